// nw_internal.h — types shared by the C ABI (nw_api.cpp) and the gfx950 kernels.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/ninwave.h"
#include "nw_host.h"

namespace nw {

// Everything a kernel needs to evaluate W[f, k] and to mask X, for one execute.
//
// The wavelet row of the reference's cache (base.py:258-279) has len_full bins,
// bin j carrying psi_f(j * delta) for j < len_valid (analytic kinds) or the
// host-supplied table value.  At execute time cwt() pad_to's it to the signal
// length n (base.py:75-82, 396-397): crop when len_full > n, else centre-pad by
// off = (n - len_full) // 2.  So output bin k uses row bin j = k - off, valid
// iff 0 <= j < len_valid.  X bins k >= xlim are zeroed (interpolate_alias on
// fft(x), base.py:400-401).  scale = 1/n folds scipy's ifft normalisation.
struct WDesc {
    int     kind;
    int     nfreq;
    int64_t n;          // signal length at execute
    int64_t nh;         // n/2 + 1: row length of the R2C half spectrum
    int64_t off;
    int64_t len_valid;
    int64_t len_full;
    int64_t xlim;
    double  delta;      // grid spacing of the cache build
    double  scale;      // 1/n
    // Morse (wavelets.py:65-74)
    double  b, r, b_over_r;
    // 1 when some Morse bin of the plan overflows the reference's fp64 x^b or exp term (large
    // b, tiny f): the rows then take the overflow-checked forms (morse_special)
    int     morse_ovf;
    // Morlet (wavelets.py:118-136): cpi = c * pi^(-1/4), kappa = k
    double  sigma, cpi, kappa;
    // per-frequency device arrays [nfreq]
    const double* freq;      // f
    const double* peak;      // Morlet p(f) = sigma / (1 - exp(-sigma f))
    const float*  xstep32;   // fp32 path: (float)(delta / f)  (Morse) or (float)(delta / f * p(f)) (Morlet)
    const void*   table;     // NW_TABLE: complex[nfreq][len_full] of the plan dtype
    const int64_t* row_len;  // NW_TABLE: true length of each (left-aligned) row
};

template <typename T> struct cplx { T re, im; };

// Timed launches (NW_TIMING): staged() (nw_api.cpp) hands the two events of a stage to the
// kernel launches the stage makes through nw_launch -- the first launch takes the start event,
// every launch the stop event -- and hipExtLaunchKernel stamps them with the dispatch's own
// begin / end (no marker packets between the kernels: recorded with hipEventRecord, the two
// markers around each launch cost a C2 step 10 %).  Other launches run untimed.
struct StageEvents {
    hipEvent_t start = nullptr, stop = nullptr;
    int launches = 0;
};
StageEvents& stage_events();   // thread-local

template <typename K, typename... Args>
inline void nw_launch(K kernel, dim3 grid, dim3 block, size_t lds, hipStream_t s, Args... args) {
    StageEvents& se = stage_events();
    if (se.stop) {
        hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, s, se.start, se.stop, 0u, args...);
        se.start = nullptr;
        ++se.launches;
    } else {
        hipLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, s, args...);
    }
}

// ---------------------------------------------------------------------------
// Analytic spectra.  fp64 follows the reference expression order exactly;
// fp32 evaluates Morse in the log2 domain (x^b overflows fp32).
// ---------------------------------------------------------------------------

__device__ __forceinline__ double psi_f64(const WDesc& d, int fi, int64_t j) {
    const double nu = (double)j * d.delta;               // np.arange fill: j * step
    if (d.kind == NW_MORSE) {
        const double x = nu / d.freq[fi];
        const double step = x > 0.0 ? 1.0 : (x == 0.0 ? x : 0.0);   // np.heaviside(x, x)
        return 2.0 * (step * pow(x, d.b) * exp(d.b_over_r * (1.0 - pow(x, d.r))));
    } else if (d.kind == NW_MORLET) {
        const double x = nu / d.freq[fi] * d.peak[fi];
        const double a = d.sigma - x;
        return d.cpi * (exp(-(a * a) / 2.0) - d.kappa * exp(-(x * x) / 2.0));
    } else {  // NW_SHANNON: 1 for nu <= 1, freq unused
        return nu <= 1.0 ? 1.0 : 0.0;
    }
}

// fp32 Morse psi at x = j * xstep (x > 0), in the log2 domain:
// log2(psi/2) = b*log2(x) + (b/r)*log2(e)*(1 - x^r).  Contractions are explicit so the W
// table (wtable_kernel), the two-pass row evaluator (RowW) and the fused kernel's in-register
// W tail produce the same bits in every compilation context.
// The reference evaluates 2 * (x^b * exp((b/r)(1 - x^r))) in fp64 (wavelets.py:65-74): where a
// factor overflows (x^b for large b and x = nu / f >> 1, or exp for b/r > 709), the product is
// inf, or NaN (inf * 0) when the other factor underflowed to 0 -- and a NaN bin makes the whole
// row NaN (ifft).  morse_special gives that value from the two factors' log magnitudes (lp of
// x^b, lq of the exp term, log base 2^(1/LN)): +inf, NaN, or 0 when neither overflows.
template <typename F>
__device__ __forceinline__ bool morse_special(F lp, F lq, F lmax, F lmin_p, F lmin_q, F* v) {
    const bool p_inf = lp >= lmax, q_inf = lq >= lmax;
    if (!(p_inf || q_inf)) return false;
    *v = ((p_inf && lq < lmin_q) || (q_inf && lp < lmin_p)) ? (F)__builtin_nan("") : (F)__builtin_inf();
    return true;
}
// CHECK: apply the reference's overflow semantics (tables, and rows of plans with morse_ovf)
// The exponentials are the raw v_exp_f32 (round 5; exp2f wrapped each in a denormal-range
// compare / select / ldexp): a psi below 2^-126 (1e-38 of the row's peak 2) is 0, which every
// table, support scan and row evaluator share, so the zeros the pruning relies on agree.
template <bool CHECK = true>
__device__ __forceinline__ float morse_f32(float x, float b, float c1, float rr) {
    const float lx = __log2f(x);
    const float lq = c1 * (1.0f - __builtin_amdgcn_exp2f(rr * lx));
    const float e2 = __builtin_fmaf(b, lx, lq);   // the contraction clang chose for the plain expression
    float v = 2.0f * __builtin_amdgcn_exp2f(e2);
    if constexpr (CHECK) {
        // fp64 thresholds in log2: overflow at 2^1024, x^b underflows below 2^-1074, exp below 2^-1075
        float sp;
        if (morse_special<float>(b * lx, lq, 1024.0f, -1074.0f, -1075.0f, &sp)) v = sp;
    }
    return v;
}
__device__ __forceinline__ float morse_c1_f32(const WDesc& d) { return (float)(d.b_over_r * 1.4426950408889634); }

__device__ __forceinline__ float psi_f32(const WDesc& d, int fi, int64_t j) {
    if (d.kind == NW_MORSE) {
        const float x = (float)j * d.xstep32[fi];
        if (!(x > 0.0f)) return 0.0f;
        return morse_f32(x, (float)d.b, morse_c1_f32(d), (float)d.r);
    } else if (d.kind == NW_MORLET) {
        const float x = (float)j * d.xstep32[fi];
        const float a = (float)d.sigma - x;
        return (float)d.cpi * (expf(-(a * a) * 0.5f) - (float)d.kappa * expf(-(x * x) * 0.5f));
    } else {
        const double nu = (double)j * d.delta;
        return nu <= 1.0 ? 1.0f : 0.0f;
    }
}

template <typename T> __device__ __forceinline__ T psi(const WDesc& d, int fi, int64_t j);
template <> __device__ __forceinline__ double psi<double>(const WDesc& d, int fi, int64_t j) { return psi_f64(d, fi, j); }
template <> __device__ __forceinline__ float  psi<float >(const WDesc& d, int fi, int64_t j) { return psi_f32(d, fi, j); }

// W[f, k] for output bin k (scaled by 1/n), complex in general (TABLE rows).
template <typename T>
__device__ __forceinline__ cplx<T> wavelet_bin(const WDesc& d, int fi, int64_t k) {
    cplx<T> w{T(0), T(0)};
    if (d.kind == NW_TABLE) {
        // every row is pad_to'd on its own (rows may differ in length)
        const int64_t len = d.row_len[fi];
        const int64_t j = k - (len < d.n ? (d.n - len) / 2 : 0);
        if (j >= 0 && j < len) {
            const cplx<T> t = reinterpret_cast<const cplx<T>*>(d.table)[(int64_t)fi * d.len_full + j];
            w.re = t.re * (T)d.scale;
            w.im = t.im * (T)d.scale;
        }
    } else {
        const int64_t j = k - d.off;
        if (j >= 0 && j < d.len_valid) w.re = psi<T>(d, fi, j) * (T)d.scale;
    }
    return w;
}

// X[k] of a real signal from its R2C half spectrum (conjugate symmetry), masked.
template <typename T>
__device__ __forceinline__ cplx<T> spectrum_bin(const cplx<T>* __restrict__ Xs, const WDesc& d, int64_t k) {
    cplx<T> x{T(0), T(0)};
    if (k < d.xlim) {
        if (k < d.nh) {
            x = Xs[k];
        } else {
            x = Xs[d.n - k];
            x.im = -x.im;
        }
    }
    return x;
}

// launchers (nw_kernels.hip)
hipError_t launch_multiply(const WDesc& d, int dtype, const void* X, void* Y, int64_t nsig, hipStream_t s);
hipError_t launch_epilogue(int dtype, int out_kind, const void* Y, void* out, int64_t count, hipStream_t s);
hipError_t launch_rows(const WDesc& d, int dtype, void* rows, hipStream_t s);
// repeated rows: dst (nsig, nf, row) from src (nsig, nu, row), scales grouped by distinct row
hipError_t launch_gather(const void* src, void* dst, const int32_t* idx, int count, size_t elem_bytes, hipStream_t s);
// debug library: one 64-lane block whose lanes >= 32 fail an NW_DCHECK (no memory access)
hipError_t launch_dcheck_selftest(hipStream_t s);
hipError_t launch_expand_rows(const void* src, void* dst, int64_t nsig, int nu, int nf, size_t row_bytes,
                              const int32_t* offs, const int32_t* order, hipStream_t s);
// epoch reductions: source kinds of launch_accumulate
enum { ACC_POWER_REAL = 0, ACC_POWER_Y = 1, ACC_PHASE_Y = 2 };
hipError_t launch_accumulate(int dtype, int src_kind, const void* src, double* acc, int64_t fn, int64_t c,
                             hipStream_t s);
hipError_t launch_finalize(int dtype, bool itc, const double* acc, void* out, int64_t fn, int64_t nsig,
                           hipStream_t s);
hipError_t launch_add_f64(double* acc, const double* src, int64_t count, hipStream_t s);
// WaveletMode.Normal rows built on the device (base.py:249-256): one row per freq, laid
// out in the FFT scratch grouped by row length (off), m timeline samples between
// `half` zeros on each side (len = m + 2*half), np.arange's fill (t0, t1, delta).
hipError_t launch_normal_time(const NormalRow* rows, int nrows, int64_t lmax, int kind, double sigma, void* buf,
                              hipStream_t s);
hipError_t launch_normal_finish(const NormalRow* rows, int nrows, int64_t lmax, bool interp, const void* buf,
                                int dtype, void* table, hipStream_t s);

// Time-domain wavelets (base.py:346-376): Reverse kinds fill an fp64 spectrum row on
// arange(0, sfreq/f*rwl, 1/f) (buffer offset `off`, m points), the time kinds a timeline
// t0, t1, t0 + i*delta (m points); `len` is the returned row length.
struct WaveRow {
    int64_t off, m, len;
    double t0, t1, delta;
};
struct WaveParams {
    int kind;
    double b, r, b_over_r;        // Morse
    double sigma, cpi, kappa;     // Morlet (cpi = c * pi^(-1/4)), MexicanHat (sigma)
};
hipError_t launch_wavelet_spectra(const WaveRow* rows, int nrows, WaveParams wp, void* buf, hipStream_t s);
hipError_t launch_wavelet_pack(const WaveRow* rows, int nrows, int64_t maxlen, const void* buf, void* out,
                               hipStream_t s);
hipError_t launch_wavelet_time(const WaveRow* rows, int nrows, int64_t maxlen, WaveParams wp, void* out,
                               hipStream_t s);

constexpr int BL_WORK_DOUBLES = 1024 + 2;   // k_bl_partial blocks + (mean, std)
hipError_t launch_baseline(int dtype, const void* x, int64_t count, int64_t b0, int64_t b1, int op, void* out,
                           double* work, hipStream_t s);
// fused engine (nw_fused.hip)
bool       fused_supported(int64_t n, int dtype);
hipError_t fused_prepare(int64_t n, int dtype);
size_t     fused_wtable_bytes(int64_t n, int nfreq, int dtype, int kind);
hipError_t build_wtable(const WDesc& d, int dtype, void* wtab, hipStream_t s);
hipError_t launch_fused(const WDesc& d, int dtype, int out_kind, const void* X, const void* wtab, void* out,
                        int64_t nsig, hipStream_t s);
int        fused_kernel_id(int64_t n, int dtype, int kind);   // NW_K_FUSED or NW_K_FUSED_PAIR
// forward R2C of nsig real rows of length n (fused sizes) into half spectra of row stride nh
hipError_t fused_forward(int64_t n, int dtype, const void* x, void* X, int64_t nsig, int64_t nh, hipStream_t s);
hipError_t fused_twiddles(int64_t n, int dtype, void** out);   // exact exp(+2 pi i j / n), cached per device
// epoch reduction partials (fused sizes, fp32 analytic rows; power up to E = 32, phase
// E <= 16): per block of signals the sum over its signals (fp64, in signal order) of |y|^2,
// or with phase of y / |y|; one
// (groups, F, n) row of fp64 (phase: complex fp64) per (group, scale);
// groups = fused_psum_groups(nsig)
// Signals per partial-sum row: the block size of both the fused kernels (kGroup) and the
// chirp-z kernel (kGroupC), each static_assert'ed equal to it, so one fused_psum_groups sizes
// and accumulates the partial rows of either form
constexpr int kPsumGroup = 8;

// W support for the pruned pass 0 / row pass (wsupport_kernel, kmax_kernel): the last bin
// whose |W| exceeds kTailRel x the row's max |W|.  The bins past it (the far tail of a Morse
// row, exactly zero only where exp underflows, ~9x the peak frequency in fp64) are left out;
// each holds |W| below kTailRel of the row's peak, so together they move y by less than
// n * kTailRel of the signal's scale: 2^-48 (fp64) / 2^-32 (fp32) at n = 2^24, far below each
// dtype's own FFT rounding (1e-15 / 1e-7) and the parity contract (1e-12 / 1e-5).  Non-finite
// bins (the reference's inf / NaN rows, morse_special) stay in the support and out of the max.
#ifdef NW_TAIL_EXACT   // diagnostic A/B: the exact support (every nonzero bin)
template <typename T> constexpr double kTailRel = 0.0;
#else
template <typename T> constexpr double kTailRel = sizeof(T) == 8 ? 0x1p-72 : 0x1p-56;
#endif
__host__ __device__ inline double tail_max_term(double mag) { return mag <= 1.7976931348623157e308 ? mag : 0.0; }
__host__ __device__ inline bool tail_in_support(double mag, double thr) { return !(mag <= thr); }
bool fused_psum_supported(int64_t n, int dtype, int kind, bool phase);
int64_t fused_psum_groups(int64_t nsig);
int fused_psum_kernel_id(int64_t n, int dtype, bool phase);   // NW_K_FUSED or NW_K_FUSED_PAIR
hipError_t fused_power_partials(const WDesc& d, int dtype, bool phase, const void* X, const void* wtab,
                                void* partials, int64_t nsig, hipStream_t s);

// chirp-z engine (nw_chirp.hip): n not taken by the power-of-two kernels, 2n - 1 <= 16384
// (fp32) / 8192 (fp64); one (scale, signal) row = two on-chip FFTs of M = 2^ceil(log2(2n-1))
bool       chirp_supported(int64_t n, int dtype);
bool       chirp_possible(int64_t n, int dtype);   // also n < M_max when every row's support fits
size_t     chirp_wtable_bytes(int64_t n, int nfreq, int dtype, int kind);
// builds W, each row's support and the rows grouped by M class (M = 1024 << c, c < 5:
// counts[c] rows each; synchronises s once); launch_chirp runs one kernel per class
// rows whose support does not fit the largest on-chip transform get no M class: *fits is
// false and (overflow non-null) their indices are listed; counts[] covers the others
hipError_t build_chirp_wtable(const WDesc& d, int dtype, void* wtab, hipStream_t s, int64_t* counts, bool* fits,
                              std::vector<int>* overflow);
hipError_t launch_chirp(const WDesc& d, int dtype, int out_kind, const void* X, const void* wtab, void* out,
                        int64_t nsig, const int64_t* counts, hipStream_t s);
bool chirp_psum_ok(int dtype, bool phase, const int64_t* counts);

// two-pass engine for long signals (nw_large.hip): power-of-two 2^15 <= n <= 2^24, fp32 or
// fp64.  scratch = Xt (n complex) + B (large_fchunk scales x n complex); support = kmax[nfreq]
// + the fp64 column-pass twiddle tables.
bool       large_supported(int64_t n, int dtype);
size_t     large_scratch_bytes(int64_t n, int nfreq, int dtype);
size_t     large_support_bytes(int nfreq);
int64_t    large_fchunk(int64_t n, int nfreq, int dtype);
hipError_t build_large_support(const WDesc& d, int dtype, void* support, hipStream_t s);
// kmax[] / wmax[] of the rows into support (its first nfreq ints are kmax): the analytic kinds
// without a full scan (support_fast_kernel), the others -- or scan = true -- by scanning every bin
hipError_t large_row_support(const WDesc& d, int dtype, void* support, bool scan, hipStream_t s);
hipError_t large_transpose(const WDesc& d, int dtype, const void* X, void* scratch, hipStream_t s);
hipError_t large_rows(const WDesc& d, int dtype, int f0, int nf, const void* support, void* scratch, hipStream_t s);
hipError_t large_cols(const WDesc& d, int dtype, int out_kind, int f0, int nf, const void* support,
                      const void* scratch, void* out, hipStream_t s);

}  // namespace nw
