// nw_large.hip — the fused CWT engine for long power-of-two signals (fp32 and fp64,
// n = 2^15 .. 2^24).
//
// One output row y_f = ifft_n(W_f * X) (reference base.py:378-407: scipy ifft, 1/n folded
// into W) is longer than one workgroup's LDS holds, so it is computed as a four-step
// transform n = N1 * N2 (N2 <= 16384 on chip per workgroup, 32 <= N1 <= 1024):
//
//   k = k1 + N1*k2,   n = n2 + N2*n1,   Z = W_f * X,   w_M = exp(+2 pi i / M)
//   y[n2 + N2 n1] = sum_k1 w_N1^(n1 k1) * ( w_n^(n2 k1) * sum_k2 Z[k1 + N1 k2] w_N2^(n2 k2) )
//
// Kernels, per signal:
//   xt_kernel    X (R2C half spectrum, conjugate-mirrored above n/2, interpolate-masked,
//                base.py:400-401) -> Xt[k1][k2] = X[k1 + N1 k2], n complex; once per signal
//   rows_kernel  per (scale f, row k1): z[k2] = W_f[k1 + N1 k2] * Xt[k1][k2] with W evaluated
//                in registers (the expression wtable_kernel uses: analytic psi or the table
//                row, pad_to + 1/n), pruned to the row's support (kmax[f], the last nonzero
//                bin), a length-N2 inverse FFT on chip (the nw_fused pass machinery), the
//                complex row stored to B[f][k1][0 .. N2)
//   cols_kernel  per (scale f, C consecutive n2): v[k1] = B[f][k1][n2] * w_n^(n2 k1), C
//                length-N1 inverse FFTs side by side (C * N1 = 32768 fp32 / 16384 fp64 points
//                per 1024-thread workgroup, C * 2e B contiguous per k1 read), epilogue y / |y|
//                / |y|^2 stored to out[f][n2 + N2 n1] (256-B contiguous runs at N1 = 1024)
//
// fp64: E = 32 rows (16 for table rows), 32 elements per thread in the column pass, the
// column twiddles from two exact split tables and a per-thread recurrence, Morse rows in
// the log domain (RowW<double>).
//
// Measured at C5 (1 x 2^24 x 512, tools/ablate.sh): the column pass is bound by its
// mixed read + write HBM stream (4.4 TB/s combined; without its stores it reads at
// 4.7 TB/s and the FFT work costs < 3 %); the row pass is the fused kernel's
// write-bound form (W evaluation 9 % of it).
//
// HBM per output point: B written and read once (16 B) and y written once; X per row
// from L2 (rows of one k1 group are swept over 8 scales per XCD tile).  The rocFFT engine
// it replaces moves K1's product + ~3 in-place passes of rocFFT at n = 2^24.
// B is written with streaming (nt) stores like every output: measured at C5, plain stores
// (to keep B in the 256 MiB Infinity Cache for the column pass) and 1-2 scales per launch
// pair (B = 134-268 MB) were slower (51.6 / 65.1 / 93.2 ms per step for 16 / 2 / 1 scales
// with plain stores vs 49.3 with nt at 16): the column pass gains <= 8 % from the cache
// hits, the row pass loses its Xt reuse across the scales of a tile.
#include <cstdlib>

#include "nw_fft_dev.h"

namespace nw {

namespace {

constexpr int kRowGroup = 4;      // rows (k1) per rows_kernel workgroup (1 when a launch holds few scales)
constexpr int kRowTileF = 8;      // scales per XCD tile
constexpr int kRowTileG = 8;      // row groups per XCD tile
// cols_kernel workgroups of 1024 threads: C = 32 columns at N1 = 1024, 256-B runs (C5 cols
// 1.039 -> 0.978 ms per launch against 512 threads)
// cols_kernel workgroup size (C * N1 / E)
// fp64: 512 threads x 32 elements (N1 = 1024 in 2 passes, one exchange; 16 columns, 256-B runs
// as before) against 1024 x 16 (3 passes, two exchanges): C5 fp64 cols 3.97-4.11 -> 3.90-3.91
// ms per 32-scale launch (profiles/r05_c5f64_cols_e32_ab.txt; -DNW_COLS64_E16: the old form)
#ifdef NW_COLS64_E16
template <typename T> constexpr int kColThreads = 1024;
#else
template <typename T> constexpr int kColThreads = sizeof(T) == 8 ? 512 : 1024;
#endif
// bytes of B per launch pair (scales chunked to fit): 8 GiB = 64 scales of fp32 / 32 of fp64 at
// C5.  Against 2 GiB (16 / 8 scales): C5 fp32 47.49 -> 46.15 ms per step, fp64 118.19 -> 113.15
// (fewer, longer launches: the row pass's XCD tiles of 8 scales fill, fewer tails;
// profiles/r04_c5_fchunk.txt)
constexpr size_t kBBudget = size_t(8) << 30;

// N2 (on-chip rows) and its elements per thread E: the nw_fused sizes (fp64: E = 16, N2 <= 8192)
template <typename T, int N2> constexpr int kRowE = N2 >= 8192 ? 32 : 16;
// complex table rows (wavelet_bin loads) spill at fp64 E = 32: E = 16 there
template <typename T, int N2> constexpr int kRowETab = sizeof(T) == 8 ? 16 : kRowE<T, N2>;
// elements per thread in cols_kernel: 32 complex fp32 (64 VGPRs) or fp64 (128 VGPRs, 2 waves/SIMD)
#ifdef NW_COLS64_E16
template <typename T> constexpr int kColE = sizeof(T) == 4 ? 32 : 16;
#else
template <typename T> constexpr int kColE = 32;
#endif
// rows of at most 16384 on chip, fp64 too (N2 = 8192 with N1 = 2048, 8-column blocks and
// 128-B runs: C5 fp64 150.0 ms/step; 16384, 16 columns, 256-B runs: 129.9)
// (fp32 rows of 32768 -- N1 = 512, 64-column workgroups writing 512-B output pieces -- measured
// in round 6: the row pass at one 1024-thread block per CU +37-43 %, the column pass 0-3 %
// faster, C5 step +10 %; profiles/r06_c5_rows32k_ab.txt)
template <typename T> constexpr int kMaxN2 = 16384;

// ---- X (R2C half spectrum) -> Xt[k1][k2], mirrored + masked (spectrum_bin)
template <typename T>
__global__ __launch_bounds__(256) void xt_kernel(WDesc d, const cplx<T>* __restrict__ X, C2<T>* __restrict__ Xt,
                                                 int n1, int n2) {
    __shared__ C2<T> tile[32][33];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    const int k1_0 = blockIdx.x * 32, k2_0 = blockIdx.y * 32;
    for (int i = ty; i < 32; i += 8) {
        const int64_t k = (int64_t)(k1_0 + tx) + (int64_t)n1 * (k2_0 + i);
        const cplx<T> x = spectrum_bin<T>(X, d, k);
        tile[i][tx] = C2<T>{x.re, x.im};
    }
    __syncthreads();
    for (int i = ty; i < 32; i += 8) Xt[(int64_t)(k1_0 + i) * n2 + k2_0 + tx] = tile[tx][i];
}

// ---- kmax[f] = last bin k < min(n, xlim) with |W_f[k]| above kTailRel x the row's max |W|
// (nw_internal.h; -1: none); pass-1 pruning.  wmax_kernel first: the row maxima as the bit
// patterns of non-negative doubles (ordered as unsigned integers, so atomicMax keeps the max)
constexpr int kSupBins = 16;   // bins per thread
template <typename T, bool REALW>
__device__ __forceinline__ double wmag(const WDesc& d, int fi, int64_t k) {
    const cplx<T> w = wavelet_bin<T>(d, fi, k);
    return REALW ? fabs((double)w.re) : fmax(fabs((double)w.re), fabs((double)w.im));
}
template <typename T, bool REALW>
__global__ __launch_bounds__(256) void wmax_kernel(WDesc d, unsigned long long* __restrict__ wmax) {
    const int fi = blockIdx.y;
    const int64_t lim = d.xlim < d.n ? d.xlim : d.n;
    const int64_t k0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * kSupBins;
    double m = 0.0;
    for (int i = 0; i < kSupBins; ++i) {
        const int64_t k = k0 + i;
        if (k >= lim) break;
        m = fmax(m, tail_max_term(wmag<T, REALW>(d, fi, k)));
    }
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0 && m > 0.0) atomicMax(&wmax[fi], (unsigned long long)__double_as_longlong(m));
}
template <typename T, bool REALW>
__global__ __launch_bounds__(256) void kmax_kernel(WDesc d, int* __restrict__ kmax, const unsigned long long* __restrict__ wmax) {
    const int fi = blockIdx.y;
    const int64_t lim = d.xlim < d.n ? d.xlim : d.n;
    const int64_t k0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * kSupBins;
    const double thr = kTailRel<T> * __longlong_as_double((long long)wmax[fi]);
    int m = -1;
    for (int i = 0; i < kSupBins; ++i) {
        const int64_t k = k0 + i;
        if (k >= lim) break;
        if (tail_in_support(wmag<T, REALW>(d, fi, k), thr)) m = (int)k;
    }
    // wave max, then one atomic per wave
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0 && m >= 0) atomicMax(&kmax[fi], m);
}

// ---- The same wmax[f] and kmax[f] for the analytic kinds without a full scan.  A Morse,
// Morlet (sigma > 0) or Shannon row is unimodal in k: |psi| rises to its peak (Morse nu = f,
// Morlet x = nu/f p(f) ~ sigma, Shannon k = 0) and falls after it (the computed value c(k) is
// the true g(x_k) times (1 + e_k), |e_k| <= eps, with x_k monotone in k).  One 256-thread block
// per row, O(window + F log n) evaluations of the scan's own wmag instead of 2 n:
//  1. max: scan a window around the analytic peak, widened 4x until both window edges lie
//     at the row's ends or below M (1 - kMu); then no bin outside exceeds the window's max M
//     (if g rose past an edge, that edge would be within 2 eps of M; if it fell, every bin
//     beyond is below the edge's value times (1 + 3 eps)), so M is the full scan's max.
//  2. kmax: a 256-ary bisection on [argmax, end) for a bin J with c(J) <= L = thr (1 - kMu);
//     every bin past J is then <= L (1 + 3 eps) < thr, so the last bin above thr lies in
//     [argmax, J): a backward scan from J finds it -- the full scan's kmax.
// kMu >> 3 eps: fp64 evaluations are within ~1e-12 relative wherever they matter, fp32's
// log2-domain Morse within ~3e-5 (v_log / v_exp on exponents of magnitude <= 200).
// Plans whose rows may hold non-finite bins (morse_ovf), tables, sigma <= 0, b <= 0 and the
// exact support (kTailRel = 0) keep wmax_kernel / kmax_kernel; a row that still meets a
// non-finite value here is scanned whole by its block (the scan kernels' rules).
template <typename T> constexpr double kMu = sizeof(T) == 8 ? 0x1p-30 : 0x1p-10;
constexpr int kFastThreads = 256, kFastBins = 16;   // bins per thread per scan round

bool support_fast_ok(const WDesc& d, int dtype) {
    if ((dtype == NW_F32 ? kTailRel<float> : kTailRel<double>) == 0.0) return false;
    if (d.kind == NW_MORSE) return !d.morse_ovf && d.b > 0.0 && d.r > 0.0;
    if (d.kind == NW_MORLET) return d.sigma > 0.0;
    return d.kind == NW_SHANNON;
}

// block reductions over kFastThreads threads (4 waves): max with its (smallest) bin, min bin
__device__ __forceinline__ void blk_max_arg(double& v, int64_t& k, double* sv, int64_t* sk) {
    for (int o = 32; o > 0; o >>= 1) {
        const double v2 = __shfl_xor(v, o, 64);
        const int64_t k2 = __shfl_xor(k, o, 64);
        if (v2 > v || (v2 == v && k2 < k)) { v = v2; k = k2; }
    }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) { sv[w] = v; sk[w] = k; }
    __syncthreads();
    v = sv[0]; k = sk[0];
    for (int i = 1; i < kFastThreads / 64; ++i)
        if (sv[i] > v || (sv[i] == v && sk[i] < k)) { v = sv[i]; k = sk[i]; }
}
__device__ __forceinline__ int64_t blk_min_i64(int64_t k, int64_t* sk) {
    for (int o = 32; o > 0; o >>= 1) k = min(k, (int64_t)__shfl_xor(k, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sk[threadIdx.x >> 6] = k;
    __syncthreads();
    for (int i = 0; i < kFastThreads / 64; ++i) k = min(k, sk[i]);
    return k;
}
__device__ __forceinline__ int64_t blk_max_i64(int64_t k, int64_t* sk) {
    for (int o = 32; o > 0; o >>= 1) k = max(k, (int64_t)__shfl_xor(k, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sk[threadIdx.x >> 6] = k;
    __syncthreads();
    for (int i = 0; i < kFastThreads / 64; ++i) k = max(k, sk[i]);
    return k;
}

template <typename T>
__global__ __launch_bounds__(kFastThreads) void support_fast_kernel(WDesc d, int* __restrict__ kmax,
                                                                    unsigned long long* __restrict__ wmax) {
    __shared__ double sv[kFastThreads / 64];
    __shared__ int64_t sk[kFastThreads / 64];
    const int fi = blockIdx.x;
    const int t = threadIdx.x;
    const int64_t lim = d.xlim < d.n ? d.xlim : d.n;
    const int64_t lo = d.off > 0 ? d.off : 0;
    const int64_t hi = min(lim, d.off + d.len_valid);   // W = 0 outside [lo, hi)
    if (hi <= lo) return;                                // kmax -1, wmax 0 (memset)
    auto mag = [&](int64_t k) { return wmag<T, true>(d, fi, k); };
    // the analytic peak's row bin j* (x = 1 for Morse, x = sigma for Morlet, 0 for Shannon)
    const double f = d.freq[fi];
    double js = 0.0;
    if (d.kind == NW_MORSE) js = f / d.delta;
    else if (d.kind == NW_MORLET) js = d.sigma * f / (d.peak[fi] * d.delta);
    const double kd = (double)d.off + (js == js ? js : 0.0);
    const int64_t kp = kd <= (double)lo ? lo : kd >= (double)(hi - 1) ? hi - 1 : (int64_t)kd;
    bool bad = false;
    // 1. the row max over a widening window around the peak
    double M = 0.0;
    int64_t m = lo;
    for (int64_t w = kFastThreads * kFastBins / 2;; w *= 4) {
        const int64_t a = max(lo, kp - w), b = min(hi - 1, kp + w);
        double v = -1.0;
        int64_t kv = b;
        for (int64_t k = a + t; k <= b; k += kFastThreads) {
            const double c = mag(k);
            if (!(c <= 1.7976931348623157e308)) bad = true;
            else if (c > v) { v = c; kv = k; }
        }
        bad = __syncthreads_or(bad);            // block-wide: the branch below holds barriers
        if (bad) break;
        blk_max_arg(v, kv, sv, sk);
        M = v;
        m = kv;
        const double edge = M * (1.0 - kMu<T>);
        if ((a == lo || mag(a) <= edge) && (b == hi - 1 || mag(b) <= edge)) break;
    }
    if (bad) {
        // the scan kernels' rules over the whole row: the max of the finite bins, then the last
        // bin above the threshold with non-finite bins in the support
        double v = 0.0;
        int64_t kv = lo;
        for (int64_t k = lo + t; k < hi; k += kFastThreads) v = fmax(v, tail_max_term(mag(k)));
        blk_max_arg(v, kv, sv, sk);
        const double thr = kTailRel<T> * v;
        int64_t found = -1;
        for (int64_t k = lo + t; k < hi; k += kFastThreads)
            if (tail_in_support(mag(k), thr)) found = k;
        found = blk_max_i64(found, sk);
        if (t == 0) {
            wmax[fi] = (unsigned long long)__double_as_longlong(v);
            kmax[fi] = (int)found;
        }
        return;
    }
    if (M <= 0.0) return;                               // an all-zero row: kmax -1, wmax 0
    const double thr = kTailRel<T> * M;
    const double L = thr * (1.0 - kMu<T>);
    // 2. a bin J >= m with c(J) <= L: 256-ary bisection on [m, hi); J = hi when none
    int64_t l = m, r = hi;                              // c(l) > L; c(r) <= L or r = hi
    if (mag(hi - 1) <= L) {
        r = hi - 1;
        while (r - l > 1) {
            const int64_t span = r - l;
            // sample points l + span * (t + 1) / 257 (distinct when span > 256)
            const int64_t p = l + (span > kFastThreads ? span * (t + 1) / (kFastThreads + 1) : t + 1);
            const bool below = p < r && mag(p) <= L;
            const int64_t first = blk_min_i64(below ? p : r, sk);   // first sampled bin <= L
            // the sample before it (or l) stays above L
            const int64_t prev = blk_max_i64(p < first ? p : l, sk);
            l = prev;
            r = first;
        }
    }
    // 3. the last bin above thr in [m, r): backward scan from r - 1 (c(m) = M > thr ends it)
    int64_t km = -1;
    for (int64_t top = r - 1; km < 0 && top >= m; top -= kFastThreads * kFastBins) {
        int64_t found = -1;
        for (int i = 0; i < kFastBins; ++i) {
            const int64_t k = top - (int64_t)i * kFastThreads - t;
            if (k >= m && k > found && tail_in_support(mag(k), thr)) found = k;
        }
        km = blk_max_i64(found, sk);
    }
    if (t == 0) {
        wmax[fi] = (unsigned long long)__double_as_longlong(M);
        kmax[fi] = (int)km;
    }
}

// ---- W_f[k] of one scale in fp32 for a compile-time kind: psi_f32 (nw_internal.h) with
// the same operations in the same order, times 1/n, as wavelet_bin<float> -- so a row
// here equals the nw_fused W table bit for bit -- but on 32-bit bin indices (n <= 2^24)
// and with the per-scale constants hoisted.  j = k - off is the cached row's bin.
template <typename T, int KIND> struct RowW;
// fp64 Morse rows with r = 3 and 2b an integer in [0, 128) (the default b = 17.5): a kernel
// instantiation of its own (host dispatch, morse_fast_of), since the general log-domain form's
// ocml constants beside it spill
constexpr int kMorseFast = 100;
// ... and its instantiation for the default b = 17.5 (2b = 35): x^17 by four squarings and one
// multiply at compile time
constexpr int kMorseFast35 = 102;
// fp32 Morse rows of a plan where some bin overflows the reference's fp64 factors
// (WDesc::morse_ovf): the overflow-checked form (its own instantiation, so the default rows
// carry no check)
constexpr int kMorseOvf = 101;
// ... and b = 17.5 rows that start at bin 0 (WDesc::off == 0: every bin of a row is >= 0) with
// the exponential factor by a product recurrence over the thread's bins (RowW<double>::Rec)
constexpr int kMorseRec = 103;
#ifdef NW_ROWS_NO_REC   // diagnostic A/B: the per-bin exp form (kMorseFast35) for every b = 17.5 row
constexpr bool kRowsRec = false;
#else
constexpr bool kRowsRec = true;
#endif
template <int KIND> struct RowW<float, KIND> {
    float xs, b, c1, rr, cpi, sigma, kappa, scale;
    int off, lenv, jlim;
    __device__ __forceinline__ void init(const WDesc& d, int fi) {
        xs = d.xstep32 ? d.xstep32[fi] : 0.0f;
        b = (float)d.b;
        c1 = morse_c1_f32(d);
        rr = (float)d.r;
        cpi = (float)d.cpi;
        sigma = (float)d.sigma;
        kappa = (float)d.kappa;
        scale = (float)d.scale;
        off = (int)d.off;
        lenv = d.len_valid < 0x7fffffff ? (int)d.len_valid : 0x7fffffff;
        if constexpr (KIND == NW_SHANNON) {   // nu = j * delta <= 1.0  <=>  j <= jlim (monotone)
            int64_t j = (int64_t)(1.0 / d.delta);
            while ((double)(j + 1) * d.delta <= 1.0) ++j;
            while (j >= 0 && (double)j * d.delta > 1.0) --j;
            jlim = j < 0x7fffffff ? (int)j : 0x7fffffff;
        } else {
            jlim = 0;
        }
    }
    __device__ __forceinline__ float operator()(int j) const {
        if constexpr (KIND == NW_MORSE) {
            // branch-free (round 5): every bin evaluated, the invalid ones (past the row, x <= 0:
            // a log2 of 0 or below gives 0 or NaN here) selected to 0, so a pass-0 group's
            // evaluations interleave; the same operations as psi_f32, so the same bits
            const float x = (float)j * xs;
            const float psi = morse_f32<false>(x, b, c1, rr) * scale;
            return ((unsigned)j < (unsigned)lenv && x > 0.0f) ? psi : 0.0f;
        }
        if ((unsigned)j >= (unsigned)lenv) return 0.0f;
        float psi;
        if constexpr (KIND == kMorseOvf) {
            const float x = (float)j * xs;
            if (!(x > 0.0f)) return 0.0f;
            psi = morse_f32<KIND == kMorseOvf>(x, b, c1, rr);
        } else if constexpr (KIND == NW_MORLET) {
            const float x = (float)j * xs;
            const float a = sigma - x;
            psi = cpi * (expf(-(a * a) * 0.5f) - kappa * expf(-(x * x) * 0.5f));
        } else {
            psi = j <= jlim ? 1.0f : 0.0f;
        }
        return psi * scale;
    }
};

// fp64 rows, per-scale constants hoisted and pinned in SGPRs.  Morse in the log domain:
// x^b e^{(b/r)(1 - x^r)} = exp(b ln x + (b/r)(1 - x^r)), x = j * (delta / f) (one multiply per
// bin for the reference's nu / f with nu = j * delta: <= 2 ulp of x, i.e. < 1e-14 relative
// in psi), x^r = exp(r ln x); psi(0) = 0 as np.heaviside(0, 0).  Relative error ~ |b ln x| eps
// < 1e-13 over the rows' support.  Measured (C5 fp64 row pass): the W evaluation is 26 % of
// it (0.937 -> 0.697 ms without it).  Morlet / Shannon: psi_f64's expression.  (x^b and x^r by
// repeated squaring measured slower: 76 B of scratch; x^3 as x*x*x for r = 3 spills 44-64 B:
// the exp / log polynomial constants of ocml sit in ~22 VGPRs hoisted out of the row loop.)
// exp(y) in fp64 (|error| < 1 ulp + the final scaling's rounding): y = k ln2 + r by Cody-Waite,
// |r| <= ln2 / 2, 2^k * (Taylor polynomial of degree 13: truncation < 5e-18).  Written out
// here so its constants are plain operands the compiler can keep in SGPRs (ocml's exp keeps
// ~22 VGPRs of constants hoisted out of the row loop, which spilled every cheaper Morse form)
// The constants are pinned ONCE per row pass in SGPR pairs (ExpK, an empty volatile asm on each
// at init: opaque, so the compiler neither folds them back into per-use materialisations nor
// hoists copies into VGPRs) and read as plain SGPR operands of the FMAs.  (Round 4 pinned each
// constant at its use: an s_mov_b64 copy + an s_nop hazard wait before every FMA of the
// polynomial -- 974 s_nop in the fp64 row kernel.)
__device__ __forceinline__ double spin(double c) {
    asm volatile("" : "+s"(c));
    return c;
}
struct ExpK {
    double log2e, ln2hi, ln2lo, lo;
    double c[11];                                            // 1/13!, 1/12!, ..., 1/3!
    __device__ __forceinline__ void init() {
        log2e = spin(1.4426950408889634074);
        ln2hi = spin(6.93147180369123816490e-01);
        ln2lo = spin(1.90821492927058770002e-10);
        lo = spin(-1100.0);
        double f = 6227020800.0;                             // 13!
#pragma unroll
        for (int i = 0; i < 11; ++i) {
            c[i] = spin(1.0 / f);
            f /= (double)(13 - i);
        }
    }
};
// FINITE: y is finite (the b = 17.5 rows): no NaN pass-through, and both bounds by plain
// constants.  Valid bins have y <= 21.4; the branch-free kMorseFast35 / kMorseRec evaluators also
// evaluate the bins before a row's start (j < 0, x < 0: y = (b/r)(1 - x^3) up to ~1e9), whose
// values the final select drops -- the upper clamp keeps rint(y log2 e) inside int there too
template <bool FINITE = false>
__device__ __forceinline__ double exp_rows(double y, const ExpK& K) {
    // k fits an int: y is bounded below here (NaN -> the bound, fixed at the end); above by the
    // fast Morse form's domain, y = (b/r)(1 - x^3) <= b/3 < 21.4 (a select, not fmax: fmax
    // canonicalises its opaque SGPR operand with two extra v_max per call)
    double yc;
    if constexpr (FINITE) yc = fmin(fmax(y, -1100.0), 1100.0);
    else yc = y > K.lo ? y : K.lo;
    const double k = __builtin_rint(yc * K.log2e);
    double rr = fma(-k, K.ln2hi, yc);
    rr = fma(-k, K.ln2lo, rr);
    double p = K.c[0];                                       // 1/13!
#pragma unroll
    for (int i = 1; i < 11; ++i) p = fma(p, rr, K.c[i]);     // (degree 11: +-0 on the C5 fp64 row pass, round 5)
    p = fma(p, rr, 0.5);
    p = fma(p, rr, 1.0);
    p = fma(p, rr, 1.0);
    const double e = ldexp(p, (int)k);
    if constexpr (FINITE) return e;
    return y == y ? e : y;
}

template <int KIND> struct RowW<double, KIND> {
    static constexpr bool MORSE = KIND == NW_MORSE || KIND == kMorseFast || KIND == kMorseFast35 || KIND == kMorseRec;
    // kMorseFast: x^b by a multiply chain (+ one sqrt for the half) and x^3 by two multiplies,
    // then ONE exp -- 2 x^b exp((b/r)(1 - x^3)), the reference's own factorisation
    // (wavelets.py:65-74) -- instead of one log and two exps.  kMorseFast35 (b = 17.5, round 5)
    // is branch-free: every bin is evaluated and the invalid ones (j past the row, x <= 0)
    // selected to 0 at the end, so the evaluations of a pass-0 group interleave (the branches
    // around each one were s_and_saveexec / s_cbranch pairs that serialised them), with the
    // sqrt without the compiler's denormal scaling and class checks (x >= delta / f is normal
    // for every valid bin)
    static constexpr bool FAST = KIND == kMorseFast || KIND == kMorseFast35 || KIND == kMorseRec;
    double delta, f, xs, peak, b, r, bor, sigma, cpi, kappa, scale, scale2;
    double dx, dd;                                           // kMorseRec: bin stride in x, e^(third difference)
    int off, lenv;
    int bint, bhalf, jm1;
    ExpK ek;
    __device__ static __forceinline__ double pin(double v) {
        const long long u = __double_as_longlong(v);
        const int lo = __builtin_amdgcn_readfirstlane((int)(u & 0xffffffffLL));
        const int hi = __builtin_amdgcn_readfirstlane((int)(u >> 32));
        return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
    }
    __device__ __forceinline__ void init(const WDesc& d, int fi) {
        delta = d.delta;
        f = pin(d.freq ? d.freq[fi] : 1.0);
        xs = pin(delta / f);
        peak = pin(d.peak ? d.peak[fi] : 1.0);
        b = d.b;
        r = d.r;
        bor = d.b_over_r;
        sigma = d.sigma;
        cpi = d.cpi;
        kappa = d.kappa;
        scale = d.scale;
        scale2 = 2.0 * d.scale;
        off = (int)d.off;
        lenv = d.len_valid < 0x7fffffff ? (int)d.len_valid : 0x7fffffff;
        bint = FAST ? (int)(2.0 * d.b) / 2 : 0;
        bhalf = FAST ? (int)(2.0 * d.b) & 1 : 0;
        if constexpr (FAST) ek.init();
        jm1 = (xs > 0.0 && lenv > 0) ? lenv - 1 : 0;
    }
    // sqrt(x) for normal x > 0 to within an ulp: the rsq estimate and two Newton-Raphson steps
    // (the compiler's sequence without its denormal scaling and special-value class checks)
    __device__ static __forceinline__ double sqrt_normal(double x) {
        const double r = __builtin_amdgcn_rsq(x);
        double s = x * r, h = 0.5 * r;
        const double e = fma(-h, s, 0.5);
        s = fma(s, e, s);
        h = fma(h, e, h);
        double d = fma(-s, s, x);
        s = fma(d, h, s);
        d = fma(-s, s, x);
        return fma(d, h, s);
    }
    // kMorseRec: the exponential factor e^{E(x)}, E(x) = (b/r)(1 - x^3), over a thread's bins
    // x_g + i D (D = the bin stride times xs) by products of its finite differences: E is a
    // cubic, so e^{E(x+D)} = e^{E(x)} a, a <- a c, c <- c dd with a = e^{E(x+D) - E(x)},
    // c = e^{second difference} and dd = e^{-6 (b/r) D^3} constant per scale -- three
    // multiplies per bin instead of an exp.  Restarted with three exps every kRecGroup bins:
    // the rounding of c and dd is raised to the C(i,2) / C(i,3) power within a group, so 16
    // keeps psi within 3.3e-14 of its row maximum (numpy emulation against long double over
    // D = 0.004 .. 10; the direct exp: 1e-15), far inside the 1e-12 parity contract
    static constexpr int kRecGroup = 16;
    struct Rec { double e, a, c; };
    __device__ __forceinline__ void init_rec(int stride) {
        dx = pin((double)stride * xs);
        dd = pin(exp_rows<true>(-bor * (6.0 * (dx * dx * dx)), ek));
    }
    __device__ __forceinline__ Rec start(int j) const {
        const double x = (double)j * xs;
        const double e0 = bor * (1.0 - (x * x) * x);
        const double d1 = -bor * (dx * (3.0 * (x * x) + dx * (3.0 * x + dx)));   // E(x + D) - E(x)
        const double d2 = -bor * (6.0 * (dx * dx) * (x + dx));                  // its difference
        return Rec{exp_rows<true>(e0, ek), exp_rows<true>(d1, ek), exp_rows<true>(d2, ek)};
    }
    __device__ __forceinline__ double step(int j, Rec& q) const {
        const double x = (double)j * xs;
        const double x2 = x * x, x4 = x2 * x2, x8 = x4 * x4, x16 = x8 * x8;
        const double xb = (x16 * x) * sqrt_normal(x);
        const double psi = (xb * q.e) * scale2;
        q.e *= q.a;
        q.a *= q.c;
        q.c *= dd;
        return (unsigned)(j - 1) < (unsigned)jm1 ? psi : 0.0;
    }
    __device__ __forceinline__ double operator()(int j) const {
        if constexpr (KIND == kMorseFast35 || KIND == kMorseRec) {
            // branch-free (the general kMorseFast form below keeps its branches: interleaved,
            // its runtime chain and sqrt select spilled 236 B)
            const double x = (double)j * xs;
            const double x2 = x * x, x4 = x2 * x2, x8 = x4 * x4, x16 = x8 * x8;
            const double xb = (x16 * x) * sqrt_normal(x);
            // 2 * (x^b e) * scale: 2 * scale is a power of two, so one multiply by it rounds alike
            const double psi = (xb * exp_rows<true>(bor * (1.0 - x2 * x), ek)) * scale2;
            // valid bins 1 <= j < lenv (x > 0 <=> j > 0 with xs > 0; none when xs <= 0: psi = 0
            // there, heaviside(x, x) of x <= 0): one unsigned compare on integers, j - 1 < jm1
            return (unsigned)(j - 1) < (unsigned)jm1 ? psi : 0.0;
        }
        if ((unsigned)j >= (unsigned)lenv) return 0.0;
        double psi;
        if constexpr (MORSE) {
            const double x = (double)j * xs;
            if (!(x > 0.0)) return 0.0;
            if constexpr (FAST) {
                double xb = bhalf ? sqrt(x) : 1.0, pw = x;
                for (int e = bint; e; e >>= 1) {                 // uniform trip count
                    if (e & 1) xb *= pw;
                    pw *= pw;
                }
                psi = 2.0 * (xb * exp_rows(bor * (1.0 - x * x * x), ek));
            } else {
                const double lx = log(x);
                const double lq = bor * (1.0 - exp(r * lx));
                psi = 2.0 * exp(b * lx + lq);
                // the reference's inf / NaN where a factor overflows (morse_special; ln thresholds)
                double sp;
                if (morse_special<double>(b * lx, lq, 709.782712893384, -744.4400719213812, -745.1332191019412, &sp))
                    psi = sp;
            }
        } else if constexpr (KIND == NW_MORLET) {
            const double nu = (double)(int64_t)j * delta;
            const double x = nu / f * peak;
            const double a = sigma - x;
            psi = cpi * (exp(-(a * a) / 2.0) - kappa * exp(-(x * x) / 2.0));
        } else {
            const double nu = (double)(int64_t)j * delta;
            psi = nu <= 1.0 ? 1.0 : 0.0;
        }
        return psi * scale;
    }
};

// the recurrence state of a row's W evaluation (kMorseRec), or nothing
template <typename T, int KIND> struct RowRec { struct type {}; };
template <> struct RowRec<double, kMorseRec> { using type = RowW<double, kMorseRec>::Rec; };

// ---- pass 1: rows
// fp32 E = 32 rows: pruned Xt rows by LDS-DMA ahead of the stores (C5 50.6 -> 48.5 ms per step);
// analytic kinds only (table rows' wavelet_bin loads would exceed 128 VGPRs, as in nw_fused);
// fp64 rows with the same DMA measured no faster (0.94 -> 0.98 ms per launch; round 5, after the
// W-evaluator changes: rows -0.5 %, step +1.4 %, profiles/r05_c5f64_rows_xd_ab.txt)
// (fp64 rows with the DMA, re-measured in round 4 beside the fast Morse form: no gain either,
// profiles/r04_c5f64_rows_ab.txt)
// NW_ABL_ROWS_STREAM (diagnostic, wrong results): the row pass as a pure stream -- the pass-0
// Xt loads (global, no LDS-DMA) and the last pass's B stores at the product's addresses and
// widths, without W, FFT arithmetic or exchanges: the floor of its write stream
#ifdef NW_ABL_ROWS_STREAM
constexpr bool kRowsStream = true;
#else
constexpr bool kRowsStream = false;
#endif
template <typename T, int E, int KIND>
constexpr bool kRowsXD = sizeof(T) == 4 && E >= 32 && KIND != NW_TABLE && !kRowsStream;
// 4 waves/SIMD; fp64: 2 (twice the registers per element, as nw_fused)
template <typename T, int N2, int E, int KIND>
__global__ __launch_bounds__(N2 / E, sizeof(T) == 8 ? 2 : 4) void rows_kernel(
    WDesc d, int f0, int nf, int n1, int rgs, const C2<T>* __restrict__ Xt, C2<T>* __restrict__ B,
    const int* __restrict__ kmax, const C2<T>* __restrict__ tw) {
    using G = Geometry<N2, E>;
    extern __shared__ __align__(16) unsigned char smem[];
    T* lds = reinterpret_cast<T*>(smem);
    const int t = threadIdx.x;

    // XCD-aware block -> (scale, row group), as nw_fused_kernel: blocks b, b+8, ... share
    // an XCD, whose resident blocks cover kRowTileF scales x kRowTileG row groups, so each
    // Xt row group is read from HBM once per tile and then from that XCD's L2
    const int b = blockIdx.x;
    const int xcd = b & 7;
    const int local = b >> 3;
    const int pos = local % (kRowTileF * kRowTileG);
    const int round = local / (kRowTileF * kRowTileG);
    const int nfr = (nf + kRowTileF - 1) / kRowTileF;
    const int fl = (round % nfr) * kRowTileF + pos % kRowTileF;
    const int rg = ((round / nfr) * kRowTileG + pos / kRowTileF) * 8 + xcd;
    const int ngroups = n1 / rgs;
    if (fl >= nf || rg >= ngroups) return;
    const int fi = f0 + fl;
    const int km = kmax[fi];
    NW_DCHECK(fi < d.nfreq && (rg + 1) * rgs <= n1 && (int64_t)n1 * N2 == d.n && km < d.n);
    RowW<T, KIND> wf;
    if constexpr (KIND != NW_TABLE) wf.init(d, fi);
    if constexpr (sizeof(T) == 8 && KIND == kMorseRec) wf.init_rec(n1 * G::T);

    Tab1<T, N2, E>::fill(lds, tw, t);
    TwSplit<T, N2, E>::fill(lds, tw, t);
    if constexpr (TwSplit<T, N2, E>::ON) lds_barrier();   // read before the first exchange
    C2<T> x[E];
    // bins k = k1 + n1*k2 with k2 = t + r*T: elements r >= need are zero for every thread;
    // pass 0 runs the variant NZ = nzv(need) elements
    auto need_of = [&](int k1) { return km < k1 ? 1 : (km - k1) / n1 / G::T + 1; };
    // pass-0 variants in steps of 4 elements at fp32 E = 32 (fp64: 4, 8, 16, 24, E)
    constexpr bool FINE = E > 16 && sizeof(T) == 4 && KIND != NW_TABLE;   // table rows: more scratch
    auto nzv_of = [](int need) {
        return need <= 4 ? 4 : need <= 8 ? 8 : (FINE && need <= 12) ? 12 : (E > 16 && need <= 16) ? 16
             : (FINE && need <= 20) ? 20 : (E > 16 && need <= 24) ? 24 : E;
    };
    // XD: a row whose pass 0 reads only Xt[k1][0 .. N2/2) (NZ <= E/2) gets those bins by
    // LDS-DMA into the idle image, issued BEFORE the previous row's stores (as nw_fused's
    // next-signal X): global loads issued after the stores would wait for all of them in
    // the in-order vmcnt queue
    constexpr bool XD = kRowsXD<T, E, KIND>;
    const int k1_begin = rg * rgs, k1_end = (rg + 1) * rgs;
    bool in_lds = false;
    if constexpr (XD) {
        const int nz0 = nzv_of(need_of(k1_begin));
        if (nz0 <= E / 2) {
            dma_x<T, N2, G::T>(Xt + (int64_t)k1_begin * N2, lds, t, dma_rounds_for<T>(nz0));
            in_lds = true;
        }
    }
    for (int k1 = k1_begin; k1 < k1_end; ++k1) {
        const int need = need_of(k1);
        const C2<T>* xrow = Xt + (int64_t)k1 * N2;
        const uint32_t xo = (uint32_t)t * (uint32_t)sizeof(C2<T>);
        C2<T> v[E];
        if constexpr (XD) {
            if (in_lds) {
                // this wave's DMA landed (only the stores issued after it may be pending), then every wave's
                if (k1 == k1_begin) wait_vmcnt<0>(); else wait_vmcnt<LastStores<T, N2, E, NW_OUT_CWT>::COUNT>();
                lds_barrier();
            }
        }
        auto pass0 = [&]<int NZ, bool FROM_LDS>() {
            int j0 = k1 + n1 * t;                  // bin k of element 0 (k2 = t)
            if constexpr (KIND != NW_TABLE) j0 -= wf.off;
            asm volatile("" : "+v"(j0));
            int tl = t;                            // opaque here: LDS reads must not hoist above the dispatch
            asm volatile("" : "+v"(tl));
            const C2<T>* xl = reinterpret_cast<const C2<T>*>(lds);
            [[maybe_unused]] typename RowRec<T, KIND>::type rec{};
#pragma unroll
            for (int r = 0; r < E; ++r) {
                if (r < NZ) {
                    C2<T> xv;
                    if constexpr (FROM_LDS) xv = xl[tl + r * G::T];
                    else xv = *at(xrow, xo, (uint32_t)(r * G::T * sizeof(C2<T>)));
                    const int j = j0 + r * n1 * G::T;
                    if constexpr (sizeof(T) == 8 && KIND == kMorseRec) {
                        if (r % RowW<T, KIND>::kRecGroup == 0) rec = wf.start(j);
                        const T w = wf.step(j, rec);
                        v[r] = C2<T>{w * xv.re, w * xv.im};
                        if (r % 4 == 3) __builtin_amdgcn_sched_barrier(0);
                    } else if constexpr (KIND == NW_TABLE) {
                        const cplx<T> w = wavelet_bin<T>(d, fi, (int64_t)j);
                        v[r] = cmul(C2<T>{w.re, w.im}, xv);
                    } else {
#if defined(NW_ABL_ROWS_NOW)
                        const T w = (T)(j & 1);
#elif defined(NW_ABL_ROWS_STREAM)
                        (void)j;
                        const T w = T(1);
#else
                        const T w = wf(j);
#endif
                        v[r] = C2<T>{w * xv.re, w * xv.im};
                        // fp64 W: at most 4 evaluations in flight (they hold ~12 VGPRs each)
                        if constexpr (sizeof(T) == 8 && (KIND == NW_MORSE || KIND == kMorseFast || KIND == kMorseFast35))
                            if (r % 4 == 3) __builtin_amdgcn_sched_barrier(0);
                    }
                } else {
                    v[r] = C2<T>{T(0), T(0)};
                }
            }
            if constexpr (!kRowsStream) idft_br<T, E, NZ>(v);
        };
        if (XD && in_lds) {
            if (need <= 4) pass0.template operator()<4, XD>();
            else if (need <= 8) pass0.template operator()<8, XD>();
            else if (FINE && need <= 12) pass0.template operator()<(FINE ? 12 : E), XD>();
            else pass0.template operator()<(E > 16 ? 16 : E), XD>();
        } else {
            if (need <= 4) pass0.template operator()<4, false>();
            else if (need <= 8) pass0.template operator()<8, false>();
            else if (FINE && need <= 12) pass0.template operator()<(FINE ? 12 : E), false>();
            else if (E > 16 && need <= 16) pass0.template operator()<(E > 16 ? 16 : E), false>();
            else if (FINE && need <= 20) pass0.template operator()<(FINE ? 20 : E), false>();
            else if (E > 16 && need <= 24) pass0.template operator()<(E > 16 ? 24 : E), false>();
            else pass0.template operator()<E, false>();
        }
        void* orow = B + ((int64_t)fl * n1 + k1) * N2;
        const C2<T>* xs_next = nullptr;
        int rounds_next = 0;
        if constexpr (XD) {
            if (k1 + 1 < k1_end) {
                const int nzn = nzv_of(need_of(k1 + 1));
                if (nzn <= E / 2) {
                    xs_next = Xt + (int64_t)(k1 + 1) * N2;
                    rounds_next = dma_rounds_for<T>(nzn);
                }
            }
            in_lds = xs_next != nullptr;
        }
        // B rows stored nt (fp64: the 16-B complex128 stores; plain ones made the C5 fp64 step
        // 129.4 ms against 125.3)
#if defined(NW_ABL_ROWS_STREAM)
        (void)x;
        (void)rounds_next;
        LastStores<T, N2, E, NW_OUT_CWT, kStoreGlobalNt>::all(v, orow, t);
#elif defined(NW_B_PLAIN)   // diagnostic: B with plain stores (kept in the Infinity Cache when it fits)
        passes_from<T, N2, E, NW_OUT_CWT, 1, XD, kStoreGlobal>(v, lds, t, tw, x, xs_next, orow, nullptr, nullptr, rounds_next);
#else
        passes_from<T, N2, E, NW_OUT_CWT, 1, XD, kStoreGlobalNt>(v, lds, t, tw, x, xs_next, orow, nullptr, nullptr, rounds_next);
#endif
    }
}

// ---- pass 2: columns.  Thread t owns column c = t % C of the workgroup's C columns and
// butterflies u + q*U (U = N1/E threads per column).  The exchange image is
// [position][column] (position-major, C reals per position), one real component at a
// time: 32-lane groups cover >= 16 consecutive columns (fp32), so reads are conflict-free
// and writes at most 2-way (free for ds_write_b32, MI355X_MICROARCH.md §LDS); fp64 lanes
// read 8 B each, so C >= 8 columns keep a 32-lane group on consecutive positions.
// NW_ABL_COLS_STREAM (diagnostic, wrong results): the column kernels as a pure stream -- the
// pass-0 B loads and the last pass's y stores at exactly the product's addresses and widths,
// with no twiddles, FFT arithmetic or LDS exchanges between them: the floor the column pass's
// access pattern alone reaches (tools/ab.sh next to the product)
#ifdef NW_ABL_COLS_STREAM
#ifndef NW_ABL_COLS_NOFFT
#define NW_ABL_COLS_NOFFT
#endif
#ifndef NW_ABL_COLS_NOTW
#define NW_ABL_COLS_NOTW
#endif
#endif
template <typename T, int N1> struct Cols {
    static constexpr int E = kColE<T>;
    static constexpr int U = N1 / E;                 // threads per column
    static constexpr int C = kColThreads<T> / U;     // columns per workgroup
    using G = Geometry<N1, E>;
    static_assert(N1 >= 32 && C >= (sizeof(T) == 4 ? 16 : 4), "cols geometry");
};

template <typename T, int N1, int P, int COMP>
__device__ __forceinline__ void col_write(C2<T>* v, T* lds, int u, int c) {
    using CL = Cols<T, N1>;
    using G = typename CL::G;
    constexpr int C = CL::C, U = CL::U;
    constexpr int R = G::radix(P), NS = G::ns(P), Q = CL::E / R;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int j = u + q * U;
        T* dst = lds + ((j / NS) * NS * R + j % NS) * C + c;
#pragma unroll
        for (int i = 0; i < R; ++i) dst[bitrev<R>(i) * NS * C] = comp<COMP>(v[q * R + i]);
    }
}

template <typename T, int N1, int P, int COMP>
__device__ __forceinline__ void col_read(C2<T>* v, const T* lds, int u, int c) {
    using CL = Cols<T, N1>;
    using G = typename CL::G;
    constexpr int C = CL::C, U = CL::U;
    constexpr int R = G::radix(P), Q = CL::E / R, STRIDE = N1 / R;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const T* src = lds + (u + q * U) * C + c;
#pragma unroll
        for (int r = 0; r < R; ++r) comp<COMP>(v[q * R + r]) = src[r * STRIDE * C];
    }
}

// tw1: fp64 only, the exact length-N1 table exp(+2 pi i j / N1) (fp32 twiddles come from
// v_sin / v_cos)
template <typename T, int N1, int N2, int OUT, int P>
__device__ __forceinline__ void col_passes(C2<T>* v, T* lds, int u, int c, void* orow, uint32_t lane_off,
                                           const C2<T>* __restrict__ tw1) {
    using CL = Cols<T, N1>;
    using G = typename CL::G;
    constexpr int U = CL::U;
    constexpr int R = G::radix(P), NS = G::ns(P), Q = CL::E / R;
#ifdef NW_ABL_COLS_NOFFT
    if constexpr (false) {
#else
    if constexpr (P > 0) {
#endif
        constexpr int LR = ilog2<R>();
        lds_barrier();
        col_write<T, N1, P - 1, 0>(v, lds, u, c);
        lds_barrier();
        col_read<T, N1, P, 0>(v, lds, u, c);
        lds_barrier();
        col_write<T, N1, P - 1, 1>(v, lds, u, c);
        lds_barrier();
        col_read<T, N1, P, 1>(v, lds, u, c);
        // twiddles after the exchange (no stores are in flight here): bases of one
        // butterfly at a time, so they never sit live across the exchange
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            C2<T> pb[LR > 0 ? LR : 1];
            twiddle_bases<T, R, N1, NS * R>(pb, (u + q * U) % NS, tw1);
            twiddle_apply<T, R>(v + q * R, pb);
            idft_br<T, R>(v + q * R);
        }
    }
    if constexpr (P + 1 < G::npass()) {
        col_passes<T, N1, N2, OUT, P + 1>(v, lds, u, c, orow, lane_off, tw1);
    } else {
        // v[q*R + i] is y at n1 = (j / NS) * NS * R + j % NS + bitrev(i) * NS, j = u + q*U.
        // The last pass has N1 / R = NS butterflies, so j < NS and n1 = u + q*U + bitrev(i)*NS:
        // every store is the lane offset (col + u * N2) plus a compile-time offset
        using O = typename OutT<OUT, T>::type;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const uint32_t cn1 = (uint32_t)(q * U + bitrev<R>(i) * NS);
                const O val = out_value<OUT, T>(v[q * R + i]);
                O* dst = at(reinterpret_cast<O*>(orow), lane_off, cn1 * (uint32_t)N2 * (uint32_t)sizeof(O));
#ifdef NW_ABL_COLS_NOSTORE
                if constexpr (OUT == NW_OUT_CWT) asm volatile("" ::"v"(val.re), "v"(val.im), "v"(dst));
                else asm volatile("" ::"v"(val), "v"(dst));
                continue;
#endif
                if constexpr (OUT == NW_OUT_CWT) {
                    using V2 = T __attribute__((ext_vector_type(2)));
                    __builtin_nontemporal_store(__builtin_bit_cast(V2, val), reinterpret_cast<V2*>(dst));
                } else {
                    __builtin_nontemporal_store(val, dst);
                }
            }
        }
    }
}

// fp64 pass-0 twiddles w_n^m (m = n2 k1 < n) as the product of two exact entries:
// tsplit[m & 4095] = w_n^(m mod 4096) and tsplit[4096 + (m >> 12)] = w_n^(4096 (m >> 12))
constexpr int kSplitLo = 4096;
constexpr int kSplitEntries = 2 * kSplitLo;   // n <= 2^24: m >> 12 < 4096

template <typename T, int N1, int N2, int OUT>
#ifdef NW_COLS64_E16
__global__ __launch_bounds__(kColThreads<T>, sizeof(T) == 8 ? 2 : 4) void cols_kernel(
#else
__global__ __launch_bounds__(kColThreads<T>, sizeof(T) == 8 ? 1 : 4) void cols_kernel(
#endif
    int f0, int nf, const C2<T>* __restrict__ B, void* __restrict__ out, const C2<T>* __restrict__ tw1,
    const C2<T>* __restrict__ tsplit) {
    using CL = Cols<T, N1>;
    constexpr int C = CL::C, U = CL::U, E = CL::E;
    constexpr int64_t n = (int64_t)N1 * N2;
    extern __shared__ __align__(16) unsigned char smem[];
    T* lds = reinterpret_cast<T*>(smem);
    const int t = threadIdx.x;
    const int c = t % C, u = t / C;
    constexpr int ngroups = N2 / C;
    const int fl = blockIdx.x / ngroups;
    const int cg = blockIdx.x % ngroups;
    if (fl >= nf) return;
    const int col = cg * C + c;                      // n2
    // B[fl] (uniform base) + 32-bit lane offsets: (k1 * N2 + col) * 16 < n * 16 <= 2^28
    const C2<T>* bf = B + (int64_t)fl * n;
    const uint32_t boff = ((uint32_t)u * N2 + (uint32_t)col) * (uint32_t)sizeof(C2<T>);

    // pass 0: v[r] = B[k1][n2] * w_n^(n2 k1), k1 = u + U r (radix E, Ns = 1)
    C2<T> v[E];
    // fp64: w_n^(n2 u) and w_n^(n2 U) from the exact split tables (4 loads per thread), the
    // E powers by repeated multiplication (<= E ulp of drift, far inside 1e-12)
    C2<T> wr{T(1), T(0)}, wstep{T(1), T(0)};
    if constexpr (sizeof(T) == 8) {
        auto wpow = [&](uint32_t m) {
            const C2<T> wl = *at(tsplit, (m & (kSplitLo - 1)) * (uint32_t)sizeof(C2<T>));
            const C2<T> wh = *at(tsplit, (kSplitLo + (m >> 12)) * (uint32_t)sizeof(C2<T>));
            return cmul(wh, wl);
        };
        wr = wpow((uint32_t)col * (uint32_t)u);
        wstep = wpow((uint32_t)col * (uint32_t)U);
    }
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int k1 = u + U * r;
        const C2<T> bv = *at(bf, boff, (uint32_t)(U * r * N2 * sizeof(C2<T>)));
        const uint32_t m = (uint32_t)col * (uint32_t)k1;                      // n2 k1 < n <= 2^24
#ifdef NW_ABL_COLS_NOTW
        (void)m;
        v[r] = bv;
#else
        if constexpr (sizeof(T) == 4) {
            constexpr float inv_n = 1.0f / (float)n;                          // exact: power of two
            const float rev = (float)m * inv_n;                               // exact: m < 2^24
            const C2<float> w{__builtin_amdgcn_cosf(rev), __builtin_amdgcn_sinf(rev)};
            v[r] = cmul(bv, w);
        } else {
            (void)m;
            v[r] = cmul(bv, wr);
            if (r + 1 < E) wr = cmul(wr, wstep);
        }
#endif
    }
#ifdef NW_ABL_COLS_NOFFT
#pragma unroll
    for (int i = 0; i < E; ++i) asm volatile("" : "+v"(v[i].re), "+v"(v[i].im));
#else
    idft_br<T, E>(v);
#endif
    using O = typename OutT<OUT, T>::type;
    void* orow = reinterpret_cast<char*>(out) + (int64_t)(f0 + fl) * n * (int64_t)sizeof(O);
    const uint32_t ooff = ((uint32_t)col + (uint32_t)u * N2) * (uint32_t)sizeof(O);
    col_passes<T, N1, N2, OUT, 0>(v, lds, u, c, orow, ooff, tw1);
}

// ---- fp32 column pass on column PAIRS: thread (cp, u) owns the adjacent columns 2cp, 2cp+1
// and E2 = 16 elements k1 = u + U2 r of each, every lane value a C2<f2> holding the two columns
// (signal-pair technique of nw_fused_pair_kernel): B is read and y written 16 B per lane
// (two complex64) instead of 8, every butterfly / twiddle / LDS access serves both columns
// (v_pk_* math, 8-B image slots [position][pair]), the same C = 2 CP columns per 1024-thread
// workgroup and 256-B runs.  Length-N1 transforms at E = 16 take one exchange more than E = 32.
// (E = 32 with 512-thread workgroups: one exchange instead of two, 198 VGPRs at 2 waves/SIMD:
// C5 cols 3.92 -> 3.95 ms per launch, not kept; profiles/r04_c5_colpairs_ab.txt)
template <int N1> struct ColsP {
    static constexpr int E = 16;
    static constexpr int THREADS = 1024;
    static constexpr int U = N1 / E;                 // threads per column pair
    static constexpr int CP = THREADS / U;           // column pairs per workgroup
    static constexpr int C = 2 * CP;
    using G = Geometry<N1, E>;
    static_assert(N1 >= 32 && CP >= 16, "column-pair geometry");
};

template <int N1, int P, int COMP>
__device__ __forceinline__ void colp_write(C2<f2>* v, f2* lds, int u, int cp) {
    using CL = ColsP<N1>;
    using G = typename CL::G;
    constexpr int CP = CL::CP, U = CL::U;
    constexpr int R = G::radix(P), NS = G::ns(P), Q = CL::E / R;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int j = u + q * U;
        f2* dst = lds + ((j / NS) * NS * R + j % NS) * CP + cp;
#pragma unroll
        for (int i = 0; i < R; ++i) dst[bitrev<R>(i) * NS * CP] = comp<COMP>(v[q * R + i]);
    }
}

template <int N1, int P, int COMP>
__device__ __forceinline__ void colp_read(C2<f2>* v, const f2* lds, int u, int cp) {
    using CL = ColsP<N1>;
    using G = typename CL::G;
    constexpr int CP = CL::CP, U = CL::U;
    constexpr int R = G::radix(P), Q = CL::E / R, STRIDE = N1 / R;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const f2* src = lds + (u + q * U) * CP + cp;
#pragma unroll
        for (int r = 0; r < R; ++r) comp<COMP>(v[q * R + r]) = src[r * STRIDE * CP];
    }
}

template <int N1, int N2, int OUT, int P>
__device__ __forceinline__ void colp_passes(C2<f2>* v, f2* lds, int u, int cp, void* orow, uint32_t lane_off) {
    using CL = ColsP<N1>;
    using G = typename CL::G;
    constexpr int U = CL::U;
    constexpr int R = G::radix(P), NS = G::ns(P), Q = CL::E / R;
#ifdef NW_ABL_COLS_STREAM
    if constexpr (false) {
#else
    if constexpr (P > 0) {
#endif
        constexpr int LR = ilog2<R>();
        lds_barrier();
        colp_write<N1, P - 1, 0>(v, lds, u, cp);
        lds_barrier();
        colp_read<N1, P, 0>(v, lds, u, cp);
        lds_barrier();
        colp_write<N1, P - 1, 1>(v, lds, u, cp);
        lds_barrier();
        colp_read<N1, P, 1>(v, lds, u, cp);
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            C2<float> pb[LR > 0 ? LR : 1];                  // shared by the two columns
            twiddle_bases<float, R, N1, NS * R>(pb, (u + q * U) % NS, nullptr);
            twiddle_apply<f2, R>(v + q * R, pb);
            idft_br<f2, R>(v + q * R);
        }
    }
    if constexpr (P + 1 < G::npass()) {
        colp_passes<N1, N2, OUT, P + 1>(v, lds, u, cp, orow, lane_off);
    } else {
        // v[q*R + i] is y at n1 = u + q*U + bitrev(i)*NS (the last pass has NS butterflies)
        using O = typename OutT<OUT, float>::type;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const uint32_t cn1 = (uint32_t)(q * U + bitrev<R>(i) * NS);
                const C2<f2> y = v[q * R + i];
                O* dst = at(reinterpret_cast<O*>(orow), lane_off, cn1 * (uint32_t)N2 * (uint32_t)sizeof(O));
                if constexpr (OUT == NW_OUT_CWT) {
                    using V4 = float __attribute__((ext_vector_type(4)));
                    __builtin_nontemporal_store(V4{y.re.x, y.im.x, y.re.y, y.im.y}, reinterpret_cast<V4*>(dst));
                } else {
                    const f2 o{out_value<OUT, float>(C2<float>{y.re.x, y.im.x}),
                               out_value<OUT, float>(C2<float>{y.re.y, y.im.y})};
                    __builtin_nontemporal_store(o, reinterpret_cast<f2*>(dst));
                }
            }
        }
    }
}

template <int N1, int N2, int OUT>
__global__ __launch_bounds__(ColsP<N1>::THREADS, ColsP<N1>::THREADS / 256) void cols_kernel(int f0, int nf, const C2<float>* __restrict__ B,
                                                       void* __restrict__ out) {
    using CL = ColsP<N1>;
    constexpr int CP = CL::CP, C = CL::C, U = CL::U, E = CL::E;
    constexpr int64_t n = (int64_t)N1 * N2;
    extern __shared__ __align__(16) unsigned char smem[];
    f2* lds = reinterpret_cast<f2*>(smem);
    const int t = threadIdx.x;
    const int cp = t % CP, u = t / CP;
    constexpr int ngroups = N2 / C;
    const int fl = blockIdx.x / ngroups;
    const int cg = blockIdx.x % ngroups;
    if (fl >= nf) return;
    const int col = cg * C + 2 * cp;                 // n2 of the pair's first column
    const C2<float>* bf = B + (int64_t)fl * n;
    const uint32_t boff = ((uint32_t)u * N2 + (uint32_t)col) * (uint32_t)sizeof(C2<float>);
    // pass 0: v[r] = B[k1][n2 .. n2+1] * w_n^(n2 k1), k1 = u + U r
    C2<f2> v[E];
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int k1 = u + U * r;
        using V4 = float __attribute__((ext_vector_type(4)));
        const V4 b4 = *reinterpret_cast<const V4*>(at(bf, boff, (uint32_t)(U * r * N2 * sizeof(C2<float>))));
#ifdef NW_ABL_COLS_STREAM
        (void)k1;
        v[r] = C2<f2>{f2{b4.x, b4.z}, f2{b4.y, b4.w}};
#else
        const uint32_t m0 = (uint32_t)col * (uint32_t)k1;                 // n2 k1 < n <= 2^24
        constexpr float inv_n = 1.0f / (float)n;                          // exact: power of two
        const float r0 = (float)m0 * inv_n, r1 = (float)(m0 + (uint32_t)k1) * inv_n;
        const C2<f2> w{f2{__builtin_amdgcn_cosf(r0), __builtin_amdgcn_cosf(r1)},
                       f2{__builtin_amdgcn_sinf(r0), __builtin_amdgcn_sinf(r1)}};
        v[r] = cmul(C2<f2>{f2{b4.x, b4.z}, f2{b4.y, b4.w}}, w);
#endif
    }
#ifndef NW_ABL_COLS_STREAM
    idft_br<f2, E>(v);
#endif
    using O = typename OutT<OUT, float>::type;
    void* orow = reinterpret_cast<char*>(out) + (int64_t)(f0 + fl) * n * (int64_t)sizeof(O);
    const uint32_t ooff = ((uint32_t)col + (uint32_t)u * N2) * (uint32_t)sizeof(O);
    colp_passes<N1, N2, OUT, 0>(v, lds, u, cp, orow, ooff);
}

// tsplit for one n (fp64 column pass), from sincospi in fp64
__global__ __launch_bounds__(256) void tsplit_kernel(C2<double>* ts, int64_t n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= kSplitEntries) return;
    const int64_t m = i < kSplitLo ? i : (int64_t)(i - kSplitLo) * kSplitLo;
    double s, c;
    sincospi(2.0 * (double)(m % n) / (double)n, &s, &c);
    ts[i] = C2<double>{c, s};
}

template <typename T, int N2, int E, int KIND>
hipError_t launch_row_pass(const WDesc& d, int f0, int nf, int n1, const C2<T>* Xt, C2<T>* B, const int* kmax,
                           hipStream_t s) {
    void* tw = nullptr;
    hipError_t e = fused_twiddles(N2, sizeof(T) == 4 ? NW_F32 : NW_F64, &tw);
    if (e != hipSuccess) return e;
    const int lds = kLdsBytes<T, N2, E>;
    e = hipFuncSetAttribute((const void*)rows_kernel<T, N2, E, KIND>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    const int rgs = nf < kRowTileF ? 1 : kRowGroup;   // few scales: one row per block, more blocks
    const int ngroups = n1 / rgs;
    const int gpad = (ngroups + 8 * kRowTileG - 1) / (8 * kRowTileG) * (8 * kRowTileG);
    const int nfr = (nf + kRowTileF - 1) / kRowTileF;
    const int64_t blocks = (int64_t)gpad * nfr * kRowTileF;
    nw_launch(rows_kernel<T, N2, E, KIND>, (unsigned)blocks, N2 / E, lds, s, d, f0, nf, n1, rgs, Xt, B, kmax,
                                                                       reinterpret_cast<const C2<T>*>(tw));
    return hipGetLastError();
}

// fp32: the column-pair kernel (C5 cols 4.02 -> 3.86 ms per 64-scale launch against the
// single-column kernel, which fp64 keeps: its lanes already read and write 16 B)
constexpr bool kColsPair = true;
template <typename T, int N1, int N2>
hipError_t launch_cols(int out_kind, int f0, int nf, const C2<T>* B, void* out, const C2<T>* tsplit, hipStream_t s) {
    if constexpr (sizeof(T) == 4 && kColsPair && ColsP<N1>::CP >= 16 && N2 % ColsP<N1>::C == 0) {
        using CL = ColsP<N1>;
        const int lds = N1 * CL::C * (int)sizeof(float);
        const int64_t blocks = (int64_t)nf * (N2 / CL::C);
        const void* fn = out_kind == NW_OUT_CWT     ? (const void*)cols_kernel<N1, N2, NW_OUT_CWT>
                         : out_kind == NW_OUT_POWER ? (const void*)cols_kernel<N1, N2, NW_OUT_POWER>
                                                    : (const void*)cols_kernel<N1, N2, NW_OUT_ABS>;
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return e;
        if (out_kind == NW_OUT_CWT)
            nw_launch(cols_kernel<N1, N2, NW_OUT_CWT>, (unsigned)blocks, CL::THREADS, lds, s, f0, nf, B, out);
        else if (out_kind == NW_OUT_POWER)
            nw_launch(cols_kernel<N1, N2, NW_OUT_POWER>, (unsigned)blocks, CL::THREADS, lds, s, f0, nf, B, out);
        else
            nw_launch(cols_kernel<N1, N2, NW_OUT_ABS>, (unsigned)blocks, CL::THREADS, lds, s, f0, nf, B, out);
        return hipGetLastError();
    }
    using CL = Cols<T, N1>;
    const int lds = N1 * CL::C * (int)sizeof(T);
    const int64_t blocks = (int64_t)nf * (N2 / CL::C);
    static_assert(N2 % CL::C == 0, "column groups");
    const C2<T>* tw1 = nullptr;
    if constexpr (sizeof(T) == 8) {
        void* tw = nullptr;
        hipError_t e = fused_twiddles(N1, NW_F64, &tw);
        if (e != hipSuccess) return e;
        tw1 = reinterpret_cast<const C2<T>*>(tw);
    }
    const void* fn = out_kind == NW_OUT_CWT     ? (const void*)cols_kernel<T, N1, N2, NW_OUT_CWT>
                     : out_kind == NW_OUT_POWER ? (const void*)cols_kernel<T, N1, N2, NW_OUT_POWER>
                                                : (const void*)cols_kernel<T, N1, N2, NW_OUT_ABS>;
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    if (out_kind == NW_OUT_CWT)
        nw_launch(cols_kernel<T, N1, N2, NW_OUT_CWT>, (unsigned)blocks, kColThreads<T>, lds, s, f0, nf, B, out, tw1, tsplit);
    else if (out_kind == NW_OUT_POWER)
        nw_launch(cols_kernel<T, N1, N2, NW_OUT_POWER>, (unsigned)blocks, kColThreads<T>, lds, s, f0, nf, B, out, tw1, tsplit);
    else
        nw_launch(cols_kernel<T, N1, N2, NW_OUT_ABS>, (unsigned)blocks, kColThreads<T>, lds, s, f0, nf, B, out, tw1, tsplit);
    return hipGetLastError();
}

// n = N1 * N2: N2 = min(n / 32, 16384 (fp32) or 8192 (fp64)), N1 = n / N2 >= 32
struct Split {
    int n1, n2;
};
Split split_of(int64_t n, int dtype) {
    const int64_t maxn2 = dtype == NW_F32 ? kMaxN2<float> : kMaxN2<double>;
    const int64_t n1 = n / maxn2 > 32 ? n / maxn2 : 32;
    return {(int)n1, (int)(n / n1)};
}

size_t cplx_bytes(int dtype) { return dtype == NW_F32 ? sizeof(C2<float>) : sizeof(C2<double>); }

int64_t fchunk_of(int64_t n, int nfreq, int dtype) {
    const int64_t per = n * (int64_t)cplx_bytes(dtype);
    int64_t fc = (int64_t)(kBBudget / (size_t)per);
    if (const char* e = std::getenv("NW_LARGE_FCHUNK")) fc = std::atoll(e);   // diagnostics
    if (fc < 1) fc = 1;
    return fc < nfreq ? fc : nfreq;
}

// support buffer: kmax[nfreq] (padded to 256 B), then the fp64 split twiddles
// support buffer: kmax (int) | row maxima (u64) | tsplit (fp64)
size_t wmax_offset(int nfreq) { return ((size_t)nfreq * sizeof(int) + 255) / 256 * 256; }
size_t tsplit_offset(int nfreq) { return wmax_offset(nfreq) + ((size_t)nfreq * sizeof(uint64_t) + 255) / 256 * 256; }

}  // namespace

bool large_supported(int64_t n, int dtype) {
    return (dtype == NW_F32 || dtype == NW_F64) && n >= (int64_t(1) << 15) && n <= (int64_t(1) << 24) &&
           !(n & (n - 1));
}

size_t large_scratch_bytes(int64_t n, int nfreq, int dtype) {
    const size_t per = (size_t)n * cplx_bytes(dtype);
    return per + (size_t)fchunk_of(n, nfreq, dtype) * per;   // Xt + B
}

size_t large_support_bytes(int nfreq) { return tsplit_offset(nfreq) + kSplitEntries * sizeof(C2<double>); }

// kmax[] and wmax[] of every row into `support`: the analytic kinds by support_fast_kernel,
// the others (or scan = true: the full-scan reference the tests compare it with) by
// wmax_kernel + kmax_kernel over every bin
hipError_t large_row_support(const WDesc& d, int dtype, void* support, bool scan, hipStream_t s) {
    int* kmax = reinterpret_cast<int*>(support);
    auto* wmax = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(support) + wmax_offset(d.nfreq));
    hipError_t e = hipMemsetAsync(kmax, 0xFF, (size_t)d.nfreq * sizeof(int), s);   // -1
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(wmax, 0, (size_t)d.nfreq * sizeof(uint64_t), s);            // +0.0
    if (e != hipSuccess) return e;
    if (!scan && support_fast_ok(d, dtype)) {
        if (dtype == NW_F32) nw_launch(support_fast_kernel<float>, d.nfreq, kFastThreads, 0, s, d, kmax, wmax);
        else nw_launch(support_fast_kernel<double>, d.nfreq, kFastThreads, 0, s, d, kmax, wmax);
        return hipGetLastError();
    }
    const int64_t per_block = 256 * kSupBins;
    dim3 grid((unsigned)((d.n + per_block - 1) / per_block), (unsigned)d.nfreq);
    const bool realw = d.kind != NW_TABLE;
    if (dtype == NW_F32) {
        if (realw) nw_launch(wmax_kernel<float, true>, grid, 256, 0, s, d, wmax);
        else nw_launch(wmax_kernel<float, false>, grid, 256, 0, s, d, wmax);
        if (realw) nw_launch(kmax_kernel<float, true>, grid, 256, 0, s, d, kmax, wmax);
        else nw_launch(kmax_kernel<float, false>, grid, 256, 0, s, d, kmax, wmax);
    } else {
        if (realw) nw_launch(wmax_kernel<double, true>, grid, 256, 0, s, d, wmax);
        else nw_launch(wmax_kernel<double, false>, grid, 256, 0, s, d, wmax);
        if (realw) nw_launch(kmax_kernel<double, true>, grid, 256, 0, s, d, kmax, wmax);
        else nw_launch(kmax_kernel<double, false>, grid, 256, 0, s, d, kmax, wmax);
    }
    return hipGetLastError();
}

hipError_t build_large_support(const WDesc& d, int dtype, void* support, hipStream_t s) {
    // NW_SUPPORT_SCAN=1: every row by the full scan (diagnostic A/B)
    static const bool force_scan = [] {
        const char* v = std::getenv("NW_SUPPORT_SCAN");
        return v && v[0] == '1';
    }();
    hipError_t e = large_row_support(d, dtype, support, force_scan, s);
    if (e != hipSuccess) return e;
    if (dtype == NW_F64) {
        nw_launch(tsplit_kernel, kSplitEntries / 256, 256, 0, s, 
            reinterpret_cast<C2<double>*>(reinterpret_cast<char*>(support) + tsplit_offset(d.nfreq)), d.n);
    }
    return hipGetLastError();
}

int64_t large_fchunk(int64_t n, int nfreq, int dtype) { return fchunk_of(n, nfreq, dtype); }

// Xt of one signal (X: its R2C half spectrum) into the scratch's first n complex
hipError_t large_transpose(const WDesc& d, int dtype, const void* X, void* scratch, hipStream_t s) {
    const Split sp = split_of(d.n, dtype);
    const dim3 grid((unsigned)(sp.n1 / 32), (unsigned)(sp.n2 / 32));
    if (dtype == NW_F32)
        nw_launch(xt_kernel<float>, grid, 256, 0, s, d, reinterpret_cast<const cplx<float>*>(X),
                                              reinterpret_cast<C2<float>*>(scratch), sp.n1, sp.n2);
    else
        nw_launch(xt_kernel<double>, grid, 256, 0, s, d, reinterpret_cast<const cplx<double>*>(X),
                                               reinterpret_cast<C2<double>*>(scratch), sp.n1, sp.n2);
    return hipGetLastError();
}

namespace {
// the fp64 row pass's fast Morse form applies (RowW<double, kMorseFast>)
bool morse_fast_of(const WDesc& d) {
    const double b2 = 2.0 * d.b;
    return d.kind == NW_MORSE && !d.morse_ovf && d.r == 3.0 && b2 >= 0.0 && b2 < 128.0 && b2 == (double)(int)b2;
}

template <typename T>
hipError_t rows_t(const WDesc& d, int f0, int nf, const int* km, void* scratch, hipStream_t s) {
    const Split sp = split_of(d.n, sizeof(T) == 4 ? NW_F32 : NW_F64);
    C2<T>* Xt = reinterpret_cast<C2<T>*>(scratch);
    C2<T>* B = Xt + d.n;
#define NW_ROWS(NN)                                                                                          \
    case NN:                                                                                                 \
        if constexpr (NN <= kMaxN2<T>) {                                                                     \
            constexpr int EE = kRowE<T, NN>;                                                                 \
            switch (d.kind) {                                                                                \
                case NW_MORSE:                                                                               \
                    if constexpr (sizeof(T) == 8)                                                            \
                        if (morse_fast_of(d))                                                                \
                            return d.b == 17.5 ? (kRowsRec && d.off == 0 ? launch_row_pass<T, NN, EE, kMorseRec>(d, f0, nf, sp.n1, Xt, B, km, s) \
                                                             : launch_row_pass<T, NN, EE, kMorseFast35>(d, f0, nf, sp.n1, Xt, B, km, s)) \
                                               : launch_row_pass<T, NN, EE, kMorseFast>(d, f0, nf, sp.n1, Xt, B, km, s);  \
                    if constexpr (sizeof(T) == 4)                                                            \
                        if (d.morse_ovf) return launch_row_pass<T, NN, EE, kMorseOvf>(d, f0, nf, sp.n1, Xt, B, km, s); \
                    return launch_row_pass<T, NN, EE, NW_MORSE>(d, f0, nf, sp.n1, Xt, B, km, s);             \
                case NW_MORLET: return launch_row_pass<T, NN, EE, NW_MORLET>(d, f0, nf, sp.n1, Xt, B, km, s);   \
                case NW_SHANNON: return launch_row_pass<T, NN, EE, NW_SHANNON>(d, f0, nf, sp.n1, Xt, B, km, s); \
                case NW_TABLE: return launch_row_pass<T, NN, kRowETab<T, NN>, NW_TABLE>(d, f0, nf, sp.n1, Xt, B, km, s); \
                default: return hipErrorNotSupported;                                                        \
            }                                                                                                \
        }                                                                                                    \
        return hipErrorNotSupported;
    switch (sp.n2) {
        NW_ROWS(1024) NW_ROWS(2048) NW_ROWS(4096) NW_ROWS(8192) NW_ROWS(16384)
        default: return hipErrorNotSupported;
    }
#undef NW_ROWS
}

template <typename T>
hipError_t cols_t(const WDesc& d, int out_kind, int f0, int nf, const void* support, const void* scratch, void* out,
                  hipStream_t s) {
    const Split sp = split_of(d.n, sizeof(T) == 4 ? NW_F32 : NW_F64);
    const C2<T>* B = reinterpret_cast<const C2<T>*>(scratch) + d.n;
    const C2<T>* ts = sizeof(T) == 8 ? reinterpret_cast<const C2<T>*>(reinterpret_cast<const char*>(support) +
                                                                      tsplit_offset(d.nfreq))
                                     : nullptr;
#define NW_COLS(A, BB) \
    if (sp.n1 == A && sp.n2 == BB) return launch_cols<T, A, BB>(out_kind, f0, nf, B, out, ts, s);
    if constexpr (sizeof(T) == 4) {
        NW_COLS(32, 1024) NW_COLS(32, 2048) NW_COLS(32, 4096) NW_COLS(32, 8192) NW_COLS(32, 16384)
        NW_COLS(64, 16384) NW_COLS(128, 16384) NW_COLS(256, 16384) NW_COLS(512, 16384) NW_COLS(1024, 16384)
    } else {
        NW_COLS(32, 1024) NW_COLS(32, 2048) NW_COLS(32, 4096) NW_COLS(32, 8192) NW_COLS(32, 16384)
        NW_COLS(64, 16384) NW_COLS(128, 16384) NW_COLS(256, 16384) NW_COLS(512, 16384) NW_COLS(1024, 16384)
    }
    return hipErrorNotSupported;
#undef NW_COLS
}
}  // namespace

// pass 1 for scales [f0, f0 + nf): Xt -> B (both in the scratch)
hipError_t large_rows(const WDesc& d, int dtype, int f0, int nf, const void* support, void* scratch, hipStream_t s) {
    const int* km = reinterpret_cast<const int*>(support);
    return dtype == NW_F32 ? rows_t<float>(d, f0, nf, km, scratch, s) : rows_t<double>(d, f0, nf, km, scratch, s);
}

// pass 2 for scales [f0, f0 + nf): B -> out rows (f, n) of one signal (out: its row 0)
hipError_t large_cols(const WDesc& d, int dtype, int out_kind, int f0, int nf, const void* support,
                      const void* scratch, void* out, hipStream_t s) {
    return dtype == NW_F32 ? cols_t<float>(d, out_kind, f0, nf, support, scratch, out, s)
                           : cols_t<double>(d, out_kind, f0, nf, support, scratch, out, s);
}

}  // namespace nw
