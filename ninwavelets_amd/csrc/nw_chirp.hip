// nw_chirp.hip — fused engine for the signal lengths the power-of-two kernels do not take
// (any n with 2n - 1 <= 16384 fp32 / 8192 fp64 that is not a power of two >= 1024: MNE
// epochs of 1201, 4097, ... samples; reference base.py:378-407 makes no distinction).
//
// The inverse DFT of length n is a chirp-z (Bluestein) convolution computed with the
// power-of-two machinery of nw_fft_dev.h on chip, M = 2^ceil(log2(2n - 1)):
//   c(k) = exp(+i pi k^2 / n),   a[k] = W[f,k] X[k] c(k)   (k < n, zero to M; W carries 1/n)
//   A = FFT_M(a)                  (the inverse passes on conj(a): A = conj(IDFT(conj a)))
//   P = A * Bh,   Bh = FFT_M(b) / M,  b[j] = b[M - j] = exp(-i pi j^2 / n) (j < n), 0 between
//   y'= IDFT_M(P)                 (= sum_k a[k] b[n - k]: the linear convolution, n < N)
//   y[n] = c(n) y'[n]            = sum_k W X exp(2 pi i n k / n)   (ifft of base.py:406)
// so one (scale, signal) row costs two M-point on-chip FFTs and is still read once (X, W)
// and written once (y, |y| or |y|^2): 8 B/pt of HBM (fp32 cwt) instead of the rocFFT
// engine's product + Bluestein passes + epilogue.  Bh (and, in fp64, the chirp c) are
// built once per (device, n) in fp64; the fp32 chirp comes from v_sin/v_cos on the exact
// phase index k^2 mod 2n.
#include <map>
#include <mutex>
#include <tuple>
#include <vector>
#include <algorithm>

#include "nw_fft_dev.h"

namespace nw {
namespace {

// signals per block; measured (n = 1201 / 4097): 4 -2 % / -1 %, 16 +0.6 % / +0.6 % (noise).
// The partial-sum form writes one row per block: execute_reduce sizes and accumulates them by
// fused_psum_groups, i.e. kPsumGroup signals per row
constexpr int kGroupC = 8;
static_assert(kGroupC == kPsumGroup, "chirp-z partial rows are counted by fused_psum_groups");
constexpr int kTileFC = 8;    // scales per XCD tile
constexpr int kTileGC = 4;    // signal groups per XCD tile
constexpr int kRegOsz = 16;   // PassInfo without last-pass pairing: j = t + q*T everywhere

// exchange P-1 -> P and pass P, as passes_from (nw_fft_dev.h) without the stores: the
// last pass leaves its outputs in registers, v[q*R + i] = output j + bitrev(i)*NS, j = t + q*T
template <typename T, int N, int E, int P>
__device__ __forceinline__ void passes_regs(C2<T>* v, T* lds, int t, const C2<Sc<T>>* __restrict__ tw) {
    using S = Sc<T>;   // T = f2: two signals per lane value, twiddles shared
    using I = PassInfo<N, E, P, kRegOsz>;
    if constexpr (P < Geometry<N, E>::npass()) {
        constexpr int R = I::R, Q = I::Q, LR = ilog2<R>();
        constexpr bool TABLED = P == 1 && Tab1<T, N, E>::ON;
        C2<S> pb[Q][LR > 0 ? LR : 1];
        if constexpr (!TABLED) {
#pragma unroll
            for (int q = 0; q < Q; ++q) twiddle_bases<S, R, N, I::NS * R>(pb[q], I::bfly(t, q) % I::NS, tw);
        }
        lds_barrier();
        lds_write<T, N, E, P - 1, 0>(v, lds, t);
        lds_barrier();
        lds_read<T, N, E, P, 0, kRegOsz>(v, lds, t);
        lds_barrier();
        lds_write<T, N, E, P - 1, 1>(v, lds, t);
        lds_barrier();
        lds_read<T, N, E, P, 1, kRegOsz>(v, lds, t);
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            if constexpr (TABLED) {
                const C2<S>* tab = Tab1<T, N, E>::table(lds) + I::bfly(t, q) % I::NS;
#pragma unroll
                for (int r = 1; r < R; ++r) v[q * R + r] = cmul(v[q * R + r], tab[(r - 1) * I::NS]);
            } else {
                twiddle_apply<T, R>(v + q * R, pb[q]);
            }
            idft_br<T, R>(v + q * R);
        }
        passes_regs<T, N, E, P + 1>(v, lds, t, tw);
    }
}

// c(k) = exp(+i pi k^2 / n): fp32 from the exact phase index k^2 mod 2n (revolutions),
// fp64 from the table built with sincospi
template <typename T>
__device__ __forceinline__ C2<T> chirp(int k, uint32_t n2, float inv_n2, const C2<T>* __restrict__ ct) {
    if constexpr (sizeof(T) == 4) {
        const uint32_t m = ((uint32_t)k * (uint32_t)k) % n2;
        const float rev = (float)m * inv_n2;
        return C2<T>{__builtin_amdgcn_cosf(rev), __builtin_amdgcn_sinf(rev)};
    } else {
        NW_DCHECK(k >= 0 && (uint32_t)k < n2 / 2);
        return ct[k];
    }
}

// (fp32 phase indices k^2 mod 2n by exact modular increments instead of one urem per
// element measured 2.7 % slower at n = 1201, power and cwt: not kept)

template <typename T, bool REALW> struct WRow;
template <typename T> struct WRow<T, true> {
    using type = T;
    __device__ static __forceinline__ C2<T> apply(T w, cplx<T> x) { return {w * x.re, w * x.im}; }
};
template <typename T> struct WRow<T, false> {
    using type = C2<T>;
    __device__ static __forceinline__ C2<T> apply(C2<T> w, cplx<T> x) { return cmul(w, C2<T>{x.re, x.im}); }
};

// waves per SIMD without scratch (tools/regs.py): fp32 M <= 4096 fit 168 VGPRs (3 waves;
// 4 spilled 44 B at M = 1024), M >= 8192 and fp64 need up to 256 (2 waves; fp32 M = 16384
// at E = 32 still spills ~230 B there)
// (the phase-sum form holds the chirp and the reciprocal on top: 2 waves/SIMD, no scratch)
template <typename T, int M, int E, int OUT>
constexpr int kChirpWps = OUT == kOutPhSum ? 2 : E <= 8 ? 4 : (sizeof(T) == 4 && M <= 4096 && E <= 16) ? 3 : 2;
template <typename T, int M, int E, int OUT, bool REALW>
__global__ __launch_bounds__(M / E, (kChirpWps<T, M, E, OUT>)) void nw_chirp_kernel(
    WDesc d, const cplx<T>* __restrict__ X, const void* __restrict__ wtab, void* __restrict__ out,
    const C2<T>* __restrict__ tw, const C2<T>* __restrict__ bh, const C2<T>* __restrict__ ct, int64_t nsig,
    int nsg_pad, const int* __restrict__ rowmap, int nrows, const int* __restrict__ ksup) {
    using G = Geometry<M, E>;
    constexpr int TT = G::T;
    constexpr int LP = G::npass() - 1;
    using IL = PassInfo<M, E, LP, kRegOsz>;
    static_assert(PassInfo<M, E, 1, kRegOsz>::R == E, "pass 1 must be radix E (pass-0 layout reads)");
    using O = typename OutT<OUT, T>::type;
    using WT = typename WRow<T, REALW>::type;
    extern __shared__ __align__(16) unsigned char smem[];
    T* lds = reinterpret_cast<T*>(smem);
    const int t = threadIdx.x;
    // XCD-aware block -> (scale, signal group), as nw_fused_kernel
    const int b = blockIdx.x;
    const int xcd = b & 7;
    const int local = b >> 3;
    const int pos = local % (kTileFC * kTileGC);
    const int round = local / (kTileFC * kTileGC);
    const int nfr = (nrows + kTileFC - 1) / kTileFC;
    const int fl = (round % nfr) * kTileFC + pos % kTileFC;   // this launch's rows: rowmap[0 .. nrows)
    const int sg = ((round / nfr) * kTileGC + pos / kTileFC) * 8 + xcd;
    if (fl >= nrows || sg >= nsg_pad || (int64_t)sg * kGroupC >= nsig) return;
    const int fi = rowmap[fl];
    const int64_t s_begin = (int64_t)sg * kGroupC;
    const int64_t s_end = min(nsig, s_begin + kGroupC);

    const int n = (int)d.n;
    const uint32_t n2 = 2u * (uint32_t)n;
    const float inv_n2 = 1.0f / (float)n2;
    const WT* wrow = reinterpret_cast<const WT*>(wtab) + (int64_t)fi * n;
    const int nz = (ksup[fi] + TT - 1) / TT;   // pass-0 elements reaching the support (<= E/2)
    // the row's M class: wrap-free (M >= n + K - 1) and the pruned pass 0 (M >= 2K, nz <= E/2)
    NW_DCHECK(fi >= 0 && fi < d.nfreq && s_end <= nsig && n + max(ksup[fi], 1) - 1 <= M && 2 * ksup[fi] <= M);
    Tab1<T, M, E>::fill(lds, tw, t);
    for (int64_t s = s_begin; s < s_end; ++s) {
        const cplx<T>* Xs = X + s * d.nh;
        C2<T> v[E];
        // a[k] = W X c(k), conjugated: the forward FFT through the inverse passes
        // only the elements r < NZ (bins k < NZ*T) can meet the row's support K <= M/2: the
        // others are zero for every thread and the DIF stages skip them (as nw_fused's pass 0)
        auto pass0 = [&]<int NZ>() {
#pragma unroll
            for (int r = 0; r < E; ++r) {
                const int k = t + r * TT;
                C2<T> a{T(0), T(0)};
                if (r < NZ && k < n) {
                    const C2<T> z = WRow<T, REALW>::apply(wrow[k], spectrum_bin<T>(Xs, d, k));
                    a = cmul(z, chirp<T>(k, n2, inv_n2, ct));
                }
                v[r] = C2<T>{a.re, -a.im};
            }
            idft_br<T, E, NZ>(v);
        };
        if (nz <= 1) pass0.template operator()<1>();
        else if (nz <= 2) pass0.template operator()<2>();
        else if (nz <= 4) pass0.template operator()<4>();
        else pass0.template operator()<E / 2>();
        passes_regs<T, M, E, 1>(v, lds, t, tw);
        // P[m] = conj(v[m]) * Bh[m]
#pragma unroll
        for (int q = 0; q < IL::Q; ++q)
#pragma unroll
            for (int i = 0; i < IL::R; ++i) {
                const int m = t + q * TT + bitrev<IL::R>(i) * IL::NS;
                C2<T>& e = v[q * IL::R + i];
                e = cmul(C2<T>{e.re, -e.im}, bh[m]);
            }
        // natural order -> the pass-0 layout (element m = t + r*T) through the image
        lds_barrier();
        lds_write<T, M, E, LP, 0>(v, lds, t);
        lds_barrier();
        lds_read<T, M, E, 1, 0, kRegOsz>(v, lds, t);
        lds_barrier();
        lds_write<T, M, E, LP, 1>(v, lds, t);
        lds_barrier();
        lds_read<T, M, E, 1, 1, kRegOsz>(v, lds, t);
        idft_br<T, E>(v);
        passes_regs<T, M, E, 1>(v, lds, t, tw);
        // y[n] = c(n) y'[n] for n < N (|y|, |y|^2: |c(n)| = 1, the chirp is skipped)
        O* orow = reinterpret_cast<O*>(out) + (s * d.nfreq + fi) * (int64_t)n;
        // epoch partial sums (kOutPSum / kOutPhSum): the block's fp64 row (group sg, scale fi)
        // of the (groups, F, n) partial buffer, read-modify-written by the lane that owns each
        // point (the same lane for every signal), in signal order -- no accumulator registers
        constexpr bool PS = OUT == kOutPSum || OUT == kOutPhSum;
        constexpr int NACC = OUT == kOutPhSum ? 2 : 1;
        double* prow = reinterpret_cast<double*>(out) + ((int64_t)sg * d.nfreq + fi) * (int64_t)n * NACC;
        const bool first = s == s_begin;
#pragma unroll
        for (int q = 0; q < IL::Q; ++q) {
            // outputs n_j = n0 + j*NS in natural j order (register i = bitrev(j)); |y| and
            // |y|^2 skip the final chirp (|c(n) y'| = |y'|: n = 1201 power 1.397 -> 1.313 ms)
            const uint32_t n0 = (uint32_t)(t + q * TT);
            constexpr bool EPI = OUT == NW_OUT_CWT || OUT == kOutPhSum;
#pragma unroll
            for (int j = 0; j < IL::R; ++j) {
                const int i = bitrev<IL::R>(j);
                const int idx = (int)n0 + j * IL::NS;
                C2<T> y = v[q * IL::R + i];
                // (idx >= n: not stored; the chirp index is clamped so the fp64 table ct[0 .. n)
                // is never read past its end, whatever the compiler hoists)
                if constexpr (EPI) y = cmul(y, chirp<T>(idx < n ? idx : 0, n2, inv_n2, ct));
                if constexpr (OUT == kOutPSum) {
                    // the power output's own value (out_value), added in fp64 like k_accumulate
                    const double pv = (double)out_value<NW_OUT_POWER, T>(y);
                    if (idx < n) prow[idx] = first ? pv : prow[idx] + pv;
                } else if constexpr (OUT == kOutPhSum) {
                    // y / |y| (fp64 y: 1 / hypot, which does not underflow; fp32: rsqrt of the
                    // exact fp64 |y|^2), 0 / 0 -> NaN like the reference (mneutils.py:68)
                    const double re = (double)y.re, im = (double)y.im;
                    const double inv = sizeof(T) == 8 ? 1.0 / hypot(re, im) : rsqrt(re * re + im * im);
                    const double pr = mul_nocontract(re, inv), pi = mul_nocontract(im, inv);
                    if (idx < n) {
                        double2* q2 = reinterpret_cast<double2*>(prow) + idx;
                        if (first) {
                            *q2 = double2{pr, pi};
                        } else {
                            const double2 o = *q2;
                            *q2 = double2{o.x + pr, o.y + pi};
                        }
                    }
                } else {
                    if (idx < n) orow[idx] = out_value<OUT, T>(y);
                }
                // partial sums: at most 4 read-modify-writes in flight (their loaded values
                // would otherwise all be live at once and spill)
                if constexpr (PS) {
                    if (j % 4 == 3) __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
    }
}

// W rows of length n (1/n folded in) for the chirp engine: the reference's cached row,
// pad_to'd (base.py:75-82, 396-397); X's interpolate mask is applied by spectrum_bin
template <typename T, bool REALW>
__global__ __launch_bounds__(256) void chirp_wtable_kernel(WDesc d, void* wtab) {
    const int fi = blockIdx.y;
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= d.n) return;
    const cplx<T> w = wavelet_bin<T>(d, fi, k);
    if constexpr (REALW)
        reinterpret_cast<T*>(wtab)[(int64_t)fi * d.n + k] = w.re;
    else
        reinterpret_cast<C2<T>*>(wtab)[(int64_t)fi * d.n + k] = C2<T>{w.re, w.im};
}

// Support of each W row: ksup[f] = last nonzero bin + 1 (0 for an all-zero row)
template <typename T, bool REALW>
__global__ __launch_bounds__(256) void chirp_support_kernel(const void* wtab, int64_t n, int* ksup) {
    __shared__ int kmax[256];
    const int fi = blockIdx.x;
    int m = -1;
    for (int64_t k = threadIdx.x; k < n; k += 256) {
        bool nzv;
        if constexpr (REALW) nzv = reinterpret_cast<const T*>(wtab)[(int64_t)fi * n + k] != T(0);
        else {
            const C2<T> w = reinterpret_cast<const C2<T>*>(wtab)[(int64_t)fi * n + k];
            nzv = w.re != T(0) || w.im != T(0);
        }
        if (nzv) m = (int)k;
    }
    kmax[threadIdx.x] = m;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) kmax[threadIdx.x] = max(kmax[threadIdx.x], kmax[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) ksup[fi] = kmax[0] + 1;
}

// Bh[m] = (1/M) sum_p b(p) exp(-2 pi i m p / M), in fp64, b(p) = exp(-i pi j^2 / n) for the
// lag j = p (p < n) or p - M (p >= n) when -n < j < n, else 0.  With M >= 2n - 1 that is the
// whole chirp; a row whose W support is K bins needs only the lags -K < j < n, so any
// M >= n + K - 1 is wrap-free for it (the circular convolution equals the linear one on the
// n outputs) -- the smaller M of band-limited rows.
template <typename T>
__global__ __launch_bounds__(256) void chirp_bhat_kernel(C2<T>* bh, int n, int m_len) {
    const int m = blockIdx.x * 256 + threadIdx.x;
    if (m >= m_len) return;
    double re = 0.0, im = 0.0;
    for (int p = 0; p < m_len; ++p) {
        const int j = p < n ? p : p - m_len;
        if (j <= -n) continue;
        const int64_t aj = j < 0 ? -(int64_t)j : j;
        double bs, bc, es, ec;
        sincospi(-(double)((aj * aj) % (2 * (int64_t)n)) / n, &bs, &bc);
        sincospi(-2.0 * (double)(((int64_t)m * p) % m_len) / m_len, &es, &ec);
        re += bc * ec - bs * es;
        im += bc * es + bs * ec;
    }
    bh[m] = C2<T>{(T)(re / m_len), (T)(im / m_len)};
}

// the fp64 chirp c(k) = exp(+i pi k^2 / n), k < n
template <typename T>
__global__ __launch_bounds__(256) void chirp_ct_kernel(C2<T>* ct, int n) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    double sn, cs;
    sincospi((double)(((int64_t)k * k) % (2 * (int64_t)n)) / n, &sn, &cs);
    ct[k] = C2<T>{(T)cs, (T)sn};
}

struct ChirpKey {
    int dev;
    int64_t n, m;
    int dtype;
    bool operator<(const ChirpKey& o) const {
        return std::tie(dev, n, m, dtype) < std::tie(o.dev, o.n, o.m, o.dtype);
    }
};
std::mutex g_chirp_mu;
std::map<ChirpKey, void*> g_chirp;   // per device, length and M: Bh[M] then (fp64) c[n]

constexpr int kChirpClasses = 5;      // M = 1024 << c, c < 5
int64_t chirp_m(int64_t n) {
    int64_t m = 1024;
    while (m < 2 * n - 1) m <<= 1;
    return m;
}

hipError_t chirp_tables(int64_t n, int64_t m, int dtype, void** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_chirp_mu);
    auto it = g_chirp.find({dev, n, m, dtype});
    if (it != g_chirp.end()) {
        *out = it->second;
        return hipSuccess;
    }
    const size_t esz = dtype == NW_F32 ? sizeof(C2<float>) : sizeof(C2<double>);
    void* p = nullptr;
    e = hipMalloc(&p, (size_t)(m + n) * esz);
    if (e != hipSuccess) return e;
    const unsigned bm = (unsigned)((m + 255) / 256), bn = (unsigned)((n + 255) / 256);
    if (dtype == NW_F32) {
        hipLaunchKernelGGL(chirp_bhat_kernel<float>, bm, 256, 0, 0, (C2<float>*)p, (int)n, (int)m);
    } else {
        hipLaunchKernelGGL(chirp_bhat_kernel<double>, bm, 256, 0, 0, (C2<double>*)p, (int)n, (int)m);
        hipLaunchKernelGGL(chirp_ct_kernel<double>, bn, 256, 0, 0, (C2<double>*)p + m, (int)n);
    }
    e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        (void)hipFree(p);
        return e;
    }
    g_chirp[{dev, n, m, dtype}] = p;
    *out = p;
    return hipSuccess;
}

template <typename T, int M, int E, bool REALW>
hipError_t launch_m_e(const WDesc& d, int out_kind, const void* X, const void* wtab, void* out, int64_t nsig,
                      const int* rowmap, int nrows, const int* ksup, hipStream_t s) {
    constexpr int threads = M / E;
    const int lds = kLdsBytes<T, M, E>;
    void* tw = nullptr;
    hipError_t e = fused_twiddles(M, sizeof(T) == 4 ? NW_F32 : NW_F64, &tw);
    if (e != hipSuccess) return e;
    void* tabs = nullptr;
    e = chirp_tables(d.n, M, sizeof(T) == 4 ? NW_F32 : NW_F64, &tabs);
    if (e != hipSuccess) return e;
    const C2<T>* bh = reinterpret_cast<const C2<T>*>(tabs);
    const C2<T>* ct = bh + M;
    const int64_t nsg = (nsig + kGroupC - 1) / kGroupC;
    const int64_t nsg_pad = (nsg + 8 * kTileGC - 1) / (8 * kTileGC) * (8 * kTileGC);
    const int64_t nfr = (nrows + kTileFC - 1) / kTileFC;
    const int64_t blocks = nsg_pad * nfr * kTileFC;
    if (blocks > 0x7fffffff || nsg_pad > 0x7fffffff) return hipErrorInvalidConfiguration;
    const cplx<T>* Xc = reinterpret_cast<const cplx<T>*>(X);
    const C2<T>* twc = reinterpret_cast<const C2<T>*>(tw);
    auto go = [&](auto kern) {
        e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return;
        nw_launch(kern, (unsigned)blocks, threads, lds, s, d, Xc, wtab, out, twc, bh, ct, nsig, (int)nsg_pad, rowmap, nrows,
                                                    ksup);
        e = hipGetLastError();
    };
    if (out_kind == NW_OUT_CWT) go(nw_chirp_kernel<T, M, E, NW_OUT_CWT, REALW>);
    else if (out_kind == NW_OUT_POWER) go(nw_chirp_kernel<T, M, E, NW_OUT_POWER, REALW>);
    else if (out_kind == kOutPSum || out_kind == kOutPhSum) {
        // partial sums at E = 16 only (chirp_psum_ok: the classes whose kernels do not spill)
        if constexpr (E == 16) {
            if (out_kind == kOutPSum) go(nw_chirp_kernel<T, M, E, kOutPSum, REALW>);
            else go(nw_chirp_kernel<T, M, E, kOutPhSum, REALW>);
        } else {
            e = hipErrorNotSupported;
        }
    } else go(nw_chirp_kernel<T, M, E, NW_OUT_ABS, REALW>);
    return e;
}

// fp32 M = 8192: |y| and |y|^2 at E = 32 (256 threads, two blocks per CU, 3 passes, no
// scratch): measured N = 4097 power 10.60 -> 8.75 ms, N = 3001 6.60 -> 5.82 ms per launch;
// the complex output spills at E = 32 (108-128 B) and keeps E = 16
template <typename T, int M, int E, bool REALW>
hipError_t launch_m(const WDesc& d, int out_kind, const void* X, const void* wtab, void* out, int64_t nsig,
                    const int* rowmap, int nrows, const int* ksup, hipStream_t s) {
    constexpr int EP = (sizeof(T) == 4 && M == 8192) ? 32 : E;
    if constexpr (EP != E) {
        if (out_kind == NW_OUT_POWER || out_kind == NW_OUT_ABS)
            return launch_m_e<T, M, EP, REALW>(d, out_kind, X, wtab, out, nsig, rowmap, nrows, ksup, s);
    }
    return launch_m_e<T, M, E, REALW>(d, out_kind, X, wtab, out, nsig, rowmap, nrows, ksup, s);
}

}  // namespace

// (dtype, M, E) of the chirp engine: fp32 M <= 16384 (E = 32 at 16384), fp64 M <= 8192
#define NW_CHIRP_TABLE(X)                                                                        \
    X(float, 1024, 16) X(float, 2048, 16) X(float, 4096, 16) X(float, 8192, 16) X(float, 16384, 32) \
    X(double, 1024, 16) X(double, 2048, 16) X(double, 4096, 16) X(double, 8192, 16)

int64_t chirp_mmax(int dtype) { return dtype == NW_F32 ? 16384 : 8192; }

bool chirp_supported(int64_t n, int dtype) {
    if (n < 1 || fused_supported(n, dtype)) return false;
    return (dtype == NW_F32 || dtype == NW_F64) && 2 * n - 1 <= chirp_mmax(dtype);
}

// longer lengths (up to M_max - 1) fit when every row's support does (M >= n + K - 1)
bool chirp_possible(int64_t n, int dtype) {
    if (n < 1 || fused_supported(n, dtype) || (dtype != NW_F32 && dtype != NW_F64)) return false;
    return n < chirp_mmax(dtype);
}

// table buffer: W rows, then ksup[nfreq], then the row map (rows grouped by M class)
size_t chirp_w_bytes(int64_t n, int nfreq, int dtype, int kind) {
    const size_t esz = dtype == NW_F32 ? sizeof(float) : sizeof(double);
    return ((size_t)n * nfreq * esz * (kind != NW_TABLE ? 1 : 2) + 15) / 16 * 16;
}
size_t chirp_wtable_bytes(int64_t n, int nfreq, int dtype, int kind) {
    return chirp_w_bytes(n, nfreq, dtype, kind) + 2 * (size_t)nfreq * sizeof(int);
}

hipError_t build_chirp_wtable(const WDesc& d, int dtype, void* wtab, hipStream_t s, int64_t* counts, bool* fits,
                              std::vector<int>* overflow) {
    dim3 grid((unsigned)((d.n + 255) / 256), (unsigned)d.nfreq);
    const bool realw = d.kind != NW_TABLE;
    int* ksup = reinterpret_cast<int*>(reinterpret_cast<char*>(wtab) + chirp_w_bytes(d.n, d.nfreq, dtype, d.kind));
    int* rowmap = ksup + d.nfreq;
    if (dtype == NW_F32) {
        if (realw) nw_launch(chirp_wtable_kernel<float, true>, grid, 256, 0, s, d, wtab);
        else nw_launch(chirp_wtable_kernel<float, false>, grid, 256, 0, s, d, wtab);
        if (realw) nw_launch(chirp_support_kernel<float, true>, d.nfreq, 256, 0, s, wtab, d.n, ksup);
        else nw_launch(chirp_support_kernel<float, false>, d.nfreq, 256, 0, s, wtab, d.n, ksup);
    } else {
        if (realw) nw_launch(chirp_wtable_kernel<double, true>, grid, 256, 0, s, d, wtab);
        else nw_launch(chirp_wtable_kernel<double, false>, grid, 256, 0, s, d, wtab);
        if (realw) nw_launch(chirp_support_kernel<double, true>, d.nfreq, 256, 0, s, wtab, d.n, ksup);
        else nw_launch(chirp_support_kernel<double, false>, d.nfreq, 256, 0, s, wtab, d.n, ksup);
    }
    hipError_t e = hipGetLastError();
    // once per wavelet: the rows' M classes on the host (M >= n + K - 1 wrap-free, >= 2K for
    // the pruned first pass 0, >= 1024, <= the full 2^ceil(log2(2n - 1)))
    std::vector<int> ks(d.nfreq);
    if (e == hipSuccess) e = hipMemcpyAsync(ks.data(), ksup, d.nfreq * sizeof(int), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    const int64_t mfull = std::min<int64_t>(chirp_m(d.n), chirp_mmax(dtype));
    std::vector<int> cls(d.nfreq);
    for (int c = 0; c < kChirpClasses; ++c) counts[c] = 0;
    *fits = true;
    if (overflow) overflow->clear();
    for (int f = 0; f < d.nfreq; ++f) {
        const int64_t need = std::max<int64_t>(d.n + std::max(ks[f], 1) - 1, 2 * (int64_t)ks[f]);
        if (need > mfull) {
            // wider than the largest on-chip transform: listed for the caller (rocFFT rows)
            *fits = false;
            if (overflow) overflow->push_back(f);
            cls[f] = -1;
            continue;
        }
        int64_t m = 1024;
        while (m < need && m < mfull) m <<= 1;
        int c = 0;
        while ((1024ll << c) < m) ++c;
        cls[f] = c;
        counts[c]++;
    }
    std::vector<int> map;
    for (int c = 0; c < kChirpClasses; ++c)
        for (int f = 0; f < d.nfreq; ++f)
            if (cls[f] == c) map.push_back(f);
    e = hipMemcpyAsync(rowmap, map.data(), map.size() * sizeof(int), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return e;
}

// Epoch partial sums on the chirp-z form: every M class of the wavelet needs a partial-sum
// kernel without scratch (tools/regs.py): fp32 M <= 8192 (E = 16), fp64 power every M, fp64
// phases M <= 2048 (44-60 B of scratch above)
bool chirp_psum_ok(int dtype, bool phase, const int64_t* counts) {
    for (int c = 0; c < kChirpClasses; ++c) {
        if (counts[c] == 0) continue;
        const int64_t m = 1024ll << c;
        if (dtype == NW_F32 ? m > 8192 : (phase && m > 2048)) return false;
    }
    return true;
}

hipError_t launch_chirp(const WDesc& d, int dtype, int out_kind, const void* X, const void* wtab, void* out,
                        int64_t nsig, const int64_t* counts, hipStream_t s) {
    if (!chirp_possible(d.n, dtype)) return hipErrorNotSupported;
    const bool realw = d.kind != NW_TABLE;
    const int* ksup = reinterpret_cast<const int*>(reinterpret_cast<const char*>(wtab) +
                                                   chirp_w_bytes(d.n, d.nfreq, dtype, d.kind));
    const int* rowmap = ksup + d.nfreq;
    int64_t off = 0;
    for (int c = 0; c < kChirpClasses; ++c) {
        const int64_t cnt = counts[c];
        if (cnt == 0) continue;
        const int64_t m = 1024ll << c;
        hipError_t e = hipErrorNotSupported;
#define NW_CHIRP_LAUNCH(TY, MM, EE)                                                                             \
        if (m == MM && dtype == (sizeof(TY) == 4 ? NW_F32 : NW_F64))                                            \
            e = realw ? launch_m<TY, MM, EE, true>(d, out_kind, X, wtab, out, nsig, rowmap + off, (int)cnt, ksup, s) \
                      : launch_m<TY, MM, EE, false>(d, out_kind, X, wtab, out, nsig, rowmap + off, (int)cnt, ksup, s);
        NW_CHIRP_TABLE(NW_CHIRP_LAUNCH)
#undef NW_CHIRP_LAUNCH
        if (e != hipSuccess) return e;
        off += cnt;
    }
    return hipSuccess;
}

}  // namespace nw
