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

#include "nw_fft_dev.h"

namespace nw {
namespace {

constexpr int kGroupC = 8;    // signals per block
constexpr int kTileFC = 8;    // scales per XCD tile
constexpr int kTileGC = 4;    // signal groups per XCD tile
constexpr int kRegOsz = 16;   // PassInfo without last-pass pairing: j = t + q*T everywhere
#ifndef NW_CHIRP_PAIR
#define NW_CHIRP_PAIR 0       // fp32 analytic rows, two signals per lane value (C2<f2>): measured
                              // +-2 % at n = 700 / 1000 / 1201 (not VALU-bound), so off
#endif
#ifndef NW_CHIRP_PAIR_MAXM
#define NW_CHIRP_PAIR_MAXM 4096   // pair kernels up to this M (2 waves/SIMD; 44-56 B scratch at 4096)
#endif

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
        return ct[k];
    }
}

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
template <typename T, int M, int E> constexpr int kChirpWps = E <= 8 ? 4 : (sizeof(T) == 4 && M <= 4096) ? 3 : 2;
template <typename T, int M, int E, int OUT, bool REALW>
__global__ __launch_bounds__(M / E, (kChirpWps<T, M, E>)) void nw_chirp_kernel(
    WDesc d, const cplx<T>* __restrict__ X, const void* __restrict__ wtab, void* __restrict__ out,
    const C2<T>* __restrict__ tw, const C2<T>* __restrict__ bh, const C2<T>* __restrict__ ct, int64_t nsig,
    int nsg_pad) {
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
    const int nfr = (d.nfreq + kTileFC - 1) / kTileFC;
    const int fi = (round % nfr) * kTileFC + pos % kTileFC;
    const int sg = ((round / nfr) * kTileGC + pos / kTileFC) * 8 + xcd;
    if (fi >= d.nfreq || sg >= nsg_pad || (int64_t)sg * kGroupC >= nsig) return;
    const int64_t s_begin = (int64_t)sg * kGroupC;
    const int64_t s_end = min(nsig, s_begin + kGroupC);

    const int n = (int)d.n;
    const uint32_t n2 = 2u * (uint32_t)n;
    const float inv_n2 = 1.0f / (float)n2;
    const WT* wrow = reinterpret_cast<const WT*>(wtab) + (int64_t)fi * n;
    Tab1<T, M, E>::fill(lds, tw, t);
    for (int64_t s = s_begin; s < s_end; ++s) {
        const cplx<T>* Xs = X + s * d.nh;
        C2<T> v[E];
        // a[k] = W X c(k), conjugated: the forward FFT through the inverse passes
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int k = t + r * TT;
            C2<T> a{T(0), T(0)};
            if (k < n) {
                const C2<T> z = WRow<T, REALW>::apply(wrow[k], spectrum_bin<T>(Xs, d, k));
                a = cmul(z, chirp<T>(k, n2, inv_n2, ct));
            }
            v[r] = C2<T>{a.re, -a.im};
        }
        idft_br<T, E, E / 2>(v);   // n <= M/2: elements r >= E/2 (k >= M/2) are zero
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
        // y[n] = c(n) y'[n] for n < N
        O* orow = reinterpret_cast<O*>(out) + (s * d.nfreq + fi) * (int64_t)n;
#pragma unroll
        for (int q = 0; q < IL::Q; ++q)
#pragma unroll
            for (int i = 0; i < IL::R; ++i) {
                const int idx = t + q * TT + bitrev<IL::R>(i) * IL::NS;
                if (idx < n) orow[idx] = out_value<OUT, T>(cmul(v[q * IL::R + i], chirp<T>(idx, n2, inv_n2, ct)));
            }
    }
}

// Signal pairs (fp32, analytic real W rows), as nw_fused_pair_kernel: every lane value is
// a C2<f2> holding signal s in the low and s+1 in the high half, so each butterfly, twiddle
// multiply, chirp / Bh multiply and LDS access of both transforms serves two signals
// (v_pk_* math, 8-B image slots); an odd last signal transforms a duplicate, not stored.
template <int M, int E, int OUT>
__global__ __launch_bounds__(M / E, 2) void nw_chirp_pair_kernel(
    WDesc d, const cplx<float>* __restrict__ X, const float* __restrict__ wtab, void* __restrict__ out,
    const C2<float>* __restrict__ tw, const C2<float>* __restrict__ bh, int64_t nsig, int nsg_pad) {
    using G = Geometry<M, E>;
    constexpr int TT = G::T;
    constexpr int LP = G::npass() - 1;
    using IL = PassInfo<M, E, LP, kRegOsz>;
    static_assert(PassInfo<M, E, 1, kRegOsz>::R == E, "pass 1 must be radix E (pass-0 layout reads)");
    using O = typename OutT<OUT, float>::type;
    extern __shared__ __align__(16) unsigned char smem[];
    f2* lds = reinterpret_cast<f2*>(smem);
    const int t = threadIdx.x;
    const int b = blockIdx.x;
    const int xcd = b & 7;
    const int local = b >> 3;
    const int pos = local % (kTileFC * kTileGC);
    const int round = local / (kTileFC * kTileGC);
    const int nfr = (d.nfreq + kTileFC - 1) / kTileFC;
    const int fi = (round % nfr) * kTileFC + pos % kTileFC;
    const int sg = ((round / nfr) * kTileGC + pos / kTileFC) * 8 + xcd;
    if (fi >= d.nfreq || sg >= nsg_pad || (int64_t)sg * kGroupC >= nsig) return;
    const int64_t s_begin = (int64_t)sg * kGroupC;
    const int64_t s_end = min(nsig, s_begin + kGroupC);

    const int n = (int)d.n;
    const uint32_t n2 = 2u * (uint32_t)n;
    const float inv_n2 = 1.0f / (float)n2;
    const float* wrow = wtab + (int64_t)fi * n;
    Tab1<f2, M, E>::fill(lds, tw, t);
    for (int64_t s = s_begin; s < s_end; s += 2) {
        const bool two = s + 1 < s_end;
        const cplx<float>* X0 = X + s * d.nh;
        const cplx<float>* X1 = X + (two ? s + 1 : s) * d.nh;
        C2<f2> v[E];
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int k = t + r * TT;
            C2<f2> a{f2{0.f, 0.f}, f2{0.f, 0.f}};
            if (k < n) {
                const float w = wrow[k];
                const cplx<float> x0 = spectrum_bin<float>(X0, d, k), x1 = spectrum_bin<float>(X1, d, k);
                a = cmul(C2<f2>{f2{w * x0.re, w * x1.re}, f2{w * x0.im, w * x1.im}},
                         chirp<float>(k, n2, inv_n2, nullptr));
            }
            v[r] = C2<f2>{a.re, -a.im};
        }
        idft_br<f2, E, E / 2>(v);
        passes_regs<f2, M, E, 1>(v, lds, t, tw);
#pragma unroll
        for (int q = 0; q < IL::Q; ++q)
#pragma unroll
            for (int i = 0; i < IL::R; ++i) {
                const int m = t + q * TT + bitrev<IL::R>(i) * IL::NS;
                C2<f2>& e = v[q * IL::R + i];
                e = cmul(C2<f2>{e.re, -e.im}, bh[m]);
            }
        lds_barrier();
        lds_write<f2, M, E, LP, 0>(v, lds, t);
        lds_barrier();
        lds_read<f2, M, E, 1, 0, kRegOsz>(v, lds, t);
        lds_barrier();
        lds_write<f2, M, E, LP, 1>(v, lds, t);
        lds_barrier();
        lds_read<f2, M, E, 1, 1, kRegOsz>(v, lds, t);
        idft_br<f2, E>(v);
        passes_regs<f2, M, E, 1>(v, lds, t, tw);
        O* o0 = reinterpret_cast<O*>(out) + (s * d.nfreq + fi) * (int64_t)n;
        O* o1 = reinterpret_cast<O*>(out) + ((s + 1) * d.nfreq + fi) * (int64_t)n;
#pragma unroll
        for (int q = 0; q < IL::Q; ++q)
#pragma unroll
            for (int i = 0; i < IL::R; ++i) {
                const int idx = t + q * TT + bitrev<IL::R>(i) * IL::NS;
                if (idx < n) {
                    const C2<f2> y = cmul(v[q * IL::R + i], chirp<float>(idx, n2, inv_n2, nullptr));
                    o0[idx] = out_value<OUT, float>(lo(y));
                    if (two) o1[idx] = out_value<OUT, float>(hi(y));
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

// Bh[m] = (1/M) sum_j b[j] exp(-2 pi i m j / M) with b symmetric (b[M-j] = b[j]), in fp64:
// (1/M) sum_{j<n} b[j] w_j cos(2 pi m j / M), w_0 = 1, w_j = 2; b[j] = exp(-i pi (j^2 mod 2n) / n)
template <typename T>
__global__ __launch_bounds__(256) void chirp_bhat_kernel(C2<T>* bh, C2<T>* ct, int n, int m_len) {
    const int m = blockIdx.x * 256 + threadIdx.x;
    if (m < n && ct) {
        double s, c;
        sincospi((double)(((int64_t)m * m) % (2 * (int64_t)n)) / n, &s, &c);
        ct[m] = C2<T>{(T)c, (T)s};
    }
    if (m >= m_len) return;
    double re = 0.0, im = 0.0;
    for (int j = 0; j < n; ++j) {
        double bs, bc;
        sincospi(-(double)(((int64_t)j * j) % (2 * (int64_t)n)) / n, &bs, &bc);
        const double cw = cospi(2.0 * (double)(((int64_t)m * j) % m_len) / m_len) * (j == 0 ? 1.0 : 2.0);
        re += bc * cw;
        im += bs * cw;
    }
    bh[m] = C2<T>{(T)(re / m_len), (T)(im / m_len)};
}

struct ChirpKey {
    int dev;
    int64_t n;
    int dtype;
    bool operator<(const ChirpKey& o) const { return std::tie(dev, n, dtype) < std::tie(o.dev, o.n, o.dtype); }
};
std::mutex g_chirp_mu;
std::map<ChirpKey, void*> g_chirp;   // Bh[M] then (fp64) c[n], per device and length

int64_t chirp_m(int64_t n) {
    int64_t m = 1024;
    while (m < 2 * n - 1) m <<= 1;
    return m;
}

hipError_t chirp_tables(int64_t n, int dtype, void** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_chirp_mu);
    auto it = g_chirp.find({dev, n, dtype});
    if (it != g_chirp.end()) {
        *out = it->second;
        return hipSuccess;
    }
    const int64_t m = chirp_m(n);
    const size_t esz = dtype == NW_F32 ? sizeof(C2<float>) : sizeof(C2<double>);
    void* p = nullptr;
    e = hipMalloc(&p, (size_t)(m + n) * esz);
    if (e != hipSuccess) return e;
    const unsigned blocks = (unsigned)((m + 255) / 256);
    if (dtype == NW_F32)
        chirp_bhat_kernel<float><<<blocks, 256>>>((C2<float>*)p, (C2<float>*)p + m, (int)n, (int)m);
    else
        chirp_bhat_kernel<double><<<blocks, 256>>>((C2<double>*)p, (C2<double>*)p + m, (int)n, (int)m);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        (void)hipFree(p);
        return e;
    }
    g_chirp[{dev, n, dtype}] = p;
    *out = p;
    return hipSuccess;
}

template <typename T, int M, int E, bool REALW>
hipError_t launch_m(const WDesc& d, int out_kind, const void* X, const void* wtab, void* out, int64_t nsig,
                    hipStream_t s) {
    constexpr int threads = M / E;
    const int lds = kLdsBytes<T, M, E>;
    void* tw = nullptr;
    hipError_t e = fused_twiddles(M, sizeof(T) == 4 ? NW_F32 : NW_F64, &tw);
    if (e != hipSuccess) return e;
    void* tabs = nullptr;
    e = chirp_tables(d.n, sizeof(T) == 4 ? NW_F32 : NW_F64, &tabs);
    if (e != hipSuccess) return e;
    const C2<T>* bh = reinterpret_cast<const C2<T>*>(tabs);
    const C2<T>* ct = bh + M;
    const int64_t nsg = (nsig + kGroupC - 1) / kGroupC;
    const int64_t nsg_pad = (nsg + 8 * kTileGC - 1) / (8 * kTileGC) * (8 * kTileGC);
    const int64_t nfr = (d.nfreq + kTileFC - 1) / kTileFC;
    const int64_t blocks = nsg_pad * nfr * kTileFC;
    if (blocks > 0x7fffffff || nsg_pad > 0x7fffffff) return hipErrorInvalidConfiguration;
    const cplx<T>* Xc = reinterpret_cast<const cplx<T>*>(X);
    const C2<T>* twc = reinterpret_cast<const C2<T>*>(tw);
    auto go = [&](auto kern) {
        e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return;
        kern<<<(unsigned)blocks, threads, lds, s>>>(d, Xc, wtab, out, twc, bh, ct, nsig, (int)nsg_pad);
        e = hipGetLastError();
    };
    if constexpr (std::is_same<T, float>::value && REALW && NW_CHIRP_PAIR && E <= 16 && M <= NW_CHIRP_PAIR_MAXM) {
        const int lp = kLdsBytes<f2, M, E>;
        const float* wt = reinterpret_cast<const float*>(wtab);
        auto gp = [&](auto kern) {
            e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lp);
            if (e != hipSuccess) return;
            kern<<<(unsigned)blocks, threads, lp, s>>>(d, Xc, wt, out, twc, bh, nsig, (int)nsg_pad);
            e = hipGetLastError();
        };
        if (out_kind == NW_OUT_CWT) gp(nw_chirp_pair_kernel<M, E, NW_OUT_CWT>);
        else if (out_kind == NW_OUT_POWER) gp(nw_chirp_pair_kernel<M, E, NW_OUT_POWER>);
        else gp(nw_chirp_pair_kernel<M, E, NW_OUT_ABS>);
        return e;
    }
    if (out_kind == NW_OUT_CWT) go(nw_chirp_kernel<T, M, E, NW_OUT_CWT, REALW>);
    else if (out_kind == NW_OUT_POWER) go(nw_chirp_kernel<T, M, E, NW_OUT_POWER, REALW>);
    else go(nw_chirp_kernel<T, M, E, NW_OUT_ABS, REALW>);
    return e;
}

}  // namespace

// (dtype, M, E) of the chirp engine: fp32 M <= 16384 (E = 32 at 16384), fp64 M <= 8192
#ifndef NW_CHIRP_E
#define NW_CHIRP_E 16   // elements per thread, fp32 M <= 8192
#endif
#define NW_CHIRP_TABLE(X)                                                                        \
    X(float, 1024, NW_CHIRP_E) X(float, 2048, NW_CHIRP_E) X(float, 4096, NW_CHIRP_E)             \
    X(float, 8192, NW_CHIRP_E) X(float, 16384, 32)                                               \
    X(double, 1024, 16) X(double, 2048, 16) X(double, 4096, 16) X(double, 8192, 16)

bool chirp_supported(int64_t n, int dtype) {
    if (n < 1 || fused_supported(n, dtype)) return false;
    const int64_t mmax = dtype == NW_F32 ? 16384 : 8192;
    return (dtype == NW_F32 || dtype == NW_F64) && 2 * n - 1 <= mmax;
}

size_t chirp_wtable_bytes(int64_t n, int nfreq, int dtype, int kind) {
    const size_t esz = dtype == NW_F32 ? sizeof(float) : sizeof(double);
    return (size_t)n * nfreq * esz * (kind != NW_TABLE ? 1 : 2);
}

hipError_t build_chirp_wtable(const WDesc& d, int dtype, void* wtab, hipStream_t s) {
    dim3 grid((unsigned)((d.n + 255) / 256), (unsigned)d.nfreq);
    const bool realw = d.kind != NW_TABLE;
    if (dtype == NW_F32) {
        if (realw) chirp_wtable_kernel<float, true><<<grid, 256, 0, s>>>(d, wtab);
        else chirp_wtable_kernel<float, false><<<grid, 256, 0, s>>>(d, wtab);
    } else {
        if (realw) chirp_wtable_kernel<double, true><<<grid, 256, 0, s>>>(d, wtab);
        else chirp_wtable_kernel<double, false><<<grid, 256, 0, s>>>(d, wtab);
    }
    return hipGetLastError();
}

hipError_t launch_chirp(const WDesc& d, int dtype, int out_kind, const void* X, const void* wtab, void* out,
                        int64_t nsig, hipStream_t s) {
    if (!chirp_supported(d.n, dtype)) return hipErrorNotSupported;
    const int64_t m = chirp_m(d.n);
    const bool realw = d.kind != NW_TABLE;
#define NW_CHIRP_LAUNCH(TY, MM, EE)                                                          \
    if (m == MM && dtype == (sizeof(TY) == 4 ? NW_F32 : NW_F64))                            \
        return realw ? launch_m<TY, MM, EE, true>(d, out_kind, X, wtab, out, nsig, s)        \
                     : launch_m<TY, MM, EE, false>(d, out_kind, X, wtab, out, nsig, s);
    NW_CHIRP_TABLE(NW_CHIRP_LAUNCH)
#undef NW_CHIRP_LAUNCH
    return hipErrorNotSupported;
}

}  // namespace nw
