// nw_fused.hip — the fused CWT engine for power-of-two n (gfx950).
//
// One workgroup owns one scale f and a group of G signals.  Per block:
//   1. W[f, k] is evaluated ONCE into registers for the thread's bins
//      k = t + r*T (analytic psi, or a table row), 1/n folded in;
//   2. per signal s: z = W * X[s] (X = R2C half spectrum in HBM, read through L2:
//      blocks on one XCD sweep the scales of the same signal group), then an
//      inverse Stockham FFT entirely on chip -- pass 0 in registers, the middle
//      passes exchanged through a padded LDS image, the last pass storing
//      straight to HBM: complex y, |y| or |y|^2 (reference base.py:378-443).
// HBM traffic is one write per output point plus X once per signal: the
// product W*X and the complex intermediate of |.|^2 never reach HBM.
//
// Stockham pass (radix R, Ns = product of earlier radices), butterfly j:
//   v[r] = src[j + r*N/R];  v[r] *= w^(r*(j mod Ns)), w = exp(+2 pi i/(Ns R));  v = IDFT_R(v)
//   dst[(j / Ns) * Ns * R + (j mod Ns) + r * Ns] = v[r]
// IDFT_R is a radix-2 decimation-in-frequency network in registers whose output
// comes out bit-reversed; stores index it with bitrev(i) (compile-time, free).
#include <map>
#include <mutex>
#include <tuple>

#include "nw_internal.h"

namespace nw {

namespace {

template <typename T> struct C2 {
    T re, im;
};

template <typename T> __device__ __forceinline__ C2<T> cmul(C2<T> a, C2<T> b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}

// --- memory ops addressed as wave-uniform base (SGPR pair) + 32-bit per-lane byte
// offset: `global_load/store ... v_off, s[base:base+1]` (saddr form), i.e. one VGPR
// per address instead of a 64-bit pair.  The empty asm makes the offset opaque so
// the compiler cannot re-associate constant parts back into 64-bit address math.
// (The raw_buffer_load/store_b64 builtins of this toolchain emit a single dword
// and are not used.)
template <typename P>
__device__ __forceinline__ P* at(P* base, uint32_t byte_off) {
    asm("" : "+v"(byte_off));
    return reinterpret_cast<P*>(reinterpret_cast<char*>(base) + byte_off);
}
template <typename P>
__device__ __forceinline__ const P* at(const P* base, uint32_t byte_off) {
    asm("" : "+v"(byte_off));
    return reinterpret_cast<const P*>(reinterpret_cast<const char*>(base) + byte_off);
}

// cos(2*pi*i/32), i = 0..31
__device__ constexpr double kCos32[32] = {
    1.0, 0.98078528040323043, 0.92387953251128674, 0.83146961230254524, 0.70710678118654757,
    0.55557023301960218, 0.38268343236508978, 0.19509032201612825, 0.0, -0.19509032201612825,
    -0.38268343236508978, -0.55557023301960218, -0.70710678118654757, -0.83146961230254524,
    -0.92387953251128674, -0.98078528040323043, -1.0, -0.98078528040323043, -0.92387953251128674,
    -0.83146961230254524, -0.70710678118654757, -0.55557023301960218, -0.38268343236508978,
    -0.19509032201612825, 0.0, 0.19509032201612825, 0.38268343236508978, 0.55557023301960218,
    0.70710678118654757, 0.83146961230254524, 0.92387953251128674, 0.98078528040323043};

// a * exp(+2 pi i K / LEN) for compile-time K, LEN (LEN | 32); trivial angles special-cased
template <typename T, int K, int LEN>
__device__ __forceinline__ C2<T> twc(C2<T> a) {
    constexpr int idx = K * (32 / LEN);
    if constexpr (idx == 0) {
        return a;
    } else if constexpr (idx == 8) {                  // +i
        return {-a.im, a.re};
    } else if constexpr (idx == 4) {                  // (1+i)/sqrt2
        constexpr T h = (T)0.70710678118654757;
        return {h * (a.re - a.im), h * (a.re + a.im)};
    } else if constexpr (idx == 12) {                 // (-1+i)/sqrt2
        constexpr T h = (T)0.70710678118654757;
        return {-h * (a.re + a.im), h * (a.re - a.im)};
    } else {
        constexpr T c = (T)kCos32[idx];
        constexpr T s = (T)kCos32[(idx + 24) % 32];   // sin(x) = cos(x - pi/2)
        return {a.re * c - a.im * s, a.re * s + a.im * c};
    }
}

template <int R> __host__ __device__ constexpr int bitrev(int i) {
    int r = 0;
    for (int b = 1; b < R; b <<= 1) {
        r = (r << 1) | (i & 1);
        i >>= 1;
    }
    return r;
}

// radix-2 DIF butterflies of one stage (half size H), unrolled by template recursion
template <typename T, int R, int H, int G, int K>
__device__ __forceinline__ void dif_bfly(C2<T>* a) {
    if constexpr (G < R) {
        if constexpr (K < H) {
            const C2<T> u = a[G + K], w = a[G + K + H];
            a[G + K] = {u.re + w.re, u.im + w.im};
            a[G + K + H] = twc<T, K, 2 * H>(C2<T>{u.re - w.re, u.im - w.im});
            dif_bfly<T, R, H, G, K + 1>(a);
        } else {
            dif_bfly<T, R, H, G + 2 * H, 0>(a);
        }
    }
}

template <typename T, int R, int H>
__device__ __forceinline__ void dif_stages(C2<T>* a) {
    if constexpr (H >= 1) {
        dif_bfly<T, R, H, 0, 0>(a);
        dif_stages<T, R, H / 2>(a);
    }
}

// inverse DFT of R registers, natural-order input, bit-reversed output
template <typename T, int R>
__device__ __forceinline__ void idft_br(C2<T>* v) {
    if constexpr (R > 1) dif_stages<T, R, R / 2>(v);
}

template <int R> constexpr int ilog2() { return R <= 1 ? 0 : 1 + ilog2<R / 2>(); }

// v[r] *= w^(r m), w = exp(2 pi i / NSR), r = 1..R-1.  The base powers w^(m 2^k)
// come from the exact table tw[i] = exp(2 pi i i / N) (L2-resident); every other
// power is a product of at most log2(R) of them: a few ulp, no recurrence drift.
template <typename T, int R, int N, int NSR>
__device__ __forceinline__ void twiddle(C2<T>* v, int m, const C2<T>* __restrict__ tw) {
    if constexpr (R > 1) {
        constexpr int LR = ilog2<R>();
        C2<T> p[LR];
#pragma unroll
        for (int k = 0; k < LR; ++k) p[k] = *at(tw, (uint32_t)((m << k) * (N / NSR) * sizeof(C2<T>)));
#pragma unroll
        for (int r = 1; r < R; ++r) {
            C2<T> w = p[__builtin_ctz(r)];
#pragma unroll
            for (int k = __builtin_ctz(r) + 1; k < LR; ++k)
                if (r & (1 << k)) w = cmul(w, p[k]);
            v[r] = cmul(v[r], w);
        }
    }
}

// Padded LDS half image (one real component at a time): 2 extra slots after
// every E slots (E = elements per thread).  The pass-0 scatter (thread t owns
// slots t*E .. t*E+E-1) then hits distinct banks with pair stores, pairs stay
// aligned, and every later access is base(thread) + compile-time offset because
// all strides are multiples of E.
template <int E> __device__ __forceinline__ int lds_idx(int i) { return i + 2 * (i / E); }
template <int E> constexpr int lds_off(int c) { return c + 2 * (c / E); }   // c a multiple of E
template <int N, int E> constexpr int lds_elems() { return N + 2 * (N / E); }

template <int N, int E> struct Geometry {
    static constexpr int T = N / E;                 // threads per block
    static constexpr int radix(int p) {             // radix of pass p; pass 0 has radix E
        int done = E;
        for (int i = 1; i < p; ++i) done *= (N / done >= E ? E : N / done);
        const int left = N / done;
        return p == 0 ? E : (left >= E ? E : left);
    }
    static constexpr int npass() {
        int done = E, p = 1;
        while (done < N) {
            done *= (N / done >= E ? E : N / done);
            ++p;
        }
        return p;
    }
    static constexpr int ns(int p) {                // Ns before pass p
        int done = 1;
        for (int i = 0; i < p; ++i) done *= radix(i);
        return done;
    }
};

// output value of one point: y, |y| or |y|^2
template <int OUT, typename T> struct OutT { using type = T; };
template <typename T> struct OutT<NW_OUT_CWT, T> { using type = C2<T>; };
template <int OUT, typename T>
__device__ __forceinline__ typename OutT<OUT, T>::type out_value(C2<T> y) {
    if constexpr (OUT == NW_OUT_CWT) return y;
    else if constexpr (OUT == NW_OUT_POWER) return y.re * y.re + y.im * y.im;
    else return (T)sqrt(y.re * y.re + y.im * y.im);
}

// store outputs idx, idx+1 of the current row (orow: wave-uniform row base) as ONE
// vector store (16 B for complex64, 8 B for float32, 2x16 B for complex128)
template <int OUT, typename T>
__device__ __forceinline__ void store_pair(void* orow, uint32_t idx, C2<T> y0, C2<T> y1) {
    using O = typename OutT<OUT, T>::type;
    struct alignas(2 * sizeof(O)) P2 { O a, b; };
#ifdef NW_ABL_NOSTORE
    asm volatile("" ::"v"(y0.re), "v"(y0.im), "v"(y1.re), "v"(y1.im), "v"(idx));
    return;
#endif
    *at(reinterpret_cast<P2*>(orow), idx * (uint32_t)sizeof(O)) = P2{out_value<OUT, T>(y0), out_value<OUT, T>(y1)};
}
template <int OUT, typename T>
__device__ __forceinline__ void store_one(void* orow, uint32_t idx, C2<T> y) {
    using O = typename OutT<OUT, T>::type;
#ifdef NW_ABL_NOSTORE
    asm volatile("" ::"v"(y.re), "v"(y.im), "v"(idx));
    return;
#endif
    *at(reinterpret_cast<O*>(orow), idx * (uint32_t)sizeof(O)) = out_value<OUT, T>(y);
}

// two adjacent real slots of the half image, one 8/16-byte LDS access
template <typename T> struct alignas(2 * sizeof(T)) Pair {
    T a, b;
};

template <int COMP, typename T> __device__ __forceinline__ T& comp(C2<T>& c) {
    if constexpr (COMP == 0) return c.re; else return c.im;
}

// ---- one component of the pass-P outputs -> LDS (P = 0: slots t*E + s, as pairs)
template <typename T, int N, int E, int P, int COMP>
__device__ __forceinline__ void lds_write(C2<T>* v, T* lds, int t) {
    using G = Geometry<N, E>;
    if constexpr (P == 0) {
        Pair<T>* dst = reinterpret_cast<Pair<T>*>(lds + lds_idx<E>(t * E));
#pragma unroll
        for (int u = 0; u < E / 2; ++u)
            dst[u] = Pair<T>{comp<COMP>(v[bitrev<E>(2 * u)]), comp<COMP>(v[bitrev<E>(2 * u + 1)])};
    } else {
        constexpr int R = G::radix(P);
        constexpr int NS = G::ns(P);
        constexpr int Q = E / R;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int j = t + q * G::T;
            T* dst = lds + lds_idx<E>((j / NS) * NS * R + j % NS);
#pragma unroll
            for (int i = 0; i < R; ++i) dst[lds_off<E>(bitrev<R>(i) * NS)] = comp<COMP>(v[q * R + i]);
        }
    }
}

// ---- one component of the pass-P inputs <- LDS.  Butterflies: j = t + q*T, except
// in the LAST pass, where j = Q*t + q so a thread's outputs come in adjacent pairs.
template <int N, int E, int P> struct PassInfo {
    using G = Geometry<N, E>;
    static constexpr int R = G::radix(P);
    static constexpr int NS = G::ns(P);
    static constexpr int Q = E / R;
    static constexpr int STRIDE = N / R;
    static constexpr bool LAST = (P == G::npass() - 1);
    static constexpr bool PAIRED = LAST && Q >= 2;
    static_assert(STRIDE % E == 0 && NS % E == 0, "pad must stay linear");
    __device__ static __forceinline__ int bfly(int t, int q) { return PAIRED ? Q * t + q : t + q * G::T; }
};

template <typename T, int N, int E, int P, int COMP>
__device__ __forceinline__ void lds_read(C2<T>* v, const T* lds, int t) {
    using I = PassInfo<N, E, P>;
    constexpr int R = I::R, Q = I::Q;
    if constexpr (I::PAIRED) {
        const T* src = lds + lds_idx<E>(Q * t);
#pragma unroll
        for (int q = 0; q < Q; q += 2)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const Pair<T> pr = *reinterpret_cast<const Pair<T>*>(src + q + lds_off<E>(r * I::STRIDE));
                comp<COMP>(v[q * R + r]) = pr.a;
                comp<COMP>(v[(q + 1) * R + r]) = pr.b;
            }
    } else {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const T* src = lds + lds_idx<E>(t + q * Geometry<N, E>::T);
#pragma unroll
            for (int r = 0; r < R; ++r) comp<COMP>(v[q * R + r]) = src[lds_off<E>(r * I::STRIDE)];
        }
    }
}

// ---- exchange pass P-1 -> P through the half image (re, then im), then compute pass P
template <typename T, int N, int E, int OUT, int P>
__device__ __forceinline__ void passes_from(C2<T>* v, T* lds, int t, void* orow, const C2<T>* __restrict__ tw) {
    using I = PassInfo<N, E, P>;
    if constexpr (P < Geometry<N, E>::npass()) {
        constexpr int R = I::R, Q = I::Q;
        __syncthreads();                       // earlier readers of the image are done
        lds_write<T, N, E, P - 1, 0>(v, lds, t);
        __syncthreads();
        lds_read<T, N, E, P, 0>(v, lds, t);
        __syncthreads();
        lds_write<T, N, E, P - 1, 1>(v, lds, t);
        __syncthreads();
        lds_read<T, N, E, P, 1>(v, lds, t);
#pragma unroll
        for (int q = 0; q < Q; ++q) {
#ifndef NW_ABL_NOTWIDDLE
            twiddle<T, R, N, I::NS * R>(v + q * R, I::bfly(t, q) % I::NS, tw);
#endif
            idft_br<T, R>(v + q * R);
        }
        if constexpr (I::LAST) {
            // NS * R == N: the output index of (j, r) is j + r*NS
#pragma unroll
            for (int q = 0; q < Q; q += (I::PAIRED ? 2 : 1))
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    const uint32_t k = (uint32_t)(I::bfly(t, q) + bitrev<R>(i) * I::NS);
                    if constexpr (I::PAIRED)
                        store_pair<OUT, T>(orow, k, v[q * R + i], v[(q + 1) * R + i]);
                    else
                        store_one<OUT, T>(orow, k, v[q * R + i]);
                }
        } else {
            passes_from<T, N, E, OUT, P + 1>(v, lds, t, orow, tw);
        }
    }
}

template <typename T, bool REALW> struct WLoad;
template <typename T> struct WLoad<T, true> {     // analytic wavelets: real rows
    using type = T;
    __device__ static __forceinline__ C2<T> apply(T w, C2<T> x) { return {w * x.re, w * x.im}; }
};
template <typename T> struct WLoad<T, false> {    // table wavelets: complex rows
    using type = C2<T>;
    __device__ static __forceinline__ C2<T> apply(C2<T> w, C2<T> x) { return cmul(w, x); }
};

// Occupancy target (waves per SIMD).  E = 16: 4 (<= 128 VGPRs; the small half images
// let several blocks share a CU, so one block's barriers and memory waits overlap
// another's arithmetic).  E = 32 (n = 16384 fp32): one signal occupies 128 KiB of
// registers, so 2 (<= 256 VGPRs); capping it at 128 spills (measured 1.6x slower).
#ifndef NW_WAVES_PER_SIMD
#define NW_WAVES_PER_SIMD(E) ((E) >= 32 ? 2 : 4)
#endif
template <typename T, int N, int E, int OUT, bool REALW>
__global__ __launch_bounds__(N / E, NW_WAVES_PER_SIMD(E)) void nw_fused_kernel(WDesc d, const cplx<T>* __restrict__ X,
                                                            const void* __restrict__ wtab, void* __restrict__ out,
                                                            const C2<T>* __restrict__ tw, int64_t nsig, int group,
                                                            int nsg_pad) {
    using G = Geometry<N, E>;
    using WT = typename WLoad<T, REALW>::type;
    extern __shared__ __align__(16) unsigned char smem[];
    T* lds = reinterpret_cast<T*>(smem);
    const int t = threadIdx.x;

    // XCD-aware block -> (scale, signal group): blocks b, b+8, b+16, ... share an
    // XCD (and its L2) and walk the scales of ONE signal group, so X[s] is
    // fetched from HBM once and re-read from L2 for every scale.
    const int b = blockIdx.x;
    const int xcd = b & 7;
    const int qb = b >> 3;
    const int fi = qb % d.nfreq;
    const int sg = (qb / d.nfreq) * 8 + xcd;
    if (sg >= nsg_pad || (int64_t)sg * group >= nsig) return;
    const int64_t s_begin = (int64_t)sg * group;
    const int64_t s_end = min(nsig, s_begin + group);
    const WT* wrow = reinterpret_cast<const WT*>(wtab) + (int64_t)fi * N;   // W[f, :] incl. pad_to and 1/n

    for (int64_t s = s_begin; s < s_end; ++s) {
        const C2<T>* xs = reinterpret_cast<const C2<T>*>(X + s * d.nh);
        C2<T> v[E];
        // pass 0 (Ns = 1): z = W * X at k = t + r*T, radix-E IDFT in registers.
        // k < N/2 exactly when r < E/2 (compile-time), so the half-spectrum read needs
        // no branch: X[k], or conj(X[N - k]) above N/2 (at k = N/2 the bin is real).
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const uint32_t k = (uint32_t)(t + r * G::T);
            C2<T> x;
#ifdef NW_ABL_NOXLOAD
            x = {(T)(t + r), (T)r};
            asm volatile("" : "+v"(x.re), "+v"(x.im));
#else
            if (r < E / 2) {
                x = *at(xs, k * (uint32_t)sizeof(C2<T>));
            } else {
                x = *at(xs, ((uint32_t)N - k) * (uint32_t)sizeof(C2<T>));
                x.im = -x.im;
            }
#endif
            const bool keep = (int64_t)k < d.xlim;     // interpolate_alias mask
            x.re = keep ? x.re : T(0);
            x.im = keep ? x.im : T(0);
            v[r] = WLoad<T, REALW>::apply(*at(wrow, k * (uint32_t)sizeof(WT)), x);
        }
        idft_br<T, E>(v);
        const int64_t row = (s * d.nfreq + fi) * (int64_t)N;
        void* orow = (char*)out + row * (int64_t)(OUT == NW_OUT_CWT ? sizeof(C2<T>) : sizeof(T));
        passes_from<T, N, E, OUT, 1>(v, lds, t, orow, tw);
    }
}

// W[f, k] for the fused engine: the reference's cached row, pad_to'd to n, 1/n folded
// in (real rows for analytic kinds, complex for tables).  Built once per plan+wavelet.
template <typename T, bool REALW>
__global__ __launch_bounds__(256) void wtable_kernel(WDesc d, void* wtab) {
    const int fi = blockIdx.y;
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= d.n) return;
    const cplx<T> w = wavelet_bin<T>(d, fi, k);
    if constexpr (REALW)
        reinterpret_cast<T*>(wtab)[(int64_t)fi * d.n + k] = w.re;
    else
        reinterpret_cast<C2<T>*>(wtab)[(int64_t)fi * d.n + k] = C2<T>{w.re, w.im};
}

template <typename T>
__global__ void twiddle_table_kernel(C2<T>* tw, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        double s, c;
        sincospi(2.0 * (double)i / (double)n, &s, &c);
        tw[i] = {(T)c, (T)s};
    }
}

struct TwKey {
    int dev;
    int64_t n;
    int dtype;
    bool operator<(const TwKey& o) const { return std::tie(dev, n, dtype) < std::tie(o.dev, o.n, o.dtype); }
};
std::mutex g_tw_mu;
std::map<TwKey, void*> g_tw;

hipError_t twiddles_for(int64_t n, int dtype, void** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_tw_mu);
    auto it = g_tw.find({dev, n, dtype});
    if (it != g_tw.end()) {
        *out = it->second;
        return hipSuccess;
    }
    const size_t esz = dtype == NW_F32 ? sizeof(C2<float>) : sizeof(C2<double>);
    void* p = nullptr;
    e = hipMalloc(&p, (size_t)n * esz);
    if (e != hipSuccess) return e;
    if (dtype == NW_F32)
        twiddle_table_kernel<float><<<(unsigned)((n + 255) / 256), 256>>>((C2<float>*)p, (int)n);
    else
        twiddle_table_kernel<double><<<(unsigned)((n + 255) / 256), 256>>>((C2<double>*)p, (int)n);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        (void)hipFree(p);
        return e;
    }
    g_tw[{dev, n, dtype}] = p;
    *out = p;
    return hipSuccess;
}

constexpr int kGroup = 8;   // signals per block

template <typename T, int N, int E, bool REALW>
hipError_t launch_n(const WDesc& d, int out_kind, const void* X, const void* wtab, void* out, int64_t nsig,
                    hipStream_t s) {
    constexpr int threads = N / E;
    const size_t lds = (size_t)lds_elems<N, E>() * sizeof(T);
    void* tw = nullptr;
    hipError_t e = twiddles_for(N, sizeof(T) == 4 ? NW_F32 : NW_F64, &tw);
    if (e != hipSuccess) return e;
    const int64_t nsg = (nsig + kGroup - 1) / kGroup;
    const int64_t nsg_pad = (nsg + 7) / 8 * 8;
    const int64_t blocks = nsg_pad * d.nfreq;
    if (blocks > 0x7fffffff || nsg_pad > 0x7fffffff) return hipErrorInvalidConfiguration;
    const cplx<T>* Xc = reinterpret_cast<const cplx<T>*>(X);
    const C2<T>* twc_ = reinterpret_cast<const C2<T>*>(tw);
    if (out_kind == NW_OUT_CWT)
        nw_fused_kernel<T, N, E, NW_OUT_CWT, REALW><<<blocks, threads, lds, s>>>(d, Xc, wtab, out, twc_, nsig, kGroup, (int)nsg_pad);
    else if (out_kind == NW_OUT_POWER)
        nw_fused_kernel<T, N, E, NW_OUT_POWER, REALW><<<blocks, threads, lds, s>>>(d, Xc, wtab, out, twc_, nsig, kGroup, (int)nsg_pad);
    else
        nw_fused_kernel<T, N, E, NW_OUT_ABS, REALW><<<blocks, threads, lds, s>>>(d, Xc, wtab, out, twc_, nsig, kGroup, (int)nsg_pad);
    return hipGetLastError();
}

template <typename T, int N, int E, bool REALW>
hipError_t prepare_one() {
    const int lds = (int)(lds_elems<N, E>() * sizeof(T));
    hipError_t e = hipFuncSetAttribute((const void*)nw_fused_kernel<T, N, E, NW_OUT_CWT, REALW>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)nw_fused_kernel<T, N, E, NW_OUT_POWER, REALW>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)nw_fused_kernel<T, N, E, NW_OUT_ABS, REALW>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    return e;
}

template <typename T, int N, int E>
hipError_t prepare_n() {
    hipError_t e = prepare_one<T, N, E, true>();
    if (e == hipSuccess) e = prepare_one<T, N, E, false>();
    void* tw = nullptr;
    if (e == hipSuccess) e = twiddles_for(N, sizeof(T) == 4 ? NW_F32 : NW_F64, &tw);
    return e;
}

}  // namespace

#ifndef NW_E16384
#define NW_E16384 32   // elements per thread at n = 16384 fp32 (512 threads)
#endif

// power-of-two n from 2^10 to 2^14, fp32 and fp64 (half image <= 144 KiB)
bool fused_supported(int64_t n, int dtype) {
    if (n < 1024 || n > 16384 || (n & (n - 1))) return false;
    return dtype == NW_F32 || dtype == NW_F64;
}

#define NW_FUSED_TABLE(X)                                                               \
    X(float, 1024, 16) X(float, 2048, 16) X(float, 4096, 16) X(float, 8192, 16)        \
    X(float, 16384, NW_E16384) X(double, 1024, 16) X(double, 2048, 16) X(double, 4096, 16) \
    X(double, 8192, 16) X(double, 16384, 16)

hipError_t fused_prepare(int64_t n, int dtype) {
#define NW_PREP(TY, NN, EE) \
    if (n == NN && dtype == (sizeof(TY) == 4 ? NW_F32 : NW_F64)) return prepare_n<TY, NN, EE>();
    NW_FUSED_TABLE(NW_PREP)
#undef NW_PREP
    return hipErrorNotSupported;
}

size_t fused_wtable_bytes(int64_t n, int nfreq, int dtype, int kind) {
    const size_t esz = dtype == NW_F32 ? sizeof(float) : sizeof(double);
    return (size_t)n * nfreq * esz * (kind == NW_TABLE ? 2 : 1);
}

hipError_t build_wtable(const WDesc& d, int dtype, void* wtab, hipStream_t s) {
    dim3 grid((unsigned)((d.n + 255) / 256), (unsigned)d.nfreq);
    const bool realw = d.kind != NW_TABLE;
    if (dtype == NW_F32) {
        if (realw) wtable_kernel<float, true><<<grid, 256, 0, s>>>(d, wtab);
        else wtable_kernel<float, false><<<grid, 256, 0, s>>>(d, wtab);
    } else {
        if (realw) wtable_kernel<double, true><<<grid, 256, 0, s>>>(d, wtab);
        else wtable_kernel<double, false><<<grid, 256, 0, s>>>(d, wtab);
    }
    return hipGetLastError();
}

hipError_t launch_fused(const WDesc& d, int dtype, int out_kind, const void* X, const void* wtab, void* out,
                        int64_t nsig, hipStream_t s) {
    const bool realw = d.kind != NW_TABLE;
#define NW_LAUNCH(TY, NN, EE)                                                                 \
    if (d.n == NN && dtype == (sizeof(TY) == 4 ? NW_F32 : NW_F64))                            \
        return realw ? launch_n<TY, NN, EE, true>(d, out_kind, X, wtab, out, nsig, s)         \
                     : launch_n<TY, NN, EE, false>(d, out_kind, X, wtab, out, nsig, s);
    NW_FUSED_TABLE(NW_LAUNCH)
#undef NW_LAUNCH
    return hipErrorNotSupported;
}

}  // namespace nw
