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

// padded LDS image: one extra element every 32 keeps the Ns=1 scatter conflict-free
__device__ __forceinline__ int lds_idx(int i) { return i + (i >> 5); }

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

// one output point of the current row (orow = wave-uniform row base)
template <int OUT, typename T>
__device__ __forceinline__ void store_out(void* orow, uint32_t idx, C2<T> y) {
    if constexpr (OUT == NW_OUT_CWT) {
        *at(reinterpret_cast<C2<T>*>(orow), idx * (uint32_t)sizeof(C2<T>)) = y;
    } else if constexpr (OUT == NW_OUT_POWER) {
        *at(reinterpret_cast<T*>(orow), idx * (uint32_t)sizeof(T)) = y.re * y.re + y.im * y.im;
    } else {
        *at(reinterpret_cast<T*>(orow), idx * (uint32_t)sizeof(T)) = (T)sqrt(y.re * y.re + y.im * y.im);
    }
}

// Stockham pass P >= 1: read the LDS image, twiddle, IDFT, write LDS (or HBM if last).
// Every LDS access is base(thread) + compile-time offset: with the 1-in-32 pad,
// lds_idx(a + c) = lds_idx(a) + c + c/32 whenever c is a multiple of 32, and for
// NS < 32 the pad of d0 + r*NS splits into a per-thread and a per-r part.
template <typename T, int N, int E, int P, int OUT>
__device__ __forceinline__ void stockham_pass(C2<T>* v, C2<T>* lds, int t, void* orow,
                                              const C2<T>* __restrict__ tw) {
    using G = Geometry<N, E>;
    constexpr int R = G::radix(P);
    constexpr int NS = G::ns(P);
    constexpr int Q = E / R;             // butterflies per thread
    constexpr int STRIDE = N / R;        // a multiple of 32 for every supported geometry
    constexpr bool LAST = (P == G::npass() - 1);
    static_assert(STRIDE % 32 == 0, "read stride must keep the pad linear");
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const C2<T>* src = lds + lds_idx(t + q * G::T);
#pragma unroll
        for (int r = 0; r < R; ++r) v[q * R + r] = src[r * (STRIDE + STRIDE / 32)];
    }
    __syncthreads();   // every read of this pass done before the image is overwritten
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int j = t + q * G::T;
        const int m = j % NS;
        twiddle<T, R, N, NS * R>(v + q * R, m, tw);
        idft_br<T, R>(v + q * R);
        const int d0 = (j / NS) * NS * R + m;
        if constexpr (LAST) {
            // NS * R == N here, so d0 == j: row-contiguous stores across the wave
#pragma unroll
            for (int i = 0; i < R; ++i)
                store_out<OUT, T>(orow, (uint32_t)(d0 + bitrev<R>(i) * NS), v[q * R + i]);
        } else {
            C2<T>* dst;
            if constexpr (NS % 32 == 0)
                dst = lds + lds_idx(d0);
            else
                dst = lds + d0 + (((j / NS) * NS * R) >> 5);
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const int c = bitrev<R>(i) * NS;
                dst[(NS % 32 == 0) ? c + c / 32 : c + (c >> 5)] = v[q * R + i];
            }
        }
    }
    if constexpr (!LAST) __syncthreads();
}

template <typename T, int N, int E, int OUT, int P>
__device__ __forceinline__ void run_passes(C2<T>* v, C2<T>* lds, int t, void* orow,
                                           const C2<T>* __restrict__ tw) {
    using G = Geometry<N, E>;
    if constexpr (P < G::npass()) {
        stockham_pass<T, N, E, P, OUT>(v, lds, t, orow, tw);
        run_passes<T, N, E, OUT, P + 1>(v, lds, t, orow, tw);
    }
}

template <typename T, bool REALW> struct WReg;
template <typename T> struct WReg<T, true> {
    T re;
    __device__ __forceinline__ void set(cplx<T> w) { re = w.re; }
    __device__ __forceinline__ C2<T> apply(cplx<T> x) const { return {re * x.re, re * x.im}; }
};
template <typename T> struct WReg<T, false> {
    T re, im;
    __device__ __forceinline__ void set(cplx<T> w) { re = w.re; im = w.im; }
    __device__ __forceinline__ C2<T> apply(cplx<T> x) const {
        return {re * x.re - im * x.im, re * x.im + im * x.re};
    }
};

template <typename T, int N, int E, int OUT, bool REALW>
__global__ __launch_bounds__(N / E) void nw_fused_kernel(WDesc d, const cplx<T>* __restrict__ X, void* __restrict__ out,
                                                         const C2<T>* __restrict__ tw, int64_t nsig, int group,
                                                         int nsg_pad) {
    using G = Geometry<N, E>;
    extern __shared__ __align__(16) unsigned char smem[];
    C2<T>* lds = reinterpret_cast<C2<T>*>(smem);
    const int t = threadIdx.x;

    // XCD-aware block -> (scale, signal group): blocks b, b+8, b+16, ... share an
    // XCD (and its L2) and walk the scales of ONE signal group, so X[s] is
    // fetched from HBM once and re-read from L2 for every scale.
    const int b = blockIdx.x;
    const int xcd = b & 7;
    const int q = b >> 3;
    const int fi = q % d.nfreq;
    const int sg = (q / d.nfreq) * 8 + xcd;
    if (sg >= nsg_pad || (int64_t)sg * group >= nsig) return;
    const int64_t s_begin = (int64_t)sg * group;
    const int64_t s_end = min(nsig, s_begin + group);

    // 1. wavelet bins of this thread, evaluated once per block (1/n folded in)
    WReg<T, REALW> w[E];
#pragma unroll
    for (int r = 0; r < E; ++r) w[r].set(wavelet_bin<T>(d, fi, t + r * G::T));

    for (int64_t s = s_begin; s < s_end; ++s) {
        const C2<T>* xs = reinterpret_cast<const C2<T>*>(X + s * d.nh);
        C2<T> v[E];
        // 2. pass 0 (Ns = 1): z = W * X at k = t + r*T, radix-E IDFT in registers.
        //    k < N/2 exactly when r < E/2 (compile-time), so the half-spectrum read
        //    needs no branch: X[k] directly, or conj(X[N - k]) for the upper half
        //    (N - k <= N/2 < nh; at k = N/2 the Nyquist bin is real).
#pragma unroll
        for (int r = 0; r < E; ++r) {
            C2<T> x;
            if (r < E / 2) {
                x = *at(xs, (uint32_t)(t + r * G::T) * (uint32_t)sizeof(C2<T>));
            } else {
                x = *at(xs, (uint32_t)(N - t - r * G::T) * (uint32_t)sizeof(C2<T>));
                x.im = -x.im;
            }
            const bool keep = t + r * G::T < d.xlim;     // interpolate_alias mask
            x.re = keep ? x.re : T(0);
            x.im = keep ? x.im : T(0);
            v[r] = w[r].apply(cplx<T>{x.re, x.im});
        }
        idft_br<T, E>(v);
        {   // E | 32, so (t*E + i) >> 5 == (t*E) >> 5 for i < E
            C2<T>* dst = lds + t * E + ((t * E) >> 5);
#pragma unroll
            for (int i = 0; i < E; ++i) dst[bitrev<E>(i)] = v[i];
        }
        __syncthreads();
        const int64_t row = (s * d.nfreq + fi) * (int64_t)N;
        void* orow = (char*)out + row * (int64_t)(OUT == NW_OUT_CWT ? sizeof(C2<T>) : sizeof(T));
        run_passes<T, N, E, OUT, 1>(v, lds, t, orow, tw);
        __syncthreads();   // the last pass's LDS reads finish before the next signal's scatter
    }
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
hipError_t launch_n(const WDesc& d, int out_kind, const void* X, void* out, int64_t nsig, hipStream_t s) {
    constexpr int threads = N / E;
    const size_t lds = (size_t)(N + N / 32) * sizeof(C2<T>);
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
        nw_fused_kernel<T, N, E, NW_OUT_CWT, REALW><<<blocks, threads, lds, s>>>(d, Xc, out, twc_, nsig, kGroup, (int)nsg_pad);
    else if (out_kind == NW_OUT_POWER)
        nw_fused_kernel<T, N, E, NW_OUT_POWER, REALW><<<blocks, threads, lds, s>>>(d, Xc, out, twc_, nsig, kGroup, (int)nsg_pad);
    else
        nw_fused_kernel<T, N, E, NW_OUT_ABS, REALW><<<blocks, threads, lds, s>>>(d, Xc, out, twc_, nsig, kGroup, (int)nsg_pad);
    return hipGetLastError();
}

template <typename T, int N, int E, bool REALW>
hipError_t prepare_one() {
    const int lds = (int)((N + N / 32) * sizeof(C2<T>));
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

// fp32: 2^10..2^14, fp64: 2^10..2^13 (the padded LDS image is <= 132 KiB)
bool fused_supported(int64_t n, int dtype) {
    if (n < 1024 || (n & (n - 1))) return false;
    return dtype == NW_F32 ? n <= 16384 : n <= 8192;
}

#define NW_FUSED_TABLE(X)                                                           \
    X(float, 1024, 16) X(float, 2048, 16) X(float, 4096, 16) X(float, 8192, 16)    \
    X(float, 16384, 32) X(double, 1024, 16) X(double, 2048, 16) X(double, 4096, 16) \
    X(double, 8192, 16)

hipError_t fused_prepare(int64_t n, int dtype) {
#define NW_PREP(TY, NN, EE) \
    if (n == NN && dtype == (sizeof(TY) == 4 ? NW_F32 : NW_F64)) return prepare_n<TY, NN, EE>();
    NW_FUSED_TABLE(NW_PREP)
#undef NW_PREP
    return hipErrorNotSupported;
}

hipError_t launch_fused(const WDesc& d, int dtype, int out_kind, const void* X, void* out, int64_t nsig,
                        hipStream_t s) {
    const bool realw = d.kind != NW_TABLE;
#define NW_LAUNCH(TY, NN, EE)                                                           \
    if (d.n == NN && dtype == (sizeof(TY) == 4 ? NW_F32 : NW_F64))                      \
        return realw ? launch_n<TY, NN, EE, true>(d, out_kind, X, out, nsig, s)         \
                     : launch_n<TY, NN, EE, false>(d, out_kind, X, out, nsig, s);
    NW_FUSED_TABLE(NW_LAUNCH)
#undef NW_LAUNCH
    return hipErrorNotSupported;
}

}  // namespace nw
