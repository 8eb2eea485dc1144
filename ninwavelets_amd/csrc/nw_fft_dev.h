// nw_fft_dev.h — device building blocks of the on-chip inverse FFT engines (gfx950):
// complex helpers, register radix-2 DIF networks, twiddles (v_sin/v_cos or exact table),
// the padded half-image LDS exchange, Stockham pass geometry, LDS-DMA, DPP transposes
// and the last-pass store forms.  Included by nw_fused.hip (n <= 16384) and
// nw_large.hip (the two-pass engine for n up to 2^24); header-only device templates.
#pragma once

#include <type_traits>

#include "nw_dcheck.h"
#include "nw_internal.h"

// Tuning constants; each was measured against its alternatives (numbers in DESIGN.md §4).
// unpaired last pass: lane-pair transposes (DPP) regroup outputs of <= 8 B into 16-B stores
// (pairs of 8-B outputs: n = 4096 cwt 0.413 -> 0.403 ms); 4-B outputs stay single stores
// (quads: 0.337 -> 0.360 ms at n = 4096 power, pairs: C3 1.253 -> 1.277 ms)
#ifndef NW_PACK_MAX   // diagnostic A/B (-DNW_PACK_MAX=4: quad-packed 4-B outputs)
#define NW_PACK_MAX 2
#endif
constexpr int kPackMax = NW_PACK_MAX;
// smallest pass-0 variant: a W row's support is rounded up to it (1 and 2 add code without a
// measurable gain)
constexpr int kPruneMin = 4;
// fp32 kernels with E >= this take the next signal's X by LDS-DMA into the idle image before
// the stores (E = 32: 1.99 -> 1.94 ms; E = 16: 0.362 -> 0.386 ms, so not there)
constexpr int kXdmaMinE = 32;
// W held in registers for the whole block when E <= this
constexpr int kWregMaxE = 16;


namespace nw {
namespace {


template <typename T> struct C2 {
    T re, im;
};

// two fp32 lanes of one VGPR pair: C2<f2> is a PAIR of complex numbers (a.re, b.re),
// (a.im, b.im) on which every DIF / twiddle template runs as packed math
// (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32: two fp32 operations per instruction)
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ C2<f2> pk(C2<float> a, C2<float> b) { return {f2{a.re, b.re}, f2{a.im, b.im}}; }
__device__ __forceinline__ C2<float> lo(C2<f2> p) { return {p.re.x, p.im.x}; }
__device__ __forceinline__ C2<float> hi(C2<f2> p) { return {p.re.y, p.im.y}; }

// a rounded product that the compiler may not fuse into a following add
__device__ __forceinline__ double mul_nocontract(double a, double b) {
#pragma clang fp contract(off)
    return a * b;
}

template <typename T> __device__ __forceinline__ C2<T> cmul(C2<T> a, C2<T> b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
// a pair of complex numbers (two signals) times one complex number (a shared twiddle):
// the scalar operand is splat across both halves of every packed op
__device__ __forceinline__ C2<f2> cmul(C2<f2> a, C2<float> b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}

// scalar type of a lane value: C2<f2> carries two signals' values of one float element
template <typename T> struct ScalarOf { using type = T; };
template <> struct ScalarOf<f2> { using type = float; };
template <typename T> using Sc = typename ScalarOf<T>::type;

// --- memory ops addressed as wave-uniform base (SGPR pair) + 32-bit per-lane byte
// offset: `global_load/store ... v_off, s[base:base+1]` (saddr form), i.e. one VGPR
// per address instead of a 64-bit pair.  The empty asm makes the offset opaque so
// the compiler cannot re-associate constant parts back into 64-bit address math.
// (The raw_buffer_load/store_b64 builtins of this toolchain emit a single dword
// and are not used.)
//
// `lane_off` is a per-thread byte offset shared by many accesses and `c` a
// compile-time byte offset.  The volatile asm re-materialises lane_off at every
// use, so neither it nor lane_off + c can be hoisted out of the signal loop as a
// per-element loop invariant (which left ~100 live offsets and spilled).
template <typename P>
__device__ __forceinline__ P* at(P* base, uint32_t lane_off, uint32_t c = 0) {
    asm volatile("" : "+v"(lane_off));
    return reinterpret_cast<P*>(reinterpret_cast<char*>(base) + (lane_off + c));
}
template <typename P>
__device__ __forceinline__ const P* at(const P* base, uint32_t lane_off, uint32_t c = 0) {
    asm volatile("" : "+v"(lane_off));
    return reinterpret_cast<const P*>(reinterpret_cast<const char*>(base) + (lane_off + c));
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

// radix-2 DIF butterflies of one stage (half size H), unrolled by template recursion.
// NZ: only the first NZ elements of every group of 2H are nonzero (pruned inputs): a
// butterfly whose partner is zero is a copy plus a twiddle, one with both zero is skipped
// (exact: u + 0 = u), and every group keeps a nonzero prefix of min(NZ, H) after the stage.
template <typename T, int R, int H, int G, int K, int NZ>
__device__ __forceinline__ void dif_bfly(C2<T>* a) {
    if constexpr (G < R) {
        if constexpr (K < H) {
            if constexpr (K + H < NZ) {
                const C2<T> u = a[G + K], w = a[G + K + H];
                a[G + K] = {u.re + w.re, u.im + w.im};
                a[G + K + H] = twc<T, K, 2 * H>(C2<T>{u.re - w.re, u.im - w.im});
            } else if constexpr (K < NZ) {
                a[G + K + H] = twc<T, K, 2 * H>(a[G + K]);
            }
            dif_bfly<T, R, H, G, K + 1, NZ>(a);
        } else {
            dif_bfly<T, R, H, G + 2 * H, 0, NZ>(a);
        }
    }
}

template <typename T, int R, int H, int NZ>
__device__ __forceinline__ void dif_stages(C2<T>* a) {
    if constexpr (H >= 1) {
        dif_bfly<T, R, H, 0, 0, NZ>(a);
        dif_stages<T, R, H / 2, (NZ < H ? NZ : H)>(a);
    }
}

// inverse DFT of R registers, natural-order input, bit-reversed output; inputs r >= NZ
// are zero (their registers must hold zeros)
template <typename T, int R, int NZ = R>
__device__ __forceinline__ void idft_br(C2<T>* v) {
    if constexpr (R > 1) dif_stages<T, R, R / 2, NZ>(v);
}

template <int R> constexpr int ilog2() { return R <= 1 ? 0 : 1 + ilog2<R / 2>(); }

// v[r] *= w^(r m), w = exp(2 pi i / NSR), r = 1..R-1.  The base powers w^(m 2^k)
// come from the exact table tw[i] = exp(2 pi i i / N) (L2-resident); every other
// power is a product of at most log2(R) of them: a few ulp, no recurrence drift.
// The bases are loaded a phase ahead of use (before the LDS exchange that feeds
// the pass) so the table latency hides under the exchange.
template <typename T, int R, int N, int NSR, bool SPLIT = false>
__device__ __forceinline__ void twiddle_bases(C2<T>* p, int m, const C2<T>* __restrict__ tw,
                                              const C2<T>* split = nullptr) {
    // the twiddles depend on the thread only: keep the compiler from hoisting all of
    // them out of the signal loop (that keeps ~120 values live and spills)
    asm volatile("" : "+v"(m));
#pragma unroll
    for (int k = 0; k < ilog2<R>(); ++k) {
        if constexpr (SPLIT) {
            // w_N^i = hi[i >> 5] * lo[i & 31] from the LDS split table (TwSplit), i < N/2
            const uint32_t i = ((uint32_t)m << k) * (uint32_t)(N / NSR);
            p[k] = cmul(split[i >> 5], split[N / 64 + (i & 31)]);
        } else if constexpr (sizeof(T) == 4) {
            // v_cos/v_sin take revolutions; (m << k) / NSR is exact in fp32 (power-of-two
            // denominator), measured max abs error 1.2e-7 over all 16384 angles: no memory
            // access, so nothing queues behind this wave's in-flight stores
            const float rev = (float)(m << k) * (1.0f / (float)NSR);
            p[k] = C2<T>{__builtin_amdgcn_cosf(rev), __builtin_amdgcn_sinf(rev)};
        } else {
            p[k] = *at(tw, (uint32_t)m * (uint32_t)((N / NSR) * sizeof(C2<T>)) << k);
        }
    }
}
template <typename T, int R, typename P>
__device__ __forceinline__ void twiddle_apply(C2<T>* v, const C2<P>* p) {
    constexpr int LR = ilog2<R>();
#pragma unroll
    for (int r = 1; r < R; ++r) {
        C2<P> w = p[__builtin_ctz(r)];
#pragma unroll
        for (int k = __builtin_ctz(r) + 1; k < LR; ++k)
            if (r & (1 << k)) w = cmul(w, p[k]);
        v[r] = cmul(v[r], w);
    }
}

// Padded LDS half image (one real component at a time): 2 extra slots after every
// kPadG<E> slots (E = elements per thread; 32 slots for E = 16, E otherwise).  Pairs
// stay 8-B aligned, and every access is base(thread) + compile-time offset: bases
// mod kPadG plus offsets mod kPadG never carry at the instantiated sizes (checked
// exhaustively for N = 1024 .. 16384).  Padding every 16 slots at E = 16 made every
// exchange access 2-way bank-conflicted (a contiguous 32-lane ds_read_b32 wrapped its
// last two lanes onto banks 0-1; rocprofv3 SQ_LDS_BANK_CONFLICT = 2.2 cycles per LDS
// instruction at C3); every 32 slots removes them at N = 4096 and leaves 1 in 8
// elsewhere (bank model: MI355X_MICROARCH.md §LDS).
template <int E> constexpr int kPadG = E < 32 ? 32 : E;
template <int E> __device__ __forceinline__ int lds_idx(int i) { return i + 2 * (i / kPadG<E>); }
template <int E> constexpr int lds_off(int c) { return c + 2 * (c / kPadG<E>); }   // c a multiple of E
template <int N, int E> constexpr int lds_elems() { return N + 2 * (N / kPadG<E>); }

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

// The image feeding pass P and its padding group (2 pad slots per kPadG<E> slots, or per 16
// for the signal-pair kernel's 0 -> 1 image at n = 4096: kPad16 below).
template <int PG> __device__ __forceinline__ int lds_idx_p(int i) { return i + 2 * (i / PG); }
template <int PG> constexpr int lds_off_p(int c) { return c + 2 * (c / PG); }
template <typename T> constexpr bool kIsPair = !std::is_same<T, Sc<T>>::value;
// Signal-pair kernel at T = 256 (n = 4096, E = 16): pass 0 writes each lane's 16 slots as
// 8 ds_write_b128; with 2 pad slots per 32 two lanes share a pad block, so lanes t, t+1 of
// every 8-lane group hit the same banks (2-way on every pass-0 write).  kPad16 pads the
// 0 -> 1 image per 16 slots (stride 18 slots = 36 dwords per lane: conflict-free writes), and
// pass 1's lanes 16-31 of each 32-lane ds_read_b64 group take the butterfly block 8 blocks
// further (PassInfo::REMAP: 8 * 18 slots = 288 = 32 mod 64 dwords), so those reads stay
// conflict-free too.  The 1 -> 2 image keeps 2 per 32 (its accesses are lane-contiguous).
// Measured: round 2, 1.4 % slower (the layout pushed the power kernel from 16 to 20 B of
// scratch); round 5, with the pair kernels at 0 B of scratch, C3 1.1258 -> 1.1156 ms per
// launch (-0.9 %, profiles/r05_c3_pad16_ab.txt).  -DNW_PAIR_PAD16=0: the per-32 image.
#ifndef NW_PAIR_PAD16
#define NW_PAIR_PAD16 1
#endif
template <typename T, int N, int E>
constexpr bool kPad16 = NW_PAIR_PAD16 && kIsPair<T> && E == 16 && N / E == 256 && Geometry<N, E>::npass() > 2;
template <typename T, int N, int E, int P> constexpr int kPadX = (kPad16<T, N, E> && P == 1) ? 16 : kPadG<E>;
template <typename T, int N, int E> constexpr int kImgElems = kPad16<T, N, E> ? N + 2 * (N / 16) : lds_elems<N, E>();

// output value of one point: y, |y| or |y|^2
template <int OUT, typename T> struct OutT { using type = T; };
template <typename T> struct OutT<NW_OUT_CWT, T> { using type = C2<T>; };
// internal output kind of the forward R2C kernel (fused_forward): conj(y[k]) for k <= n/2,
// stored lane-contiguous (a 16-B "output" size keeps the last pass unpaired)
constexpr int kOutXHalf = 1000;
// internal output kind of the fused power partial sums: the last pass adds |y|^2 into the
// caller's per-thread fp64 accumulators instead of storing (epoch reductions, fused_power_partials)
constexpr int kOutPSum = 1001;
// ... and the phase sums of ITC: acc[2e], acc[2e + 1] += y / |y| in fp64
constexpr int kOutPhSum = 1002;
struct alignas(16) XHalfSlot { double a, b; };
template <typename T> struct OutT<kOutXHalf, T> { using type = XHalfSlot; };
template <int OUT, typename T>
__device__ __forceinline__ typename OutT<OUT, T>::type out_value(C2<T> y) {
    if constexpr (OUT == NW_OUT_CWT) return y;
    else if constexpr (OUT == NW_OUT_POWER) return y.re * y.re + y.im * y.im;
    else return (T)sqrt(y.re * y.re + y.im * y.im);
}

// Output store policies (each kernel picks one; measured with tools/ab.sh on one box):
//   kStoreGlobal: global stores, streaming (nt) for paired / packed outputs, plain for the
//     16-B unpaired ones (fp32 C4 3.364 ms; nt there too 3.36; the C5 passes);
//   kStoreGlobalNt: global nt for every output (fp64 C4 shape 9.14-9.34 -> 8.29-8.40 ms per
//     launch, the C5 fp64 row pass: plain 16-B complex128 stores were the slow ones);
//   kStoreBuffer: raw buffer nt stores, the compile-time offset in the descriptor base (scalar
//     adds instead of per-store VGPR address adds): the signal-pair kernel, C3 1.268 -> 1.222 ms
//     (fp32 C4 3.364 -> 3.402, the C5 fp64 row pass 0.93 -> 1.06 and the chirp-z kernel
//     1.23 -> 1.44 ms were slower with it).
// The buffer form keeps the descriptor's SGPR offset field 0: with a register there, a VALU
// write of the store's data VGPRs in the very next instruction (which the compiler does not
// guard for that form) corrupted the first dword of 16-B stores on gfx950.
constexpr int kStoreGlobal = 0, kStoreGlobalNt = 1, kStoreBuffer = 2;
// (NW_LINT_HAZARD_SOFFSET: the old, hazardous form with the offset in the soffset field --
// built only by tests/test_isa_lint.py, device code only and never run, to show that
// tools/isa_lint.py catches it)
#ifdef NW_LINT_HAZARD_SOFFSET
constexpr bool kSoffsetInField = true;
#else
constexpr bool kSoffsetInField = false;
#endif
template <int SP, typename V>
__device__ __forceinline__ void store_row(V val, void* row, uint32_t lane_off, uint32_t c_off) {
    if constexpr (SP == kStoreBuffer) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<char*>(row) + (kSoffsetInField ? 0 : c_off), 0, 0x7fffffff, 0x00020000);
        const int so = kSoffsetInField ? (int)c_off : 0;
        if constexpr (sizeof(V) == 16)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, val),
                                                   rs, (int)lane_off, so, 2);
        else if constexpr (sizeof(V) == 8)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, val),
                                                  rs, (int)lane_off, so, 2);
        else
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, val), rs, (int)lane_off, so, 2);
    } else {
        __builtin_nontemporal_store(val, reinterpret_cast<V*>(at(reinterpret_cast<char*>(row), lane_off, c_off)));
    }
}
template <typename O> using StoreVec =
    typename std::conditional<sizeof(O) == 16, float __attribute__((ext_vector_type(4))),
    typename std::conditional<sizeof(O) == 8, float __attribute__((ext_vector_type(2))), float>::type>::type;

// store outputs idx, idx+1 of the current row (orow: wave-uniform row base) as ONE
// vector store (16 B for complex64, 8 B for float32, 2x16 B for complex128)
// outputs lane_idx + c_idx (pair: and the next one) of the current row
template <int OUT, typename T, int SP>
__device__ __forceinline__ void store_pair(void* orow, uint32_t lane_idx, uint32_t c_idx, C2<T> y0, C2<T> y1) {
    using O = typename OutT<OUT, T>::type;
    struct alignas(2 * sizeof(O)) P2 { O a, b; };
#ifdef NW_ABL_NOSTORE
    asm volatile("" ::"v"(y0.re), "v"(y0.im), "v"(y1.re), "v"(y1.im), "v"(lane_idx));
    return;
#endif
    using V = typename std::conditional<sizeof(P2) == 16, float __attribute__((ext_vector_type(4))),
              typename std::conditional<sizeof(P2) == 8, float __attribute__((ext_vector_type(2))),
                                        double __attribute__((ext_vector_type(4)))>::type>::type;
    const P2 pv{out_value<OUT, T>(y0), out_value<OUT, T>(y1)};
    store_row<SP>(__builtin_bit_cast(V, pv), orow, lane_idx * (uint32_t)sizeof(O), c_idx * (uint32_t)sizeof(O));
}
template <int OUT, typename T, int SP>
__device__ __forceinline__ void store_one(void* orow, uint32_t lane_idx, uint32_t c_idx, C2<T> y) {
    using O = typename OutT<OUT, T>::type;
#ifdef NW_ABL_NOSTORE
    asm volatile("" ::"v"(y.re), "v"(y.im), "v"(lane_idx));
    return;
#endif
    if constexpr (SP == kStoreGlobal)
        *at(reinterpret_cast<O*>(orow), lane_idx * (uint32_t)sizeof(O), c_idx * (uint32_t)sizeof(O)) =
            out_value<OUT, T>(y);
    else
        store_row<SP>(__builtin_bit_cast(StoreVec<O>, out_value<OUT, T>(y)), orow, lane_idx * (uint32_t)sizeof(O),
                      c_idx * (uint32_t)sizeof(O));
}

// ---- diagnostic phase stamps (NW_STAMPS builds only; never in the product build).
// Per wave: cycles between consecutive stamps are summed into SGPR-resident
// counters and lane 0 adds them to g_nw_stamps at the end (cdna_hip_programming.md
// §7 "In-kernel stamps"): read the SHARES, not the run time of a stamped build.
#ifdef NW_STAMPS
constexpr int kStamps = 8;
__device__ unsigned long long g_nw_stamps[kStamps + 1];
struct Stamps {
    unsigned long long last, acc[kStamps];
};
__device__ __forceinline__ unsigned long long nw_now() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define NW_STAMP(st, k)                                 \
    do {                                                \
        if (st) {   /* callers without stamps pass nullptr (fwd_r2c, rows, chirp) */ \
            const unsigned long long now_ = nw_now();   \
            (st)->acc[k] += now_ - (st)->last;          \
            (st)->last = now_;                          \
        }                                               \
    } while (0)
constexpr int kStampsStore = kStamps - 1;
#else
struct Stamps {};
#define NW_STAMP(st, k) ((void)(st))
#endif

// two adjacent real slots of the half image, one 8/16-byte LDS access
template <typename T> struct alignas(2 * sizeof(T)) Pair {
    T a, b;
};

template <int COMP, typename T> __device__ __forceinline__ T& comp(C2<T>& c) {
    if constexpr (COMP == 0) return c.re; else return c.im;
}

template <int N, int E, int P, int OSZ = 8, bool PK = false> struct PassInfo;

// ---- one component of the pass-P outputs -> LDS (P = 0: slots t*E + s, as pairs)
template <typename T, int N, int E, int P, int COMP>
__device__ __forceinline__ void lds_write(C2<T>* v, T* lds, int t) {
    using G = Geometry<N, E>;
    constexpr int PG = kPadX<T, N, E, P + 1>;
    if constexpr (P == 0) {
        NW_DCHECK_H(lds_idx_p<PG>(t * E + E - 1) < kImgElems<T, N, E>);
        Pair<T>* dst = reinterpret_cast<Pair<T>*>(lds + lds_idx_p<PG>(t * E));
#pragma unroll
        for (int u = 0; u < E / 2; ++u)
            dst[u] = Pair<T>{comp<COMP>(v[bitrev<E>(2 * u)]), comp<COMP>(v[bitrev<E>(2 * u + 1)])};
    } else {
        constexpr int R = G::radix(P);
        constexpr int NS = G::ns(P);
        constexpr int Q = E / R;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            // lane-contiguous butterflies (OSZ 16: never the paired last-pass order), or pass 1's remap
            const int j = PassInfo<N, E, P, 16, kIsPair<T>>::bfly(t, q);
            NW_DCHECK_H(lds_idx_p<PG>((j / NS) * NS * R + j % NS) + lds_off_p<PG>((R - 1) * NS) < kImgElems<T, N, E>);
            T* dst = lds + lds_idx_p<PG>((j / NS) * NS * R + j % NS);
#pragma unroll
            for (int i = 0; i < R; ++i) dst[lds_off_p<PG>(bitrev<R>(i) * NS)] = comp<COMP>(v[q * R + i]);
        }
    }
}

// ---- one component of the pass-P inputs <- LDS.  Butterflies: j = t + q*T, except
// in the LAST pass, where j = Q*t + q so a thread's outputs come in adjacent pairs.
// OSZ: bytes of one output value (pairing is only worth it for outputs <= 8 B: a pair of
// 16-B complex128 outputs is two 16-B stores per lane, each touching every other 16 B)
template <int N, int E, int P, int OSZ, bool PK> struct PassInfo {
    using G = Geometry<N, E>;
    static constexpr int R = G::radix(P);
    static constexpr int NS = G::ns(P);
    static constexpr int Q = E / R;
    static constexpr int STRIDE = N / R;
    static constexpr bool LAST = (P == G::npass() - 1);
    // pairs (j = Q*t + q) only when Q == 2: the two outputs of a lane are then adjacent AND
    // neighbouring lanes are too (16-B stores, whole lines).  At Q >= 4 pairing put lanes Q
    // outputs apart (a store instruction touched 1/2 .. 1/4 of each line: 4x slower at
    // n = 8192); the lane-contiguous j = t + q*T plus DPP packing keeps stores whole.
    static constexpr bool PAIRED = LAST && Q == 2 && OSZ <= 8;
    static_assert(STRIDE % E == 0 && NS % E == 0, "pad must stay linear");
    // Paired reads at T = 512 (n = 16384 fp32, E = 32; image padded 2 slots per 32): with
    // lane-contiguous pairs j = 2t the second 16 lanes of every 32-lane ds_read_b64 group
    // start 34 dwords after the first, so lane 31 lands on lane 0's banks 0-1: every read
    // of the pass 2-way conflicted (SQ_LDS_BANK_CONFLICT 20 % of LDS cycles at C4).  Lanes
    // 16-31 of each group take the pair block 16 blocks further (512 slots: 16 * 34 =
    // 544 = 32 mod 64 dwords), so a group covers the 64 banks once.  Stores stay whole:
    // each store instruction writes two 512-B runs.
    static constexpr bool SWZ = PAIRED && G::T == 512 && kPadG<E> == 32;
    // the signal-pair kernel's pass 1 reads the per-16-padded image (kPad16)
    static constexpr bool REMAP = PK && NW_PAIR_PAD16 && P == 1 && !LAST && E == 16 && G::T == 256 && Q == 1;
    __device__ static __forceinline__ int bfly(int t, int q) {
        if constexpr (SWZ) return 2 * (((t >> 5) << 4) + (((t >> 4) & 1) << 8) + (t & 15)) + q;
        if constexpr (REMAP) return ((t >> 5) << 4) + (((t >> 4) & 1) << 7) + (t & 15);
        return PAIRED ? Q * t + q : t + q * G::T;
    }
};

// Pass-1 twiddles w_{NS*R}^{(j % NS) * r} depend on j % NS only (NS = E, the pass-0
// radix): an NS x (R-1) table in LDS after the image (7.75 KiB at n = 16384 fp32),
// filled once per block from the exact global table, replaces that pass's v_sin/v_cos
// bases and their products (the kernel is power-bound: every VALU op saved counts).
template <typename T, int N, int E> struct Tab1 {
    using I = PassInfo<N, E, 1>;
    using S = Sc<T>;                                // entries in the scalar type (shared by a pair)
    static constexpr int NS = I::NS, R = I::R;
    static constexpr int COUNT = Geometry<N, E>::npass() >= 2 ? NS * (R - 1) : 0;
    // fp64 at n = 16384: one block per CU whatever the table costs (256 VGPRs), and image +
    // table (155 KiB) fit the CU's LDS
    // (fp64 at n = 16384, 15.5 KiB beside the 136 KiB image, measured +2.5 % alone and
    // slower than the X LDS-DMA it would share the space with: not kept)
    // fp64 at n = 16384 (one block per CU either way): the 15.5 KiB table beside the 136 KiB
    // image (155 KiB of the CU's 160), in the translation units that define NW_TAB1_F64_16384
    // (nw_fused.hip: C4 shape fp64 8.19-8.21 -> 7.96 ms per launch, 0.525 -> 0.541 of HBM peak;
    // the C5 fp64 row pass +-0 with it and its step 3 % slower, so nw_large.hip keeps the bases;
    // profiles/r05_f64_tab1_ab.txt)
    // (A per-file choice without an ODR question: this header's templates live in an unnamed
    // namespace, so every translation unit instantiates its own Tab1 -- internal linkage, as
    // `static` -- and nw_fused.hip's Tab1<double, 16384, 32> is not nw_large.hip's; the
    // device code is compiled per file, without -fgpu-rdc, too.)
#ifdef NW_TAB1_F64_16384
    static constexpr bool BIG = sizeof(S) == 8 && N == 16384 && E == 32;
#else
    static constexpr bool BIG = false;
#endif
    static constexpr bool ON = COUNT > 0 && (COUNT * (int)sizeof(C2<S>) <= 8192 || BIG);
    static constexpr int BYTES = ON ? COUNT * (int)sizeof(C2<S>) : 0;
    static_assert((kImgElems<T, N, E> * sizeof(T)) % 16 == 0, "table alignment");
    __device__ static __forceinline__ const C2<S>* table(const T* lds) {
        return reinterpret_cast<const C2<S>*>(lds + kImgElems<T, N, E>);
    }
    // w_N^e entries from the exact table tw (tw[i] = exp(+2 pi i / N))
    __device__ static __forceinline__ void fill(T* lds, const C2<S>* __restrict__ tw, int t) {
        if constexpr (ON) {
            C2<S>* tab = reinterpret_cast<C2<S>*>(lds + kImgElems<T, N, E>);
            for (int i = t; i < COUNT; i += Geometry<N, E>::T) {
                const int jj = i % NS, r = i / NS + 1;
                tab[i] = tw[(jj * r * (N / (NS * R))) % N];
            }
        }
    }
};

template <typename T, int N, int E, int P, int COMP, int OSZ>
__device__ __forceinline__ void lds_read(C2<T>* v, const T* lds, int t) {
    using I = PassInfo<N, E, P, OSZ, kIsPair<T>>;
    constexpr int R = I::R, Q = I::Q;
    constexpr int PG = kPadX<T, N, E, P>;
    if constexpr (I::PAIRED) {
        NW_DCHECK_H(lds_idx_p<PG>(I::bfly(t, 0)) + (Q - 1) + lds_off_p<PG>((R - 1) * I::STRIDE) < kImgElems<T, N, E>);
        const T* src = lds + lds_idx_p<PG>(I::bfly(t, 0));
#pragma unroll
        for (int q = 0; q < Q; q += 2)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const Pair<T> pr = *reinterpret_cast<const Pair<T>*>(src + q + lds_off_p<PG>(r * I::STRIDE));
                comp<COMP>(v[q * R + r]) = pr.a;
                comp<COMP>(v[(q + 1) * R + r]) = pr.b;
            }
    } else {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            NW_DCHECK_H(lds_idx_p<PG>(I::bfly(t, q)) + lds_off_p<PG>((R - 1) * I::STRIDE) < kImgElems<T, N, E>);
            const T* src = lds + lds_idx_p<PG>(I::bfly(t, q));
#pragma unroll
            for (int r = 0; r < R; ++r) comp<COMP>(v[q * R + r]) = src[lds_off_p<PG>(r * I::STRIDE)];
        }
    }
}

// Workgroup barrier for the LDS image only.  __syncthreads() carries a workgroup
// release fence that gfx950 lowers to s_waitcnt vmcnt(0): every exchange would
// wait for ALL of the wave's in-flight global stores.  The exchanges only need
// this wave's LDS operations complete (lgkmcnt(0)) before the s_barrier.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);   // vmcnt(63) expcnt(7) lgkmcnt(0): LDS ops only
    __builtin_amdgcn_s_barrier();
}

// ---- LDS-DMA of the next signal's half spectrum X[0 .. N/2) (N*4 bytes) into the idle
// LDS image: 16 B per lane per instruction, global_load_lds_dwordx4 writes lane l of
// a wave at (wave-uniform base) + 16*l.  X[N/2] (the real Nyquist bin) travels by a
// scalar load.  The DMA is issued before the stores, so the next pass 0 waits for
// it with vmcnt(#stores issued after it), not for the stores.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

// LDS-DMA of X[0 .. N/2) (the R2C half spectrum without its Nyquist bin) into LDS at dst:
// 16 B per lane per instruction, wave w filling its own 1 KiB slices of each round.
// nround < CH / TT copies only the first nround rounds (2*TT bins each): the bins a pruned
// pass 0 reads (wave-uniform count)
template <typename T, int N, int TT>
__device__ __forceinline__ void dma_x(const C2<T>* xs, void* dst, int t, int nround = 1 << 30) {
    constexpr int CH = (N / 2) * (int)sizeof(C2<T>) / 16;   // 16-byte chunks
    static_assert(CH % TT == 0, "whole DMA rounds");
    // wave-uniform LDS destination base in an SGPR (M0 takes it directly; a VGPR copy
    // per chunk would be hoisted out of the signal loop and spilled)
    const int wave_base = __builtin_amdgcn_readfirstlane((t & ~63) * 16);
    const uint32_t lane_off = (uint32_t)t * 16u;
#pragma unroll
    for (int i = 0; i < CH / TT; ++i) {
        if (i >= nround) break;
        // uniform chunk base + 32-bit lane offset: the saddr form, no 64-bit VGPR pairs
        const char* chunk = reinterpret_cast<const char*>(xs) + (size_t)i * TT * 16;
        asm volatile("" : "+s"(chunk));           // computed here, in SGPRs (not hoisted)
        const uint32_t lds_addr = (uint32_t)(uintptr_t)(lds_void_t*)(reinterpret_cast<char*>(dst) + i * TT * 16 + wave_base);
        // Issued as inline asm, not __builtin_amdgcn_global_load_lds: for the builtin the
        // compiler puts a vmcnt(0) before every later LDS read (it cannot count a loop-carried,
        // variably sized DMA), which also waits for all of the previous signal's stores.  The
        // callers order it themselves: a barrier before (the image's readers are done) and
        // wait_vmcnt<#stores issued after it> + a barrier before the first read.
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
                     :: "s"(lds_addr), "v"(lane_off), "s"(chunk) : "memory", "m0");
    }
}

// One uniform complex value by a scalar load (lgkmcnt, not vmcnt): a vector load issued
// after the previous signal's stores would wait for all of them (in-order vmcnt), and the
// compiler put a vmcnt(0) before it (a register of the merged pass-0 variants still pending)
// fp32: the raw 8 bytes (kept uniform, in SGPRs, across a loop; C2 values of it were moved
// to VGPRs and spilled to scratch, whose reload is a vector load behind the stores)
__device__ __forceinline__ unsigned long long sload_u64(const void* p) {
    unsigned long long u;
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(u) : "s"(p) : "memory");
    return u;
}
__device__ __forceinline__ C2<float> c2_of_u64(unsigned long long u) {
    return C2<float>{__uint_as_float((unsigned)u), __uint_as_float((unsigned)(u >> 32))};
}
template <typename T> __device__ __forceinline__ C2<T> sload_c2(const C2<T>* p) {
    if constexpr (sizeof(T) == 4) {
        unsigned long long u;
        asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(u) : "s"(p) : "memory");
        return C2<T>{__uint_as_float((unsigned)u), __uint_as_float((unsigned)(u >> 32))};
    } else {
        typedef unsigned long long u2 __attribute__((ext_vector_type(2)));
        u2 u;
        asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(u) : "s"(p) : "memory");
        return C2<T>{__longlong_as_double((long long)u.x), __longlong_as_double((long long)u.y)};
    }
}

// s_waitcnt vmcnt(V) with expcnt/lgkmcnt left free (gfx9 encoding: vmcnt[3:0] + [15:14])
template <int V>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(V >= 0 && V < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((V & 0xF) | ((V >> 4) << 14) | 0x70 | 0xF00);
}

// ---- lane-group transposes for the last pass's stores (DPP quad_perm, no LDS)
template <int CTRL> __device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL> __device__ __forceinline__ double dpp_f(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffLL), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// 2x2 transpose of (register a, register b) x (lane l, lane l ^ D): the lane with bit D
// clear keeps a and takes its partner's a as b; the other keeps b and takes the partner's b as a
template <int D, typename F> __device__ __forceinline__ void xpose2(F& a, F& b, bool hi) {
    constexpr int CTRL = D == 1 ? 0xB1 : 0x4E;      // quad_perm [1,0,3,2] / [2,3,0,1]
    const F recv = dpp_f<CTRL>(hi ? a : b);
    if (hi) a = recv; else b = recv;
}
template <typename F> __device__ __forceinline__ void xpose2(C2<F>& a, C2<F>& b, bool hi, int d) {
    if (d == 1) { xpose2<1>(a.re, b.re, hi); xpose2<1>(a.im, b.im, hi); }
    else { xpose2<2>(a.re, b.re, hi); xpose2<2>(a.im, b.im, hi); }
}

// ---- the last pass's outputs: store number i (0 .. nstores-1) of a thread
// Unpaired last pass (Q = 1: lane t owns outputs t + NS*m, NS apart): PACK lanes swap
// PACK rows with a PACK x PACK transpose, so each lane stores PACK consecutive outputs
// as ONE 16-B store -- 4x fewer store instructions for |y|^2 (fp32), 2x for y.  The
// stores, not their bytes, limited these sizes (n = 4096: 2x the bytes of cwt over
// power cost +20 % time).
template <typename T, int N, int E, int OUT, int SP = kStoreGlobal>
struct LastStores {
    using O = typename OutT<OUT, T>::type;
    using I = PassInfo<N, E, Geometry<N, E>::npass() - 1, (int)sizeof(O)>;
    static constexpr int R = I::R, Q = I::Q;
    static constexpr int STEP = I::PAIRED ? 2 : 1;
    static constexpr int PACK_W = (int)(16 / sizeof(O));
    static constexpr int PACK = (!I::PAIRED && PACK_W <= kPackMax && R % PACK_W == 0) ? PACK_W : 1;
    static_assert(PACK == 1 || PACK == 2 || PACK == 4, "pack");
    static constexpr int COUNT = PACK > 1 ? Q * R / PACK : Q / STEP * R;   // store instructions per thread per signal
    // all stores of one signal (v: the last pass's registers, bit-reversed rows)
    __device__ static __forceinline__ void all(const C2<T>* v, void* orow, int t) {
        if constexpr (PACK == 1) {
            chunk<0, 1>(v, orow, t);
        } else {
            const int c = t & (PACK - 1);
            const uint32_t lane = (uint32_t)((t & ~(PACK - 1)) + I::NS * c) * (uint32_t)sizeof(O);
#pragma unroll
            for (int qg = 0; qg < Q * (R / PACK); ++qg) {
                const int q = qg / (R / PACK), g = qg % (R / PACK);   // butterfly t + q*T, row group g
                O val[PACK];
#pragma unroll
                for (int b = 0; b < PACK; ++b) val[b] = out_value<OUT, T>(v[q * R + bitrev<R>(g * PACK + b)]);
                if constexpr (PACK >= 2) {
                    const bool hi1 = c & 1;
#pragma unroll
                    for (int b = 0; b < PACK; b += 2) xpose_any<1>(val[b], val[b + 1], hi1);
                }
                if constexpr (PACK == 4) {
                    const bool hi2 = c & 2;
                    xpose_any<2>(val[0], val[2], hi2);
                    xpose_any<2>(val[1], val[3], hi2);
                }
                using V = float __attribute__((ext_vector_type(4)));
                struct alignas(16) P16 { O a[PACK]; };
                P16 pk;
#pragma unroll
                for (int b = 0; b < PACK; ++b) pk.a[b] = val[b];
#ifdef NW_ABL_NOSTORE
                asm volatile("" ::"v"(__builtin_bit_cast(V, pk)));
#else
                store_row<SP>(__builtin_bit_cast(V, pk), orow, lane,
                              (uint32_t)((q * Geometry<N, E>::T + g * PACK * I::NS) * sizeof(O)));
#endif
            }
        }
    }
    template <int D, typename F> __device__ static __forceinline__ void xpose_any(F& a, F& b, bool hi) {
        if constexpr (std::is_same<F, float>::value || std::is_same<F, double>::value) xpose2<D>(a, b, hi);
        else xpose2(a, b, hi, D);
    }
    template <int K>
    __device__ static __forceinline__ void one(const C2<T>* o, void* orow, int t) {
        constexpr int q = (K / R) * STEP, i = K % R;
        const uint32_t lane = (uint32_t)I::bfly(t, 0);        // Q*t (paired) or t
        constexpr uint32_t c = (uint32_t)((I::PAIRED ? q : q * Geometry<N, E>::T) + bitrev<R>(i) * I::NS);
        NW_DCHECK_H(lane + c + (I::PAIRED ? 1u : 0u) < (uint32_t)N);
        if constexpr (I::PAIRED)
            store_pair<OUT, T, SP>(orow, lane, c, o[q * R + i], o[(q + 1) * R + i]);
        else
            store_one<OUT, T, SP>(orow, lane, c, o[q * R + i]);
    }
    // stores [C*COUNT/NCH, (C+1)*COUNT/NCH) -- one chunk of a deferred signal
    template <int C, int NCH, int K = C * COUNT / NCH>
    __device__ static __forceinline__ void chunk(const C2<T>* o, void* orow, int t) {
        if constexpr (K < (C + 1) * COUNT / NCH) {
            one<K>(o, orow, t);
            chunk<C, NCH, K + 1>(o, orow, t);
        }
    }
};



// LDS-DMA of the next signal's X: fp32 at E >= kXdmaMinE, fp64 at E = 32 (n = 16384 fp64 cwt
// 10.90 -> 9.88 ms per 512-signal launch); analytic rows only (complex table rows keep the
// register path: with LDS-DMA they exceed 128 VGPRs)
template <typename T, int E, bool REALW>
constexpr bool kXDMA = E >= (sizeof(T) == 4 ? kXdmaMinE : 32) && REALW;
// DMA rounds (T lanes x 16 B each) holding the first nz pass-0 elements (T bins each)
template <typename T> __device__ __forceinline__ int dma_rounds_for(int nz) {
    return (nz * (int)sizeof(C2<T>) + 15) / 16;
}

// fp64 twiddle bases from a split table in LDS: w_N^i = hi[i >> 5] * lo[i & 31] for i < N/2,
// N/64 + 32 exact entries (4.5 KiB at N = 16384) filled once per block from the exact global
// table, so no base is a global load (a load issued after this wave's stores waits for all
// of them in the in-order vmcnt queue; fp32 takes v_sin/v_cos for the same reason).  The
// product of two exact entries is within 1 ulp of a direct entry.
// Measured (one box, interleaved): fp64 N = 4096 1.950 -> 1.900 ms per launch (+2.7 %), but
// N = 16384 (E = 32, X by LDS-DMA) 9.80 -> 10.0-10.3 ms and the C5 fp64 row pass 0.94 -> 0.95:
// on for N <= 4096 only.
// (At N = 16384 measured again in round 4, beside the next signal's W loaded before the
// stores and alone: +-0 / slower, profiles/r04_ab_fused.txt.)
template <typename T, int N, int E> struct TwSplit {
    static constexpr bool ON = std::is_same<T, double>::value && N >= 2048 && N <= 4096;
    static constexpr int NHI = N / 64, COUNT = NHI + 32;
    static constexpr int OFFSET = kImgElems<T, N, E> * (int)sizeof(T) + Tab1<T, N, E>::BYTES;
    static_assert(OFFSET % 16 == 0, "table alignment");
    static constexpr int BYTES = ON ? COUNT * (int)sizeof(C2<T>) : 0;
    __device__ static __forceinline__ const C2<T>* table(const T* lds) {
        return reinterpret_cast<const C2<T>*>(reinterpret_cast<const char*>(lds) + OFFSET);
    }
    // call before the first lds_barrier that precedes any use
    __device__ static __forceinline__ void fill(T* lds, const C2<T>* __restrict__ tw, int t) {
        if constexpr (ON) {
            C2<T>* tab = reinterpret_cast<C2<T>*>(reinterpret_cast<char*>(lds) + OFFSET);
            for (int i = t; i < COUNT; i += Geometry<N, E>::T) tab[i] = i < NHI ? tw[i * 32] : tw[i - NHI];
        }
    }
};
template <typename T, int N, int E> constexpr int kLdsBytes =
    kImgElems<T, N, E> * (int)sizeof(T) + Tab1<T, N, E>::BYTES + TwSplit<T, N, E>::BYTES;


// ---- exchange pass P-1 -> P through the half image (re, then im), then compute pass P.
// In the last pass (LDS-DMA kernels) the NEXT signal's X is DMA'd into the idle image
// before this signal's stores are issued: loads, stores and LDS-DMA retire in one
// in-order vmcnt queue, so the next pass 0 waits for that DMA only.  The last pass
// stores its outputs straight to HBM.
//
// T = f2 (signal pairs): every element carries two signals' values; twiddles and the Tab1
// table stay scalar (shared), and the last pass stores the low halves to ocur and the high
// halves to ocur2 (nullptr: an odd last signal, its high half is not stored).
template <typename T, int N, int E, int OUT, int P, bool XD, int SP = kStoreGlobal>
__device__ __forceinline__ void passes_from(C2<T>* v, T* lds, int t, const C2<Sc<T>>* __restrict__ tw, C2<T>* x,
                                            const C2<T>* xs_next, void* ocur,
                                            Stamps* st, void* ocur2 = nullptr, int dma_rounds = 1 << 30,
                                            double* acc = nullptr, const void* xs_next2 = nullptr) {
    using S = Sc<T>;
    constexpr bool PAIRSIG = !std::is_same<T, S>::value;
    constexpr int OSZ = (int)sizeof(typename OutT<OUT, S>::type);
    using I = PassInfo<N, E, P, OSZ, kIsPair<T>>;
    if constexpr (P < Geometry<N, E>::npass()) {
        constexpr int R = I::R, Q = I::Q, LR = ilog2<R>();
        constexpr bool TABLED = P == 1 && Tab1<T, N, E>::ON;
        constexpr bool SPLIT = TwSplit<T, N, E>::ON;
        const C2<S>* split = nullptr;
        if constexpr (SPLIT) split = reinterpret_cast<const C2<S>*>(TwSplit<T, N, E>::table(lds));
        C2<S> pb[Q][LR > 0 ? LR : 1];
#ifndef NW_ABL_NOTWIDDLE
        if constexpr (!TABLED && I::PAIRED && Q == 2) {
            // the lane's second butterfly is j + 1 (j even, no wrap mod NS): its bases are the
            // first's times the constants w^(2^k) -- uniform loads from the exact table
            twiddle_bases<S, R, N, I::NS * R, SPLIT>(pb[0], I::bfly(t, 0) % I::NS, tw, split);
#pragma unroll
            for (int k = 0; k < LR; ++k) pb[1][k] = cmul(pb[0][k], tw[(N / (I::NS * R)) << k]);
        } else if constexpr (!TABLED) {
#pragma unroll
            for (int q = 0; q < Q; ++q) twiddle_bases<S, R, N, I::NS * R, SPLIT>(pb[q], I::bfly(t, q) % I::NS, tw, split);
        }
#endif
#ifndef NW_ABL_NOEXCH
        lds_barrier();                         // earlier readers of the image are done
        lds_write<T, N, E, P - 1, 0>(v, lds, t);
        lds_barrier();
        lds_read<T, N, E, P, 0, OSZ>(v, lds, t);
        lds_barrier();
        lds_write<T, N, E, P - 1, 1>(v, lds, t);
        lds_barrier();
        lds_read<T, N, E, P, 1, OSZ>(v, lds, t);
#else   // ablation (diagnostic builds only): no exchange, the registers stay live
#pragma unroll
        for (int i = 0; i < E; ++i) asm volatile("" : "+v"(v[i].re), "+v"(v[i].im));
#endif
        if constexpr (I::LAST && XD) {
            if (xs_next) {                     // the image is idle once every wave has read it
                lds_barrier();
                if constexpr (PAIRSIG) {
                    // the next pair's two half spectra side by side: [0, N/2) and [N/2, N) complex
                    dma_x<S, N, Geometry<N, E>::T>(reinterpret_cast<const C2<S>*>(xs_next), lds, t, dma_rounds);
                    dma_x<S, N, Geometry<N, E>::T>(reinterpret_cast<const C2<S>*>(xs_next2),
                                                   reinterpret_cast<char*>(lds) + (N / 2) * sizeof(C2<S>), t, dma_rounds);
                } else {
                    dma_x<T, N, Geometry<N, E>::T>(xs_next, lds, t, dma_rounds);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        NW_STAMP(st, 2 * P - 1);               // exchange P-1 -> P
#pragma unroll
        for (int q = 0; q < Q; ++q) {
#ifndef NW_ABL_NOTWIDDLE
            if constexpr (TABLED) {
                const C2<S>* tab = Tab1<T, N, E>::table(lds) + I::bfly(t, q) % I::NS;
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    v[q * R + r] = cmul(v[q * R + r], tab[(r - 1) * I::NS]);
                    if (r % 8 == 7) __builtin_amdgcn_sched_barrier(0);   // <= 8 twiddles in flight
                }
            } else if constexpr (!(std::is_same<T, float>::value && Q % 2 == 0)) {
                twiddle_apply<T, R>(v + q * R, pb[q]);
            }
#endif
            if constexpr (std::is_same<T, float>::value && Q % 2 == 0) {
                // butterflies q, q+1 as one packed pair: identical DIF networks, per-butterfly
                // twiddles packed side by side
                if (q % 2 == 0) {
                    C2<f2> pv[R];
#pragma unroll
                    for (int i = 0; i < R; ++i)
                        pv[i] = pk(reinterpret_cast<C2<float>*>(v)[q * R + i],
                                   reinterpret_cast<C2<float>*>(v)[(q + 1) * R + i]);
#ifndef NW_ABL_NOTWIDDLE
                    if constexpr (!TABLED) {
                        C2<f2> pp[LR > 0 ? LR : 1];
#pragma unroll
                        for (int k = 0; k < LR; ++k)
                            pp[k] = pk(reinterpret_cast<C2<float>*>(pb[q])[k], reinterpret_cast<C2<float>*>(pb[q + 1])[k]);
                        twiddle_apply<f2, R>(pv, pp);
                    }
#endif
                    idft_br<f2, R>(pv);
#pragma unroll
                    for (int i = 0; i < R; ++i) {
                        reinterpret_cast<C2<float>*>(v)[q * R + i] = lo(pv[i]);
                        reinterpret_cast<C2<float>*>(v)[(q + 1) * R + i] = hi(pv[i]);
                    }
                }
            } else {
                idft_br<T, R>(v + q * R);
            }
        }
        NW_STAMP(st, 2 * P);                   // pass P arithmetic
        if constexpr (I::LAST && OUT == kOutPSum) {
            // acc[q*R + i] += |y|^2 of output bfly(t, q) + bitrev(i)*NS (the same positions for
            // every signal of the block): the power output's value, added in fp64 in signal order
            // like k_accumulate, so the partials reproduce its sums
            if constexpr (PAIRSIG) {
                // signal s (low halves), then s + 1 (high halves) when the pair has one: the
                // pair kernel's power-output values, in signal order
#pragma unroll
                for (int e = 0; e < Q * R; ++e) {
                    const C2<S> a{v[e].re.x, v[e].im.x};
                    acc[e] += (double)(a.re * a.re + a.im * a.im);
                }
                if (ocur2) {
#pragma unroll
                    for (int e = 0; e < Q * R; ++e) {
                        const C2<S> b{v[e].re.y, v[e].im.y};
                        acc[e] += (double)(b.re * b.re + b.im * b.im);
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < Q * R; ++e) acc[e] += (double)(v[e].re * v[e].re + v[e].im * v[e].im);
            }
        } else if constexpr (I::LAST && OUT == kOutPhSum) {
            static_assert(!PAIRSIG, "partial sums run the single-signal kernel");
#pragma unroll
            for (int e = 0; e < Q * R; ++e) {
                const double re = (double)v[e].re, im = (double)v[e].im;
                if constexpr (sizeof(S) == 8) {
                    // fp64 y: hypot, as k_accumulate (|y|^2 of fp64 parts can underflow: rows of
                    // tiny magnitude, e.g. |y| ~ 1e-260 at the edge of a 1 Hz row), then one
                    // reciprocal for both parts (within 1 ulp of its two divisions); y = 0 gives
                    // 0 * inf = NaN like the reference's 0/0
                    const double inv = 1.0 / hypot(re, im);
                    acc[2 * e] += mul_nocontract(re, inv);
                    acc[2 * e + 1] += mul_nocontract(im, inv);
                } else {
                    // |y|^2 of fp32 parts is exact in fp64 up to one rounding (no overflow), so
                    // rsqrt replaces hypot + two divisions (k_accumulate) to within a few fp64
                    // ulp; y = 0 gives 0 * inf = NaN like the reference's 0/0 (mneutils.py:68)
                    const double inv = rsqrt(re * re + im * im);
                    // products rounded before the add (no fma into acc): a partial then adds the
                    // same values whichever block boundaries the chunking draws
                    acc[2 * e] += mul_nocontract(re, inv);
                    acc[2 * e + 1] += mul_nocontract(im, inv);
                }
            }
        } else if constexpr (I::LAST && OUT == kOutXHalf) {
            // forward R2C: X[k] = conj(sum_n x[n] w^(+kn)) for k <= n/2 (row stride n/2 + 1)
            static_assert(!I::PAIRED, "forward stores are lane-contiguous");
            C2<S>* xr = reinterpret_cast<C2<S>*>(ocur);
#pragma unroll
            for (int q = 0; q < Q; ++q)
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    const int k = I::bfly(t, q) + bitrev<R>(i) * I::NS;
                    if (k <= N / 2) xr[k] = C2<S>{v[q * R + i].re, -v[q * R + i].im};
                }
        } else if constexpr (I::LAST) {
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (PAIRSIG) {
                C2<S> a[E], b[E];
#pragma unroll
                for (int i = 0; i < E; ++i) {
                    a[i] = C2<S>{v[i].re.x, v[i].im.x};
                    b[i] = C2<S>{v[i].re.y, v[i].im.y};
                }
                LastStores<S, N, E, OUT, SP>::all(a, ocur, t);
                if (ocur2) LastStores<S, N, E, OUT, SP>::all(b, ocur2, t);
            } else {
                LastStores<T, N, E, OUT, SP>::all(v, ocur, t);
            }
        } else {
            passes_from<T, N, E, OUT, P + 1, XD, SP>(v, lds, t, tw, x, xs_next, ocur, st, ocur2, dma_rounds, acc, xs_next2);
        }
    }
}
}  // namespace
}  // namespace nw
