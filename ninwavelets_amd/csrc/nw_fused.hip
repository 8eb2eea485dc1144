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
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

// the fp64 n = 16384 pass-1 twiddle table (Tab1, nw_fft_dev.h) is on in this file's kernels
#define NW_TAB1_F64_16384 1
#include "nw_fft_dev.h"

namespace nw {

namespace {

// X[k] at the thread's pass-0 bins k = t + r*T from the R2C half spectrum xs.
// k < N/2 exactly when r < E/2 (compile-time), so no branch: X[k], or conj(X[N - k])
// above N/2 (at k = N/2 the bin is real).  interpolate_alias (zero X[k], k >= int(N/2),
// base.py:400-401) is folded into the W table (W[f, k] = 0 there): same product for
// every finite X, and no per-element masking in the kernel.
template <typename T, int N, int E, int NZ = E>
__device__ __forceinline__ void load_x(C2<T>* x, const C2<T>* xs, int t) {
    constexpr int TT = N / E;
    const uint32_t xo = (uint32_t)t * (uint32_t)sizeof(C2<T>);
#pragma unroll
    for (int r = 0; r < NZ; ++r) {
        if (r < E / 2) {
            x[r] = *at(xs, xo, (uint32_t)(r * TT * sizeof(C2<T>)));
        } else {   // X[N - k] = X[(N - r*T) - t]
            x[r] = *at(xs, (uint32_t)((N - r * TT) * sizeof(C2<T>)) - xo);
            x[r].im = -x[r].im;
        }
    }
}

template <typename T, bool REALW>
__device__ __forceinline__ auto wsel(cplx<T> w) {
    if constexpr (REALW) return w.re; else return C2<T>{w.re, w.im};
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

// Tuning constants (each measured against its alternatives):
// E = 32 kernels keep the first kWKeep32 elements of W in registers for the block (a row
// pruned to NZ <= 16 then reads no W per signal): C4 0 / 8 / 16 -> 3.537 / 3.486 / 3.456 ms
// per launch; fp64 has no registers to spare (4 and 8 measured +-0 / slower, with spills);
// n = 8192 (256-thread blocks) keeps 8: 16 spilled 12-16 B there
constexpr int kWKeep32 = 16, kWKeep32Small = 8;
// fp64 n = 16384: the pass-1 twiddle table (Tab1) left room for 8 W elements in the 256 VGPRs:
// C4 shape fp64 8.21 -> 8.02 ms per launch (4: 8.10; 12 / 16 spill 28 / 52 B;
// profiles/r05_f64_wkeep_ab.txt)
#ifndef NW_WKEEP64   // diagnostic A/B
#define NW_WKEEP64 8
#endif
constexpr int kWKeep64 = NW_WKEEP64;
// the pair kernel (E = 16): W elements kept in registers for the block (nw_fused_pair_kernel)
constexpr int kPairWKeep = 12;
// ... in the |y| and power-partial pair kernels (their sqrt / fp64 accumulators take the registers)
constexpr int kPairWKeepRed = 10;
// (W elements beyond kWKeep32 evaluated in registers for Morse rows instead of re-read:
// C4 3.360-3.368 -> 3.420-3.430 ms per launch; removing those loads altogether (diagnostic)
// 3.367-3.369: the re-read costs nothing, the evaluation's VALU does)
// E = 32: a pass-0 variant for rows whose support ends below 3/4 of n (NZ = 24: C4's rows
// above 186 Hz), between the power-of-two variants: C4 3.360-3.368 -> 3.346-3.351 ms
constexpr bool kNz24 = true;
// signal-pair kernel: the next pair's X by LDS-DMA before the stores (cwt output only, below)
constexpr bool kPairXD = true;
template <typename T, int N, int E> constexpr bool kNz24Of = kNz24 && E > 16;
// NZ = 12 and 20 between them (fp32 only: fp64 n = 16384 |y| spills 20 B with them)
template <typename T, int N, int E> constexpr bool kNzFineOf = kNz24Of<T, N, E> && sizeof(T) == 4;
// ... and for the fp64 cwt output (round 6: C4 shape fp64 -0.7 to -0.9 %; its |y| spills with
// them; -DNW_F64_FINE=0 for the A/B)
#ifndef NW_F64_FINE
#define NW_F64_FINE 1
#endif
#if NW_F64_FINE
template <typename T, int N, int E, int OUT> constexpr bool kNzFineOut = kNzFineOf<T, N, E> ||
    (kNz24Of<T, N, E> && OUT == NW_OUT_CWT);
#else
template <typename T, int N, int E, int OUT> constexpr bool kNzFineOut = kNzFineOf<T, N, E>;
#endif
// The pass-0 variant (elements read and multiplied per thread) that runs a row of support nz:
// the smallest instantiated NZ >= nz.  The X LDS-DMA copies what THAT variant reads (a row
// of support 12 on a kernel without the NZ = 12 variant runs NZ = 16, which reads 16 elements)
template <typename T, int N, int E, int OUT>
__device__ __forceinline__ int pass0_variant(int nz) {
    if (nz <= 4) return 4;
    if (nz <= 8) return 8;
    if (kNzFineOut<T, N, E, OUT> && nz <= 12) return 12;
    if (E > 16 && nz <= 16) return 16;
    if (kNzFineOut<T, N, E, OUT> && nz <= 20) return 20;
    if (kNz24Of<T, N, E> && nz <= 24) return 24;
    return E;
}
// signals per block: C3 0.354 -> 0.348 ms, C4 1.774 -> 1.770 vs 4 (2 and 16 slower or equal).
// fp64 (one block per CU): 8 since round 6 (C4 shape fp64 7.31-7.32 -> 7.25-7.28 ms per launch,
// with the fine pass-0 variants below 7.21-7.24; 2 signals +2.6 %, tiles 4 x 8 +1.5 %, 8 x 2
// +0.3 %; profiles/r06_f64_group_ab.txt).  Round 3 had taken 4 (then 10.04 -> 9.66 ms against
// 8 signals, when X was re-read from L2 per scale without the LDS-DMA)
constexpr int kGroup = 8;
static_assert(kGroup == kPsumGroup, "fused partial rows are counted by fused_psum_groups");
// (-DNW_GROUP64 / NW_TILE64_F / NW_TILE64_G: diagnostic A/B of the fp64 block and tile shape)
#ifndef NW_GROUP64
#define NW_GROUP64 8
#endif
constexpr int kGroup64 = NW_GROUP64;
// XCD tile: kTileF scales x kTileG signal groups per XCD round (fp64 tiles 16 x 2, 4 x 8,
// 32 x 1, 2 x 16 measured -2.4 / -0.2 / -4.8 / -3.5 % against 8 x 4)
constexpr int kTileF = 8, kTileG = 4;
#ifndef NW_TILE64_F
#define NW_TILE64_F kTileF
#endif
#ifndef NW_TILE64_G
#define NW_TILE64_G kTileG
#endif
template <typename T> constexpr int kTileFT = sizeof(T) == 8 ? NW_TILE64_F : kTileF;
template <typename T> constexpr int kTileGT = sizeof(T) == 8 ? NW_TILE64_G : kTileG;
// fp64 output kernels at n = 16384 (one block per CU): 16-signal blocks in XCD tiles of 8 scales
// x 2 groups -- the same X + W working set per XCD round as 8 x 4 of 8 signals, half the blocks
// (C4 shape fp64 7.175 -> 7.12-7.13 and 7.246 -> 7.212 ms per launch on two boxes, -0.5 %;
// 32 x 1 -0.3 %, 16 signals in 8 x 4 tiles -0.4 %, 16 in 8 x 1 +-0; profiles/r06_f64_g16_ab.txt).
// Smaller n (two blocks per CU) and the partial-sum kernels keep kGroup64 / kTileGT.
#ifndef NW_GROUP64_16K
#define NW_GROUP64_16K 16
#endif
#ifndef NW_TILE64_G_16K
#define NW_TILE64_G_16K 2
#endif
template <typename T, int N> constexpr int kGroupOut = sizeof(T) == 8 ? (N == 16384 ? NW_GROUP64_16K : kGroup64) : kGroup;
template <typename T, int N> constexpr int kTileGOut = sizeof(T) == 8 && N == 16384 ? NW_TILE64_G_16K : kTileGT<T>;
// ... and at most as many groups as a launch has (in units of 8 XCD slots): C2 (64 signals =
// 8 groups) with 4-group tiles padded its grid to 4x its real blocks
__host__ __device__ constexpr int tile_g_of(int64_t nsg, int tg_max) {
    const int64_t per = (nsg + 7) / 8;
    return per < tg_max ? (int)(per < 1 ? 1 : per) : tg_max;
}
// Occupancy: 4 waves/SIMD (128 VGPRs) for fp32 -- the half image is <= 74 KiB, so two
// 512-thread blocks share a CU at n = 16384 (more at smaller n) and one block's barriers,
// memory waits and store bursts overlap another's arithmetic -- and 2 for fp64 (twice the
// registers per element); the partial-sum kernels hold fp64 accumulators on top: ITC (2E) at 3 waves/SIMD,
// power at E = 32 at 2
constexpr int kWpsF32 = 4, kWpsF64 = 2, kWpsPhSum = 3, kWpsPSum32 = 2;
// fp64 one-pass kernels (E = 32, X by LDS-DMA): the second half of a block's waves at s_setprio 1 (MI355X_MICROARCH.md
// "Two waves per SIMD", item 4: at equal priority the younger half loses every arbitration).
// fp64 C4 shape 7.92-7.99 -> 7.89-7.90 ms per launch; fp32 C4 +-0, C3 (signal pairs) +10 %:
// fp64 only (tools/ab.sh, profiles/r04_ab_fused.txt)
#ifndef NW_PRIO64   // diagnostic A/B (-DNW_PRIO64=0)
#define NW_PRIO64 1
#endif
template <typename T> constexpr bool kPrioHalf = sizeof(T) == 8 && NW_PRIO64;
__device__ __forceinline__ void prio_half(int t, int threads) {
    if (__builtin_amdgcn_readfirstlane(t) >= threads / 2) __builtin_amdgcn_s_setprio(1);
}
template <typename T, int E, int OUT>
constexpr int kWpsOf = sizeof(T) == 8 ? kWpsF64 : OUT == kOutPhSum ? kWpsPhSum
                     : (OUT == kOutPSum && E >= 32) ? kWpsPSum32 : kWpsF32;

// WSH: the W-row support table wnz was built for the output kernels' E << WSH elements per
// thread (the partial-sum kernels may run at a smaller E): a row whose elements r >= nz are
// zero at E << WSH has elements r >= max(1, nz >> WSH) zero here
template <typename T, int N, int E, int OUT, bool REALW, int WSH = 0>
__global__ __launch_bounds__(N / E, (kWpsOf<T, E, OUT>)) void nw_fused_kernel(WDesc d, const cplx<T>* __restrict__ X,
                                                            const void* __restrict__ wtab, void* __restrict__ out,
                                                            const C2<T>* __restrict__ tw, int64_t nsig, int group,
                                                            int nsg_pad, const int* __restrict__ wnz, int tg) {
    using G = Geometry<N, E>;
    using WT = typename WLoad<T, REALW>::type;
    constexpr bool XD = kXDMA<T, E, REALW>;
    // the LDS-DMA copies dma_rounds_for(nzv) rounds of the bins pass-0 variant nzv reads; with a
    // shifted support table (WSH > 0: nz = wnz >> WSH can be 6 or 10, between the variants) it
    // would copy fewer bins than the dispatched variant reads.  The shift only occurs for the
    // E = 16 partial-sum kernels, which never DMA (kXdmaMinE = 32)
    static_assert(!XD || WSH == 0, "X LDS-DMA needs the unshifted W-support table");
    extern __shared__ __align__(16) unsigned char smem[];
    T* lds = reinterpret_cast<T*>(smem);
    const int t = threadIdx.x;
    if constexpr (kPrioHalf<T> && XD) prio_half(t, N / E);   // the measured case: E = 32 output kernels

    // XCD-aware block -> (scale, signal group).  Blocks b, b+8, b+16, ... share an XCD
    // (and its 4 MiB L2); the ~64 of them resident at a time cover a tile of
    // kTileF scales x kTileG signal groups, so each W row is read by kTileG blocks
    // and each X group by kTileF blocks from L2 (W + X of a tile ~2.5 MiB), and
    // the XCD sweeps all scales of its groups before moving on.
    const int b = blockIdx.x;
    const int xcd = b & 7;
    const int local = b >> 3;
    constexpr int TF = kTileFT<T>;
    const int pos = local % (TF * tg);
    const int round = local / (TF * tg);
    const int nfr = (d.nfreq + TF - 1) / TF;
    const int fi = (round % nfr) * TF + pos % TF;
    const int sg = ((round / nfr) * tg + pos / TF) * 8 + xcd;
    if (fi >= d.nfreq || sg >= nsg_pad || (int64_t)sg * group >= nsig) return;
    const int64_t s_begin = (int64_t)sg * group;
    const int64_t s_end = min(nsig, s_begin + group);

    // W[f, k] at the thread's bins (1/n folded in), from the device-built table (L2-shared
    // by the XCD tile).  E <= kWregMaxE: held in registers for the whole block, loaded
    // before any store is in flight; E = 32: re-read per signal (no VGPRs to spare).
    const WT* wrow = reinterpret_cast<const WT*>(wtab) + (int64_t)fi * N;
    const uint32_t wo = (uint32_t)t * (uint32_t)sizeof(WT);
    constexpr bool WREG = E <= kWregMaxE && !(sizeof(T) == 8 && N / E > 512);
    WT w[WREG ? E : 1];
    if constexpr (WREG) {
#pragma unroll
        for (int r = 0; r < E; ++r) w[r] = *at(wrow, wo, (uint32_t)(r * G::T * sizeof(WT)));
    }
    // E = 32: the first WKEEP elements of W stay in registers for the block (a row pruned to
    // NZ <= WKEEP reads no W per signal; loads issued after the previous signal's stores
    // wait for all of them in the in-order vmcnt queue)
    constexpr int WKEEP = (!WREG && REALW && sizeof(T) == 4) ? (N >= 16384 ? kWKeep32 : kWKeep32Small)
                        : (!WREG && REALW && sizeof(T) == 8 && N == 16384) ? kWKeep64 : 0;
    WT wk[WKEEP > 0 ? WKEEP : 1];
    if constexpr (WKEEP > 0) {
#pragma unroll
        for (int r = 0; r < WKEEP; ++r) wk[r] = *at(wrow, wo, (uint32_t)(r * G::T * sizeof(WT)));
    }
    auto w_at = [&](int r) -> WT {
        if constexpr (WREG) return w[r];
        else if (r < WKEEP) return wk[r < WKEEP ? r : 0];
#ifdef NW_ABL_NOWLOAD   // diagnostic only (wrong results): W beyond WKEEP without its global loads
        else { WT z{}; if constexpr (REALW) z = (T)(r + 1); return z; }
#else
        else return *at(wrow, wo, (uint32_t)(r * G::T * sizeof(WT)));
#endif
    };

#ifdef NW_STAMPS
    Stamps stamps{};
    Stamps* st = &stamps;
    st->last = nw_now();
#else
    Stamps* st = nullptr;
#endif
    Tab1<T, N, E>::fill(lds, tw, t);   // read after the first exchange's barriers
    TwSplit<T, N, E>::fill(lds, tw, t);
    if constexpr (TwSplit<T, N, E>::ON) lds_barrier();   // read before the first exchange
    C2<T> x[E];
    const int64_t out_esz = (int64_t)(OUT == NW_OUT_CWT ? sizeof(C2<T>) : sizeof(T));
    // XDMA: X[N/2] (the real Nyquist bin, outside the DMA'd half) of the signal being
    // transformed, carried one signal ahead in registers so its load never queues behind
    // a store and is never folded into a private/LDS pointer select
    C2<T> nyq{T(0), T(0)};
    if constexpr (XD) {
        nyq = reinterpret_cast<const C2<T>*>(X + s_begin * d.nh)[N / 2];
        const int nzv0 = pass0_variant<T, N, E, OUT>(max(1, wnz[fi] >> WSH));
        dma_x<T, N, G::T>(reinterpret_cast<const C2<T>*>(X + s_begin * d.nh),
                          lds, t, nzv0 <= E / 2 ? dma_rounds_for<T>(nzv0) : 1 << 30);
    }
    // W row support (device-built with the table): elements r >= nz of pass 0 multiply an
    // exactly-zero W for every thread of the block (k = t + r*T beyond the row's last
    // nonzero bin), so they are neither read nor multiplied and the DIF stages skip them
    const int nz = max(1, wnz[fi] >> WSH);
    NW_DCHECK(fi < d.nfreq && s_end <= nsig && d.n == N && nz <= E);
    // LDS-DMA only the X bins the pruned pass 0 reads: variant NZ (>= 4) reads bins < NZ*T,
    // i.e. NZ/2 rounds of 2*T bins (fp32; NZ rounds of T bins in fp64), when it reads no
    // mirrored bin (NZ <= E/2)
    const int nzv = pass0_variant<T, N, E, OUT>(nz);
    static_assert(kPruneMin == 4, "the smallest pass-0 variant");
    const int dma_rounds = nzv <= E / 2 ? dma_rounds_for<T>(nzv) : 1 << 30;
    // power partial sums (kOutPSum): sum over the block's signals of |y|^2 per output point
    // (kOutPhSum: the sums of y / |y|, two fp64 values per point)
    constexpr bool PSUM = OUT == kOutPSum || OUT == kOutPhSum;
    constexpr int NACC = OUT == kOutPhSum ? 2 : 1;
    double acc[PSUM ? NACC * E : 1];
    if constexpr (PSUM) {
#pragma unroll
        for (int e = 0; e < NACC * E; ++e) acc[e] = 0.0;
    }
    for (int64_t s = s_begin; s < s_end; ++s) {
        const C2<T>* xl = nullptr;
        if constexpr (XD) {
            // this wave's DMA landed (only the stores issued after it may be pending),
            // then every wave's: the whole X[0 .. N/2) is in LDS
            // (the partial-sum modes store nothing after the DMA: nothing may stay pending)
            if (s == s_begin || PSUM) wait_vmcnt<0>(); else wait_vmcnt<LastStores<T, N, E, OUT>::COUNT>();
            lds_barrier();
            xl = reinterpret_cast<const C2<T>*>(lds);
        }
        C2<T> v[E];
        // pass 0 (Ns = 1): z = W * X at k = t + r*T, r < NZ, radix-E IDFT in registers
        auto pass0 = [&]<int NZ>() {
            if constexpr (XD) {
                // the lane index made opaque HERE: LDS reads are speculatable, and hoisted
                // above the variant dispatch they would all be live at once and spill
                int tl = t;
                asm volatile("" : "+v"(tl));
                // X[N - k] for r >= E/2 from ONE base (the lowest address, r = E-1) and positive
                // immediate offsets: DS offsets are unsigned, so N - t - r*T per r would hold
                // E/2 address registers
                const C2<T>* xm = xl + (N - (E - 1) * G::T - tl);
#pragma unroll
                for (int r = 0; r < NZ; ++r) {
                    if (r < E / 2) {
                        x[r] = xl[tl + r * G::T];
                    } else {                        // X[N - k]; k = N/2 (t = 0, r = E/2) is the Nyquist bin
                        x[r] = xm[(E - 1 - r) * G::T];  // value copies: `c ? nyq : xl[m]` is an
                        if (r == E / 2 && t == 0) x[r] = nyq;   // lvalue select (nyq -> scratch)
                        x[r].im = -x[r].im;
                    }
                }
            } else {
                load_x<T, N, E, NZ>(x, reinterpret_cast<const C2<T>*>(X + s * d.nh), t);
            }
#pragma unroll
            for (int r = 0; r < E; ++r)
                v[r] = r < NZ ? WLoad<T, REALW>::apply(w_at(r), x[r]) : C2<T>{T(0), T(0)};
            idft_br<T, E, NZ>(v);
        };
        if (nzv == 4) pass0.template operator()<4>();
        else if (nzv == 8) pass0.template operator()<8>();
        else if (kNzFineOut<T, N, E, OUT> && nzv == 12) pass0.template operator()<(E > 16 ? 12 : E)>();
        else if (E > 16 && nzv == 16) pass0.template operator()<(E > 16 ? 16 : E)>();
        else if (kNzFineOut<T, N, E, OUT> && nzv == 20) pass0.template operator()<(E > 16 ? 20 : E)>();
        else if (kNz24Of<T, N, E> && nzv == 24) pass0.template operator()<(E > 16 ? 24 : E)>();
        else pass0.template operator()<E>();
        if constexpr (XD) {
            if (s + 1 < s_end) nyq = sload_c2(reinterpret_cast<const C2<T>*>(X + (s + 1) * d.nh) + N / 2);
        }
        NW_STAMP(st, 0);                       // pass 0: X wait + radix-E arithmetic
        const C2<T>* xs_next = s + 1 < s_end ? reinterpret_cast<const C2<T>*>(X + (s + 1) * d.nh) : nullptr;
        void* ocur = (char*)out + (s * d.nfreq + fi) * (int64_t)N * out_esz;   // row of signal s
        passes_from<T, N, E, OUT, 1, XD, (sizeof(T) == 8 ? kStoreGlobalNt : kStoreGlobal)>(
            v, lds, t, tw, x, xs_next, ocur, st, nullptr, dma_rounds, PSUM ? acc : nullptr);
    }
    if constexpr (PSUM) {
        // the block's partial: row (group sg, scale fi) of the (groups, F, N) partial buffer
        using IL = PassInfo<N, E, G::npass() - 1, (int)sizeof(T)>;
        double* prow = reinterpret_cast<double*>(out) + ((int64_t)sg * d.nfreq + fi) * (int64_t)N * NACC;
#pragma unroll
        for (int q = 0; q < IL::Q; ++q)
#pragma unroll
            for (int i = 0; i < IL::R; ++i) {
                const int k = IL::bfly(t, q) + bitrev<IL::R>(i) * IL::NS, e = q * IL::R + i;
                if constexpr (NACC == 1) {
                    prow[k] = acc[e];
                } else {
                    *reinterpret_cast<double2*>(prow + 2 * k) = double2{acc[2 * e], acc[2 * e + 1]};
                }
            }
    }
    // the last signal's outputs
    NW_STAMP(st, kStampsStore);
#ifdef NW_STAMPS
    if ((t & 63) == 0) {
        for (int k = 0; k < kStamps; ++k) atomicAdd(&g_nw_stamps[k], stamps.acc[k]);
        atomicAdd(&g_nw_stamps[kStamps], (unsigned long long)(s_end - s_begin));
    }
#endif
}

// Signal pairs (fp32, E = 16, analytic real W rows): the block's signals are transformed
// two at a time, each lane value a C2<f2> holding signal s in the low and s+1 in the high
// half, so every butterfly, twiddle multiply and LDS access of the FFT serves two signals
// (v_pk_add/mul/fma_f32; 8-B image slots; twiddles and the pass-1 table shared).  Pass 0
// reads both X rows and the block's W registers; the last pass stores each half to its
// own row (an odd last signal transforms a duplicate whose high half is not stored).
// |y| and |y|^2 read X from L2 in pass 0; cwt takes the next pair's X by LDS-DMA before the
// stores (XD below).  4 waves/SIMD; the power partials' E fp64 accumulators take it to 3.
template <int N, int E, int OUT>
__global__ __launch_bounds__(N / E, OUT == kOutPSum ? 3 : 4) void nw_fused_pair_kernel(WDesc d, const cplx<float>* __restrict__ X,
                                                                  const void* __restrict__ wtab, void* __restrict__ out,
                                                                  const C2<float>* __restrict__ tw, int64_t nsig,
                                                                  int group, int nsg_pad, const int* __restrict__ wnz,
                                                                  int tg) {
    using G = Geometry<N, E>;
    static_assert(E <= 16, "pair mode holds 2 x E complex values per lane");
    extern __shared__ __align__(16) unsigned char smem[];
    f2* lds = reinterpret_cast<f2*>(smem);
    const int t = threadIdx.x;
    // XCD-aware block -> (scale, signal group): as nw_fused_kernel
    const int b = blockIdx.x;
    const int xcd = b & 7;
    const int local = b >> 3;
    const int pos = local % (kTileF * tg);
    const int round = local / (kTileF * tg);
    const int nfr = (d.nfreq + kTileF - 1) / kTileF;
    const int fi = (round % nfr) * kTileF + pos % kTileF;
    const int sg = ((round / nfr) * tg + pos / kTileF) * 8 + xcd;
    if (fi >= d.nfreq || sg >= nsg_pad || (int64_t)sg * group >= nsig) return;
    const int64_t s_begin = (int64_t)sg * group;
    // the block's signal count, pinned in an SGPR: as an int64 min it sat in a VGPR pair that
    // was spilled, and its reload at the top of every pair iteration waited (vmcnt(0)) for all
    // of the previous pair's stores
    const int cnt = __builtin_amdgcn_readfirstlane((int)(min(nsig, s_begin + group) - s_begin));

    const float* wrow = reinterpret_cast<const float*>(wtab) + (int64_t)fi * N;
    const uint32_t wo = (uint32_t)t * (uint32_t)sizeof(float);
    // the block's W elements r < kPairWKeep in registers; the rest (read only by the NZ = E
    // pass 0: analytic rows end at the Nyquist bin, r <= E/2) re-read from L2 there.  All E
    // kept spilled 4 of them (16-24 B of scratch at 128 VGPRs) in the |y| / |y|^2 kernels
    constexpr int WK = (OUT == NW_OUT_CWT || OUT == NW_OUT_POWER ? kPairWKeep : kPairWKeepRed) < E
                           ? (OUT == NW_OUT_CWT || OUT == NW_OUT_POWER ? kPairWKeep : kPairWKeepRed) : E;
    float w[WK];
#pragma unroll
    for (int r = 0; r < WK; ++r) w[r] = *at(wrow, wo, (uint32_t)(r * G::T * sizeof(float)));
    auto w_at = [&](int r) { return r < WK ? w[r < WK ? r : 0] : *at(wrow, wo, (uint32_t)(r * G::T * sizeof(float))); };
    Tab1<f2, N, E>::fill(lds, tw, t);
    const int64_t out_esz = (int64_t)(OUT == NW_OUT_CWT ? sizeof(C2<float>) : sizeof(float));
    const int nz = wnz[fi];
    NW_DCHECK(fi < d.nfreq && s_begin + cnt <= nsig && d.n == N && nz >= 1 && nz <= E);
    auto xrow = [&](int64_t s) { return reinterpret_cast<const C2<float>*>(X + s * d.nh); };
    // XD: the next pair's X[0 .. N/2) (both signals, or only the bins a pruned pass 0 reads) by
    // LDS-DMA into the idle image before the stores, as nw_fused_kernel at E = 32; the Nyquist
    // bins by scalar loads
    // (cwt only: n = 4096 cwt 1.585 -> 1.567 ms per 256-signal launch; |y|^2 slower, C3 1.180 ->
    // 1.210, n = 1024 power equal)
#ifdef NW_PAIR_XD_ALL   // diagnostic A/B: the LDS-DMA for every output kind
    constexpr bool XD = kPairXD && OUT != kOutPSum;
#else
    constexpr bool XD = kPairXD && OUT == NW_OUT_CWT;
#endif
    const int nzv = nz < kPruneMin ? kPruneMin : nz;
    const int dma_rounds = nzv <= E / 2 ? dma_rounds_for<float>(nzv) : 1 << 30;
    unsigned long long nyq_a = 0, nyq_b = 0;
    if constexpr (XD) {
        const int64_t sb = cnt > 1 ? s_begin + 1 : s_begin;
        nyq_a = sload_u64(xrow(s_begin) + N / 2);
        nyq_b = sload_u64(xrow(sb) + N / 2);
        dma_x<float, N, G::T>(xrow(s_begin), lds, t, dma_rounds);
        dma_x<float, N, G::T>(xrow(sb), reinterpret_cast<char*>(lds) + (N / 2) * sizeof(C2<float>), t, dma_rounds);
    }
    // power partial sums (kOutPSum): as nw_fused_kernel, both signals of a pair into one sum
    constexpr bool PSUM = OUT == kOutPSum;
    double acc[PSUM ? E : 1];
    if constexpr (PSUM) {
#pragma unroll
        for (int e = 0; e < E; ++e) acc[e] = 0.0;
    }
    for (int i = 0; i < cnt; i += 2) {
        const int64_t s = s_begin + i;
        const bool two = i + 1 < cnt;
        const int64_t s2 = two ? s + 1 : s;
        C2<f2> v[E];
        if constexpr (XD) {
            // this wave's DMA landed (only the previous pair's 2 x COUNT stores may be pending),
            // then every wave's
            if (i == 0) wait_vmcnt<0>(); else wait_vmcnt<2 * LastStores<float, N, E, OUT, kStoreBuffer>::COUNT>();
            lds_barrier();
        }
        auto pass0 = [&]<int NZ>() {
            C2<float> xa[E], xb[E];
            if constexpr (XD) {
                int tl = t;                         // opaque: the LDS reads stay below the dispatch
                asm volatile("" : "+v"(tl));
                const C2<float>* la = reinterpret_cast<const C2<float>*>(lds);
                const C2<float>* lb = la + N / 2;
                const C2<float>* ma = la + (N - (E - 1) * G::T - tl);
                const C2<float>* mb = lb + (N - (E - 1) * G::T - tl);
#pragma unroll
                for (int r = 0; r < NZ; ++r) {
                    if (r < E / 2) {
                        xa[r] = la[tl + r * G::T];
                        xb[r] = lb[tl + r * G::T];
                    } else {                        // X[N - k]; k = N/2 (t = 0, r = E/2) is the Nyquist bin
                        C2<float> va = ma[(E - 1 - r) * G::T], vb = mb[(E - 1 - r) * G::T];
                        if (r == E / 2) {
                            // values in registers first: a select of the two sources would become
                            // a load through a selected pointer (the Nyquist bin via scratch)
                            asm volatile("" : "+v"(va.re), "+v"(va.im), "+v"(vb.re), "+v"(vb.im));
                            const C2<float> na = c2_of_u64(nyq_a), nb = c2_of_u64(nyq_b);
                            const bool z = t == 0;
                            va = C2<float>{z ? na.re : va.re, z ? na.im : va.im};
                            vb = C2<float>{z ? nb.re : vb.re, z ? nb.im : vb.im};
                        }
                        xa[r] = C2<float>{va.re, -va.im};
                        xb[r] = C2<float>{vb.re, -vb.im};
                    }
                }
            } else {
                load_x<float, N, E, NZ>(xa, xrow(s), t);
                load_x<float, N, E, NZ>(xb, xrow(s2), t);
            }
#pragma unroll
            for (int r = 0; r < E; ++r) {
                if (r < NZ) {
                    const float wr = w_at(r);
                    v[r] = C2<f2>{f2{wr * xa[r].re, wr * xb[r].re}, f2{wr * xa[r].im, wr * xb[r].im}};
                } else {
                    v[r] = C2<f2>{f2{0.0f, 0.0f}, f2{0.0f, 0.0f}};
                }
            }
            idft_br<f2, E, NZ>(v);
        };
        if (nz <= 4) pass0.template operator()<4>();
        else if (nz <= 8) pass0.template operator()<8>();
        else if (nz <= 12) pass0.template operator()<12>();
        else pass0.template operator()<E>();
        void* o1 = (char*)out + (s * d.nfreq + fi) * (int64_t)N * out_esz;
        void* o2 = two ? (void*)((char*)out + (s2 * d.nfreq + fi) * (int64_t)N * out_esz) : nullptr;
        // the next pair (signals s + 2 and s + 3, or s + 2 twice when it is the odd last one)
        const C2<float>* xn_a = nullptr;
        const C2<float>* xn_b = nullptr;
        if constexpr (XD) {
            if (i + 2 < cnt) {
                xn_a = xrow(s + 2);
                xn_b = i + 3 < cnt ? xrow(s + 3) : xn_a;
                nyq_a = sload_u64(xn_a + N / 2);
                nyq_b = sload_u64(xn_b + N / 2);
            }
        }
        passes_from<f2, N, E, OUT, 1, XD, kStoreBuffer>(v, lds, t, tw, nullptr,
                                                       reinterpret_cast<const C2<f2>*>(xn_a), o1, nullptr, o2,
                                                       dma_rounds, PSUM ? acc : nullptr, xn_b);
    }
    if constexpr (PSUM) {
        using IL = PassInfo<N, E, G::npass() - 1, (int)sizeof(float), true>;
        double* prow = reinterpret_cast<double*>(out) + ((int64_t)sg * d.nfreq + fi) * (int64_t)N;
#pragma unroll
        for (int q = 0; q < IL::Q; ++q)
#pragma unroll
            for (int i = 0; i < IL::R; ++i) prow[IL::bfly(t, q) + bitrev<IL::R>(i) * IL::NS] = acc[q * IL::R + i];
    }
}

// Forward R2C of the signals for the fused engine (replaces rocFFT's two-kernel R2C and the
// copy it needs, since rocFFT may use its input as scratch): one block per signal, the same
// pass machinery on v[r] = x[t + r*T] (imaginary parts zero), X[k] = conj(y[k]) for k <= n/2
// (scipy/rocFFT's unnormalised forward transform, base.py:399).
template <typename T, int N, int E>
__global__ __launch_bounds__(N / E, sizeof(T) == 8 ? kWpsF64 : kWpsF32) void fwd_r2c_kernel(const T* __restrict__ x,
                                                                              C2<T>* __restrict__ X,
                                                                              const C2<T>* __restrict__ tw,
                                                                              int64_t nh) {
    using G = Geometry<N, E>;
    extern __shared__ __align__(16) unsigned char smem[];
    T* lds = reinterpret_cast<T*>(smem);
    const int t = threadIdx.x;
    const int64_t s = blockIdx.x;
    Tab1<T, N, E>::fill(lds, tw, t);
    TwSplit<T, N, E>::fill(lds, tw, t);
    if constexpr (TwSplit<T, N, E>::ON) lds_barrier();
    const T* xs = x + s * (int64_t)N;
    const uint32_t xo = (uint32_t)t * (uint32_t)sizeof(T);
    C2<T> v[E];
#pragma unroll
    for (int r = 0; r < E; ++r) v[r] = C2<T>{*at(xs, xo, (uint32_t)(r * G::T * sizeof(T))), T(0)};
    idft_br<T, E>(v);
    passes_from<T, N, E, kOutXHalf, 1, false>(v, lds, t, tw, nullptr, nullptr, X + s * nh, nullptr);
}

// W[f, k] for the fused engine: the reference's cached row, pad_to'd to n, 1/n folded
// in (real rows for analytic kinds, complex for tables).  Built once per plan+wavelet.
template <typename T, bool REALW>
__global__ __launch_bounds__(256) void wtable_kernel(WDesc d, void* wtab) {
    const int fi = blockIdx.y;
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= d.n) return;
    cplx<T> w = wavelet_bin<T>(d, fi, k);
    if (k >= d.xlim) w = cplx<T>{T(0), T(0)};   // interpolate_alias of X (base.py:400-401)
    if constexpr (REALW)
        reinterpret_cast<T*>(wtab)[(int64_t)fi * d.n + k] = w.re;
    else
        reinterpret_cast<C2<T>*>(wtab)[(int64_t)fi * d.n + k] = C2<T>{w.re, w.im};
}

// Support of each W row for pass-0 pruning: wnz[f] >= the number of pass-0 elements r
// (bins k = t + r*T, t < T) reaching the row's last bin above kTailRel x its max, i.e. elements
// r >= wnz[f] see only the row's negligible tail for every thread (they run as zeros): the
// next power of two up to 4, then the next multiple
// of 4 (the pass-0 variants: NZ = 4, 8, 12, 16 at E = 16; 4, 8, 12, 16, 20, 24, 32 at E = 32
// fp32; a multiple of 2^WSH, so nz >> WSH is exact for the partial-sum kernels' smaller E).
// Rows pruned in steps of 4 elements: C3 1.205 -> 1.186 ms per launch (NZ = 12 at E = 16).
// The support ends at the last bin above kTailRel x the row's max |W| (nw_internal.h).
template <typename T, bool REALW>
__global__ __launch_bounds__(256) void wsupport_kernel(const void* wtab, int64_t n, int tt, int e, int* wnz) {
    __shared__ int kmax[256];
    __shared__ T wmax[256];
    const int fi = blockIdx.x;
    auto mag = [&](int64_t k) -> T {
        if constexpr (REALW) return fabs(reinterpret_cast<const T*>(wtab)[(int64_t)fi * n + k]);
        const C2<T> w = reinterpret_cast<const C2<T>*>(wtab)[(int64_t)fi * n + k];
        return fmax(fabs(w.re), fabs(w.im));
    };
    T mx = T(0);
    for (int64_t k = threadIdx.x; k < n; k += 256) mx = fmax(mx, (T)tail_max_term((double)mag(k)));
    wmax[threadIdx.x] = mx;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) wmax[threadIdx.x] = fmax(wmax[threadIdx.x], wmax[threadIdx.x + w]);
        __syncthreads();
    }
    const double thr = kTailRel<T> * (double)wmax[0];
    int m = -1;
    for (int64_t k = threadIdx.x; k < n; k += 256)
        if (tail_in_support((double)mag(k), thr)) m = (int)k;
    kmax[threadIdx.x] = m;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) kmax[threadIdx.x] = max(kmax[threadIdx.x], kmax[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const int need = kmax[0] < 0 ? 1 : kmax[0] / tt + 1;   // elements 0 .. need-1 can be nonzero
        int p2 = 1;
        while (p2 < need && p2 < 8) p2 <<= 1;
        if (p2 < need) p2 = (need + 3) / 4 * 4;
        wnz[fi] = p2 < e ? p2 : e;
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
        hipLaunchKernelGGL(twiddle_table_kernel<float>, (unsigned)((n + 255) / 256), 256, 0, 0, (C2<float>*)p, (int)n);
    else
        hipLaunchKernelGGL(twiddle_table_kernel<double>, (unsigned)((n + 255) / 256), 256, 0, 0, (C2<double>*)p, (int)n);
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


template <typename T, int N, int E>
hipError_t launch_forward(const void* x, void* X, int64_t nsig, int64_t nh, hipStream_t s) {
    void* tw = nullptr;
    hipError_t e = twiddles_for(N, sizeof(T) == 4 ? NW_F32 : NW_F64, &tw);
    if (e != hipSuccess) return e;
    const int lds = kLdsBytes<T, N, E>;
    e = hipFuncSetAttribute((const void*)fwd_r2c_kernel<T, N, E>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    if (nsig > 0x7fffffff) return hipErrorInvalidConfiguration;
    nw_launch(fwd_r2c_kernel<T, N, E>, (unsigned)nsig, N / E, lds, s, reinterpret_cast<const T*>(x), reinterpret_cast<C2<T>*>(X),
                                                             reinterpret_cast<const C2<T>*>(tw), nh);
    return hipGetLastError();
}

// bytes of the W rows in the table buffer (the wnz[nfreq] support array follows them)
size_t wtab_row_bytes(int64_t n, int nfreq, size_t esz, bool realw) {
    const size_t b = (size_t)n * nfreq * esz * (realw ? 1 : 2);
    return (b + 15) / 16 * 16;
}

template <typename T, int E, bool REALW>
constexpr bool kPairMode = std::is_same<T, float>::value && E <= 16 && REALW;

// Signals per block of the output kernels: `base`, halved (to 2) while a launch would fill the
// chip fewer than kMinRounds times over (512 resident 512-thread blocks): a small launch (C2:
// 64 signals x 128 scales = 1024 blocks of 8, two rounds) otherwise ends on a tail of long
// blocks.  NW_FUSED_GROUP=<g> fixes it (diagnostic A/B).
constexpr int64_t kMinRounds = 4, kResidentBlocks = 512;
int group_for(int base, int64_t nsig, int nfreq) {
    static const int fixed = [] {
        const char* v = std::getenv("NW_FUSED_GROUP");
        return v ? std::atoi(v) : 0;
    }();
    if (fixed > 0) return fixed;
    int g = base;
    while (g > 2 && (nsig + g - 1) / g * (int64_t)nfreq < kMinRounds * kResidentBlocks) g /= 2;
    return g;
}

template <typename T, int N, int E, bool REALW>
hipError_t launch_n(const WDesc& d, int out_kind, const void* X, const void* wtab, void* out, int64_t nsig,
                    hipStream_t s) {
    constexpr int threads = N / E;
    const size_t lds = (size_t)kLdsBytes<T, N, E>;
    void* tw = nullptr;
    hipError_t e = twiddles_for(N, sizeof(T) == 4 ? NW_F32 : NW_F64, &tw);
    if (e != hipSuccess) return e;
    const int grp = kPairMode<T, E, REALW> ? kGroup : group_for(kGroupOut<T, N>, nsig, d.nfreq);
    const int64_t nsg = (nsig + grp - 1) / grp;
    constexpr int TF = kTileFT<T>;
    const int TG = tile_g_of(nsg, kTileGOut<T, N>);
    const int64_t nsg_pad = (nsg + 8 * TG - 1) / (8 * TG) * (8 * TG);
    const int64_t nfr = (d.nfreq + TF - 1) / TF;
    const int64_t blocks = nsg_pad * nfr * TF;
    if (blocks > 0x7fffffff || nsg_pad > 0x7fffffff) return hipErrorInvalidConfiguration;
    const cplx<T>* Xc = reinterpret_cast<const cplx<T>*>(X);
    const C2<T>* twc_ = reinterpret_cast<const C2<T>*>(tw);
    const int* wnz = reinterpret_cast<const int*>(reinterpret_cast<const char*>(wtab) +
                                                  wtab_row_bytes(N, d.nfreq, sizeof(T), REALW));
    if constexpr (kPairMode<T, E, REALW>) {
        const size_t lp = (size_t)kLdsBytes<f2, N, E>;
        const C2<float>* twf = reinterpret_cast<const C2<float>*>(tw);
        const cplx<float>* Xf = reinterpret_cast<const cplx<float>*>(X);
        if (out_kind == NW_OUT_CWT)
            nw_launch(nw_fused_pair_kernel<N, E, NW_OUT_CWT>, blocks, threads, lp, s, d, Xf, wtab, out, twf, nsig, kGroup, (int)nsg_pad, wnz, TG);
        else if (out_kind == NW_OUT_POWER)
            nw_launch(nw_fused_pair_kernel<N, E, NW_OUT_POWER>, blocks, threads, lp, s, d, Xf, wtab, out, twf, nsig, kGroup, (int)nsg_pad, wnz, TG);
        else
            nw_launch(nw_fused_pair_kernel<N, E, NW_OUT_ABS>, blocks, threads, lp, s, d, Xf, wtab, out, twf, nsig, kGroup, (int)nsg_pad, wnz, TG);
        return hipGetLastError();
    }
    if (out_kind == NW_OUT_CWT)
        nw_launch(nw_fused_kernel<T, N, E, NW_OUT_CWT, REALW>, blocks, threads, lds, s, d, Xc, wtab, out, twc_, nsig, grp, (int)nsg_pad, wnz, TG);
    else if (out_kind == NW_OUT_POWER)
        nw_launch(nw_fused_kernel<T, N, E, NW_OUT_POWER, REALW>, blocks, threads, lds, s, d, Xc, wtab, out, twc_, nsig, grp, (int)nsg_pad, wnz, TG);
    else
        nw_launch(nw_fused_kernel<T, N, E, NW_OUT_ABS, REALW>, blocks, threads, lds, s, d, Xc, wtab, out, twc_, nsig, grp, (int)nsg_pad, wnz, TG);
    return hipGetLastError();
}

template <typename T, int N, int E, int OUT, int WSH>
hipError_t launch_psum(const WDesc& d, const void* X, const void* wtab, void* partials, int64_t nsig, hipStream_t s) {
    constexpr int threads = N / E;
    const int lds = kLdsBytes<T, N, E>;
    void* tw = nullptr;
    hipError_t e = twiddles_for(N, sizeof(T) == 4 ? NW_F32 : NW_F64, &tw);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute((const void*)nw_fused_kernel<T, N, E, OUT, true, WSH>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    const int64_t nsg = (nsig + kGroup - 1) / kGroup;
    constexpr int TF = kTileFT<T>;
    const int TG = tile_g_of(nsg, kTileGT<T>);
    const int64_t nsg_pad = (nsg + 8 * TG - 1) / (8 * TG) * (8 * TG);
    const int64_t nfr = (d.nfreq + TF - 1) / TF;
    const int64_t blocks = nsg_pad * nfr * TF;
    if (blocks > 0x7fffffff || nsg_pad > 0x7fffffff) return hipErrorInvalidConfiguration;
    const int* wnz = reinterpret_cast<const int*>(reinterpret_cast<const char*>(wtab) +
                                                  wtab_row_bytes(N, d.nfreq, sizeof(T), true));
    if constexpr (OUT == kOutPSum && kPairMode<T, E, true>) {
        // power partials on the signal-pair kernel: the same values as its power output
        const int lp = kLdsBytes<f2, N, E>;
        e = hipFuncSetAttribute((const void*)nw_fused_pair_kernel<N, E, kOutPSum>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lp);
        if (e != hipSuccess) return e;
        nw_launch(nw_fused_pair_kernel<N, E, kOutPSum>, blocks, threads, lp, s, 
            d, reinterpret_cast<const cplx<float>*>(X), wtab, partials, reinterpret_cast<const C2<float>*>(tw), nsig,
            kGroup, (int)nsg_pad, wnz, TG);
        return hipGetLastError();
    }
    nw_launch(nw_fused_kernel<T, N, E, OUT, true, WSH>, blocks, threads, lds, s, 
        d, reinterpret_cast<const cplx<T>*>(X), wtab, partials, reinterpret_cast<const C2<T>*>(tw), nsig, kGroup,
        (int)nsg_pad, wnz, TG);
    return hipGetLastError();
}

template <typename T, int N, int E, bool REALW>
hipError_t prepare_one() {
    if constexpr (kPairMode<T, E, REALW>) {
        const int lp = kLdsBytes<f2, N, E>;
        hipError_t e = hipFuncSetAttribute((const void*)nw_fused_pair_kernel<N, E, NW_OUT_CWT>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lp);
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void*)nw_fused_pair_kernel<N, E, NW_OUT_POWER>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lp);
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void*)nw_fused_pair_kernel<N, E, NW_OUT_ABS>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lp);
        if (e != hipSuccess) return e;
    }
    const int lds = kLdsBytes<T, N, E>;
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

hipError_t fused_twiddles(int64_t n, int dtype, void** out) { return twiddles_for(n, dtype, out); }

// power-of-two n: 2^10..2^14 in fp32 and fp64 (fp64 at 8192 / 16384: E = 32 with 256 VGPRs,
// W re-read per signal)
bool fused_supported(int64_t n, int dtype) {
    if (n < 1024 || (n & (n - 1))) return false;
    return (dtype == NW_F32 || dtype == NW_F64) && n <= 16384;
}

// Elements per thread E of each fused size (threads = n / E).  Measured: fp32 n = 4096 at
// E = 32 slower (0.350 -> 0.404 ms power); n = 8192 at E = 32 vs 16: power 0.887 -> 0.768 ms,
// cwt 1.034 -> 0.926; fp64 at n >= 8192: E = 32 (3 passes, 256 VGPRs, 2 waves/SIMD) vs E = 16
// (4 passes): 8192 cwt 2.907 -> 2.573 ms, power 2.397 -> 1.991; 16384 cwt 3.447 -> 3.124,
// power 2.615 -> 2.312 (256 x 256 rows; 128 x 256 at 16384).
#define NW_FUSED_TABLE(X)                                                               \
    X(float, 1024, 16) X(float, 2048, 16) X(float, 4096, 16) X(float, 8192, 32) X(float, 16384, 32) \
    X(double, 1024, 16) X(double, 2048, 16) X(double, 4096, 16) X(double, 8192, 32) X(double, 16384, 32)

hipError_t fused_prepare(int64_t n, int dtype) {
#define NW_PREP(TY, NN, EE) \
    if (n == NN && dtype == (sizeof(TY) == 4 ? NW_F32 : NW_F64)) return prepare_n<TY, NN, EE>();
    NW_FUSED_TABLE(NW_PREP)
#undef NW_PREP
    return hipErrorNotSupported;
}

size_t fused_wtable_bytes(int64_t n, int nfreq, int dtype, int kind) {
    const size_t esz = dtype == NW_F32 ? sizeof(float) : sizeof(double);
    return wtab_row_bytes(n, nfreq, esz, kind != NW_TABLE) + (size_t)nfreq * sizeof(int);   // + wnz[nfreq]
}

hipError_t build_wtable(const WDesc& d, int dtype, void* wtab, hipStream_t s) {
    dim3 grid((unsigned)((d.n + 255) / 256), (unsigned)d.nfreq);
    const bool realw = d.kind != NW_TABLE;
    const size_t esz = dtype == NW_F32 ? sizeof(float) : sizeof(double);
    int* wnz = reinterpret_cast<int*>(reinterpret_cast<char*>(wtab) + wtab_row_bytes(d.n, d.nfreq, esz, realw));
    int e = 0;
#define NW_E_OF(TY, NN, EE) \
    if (d.n == NN && dtype == (sizeof(TY) == 4 ? NW_F32 : NW_F64)) e = EE;
    NW_FUSED_TABLE(NW_E_OF)
#undef NW_E_OF
    if (e == 0) return hipErrorNotSupported;
    const int tt = (int)(d.n / e);
    if (dtype == NW_F32) {
        if (realw) nw_launch(wtable_kernel<float, true>, grid, 256, 0, s, d, wtab);
        else nw_launch(wtable_kernel<float, false>, grid, 256, 0, s, d, wtab);
        if (realw) nw_launch(wsupport_kernel<float, true>, d.nfreq, 256, 0, s, wtab, d.n, tt, e, wnz);
        else nw_launch(wsupport_kernel<float, false>, d.nfreq, 256, 0, s, wtab, d.n, tt, e, wnz);
    } else {
        if (realw) nw_launch(wtable_kernel<double, true>, grid, 256, 0, s, d, wtab);
        else nw_launch(wtable_kernel<double, false>, grid, 256, 0, s, d, wtab);
        if (realw) nw_launch(wsupport_kernel<double, true>, d.nfreq, 256, 0, s, wtab, d.n, tt, e, wnz);
        else nw_launch(wsupport_kernel<double, false>, d.nfreq, 256, 0, s, wtab, d.n, tt, e, wnz);
    }
    return hipGetLastError();
}

// epoch power / phase partials: analytic rows; fp32 power to E = 32, fp32 phases and fp64 at E = 16
// Elements per thread of the partial-sum kernels (EO: the output kernels'): fp32 power keeps
// EO (E = 32 at n = 8192 / 16384: E fp64 accumulators at 2 waves/SIMD); fp32 phases (2E fp64
// accumulators) and fp64 (the drop-in's default dtype, 2 waves/SIMD already at 256 VGPRs)
// run at E = 16 -- n = 8192 / 16384 then take 512 / 1024 threads, the W-support table
// shifted by log2(EO / 16) (nw_fused_kernel's WSH)
template <typename T, int EO, bool PHASE>
constexpr int kPsE = (EO >= 32 && (PHASE || sizeof(T) == 8)) ? 16 : EO;
template <int EO, int E> constexpr int kPsShift = EO == E ? 0 : EO == 2 * E ? 1 : 2;
// combinations whose accumulators fit without spilling (tools/regs.py): at 1024 threads
// (n = 16384, E = 16) a wave has 128 VGPRs, and neither fp64 power (228 B of scratch) nor
// phases (fp32: 84 B) fit there -- n = 16384 keeps the chunk path for those
template <typename T, int N, int EO>
constexpr bool kPSumOK = !(sizeof(T) == 8 && N / kPsE<T, EO, false> > 512);
template <typename T, int N, int EO>
constexpr bool kPhSumOK = N / kPsE<T, EO, true> <= 512;

bool fused_psum_supported(int64_t n, int dtype, int kind, bool phase) {
    if (kind == NW_TABLE) return false;
#define NW_PS(TY, NN, EE) \
    if (n == NN && dtype == (sizeof(TY) == 4 ? NW_F32 : NW_F64)) return phase ? kPhSumOK<TY, NN, EE> : kPSumOK<TY, NN, EE>;
    NW_FUSED_TABLE(NW_PS)
#undef NW_PS
    return false;
}

int64_t fused_psum_groups(int64_t nsig) { return (nsig + kGroup - 1) / kGroup; }

int fused_psum_kernel_id(int64_t n, int dtype, bool phase) {
#define NW_PK_ID(TY, NN, EE) \
    if (n == NN && dtype == (sizeof(TY) == 4 ? NW_F32 : NW_F64)) \
        return (!phase && kPairMode<TY, EE, true>) ? NW_K_FUSED_PAIR : NW_K_FUSED;
    NW_FUSED_TABLE(NW_PK_ID)
#undef NW_PK_ID
    return NW_K_NONE;
}

hipError_t fused_power_partials(const WDesc& d, int dtype, bool phase, const void* X, const void* wtab,
                                void* partials, int64_t nsig, hipStream_t s) {
#define NW_PSL(TY, NN, EE)                                                                                    \
    if (d.n == NN && dtype == (sizeof(TY) == 4 ? NW_F32 : NW_F64)) {                                          \
        if constexpr (kPhSumOK<TY, NN, EE>) {                                                                 \
            constexpr int PE = kPsE<TY, EE, true>;                                                            \
            if (phase) return launch_psum<TY, NN, PE, kOutPhSum, kPsShift<EE, PE>>(d, X, wtab, partials, nsig, s); \
        }                                                                                                     \
        if constexpr (kPSumOK<TY, NN, EE>) {                                                                  \
            constexpr int PE = kPsE<TY, EE, false>;                                                           \
            if (!phase) return launch_psum<TY, NN, PE, kOutPSum, kPsShift<EE, PE>>(d, X, wtab, partials, nsig, s); \
        }                                                                                                     \
        return hipErrorNotSupported;                                                                          \
    }
    NW_FUSED_TABLE(NW_PSL)
#undef NW_PSL
    return hipErrorNotSupported;
}

hipError_t fused_forward(int64_t n, int dtype, const void* x, void* X, int64_t nsig, int64_t nh, hipStream_t s) {
#define NW_FWD(TY, NN, EE) \
    if (n == NN && dtype == (sizeof(TY) == 4 ? NW_F32 : NW_F64)) return launch_forward<TY, NN, EE>(x, X, nsig, nh, s);
    NW_FUSED_TABLE(NW_FWD)
#undef NW_FWD
    return hipErrorNotSupported;
}

int fused_kernel_id(int64_t n, int dtype, int kind) {
    const bool realw = kind != NW_TABLE;
#define NW_KID(TY, NN, EE)                                                                      \
    if (n == NN && dtype == (sizeof(TY) == 4 ? NW_F32 : NW_F64))                                \
        return (realw ? kPairMode<TY, EE, true> : kPairMode<TY, EE, false>) ? NW_K_FUSED_PAIR : NW_K_FUSED;
    NW_FUSED_TABLE(NW_KID)
#undef NW_KID
    return NW_K_NONE;
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

#ifdef NW_STAMPS
// diagnostic builds only: per-phase cycle sums (and the signal-wave count in [8])
extern "C" int nw_debug_stamps(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(nw::g_nw_stamps), sizeof(unsigned long long) * 9) != hipSuccess)
        return -2;
    if (reset) {
        unsigned long long z[9] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(nw::g_nw_stamps), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#endif
