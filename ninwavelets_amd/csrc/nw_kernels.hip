// nw_kernels.hip — gfx950 kernels of the rocFFT engine:
//   K1  spectrum multiply  Y[s,f,k] = W[f,k] * X[s,k] / n      (base.py:396-406)
//   K2  epilogue           |Y| or |Y|^2                          (base.py:409-443)
//   rows                   the cached wavelet rows themselves     (base.py:221-279)
//   accumulate / finalize  epoch reductions power / ITC          (mneutils.py:42-71)
//   baseline               Baseline correction                   (base.py:18-68)
//   normal_time / finish   MexicanHat / Haar rows on the device  (base.py:249-256)
//   wavelet_*              time-domain wavelets, make_wavelet(s)  (base.py:346-376)
//   expand_rows            copies of repeated scale rows (Shannon ignores f)
//
// K1 is HBM-write bound (8 or 16 B per output point, X re-read from L2): each
// block evaluates W for one scale f and a 256*V-bin tile ONCE into registers,
// then sweeps a group of signals, so the transcendental cost of psi is
// amortised over the group.  Stores are 16 B per lane (float4 / double2).
#include <type_traits>

#include "nw_dcheck.h"
#include "nw_internal.h"

namespace nw {

constexpr int K1_THREADS = 256;
constexpr int K1_GROUP = 16;   // signals per block

template <typename T, int V, bool ALIGNED>
__global__ __launch_bounds__(K1_THREADS) void k1_multiply(WDesc d, const cplx<T>* __restrict__ X,
                                                          cplx<T>* __restrict__ Y, int64_t nsig) {
    const int fi = blockIdx.y;
    const int64_t k0 = ((int64_t)blockIdx.x * K1_THREADS + threadIdx.x) * V;
    if (k0 >= d.n) return;
    cplx<T> w[V];
#pragma unroll
    for (int v = 0; v < V; ++v) w[v] = (k0 + v < d.n) ? wavelet_bin<T>(d, fi, k0 + v) : cplx<T>{T(0), T(0)};

    const int64_t s_begin = (int64_t)blockIdx.z * K1_GROUP;
    const int64_t s_end = min(nsig, s_begin + K1_GROUP);
    for (int64_t s = s_begin; s < s_end; ++s) {
        const cplx<T>* Xs = X + s * d.nh;
        cplx<T> y[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const cplx<T> x = spectrum_bin<T>(Xs, d, k0 + v);
            y[v].re = w[v].re * x.re - w[v].im * x.im;
            y[v].im = w[v].re * x.im + w[v].im * x.re;
        }
        cplx<T>* Yrow = Y + (s * d.nfreq + fi) * d.n;
        if (ALIGNED) {
            // V complex values = 16 B contiguous (V=2 for fp32, V=1 for fp64)
            using vec = typename std::conditional<sizeof(T) == 4, float4, double2>::type;
            vec o;
            if constexpr (sizeof(T) == 4) {
                o.x = y[0].re; o.y = y[0].im; o.z = y[V - 1].re; o.w = y[V - 1].im;
            } else {
                o.x = y[0].re; o.y = y[0].im;
            }
            *reinterpret_cast<vec*>(Yrow + k0) = o;
        } else {
#pragma unroll
            for (int v = 0; v < V; ++v)
                if (k0 + v < d.n) Yrow[k0 + v] = y[v];
        }
    }
}

hipError_t launch_multiply(const WDesc& d, int dtype, const void* X, void* Y, int64_t nsig, hipStream_t s) {
    const int V = dtype == NW_F32 ? 2 : 1;
    dim3 grid((unsigned)((d.n + (int64_t)K1_THREADS * V - 1) / ((int64_t)K1_THREADS * V)), (unsigned)d.nfreq,
              (unsigned)((nsig + K1_GROUP - 1) / K1_GROUP));
    if (dtype == NW_F32) {
        if (d.n % 2 == 0)
            nw_launch(k1_multiply<float, 2, true>, grid, K1_THREADS, 0, s, d, (const cplx<float>*)X, (cplx<float>*)Y, nsig);
        else
            nw_launch(k1_multiply<float, 2, false>, grid, K1_THREADS, 0, s, d, (const cplx<float>*)X, (cplx<float>*)Y, nsig);
    } else {
        nw_launch(k1_multiply<double, 1, true>, grid, K1_THREADS, 0, s, d, (const cplx<double>*)X, (cplx<double>*)Y, nsig);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K2: |y|^2 (power) or |y| (abs), grid-stride, 2 complex per lane per step.
// ---------------------------------------------------------------------------
template <typename T, bool POWER>
__global__ __launch_bounds__(256) void k2_epilogue(const cplx<T>* __restrict__ Y, T* __restrict__ out, int64_t count) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
        const cplx<T> y = Y[i];
        const T p = y.re * y.re + y.im * y.im;
        out[i] = POWER ? p : (T)hypot(y.re, y.im);
    }
}

hipError_t launch_epilogue(int dtype, int out_kind, const void* Y, void* out, int64_t count, hipStream_t s) {
    const int64_t blocks = std::min<int64_t>((count + 255) / 256, 256 * 16);
    if (dtype == NW_F32) {
        if (out_kind == NW_OUT_POWER)
            nw_launch(k2_epilogue<float, true>, blocks, 256, 0, s, (const cplx<float>*)Y, (float*)out, count);
        else
            nw_launch(k2_epilogue<float, false>, blocks, 256, 0, s, (const cplx<float>*)Y, (float*)out, count);
    } else {
        if (out_kind == NW_OUT_POWER)
            nw_launch(k2_epilogue<double, true>, blocks, 256, 0, s, (const cplx<double>*)Y, (double*)out, count);
        else
            nw_launch(k2_epilogue<double, false>, blocks, 256, 0, s, (const cplx<double>*)Y, (double*)out, count);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// rows: the reference's cached fft_wavelets rows on the build grid (no pad_to,
// no 1/n): real rows for analytic kinds, complex rows for TABLE.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_rows(WDesc d, T* __restrict__ rows) {
    const int fi = blockIdx.y;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= d.len_full) return;
    if (d.kind == NW_TABLE) {
        const cplx<T>* t = reinterpret_cast<const cplx<T>*>(d.table) + (int64_t)fi * d.len_full;
        reinterpret_cast<cplx<T>*>(rows)[(int64_t)fi * d.len_full + j] = j < d.row_len[fi] ? t[j] : cplx<T>{T(0), T(0)};
    } else {
        rows[(int64_t)fi * d.len_full + j] = j < d.len_valid ? psi<T>(d, fi, j) : T(0);
    }
}

hipError_t launch_rows(const WDesc& d, int dtype, void* rows, hipStream_t s) {
    dim3 grid((unsigned)((d.len_full + 255) / 256), (unsigned)d.nfreq);
    if (dtype == NW_F32)
        nw_launch(k_rows<float>, grid, 256, 0, s, d, (float*)rows);
    else
        nw_launch(k_rows<double>, grid, 256, 0, s, d, (double*)rows);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Epoch reductions (mneutils.py:42-71).  acc[f, k] (fp64) += the chunk's signals in
// signal order -- numpy's np.mean(axis=0) adds the (F, N) slabs one after another,
// then divides by the count.  One thread per (f, k), coalesced across k; each
// signal's slab is S_STRIDE = F*n elements further on.
//   ACC_POWER_REAL : src = |y|^2 (real T, the fused kernel's power output)
//   ACC_POWER_Y    : src = y (complex T)  -> |y|^2
//   ACC_PHASE_Y    : src = y (complex T)  -> y/|y| in fp64; 0/0 -> NaN (mneutils.py:68)
// ---------------------------------------------------------------------------
template <typename T, int SRC>
__global__ __launch_bounds__(256) void k_accumulate(const void* __restrict__ src, double* __restrict__ acc,
                                                    int64_t fn, int64_t c) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < fn; i += stride) {
        if constexpr (SRC == ACC_PHASE_Y) {
            double re = acc[2 * i], im = acc[2 * i + 1];
            const cplx<T>* y = reinterpret_cast<const cplx<T>*>(src) + i;
            for (int64_t s = 0; s < c; ++s) {
                const cplx<T> v = y[s * fn];
                const double a = hypot((double)v.re, (double)v.im);
                re += (double)v.re / a;
                im += (double)v.im / a;
            }
            acc[2 * i] = re;
            acc[2 * i + 1] = im;
        } else {
            double p = acc[i];
            for (int64_t s = 0; s < c; ++s) {
                if constexpr (SRC == ACC_POWER_REAL) {
                    p += (double)reinterpret_cast<const T*>(src)[s * fn + i];
                } else {
                    const cplx<T> v = reinterpret_cast<const cplx<T>*>(src)[s * fn + i];
                    p += (double)v.re * (double)v.re + (double)v.im * (double)v.im;
                }
            }
            acc[i] = p;
        }
    }
}

hipError_t launch_accumulate(int dtype, int src_kind, const void* src, double* acc, int64_t fn, int64_t c,
                             hipStream_t s) {
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((fn + 255) / 256, 256 * 32));
#define NW_ACC(T)                                                                                         \
    switch (src_kind) {                                                                                   \
        case ACC_POWER_REAL: nw_launch(k_accumulate<T, ACC_POWER_REAL>, blocks, 256, 0, s, src, acc, fn, c); break; \
        case ACC_POWER_Y: nw_launch(k_accumulate<T, ACC_POWER_Y>, blocks, 256, 0, s, src, acc, fn, c); break;       \
        default: nw_launch(k_accumulate<T, ACC_PHASE_Y>, blocks, 256, 0, s, src, acc, fn, c); break;               \
    }
    if (dtype == NW_F32) {
        NW_ACC(float)
    } else {
        NW_ACC(double)
    }
#undef NW_ACC
    return hipGetLastError();
}

// mean = acc / nsig (np.mean's true_divide by the count); ITC = |(re, im) / nsig|
template <typename T, bool ITC>
__global__ __launch_bounds__(256) void k_finalize(const double* __restrict__ acc, T* __restrict__ out, int64_t fn,
                                                  double nsig) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < fn; i += stride) {
        if constexpr (ITC)
            out[i] = (T)hypot(acc[2 * i] / nsig, acc[2 * i + 1] / nsig);
        else
            out[i] = (T)(acc[i] / nsig);
    }
}

hipError_t launch_finalize(int dtype, bool itc, const double* acc, void* out, int64_t fn, int64_t nsig,
                           hipStream_t s) {
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((fn + 255) / 256, 256 * 32));
    const double d = (double)nsig;
    if (dtype == NW_F32) {
        if (itc) nw_launch(k_finalize<float, true>, blocks, 256, 0, s, acc, (float*)out, fn, d);
        else nw_launch(k_finalize<float, false>, blocks, 256, 0, s, acc, (float*)out, fn, d);
    } else {
        if (itc) nw_launch(k_finalize<double, true>, blocks, 256, 0, s, acc, (double*)out, fn, d);
        else nw_launch(k_finalize<double, false>, blocks, 256, 0, s, acc, (double*)out, fn, d);
    }
    return hipGetLastError();
}

// acc[i] += src[i] (fp64 partial sums of several devices, added in device order)
__global__ __launch_bounds__(256) void k_add_f64(double* __restrict__ acc, const double* __restrict__ src,
                                                 int64_t count) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) acc[i] += src[i];
}

hipError_t launch_add_f64(double* acc, const double* src, int64_t count, hipStream_t s) {
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((count + 255) / 256, 256 * 32));
    nw_launch(k_add_f64, blocks, 256, 0, s, acc, src, count);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// WaveletMode.Normal rows (base.py:249-256 with make_wavelet 346-359 and
// _setup_waveletshape 196-216).  Row f of the FFT scratch: `half` zeros, the
// time-domain wavelet at np.arange's points (t0, t1 = t0 + step, then t0 + i*delta
// with delta = t1 - t0, exactly as numpy fills a float arange), `half` zeros.
// Round-to-nearest intrinsics keep every product and sum unfused, as numpy's.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double mexican_hat_f(double tc, double sigma) {
    // (1 - np.power(tc / sigma, 2)) * np.exp(-np.square(tc) / np.square(sigma) / 2)  (wavelets.py:219-221)
    const double a = __ddiv_rn(tc, sigma);
    const double e = exp(__ddiv_rn(__ddiv_rn(-__dmul_rn(tc, tc), __dmul_rn(sigma, sigma)), 2.0));
    return __dmul_rn(__dsub_rn(1.0, __dmul_rn(a, a)), e);
}
__device__ __forceinline__ double haar_f(double tc) {          // wavelets.py:272-280
    return (tc > 0.0 && tc <= 1.0) ? 1.0 : ((tc > -1.0 && tc <= 0.0) ? -1.0 : 0.0);
}

__global__ __launch_bounds__(256) void k_normal_time(const NormalRow* __restrict__ rows, int kind, double sigma,
                                                     double2* __restrict__ buf) {
    const NormalRow r = rows[blockIdx.x];
    for (int64_t j = threadIdx.x; j < r.len; j += blockDim.x) {
        const int64_t i = j - r.half;
        double v = 0.0;
        if (i >= 0 && i < r.m) {
            const double t = i == 0 ? r.t0 : (i == 1 ? r.t1 : __dadd_rn(r.t0, __dmul_rn((double)i, r.delta)));
            v = kind == NW_MEXICAN_HAT ? mexican_hat_f(t, sigma) : haar_f(t);
        }
        buf[r.off + j] = double2{v, 0.0};
    }
}

hipError_t launch_normal_time(const NormalRow* rows, int nrows, int64_t, int kind, double sigma, void* buf,
                              hipStream_t s) {
    if (nrows > 0) nw_launch(k_normal_time, nrows, 256, 0, s, rows, kind, sigma, (double2*)buf);
    return hipGetLastError();
}

// table[f][j] = |Re| + i|Im| of the row's spectrum (base.py:255-256), zero past its
// length and, when interpolating, from int(len/2) on (interpolate_alias, base.py:107-123)
template <typename T>
__global__ __launch_bounds__(256) void k_normal_finish(const NormalRow* __restrict__ rows, int64_t lmax, int interp,
                                                       const double2* __restrict__ buf, cplx<T>* __restrict__ table) {
    const NormalRow r = rows[blockIdx.x];
    const int64_t keep = interp ? r.len / 2 : r.len;
    cplx<T>* row = table + (int64_t)blockIdx.x * lmax;
    for (int64_t j = threadIdx.x; j < lmax; j += blockDim.x) {
        cplx<T> v{T(0), T(0)};
        if (j < keep) {
            const double2 z = buf[r.off + j];
            v = cplx<T>{(T)fabs(z.x), (T)fabs(z.y)};
        }
        row[j] = v;
    }
}

hipError_t launch_normal_finish(const NormalRow* rows, int nrows, int64_t lmax, bool interp, const void* buf,
                                int dtype, void* table, hipStream_t s) {
    if (nrows > 0) {
        if (dtype == NW_F32)
            nw_launch(k_normal_finish<float>, nrows, 256, 0, s, rows, lmax, interp, (const double2*)buf, (cplx<float>*)table);
        else
            nw_launch(k_normal_finish<double>, nrows, 256, 0, s, rows, lmax, interp, (const double2*)buf, (cplx<double>*)table);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Time-domain wavelets (make_wavelet, base.py:346-376).
// Reverse kinds (Morse, Shannon): the spectrum with its default freq = 1 on
// t_j = j * (1/f) (np.arange(0, sfreq/f*rwl, 1/f): start 0, so the fill is exact j*step),
// then rocFFT's unnormalised inverse, then `wavelet_pack`: the centre slice
// [m//2, m//2*3) of hstack(conj(flip(w)), w), scaled by 1/m as scipy's ifft.
// Time kinds (Morlet, MexicanHat, Haar): the formula on the zero-mean timeline.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_wavelet_spectra(const WaveRow* __restrict__ rows, WaveParams wp,
                                                         double2* __restrict__ buf) {
    const WaveRow r = rows[blockIdx.x];
    for (int64_t j = threadIdx.x; j < r.m; j += blockDim.x) {
        const double x = (double)j * r.delta;
        double v;
        if (wp.kind == NW_MORSE) {        // wavelets.py:65-74 with freq = 1
            const double step = x > 0.0 ? 1.0 : (x == 0.0 ? x : 0.0);
            v = 2.0 * (step * pow(x, wp.b) * exp(wp.b_over_r * (1.0 - pow(x, wp.r))));
        } else {                          // Shannon, wavelets.py:256-262
            v = x <= 1.0 ? 1.0 : 0.0;
        }
        buf[r.off + j] = double2{v, 0.0};
    }
}

hipError_t launch_wavelet_spectra(const WaveRow* rows, int nrows, WaveParams wp, void* buf, hipStream_t s) {
    if (nrows > 0) nw_launch(k_wavelet_spectra, nrows, 256, 0, s, rows, wp, (double2*)buf);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_wavelet_pack(const WaveRow* __restrict__ rows, int64_t maxlen,
                                                      const double2* __restrict__ buf, double2* __restrict__ out) {
    const WaveRow r = rows[blockIdx.x];
    const double fct = 1.0 / (double)r.m;
    double2* row = out + (int64_t)blockIdx.x * maxlen;
    for (int64_t j = threadIdx.x; j < maxlen; j += blockDim.x) {
        double2 v{0.0, 0.0};
        if (j < r.len) {
            const int64_t pos = j + r.m / 2;
            if (pos < r.m) {
                const double2 w = buf[r.off + (r.m - 1 - pos)];
                v = double2{w.x * fct, -(w.y * fct)};
            } else {
                const double2 w = buf[r.off + (pos - r.m)];
                v = double2{w.x * fct, w.y * fct};
            }
        }
        row[j] = v;
    }
}

hipError_t launch_wavelet_pack(const WaveRow* rows, int nrows, int64_t maxlen, const void* buf, void* out,
                               hipStream_t s) {
    if (nrows > 0) nw_launch(k_wavelet_pack, nrows, 256, 0, s, rows, maxlen, (const double2*)buf, (double2*)out);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_wavelet_time(const WaveRow* __restrict__ rows, int64_t maxlen, WaveParams wp,
                                                      double2* __restrict__ out) {
    const WaveRow r = rows[blockIdx.x];
    double2* row = out + (int64_t)blockIdx.x * maxlen;
    for (int64_t j = threadIdx.x; j < maxlen; j += blockDim.x) {
        double2 v{0.0, 0.0};
        if (j < r.m) {
            const double t = j == 0 ? r.t0 : (j == 1 ? r.t1 : __dadd_rn(r.t0, __dmul_rn((double)j, r.delta)));
            if (wp.kind == NW_MORLET) {   // c pi^-1/4 exp(-t^2/2) (exp(i sigma t) - k), wavelets.py:138-141
                const double a = __dmul_rn(wp.cpi, exp(__ddiv_rn(-__dmul_rn(t, t), 2.0)));
                const double ph = __dmul_rn(wp.sigma, t);
                v = double2{__dmul_rn(a, __dsub_rn(cos(ph), wp.kappa)), __dmul_rn(a, sin(ph))};
            } else if (wp.kind == NW_MEXICAN_HAT) {
                v = double2{mexican_hat_f(t, wp.sigma), 0.0};
            } else {
                v = double2{haar_f(t), 0.0};
            }
        }
        row[j] = v;
    }
}

hipError_t launch_wavelet_time(const WaveRow* rows, int nrows, int64_t maxlen, WaveParams wp, void* out,
                               hipStream_t s) {
    if (nrows > 0) nw_launch(k_wavelet_time, nrows, 256, 0, s, rows, maxlen, wp, (double2*)out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Baseline correction (base.py:18-68).  The statistics of the slice x[b0, b1) -- one
// scalar mean and population std over ALL its elements (baseline.mean(), np.std) -- are
// reduced in fp64 in a fixed order: per-block partials over a grid-stride loop, then
// one block over the partials (deterministic, run to run).  PASS 0 sums x, PASS 1 sums
// (x - mean)^2 with the mean read back from stats[0].
// ---------------------------------------------------------------------------
constexpr int BL_THREADS = 256;
constexpr int BL_BLOCKS = 1024;

template <int PASS>
__device__ __forceinline__ double block_sum(double v) {
    __shared__ double sh[BL_THREADS];
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int w = BL_THREADS / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    return sh[0];
}

template <typename T, int PASS>
__global__ __launch_bounds__(BL_THREADS) void k_bl_partial(const T* __restrict__ x, int64_t b0, int64_t b1,
                                                           const double* __restrict__ stats,
                                                           double* __restrict__ part) {
    const double m = PASS == 1 ? stats[0] : 0.0;
    double acc = 0.0;
    for (int64_t i = b0 + (int64_t)blockIdx.x * BL_THREADS + threadIdx.x; i < b1; i += (int64_t)gridDim.x * BL_THREADS) {
        const double v = (double)x[i];
        acc += PASS == 0 ? v : (v - m) * (v - m);
    }
    const double tot = block_sum<PASS>(acc);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// stats[PASS] = sum(part) / count  (PASS 1: sqrt -> population std); 0/0 = NaN for an
// empty slice, as numpy's mean / std of nothing
template <int PASS>
__global__ __launch_bounds__(BL_THREADS) void k_bl_final(const double* __restrict__ part, int nparts, int64_t count,
                                                         double* __restrict__ stats) {
    double acc = 0.0;
    for (int i = threadIdx.x; i < nparts; i += BL_THREADS) acc += part[i];
    const double tot = block_sum<PASS>(acc);
    if (threadIdx.x == 0) {
        const double q = tot / (double)count;
        stats[PASS] = PASS == 0 ? q : sqrt(q);
    }
}

// out = op(x) in the data's precision, with the statistics rounded to it (a float32 array
// has float32 basemean / std in the reference, whose arithmetic order is kept:
// base.py:53-68)
template <typename T>
__global__ __launch_bounds__(256) void k_bl_apply(const T* __restrict__ x, T* __restrict__ out, int64_t count,
                                                  int op, const double* __restrict__ stats) {
    const T m = (T)stats[0], sd = (T)stats[1];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
        const T v = x[i];
        T r;
        switch (op) {
            case NW_BL_MEAN: r = v - m; break;
            case NW_BL_RATIO: r = v / m; break;
            case NW_BL_PERCENT: r = (v - m) / m; break;
            case NW_BL_LOG: r = log10(v / m); break;
            case NW_BL_ZSCORE: r = (v - m) / sd; break;
            default: r = log10(v / m) / sd; break;      // NW_BL_ZLOG
        }
        out[i] = r;
    }
}

hipError_t launch_baseline(int dtype, const void* x, int64_t count, int64_t b0, int64_t b1, int op, void* out,
                           double* work /* BL_BLOCKS + 2 doubles */, hipStream_t s) {
    double* part = work;
    double* stats = work + BL_BLOCKS;
    const int64_t n = std::max<int64_t>(0, b1 - b0);
    const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(BL_BLOCKS, (n + BL_THREADS - 1) / BL_THREADS));
    const int64_t ab = std::max<int64_t>(1, std::min<int64_t>((count + 255) / 256, 256 * 32));
    if (dtype == NW_F32) {
        nw_launch(k_bl_partial<float, 0>, nb, BL_THREADS, 0, s, (const float*)x, b0, b1, stats, part);
        nw_launch(k_bl_final<0>, 1, BL_THREADS, 0, s, part, nb, n, stats);
        nw_launch(k_bl_partial<float, 1>, nb, BL_THREADS, 0, s, (const float*)x, b0, b1, stats, part);
        nw_launch(k_bl_final<1>, 1, BL_THREADS, 0, s, part, nb, n, stats);
        if (count > 0) nw_launch(k_bl_apply<float>, ab, 256, 0, s, (const float*)x, (float*)out, count, op, stats);
    } else {
        nw_launch(k_bl_partial<double, 0>, nb, BL_THREADS, 0, s, (const double*)x, b0, b1, stats, part);
        nw_launch(k_bl_final<0>, 1, BL_THREADS, 0, s, part, nb, n, stats);
        nw_launch(k_bl_partial<double, 1>, nb, BL_THREADS, 0, s, (const double*)x, b0, b1, stats, part);
        nw_launch(k_bl_final<1>, 1, BL_THREADS, 0, s, part, nb, n, stats);
        if (count > 0) nw_launch(k_bl_apply<double>, ab, 256, 0, s, (const double*)x, (double*)out, count, op, stats);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Repeated rows (nw_plan::dedup): dst[s][f][:] = src[s][u][:] for every scale f whose
// wavelet row is the u-th distinct one (order[offs[u] .. offs[u + 1])).  Each block
// reads one tile of a computed row once and streams it to all of its copies, so the
// HBM traffic is the output write plus 1/(F/U) of it read: write-bound.
// ---------------------------------------------------------------------------
template <typename V>
__global__ __launch_bounds__(256) void k_expand_rows(const V* __restrict__ src, V* __restrict__ dst, int64_t rowv,
                                                     int64_t tiles, int64_t nblk, int nu, int nf,
                                                     const int32_t* __restrict__ offs,
                                                     const int32_t* __restrict__ order) {
    for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        const int64_t su = b / tiles;               // s * nu + u
        const int64_t k = (b - su * tiles) * 256 + threadIdx.x;
        if (k >= rowv) continue;
        const int u = (int)(su % nu);
        const V v = src[su * rowv + k];
        V* base = dst + (su / nu) * nf * rowv + k;
        const int i1 = offs[u + 1];
        NW_DCHECK(offs[u] <= i1 && i1 <= nf);
        for (int i = offs[u]; i < i1; ++i) {
            NW_DCHECK(order[i] >= 0 && order[i] < nf);
            __builtin_nontemporal_store(v, base + (int64_t)order[i] * rowv);
        }
    }
}

// dst[i] = src[idx[i]] for elements of elem_bytes (a multiple of 4): the compacted per-row
// arrays (and table rows) of a row subset
__global__ __launch_bounds__(256) void k_gather_elems(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                      const int32_t* __restrict__ idx, int count, int64_t words) {
    const int64_t total = (int64_t)count * words;
    for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < total; g += (int64_t)gridDim.x * 256) {
        const int64_t i = g / words, w = g - i * words;
        dst[g] = src[(int64_t)idx[i] * words + w];
    }
}

__global__ __launch_bounds__(64) void k_dcheck_selftest(int n) { NW_DCHECK((int)threadIdx.x < n); }

hipError_t launch_dcheck_selftest(hipStream_t s) {
    nw_launch(k_dcheck_selftest, 1, 64, 0, s, 32);
    return hipGetLastError();
}

hipError_t launch_gather(const void* src, void* dst, const int32_t* idx, int count, size_t elem_bytes, hipStream_t s) {
    if (count <= 0 || elem_bytes == 0) return hipSuccess;
    if (elem_bytes % 4) return hipErrorInvalidValue;
    const int64_t words = (int64_t)(elem_bytes / 4);
    const int64_t blocks = std::min<int64_t>(((int64_t)count * words + 255) / 256, int64_t(1) << 16);
    nw_launch(k_gather_elems, (unsigned)blocks, 256, 0, s, (const uint32_t*)src, (uint32_t*)dst, idx, count, words);
    return hipGetLastError();
}

hipError_t launch_expand_rows(const void* src, void* dst, int64_t nsig, int nu, int nf, size_t row_bytes,
                              const int32_t* offs, const int32_t* order, hipStream_t s) {
    using V4 = unsigned int __attribute__((ext_vector_type(4)));
    using V2 = unsigned int __attribute__((ext_vector_type(2)));
    auto go = [&](auto* tag, size_t vb) {
        using V = std::remove_pointer_t<decltype(tag)>;
        const int64_t rowv = (int64_t)(row_bytes / vb);
        const int64_t tiles = (rowv + 255) / 256;
        const int64_t nblk = nsig * nu * tiles;
        if (nblk == 0) return;
        const int64_t grid = std::min<int64_t>(nblk, int64_t(1) << 20);
        nw_launch(k_expand_rows<V>, (unsigned)grid, 256, 0, s, (const V*)src, (V*)dst, rowv, tiles, nblk, nu, nf, offs, order);
    };
    if (row_bytes % 16 == 0) go((V4*)nullptr, 16);
    else if (row_bytes % 8 == 0) go((V2*)nullptr, 8);
    else go((unsigned int*)nullptr, 4);
    return hipGetLastError();
}

}  // namespace nw
