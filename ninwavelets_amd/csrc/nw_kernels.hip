// nw_kernels.hip — gfx950 kernels of the rocFFT engine:
//   K1  spectrum multiply  Y[s,f,k] = W[f,k] * X[s,k] / n      (base.py:396-406)
//   K2  epilogue           |Y| or |Y|^2                          (base.py:409-443)
//   rows                   the cached wavelet rows themselves     (base.py:221-279)
//
// K1 is HBM-write bound (8 or 16 B per output point, X re-read from L2): each
// block evaluates W for one scale f and a 256*V-bin tile ONCE into registers,
// then sweeps a group of signals, so the transcendental cost of psi is
// amortised over the group.  Stores are 16 B per lane (float4 / double2).
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
            k1_multiply<float, 2, true><<<grid, K1_THREADS, 0, s>>>(d, (const cplx<float>*)X, (cplx<float>*)Y, nsig);
        else
            k1_multiply<float, 2, false><<<grid, K1_THREADS, 0, s>>>(d, (const cplx<float>*)X, (cplx<float>*)Y, nsig);
    } else {
        k1_multiply<double, 1, true><<<grid, K1_THREADS, 0, s>>>(d, (const cplx<double>*)X, (cplx<double>*)Y, nsig);
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
            k2_epilogue<float, true><<<blocks, 256, 0, s>>>((const cplx<float>*)Y, (float*)out, count);
        else
            k2_epilogue<float, false><<<blocks, 256, 0, s>>>((const cplx<float>*)Y, (float*)out, count);
    } else {
        if (out_kind == NW_OUT_POWER)
            k2_epilogue<double, true><<<blocks, 256, 0, s>>>((const cplx<double>*)Y, (double*)out, count);
        else
            k2_epilogue<double, false><<<blocks, 256, 0, s>>>((const cplx<double>*)Y, (double*)out, count);
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
        k_rows<float><<<grid, 256, 0, s>>>(d, (float*)rows);
    else
        k_rows<double><<<grid, 256, 0, s>>>(d, (double*)rows);
    return hipGetLastError();
}

}  // namespace nw
