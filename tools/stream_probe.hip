// stream_probe.hip -- the HBM floor of the C5 column pass's traffic.
//
// The column pass (nw_large.hip cols_kernel, fp32 at C5) reads B[f][k1][n2] (complex64,
// k1 < N1 = 1024, n2 < N2 = 16384) and writes out[f][n2 + N2 * n1]: per workgroup C
// consecutive columns n2, i.e. N1 pieces of C * 8 bytes strided by N2 * 8 = 128 KiB on both
// sides.  This program moves exactly those bytes (read B once, write out once, no arithmetic)
// in several geometries and prints the rate of each:
//   copy      : contiguous 16-B float4 copy of the same bytes (the device's mixed-stream roof)
//   colsC     : the column pass's geometry with C columns per workgroup (C * 8-B pieces):
//               C = 32 is the product (256-B pieces), 64 / 128 what larger column blocks would do
//   rowsonly  : the row pass's write pattern (contiguous 128-KiB rows of B) for reference
// Every workgroup loads all its pieces into registers before storing any (the product's order).
//   hipcc --offload-arch=gfx950 -O3 -o tools/stream_probe tools/stream_probe.hip
//   ./tools/stream_probe [scales=64] [reps=5]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

constexpr int N1 = 1024, N2 = 16384;
typedef float f4 __attribute__((ext_vector_type(4)));

// contiguous copy: every thread moves 16 float4 (256 B), loads first
__global__ __launch_bounds__(1024) void copy_kernel(const f4* __restrict__ src, f4* __restrict__ dst, long n4) {
    const long base = ((long)blockIdx.x * 1024 * 16) + threadIdx.x;
    f4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const long k = base + (long)i * 1024;
        v[i] = k < n4 ? __builtin_nontemporal_load(src + k) : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const long k = base + (long)i * 1024;
        if (k < n4) __builtin_nontemporal_store(v[i], dst + k);
    }
}

// column geometry: workgroup (f, group of C columns); lanes own 2 columns (16 B); the
// workgroup's 1024 threads cover C/2 lanes per k1 row and 2048/C rows per pass over the
// threads; N1 rows in total -> PER = N1 * C / 2048 float4 per thread
// RS / WS: read / write side in the strided column geometry (false: the workgroup's N1 * C
// complex values as one contiguous block instead).  XCD: workgroup b runs on XCD b % 8; with
// XCD = true each XCD takes a contiguous run of (scale, column group)s, so the ~32 workgroups
// resident on one XCD at a time hold ADJACENT column groups (their pieces of one output row
// form one 8-KiB span); false: consecutive workgroups (on 8 different XCDs) take adjacent
// groups.  NT: nontemporal stores (the product's), else plain (write-back through L2).
// ROT: output row order rotated per workgroup, n1 -> (n1 + g * ROT) % N1 (0: the product's order,
// every workgroup walks the rows from 0 at the same time)
template <int C, bool RS = true, bool WS = true, bool XCD = false, bool NT = true, int ROT = 0>
__global__ __launch_bounds__(1024) void cols_kernel(const f4* __restrict__ B, f4* __restrict__ out, int nf) {
    constexpr int LANES = C / 2;             // float4 per piece
    constexpr int ROWS = 1024 / LANES;       // k1 rows per pass over the threads
    constexpr int PER = N1 / ROWS;           // float4 per thread
    const int groups = N2 / C;
    const int nb = nf * groups;
    const int v = XCD ? (int)(blockIdx.x & 7) * (nb / 8) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
    const int f = v / groups;
    const int g = v % groups;
    if (f >= nf) return;
    const int lane = threadIdx.x % LANES, row0 = threadIdx.x / LANES;
    const long fb = (long)f * N1 * N2 / 2;   // float4 offset of scale f (N1 * N2 complex64)
    constexpr int CH = PER < 16 ? PER : 16;  // float4 in registers at a time (64 VGPRs)
    for (int c0 = 0; c0 < PER; c0 += CH) {
        f4 v[CH];
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const int k1 = row0 + (c0 + i) * ROWS;
            const long ro = RS ? ((long)k1 * N2 + (long)g * C) / 2 + lane : (long)g * (N1 * C / 2) + (long)k1 * LANES + lane;
            v[i] = __builtin_nontemporal_load(B + fb + ro);
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const int n1 = (row0 + (c0 + i) * ROWS + g * ROT) & (N1 - 1);   // output row n1: out[f][g*C + n2 + N2*n1]
            const long wo = WS ? ((long)n1 * N2 + (long)g * C) / 2 + lane : (long)g * (N1 * C / 2) + (long)n1 * LANES + lane;
            if constexpr (NT) __builtin_nontemporal_store(v[i], out + fb + wo);
            else out[fb + wo] = v[i];
        }
    }
}

// the row pass's B stores: contiguous rows (write-only stream of the same bytes)
__global__ __launch_bounds__(1024) void rows_kernel(f4* __restrict__ B, long n4) {
    const long base = ((long)blockIdx.x * 1024 * 16) + threadIdx.x;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const long k = base + (long)i * 1024;
        if (k < n4) __builtin_nontemporal_store(f4{1.f, 2.f, 3.f, (float)i}, B + k);
    }
}

int main(int argc, char** argv) {
    const int nf = argc > 1 ? std::atoi(argv[1]) : 64;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const size_t bytes = (size_t)nf * N1 * N2 * 8;   // complex64
    const long n4 = (long)(bytes / 16);
    f4 *B = nullptr, *out = nullptr;
    CHECK(hipMalloc(&B, bytes));
    CHECK(hipMalloc(&out, bytes));
    CHECK(hipMemset(B, 0, bytes));
    CHECK(hipMemset(out, 0, bytes));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto time = [&](const char* name, double moved, auto launch) {
        launch();                                    // warm
        CHECK(hipDeviceSynchronize());
        std::vector<float> ms(reps);
        for (int r = 0; r < reps; ++r) {
            CHECK(hipEventRecord(a));
            launch();
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            CHECK(hipEventElapsedTime(&ms[r], a, b));
        }
        float best = ms[0], sum = 0;
        for (float m : ms) { best = m < best ? m : best; sum += m; }
        std::printf("{\"geometry\": \"%s\", \"bytes\": %.6g, \"ms_mean\": %.4f, \"ms_best\": %.4f, \"TBps_mean\": %.3f}\n",
                    name, moved, sum / reps, best, moved / (sum / reps * 1e-3) / 1e12);
        std::fflush(stdout);
    };
    const unsigned cblocks = (unsigned)((n4 + 1024 * 16 - 1) / (1024 * 16));
    time("copy (contiguous float4, read + write)", 2.0 * bytes,
         [&] { copy_kernel<<<cblocks, 1024>>>(B, out, n4); });
    time("cols32 (the product: 256-B pieces, read + write)", 2.0 * bytes,
         [&] { cols_kernel<32><<<nf * (N2 / 32), 1024>>>(B, out, nf); });
    time("cols64 (512-B pieces, read + write)", 2.0 * bytes,
         [&] { cols_kernel<64><<<nf * (N2 / 64), 1024>>>(B, out, nf); });
    time("cols128 (1-KiB pieces, read + write)", 2.0 * bytes,
         [&] { cols_kernel<128><<<nf * (N2 / 128), 1024>>>(B, out, nf); });
    time("cols32 reads contiguous, writes 256-B pieces", 2.0 * bytes,
         [&] { cols_kernel<32, false, true><<<nf * (N2 / 32), 1024>>>(B, out, nf); });
    time("cols32 reads 256-B pieces, writes contiguous", 2.0 * bytes,
         [&] { cols_kernel<32, true, false><<<nf * (N2 / 32), 1024>>>(B, out, nf); });
    time("cols32 both contiguous (the same workgroup shape)", 2.0 * bytes,
         [&] { cols_kernel<32, false, false><<<nf * (N2 / 32), 1024>>>(B, out, nf); });
    time("cols32 plain stores", 2.0 * bytes,
         [&] { cols_kernel<32, true, true, false, false><<<nf * (N2 / 32), 1024>>>(B, out, nf); });
    time("cols32 XCD-adjacent groups, nt stores", 2.0 * bytes,
         [&] { cols_kernel<32, true, true, true, true><<<nf * (N2 / 32), 1024>>>(B, out, nf); });
    time("cols32 XCD-adjacent groups, plain stores", 2.0 * bytes,
         [&] { cols_kernel<32, true, true, true, false><<<nf * (N2 / 32), 1024>>>(B, out, nf); });
    time("cols32 rows rotated by 37 per group", 2.0 * bytes,
         [&] { cols_kernel<32, true, true, false, true, 37><<<nf * (N2 / 32), 1024>>>(B, out, nf); });
    time("cols32 rows rotated by 128 per group", 2.0 * bytes,
         [&] { cols_kernel<32, true, true, false, true, 128><<<nf * (N2 / 32), 1024>>>(B, out, nf); });
    time("cols32 rows rotated by 1 per group", 2.0 * bytes,
         [&] { cols_kernel<32, true, true, false, true, 1><<<nf * (N2 / 32), 1024>>>(B, out, nf); });
    time("cols32 rows rotated by 32 per group", 2.0 * bytes,
         [&] { cols_kernel<32, true, true, false, true, 32><<<nf * (N2 / 32), 1024>>>(B, out, nf); });
    time("rows (contiguous write only)", 1.0 * bytes, [&] { rows_kernel<<<cblocks, 1024>>>(B, n4); });
    CHECK(hipFree(B));
    CHECK(hipFree(out));
    return 0;
}
