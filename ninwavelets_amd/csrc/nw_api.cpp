// nw_api.cpp — the C ABI of libninwave.so (include/ninwave.h).
//
// Pipeline per device chunk of signals:
//   x (S, n) --H2D/D2D--> d_x --rocFFT R2C--> d_X (S, n/2+1)
//   engine ROCFFT: K1 multiply -> d_Y (S, F, n) -> rocFFT C2C inverse in place -> K2 epilogue
//   engine FUSED : one kernel: W*X -> LDS Stockham inverse FFT -> epilogue store
// The wavelet is never materialised on the host: analytic kinds are evaluated
// inside the kernels from (kind, params, freqs, grid).
#include <hip/hip_runtime.h>
#include <rocfft/rocfft.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "nw_dcheck.h"
#include "nw_internal.h"

namespace {

thread_local std::string g_last_error;

// NW_LOG (SURVEY.md §5 "Metrics / logging"; the reference only prints SizeError, base.py:71-72):
// 0 = silent (default), 1 = plan / engine / reduction-path decisions and every error status,
// 2 = also every launch stage with its kernel and, under NW_TIMING, its time.  Read from the
// environment at first use; nw_set_log_level() overrides it.  One line per event on stderr.
std::atomic<int> g_log_level{-1};
std::mutex g_log_mu;

int log_level() {
    int l = g_log_level.load(std::memory_order_relaxed);
    if (l >= 0) return l;
    const char* s = std::getenv("NW_LOG");
    int expect = -1;
    g_log_level.compare_exchange_strong(expect, s ? std::max(0, std::atoi(s)) : 0);
    return g_log_level.load();
}

__attribute__((format(printf, 2, 3))) void nw_logf(int level, const char* fmt, ...) {
    if (log_level() < level) return;
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    std::lock_guard<std::mutex> g(g_log_mu);
    std::fprintf(stderr, "[ninwave] %s\n", buf);
}

const char* out_name(int k) {
    static const char* names[] = {"cwt", "abs", "power", "power_mean", "itc", "power_sum", "phase_sum"};
    if (k == 1001) return "power partials";
    if (k == 1002) return "phase partials";
    return k >= 0 && k < 7 ? names[k] : "?";
}
const char* kernel_name(int64_t k) {
    static const char* names[] = {"none", "nw_fused_kernel", "nw_fused_pair_kernel", "nw_chirp_kernel",
                                  "rows_kernel + cols_kernel", "k1_multiply + rocFFT"};
    return k >= 0 && k < 6 ? names[k] : "?";
}
const char* dtype_name(int dt) { return dt == NW_F32 ? "float32" : "float64"; }

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    nw_logf(1, "error %d: %s", code, msg.c_str());
    return code;
}

#define NW_HIP(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(e_ == hipErrorOutOfMemory ? NW_E_NOMEM : NW_E_HIP,                    \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                   \
    } while (0)

#define NW_RF(expr)                                                                           \
    do {                                                                                      \
        rocfft_status s_ = (expr);                                                            \
        if (s_ != rocfft_status_success)                                                      \
            return fail(NW_E_ROCFFT, std::string(#expr) + ": rocfft status " + std::to_string((int)s_)); \
    } while (0)

#define NW_TRY(expr)                 \
    do {                             \
        int r_ = (expr);             \
        if (r_ != NW_OK) return r_;  \
    } while (0)

std::once_flag g_rocfft_once;

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// debug library: every kernel file's check words (nw_dcheck.h), read and cleared after each
// synchronising call; the product library registers none
std::vector<nw::DcheckTake>& dcheck_registry() {
    static std::vector<nw::DcheckTake> r;
    return r;
}

#ifdef NW_DEBUG_BOUNDS
constexpr bool kDebugBounds = true;
#else
constexpr bool kDebugBounds = false;
#endif

// after the device's work is complete: NW_E_BOUNDS if any kernel check failed since the last call
int dcheck_collect(hipStream_t stream) {
    if (!kDebugBounds) return NW_OK;
    hipError_t e = stream ? hipStreamSynchronize(stream) : hipDeviceSynchronize();
    if (e != hipSuccess) return fail(NW_E_HIP, std::string("synchronize: ") + hipGetErrorString(e));
    std::string msg;
    for (nw::DcheckTake take : dcheck_registry()) {
        unsigned fails = 0, site = 0;
        const char* file = "";
        e = take(&fails, &site, &file);
        if (e != hipSuccess) return fail(NW_E_HIP, std::string("bounds-check readback: ") + hipGetErrorString(e));
        if (!fails) continue;
        std::string where = site >= nw::kDcheckHeaderSite
                                ? "nw_fft_dev.h:" + std::to_string(site - nw::kDcheckHeaderSite)
                                : std::string(file) + ":" + std::to_string(site);
        msg += (msg.empty() ? "" : "; ") + std::to_string(fails) + " failing check(s), first at " + where;
    }
    return msg.empty() ? NW_OK : fail(NW_E_BOUNDS, "kernel bounds check: " + msg);
}

enum Stage { ST_FWD = 0, ST_MUL, ST_INV, ST_EPI, ST_FUSED, ST_COPY, ST_ROWS, ST_EXPAND, ST_N };
const char* const kStageName[ST_N] = {"forward", "multiply", "inverse", "epilogue", "fused", "copy", "rows", "expand"};

struct Pending {
    int stage;
    hipEvent_t a, b;
    bool own_a = true;   // false: a is the previous stage's b (chained), released with it
};

}  // namespace

struct nw_plan {
    int device = 0;
    int64_t n = 0, nh = 0, max_batch = 0;
    int nfreq = 0, dtype = NW_F32;
    uint32_t flags = 0;
    int engine = NW_ENGINE_ROCFFT;
    size_t esz = 4;  // real element size

    hipStream_t own_stream = nullptr, stream = nullptr;

    // wavelet
    bool has_wavelet = false;
    nw::WDesc desc{};
    double* d_freq = nullptr;
    double* d_peak = nullptr;
    float* d_xstep32 = nullptr;
    void* d_table = nullptr;
    size_t d_table_bytes = 0;
    int64_t* d_row_len = nullptr;
    std::vector<int64_t> row_len_host;   // tables: true length of each row

    // repeated rows: when at most half the F rows of W are distinct (Shannon ignores f,
    // wavelets.py:256-262; repeated freqs), the engines run on the U distinct rows
    // (udesc, compacted per-freq arrays) into d_uout and k_expand_rows copies each
    // computed row to every scale that repeats it (d_rep_offs / d_rep_order: the scales
    // grouped by distinct row).  NW_NO_DEDUP turns it off.
    bool dedup = false;
    int nuniq = 0;
    nw::WDesc udesc{};
    void* d_ubuf = nullptr;          // udesc's freq / peak / xstep32 / row_len (+ table rows)
    int32_t* d_rep = nullptr;        // offs[U + 1] then order[F]
    void* d_uout = nullptr;
    size_t d_uout_bytes = 0;

    // buffers
    void* d_x = nullptr;
    void* d_X = nullptr;
    void* d_Y = nullptr;
    size_t d_Y_bytes = 0;
    void* d_out = nullptr;
    size_t d_out_bytes = 0;
    void* d_acc = nullptr;           // epoch reductions: fp64 (F, n) sums (x2 for phases)
    size_t d_acc_bytes = 0;
    // nw_execute_multi_device reductions: this device's fp64 partial sums, and (device 0's
    // plan) the peer-copy landing buffer; kept across calls (a hipFree per call would
    // synchronise the device on every epoch-loop iteration)
    void* d_part = nullptr;
    size_t d_part_bytes = 0;
    void* d_gather = nullptr;
    size_t d_gather_bytes = 0;
    void* d_wtab = nullptr;          // fused engine: W[f, k] (pad_to + 1/n applied); n > 16384: kmax[f]
    size_t d_wtab_bytes = 0;
    bool wtab_valid = false;
    bool large = false;              // fused engine, two-pass form (nw_large.hip)
    bool chirp = false;              // fused engine, chirp-z form (nw_chirp.hip): other n
    int64_t chirp_counts[5] = {0, 0, 0, 0, 0};   // rows per M class (M = 1024 << c)
    bool chirp_tentative = false;    // auto engine, 2n - 1 > M_max: chirp-z only if every row's
                                     // support fits (checked when the table is built), else rocFFT
    // chirp-z rows of a tentative length wider than the largest on-chip transform: computed
    // by the rocFFT path on a compacted view of just those rows (over_desc) into d_oscr and
    // scattered to their scales (k_expand_rows), the other rows stay on chip
    std::vector<int> chirp_over;
    nw::WDesc over_desc{};
    void* d_obuf = nullptr;          // idx[U], offs[U + 1], order[U], then over_desc's per-row arrays
    void* d_oscr = nullptr;
    size_t d_oscr_bytes = 0;
    void* d_scratch = nullptr;       // two-pass form: Xt + B
    size_t d_scratch_bytes = 0;

    // rocFFT, keyed by batch count
    std::map<int64_t, rocfft_plan> fwd, inv;
    rocfft_execution_info info = nullptr;
    void* work = nullptr;
    size_t work_bytes = 0;

    // host-buffer output: two pinned staging pieces (the DMA of piece i overlaps the
    // host copy of piece i-1 into the caller's pageable array)
    void* pinned[2] = {nullptr, nullptr};
    hipEvent_t pinned_ev[2] = {nullptr, nullptr};

    // timing
    std::vector<Pending> pending;
    std::vector<hipEvent_t> event_pool;
    nw_stats stats{};
};

namespace {

int ensure(void** ptr, size_t* cur, size_t want) {
    if (*cur >= want && *ptr) return NW_OK;
    if (*ptr) {
        NW_HIP(hipFree(*ptr));
        *ptr = nullptr;
        *cur = 0;
    }
    NW_HIP(hipMalloc(ptr, want));
    *cur = want;
    return NW_OK;
}

}  // namespace

nw::StageEvents& nw::stage_events() {
    static thread_local StageEvents se;
    return se;
}

namespace {

int take_event(nw_plan* p, hipEvent_t* ev) {
    if (!p->event_pool.empty()) {
        *ev = p->event_pool.back();
        p->event_pool.pop_back();
        return NW_OK;
    }
    // timing only (resolve_timing synchronises the stream before reading them): no system-scope
    // fence at record, whose L2 writeback + invalidate between a step's two launches cost C2
    // (one 0.23 ms launch per step) 0.04 ms per step and showed up in the stage times
    NW_HIP(hipEventCreateWithFlags(ev, hipEventDisableSystemFence));
    return NW_OK;
}

// Run `fn` on the plan stream, bracketed by events when NW_TIMING is set.
// launch counts are kept with or without NW_TIMING (they tell which kernels ran)
void count_launch(nw_plan* p, int stage) {
    switch (stage) {
        case ST_MUL: p->stats.launches_multiply++; break;
        case ST_FUSED: p->stats.launches_fused++; break;
        case ST_ROWS: p->stats.launches_rows++; break;
        case ST_EXPAND: p->stats.launches_expand++; break;
        default: break;
    }
}

// chain = true: the caller enqueued nothing on the stream since the previous staged() call
// returned, so that stage's end event is this one's start (one event record less per
// boundary: each costs the stream a few microseconds, 3 % of a C2 step)
template <typename F>
int staged(nw_plan* p, int stage, F&& fn, bool chain = false) {
    count_launch(p, stage);
    nw_logf(2, "plan %p: launch %s%s%s", (void*)p, kStageName[stage], stage == ST_FUSED || stage == ST_ROWS ? ": " : "",
            stage == ST_FUSED || stage == ST_ROWS ? kernel_name(p->stats.kernel) : "");
    if (!(p->flags & NW_TIMING)) return fn();
    Pending pe{stage, nullptr, nullptr};
    if ((chain || (p->flags & NW_TIMING_CHAIN)) && !p->pending.empty()) {
        pe.a = p->pending.back().b;
        pe.own_a = false;
    } else {
        NW_TRY(take_event(p, &pe.a));
        NW_HIP(hipEventRecord(pe.a, p->stream));
    }
    NW_TRY(take_event(p, &pe.b));
    int r = fn();
    NW_HIP(hipEventRecord(pe.b, p->stream));
    p->pending.push_back(pe);
    return r;
}

// A stage whose work is kernels launched through nw_launch (nw_internal.h): with NW_TIMING
// its events ride on those launches (hipExtLaunchKernel: the stop event is the last dispatch's
// own end; the start event is one marker before the first), and a chained stage (the previous
// stage was the last thing enqueued) starts at that stage's stop, so it adds no marker at all;
// a stage that launched nothing records both at once (0 ms)
template <typename F>
int staged_k(nw_plan* p, int stage, F&& fn, bool chain = false) {
    if (!(p->flags & NW_TIMING)) return staged(p, stage, fn);
    count_launch(p, stage);
    nw_logf(2, "plan %p: launch %s%s%s", (void*)p, kStageName[stage], stage == ST_FUSED || stage == ST_ROWS ? ": " : "",
            stage == ST_FUSED || stage == ST_ROWS ? kernel_name(p->stats.kernel) : "");
    Pending pe{stage, nullptr, nullptr};
    const bool chained = (chain || (p->flags & NW_TIMING_CHAIN)) && !p->pending.empty();
    if (chained) {
        pe.a = p->pending.back().b;
        pe.own_a = false;
    } else {
        NW_TRY(take_event(p, &pe.a));
    }
    NW_TRY(take_event(p, &pe.b));
    nw::StageEvents& se = nw::stage_events();
    se = nw::StageEvents{chained ? nullptr : pe.a, pe.b, 0};
    const int r = fn();
    const int launched = se.launches;
    se = nw::StageEvents{};
    if (launched == 0) {
        if (!chained) NW_HIP(hipEventRecord(pe.a, p->stream));
        NW_HIP(hipEventRecord(pe.b, p->stream));
    }
    p->pending.push_back(pe);
    return r;
}

int resolve_timing(nw_plan* p) {
    if (p->pending.empty()) return NW_OK;
    NW_HIP(hipStreamSynchronize(p->stream));
    for (const Pending& pe : p->pending) {
        float ms = 0.f;
        NW_HIP(hipEventElapsedTime(&ms, pe.a, pe.b));
        nw_logf(2, "plan %p: %s %.3f ms", (void*)p, kStageName[pe.stage], ms);
        switch (pe.stage) {
            case ST_FWD: p->stats.ms_forward += ms; break;
            case ST_MUL: p->stats.ms_multiply += ms; break;
            case ST_INV: p->stats.ms_inverse += ms; break;
            case ST_EPI: p->stats.ms_epilogue += ms; break;
            case ST_FUSED: p->stats.ms_fused += ms; break;
            case ST_ROWS: p->stats.ms_rows += ms; break;
            case ST_EXPAND: p->stats.ms_expand += ms; break;
            default: p->stats.ms_copy += ms; break;
        }
        if (pe.own_a) p->event_pool.push_back(pe.a);
        p->event_pool.push_back(pe.b);
    }
    p->pending.clear();
    return NW_OK;
}

// execute-time geometry: pad_to the cached rows to n, mask X (base.py:396-401)
void set_exec_geometry(nw_plan* p) {
    nw::WDesc& d = p->desc;
    d.n = p->n;
    d.nh = p->nh;
    d.scale = 1.0 / (double)p->n;
    d.off = d.len_full < p->n ? (p->n - d.len_full) / 2 : 0;
    d.xlim = (p->flags & NW_INTERPOLATE) ? p->n / 2 : p->n;   // int(n / 2) (base.py:120)
}

rocfft_precision prec(const nw_plan* p) {
    return p->dtype == NW_F32 ? rocfft_precision_single : rocfft_precision_double;
}

// rocFFT plans keyed by batch count: R2C forward over signals, C2C inverse (in place)
// over (signal, scale) rows.
int get_plan(nw_plan* p, bool inverse, int64_t batch, rocfft_plan* out) {
    auto& m = inverse ? p->inv : p->fwd;
    auto it = m.find(batch);
    if (it == m.end()) {
        size_t len = (size_t)p->n;
        rocfft_plan pl = nullptr;
        NW_RF(rocfft_plan_create(&pl, inverse ? rocfft_placement_inplace : rocfft_placement_notinplace,
                                 inverse ? rocfft_transform_type_complex_inverse : rocfft_transform_type_real_forward,
                                 prec(p), 1, &len, (size_t)batch, nullptr));
        m[batch] = pl;
        size_t ws = 0;
        NW_RF(rocfft_plan_get_work_buffer_size(pl, &ws));
        if (ws > p->work_bytes) NW_TRY(ensure(&p->work, &p->work_bytes, ws));
        it = m.find(batch);
    }
    *out = it->second;
    return NW_OK;
}

// One rocFFT execution covers at most 2^31 elements: a single 512 x 2^24 batch
// (C5, 8.6e9 elements) completes only part of its rows, so longer batches run as
// several executions of <= kFftElems / n rows each.
constexpr int64_t kFftElems = int64_t(1) << 31;

int run_fft(nw_plan* p, rocfft_plan plan, void* in, void* out) {
    NW_RF(rocfft_execution_info_set_stream(p->info, p->stream));
    if (p->work_bytes) NW_RF(rocfft_execution_info_set_work_buffer(p->info, p->work, p->work_bytes));
    void* ib[1] = {in};
    void* ob[1] = {out};
    NW_RF(rocfft_execute(plan, ib, out ? ob : nullptr, p->info));
    return NW_OK;
}

// The rocFFT engine's Y buffer (max_batch x F x n complex) is allocated on first need:
// a device-output CWT writes Y straight into the caller's buffer and never needs it
// (at C5, 512 x 2^24 complex64 = 68.7 GB of HBM saved).
int need_Y(nw_plan* p) {
    return ensure(&p->d_Y, &p->d_Y_bytes, (size_t)p->max_batch * p->nfreq * p->n * 2 * p->esz);
}

// One device chunk: xs (device, c signals) -> dst (device).
// rows transforms of length n starting at in/out (elem bytes per input / output element)
int run_fft_rows(nw_plan* p, bool inverse, int64_t rows, char* in, char* out, size_t in_row, size_t out_row) {
    const int64_t group = std::max<int64_t>(1, kFftElems / p->n);
    for (int64_t r0 = 0; r0 < rows; r0 += group) {
        const int64_t nb = std::min<int64_t>(group, rows - r0);
        rocfft_plan pl = nullptr;
        NW_TRY(get_plan(p, inverse, nb, &pl));
        NW_TRY(run_fft(p, pl, in + r0 * in_row, out ? out + r0 * out_row : nullptr));
    }
    return NW_OK;
}

// The chirp-z table (W rows, supports, rows grouped by M) of the current wavelet.  A
// tentative length (2n - 1 > M_max) whose rows do not all fit switches the plan to the
// rocFFT engine until the next nw_plan_set_wavelet.

// The compacted view of the rows `rows` of the current desc (device arrays gathered on the
// device): per-row freq / peak / xstep32 / row_len and table rows, plus the scatter map
// (offs = 0 .. U, order = rows) for k_expand_rows.
int build_overflow_view(nw_plan* p, const std::vector<int>& rows) {
    const int U = (int)rows.size();
    const nw::WDesc& d = p->desc;
    const bool table = d.kind == NW_TABLE;
    const size_t trow = table ? (size_t)d.len_full * 2 * p->esz : 0;
    const size_t o_offs = ((size_t)U * 4 + 15) / 16 * 16, o_order = o_offs + ((size_t)(U + 1) * 4 + 15) / 16 * 16,
                 o_freq = o_order + ((size_t)U * 4 + 15) / 16 * 16, o_peak = o_freq + (size_t)U * 8,
                 o_x = o_peak + (size_t)U * 8, o_rl = (o_x + (size_t)U * 4 + 15) / 16 * 16,
                 o_tab = (o_rl + (size_t)U * 8 + 255) / 256 * 256, bytes = o_tab + (size_t)U * trow;
    if (p->d_obuf) NW_HIP(hipFree(p->d_obuf));
    p->d_obuf = nullptr;
    char* b = nullptr;
    NW_HIP(hipMalloc((void**)&b, bytes));
    p->d_obuf = b;
    std::vector<int32_t> head(o_freq / 4, 0);
    for (int u = 0; u < U; ++u) {
        head[u] = rows[u];
        head[o_offs / 4 + u] = u;
        head[o_order / 4 + u] = rows[u];
    }
    head[o_offs / 4 + U] = U;
    NW_HIP(hipMemcpy(b, head.data(), o_freq, hipMemcpyHostToDevice));
    const int32_t* idx = (const int32_t*)b;
    nw::WDesc o = d;
    o.nfreq = U;
    if (d.freq) {
        NW_HIP(nw::launch_gather(d.freq, b + o_freq, idx, U, 8, p->stream));
        o.freq = (const double*)(b + o_freq);
    }
    if (d.peak) {
        NW_HIP(nw::launch_gather(d.peak, b + o_peak, idx, U, 8, p->stream));
        o.peak = (const double*)(b + o_peak);
    }
    if (d.xstep32) {
        NW_HIP(nw::launch_gather(d.xstep32, b + o_x, idx, U, 4, p->stream));
        o.xstep32 = (const float*)(b + o_x);
    }
    if (table && d.row_len) {
        NW_HIP(nw::launch_gather(d.row_len, b + o_rl, idx, U, 8, p->stream));
        o.row_len = (const int64_t*)(b + o_rl);
    }
    if (table && trow) {
        NW_HIP(nw::launch_gather(d.table, b + o_tab, idx, U, trow, p->stream));
        o.table = b + o_tab;
    }
    NW_HIP(hipStreamSynchronize(p->stream));
    p->over_desc = o;
    p->chirp_over = rows;
    return NW_OK;
}

int chirp_table(nw_plan* p) {
    if (p->wtab_valid) return NW_OK;
    NW_TRY(ensure(&p->d_wtab, &p->d_wtab_bytes, nw::chirp_wtable_bytes(p->n, p->nfreq, p->dtype, p->desc.kind)));
    bool fits = true;
    std::vector<int> over;
    p->chirp_over.clear();
    NW_HIP(nw::build_chirp_wtable(p->desc, p->dtype, p->d_wtab, p->stream, p->chirp_counts, &fits, &over));
    if (!fits) {
        if (!p->chirp_tentative)
            return fail(NW_E_INVALID, "chirp-z form: a wavelet row is wider than the largest on-chip transform");
        if ((int)over.size() >= p->nfreq) {   // no row fits: the rocFFT engine
            p->chirp = false;
            p->engine = NW_ENGINE_ROCFFT;
            p->stats.engine = NW_ENGINE_ROCFFT;
            nw_logf(1, "plan %p: no wavelet row fits the on-chip chirp-z transform: rocFFT engine", (void*)p);
            return NW_OK;
        }
        NW_TRY(build_overflow_view(p, over));
        nw_logf(1, "plan %p: chirp-z form, %d of %d rows too wide for the chip run through rocFFT (hybrid)",
                (void*)p, (int)over.size(), p->nfreq);
    }
    p->wtab_valid = true;
    return NW_OK;
}

// The overflow rows of a hybrid chirp-z plan through the rocFFT path (K1 on the compacted
// view, in-place C2C inverse, epilogue), then scattered to their scales of dst.
int run_overflow_rows(nw_plan* p, int64_t c, void* dst, int out_kind) {
    const int U = (int)p->chirp_over.size();
    nw::WDesc od = p->over_desc;
    od.n = p->desc.n;
    od.nh = p->desc.nh;
    od.scale = p->desc.scale;
    od.off = p->desc.off;
    od.xlim = p->desc.xlim;
    const size_t crow = (size_t)p->n * 2 * p->esz;
    const size_t orow = (size_t)p->n * (out_kind == NW_OUT_CWT ? 2 : 1) * p->esz;
    const size_t ybytes = (size_t)c * U * crow;
    NW_TRY(ensure(&p->d_oscr, &p->d_oscr_bytes, ybytes + (out_kind == NW_OUT_CWT ? 0 : (size_t)c * U * orow)));
    char* Y = (char*)p->d_oscr;
    NW_TRY(staged_k(p, ST_MUL, [&] {
        NW_HIP(nw::launch_multiply(od, p->dtype, p->d_X, Y, c, p->stream));
        return NW_OK;
    }));
    NW_TRY(staged(p, ST_INV, [&] { return run_fft_rows(p, true, c * U, Y, nullptr, crow, crow); }));
    const char* src = Y;
    if (out_kind != NW_OUT_CWT) {
        char* Z = Y + ybytes;
        NW_TRY(staged_k(p, ST_EPI, [&] {
            NW_HIP(nw::launch_epilogue(p->dtype, out_kind, Y, Z, c * U * p->n, p->stream));
            return NW_OK;
        }));
        src = Z;
    }
    const int32_t* hb = (const int32_t*)p->d_obuf;
    const size_t o_offs = ((size_t)U * 4 + 15) / 16 * 16, o_order = o_offs + ((size_t)(U + 1) * 4 + 15) / 16 * 16;
    return staged_k(p, ST_EXPAND, [&] {
        NW_HIP(nw::launch_expand_rows(src, dst, c, U, p->nfreq, orow, hb + o_offs / 4, hb + o_order / 4, p->stream));
        return NW_OK;
    });
}

constexpr int OUT_PSUM = 1001;    // internal run_chunk kinds: (ceil(c / 8), F, n) fp64 power partials,
constexpr int OUT_PHSUM = 1002;   // complex fp64 phase partials (y / |y|)

int run_chunk_rows(nw_plan* p, const void* xs_dev, int64_t c, void* dst, int out_kind, bool dst_is_final) {
    bool rocfft_engine = p->engine == NW_ENGINE_ROCFFT;
    // fused sizes: the forward R2C by nw_fused.hip's fwd_r2c_kernel (no copy, one kernel)
    // the forward stage was the last thing enqueued (the fused form's launch may chain onto it)
    bool fwd_chain = false;
    const bool table_was_valid = p->wtab_valid;
    if (!rocfft_engine && !p->large && !p->chirp) {
        // power-of-two n <= 16384: the on-chip forward transform reads the caller's rows directly
        fwd_chain = true;
        NW_TRY(staged_k(p, ST_FWD, [&] {
            NW_HIP(nw::fused_forward(p->n, p->dtype, xs_dev, p->d_X, c, p->nh, p->stream));
            return NW_OK;
        }));
    } else {
        // rocFFT may use its input as scratch: transform from the plan's own copy.
        if (xs_dev != p->d_x)
            NW_TRY(staged(p, ST_COPY, [&] {
                NW_HIP(hipMemcpyAsync(p->d_x, xs_dev, (size_t)c * p->n * p->esz, hipMemcpyDeviceToDevice, p->stream));
                return NW_OK;
            }));
        NW_TRY(staged(p, ST_FWD, [&] {
            return run_fft_rows(p, false, c, (char*)p->d_x, (char*)p->d_X, (size_t)p->n * p->esz,
                                (size_t)p->nh * 2 * p->esz);
        }));
    }

    if (!rocfft_engine && p->large) {
        // two-pass form (n > 16384): per signal, X -> Xt, then per chunk of scales the
        // row pass (W * X, length-N2 FFTs) into B and the column pass (length-N1 FFTs +
        // epilogue) into the destination rows
        if (!p->wtab_valid) {
            NW_TRY(ensure(&p->d_wtab, &p->d_wtab_bytes, nw::large_support_bytes(p->nfreq)));
            NW_HIP(nw::build_large_support(p->desc, p->dtype, p->d_wtab, p->stream));
            p->wtab_valid = true;
        }
        NW_TRY(ensure(&p->d_scratch, &p->d_scratch_bytes, nw::large_scratch_bytes(p->n, p->nfreq, p->dtype)));
        const size_t out_row = (size_t)p->n * (out_kind == NW_OUT_CWT ? 2 : 1) * p->esz;
        const int64_t fc = nw::large_fchunk(p->n, p->nfreq, p->dtype);
        p->stats.kernel = NW_K_TWO_PASS;
        for (int64_t sidx = 0; sidx < c; ++sidx) {
            const char* Xs = (const char*)p->d_X + (size_t)sidx * p->nh * 2 * p->esz;
            char* os = (char*)dst + (size_t)sidx * p->nfreq * out_row;
            NW_TRY(staged_k(p, ST_COPY, [&] {   // the spectrum transpose: timed with the copies
                NW_HIP(nw::large_transpose(p->desc, p->dtype, Xs, p->d_scratch, p->stream));
                return NW_OK;
            }));
            for (int64_t f0 = 0; f0 < p->nfreq; f0 += fc) {
                const int nf = (int)std::min<int64_t>(fc, p->nfreq - f0);
                NW_TRY(staged_k(p, ST_ROWS, [&] {
                    NW_HIP(nw::large_rows(p->desc, p->dtype, (int)f0, nf, p->d_wtab, p->d_scratch, p->stream));
                    return NW_OK;
                }, true));
                NW_TRY(staged_k(p, ST_FUSED, [&] {
                    NW_HIP(nw::large_cols(p->desc, p->dtype, out_kind, (int)f0, nf, p->d_wtab, p->d_scratch, os, p->stream));
                    return NW_OK;
                }, true));
            }
        }
        return NW_OK;
    }
    if (!rocfft_engine && p->chirp) {
        // chirp-z form (any other n up to 8192 fp32 / 4096 fp64): two on-chip FFTs per row
        NW_TRY(chirp_table(p));
        p->stats.kernel = NW_K_CHIRP;
        if (p->chirp) {
            NW_TRY(staged_k(p, ST_FUSED, [&] {
                NW_HIP(nw::launch_chirp(p->desc, p->dtype, out_kind, p->d_X, p->d_wtab, dst, c, p->chirp_counts,
                                        p->stream));
                return NW_OK;
            }));
            if (!p->chirp_over.empty()) NW_TRY(run_overflow_rows(p, c, dst, out_kind));
            return NW_OK;
        }
        rocfft_engine = true;   // a tentative length none of whose rows fit: the rocFFT engine
    }
    if (!rocfft_engine) {
        if (!p->wtab_valid) {
            NW_TRY(ensure(&p->d_wtab, &p->d_wtab_bytes,
                          nw::fused_wtable_bytes(p->n, p->nfreq, p->dtype, p->desc.kind)));
            NW_HIP(nw::build_wtable(p->desc, p->dtype, p->d_wtab, p->stream));
            p->wtab_valid = true;
        }
        if (out_kind == OUT_PSUM || out_kind == OUT_PHSUM) {
            p->stats.kernel = nw::fused_psum_kernel_id(p->n, p->dtype, out_kind == OUT_PHSUM);
            return staged_k(p, ST_FUSED, [&] {
                NW_HIP(nw::fused_power_partials(p->desc, p->dtype, out_kind == OUT_PHSUM, p->d_X, p->d_wtab, dst, c,
                                                p->stream));
                return NW_OK;
            });
        }
        p->stats.kernel = nw::fused_kernel_id(p->n, p->dtype, p->desc.kind);
        return staged_k(p, ST_FUSED, [&] {
            NW_HIP(nw::launch_fused(p->desc, p->dtype, out_kind, p->d_X, p->d_wtab, dst, c, p->stream));
            return NW_OK;
        }, fwd_chain && table_was_valid);
    }
    // K1 writes the product straight into the destination when the caller wants
    // the complex CWT on the device; otherwise into the plan's Y buffer.
    void* Y = dst;
    if (!(out_kind == NW_OUT_CWT && dst_is_final)) {
        NW_TRY(need_Y(p));
        Y = p->d_Y;
    }
    p->stats.kernel = NW_K_MULTIPLY;
    NW_TRY(staged_k(p, ST_MUL, [&] {
        NW_HIP(nw::launch_multiply(p->desc, p->dtype, p->d_X, Y, c, p->stream));
        return NW_OK;
    }));
    NW_TRY(staged(p, ST_INV, [&] {
        const size_t row = (size_t)p->n * 2 * p->esz;
        return run_fft_rows(p, true, c * p->nfreq, (char*)Y, nullptr, row, row);
    }));
    if (out_kind == NW_OUT_CWT) {
        if (Y != dst)
            NW_TRY(staged(p, ST_COPY, [&] {
                NW_HIP(hipMemcpyAsync(dst, Y, (size_t)c * p->nfreq * p->n * 2 * p->esz, hipMemcpyDeviceToDevice,
                                      p->stream));
                return NW_OK;
            }));
        return NW_OK;
    }
    return staged_k(p, ST_EPI, [&] {
        NW_HIP(nw::launch_epilogue(p->dtype, out_kind, Y, dst, c * p->nfreq * p->n, p->stream));
        return NW_OK;
    });
}

// The engines see the plan as if it had only the U distinct rows (desc, nfreq); the
// execute-time geometry nw_execute set on desc is carried over.
struct UniqueRows {
    nw_plan* p;
    nw::WDesc saved;
    explicit UniqueRows(nw_plan* pl) : p(pl), saved(pl->desc) {
        nw::WDesc u = p->udesc;
        u.n = saved.n;
        u.nh = saved.nh;
        u.scale = saved.scale;
        u.off = saved.off;
        u.xlim = saved.xlim;
        p->desc = u;
        p->nfreq = p->nuniq;
    }
    ~UniqueRows() {
        p->desc = saved;
        p->nfreq = saved.nfreq;
    }
};

// One device chunk: (c, F, n) outputs of kind out_kind into dst (device).
int run_chunk(nw_plan* p, const void* xs_dev, int64_t c, void* dst, int out_kind, bool dst_is_final) {
    if (!p->dedup) return run_chunk_rows(p, xs_dev, c, dst, out_kind, dst_is_final);
    const bool psum = out_kind == OUT_PSUM || out_kind == OUT_PHSUM;   // fp64 partial rows, one per block of signals
    const size_t row = psum ? (size_t)p->n * sizeof(double) * (out_kind == OUT_PHSUM ? 2 : 1)
                            : (size_t)p->n * (out_kind == NW_OUT_CWT ? 2 : 1) * p->esz;
    const int64_t crows = psum ? nw::fused_psum_groups(c) : c;
    NW_TRY(ensure(&p->d_uout, &p->d_uout_bytes, (size_t)c * p->nuniq * row));   // crows <= c
    {
        UniqueRows u(p);   // d_uout is scratch of the CWT's row size: K1 may write it
        NW_TRY(run_chunk_rows(p, xs_dev, c, p->d_uout, out_kind, true));
    }
    return staged_k(p, ST_EXPAND, [&] {   // run_chunk_rows ends with a staged stage: chain onto it
        NW_HIP(nw::launch_expand_rows(p->d_uout, dst, crows, p->nuniq, p->nfreq, row, p->d_rep, p->d_rep + p->nuniq + 1,
                                      p->stream));
        return NW_OK;
    }, true);
}

bool is_reduction(int out_kind) { return out_kind >= NW_OUT_POWER_MEAN && out_kind <= NW_OUT_PHASE_SUM; }
bool is_phase(int out_kind) { return out_kind == NW_OUT_ITC || out_kind == NW_OUT_PHASE_SUM; }

// Epoch reductions (mneutils.py:42-71): every chunk's per-signal results (|y|^2 from
// the fused kernel, or y from the rocFFT engine's Y / the fused CWT for phases) are
// added in signal order into the fp64 accumulator; the (S, F, n) result never exists
// beyond one chunk.  nsig = 0 leaves acc = 0, so the mean is 0/0 = NaN like
// np.mean over an empty axis.
int execute_reduce(nw_plan* p, const void* x, int64_t nsig, void* out, int out_kind, bool host) {
    const bool phase = is_phase(out_kind);
    const int64_t fn = (int64_t)p->nfreq * p->n;
    const size_t acc_bytes = (size_t)fn * (phase ? 2 : 1) * sizeof(double);
    NW_TRY(ensure(&p->d_acc, &p->d_acc_bytes, acc_bytes));
    NW_HIP(hipMemsetAsync(p->d_acc, 0, acc_bytes, p->stream));
    const bool fused = p->engine == NW_ENGINE_FUSED;
    // fp32 reductions at the register-resident fused sizes: the kernel sums |y|^2 (ITC: y / |y|)
    // over each block of 8 signals in fp64, the accumulator adds the ceil(c / 8) fp64 partials
    // (the same fp64 additions of the same fp32-derived values, regrouped; with the dedup view
    // the partials of the distinct rows are expanded like any output row)
    // The chirp-z form (lengths 2n - 1 <= M_max, every row on chip) read-modify-writes its
    // block partial rows instead (no accumulator registers; any kind, fp32 and fp64); its
    // tentative lengths (rows may leave the chip) and the repeated-row view keep the chunk path;
    // so do complex table rows (MexicanHat, Haar, user tables), as on the fused form: their
    // partial-sum instantiations are not scratch-free (fp32 M = 4096: 20 B)
    bool chirp_psum = fused && p->chirp && !p->chirp_tentative && !p->dedup && p->desc.kind != NW_TABLE;
    if (chirp_psum) {
        NW_TRY(chirp_table(p));   // the rows' M classes decide (chirp_psum_ok)
        chirp_psum = p->chirp && p->chirp_over.empty() && nw::chirp_psum_ok(p->dtype, phase, p->chirp_counts);
    }
    const bool psum = (fused && !p->large && !p->chirp &&
                       nw::fused_psum_supported(p->n, p->dtype, p->desc.kind, phase)) || chirp_psum;
    const int sig_kind = psum ? (phase ? OUT_PHSUM : OUT_PSUM) : (fused && !phase) ? NW_OUT_POWER : NW_OUT_CWT;
    nw_logf(1, "plan %p: %s over %lld signals: %s", (void*)p, out_name(out_kind), (long long)nsig,
            psum ? "fp64 block partial sums inside the transform kernel"
                 : "per-signal rows per chunk, added in signal order in fp64");
    // partials: plain fp64 sums (phase partials as 2 fn reals)
    const int src_kind = psum ? nw::ACC_POWER_REAL
                              : phase ? nw::ACC_PHASE_Y : (fused ? nw::ACC_POWER_REAL : nw::ACC_POWER_Y);
    void* scratch = nullptr;            // rocFFT engine: run_chunk leaves y in d_Y
    if (!fused) {
        NW_TRY(need_Y(p));
        scratch = p->d_Y;
    } else {
        size_t sb = (size_t)p->max_batch * fn * (phase ? 2 : 1) * p->esz;
        if (psum) sb = std::max(sb, (size_t)nw::fused_psum_groups(p->max_batch) * fn * (phase ? 2 : 1) * sizeof(double));
        NW_TRY(ensure(&p->d_out, &p->d_out_bytes, sb));
        scratch = p->d_out;
    }
    for (int64_t s0 = 0; s0 < nsig; s0 += p->max_batch) {
        const int64_t c = std::min<int64_t>(p->max_batch, nsig - s0);
        const void* xs = (const char*)x + (size_t)s0 * p->n * p->esz;
        if (host) {
            NW_TRY(staged(p, ST_COPY, [&] {
                NW_HIP(hipMemcpyAsync(p->d_x, xs, (size_t)c * p->n * p->esz, hipMemcpyHostToDevice, p->stream));
                return NW_OK;
            }));
            xs = p->d_x;
        }
        NW_TRY(run_chunk(p, xs, c, scratch, sig_kind, false));
        NW_TRY(staged_k(p, ST_EPI, [&] {   // chained: run_chunk ends with a staged stage
            const int64_t rows = psum ? nw::fused_psum_groups(c) : c;
            NW_HIP(nw::launch_accumulate(psum ? NW_F64 : p->dtype, src_kind, scratch, (double*)p->d_acc,
                                         psum && phase ? 2 * fn : fn, rows, p->stream));
            return NW_OK;
        }, true));
        p->stats.chunks++;
    }
    const hipMemcpyKind back = host ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    if (out_kind == NW_OUT_POWER_SUM || out_kind == NW_OUT_PHASE_SUM) {
        NW_HIP(hipMemcpyAsync(out, p->d_acc, acc_bytes, back, p->stream));
    } else {
        // scratch is >= fn elements of the plan dtype on both engines
        void* dst = host ? scratch : out;
        NW_TRY(staged_k(p, ST_EPI, [&] {
            NW_HIP(nw::launch_finalize(p->dtype, phase, (const double*)p->d_acc, dst, fn, nsig, p->stream));
            return NW_OK;
        }));
        if (host) NW_HIP(hipMemcpyAsync(out, dst, (size_t)fn * p->esz, hipMemcpyDeviceToHost, p->stream));
    }
    p->stats.executes++;
    if (host) {
        NW_HIP(hipStreamSynchronize(p->stream));
        NW_TRY(resolve_timing(p));
    }
    return NW_OK;
}

// ---- page-locked result buffers (nw_host_alloc): a destination inside one is written by DMA
std::mutex g_host_mu;
std::map<uintptr_t, size_t> g_host_bufs;   // base -> bytes

bool host_pinned(const void* p, size_t bytes) {
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> lk(g_host_mu);
    auto it = g_host_bufs.upper_bound(a);
    if (it == g_host_bufs.begin()) return false;
    --it;
    return a >= it->first && a + bytes <= it->first + it->second;
}

// ---- host-buffer copy-out: pinned double-buffered pieces + a multi-threaded host copy
constexpr size_t kPiece = size_t(64) << 20;
// host copy threads (NW_COPY_THREADS overrides, diagnostics)
int copy_threads() {
    static const int n = [] {
        const char* e = std::getenv("NW_COPY_THREADS");
        const int v = e ? std::atoi(e) : 8;
        return v > 0 ? v : 8;
    }();
    return n;
}

int copy_out(nw_plan* p, char* dst, const char* src, size_t bytes) {
    if (!p->pinned[0]) {
        for (int i = 0; i < 2; ++i) {
            NW_HIP(hipHostMalloc(&p->pinned[i], kPiece, hipHostMallocDefault));
            NW_HIP(hipEventCreateWithFlags(&p->pinned_ev[i], hipEventDisableTiming));
        }
    }
    const size_t npieces = (bytes + kPiece - 1) / kPiece;
    for (size_t i = 0; i <= npieces; ++i) {
        if (i < npieces) {
            const size_t off = i * kPiece;
            NW_HIP(hipMemcpyAsync(p->pinned[i & 1], src + off, std::min(kPiece, bytes - off), hipMemcpyDeviceToHost,
                                  p->stream));
            NW_HIP(hipEventRecord(p->pinned_ev[i & 1], p->stream));
        }
        if (i > 0) {                                  // piece i-1 landed: copy it out while piece i flies
            const size_t k = i - 1, off = k * kPiece;
            NW_HIP(hipEventSynchronize(p->pinned_ev[k & 1]));
            nw::host::parallel_copy(dst + off, (const char*)p->pinned[k & 1], std::min(kPiece, bytes - off),
                                   copy_threads());
        }
    }
    return NW_OK;
}

void free_plan(nw_plan* p) {
    for (auto& kv : p->fwd) rocfft_plan_destroy(kv.second);
    for (auto& kv : p->inv) rocfft_plan_destroy(kv.second);
    if (p->info) rocfft_execution_info_destroy(p->info);
    void* bufs[] = {p->work,   p->d_x,    p->d_X,        p->d_Y,     p->d_out,      p->d_wtab,
                    p->d_freq, p->d_peak, p->d_xstep32, p->d_table, p->d_row_len, p->d_acc, p->d_scratch,
                    p->d_ubuf, p->d_rep,  p->d_uout, p->d_obuf, p->d_oscr, p->d_part, p->d_gather};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (auto& pe : p->pending) {
        (void)hipEventDestroy(pe.a);
        (void)hipEventDestroy(pe.b);
    }
    for (auto e : p->event_pool) (void)hipEventDestroy(e);
    for (int i = 0; i < 2; ++i) {
        if (p->pinned[i]) (void)hipHostFree(p->pinned[i]);
        if (p->pinned_ev[i]) (void)hipEventDestroy(p->pinned_ev[i]);
    }
    if (p->own_stream) (void)hipStreamDestroy(p->own_stream);
    delete p;
}

}  // namespace

namespace nw {
int dcheck_register(DcheckTake fn) {
    dcheck_registry().push_back(fn);
    return (int)dcheck_registry().size();
}
}  // namespace nw

extern "C" {

const char* nw_last_error(void) { return g_last_error.c_str(); }

const char* nw_version(void) { return "ninwave 0.1.0 (gfx950)"; }

int nw_debug_bounds(void) { return kDebugBounds ? 1 : 0; }

int nw_debug_selftest(int device) {
    if (!kDebugBounds) return fail(NW_E_STATE, "nw_debug_selftest: not the debug library");
    int ndev = 0;
    NW_TRY(nw_device_count(&ndev));
    if (device < 0 || device >= ndev) return fail(NW_E_INVALID, "nw_debug_selftest: device out of range");
    DeviceGuard guard(device);
    NW_TRY(dcheck_collect(nullptr));   // nothing pending from earlier calls
    NW_HIP(nw::launch_dcheck_selftest(nullptr));
    return dcheck_collect(nullptr);
}

int nw_set_log_level(int level) {
    const int prev = log_level();
    g_log_level.store(std::max(0, level));
    return prev;
}

int nw_device_count(int* n) {
    if (!n) return fail(NW_E_INVALID, "nw_device_count: null pointer");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *n = 0;
        return fail(NW_E_NODEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    }
    *n = c;
    return NW_OK;
}

int nw_trans_grid(double real_length, double sfreq, int interpolate, nw_grid* g) {
    if (!g || !(real_length > 0.0) || !(sfreq > 0.0))
        return fail(NW_E_INVALID, "nw_trans_grid: need real_length > 0, sfreq > 0");
    nw::host::trans_grid(real_length, sfreq, interpolate != 0, &g->delta, &g->len_valid, &g->len_full);
    return NW_OK;
}

int nw_fused_supported(int64_t n, int dtype) {
    return nw::fused_supported(n, dtype) || nw::large_supported(n, dtype) || nw::chirp_supported(n, dtype) ? 1 : 0;
}

int nw_plan_create(nw_plan** out, int device, int64_t n, int64_t max_batch, int32_t nfreq, int dtype,
                   uint32_t flags) {
    if (!out) return fail(NW_E_INVALID, "nw_plan_create: null plan pointer");
    *out = nullptr;
    if (n < 1 || max_batch < 1 || nfreq < 1) return fail(NW_E_INVALID, "nw_plan_create: n, max_batch, nfreq must be >= 1");
    if (dtype != NW_F32 && dtype != NW_F64) return fail(NW_E_INVALID, "nw_plan_create: dtype must be NW_F32 or NW_F64");
    if ((flags & NW_ENGINE_ROCFFT) && (flags & NW_ENGINE_FUSED))
        return fail(NW_E_INVALID, "nw_plan_create: choose one engine");
    int ndev = 0;
    NW_TRY(nw_device_count(&ndev));
    if (ndev == 0) return fail(NW_E_NODEVICE, "nw_plan_create: no HIP device");
    if (device < 0 || device >= ndev) return fail(NW_E_INVALID, "nw_plan_create: device out of range");
    std::call_once(g_rocfft_once, [] { rocfft_setup(); });

    DeviceGuard guard(device);
    nw_plan* p = new nw_plan();
    p->device = device;
    p->n = n;
    p->nh = n / 2 + 1;
    p->max_batch = max_batch;
    p->nfreq = nfreq;
    p->dtype = dtype;
    p->flags = flags;
    p->esz = dtype == NW_F32 ? 4 : 8;
    const bool large_ok = !nw::fused_supported(n, dtype) && nw::large_supported(n, dtype);
    const bool chirp_sure = nw::chirp_supported(n, dtype) && !(flags & NW_NO_CHIRP);
    // 2n - 1 > M_max: the chirp-z form only if the auto engine finds every row narrow enough
    const bool chirp_maybe = !chirp_sure && !large_ok && nw::chirp_possible(n, dtype) && !(flags & NW_NO_CHIRP) &&
                             !(flags & (NW_ENGINE_ROCFFT | NW_ENGINE_FUSED));
    const bool chirp_ok = chirp_sure || chirp_maybe;
    const bool fused_ok = nw::fused_supported(n, dtype) || large_ok || chirp_sure;
    if (flags & NW_ENGINE_FUSED) {
        if (!fused_ok) {
            free_plan(p);
            return fail(NW_E_INVALID, "nw_plan_create: fused engine does not support this n/dtype");
        }
        p->engine = NW_ENGINE_FUSED;
    } else if (flags & NW_ENGINE_ROCFFT) {
        p->engine = NW_ENGINE_ROCFFT;
    } else {
        p->engine = (fused_ok || chirp_maybe) ? NW_ENGINE_FUSED : NW_ENGINE_ROCFFT;
    }
    p->large = p->engine == NW_ENGINE_FUSED && large_ok;
    p->chirp = p->engine == NW_ENGINE_FUSED && chirp_ok;
    p->chirp_tentative = p->chirp && chirp_maybe;
    p->stats.engine = p->engine;
    auto bail = [&](int code) {
        free_plan(p);
        return code;
    };
    hipError_t e = hipStreamCreateWithFlags(&p->own_stream, hipStreamNonBlocking);
    if (e != hipSuccess) return bail(fail(NW_E_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e)));
    p->stream = p->own_stream;
    if (rocfft_execution_info_create(&p->info) != rocfft_status_success)
        return bail(fail(NW_E_ROCFFT, "rocfft_execution_info_create failed"));
    size_t sz = 0;
    int r = ensure(&p->d_x, &sz, (size_t)max_batch * n * p->esz);
    if (r != NW_OK) return bail(r);
    sz = 0;
    r = ensure(&p->d_X, &sz, (size_t)max_batch * p->nh * 2 * p->esz);
    if (r != NW_OK) return bail(r);
    if (p->engine == NW_ENGINE_FUSED && !p->large && !p->chirp) {
        e = nw::fused_prepare(n, dtype);
        if (e != hipSuccess) return bail(fail(NW_E_HIP, std::string("fused_prepare: ") + hipGetErrorString(e)));
    }
    nw_logf(1, "plan %p: device %d n %lld nfreq %d %s max_batch %lld: %s engine, %s", (void*)p, device, (long long)n,
            (int)nfreq, dtype_name(dtype), (long long)max_batch,
            p->engine == NW_ENGINE_FUSED ? "fused" : "rocFFT",
            p->engine == NW_ENGINE_ROCFFT ? "rocFFT forward / K1 multiply / rocFFT inverse / K2 epilogue"
            : p->large ? "two-pass form (rows_kernel + cols_kernel)"
            : p->chirp_tentative ? "chirp-z form if every row fits on chip (settled at the first execute)"
            : p->chirp ? "chirp-z form (nw_chirp_kernel)" : "one-pass form (fwd_r2c_kernel + nw_fused_kernel)");
    *out = p;
    return NW_OK;
}

// WaveletMode.Normal table on the device (MexicanHat / Haar; base.py:249-256).  The row
// geometry mirrors numpy on the host: _setup_waveletshape's span and step
// (base.py:196-216, real_length = 1, zero_mean), np.arange's length ceil((stop - start)
// / step) and fill, half = int((sfreq * real_wave_length - m) / 2) zeros per side
// (base.py:253-254).  Rows of equal length share one batched fp64 rocFFT.
static int build_normal_table(nw_plan* p, int kind, const double* params, int nparams, const double* freqs,
                              int64_t* lmax_out) {
    const int F = p->nfreq;
    std::vector<nw::NormalRow> rows;
    int64_t lmax = 0, off = 0;
    double sigma = 0.0;
    if (!nw::host::normal_rows(kind == NW_MEXICAN_HAT, params, nparams, freqs, F, rows, &lmax, &off, &sigma))
        return fail(NW_E_INVALID, "nw_plan_set_wavelet: negative padding (np.zeros of a negative size)");
    std::map<int64_t, std::vector<int>> by_len;
    for (int f = 0; f < F; ++f) by_len[rows[f].len].push_back(f);
    const size_t tbytes = (size_t)F * lmax * 2 * p->esz;
    std::vector<int64_t> lens(F);
    for (int f = 0; f < F; ++f) lens[f] = rows[f].len;
    p->row_len_host = lens;
    void* d_rows = nullptr;
    void* d_buf = nullptr;
    void* d_work = nullptr;
    int rc = NW_OK;
    auto hip = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && rc == NW_OK) rc = fail(NW_E_HIP, std::string("normal table: ") + what + ": " + hipGetErrorString(e));
        return rc == NW_OK;
    };
    if (hip(hipMalloc(&d_rows, F * sizeof(nw::NormalRow)), "hipMalloc") &&
        hip(hipMalloc(&d_buf, (size_t)std::max<int64_t>(off, 1) * 2 * sizeof(double)), "hipMalloc") &&
        hip(hipMalloc(&p->d_table, std::max<size_t>(tbytes, 16)), "hipMalloc") &&
        ((p->d_table_bytes = std::max<size_t>(tbytes, 16)), true) &&
        hip(hipMalloc((void**)&p->d_row_len, F * sizeof(int64_t)), "hipMalloc") &&
        hip(hipMemcpy(d_rows, rows.data(), F * sizeof(nw::NormalRow), hipMemcpyHostToDevice), "H2D") &&
        hip(hipMemcpy(p->d_row_len, lens.data(), F * sizeof(int64_t), hipMemcpyHostToDevice), "H2D") &&
        hip(nw::launch_normal_time((const nw::NormalRow*)d_rows, F, lmax, kind, sigma, d_buf, p->stream), "time rows")) {
        for (auto& kv : by_len) {
            if (kv.first == 0) continue;
            rocfft_plan pl = nullptr;
            size_t len = (size_t)kv.first, ws = 0;
            if (rocfft_plan_create(&pl, rocfft_placement_inplace, rocfft_transform_type_complex_forward,
                                   rocfft_precision_double, 1, &len, kv.second.size(), nullptr) != rocfft_status_success) {
                rc = fail(NW_E_ROCFFT, "normal table: rocfft_plan_create");
                break;
            }
            rocfft_plan_get_work_buffer_size(pl, &ws);
            if (ws > 0 && !hip(hipMalloc(&d_work, ws), "hipMalloc")) {
                rocfft_plan_destroy(pl);
                break;
            }
            rocfft_execution_info_set_stream(p->info, p->stream);
            if (ws) rocfft_execution_info_set_work_buffer(p->info, d_work, ws);
            void* ib[1] = {(char*)d_buf + (size_t)rows[kv.second[0]].off * 2 * sizeof(double)};
            const bool ok = rocfft_execute(pl, ib, nullptr, p->info) == rocfft_status_success;
            hip(hipStreamSynchronize(p->stream), "sync");
            if (p->work_bytes) rocfft_execution_info_set_work_buffer(p->info, p->work, p->work_bytes);
            rocfft_plan_destroy(pl);
            if (d_work) {
                (void)hipFree(d_work);
                d_work = nullptr;
            }
            if (!ok) {
                rc = fail(NW_E_ROCFFT, "normal table: rocfft_execute");
                break;
            }
        }
        if (rc == NW_OK)
            hip(nw::launch_normal_finish((const nw::NormalRow*)d_rows, F, lmax, (p->flags & NW_INTERPOLATE) != 0,
                                         d_buf, p->dtype, p->d_table, p->stream), "finish");
        if (rc == NW_OK) hip(hipStreamSynchronize(p->stream), "sync");
    }
    if (d_rows) (void)hipFree(d_rows);
    if (d_buf) (void)hipFree(d_buf);
    *lmax_out = lmax;
    return rc;
}

// Distinct rows of W (see nw_plan::dedup).  A row is a function of (kind, params, grid)
// and, except for Shannon, of its freq (tables: of its contents), so equal freqs (equal
// table rows) give bit-identical outputs.  rep[f] = first scale with the same row.
static int setup_unique_rows(nw_plan* p, int kind, const double* freqs, const std::vector<double>& peak,
                             const std::vector<float>& xstep, const void* host_table) {
    const int F = p->nfreq;
    p->dedup = false;
    p->nuniq = F;
    p->stats.unique_rows = F;
    if (p->d_ubuf) NW_HIP(hipFree(p->d_ubuf));
    if (p->d_rep) NW_HIP(hipFree(p->d_rep));
    p->d_ubuf = nullptr;
    p->d_rep = nullptr;
    const bool user_table = kind == NW_TABLE && host_table;
    const nw::host::RowGroups groups =
        nw::host::group_rows(kind == NW_SHANNON, F, freqs, user_table ? (const double*)host_table : nullptr,
                             p->desc.len_full, user_table && !p->row_len_host.empty() ? p->row_len_host.data() : nullptr);
    const std::vector<int>& uniq = groups.uniq;
    const int U = (int)uniq.size();
    if ((p->flags & NW_NO_DEDUP) || 2 * U > F) return NW_OK;
    const std::vector<int32_t>& host = groups.packed;
    // compacted per-freq arrays of the distinct rows
    const nw::WDesc& d = p->desc;
    const bool table = d.kind == NW_TABLE;
    const size_t trow = table ? (size_t)d.len_full * 2 * p->esz : 0;
    const size_t o_peak = (size_t)U * 8, o_x = o_peak + (size_t)U * 8, o_rl = (o_x + (size_t)U * 4 + 15) / 16 * 16,
                 o_tab = (o_rl + (size_t)U * 8 + 255) / 256 * 256, bytes = o_tab + (size_t)U * trow;
    std::vector<double> uf(U), up(U);
    std::vector<float> ux(U);
    std::vector<int64_t> url(U, d.len_full);
    for (int u = 0; u < U; ++u) {
        uf[u] = freqs[uniq[u]];
        up[u] = peak[uniq[u]];
        ux[u] = xstep[uniq[u]];
        if (table && !p->row_len_host.empty()) url[u] = p->row_len_host[uniq[u]];
    }
    char* b = nullptr;
    NW_HIP(hipMalloc((void**)&b, bytes));
    p->d_ubuf = b;
    NW_HIP(hipMemcpy(b, uf.data(), U * 8, hipMemcpyHostToDevice));
    NW_HIP(hipMemcpy(b + o_peak, up.data(), U * 8, hipMemcpyHostToDevice));
    NW_HIP(hipMemcpy(b + o_x, ux.data(), U * 4, hipMemcpyHostToDevice));
    nw::WDesc u = d;
    u.nfreq = U;
    u.freq = (const double*)b;
    u.peak = (const double*)(b + o_peak);
    u.xstep32 = (const float*)(b + o_x);
    if (table) {
        if (d.row_len) {
            NW_HIP(hipMemcpy(b + o_rl, url.data(), U * 8, hipMemcpyHostToDevice));
            u.row_len = (const int64_t*)(b + o_rl);
        }
        for (int k = 0; k < U && trow > 0; ++k)
            NW_HIP(hipMemcpy(b + o_tab + (size_t)k * trow, (const char*)d.table + (size_t)uniq[k] * trow, trow,
                             hipMemcpyDeviceToDevice));
        u.table = b + o_tab;
    }
    NW_HIP(hipMalloc((void**)&p->d_rep, host.size() * sizeof(int32_t)));
    NW_HIP(hipMemcpy(p->d_rep, host.data(), host.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    p->udesc = u;
    p->nuniq = U;
    p->dedup = true;
    p->stats.unique_rows = U;
    return NW_OK;
}

int nw_plan_set_wavelet(nw_plan* p, int kind, const double* params, int nparams, const double* freqs,
                        const nw_grid* grid, const void* table, const int64_t* row_len) {
    if (!p || !freqs || !grid) return fail(NW_E_INVALID, "nw_plan_set_wavelet: null argument");
    if (kind < NW_MORSE || kind > NW_HAAR) return fail(NW_E_INVALID, "nw_plan_set_wavelet: unknown kind");
    const bool normal = kind == NW_MEXICAN_HAT || kind == NW_HAAR;
    if (kind == NW_TABLE && !table) return fail(NW_E_INVALID, "nw_plan_set_wavelet: NW_TABLE needs a table");
    if (grid->len_full < 0 || grid->len_valid < 0 || grid->len_valid > grid->len_full)
        return fail(NW_E_INVALID, "nw_plan_set_wavelet: bad grid lengths");
    const int F = p->nfreq;
    for (int i = 0; i < F; ++i)
        if (kind != NW_TABLE && kind != NW_SHANNON && freqs[i] == 0.0)
            return fail(NW_E_INVALID, "nw_plan_set_wavelet: freq == 0 (ZeroDivisionError in base.py:234-235)");
    DeviceGuard guard(p->device);
    nw::WDesc d{};
    d.kind = kind;
    d.nfreq = F;
    d.delta = grid->delta;
    d.len_full = grid->len_full;
    d.len_valid = grid->len_valid;
    std::vector<double> peak(F, 1.0);
    std::vector<float> xstep(F, 0.f);
    if (kind == NW_MORSE) {
        d.b = nparams > 0 ? params[0] : 17.5;
        d.r = nparams > 1 ? params[1] : 3.0;
        d.b_over_r = d.b / d.r;
        for (int i = 0; i < F; ++i) xstep[i] = (float)(grid->delta / freqs[i]);
        d.morse_ovf = nw::host::morse_may_overflow(d.b, d.r, grid->delta, grid->len_valid, freqs, F) ? 1 : 0;
    } else if (kind == NW_MORLET) {
        d.sigma = nparams > 0 ? params[0] : 7.0;
        const bool gabor = nparams > 1 && params[1] != 0.0;
        const double s2 = d.sigma * d.sigma;
        const double c = std::pow(1.0 + std::exp(-s2) - 2.0 * std::exp(-3.0 / 4.0 * s2), -0.5);
        d.cpi = (nparams > 2 ? params[2] : c) * std::pow(M_PI, -0.25);
        d.kappa = nparams > 3 ? params[3] : (gabor ? 0.0 : std::exp(-std::pow(d.sigma, 2.0) / 2.0));
        for (int i = 0; i < F; ++i) {
            peak[i] = d.sigma / (1.0 - std::exp(-d.sigma * freqs[i]));
            xstep[i] = (float)(grid->delta / freqs[i] * peak[i]);
        }
    }
    size_t cur = 0;
    if (!p->d_freq) {
        NW_TRY(ensure((void**)&p->d_freq, &cur, F * sizeof(double)));
        cur = 0;
        NW_TRY(ensure((void**)&p->d_peak, &cur, F * sizeof(double)));
        cur = 0;
        NW_TRY(ensure((void**)&p->d_xstep32, &cur, F * sizeof(float)));
    }
    NW_HIP(hipMemcpy(p->d_freq, freqs, F * sizeof(double), hipMemcpyHostToDevice));
    NW_HIP(hipMemcpy(p->d_peak, peak.data(), F * sizeof(double), hipMemcpyHostToDevice));
    NW_HIP(hipMemcpy(p->d_xstep32, xstep.data(), F * sizeof(float), hipMemcpyHostToDevice));
    if (p->d_table) {
        NW_HIP(hipFree(p->d_table));
        p->d_table = nullptr;
        p->d_table_bytes = 0;
    }
    if (p->d_row_len) {
        NW_HIP(hipFree(p->d_row_len));
        p->d_row_len = nullptr;
    }
    if (kind == NW_TABLE && !normal) {
        std::vector<int64_t> rl(F, grid->len_full);
        if (row_len)
            for (int i = 0; i < F; ++i) {
                if (row_len[i] < 0 || row_len[i] > grid->len_full)
                    return fail(NW_E_INVALID, "nw_plan_set_wavelet: row_len out of range");
                rl[i] = row_len[i];
            }
        NW_HIP(hipMalloc((void**)&p->d_row_len, F * sizeof(int64_t)));
        NW_HIP(hipMemcpy(p->d_row_len, rl.data(), F * sizeof(int64_t), hipMemcpyHostToDevice));
        p->row_len_host = rl;
    }
    if (normal) {
        int64_t lmax = 0;
        NW_TRY(build_normal_table(p, kind, params, nparams, freqs, &lmax));
        kind = NW_TABLE;               // from here on a (device-built) table like any other
        d.kind = NW_TABLE;
        d.delta = 1.0;
        d.len_full = d.len_valid = lmax;
    }
    if (kind == NW_TABLE && !normal && grid->len_full > 0) {
        const size_t cnt = (size_t)F * grid->len_full;
        const size_t bytes = cnt * 2 * p->esz;
        NW_HIP(hipMalloc(&p->d_table, bytes));
        p->d_table_bytes = bytes;
        if (p->dtype == NW_F64) {
            NW_HIP(hipMemcpy(p->d_table, table, bytes, hipMemcpyHostToDevice));
        } else {
            std::vector<float> tmp(cnt * 2);
            const double* src = (const double*)table;
            for (size_t i = 0; i < cnt * 2; ++i) tmp[i] = (float)src[i];
            NW_HIP(hipMemcpy(p->d_table, tmp.data(), bytes, hipMemcpyHostToDevice));
        }
    }
    d.freq = p->d_freq;
    d.peak = p->d_peak;
    d.xstep32 = p->d_xstep32;
    d.table = p->d_table;
    d.row_len = p->d_row_len;
    p->desc = d;
    p->has_wavelet = true;
    p->wtab_valid = false;
    if (p->chirp_tentative) {   // a new wavelet may fit where the last one did not
        p->chirp = true;
        p->engine = NW_ENGINE_FUSED;
        p->stats.engine = NW_ENGINE_FUSED;
    }
    NW_TRY(setup_unique_rows(p, kind, freqs, peak, xstep, normal ? nullptr : table));
    nw_logf(1, "plan %p: wavelet kind %d, %d scales (%s), row length %lld", (void*)p, kind, F,
            p->dedup ? (std::to_string(p->nuniq) + " distinct rows, expanded after the transform").c_str()
                     : "every row distinct",
            (long long)d.len_full);
    return NW_OK;
}

int nw_plan_wavelet_shape(nw_plan* p, int64_t* len_full, int64_t* row_len) {
    if (!p || !len_full) return fail(NW_E_INVALID, "nw_plan_wavelet_shape: null argument");
    if (!p->has_wavelet) return fail(NW_E_STATE, "nw_plan_wavelet_shape: no wavelet attached");
    *len_full = p->desc.len_full;
    if (row_len)
        for (int f = 0; f < p->nfreq; ++f)
            row_len[f] = (p->desc.kind == NW_TABLE && !p->row_len_host.empty()) ? p->row_len_host[f] : p->desc.len_full;
    return NW_OK;
}

int nw_plan_wavelet_rows(nw_plan* p, void* out_host) {
    if (!p || !out_host) return fail(NW_E_INVALID, "nw_plan_wavelet_rows: null argument");
    if (!p->has_wavelet) return fail(NW_E_STATE, "nw_plan_wavelet_rows: no wavelet attached");
    if (p->desc.len_full == 0) return NW_OK;
    DeviceGuard guard(p->device);
    const size_t bytes = (size_t)p->nfreq * p->desc.len_full * p->esz * (p->desc.kind == NW_TABLE ? 2 : 1);
    void* d_rows = nullptr;
    NW_HIP(hipMalloc(&d_rows, bytes));
    hipError_t e = nw::launch_rows(p->desc, p->dtype, d_rows, p->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(out_host, d_rows, bytes, hipMemcpyDeviceToHost, p->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
    (void)hipFree(d_rows);
    if (e != hipSuccess) return fail(NW_E_HIP, std::string("nw_plan_wavelet_rows: ") + hipGetErrorString(e));
    return NW_OK;
}

int nw_plan_row_support(nw_plan* p, int method, int32_t* kmax_out) {
    if (!p || !kmax_out) return fail(NW_E_INVALID, "nw_plan_row_support: null argument");
    if (!p->has_wavelet) return fail(NW_E_STATE, "nw_plan_row_support: no wavelet attached");
    if (!p->large || p->engine == NW_ENGINE_ROCFFT)
        return fail(NW_E_STATE, "nw_plan_row_support: the plan does not run the two-pass engine");
    if (method != 0 && method != 1) return fail(NW_E_INVALID, "nw_plan_row_support: bad method");
    DeviceGuard guard(p->device);
    set_exec_geometry(p);
    // into a scratch buffer (the plan's own support stays as built: under a repeated-rows view
    // it holds the distinct rows only)
    void* tmp = nullptr;
    NW_HIP(hipMalloc(&tmp, nw::large_support_bytes(p->nfreq)));
    hipError_t e = nw::large_row_support(p->desc, p->dtype, tmp, method == 1, p->stream);
    const void* src = tmp;
    if (e == hipSuccess) e = hipMemcpyAsync(kmax_out, src, (size_t)p->nfreq * sizeof(int32_t), hipMemcpyDeviceToHost, p->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
    if (tmp) (void)hipFree(tmp);
    if (e != hipSuccess) return fail(NW_E_HIP, std::string("nw_plan_row_support: ") + hipGetErrorString(e));
    return NW_OK;
}

int nw_execute(nw_plan* p, const void* x, int64_t nsig, void* out, int out_kind, int mem) {
    if (!p || (!x && nsig > 0) || (!out && nsig > 0)) return fail(NW_E_INVALID, "nw_execute: null argument");
    if (!p->has_wavelet) return fail(NW_E_STATE, "nw_execute: nw_plan_set_wavelet first");
    if (out_kind < NW_OUT_CWT || out_kind > NW_OUT_PHASE_SUM) return fail(NW_E_INVALID, "nw_execute: bad out_kind");
    if (mem != NW_MEM_HOST && mem != NW_MEM_DEVICE) return fail(NW_E_INVALID, "nw_execute: bad mem");
    if (nsig < 0) return fail(NW_E_INVALID, "nw_execute: nsig < 0");
    if (is_reduction(out_kind) && !out) return fail(NW_E_INVALID, "nw_execute: null out");
    if (nsig == 0 && !is_reduction(out_kind)) return NW_OK;
    DeviceGuard guard(p->device);
    set_exec_geometry(p);
    if (p->chirp && p->chirp_tentative && !p->wtab_valid) {   // settle the engine before any buffer choice
        if (p->dedup) {
            UniqueRows u(p);
            NW_TRY(chirp_table(p));
        } else {
            NW_TRY(chirp_table(p));
        }
    }

    nw_logf(1, "plan %p: execute %s, %lld signals, %s buffers", (void*)p, out_name(out_kind), (long long)nsig,
            mem == NW_MEM_HOST ? "host" : "device");
    if (is_reduction(out_kind)) {
        NW_TRY(execute_reduce(p, x, nsig, out, out_kind, mem == NW_MEM_HOST));
        return dcheck_collect(p->stream);
    }

    const size_t out_elem = (out_kind == NW_OUT_CWT ? 2 : 1) * p->esz;
    const size_t row_out = (size_t)p->nfreq * p->n * out_elem;  // one signal's output bytes
    const bool host = mem == NW_MEM_HOST;
    if (host && out_kind != NW_OUT_CWT && p->engine == NW_ENGINE_ROCFFT)
        NW_TRY(ensure(&p->d_out, &p->d_out_bytes, (size_t)p->max_batch * row_out));
    if (host && p->engine == NW_ENGINE_FUSED) NW_TRY(ensure(&p->d_out, &p->d_out_bytes, (size_t)p->max_batch * row_out));
    if (host && p->engine == NW_ENGINE_ROCFFT && out_kind == NW_OUT_CWT) NW_TRY(need_Y(p));
    // (rocFFT engine, host CWT: the complex result is read back straight from d_Y)
    // a page-locked destination (nw_host_alloc) is written by DMA directly (a fresh pageable
    // array the caller allocated may have been advised onto huge pages by it, nw_host_advise;
    // the caller's memory policy is never changed here)
    const bool direct = host && host_pinned(out, (size_t)nsig * row_out);

    for (int64_t s0 = 0; s0 < nsig; s0 += p->max_batch) {
        const int64_t c = std::min<int64_t>(p->max_batch, nsig - s0);
        const char* xs = (const char*)x + (size_t)s0 * p->n * p->esz;
        char* os = (char*)out + (size_t)s0 * row_out;
        if (host) {
            NW_TRY(staged(p, ST_COPY, [&] {
                NW_HIP(hipMemcpyAsync(p->d_x, xs, (size_t)c * p->n * p->esz, hipMemcpyHostToDevice, p->stream));
                return NW_OK;
            }));
            void* dst = (p->engine == NW_ENGINE_ROCFFT && out_kind == NW_OUT_CWT) ? p->d_Y : p->d_out;
            NW_TRY(run_chunk(p, p->d_x, c, dst, out_kind, true));
            NW_TRY(staged(p, ST_COPY, [&] {
                if (direct) {
                    NW_HIP(hipMemcpyAsync(os, dst, (size_t)c * row_out, hipMemcpyDeviceToHost, p->stream));
                    return NW_OK;
                }
                return copy_out(p, os, (const char*)dst, (size_t)c * row_out);
            }));
            NW_HIP(hipStreamSynchronize(p->stream));
        } else {
            NW_TRY(run_chunk(p, xs, c, os, out_kind, true));
        }
        p->stats.chunks++;
    }
    p->stats.executes++;
    if (host) NW_TRY(resolve_timing(p));
    return dcheck_collect(p->stream);
}

}  // extern "C"

namespace {

using nw::host::block_of;   // balanced contiguous blocks, as dist.shard

// A plan is not reentrant: one host thread per plan, so a plan may appear only once.
int check_distinct(nw_plan* const* plans, int nplans, const char* who) {
    for (int i = 0; i < nplans; ++i) {
        if (!plans[i]) return fail(NW_E_INVALID, std::string(who) + ": null plan");
        for (int j = 0; j < i; ++j)
            if (plans[j] == plans[i])
                return fail(NW_E_INVALID, std::string(who) + ": plan " + std::to_string(i) +
                                              " repeats plan " + std::to_string(j) +
                                              " (a plan is not reentrant: create one plan per shard)");
    }
    return NW_OK;
}

// Reductions over devices: each device sums its contiguous block (fp64 partial sums),
// the host adds them in device order, then takes the mean / |mean| exactly as
// k_finalize does.
static int execute_multi_reduce(nw_plan* const* plans, int nplans, const void* x, int64_t nsig, void* out,
                                int out_kind) {
    const nw_plan* p0 = plans[0];
    const bool phase = is_phase(out_kind);
    const int64_t fn = (int64_t)p0->nfreq * p0->n;
    const size_t comps = (size_t)fn * (phase ? 2 : 1);
    const size_t x_row = (size_t)p0->n * p0->esz;
    std::vector<std::vector<double>> part(nplans);
    std::vector<int> rc(nplans, NW_OK);
    std::vector<std::string> err(nplans);
    std::vector<std::thread> th;
    for (int i = 0; i < nplans; ++i) {
        int64_t s0 = 0, cnt = 0;
        block_of(nsig, i, nplans, &s0, &cnt);
        if (cnt <= 0) continue;
        part[i].assign(comps, 0.0);
        th.emplace_back([&, i, s0, cnt] {
            rc[i] = nw_execute(plans[i], (const char*)x + s0 * x_row, cnt, part[i].data(),
                               phase ? NW_OUT_PHASE_SUM : NW_OUT_POWER_SUM, NW_MEM_HOST);
            if (rc[i] != NW_OK) err[i] = g_last_error;
        });
    }
    for (auto& t : th) t.join();
    for (int i = 0; i < nplans; ++i)
        if (rc[i] != NW_OK) return fail(rc[i], "device " + std::to_string(plans[i]->device) + ": " + err[i]);
    std::vector<double> tot(comps, 0.0);
    for (int i = 0; i < nplans; ++i)
        for (size_t j = 0; j < part[i].size(); ++j) tot[j] += part[i][j];
    if (out_kind == NW_OUT_POWER_SUM || out_kind == NW_OUT_PHASE_SUM) {
        std::memcpy(out, tot.data(), comps * sizeof(double));
        return NW_OK;
    }
    const double d = (double)nsig;
    for (int64_t j = 0; j < fn; ++j) {
        const double v = phase ? std::hypot(tot[2 * j] / d, tot[2 * j + 1] / d) : tot[j] / d;
        if (p0->dtype == NW_F32)
            static_cast<float*>(out)[j] = (float)v;
        else
            static_cast<double*>(out)[j] = v;
    }
    return NW_OK;
}

int check_same_config(nw_plan* const* plans, int nplans, const char* who) {
    for (int i = 1; i < nplans; ++i)
        if (plans[i]->n != plans[0]->n || plans[i]->nfreq != plans[0]->nfreq || plans[i]->dtype != plans[0]->dtype)
            return fail(NW_E_INVALID, std::string(who) + ": plans must share n, nfreq and dtype");
    return NW_OK;
}

}  // namespace

extern "C" {

int nw_execute_multi(nw_plan* const* plans, int nplans, const void* x, int64_t nsig, void* out, int out_kind) {
    if (!plans || nplans < 1) return fail(NW_E_INVALID, "nw_execute_multi: no plans");
    NW_TRY(check_distinct(plans, nplans, "nw_execute_multi"));
    NW_TRY(check_same_config(plans, nplans, "nw_execute_multi"));
    const nw_plan* p0 = plans[0];
    if (out_kind < NW_OUT_CWT || out_kind > NW_OUT_PHASE_SUM) return fail(NW_E_INVALID, "nw_execute_multi: bad out_kind");
    if (nsig < 0) return fail(NW_E_INVALID, "nw_execute_multi: nsig < 0");
    if (is_reduction(out_kind)) return execute_multi_reduce(plans, nplans, x, nsig, out, out_kind);
    const size_t x_row = (size_t)p0->n * p0->esz;
    const size_t o_row = (size_t)p0->nfreq * p0->n * (out_kind == NW_OUT_CWT ? 2 : 1) * p0->esz;
    std::vector<int> rc(nplans, NW_OK);
    std::vector<std::string> err(nplans);
    std::vector<std::thread> th;
    for (int i = 0; i < nplans; ++i) {
        int64_t s0 = 0, cnt = 0;
        block_of(nsig, i, nplans, &s0, &cnt);
        if (cnt <= 0) continue;
        th.emplace_back([&, i, s0, cnt] {
            rc[i] = nw_execute(plans[i], (const char*)x + s0 * x_row, cnt, (char*)out + s0 * o_row, out_kind,
                               NW_MEM_HOST);
            if (rc[i] != NW_OK) err[i] = g_last_error;
        });
    }
    for (auto& t : th) t.join();
    for (int i = 0; i < nplans; ++i)
        if (rc[i] != NW_OK)
            return fail(rc[i], "device " + std::to_string(plans[i]->device) + ": " + err[i]);
    return NW_OK;
}

// Device-resident sharding (one process, one host thread per device).  Plan i
// transforms its own device-resident block x[i] (nsig[i] signals) into out[i]; nothing
// crosses PCIe.  Reductions: every device sums its block into fp64 partials, device 0
// gathers them peer-to-peer, adds them in device order and finalises into out[0].
int nw_execute_multi_device(nw_plan* const* plans, int nplans, const void* const* x, const int64_t* nsig,
                            void* const* out, int out_kind) {
    if (!plans || nplans < 1 || !x || !nsig || !out) return fail(NW_E_INVALID, "nw_execute_multi_device: null argument");
    NW_TRY(check_distinct(plans, nplans, "nw_execute_multi_device"));
    NW_TRY(check_same_config(plans, nplans, "nw_execute_multi_device"));
    if (out_kind < NW_OUT_CWT || out_kind > NW_OUT_PHASE_SUM)
        return fail(NW_E_INVALID, "nw_execute_multi_device: bad out_kind");
    int64_t total = 0;
    for (int i = 0; i < nplans; ++i) {
        if (nsig[i] < 0) return fail(NW_E_INVALID, "nw_execute_multi_device: nsig < 0");
        total += nsig[i];
    }
    const bool reduce = is_reduction(out_kind);
    if (reduce && !out[0]) return fail(NW_E_INVALID, "nw_execute_multi_device: null out[0]");
    nw_plan* p0 = plans[0];
    const bool phase = is_phase(out_kind);
    const int64_t fn = (int64_t)p0->nfreq * p0->n;
    const size_t acc_bytes = (size_t)fn * (phase ? 2 : 1) * sizeof(double);
    // reductions: per-device fp64 partial sums (each plan's d_part), then device 0's gather
    // buffer (plans[0]->d_gather); both persist on the plans and are freed with them
    std::vector<void*> part(nplans, nullptr);
    if (reduce) {
        for (int i = 0; i < nplans; ++i) {
            DeviceGuard g(plans[i]->device);
            const int r = ensure(&plans[i]->d_part, &plans[i]->d_part_bytes, acc_bytes);
            if (r != NW_OK) return fail(r, "device " + std::to_string(plans[i]->device) +
                                                ": nw_execute_multi_device: partial-sum buffer: " + g_last_error);
            part[i] = plans[i]->d_part;
        }
    }
    std::vector<int> rc(nplans, NW_OK);
    std::vector<std::string> err(nplans);
    std::vector<std::thread> th;
    for (int i = 0; i < nplans; ++i) {
        th.emplace_back([&, i] {
            nw_plan* p = plans[i];
            rc[i] = nw_execute(p, x[i], nsig[i], reduce ? part[i] : out[i],
                               reduce ? (phase ? NW_OUT_PHASE_SUM : NW_OUT_POWER_SUM) : out_kind, NW_MEM_DEVICE);
            if (rc[i] == NW_OK) rc[i] = nw_plan_sync(p);
            if (rc[i] != NW_OK) err[i] = g_last_error;
        });
    }
    for (auto& t : th) t.join();
    for (int i = 0; i < nplans; ++i)
        if (rc[i] != NW_OK) return fail(rc[i], "device " + std::to_string(plans[i]->device) + ": " + err[i]);
    if (!reduce) return NW_OK;
    int r = NW_OK;
    {
        DeviceGuard g(p0->device);
        auto hip = [&](hipError_t e, const char* what) {
            if (e != hipSuccess && r == NW_OK)
                r = fail(NW_E_HIP, std::string("nw_execute_multi_device: ") + what + ": " + hipGetErrorString(e));
            return r == NW_OK;
        };
        const int64_t comps = fn * (phase ? 2 : 1);
        double* acc = (double*)part[0];
        void* gather = nullptr;
        if (nplans > 1) {
            r = ensure(&p0->d_gather, &p0->d_gather_bytes, acc_bytes);
            gather = p0->d_gather;
        }
        for (int i = 1; i < nplans && r == NW_OK; ++i) {
            if (hip(hipMemcpyPeerAsync(gather, p0->device, part[i], plans[i]->device, acc_bytes, p0->stream), "peer copy"))
                hip(nw::launch_add_f64(acc, (const double*)gather, comps, p0->stream), "add");
        }
        if (r == NW_OK) {
            if (out_kind == NW_OUT_POWER_SUM || out_kind == NW_OUT_PHASE_SUM)
                hip(hipMemcpyAsync(out[0], acc, acc_bytes, hipMemcpyDeviceToDevice, p0->stream), "copy");
            else
                hip(nw::launch_finalize(p0->dtype, phase, acc, out[0], fn, total, p0->stream), "finalize");
        }
        hip(hipStreamSynchronize(p0->stream), "sync");
    }
    return r;
}

int nw_execute_multi_scales(nw_plan* const* plans, int nplans, const void* x, int64_t nsig, void* out,
                            int out_kind) {
    if (!plans || nplans < 1 || !plans[0]) return fail(NW_E_INVALID, "nw_execute_multi_scales: no plans");
    NW_TRY(check_distinct(plans, nplans, "nw_execute_multi_scales"));
    const nw_plan* p0 = plans[0];
    for (int i = 1; i < nplans; ++i)
        if (!plans[i] || plans[i]->n != p0->n || plans[i]->dtype != p0->dtype ||
            (plans[i]->flags & NW_INTERPOLATE) != (p0->flags & NW_INTERPOLATE))
            return fail(NW_E_INVALID, "nw_execute_multi_scales: plans must share n, dtype and interpolate");
    if (out_kind < NW_OUT_CWT || out_kind > NW_OUT_PHASE_SUM)
        return fail(NW_E_INVALID, "nw_execute_multi_scales: bad out_kind");
    if (nsig < 0) return fail(NW_E_INVALID, "nw_execute_multi_scales: nsig < 0");
    if (nsig > 0 && (!x || !out)) return fail(NW_E_INVALID, "nw_execute_multi_scales: null argument");
    int64_t F = 0;
    std::vector<int64_t> f0(nplans);
    for (int i = 0; i < nplans; ++i) {
        f0[i] = F;
        F += plans[i]->nfreq;
    }
    // bytes of one output element: reductions keep their own types (include/ninwave.h)
    size_t oe = (out_kind == NW_OUT_CWT ? 2 : 1) * p0->esz;
    if (out_kind == NW_OUT_POWER_SUM) oe = sizeof(double);
    if (out_kind == NW_OUT_PHASE_SUM) oe = 2 * sizeof(double);
    const size_t x_row = (size_t)p0->n * p0->esz, o_scale = (size_t)p0->n * oe;
    std::vector<int> rc(nplans, NW_OK);
    std::vector<std::string> err(nplans);
    std::vector<std::thread> th;
    for (int i = 0; i < nplans; ++i) {
        th.emplace_back([&, i] {
            nw_plan* p = plans[i];
            if (is_reduction(out_kind) || nsig <= 1) {   // the rows are contiguous in out
                rc[i] = nw_execute(p, x, nsig, (char*)out + f0[i] * o_scale, out_kind, NW_MEM_HOST);
            } else {
                for (int64_t s = 0; s < nsig && rc[i] == NW_OK; ++s)
                    rc[i] = nw_execute(p, (const char*)x + s * x_row, 1,
                                       (char*)out + ((size_t)s * F + f0[i]) * o_scale, out_kind, NW_MEM_HOST);
            }
            if (rc[i] != NW_OK) err[i] = g_last_error;
        });
    }
    for (auto& t : th) t.join();
    for (int i = 0; i < nplans; ++i)
        if (rc[i] != NW_OK)
            return fail(rc[i], "device " + std::to_string(plans[i]->device) + ": " + err[i]);
    return NW_OK;
}

int nw_baseline(int device, int dtype, const void* x, int64_t count, int64_t row_len, int64_t row0, int64_t row1,
                int op, void* out, int mem, double* stats) {
    if (dtype != NW_F32 && dtype != NW_F64) return fail(NW_E_INVALID, "nw_baseline: dtype must be NW_F32 or NW_F64");
    if (op < NW_BL_MEAN || op > NW_BL_ZLOG) return fail(NW_E_INVALID, "nw_baseline: unknown op");
    if (mem != NW_MEM_HOST && mem != NW_MEM_DEVICE) return fail(NW_E_INVALID, "nw_baseline: bad mem");
    if (count < 0 || row_len < 1 || row0 < 0 || row1 < row0 || row1 > count / row_len)
        return fail(NW_E_INVALID, "nw_baseline: baseline rows out of range");
    if (count > 0 && (!x || !out)) return fail(NW_E_INVALID, "nw_baseline: null array");
    int ndev = 0;
    NW_TRY(nw_device_count(&ndev));
    if (device < 0 || device >= ndev) return fail(NW_E_INVALID, "nw_baseline: device out of range");
    DeviceGuard guard(device);
    const size_t esz = dtype == NW_F32 ? sizeof(float) : sizeof(double);
    const size_t bytes = (size_t)count * esz;
    void* dx = const_cast<void*>(x);
    void* dout = out;
    void* work = nullptr;
    int rc = NW_OK;
    auto hip = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && rc == NW_OK) rc = fail(NW_E_HIP, std::string("nw_baseline: ") + what + ": " + hipGetErrorString(e));
        return e == hipSuccess;
    };
    const bool host = mem == NW_MEM_HOST;
    if (hip(hipMalloc(&work, nw::BL_WORK_DOUBLES * sizeof(double)), "hipMalloc") && host && bytes) {
        dx = dout = nullptr;
        if (hip(hipMalloc(&dx, bytes), "hipMalloc") && hip(hipMalloc(&dout, bytes), "hipMalloc"))
            hip(hipMemcpy(dx, x, bytes, hipMemcpyHostToDevice), "H2D");
    }
    if (rc == NW_OK)
        hip(nw::launch_baseline(dtype, dx, count, row0 * row_len, row1 * row_len, op, dout, (double*)work, nullptr),
            "launch");
    if (rc == NW_OK) hip(hipStreamSynchronize(nullptr), "sync");
    if (rc == NW_OK && host && bytes) hip(hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost), "D2H");
    if (rc == NW_OK && stats)
        hip(hipMemcpy(stats, (double*)work + (nw::BL_WORK_DOUBLES - 2), 2 * sizeof(double), hipMemcpyDeviceToHost),
            "D2H stats");
    if (work) (void)hipFree(work);
    if (host && bytes) {
        if (dx) (void)hipFree(dx);
        if (dout) (void)hipFree(dout);
    }
    return rc == NW_OK ? dcheck_collect(nullptr) : rc;
}

int nw_make_wavelets(int device, int kind, const double* params, int nparams, const double* freqs, int nfreq,
                     double sfreq, double rwl, void* out, int64_t* max_len, int64_t* row_len) {
    const bool reverse = kind == NW_MORSE || kind == NW_SHANNON;
    if (!reverse && kind != NW_MORLET && kind != NW_MEXICAN_HAT && kind != NW_HAAR)
        return fail(NW_E_INVALID, "nw_make_wavelets: kind must be a stock wavelet");
    if (nfreq < 0 || (nfreq > 0 && !freqs) || !max_len || !row_len) return fail(NW_E_INVALID, "nw_make_wavelets: null argument");
    if (!(sfreq > 0.0)) return fail(NW_E_INVALID, "nw_make_wavelets: sfreq must be > 0");
    nw::WaveParams wp{};
    wp.kind = kind;
    if (kind == NW_MORSE) {
        wp.b = nparams > 0 ? params[0] : 17.5;
        wp.r = nparams > 1 ? params[1] : 3.0;
        wp.b_over_r = wp.b / wp.r;
    } else if (kind == NW_MORLET) {
        wp.sigma = nparams > 0 ? params[0] : 7.0;
        const bool gabor = nparams > 1 && params[1] != 0.0;
        const double s2 = wp.sigma * wp.sigma;
        const double c = nparams > 2 ? params[2] : std::pow(1.0 + std::exp(-s2) - 2.0 * std::exp(-3.0 / 4.0 * s2), -0.5);
        wp.cpi = c * std::pow(M_PI, -0.25);
        wp.kappa = nparams > 3 ? params[3] : (gabor ? 0.0 : std::exp(-std::pow(wp.sigma, 2.0) / 2.0));
    } else if (kind == NW_MEXICAN_HAT) {
        wp.sigma = nparams > 0 ? params[0] : 7.0;
    }
    std::vector<nw::WaveRow> rows(nfreq);
    std::map<int64_t, std::vector<int>> by_m;
    int64_t lmax = 0, off = 0;
    for (int f = 0; f < nfreq; ++f) {
        const double fr = freqs[f];
        if (fr == 0.0) return fail(NW_E_INVALID, "nw_make_wavelets: freq == 0 (ZeroDivisionError, base.py:347-348)");
        nw::WaveRow r{};
        if (reverse) {                        // _setup_trans_shape(freq, real_wave_length), base.py:191-194
            const double one = 1.0 / fr;
            r.m = nw::host::arange_len(sfreq / fr * rwl, one);
            r.len = 2 * (r.m / 2);
            r.t0 = 0.0;
            r.delta = one;
            r.t1 = one;
            by_m[r.m].push_back(f);
        } else {                              // _setup_waveletshape(freq, 1, zero_mean=True), base.py:211-216
            const double peak = kind == NW_MORLET ? wp.sigma / (1.0 - std::exp(-wp.sigma * fr))
                                : kind == NW_MEXICAN_HAT ? std::sqrt(6.0) / M_PI / M_PI : 1.0;
            const double total = 1.0 / peak * fr * 2.0 * M_PI;
            const double one = 1.0 / sfreq * 2.0 * M_PI * fr / peak;
            r.t0 = -total / 2.0;
            r.m = nw::host::arange_len_from(r.t0, total / 2.0, one);
            r.len = r.m;
            r.t1 = r.t0 + one;
            r.delta = r.t1 - r.t0;
        }
        row_len[f] = r.len;
        lmax = std::max(lmax, r.len);
        rows[f] = r;
    }
    for (auto& kv : by_m)
        for (int f : kv.second) {
            rows[f].off = off;
            off += kv.first;
        }
    *max_len = lmax;
    if (!out || nfreq == 0 || lmax == 0) {
        if (out && nfreq > 0) std::memset(out, 0, (size_t)nfreq * lmax * 16);
        return NW_OK;
    }
    int ndev = 0;
    NW_TRY(nw_device_count(&ndev));
    if (device < 0 || device >= ndev) return fail(NW_E_INVALID, "nw_make_wavelets: device out of range");
    std::call_once(g_rocfft_once, [] { rocfft_setup(); });
    DeviceGuard guard(device);
    void *d_rows = nullptr, *d_buf = nullptr, *d_out = nullptr, *d_work = nullptr;
    rocfft_execution_info info = nullptr;
    int rc = NW_OK;
    auto hip = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && rc == NW_OK) rc = fail(NW_E_HIP, std::string("nw_make_wavelets: ") + what + ": " + hipGetErrorString(e));
        return rc == NW_OK;
    };
    const size_t obytes = (size_t)nfreq * lmax * 16;
    if (hip(hipMalloc(&d_rows, nfreq * sizeof(nw::WaveRow)), "hipMalloc") &&
        hip(hipMalloc(&d_out, obytes), "hipMalloc") &&
        hip(hipMemcpy(d_rows, rows.data(), nfreq * sizeof(nw::WaveRow), hipMemcpyHostToDevice), "H2D")) {
        if (!reverse) {
            hip(nw::launch_wavelet_time((const nw::WaveRow*)d_rows, nfreq, lmax, wp, d_out, nullptr), "time rows");
        } else if (hip(hipMalloc(&d_buf, (size_t)std::max<int64_t>(off, 1) * 16), "hipMalloc") &&
                   hip(nw::launch_wavelet_spectra((const nw::WaveRow*)d_rows, nfreq, wp, d_buf, nullptr), "spectra")) {
            if (rocfft_execution_info_create(&info) != rocfft_status_success) rc = fail(NW_E_ROCFFT, "nw_make_wavelets: rocfft info");
            for (auto& kv : by_m) {
                if (rc != NW_OK || kv.first == 0) continue;
                rocfft_plan pl = nullptr;
                size_t len = (size_t)kv.first, ws = 0;
                if (rocfft_plan_create(&pl, rocfft_placement_inplace, rocfft_transform_type_complex_inverse,
                                       rocfft_precision_double, 1, &len, kv.second.size(), nullptr) != rocfft_status_success) {
                    rc = fail(NW_E_ROCFFT, "nw_make_wavelets: rocfft_plan_create");
                    break;
                }
                rocfft_plan_get_work_buffer_size(pl, &ws);
                if (ws && hip(hipMalloc(&d_work, ws), "hipMalloc")) rocfft_execution_info_set_work_buffer(info, d_work, ws);
                void* ib[1] = {(char*)d_buf + (size_t)rows[kv.second[0]].off * 16};
                if (rc == NW_OK && rocfft_execute(pl, ib, nullptr, info) != rocfft_status_success)
                    rc = fail(NW_E_ROCFFT, "nw_make_wavelets: rocfft_execute");
                hip(hipDeviceSynchronize(), "sync");
                rocfft_plan_destroy(pl);
                if (d_work) {
                    (void)hipFree(d_work);
                    d_work = nullptr;
                }
            }
            if (rc == NW_OK) hip(nw::launch_wavelet_pack((const nw::WaveRow*)d_rows, nfreq, lmax, d_buf, d_out, nullptr), "pack");
        }
        if (rc == NW_OK) hip(hipDeviceSynchronize(), "sync");
        if (rc == NW_OK) hip(hipMemcpy(out, d_out, obytes, hipMemcpyDeviceToHost), "D2H");
    }
    if (info) rocfft_execution_info_destroy(info);
    for (void* b : {d_rows, d_buf, d_out})
        if (b) (void)hipFree(b);
    return rc == NW_OK ? dcheck_collect(nullptr) : rc;
}

int nw_plan_set_stream(nw_plan* p, void* stream) {
    if (!p) return fail(NW_E_INVALID, "nw_plan_set_stream: null plan");
    p->stream = stream ? (hipStream_t)stream : p->own_stream;
    return NW_OK;
}

int nw_plan_get_stream(nw_plan* p, void** stream) {
    if (!p || !stream) return fail(NW_E_INVALID, "nw_plan_get_stream: null argument");
    *stream = (void*)p->stream;
    return NW_OK;
}

int nw_host_alloc(int64_t bytes, void** ptr) {
    if (!ptr || bytes <= 0) return fail(NW_E_INVALID, "nw_host_alloc: bad argument");
    *ptr = nullptr;
    NW_HIP(hipHostMalloc(ptr, (size_t)bytes, hipHostMallocDefault));
    std::lock_guard<std::mutex> lk(g_host_mu);
    g_host_bufs[(uintptr_t)*ptr] = (size_t)bytes;
    return NW_OK;
}

int nw_host_advise(void* ptr, int64_t bytes, int64_t* advised) {
    if (!ptr || bytes < 0) return fail(NW_E_INVALID, "nw_host_advise: bad argument");
    const size_t a = nw::host::advise_output(reinterpret_cast<char*>(ptr), (size_t)bytes);
    if (advised) *advised = (int64_t)a;
    return NW_OK;
}

int nw_host_free(void* ptr) {
    {
        std::lock_guard<std::mutex> lk(g_host_mu);
        auto it = g_host_bufs.find((uintptr_t)ptr);
        if (it == g_host_bufs.end()) return fail(NW_E_INVALID, "nw_host_free: not an nw_host_alloc pointer");
        g_host_bufs.erase(it);
    }
    NW_HIP(hipHostFree(ptr));
    return NW_OK;
}

int nw_plan_sync(nw_plan* p) {
    if (!p) return fail(NW_E_INVALID, "nw_plan_sync: null plan");
    DeviceGuard guard(p->device);
    NW_HIP(hipStreamSynchronize(p->stream));
    NW_TRY(resolve_timing(p));
    return dcheck_collect(p->stream);
}

int nw_plan_stats(nw_plan* p, nw_stats* s) {
    if (!p || !s) return fail(NW_E_INVALID, "nw_plan_stats: null argument");
    DeviceGuard guard(p->device);
    NW_TRY(resolve_timing(p));
    *s = p->stats;
    // the sized buffers (the per-freq arrays, row maps and rocFFT plan objects are small)
    s->device_bytes = (int64_t)((size_t)p->max_batch * p->n * p->esz + (size_t)p->max_batch * p->nh * 2 * p->esz +
                                p->d_table_bytes + p->d_uout_bytes + p->d_Y_bytes + p->d_out_bytes + p->d_acc_bytes +
                                p->d_part_bytes + p->d_gather_bytes + p->d_wtab_bytes + p->d_oscr_bytes +
                                p->d_scratch_bytes + p->work_bytes);
    return NW_OK;
}

int nw_plan_reset_stats(nw_plan* p) {
    if (!p) return fail(NW_E_INVALID, "nw_plan_reset_stats: null plan");
    DeviceGuard guard(p->device);
    NW_TRY(resolve_timing(p));
    const int64_t engine = p->stats.engine, uniq = p->stats.unique_rows, kernel = p->stats.kernel;
    p->stats = nw_stats{};
    p->stats.engine = engine;
    p->stats.unique_rows = uniq;
    p->stats.kernel = kernel;
    return NW_OK;
}

int nw_plan_destroy(nw_plan* p) {
    if (!p) return NW_OK;
    DeviceGuard guard(p->device);
    (void)hipStreamSynchronize(p->stream);
    free_plan(p);
    return NW_OK;
}

}  // extern "C"
