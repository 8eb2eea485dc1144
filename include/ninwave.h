/*
 * ninwave.h — C ABI of libninwave.so, the MI355X (gfx950) FFT-domain CWT engine.
 *
 * This is the drop-in boundary for ninwavelets' hot path:
 *   WaveletBase.cwt / power / abs         reference base.py:378-443
 *   WaveletBase.make_fft_wavelet(s)       reference base.py:221-279
 *   WaveletBase._setup_trans_shape        reference base.py:173-194
 *   pad_to / interpolate_alias            reference base.py:75-82, 107-123
 *   Morse / Morlet / Shannon spectra      reference wavelets.py:65-74, 132-136, 256-262
 *   EpochsWavelet.cwt (batched caller)    reference mneutils.py:26-40
 * The reference is pure Python/numpy, so it has no FFI of its own; the Python
 * host layer (ninwavelets_amd/_lib.py, ctypes) binds exactly these symbols, and
 * INTEGRATION.md shows the binding a maintainer would add to the reference.
 *
 * Conventions
 *  - Every function returns int status: NW_OK (0) or a negative NW_E* code;
 *    nw_last_error() returns a thread-local message for the last failure.
 *  - Plain pointers and sizes only.  Host buffers are C-contiguous row-major.
 *  - A plan is bound to one device and one HIP stream; it is not reentrant.
 *  - Complex numbers are interleaved (re, im) of the plan's real dtype.
 */
#ifndef NINWAVE_H
#define NINWAVE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define NW_OK              0
#define NW_E_INVALID      -1   /* bad argument (maps to ValueError) */
#define NW_E_HIP          -2   /* HIP runtime error */
#define NW_E_ROCFFT       -3   /* rocFFT error */
#define NW_E_NOMEM        -4   /* device allocation failed */
#define NW_E_STATE        -5   /* call out of order (e.g. execute before set_wavelet) */
#define NW_E_NODEVICE     -6   /* no HIP device visible */
#define NW_E_BOUNDS       -7   /* debug library only: a kernel bounds check failed */

/* compute dtypes (the arithmetic type of the whole path) */
#define NW_F32 0
#define NW_F64 1

/* wavelet kinds */
#define NW_MORSE   1   /* params: b, r                      wavelets.py:38-74  */
#define NW_MORLET  2   /* params: sigma, gabor(0/1)         wavelets.py:110-144 */
#define NW_SHANNON 3   /* params: none (freq is ignored)    wavelets.py:256-262 */
#define NW_TABLE   4   /* complex128 rows supplied by the host (WaveletMode.Normal,
                          user plugins overriding trans_formula/formula)          */
#define NW_MEXICAN_HAT 5  /* params: sigma, sfreq, real_wave_length   wavelets.py:194-228 */
#define NW_HAAR        6  /* params: sfreq, real_wave_length          wavelets.py:265-280
                             Both are WaveletMode.Normal tables built ON THE DEVICE
                             (base.py:249-256): the time-domain wavelet on np.arange's
                             grid, zero-padded to ~sfreq*real_wave_length, fp64 rocFFT,
                             |Re| + i|Im| (+ interpolate_alias), ragged row lengths. */

/* plan flags */
#define NW_INTERPOLATE   0x1u  /* zero the upper half of fft(x) (interpolate_alias, base.py:400-401) */
#define NW_ENGINE_ROCFFT 0x10u /* force: rocFFT fwd -> K1 multiply -> rocFFT inv -> K2 epilogue   */
#define NW_ENGINE_FUSED  0x20u /* force: rocFFT fwd -> fused multiply+LDS inverse FFT+epilogue
                                  (n > 16384: the two-pass form, nw_large.hip; n not a power
                                  of two >= 1024 with 2n-1 <= 16384 fp32 / 8192 fp64: the
                                  chirp-z form, nw_chirp.hip)                                  */
#define NW_TIMING        0x100u/* record HIP events around every stage (nw_plan_stats)            */
#define NW_TIMING_CHAIN  0x800u/* with NW_TIMING: the plan's stream carries nothing but this plan's
                                  executes between two nw_plan_sync / nw_plan_stats calls (a
                                  dedicated benchmark stream), so each stage -- the first of an
                                  execute too -- starts at the previous stage's end event and no
                                  event marker enters the stream (the stop events ride on the
                                  kernel dispatches themselves)                                 */
#define NW_NO_CHIRP      0x400u/* auto engine: keep the rocFFT engine for lengths the chirp-z fused
                                  form would take (non-power-of-two n, 2n-1 <= 16384 fp32 /
                                  8192 fp64, and n < 1024; up to n < 16384 / 8192 when every
                                  wavelet row's support K fits n + K - 1 <= 16384 / 8192)      */
#define NW_NO_DEDUP      0x200u/* compute every scale row even when wavelet rows repeat (by
                                  default rows with identical W -- Shannon ignores f
                                  (wavelets.py:256-262), repeated freqs -- are computed once
                                  and copied: bit-identical output, nw_stats.unique_rows)      */

/* execute outputs */
#define NW_OUT_CWT   0   /* complex (S, F, N)   base.py:378-407 */
#define NW_OUT_ABS   1   /* real    (S, F, N)   base.py:427-443 */
#define NW_OUT_POWER 2   /* real    (S, F, N)   base.py:409-425 */
/* Reductions over the nsig signals (EpochsWavelet, mneutils.py:42-71): out is (F, N),
 * summed in signal order in fp64 on the device; (E, F, N) is never materialised. */
#define NW_OUT_POWER_MEAN 3  /* real (F, N), compute dtype: mean_s |y|^2    mneutils.py:42-55 */
#define NW_OUT_ITC        4  /* real (F, N), compute dtype: |mean_s y/|y||  mneutils.py:57-71;
                                |y| = 0 gives NaN, as 0/0 does in the reference */
#define NW_OUT_POWER_SUM  5  /* float64 (F, N): sum_s |y|^2 (partial sums to combine over
                                devices or ranks, then divide by the total count) */
#define NW_OUT_PHASE_SUM  6  /* complex128 (F, N): sum_s y/|y| (partial sums; ITC = |sum/S|) */

/* memory placement of x / out in nw_execute */
#define NW_MEM_HOST   0
#define NW_MEM_DEVICE 1

/* Analytic-spectrum grid of one cache build (base.py:173-194, 238-246, 274-276):
 *   nu_j = j * delta for j < len_valid, and zero for len_valid <= j < len_full.
 * delta = 1/(n/sfreq); len_full is the row length of the reference's cached
 * wavelet (len(np.arange(...)), doubled by the hstack when interpolating). */
typedef struct nw_grid {
    double  delta;
    int64_t len_full;
    int64_t len_valid;
} nw_grid;

/* Per-stage device time accumulated since the plan was created or reset. */
typedef struct nw_stats {
    int64_t executes;       /* nw_execute calls */
    int64_t chunks;         /* device chunks run */
    double  ms_forward;     /* rocFFT forward (R2C) */
    double  ms_multiply;    /* K1 spectrum multiply (rocFFT engine) */
    double  ms_inverse;     /* rocFFT inverse (rocFFT engine) */
    double  ms_epilogue;    /* K2 |.| / |.|^2 (rocFFT engine) */
    double  ms_fused;       /* fused multiply + inverse FFT + epilogue (fused engine) */
    double  ms_copy;        /* copies (host<->device, input staging, spectrum transposes) */
    int64_t launches_multiply;
    int64_t launches_fused;
    int64_t engine;         /* NW_ENGINE_ROCFFT or NW_ENGINE_FUSED actually used */
    double  ms_rows;        /* fused engine, n > 16384: pass-1 row FFTs (ms_fused then times
                               pass 2, the column FFTs + epilogue; the spectrum transpose is
                               timed in ms_copy) */
    int64_t launches_rows;
    double  ms_expand;      /* repeated rows: copies of the computed unique rows */
    int64_t launches_expand;
    int64_t unique_rows;    /* scale rows actually computed (nfreq unless rows repeat) */
    int64_t kernel;         /* NW_K_*: the output-writing kernel of the last chunk */
    int64_t device_bytes;   /* device memory the plan holds now: input / spectrum / output /
                               reduction buffers, wavelet tables, two-pass scratch, rocFFT work
                               (it grows as calls need larger buffers; the Python classes
                               bound their plan cache by it) */
} nw_stats;

/* nw_stats.kernel: which kernel wrote the output rows (the dominant kernel of a step) */
#define NW_K_NONE        0
#define NW_K_FUSED       1   /* nw_fused_kernel (one pass, one signal per lane value)        */
#define NW_K_FUSED_PAIR  2   /* nw_fused_pair_kernel (one pass, two signals per lane value)  */
#define NW_K_CHIRP       3   /* nw_chirp_kernel (chirp-z form)                               */
#define NW_K_TWO_PASS    4   /* rows_kernel + cols_kernel (n > 16384; cols writes the output) */
#define NW_K_MULTIPLY    5   /* k1_multiply + rocFFT inverse (+ k2_epilogue): rocFFT engine   */

typedef struct nw_plan nw_plan;

const char* nw_last_error(void);
const char* nw_version(void);
/* Diagnostics on stderr ("[ninwave] ..." lines): 0 silent, 1 plan / engine / reduction-path
 * decisions and every error status, 2 also every launch stage (and its time under NW_TIMING).
 * Default: the NW_LOG environment variable, else 0.  Returns the previous level. */
int nw_set_log_level(int level);
/* 1 in the debug library (libninwave_debug.so: kernel bounds checks, every call synchronous,
 * NW_E_BOUNDS names the failing file:line), 0 in the product library. */
int nw_debug_bounds(void);
/* Debug library: launches one kernel whose checks fail on purpose (no memory is touched) and
 * returns the resulting NW_E_BOUNDS status; the product library returns NW_E_STATE. */
int nw_debug_selftest(int device);
int nw_device_count(int* n);

/* Host-only (no GPU): the grid of the reference's make_fft_wavelet(freq, real_length)
 * -- cwt passes real_length = n / sfreq (base.py:395).  Replaces _setup_trans_shape
 * (base.py:173-194) as called from base.py:238-245. */
int nw_trans_grid(double real_length, double sfreq, int interpolate, nw_grid* grid);

/* Host-only (no GPU): whether the fused engine supports (n, dtype): power-of-two n with
 * 1024 <= n <= 16384 in one on-chip pass, or 2^15 <= n <= 2^24 in its two-pass form (row
 * FFTs of W*X, then column FFTs + epilogue); fp32 and fp64 alike. */
int nw_fused_supported(int64_t n, int dtype);

/* Create a plan for signals of n samples, up to max_batch signals per device
 * chunk, nfreq scales.  flags: NW_INTERPOLATE | NW_ENGINE_* | NW_TIMING. */
int nw_plan_create(nw_plan** plan, int device, int64_t n, int64_t max_batch,
                   int32_t nfreq, int dtype, uint32_t flags);

/* Attach the wavelet (the reference's cached fft_wavelets, base.py:258-279).
 *   freqs[nfreq]: scale frequencies; grid: the cache-build grid (nw_trans_grid of
 *   the build length -- it may differ from the plan's n: base.py:394-397 reuses
 *   the cache and pad_to's it to the current n).
 *   params: NW_MORSE {b, r}; NW_MORLET {sigma, gabor[, c, k]} (c, k of wavelets.py:118-122,
 *   derived from sigma when absent); NW_SHANNON {}; NW_TABLE {}.
 *   table: NW_TABLE only, complex128 [nfreq][grid.len_full], copied to the device.
 *   row_len: NW_TABLE only, optional [nfreq] true length of each row (rows are
 *   left-aligned in the table); the reference pad_to's every row on its own
 *   (base.py:396-397) and time-domain rows can differ by one sample.  NULL: all
 *   rows are grid.len_full long. */
int nw_plan_set_wavelet(nw_plan* plan, int kind, const double* params, int nparams,
                        const double* freqs, const nw_grid* grid, const void* table,
                        const int64_t* row_len);

/* Shape of the attached wavelet's cached rows: len_full (the table width; for the
 * device-built NW_MEXICAN_HAT / NW_HAAR tables the longest row) and, if row_len is not
 * NULL, each row's true length [nfreq] (ragged Normal-mode rows, base.py:253-254). */
int nw_plan_wavelet_shape(nw_plan* plan, int64_t* len_full, int64_t* row_len);

/* Evaluate the attached wavelet rows on the device and copy them to the host:
 * out[nfreq][len_full] of the plan dtype (real for analytic kinds, complex for the
 * table kinds) -- the reference's self.fft_wavelets. */
int nw_plan_wavelet_rows(nw_plan* plan, void* out_host);

/* Diagnostic: the W-row support the two-pass engine (2^15 <= n <= 2^24) prunes its row pass
 * to -- kmax_out[nfreq] = the last bin k whose |W_f[k]| exceeds the tail threshold (2^-72 fp64,
 * 2^-56 fp32, of the row's max |W|; -1 for an all-zero row) of every scale of the plan.  method
 * 0: as the engine builds it (no full scan for Morse / Morlet / Shannon rows), 1: by scanning every bin
 * (the reference the tests compare method 0 with).  No reference counterpart: the reference
 * multiplies every bin (base.py:404-406); the cut bins together move y by < n * 2^-72 (fp64)
 * of the signal's scale.  NW_E_STATE for plans on another engine. */
int nw_plan_row_support(nw_plan* plan, int method, int32_t* kmax_out);

/* Run the CWT of nsig signals x[nsig][n] (plan dtype) into out[nsig][nfreq][n]
 * (complex for NW_OUT_CWT, real otherwise), or (F, N) for the reduction kinds
 * NW_OUT_POWER_MEAN .. NW_OUT_PHASE_SUM.  mem = NW_MEM_HOST: synchronous;
 * NW_MEM_DEVICE: x/out are device pointers on the plan's device, the call is
 * asynchronous on the plan stream (see nw_plan_sync). */
int nw_execute(nw_plan* plan, const void* x, int64_t nsig, void* out, int out_kind, int mem);

/* Shard nsig host signals over nplans plans (one per device, identical config),
 * one host thread per plan; balanced contiguous blocks (nsig / nplans signals, one
 * more for the first nsig % nplans plans).  A plan is not reentrant, so a plan
 * pointer may appear only once (NW_E_INVALID otherwise; two plans on one device are
 * fine).  For the reduction kinds each device sums its block and the host adds the
 * fp64 partial sums in device order before the mean / |.| of the result.
 * Replaces the serial per-epoch loop of EpochsWavelet.cwt (mneutils.py:39). */
int nw_execute_multi(nw_plan* const* plans, int nplans, const void* x, int64_t nsig,
                     void* out, int out_kind);

/* Device-resident sharding (one process, one host thread per device, no
 * PCIe): plan i transforms nsig[i] signals x[i] -- a DEVICE pointer on plan i's
 * device -- into out[i] (device pointer, same device, (nsig[i], F, n)).  Returns when
 * every device has finished.  Reduction kinds: each device sums its block in fp64,
 * device 0 gathers the partial sums peer-to-peer, adds them in device order and
 * writes the (F, n) result to out[0] (out[i > 0] unused).  Plans must be distinct and
 * share n, nfreq and dtype. */
int nw_execute_multi_device(nw_plan* const* plans, int nplans, const void* const* x,
                            const int64_t* nsig, void* const* out, int out_kind);

/* Shard the SCALES instead (one long signal, e.g. C5, cannot shard by
 * signal): plan i (its own device, same n / dtype / flags) holds the i-th contiguous
 * slice of the scale list, nfreq_i scales, sum nfreq_i = F.  Every device transforms all
 * nsig host signals for its scales (its own forward FFT: ~0.2 ms at 2^24, cheaper than a
 * broadcast) and writes its rows of out (nsig, F, n) -- or (F, n) for the reduction
 * kinds -- in place; no exchange.  Meant for nsig below the device count (the host
 * output is written one signal at a time). */
int nw_execute_multi_scales(nw_plan* const* plans, int nplans, const void* x, int64_t nsig,
                            void* out, int out_kind);

/* Baseline correction (base.py:18-68: class Baseline; baseline_of at 18-20) of a real
 * array x[count] (dtype NW_F32 / NW_F64).  The reference slices AXIS 0: for an array
 * whose rows hold row_len elements the baseline is rows [row0, row1) (already
 * normalised like a Python slice), i.e. the contiguous elements [row0*row_len,
 * row1*row_len).  basemean = its mean and std = its population std (np.std), both over
 * all of its elements, are reduced on the device in fp64; then out[i] = op(x[i]) in the
 * array's precision:
 *   NW_BL_MEAN    x - basemean                 (base.py:53-54)
 *   NW_BL_RATIO   x / basemean                 (56-57)
 *   NW_BL_PERCENT (x - basemean) / basemean    (59-60)
 *   NW_BL_LOG     log10(x / basemean)          (62-63)
 *   NW_BL_ZSCORE  (x - basemean) / std         (65-66)
 *   NW_BL_ZLOG    log10(x / basemean) / std    (68-69)
 * mem = NW_MEM_HOST (synchronous) or NW_MEM_DEVICE (pointers on `device`, synchronous
 * on the device's null stream).  stats (optional, host) receives {basemean, std}.
 * An empty baseline gives NaN statistics, like numpy. */
#define NW_BL_MEAN    0
#define NW_BL_RATIO   1
#define NW_BL_PERCENT 2
#define NW_BL_LOG     3
#define NW_BL_ZSCORE  4
#define NW_BL_ZLOG    5
int nw_baseline(int device, int dtype, const void* x, int64_t count, int64_t row_len, int64_t row0,
                int64_t row1, int op, void* out, int mem, double* stats);

/* Time-domain wavelets of the stock kinds, make_wavelet(s) (base.py:346-376), computed on
 * `device`: one row per freq, complex128, left-aligned in out[nfreq][*max_len] (host).
 *   NW_MORSE {b, r}, NW_SHANNON {}  (WaveletMode.Reverse): ifft of the spectrum (its
 *     default freq = 1) on np.arange(0, sfreq/f*real_wave_length, 1/f), then the centre
 *     slice [m//2, m//2*3) of hstack(conj(flip(w)), w)  -> 2*(m//2) points;
 *   NW_MORLET {sigma, gabor[, c, k]}, NW_MEXICAN_HAT {sigma}, NW_HAAR {}: the time-domain
 *     formula on np.arange(-T/2, T/2, step) of _setup_waveletshape (base.py:196-216).
 * row_len[nfreq] receives each row's length.  out == NULL: lengths only (to size out). */
int nw_make_wavelets(int device, int kind, const double* params, int nparams, const double* freqs, int nfreq,
                     double sfreq, double real_wave_length, void* out, int64_t* max_len, int64_t* row_len);

/* Page-locked host memory for results (no reference counterpart: the drop-in classes pool
 * their result arrays in it, ninwavelets_amd/engine.py HostPool).  nw_execute with
 * NW_MEM_HOST writes an output that lies inside such an allocation by DMA directly, without
 * the staging copy; a fresh pageable array instead is faulted in page by page during the
 * copy-out.  nw_host_free takes exactly a pointer nw_host_alloc returned. */
int nw_host_alloc(int64_t bytes, void** ptr);
int nw_host_free(void* ptr);
/* Advise a pageable host buffer the CALLER has just allocated for a result onto transparent
 * huge pages (madvise MADV_HUGEPAGE over its whole 2 MiB pages; no reference counterpart:
 * the drop-in classes call it for the fresh arrays they return when the page-locked pool is
 * full, ninwavelets_amd/engine.py).  A fresh array is then faulted in 2 MiB at a time during
 * the copy-out instead of 4 KiB.  nw_execute never changes the page policy of the memory it
 * is handed.  *advised (may be NULL) receives the bytes advised (0 below one huge page). */
int nw_host_advise(void* ptr, int64_t bytes, int64_t* advised);

int nw_plan_set_stream(nw_plan* plan, void* hip_stream);   /* NULL: the plan's own stream */
/* The hipStream_t the plan currently launches on (for event ordering with the caller's
 * streams: device-buffer executes are asynchronous on it). */
int nw_plan_get_stream(nw_plan* plan, void** hip_stream);
int nw_plan_sync(nw_plan* plan);
int nw_plan_stats(nw_plan* plan, nw_stats* stats);
int nw_plan_reset_stats(nw_plan* plan);
int nw_plan_destroy(nw_plan* plan);

#ifdef __cplusplus
}
#endif
#endif /* NINWAVE_H */
