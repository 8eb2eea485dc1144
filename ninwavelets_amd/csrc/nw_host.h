// nw_host.h — the host-only logic of the C ABI (no HIP calls): numpy-exact grid lengths,
// the Normal-mode row timelines, distinct-row grouping, signal blocks and the pinned
// copy-out.  Built into libninwave.so and, with -fsanitize=address,undefined, into the
// CPU test driver tests/asan/host_asan.cpp (sanitizer build of the host path).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace nw {

// One WaveletMode.Normal row (base.py:196-216, 249-256): an np.arange timeline
// t0, t0 + delta, ... of m points, zero-padded by `half` per side to `len`, at `off`
// in the batched transform buffer.
struct NormalRow {
    int64_t off, m, half, len;
    double t0, t1, delta;
};

namespace host {

// len(np.arange(0, stop, step)) for Python floats: ceil(stop / step) (numpy _calc_length)
int64_t arange_len(double stop, double step);
// len(np.arange(start, stop, step))
int64_t arange_len_from(double start, double stop, double step);

// _setup_trans_shape's grid for make_fft_wavelet (base.py:173-194, 238-245):
// spacing 1 / real_length, numpy's row length, doubled when interpolating.
void trans_grid(double real_length, double sfreq, bool interpolate, double* delta, int64_t* len_valid,
                int64_t* len_full);

// Timelines of the Normal-mode rows (MexicanHat / Haar, wavelets.py:194-228, 272-280):
// rows[f] for every freq, rows of equal length consecutive (off), sigma out.
// Returns false on a negative padding (np.zeros of a negative size in the reference).
bool normal_rows(bool mexican_hat, const double* params, int nparams, const double* freqs, int F,
                 std::vector<NormalRow>& rows, int64_t* lmax, int64_t* total, double* sigma);

// Distinct wavelet rows (nw_plan::dedup).  shannon: every row equal.  table (may be null):
// complex128 rows of stride L, row f of true length row_len[f] (row_len may be null: L),
// equal iff equal length and contents.  Otherwise rows are equal iff their freqs are
// bitwise equal.  rep[f] = first scale with f's row; uniq = first scale of each distinct
// row in order; packed = offs[0..U] followed by the scales grouped by distinct row.
struct RowGroups {
    std::vector<int> rep, uniq;
    std::vector<int32_t> packed;
};
RowGroups group_rows(bool shannon, int F, const double* freqs, const double* table, int64_t L,
                     const int64_t* row_len);

// Balanced contiguous blocks: nsig / n per part, one more for the first nsig % n parts.
void block_of(int64_t nsig, int i, int n, int64_t* s0, int64_t* cnt);

// memcpy split over up to max_threads host threads (>= 4 MiB per thread).
void parallel_copy(char* dst, const char* src, size_t bytes, unsigned max_threads);

// Ask for transparent huge pages on the 2-MiB-aligned interior of a host output range before
// the copy-out writes it (MADV_HUGEPAGE; a no-op where THP is off).  A fresh numpy array is
// untouched anonymous memory: faulted 4 KiB at a time inside the copy-out (and unmapped page by
// page when the caller drops it) it bounded the reference-style fresh-array path at 1/3 of the
// PCIe rate.  Measured on 1 GiB (8 threads): copy with faults 10 -> 13-17 GB/s, munmap 30-50 ->
// 3 ms; populating ahead (MADV_POPULATE_WRITE) was slower than faulting inside the copy.
// Returns the advised bytes (0: range below one huge page).
size_t advise_output(char* dst, size_t bytes);
// Whether some bin x = j * delta / f (j < len_valid) of a Morse plan comes within 2^24 of the
// fp64 overflow of the reference's x^b (or its exp term: b/r > 709): the rows then take the
// overflow-checked forms, which reproduce the reference's inf / NaN (wavelets.py:65-74)
bool morse_may_overflow(double b, double r, double delta, int64_t len_valid, const double* freqs, int nfreq);

}  // namespace host
}  // namespace nw
