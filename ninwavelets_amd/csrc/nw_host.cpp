// nw_host.cpp — host-only logic of the C ABI (see nw_host.h); no HIP calls.
#include "nw_host.h"

#include <sys/mman.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <thread>
#include <unordered_map>

namespace nw {
namespace host {

int64_t arange_len(double stop, double step) {
    const double q = stop / step;
    if (q == 0.0 && stop != 0.0) return std::signbit(q) ? 0 : 1;
    if (!(q > 0.0)) return 0;
    return (int64_t)std::ceil(q);
}

int64_t arange_len_from(double start, double stop, double step) {
    const double q = (stop - start) / step;
    if (!(q > 0.0)) return 0;
    return (int64_t)std::ceil(q);
}

void trans_grid(double real_length, double sfreq, bool interpolate, double* delta, int64_t* len_valid,
                int64_t* len_full) {
    // make_fft_wavelet(freq, real_length) -> _setup_trans_shape(real_length, rl'):
    //   one = 1 / real_length; total = sfreq / real_length * rl'   (base.py:191-194, 238-245)
    const double rl = real_length;
    const double one = 1.0 / rl;
    const double rwl = interpolate ? rl / 2.0 : rl;
    const double total = sfreq / rl * rwl;
    const int64_t len = arange_len(total, one);
    *delta = one;
    *len_valid = len;
    *len_full = interpolate ? 2 * len : len;   // hstack with zeros(len(t)) (base.py:241-242)
}

bool normal_rows(bool mexican_hat, const double* params, int nparams, const double* freqs, int F,
                 std::vector<NormalRow>& rows, int64_t* lmax_out, int64_t* total_out, double* sigma_out) {
    const double sigma = mexican_hat ? (nparams > 0 ? params[0] : 7.0) : 0.0;
    const int o = mexican_hat ? 1 : 0;
    const double sfreq = nparams > o ? params[o] : 1000.0;
    const double rwl = nparams > o + 1 ? params[o + 1] : 1.0;
    const double peak = mexican_hat ? std::sqrt(6.0) / M_PI / M_PI : 1.0;   // wavelets.py:227-228
    rows.assign(F, NormalRow{});
    std::map<int64_t, std::vector<int>> by_len;
    int64_t lmax = 0;
    for (int f = 0; f < F; ++f) {
        const double fr = freqs[f];
        const double total = 1.0 / peak * fr * 2.0 * M_PI;
        const double one = 1.0 / sfreq * 2.0 * M_PI * fr / peak;
        const double t0 = -total / 2.0, stop = total / 2.0;
        const int64_t m = arange_len_from(t0, stop, one);
        const int64_t half = (int64_t)((sfreq * rwl - (double)m) / 2.0);
        if (half < 0) return false;
        NormalRow& r = rows[f];
        r.m = m;
        r.half = half;
        r.len = m + 2 * half;
        r.t0 = t0;
        r.t1 = t0 + one;
        r.delta = r.t1 - t0;
        by_len[r.len].push_back(f);
        lmax = std::max(lmax, r.len);
    }
    int64_t off = 0;
    for (auto& kv : by_len)
        for (int f : kv.second) {
            rows[f].off = off;
            off += kv.first;
        }
    *lmax_out = lmax;
    *total_out = off;
    *sigma_out = sigma;
    return true;
}

RowGroups group_rows(bool shannon, int F, const double* freqs, const double* table, int64_t L,
                     const int64_t* row_len) {
    RowGroups g;
    g.rep.assign(F, 0);
    if (F <= 0) {
        g.packed.assign(1, 0);
        return g;
    }
    if (shannon) {
        g.uniq.push_back(0);
    } else if (table) {
        // user rows: equal length and equal contents (FNV-1a over 8-byte words, then compare)
        std::unordered_map<uint64_t, std::vector<int>> seen;
        for (int f = 0; f < F; ++f) {
            const int64_t len = row_len ? row_len[f] : L;
            const unsigned char* b = (const unsigned char*)(table + (size_t)f * L * 2);
            uint64_t h = 1469598103934665603ull ^ (uint64_t)len;
            for (size_t i = 0; i < (size_t)len * 2; ++i) {
                uint64_t w;
                std::memcpy(&w, b + 8 * i, 8);
                h = (h ^ w) * 1099511628211ull;
            }
            int found = -1;
            for (int o : seen[h]) {
                const int64_t lo = row_len ? row_len[o] : L;
                if (lo == len && std::memcmp(b, table + (size_t)o * L * 2, (size_t)len * 16) == 0) {
                    found = o;
                    break;
                }
            }
            if (found < 0) {
                seen[h].push_back(f);
                g.uniq.push_back(f);
                g.rep[f] = f;
            } else {
                g.rep[f] = found;
            }
        }
    } else {
        // analytic kinds and Normal tables: a row is a function of its freq (bitwise)
        std::unordered_map<uint64_t, int> first;
        for (int f = 0; f < F; ++f) {
            uint64_t key;
            std::memcpy(&key, &freqs[f], sizeof(key));
            auto it = first.find(key);
            if (it == first.end()) {
                first.emplace(key, f);
                g.uniq.push_back(f);
                g.rep[f] = f;
            } else {
                g.rep[f] = it->second;
            }
        }
    }
    // scales grouped by distinct row: packed[u] .. packed[u + 1] index packed[U + 1 + ...]
    const int U = (int)g.uniq.size();
    std::vector<int> uidx(F, -1), counts(U, 0);
    for (int u = 0; u < U; ++u) uidx[g.uniq[u]] = u;
    for (int f = 0; f < F; ++f) counts[uidx[g.rep[f]]]++;
    g.packed.assign(U + 1 + F, 0);
    for (int u = 0; u < U; ++u) g.packed[u + 1] = g.packed[u] + counts[u];
    std::vector<int> fill(g.packed.begin(), g.packed.begin() + U);
    for (int f = 0; f < F; ++f) g.packed[U + 1 + fill[uidx[g.rep[f]]]++] = f;
    return g;
}

void block_of(int64_t nsig, int i, int n, int64_t* s0, int64_t* cnt) {
    const int64_t base = nsig / n, extra = nsig % n;
    *s0 = (int64_t)i * base + std::min<int64_t>(i, extra);
    *cnt = base + (i < extra ? 1 : 0);
}

void parallel_copy(char* dst, const char* src, size_t bytes, unsigned max_threads) {
    const size_t min_share = size_t(4) << 20;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nth = std::min<size_t>(std::min<size_t>(std::max(1u, max_threads), hw),
                                        std::max<size_t>(1, bytes / min_share));
    if (nth <= 1) {
        if (bytes) std::memcpy(dst, src, bytes);
        return;
    }
    const size_t share = (bytes + nth - 1) / nth;
    std::vector<std::thread> th;
    for (size_t i = 1; i < nth; ++i) {
        const size_t off = i * share;
        if (off >= bytes) break;
        th.emplace_back([=] { std::memcpy(dst + off, src + off, std::min(share, bytes - off)); });
    }
    std::memcpy(dst, src, std::min(share, bytes));
    for (auto& t : th) t.join();
}

bool morse_may_overflow(double b, double r, double delta, int64_t len_valid, const double* freqs, int nfreq) {
    if (r != 0.0 && b / r * 1.4426950408889634 >= 1000.0) return true;      // exp((b/r)(1 - x^r)) near x = 0
    double fmin = 0.0;
    for (int i = 0; i < nfreq; ++i)
        if (freqs[i] > 0.0 && (fmin == 0.0 || freqs[i] < fmin)) fmin = freqs[i];
    if (fmin == 0.0 || len_valid < 2 || b <= 0.0) return false;
    const double xmax = (double)(len_valid - 1) * delta / fmin;
    return xmax > 1.0 && b * std::log2(xmax) >= 1000.0;
}

size_t advise_output(char* dst, size_t bytes) {
    const size_t huge = size_t(2) << 20;
    const uintptr_t b = (uintptr_t)dst, e = b + bytes;
    const uintptr_t hb = (b + huge - 1) / huge * huge, he = e / huge * huge;
    if (bytes < huge || he <= hb) return 0;
    (void)madvise(reinterpret_cast<void*>(hb), he - hb, MADV_HUGEPAGE);
    return he - hb;
}

}  // namespace host
}  // namespace nw
