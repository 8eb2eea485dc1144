// CPU driver for the sanitizer build of the engine's host-only logic (nw_host.cpp):
// built with -fsanitize=address,undefined by tests/test_host_asan.py.
//   host_asan self      : invariant checks of group_rows / block_of / parallel_copy / advise_output /
//                         normal_rows
//   host_asan grid      : stdin "real_length sfreq interpolate" -> "len_valid len_full delta"
#include <cstdio>
#include <functional>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../ninwavelets_amd/csrc/nw_host.h"

using namespace nw::host;

static int g_fail = 0;
#define CHECK(c)                                                            \
    do {                                                                    \
        if (!(c)) {                                                         \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                       \
        }                                                                   \
    } while (0)

// brute-force equality of rows f and g under group_rows' rules
static bool rows_equal(const std::vector<double>& tab, int64_t L, const std::vector<int64_t>* rl, int f, int g) {
    const int64_t lf = rl ? (*rl)[f] : L, lg = rl ? (*rl)[g] : L;
    return lf == lg && std::memcmp(&tab[(size_t)f * L * 2], &tab[(size_t)g * L * 2], (size_t)lf * 16) == 0;
}

static void check_groups(const RowGroups& g, int F, const std::function<bool(int, int)>& eq) {
    CHECK((int)g.rep.size() == F);
    const int U = (int)g.uniq.size();
    CHECK((int)g.packed.size() == U + 1 + F);
    for (int f = 0; f < F; ++f) {
        int first = f;
        for (int h = 0; h < f; ++h)
            if (eq(h, f)) { first = h; break; }
        CHECK(g.rep[f] == first);
    }
    std::vector<int> seen(F, 0);
    CHECK(g.packed[0] == 0 && g.packed[U] == F);
    for (int u = 0; u < U; ++u)
        for (int i = g.packed[u]; i < g.packed[u + 1]; ++i) {
            const int f = g.packed[U + 1 + i];
            CHECK(f >= 0 && f < F);
            if (f < 0 || f >= F) continue;
            seen[f]++;
            CHECK(g.rep[f] == g.uniq[u]);
        }
    for (int f = 0; f < F; ++f) CHECK(seen[f] == 1);
}

static void self_checks() {
    std::mt19937_64 rng(7);
    // group_rows: user tables with repeats and ragged rows
    for (int trial = 0; trial < 200; ++trial) {
        const int F = (int)(rng() % 40);
        const int64_t L = 1 + (int64_t)(rng() % 33);
        std::vector<double> tab((size_t)F * L * 2 + 1);
        std::vector<int64_t> rl(F);
        const int distinct = 1 + (int)(rng() % 5);
        for (int f = 0; f < F; ++f) {
            const int pick = (int)(rng() % distinct);
            rl[f] = 1 + (pick * 7) % L;
            for (int64_t i = 0; i < L * 2; ++i) tab[(size_t)f * L * 2 + i] = (i < rl[f] * 2) ? pick * 1.5 + i : 0.0;
        }
        const bool ragged = trial & 1;
        RowGroups g = group_rows(false, F, nullptr, tab.data(), L, ragged ? rl.data() : nullptr);
        check_groups(g, F, [&](int a, int b) { return rows_equal(tab, L, ragged ? &rl : nullptr, a, b); });
        // freq-keyed rows (analytic kinds) with repeated values, and Shannon
        std::vector<double> fr(F);
        for (int f = 0; f < F; ++f) fr[f] = 0.5 * (double)(rng() % 6);
        RowGroups h = group_rows(false, F, fr.data(), nullptr, L, nullptr);
        check_groups(h, F, [&](int a, int b) { return std::memcmp(&fr[a], &fr[b], 8) == 0; });
        if (F > 0) {
            RowGroups s = group_rows(true, F, fr.data(), nullptr, L, nullptr);
            check_groups(s, F, [](int, int) { return true; });
            CHECK(s.uniq.size() == 1);
        }
    }
    // -0.0 and 0.0 are different bits: different rows (the engine keys on bits)
    {
        const double fr[2] = {0.0, -0.0};
        CHECK(group_rows(false, 2, fr, nullptr, 4, nullptr).uniq.size() == 2);
    }
    // block_of: a partition into balanced contiguous blocks
    for (int64_t nsig = 0; nsig < 200; ++nsig)
        for (int n = 1; n < 12; ++n) {
            int64_t next = 0;
            for (int i = 0; i < n; ++i) {
                int64_t s0, cnt;
                block_of(nsig, i, n, &s0, &cnt);
                CHECK(s0 == next && cnt >= nsig / n && cnt <= nsig / n + 1);
                next = s0 + cnt;
            }
            CHECK(next == nsig);
        }
    // parallel_copy at odd sizes and thread counts
    const size_t sizes[] = {0, 1, 7, (size_t(4) << 20) - 1, (size_t(4) << 20) + 3, (size_t(33) << 20) + 5};
    for (size_t bytes : sizes)
        for (unsigned th : {0u, 1u, 3u, 8u, 64u}) {
            std::vector<char> src(bytes + 1), dst(bytes + 1, 0);
            for (size_t i = 0; i < bytes; ++i) src[i] = (char)(i * 131 + th);
            parallel_copy(dst.data(), src.data(), bytes, th);
            CHECK(std::memcmp(dst.data(), src.data(), bytes) == 0);
        }
    // advise_output: contents kept, whole range writable afterwards, odd bounds and sizes
    for (size_t bytes : {size_t(0), size_t(100), (size_t(2) << 20) - 1, (size_t(37) << 20) + 11,
                         (size_t(130) << 20) + 4097}) {
        std::vector<char> buf(bytes + 64);
        char* dst = buf.data() + 5;                      // not page aligned
        for (size_t i = 0; i < bytes; i += 4093) dst[i] = (char)(i * 7);
        const size_t adv = advise_output(dst, bytes);
        CHECK(adv <= bytes && adv % (size_t(2) << 20) == 0);
        CHECK(bytes >= (size_t(4) << 20) || adv <= (size_t(2) << 20));
        for (size_t i = 0; i < bytes; i += 4093) CHECK(dst[i] == (char)(i * 7));
        std::memset(dst, 1, bytes);
    }
    // normal_rows: offsets tile the batched buffer, rows of equal length consecutive
    for (int mh = 0; mh < 2; ++mh) {
        const double params[3] = {7.0, 1000.0, 1.0};
        std::vector<double> fr = {1., 2., 3., 5., 2., 40., 80., 160.};
        std::vector<nw::NormalRow> rows;
        int64_t lmax = 0, total = 0;
        double sigma = -1;
        const bool ok = normal_rows(mh == 1, params + (mh ? 0 : 1), mh ? 3 : 2, fr.data(), (int)fr.size(), rows,
                                    &lmax, &total, &sigma);
        CHECK(ok);
        int64_t sum = 0;
        for (auto& r : rows) {
            CHECK(r.len == r.m + 2 * r.half && r.half >= 0 && r.len <= lmax);
            CHECK(r.off >= 0 && r.off + r.len <= total);
            sum += r.len;
        }
        CHECK(sum == total);
        // a wavelet longer than sfreq * real_wave_length: negative padding is refused
        const double tiny[3] = {7.0, 10.0, 0.01};
        CHECK(!normal_rows(mh == 1, tiny + (mh ? 0 : 1), mh ? 3 : 2, fr.data(), (int)fr.size(), rows, &lmax, &total,
                           &sigma));
    }
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "self";
    if (mode == "grid") {
        double rl, sf;
        int interp;
        while (std::scanf("%lf %lf %d", &rl, &sf, &interp) == 3) {
            double d;
            int64_t lv, lf;
            trans_grid(rl, sf, interp != 0, &d, &lv, &lf);
            std::printf("%lld %lld %.17g\n", (long long)lv, (long long)lf, d);
        }
        return 0;
    }
    self_checks();
    std::printf("%s\n", g_fail ? "FAIL" : "ok");
    return g_fail ? 1 : 0;
}
