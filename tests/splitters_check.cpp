// Checker for dist::choose_splitters (csrc/dist_plan.h), compiled by tests/test_splitters.py:
// the selection over the p sorted sample runs must pick exactly the splitters that a stable
// sort of the pooled samples by (key, rank) picks -- pooled index j * N / p, N = samples of
// the non-empty shards -- on random rank counts, key distributions with heavy ties, both key
// orders, empty shards, and runs that are not sorted (the pooled-sort path).
#include <stdio.h>

#include <random>

#include "dist_plan.h"

using labsort::dist::Splitter;

static std::vector<Splitter> by_pool_sort(int p, const uint64_t *m, const uint32_t *smp, size_t s, uint32_t flip) {
    std::vector<Splitter> pool;
    for (int r = 0; r < p; ++r) {
        if (!m[r]) continue;
        for (size_t k = 0; k < s; ++k) {
            const uint32_t key = smp[(size_t)r * s + k];
            pool.push_back({key ^ flip, (uint32_t)r, (uint64_t)labsort::dist::sample_pos(m[r], s, k), key});
        }
    }
    std::stable_sort(pool.begin(), pool.end(), [](const Splitter &a, const Splitter &b) {
        return a.ord != b.ord ? a.ord < b.ord : a.rank < b.rank;
    });
    std::vector<Splitter> spl(p > 1 ? p - 1 : 0, Splitter{0u, 0u, 0u, 0u});
    if (pool.empty()) return spl;
    for (int j = 1; j < p; ++j) spl[j - 1] = pool[(size_t)j * pool.size() / p];
    return spl;
}

int main(int argc, char **argv) {
    const int cases = argc > 1 ? atoi(argv[1]) : 2000;
    std::mt19937_64 g(0x5A3F1E);
    int bad = 0, sel = 0;
    for (int c = 0; c < cases; ++c) {
        const int p = 1 + (int)(g() % 16);
        const size_t s = labsort::dist::samples_per_rank(p);
        const uint32_t flip = (g() & 1) ? 0x80000000u : 0u;
        const uint32_t mods[] = {0xFFFFFFFFu, 1u, 2u, 3u, 100u, 5000u};
        const uint32_t mod = mods[g() % 6];
        const bool unsorted_run = g() % 8 == 0;
        std::vector<uint64_t> m(p);
        std::vector<uint32_t> smp((size_t)p * s);
        for (int r = 0; r < p; ++r) {
            m[r] = g() % 6 == 0 ? 0 : 1 + g() % (1u << 20);
            uint32_t *x = &smp[(size_t)r * s];
            for (size_t k = 0; k < s; ++k) x[k] = ((uint32_t)(g() % ((uint64_t)mod + 1))) ^ flip;
            if (!(unsorted_run && r == p / 2))
                std::sort(x, x + s, [flip](uint32_t a, uint32_t b) { return (a ^ flip) < (b ^ flip); });
        }
        const auto a = labsort::dist::choose_splitters(p, m.data(), smp.data(), s, flip);
        const auto b = by_pool_sort(p, m.data(), smp.data(), s, flip);
        sel += !unsorted_run;
        bool ok = a.size() == b.size();
        for (size_t j = 0; ok && j < a.size(); ++j)
            ok = a[j].ord == b[j].ord && a[j].rank == b[j].rank && a[j].pos == b[j].pos && a[j].key == b[j].key;
        if (!ok && bad++ < 5) fprintf(stderr, "case %d: p=%d mod=%u flip=%x differs\n", c, p, mod, flip);
    }
    printf("cases %d selection %d mismatches %d\n", cases, sel, bad);
    return bad != 0;
}
