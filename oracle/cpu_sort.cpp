// oracle/cpu_sort.cpp -- TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline).
//
// The specification oracle for the sort path.  The reference's order_array is
// specified as "sort the int array ascending" (letra.pdf p.3, "Consigna";
// lab.h:9), and its comparator order_with_trust is thrust::sort on host
// pointers (lab.cu:404-406), i.e. a sequential host sort.  A
// keys-only ascending sort has exactly one correct output, so std::sort is a
// complete oracle for both entry points.
//
// Also holds the counter-based input generator: the product has
// its own device implementation of the same formula, and the tests check that
// the two agree word for word.
//
// Pinning: parity unpinned by reference artifacts (the reference has no tests or
// golden outputs and its CUDA source cannot be built here); see oracle/oracle.py.
//
// Build: oracle/Makefile -> oracle/liboracle.so (gcc, -fopenmp for the
// __gnu_parallel baseline).
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <parallel/algorithm>
#include <omp.h>
#include <vector>

extern "C" {

// ---- generator: key[i] = f(splitmix64(seed ^ (i * golden))) -------------------
static inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// dist codes shared with the product's device generator (include/labsort.h)
enum {
    DIST_U32 = 0,      // uniform on [0, 2^32)
    DIST_U31 = 1,      // uniform on [0, 2^31): the reference's valid int domain
    DIST_MOD100 = 2,   // like rand()%100  (main.cpp:10)
    DIST_MOD1000 = 3,  // like rand()%1000 (performanceTest.cpp:35)
    DIST_SORTED = 4,   // i
    DIST_REVERSED = 5, // n-1-i  (needs the global n: passed as `param`)
    DIST_CONST = 6,    // every key equal to `param`
    DIST_LOWBITS = 7,  // uniform on [0, 2^param)
};

static inline uint32_t gen_one(uint64_t seed, uint64_t i, int dist, uint64_t param) {
    uint64_t z = mix64(seed ^ (i * 0x9E3779B97F4A7C15ull));
    uint32_t hi = (uint32_t)(z >> 32);
    switch (dist) {
    case DIST_U32: return hi;
    case DIST_U31: return (uint32_t)(z >> 33);
    case DIST_MOD100: return hi % 100u;
    case DIST_MOD1000: return hi % 1000u;
    case DIST_SORTED: return (uint32_t)i;
    case DIST_REVERSED: return (uint32_t)(param - 1 - i);
    case DIST_CONST: return (uint32_t)param;
    case DIST_LOWBITS: return param >= 32 ? hi : (hi & (uint32_t)((1ull << param) - 1));
    default: return hi;
    }
}

// fills out[0..n) with keys first..first+n of the stream (first lets a rank
// generate its own shard of a global array)
void oracle_fill(uint32_t *out, uint64_t n, uint64_t seed, int dist, uint64_t param, uint64_t first) {
#pragma omp parallel for schedule(static) if (n > (1u << 20))
    for (int64_t i = 0; i < (int64_t)n; ++i) out[i] = gen_one(seed, first + (uint64_t)i, dist, param);
}

// ---- sort oracles -----------------------------------------------------------------
void oracle_sort_u32(uint32_t *a, uint64_t n) { std::sort(a, a + n); }
void oracle_sort_i32(int32_t *a, uint64_t n) { std::sort(a, a + n); }

void oracle_par_sort_u32(uint32_t *a, uint64_t n, int threads) {
    omp_set_num_threads(threads);
    __gnu_parallel::sort(a, a + n);
}

int oracle_is_sorted_u32(const uint32_t *a, uint64_t n) { return std::is_sorted(a, a + n) ? 1 : 0; }
int oracle_is_sorted_i32(const int32_t *a, uint64_t n) { return std::is_sorted(a, a + n) ? 1 : 0; }

// Key/value oracle (sort_by_key): std::stable_sort of (key, payload) pairs
// by key in u32 (flip = 0) or i32 (flip = 0x80000000) order; equal keys keep input order.
void oracle_stable_sort_pairs(uint32_t *keys, uint32_t *vals, uint64_t n, uint32_t flip) {
    std::vector<uint64_t> idx(n);
    for (uint64_t i = 0; i < n; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](uint64_t x, uint64_t y) { return (keys[x] ^ flip) < (keys[y] ^ flip); });
    std::vector<uint32_t> k(n), v(n);
    for (uint64_t i = 0; i < n; ++i) {
        k[i] = keys[idx[i]];
        v[i] = vals[idx[i]];
    }
    std::memcpy(keys, k.data(), n * 4);
    std::memcpy(vals, v.data(), n * 4);
}

// Merge-split oracle for the multi-GPU exchange step: the lower (keep_low=1)
// or upper half of merge(A, B) with A-before-B on ties (lab.cu:163-170 rule).
void oracle_merge_split_u32(const uint32_t *a, uint64_t la, const uint32_t *b, uint64_t lb, uint32_t *out,
                            uint64_t lo_diag, uint64_t hi_diag) {
    uint64_t i = 0, j = 0, d = 0;
    while (d < hi_diag) {
        uint32_t v;
        if (j >= lb || (i < la && a[i] <= b[j])) v = a[i++];
        else v = b[j++];
        if (d >= lo_diag) out[d - lo_diag] = v;
        ++d;
    }
}

// Times std::sort (threads == 1) or __gnu_parallel::sort on a private copy of
// `keys`; returns seconds for `reps` sorts (each on a fresh copy, copy untimed).
double oracle_time_sort_u32(const uint32_t *keys, uint64_t n, int threads, int reps, uint32_t *scratch) {
    double total = 0.0;
    for (int r = 0; r < reps; ++r) {
        std::memcpy(scratch, keys, n * sizeof(uint32_t));
        auto t0 = std::chrono::steady_clock::now();
        if (threads <= 1) std::sort(scratch, scratch + n);
        else {
            omp_set_num_threads(threads);
            __gnu_parallel::sort(scratch, scratch + n);
        }
        auto t1 = std::chrono::steady_clock::now();
        total += std::chrono::duration<double>(t1 - t0).count();
    }
    return total;
}

} // extern "C"
