// dist_plan.h -- the multi-GPU merge-sort schedule, written ONCE and
// instantiated for every transport:
//   * csrc/multi.hip: HIP rank operations with RCCL (one process per GPU, or one host
//     thread per GPU), in-process peer copies, or host-staged callbacks (tests);
//   * oracle/dist_host.cpp (test infrastructure): host operations (std::sort,
//     std::upper_bound, std::merge) over the same host-staged callbacks, so the CPU
//     tests run this exact schedule over torch.distributed gloo.
// Host C++17 only (no HIP types): the rank operations and the communicator are
// template parameters.
//
// The reference is single-GPU (lab.cu:303-402); its stage 3 (separators_kernel
// lab.cu:209-270 + merge_segments_kernel lab.cu:272-300) is the model: splitters are
// taken every few hundred keys of each sorted run, each splitter's co-rank in the
// other runs is found by binary search (busquedaPorBiparticion lab.cu:102-132,
// here labsort_upper_bound), and the segments between consecutive splitters are
// merged independently.  Across ranks:
//   1. each rank sorts its shard (labsort_sort_device);
//   2. every rank contributes a regular sample of its sorted shard (allgather);
//   3. all ranks pick the same p-1 splitters -- (key, rank, position) triples, so runs
//      of one repeated key are cut between ranks like any other keys;
//   4. each rank cuts its sorted shard at the splitters (bound queries);
//   5. the piece counts are allgathered, piece j of rank i goes to rank j by pairwise
//      send/recv with every peer at once (RCCL ncclSend/ncclRecv in one group);
//   6. each rank merges its p received runs in rank order (equal keys keep rank order),
//      and holds the contiguous range [goff, goff + total) of the sorted array.
#pragma once
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/labsort.h"

namespace labsort {
namespace dist {

struct Splitter {
    uint32_t ord;   // key ^ flip: monotone in key order
    uint32_t rank;  // rank whose sample it is
    uint64_t pos;   // position in that rank's sorted shard
    uint32_t key;   // the 32-bit word
};

// regular sample: s keys per rank at positions k*m/s (ranges end within ~m/s of n/p)
inline size_t samples_per_rank(int p) { return (size_t)256 * (size_t)p; }
inline size_t sample_pos(size_t m, size_t s, size_t k) { return (size_t)((unsigned __int128)k * m / s); }

// p-1 splitters at the quantiles of the pooled samples, in (key, rank, position) order
inline std::vector<Splitter> choose_splitters(int p, const uint64_t *m, const uint32_t *samples, size_t s,
                                              uint32_t flip) {
    std::vector<Splitter> pool;
    pool.reserve(s * (size_t)p);
    for (int r = 0; r < p; ++r) {
        if (!m[r]) continue;  // an empty shard samples nothing
        for (size_t k = 0; k < s; ++k) {
            const uint32_t key = samples[(size_t)r * s + k];
            pool.push_back({key ^ flip, (uint32_t)r, (uint64_t)sample_pos(m[r], s, k), key});
        }
    }
    // a sorted shard's sample positions ascend, so a stable sort by (key, rank) is
    // the (key, rank, position) order
    std::stable_sort(pool.begin(), pool.end(), [](const Splitter &a, const Splitter &b) {
        return a.ord != b.ord ? a.ord < b.ord : a.rank < b.rank;
    });
    std::vector<Splitter> spl(p > 1 ? p - 1 : 0);
    if (pool.empty()) {
        for (auto &x : spl) x = {0u, 0u, 0u, 0u};
        return spl;
    }
    for (int j = 1; j < p; ++j) spl[j - 1] = pool[(size_t)j * pool.size() / p];
    return spl;
}

// bound-query values of one rank: the splitter keys, then the key just below each
inline std::vector<uint32_t> plan_values(const std::vector<Splitter> &spl, int p, uint32_t flip) {
    std::vector<uint32_t> vals(p > 1 ? 2 * (p - 1) : 0);
    for (int j = 0; j < p - 1; ++j) {
        vals[j] = spl[j].key;
        vals[p - 1 + j] = spl[j].ord ? ((spl[j].ord - 1) ^ flip) : spl[j].key;
    }
    return vals;
}

// cut[0..p] of rank r's sorted shard of m keys: piece j = [cut[j], cut[j+1]) goes to
// rank j.  `ub` = the answers of plan_values' bound queries (keys <= value).
inline int rank_cuts(int r, uint64_t m, const std::vector<Splitter> &spl, const uint32_t *ub, int p,
                     uint64_t *cut) {
    cut[0] = 0;
    cut[p] = m;
    if (!m || p == 1) {
        for (int j = 1; j < p; ++j) cut[j] = 0;
        return LABSORT_OK;
    }
    for (int j = 0; j < p - 1; ++j) {
        const uint64_t upper = ub[j], lower = spl[j].ord ? ub[p - 1 + j] : 0;
        uint64_t x;
        if (spl[j].rank > (uint32_t)r) x = upper;       // rank r's equal keys precede the splitter
        else if (spl[j].rank < (uint32_t)r) x = lower;  // ... or follow it
        else x = spl[j].pos + 1;                        // the splitter itself ends piece j
        if (x < cut[j] || x > m) return LABSORT_ERR_DEVICE;  // inconsistent bounds
        cut[j + 1] = x;
    }
    return LABSORT_OK;
}

struct Result {
    const uint32_t *data = nullptr;  // this rank's sorted range (owned by the rank operations)
    uint64_t count = 0;              // keys in it
    uint64_t goff = 0;               // its offset in the global sorted array
    uint64_t sent = 0;               // key bytes this rank sent to its peers
};

// Phase marks the schedule reports to the rank operations (timing hooks)
enum Mark { M_START = 0, M_SORTED, M_PLANNED, M_EXCHANGED, M_MERGED, M_NMARKS };

// One rank of the distributed sort.
//   Ops  (rank operations, on the rank's device or on the host):
//     int local_sort(const uint32_t *in, uint64_t m, const uint32_t **sorted)
//     int sample(const uint32_t *sorted, uint64_t m, size_t s, uint32_t *h_out)       (blocking)
//     int bounds(const uint32_t *sorted, uint64_t m, const uint32_t *h_vals, size_t nv,
//                uint32_t *h_out)                                                     (blocking)
//     int recv_buffer(uint64_t total, uint32_t **recv)
//     int copy_local(uint32_t *dst, const uint32_t *src, uint64_t count)
//     int merge(const uint32_t *recv, const uint64_t *offs, int p, uint32_t *h_sink,
//               const uint32_t **result)   -- h_sink: also copy the result to this host address
//     void mark(Mark)
//   Comm (the ranks' communicator):
//     int size(), rank()
//     int allgather(const void *h_in, void *h_out, size_t bytes)                      (blocking)
//     int exchange(const uint32_t *const *send, const uint64_t *scount,
//                  uint32_t *const *recv, const uint64_t *rcount)   -- self pieces excluded
// `h_out_base` (nullable): the caller's host array of the whole sorted output; this
// rank's range is copied to h_out_base + goff.
template <class Ops, class Comm>
int sort_rank(Ops &ops, Comm &comm, const uint32_t *in, uint64_t m, uint32_t flip, uint32_t *h_out_base,
              Result &res) {
    const int p = comm.size(), r = comm.rank();
    int st;
    ops.mark(M_START);
    const uint32_t *S = nullptr;
    if ((st = ops.local_sort(in, m, &S))) return st;
    ops.mark(M_SORTED);
    res = Result{};
    // (one rank runs the whole schedule too: its communicator is exercised, at the
    // price of one copy of the shard)
    // 2. shard sizes and samples of every rank
    const size_t s = samples_per_rank(p), rec = 8 + 4 * s;
    std::vector<uint8_t> mine(rec, 0), all(rec * (size_t)p, 0);
    memcpy(mine.data(), &m, 8);
    if (m && (st = ops.sample(S, m, s, reinterpret_cast<uint32_t *>(mine.data() + 8)))) return st;
    if ((st = comm.allgather(mine.data(), all.data(), rec))) return st;
    std::vector<uint64_t> ms(p);
    std::vector<uint32_t> samples((size_t)p * s);
    for (int i = 0; i < p; ++i) {
        memcpy(&ms[i], all.data() + (size_t)i * rec, 8);
        memcpy(&samples[(size_t)i * s], all.data() + (size_t)i * rec + 8, 4 * s);
    }
    if (ms[r] != m) return LABSORT_ERR_ARG;  // the communicator mixed up the ranks
    // 3-4. splitters (the same on every rank) and this rank's cut points
    const std::vector<Splitter> spl = choose_splitters(p, ms.data(), samples.data(), s, flip);
    const std::vector<uint32_t> vals = plan_values(spl, p, flip);
    std::vector<uint32_t> ub(vals.size(), 0u);
    if (m && (st = ops.bounds(S, m, vals.data(), vals.size(), ub.data()))) return st;
    std::vector<uint64_t> cut(p + 1);
    if ((st = rank_cuts(r, m, spl, ub.data(), p, cut.data()))) return st;
    // 5. piece counts of every rank: C[i * p + j] = keys rank i sends to rank j
    std::vector<uint64_t> sc(p), C((size_t)p * p);
    for (int j = 0; j < p; ++j) sc[j] = cut[j + 1] - cut[j];
    if ((st = comm.allgather(sc.data(), C.data(), 8 * (size_t)p))) return st;
    for (int j = 0; j < p; ++j)
        if (C[(size_t)r * p + j] != sc[j]) return LABSORT_ERR_ARG;
    std::vector<uint64_t> roff(p + 1, 0);
    for (int i = 0; i < p; ++i) roff[i + 1] = roff[i] + C[(size_t)i * p + r];
    uint64_t goff = 0;
    for (int i = 0; i < p; ++i)
        for (int j = 0; j < r; ++j) goff += C[(size_t)i * p + j];
    const uint64_t total = roff[p];
    ops.mark(M_PLANNED);
    uint32_t *R = nullptr;
    if ((st = ops.recv_buffer(total, &R))) return st;
    if (sc[r] && (st = ops.copy_local(R + roff[r], S + cut[r], sc[r]))) return st;
    std::vector<const uint32_t *> sp(p, nullptr);
    std::vector<uint32_t *> rp(p, nullptr);
    std::vector<uint64_t> scount(p, 0), rcount(p, 0);
    uint64_t sent = 0;
    for (int j = 0; j < p; ++j) {
        if (j == r) continue;
        sp[j] = S + cut[j];
        scount[j] = sc[j];
        rp[j] = R + roff[j];
        rcount[j] = C[(size_t)j * p + r];
        sent += 4 * sc[j];
    }
    if ((st = comm.exchange(sp.data(), scount.data(), rp.data(), rcount.data()))) return st;
    ops.mark(M_EXCHANGED);
    // 6. merge of the p received runs in rank order
    const uint32_t *out = nullptr;
    if ((st = ops.merge(R, roff.data(), p, h_out_base ? h_out_base + goff : nullptr, &out))) return st;
    ops.mark(M_MERGED);
    res.data = out;
    res.count = total;
    res.goff = goff;
    res.sent = sent;
    return LABSORT_OK;
}

}  // namespace dist
}  // namespace labsort
