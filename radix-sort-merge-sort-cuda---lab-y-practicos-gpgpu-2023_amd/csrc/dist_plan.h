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
#include <stdlib.h>
#include <string.h>

#include <chrono>

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

// p-1 splitters at the quantiles of the pooled samples, in (key, rank, position) order:
// splitter j is the pooled sample of index j * N / p (N = samples of the non-empty shards).
inline std::vector<Splitter> choose_splitters(int p, const uint64_t *m, const uint32_t *samples, size_t s,
                                              uint32_t flip) {
    std::vector<Splitter> spl(p > 1 ? p - 1 : 0);
    std::vector<int> src;  // ranks that sampled (non-empty shards), ascending
    bool ascending = true;
    for (int r = 0; r < p; ++r) {
        if (!m[r]) continue;  // an empty shard samples nothing
        src.push_back(r);
        const uint32_t *x = samples + (size_t)r * s;
        for (size_t k = 1; k < s && ascending; ++k) ascending = (x[k] ^ flip) >= (x[k - 1] ^ flip);
    }
    const size_t N = s * src.size();
    if (!N) {
        for (auto &x : spl) x = {0u, 0u, 0u, 0u};
        return spl;
    }
    auto make = [&](int r, size_t k) {
        const uint32_t key = samples[(size_t)r * s + k];
        return Splitter{key ^ flip, (uint32_t)r, (uint64_t)sample_pos(m[r], s, k), key};
    };
    if (!ascending) {  // samples of a shard that was not sorted: order the pool outright
        std::vector<Splitter> pool;
        pool.reserve(N);
        for (int r : src)
            for (size_t k = 0; k < s; ++k) pool.push_back(make(r, k));
        // sample positions ascend within a rank, so a stable sort by (key, rank) is the
        // (key, rank, position) order
        std::stable_sort(pool.begin(), pool.end(), [](const Splitter &a, const Splitter &b) {
            return a.ord != b.ord ? a.ord < b.ord : a.rank < b.rank;
        });
        for (int j = 1; j < p; ++j) spl[j - 1] = pool[(size_t)j * N / p];
        return spl;
    }
    // Sorted shards (the schedule's case): each rank's samples are one ascending run, so
    // the pooled sample of index t is found without forming the pool -- the smallest key X
    // with more than t samples <= X (a binary search over the 32-bit key order, counting
    // by one bound search per run), then among the samples equal to X, taken in (rank,
    // position) order, the (t - #samples < X)-th.  O(p log s) per key step, no allocation:
    // at p = 8 (16 Ki samples) a few tens of microseconds on every rank instead of the
    // ~1 ms a sort of the pool takes.
    auto count = [&](uint32_t ord, bool le) {  // samples with key < ord (le: <= ord)
        size_t c = 0;
        for (int r : src) {
            const uint32_t *x = samples + (size_t)r * s;
            size_t lo = 0, hi = s;
            while (lo < hi) {
                const size_t mid = (lo + hi) / 2;
                const uint32_t v = x[mid] ^ flip;
                if (v < ord || (le && v == ord)) lo = mid + 1;
                else hi = mid;
            }
            c += lo;
        }
        return c;
    };
    for (int j = 1; j < p; ++j) {
        const size_t t = (size_t)j * N / p;
        uint64_t lo = 0, hi = 0xFFFFFFFFull;  // smallest ord in [lo, hi] with count(<= ord) > t
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            if (count((uint32_t)mid, true) > t) hi = mid;
            else lo = mid + 1;
        }
        const uint32_t X = (uint32_t)lo;
        size_t rem = t - count(X, false);
        for (int r : src) {
            const uint32_t *x = samples + (size_t)r * s;
            const size_t b = (size_t)(std::lower_bound(x, x + s, X, [&](uint32_t a, uint32_t v) {
                                          return (a ^ flip) < v;
                                      }) - x);
            const size_t e = (size_t)(std::upper_bound(x + b, x + s, X, [&](uint32_t v, uint32_t a) {
                                          return v < (a ^ flip);
                                      }) - x);
            if (rem < e - b) {
                spl[j - 1] = make(r, b + rem);
                break;
            }
            rem -= e - b;
        }
    }
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

// Collectives of one sort_rank call, in order (the timing records index them)
enum Coll { C_SAMPLES = 0, C_COUNTS, C_GROW, C_NCOLL };

struct Result {
    const uint32_t *data = nullptr;  // this rank's sorted range (owned by the rank operations)
    uint64_t count = 0;              // keys in it
    uint64_t goff = 0;               // its offset in the global sorted array
    uint64_t sent = 0;               // key bytes this rank sent to its peers
    // host wall clock, ms since the call started: arrival at / return from each collective
    // (C_GROW runs only when some rank's range outgrew the pre-sized receive buffer; -1
    // when it did not run).  leave - arrive = time spent waiting for the slowest peer
    // (plus the collective's own latency); the rest of the plan phase is this rank's work.
    double arrive[C_NCOLL] = {-1.0, -1.0, -1.0}, leave[C_NCOLL] = {-1.0, -1.0, -1.0};
    // host wall clock, ms since the call started: the plan phase as this rank's host sees
    // it, from its local sort observed complete (wait_sorted) to the plan's end.  Its work
    // = this span minus the time inside the collectives, on one clock (a device-event span
    // would also count marker packets queued behind other ranks' work when several ranks
    // share one GPU's hardware queues).
    double plan_host[2] = {-1.0, -1.0};
    int failed_rank = -1;  // the lowest rank that reported a failure (-1: none)
};

// Phase marks the schedule reports to the rank operations (timing hooks)
enum Mark { M_START = 0, M_SORTED, M_PLANNED, M_EXCHANGED, M_MERGED, M_NMARKS };

// Test hook: the named rank reports a failure at that step, as an out-of-memory or an
// expired device spin would (F_EXCHANGE: its transport breaks -- it leaves without taking
// part in the exchange); the tests check that every rank then returns an error instead of
// waiting for the failed one.  Armed only through the test entry points
// (labsort_test_fault, oracle_test_fault): no environment variable is read on a sort.
enum FaultPhase { F_NONE = 0, F_LOCAL_SORT, F_BOUNDS, F_RECV, F_GROW, F_EXCHANGE, F_NPHASES };
struct Fault {
    int phase = F_NONE;
    int rank = -1;
};
// phase name of the test entry points ("local_sort", "bounds", "recv", "grow", "exchange")
inline int fault_phase(const char *name) {
    static const char *const names[F_NPHASES] = {"", "local_sort", "bounds", "recv", "grow", "exchange"};
    for (int i = 1; name && i < F_NPHASES; ++i)
        if (!strcmp(name, names[i])) return i;
    return F_NONE;
}
inline int injected(const Fault &f, int phase, int r) {
    return f.phase == phase && f.rank == r ? LABSORT_ERR_DEVICE : LABSORT_OK;
}

// Receive buffer sized before the counts are known.  With equal shards every range lies
// within about m / (256 p) keys of n / p (samples_per_rank), so 1.25 n / p (+ 64 Ki keys)
// covers it.  The samples are not weighted by shard size, so unequal shards can exceed it
// (shards of 10^6 and 10^3 keys, the small one holding the largest keys: range 0 is the
// whole big shard); a rank whose range is larger grows its buffer in an extra status
// round that every rank takes part in (all ranks see all the counts, so all take it).
inline uint64_t recv_estimate(uint64_t total, int p) {
    const uint64_t share = (total + (uint64_t)p - 1) / (uint64_t)p;
    return share + share / 4 + ((uint64_t)1 << 16);
}

// One rank of the distributed sort.
//   Ops  (rank operations, on the rank's device or on the host):
//     int local_sort(const uint32_t *in, uint64_t m, const uint32_t **sorted)
//     int sample(const uint32_t *sorted, uint64_t m, size_t s, uint32_t *h_out)       (blocking)
//     int bounds(const uint32_t *sorted, uint64_t m, const uint32_t *h_vals, size_t nv,
//                uint32_t *h_out)                                                     (blocking)
//     int recv_buffer(uint64_t total, uint32_t **recv)      -- grows, never shrinks
//     int copy_local(uint32_t *dst, const uint32_t *src, uint64_t count)
//     int merge(const uint32_t *recv, const uint64_t *offs, int p, uint32_t *h_sink,
//               const uint32_t **result)   -- h_sink: also copy the result to this host address
//     void mark(Mark)
//     int wait_sorted()   -- blocks until the local sort has completed
//   Comm (the ranks' communicator):
//     int size(), rank()
//     int allgather(const void *h_in, void *h_out, size_t bytes)                      (blocking)
//     int exchange(const uint32_t *const *send, const uint64_t *scount,
//                  uint32_t *const *recv, const uint64_t *rcount)   -- self pieces excluded;
//                  a peer that never takes part must not block it forever (RCCL: a
//                  deadline, then ncclCommAbort; host callbacks: the caller's timeout)
//     void abandon()   -- this rank leaves without taking part in the exchange (its
//                  transport broke): tell the peers now where the communicator can
//                  (in-process ranks: the shared failure flag their waits poll);
//                  otherwise the peers' exchange ends at their own deadline (RCCL:
//                  ncclCommAbort after it; host callbacks: the caller's timeout)
// `h_out_base` (nullable): the caller's host array of the whole sorted output; this
// rank's range is copied to h_out_base + goff.
//
// Failures: a rank whose own step fails (local sort, samples, bounds, buffers) still takes
// part in every collective up to the exchange and reports its status word in the record;
// after each allgather every rank checks all status words and, if any is set, returns --
// its own error, or LABSORT_ERR_PEER when only another rank failed -- so no rank is left
// waiting in a collective for a rank that gave up.  A communicator whose collective itself
// fails returns that failure at once.
template <class Ops, class Comm>
int sort_rank(Ops &ops, Comm &comm, const uint32_t *in, uint64_t m, uint32_t flip, uint32_t *h_out_base,
              Result &res, const Fault &fault = Fault{}) {
    const int p = comm.size(), r = comm.rank();
    const auto t_start = std::chrono::steady_clock::now();
    auto now_ms = [&]() {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    };
    res = Result{};
    // one collective with every rank's status word at offset 0 of its record
    auto gather = [&](int k, const std::vector<uint8_t> &mine, std::vector<uint8_t> &all, int &st) {
        res.arrive[k] = now_ms();
        const int c = comm.allgather(mine.data(), all.data(), mine.size());
        res.leave[k] = now_ms();
        if (c) return c;  // the communicator failed: nothing was agreed
        for (int i = 0; i < p; ++i) {
            uint32_t w;
            memcpy(&w, all.data() + (size_t)i * mine.size(), 4);
            if (w && res.failed_rank < 0) res.failed_rank = i;
        }
        if (res.failed_rank >= 0) return st ? st : LABSORT_ERR_PEER;
        return LABSORT_OK;
    };
    ops.mark(M_START);
    const uint32_t *S = nullptr;
    int st = injected(fault, F_LOCAL_SORT, r);
    if (!st) st = ops.local_sort(in, m, &S);
    ops.mark(M_SORTED);
    if (!st) st = ops.wait_sorted();
    res.plan_host[0] = now_ms();
    // 2. status, shard size and samples of every rank
    const size_t s = samples_per_rank(p), rec = 16 + 4 * s;
    std::vector<uint8_t> mine(rec, 0), all(rec * (size_t)p, 0);
    if (!st && m) st = ops.sample(S, m, s, reinterpret_cast<uint32_t *>(mine.data() + 16));
    uint32_t sw = (uint32_t)st;
    memcpy(mine.data(), &sw, 4);
    memcpy(mine.data() + 8, &m, 8);
    if (int c = gather(C_SAMPLES, mine, all, st)) return c;
    std::vector<uint64_t> ms(p);
    std::vector<uint32_t> samples((size_t)p * s);
    uint64_t ntot = 0;
    for (int i = 0; i < p; ++i) {
        memcpy(&ms[i], all.data() + (size_t)i * rec + 8, 8);
        memcpy(&samples[(size_t)i * s], all.data() + (size_t)i * rec + 16, 4 * s);
        ntot += ms[i];
    }
    if (ms[r] != m) st = LABSORT_ERR_ARG;  // the communicator mixed up the ranks
    // 3-4. splitters (the same on every rank) and this rank's cut points; the receive
    // buffer pre-sized
    const std::vector<Splitter> spl = choose_splitters(p, ms.data(), samples.data(), s, flip);
    const std::vector<uint32_t> vals = plan_values(spl, p, flip);
    std::vector<uint32_t> ub(vals.size(), 0u);
    std::vector<uint64_t> cut(p + 1, 0);
    if (!st) st = injected(fault, F_BOUNDS, r);
    if (!st && m) st = ops.bounds(S, m, vals.data(), vals.size(), ub.data());
    if (!st) st = rank_cuts(r, m, spl, ub.data(), p, cut.data());
    const uint64_t est = recv_estimate(ntot, p);
    uint32_t *R = nullptr;
    if (!st) st = injected(fault, F_RECV, r);
    if (!st) st = ops.recv_buffer(est, &R);
    // 5. status and piece counts of every rank: C[i * p + j] = keys rank i sends to rank j
    std::vector<uint64_t> sc(p, 0), C((size_t)p * p);
    for (int j = 0; j < p && !st; ++j) sc[j] = cut[j + 1] - cut[j];
    {
        std::vector<uint8_t> cm(8 * ((size_t)p + 1), 0), ca(cm.size() * (size_t)p, 0);
        sw = (uint32_t)st;
        memcpy(cm.data(), &sw, 4);
        memcpy(cm.data() + 8, sc.data(), 8 * (size_t)p);
        if (int c = gather(C_COUNTS, cm, ca, st)) return c;
        for (int i = 0; i < p; ++i) memcpy(&C[(size_t)i * p], ca.data() + (size_t)i * cm.size() + 8, 8 * (size_t)p);
    }
    // every row must add up to its rank's shard: a check all ranks reach the same verdict on
    uint64_t rmax = 0;
    for (int i = 0; i < p; ++i) {
        uint64_t row = 0, col = 0;
        for (int j = 0; j < p; ++j) {
            row += C[(size_t)i * p + j];
            col += C[(size_t)j * p + i];
        }
        if (row != ms[i]) return LABSORT_ERR_ARG;
        rmax = col > rmax ? col : rmax;
    }
    std::vector<uint64_t> roff(p + 1, 0);
    for (int i = 0; i < p; ++i) roff[i + 1] = roff[i] + C[(size_t)i * p + r];
    uint64_t goff = 0;
    for (int i = 0; i < p; ++i)
        for (int j = 0; j < r; ++j) goff += C[(size_t)i * p + j];
    const uint64_t total = roff[p];
    if (rmax > est) {  // some range outgrew the pre-sized buffers: grow, then agree again
        st = injected(fault, F_GROW, r);
        if (!st) st = ops.recv_buffer(total, &R);
        std::vector<uint8_t> gm(8, 0), ga(8 * (size_t)p, 0);
        sw = (uint32_t)st;
        memcpy(gm.data(), &sw, 4);
        if (int c = gather(C_GROW, gm, ga, st)) return c;
    } else if ((st = ops.recv_buffer(total, &R))) {
        return st;  // (cannot allocate: total <= est was allocated above)
    }
    ops.mark(M_PLANNED);
    res.plan_host[1] = now_ms();
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
    // (a rank whose transport breaks here leaves its peers inside the exchange: the
    // communicators bound that wait -- RCCL by a deadline and ncclCommAbort)
    if ((st = injected(fault, F_EXCHANGE, r))) {
        comm.abandon();
        return st;
    }
    if ((st = comm.exchange(sp.data(), scount.data(), rp.data(), rcount.data()))) return st;
    // (the own piece after the exchange: nothing can fail between the agreement and it)
    if (sc[r] && (st = ops.copy_local(R + roff[r], S + cut[r], sc[r]))) return st;
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
