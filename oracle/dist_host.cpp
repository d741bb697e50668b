// dist_host.cpp -- TEST INFRASTRUCTURE ONLY (tests/ may call it; the product never does).
//
// The multi-GPU merge-sort schedule of the product (csrc/dist_plan.h, dist::sort_rank:
// the one copy of the schedule, also run by csrc/multi.hip on the GPUs) instantiated
// with HOST rank operations -- std::sort for the local sort (the spec oracle), regular
// samples, std::upper_bound for the bound queries, std::merge of the received runs in
// rank order (A before B on ties, as lab.cu:163-170) -- over the caller's host
// collectives (labsort_host_coll; the CPU tests pass torch.distributed gloo callbacks).
// So `pytest -m "not gpu"` runs the product's exchange schedule with 2-8 gloo ranks on
// machines without GPUs.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/csrc/dist_plan.h"

namespace {

using labsort::dist::Mark;

struct HostOps {
    uint32_t flip;
    std::vector<uint32_t> S, R, T;
    bool less(uint32_t a, uint32_t b) const { return (a ^ flip) < (b ^ flip); }
    void mark(Mark) {}
    int wait_sorted() { return LABSORT_OK; }
    int local_sort(const uint32_t *in, uint64_t m, const uint32_t **sorted) {
        S.assign(in, in + m);
        std::sort(S.begin(), S.end(), [this](uint32_t a, uint32_t b) { return less(a, b); });
        *sorted = S.data();
        return LABSORT_OK;
    }
    int sample(const uint32_t *s, uint64_t m, size_t n, uint32_t *h_out) {
        for (size_t k = 0; k < n; ++k) h_out[k] = s[labsort::dist::sample_pos(m, n, k)];
        return LABSORT_OK;
    }
    int bounds(const uint32_t *s, uint64_t m, const uint32_t *vals, size_t nv, uint32_t *h_out) {
        for (size_t v = 0; v < nv; ++v)
            h_out[v] = (uint32_t)(std::upper_bound(s, s + m, vals[v],
                                                   [this](uint32_t x, uint32_t y) { return less(x, y); }) -
                                  s);
        return LABSORT_OK;
    }
    int recv_buffer(uint64_t total, uint32_t **recv) {
        if (R.size() < total || R.empty()) R.resize(total ? total : 1, 0u);
        *recv = R.data();
        return LABSORT_OK;
    }
    int copy_local(uint32_t *dst, const uint32_t *src, uint64_t count) {
        memmove(dst, src, count * 4);
        return LABSORT_OK;
    }
    int merge(const uint32_t *recv, const uint64_t *offs, int p, uint32_t *h_sink, const uint32_t **result) {
        // runs merged left to right: (((r0 + r1) + r2) + ...), A before B on ties
        T.assign(recv, recv + offs[p]);
        std::vector<uint32_t> tmp(offs[p]);
        for (int q = 1; q < p; ++q) {
            std::merge(T.begin(), T.begin() + offs[q], T.begin() + offs[q], T.begin() + offs[q + 1], tmp.begin(),
                       [this](uint32_t a, uint32_t b) { return less(a, b); });
            std::copy(tmp.begin(), tmp.begin() + offs[q + 1], T.begin());
        }
        if (h_sink) std::copy(T.begin(), T.begin() + offs[p], h_sink);
        *result = T.data();
        return LABSORT_OK;
    }
};

struct CbComm {
    labsort_host_coll cb;
    int p, me;
    int size() const { return p; }
    int rank() const { return me; }
    // a failed callback: the caller's transport failed or a peer left it (as multi.hip's HostCbComm)
    int allgather(const void *in, void *out, size_t bytes) {
        return cb.allgather(cb.ctx, in, out, bytes) ? LABSORT_ERR_PEER : LABSORT_OK;
    }
    int exchange(const uint32_t *const *send, const uint64_t *sc, uint32_t *const *recv, const uint64_t *rc) {
        std::vector<size_t> sb(p), rb(p);
        std::vector<uint32_t> hs, hr;
        for (int j = 0; j < p; ++j) {
            sb[j] = j == me ? 0 : sc[j] * 4;
            rb[j] = j == me ? 0 : rc[j] * 4;
            if (sb[j]) hs.insert(hs.end(), send[j], send[j] + sc[j]);
        }
        size_t tr = 0;
        for (int j = 0; j < p; ++j) tr += rb[j] / 4;
        hs.resize(std::max<size_t>(hs.size(), 1));
        hr.resize(std::max<size_t>(tr, 1));
        if (cb.alltoallv(cb.ctx, hs.data(), sb.data(), hr.data(), rb.data())) return LABSORT_ERR_PEER;
        size_t o = 0;
        for (int j = 0; j < p; ++j) {
            if (rb[j]) memcpy(recv[j], hr.data() + o, rb[j]);
            o += rb[j] / 4;
        }
        return LABSORT_OK;
    }
    void abandon() {}  // the peers' gloo collective ends at the group's timeout
};

labsort::dist::Fault g_fault;  // armed by oracle_test_fault (tests only)

}  // namespace

extern "C" {

// Arm (phase "local_sort" | "bounds" | "recv" | "grow" | "exchange", rank) or disarm
// (NULL / unknown phase) the schedule's test failure for the following oracle_dist_sort calls.
void oracle_test_fault(const char *phase, int rank) {
    g_fault.phase = labsort::dist::fault_phase(phase);
    g_fault.rank = g_fault.phase ? rank : -1;
}

// One rank of the product's distributed sort schedule on host shards.  out: room for
// `cap` keys; *count = keys of this rank's range, *goff = its global offset.  Returns a
// LABSORT_* status (LABSORT_ERR_ARG also when cap is too small).
int oracle_dist_sort(const uint32_t *shard, uint64_t m, int key_type, int world, int rank,
                     const labsort_host_coll *coll, uint32_t *out, uint64_t cap, uint64_t *count, uint64_t *goff) {
    if (!coll || world < 1 || rank < 0 || rank >= world || !count || !goff) return LABSORT_ERR_ARG;
    HostOps ops{key_type == LABSORT_KEY_I32 ? 0x80000000u : 0u, {}, {}, {}};
    CbComm comm{*coll, world, rank};
    labsort::dist::Result res;
    const int st = labsort::dist::sort_rank(ops, comm, shard, m, ops.flip, nullptr, res, g_fault);
    if (st) return st;
    *count = res.count;
    *goff = res.goff;
    if (res.count > cap) return LABSORT_ERR_ARG;
    if (res.count) memcpy(out, res.data, res.count * 4);
    return LABSORT_OK;
}

}  // extern "C"
