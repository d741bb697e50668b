// multi.hip -- order_array across the GPUs of one node, from one host process
// (the reference is single-GPU: lab.cu:303-402).
//
//   labsort_sort_host_multi(h, n, key, p)   ranks 0..p-1 on devices 0..p-1, RCCL
//   labsort_sort_host_ranks(h, n, key, p, devices, transport)   any rank -> device map
//
// Schedule (one call = one completed sort of the caller's host buffer, in place):
//   1. shard r = h[r*n/p, (r+1)*n/p): H2D over rank r's own PCIe link (one host
//      thread per rank, so the p links copy at once), local radix/merge sort;
//   2. a regular sample of every sorted shard -> p-1 splitters, each a
//      (key, rank, position) triple, so runs of one repeated key are cut between
//      ranks like any other keys (every range stays near n/p);
//   3. each rank's cut points at the splitters (labsort_upper_bound on its shard);
//   4. exchange: piece j of rank i -> rank j, straight into rank j's receive buffer
//      at its rank-ordered slot: RCCL ncclSend/ncclRecv to all peers in one group
//      (every xGMI link of a GPU carries data at once) or, for ranks that share a
//      device, peer copies (hipMemcpyPeerAsync);
//   5. rank j merges its p received runs in one K-way pass (labsort_merge_runs,
//      equal keys keep rank order) and copies its range D2H to its global offset.
// The plan of steps 2-3 is host code shared with labsort_multi_plan, which runs it
// on host shards (std::upper_bound bound queries) so the CPU tests check it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/labsort.h"
#include "common.h"

namespace labsort {
namespace {

// ---------------------------------------------------------------------------------
// the exchange plan (host only)
// ---------------------------------------------------------------------------------
struct Splitter {
    uint32_t ord;   // key ^ flip: monotone in key order
    uint32_t rank;  // rank whose sample it is
    uint64_t pos;   // position in that rank's sorted shard
    uint32_t key;   // the 32-bit word
};

struct ExPlan {
    int p = 0;
    std::vector<size_t> m;         // shard sizes
    std::vector<size_t> cut;       // [r * (p+1) + j]: first position of piece j on rank r
    std::vector<size_t> recv_off;  // [j * (p+1) + i]: slot of piece i->j in rank j's receive buffer
    size_t count(int i, int j) const { return cut[i * (p + 1) + j + 1] - cut[i * (p + 1) + j]; }
    size_t total(int j) const { return recv_off[j * (p + 1) + p]; }
    size_t roff(int j, int i) const { return recv_off[j * (p + 1) + i]; }
};

inline size_t sample_pos(size_t m, size_t s, size_t k) { return k * m / s; }
inline size_t samples_per_rank(int p) { return (size_t)256 * (size_t)p; }  // ranges within ~m/(256p) keys of n/p

// bound query: out[v] = number of keys of rank r's sorted shard <= values[v] (key order)
using BoundFn = std::function<int(int r, const std::vector<uint32_t> &values, std::vector<uint32_t> &out)>;

std::vector<Splitter> choose_splitters(int p, const std::vector<size_t> &m,
                                       const std::vector<std::vector<uint32_t>> &samples, uint32_t flip) {
    const size_t s = samples_per_rank(p);
    std::vector<Splitter> pool;
    pool.reserve(s * p);
    for (int r = 0; r < p; ++r) {
        if (!m[r]) continue;  // an empty shard samples nothing
        for (size_t k = 0; k < s; ++k) {
            const uint32_t key = samples[r][k];
            pool.push_back({key ^ flip, (uint32_t)r, (uint64_t)sample_pos(m[r], s, k), key});
        }
    }
    // (key, rank, position) order: a sorted shard's positions are already ascending
    std::stable_sort(pool.begin(), pool.end(), [](const Splitter &a, const Splitter &b) {
        return a.ord != b.ord ? a.ord < b.ord : a.rank < b.rank;
    });
    std::vector<Splitter> spl(p > 1 ? p - 1 : 0);
    for (int j = 1; j < p; ++j) spl[j - 1] = pool[(size_t)j * pool.size() / p];
    return spl;
}

// bound-query values: the splitter keys, then the key just below each (its lower bound)
std::vector<uint32_t> plan_values(const std::vector<Splitter> &spl, int p, uint32_t flip) {
    std::vector<uint32_t> vals(p > 1 ? 2 * (p - 1) : 0);
    for (int j = 0; j < p - 1; ++j) {
        vals[j] = spl[j].key;
        vals[p - 1 + j] = spl[j].ord ? ((spl[j].ord - 1) ^ flip) : spl[j].key;
    }
    return vals;
}

int make_plan(ExPlan &P, const std::vector<Splitter> &spl, uint32_t flip, const BoundFn &ub) {
    const int p = P.p;
    P.cut.assign((size_t)p * (p + 1), 0);
    P.recv_off.assign((size_t)p * (p + 1), 0);
    const std::vector<uint32_t> vals = plan_values(spl, p, flip);
    std::vector<uint32_t> out;
    for (int r = 0; r < p; ++r) {
        size_t *c = &P.cut[(size_t)r * (p + 1)];
        c[p] = P.m[r];
        if (!P.m[r] || p == 1) continue;
        out.assign(vals.size(), 0);
        const int st = ub(r, vals, out);
        if (st) return st;
        for (int j = 0; j < p - 1; ++j) {
            const size_t upper = out[j], lower = spl[j].ord ? out[p - 1 + j] : 0;
            size_t x;
            if (spl[j].rank > (uint32_t)r) x = upper;       // rank r's equal keys precede the splitter
            else if (spl[j].rank < (uint32_t)r) x = lower;  // ... or follow it
            else x = (size_t)spl[j].pos + 1;                // the splitter itself ends piece j
            if (x < c[j] || x > P.m[r]) return LABSORT_ERR_DEVICE;  // inconsistent bounds
            c[j + 1] = x;
        }
    }
    for (int j = 0; j < p; ++j) {
        size_t *o = &P.recv_off[(size_t)j * (p + 1)];
        for (int i = 0; i < p; ++i) o[i + 1] = o[i] + P.count(i, j);
    }
    return LABSORT_OK;
}

// ---------------------------------------------------------------------------------
// device side
// ---------------------------------------------------------------------------------
__global__ void k_sample(const uint32_t *__restrict__ keys, uint64_t m, uint32_t s, uint32_t *__restrict__ out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < s) out[k] = keys[(uint64_t)k * m / s];
}

thread_local int t_last_hip = 0;
#define MHIP(x)                                  \
    do {                                         \
        hipError_t _e = (x);                     \
        if (_e != hipSuccess) {                  \
            t_last_hip = (int)_e;                \
            return LABSORT_ERR_HIP;              \
        }                                        \
    } while (0)

struct Buf {
    void *p = nullptr;
    size_t bytes = 0;
};
int grow(Buf &b, size_t need) {
    if (b.p && b.bytes >= need) return LABSORT_OK;
    if (b.p) MHIP(hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
    const size_t want = std::max(need, (size_t)1 << 16);
    MHIP(hipMalloc(&b.p, want));
    b.bytes = want;
    return LABSORT_OK;
}

struct RankState {
    int dev = -1;
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;
    Buf keys, recv, out, ws, kmws, small;
};

// RCCL, loaded on first use (no link-time dependency; in a torch process the
// already-loaded librccl.so.1 is the one dlopen returns)
struct Rccl {
    bool tried = false;
    void *h = nullptr;
    decltype(&ncclCommInitAll) init = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) gstart = nullptr;
    decltype(&ncclGroupEnd) gend = nullptr;
    decltype(&ncclGetErrorString) errstr = nullptr;
    std::vector<int> devs;
    std::vector<ncclComm_t> comms;
    bool load() {
        if (tried) return h != nullptr;
        tried = true;
        h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return false;
        init = (decltype(init))dlsym(h, "ncclCommInitAll");
        send = (decltype(send))dlsym(h, "ncclSend");
        recv = (decltype(recv))dlsym(h, "ncclRecv");
        gstart = (decltype(gstart))dlsym(h, "ncclGroupStart");
        gend = (decltype(gend))dlsym(h, "ncclGroupEnd");
        errstr = (decltype(errstr))dlsym(h, "ncclGetErrorString");
        if (!init || !send || !recv || !gstart || !gend) h = nullptr;
        return h != nullptr;
    }
};

std::mutex g_mu;                 // one multi-GPU sort at a time
std::vector<RankState> g_ranks;  // per rank slot, re-bound when its device changes
Rccl g_rccl;
double g_phase_ms[LABSORT_MULTI_PHASES];
size_t g_sent_bytes = 0;

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int bind_rank(RankState &R, int dev) {
    if (R.dev == dev && R.s) return LABSORT_OK;
    if (R.dev >= 0) {  // device changed: drop the old buffers on their device
        MHIP(hipSetDevice(R.dev));
        for (Buf *b : {&R.keys, &R.recv, &R.out, &R.ws, &R.kmws, &R.small})
            if (b->p) MHIP(hipFree(b->p));
        if (R.s) MHIP(hipStreamDestroy(R.s));
        if (R.ev) MHIP(hipEventDestroy(R.ev));
        R = RankState{};
    }
    MHIP(hipSetDevice(dev));
    MHIP(hipStreamCreateWithFlags(&R.s, hipStreamNonBlocking));
    MHIP(hipEventCreateWithFlags(&R.ev, hipEventDisableTiming));
    R.dev = dev;
    return LABSORT_OK;
}

// run f(r) for every rank on its own host thread (each binds its rank's device)
int for_ranks(int p, const std::function<int(int)> &f) {
    std::vector<int> st(p, LABSORT_OK);
    std::vector<int> hip(p, 0);
    std::vector<std::thread> th;
    th.reserve(p);
    for (int r = 0; r < p; ++r)
        th.emplace_back([&, r] {
            st[r] = f(r);
            hip[r] = t_last_hip;
        });
    for (auto &t : th) t.join();
    for (int r = 0; r < p; ++r)
        if (st[r]) {
            t_last_hip = hip[r];
            return st[r];
        }
    return LABSORT_OK;
}

int exchange_peer(const ExPlan &P, std::vector<RankState> &R) {
    const int p = P.p;
    for (int i = 0; i < p; ++i) {
        MHIP(hipSetDevice(R[i].dev));
        const uint32_t *src = static_cast<const uint32_t *>(R[i].keys.p);
        for (int j = 0; j < p; ++j) {
            const size_t c = P.count(i, j);
            if (!c) continue;
            uint32_t *dst = static_cast<uint32_t *>(R[j].recv.p) + P.roff(j, i);
            MHIP(hipMemcpyPeerAsync(dst, R[j].dev, src + P.cut[(size_t)i * (p + 1) + j], R[i].dev, c * 4, R[i].s));
        }
        MHIP(hipEventRecord(R[i].ev, R[i].s));
    }
    for (int j = 0; j < p; ++j) {
        MHIP(hipSetDevice(R[j].dev));
        for (int i = 0; i < p; ++i)
            if (i != j) MHIP(hipStreamWaitEvent(R[j].s, R[i].ev, 0));
    }
    return LABSORT_OK;
}

int exchange_rccl(const ExPlan &P, std::vector<RankState> &R) {
    const int p = P.p;
    std::vector<int> devs(p);
    for (int r = 0; r < p; ++r) devs[r] = R[r].dev;
    if (g_rccl.devs != devs) {
        g_rccl.comms.assign(p, nullptr);
        if (g_rccl.init(g_rccl.comms.data(), p, devs.data()) != ncclSuccess) return LABSORT_ERR_HIP;
        g_rccl.devs = devs;
    }
    for (int i = 0; i < p && p > 1; ++i) {  // the piece a rank keeps: a local copy
        const size_t c = P.count(i, i);
        if (!c) continue;
        MHIP(hipSetDevice(R[i].dev));
        MHIP(hipMemcpyAsync(static_cast<uint32_t *>(R[i].recv.p) + P.roff(i, i),
                            static_cast<const uint32_t *>(R[i].keys.p) + P.cut[(size_t)i * (p + 1) + i], c * 4,
                            hipMemcpyDeviceToDevice, R[i].s));
    }
    if (g_rccl.gstart() != ncclSuccess) return LABSORT_ERR_HIP;
    int bad = 0;
    // (one rank: the send to itself goes through RCCL too -- the 1-GPU check of this path)
    for (int i = 0; i < p && !bad; ++i) {
        for (int j = 0; j < p && !bad; ++j) {
            if (j == i && p > 1) continue;
            const size_t cs = P.count(i, j), cr = P.count(j, i);
            if (cs && g_rccl.send(static_cast<const uint32_t *>(R[i].keys.p) + P.cut[(size_t)i * (p + 1) + j], cs,
                                  ncclUint32, j, g_rccl.comms[i], R[i].s) != ncclSuccess)
                bad = 1;
            if (cr && g_rccl.recv(static_cast<uint32_t *>(R[i].recv.p) + P.roff(i, j), cr, ncclUint32, j,
                                  g_rccl.comms[i], R[i].s) != ncclSuccess)
                bad = 1;
        }
    }
    if (g_rccl.gend() != ncclSuccess || bad) return LABSORT_ERR_HIP;
    return LABSORT_OK;
}

int sort_ranks(uint32_t *h, size_t n, int key_type, int p, const int *devices, int transport) {
    const uint32_t flip = key_type == LABSORT_KEY_I32 ? 0x80000000u : 0u;
    int ndev = 0;
    MHIP(hipGetDeviceCount(&ndev));
    std::vector<int> devs(p);
    bool distinct = true;
    for (int r = 0; r < p; ++r) {
        devs[r] = devices ? devices[r] : r;
        if (devs[r] < 0 || devs[r] >= ndev) return LABSORT_ERR_ARG;
        for (int q = 0; q < r; ++q) distinct = distinct && devs[q] != devs[r];
    }
    if (transport == LABSORT_XFER_AUTO) transport = (distinct && p > 1) ? LABSORT_XFER_RCCL : LABSORT_XFER_PEER;
    if (transport == LABSORT_XFER_RCCL && !distinct) return LABSORT_ERR_ARG;  // RCCL: one rank per device
    if (transport == LABSORT_XFER_RCCL && !g_rccl.load()) return LABSORT_ERR_HIP;
    if ((int)g_ranks.size() < p) g_ranks.resize(p);
    std::vector<RankState> &R = g_ranks;
    for (int r = 0; r < p; ++r)
        if (int st = bind_rank(R[r], devs[r])) return st;
    if (transport == LABSORT_XFER_PEER) {
        for (int a = 0; a < p; ++a)
            for (int b = 0; b < p; ++b) {
                if (devs[a] == devs[b]) continue;
                int can = 0;
                MHIP(hipDeviceCanAccessPeer(&can, devs[a], devs[b]));
                if (!can) continue;
                MHIP(hipSetDevice(devs[a]));
                const hipError_t e = hipDeviceEnablePeerAccess(devs[b], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) MHIP(e);
                (void)hipGetLastError();
            }
    }
    ExPlan P;
    P.p = p;
    P.m.resize(p);
    std::vector<size_t> off(p + 1);
    for (int r = 0; r <= p; ++r) off[r] = (size_t)((unsigned __int128)n * r / p);
    for (int r = 0; r < p; ++r) P.m[r] = off[r + 1] - off[r];
    const size_t s = samples_per_rank(p);
    std::vector<std::vector<uint32_t>> samples(p, std::vector<uint32_t>(s));
    std::vector<double> t_h2d(p, 0), t_sort(p, 0);
    for (int i = 0; i < LABSORT_MULTI_PHASES; ++i) g_phase_ms[i] = 0;
    double t0 = now_ms();

    // 1. H2D + local sort + sample, one host thread per rank
    int st = for_ranks(p, [&](int r) -> int {
        RankState &Q = R[r];
        const size_t m = P.m[r];
        MHIP(hipSetDevice(Q.dev));
        if (!m) return LABSORT_OK;
        if (int e = grow(Q.keys, m * 4)) return e;
        const size_t wsb = labsort_workspace_bytes(m, LABSORT_ALGO_AUTO);
        if (int e = grow(Q.ws, wsb)) return e;
        if (int e = grow(Q.small, std::max(s, (size_t)4 * p) * 4)) return e;
        const double a = now_ms();
        MHIP(hipMemcpyAsync(Q.keys.p, h + off[r], m * 4, hipMemcpyHostToDevice, Q.s));
        MHIP(hipStreamSynchronize(Q.s));
        const double b = now_ms();
        if (int e = labsort_sort_device(Q.keys.p, Q.keys.p, m, key_type, LABSORT_ALGO_AUTO, Q.ws.p, Q.ws.bytes, Q.s))
            return e;
        if (int e = labsort_workspace_status(Q.ws.p, m, LABSORT_ALGO_AUTO, Q.s)) return e;  // synchronises
        t_h2d[r] = b - a;
        t_sort[r] = now_ms() - b;
        k_sample<<<(unsigned)((s + 255) / 256), 256, 0, Q.s>>>(static_cast<const uint32_t *>(Q.keys.p), m, (uint32_t)s,
                                                               static_cast<uint32_t *>(Q.small.p));
        MHIP(hipGetLastError());
        MHIP(hipMemcpyAsync(samples[r].data(), Q.small.p, s * 4, hipMemcpyDeviceToHost, Q.s));
        MHIP(hipStreamSynchronize(Q.s));
        return LABSORT_OK;
    });
    if (st) return st;
    double t1 = now_ms();
    g_phase_ms[0] = *std::max_element(t_h2d.begin(), t_h2d.end());
    g_phase_ms[1] = *std::max_element(t_sort.begin(), t_sort.end());

    // 2-3. splitters and cut points
    if (p > 1) {
        const std::vector<Splitter> spl = choose_splitters(p, P.m, samples, flip);
        // every rank's bound queries at once, one host thread per rank
        const std::vector<uint32_t> vals = plan_values(spl, p, flip);
        std::vector<std::vector<uint32_t>> bounds(p, std::vector<uint32_t>(vals.size(), 0u));
        st = for_ranks(p, [&](int r) -> int {
            RankState &Q = R[r];
            if (!P.m[r]) return LABSORT_OK;
            MHIP(hipSetDevice(Q.dev));
            uint32_t *d = static_cast<uint32_t *>(Q.small.p);
            MHIP(hipMemcpyAsync(d, vals.data(), vals.size() * 4, hipMemcpyHostToDevice, Q.s));
            MHIP(launch_upper_bound(static_cast<const uint32_t *>(Q.keys.p), P.m[r], flip, d, vals.size(),
                                    d + vals.size(), Q.s));
            MHIP(hipMemcpyAsync(bounds[r].data(), d + vals.size(), vals.size() * 4, hipMemcpyDeviceToHost, Q.s));
            MHIP(hipStreamSynchronize(Q.s));
            return LABSORT_OK;
        });
        if (st) return st;
        st = make_plan(P, spl, flip, [&](int r, const std::vector<uint32_t> &, std::vector<uint32_t> &out) -> int {
            out = bounds[r];
            return LABSORT_OK;
        });
        if (st) return st;
    } else {
        make_plan(P, {}, flip, nullptr);
    }
    for (int j = 0; j < p; ++j)
        if (P.total(j) > 0x7FFFFFFFu) return LABSORT_ERR_ARG;  // one rank's range beyond a device merge
    double t2 = now_ms();
    g_phase_ms[2] = t2 - t1;

    // 4. exchange into the receive buffers
    {  // the most key bytes one rank sends to its peers (the xGMI volume per link set)
        size_t worst = 0;
        for (int i = 0; i < p; ++i) {
            size_t b = 0;
            for (int j = 0; j < p; ++j)
                if (j != i) b += P.count(i, j) * 4;
            worst = std::max(worst, b);
        }
        g_sent_bytes = worst;
    }
    for (int j = 0; j < p; ++j) {
        MHIP(hipSetDevice(R[j].dev));
        if (int e = grow(R[j].recv, P.total(j) * 4)) return e;
        if (int e = grow(R[j].out, P.total(j) * 4)) return e;
        if (int e = grow(R[j].kmws, labsort_merge_runs_workspace_bytes(P.total(j)))) return e;
    }
    const bool direct = p == 1 && transport != LABSORT_XFER_RCCL;  // one rank: nothing to exchange
    st = direct ? LABSORT_OK : transport == LABSORT_XFER_RCCL ? exchange_rccl(P, R) : exchange_peer(P, R);
    if (st) return st;
    for (int j = 0; j < p; ++j) {
        MHIP(hipSetDevice(R[j].dev));
        MHIP(hipStreamSynchronize(R[j].s));
    }
    double t3 = now_ms();
    g_phase_ms[3] = t3 - t2;

    // 5. K-way merge of the received runs, D2H of each range to its global offset
    std::vector<size_t> goff(p + 1, 0);
    for (int j = 0; j < p; ++j) goff[j + 1] = goff[j] + P.total(j);
    std::vector<double> t_merge(p, 0), t_d2h(p, 0);
    st = for_ranks(p, [&](int j) -> int {
        RankState &Q = R[j];
        const size_t tot = P.total(j);
        MHIP(hipSetDevice(Q.dev));
        if (!tot) return LABSORT_OK;
        const double a = now_ms();
        const uint32_t *res;
        if (direct) {
            res = static_cast<const uint32_t *>(Q.keys.p);
        } else {
            std::vector<size_t> o(P.recv_off.begin() + (size_t)j * (p + 1), P.recv_off.begin() + (size_t)(j + 1) * (p + 1));
            if (int e = labsort_merge_runs(Q.recv.p, Q.out.p, o.data(), p, key_type, Q.kmws.p, Q.kmws.bytes, Q.s))
                return e;
            res = static_cast<const uint32_t *>(Q.out.p);
        }
        MHIP(hipStreamSynchronize(Q.s));
        const double b = now_ms();
        MHIP(hipMemcpyAsync(h + goff[j], res, tot * 4, hipMemcpyDeviceToHost, Q.s));
        MHIP(hipStreamSynchronize(Q.s));
        t_merge[j] = b - a;
        t_d2h[j] = now_ms() - b;
        return LABSORT_OK;
    });
    if (st) return st;
    g_phase_ms[4] = *std::max_element(t_merge.begin(), t_merge.end());
    g_phase_ms[5] = *std::max_element(t_d2h.begin(), t_d2h.end());
    g_phase_ms[6] = now_ms() - t0;
    return LABSORT_OK;
}

}  // namespace
}  // namespace labsort

using namespace labsort;

extern "C" {

int labsort_sort_host_ranks(void *h_keys, size_t n, int key_type, int nranks, const int *devices, int transport) {
    if (nranks < 1 || nranks > LABSORT_MULTI_MAX_RANKS) return LABSORT_ERR_ARG;
    if (key_type != LABSORT_KEY_U32 && key_type != LABSORT_KEY_I32) return LABSORT_ERR_ARG;
    if (transport != LABSORT_XFER_AUTO && transport != LABSORT_XFER_RCCL && transport != LABSORT_XFER_PEER)
        return LABSORT_ERR_ARG;
    if (n == 0) return LABSORT_OK;
    if (!h_keys) return LABSORT_ERR_ARG;
    if ((n + nranks - 1) / nranks > labsort_max_keys(LABSORT_ALGO_RADIX)) return LABSORT_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) cur = 0;
    const int st = sort_ranks(static_cast<uint32_t *>(h_keys), n, key_type, nranks, devices, transport);
    const int hip = t_last_hip;
    (void)hipSetDevice(cur);
    t_last_hip = hip;
    return st;
}

int labsort_sort_host_multi(void *h_keys, size_t n, int key_type, int ngpus) {
    return labsort_sort_host_ranks(h_keys, n, key_type, ngpus, nullptr, LABSORT_XFER_AUTO);
}

int labsort_multi_last_hip_error(void) { return t_last_hip; }

int labsort_multi_timing(double *phase_ms, int nphases, size_t *max_sent_bytes) {
    if (!phase_ms || nphases < 0 || nphases > LABSORT_MULTI_PHASES) return LABSORT_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    for (int i = 0; i < nphases; ++i) phase_ms[i] = g_phase_ms[i];
    if (max_sent_bytes) *max_sent_bytes = g_sent_bytes;
    return LABSORT_OK;
}

int labsort_multi_plan(const uint32_t *const *h_shards, const size_t *m, int nranks, int key_type,
                       size_t *h_cuts) {
    if (nranks < 1 || nranks > LABSORT_MULTI_MAX_RANKS || !h_shards || !m || !h_cuts) return LABSORT_ERR_ARG;
    const uint32_t flip = key_type == LABSORT_KEY_I32 ? 0x80000000u : 0u;
    const int p = nranks;
    ExPlan P;
    P.p = p;
    P.m.assign(m, m + p);
    const size_t s = samples_per_rank(p);
    std::vector<std::vector<uint32_t>> samples(p, std::vector<uint32_t>(s));
    size_t total = 0;
    for (int r = 0; r < p; ++r) {
        total += m[r];
        if (m[r] && !h_shards[r]) return LABSORT_ERR_ARG;
        for (size_t k = 0; m[r] && k < s; ++k) samples[r][k] = h_shards[r][sample_pos(m[r], s, k)];
    }
    int st = LABSORT_OK;
    if (p > 1 && total) {
        const std::vector<Splitter> spl = choose_splitters(p, P.m, samples, flip);
        st = make_plan(P, spl, flip, [&](int r, const std::vector<uint32_t> &vals, std::vector<uint32_t> &out) -> int {
            const uint32_t *a = h_shards[r];
            for (size_t v = 0; v < vals.size(); ++v)
                out[v] = (uint32_t)(std::upper_bound(a, a + m[r], vals[v] ^ flip,
                                                     [flip](uint32_t x, uint32_t y) { return x < (y ^ flip); }) -
                                    a);
            return LABSORT_OK;
        });
    } else {  // one rank, or no keys: every rank keeps its (empty) shard as its last piece
        P.cut.assign((size_t)p * (p + 1), 0);
        for (int r = 0; r < p; ++r) P.cut[(size_t)r * (p + 1) + p] = m[r];
    }
    if (st) return st;
    std::copy(P.cut.begin(), P.cut.end(), h_cuts);
    return LABSORT_OK;
}

}  // extern "C"
