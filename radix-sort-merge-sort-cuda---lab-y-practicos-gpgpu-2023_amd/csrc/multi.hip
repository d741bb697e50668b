// multi.hip -- the merge-sort path across GPUs (the
// reference is single-GPU: lab.cu:303-402).  The schedule itself is dist_plan.h's
// dist::sort_rank, written once; this file supplies its HIP rank operations and three
// communicators, and the C-ABI entries that drive them:
//
//   labsort_sort_host_multi / labsort_sort_host_ranks   one process, one host thread per
//       rank (order_array with LABSORT_GPUS=p): rank r copies its shard of the caller's
//       host array over its own PCIe link in chunks while earlier chunks sort, takes part
//       in the exchange (in-process peer copies, or RCCL on communicators from
//       ncclCommInitAll), and copies its merged range back to its global offset in
//       diagonal ranges as each lands;
//   labsort_dist_sort on a labsort_comm_t               one process per GPU (bench.py
//       --gpus N under torch.distributed.run): device-resident shard in, this rank's
//       range of the sorted array out; RCCL communicator from ncclCommInitRank
//       (labsort_comm_init_rccl), or host-staged callbacks (labsort_comm_init_host: the
//       tests run several ranks on one GPU over torch.distributed gloo).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/labsort.h"
#include "common.h"
#include "dist_plan.h"

namespace labsort {
namespace {

// ---------------------------------------------------------------------------------
// errors: the HIP code of the failing call (per thread) and a detail message
// ---------------------------------------------------------------------------------
thread_local int t_last_hip = 0;
std::mutex g_err_mu;
std::string g_detail;  // last failure of a multi-GPU call, human readable

void set_detail(const std::string &s) {
    std::lock_guard<std::mutex> lk(g_err_mu);
    g_detail = s;
}

#define MHIP(x)                                                                                    \
    do {                                                                                           \
        hipError_t _e = (x);                                                                       \
        if (_e != hipSuccess) {                                                                    \
            t_last_hip = (int)_e;                                                                  \
            set_detail(std::string(#x) + ": " + hipGetErrorString(_e));                            \
            return LABSORT_ERR_HIP;                                                                \
        }                                                                                          \
    } while (0)
// a labsort_* call: an ERR_HIP it returns recorded its code in api.hip's thread-local slot
#define LCALL(x)                                                                                   \
    do {                                                                                           \
        const int _s = (x);                                                                        \
        if (_s != LABSORT_OK) {                                                                    \
            if (_s == LABSORT_ERR_HIP) {                                                           \
                t_last_hip = labsort_last_hip_error();                                             \
                set_detail(std::string(#x) + ": " + hipGetErrorString((hipError_t)t_last_hip));    \
            } else {                                                                               \
                set_detail(std::string(#x) + ": " + labsort_error_string(_s));                     \
            }                                                                                      \
            return _s;                                                                             \
        }                                                                                          \
    } while (0)

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

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
template <class T>
T *as(Buf &b) {
    return static_cast<T *>(b.p);
}

__global__ void k_sample(const uint32_t *__restrict__ keys, uint64_t m, uint32_t s, uint32_t *__restrict__ out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < s) out[k] = keys[(uint64_t)k * m / s];  // = dist::sample_pos (k * m < 2^42)
}

// ---------------------------------------------------------------------------------
// one rank's device state (persistent across calls) and its HIP operations
// ---------------------------------------------------------------------------------
constexpr int RANK_CHUNKS = 8;   // host input: shard copied and sorted in chunks
constexpr int RANK_RANGES = 8;   // host output: the last merge level in diagonal ranges, D2H per range
constexpr size_t RANK_PIPE_MIN = (size_t)1 << 24;  // keys per rank from which the host input is chunked

// LABSORT_HOST_PIPE: "0" never chunk, "1" from 2^16 keys per rank (tests), unset RANK_PIPE_MIN
size_t rank_pipe_min() {
    const char *e = std::getenv("LABSORT_HOST_PIPE");
    if (e && !std::strcmp(e, "0")) return ~(size_t)0;
    if (e && !std::strcmp(e, "1")) return (size_t)1 << 16;
    return RANK_PIPE_MIN;
}

enum { EV_H2D = dist::M_NMARKS, EV_D2H, EV_NEV };

struct RankState {
    int dev = -1;
    hipStream_t own = nullptr, copy = nullptr;  // own compute stream (in-process ranks), copy stream
    // the plan's small launches (samples, bounds), at the highest stream priority: the
    // runtime gives each priority its own hardware queues, so when several ranks share a
    // GPU they do not wait in a queue behind another rank's queued sort or merge kernels
    hipStream_t plan = nullptr;
    hipEvent_t chunk_ev[RANK_CHUNKS] = {}, range_ev[RANK_RANGES] = {};
    hipEvent_t tev[EV_NEV] = {};  // timing: schedule marks, end of H2D, end of D2H
    Buf x, y, ws, mws, recv, out, small, part, errs;
    int nerrs = 0;
    uint32_t *pin = nullptr;  // pinned host staging of the plan's small copies (samples, bounds)
    size_t pin_words = 0;
};

// the rank's pinned staging, at least `words` long (DMA copies instead of pageable staging)
int grow_pin(RankState &R, size_t words) {
    if (R.pin && R.pin_words >= words) return LABSORT_OK;
    if (R.pin) MHIP(hipHostFree(R.pin));
    R.pin = nullptr;
    R.pin_words = 0;
    const size_t want = std::max(words, (size_t)4096);
    MHIP(hipHostMalloc(reinterpret_cast<void **>(&R.pin), want * 4, hipHostMallocDefault));
    R.pin_words = want;
    return LABSORT_OK;
}

int bind_rank(RankState &R, int dev) {
    if (R.dev == dev && R.own) return LABSORT_OK;
    if (R.dev >= 0) {  // device changed: drop the old buffers on their device
        MHIP(hipSetDevice(R.dev));
        for (Buf *b : {&R.x, &R.y, &R.ws, &R.mws, &R.recv, &R.out, &R.small, &R.part, &R.errs})
            if (b->p) MHIP(hipFree(b->p));
        for (hipStream_t s : {R.own, R.copy, R.plan})
            if (s) MHIP(hipStreamDestroy(s));
        for (hipEvent_t e : R.chunk_ev)
            if (e) MHIP(hipEventDestroy(e));
        for (hipEvent_t e : R.range_ev)
            if (e) MHIP(hipEventDestroy(e));
        for (hipEvent_t e : R.tev)
            if (e) MHIP(hipEventDestroy(e));
        if (R.pin) MHIP(hipHostFree(R.pin));
        R = RankState{};
    }
    MHIP(hipSetDevice(dev));
    MHIP(hipStreamCreateWithFlags(&R.own, hipStreamNonBlocking));
    MHIP(hipStreamCreateWithFlags(&R.copy, hipStreamNonBlocking));
    int least = 0, greatest = 0;
    MHIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    MHIP(hipStreamCreateWithPriority(&R.plan, hipStreamNonBlocking, greatest));
    for (hipEvent_t &e : R.chunk_ev) MHIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t &e : R.range_ev) MHIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t &e : R.tev) MHIP(hipEventCreate(&e));
    R.dev = dev;
    return LABSORT_OK;
}

// dist::sort_rank's Ops on one GPU.  host_in: `in` is a host address (the caller's
// array); otherwise a device address.
struct HipRankOps {
    RankState &R;
    hipStream_t s;
    int key_type;
    bool host_in;
    uint32_t flip() const { return key_type == LABSORT_KEY_I32 ? 0x80000000u : 0u; }

    void mark(dist::Mark k) { (void)hipEventRecord(R.tev[k], s); }
    int wait_sorted() {
        MHIP(hipEventSynchronize(R.tev[dist::M_SORTED]));
        return LABSORT_OK;
    }

    // sort one piece in -> out (device) with the workspace; its radix error word copied aside
    int sort_piece(const uint32_t *in, uint32_t *out, size_t len) {
        const int algo = LABSORT_ALGO_AUTO;
        LCALL(labsort_sort_device(in, out, len, key_type, algo, R.ws.p, R.ws.bytes, s));
        // every layout but the one-tile sort's starts with a device error word (radix: a
        // look-back spin that expired; merge: a four-way block with inconsistent cuts)
        if (R.nerrs < RANK_CHUNKS && len > labsort_tile_keys())
            MHIP(hipMemcpyAsync(as<uint32_t>(R.errs) + R.nerrs++, R.ws.p, 4, hipMemcpyDeviceToDevice, s));
        return LABSORT_OK;
    }

    int local_sort(const uint32_t *in, uint64_t m, const uint32_t **sorted) {
        int st;
        R.nerrs = 0;
        if ((st = grow(R.errs, RANK_CHUNKS * 4))) return st;
        MHIP(hipMemsetAsync(R.errs.p, 0, RANK_CHUNKS * 4, s));
        if ((st = grow(R.x, m * 4)) || (st = grow(R.y, m * 4))) return st;
        uint32_t *X = as<uint32_t>(R.x), *Y = as<uint32_t>(R.y);
        if (!m) {
            *sorted = X;
            if (host_in) MHIP(hipEventRecord(R.tev[EV_H2D], s));
            return LABSORT_OK;
        }
        if (!host_in) {  // device-resident shard: one sort into X
            if ((st = grow(R.ws, labsort_workspace_bytes(m, LABSORT_ALGO_AUTO)))) return st;
            if ((st = sort_piece(in, X, m))) return st;
            *sorted = X;
            return LABSORT_OK;
        }
        // host shard: chunk i copied H2D into X on the copy stream while the compute stream
        // sorts the chunks that have landed (X -> Y); then the chunk runs merged Y -> X
        const int K = m >= rank_pipe_min() ? RANK_CHUNKS : 1;
        const size_t c = (m + K - 1) / K;
        if ((st = grow(R.ws, labsort_workspace_bytes(c, LABSORT_ALGO_AUTO)))) return st;
        MHIP(hipEventRecord(R.tev[dist::M_START], s));  // the copy stream starts after the zeroed error words
        MHIP(hipStreamWaitEvent(R.copy, R.tev[dist::M_START], 0));
        size_t off[RANK_CHUNKS + 1];
        int nr = 0;
        for (int i = 0; i < K; ++i) {
            const size_t o = (size_t)i * c;
            if (o >= m) break;
            const size_t len = std::min(c, (size_t)m - o);
            off[nr++] = o;
            MHIP(hipMemcpyAsync(X + o, in + o, len * 4, hipMemcpyHostToDevice, R.copy));
            MHIP(hipEventRecord(R.chunk_ev[i], R.copy));
            MHIP(hipStreamWaitEvent(s, R.chunk_ev[i], 0));
            if ((st = sort_piece(X + o, (nr == 1 && K == 1) ? X + o : Y + o, len))) return st;
        }
        MHIP(hipEventRecord(R.tev[EV_H2D], R.copy));
        off[nr] = m;
        if (nr == 1 && K == 1) {
            *sorted = X;
            return LABSORT_OK;
        }
        if ((st = grow(R.mws, labsort_merge_runs_workspace_bytes(m)))) return st;
        LCALL(labsort_merge_runs(Y, X, off, nr, key_type, R.mws.p, R.mws.bytes, s));
        *sorted = X;
        return LABSORT_OK;
    }

    int sample(const uint32_t *S, uint64_t m, size_t n, uint32_t *h_out) {
        int st;
        if ((st = grow(R.small, std::max(n, (size_t)4096) * 4))) return st;
        if ((st = grow_pin(R, n))) return st;
        MHIP(hipStreamWaitEvent(R.plan, R.tev[dist::M_SORTED], 0));  // after the local sort
        k_sample<<<(unsigned)((n + 255) / 256), 256, 0, R.plan>>>(S, m, (uint32_t)n, as<uint32_t>(R.small));
        MHIP(hipGetLastError());
        MHIP(hipMemcpyAsync(R.pin, R.small.p, n * 4, hipMemcpyDeviceToHost, R.plan));
        MHIP(hipStreamSynchronize(R.plan));
        memcpy(h_out, R.pin, n * 4);
        return LABSORT_OK;
    }

    int bounds(const uint32_t *S, uint64_t m, const uint32_t *h_vals, size_t nv, uint32_t *h_out) {
        int st;
        if (!nv) return LABSORT_OK;
        if ((st = grow(R.small, std::max(2 * nv, (size_t)4096) * 4))) return st;
        if ((st = grow_pin(R, 2 * nv))) return st;
        uint32_t *d = as<uint32_t>(R.small);
        memcpy(R.pin, h_vals, nv * 4);
        MHIP(hipStreamWaitEvent(R.plan, R.tev[dist::M_SORTED], 0));  // after the local sort
        MHIP(hipMemcpyAsync(d, R.pin, nv * 4, hipMemcpyHostToDevice, R.plan));
        LCALL(labsort_upper_bound(S, m, key_type, d, nv, d + nv, R.plan));
        MHIP(hipMemcpyAsync(R.pin + nv, d + nv, nv * 4, hipMemcpyDeviceToHost, R.plan));
        MHIP(hipStreamSynchronize(R.plan));
        memcpy(h_out, R.pin + nv, nv * 4);
        return LABSORT_OK;
    }

    int recv_buffer(uint64_t total, uint32_t **recv) {
        int st;
        if ((st = grow(R.recv, total * 4)) || (st = grow(R.out, total * 4)) ||
            (st = grow(R.mws, labsort_merge_runs_workspace_bytes(total))) ||
            (st = grow(R.part, labsort_merge_parts((total + RANK_RANGES - 1) / RANK_RANGES) * 4)))
            return st;
        *recv = as<uint32_t>(R.recv);
        return LABSORT_OK;
    }

    int copy_local(uint32_t *dst, const uint32_t *src, uint64_t count) {
        MHIP(hipMemcpyAsync(dst, src, count * 4, hipMemcpyDeviceToDevice, s));
        return LABSORT_OK;
    }

    int to_host(const uint32_t *src, uint64_t count, uint32_t *h_dst) {
        MHIP(hipEventRecord(R.range_ev[0], s));
        MHIP(hipStreamWaitEvent(R.copy, R.range_ev[0], 0));
        MHIP(hipMemcpyAsync(h_dst, src, count * 4, hipMemcpyDeviceToHost, R.copy));
        MHIP(hipEventRecord(R.tev[EV_D2H], R.copy));
        return LABSORT_OK;
    }

    // the p received runs (rank order) merged: the first and second halves of the runs
    // by labsort_merge_runs (pair passes) into `out`, then the two halves merged back
    // into `recv` as RANK_RANGES diagonal ranges, each range's D2H (h_sink) on the copy
    // stream as soon as it lands
    int merge(const uint32_t *Rv, const uint64_t *offs, int p, uint32_t *h_sink, const uint32_t **result) {
        const size_t total = offs[p];
        uint32_t *recv = const_cast<uint32_t *>(Rv), *O = as<uint32_t>(R.out);
        if (p == 1 || total == 0) {
            *result = recv;
            return h_sink && total ? to_host(recv, total, h_sink) : LABSORT_OK;
        }
        const int h = (p + 1) / 2;
        auto half = [&](int q0, int q1) -> int {  // runs [q0, q1) -> O
            const size_t b = offs[q0], e = offs[q1];
            if (e == b) return LABSORT_OK;
            if (q1 - q0 == 1) {
                MHIP(hipMemcpyAsync(O + b, recv + b, (e - b) * 4, hipMemcpyDeviceToDevice, s));
                return LABSORT_OK;
            }
            std::vector<size_t> o(offs + q0, offs + q1 + 1);  // (q1 - q0 <= 8: LABSORT_DIST_MAX_RANKS)
            LCALL(labsort_merge_runs(recv, O, o.data(), q1 - q0, key_type, R.mws.p, R.mws.bytes, s));
            return LABSORT_OK;
        };
        int st;
        if ((st = half(0, h)) || (st = half(h, p))) return st;
        const size_t la = offs[h], lb = total - la, rl = (total + RANK_RANGES - 1) / RANK_RANGES;
        for (int q = 0; q < RANK_RANGES; ++q) {
            const size_t d0 = (size_t)q * rl, d1 = std::min(total, d0 + rl);
            if (d0 >= d1) break;
            LCALL(labsort_merge(O, la, O + la, lb, recv + d0, d0, d1, key_type, as<uint32_t>(R.part), s));
            if (h_sink) {
                MHIP(hipEventRecord(R.range_ev[q], s));
                MHIP(hipStreamWaitEvent(R.copy, R.range_ev[q], 0));
                MHIP(hipMemcpyAsync(h_sink + d0, recv + d0, (d1 - d0) * 4, hipMemcpyDeviceToHost, R.copy));
            }
        }
        if (h_sink) MHIP(hipEventRecord(R.tev[EV_D2H], R.copy));
        *result = recv;
        return LABSORT_OK;
    }

    // after the schedule: wait for both streams, then the sorts' device error words
    int finish() {
        MHIP(hipStreamSynchronize(s));
        MHIP(hipStreamSynchronize(R.copy));
        if (R.nerrs) {
            uint32_t e[RANK_CHUNKS] = {};
            MHIP(hipMemcpy(e, R.errs.p, R.nerrs * 4, hipMemcpyDeviceToHost));
            for (int i = 0; i < R.nerrs; ++i)
                if (e[i]) {
                    set_detail("a sort kernel reported a device-side error (radix look-back spin limit or merge block cuts)");
                    return LABSORT_ERR_DEVICE;
                }
        }
        return LABSORT_OK;
    }

    // phases (ms, device timeline) of the call just finished; the plan's work and wait from
    // the host times at its collectives
    void phases(double *ph, bool host, const dist::Result &res) {
        auto el = [&](hipEvent_t a, hipEvent_t b) {
            float ms = 0.f;
            return hipEventElapsedTime(&ms, a, b) == hipSuccess ? (double)ms : 0.0;
        };
        ph[0] = host ? el(R.tev[dist::M_START], R.tev[EV_H2D]) : 0.0;
        ph[1] = el(R.tev[dist::M_START], R.tev[dist::M_SORTED]);
        ph[2] = el(R.tev[dist::M_SORTED], R.tev[dist::M_PLANNED]);
        ph[3] = el(R.tev[dist::M_PLANNED], R.tev[dist::M_EXCHANGED]);
        ph[4] = el(R.tev[dist::M_EXCHANGED], R.tev[dist::M_MERGED]);
        ph[5] = host ? el(R.tev[dist::M_MERGED], R.tev[EV_D2H]) : 0.0;
        double wait = 0.0;
        for (int k = 0; k < dist::C_NCOLL; ++k)
            if (res.arrive[k] >= 0.0) wait += res.leave[k] - res.arrive[k];
        ph[8] = wait;
        const double span = res.plan_host[1] - res.plan_host[0];  // host clock, as the waits
        ph[7] = span > wait ? span - wait : 0.0;
    }
};

// ---------------------------------------------------------------------------------
// RCCL, loaded on first use (no link-time dependency; in a torch process the
// already-loaded librccl.so.1 is the one dlopen returns)
// ---------------------------------------------------------------------------------
struct Rccl {
    bool tried = false;
    void *h = nullptr;
    decltype(&ncclGetUniqueId) uid = nullptr;
    decltype(&ncclCommInitRankConfig) init_rank_cfg = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclCommFinalize) finalize = nullptr;  // optional: older RCCL lacks it
    decltype(&ncclCommAbort) abort = nullptr;
    decltype(&ncclCommGetAsyncError) async_err = nullptr;
    decltype(&ncclAllGather) allgather = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) gstart = nullptr;
    decltype(&ncclGroupEnd) gend = nullptr;
    decltype(&ncclGetErrorString) errstr = nullptr;
    bool load() {
        static std::mutex mu;
        std::lock_guard<std::mutex> lk(mu);
        if (tried) return h != nullptr;
        tried = true;
        h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            set_detail("RCCL: librccl.so could not be loaded");
            return false;
        }
        uid = (decltype(uid))dlsym(h, "ncclGetUniqueId");
        init_rank_cfg = (decltype(init_rank_cfg))dlsym(h, "ncclCommInitRankConfig");
        destroy = (decltype(destroy))dlsym(h, "ncclCommDestroy");
        finalize = (decltype(finalize))dlsym(h, "ncclCommFinalize");
        abort = (decltype(abort))dlsym(h, "ncclCommAbort");
        async_err = (decltype(async_err))dlsym(h, "ncclCommGetAsyncError");
        allgather = (decltype(allgather))dlsym(h, "ncclAllGather");
        send = (decltype(send))dlsym(h, "ncclSend");
        recv = (decltype(recv))dlsym(h, "ncclRecv");
        gstart = (decltype(gstart))dlsym(h, "ncclGroupStart");
        gend = (decltype(gend))dlsym(h, "ncclGroupEnd");
        errstr = (decltype(errstr))dlsym(h, "ncclGetErrorString");
        if (!uid || !init_rank_cfg || !destroy || !abort || !async_err || !allgather || !send || !recv || !gstart ||
            !gend) {
            set_detail("RCCL: a symbol is missing from librccl.so");
            h = nullptr;
        }
        return h != nullptr;
    }
    // record an ncclResult as the call's failure detail
    int fail(const char *what, ncclResult_t r) {
        set_detail(std::string("RCCL ") + what + ": " + (errstr ? errstr(r) : "error") + " (ncclResult " +
                   std::to_string((int)r) + ")");
        t_last_hip = 0;
        return LABSORT_ERR_HIP;
    }
};
Rccl g_rccl;

#define NCHK(what, x)                                        \
    do {                                                     \
        const ncclResult_t _r = (x);                         \
        if (_r != ncclSuccess) return g_rccl.fail(what, _r); \
    } while (0)

// ---------------------------------------------------------------------------------
// Bounded waits on RCCL.  Communicators are created nonblocking (ncclConfig_t
// blocking = 0), so no RCCL call blocks the host: a call may return ncclInProgress and
// the communicator is then polled (ncclCommGetAsyncError) until it settles, and a stream
// carrying RCCL work is polled (hipStreamQuery) instead of synchronised.  Both polls
// end at the communicator's deadline, or at once when an in-process peer reports a
// failure: a rank whose peer never arrives -- its transport broke, or it left -- then
// returns LABSORT_ERR_PEER instead of blocking forever, and its caller aborts the
// communicator (ncclCommAbort), which stops its kernels and proxy thread.  (The
// reference ends the process on any CUDA error, utils.h:18-26; here a failure ends every
// rank's call and leaves the process usable.)
// ---------------------------------------------------------------------------------
constexpr double COMM_TIMEOUT_MS = 1000.0 * LABSORT_COMM_TIMEOUT_S;

void poll_pause(double t0) {
    if (now_ms() - t0 < 2.0) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(50));
}
int peer_gone(const char *what, const char *why) {
    set_detail(std::string("RCCL ") + what + ": " + why + " (the communicator is aborted)");
    t_last_hip = 0;
    return LABSORT_ERR_PEER;
}
// the communicator's pending host-side work done (after a call that returned ncclInProgress)
int rccl_settle(ncclComm_t c, double deadline, const char *what, const std::atomic<bool> *peer_failed = nullptr) {
    const double t0 = now_ms();
    for (;;) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t q = g_rccl.async_err(c, &st);
        if (q != ncclSuccess) return g_rccl.fail(what, q);
        if (st == ncclSuccess) return LABSORT_OK;
        if (st != ncclInProgress) return g_rccl.fail(what, st);
        if (peer_failed && peer_failed->load()) return peer_gone(what, "a peer rank failed");
        if (now_ms() > deadline) return peer_gone(what, "timed out waiting for the peers");
        poll_pause(t0);
    }
}
// a nonblocking RCCL call: queued (ncclSuccess / ncclInProgress), then settled
int rccl_call(ncclComm_t c, ncclResult_t r, double deadline, const char *what,
              const std::atomic<bool> *peer_failed = nullptr) {
    if (r != ncclSuccess && r != ncclInProgress) return g_rccl.fail(what, r);
    return rccl_settle(c, deadline, what, peer_failed);
}
// stream s, which carries RCCL work of c, complete (the communicator's errors polled)
int rccl_stream_wait(ncclComm_t c, hipStream_t s, double deadline, const char *what,
                     const std::atomic<bool> *peer_failed = nullptr) {
    const double t0 = now_ms();
    for (;;) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) return LABSORT_OK;
        if (q != hipErrorNotReady) MHIP(q);
        ncclResult_t st = ncclSuccess;
        if (g_rccl.async_err(c, &st) != ncclSuccess || (st != ncclSuccess && st != ncclInProgress))
            return g_rccl.fail(what, st);
        if (peer_failed && peer_failed->load()) return peer_gone(what, "a peer rank failed");
        if (now_ms() > deadline) return peer_gone(what, "timed out waiting for the peers");
        poll_pause(t0);
    }
}
ncclConfig_t nonblocking_config() {
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    return cfg;
}

// Release communicators, the documented teardown of nonblocking ones: ncclCommFinalize on
// each (it returns at once, ncclInProgress), each polled to ncclSuccess by the deadline
// (the peers finalize too), then ncclCommDestroy.  One that does not settle (a peer that
// never finalizes) is aborted instead.  The pointers are cleared.
constexpr double COMM_TEARDOWN_MS = 10000.0;
int rccl_release(ncclComm_t *cs, size_t k, double deadline) {
    int st = LABSORT_OK;
    std::vector<char> fin(k, 0);
    for (size_t i = 0; i < k; ++i)
        if (cs[i] && g_rccl.finalize) {
            const ncclResult_t r = g_rccl.finalize(cs[i]);
            fin[i] = r == ncclSuccess || r == ncclInProgress;
            if (!fin[i] && !st) st = g_rccl.fail("ncclCommFinalize", r);
        }
    for (size_t i = 0; i < k; ++i) {
        if (!cs[i]) continue;
        const int e = fin[i] ? rccl_settle(cs[i], deadline, "ncclCommFinalize") : (g_rccl.finalize ? st : LABSORT_OK);
        if (e || (g_rccl.finalize && !fin[i])) {
            (void)g_rccl.abort(cs[i]);
            if (!st) st = e ? e : LABSORT_ERR_HIP;
        } else {
            const ncclResult_t r = g_rccl.destroy(cs[i]);
            if (r != ncclSuccess && r != ncclInProgress && !st) st = g_rccl.fail("ncclCommDestroy", r);
        }
        cs[i] = nullptr;
    }
    return st;
}

// grouped pairwise send/recv with every peer at once: every xGMI link of the GPU
// carries data together (the "pairwise RCCL send/recv merge" of the north_star).  The
// group is queued whole or not at all (ncclGroupEnd), then settled by the deadline.
int rccl_exchange(ncclComm_t c, int p, int me, hipStream_t s, const uint32_t *const *send, const uint64_t *sc,
                  uint32_t *const *recv, const uint64_t *rc, double deadline,
                  const std::atomic<bool> *peer_failed = nullptr) {
    const ncclResult_t g = g_rccl.gstart();
    if (g != ncclSuccess) return g_rccl.fail("ncclGroupStart", g);
    ncclResult_t bad = ncclSuccess;
    for (int j = 0; j < p && bad == ncclSuccess; ++j) {
        if (j == me) continue;
        if (sc[j]) bad = g_rccl.send(send[j], sc[j], ncclUint32, j, c, s);
        if (bad == ncclSuccess && rc[j]) bad = g_rccl.recv(recv[j], rc[j], ncclUint32, j, c, s);
    }
    const ncclResult_t e = g_rccl.gend();
    if (bad != ncclSuccess && bad != ncclInProgress) return g_rccl.fail("ncclSend/ncclRecv", bad);
    return rccl_call(c, e, deadline, "ncclGroupEnd (exchange)", peer_failed);
}

// ---------------------------------------------------------------------------------
// communicator 1: in-process ranks (one host thread each)
// ---------------------------------------------------------------------------------
struct ThreadShared {
    int p = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    unsigned gen = 0;
    std::atomic<bool> failed{false};
    std::vector<std::vector<uint8_t>> slot;
    std::vector<uint32_t *const *> rptr;  // each rank's receive addresses (during an exchange)
    std::vector<hipEvent_t> sent;          // each rank's "my sends are queued" event
    std::vector<int> dev;
    std::vector<ncclComm_t> comms;         // RCCL transport: one communicator per rank
    double deadline = 0.0;                 // RCCL transport: the call's deadline (now_ms clock)
    explicit ThreadShared(int n) : p(n), slot(n), rptr(n, nullptr), sent(n, nullptr), dev(n, -1) {}

    // all ranks arrive; LABSORT_ERR_PEER if one of them failed without arriving (a rank
    // that failed in its own step still arrives: the schedule's status words report it)
    int barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (failed) return LABSORT_ERR_PEER;
        const unsigned g = gen;
        if (++arrived == p) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return LABSORT_OK;
        }
        cv.wait(lk, [&] { return gen != g || failed; });
        return gen != g ? LABSORT_OK : LABSORT_ERR_PEER;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        failed = true;
        cv.notify_all();
    }
};

struct ThreadComm {
    ThreadShared &sh;
    int me;
    hipStream_t s;
    bool rccl;
    int size() const { return sh.p; }
    int rank() const { return me; }
    int allgather(const void *in, void *out, size_t bytes) {
        int st;
        sh.slot[me].assign(static_cast<const uint8_t *>(in), static_cast<const uint8_t *>(in) + bytes);
        if ((st = sh.barrier())) return st;
        for (int i = 0; i < sh.p; ++i) {
            if (sh.slot[i].size() != bytes) return LABSORT_ERR_ARG;
            memcpy(static_cast<uint8_t *>(out) + (size_t)i * bytes, sh.slot[i].data(), bytes);
        }
        return sh.barrier();  // every rank has read every slot
    }
    int exchange(const uint32_t *const *send, const uint64_t *sc, uint32_t *const *recv, const uint64_t *rc) {
        int st;
        if (rccl) {
            // queued, then waited for here, bounded: the merge that follows issues copies that
            // can block the host behind the stream, where a peer that left would hold it
            // forever (ncclGroupEnd can settle before the peers' kernels have run)
            st = rccl_exchange(sh.comms[me], sh.p, me, s, send, sc, recv, rc, sh.deadline, &sh.failed);
            return st ? st : rccl_stream_wait(sh.comms[me], s, sh.deadline, "exchange", &sh.failed);
        }
        // peer copies straight into each receiver's slot, on the sender's stream; the
        // receivers' streams then wait for every sender's event
        sh.rptr[me] = recv;
        if ((st = sh.barrier())) return st;
        for (int j = 0; j < sh.p; ++j) {
            if (j == me || !sc[j]) continue;
            MHIP(hipMemcpyPeerAsync(sh.rptr[j][me], sh.dev[j], send[j], sh.dev[me], sc[j] * 4, s));
        }
        MHIP(hipEventRecord(sh.sent[me], s));
        if ((st = sh.barrier())) return st;
        for (int i = 0; i < sh.p; ++i)
            if (i != me && rc[i]) MHIP(hipStreamWaitEvent(s, sh.sent[i], 0));
        return sh.barrier();  // the receive addresses are no longer read
    }
    void abandon() { sh.abort(); }  // this rank leaves the exchange: its peers stop waiting now
};

// ---------------------------------------------------------------------------------
// communicator 2: one process per rank over RCCL (ncclCommInitRankConfig, nonblocking)
// communicator 3: host-staged callbacks (tests: torch.distributed gloo)
// ---------------------------------------------------------------------------------
struct RcclState {
    ncclComm_t nc = nullptr;
    bool broken = false;                   // aborted after a transport failure: every later call fails
    double timeout_ms = COMM_TIMEOUT_MS;   // bound of every wait on the peers
    Buf stage;                             // allgather staging, sized at init for the schedule's records
    // abort after a transport failure (the peers' own waits then end at their deadlines)
    void abort() {
        if (nc) (void)g_rccl.abort(nc);
        nc = nullptr;
        broken = true;
    }
};
// largest allgather of dist::sort_rank at p ranks, per rank: the sample record
inline size_t stage_bytes(int p) { return (16 + 4 * dist::samples_per_rank(p)) * (size_t)(p + 1); }

struct RcclComm {
    RcclState &o;
    int p, me;
    hipStream_t s;
    int size() const { return p; }
    int rank() const { return me; }
    int failed(int st) {
        o.abort();
        return st;
    }
    int allgather(const void *in, void *out, size_t bytes) {
        const double deadline = now_ms() + o.timeout_ms;
        if (bytes * (p + 1) > o.stage.bytes) {  // (cannot happen: pre-sized for the schedule's records)
            set_detail("RCCL allgather: record larger than the communicator's staging");
            return failed(LABSORT_ERR_ARG);
        }
        uint8_t *d = as<uint8_t>(o.stage);
        hipError_t h = hipMemcpyAsync(d + bytes * p, in, bytes, hipMemcpyHostToDevice, s);
        if (h != hipSuccess) {
            t_last_hip = (int)h;
            set_detail(std::string("allgather staging: ") + hipGetErrorString(h));
            return failed(LABSORT_ERR_HIP);
        }
        int st = rccl_call(o.nc, g_rccl.allgather(d + bytes * p, d, bytes, ncclUint8, o.nc, s), deadline,
                           "ncclAllGather");
        if (!st) {
            h = hipMemcpyAsync(out, d, bytes * p, hipMemcpyDeviceToHost, s);
            if (h != hipSuccess) {
                t_last_hip = (int)h;
                set_detail(std::string("allgather staging: ") + hipGetErrorString(h));
                st = LABSORT_ERR_HIP;
            }
        }
        if (!st) st = rccl_stream_wait(o.nc, s, deadline, "ncclAllGather");
        return st ? failed(st) : LABSORT_OK;
    }
    int exchange(const uint32_t *const *send, const uint64_t *sc, uint32_t *const *recv, const uint64_t *rc) {
        const double deadline = now_ms() + o.timeout_ms;
        int st = rccl_exchange(o.nc, p, me, s, send, sc, recv, rc, deadline);
        if (!st) st = rccl_stream_wait(o.nc, s, deadline, "exchange");  // as ThreadComm::exchange
        return st ? failed(st) : LABSORT_OK;
    }
    void abandon() { o.abort(); }  // a transport that breaks is gone for every later sort too
};

struct HostCbComm {
    labsort_host_coll cb;
    int p, me;
    hipStream_t s;
    std::vector<uint32_t> &hs, &hr;  // host staging of the key pieces
    int size() const { return p; }
    int rank() const { return me; }
    // a failed callback: the caller's transport failed or a peer left it
    int allgather(const void *in, void *out, size_t bytes) {
        if (cb.allgather(cb.ctx, in, out, bytes)) {
            set_detail("labsort_host_coll.allgather failed");
            return LABSORT_ERR_PEER;
        }
        return LABSORT_OK;
    }
    int exchange(const uint32_t *const *send, const uint64_t *sc, uint32_t *const *recv, const uint64_t *rc) {
        std::vector<size_t> sb(p), rb(p);
        size_t ts = 0, tr = 0;
        for (int j = 0; j < p; ++j) {
            sb[j] = j == me ? 0 : sc[j] * 4;
            rb[j] = j == me ? 0 : rc[j] * 4;
            ts += sb[j] / 4;
            tr += rb[j] / 4;
        }
        hs.resize(std::max<size_t>(ts, 1));
        hr.resize(std::max<size_t>(tr, 1));
        size_t o = 0;
        for (int j = 0; j < p; ++j) {
            if (sb[j]) MHIP(hipMemcpyAsync(hs.data() + o, send[j], sb[j], hipMemcpyDeviceToHost, s));
            o += sb[j] / 4;
        }
        MHIP(hipStreamSynchronize(s));
        if (cb.alltoallv(cb.ctx, hs.data(), sb.data(), hr.data(), rb.data())) {
            set_detail("labsort_host_coll.alltoallv failed");
            return LABSORT_ERR_PEER;
        }
        o = 0;
        for (int j = 0; j < p; ++j) {
            if (rb[j]) MHIP(hipMemcpyAsync(recv[j], hr.data() + o, rb[j], hipMemcpyHostToDevice, s));
            o += rb[j] / 4;
        }
        MHIP(hipStreamSynchronize(s));  // the staging buffer may be reused
        return LABSORT_OK;
    }
    void abandon() {}  // the caller's collectives bound their own waits (gloo: the group's timeout)
};

// test hook of the schedule (labsort_test_fault; dist_plan.h dist::Fault)
std::mutex g_fault_mu;
dist::Fault g_fault;
dist::Fault armed_fault() {
    std::lock_guard<std::mutex> lk(g_fault_mu);
    return g_fault;
}

// ---------------------------------------------------------------------------------
// in-process ranks: labsort_sort_host_ranks
// ---------------------------------------------------------------------------------
std::mutex g_mu;                 // one in-process multi-GPU sort at a time
std::vector<RankState> g_ranks;  // per rank slot, re-bound when its device changes
std::vector<int> g_comm_devs;    // devices of the cached in-process communicators
std::vector<ncclComm_t> g_comms;
double g_phase_ms[LABSORT_MULTI_PHASES];
std::vector<dist::Result> g_res;  // each rank's collective times in the last call
size_t g_sent_bytes = 0;
std::vector<size_t> g_range_counts;  // keys of each rank's range in the last call
double g_timeout_ms = COMM_TIMEOUT_MS;  // labsort_comm_set_timeout(NULL, s): in-process ranks, new communicators

// abort the cached in-process communicators (after a transport failure): recreated next call
void drop_comms() {
    for (ncclComm_t &c : g_comms)
        if (c) (void)g_rccl.abort(c);
    g_comms.clear();
    g_comm_devs.clear();
}

// one nonblocking communicator per device, created from this thread in one group
// (ncclCommInitRankConfig x p between ncclGroupStart/End), each settled by the deadline
int rccl_comms(const std::vector<int> &devs, double deadline) {
    if (!g_rccl.load()) return LABSORT_ERR_HIP;
    if (g_comm_devs == devs) return LABSORT_OK;
    // the device set changed: release the old communicators
    (void)rccl_release(g_comms.data(), g_comms.size(), now_ms() + std::min(g_timeout_ms, COMM_TEARDOWN_MS));
    g_comms.assign(devs.size(), nullptr);
    g_comm_devs.clear();
    ncclUniqueId u;
    NCHK("ncclGetUniqueId", g_rccl.uid(&u));
    ncclConfig_t cfg = nonblocking_config();
    NCHK("ncclGroupStart", g_rccl.gstart());
    ncclResult_t bad = ncclSuccess;
    for (size_t r = 0; r < devs.size() && (bad == ncclSuccess || bad == ncclInProgress); ++r) {
        MHIP(hipSetDevice(devs[r]));
        bad = g_rccl.init_rank_cfg(&g_comms[r], (int)devs.size(), u, (int)r, &cfg);
    }
    const ncclResult_t e = g_rccl.gend();
    int st = (bad != ncclSuccess && bad != ncclInProgress) ? g_rccl.fail("ncclCommInitRankConfig", bad)
             : (e != ncclSuccess && e != ncclInProgress)   ? g_rccl.fail("ncclGroupEnd (init)", e)
                                                           : LABSORT_OK;
    for (size_t r = 0; r < devs.size() && !st; ++r) st = rccl_settle(g_comms[r], deadline, "ncclCommInitRankConfig");
    if (st) {
        drop_comms();
        return st;
    }
    g_comm_devs = devs;
    return LABSORT_OK;
}

// LABSORT_PIN=1: page-lock the caller's array for the call (hipHostRegister), so the p
// ranks' copies run at the links' pinned rate instead of through the runtime's
// pageable staging buffers
bool pin_requested() {
    const char *e = std::getenv("LABSORT_PIN");
    return e && !std::strcmp(e, "1");
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
    // AUTO: the peer-copy transport (measured on hardware); RCCL on request
    if (transport == LABSORT_XFER_AUTO) transport = LABSORT_XFER_PEER;
    if (transport == LABSORT_XFER_RCCL && !distinct) return LABSORT_ERR_ARG;  // RCCL: one rank per device
    if ((int)g_ranks.size() < p) g_ranks.resize(p);
    for (int r = 0; r < p; ++r)
        if (int st = bind_rank(g_ranks[r], devs[r])) return st;
    ThreadShared sh(p);
    sh.dev = devs;
    const bool rccl = transport == LABSORT_XFER_RCCL;
    sh.deadline = now_ms() + g_timeout_ms;
    if (rccl) {
        if (int st = rccl_comms(devs, sh.deadline)) return st;
        sh.comms = g_comms;
    } else {
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
    std::vector<hipEvent_t> sent_ev(p, nullptr);  // each rank's "my sends are queued" event
    for (int r = 0; r < p; ++r) {
        MHIP(hipSetDevice(devs[r]));
        MHIP(hipEventCreateWithFlags(&sent_ev[r], hipEventDisableTiming));
        sh.sent[r] = sent_ev[r];
    }
    const bool pin = pin_requested();
    if (pin) MHIP(hipHostRegister(h, n * 4, hipHostRegisterDefault));
    std::vector<size_t> off(p + 1);
    for (int r = 0; r <= p; ++r) off[r] = (size_t)((unsigned __int128)n * r / p);
    std::vector<int> st(p, LABSORT_OK), hip(p, 0);
    std::vector<dist::Result> res(p);
    std::vector<std::vector<double>> ph(p, std::vector<double>(LABSORT_MULTI_PHASES, 0.0));
    const double t0 = now_ms();
    const dist::Fault fault = armed_fault();
    std::vector<std::thread> th;
    th.reserve(p);
    for (int r = 0; r < p; ++r)
        th.emplace_back([&, r] {
            t_last_hip = 0;
            RankState &R = g_ranks[r];
            int e = hipSetDevice(R.dev) == hipSuccess ? LABSORT_OK : LABSORT_ERR_HIP;
            HipRankOps ops{R, R.own, key_type, true};
            ThreadComm comm{sh, r, R.own, rccl};
            if (!e) e = dist::sort_rank(ops, comm, h + off[r], off[r + 1] - off[r], flip, h, res[r], fault);
            if (rccl) {
                // the rank's RCCL work (its exchange) done, bounded by the deadline and by the
                // peers' failures; a failed rank aborts its communicator before draining its
                // streams, so none of its kernels waits for a peer that is gone
                if (!e) e = rccl_stream_wait(sh.comms[r], R.own, sh.deadline, "exchange", &sh.failed);
                if (e) {
                    sh.abort();
                    (void)g_rccl.abort(sh.comms[r]);
                    sh.comms[r] = nullptr;
                }
            }
            const int f = ops.finish();  // drain the streams even after a failure
            if (!e) e = f;
            if (e) sh.abort();
            else ops.phases(ph[r].data(), true, res[r]);
            st[r] = e;
            hip[r] = t_last_hip;
        });
    for (auto &t : th) t.join();
    const double t1 = now_ms();
    if (rccl) {
        bool any = false;
        for (int r = 0; r < p; ++r) any = any || st[r];
        if (any) {  // the aborted communicators (and the survivors of the failed call) go
            for (int r = 0; r < p; ++r)
                if (!sh.comms[r]) g_comms[r] = nullptr;
            drop_comms();
        }
    }
    for (int r = 0; r < p; ++r) {
        (void)hipSetDevice(devs[r]);
        (void)hipEventDestroy(sent_ev[r]);
    }
    if (pin) MHIP(hipHostUnregister(h));
    // the first rank that failed for a reason of its own (the others report its failure)
    for (int pass = 0; pass < 2; ++pass)
        for (int r = 0; r < p; ++r)
            if (st[r] && (pass == 1 || st[r] != LABSORT_ERR_PEER)) {
                t_last_hip = hip[r];
                return st[r];
            }
    for (int i = 0; i < LABSORT_MULTI_PHASES; ++i) g_phase_ms[i] = 0.0;
    size_t sent = 0;
    for (int r = 0; r < p; ++r) {
        for (int i = 0; i < LABSORT_MULTI_PHASES; ++i)
            if (i != 6) g_phase_ms[i] = std::max(g_phase_ms[i], ph[r][i]);
        sent = std::max(sent, (size_t)res[r].sent);
    }
    g_phase_ms[6] = t1 - t0;
    g_sent_bytes = sent;
    g_range_counts.assign(p, 0);
    for (int r = 0; r < p; ++r) g_range_counts[r] = (size_t)res[r].count;
    g_res = res;
    return LABSORT_OK;
}

}  // namespace
}  // namespace labsort

// ---------------------------------------------------------------------------------
// one process per GPU: the communicator handle of the C-ABI
// ---------------------------------------------------------------------------------
struct labsort_comm {
    int kind = 0;  // 1 RCCL, 2 host callbacks
    int p = 0, me = 0, dev = -1;
    labsort::RcclState rc;  // RCCL: the nonblocking communicator, its deadline and staging
    labsort_host_coll cb{};
    labsort::RankState R;
    std::vector<uint32_t> hs, hr;
    double phase[LABSORT_MULTI_PHASES] = {};
    labsort::dist::Result res;  // collective times of the last sort
    size_t sent = 0;
    int last_hip = 0;
};

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
    t_last_hip = 0;
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

const char *labsort_multi_error_detail(void) {
    static thread_local std::string copy;
    std::lock_guard<std::mutex> lk(g_err_mu);
    copy = g_detail;
    return copy.c_str();
}

int labsort_multi_timing(double *phase_ms, int nphases, size_t *max_sent_bytes) {
    if (!phase_ms || nphases < 0 || nphases > LABSORT_MULTI_PHASES) return LABSORT_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    for (int i = 0; i < nphases; ++i) phase_ms[i] = g_phase_ms[i];
    if (max_sent_bytes) *max_sent_bytes = g_sent_bytes;
    return LABSORT_OK;
}

int labsort_multi_collectives(double *arrive, double *leave, int nranks, int ncoll) {
    if (!arrive || !leave || nranks < 0 || ncoll < 0 || ncoll > dist::C_NCOLL) return LABSORT_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    if ((size_t)nranks > g_res.size()) return LABSORT_ERR_ARG;
    for (int r = 0; r < nranks; ++r)
        for (int k = 0; k < ncoll; ++k) {
            arrive[r * ncoll + k] = g_res[r].arrive[k];
            leave[r * ncoll + k] = g_res[r].leave[k];
        }
    return LABSORT_OK;
}

int labsort_multi_range_counts(size_t *counts, int nranks) {
    if (!counts || nranks < 0) return LABSORT_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    if ((size_t)nranks > g_range_counts.size()) return LABSORT_ERR_ARG;
    for (int r = 0; r < nranks; ++r) counts[r] = g_range_counts[r];
    return LABSORT_OK;
}

int labsort_multi_plan(const uint32_t *const *h_shards, const size_t *m, int nranks, int key_type,
                       size_t *h_cuts) {
    if (nranks < 1 || nranks > LABSORT_MULTI_MAX_RANKS || !h_shards || !m || !h_cuts) return LABSORT_ERR_ARG;
    const uint32_t flip = key_type == LABSORT_KEY_I32 ? 0x80000000u : 0u;
    const int p = nranks;
    const size_t s = dist::samples_per_rank(p);
    std::vector<uint64_t> ms(m, m + p);
    std::vector<uint32_t> samples((size_t)p * s, 0u);
    for (int r = 0; r < p; ++r) {
        if (m[r] && !h_shards[r]) return LABSORT_ERR_ARG;
        for (size_t k = 0; m[r] && k < s; ++k) samples[(size_t)r * s + k] = h_shards[r][dist::sample_pos(m[r], s, k)];
    }
    const std::vector<dist::Splitter> spl = dist::choose_splitters(p, ms.data(), samples.data(), s, flip);
    const std::vector<uint32_t> vals = dist::plan_values(spl, p, flip);
    std::vector<uint64_t> cut(p + 1);
    for (int r = 0; r < p; ++r) {
        const uint32_t *a = h_shards[r];
        std::vector<uint32_t> ub(vals.size());
        for (size_t v = 0; v < vals.size(); ++v)  // number of keys <= vals[v] in key order
            ub[v] = (uint32_t)(std::upper_bound(a, a + m[r], vals[v] ^ flip,
                                                [flip](uint32_t x, uint32_t y) { return x < (y ^ flip); }) -
                               a);
        if (int st = dist::rank_cuts(r, m[r], spl, ub.data(), p, cut.data())) return st;
        for (int j = 0; j <= p; ++j) h_cuts[(size_t)r * (p + 1) + j] = (size_t)cut[j];
    }
    return LABSORT_OK;
}

int labsort_comm_unique_id(void *id) {
    if (!id) return LABSORT_ERR_ARG;
    if (!g_rccl.load()) return LABSORT_ERR_HIP;
    ncclUniqueId u;
    NCHK("ncclGetUniqueId", g_rccl.uid(&u));
    memcpy(id, &u, sizeof u);
    return LABSORT_OK;
}

int labsort_comm_init_rccl(labsort_comm_t *comm, const void *id, int nranks, int rank) {
    if (!comm || !id || nranks < 1 || nranks > LABSORT_DIST_MAX_RANKS || rank < 0 || rank >= nranks)
        return LABSORT_ERR_ARG;
    *comm = nullptr;
    if (!g_rccl.load()) return LABSORT_ERR_HIP;
    labsort_comm *c = new labsort_comm;
    c->kind = 1;
    c->p = nranks;
    c->me = rank;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        c->rc.timeout_ms = g_timeout_ms;
    }
    if (hipGetDevice(&c->dev) != hipSuccess) {
        delete c;
        return LABSORT_ERR_HIP;
    }
    // the allgather staging is sized here for the schedule's largest record, so nothing
    // can fail between a rank's status word and its collective
    if (int st = grow(c->rc.stage, stage_bytes(nranks))) {
        delete c;
        return st;
    }
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    ncclConfig_t cfg = nonblocking_config();
    const ncclResult_t r = g_rccl.init_rank_cfg(&c->rc.nc, nranks, u, rank, &cfg);  // (sets rc.nc first)
    const int st = rccl_call(c->rc.nc, r, now_ms() + c->rc.timeout_ms, "ncclCommInitRankConfig");
    if (st) {  // (a peer that never joins: the deadline, then the half-made communicator aborted)
        c->rc.abort();
        (void)hipFree(c->rc.stage.p);
        delete c;
        return st;
    }
    *comm = c;
    return LABSORT_OK;
}

int labsort_comm_set_timeout(labsort_comm_t c, double seconds) {
    if (!(seconds > 0.0)) return LABSORT_ERR_ARG;
    if (c) c->rc.timeout_ms = 1000.0 * seconds;
    else {
        std::lock_guard<std::mutex> lk(g_mu);
        g_timeout_ms = 1000.0 * seconds;
    }
    return LABSORT_OK;
}

int labsort_test_fault(const char *phase, int rank) {
    const int ph = dist::fault_phase(phase);
    if (phase && !ph) return LABSORT_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_fault_mu);
    g_fault.phase = ph;
    g_fault.rank = ph ? rank : -1;
    return LABSORT_OK;
}

int labsort_comm_init_host(labsort_comm_t *comm, int nranks, int rank, const labsort_host_coll *coll) {
    if (!comm || !coll || !coll->allgather || !coll->alltoallv || nranks < 1 || nranks > LABSORT_DIST_MAX_RANKS ||
        rank < 0 || rank >= nranks)
        return LABSORT_ERR_ARG;
    labsort_comm *c = new labsort_comm;
    c->kind = 2;
    c->p = nranks;
    c->me = rank;
    c->cb = *coll;
    if (hipGetDevice(&c->dev) != hipSuccess) {
        delete c;
        return LABSORT_ERR_HIP;
    }
    *comm = c;
    return LABSORT_OK;
}

int labsort_comm_destroy(labsort_comm_t c) {
    if (!c) return LABSORT_OK;
    int st = LABSORT_OK;
    if (c->rc.nc) st = rccl_release(&c->rc.nc, 1, now_ms() + std::min(c->rc.timeout_ms, COMM_TEARDOWN_MS));
    if (c->R.dev >= 0) {
        (void)hipSetDevice(c->R.dev);
        for (Buf *b : {&c->R.x, &c->R.y, &c->R.ws, &c->R.mws, &c->R.recv, &c->R.out, &c->R.small, &c->R.part,
                       &c->R.errs, &c->rc.stage})
            if (b->p) (void)hipFree(b->p);
        for (hipStream_t s : {c->R.own, c->R.copy, c->R.plan})
            if (s) (void)hipStreamDestroy(s);
        for (hipEvent_t e : c->R.chunk_ev) (void)hipEventDestroy(e);
        for (hipEvent_t e : c->R.range_ev) (void)hipEventDestroy(e);
        for (hipEvent_t e : c->R.tev) (void)hipEventDestroy(e);
        if (c->R.pin) (void)hipHostFree(c->R.pin);
    }
    delete c;
    return st;
}

int labsort_dist_sort(labsort_comm_t c, const void *d_keys, size_t m, int key_type, void *stream,
                      const void **d_result, size_t *count, size_t *global_offset) {
    if (!c || !d_result || !count || (m && !d_keys)) return LABSORT_ERR_ARG;
    if (key_type != LABSORT_KEY_U32 && key_type != LABSORT_KEY_I32) return LABSORT_ERR_ARG;
    if (m > labsort_max_keys(LABSORT_ALGO_RADIX)) return LABSORT_ERR_ARG;
    t_last_hip = 0;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || cur != c->dev) return LABSORT_ERR_ARG;  // the comm's device
    if (c->kind == 1 && c->rc.broken) {  // aborted after a transport failure in an earlier call
        set_detail("RCCL communicator aborted by an earlier transport failure: create a new one");
        return LABSORT_ERR_PEER;
    }
    if (int st = bind_rank(c->R, c->dev)) return st;
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL: the null stream, as everywhere in the C-ABI
    HipRankOps ops{c->R, s, key_type, false};
    dist::Result res;
    const double t0 = now_ms();
    const dist::Fault fault = armed_fault();
    const uint32_t flip = key_type == LABSORT_KEY_I32 ? 0x80000000u : 0u;
    int st;
    if (c->kind == 1) {
        RcclComm comm{c->rc, c->p, c->me, s};
        st = dist::sort_rank(ops, comm, static_cast<const uint32_t *>(d_keys), m, flip, nullptr, res, fault);
        // the exchange (queued on s) done, bounded: a peer that left ends this rank's wait at
        // the deadline, and the aborted communicator stops its kernels before the drain below
        if (!st && !c->rc.broken) {
            st = rccl_stream_wait(c->rc.nc, s, now_ms() + c->rc.timeout_ms, "exchange");
            if (st) c->rc.abort();
        }
    } else {
        HostCbComm comm{c->cb, c->p, c->me, s, c->hs, c->hr};
        st = dist::sort_rank(ops, comm, static_cast<const uint32_t *>(d_keys), m, flip, nullptr, res, fault);
    }
    const int f = ops.finish();
    if (!st) st = f;
    c->last_hip = t_last_hip;
    c->res = res;  // (collective times also after a failure)
    if (st) return st;
    ops.phases(c->phase, false, res);
    c->phase[6] = now_ms() - t0;
    c->sent = res.sent;
    *d_result = res.data;
    *count = res.count;
    if (global_offset) *global_offset = res.goff;
    return LABSORT_OK;
}

int labsort_dist_timing(labsort_comm_t c, double *phase_ms, int nphases, size_t *sent_bytes) {
    if (!c || !phase_ms || nphases < 0 || nphases > LABSORT_MULTI_PHASES) return LABSORT_ERR_ARG;
    for (int i = 0; i < nphases; ++i) phase_ms[i] = c->phase[i];
    if (sent_bytes) *sent_bytes = c->sent;
    return LABSORT_OK;
}

int labsort_dist_collectives(labsort_comm_t c, double *arrive, double *leave, int ncoll) {
    if (!c || !arrive || !leave || ncoll < 0 || ncoll > dist::C_NCOLL) return LABSORT_ERR_ARG;
    for (int k = 0; k < ncoll; ++k) {
        arrive[k] = c->res.arrive[k];
        leave[k] = c->res.leave[k];
    }
    return LABSORT_OK;
}

int labsort_dist_last_hip_error(labsort_comm_t c) { return c ? c->last_hip : 0; }

}  // extern "C"
