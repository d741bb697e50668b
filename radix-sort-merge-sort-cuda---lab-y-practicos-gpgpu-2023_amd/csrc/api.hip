// api.hip -- host orchestration and the C-ABI of liblabsort.so (include/labsort.h).
//
// Replaces the reference's host pipeline `order_array` (lab.cu:303-402):
//   * device memory is a persistent, grown-on-demand workspace per device instead
//     of cudaMalloc/cudaFree on every call (lab.cu:313-316, 398-401);
//   * all stages are queued on one stream with no intermediate device-wide
//     synchronisation (the reference syncs after each of its 19-21 launches);
//   * the only host synchronisation is the final D2H copy of the host-pointer API.
// Error policy of the drop-in order_array: print "GPUassert: ..." and exit(code),
// as CUDA_CHK/gpuAssert do (utils.h:30-38).  The extern "C" API returns codes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/labsort.h"
#include "common.h"

using namespace labsort;

namespace {

thread_local int g_last_hip = 0;

int fail_hip(hipError_t e) {
    g_last_hip = (int)e;
    return LABSORT_ERR_HIP;
}
#define HIP_TRY(x)                                   \
    do {                                             \
        hipError_t _e = (x);                         \
        if (_e != hipSuccess) return fail_hip(_e);   \
    } while (0)

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
inline uint32_t flip_of(int key_type) { return key_type == LABSORT_KEY_I32 ? 0x80000000u : 0u; }
inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------------------------
// timing hooks
// ---------------------------------------------------------------------------------
struct TimedLaunch {
    int cls;
    hipEvent_t a, b;
};
std::mutex g_timing_mu;
bool g_timing_on = false;
std::vector<TimedLaunch> g_pending;
double g_total_ms[LABSORT_K_COUNT];
long long g_launches[LABSORT_K_COUNT];

struct TimingScope {
    int cls;
    hipStream_t s;
    hipEvent_t a = nullptr, b = nullptr;
    TimingScope(int c, hipStream_t st) : cls(c), s(st) {
        if (!g_timing_on) return;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) { a = b = nullptr; return; }
        (void)hipEventRecord(a, s);
    }
    ~TimingScope() {
        if (!a) return;
        (void)hipEventRecord(b, s);
        std::lock_guard<std::mutex> lk(g_timing_mu);
        g_pending.push_back({cls, a, b});
    }
};

void timing_collect() {
    std::lock_guard<std::mutex> lk(g_timing_mu);
    for (auto &t : g_pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess) {
            g_total_ms[t.cls] += ms;
            g_launches[t.cls] += 1;
        }
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
    g_pending.clear();
}

// ---------------------------------------------------------------------------------
// workspace layouts
// ---------------------------------------------------------------------------------
struct RadixLayout {
    int bits, R, P;
    size_t ntiles;  // look-back slots per pass (tiles + one partial tile per segment)
    size_t off_tmp, off_hist, off_hps, off_joint, off_counter, off_err, off_lookback, zero_bytes, off_plan,
        off_segplan, total;
};

// `tile`: keys per look-back slot of the pass kernel that will run (OSP_TILE for the
// persistent k_onesweep_p, OS_TILE for the non-persistent k_onesweep)
RadixLayout radix_layout(size_t n, int bits, size_t tile) {
    RadixLayout L{};
    L.bits = bits;
    L.R = 1 << bits;
    L.P = (32 + bits - 1) / bits;
    L.ntiles = (n + tile - 1) / tile + (bits == 8 ? NSEG : 0);
    // zeroed block: err | hist | segment histograms | counters | lookback.  The device
    // error word is the workspace's first word (labsort_workspace_status reads it).
    size_t o = 0;
    L.off_err = o;
    o += 256;
    L.off_hist = o;
    o += (size_t)L.P * L.R * 4;
    L.off_hps = o;
    if (bits == 8) o += (size_t)NSEG * 256 * 4;
    L.off_joint = o;
    if (bits == 8) o += (size_t)4 * NSEG * 256 * 4;
    L.off_counter = o;
    o += (size_t)L.P * OSP_NCTR * 4;
    o = align_up(o, 256);
    L.off_lookback = o;
    o += (size_t)L.P * L.ntiles * L.R * 4;
    o = align_up(o, 256);
    L.zero_bytes = o;
    L.off_plan = o;
    o = align_up(o + sizeof(Plan), 256);
    L.off_segplan = o;
    if (bits == 8) o = align_up(o + 4 * sizeof(SegPlan), 256);
    // the ping-pong key buffer last, 64 KiB aligned (tiles are 64 KiB of keys)
    L.off_tmp = align_up(o, 65536);
    L.total = align_up(L.off_tmp + n * 4, 256);
    return L;
}

// Merge sort levels after the tile sort: runs of TS_TILE keys doubled until one run.
// LABSORT_MERGE4 (build knob, default 1): two levels per four-way pass (merge4.hip), the odd
// level first as a pairwise pass; 0: pairwise passes only.
#ifndef LABSORT_MERGE4
#define LABSORT_MERGE4 1
#endif
int merge_levels(size_t n) {
    int m = 0;
    for (size_t run = TS_TILE; run < n; run *= 2) ++m;
    return m;
}

// the error word first (labsort_workspace_status reads the workspace's first word, as for
// the radix layout), then the ping-pong keys, ...
struct MergeLayout {
    size_t off_err, off_tmp, off_part, off_bnd, off_samp[2], total;
};
MergeLayout merge_layout(size_t n) {
    MergeLayout L{};
    size_t o = 0;
    L.off_err = o;
    o += 256;
    L.off_tmp = o;
    o = align_up(o + n * 4, 256);
    L.off_part = o;
    o = align_up(o + (labsort_merge_parts(n)) * 4, 256);
    L.off_bnd = o;
    size_t bw = 0;  // the four-way passes' boundary tables (one at a time)
    if (LABSORT_MERGE4)
        for (size_t r = (merge_levels(n) % 2 ? 2 : 1) * (size_t)TS_TILE; r < n; r *= 4) bw = std::max(bw, merge4_bnd_words(n, r));
    o = align_up(o + bw * 4, 256);
    for (int i = 0; i < 2; ++i) {  // the four-way passes' samples, written by the pass before (ping-pong)
        L.off_samp[i] = o;
        if (bw) o = align_up(o + merge4_samp_words(n) * 4, 256);
    }
    L.total = o;
    return L;
}

// LABSORT_ALGO_RADIX for GS_MIN_N <= n < GS_MAX_N: the gathered passes (gsweep.hip);
// LABSORT_RADIX_IMPL=onesweep selects the scatter passes there too, =gather the
// gathered passes at any n (tests)
bool use_gather(size_t n) {
    const char *e = std::getenv("LABSORT_RADIX_IMPL");
    if (e && !std::strcmp(e, "gather")) return true;
    if (n < GS_MIN_N || n >= GS_MAX_N) return false;
    return !(e && !std::strcmp(e, "onesweep"));
}

// GsHooks callbacks: the same event pairs as TimingScope
struct HookCtx {
    hipEvent_t a = nullptr, b = nullptr;
};
void hook_begin(void *ctx, int cls, hipStream_t s) {
    (void)cls;
    HookCtx *h = static_cast<HookCtx *>(ctx);
    h->a = h->b = nullptr;
    if (!g_timing_on) return;
    if (hipEventCreate(&h->a) != hipSuccess || hipEventCreate(&h->b) != hipSuccess) {
        h->a = h->b = nullptr;
        return;
    }
    (void)hipEventRecord(h->a, s);
}
void hook_end(void *ctx, int cls, hipStream_t s) {
    HookCtx *h = static_cast<HookCtx *>(ctx);
    if (!h->a) return;
    (void)hipEventRecord(h->b, s);
    std::lock_guard<std::mutex> lk(g_timing_mu);
    g_pending.push_back({cls, h->a, h->b});
    h->a = h->b = nullptr;
}

bool small_path(size_t n, int algo) { return algo != LABSORT_ALGO_RADIX1 && n <= (size_t)TS_TILE; }

int sort_radix(const uint32_t *in, uint32_t *out, size_t n, uint32_t flip, int bits, char *ws, hipStream_t s) {
    const RadixLayout L = radix_layout(n, bits, bits == 8 ? OSP_TILE : OS_TILE);
    Bufs b;
    b.p[SEL_IN] = const_cast<uint32_t *>(in);
    b.p[SEL_OUT] = out;
    b.p[SEL_TMP] = reinterpret_cast<uint32_t *>(ws + L.off_tmp);
    uint32_t *hist = reinterpret_cast<uint32_t *>(ws + L.off_hist);
    uint32_t *counters = reinterpret_cast<uint32_t *>(ws + L.off_counter);
    uint32_t *err = reinterpret_cast<uint32_t *>(ws + L.off_err);
    uint32_t *lookback = reinterpret_cast<uint32_t *>(ws + L.off_lookback);
    Plan *plan = reinterpret_cast<Plan *>(ws + L.off_plan);
    if (bits == 8) {
        // histograms first; the look-back words (tens of MB) are cleared after the
        // histogram so their dirty lines do not compete with its read of the keys
        HIP_TRY(launch_zero(ws, L.off_lookback, s));
        uint32_t *hps = reinterpret_cast<uint32_t *>(ws + L.off_hps);
        uint32_t *joint = reinterpret_cast<uint32_t *>(ws + L.off_joint);
        SegPlan *sps = reinterpret_cast<SegPlan *>(ws + L.off_segplan);
        {
            TimingScope ts(LABSORT_K_HISTOGRAM, s);
            HIP_TRY(launch_hist_seg(in, n, flip, hps, joint, s));
        }
        // the look-back clear rides in the plan launch (k_plan8's workgroups 1..)
        HIP_TRY(launch_plan8(hps, joint, n, in == out ? 1 : 0, plan, sps, hist, ws + L.off_lookback,
                             L.zero_bytes - L.off_lookback, s));
        for (int p = 0; p < L.P; ++p) {
            TimingScope ts(LABSORT_K_ONESWEEP, s);
            HIP_TRY(launch_onesweep_p(b, plan, p, n, flip, sps + p, lookback + (size_t)p * L.ntiles * L.R,
                                      counters + (size_t)p * OSP_NCTR, err, s));
        }
    } else {
        HIP_TRY(launch_zero(ws, L.zero_bytes, s));
        {
            TimingScope ts(LABSORT_K_HISTOGRAM, s);
            HIP_TRY(launch_histogram(in, n, flip, bits, hist, s));
        }
        HIP_TRY(launch_plan(hist, n, bits, in == out ? 1 : 0, plan, s));
        for (int p = 0; p < L.P; ++p) {
            TimingScope ts(LABSORT_K_ONESWEEP, s);
            HIP_TRY(launch_onesweep(b, plan, p, bits, n, flip, hist, lookback + (size_t)p * L.ntiles * L.R,
                                    counters + (size_t)p * OSP_NCTR, err, s));
        }
    }
    // 8-bit: pass 0's launch copies an input whose every digit is constant (IN -> OUT), so
    // only an in-place sort (its odd pass count ends in TMP) needs the final copy launch
    if (bits != 8 || in == out) HIP_TRY(launch_final_copy(b, plan, n, s));
    return LABSORT_OK;
}

// Merge passes after the tile sort (runs of TS_TILE keys): four-way passes (two levels per
// HBM read and write, merge4.hip) and, for an odd level count, one pairwise merge-path pass
// first.  (An earlier K-way pass, LDS merges with binary searches per key, measured slower
// than pairwise passes: 9.7-14 vs 7.9 ms)
int sort_merge(const uint32_t *in, uint32_t *out, size_t n, uint32_t flip, char *ws, hipStream_t s) {
    const MergeLayout L = merge_layout(n);
    uint32_t *err = reinterpret_cast<uint32_t *>(ws + L.off_err);
    HIP_TRY(launch_zero(err, 16, s));  // (a kernel: graph-replayable)
    uint32_t *tmp = reinterpret_cast<uint32_t *>(ws + L.off_tmp);
    uint32_t *part = reinterpret_cast<uint32_t *>(ws + L.off_part);
    uint32_t *bnd = reinterpret_cast<uint32_t *>(ws + L.off_bnd);
    const int m = merge_levels(n);
    const bool four = LABSORT_MERGE4 && (((uintptr_t)out | (uintptr_t)tmp) & 15u) == 0;
    const int npass = four ? m / 2 + m % 2 : m;
    uint32_t *cur = (npass % 2 == 0) ? out : tmp;
    // samples for a four-way pass are written by the pass before it (samp[0], samp[1] in turn)
    uint32_t *samp[2] = {reinterpret_cast<uint32_t *>(ws + L.off_samp[0]), reinterpret_cast<uint32_t *>(ws + L.off_samp[1])};
    int sb = 0;
    auto next_is_four = [&](int lv) { return four && lv < m && (m - lv) % 2 == 0; };
    {
        TimingScope ts(LABSORT_K_TILE_SORT, s);
        HIP_TRY(launch_tile_sort(in, cur, n, flip, s, next_is_four(0) ? samp[sb] : nullptr));
    }
    size_t run = TS_TILE;
    for (int lv = 0; lv < m;) {
        uint32_t *nxt = (cur == out) ? tmp : out;
        if (next_is_four(lv)) {
            TimingScope ts(LABSORT_K_MERGE4, s);
            HIP_TRY(launch_merge4_pass(cur, nxt, n, run, flip, bnd, samp[sb], next_is_four(lv + 2) ? samp[sb ^ 1] : nullptr,
                                       s, nullptr, nullptr, err));
            sb ^= 1;
            run *= 4;
            lv += 2;
        } else {
            TimingScope ts(LABSORT_K_MERGE, s);
            HIP_TRY(launch_merge_pass(cur, nxt, n, run, flip, part, s, nullptr, nullptr, nullptr,
                                      next_is_four(lv + 1) ? samp[sb] : nullptr));
            run *= 2;
            lv += 1;
        }
        cur = nxt;
    }
    return LABSORT_OK;
}

// ---------------------------------------------------------------------------------
// host-pointer API state: one cached device buffer + workspace per device
// ---------------------------------------------------------------------------------
// Host-pointer pipeline (labsort_sort_host, n >= HOST_PIPE_MIN): HOST_CHUNKS chunks
// copied H2D on `copy` while `stream` sorts the chunks that have landed; the chunk
// runs are merged in two halves (labsort_merge_runs), then the final merge of the
// halves runs as HOST_RANGES diagonal ranges whose D2H copies start as each lands.
constexpr int HOST_CHUNKS = 8, HOST_RANGES = 8;
constexpr size_t HOST_PIPE_MIN = (size_t)1 << 27;  // r19: 2^26 0.3 ms slower, 2^27 even, 2^28 0.7 ms
                                                    // faster, 2^30 187 -> 157 ms (PCIe-bound)

struct DeviceCache {
    void *keys = nullptr;
    size_t keys_bytes = 0;
    void *ws = nullptr;
    size_t ws_bytes = 0;
    hipStream_t stream = nullptr;
    // pipeline only
    void *keys2 = nullptr, *mws = nullptr, *part = nullptr, *errs = nullptr;
    size_t keys2_bytes = 0, mws_bytes = 0, part_bytes = 0, errs_bytes = 0;
    hipStream_t copy = nullptr;
    hipEvent_t ev[HOST_CHUNKS + HOST_RANGES] = {};
};
std::mutex g_host_mu;
std::vector<DeviceCache> g_cache;

int ensure_buffer(void **p, size_t *have, size_t need) {
    if (*have >= need && *p) return LABSORT_OK;
    if (*p) {
        HIP_TRY(hipFree(*p));
        *p = nullptr;
        *have = 0;
    }
    size_t want = need < (1u << 20) ? (1u << 20) : need;
    HIP_TRY(hipMalloc(p, want));
    *have = want;
    return LABSORT_OK;
}

int default_algo() {
    const char *e = std::getenv("LABSORT_ALGO");
    if (!e) return LABSORT_ALGO_AUTO;
    if (!std::strcmp(e, "merge")) return LABSORT_ALGO_MERGE;
    if (!std::strcmp(e, "radix1")) return LABSORT_ALGO_RADIX1;
    if (!std::strcmp(e, "radix")) return LABSORT_ALGO_RADIX;
    return LABSORT_ALGO_AUTO;
}

// LABSORT_GPUS=p (p > 1): the host drop-ins sort across devices 0..p-1
// (labsort_sort_host_multi); unset, 0 or 1: one GPU.
int multi_gpus() {
    const char *e = std::getenv("LABSORT_GPUS");
    return e ? std::atoi(e) : 0;
}

// LABSORT_ALGO_AUTO -> the algorithm that runs.  Measured on MI355X (r15,
// harness/exp/small_n.py, device-resident): merge 0.054 / 0.119 / 0.202 ms vs radix
// 0.134 / 0.220 / 0.286 ms at 2^16 / 2^20 / 2^22; equal at 2^23; radix faster above.
int resolve_algo(int algo, size_t n) {
    if (algo != LABSORT_ALGO_AUTO) return algo;
    // merge for small arrays (fewer launches) and past the radix limit (2^30 - 1 keys)
    return n <= (size_t)LABSORT_AUTO_MERGE_MAX_KEYS || n > RADIX_MAX_N ? LABSORT_ALGO_MERGE : LABSORT_ALGO_RADIX;
}
// The same for key/value sorts: their radix has no fused small path (the histogram, the
// plan and four persistent passes at every size), so merge up to its own, higher bound
int resolve_pairs_algo(int algo, size_t n) {
    if (algo != LABSORT_ALGO_AUTO) return algo;
    return n <= (size_t)LABSORT_AUTO_PAIRS_MERGE_MAX_KEYS || n > RADIX_MAX_N ? LABSORT_ALGO_MERGE : LABSORT_ALGO_RADIX;
}

// Workspace of LABSORT_ALGO_RADIX at n keys: the layout of the implementation that runs,
// and never less than the gathered layout of any smaller n, so the function is
// monotone in n: a workspace sized for a chunk of m keys serves every shorter chunk
// (labsort_sort_host's ragged last chunk, a rank's smaller shard) whichever
// implementation that length selects.
size_t radix_ws_bytes(size_t n) {
    size_t w = radix_layout(n, 8, OSP_TILE).total;
    if (n >= GS_MIN_N) {
        const size_t g = gs_layout(n < GS_MAX_N ? n : GS_MAX_N - 1).total;
        w = g > w ? g : w;
    }
    if (use_gather(n)) {  // LABSORT_RADIX_IMPL=gather beyond the window
        const size_t g = gs_layout(n).total;
        w = g > w ? g : w;
    }
    return w;
}

}  // namespace

// ---------------------------------------------------------------------------------
// LABSORT_VERIFY=1: every host-pointer drop-in call (order_array / sort /
// order_with_trust) checks its own result -- no descents in int32 order, and the
// same multiset as the input (sum, sum of squares and xor of a mixed hash, all mod
// 2^64) -- prints "labsort-verify,<caller>,<n>,ok" on stderr, and on a mismatch
// fails with the reference's error policy (GPUassert line + exit, utils.h:18-26).
// This is the harness's verify column without editing main.cpp.
// ---------------------------------------------------------------------------------
namespace labsort {
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
bool verify_enabled() {
    const char *e = std::getenv("LABSORT_VERIFY");
    return e && *e && std::strcmp(e, "0") != 0;
}
KeyPrint key_print(const int *a, size_t n) {
    KeyPrint p{0, 0, 0};
    for (size_t i = 0; i < n; ++i) {
        const uint64_t v = (uint32_t)a[i];
        p.s1 += v;
        p.s2 += v * v;
        p.x ^= mix64(v + 0x9E3779B97F4A7C15ull);
    }
    return p;
}
void verify_or_exit(const char *who, const int *a, size_t n, const KeyPrint &before) {
    size_t desc = 0;
    for (size_t i = 1; i < n; ++i) desc += a[i - 1] > a[i];
    const KeyPrint after = key_print(a, n);
    const bool perm = after.s1 == before.s1 && after.s2 == before.s2 && after.x == before.x;
    if (desc || !perm) {
        std::fprintf(stderr, "GPUassert: labsort verify failed in %s: n=%zu, %zu descents, %s %s %d\n", who, n, desc,
                     perm ? "same multiset" : "NOT a permutation of the input", __FILE__, __LINE__);
        std::exit(1);
    }
    std::fprintf(stderr, "labsort-verify,%s,%zu,ok\n", who, n);
}
}  // namespace labsort


// =================================================================================
// C-ABI
// =================================================================================
extern "C" {

const char *labsort_version(void) { return "labsort 0.1 (gfx950)"; }

const char *labsort_error_string(int status) {
    switch (status) {
    case LABSORT_OK: return "ok";
    case LABSORT_ERR_ARG: return "invalid argument";
    case LABSORT_ERR_HIP: return "HIP runtime error";
    case LABSORT_ERR_DEVICE: return "device-side error (look-back spin limit)";
    case LABSORT_ERR_PEER: return "another rank of the distributed sort failed";
    default: return "unknown status";
    }
}

int labsort_last_hip_error(void) { return g_last_hip; }
const char *labsort_hip_error_string(int e) { return hipGetErrorString((hipError_t)e); }

size_t labsort_max_keys(int algo) {
    if (algo == LABSORT_ALGO_MERGE || algo == LABSORT_ALGO_AUTO) return (size_t)0x7FFFFFFFu;
    return RADIX_MAX_N;
}
size_t labsort_tile_keys(void) { return (size_t)TS_TILE; }
size_t labsort_merge_tile_keys(void) { return (size_t)MG_TILE; }
size_t labsort_merge_parts(size_t n) { return (n + MG_TILE - 1) / MG_TILE + 2; }

size_t labsort_workspace_bytes(size_t n, int algo) {
    algo = resolve_algo(algo, n);
    if (small_path(n, algo)) return 256;
    switch (algo) {
    // the implementation that will run (use_gather reads LABSORT_RADIX_IMPL; a sort run
    // after that variable changes is checked against the same function: ERR_ARG if the
    // caller's workspace was sized for the other one)
    case LABSORT_ALGO_RADIX: return radix_ws_bytes(n);
    case LABSORT_ALGO_RADIX1: return radix_layout(n, 1, OS_TILE).total;
    case LABSORT_ALGO_MERGE: return merge_layout(n).total;
    default: return 0;
    }
}

int labsort_sort_device(const void *d_in, void *d_out, size_t n, int key_type, int algo, void *d_ws,
                        size_t ws_bytes, void *stream) {
    if (n == 0) return LABSORT_OK;
    if (!d_in || !d_out) return LABSORT_ERR_ARG;
    if (key_type != LABSORT_KEY_U32 && key_type != LABSORT_KEY_I32) return LABSORT_ERR_ARG;
    if (algo != LABSORT_ALGO_RADIX && algo != LABSORT_ALGO_MERGE && algo != LABSORT_ALGO_RADIX1 &&
        algo != LABSORT_ALGO_AUTO)
        return LABSORT_ERR_ARG;
    if (n > labsort_max_keys(algo)) return LABSORT_ERR_ARG;
    algo = resolve_algo(algo, n);
    if (ws_bytes < labsort_workspace_bytes(n, algo) || !d_ws) return LABSORT_ERR_ARG;
    const uint32_t flip = flip_of(key_type);
    hipStream_t s = as_stream(stream);
    const uint32_t *in = static_cast<const uint32_t *>(d_in);
    uint32_t *out = static_cast<uint32_t *>(d_out);
    if (small_path(n, algo)) {
        TimingScope ts(LABSORT_K_TILE_SORT, s);
        HIP_TRY(launch_tile_sort(in, out, n, flip, s));
        return LABSORT_OK;
    }
    char *ws = static_cast<char *>(d_ws);
    if (algo == LABSORT_ALGO_MERGE) return sort_merge(in, out, n, flip, ws, s);
    if (algo == LABSORT_ALGO_RADIX && use_gather(n)) {
        HookCtx hc;
        HIP_TRY(launch_gsweep_sort(in, out, n, flip, ws, s, GsHooks{&hc, hook_begin, hook_end}));
        return LABSORT_OK;
    }
    return sort_radix(in, out, n, flip, algo == LABSORT_ALGO_RADIX1 ? 1 : 8, ws, s);
}

namespace {
// Synchronise the stream, then read the device error word (the workspace's first
// word) when the sort that used the workspace had one (radix and merge layouts beyond one tile).
int read_status(const void *d_ws, bool has_err_word, hipStream_t s) {
    HIP_TRY(hipStreamSynchronize(s));
    if (!has_err_word) return LABSORT_OK;
    if (!d_ws) return LABSORT_ERR_ARG;
    uint32_t err = 0;
    HIP_TRY(hipMemcpyAsync(&err, d_ws, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return err ? LABSORT_ERR_DEVICE : LABSORT_OK;
}
}  // namespace

int labsort_workspace_status(const void *d_ws, size_t n, int algo, void *stream) {
    if (n == 0) return read_status(d_ws, false, as_stream(stream));
    algo = resolve_algo(algo, n);
    return read_status(d_ws, !small_path(n, algo), as_stream(stream));
}

int labsort_pairs_workspace_status(const void *d_ws, size_t n, int algo, void *stream) {
    algo = resolve_pairs_algo(algo, n);
    return read_status(d_ws, n > (size_t)TS_TILE_KV, as_stream(stream));
}

namespace {
// LABSORT_HOST_PIPE: "0" never, "1" from 2^16 keys (tests), unset from HOST_PIPE_MIN
bool host_pipe_enabled(size_t n, int algo) {
    if (algo == LABSORT_ALGO_RADIX1) return false;
    const char *e = std::getenv("LABSORT_HOST_PIPE");
    if (e && !std::strcmp(e, "0")) return false;
    return n >= (e && !std::strcmp(e, "1") ? (size_t)1 << 16 : HOST_PIPE_MIN);
}

// The pipelined host sort (see HOST_CHUNKS).  Chunk i: H2D into X on c.copy (a pageable
// copy returns once staged, so the host issues chunk i+1's copy while the GPU sorts
// chunk i), then sorted X -> Y on c.stream; its device error word is copied aside.
// Halves: Y's 4 + 4 chunk runs merged into X (the left half while the right half
// is still being copied).  Final: merge(X left, X right) -> Y by
// ranges, each range's D2H on c.copy after its merge.
int sort_host_pipelined(DeviceCache &c, void *h_keys, size_t n, int key_type, int algo) {
    const size_t m = (n + HOST_CHUNKS - 1) / HOST_CHUNKS;  // chunk keys (last one ragged)
    const int calgo = resolve_algo(algo, m);
    const size_t half = m * (HOST_CHUNKS / 2);
    int st;
    if ((st = ensure_buffer(&c.keys, &c.keys_bytes, n * 4))) return st;
    if ((st = ensure_buffer(&c.keys2, &c.keys2_bytes, n * 4))) return st;
    if ((st = ensure_buffer(&c.ws, &c.ws_bytes, labsort_workspace_bytes(m, calgo)))) return st;
    const size_t mwb = labsort_merge_runs_workspace_bytes(half > n - half ? half : n - half);
    if ((st = ensure_buffer(&c.mws, &c.mws_bytes, mwb))) return st;
    if ((st = ensure_buffer(&c.part, &c.part_bytes, labsort_merge_parts((n + HOST_RANGES - 1) / HOST_RANGES) * 4)))
        return st;
    if ((st = ensure_buffer(&c.errs, &c.errs_bytes, HOST_CHUNKS * 4))) return st;
    if (!c.copy) HIP_TRY(hipStreamCreateWithFlags(&c.copy, hipStreamNonBlocking));
    for (auto &e : c.ev)
        if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    uint32_t *h = static_cast<uint32_t *>(h_keys);
    uint32_t *X = static_cast<uint32_t *>(c.keys), *Y = static_cast<uint32_t *>(c.keys2);
    uint32_t *errs = static_cast<uint32_t *>(c.errs);
    // the previous call's D2H copies of Y have finished (c.copy), before Y is written
    HIP_TRY(hipEventRecord(c.ev[0], c.copy));
    HIP_TRY(hipStreamWaitEvent(c.stream, c.ev[0], 0));
    HIP_TRY(launch_zero(errs, HOST_CHUNKS * 4, c.stream));
    HIP_TRY(hipEventRecord(c.ev[1], c.stream));
    HIP_TRY(hipStreamWaitEvent(c.copy, c.ev[1], 0));
    // the two halves of HOST_CHUNKS / 2 chunk runs each, Y -> X: the left half is merged
    // while the right half's chunks are still being copied
    auto merge_half = [&](int hf) -> int {
        const size_t b = hf ? half : 0, e = hf ? n : (half < n ? half : n);
        if (e <= b) return LABSORT_OK;
        size_t off[HOST_CHUNKS / 2 + 1];
        int nr = 0;
        for (int q = 0; q < HOST_CHUNKS / 2; ++q) {
            const size_t o = b + (size_t)q * m;
            if (o >= e) break;
            off[nr++] = o - b;
        }
        off[nr] = e - b;
        return labsort_merge_runs(Y + b, X + b, off, nr, key_type, c.mws, c.mws_bytes, c.stream);
    };
    for (int i = 0; i < HOST_CHUNKS; ++i) {
        const size_t o = (size_t)i * m, len = o < n ? (n - o < m ? n - o : m) : 0;
        if (len) {
            HIP_TRY(hipMemcpyAsync(X + o, h + o, len * 4, hipMemcpyHostToDevice, c.copy));
            HIP_TRY(hipEventRecord(c.ev[i], c.copy));
            HIP_TRY(hipStreamWaitEvent(c.stream, c.ev[i], 0));
            if ((st = labsort_sort_device(X + o, Y + o, len, key_type, calgo, c.ws, c.ws_bytes, c.stream))) return st;
            if (!small_path(len, calgo))  // the workspace's error word (radix and merge layouts)
                HIP_TRY(hipMemcpyAsync(errs + i, c.ws, 4, hipMemcpyDeviceToDevice, c.stream));
        }
        if (i == HOST_CHUNKS / 2 - 1 && (st = merge_half(0))) return st;
    }
    if ((st = merge_half(1))) return st;
    // final merge X[0, half) with X[half, n) into Y by ranges; D2H as each lands
    const size_t la = half < n ? half : n, lb = n - la, rl = (n + HOST_RANGES - 1) / HOST_RANGES;
    for (int r = 0; r < HOST_RANGES; ++r) {
        const size_t d0 = (size_t)r * rl, d1 = d0 + rl < n ? d0 + rl : n;
        if (d0 >= d1) break;
        if ((st = labsort_merge(X, la, X + la, lb, Y + d0, d0, d1, key_type, static_cast<uint32_t *>(c.part),
                                c.stream)))
            return st;
        HIP_TRY(hipEventRecord(c.ev[HOST_CHUNKS + r], c.stream));
    }
    for (int r = 0; r < HOST_RANGES; ++r) {
        const size_t d0 = (size_t)r * rl, d1 = d0 + rl < n ? d0 + rl : n;
        if (d0 >= d1) break;
        HIP_TRY(hipStreamWaitEvent(c.copy, c.ev[HOST_CHUNKS + r], 0));
        HIP_TRY(hipMemcpyAsync(h + d0, Y + d0, (d1 - d0) * 4, hipMemcpyDeviceToHost, c.copy));
    }
    HIP_TRY(hipStreamSynchronize(c.copy));
    HIP_TRY(hipStreamSynchronize(c.stream));
    uint32_t herr[HOST_CHUNKS];
    HIP_TRY(hipMemcpy(herr, errs, sizeof herr, hipMemcpyDeviceToHost));
    for (int i = 0; i < HOST_CHUNKS; ++i)
        if (herr[i]) return LABSORT_ERR_DEVICE;
    return LABSORT_OK;
}
}  // namespace

int labsort_sort_host(void *h_keys, size_t n, int key_type, int algo) {
    if (n == 0) return LABSORT_OK;
    if (!h_keys) return LABSORT_ERR_ARG;
    if (n > labsort_max_keys(algo)) return LABSORT_ERR_ARG;
    if (key_type != LABSORT_KEY_U32 && key_type != LABSORT_KEY_I32) return LABSORT_ERR_ARG;
    const int requested = algo;  // AUTO is resolved again per chunk by the pipeline
    algo = resolve_algo(algo, n);
    std::lock_guard<std::mutex> lk(g_host_mu);
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    if ((int)g_cache.size() <= dev) g_cache.resize(dev + 1);
    DeviceCache &c = g_cache[dev];
    if (!c.stream) HIP_TRY(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    if (host_pipe_enabled(n, algo)) return sort_host_pipelined(c, h_keys, n, key_type, requested);
    int st = ensure_buffer(&c.keys, &c.keys_bytes, n * 4);
    if (st) return st;
    const size_t wsb = labsort_workspace_bytes(n, algo);
    st = ensure_buffer(&c.ws, &c.ws_bytes, wsb);
    if (st) return st;
    HIP_TRY(hipMemcpyAsync(c.keys, h_keys, n * 4, hipMemcpyHostToDevice, c.stream));
    st = labsort_sort_device(c.keys, c.keys, n, key_type, algo, c.ws, c.ws_bytes, c.stream);
    if (st) return st;
    HIP_TRY(hipMemcpyAsync(h_keys, c.keys, n * 4, hipMemcpyDeviceToHost, c.stream));
    return labsort_workspace_status(c.ws, n, algo, c.stream);
}

int labsort_wave_tile_sort(void *d_keys, size_t n, int key_type, void *stream) {
    if (n == 0) return LABSORT_OK;
    if (!d_keys || n > 0xFFFFFFC0u) return LABSORT_ERR_ARG;
    HIP_TRY(launch_wave_tile_sort(static_cast<uint32_t *>(d_keys), n, flip_of(key_type), as_stream(stream)));
    return LABSORT_OK;
}

int labsort_tile_sort(const void *d_in, void *d_out, size_t n, int key_type, void *stream) {
    if (n == 0) return LABSORT_OK;
    if (!d_in || !d_out || n > 0x7FFFFFFFu) return LABSORT_ERR_ARG;
    TimingScope ts(LABSORT_K_TILE_SORT, as_stream(stream));
    HIP_TRY(launch_tile_sort(static_cast<const uint32_t *>(d_in), static_cast<uint32_t *>(d_out), n,
                             flip_of(key_type), as_stream(stream)));
    return LABSORT_OK;
}

int labsort_merge_pass(const void *d_in, void *d_out, size_t n, size_t run, int key_type, uint32_t *d_part,
                       void *stream) {
    if (n == 0) return LABSORT_OK;
    if (!d_in || !d_out || !d_part || d_in == d_out || n > 0x7FFFFFFFu) return LABSORT_ERR_ARG;
    if (run == 0 || (run & (run - 1)) != 0 || 2 * run < (size_t)MG_TILE) return LABSORT_ERR_ARG;
    TimingScope ts(LABSORT_K_MERGE, as_stream(stream));
    HIP_TRY(launch_merge_pass(static_cast<const uint32_t *>(d_in), static_cast<uint32_t *>(d_out), n, run,
                              flip_of(key_type), d_part, as_stream(stream)));
    return LABSORT_OK;
}

int labsort_merge(const void *d_a, size_t la, const void *d_b, size_t lb, void *d_out, size_t d0, size_t d1,
                  int key_type, uint32_t *d_part, void *stream) {
    if (d1 < d0 || d1 > la + lb || la + lb > 0x7FFFFFFFu) return LABSORT_ERR_ARG;
    if (d1 == d0) return LABSORT_OK;
    if (!d_out || !d_part || (la && !d_a) || (lb && !d_b)) return LABSORT_ERR_ARG;
    TimingScope ts(LABSORT_K_MERGE, as_stream(stream));
    HIP_TRY(launch_merge_ab(static_cast<const uint32_t *>(d_a), la, static_cast<const uint32_t *>(d_b), lb,
                            static_cast<uint32_t *>(d_out), d0, d1, flip_of(key_type), d_part, as_stream(stream)));
    return LABSORT_OK;
}

size_t labsort_merge_runs_workspace_bytes(size_t n) { return align_up(n * 4, 256); }  // ping-pong keys

int labsort_merge_runs(const void *d_in, void *d_out, const size_t *h_offsets, int nruns, int key_type,
                       void *d_ws, size_t ws_bytes, void *stream) {
    if (nruns < 1 || nruns > 8 || !h_offsets) return LABSORT_ERR_ARG;
    const size_t n = h_offsets[nruns] - h_offsets[0];
    for (int q = 0; q < nruns; ++q)
        if (h_offsets[q + 1] < h_offsets[q]) return LABSORT_ERR_ARG;
    if (h_offsets[nruns] > 0xFFFFFFFFu || n > 0x7FFFFFFFu) return LABSORT_ERR_ARG;
    if (key_type != LABSORT_KEY_U32 && key_type != LABSORT_KEY_I32) return LABSORT_ERR_ARG;
    if (n == 0) return LABSORT_OK;
    if (!d_in || !d_out || d_in == d_out) return LABSORT_ERR_ARG;
    if (!d_ws || ws_bytes < labsort_merge_runs_workspace_bytes(h_offsets[nruns])) return LABSORT_ERR_ARG;
    hipStream_t s = as_stream(stream);
    if (nruns == 1) {
        HIP_TRY(hipMemcpyAsync(static_cast<uint32_t *>(d_out) + h_offsets[0],
                               static_cast<const uint32_t *>(d_in) + h_offsets[0], n * 4, hipMemcpyDeviceToDevice, s));
        return LABSORT_OK;
    }
        // log2(nruns) levels of pairwise merge-path passes over explicit pairs of runs
        // (k_merge_pass_p, one launch per pair), ping-ponging through the workspace so
        // that the last level writes d_out
        const uint32_t *src = static_cast<const uint32_t *>(d_in) + h_offsets[0];
        uint32_t *outp = static_cast<uint32_t *>(d_out) + h_offsets[0];
        uint32_t *tmp = static_cast<uint32_t *>(d_ws);
        std::vector<size_t> o(h_offsets, h_offsets + nruns + 1);
        for (auto &x : o) x -= h_offsets[0];
        int levels = 0;
        while ((1 << levels) < nruns) ++levels;
        const uint32_t flip = flip_of(key_type);
        TimingScope ts(LABSORT_K_MERGE, s);
        for (int l = 0; l < levels; ++l) {
            uint32_t *dst = ((levels - 1 - l) % 2 == 0) ? outp : tmp;
            std::vector<size_t> no;
            for (size_t i = 0; i + 1 < o.size(); i += 2) {
                const size_t a0 = o[i], a1 = o[i + 1], b1 = i + 2 < o.size() ? o[i + 2] : a1;
                no.push_back(a0);
                if (b1 == a1) {  // no partner: carried over
                    if (a1 > a0) HIP_TRY(hipMemcpyAsync(dst + a0, src + a0, (a1 - a0) * 4, hipMemcpyDeviceToDevice, s));
                    continue;
                }
                MgPairs pr{};
                pr.np = 1;
                pr.pb[0] = 0;
                pr.pb[1] = (uint32_t)(b1 - a0);
                pr.la[0] = (uint32_t)(a1 - a0);
                HIP_TRY(launch_merge_pass(src + a0, dst + a0, b1 - a0, 0, flip, nullptr, s, nullptr, nullptr, &pr));
            }
            no.push_back(o.back());
            o.swap(no);
            src = dst;
        }
        return LABSORT_OK;
}

size_t labsort_pair_tile_keys(void) { return (size_t)TS_TILE_KV; }

namespace {
// key/value merge sort: levels above the TS_TILE_KV-pair tiles, and its workspace: the keys'
// and payloads' ping-pong buffers, then (LABSORT_MERGE4) the four-way passes' boundary
// tables and the two sample buffers
int pairs_merge_levels(size_t n) {
    int m = 0;
    for (size_t run = TS_TILE_KV; run < n; run *= 2) ++m;
    return m;
}
struct PairsMergeLayout {
    size_t off_err, off_tk, off_tv, off_bnd, off_samp[2], total;
};
PairsMergeLayout pairs_merge_layout(size_t n) {
    PairsMergeLayout L{};
    size_t o = 0;
    L.off_err = o;  // (first word: labsort_pairs_workspace_status)
    o += 256;
    L.off_tk = o;
    o = align_up(o + n * 4, 256);
    L.off_tv = o;
    o = align_up(o + n * 4, 256);
    L.off_bnd = o;
    size_t bw = 0;
    if (LABSORT_MERGE4)
        for (size_t r = (pairs_merge_levels(n) % 2 ? 2 : 1) * (size_t)TS_TILE_KV; r < n; r *= 4)
            bw = std::max(bw, merge4_bnd_words(n, r));
    o = align_up(o + bw * 4, 256);
    for (int i = 0; i < 2; ++i) {
        L.off_samp[i] = o;
        if (bw) o = align_up(o + merge4_samp_words(n) * 4, 256);
    }
    L.total = o;
    return L;
}
}  // namespace

size_t labsort_pairs_workspace_bytes(size_t n, int algo) {
    if (n <= (size_t)TS_TILE_KV) return 256;
    algo = resolve_pairs_algo(algo, n);
    if (algo == LABSORT_ALGO_MERGE) return pairs_merge_layout(n).total;  // ping-pong keys | payloads | four-way tables
    // radix workspace | payload ping-pong
    return align_up(radix_layout(n, 8, OSP_TILE).total, 256) + align_up(n * 4, 256);
}

namespace {
// 8-bit LSD radix of (key, payload) pairs: the keys' segmented histogram and plans,
// then the persistent onesweep passes carrying each payload with its key
// (k_onesweep_p<true>), the final copy of keys and payloads under the same buffer plan.
int sort_pairs_radix(const uint32_t *ki, const uint32_t *vi, uint32_t *ko, uint32_t *vo, size_t n, uint32_t flip,
                     char *ws, hipStream_t s) {
    const RadixLayout L = radix_layout(n, 8, OSP_TILE);
    Bufs b, vb;
    b.p[SEL_IN] = const_cast<uint32_t *>(ki);
    b.p[SEL_OUT] = ko;
    b.p[SEL_TMP] = reinterpret_cast<uint32_t *>(ws + L.off_tmp);
    vb.p[SEL_IN] = const_cast<uint32_t *>(vi);
    vb.p[SEL_OUT] = vo;
    vb.p[SEL_TMP] = reinterpret_cast<uint32_t *>(ws + align_up(L.total, 256));
    uint32_t *hist = reinterpret_cast<uint32_t *>(ws + L.off_hist);
    uint32_t *counters = reinterpret_cast<uint32_t *>(ws + L.off_counter);
    uint32_t *err = reinterpret_cast<uint32_t *>(ws + L.off_err);
    uint32_t *lookback = reinterpret_cast<uint32_t *>(ws + L.off_lookback);
    Plan *plan = reinterpret_cast<Plan *>(ws + L.off_plan);
    HIP_TRY(launch_zero(ws, L.off_lookback, s));
    uint32_t *hps = reinterpret_cast<uint32_t *>(ws + L.off_hps);
    uint32_t *joint = reinterpret_cast<uint32_t *>(ws + L.off_joint);
    SegPlan *sps = reinterpret_cast<SegPlan *>(ws + L.off_segplan);
    {
        TimingScope ts(LABSORT_K_HISTOGRAM, s);
        HIP_TRY(launch_hist_seg(ki, n, flip, hps, joint, s));
    }
    HIP_TRY(launch_plan8(hps, joint, n, ki == ko ? 1 : 0, plan, sps, hist, ws + L.off_lookback,
                         L.zero_bytes - L.off_lookback, s));
    for (int p = 0; p < L.P; ++p) {
        TimingScope ts(LABSORT_K_ONESWEEP, s);
        HIP_TRY(launch_onesweep_p(b, plan, p, n, flip, sps + p, lookback + (size_t)p * L.ntiles * L.R,
                                  counters + (size_t)p * OSP_NCTR, err, s, &vb));
    }
    if (ki == ko) {  // (out of place: pass 0's launch copies an all-constant input)
        HIP_TRY(launch_final_copy(b, plan, n, s));
        HIP_TRY(launch_final_copy(vb, plan, n, s));
    }
    return LABSORT_OK;
}
}  // namespace

int labsort_sort_pairs_device(const void *d_keys_in, const void *d_vals_in, void *d_keys_out, void *d_vals_out,
                              size_t n, int key_type, int algo, void *d_ws, size_t ws_bytes, void *stream) {
    if (n == 0) return LABSORT_OK;
    if (!d_keys_in || !d_vals_in || !d_keys_out || !d_vals_out) return LABSORT_ERR_ARG;
    if (key_type != LABSORT_KEY_U32 && key_type != LABSORT_KEY_I32) return LABSORT_ERR_ARG;
    if (algo != LABSORT_ALGO_RADIX && algo != LABSORT_ALGO_MERGE && algo != LABSORT_ALGO_AUTO) return LABSORT_ERR_ARG;
    algo = resolve_pairs_algo(algo, n);
    if (n > (algo == LABSORT_ALGO_MERGE ? (size_t)0x7FFFFFFFu : RADIX_MAX_N)) return LABSORT_ERR_ARG;
    // in place only as a whole: one side aliased and the other not would read
    // payloads that the key side's passes already overwrote
    if ((d_keys_in == d_keys_out) != (d_vals_in == d_vals_out)) return LABSORT_ERR_ARG;
    if (d_keys_out == d_vals_out) return LABSORT_ERR_ARG;
    if (!d_ws || ws_bytes < labsort_pairs_workspace_bytes(n, algo)) return LABSORT_ERR_ARG;
    const uint32_t flip = flip_of(key_type);
    hipStream_t s = as_stream(stream);
    const uint32_t *ki = static_cast<const uint32_t *>(d_keys_in), *vi = static_cast<const uint32_t *>(d_vals_in);
    uint32_t *ko = static_cast<uint32_t *>(d_keys_out), *vo = static_cast<uint32_t *>(d_vals_out);
    if (n <= (size_t)TS_TILE_KV) {
        TimingScope ts(LABSORT_K_TILE_SORT, s);
        HIP_TRY(launch_tile_sort_kv(ki, ko, vi, vo, n, flip, s));
        return LABSORT_OK;
    }
    if (algo == LABSORT_ALGO_RADIX) return sort_pairs_radix(ki, vi, ko, vo, n, flip, static_cast<char *>(d_ws), s);
    // merge passes over runs of TS_TILE_KV pairs, ping-pong between out and the workspace:
    // four-way passes carrying the payloads (k_m4_merge_kv) and, for an odd level count,
    // one pairwise pass first (as sort_merge); the tile sort writes where the pass count
    // makes the last pass land in out
    const PairsMergeLayout L = pairs_merge_layout(n);
    char *ws = static_cast<char *>(d_ws);
    uint32_t *tk = reinterpret_cast<uint32_t *>(ws + L.off_tk), *tv = reinterpret_cast<uint32_t *>(ws + L.off_tv);
    uint32_t *bnd = reinterpret_cast<uint32_t *>(ws + L.off_bnd);
    uint32_t *samp[2] = {reinterpret_cast<uint32_t *>(ws + L.off_samp[0]), reinterpret_cast<uint32_t *>(ws + L.off_samp[1])};
    uint32_t *err = reinterpret_cast<uint32_t *>(ws + L.off_err);
    HIP_TRY(launch_zero(err, 16, s));  // (a kernel: graph-replayable)
    const int m = pairs_merge_levels(n);
    const bool four = LABSORT_MERGE4 && (((uintptr_t)ko | (uintptr_t)vo | (uintptr_t)tk | (uintptr_t)tv) & 15u) == 0;
    const int npass = four ? m / 2 + m % 2 : m;
    uint32_t *ck = (npass % 2 == 0) ? ko : tk, *cv = (npass % 2 == 0) ? vo : tv;
    int sb = 0;
    auto next_is_four = [&](int lv) { return four && lv < m && (m - lv) % 2 == 0; };
    {
        TimingScope ts(LABSORT_K_TILE_SORT, s);
        HIP_TRY(launch_tile_sort_kv(ki, ck, vi, cv, n, flip, s, next_is_four(0) ? samp[sb] : nullptr));
    }
    size_t run = TS_TILE_KV;
    for (int lv = 0; lv < m;) {
        uint32_t *nk = (ck == ko) ? tk : ko, *nv = (cv == vo) ? tv : vo;
        if (next_is_four(lv)) {
            TimingScope ts(LABSORT_K_MERGE4, s);
            HIP_TRY(launch_merge4_pass(ck, nk, n, run, flip, bnd, samp[sb], next_is_four(lv + 2) ? samp[sb ^ 1] : nullptr,
                                       s, cv, nv, err));
            sb ^= 1;
            run *= 4;
            lv += 2;
        } else {
            TimingScope ts(LABSORT_K_MERGE, s);
            HIP_TRY(launch_merge_pass(ck, nk, n, run, flip, nullptr, s, cv, nv, nullptr,
                                      next_is_four(lv + 1) ? samp[sb] : nullptr));
            run *= 2;
            lv += 1;
        }
        ck = nk;
        cv = nv;
    }
    return LABSORT_OK;
}

int labsort_histogram(const void *d_keys, size_t n, int key_type, int bits, uint32_t *d_hist, void *stream) {
    if (n == 0) return LABSORT_OK;
    if (!d_keys || !d_hist || (bits != 8 && bits != 1)) return LABSORT_ERR_ARG;
    TimingScope ts(LABSORT_K_HISTOGRAM, as_stream(stream));
    HIP_TRY(launch_histogram(static_cast<const uint32_t *>(d_keys), n, flip_of(key_type), bits, d_hist,
                             as_stream(stream)));
    return LABSORT_OK;
}

int labsort_fill(void *d_out, size_t n, uint64_t seed, int dist, uint64_t param, uint64_t first, void *stream) {
    if (n == 0) return LABSORT_OK;
    if (!d_out || dist < 0 || dist > 7) return LABSORT_ERR_ARG;
    HIP_TRY(launch_fill(static_cast<uint32_t *>(d_out), n, seed, dist, param, first, as_stream(stream)));
    return LABSORT_OK;
}

int labsort_upper_bound(const void *d_sorted, size_t n, int key_type, const uint32_t *d_values, size_t nv,
                        uint32_t *d_out, void *stream) {
    if (nv == 0) return LABSORT_OK;
    if (!d_values || !d_out || (n && !d_sorted) || n > 0xFFFFFFFFu) return LABSORT_ERR_ARG;
    if (key_type != LABSORT_KEY_U32 && key_type != LABSORT_KEY_I32) return LABSORT_ERR_ARG;
    HIP_TRY(launch_upper_bound(static_cast<const uint32_t *>(d_sorted), n, flip_of(key_type), d_values, nv, d_out,
                               as_stream(stream)));
    return LABSORT_OK;
}

int labsort_copy(const void *d_in, void *d_out, size_t n, void *stream) {
    if (n == 0) return LABSORT_OK;
    if (!d_in || !d_out) return LABSORT_ERR_ARG;
    TimingScope ts(LABSORT_K_COPY, as_stream(stream));
    HIP_TRY(launch_stream_copy(static_cast<const uint32_t *>(d_in), static_cast<uint32_t *>(d_out), n, as_stream(stream)));
    return LABSORT_OK;
}

int labsort_count_descents(const void *d_keys, size_t n, int key_type, uint32_t *d_count, void *stream) {
    if (n < 2) return LABSORT_OK;
    if (!d_keys || !d_count) return LABSORT_ERR_ARG;
    HIP_TRY(launch_count_descents(static_cast<const uint32_t *>(d_keys), n, flip_of(key_type), d_count,
                                  as_stream(stream)));
    return LABSORT_OK;
}

int labsort_timing_enable(int on) {
    timing_collect();
    std::lock_guard<std::mutex> lk(g_timing_mu);
    g_timing_on = on != 0;
    for (int i = 0; i < LABSORT_K_COUNT; ++i) {
        g_total_ms[i] = 0.0;
        g_launches[i] = 0;
    }
    return LABSORT_OK;
}

int labsort_timing_read(int cls, double *total_ms, long long *launches) {
    if (cls < 0 || cls >= LABSORT_K_COUNT || !total_ms || !launches) return LABSORT_ERR_ARG;
    timing_collect();
    std::lock_guard<std::mutex> lk(g_timing_mu);
    *total_ms = g_total_ms[cls];
    *launches = g_launches[cls];
    return LABSORT_OK;
}

void sort(int *in, int n) {
    if (n <= 0) return;
    const bool verify = verify_enabled();
    KeyPrint before{};
    if (verify) before = key_print(in, (size_t)n);
    const int gpus = multi_gpus();
    const int st = gpus > 1 ? labsort_sort_host_multi(in, (size_t)n, LABSORT_KEY_I32, gpus)
                            : labsort_sort_host(in, (size_t)n, LABSORT_KEY_I32, default_algo());
    if (st != LABSORT_OK) {
        const int hip = gpus > 1 ? labsort_multi_last_hip_error() : g_last_hip;
        // the multi-GPU path records what failed (HIP call, RCCL result) in words
        const char *what = gpus > 1 && *labsort_multi_error_detail() ? labsort_multi_error_detail()
                           : st == LABSORT_ERR_HIP                      ? hipGetErrorString((hipError_t)hip)
                                                                        : labsort_error_string(st);
        std::fprintf(stderr, "GPUassert: %s %s %d\n", what, __FILE__, __LINE__);
        std::exit(st == LABSORT_ERR_HIP && hip ? hip : 1);
    }
    if (verify) verify_or_exit("order_array", in, (size_t)n, before);
}

}  // extern "C"

// =================================================================================
// C++-linkage drop-ins (lab.h:9-10): same mangled names as the reference build.
// =================================================================================
void order_array(int *srcCpu, int length) { sort(srcCpu, length); }
