// common.h -- shared definitions of the labsort HIP kernels and host launchers.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace labsort {

constexpr int WAVE = 64;

// ---- radix configuration (8-bit digits, onesweep) ----
constexpr int RADIX_BITS = 8;
constexpr int OS_BLOCK = 512;     // threads per onesweep workgroup (8 waves)
constexpr int OS_KPT = 16;        // keys per thread
constexpr int OS_TILE = OS_BLOCK * OS_KPT;  // 8192 keys per tile
constexpr int HIST_BLOCK = 1024;

// ---- persistent pipelined onesweep (8-bit digits) ----
// The OSP_* shape constants can be overridden (-DLABSORT_OSP_BLOCK=... etc.) for
// diagnostic builds under harness/exp; the shipped library uses the defaults.
// r26 A/B at 2^28 (profiles/r26_ab_shapes_tilesort.txt): 768 threads x 20 keys (15360-key
// tiles, 12 waves, 168 VGPRs: the prefetch without spills, no match buffer) 0.487 / 0.465
// ms per pass (uniform / sorted keys) vs 0.492 / 0.489 for 1024 x 16, but 0.512 / 0.489
// with the match-rank buffer in LDS, and its key/value pass 1.00 vs 0.925 ms (11 VGPRs
// spilled); 768 x 24-32 without the prefetch 0.507-0.513; 512 x 16 at 2 workgroups per
// CU 0.585.  1024 x 16 is kept: one shape for the key and key/value passes.
#ifndef LABSORT_OSP_BLOCK
#define LABSORT_OSP_BLOCK 1024
#endif
#ifndef LABSORT_OSP_KPT
#define LABSORT_OSP_KPT 16
#endif
#ifndef LABSORT_OSP_LBW
#define LABSORT_OSP_LBW 8  // r20 sweep (2^28, with prefetch): 2 0.562, 4 0.505, 6 0.487, 8 0.486, 10 0.530, 16 0.709 ms per pass
#endif
#ifndef LABSORT_OSP_LBW2
#define LABSORT_OSP_LBW2 8
#endif
#ifndef LABSORT_OSP_PREFETCH
#define LABSORT_OSP_PREFETCH 1  // r19 with nontemporal loads: 2^28 sort 2.45 -> 2.33 ms (without them it was slower)
#endif
#ifndef LABSORT_OSP_NT
#define LABSORT_OSP_NT 0  // bit 0: nontemporal scatter stores (measured slower, r19)
#endif
// Nontemporal key loads per kernel family (ld_stream in devutil.h).  r19 A/B at 2^28:
// onesweep passes 0.556 -> 0.523 ms, the upfront histogram ~0.02 ms faster; the tile
// sort, merge pass and gathered passes were slightly slower with them (not set).
constexpr int NT_OSP = 1, NT_HIST = 2, NT_TILE = 4, NT_MERGE = 8, NT_GS = 16, NT_OS = 32;
#ifndef LABSORT_NT_LOADS
#define LABSORT_NT_LOADS 3  // NT_OSP | NT_HIST
#endif
#ifndef LABSORT_OSP_XCD
#define LABSORT_OSP_XCD 1
#endif
#ifndef LABSORT_OSP_BPC
#define LABSORT_OSP_BPC 1
#endif
constexpr int OSP_BLOCK = LABSORT_OSP_BLOCK;
constexpr int OSP_KPT = LABSORT_OSP_KPT;
constexpr int OSP_TILE = OSP_BLOCK * OSP_KPT;  // 16384 keys per tile
// key/value pass threads (the same tile: OSP_TILE / OSP_KV_BLOCK pairs per thread)
#ifndef LABSORT_OSP_KV_BLOCK
#define LABSORT_OSP_KV_BLOCK 512  // r26: 0.902 vs 0.939 ms per pair pass (1024 x 16); with the prefetch 1.020
#endif
constexpr int OSP_KV_BLOCK = LABSORT_OSP_KV_BLOCK;
#ifndef LABSORT_OSP_JCOUNT
#define LABSORT_OSP_JCOUNT 0  // timing build: in-pass joint counting (kernels.hip)
#endif
constexpr int OSP_LBW = LABSORT_OSP_LBW;    // look-back window of the first round (predecessor tiles)
constexpr int OSP_LBW2 = LABSORT_OSP_LBW2;  // look-back window of the later rounds
constexpr bool OSP_PREFETCH = LABSORT_OSP_PREFETCH != 0;  // next tile's keys loaded one iteration ahead
// A's keys are scattered straight from the LDS reorder buffer (read at scatter
// time, before B's reorder overwrites it) instead of being read back into registers at the
// end of the previous iteration: 16 VGPRs fewer across the look-back
#ifndef LABSORT_OSP_LDS_SCATTER
#define LABSORT_OSP_LDS_SCATTER 0  // r19: slower (2.33 -> 2.59 ms with prefetch, 2.46 without)
#endif
constexpr bool OSP_LDS_SCATTER = LABSORT_OSP_LDS_SCATTER != 0;
constexpr int OSP_RANK_BALLOT = 0, OSP_RANK_MATCH = 1, OSP_RANK_ATOMIC = 2;  // k_onesweep_p<RANK, HIST_FIRST>
constexpr int OSP_SEG_LATER = 1;  // 1: digit-group segments after the first active pass (LABSORT_SEG)
constexpr int OSP_DEFAULT_VARIANT = 4;          // variant = RANK * 2 + HIST_FIRST
// Tile acquisition: OSP_NCTR counters per pass.  With OSP_XCD each XCD (HW_REG_XCC_ID)
// first takes the tiles of its own segments {x, x + 8} in order, then helps the
// others; consecutive tiles of a segment then write their shared run-boundary lines
// through one L2 (harness/exp/bw_probe.hip: abutting 64-key runs 0.67 -> 0.58 ms).
constexpr bool OSP_XCD = LABSORT_OSP_XCD != 0;
constexpr int OSP_NCTR = 8;
constexpr int OSP_BLOCKS_PER_CU = LABSORT_OSP_BPC;           // persistent grid = CUs (16-wave workgroups, LDS ~130 KB, 128 VGPRs)
static_assert(OSP_TILE >= OS_TILE, "look-back layout sized by the 1-bit pass tiles");

// ---- segmented look-back chains (8-bit radix) ----
// Each pass's input is split into NSEG contiguous segments, each with its own
// decoupled look-back chain; a segment's base offsets come from histograms the
// upfront histogram kernel computes (see k_hist_seg / k_plan8).
constexpr int NSEG = 16;
#ifndef LABSORT_HS_BPS
#define LABSORT_HS_BPS 16  // r21: k_hist_seg at 2^28 0.273 ms (32), 0.255 (16), 0.420 (8)
#endif
constexpr int HS_BPS = LABSORT_HS_BPS;  // histogram workgroups per position segment (80 KB LDS each)
constexpr size_t HS_MIN_KEYS = 65536;  // fewest keys per histogram workgroup below 2^25 keys
#ifndef LABSORT_HS_ROT
#define LABSORT_HS_ROT 1
#endif
constexpr bool HS_ROT = LABSORT_HS_ROT != 0;  // rotated flush order per histogram workgroup
// first position of segment s of an n-key pass input (first active pass)
__host__ __device__ inline uint32_t seg_start(uint32_t s, size_t n) { return (uint32_t)((size_t)s * n / NSEG); }
struct SegPlan {
    uint32_t start[NSEG + 1];  // segment s = pass input positions [start[s], start[s+1])
    uint32_t tpre[NSEG + 1];   // tiles in segments < s = look-back slot of segment s's first tile
    uint32_t maxt;             // most tiles in one segment
    uint32_t mode;             // 0 position segments, 1 digit-group segments, 2 one segment
    uint32_t segbits;          // tile id c -> segment c & (2^segbits - 1), tile c >> segbits
    uint32_t pad[11];
    uint32_t base[NSEG * 256];  // output offset of the first key of digit d in segment s
};

// ---- LDS tile sort (merge path stage 1 / small sorts) ----
// 32768-key runs (one 16-wave workgroup per CU, ~146 KB LDS): two merge passes fewer
// than 8192-key runs; measured 9.45 -> 8.60 ms for the 2^28 merge sort (r11).
#ifndef LABSORT_TS_BLOCK
#define LABSORT_TS_BLOCK 1024
#endif
#ifndef LABSORT_TS_KPT
#define LABSORT_TS_KPT 32
#endif
constexpr int TS_BLOCK = LABSORT_TS_BLOCK;
constexpr int TS_KPT = LABSORT_TS_KPT;
constexpr int TS_TILE = TS_BLOCK * TS_KPT;  // sorted run length of the tile sort
// key/value tile sort: keys and payloads both in LDS (2 x 64 KB)
constexpr int TS_KPT_KV = 16;
constexpr int TS_TILE_KV = TS_BLOCK * TS_KPT_KV;

// ---- merge path ----
#ifndef LABSORT_MG_BLOCK
#define LABSORT_MG_BLOCK 512
#endif
#ifndef LABSORT_MG_KPT
#define LABSORT_MG_KPT 8
#endif
#ifndef LABSORT_MG_BPC
#define LABSORT_MG_BPC 8
#endif
constexpr int MG_BLOCK = LABSORT_MG_BLOCK;  // r15 sweep: 512 x 8 keys (4096-key tiles) 0.488 ms/pass vs 256 x 8 0.521
constexpr int MG_KPT = LABSORT_MG_KPT;
constexpr int MG_TILE = MG_BLOCK * MG_KPT;
constexpr int MG_MAX_TPB = 256;       // most consecutive output tiles per merge workgroup
constexpr int MG_MAX_PAIRS = 4;       // explicit pairs of runs per merge level (up to 8 runs)
// One merge level over explicit runs: pair i = runs A = [pb[i], pb[i] + la[i]) and
// B = [pb[i] + la[i], pb[i+1]) merged in place of the pair (labsort_merge_runs); np = 0:
// uniform runs of `run` keys (the merge sort's passes)
struct MgPairs {
    uint32_t np;
    uint32_t pb[MG_MAX_PAIRS + 1];
    uint32_t la[MG_MAX_PAIRS];
};
#ifndef LABSORT_MG_BRACKET
#define LABSORT_MG_BRACKET 8
#endif
constexpr int MG_BRACKET = LABSORT_MG_BRACKET;  // co-rank search: every 8th tile first, the rest bracketed
constexpr int MG_BLOCKS_PER_CU = LABSORT_MG_BPC;  // persistent merge pass grid
// co-rank searches by lane groups (k-ary: fewer dependent load rounds) instead of one
// binary search per thread
#ifndef LABSORT_MG_KARY
#define LABSORT_MG_KARY 0
#endif
constexpr bool MG_KARY = LABSORT_MG_KARY != 0;
#ifndef LABSORT_MG_K1
#define LABSORT_MG_K1 64  // lanes per round-1 search
#endif
#ifndef LABSORT_MG_K2
#define LABSORT_MG_K2 16  // lanes per round-2 (bracketed) search
#endif
constexpr int MG_K1 = LABSORT_MG_K1, MG_K2 = LABSORT_MG_K2;

// ---- K-way merge (kmerge.hip) ----
// (overridable for diagnostic builds under harness/exp)
#ifndef LABSORT_KM_S
#define LABSORT_KM_S 256
#endif
#ifndef LABSORT_KM_M
#define LABSORT_KM_M 16
#endif
#ifndef LABSORT_KM_BLOCK
#define LABSORT_KM_BLOCK 512
#endif
#ifndef LABSORT_KM_SEQ
#define LABSORT_KM_SEQ 0
#endif
constexpr uint32_t KM_S = LABSORT_KM_S;  // sample stride (the reference's separators: every 256 keys)
constexpr uint32_t KM_M = LABSORT_KM_M;  // samples per block: blocks average KM_M * KM_S keys
constexpr int KM_BLOCK = LABSORT_KM_BLOCK;  // threads per block-merge workgroup
constexpr bool KM_SEQ = LABSORT_KM_SEQ != 0;  // per-thread chunk: sequential merge (1) or bitonic (0)
#ifndef LABSORT_KM_PERSIST
#define LABSORT_KM_PERSIST 0
#endif
#ifndef LABSORT_KM_PERSIST_OVER
#define LABSORT_KM_PERSIST_OVER 1
#endif
constexpr bool KM_PERSIST = LABSORT_KM_PERSIST != 0;  // persistent pipelined block merge (k_km_blocks_p)
constexpr int KM_PERSIST_OVER = LABSORT_KM_PERSIST_OVER;  // persistent grid = CUs x fit x this
#ifndef LABSORT_KM_SORT_K
#define LABSORT_KM_SORT_K 2
#endif
constexpr int KM_SORT_K = LABSORT_KM_SORT_K;  // merge sort: 2 = pairwise merge-path passes, 4/8 = K-way passes
#define KM_BMAX(K) ((KM_M + (K)) * KM_S)  // most keys in one block
struct KmRuns {
    uint32_t explicit_runs;  // 1: one job, runs [offs[q], offs[q+1]); 0: runs of `run` keys tiling [0, n)
    uint32_t K;              // runs per job: 2, 4 or 8 (missing runs are empty)
    uint32_t n;
    uint32_t run;            // uniform: run length (a multiple of KM_S)
    uint32_t njobs;          // uniform: ceil(n / (K * run)); explicit: 1
    uint32_t nspl_max;       // set by launch_kmerge: splitters of the largest job
    uint32_t offs[9];
};
hipError_t launch_kmerge(const uint32_t *in, uint32_t *out, KmRuns rs, uint32_t flip, uint32_t *ws, hipStream_t s);
size_t km_workspace_words(size_t n);

// ---- gathered LSD radix (gsweep.hip): tiles gathered run by run, sorted in LDS,
// written contiguously; 8-bit digits, one tile per 512-thread workgroup, 3 per CU ----
constexpr int GS_BLOCK = 512;
#ifndef LABSORT_GS_KPT
#define LABSORT_GS_KPT 16
#endif
constexpr int GS_KPT = LABSORT_GS_KPT;
constexpr int GS_TILE = GS_BLOCK * GS_KPT;      // 8192 keys
constexpr int GS_KMAX = 1024;                   // runs per tile listed in LDS (else per-lane search)
constexpr int GS_GROUP = 64;                    // tiles per scan workgroup
#ifndef LABSORT_GS_SMALL_NG
#define LABSORT_GS_SMALL_NG 2
#endif
constexpr int GS_SMALL_NG = LABSORT_GS_SMALL_NG;  // up to this many groups (2^20 keys): one scan launch per pass
constexpr size_t GS_MIN_N = (size_t)1 << 16;    // LABSORT_ALGO_RADIX uses it for GS_MIN_N <= n < GS_MAX_N
constexpr size_t GS_MAX_N = (size_t)1 << 25;    // (onesweep outside; r26 crossover at 2^25: 0.420 vs 0.442 ms)
struct GsLayout {
    size_t off_state, off_a, off_b, off_rt, off_rt2, off_mm, off_gsx, off_gx, off_gmm, off_ls[2], off_sr[2],
        off_first[2], total;
};
GsLayout gs_layout(size_t n);
// timing hooks around the pass and final-copy launches (api.hip's event scopes)
struct GsHooks {
    void *ctx;
    void (*begin)(void *ctx, int kernel_class, hipStream_t s);
    void (*end)(void *ctx, int kernel_class, hipStream_t s);
};
hipError_t launch_gsweep_sort(const uint32_t *in, uint32_t *out, size_t n, uint32_t flip, char *ws, hipStream_t s,
                              const GsHooks &hooks);

// ---- single-launch LSD radix for small arrays (small.hip): one cooperative launch,
// one 16384-key tile per workgroup, grid barriers between phases ----
constexpr int SR_BLOCK = 1024, SR_KPT = 16;
constexpr int SR_TILE = SR_BLOCK * SR_KPT;
constexpr size_t SR_MAX_N = (size_t)256 * SR_TILE;  // one co-resident workgroup per CU (2^22 keys)
struct SrLayout {
    size_t off_err, off_bar, off_andor, off_cnt, off_tmp, total;
};
SrLayout sr_layout(size_t n);
hipError_t launch_small_radix(const uint32_t *in, uint32_t *out, size_t n, uint32_t flip, char *ws, hipStream_t s);

constexpr int MAX_PASSES = 32;
constexpr uint32_t SEL_IN = 0, SEL_OUT = 1, SEL_TMP = 2, SEL_SKIP = 0xFFu;
constexpr uint32_t NEXT_NONE = 0xFFFFFFFFu;

// Per-sort plan written on the device after the histogram (no host sync):
// which buffer each digit pass reads and writes, or SKIP when every key has
// the same digit in that pass (the deterministic counterpart of the
// reference's "stop when sorted" test, lab.cu:61).
struct Plan {
    uint32_t src[MAX_PASSES];
    uint32_t dst[MAX_PASSES];
    uint32_t next[MAX_PASSES];  // 8-bit radix: next active pass after this one (NEXT_NONE)
    uint32_t prev[MAX_PASSES];  // 8-bit radix: previous active pass (NEXT_NONE for the first)
    uint32_t copy_from;  // SEL_SKIP: result already in OUT
    uint32_t active;     // number of non-trivial passes
    uint32_t pad[2];
};

struct Bufs {
    uint32_t *p[3];  // IN, OUT, TMP
};

// lookback word: 2 status bits + 30-bit count (n < 2^30 per radix sort)
constexpr uint32_t LB_AGG = 1u << 30;
constexpr uint32_t LB_INC = 2u << 30;
constexpr uint32_t LB_VAL = (1u << 30) - 1u;
constexpr size_t RADIX_MAX_N = (size_t)LB_VAL;  // 2^30 - 1

// ---- host launchers (kernels.hip) ----
hipError_t launch_fill(uint32_t *out, size_t n, uint64_t seed, int dist, uint64_t param, uint64_t first,
                       hipStream_t s);
hipError_t launch_histogram(const uint32_t *keys, size_t n, uint32_t flip, int bits, uint32_t *hist,
                            hipStream_t s);
hipError_t launch_plan(const uint32_t *hist, size_t n, int bits, int in_is_out, Plan *plan, hipStream_t s);
hipError_t launch_onesweep(Bufs b, const Plan *plan, int pass, int bits, size_t n, uint32_t flip,
                           const uint32_t *hist, uint32_t *lookback, uint32_t *counter, uint32_t *err,
                           hipStream_t s, const Bufs *vb = nullptr);
hipError_t launch_hist_seg(const uint32_t *keys, size_t n, uint32_t flip, uint32_t *hps, uint32_t *joint,
                           hipStream_t s);
hipError_t launch_plan8(const uint32_t *hps, const uint32_t *joint, size_t n, int in_is_out, Plan *plan,
                        SegPlan *segplans, uint32_t *hist, void *zero_p, size_t zero_bytes, hipStream_t s);
hipError_t launch_onesweep_p(Bufs b, const Plan *plan, int pass, size_t n, uint32_t flip, const SegPlan *sp,
                             uint32_t *lookback, uint32_t *counter, uint32_t *err, hipStream_t s,
                             const Bufs *vb = nullptr, uint32_t *jout = nullptr);
hipError_t launch_final_copy(Bufs b, const Plan *plan, size_t n, hipStream_t s);
hipError_t launch_tile_sort(const uint32_t *in, uint32_t *out, size_t n, uint32_t flip, hipStream_t s);
hipError_t launch_wave_tile_sort(uint32_t *keys, size_t n, uint32_t flip, hipStream_t s);
hipError_t launch_merge_pass(const uint32_t *in, uint32_t *out, size_t n, size_t run, uint32_t flip,
                             uint32_t *part, hipStream_t s, const uint32_t *vin = nullptr, uint32_t *vout = nullptr,
                             const MgPairs *pairs = nullptr);
hipError_t launch_tile_sort_kv(const uint32_t *in, uint32_t *out, const uint32_t *vin, uint32_t *vout, size_t n,
                               uint32_t flip, hipStream_t s);
hipError_t launch_merge_ab(const uint32_t *a, size_t la, const uint32_t *b, size_t lb, uint32_t *out, size_t d0,
                           size_t d1, uint32_t flip, uint32_t *part, hipStream_t s);
hipError_t launch_upper_bound(const uint32_t *keys, size_t n, uint32_t flip, const uint32_t *values, size_t nv,
                              uint32_t *out, hipStream_t s);
// LABSORT_VERIFY=1 checks of the host-pointer drop-ins (api.hip)
struct KeyPrint {
    uint64_t s1, s2, x;  // sum, sum of squares, xor of a mixed hash (mod 2^64)
};
bool verify_enabled();
KeyPrint key_print(const int *a, size_t n);
void verify_or_exit(const char *who, const int *a, size_t n, const KeyPrint &before);

hipError_t launch_zero(void *p, size_t bytes, hipStream_t s);  // graph-replayable memset (16-B aligned p)
hipError_t launch_count_descents(const uint32_t *keys, size_t n, uint32_t flip, uint32_t *count, hipStream_t s);

}  // namespace labsort
