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
// One 1024-thread workgroup per CU (16 wave64s, ~130 KB LDS, 128 VGPRs), 16384-key
// tiles.  Shapes measured and not kept: 768 x 20 (faster for keys only
// without the match buffer, its key/value pass 8 % slower), 512 x 32, 2 x 512 per CU,
// 20K-32K-key tiles (no registers left for the next tile's prefetch).
constexpr int OSP_BLOCK = 1024;
constexpr int OSP_KPT = 16;
constexpr int OSP_TILE = OSP_BLOCK * OSP_KPT;  // 16384 keys per tile
constexpr int OSP_KV_BLOCK = 512;  // key/value pass threads (32 pairs each; r26: 0.902 vs 0.939 ms at 1024)
// look-back window (predecessor tiles per round); r20 sweep at 2^28 with the prefetch:
// 2 0.562, 4 0.505, 6 0.487, 8 0.486, 10 0.530, 16 0.709 ms per pass
constexpr int OSP_LBW = 8;
// Nontemporal key loads per kernel family (ld_stream in devutil.h).  r19 A/B at 2^28:
// onesweep passes 0.556 -> 0.523 ms, the upfront histogram ~0.02 ms faster; the tile
// sort, merge pass and gathered passes were slightly slower with them (not set).  r28:
// since the merge pass stores through its transpose, nontemporal loads are faster there,
// 0.4649 -> 0.4608 ms per pass (alternating runs, profiles/r28_ab_merge_nt_kpt.txt).
constexpr int NT_OSP = 1, NT_HIST = 2, NT_TILE = 4, NT_MERGE = 8, NT_GS = 16, NT_OS = 32;
constexpr int NT_LOADS = NT_OSP | NT_HIST | NT_MERGE;
constexpr int OSP_NCTR = 8;  // tile acquisition counters per pass: one per XCD group of segments
static_assert(OSP_TILE >= OS_TILE, "look-back layout sized by the 1-bit pass tiles");

// ---- segmented look-back chains (8-bit radix) ----
// Each pass's input is split into NSEG contiguous segments, each with its own
// decoupled look-back chain; a segment's base offsets come from histograms the
// upfront histogram kernel computes (see k_hist_seg / k_plan8).
constexpr int NSEG = 16;
constexpr int HS_BPS = 16;  // histogram workgroups per position segment (r21: 0.273 ms at 32, 0.255 at 16, 0.420 at 8)
constexpr size_t HS_MIN_KEYS = 65536;  // fewest keys per histogram workgroup below 2^25 keys
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
constexpr int TS_BLOCK = 1024;
constexpr int TS_KPT = 32;
#ifndef LABSORT_TS_KBLOCK
#define LABSORT_TS_KBLOCK 1024  // keys-only tile sort threads (A/B build knob: 512 = 16K-key tiles, 2 per CU)
#endif
constexpr int TS_KBLOCK = LABSORT_TS_KBLOCK;
constexpr int TS_TILE = TS_KBLOCK * TS_KPT;  // sorted run length of the tile sort
// key/value tile sort: keys and payloads both in LDS (2 x 64 KB)
constexpr int TS_KPT_KV = 16;
constexpr int TS_TILE_KV = TS_BLOCK * TS_KPT_KV;

// ---- merge path ----
// r15 sweep: 512 threads x 8 keys (4096-key tiles), 8 workgroups per CU: 0.488 ms/pass
// (256 x 8 0.521, 256 x 16 0.553, 1024 x 8 0.510, 4 per CU 0.498-0.627); r28 with the
// transposed stores: 512 x 16 0.536-0.539 vs 0.464, 4 / 16 workgroups per CU 0.490 / 0.486
// vs 0.486, co-rank bracket 1 / 2 / 4 / 16 within 1 % of 8; with the network merge 1024 x 8
// 0.4404 vs 0.4360 (profiles/r28_ab_merge_block1024.txt)
constexpr int MG_BLOCK = 512;
constexpr int MG_KPT = 8;
constexpr int MG_TILE = MG_BLOCK * MG_KPT;
constexpr int MG_BLOCKS_PER_CU = 8;   // persistent merge pass grid
constexpr int MG_MAX_TPB = 256;       // most consecutive output tiles per merge workgroup
constexpr int MG_MAX_PAIRS = 4;       // explicit pairs of runs per merge level (up to 8 runs)
constexpr int MG_BRACKET = 8;         // co-rank search: every 8th tile first, the rest bracketed
// One merge level over explicit runs: pair i = runs A = [pb[i], pb[i] + la[i]) and
// B = [pb[i] + la[i], pb[i+1]) merged in place of the pair (labsort_merge_runs); np = 0:
// uniform runs of `run` keys (the merge sort's passes)
struct MgPairs {
    uint32_t np;
    uint32_t pb[MG_MAX_PAIRS + 1];
    uint32_t la[MG_MAX_PAIRS];
};

// ---- gathered LSD radix (gsweep.hip): tiles gathered run by run, sorted in LDS,
// written contiguously; 8-bit digits, one tile per 512-thread workgroup, 3 per CU ----
constexpr int GS_BLOCK = 512;
constexpr int GS_KPT = 16;
constexpr int GS_TILE = GS_BLOCK * GS_KPT;      // 8192 keys
constexpr int GS_KMAX = 1024;                   // runs per tile listed in LDS (else per-lane search)
constexpr int GS_GROUP = 64;                    // tiles per scan workgroup
constexpr int GS_SMALL_NG = 2;                  // up to this many groups (2^20 keys): the fused small path
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

constexpr int MAX_PASSES = 32;
constexpr uint32_t SEL_IN = 0, SEL_OUT = 1, SEL_TMP = 2, SEL_SKIP = 0xFFu;
constexpr uint32_t SPIN_LIMIT = 1u << 22;  // bounded look-back spins: past it the error word is set
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
                           hipStream_t s);
hipError_t launch_hist_seg(const uint32_t *keys, size_t n, uint32_t flip, uint32_t *hps, uint32_t *joint,
                           hipStream_t s);
hipError_t launch_plan8(const uint32_t *hps, const uint32_t *joint, size_t n, int in_is_out, Plan *plan,
                        SegPlan *segplans, uint32_t *hist, void *zero_p, size_t zero_bytes, hipStream_t s);
hipError_t launch_onesweep_p(Bufs b, const Plan *plan, int pass, size_t n, uint32_t flip, const SegPlan *sp,
                             uint32_t *lookback, uint32_t *counter, uint32_t *err, hipStream_t s,
                             const Bufs *vb = nullptr);
hipError_t launch_final_copy(Bufs b, const Plan *plan, size_t n, hipStream_t s);
hipError_t launch_tile_sort(const uint32_t *in, uint32_t *out, size_t n, uint32_t flip, hipStream_t s,
                            uint32_t *samp_out = nullptr);
hipError_t launch_wave_tile_sort(uint32_t *keys, size_t n, uint32_t flip, hipStream_t s);
hipError_t launch_merge_pass(const uint32_t *in, uint32_t *out, size_t n, size_t run, uint32_t flip,
                             uint32_t *part, hipStream_t s, const uint32_t *vin = nullptr, uint32_t *vout = nullptr,
                             const MgPairs *pairs = nullptr, uint32_t *samp_out = nullptr);
hipError_t launch_tile_sort_kv(const uint32_t *in, uint32_t *out, const uint32_t *vin, uint32_t *vout, size_t n,
                               uint32_t flip, hipStream_t s, uint32_t *samp_out = nullptr);
// four-way merge pass (merge4.hip): runs of r keys (a multiple of M4_S) -> runs of 4r;
// bnd: merge4_bnd_words(n, r) words of workspace (16-B aligned); out 16-B aligned.
// vin / vout (both or neither): 4-byte payloads carried with their keys (vout 16-B aligned).
// err: set to 1 if a block's cuts are inconsistent (cannot happen; the block is skipped).
// Samples: every M4_S-th key of a pass's output, samp[pos / M4_S] = out[pos] -- written by
// the pass before a four-way pass (samp_out of the tile sort, the pairwise pass or a
// four-way pass) and read by it (samp_in; nullptr: gathered by the pass itself).
#ifndef LABSORT_M4_S
#define LABSORT_M4_S 128
#endif
constexpr uint32_t M4_S = LABSORT_M4_S;
inline size_t merge4_samp_words(size_t n) { return (n + M4_S - 1) / M4_S + 4; }
size_t merge4_bnd_words(size_t n, size_t r);
hipError_t launch_merge4_pass(const uint32_t *in, uint32_t *out, size_t n, size_t r, uint32_t flip, uint32_t *bnd,
                              const uint32_t *samp_in, uint32_t *samp_out, hipStream_t s, const uint32_t *vin = nullptr,
                              uint32_t *vout = nullptr, uint32_t *err = nullptr);
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
hipError_t launch_stream_copy(const uint32_t *in, uint32_t *out, size_t n, hipStream_t s);
hipError_t launch_count_descents(const uint32_t *keys, size_t n, uint32_t flip, uint32_t *count, hipStream_t s);

}  // namespace labsort
