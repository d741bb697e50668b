// merge4.hip -- 4-way merge pass of the merge sort (config 4): one HBM read and write merges
// four sorted runs of r keys into one of 4r, so two of the pairwise passes' doublings cost
// one pass (13 passes at 2^28 become 6 four-way + 1 pairwise).
//
// The reference's stage 3 is the model (lab.cu:209-300): splitters taken at a fixed stride
// of each run (separators_kernel :219-224), each splitter's co-rank in the other run found
// by binary search (busquedaPorBiparticion :102-132, with the tie rule "A before equal B",
// :163-170), and the segments between consecutive splitters merged independently
// (merge_segments_kernel :272-300).  Here, over four runs A, B, C, D of a group:
//   k_m4_rank  every M4_S-th key of every run is a sample; a sample's index in the merged
//              order of all the group's samples, under the order (key, run, position), is
//              its own index plus, per other run, the samples that precede it (searched
//              over that run's samples: upper bound for earlier runs, lower bound for
//              later ones -- the reference's tie rule generalised to four runs).  Every
//              M4_M-th sample in that order is a block boundary: its co-rank in each other
//              run (the same bound over the run's keys, bracketed to one sample gap) gives
//              the boundary's four cuts.  A block between consecutive boundaries holds at
//              most (M4_M + 3) M4_S keys (each run adds at most one sample gap beyond the
//              samples inside it) and M4_S M4_M on average.
//   k_m4_merge persistent workgroups take consecutive blocks: the block's four windows are
//              loaded into LDS (the next block's keys load into registers while the current
//              one merges), then two merge levels, each thread taking 8 outputs at its
//              merge-path diagonal and merging the two 8-key windows there with a 16-input
//              bitonic network in registers (equal keys are identical words, so the order
//              among them does not change the output): A+B and C+D into LDS, then
//              (A+B)+(C+D) into an LDS staging buffer aligned to the block's output offset,
//              stored as 16-B nontemporal stores (and every M4_S-th output word as the next
//              four-way pass's sample).
//   k_m4_merge_kv the same with 4-byte payloads beside the keys, stable level merges.
// r29 at 2^28 (profiles/r29_ab_merge4_v2.txt): merge sort 6.79 -> 6.04 ms
// (pass 0.745 ms: rank 0.077 + merge 0.68, VALU- and LDS-bound), key/value 13.95 -> 11.61 ms.
#include "common.h"
#include "devutil.h"

namespace labsort {

// M4_S (common.h): sample stride (keys)
// (M4_S 128 / M4_M 28 measured against 64 / 60, 64 / 56 and 256 / 12 in r30: 6.08 ms per
// 2^28 merge sort against 6.37, 6.42 and 6.39; profiles/r30_ab_sample_stride.txt)
#ifndef LABSORT_M4_M
#define LABSORT_M4_M 28
#endif
constexpr uint32_t M4_M = LABSORT_M4_M;  // samples per block (merged order)
constexpr int M4_KPT = 8;                // outputs per thread and merge level (r29: 16, with 256
constexpr int M4_BLOCK = 4096 / M4_KPT;  // threads and half the co-rank searches, measured equal)
constexpr uint32_t M4_CAP = (uint32_t)(M4_BLOCK * M4_KPT);  // keys per block at most
static_assert((M4_M + 3) * M4_S <= M4_CAP - 2 * M4_KPT, "a block (and its level-1 padding) fits one pass of the threads");
constexpr int M4_BLOCKS_PER_CU = 4;
constexpr uint32_t M4_MAX_PER = 256;  // most consecutive blocks per merge workgroup (their cuts held in LDS)

struct M4Geo {
    uint32_t n, r;        // keys, input run length (a multiple of M4_S)
    uint32_t ngroups;     // groups of four runs
    uint32_t spg, bpg;    // samples / blocks of a full group
    uint32_t nblocks;     // blocks over all groups (flat ids g * bpg + b, the last group's nb <= bpg)
};

// run k of group g: [g 4r + k r, min(n, g 4r + (k + 1) r))
__device__ __forceinline__ uint32_t m4_run_len(const M4Geo &G, uint32_t g, uint32_t k) {
    const uint64_t b = (uint64_t)g * 4u * G.r + (uint64_t)k * G.r;
    if (b >= G.n) return 0u;
    const uint64_t e = b + G.r;
    return (uint32_t)((e < G.n ? e : G.n) - b);
}

// number of keys of run[0, len) that precede key x of a later (le = true: x's run comes
// after this one, so equal keys precede: upper bound) or earlier (lower bound) run,
// searched in [lo, hi]
__device__ __forceinline__ uint32_t m4_bound(const uint32_t *run, uint32_t lo, uint32_t hi, uint32_t x, bool le,
                                             uint32_t flip) {
    const uint32_t xf = x ^ flip;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint32_t v = run[mid] ^ flip;
        if (v < xf || (le && v == xf)) lo = mid + 1u;
        else hi = mid;
    }
    return lo;
}

// every M4_S-th key of every run, compacted: samp[g spg + k spr + q] = run k of group g at q M4_S
// (the rank searches then run over n / M4_S contiguous words instead of one 64-B line per
// probe scattered over the whole array)
__global__ __launch_bounds__(256) void k_m4_sample(const uint32_t *__restrict__ src, M4Geo G,
                                                   uint32_t *__restrict__ samp) {
    const uint32_t sid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t g = sid / G.spg, w = sid % G.spg, spr = G.r / M4_S;
    if (g >= G.ngroups) return;
    const uint32_t k = w / spr, q = w % spr;
    const uint64_t pos = (uint64_t)g * 4u * G.r + (uint64_t)k * G.r + (uint64_t)q * M4_S;
    samp[sid] = pos < G.n ? ld_stream<NT_MERGE>(src + pos) : 0u;
}

constexpr uint32_t M4_RB = 256;                // threads per rank workgroup
constexpr uint32_t M4_RSPT = 2;                // samples per thread
constexpr uint32_t M4_RT = M4_RB * M4_RSPT;    // samples per rank workgroup
constexpr uint32_t M4_RW = 1024;               // most samples of another run held in LDS per workgroup

// one round of the cut search: A - 1 probes of each of the three runs loaded at once, each
// run's range [lo, hi] narrowed A-fold
template <int A>
__device__ __forceinline__ void m4_cut_round(const uint32_t *const (&run)[3], uint32_t (&lo)[3], uint32_t (&hi)[3],
                                             const bool (&le)[3], uint32_t xf, uint32_t flip) {
    uint32_t v[3][A - 1], step[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        step[i] = (hi[i] - lo[i] + (uint32_t)(A - 1)) / (uint32_t)A;
#pragma unroll
        for (int p = 0; p < A - 1; ++p) {  // probe key lo + (p + 1) step - 1, clamped into the run (unused then)
            const uint32_t idx = lo[i] + (uint32_t)(p + 1) * step[i] - 1u;
            const uint32_t top = hi[i] ? hi[i] - 1u : 0u;
            v[i][p] = run[i][idx < top ? idx : top];
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        uint32_t t = 0u;
#pragma unroll
        for (int p = 0; p < A - 1; ++p) {
            const uint32_t idx = lo[i] + (uint32_t)(p + 1) * step[i] - 1u, vf = v[i][p] ^ flip;
            t += (idx < hi[i] && (vf < xf || (le[i] && vf == xf))) ? 1u : 0u;
        }
        const uint32_t nhi = lo[i] + (t + 1u) * step[i] - 1u;  // probe t failed (none does when t = A - 1)
        hi[i] = step[i] && t < (uint32_t)(A - 1) ? (nhi < hi[i] ? nhi : hi[i]) : hi[i];
        lo[i] += t * step[i];
    }
}

// a boundary sample (merged index m, a multiple of M4_M): its cut in every run -- in run j
// between the last preceding sample and the next, so within one sample gap.  The other three
// runs are searched together, 8-ary: each round loads 7 probes of every run at once and
// narrows each gap 8-fold, so the < M4_S keys of a gap take 3 rounds of loads.  (r29, per pass
// at 2^28: one binary search per run in turn, 21 dependent HBM loads, left the rank kernel at
// 0.075 ms, 0.047 without any cut; 16 + 7 probes per run written with conditional loads,
// which the compiler serialised, 0.149 ms; r30: 15 + 7 probes in two rounds of m4_cut_round,
// 0.090 against 0.075 ms for the three rounds.)
__device__ __forceinline__ void m4_write_cut(const uint32_t *src, const M4Geo &G, uint32_t flip, uint32_t g, uint32_t k,
                                             uint32_t q, uint32_t x, const uint32_t (&cnt)[4], const uint32_t (&len)[4],
                                             uint4 *bnd) {
    static_assert(M4_S <= 8 * 8 * 8, "three 8-ary rounds cover a sample gap");
    const uint32_t m = q + cnt[0] + cnt[1] + cnt[2] + cnt[3];
    if (m == 0u || m % M4_M != 0u) return;
    const uint32_t *gb = src + (size_t)g * 4u * G.r;
    const uint32_t xf = x ^ flip;
    const uint32_t *run[3];
    uint32_t lo[3], hi[3];  // the cut (keys of the run preceding x) is in [lo, hi]
    bool le[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const uint32_t j = (uint32_t)i + ((uint32_t)i >= k);
        run[i] = len[j] ? gb + (size_t)j * G.r : src;  // (an empty run's probes read a valid word, unused)
        le[i] = j < k;
        lo[i] = cnt[j] ? (cnt[j] - 1u) * M4_S + 1u : 0u;
        hi[i] = cnt[j] * M4_S < len[j] ? cnt[j] * M4_S : len[j];
        hi[i] = hi[i] < lo[i] ? lo[i] : hi[i];
    }
#pragma unroll
    for (int round = 0; round < 3; ++round) m4_cut_round<8>(run, lo, hi, le, xf, flip);
    uint32_t cut[4];
#pragma unroll
    for (int i = 0; i < 3; ++i) cut[i + (i >= (int)k)] = lo[i];
    cut[k] = q * M4_S;
    bnd[(size_t)g * G.bpg + m / M4_M] = make_uint4(cut[0], cut[1], cut[2], cut[3]);
}

// every sample's merged-order index; boundaries (every M4_M-th) write their cuts.  A
// workgroup's M4_RT samples are consecutive in one run k (when the run has that many), so
// each count is monotone over them: six 32-lane groups first count the tile's first and last
// sample in the three other runs (32-ary searches over the compacted samples: log32(r / M4_S)
// rounds of loads), the windows of samples between those brackets are loaded into LDS (for
// uniform keys about M4_RT each), and every thread then searches its samples' brackets in
// LDS.  r29 at 2^28, per pass: one full binary search per sample and run 0.116 ms (a chain
// of log2(r / M4_S) scattered L2 loads); this form 0.074-0.078 ms with 1 or 2 samples per
// thread, 0.101 with 4.
// waves per SIMD the register budget is set for: 6 = 80 VGPRs, 19 of them spilled (r30:
// 0.075 -> 0.072 ms per pass; 84 VGPRs, 5 waves, no spill before; 8 waves = 64 VGPRs, 62
// spilled, 0.096 ms; profiles/r30_ab_rank_cuts.txt)
#ifndef LABSORT_RANK_OCC
#define LABSORT_RANK_OCC 6
#endif
#define M4_RANK_LB __launch_bounds__(M4_RB, LABSORT_RANK_OCC)
__global__ M4_RANK_LB void k_m4_rank(const uint32_t *__restrict__ src, M4Geo G, uint32_t flip,
                                                   const uint32_t *__restrict__ samp, uint4 *__restrict__ bnd) {
    __shared__ uint32_t win[3][M4_RW];
    __shared__ uint32_t s_br[6];
    const uint32_t tid = threadIdx.x, s0 = blockIdx.x * M4_RT, spr = G.r / M4_S;  // samples per full run
    const uint32_t g = s0 / G.spg, k = (s0 % G.spg) / spr, q0 = (s0 % G.spg) % spr;
    if (g >= G.ngroups) return;
    if (q0 + M4_RT > spr) {
        // runs shorter than a tile: one full search per sample and run (the tile may span
        // groups: each sample's own group, run and run lengths)
        for (uint32_t e = 0; e < M4_RSPT; ++e) {
            const uint32_t sid = s0 + tid + e * M4_RB, w = sid % G.spg, gg = sid / G.spg, kk = w / spr, q = w % spr;
            if (gg >= G.ngroups) continue;
            uint32_t len[4], cnt[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) len[j] = m4_run_len(G, gg, (uint32_t)j);
            if (q >= (len[kk] + M4_S - 1) / M4_S) continue;
            const uint32_t *ts = samp + (size_t)gg * G.spg;
            const uint32_t x = ts[(size_t)kk * spr + q];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                cnt[j] = (uint32_t)j == kk ? 0u
                                           : m4_bound(ts + (size_t)j * spr, 0u, (len[j] + M4_S - 1) / M4_S, x, (uint32_t)j < kk, flip);
            m4_write_cut(src, G, flip, gg, kk, q, x, cnt, len, bnd);
        }
        return;
    }
    uint32_t len[4], ns[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        len[j] = m4_run_len(G, g, (uint32_t)j);
        ns[j] = (len[j] + M4_S - 1) / M4_S;
    }
    if (q0 >= ns[k]) return;  // past a short last run: every sample of the tile (uniform)
    const uint32_t *gs = samp + (size_t)g * G.spg;  // the group's samples, run j at j spr
    const uint32_t qlast = q0 + M4_RT - 1u < ns[k] - 1u ? q0 + M4_RT - 1u : ns[k] - 1u;
    if (tid < 192u) {
        const uint32_t l = tid & 31u, sidx = tid >> 5;  // search 0..5: run i = sidx % 3, first / last sample
        const uint32_t i = sidx % 3u, j = i + (i >= k);
        const uint32_t *js = gs + (size_t)j * spr;
        const uint32_t xf = gs[(size_t)k * spr + (sidx < 3u ? q0 : qlast)] ^ flip;
        const bool le = j < k;
        uint32_t lo = 0u, hi = ns[j];  // the count is in [lo, hi]
        while (lo < hi) {
            const uint32_t step = (hi - lo + 31u) >> 5;
            const uint32_t pp = lo + (l + 1u) * step - 1u;  // probe sample pp
            bool pred = false;
            if (pp < hi) {
                const uint32_t v = js[pp] ^ flip;
                pred = v < xf || (le && v == xf);
            }
            const uint64_t bal = __ballot(pred);
            const uint32_t t = __builtin_popcount((uint32_t)(tid & 32u ? bal >> 32 : bal));
            const uint32_t nhi = lo + (t + 1u) * step - 1u;
            hi = nhi < hi ? nhi : hi;
            lo += t * step;
        }
        if (l == 0u) s_br[sidx] = lo;
    }
    __syncthreads();
    uint32_t lo[3], w[3], wmax = 0u;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        lo[i] = s_br[i];
        w[i] = s_br[i + 3] - s_br[i];
        wmax = w[i] > wmax ? w[i] : wmax;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const uint32_t j = (uint32_t)i + ((uint32_t)i >= k);
        if (w[i] <= M4_RW)
            for (uint32_t e = tid; e < w[i]; e += M4_RB) win[i][e] = gs[(size_t)j * spr + lo[i] + e];
    }
    __syncthreads();
    uint32_t xf[M4_RSPT], c[M4_RSPT][3];
#pragma unroll
    for (uint32_t e = 0; e < M4_RSPT; ++e) {
        const uint32_t q = q0 + tid + e * M4_RB;
        xf[e] = gs[(size_t)k * spr + (q < ns[k] ? q : qlast)] ^ flip;
#pragma unroll
        for (int i = 0; i < 3; ++i) c[e][i] = lo[i];
    }
    // the bracketed searches of all the thread's samples and runs interleaved, branch-free
    for (uint32_t step = wmax ? 1u << (31 - __builtin_clz(wmax)) : 0u; step; step >>= 1) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const uint32_t j = (uint32_t)i + ((uint32_t)i >= k);
#pragma unroll
            for (uint32_t e = 0; e < M4_RSPT; ++e) {
                const uint32_t p = c[e][i] + step;  // probe sample p - 1
                const bool in = p <= lo[i] + w[i];
                const uint32_t v = in ? (w[i] <= M4_RW ? win[i][p - 1u - lo[i]] : gs[(size_t)j * spr + p - 1u]) ^ flip : 0u;
                if (in && (v < xf[e] || (j < k && v == xf[e]))) c[e][i] = p;
            }
        }
    }
    // the thread's boundary samples (about one in M4_M) taken one per round: a wave runs the
    // cut's three dependent load rounds once when no lane holds two boundaries, instead of
    // once per sample slot (r30 at 2^28: 0.077 -> 0.070 ms and 0.087 -> 0.075 ms per pass on
    // two boxes; two rounds, 16-ary then 8-ary, 0.090 ms: profiles/r30_ab_rank_cuts.txt)
    uint32_t pend = 0u;
#pragma unroll
    for (uint32_t e = 0; e < M4_RSPT; ++e) {
        const uint32_t q = q0 + tid + e * M4_RB;
        const uint32_t m = q + c[e][0] + c[e][1] + c[e][2];
        if (q < ns[k] && m != 0u && m % M4_M == 0u) pend |= 1u << e;
    }
    while (__any(pend != 0u)) {
        if (pend != 0u) {
            const uint32_t e = (uint32_t)__builtin_ctz(pend);
            pend &= pend - 1u;
            uint32_t cnt[4], cc[3], x = 0u;
#pragma unroll
            for (uint32_t ee = 0; ee < M4_RSPT; ++ee)
                if (ee == e) {
                    x = xf[ee];
#pragma unroll
                    for (int i = 0; i < 3; ++i) cc[i] = c[ee][i];
                }
            cnt[k] = 0u;
#pragma unroll
            for (int i = 0; i < 3; ++i) cnt[i + (i >= (int)k)] = cc[i];
            m4_write_cut(src, G, flip, g, k, q0 + tid + e * M4_RB, x ^ flip, cnt, len, bnd);
        }
    }
}

// merge-path co-rank in LDS: A elements among the first d of merge(A, B) (FLIP: int32 order).
// r31, measured slower (profiles/r31_ab_merge4.txt): fixed power-of-two steps with a wave-uniform
// count (the wave's largest range, from the block geometry on scalars) and running probe
// pointers: 10 % fewer VALU per pass, but every lane's first probes share A's word and fall
// on B at an 8-word lane stride, and LDS bank conflicts rose 150 M -> 222 M cycles: 0.771 vs
// 0.653 ms.  The probes of this loop (midpoints ~4 words apart across lanes, 4-way conflicts)
// are most of the kernel's conflict cycles, and the kernel is VALU- (~80 %) and LDS- (~67 %)
// busy at once.  r29, measured slower: a branch-free form with a workgroup-uniform number of halving steps
// (7 VALU per step instead of 9; +0.09 ms per pass: the data-dependent loop stops early), and
// two-step searches (the co-ranks of every 64th diagonal first, by two waves, then each thread
// within its 64: +0.10 ms per pass from the two extra barriers per block)
typedef __attribute__((address_space(3))) const uint32_t m4_lds_u32;
__device__ __forceinline__ uint32_t m4_lds_addr(const uint32_t *p) { return (uint32_t)(uintptr_t)(m4_lds_u32 *)p; }
__device__ __forceinline__ uint32_t m4_lds_ld(uint32_t a) { return *(m4_lds_u32 *)(uintptr_t)a; }
// (r31) the bounds are kept as LDS byte addresses of A: the midpoint's address is
// ((lo + hi) / 2) & ~3 and its B partner one subtraction away (B[d - 1 - mid] at bk - mid):
// 9 VALU per step instead of 10, the same probes (0.718 -> 0.709 ms per four-way pass)
template <bool FLIP>
__device__ __forceinline__ uint32_t m4_corank(const uint32_t *A, uint32_t la, const uint32_t *B, uint32_t lb, uint32_t d) {
    constexpr uint32_t flip = FLIP ? 0x80000000u : 0u;
    const uint32_t lo = d > lb ? d - lb : 0u, hi = d < la ? d : la;
    const uint32_t a0 = m4_lds_addr(A), bk = m4_lds_addr(B) + 4u * (d - 1u) + a0;
    uint32_t lob = a0 + 4u * lo, hib = a0 + 4u * hi;
    while (lob < hib) {
        const uint32_t midb = ((lob + hib) >> 1) & ~3u;
        if ((m4_lds_ld(midb) ^ flip) <= (m4_lds_ld(bk - midb) ^ flip)) lob = midb + 4u;
        else hib = midb;
    }
    return (lob - a0) >> 2;
}

// 8 consecutive LDS words base[i .. i + 8) by five 8-B reads of the 10 words from i rounded
// down to even, and one select per word (16-B reads needed three selects per word; eight 4-B
// reads, no selects: 0.691 vs 0.687 ms per pass, r29; r31 again, as four ds_read2_b32 with
// 46 VALU fewer per block: 0.782 vs 0.771 ms and 0.7138 vs 0.7089 ms, profiles/r31_ab_merge4.txt)
template <int W = M4_KPT>
__device__ __forceinline__ void m4_read8(const uint32_t *base, uint32_t i, uint32_t (&w)[W]) {
    const uint32_t a = i & ~1u;
    const bool odd = (i & 1u) != 0u;
    const uint2 *p = reinterpret_cast<const uint2 *>(base + a);
    uint32_t b[W + 2];
#pragma unroll
    for (int q = 0; q < W / 2 + 1; ++q) {
        const uint2 v = p[q];
        b[2 * q] = v.x;
        b[2 * q + 1] = v.y;
    }
    // (a bit select: as `odd ? b[j + 1] : b[j]` the compiler indexed b[] dynamically through
    // the scratch stack)
    const uint32_t m = odd ? 0xFFFFFFFFu : 0u;
#pragma unroll
    for (int j = 0; j < W; ++j) w[j] = (b[j] & ~m) | (b[j + 1] & m);
}

// the W smallest of A[ai, ai + W) and B[bi, bi + W), by a bitonic merge of A ascending with B
// descending (only the lower half of the network is kept).  A and B are LDS word offsets into
// `buf` (8-B aligned); each run is followed by W pad words of +inf, so the windows need no
// bounds (equal keys are identical words: a pad equal to a key changes no output).
template <bool FLIP, int W = M4_KPT>
__device__ __forceinline__ void m4_window_merge(const uint32_t *buf, uint32_t A, uint32_t ai, uint32_t B, uint32_t bi,
                                                uint32_t (&r)[W]) {
    constexpr uint32_t flip = FLIP ? 0x80000000u : 0u;
    uint32_t wa[W], wb[W], x[2 * W];
    m4_read8<W>(buf, A + ai, wa);
    m4_read8<W>(buf, B + bi, wb);
#pragma unroll
    for (int j = 0; j < W; ++j) {
        x[j] = wa[j] ^ flip;
        x[2 * W - 1 - j] = wb[j] ^ flip;
    }
#pragma unroll
    for (int s = W; s >= 1; s >>= 1) {
#pragma unroll
        for (int i = 0; i < 2 * W; ++i) {
            if ((i & s) == 0) {
                const uint32_t lo = min(x[i], x[i + s]), hi = max(x[i], x[i + s]);
                x[i] = lo;
                x[i + s] = hi;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < W; ++j) r[j] = x[j] ^ flip;
}

// (r31: level 2 at 16 outputs per thread -- half that level's co-rank searches, by the first
// 256 threads, with 16-word pads after A+B and C+D -- needs 18 VGPRs of spills at the kernel's
// 64-register budget: 1.097 vs 0.660 ms, profiles/r31_ab_merge4.txt)

constexpr uint32_t M4_PAD = M4_KPT;  // +inf words after every run in LDS
static_assert((M4_M + 3) * M4_S + 4 * M4_PAD <= M4_CAP, "a block's padded LDS image fits one load pass of the threads");
// buf[p]: a block's keys A | pad | B | pad | C | pad | D | pad, then its output staging;
// buf[1 - p]: level 1's A+B | pad | C+D | pad, then the next block's keys (p alternates)
constexpr uint32_t M4_BUFW = M4_CAP + 4 * M4_PAD + 16;
struct alignas(16) M4Smem {
    alignas(16) uint32_t buf[2][M4_BUFW];
    uint4 lo[M4_MAX_PER + 1];  // each of the workgroup's blocks' start cuts (read once, at entry)
};

struct M4Blk {
    uint32_t bad;  // inconsistent cuts (cannot happen): the block is skipped and reported
    uint32_t g;    // group
    uint32_t lo[4], len[4];
    uint32_t out;  // output position of the block's first key
    uint32_t tot;
};

// block id's geometry; lo = the LDS table of the workgroup's start cuts, t = id's entry in it
// (the next entry is the block's end when it is in the same group)
__device__ __forceinline__ M4Blk m4_block(const M4Geo &G, const uint4 *lo, uint32_t id, uint32_t t) {
    M4Blk q;
    const uint32_t g = id / G.bpg, b = id % G.bpg;
    uint32_t rl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) rl[j] = m4_run_len(G, g, (uint32_t)j);
    uint32_t ns = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) ns += (rl[j] + M4_S - 1) / M4_S;
    const uint32_t nb = (ns + M4_M - 1) / M4_M;
    // (workgroup-uniform: readfirstlane keeps the geometry in SGPRs)
    auto uni = [](uint4 v) {
        return make_uint4(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                          __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w));
    };
    const uint4 l4 = uni(lo[t]);
    const uint4 h4 = b + 1u < nb ? uni(lo[t + 1u]) : make_uint4(rl[0], rl[1], rl[2], rl[3]);
    q.lo[0] = l4.x, q.lo[1] = l4.y, q.lo[2] = l4.z, q.lo[3] = l4.w;
    q.len[0] = h4.x - l4.x, q.len[1] = h4.y - l4.y, q.len[2] = h4.z - l4.z, q.len[3] = h4.w - l4.w;
    q.g = g;
    q.out = g * 4u * G.r + l4.x + l4.y + l4.z + l4.w;
    q.tot = q.len[0] + q.len[1] + q.len[2] + q.len[3];
    // (cannot happen with consistent cuts; a broken table must not send loads or stores out
    // of the runs: the block is skipped and the kernel sets the workspace's error word, which
    // labsort_workspace_status reports as LABSORT_ERR_DEVICE)
    q.bad = 0u;
    if (h4.x < l4.x || h4.y < l4.y || h4.z < l4.z || h4.w < l4.w || h4.x > rl[0] || h4.y > rl[1] || h4.z > rl[2] ||
        h4.w > rl[3] || q.tot > M4_CAP - 4 * M4_PAD) {
        q.tot = 0u;
        q.bad = 1u;
#pragma unroll
        for (int j = 0; j < 4; ++j) q.len[j] = 0u;
    }
    return q;
}

// workgroup: blocks [b0, b1) of the flat list in turn.  Two LDS buffers alternate roles, so
// a block takes three barriers: keys in X -> level 1 into Y -> level 2 back into X (staging)
// -> the stores read X while the next block's keys go into Y, which becomes its X (r29: four
// barriers with fixed in / mid / staging roles, 0.685 ms per pass at 2^28)
// WIDE: groups of more than 2^30 keys (runs of 2^29, n > 2^30): 64-bit byte offsets from
// the group base (below that a 32-bit offset, added to the base in the load's address)
template <bool FLIP, bool WIDE>
__global__ __launch_bounds__(M4_BLOCK, 8) void k_m4_merge(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                                          M4Geo G, const uint4 *__restrict__ bnd, uint32_t per,
                                                          uint32_t *__restrict__ samp_out, uint32_t *__restrict__ err) {
    constexpr uint32_t PADV = FLIP ? 0x7FFFFFFFu : 0xFFFFFFFFu;  // +inf in key order
    __shared__ M4Smem sm;
    const uint32_t tid = threadIdx.x;
    const uint32_t b0 = blockIdx.x * per;
    if (b0 >= G.nblocks) return;
    const uint32_t b1 = b0 + per < G.nblocks ? b0 + per : G.nblocks;
    // block q's LDS image into registers, by LDS position: position p = tid + j BLOCK of
    // A | pad | B | pad | C | pad | D | pad (window k at S_k, its keys at a 32-bit offset
    // delta_k + p from the group's base; the pads and everything past D hold +inf), so the
    // store into LDS is one write per word at a fixed offset (r31: the put's per-word LDS
    // shifts and pad writes were ~12 % of the kernel's VALU; a wave-uniform fast path for
    // chunks inside one window, tested on scalars, measured slower: 0.757 vs 0.680 ms)
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(tid) & ~63u, lane = tid & 63u;
    auto load = [&](const M4Blk &q, uint32_t (&v)[M4_KPT]) {
        const uint32_t S1 = q.len[0] + M4_PAD, S2 = S1 + q.len[1] + M4_PAD, S3 = S2 + q.len[2] + M4_PAD;
        const uint32_t E0 = q.len[0], E1 = S1 + q.len[1], E2 = S2 + q.len[2], E3 = S3 + q.len[3];
        const uint32_t D0 = q.lo[0], D1 = G.r + q.lo[1] - S1, D2 = 2u * G.r + q.lo[2] - S2, D3 = 3u * G.r + q.lo[3] - S3;
        const uint32_t *gbase = src + (size_t)q.g * 4u * G.r;
        // the selected values held in VGPRs once per block: as scalars every select of the
        // chains below needed a v_mov of its operand first (one scalar operand per VALU op)
        uint32_t e[4] = {E0, E1, E2, E3}, dl[4] = {D0, D1, D2, D3};
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            asm("" : "+v"(e[w]));
            asm("" : "+v"(dl[w]));
        }
#pragma unroll
        for (int j = 0; j < M4_KPT; ++j) {
            const uint32_t p = wbase + lane + (uint32_t)j * M4_BLOCK;
            const uint32_t ee = p >= S3 ? e[3] : p >= S2 ? e[2] : p >= S1 ? e[1] : e[0];
            const uint32_t d = p >= S3 ? dl[3] : p >= S2 ? dl[2] : p >= S1 ? dl[1] : dl[0];
            // (a saddr load at a 32-bit byte offset unless the group's bytes pass 2^32)
            const size_t off = WIDE ? (size_t)(p + d) * 4u : (size_t)(uint32_t)((p + d) * 4u);
            v[j] = p < ee ? ld_stream<NT_MERGE>(reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(gbase) + off))
                         : PADV;
        }
    };
    auto put = [&](uint32_t *X, const uint32_t (&v)[M4_KPT]) {
#pragma unroll
        for (int j = 0; j < M4_KPT; ++j) X[wbase + lane + (uint32_t)j * M4_BLOCK] = v[j];
    };
    // the start cuts of blocks b0 .. b1 (a group's first block starts at 0) into LDS: one
    // global round trip here instead of one before every block's key loads
    for (uint32_t t = tid; t <= b1 - b0; t += M4_BLOCK) {
        const uint32_t id = b0 + t;
        sm.lo[t] = (id < G.nblocks && id % G.bpg) ? bnd[id] : make_uint4(0u, 0u, 0u, 0u);
    }
    __syncthreads();
    uint32_t nx[M4_KPT];
    M4Blk cur = m4_block(G, sm.lo, b0, 0u);
    load(cur, nx);
    put(sm.buf[0], nx);
    M4Blk nxt = cur;
    if (b0 + 1u < b1) {
        nxt = m4_block(G, sm.lo, b0 + 1u, 1u);
        load(nxt, nx);
    }
    uint32_t p = 0u;
    for (uint32_t id = b0; id < b1; ++id) {
        uint32_t *X = sm.buf[p], *Y = sm.buf[p ^ 1u];
        if (cur.bad && err && tid == 0u) err[0] = 1u;
        const uint32_t la = cur.len[0], lb = cur.len[1], lc = cur.len[2], ld = cur.len[3];
        const uint32_t oB = la + M4_PAD, oC = oB + lb + M4_PAD, oD = oC + lc + M4_PAD;  // LDS offsets (A at 0)
        const uint32_t lab = la + lb, lcd = lc + ld, nab = (lab + M4_KPT - 1) / M4_KPT, ncd = (lcd + M4_KPT - 1) / M4_KPT;
        const uint32_t cdo = nab * M4_KPT + M4_PAD;  // C+D's offset in Y
        __syncthreads();  // X holds the block; the previous block's stores (from Y) are done
        // level 1: A+B (threads < nab) and C+D, X -> Y
        {
            const bool ab = tid < nab;
            const uint32_t d = (ab ? tid : tid - nab) * M4_KPT;
            const uint32_t oX = ab ? 0u : oC, oY = ab ? oB : oD;
            const uint32_t l1 = ab ? la : lc, l2 = ab ? lb : ld;
            if (d < l1 + l2) {
                const uint32_t ai = m4_corank<FLIP>(X + oX, l1, X + oY, l2, d);
                uint32_t r[M4_KPT];
                m4_window_merge<FLIP>(X, oX, ai, oY, d - ai, r);
                uint32_t *o = Y + (ab ? 0u : cdo) + d;
#pragma unroll
                for (int j = 0; j < M4_KPT; j += 4)
                    *reinterpret_cast<uint4 *>(o + j) = make_uint4(r[j], r[j + 1], r[j + 2], r[j + 3]);
            }
            if (tid < 2u * M4_PAD)  // pads after A+B's and C+D's last 8-word rows
                Y[(tid < M4_PAD ? nab * M4_KPT : cdo + ncd * M4_KPT) + tid % M4_PAD] = PADV;
        }
        __syncthreads();  // Y holds A+B and C+D; X is free
        // level 2: (A+B)+(C+D), Y -> X (16-B writes at the thread's diagonal)
        const uint32_t tot = cur.tot, ph = cur.out & 3u;
        {
            const uint32_t d = tid * M4_KPT;
            if (d < tot) {
                const uint32_t ai = m4_corank<FLIP>(Y, lab, Y + cdo, lcd, d);
                uint32_t r[M4_KPT];
                m4_window_merge<FLIP>(Y, 0u, ai, cdo, d - ai, r);
#pragma unroll
                for (int j = 0; j < M4_KPT; j += 4)
                    *reinterpret_cast<uint4 *>(X + d + j) = make_uint4(r[j], r[j + 1], r[j + 2], r[j + 3]);
            }
        }
        __syncthreads();  // the block's output staged in X; Y is free
        // store: 16-B chunks aligned in the output (staging word = output word - ph), the
        // partial chunks at both ends by words
        const uint32_t nch = (ph + tot + 3u) / 4u;
        uint32_t *ob = dst + (cur.out - ph);
        // (samp_out: the next four-way pass's samples, every M4_S-th output word)
        const uint32_t obase = cur.out - ph;
        for (uint32_t c = tid; c < nch; c += M4_BLOCK) {
            const uint32_t w0 = 4u * c;
            if (w0 >= ph && w0 + 4u <= ph + tot) {
                const uint32_t *sw = X + (w0 - ph);
                __builtin_nontemporal_store(u32x4{sw[0], sw[1], sw[2], sw[3]}, reinterpret_cast<u32x4 *>(ob + w0));
                if (samp_out && ((obase + w0) & (M4_S - 1u)) == 0u) samp_out[(obase + w0) / M4_S] = sw[0];
            } else {
#pragma unroll
                for (uint32_t e = 0; e < 4u; ++e)
                    if (w0 + e >= ph && w0 + e < ph + tot) {
                        ob[w0 + e] = X[w0 + e - ph];
                        if (samp_out && ((obase + w0 + e) & (M4_S - 1u)) == 0u)
                            samp_out[(obase + w0 + e) / M4_S] = X[w0 + e - ph];
                    }
            }
        }
        // the next block's keys into Y (its X), and the one after into registers
        if (id + 1u < b1) {
            put(Y, nx);
            cur = nxt;
            if (id + 2u < b1) {
                nxt = m4_block(G, sm.lo, id + 2u, id + 2u - b0);
                load(nxt, nx);
            }
        }
        p ^= 1u;
    }
}

// Key/value four-way merge (payloads of 4 bytes; labsort_sort_pairs_device with
// LABSORT_ALGO_MERGE).  The same blocks, rank and schedule as k_m4_merge, with every key's
// payload carried beside it through both LDS buffers; each level merges stably ("A before
// equal B", lab.cu:163-170) by sorting (key, slot) words, m4_merge8_kv.  The four-way
// order (key, run, position) and the runs' input order make the merge sort stable, as the
// pairwise passes were.
struct alignas(16) M4SmemKV {
    alignas(16) uint32_t buf[2][M4_BUFW];
    alignas(16) uint32_t vbuf[2][M4_BUFW];
    uint4 lo[M4_MAX_PER + 1];
};

// the thread's 8 outputs at diagonal d of the stable merge of K[oa, oa + la) and
// K[ob, ob + lb): the bitonic network of the keys-only pass on (key, LDS slot) words -- A's
// slots precede B's, so equal keys keep "A before B" and each run's own order -- and the
// payloads read from the winners' slots (r29: 1.366 vs 1.410 ms per pass against the
// pairwise pass's sequential stable merge, 8 dependent LDS reads per thread and level)
template <bool FLIP>
__device__ __forceinline__ void m4_merge8_kv(const uint32_t *K, const uint32_t *V, uint32_t oa, uint32_t la, uint32_t ob,
                                             uint32_t lb, uint32_t d, uint32_t (&r)[M4_KPT], uint32_t (&pv)[M4_KPT]) {
    constexpr uint32_t flip = FLIP ? 0x80000000u : 0u;
    const uint32_t ai = m4_corank<FLIP>(K + oa, la, K + ob, lb, d), bi = d - ai;
    uint64_t x[2 * M4_KPT];
#pragma unroll
    for (int j = 0; j < M4_KPT; ++j) {
        const uint32_t ia = ai + (uint32_t)j, ib = bi + (uint32_t)j;
        const uint32_t ka = K[oa + (ia < la ? ia : 0u)] ^ flip, kb = K[ob + (ib < lb ? ib : 0u)] ^ flip;
        x[j] = ia < la ? ((uint64_t)ka << 32 | (oa + ia)) : ~0ull;
        x[2 * M4_KPT - 1 - j] = ib < lb ? ((uint64_t)kb << 32 | (ob + ib)) : ~0ull;
    }
#pragma unroll
    for (int st = M4_KPT; st >= 1; st >>= 1) {
#pragma unroll
        for (int i = 0; i < 2 * M4_KPT; ++i) {
            if ((i & st) == 0) {
                const uint64_t lo = x[i] < x[i + st] ? x[i] : x[i + st], hi = x[i] < x[i + st] ? x[i + st] : x[i];
                x[i] = lo;
                x[i + st] = hi;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < M4_KPT; ++j) r[j] = (uint32_t)(x[j] >> 32) ^ flip;
#pragma unroll
    for (int j = 0; j < M4_KPT; ++j) {
        const uint32_t sl = (uint32_t)x[j];  // (past both windows: an unused output, any valid slot)
        pv[j] = V[sl < M4_BUFW ? sl : 0u];
    }
}

template <bool FLIP, bool WIDE>
__global__ __launch_bounds__(M4_BLOCK, 4) void k_m4_merge_kv(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                                             const uint32_t *__restrict__ vsrc, uint32_t *__restrict__ vdst,
                                                             M4Geo G, const uint4 *__restrict__ bnd, uint32_t per,
                                                             uint32_t *__restrict__ samp_out, uint32_t *__restrict__ err) {
    __shared__ M4SmemKV sm;
    const uint32_t tid = threadIdx.x;
    const uint32_t b0 = blockIdx.x * per;
    if (b0 >= G.nblocks) return;
    const uint32_t b1 = b0 + per < G.nblocks ? b0 + per : G.nblocks;
    // keys and payloads of block q into registers by LDS position, as k_m4_merge (no +inf
    // pads: the key/value merges check their bounds, so pad positions load nothing)
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(tid) & ~63u, lane = tid & 63u;
    auto load = [&](const M4Blk &q, uint32_t (&v)[M4_KPT], uint32_t (&pl)[M4_KPT]) {
        const uint32_t S1 = q.len[0] + M4_PAD, S2 = S1 + q.len[1] + M4_PAD, S3 = S2 + q.len[2] + M4_PAD;
        uint32_t e[4] = {q.len[0], S1 + q.len[1], S2 + q.len[2], S3 + q.len[3]};
        uint32_t dl[4] = {q.lo[0], G.r + q.lo[1] - S1, 2u * G.r + q.lo[2] - S2, 3u * G.r + q.lo[3] - S3};
#pragma unroll
        for (int w = 0; w < 4; ++w) {  // (held in VGPRs: see k_m4_merge)
            asm("" : "+v"(e[w]));
            asm("" : "+v"(dl[w]));
        }
        const size_t gofs = (size_t)q.g * 4u * G.r;
        const char *gb = reinterpret_cast<const char *>(src + gofs), *vb = reinterpret_cast<const char *>(vsrc + gofs);
#pragma unroll
        for (int j = 0; j < M4_KPT; ++j) {
            const uint32_t p = wbase + lane + (uint32_t)j * M4_BLOCK;
            const uint32_t ee = p >= S3 ? e[3] : p >= S2 ? e[2] : p >= S1 ? e[1] : e[0];
            const uint32_t d = p >= S3 ? dl[3] : p >= S2 ? dl[2] : p >= S1 ? dl[1] : dl[0];
            const size_t off = WIDE ? (size_t)(p + d) * 4u : (size_t)(uint32_t)((p + d) * 4u);
            const bool ok = p < ee;
            v[j] = ok ? ld_stream<NT_MERGE>(reinterpret_cast<const uint32_t *>(gb + off)) : 0u;
            pl[j] = ok ? ld_stream<NT_MERGE>(reinterpret_cast<const uint32_t *>(vb + off)) : 0u;
        }
    };
    auto put = [&](uint32_t *X, uint32_t *XV, const uint32_t (&v)[M4_KPT], const uint32_t (&pl)[M4_KPT]) {
#pragma unroll
        for (int j = 0; j < M4_KPT; ++j) {
            X[wbase + lane + (uint32_t)j * M4_BLOCK] = v[j];
            XV[wbase + lane + (uint32_t)j * M4_BLOCK] = pl[j];
        }
    };
    for (uint32_t t = tid; t <= b1 - b0; t += M4_BLOCK) {
        const uint32_t id = b0 + t;
        sm.lo[t] = (id < G.nblocks && id % G.bpg) ? bnd[id] : make_uint4(0u, 0u, 0u, 0u);
    }
    __syncthreads();
    uint32_t nx[M4_KPT], nv[M4_KPT];
    M4Blk cur = m4_block(G, sm.lo, b0, 0u);
    load(cur, nx, nv);
    put(sm.buf[0], sm.vbuf[0], nx, nv);
    M4Blk nxt = cur;
    if (b0 + 1u < b1) {
        nxt = m4_block(G, sm.lo, b0 + 1u, 1u);
        load(nxt, nx, nv);
    }
    uint32_t p = 0u;
    for (uint32_t id = b0; id < b1; ++id) {
        uint32_t *X = sm.buf[p], *Y = sm.buf[p ^ 1u], *XV = sm.vbuf[p], *YV = sm.vbuf[p ^ 1u];
        if (cur.bad && err && tid == 0u) err[0] = 1u;
        const uint32_t la = cur.len[0], lb = cur.len[1], lc = cur.len[2], ld = cur.len[3];
        const uint32_t oB = la + M4_PAD, oC = oB + lb + M4_PAD, oD = oC + lc + M4_PAD;
        const uint32_t lab = la + lb, lcd = lc + ld, nab = (lab + M4_KPT - 1) / M4_KPT;
        const uint32_t cdo = nab * M4_KPT + M4_PAD;
        __syncthreads();  // X holds the block; the previous block's stores (from Y) are done
        {
            const bool ab = tid < nab;
            const uint32_t d = (ab ? tid : tid - nab) * M4_KPT;
            const uint32_t oX = ab ? 0u : oC, oY = ab ? oB : oD, l1 = ab ? la : lc, l2 = ab ? lb : ld;
            if (d < l1 + l2) {
                uint32_t r[M4_KPT], pv[M4_KPT];
                m4_merge8_kv<FLIP>(X, XV, oX, l1, oY, l2, d, r, pv);
                const uint32_t o = (ab ? 0u : cdo) + d;
#pragma unroll
                for (int j = 0; j < M4_KPT; j += 4) {
                    *reinterpret_cast<uint4 *>(Y + o + j) = make_uint4(r[j], r[j + 1], r[j + 2], r[j + 3]);
                    *reinterpret_cast<uint4 *>(YV + o + j) = make_uint4(pv[j], pv[j + 1], pv[j + 2], pv[j + 3]);
                }
            }
        }
        __syncthreads();  // Y holds A+B and C+D; X is free
        const uint32_t tot = cur.tot, ph = cur.out & 3u;
        {
            const uint32_t d = tid * M4_KPT;
            if (d < tot) {
                uint32_t r[M4_KPT], pv[M4_KPT];
                m4_merge8_kv<FLIP>(Y, YV, 0u, lab, cdo, lcd, d, r, pv);
#pragma unroll
                for (int j = 0; j < M4_KPT; j += 4) {
                    *reinterpret_cast<uint4 *>(X + d + j) = make_uint4(r[j], r[j + 1], r[j + 2], r[j + 3]);
                    *reinterpret_cast<uint4 *>(XV + d + j) = make_uint4(pv[j], pv[j + 1], pv[j + 2], pv[j + 3]);
                }
            }
        }
        __syncthreads();  // the block's output staged in X / XV; Y is free
        const uint32_t nch = (ph + tot + 3u) / 4u;
        uint32_t *ob = dst + (cur.out - ph), *vob = vdst + (cur.out - ph);
        const uint32_t obase = cur.out - ph;
        for (uint32_t c = tid; c < nch; c += M4_BLOCK) {
            const uint32_t w0 = 4u * c;
            if (w0 >= ph && w0 + 4u <= ph + tot) {
                const uint32_t *sw = X + (w0 - ph), *sv = XV + (w0 - ph);
                __builtin_nontemporal_store(u32x4{sw[0], sw[1], sw[2], sw[3]}, reinterpret_cast<u32x4 *>(ob + w0));
                __builtin_nontemporal_store(u32x4{sv[0], sv[1], sv[2], sv[3]}, reinterpret_cast<u32x4 *>(vob + w0));
                if (samp_out && ((obase + w0) & (M4_S - 1u)) == 0u) samp_out[(obase + w0) / M4_S] = sw[0];
            } else {
#pragma unroll
                for (uint32_t e = 0; e < 4u; ++e)
                    if (w0 + e >= ph && w0 + e < ph + tot) {
                        ob[w0 + e] = X[w0 + e - ph];
                        vob[w0 + e] = XV[w0 + e - ph];
                        if (samp_out && ((obase + w0 + e) & (M4_S - 1u)) == 0u)
                            samp_out[(obase + w0 + e) / M4_S] = X[w0 + e - ph];
                    }
            }
        }
        if (id + 1u < b1) {
            put(Y, YV, nx, nv);
            cur = nxt;
            if (id + 2u < b1) {
                nxt = m4_block(G, sm.lo, id + 2u, id + 2u - b0);
                load(nxt, nx, nv);
            }
        }
        p ^= 1u;
    }
}

// geometry of a four-way pass over runs of r keys
M4Geo m4_geo(size_t n, size_t r) {
    M4Geo G{};
    G.n = (uint32_t)n;
    G.r = (uint32_t)r;
    G.ngroups = (uint32_t)((n + 4 * r - 1) / (4 * r));
    G.spg = (uint32_t)(4 * r / M4_S);
    G.bpg = (G.spg + M4_M - 1) / M4_M;
    // the last group's block count (its runs may be short or missing)
    const size_t gb = (size_t)(G.ngroups - 1) * 4 * r;
    size_t ns = 0;
    for (int k = 0; k < 4; ++k) {
        const size_t b = gb + (size_t)k * r;
        const size_t len = b >= n ? 0 : (n - b < r ? n - b : r);
        ns += (len + M4_S - 1) / M4_S;
    }
    G.nblocks = (G.ngroups - 1) * G.bpg + (uint32_t)((ns + M4_M - 1) / M4_M);
    return G;
}

// boundary table (uint4 per block) + the compacted samples
size_t merge4_bnd_words(size_t n, size_t r) {
    if (n <= r) return 0;
    const M4Geo G = m4_geo(n, r);
    return (size_t)G.ngroups * G.bpg * 4 + (((size_t)G.ngroups * G.spg + 3) & ~(size_t)3);
}

hipError_t launch_merge4_pass(const uint32_t *in, uint32_t *out, size_t n, size_t r, uint32_t flip, uint32_t *bnd,
                              const uint32_t *samp_in, uint32_t *samp_out, hipStream_t s, const uint32_t *vin,
                              uint32_t *vout, uint32_t *err) {
    if (n == 0) return hipSuccess;
    if (r % M4_S || n > 0xFFFFFFFFull - 4 * r || !vin != !vout) return hipErrorInvalidValue;
    if ((((uintptr_t)out | (uintptr_t)vout) & 15u) != 0) return hipErrorInvalidValue;  // 16-B stores
    const M4Geo G = m4_geo(n, r);
    const size_t nsamp = (size_t)G.ngroups * G.spg;
    const uint32_t *samp = samp_in;
    if (!samp) {  // no pass before wrote them: gathered here
        uint32_t *own = bnd + (size_t)G.ngroups * G.bpg * 4;
        k_m4_sample<<<(unsigned)((nsamp + 255) / 256), 256, 0, s>>>(in, G, own);
        samp = own;
    }
    k_m4_rank<<<(unsigned)((nsamp + M4_RT - 1) / M4_RT), M4_RB, 0, s>>>(in, G, flip, samp, reinterpret_cast<uint4 *>(bnd));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t want = (uint32_t)(M4_BLOCKS_PER_CU * (cus > 0 ? cus : 256));
    uint32_t per = (G.nblocks + want - 1) / want;
    if (per > M4_MAX_PER) per = M4_MAX_PER;
    const uint32_t g = (G.nblocks + per - 1) / per;
    const bool wide = r > ((size_t)1 << 28);  // a group's byte offsets pass 2^32
    const uint4 *bt = reinterpret_cast<const uint4 *>(bnd);
    if (vin) {
        const uint32_t want_kv = (uint32_t)(2 * (cus > 0 ? cus : 256));  // two 70 KB workgroups per CU
        uint32_t pkv = (G.nblocks + want_kv - 1) / want_kv;
        if (pkv > M4_MAX_PER) pkv = M4_MAX_PER;
        const uint32_t gkv = (G.nblocks + pkv - 1) / pkv;
        auto kv = flip ? (wide ? k_m4_merge_kv<true, true> : k_m4_merge_kv<true, false>)
                       : (wide ? k_m4_merge_kv<false, true> : k_m4_merge_kv<false, false>);
        kv<<<gkv, M4_BLOCK, 0, s>>>(in, out, vin, vout, G, bt, pkv, samp_out, err);
        return hipGetLastError();
    }
    auto k = flip ? (wide ? k_m4_merge<true, true> : k_m4_merge<true, false>)
                  : (wide ? k_m4_merge<false, true> : k_m4_merge<false, false>);
    k<<<g, M4_BLOCK, 0, s>>>(in, out, G, bt, per, samp_out, err);
    return hipGetLastError();
}

}  // namespace labsort
