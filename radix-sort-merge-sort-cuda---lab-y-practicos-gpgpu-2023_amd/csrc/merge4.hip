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
//              its own index plus, per other run, the samples that precede it (binary
//              search over that run's samples: upper bound for earlier runs, lower bound
//              for later ones -- the reference's tie rule generalised to four runs).  Every
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
//              stored as 16-B nontemporal stores.
#include "common.h"
#include "devutil.h"

namespace labsort {

// M4_S (common.h): sample stride (keys)
constexpr uint32_t M4_M = 28;    // samples per block (merged order)
constexpr int M4_BLOCK = 512;    // threads per merge workgroup
constexpr int M4_KPT = 8;        // outputs per thread and merge level
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

// one thread per sample: merged-order index; boundaries (every M4_M-th) write their cuts
__global__ __launch_bounds__(256) void k_m4_rank(const uint32_t *__restrict__ src, M4Geo G, uint32_t flip,
                                                 const uint32_t *__restrict__ samp, uint4 *__restrict__ bnd) {
    const uint32_t sid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t g = sid / G.spg, w = sid % G.spg, spr = G.r / M4_S;  // samples per full run
    if (g >= G.ngroups) return;
    const uint32_t k = w / spr, q = w % spr;
    uint32_t len[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) len[j] = m4_run_len(G, g, (uint32_t)j);
    if ((uint64_t)q * M4_S >= len[k]) return;  // past a short last run
    const uint32_t *gb = src + (size_t)g * 4u * G.r;
    const uint32_t x = samp[sid];
    // samples of the other runs that precede (x, k) in (key, run) order: upper bound in the
    // runs before k, lower bound in the runs after it.  The three searches run interleaved,
    // branch-free, one probe of each per step, so the thread waits on one chain of
    // log2(r / M4_S) dependent loads instead of three in a row.
    const uint32_t xf = x ^ flip;
    uint32_t cnt[4], ns[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        cnt[j] = 0u;
        ns[j] = (uint32_t)j == k ? 0u : (len[j] + M4_S - 1) / M4_S;
    }
    for (uint32_t step = 1u << (31 - __builtin_clz(spr)); step; step >>= 1) {
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t p = cnt[j] + step;
            v[j] = p <= ns[j] ? samp[(size_t)g * G.spg + (size_t)j * spr + p - 1u] ^ flip : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t p = cnt[j] + step;
            const bool le = (uint32_t)j < k;
            if (p <= ns[j] && (v[j] < xf || (le && v[j] == xf))) cnt[j] = p;
        }
    }
    const uint32_t m = q + cnt[0] + cnt[1] + cnt[2] + cnt[3];
    if (m == 0u || m % M4_M != 0u) return;
    // a boundary: its cut in every run -- in run j between the last preceding sample and the
    // next, so within one sample gap (one in M4_M threads gets here; an interleaved
    // branch-free form of these three searches stopped at the gap's start on the device when
    // every sample of the run preceded, r29)
    uint32_t cut[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if ((uint32_t)j == k) {
            cut[j] = q * M4_S;
            continue;
        }
        if (!len[j]) {
            cut[j] = 0u;
            continue;
        }
        const uint32_t lo = cnt[j] ? (cnt[j] - 1u) * M4_S + 1u : 0u;
        const uint32_t hi = cnt[j] * M4_S < len[j] ? cnt[j] * M4_S : len[j];
        cut[j] = m4_bound(gb + (size_t)j * G.r, lo, hi, x, (uint32_t)j < k, flip);
    }
    bnd[(size_t)g * G.bpg + m / M4_M] = make_uint4(cut[0], cut[1], cut[2], cut[3]);
}

// merge-path co-rank in LDS: A elements among the first d of merge(A, B) (FLIP: int32 order)
template <bool FLIP>
__device__ __forceinline__ uint32_t m4_corank(const uint32_t *A, uint32_t la, const uint32_t *B, uint32_t lb, uint32_t d) {
    constexpr uint32_t flip = FLIP ? 0x80000000u : 0u;
    uint32_t lo = d > lb ? d - lb : 0u, hi = d < la ? d : la;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((A[mid] ^ flip) <= (B[d - 1u - mid] ^ flip)) lo = mid + 1u;
        else hi = mid;
    }
    return lo;
}

// 8 consecutive LDS words base[i .. i + 8) by five 8-B reads of the 10 words from i rounded
// down to even, and one select per word (the pass is VALU-bound: r29 counters; 16-B reads
// needed three selects per word, 4-B reads hit the lanes' shared banks 4 ways)
__device__ __forceinline__ void m4_read8(const uint32_t *base, uint32_t i, uint32_t (&w)[M4_KPT]) {
    const uint32_t a = i & ~1u;
    const bool odd = (i & 1u) != 0u;
    const uint2 *p = reinterpret_cast<const uint2 *>(base + a);
    uint32_t b[M4_KPT + 2];
#pragma unroll
    for (int q = 0; q < M4_KPT / 2 + 1; ++q) {
        const uint2 v = p[q];
        b[2 * q] = v.x;
        b[2 * q + 1] = v.y;
    }
    // (a bit select: as `odd ? b[j + 1] : b[j]` the compiler indexed b[] dynamically through
    // the scratch stack)
    const uint32_t m = odd ? 0xFFFFFFFFu : 0u;
#pragma unroll
    for (int j = 0; j < M4_KPT; ++j) w[j] = (b[j] & ~m) | (b[j + 1] & m);
}

// the 8 smallest of A[ai, ai + 8) and B[bi, bi + 8), by a bitonic merge of A ascending with B
// descending.  A and B are LDS word offsets into `buf` (8-B aligned); each run is followed by
// 8 pad words of +inf, so the windows need no bounds (equal keys are identical words: a pad
// equal to a key changes no output).
template <bool FLIP>
__device__ __forceinline__ void m4_window_merge(const uint32_t *buf, uint32_t A, uint32_t ai, uint32_t B, uint32_t bi,
                                                uint32_t (&r)[M4_KPT]) {
    constexpr uint32_t flip = FLIP ? 0x80000000u : 0u;
    uint32_t wa[M4_KPT], wb[M4_KPT], x[2 * M4_KPT];
    m4_read8(buf, A + ai, wa);
    m4_read8(buf, B + bi, wb);
#pragma unroll
    for (int j = 0; j < M4_KPT; ++j) {
        x[j] = wa[j] ^ flip;
        x[2 * M4_KPT - 1 - j] = wb[j] ^ flip;
    }
#pragma unroll
    for (int s = M4_KPT; s >= 1; s >>= 1) {
#pragma unroll
        for (int i = 0; i < 2 * M4_KPT; ++i) {
            if ((i & s) == 0) {
                const uint32_t lo = min(x[i], x[i + s]), hi = max(x[i], x[i + s]);
                x[i] = lo;
                x[i + s] = hi;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < M4_KPT; ++j) r[j] = x[j] ^ flip;
}

constexpr uint32_t M4_PAD = M4_KPT;  // +inf words after every run in LDS
struct alignas(16) M4Smem {
    alignas(16) uint32_t in[M4_CAP + 4 * M4_PAD + 16];  // A | pad | B | pad | C | pad | D | pad; then the output staging
    alignas(16) uint32_t mid[M4_CAP + 4 * M4_PAD + 16]; // level 1: A+B | pad | C+D | pad
    uint4 lo[M4_MAX_PER + 1];                           // each of the workgroup's blocks' start cuts (read once, at entry)
};

struct M4Blk {
    uint32_t g;  // group
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
    // of the runs: the block is skipped and the sort's output check fails instead)
    if (h4.x < l4.x || h4.y < l4.y || h4.z < l4.z || h4.w < l4.w || q.tot > M4_CAP - 2 * M4_KPT) {
        q.tot = 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) q.len[j] = 0u;
    }
    return q;
}

// LABSORT_M4_DIAG (timing builds only, wrong output): 1 = level 1 skipped, 2 = level 2
// skipped (level 1's result stored), 3 = co-rank searches replaced by d / 2
#ifndef LABSORT_M4_DIAG
#define LABSORT_M4_DIAG 0
#endif
// workgroup: blocks [b0, b1) of the flat list in turn
template <bool FLIP>
__global__ __launch_bounds__(M4_BLOCK, 8) void k_m4_merge(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                                          M4Geo G, const uint4 *__restrict__ bnd, uint32_t per,
                                                          uint32_t *__restrict__ samp_out) {
    constexpr uint32_t PADV = FLIP ? 0x7FFFFFFFu : 0xFFFFFFFFu;  // +inf in key order
    __shared__ M4Smem sm;
    const uint32_t tid = threadIdx.x;
    const uint32_t b0 = blockIdx.x * per;
    if (b0 >= G.nblocks) return;
    const uint32_t b1 = b0 + per < G.nblocks ? b0 + per : G.nblocks;
    // keys of block q into registers: element tid + j BLOCK of the windows A | B | C | D.
    // (Each window's source address is a running select over the four, not an index into
    // q.lo[]: a dynamic index put the four bases on the scratch stack, one scratch load per key.)
    auto load = [&](const M4Blk &q, uint32_t (&v)[M4_KPT]) {
        const uint32_t o1 = q.len[0], o2 = o1 + q.len[1], o3 = o2 + q.len[2];
        const uint32_t *gb = src + (size_t)q.g * 4u * G.r;
        const uint32_t *b0 = gb + q.lo[0], *b1 = gb + G.r + q.lo[1] - o1, *b2 = gb + 2u * G.r + q.lo[2] - o2,
                       *b3 = gb + 3u * G.r + q.lo[3] - o3;
#pragma unroll
        for (int j = 0; j < M4_KPT; ++j) {
            const uint32_t i = tid + (uint32_t)j * M4_BLOCK;
            const uint32_t *a = b0;
            a = i >= o1 ? b1 : a;
            a = i >= o2 ? b2 : a;
            a = i >= o3 ? b3 : a;
            v[j] = i < q.tot ? ld_stream<NT_MERGE>(a + i) : 0u;
        }
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
    for (uint32_t id = b0; id < b1; ++id) {
        const uint32_t la = cur.len[0], lb = cur.len[1], lc = cur.len[2], ld = cur.len[3];
        const uint32_t oB = la + M4_PAD, oC = oB + lb + M4_PAD, oD = oC + lc + M4_PAD;  // LDS offsets (A at 0)
        __syncthreads();  // the previous block's output staging (sm.in) has been stored
#pragma unroll
        for (int j = 0; j < M4_KPT; ++j) {
            const uint32_t i = tid + (uint32_t)j * M4_BLOCK;
            const uint32_t k = (i >= la) + (i >= la + lb) + (i >= la + lb + lc);  // window of element i
            if (i < cur.tot) sm.in[i + k * M4_PAD] = nx[j];
        }
        if (tid < 4u * M4_PAD) {  // the pads
            const uint32_t k = tid / M4_PAD, e = tid % M4_PAD;
            const uint32_t end = k == 0 ? la : k == 1 ? oB + lb : k == 2 ? oC + lc : oD + ld;
            sm.in[end + e] = PADV;
        }
        M4Blk nxt = cur;
        if (id + 1u < b1) {
            nxt = m4_block(G, sm.lo, id + 1u, id + 1u - b0);
            load(nxt, nx);
        }
        __syncthreads();  // sm.in holds the block
        const uint32_t lab = la + lb, lcd = lc + ld, nab = (lab + M4_KPT - 1) / M4_KPT, ncd = (lcd + M4_KPT - 1) / M4_KPT;
        const uint32_t cdo = nab * M4_KPT + M4_PAD;  // C+D's offset in sm.mid
        // level 1: A+B (threads < nab) and C+D
        {
            const bool ab = tid < nab;
            const uint32_t d = (ab ? tid : tid - nab) * M4_KPT;
            const uint32_t oX = ab ? 0u : oC, oY = ab ? oB : oD;
            const uint32_t l1 = ab ? la : lc, l2 = ab ? lb : ld;
            if (LABSORT_M4_DIAG != 1 && d < l1 + l2) {
                const uint32_t ai = LABSORT_M4_DIAG == 3 ? min(d / 2, l1) : m4_corank<FLIP>(sm.in + oX, l1, sm.in + oY, l2, d);
                uint32_t r[M4_KPT];
                m4_window_merge<FLIP>(sm.in, oX, ai, oY, d - ai, r);
                uint32_t *o = sm.mid + (ab ? 0u : cdo) + d;
#pragma unroll
                for (int j = 0; j < M4_KPT; j += 4)
                    *reinterpret_cast<uint4 *>(o + j) = make_uint4(r[j], r[j + 1], r[j + 2], r[j + 3]);
            }
            if (tid < 2u * M4_PAD)  // pads after A+B's and C+D's last 8-word rows
                sm.mid[(tid < M4_PAD ? nab * M4_KPT : cdo + ncd * M4_KPT) + tid % M4_PAD] = PADV;
        }
        __syncthreads();  // sm.mid holds A+B and C+D; sm.in is free
        // level 2: (A+B)+(C+D) into the staging buffer (16-B writes at the thread's diagonal)
        const uint32_t tot = cur.tot, ph = cur.out & 3u;
        {
            const uint32_t d = tid * M4_KPT;
            if (LABSORT_M4_DIAG != 2 && d < tot) {
                const uint32_t ai = LABSORT_M4_DIAG == 3 ? min(d / 2, lab) : m4_corank<FLIP>(sm.mid, lab, sm.mid + cdo, lcd, d);
                uint32_t r[M4_KPT];
                m4_window_merge<FLIP>(sm.mid, 0u, ai, cdo, d - ai, r);
#pragma unroll
                for (int j = 0; j < M4_KPT; j += 4)
                    *reinterpret_cast<uint4 *>(sm.in + d + j) = make_uint4(r[j], r[j + 1], r[j + 2], r[j + 3]);
            }
        }
        __syncthreads();  // the block's output staged
        // store: 16-B chunks aligned in the output (staging word = output word - ph), the
        // partial chunks at both ends by words
        const uint32_t nch = (ph + tot + 3u) / 4u;
        uint32_t *ob = dst + (cur.out - ph);
        // (samp_out: the next four-way pass's samples, every M4_S-th output word)
        const uint32_t obase = cur.out - ph;
        for (uint32_t c = tid; c < nch; c += M4_BLOCK) {
            const uint32_t w0 = 4u * c;
            if (w0 >= ph && w0 + 4u <= ph + tot) {
                const uint32_t *sw = sm.in + (w0 - ph);
                __builtin_nontemporal_store(u32x4{sw[0], sw[1], sw[2], sw[3]}, reinterpret_cast<u32x4 *>(ob + w0));
                if (samp_out && ((obase + w0) & (M4_S - 1u)) == 0u) samp_out[(obase + w0) / M4_S] = sw[0];
            } else {
#pragma unroll
                for (uint32_t e = 0; e < 4u; ++e)
                    if (w0 + e >= ph && w0 + e < ph + tot) {
                        ob[w0 + e] = sm.in[w0 + e - ph];
                        if (samp_out && ((obase + w0 + e) & (M4_S - 1u)) == 0u)
                            samp_out[(obase + w0 + e) / M4_S] = sm.in[w0 + e - ph];
                    }
            }
        }
        cur = nxt;
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
                              const uint32_t *samp_in, uint32_t *samp_out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (r % M4_S || n > 0xFFFFFFFFull - 4 * r) return hipErrorInvalidValue;
    const M4Geo G = m4_geo(n, r);
    const size_t nsamp = (size_t)G.ngroups * G.spg;
    const uint32_t *samp = samp_in;
    if (!samp) {  // no pass before wrote them: gathered here
        uint32_t *own = bnd + (size_t)G.ngroups * G.bpg * 4;
        k_m4_sample<<<(unsigned)((nsamp + 255) / 256), 256, 0, s>>>(in, G, own);
        samp = own;
    }
    k_m4_rank<<<(unsigned)((nsamp + 255) / 256), 256, 0, s>>>(in, G, flip, samp, reinterpret_cast<uint4 *>(bnd));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t want = (uint32_t)(M4_BLOCKS_PER_CU * (cus > 0 ? cus : 256));
    uint32_t per = (G.nblocks + want - 1) / want;
    if (per > M4_MAX_PER) per = M4_MAX_PER;
    const uint32_t g = (G.nblocks + per - 1) / per;
    if (flip)
        k_m4_merge<true><<<g, M4_BLOCK, 0, s>>>(in, out, G, reinterpret_cast<const uint4 *>(bnd), per, samp_out);
    else
        k_m4_merge<false><<<g, M4_BLOCK, 0, s>>>(in, out, G, reinterpret_cast<const uint4 *>(bnd), per, samp_out);
    return hipGetLastError();
}

}  // namespace labsort
