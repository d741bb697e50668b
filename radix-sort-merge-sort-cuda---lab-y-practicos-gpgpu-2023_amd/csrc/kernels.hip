// kernels.hip -- hand-written HIP kernels of the labsort path for gfx950 (CDNA4).
//
// Everything here is 32-bit integer / permute work: no MFMA.  Keys are plain
// 32-bit words; signed (int) order is obtained by XOR-ing the sign bit into
// every digit extraction and comparison (`flip`), so one code path serves the
// reference's int keys (lab.h:9) and the north_star's uint32 keys.
//
// Kernel map (reference counterpart in `Sord Radix y Merge/lab.cu`):
//   k_wave_split      radix_sort_kernel :47-87 + exlusiveScan :11-41 -- a 64-key
//                     tile per wave, 1-bit split per iteration with ballot/mbcnt
//                     (the split's scan) and ds_permute (the scatter), early exit
//                     when the tile is sorted (:61).
//   k_hist_seg        letra.pdf's global "totalFalses" generalised to 8-bit digits:
//                     digit 0 per position segment and the joint fields that size the
//                     later passes' segments, in one read of the keys (k_histogram:
//                     the plain form); k_plan8 turns them into every pass's plan.
//   k_onesweep_p      one persistent LSD pass (the default radix above 2^25 keys): lane-
//                     ordered LDS-atomic rank, segmented decoupled look-back for the
//                     global offsets, LDS reorder, coalesced scatter; <true>: key/value.
//                     (k_onesweep: the non-persistent form, 1-bit digits for radix1.)
//   k_tile_sort       stage 1+2 of order_array (lab.cu:323-346): an LDS-resident
//                     32768-key (16384 pairs) LSD radix sort per workgroup.
//   k_merge_pass_p    stage 3 (separators_kernel :209-270 + merge_segments_kernel
//                     :272-300) as merge-path: co-rank searches per output tile
//                     (busquedaPorBiparticion :102-132, same tie rule: A before B on
//                     equal keys) and an LDS merge per tile; k_merge_ab: two arrays.
//                     The four-way pass of the merge sort is in merge4.hip, the
//                     gathered radix (2^16 <= n < 2^25) in gsweep.hip.
#include "common.h"
#include "devutil.h"

#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace labsort {

// ---------------------------------------------------------------------------------
// generator (same formula as oracle/cpu_sort.cpp)
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_fill(uint32_t *__restrict__ out, size_t n, uint64_t seed, int dist,
                                              uint64_t param, uint64_t first) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t gi = first + i;
        const uint64_t z = mix64(seed ^ (gi * 0x9E3779B97F4A7C15ull));
        const uint32_t hi = (uint32_t)(z >> 32);
        uint32_t v;
        switch (dist) {
        case 1: v = (uint32_t)(z >> 33); break;
        case 2: v = hi % 100u; break;
        case 3: v = hi % 1000u; break;
        case 4: v = (uint32_t)gi; break;
        case 5: v = (uint32_t)(param - 1 - gi); break;
        case 6: v = (uint32_t)param; break;
        case 7: v = param >= 32 ? hi : (hi & (uint32_t)((1ull << param) - 1)); break;
        default: v = hi; break;
        }
        out[i] = v;
    }
}

// ---------------------------------------------------------------------------------
// upfront histogram of every digit pass (one read of the keys)
// LDS counters laid out [pass][digit][32 slots], slot = lane & 31, so the 32 lanes
// of a ds_add group always hit 32 different banks (conflict-free for any data).
// ---------------------------------------------------------------------------------
template <int BITS>
__global__ __launch_bounds__(HIST_BLOCK) void k_histogram(const uint32_t *__restrict__ keys, size_t n, uint32_t flip,
                                                          uint32_t *__restrict__ hist) {
    constexpr int R = 1 << BITS, P = (32 + BITS - 1) / BITS, SLOTS = 32;
    constexpr uint32_t RM = R - 1;
    __shared__ uint32_t h[P * R * SLOTS];
    for (int i = threadIdx.x; i < P * R * SLOTS; i += HIST_BLOCK) h[i] = 0u;
    __syncthreads();
    const uint32_t slot = threadIdx.x & 31u;
    auto count = [&](uint32_t k) {
        k ^= flip;
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const uint32_t d = (k >> (p * BITS)) & RM;
            atomicAdd(&h[(p * R + d) * SLOTS + slot], 1u);
        }
    };
    // contiguous chunk per workgroup, multiple of 64 keys
    const size_t per = (((n + gridDim.x - 1) / gridDim.x) + 63) & ~(size_t)63;
    const size_t beg = (size_t)blockIdx.x * per;
    const size_t end = beg + per < n ? beg + per : n;
    if (beg < end) {
        if ((((uintptr_t)(keys + beg)) & 15u) == 0) {
            const uint4 *v = reinterpret_cast<const uint4 *>(keys + beg);
            const size_t nv = (end - beg) / 4;
            size_t i = threadIdx.x;
            for (; i + 3 * HIST_BLOCK < nv; i += 4 * HIST_BLOCK) {
                uint4 x[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) x[u] = v[i + u * HIST_BLOCK];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    count(x[u].x); count(x[u].y); count(x[u].z); count(x[u].w);
                }
            }
            for (; i < nv; i += HIST_BLOCK) {
                const uint4 x = v[i];
                count(x.x); count(x.y); count(x.z); count(x.w);
            }
            for (size_t t = beg + nv * 4 + threadIdx.x; t < end; t += HIST_BLOCK) count(keys[t]);
        } else {
            for (size_t t = beg + threadIdx.x; t < end; t += HIST_BLOCK) count(keys[t]);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < P * R; i += HIST_BLOCK) {
        uint32_t s = 0;
#pragma unroll 8
        for (int q = 0; q < SLOTS; ++q) s += h[i * SLOTS + ((q + i) & (SLOTS - 1))];
        if (s) atomicAdd(&hist[i], s);
    }
}

// ---------------------------------------------------------------------------------
// pass plan: skip passes whose digit is the same for every key; choose buffers so
// the last non-trivial pass writes OUT and no pass scatters in place.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_plan(const uint32_t *__restrict__ hist, uint32_t n, int bits,
                                              int in_is_out, Plan *__restrict__ plan) {
    __shared__ uint32_t triv[MAX_PASSES];
    const int R = 1 << bits, P = (32 + bits - 1) / bits;
    if (threadIdx.x < MAX_PASSES) triv[threadIdx.x] = 0;
    __syncthreads();
    for (int p = 0; p < P; ++p)
        for (int d = threadIdx.x; d < R; d += blockDim.x)
            if (hist[p * R + d] == n) triv[p] = 1;
    __syncthreads();
    if (threadIdx.x != 0) return;
    int act[MAX_PASSES];
    int k = 0;
    for (int p = 0; p < MAX_PASSES; ++p) {
        plan->src[p] = SEL_SKIP;
        plan->dst[p] = SEL_SKIP;
        if (p < P && !triv[p]) act[k++] = p;
    }
    plan->active = (uint32_t)k;
    if (k == 0) {
        plan->copy_from = in_is_out ? SEL_SKIP : SEL_IN;
        return;
    }
    uint32_t d[MAX_PASSES];
    uint32_t cur = SEL_OUT;
    for (int i = k - 1; i >= 0; --i) {
        d[i] = cur;
        cur = (cur == SEL_OUT) ? SEL_TMP : SEL_OUT;
    }
    if (in_is_out && d[0] == SEL_OUT)  // first pass would read and write the same buffer
        for (int i = 0; i < k; ++i) d[i] = (i & 1) ? SEL_OUT : SEL_TMP;
    uint32_t src = SEL_IN;
    for (int i = 0; i < k; ++i) {
        plan->src[act[i]] = src;
        plan->dst[act[i]] = d[i];
        src = d[i];
    }
    plan->copy_from = (d[k - 1] == SEL_OUT) ? SEL_SKIP : d[k - 1];
}

// ---------------------------------------------------------------------------------
// 8-bit radix front end and segment plans.
//
// Every pass runs NSEG independent decoupled look-back chains, one per contiguous
// segment of its input; a segment's base offsets must therefore be known before
// the pass starts:
//   * first active pass: the input is split into NSEG equal position ranges and
//     k_hist_seg (the upfront histogram, workgroups aligned to the ranges) gives
//     each range's digit-0 histogram hps[s][d] (if digit 0 is trivial, the first
//     active pass runs as one chain);
//   * later passes: after a pass on digit p the data is ordered (stably) by digit
//     p, so the keys whose digit p has top nibble g form one contiguous range of the
//     next pass's input (digit p + 1).  That segment's digit-(p+1) histogram is the
//     joint count of (top nibble of digit p, digit p + 1) = a histogram of the 12-bit
//     key field [8p + 4, 8p + 16): a property of the key multiset, so k_hist_seg
//     counts it for p = 0, 1, 2 in the same read of the keys, into joint[p+1][g][d].
//     Digit histograms of passes 1-3 are its marginals.
//     (A pass whose previous active digit is not p - 1 runs as one chain.)
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(HIST_BLOCK) void k_hist_seg(const uint32_t *__restrict__ keys, size_t n, uint32_t flip,
                                                         uint32_t *__restrict__ hps, uint32_t *__restrict__ joint,
                                                         uint32_t bps) {
    constexpr int SL = 32;  // replicated digit-0 counters: the 32 lanes of a ds_add group hit 32 banks
    constexpr int JF = 4096;  // 12-bit joint fields per pass
    __shared__ uint32_t h[256 * SL];
    __shared__ uint32_t hj[3 * JF];
    for (int i = threadIdx.x; i < 256 * SL; i += HIST_BLOCK) h[i] = 0u;
    for (int i = threadIdx.x; i < 3 * JF; i += HIST_BLOCK) hj[i] = 0u;
    __syncthreads();
    const uint32_t slot = threadIdx.x & (SL - 1);
    auto count = [&](uint32_t k) {
        k ^= flip;
        atomicAdd(&h[(k & 255u) * SL + slot], 1u);
#pragma unroll
        for (int p = 0; p < 3; ++p) atomicAdd(&hj[p * JF + ((k >> (8 * p + 4)) & (JF - 1))], 1u);
    };
    // 16 keys of one lane (4 uint4 of 4 consecutive keys): digit 0 as above
    // (replicated slots: contention-free for any data).  Joint fields: with one add per
    // key, keys whose field repeats (small keys: %100, %1000; sorted or clustered input)
    // put many lanes on one LDS counter, which serialises them -- at 2^28 the kernel
    // took 1.85-1.99 ms (%1000, %100) and 1.06 ms (sorted) instead of 0.27 ms (r19).
    // So a field that is the same for a lane's 16 keys, or for one uint4, is added once.
    // The tests run only in waves where some lane's top field repeats within its first
    // uint4 (one compare and a ballot per 16 keys): uniform keys keep the plain adds.
    auto fld = [&](uint32_t k, int p) { return (k >> (8 * p + 4)) & (JF - 1); };
    auto count16 = [&](const uint4 (&c)[4]) {
        uint32_t k[16];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            k[4 * u] = c[u].x ^ flip;
            k[4 * u + 1] = c[u].y ^ flip;
            k[4 * u + 2] = c[u].z ^ flip;
            k[4 * u + 3] = c[u].w ^ flip;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) atomicAdd(&h[(k[j] & 255u) * SL + slot], 1u);
        if (__ballot(fld(k[0], 2) == fld(k[3], 2)) == 0ull) {  // no repeats here
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int j = 0; j < 16; ++j) atomicAdd(&hj[p * JF + fld(k[j], p)], 1u);
            return;
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const uint32_t f0 = fld(k[0], p);
            bool same = fld(k[15], p) == f0;
            if (same) {  // first and last agree: check the rest
#pragma unroll
                for (int j = 1; j < 15; ++j) same &= fld(k[j], p) == f0;
            }
            // the whole wave on one field (sorted or clustered input): one add for it
            const uint32_t w0 = __builtin_amdgcn_readfirstlane(f0);
            const uint64_t act = __ballot(true);
            if (__ballot(same && f0 == w0) == act) {
                if (mbcnt64(act) == 0u) atomicAdd(&hj[p * JF + w0], 16u * (uint32_t)__popcll(act));
                continue;
            }
            if (same) {
                atomicAdd(&hj[p * JF + f0], 16u);
                continue;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t fa = fld(k[4 * u], p);
                const bool s4 = fld(k[4 * u + 3], p) == fa && fld(k[4 * u + 1], p) == fa && fld(k[4 * u + 2], p) == fa;
                if (s4) {
                    atomicAdd(&hj[p * JF + fa], 4u);
                } else {
#pragma unroll
                    for (int j = 4 * u; j < 4 * u + 4; ++j) atomicAdd(&hj[p * JF + fld(k[j], p)], 1u);
                }
            }
        }
    };
    const uint32_t seg = blockIdx.x / bps, part = blockIdx.x % bps;
    const size_t sb = seg_start(seg, n), se = seg_start(seg + 1, n);
    const size_t per = (se - sb + bps - 1) / bps;
    const size_t beg = sb + (size_t)part * per < se ? sb + (size_t)part * per : se;
    const size_t end = beg + per < se ? beg + per : se;
    if ((((uintptr_t)keys) & 15u) == 0) {
        // scalar head up to 16-B alignment, uint4 body, scalar tail
        const size_t abeg = (beg + 3) & ~(size_t)3;
        const size_t vbeg = abeg < end ? abeg : end;
        for (size_t t = beg + threadIdx.x; t < vbeg; t += HIST_BLOCK) count(keys[t]);
        const size_t nv = (end - vbeg) / 4;
        const uint4 *v = reinterpret_cast<const uint4 *>(keys + vbeg);
        size_t i = threadIdx.x;
        // software-pipelined: the next 4 x uint4 load while the current ones are counted
        // (harness/exp/hist_probe.hip: 0.246 -> 0.204 ms at 2^28)
        uint4 c[4], x[4];
        if (i + 3 * HIST_BLOCK < nv) {
#pragma unroll
            for (int u = 0; u < 4; ++u) c[u] = ld_stream4<NT_HIST>(v + i + u * HIST_BLOCK);
        }
        for (; i + 3 * HIST_BLOCK < nv; i += 4 * HIST_BLOCK) {
            if (i + 7 * HIST_BLOCK < nv) {
#pragma unroll
                for (int u = 0; u < 4; ++u) x[u] = ld_stream4<NT_HIST>(v + i + (4 + u) * HIST_BLOCK);
            }
            count16(c);
#pragma unroll
            for (int u = 0; u < 4; ++u) c[u] = x[u];
        }
        for (; i < nv; i += HIST_BLOCK) {
            const uint4 x = ld_stream4<NT_HIST>(v + i);
            count(x.x); count(x.y); count(x.z); count(x.w);
        }
        for (size_t r = vbeg + nv * 4 + threadIdx.x; r < end; r += HIST_BLOCK) count(keys[r]);
    } else {
        for (size_t t = beg + threadIdx.x; t < end; t += HIST_BLOCK) count(keys[t]);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += HIST_BLOCK) {
        uint32_t c = 0;
#pragma unroll 8
        for (int q = 0; q < SL; ++q) c += h[i * SL + ((q + i) & (SL - 1))];
        if (c) atomicAdd(&hps[seg * 256 + i], c);
    }
    // field f = (digit p+1) << 4 | (top nibble of digit p) -> joint[p+1][nibble][digit].
    // Each workgroup starts its flush at a different place, so the ~12 K
    // atomics of workgroups that finish together do not queue on the same lines.
    const uint32_t rot = (blockIdx.x * (uint32_t)HIST_BLOCK) % (3u * JF);
    for (int i0 = threadIdx.x; i0 < 3 * JF; i0 += HIST_BLOCK) {
        int i = i0 + (int)rot;
        i = i >= 3 * JF ? i - 3 * JF : i;
        const uint32_t c = hj[i];
        const uint32_t p = (uint32_t)i / JF, f = (uint32_t)i % JF;
        if (c) atomicAdd(&joint[((p + 1) * NSEG + (f & 15u)) * 256 + (f >> 4)], c);
    }
}

// Writes SegPlan `sp` for a pass on digit q from per-segment digit-q histograms
// hs[s][d] (s < NSEG) and segment starts.  256 threads (one per digit).
__device__ void build_segplan(SegPlan *__restrict__ sp, const uint32_t *__restrict__ hs, const uint32_t *start,
                              uint32_t mode, uint32_t *sh /* LDS: NSEG*256 + 8 words */) {
    const uint32_t t = threadIdx.x, lane = t & 63u, wid = t >> 6;
    uint32_t tot = 0;
    for (int s = 0; s < NSEG; ++s) {
        const uint32_t v = hs[s * 256 + t];
        sh[s * 256 + t] = v;
        tot += v;
    }
    uint32_t x = tot;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= (uint32_t)off) x += y;
    }
    uint32_t *wsum = sh + NSEG * 256;
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t add = 0;
    for (uint32_t w = 0; w < wid; ++w) add += wsum[w];
    uint32_t run = x + add - tot;  // global start of digit t
    for (int s = 0; s < NSEG; ++s) {
        sp->base[s * 256 + t] = run;
        run += sh[s * 256 + t];
    }
    if (t <= (uint32_t)NSEG) sp->start[t] = start[t];
    if (t == 0) {
        uint32_t tp = 0, mx = 0;
        for (int s = 0; s <= NSEG; ++s) {
            sp->tpre[s] = tp;
            if (s < NSEG) {
                // tiles aligned to OSP_TILE boundaries (k_onesweep_p's tile_range)
                const uint32_t a0 = start[s] - start[s] % (uint32_t)OSP_TILE;
                const uint32_t ts = start[s + 1] > start[s] ? (start[s + 1] - a0 + OSP_TILE - 1) / OSP_TILE : 0u;
                tp += ts;
                mx = ts > mx ? ts : mx;
            }
        }
        sp->maxt = mx;
        sp->mode = mode;
        sp->segbits = mode == 2u ? 0u : 4u;
    }
}

// SegPlan of pass q when q is active and not the first: segments = ranges of the
// previous digit's top nibble (starts from its histogram), histograms = the joint
// counts k_hist_seg wrote; one chain when the previous active digit is not q - 1.
// 256 threads; hist: the 4 digit histograms; sh, start: LDS scratch.
__device__ void build_segplan_later(SegPlan *__restrict__ out, int q, uint32_t prev, uint32_t n, int seg_later,
                                    const uint32_t *hist, const uint32_t *__restrict__ joint, uint32_t *sh,
                                    uint32_t *start) {
    const uint32_t t = threadIdx.x, lane = t & 63u, wid = t >> 6;
    if (seg_later <= 0 || prev + 1u != (uint32_t)q) {  // one chain over the whole input
        for (int s = 0; s < NSEG; ++s) sh[s * 256 + t] = s ? 0u : hist[q * 256 + t];
        if (t <= (uint32_t)NSEG) start[t] = t ? n : 0u;
        __syncthreads();
        build_segplan(out, sh, start, 2u, sh);
        return;
    }
    // segment starts: exclusive prefix over nibble groups of hist[prev]
    const uint32_t v = hist[prev * 256 + t];
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= (uint32_t)off) x += y;
    }
    if (lane == 63) sh[NSEG * 256 + wid] = x;
    __syncthreads();
    uint32_t add = 0;
    for (uint32_t w = 0; w < wid; ++w) add += sh[NSEG * 256 + w];
    if ((t & 15u) == 0) start[t >> 4] = x + add - v;
    if (t == 0) start[NSEG] = n;
    __syncthreads();
    build_segplan(out, joint + (size_t)q * NSEG * 256, start, 1u, sh);
}

// Pass plan for the 8-bit radix (as k_plan: totals, trivial passes, ping-pong
// buffers; plus each pass's next active digit) and every active pass's SegPlan (the
// later passes' plans depend only on the histograms, so they are built here, not by
// a launch before each pass).
// Workgroups 0-3 each derive the whole pass structure from the histograms (a few us of
// redundant reads) and workgroup q builds pass q's SegPlan, so the four plans are built at
// once (r31: one workgroup building them in turn took 18.7 us per sort); workgroup 0 also
// writes the Plan.  Workgroups 4.. clear the look-back region (zp, zn4 uint4s): one launch
// instead of a k_zero launch and this one (the look-back words are only read by the
// passes after it).
__global__ __launch_bounds__(256) void k_plan8(const uint32_t *__restrict__ hps, const uint32_t *__restrict__ joint,
                                               uint32_t n, int in_is_out, int seg_later, Plan *__restrict__ plan,
                                               SegPlan *__restrict__ sps, uint32_t *__restrict__ hist_out,
                                               uint4 *__restrict__ zp, size_t zn4) {
    constexpr uint32_t PW = 4;  // plan workgroups, one per pass
    if (blockIdx.x >= PW) {
        const size_t stride = (size_t)(gridDim.x - PW) * blockDim.x;
        for (size_t i = (size_t)(blockIdx.x - PW) * blockDim.x + threadIdx.x; i < zn4; i += stride)
            zp[i] = make_uint4(0u, 0u, 0u, 0u);
        return;
    }
    const int me = (int)blockIdx.x;  // the pass whose SegPlan this workgroup builds
    __shared__ uint32_t hist[4 * 256];
    __shared__ uint32_t sh[NSEG * 256 + 8];
    __shared__ uint32_t triv[4];
    __shared__ uint32_t start[NSEG + 1];
    __shared__ uint32_t prevs[4];
    __shared__ int first;
    const uint32_t t = threadIdx.x;
    if (t < 4) triv[t] = 0;
    __syncthreads();
    uint32_t v[4] = {0, 0, 0, 0};
    for (int s = 0; s < NSEG; ++s) {
        v[0] += hps[s * 256 + t];
#pragma unroll
        for (int p = 1; p < 4; ++p) v[p] += joint[(p * NSEG + s) * 256 + t];  // marginal over the nibble
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        hist[p * 256 + t] = v[p];
        if (me == 0) hist_out[p * 256 + t] = v[p];
        if (v[p] == n) triv[p] = 1;
    }
    if (t <= (uint32_t)NSEG) start[t] = seg_later < 0 ? (t ? n : 0u) : seg_start(t, n);
    __syncthreads();
    if (t == 0 && me != 0) {  // the pass structure only
        int k = 0, last = -1;
        for (int p = 0; p < 4; ++p) {
            prevs[p] = NEXT_NONE;
            if (!triv[p]) {
                if (last >= 0) prevs[p] = (uint32_t)last;
                last = p;
                if (!k++) first = p;
            }
        }
        if (!k) first = -1;
    }
    if (t == 0 && me == 0) {
        int act[4];
        int k = 0;
        for (int p = 0; p < MAX_PASSES; ++p) {
            plan->src[p] = SEL_SKIP;
            plan->dst[p] = SEL_SKIP;
            plan->next[p] = NEXT_NONE;
            plan->prev[p] = NEXT_NONE;
        }
        for (int p = 0; p < 4; ++p) {
            prevs[p] = NEXT_NONE;
            if (!triv[p]) act[k++] = p;
        }
        for (int i = 0; i + 1 < k; ++i) {
            plan->next[act[i]] = (uint32_t)act[i + 1];
            prevs[act[i + 1]] = (uint32_t)act[i];
        }
        plan->active = (uint32_t)k;
        first = k ? act[0] : -1;
        if (k == 0) {
            plan->copy_from = in_is_out ? SEL_SKIP : SEL_IN;
        } else {
            uint32_t d[4];
            uint32_t cur = SEL_OUT;
            for (int i = k - 1; i >= 0; --i) {
                d[i] = cur;
                cur = (cur == SEL_OUT) ? SEL_TMP : SEL_OUT;
            }
            if (in_is_out && d[0] == SEL_OUT)
                for (int i = 0; i < k; ++i) d[i] = (i & 1) ? SEL_OUT : SEL_TMP;
            uint32_t src = SEL_IN;
            for (int i = 0; i < k; ++i) {
                plan->src[act[i]] = src;
                plan->dst[act[i]] = d[i];
                plan->prev[act[i]] = i ? (uint32_t)act[i - 1] : NEXT_NONE;
                src = d[i];
            }
            plan->copy_from = (d[k - 1] == SEL_OUT) ? SEL_SKIP : d[k - 1];
        }
    }
    __syncthreads();
    if (first < 0 || me < first) return;
    // first active pass: position segments when it is digit 0 (hps), else one chain
    if (me != first) {
        if (prevs[me] != NEXT_NONE)  // (block-uniform) a later active pass
            build_segplan_later(sps + me, me, prevs[me], n, seg_later, hist, joint, sh, start);
        return;
    }
    if (seg_later < 0 || first != 0) {
        if (t <= (uint32_t)NSEG) start[t] = t ? n : 0u;
        for (int s = 0; s < NSEG; ++s) sh[s * 256 + t] = s ? 0u : hist[first * 256 + t];
        __syncthreads();
        build_segplan(sps + first, sh, start, 2u, sh);
    } else {
        for (int s = 0; s < NSEG; ++s) sh[s * 256 + t] = hps[s * 256 + t];
        __syncthreads();
        build_segplan(sps + first, sh, start, 0u, sh);
    }
}

__global__ __launch_bounds__(256) void k_final_copy(Bufs b, const Plan *__restrict__ plan, size_t n) {
    const uint32_t from = plan->copy_from;
    if (from == SEL_SKIP) return;
    const uint32_t *__restrict__ src = b.p[from];
    uint32_t *__restrict__ dst = b.p[SEL_OUT];
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (((((uintptr_t)src) | ((uintptr_t)dst)) & 15u) == 0) {
        const size_t nv = n / 4;
        for (size_t i = tid; i < nv; i += stride)
            reinterpret_cast<uint4 *>(dst)[i] = reinterpret_cast<const uint4 *>(src)[i];
        for (size_t i = nv * 4 + tid; i < n; i += stride) dst[i] = src[i];
    } else {
        for (size_t i = tid; i < n; i += stride) dst[i] = src[i];
    }
}

// ---------------------------------------------------------------------------------
// one LSD radix pass ("onesweep"): rank, look-back, LDS reorder, coalesced scatter
// ---------------------------------------------------------------------------------
// LDS index of tile slot i in the reorder buffer: one pad word per 32 slots, so a
// wave's stores to slots 64 apart (one per digit: sorted or strided input, where every
// digit of a tile has the same count) spread over the banks instead of all landing on
// one, and the slot-order read-back stays conflict-free.
__device__ __forceinline__ uint32_t osp_pad(uint32_t i) { return i + (i >> 5); }

template <int BITS, int BLOCK, int KPT>
struct OsSmem {
    static constexpr int R = 1 << BITS, W = BLOCK / WAVE, TILE = BLOCK * KPT;
    uint32_t keys[TILE + TILE / 32];  // padded (osp_pad)
    uint32_t whist[W * R];
    uint32_t gscan[R];
    uint32_t dstart[R];
    uint32_t delta[R];
    uint32_t wsum0[W];
    uint32_t wsum1[W];
    uint32_t tile;
};

// (LABSORT_ALGO_RADIX1: letra.pdf's literal 1-bit passes, BITS = 1)
template <int BITS, int BLOCK, int KPT>
__global__ __launch_bounds__(BLOCK) void k_onesweep(Bufs bufs, const Plan *__restrict__ plan, int pass, uint32_t n,
                                                    uint32_t flip, const uint32_t *__restrict__ ghist,
                                                    uint32_t *lookback, uint32_t *counter, uint32_t *err) {
    using S = OsSmem<BITS, BLOCK, KPT>;
    constexpr int R = S::R, W = S::W, TILE = S::TILE;
    constexpr uint32_t RM = R - 1;
    static_assert(R <= BLOCK, "one thread per digit");
    __shared__ S sm;

    const uint32_t srcsel = plan->src[pass];
    if (srcsel == SEL_SKIP) return;  // every key has the same digit: identity pass
    const uint32_t *__restrict__ in = bufs.p[srcsel];
    uint32_t *__restrict__ out = bufs.p[plan->dst[pass]];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t shift = (uint32_t)pass * BITS;

    if (tid == 0) sm.tile = atomicAdd(counter, 1u);  // dynamic tile id: predecessors already run
    for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLOCK) sm.whist[i] = 0u;
    const uint32_t gcount = tid < (uint32_t)R ? ghist[pass * R + tid] : 0u;
    const uint32_t gex = block_excl_scan<BLOCK, R>(gcount, sm.wsum0);
    if (tid < (uint32_t)R) sm.gscan[tid] = gex;
    __syncthreads();

    const uint32_t tile = sm.tile;
    const uint32_t base = tile * (uint32_t)TILE;
    const uint32_t nvalid = (n - base) < (uint32_t)TILE ? (n - base) : (uint32_t)TILE;
    const uint32_t sentinel = ~flip;  // digit RM in every pass: ranks after all real keys

    uint32_t k[KPT];
    const uint32_t wbase = base + wid * (KPT * WAVE) + lane;
    if (nvalid == (uint32_t)TILE) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) k[j] = ld_stream<NT_OS>(in + wbase + j * WAVE);
    } else {
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t idx = wbase + j * WAVE;
            k[j] = idx < n ? ld_stream<NT_OS>(in + idx) : sentinel;
        }
    }
    uint32_t dig[KPT], rank[KPT];
#pragma unroll
    for (int j = 0; j < KPT; ++j) dig[j] = ((k[j] ^ flip) >> shift) & RM;
    uint32_t *wh = sm.whist + wid * R;
    wave_rank<BITS, KPT>(dig, rank, wh);
    __syncthreads();

    // per digit: exclusive prefix over waves, tile total
    uint32_t tot = 0;
    if (tid < (uint32_t)R) {
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint32_t c = sm.whist[w * R + tid];
            sm.whist[w * R + tid] = tot;
            tot += c;
        }
    }
    const uint32_t agg = (tid == RM) ? tot - ((uint32_t)TILE - nvalid) : tot;  // drop sentinels
    uint32_t *lb_mine = lookback + (size_t)tile * R + tid;
    if (tid < (uint32_t)R) st_agent(lb_mine, (tile == 0 ? LB_INC : LB_AGG) | agg);  // publish early
    const uint32_t dstart = block_excl_scan<BLOCK, R>(tot, sm.wsum1);
    if (tid < (uint32_t)R) sm.dstart[tid] = dstart;
    __syncthreads();

    // reorder the tile by digit in LDS
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t pos = osp_pad(sm.dstart[dig[j]] + wh[dig[j]] + rank[j]);
        sm.keys[pos] = k[j];
    }

    // decoupled look-back: exclusive count of my digit in all earlier tiles
    if (tid < (uint32_t)R) {
        uint32_t excl = 0;
        if (tile > 0) {
            uint32_t t = tile - 1, spins = 0;
            for (;;) {
                const uint32_t w = ld_agent(lookback + (size_t)t * R + tid);
                if ((w & ~LB_VAL) == 0u) {
                    if (++spins > SPIN_LIMIT) {
                        atomicOr(err, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += w & LB_VAL;
                if (w & LB_INC) break;
                --t;
            }
            st_agent(lb_mine, LB_INC | (excl + agg));
        }
        sm.delta[tid] = sm.gscan[tid] + excl - dstart;
    }
    __syncthreads();

    // coalesced scatter: consecutive threads write consecutive slots of a digit run
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t i = (uint32_t)j * BLOCK + tid;
        if (i < nvalid) {
            const uint32_t key = sm.keys[osp_pad(i)];
            const uint32_t d = ((key ^ flip) >> shift) & RM;
            out[sm.delta[d] + i] = key;
        }
    }
}

// ---------------------------------------------------------------------------------
// persistent, software-pipelined onesweep pass (8-bit digits)
//
// The non-persistent pass above spends ~40 % of each tile waiting on the decoupled
// look-back (the inclusive-prefix chain advances only as fast as tiles finish their
// walks under loaded memory latency).  Here each workgroup loops over dynamically
// acquired tiles and keeps two in flight: tile A (ranked and reordered, keys in
// registers in scatter order) waits for its look-back while the workgroup ranks tile B,
// whose keys were loaded one iteration ahead.  Per iteration:
//   (top)  A's look-back window (LBW predecessors) and tile C's key loads are issued,
//          and tid 0 issues the next tile's acquisition atomic;
//   rank   B's keys are ranked per wave by one returning LDS atomic per key;
//   (2)    A's look-back completes (waves 0-3, one digit per thread); A's INC published;
//   (2b)   B's tile histogram is summed from the wave counts, its AGG published, scanned;
//          A's keys are scattered (groups of 4 sorted slots within one digit run as one
//          16-B store);
//   (3)    B's per-wave digit offsets; the acquisition resolved;
//   (4)    B reordered into LDS, read back in scatter order: B becomes A.
// Dynamic tile ids order the tiles by acquisition, so a tile only ever waits on tiles
// acquired earlier, whose aggregates are published unconditionally after their rank:
// forward progress holds for any grid size or residency.  Every spin is bounded.
// The measured history of this loop (shapes, barriers, prefetch, store widths,
// acquisition) is in DESIGN.md §3.1; the variants measured slower are gone from here.
// ---------------------------------------------------------------------------------
// A buffer descriptor's num_records is a 32-bit byte count: n words fit only while
// 4 n < 2^32.  The radix passes stop at RADIX_MAX_N (2^30 - 1) keys, which the launcher
// checks (launch_onesweep_p); any kernel on the merge path (n up to 2^31 - 1) that adopts
// buffer loads must split its descriptor instead (a 2^30-key merge once read zeros this way).
static_assert((uint64_t)RADIX_MAX_N * 4u <= 0xFFFFFFFFull, "buffer descriptor byte count wraps");
__device__ __forceinline__ __amdgpu_buffer_rsrc_t osp_rsrc(const uint32_t *p, uint32_t n) {
    const uint64_t a = (uint64_t)p;  // wave-uniform: readfirstlane lets the compiler prove it
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0, (int)(n * 4u), 0x00020000);
}
constexpr int OSP_BUF_NT = (NT_LOADS & NT_OSP) ? 2 : 0;  // aux bit 1 = nontemporal

template <bool KV>
struct OspSmem {
    static constexpr int BLOCK = KV ? OSP_KV_BLOCK : OSP_BLOCK;  // threads (key/value: its own shape)
    static constexpr int R = 256, W = BLOCK / WAVE, TILE = OSP_TILE;
    uint32_t keys[TILE + TILE / 32];     // reorder buffer, padded (osp_pad)
    uint32_t vals[KV ? TILE + TILE / 32 : 1];  // key/value: payloads, reordered alike
    uint32_t wh[W * R];                  // per-wave digit counters, then offsets
    uint64_t match[KV ? 1 : W * R];      // rank fallback (LDS match) if the lane-order check fails
    uint32_t probe[WAVE];
    uint32_t ordered;
    uint32_t delta[R];                   // A: output position of its slot 0 per digit
    uint32_t base[KV ? 1 : NSEG * R];    // the segments' output bases (SegPlan::base)
    uint32_t start[NSEG + 1];
    uint32_t tpre[NSEG + 1];
    uint32_t wsum[8];
    uint32_t next, next2;
};

constexpr uint32_t OSP_DONE = 0xFFFFFFFFu;

// KV: key/value pairs: each payload (vbufs, selected by the plan like
// the keys) is loaded with its key, reordered in a second LDS buffer and scattered to
// its key's destination.  No room in LDS for the match buffer (the rank's fallback is
// then 8 ballots) nor the bases table, and no registers for the next tile's prefetch:
// 512-thread workgroups, the acquisition at the end of the iteration.
template <bool KV = false>
__global__ __launch_bounds__(KV ? OSP_KV_BLOCK : OSP_BLOCK, (KV ? OSP_KV_BLOCK : OSP_BLOCK) / 256)
void k_onesweep_p(Bufs bufs, const Plan *__restrict__ plan, int pass, uint32_t n, uint32_t flip,
                  const SegPlan *__restrict__ sp, uint32_t *lookback, uint32_t *counter, uint32_t *err, Bufs vbufs) {
    using S = OspSmem<KV>;
    constexpr bool PF = !KV;  // next tile's keys loaded one iteration ahead
    constexpr bool ST4 = !KV;  // grouped 16-B scatter stores (r26; the key/value pass measured 2-5 % slower with them)
    constexpr int R = S::R, W = S::W, TILE = S::TILE, BLK = S::BLOCK, KPT = TILE / BLK, LBW = OSP_LBW;
    static_assert(BLK >= 512 && NSEG == 16 && KPT * BLK == TILE && KPT % 4 == 0, "digit threads = waves 0-3");
    __shared__ S sm;

    const uint32_t srcsel = plan->src[pass];
    if (srcsel == SEL_SKIP) {  // every key has the same digit: identity pass
        if (pass == 0 && plan->copy_from == SEL_IN) {
            // no active pass at all (every digit constant): the input is the result, and
            // pass 0's launch copies it (api.hip launches no final copy for in != out)
            const uint4 *src = reinterpret_cast<const uint4 *>(bufs.p[SEL_IN]);
            uint4 *dst = reinterpret_cast<uint4 *>(bufs.p[SEL_OUT]);
            const size_t stride = (size_t)gridDim.x * BLK, g0 = (size_t)blockIdx.x * BLK + threadIdx.x;
            if (((((uintptr_t)src) | ((uintptr_t)dst)) & 15u) == 0) {
                for (size_t i = g0; i < n / 4; i += stride) dst[i] = src[i];
                for (size_t i = (n / 4) * 4 + g0; i < n; i += stride) bufs.p[SEL_OUT][i] = bufs.p[SEL_IN][i];
            } else {
                for (size_t i = g0; i < n; i += stride) bufs.p[SEL_OUT][i] = bufs.p[SEL_IN][i];
            }
            if constexpr (KV)
                for (size_t i = g0; i < n; i += stride) vbufs.p[SEL_OUT][i] = vbufs.p[SEL_IN][i];
        }
        return;
    }
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t shift = (uint32_t)pass * 8u;
    const uint32_t sentinel = ~flip;  // digit 255 in every pass: ranks after all real keys
    // tile id c = l * NSEG + segment (tile l of the segment)
    constexpr uint32_t segbits = 4, segmask = NSEG - 1;
    // XCD-grouped acquisition: counter group g = segments {g, g + 8}; a workgroup takes
    // the tiles of its own XCD's group first, then helps the others (consecutive tiles
    // of a chain then meet in one L2).  One group when there is a single chain (mode 2).
    const bool grouped = sp->mode != 2u;
    const uint32_t gbits = grouped ? 3u : 0u, G = 1u << gbits;
    const uint32_t lbits = sp->segbits - gbits, lmask = (1u << lbits) - 1u;
    const uint32_t climit = sp->maxt << lbits;

    for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLK) sm.wh[i] = 0u;
    if constexpr (!KV)
        for (uint32_t i = tid; i < (uint32_t)(NSEG * R); i += BLK) sm.base[i] = sp->base[i];
    const uint32_t *__restrict__ in = bufs.p[srcsel];
    uint32_t *__restrict__ out = bufs.p[plan->dst[pass]];
    const __amdgpu_buffer_rsrc_t rin = osp_rsrc(in, n), rout = osp_rsrc(out, n);
    const __amdgpu_buffer_rsrc_t rvin = osp_rsrc(KV ? vbufs.p[srcsel] : in, n),
                                 rvout = osp_rsrc(KV ? vbufs.p[plan->dst[pass]] : out, n);
    if (tid <= (uint32_t)NSEG) {
        sm.start[tid] = sp->start[tid];
        sm.tpre[tid] = sp->tpre[tid];
    }
    // tile acquisition (tid 0): c -> segment c & 15, tile c >> 4 of that segment; ids past
    // a segment's last tile are skipped, so every segment's tiles are acquired in order
    const uint32_t home = grouped ? (__builtin_amdgcn_s_getreg((3 << 11) | 20) & (G - 1u)) : 0u;  // HW_REG_XCC_ID
    uint32_t gk = 0;
    auto acquire = [&]() {
        while (gk < G) {
            const uint32_t grp = (home + gk) & (G - 1u);
            const uint32_t c = atomicAdd(counter + grp, 1u);
            if (c >= climit) {
                ++gk;
                continue;
            }
            const uint32_t sg = grp | ((c & lmask) << gbits), l = c >> lbits;
            if (l < sp->tpre[sg + 1] - sp->tpre[sg]) return l * NSEG + sg;
        }
        return OSP_DONE;
    };
    // early acquisition: the counter increment was issued by tid 0 at the top of the
    // iteration and is resolved here, before barrier (3), so its round trip overlaps the
    // iteration instead of holding every wave at the barrier (r26: 0.491 -> 0.473 ms/pass)
    auto acquire_done = [&](uint32_t c) {
        while (gk < G) {
            const uint32_t grp = (home + gk) & (G - 1u);
            if (c >= climit) {
                if (++gk < G) c = atomicAdd(counter + ((home + gk) & (G - 1u)), 1u);
                continue;
            }
            const uint32_t sg = grp | ((c & lmask) << gbits), l = c >> lbits;
            if (l < sm.tpre[sg + 1] - sm.tpre[sg]) return l * NSEG + sg;
            c = atomicAdd(counter + grp, 1u);
        }
        return OSP_DONE;
    };
    if (tid == 0) {
        const uint32_t c0 = acquire();
        sm.next = c0;
        sm.next2 = (PF && c0 != OSP_DONE) ? acquire() : OSP_DONE;
    }
    if (wid == 0) {
        const bool ord = lds_lane_ordered(sm.probe, lane);
        if (lane == 0) sm.ordered = ord ? 1u : 0u;
    }
    __syncthreads();
    uint32_t cB = sm.next, cC = sm.next2;
    const bool atomic_rank = __builtin_amdgcn_readfirstlane(sm.ordered) != 0u;

    // carried state of tile A (slot = look-back slot, lo = slot of its segment's first tile)
    uint32_t slotA = OSP_DONE, loA = 0, segA = 0, nvalidA = 0;
    uint32_t kA[KPT];
    uint32_t vA[KV ? KPT : 1];
    uint32_t lwA[LBW];
    uint32_t aggA = 0, dstartA = 0;
    uint32_t *wh = sm.wh + wid * R;
    uint64_t *wm = sm.match + (KV ? 0 : wid * R);
    // input range of tile c: [beg, beg + nvalid).  Tiles are aligned to TILE-key
    // boundaries of the input (line-aligned wave loads): a segment's first tile runs
    // from its start to the next boundary.
    auto tile_range = [&](uint32_t c, uint32_t &beg, uint32_t &nvalid) {
        const uint32_t sg = c & segmask, l = c >> segbits;
        const uint32_t s0 = sm.start[sg], a0 = s0 - s0 % (uint32_t)TILE;
        beg = l ? a0 + l * (uint32_t)TILE : s0;
        const uint32_t tend = a0 + (l + 1u) * (uint32_t)TILE, send = sm.start[sg + 1];
        nvalid = (tend < send ? tend : send) - beg;
    };
    // keys of tile c in the wave's blocked layout (buffer loads: out-of-range offsets read
    // 0, replaced by the sentinel, digit 255)
    auto load_tile = [&](uint32_t c, uint32_t (&k)[KPT]) {
        uint32_t beg, nv;
        tile_range(c, beg, nv);
        const uint32_t woff = wid * (KPT * WAVE) + lane;
        const uint32_t o = (beg + woff) * 4u;
        if (nv == (uint32_t)TILE) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) k[j] = __builtin_amdgcn_raw_buffer_load_b32(rin, o + j * WAVE * 4, 0, OSP_BUF_NT);
        } else {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rin, o + j * WAVE * 4, 0, OSP_BUF_NT);
                k[j] = woff + j * WAVE < nv ? v : sentinel;
            }
        }
    };
    // payloads of tile c, in the keys' layout (key/value passes)
    auto load_vals = [&](uint32_t c, uint32_t (&v)[KPT]) {
        uint32_t beg, nv;
        tile_range(c, beg, nv);
        const uint32_t o = (beg + wid * (KPT * WAVE) + lane) * 4u;
#pragma unroll
        for (int j = 0; j < KPT; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b32(rvin, o + j * WAVE * 4, 0, OSP_BUF_NT);
    };
    uint32_t kB[KPT], kN[PF ? KPT : 1];
    uint32_t vB[KV ? KPT : 1];
    if constexpr (PF) {
        if (cB != OSP_DONE) load_tile(cB, kN);
    }

    for (;;) {
        if constexpr (PF) {  // B's keys, loaded one iteration ahead
#pragma unroll
            for (int j = 0; j < KPT; ++j) kB[j] = kN[j < (PF ? KPT : 1) ? j : 0];
        }
        const bool haveB = cB != OSP_DONE;
        uint32_t acq_c = 0;  // tid 0: the early counter increment
        const uint32_t cLast = cC;  // the last tile acquired so far
        if (PF && tid == 0 && cLast != OSP_DONE && gk < G) acq_c = atomicAdd(counter + ((home + gk) & (G - 1u)), 1u);
        const uint32_t segB = cB & segmask, lB = cB >> segbits;
        const uint32_t loB = haveB ? sm.tpre[segB] : 0u, slotB = loB + lB;
        uint32_t begB = 0, nvalidB = 0;
        if (haveB) tile_range(cB, begB, nvalidB);
        uint32_t rB[KPT / 2];  // wave-local ranks of B, two 16-bit ranks per register
        uint32_t hB = 0, xB = 0;
        // look-back window of A (its latency hides behind B's rank)
        if (slotA != OSP_DONE && tid < (uint32_t)R) {
            const int32_t hi = (int32_t)slotA - 1;
#pragma unroll
            for (int i = 0; i < LBW; ++i)
                lwA[i] = (hi - i >= (int32_t)loA) ? ld_agent(lookback + (size_t)(hi - i) * R + tid) : LB_INC;
        }
        if constexpr (PF) {
            if (cC != OSP_DONE) load_tile(cC, kN);
        } else if (haveB) {
            load_tile(cB, kB);
            if constexpr (KV) load_vals(cB, vB);
        }
        // key/value: the lane-order check hoisted out of the key loop (r29, same box: 0.899 vs
        // 0.909 ms per pass, r27's 0.899; for keys only it measured slower, 0.485 vs 0.466:
        // profiles/r29_ab_rank_hoist.txt)
        if (KV && haveB && atomic_rank) {  // stable wave rank of B
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t r = wave_atomic_rank(wh, ((kB[j] ^ flip) >> shift) & 255u, lane);
                rB[j / 2] = (j & 1) ? rB[j / 2] | (r << 16) : r;
            }
        } else if (haveB) {  // stable wave rank of B
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t d = ((kB[j] ^ flip) >> shift) & 255u;
                if (atomic_rank) {
                    const uint32_t r = wave_atomic_rank(wh, d, lane);
                    rB[j / 2] = (j & 1) ? rB[j / 2] | (r << 16) : r;
                } else {
                    const uint64_t m = KV ? match8(d) : lds_peers(wm + d, lane);
                    const uint32_t pre = mbcnt64(m);
                    const uint32_t old = wh[d];
                    if (pre == 0) wh[d] = old + (uint32_t)__popcll(m);
                    rB[j / 2] = (j & 1) ? rB[j / 2] | ((old + pre) << 16) : old + pre;
                }
            }
        }
        // complete the look-back of A; publish its inclusive prefix (within its segment)
        if (slotA != OSP_DONE && tid < (uint32_t)R) {
            // first round: the LBW words loaded at the top of the iteration; later rounds
            // (each a dependent memory round trip) read LBW words at once
            uint32_t excl = 0, spins = 0;
            int32_t hi = (int32_t)slotA - 1;
            int consumed = 0;
            bool done = false, stall = false;
#pragma unroll
            for (int i = 0; i < LBW; ++i) {
                if (!done && !stall) {
                    if ((lwA[i] & ~LB_VAL) == 0u) stall = true;
                    else {
                        excl += lwA[i] & LB_VAL;
                        ++consumed;
                        done = (lwA[i] & LB_INC) != 0u;
                    }
                }
            }
            while (!done) {
                hi -= consumed;
                if (stall) {
                    if (++spins > SPIN_LIMIT) {
                        atomicOr(err, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                uint32_t lw[LBW];
#pragma unroll
                for (int i = 0; i < LBW; ++i)
                    lw[i] = (hi - i >= (int32_t)loA) ? ld_agent(lookback + (size_t)(hi - i) * R + tid) : LB_INC;
                consumed = 0;
                stall = false;
#pragma unroll
                for (int i = 0; i < LBW; ++i) {
                    if (!done && !stall) {
                        if ((lw[i] & ~LB_VAL) == 0u) stall = true;
                        else {
                            excl += lw[i] & LB_VAL;
                            ++consumed;
                            done = (lw[i] & LB_INC) != 0u;
                        }
                    }
                }
            }
            if (slotA > loA) st_agent(lookback + (size_t)slotA * R + tid, LB_INC | (excl + aggA));
            sm.delta[tid] = (KV ? sp->base[segA * R + tid] : sm.base[segA * R + tid]) + excl - dstartA;
        }
        __syncthreads();  // (2) delta of A, wave counts of B
        if (haveB && tid < (uint32_t)R) {
            // tile histogram = sum of the per-wave counts; publish B's aggregate, scan it
            uint32_t tot = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) tot += sm.wh[w * R + tid];
            if (tid == (uint32_t)R - 1) tot -= (uint32_t)TILE - nvalidB;  // sentinels
            hB = tot;
            st_agent(lookback + (size_t)slotB * R + tid, (lB == 0 ? LB_INC : LB_AGG) | hB);
            xB = hB;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t t = __shfl_up(xB, off);
                if (lane >= (uint32_t)off) xB += t;
            }
            if (lane == 63) sm.wsum[wid] = xB;
        }
        if (slotA != OSP_DONE) {
            if constexpr (ST4) {
                // lane holds sorted slots 4 (g BLK + tid) + q: 4 keys in one digit run (their
                // first and last digits agree) leave as one 16-B store, else 4 dword stores;
                // a partial tile's sentinels (slot >= nvalidA) go past the array's end: dropped
#pragma unroll
                for (int g = 0; g < KPT / 4; ++g) {
                    const uint32_t i0 = 4u * ((uint32_t)g * BLK + tid);
                    uint32_t d[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) d[q] = ((kA[4 * g + q] ^ flip) >> shift) & 255u;
                    const uint32_t dst0 = sm.delta[d[0]] + i0;
                    if (d[0] == d[3] && i0 + 3u < nvalidA) {
                        const u32x4 v = {kA[4 * g], kA[4 * g + 1], kA[4 * g + 2], kA[4 * g + 3]};
                        __builtin_amdgcn_raw_buffer_store_b128(v, rout, dst0 * 4u, 0, 0);
                    } else {
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const uint32_t i = i0 + (uint32_t)q;
                            const uint32_t dst = i < nvalidA ? sm.delta[d[q]] + i : n;
                            __builtin_amdgcn_raw_buffer_store_b32(kA[4 * g + q], rout, dst * 4u, 0, 0);
                        }
                    }
                }
            } else {
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t i = (uint32_t)j * BLK + tid;
                    const uint32_t dst = i < nvalidA ? sm.delta[((kA[j] ^ flip) >> shift) & 255u] + i : n;
                    __builtin_amdgcn_raw_buffer_store_b32(kA[j], rout, dst * 4u, 0, 0);
                    if constexpr (KV) __builtin_amdgcn_raw_buffer_store_b32(vA[j], rvout, dst * 4u, 0, 0);
                }
            }
        }
        if (!haveB) break;
        __syncthreads();  // (2b) wave sums of B's digit scan
        if (tid < (uint32_t)R) {
            uint32_t add = 0;
#pragma unroll
            for (int w = 0; w < 4; ++w)
                if ((uint32_t)w < wid) add += sm.wsum[w];
            const uint32_t ds = xB + add - hB;  // tile-local start of digit tid
            uint32_t run = ds;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint32_t c = sm.wh[w * R + tid];
                sm.wh[w * R + tid] = run;
                run += c;
            }
            dstartA = ds;
        }
        if (tid == 0) sm.next = !PF ? acquire() : cLast != OSP_DONE ? acquire_done(acq_c) : OSP_DONE;
        __syncthreads();  // (3) wave offsets of B
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t pos = osp_pad(wh[((kB[j] ^ flip) >> shift) & 255u] + ((rB[j / 2] >> ((j & 1) * 16)) & 0xFFFFu));
            sm.keys[pos] = kB[j];
            if constexpr (KV) sm.vals[pos] = vB[j];
        }
        __syncthreads();  // (4) B reordered in LDS
        if constexpr (ST4) {  // slots 4 (g BLK + tid) + q, q = 0..3 (never across a pad word)
#pragma unroll
            for (int g = 0; g < KPT / 4; ++g)
#pragma unroll
                for (int q = 0; q < 4; ++q) kA[4 * g + q] = sm.keys[osp_pad(4u * ((uint32_t)g * BLK + tid) + (uint32_t)q)];
        } else {
            // keys first, then the payloads (interleaved reads measured 1.6 % slower for the
            // key/value pass: 0.887 vs 0.873 ms, r29 harness/exp/pairs_ab.py)
#pragma unroll
            for (int j = 0; j < KPT; ++j) kA[j] = sm.keys[osp_pad(j * BLK + tid)];
            if constexpr (KV) {
#pragma unroll
                for (int j = 0; j < KPT; ++j) vA[j] = sm.vals[osp_pad(j * BLK + tid)];
            }
        }
        // each wave clears its own counters (no barrier before the next ranking)
        for (uint32_t i = lane; i < (uint32_t)R; i += WAVE) wh[i] = 0u;
        slotA = slotB;
        loA = loB;
        segA = segB;
        nvalidA = nvalidB;
        aggA = hB;
        if constexpr (PF) {
            cB = cC;
            cC = sm.next;
        } else {
            cB = sm.next;
        }
    }
}

// ---------------------------------------------------------------------------------
// LDS-resident tile sort: 8-bit LSD passes entirely in LDS, one global read and write
// ---------------------------------------------------------------------------------
template <int BLOCK, int KPT, bool KV = false>
struct TsSmem {
    static constexpr int R = 256, W = BLOCK / WAVE, TILE = BLOCK * KPT;
    uint32_t keys[TILE];
    uint32_t vals[KV ? TILE : 1];  // key/value: the payload follows its key through every pass
    uint32_t whist[W * R];
    uint32_t wsum[W];
    uint32_t red_and[W];
    uint32_t red_or[W];
    uint32_t probe[WAVE];
    uint32_t ordered;
};

// One TILE-key tile per workgroup, sorted by up to four 8-bit LSD passes in LDS (passes
// whose digit is uniform over the tile are skipped: the reference's "stop when sorted",
// lab.cu:61, per tile).  KV: key/value pairs (vin/vout, 4-byte payloads); the sort is
// stable, so equal keys keep their input order and their payloads with them.
// Measured and not kept (r26): a persistent grid, the next tile's keys
// loaded before the last pass, 16-B grouped loads and stores; r28: nontemporal output
// stores (1.10 vs 1.07 ms at 2^28), as 16-B stores read from the sorted LDS tile 1.12;
// the rank loop's per-key uniform-digit branch makes each pass's 32 returning atomics
// wait one at a time (lgkmcnt(0) at every join), but a per-wave pre-check that runs them
// branch-free when no digit is wave-uniform measured 1.085-1.092 vs 1.080-1.083 ms (128
// VGPRs, 3 spilled; profiles/r28_ab_tile_sort_precheck.txt).
template <int BLOCK, int KPT, bool KV = false>
__global__ __launch_bounds__(BLOCK, 4) void k_tile_sort(const uint32_t *in, uint32_t *out, const uint32_t *vin,
                                                         uint32_t *vout, uint32_t n, uint32_t flip,
                                                         uint32_t *samp_out = nullptr) {
    using S = TsSmem<BLOCK, KPT, KV>;
    constexpr int R = S::R, W = S::W, TILE = S::TILE;
    __shared__ S sm;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t sentinel = ~flip;
    if (wid == 0) {  // lane-ordered LDS atomics (see k_onesweep_p): rank by one atomic per key
        const bool ord = lds_lane_ordered(sm.probe, lane);
        if (lane == 0) sm.ordered = ord ? 1u : 0u;
    }
    const uint32_t base = blockIdx.x * (uint32_t)TILE;
    const uint32_t wbase = base + wid * (KPT * WAVE) + lane;
    uint32_t k[KPT];
    uint32_t v[KV ? KPT : 1];
    uint32_t a = ~0u, o = 0u;
    const bool full = base + (uint32_t)TILE <= n;
    if constexpr (KV) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t idx = wbase + j * WAVE;
            v[j] = idx < n ? vin[idx] : 0u;
        }
    }
    if (full) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) k[j] = ld_stream<NT_TILE>(in + wbase + j * WAVE);
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            a &= k[j] ^ flip;
            o |= k[j] ^ flip;
        }
    } else {
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t idx = wbase + j * WAVE;
            const bool ok = idx < n;
            k[j] = ok ? ld_stream<NT_TILE>(in + idx) : sentinel;
            const uint32_t x = k[j] ^ flip;
            a &= ok ? x : ~0u;
            o |= ok ? x : 0u;
        }
    }
    // bits on which the tile's keys differ -> passes that are not the identity
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a &= __shfl_xor(a, off);
        o |= __shfl_xor(o, off);
    }
    if (lane == 0) {
        sm.red_and[wid] = a;
        sm.red_or[wid] = o;
    }
    __syncthreads();
    const bool atomic_rank = __builtin_amdgcn_readfirstlane(sm.ordered) != 0u;
    uint32_t diff = 0;
    {
        uint32_t aa = ~0u, oo = 0u;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            aa &= sm.red_and[w];
            oo |= sm.red_or[w];
        }
        diff = aa ^ oo;
    }
    uint32_t *wh = sm.whist + wid * R;
    for (int pass = 0; pass < 4; ++pass) {
        const uint32_t shift = pass * 8;
        if (((diff >> shift) & 0xFFu) == 0u) continue;  // uniform over the tile
        for (uint32_t i = lane; i < (uint32_t)R; i += WAVE) wh[i] = 0u;
        uint32_t rank[KPT / 2];  // two 16-bit wave-local ranks per register
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            // stable wave rank: lane-ordered returning atomic, else peers by 8 ballots
            const uint32_t d = ((k[j] ^ flip) >> shift) & 0xFFu;
            uint32_t r;
            if (atomic_rank) {
                r = wave_atomic_rank(wh, d, lane);
            } else {
                const uint64_t m = match8(d);
                const uint32_t pre = mbcnt64(m);
                const uint32_t old = wh[d];
                if (pre == 0) wh[d] = old + (uint32_t)__popcll(m);
                r = old + pre;
            }
            rank[j / 2] = (j & 1) ? rank[j / 2] | (r << 16) : r;
        }
        __syncthreads();
        // tile-wide digit offsets folded into the per-wave offsets: the reorder then
        // reads one LDS word per key instead of two (r17)
        uint32_t tot = 0;
        if (tid < (uint32_t)R) {
#pragma unroll
            for (int w = 0; w < W; ++w) tot += sm.whist[w * R + tid];
        }
        const uint32_t ds = block_excl_scan<BLOCK, R>(tot, sm.wsum);
        if (tid < (uint32_t)R) {
            uint32_t run = ds;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint32_t c = sm.whist[w * R + tid];
                sm.whist[w * R + tid] = run;
                run += c;
            }
        }
        __syncthreads();
        // every destination first (replacing its 16-bit rank: dst < TILE), the stores after:
        // interleaved, each counter read would wait for the store before it (the compiler
        // cannot tell the stores from the counters), 32 LDS round trips in a row per wave
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t d = ((k[j] ^ flip) >> shift) & 0xFFu;
            const uint32_t dst = wh[d] + ((rank[j / 2] >> ((j & 1) * 16)) & 0xFFFFu);
            rank[j / 2] = (j & 1) ? (rank[j / 2] & 0xFFFFu) | (dst << 16) : (rank[j / 2] & 0xFFFF0000u) | dst;
        }
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t dst = (rank[j / 2] >> ((j & 1) * 16)) & 0xFFFFu;
            sm.keys[dst] = k[j];
            if constexpr (KV) sm.vals[dst] = v[j];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < KPT; ++j) k[j] = sm.keys[wid * (KPT * WAVE) + j * WAVE + lane];
        if constexpr (KV) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) v[j] = sm.vals[wid * (KPT * WAVE) + j * WAVE + lane];
        }
        // (the next pass's reorder writes sm.keys two barriers later)
    }
    // samp_out: every M4_S-th output key for a four-way merge pass next (merge4.hip)
    static_assert((KPT * WAVE) % M4_S == 0 && M4_S % WAVE == 0, "samples at lane 0 of fixed slots");
    if (samp_out && lane == 0) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t idx = wbase + j * WAVE;
            if (((uint32_t)j * WAVE) % M4_S == 0 && idx < n) samp_out[idx / M4_S] = k[j];
        }
    }
    if (full) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) out[wbase + j * WAVE] = k[j];
    } else {
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t idx = wbase + j * WAVE;
            if (idx < n) out[idx] = k[j];
        }
    }
    if constexpr (KV) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t idx = wbase + j * WAVE;
            if (idx < n) vout[idx] = v[j];
        }
    }
}

// ---------------------------------------------------------------------------------
// 64-key tile bit-split sort (radix_sort_kernel's job on a wave64)
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_wave_split(uint32_t *keys, uint32_t n, uint32_t flip) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t idx = gw * 64u + lane;
    if (gw * 64u >= n) return;  // wave-uniform
    uint32_t v = idx < n ? (keys[idx] ^ flip) : 0xFFFFFFFFu;
    for (int b = 0; b < 32; ++b) {
        const uint32_t prev = __shfl_up(v, 1);
        if (__all(lane == 0 || prev <= v)) break;  // tile sorted: stop (lab.cu:61)
        const bool zero = ((v >> b) & 1u) == 0u;
        const uint64_t bal = __ballot(zero);        // the split's flags
        const uint32_t below = mbcnt64(bal);          // exclusive scan of the flags
        const uint32_t nz = (uint32_t)__popcll(bal);  // totalFalses
        const uint32_t pos = zero ? below : nz + (lane - below);
        v = (uint32_t)__builtin_amdgcn_ds_permute((int)(pos << 2), (int)v);  // scatter
    }
    if (idx < n) keys[idx] = v ^ flip;
}

// ---------------------------------------------------------------------------------
// merge path
// ---------------------------------------------------------------------------------
__device__ __forceinline__ bool key_le(uint32_t a, uint32_t b, uint32_t flip) { return (a ^ flip) <= (b ^ flip); }

// number of A elements among the first `diag` of merge(A,B), A first on ties; the
// answer is searched in [lo, hi] (callers may pass a bracket known from neighbouring
// diagonals; it is clipped to the feasible range)
__device__ __forceinline__ uint32_t corank(const uint32_t *A, uint32_t la, const uint32_t *B, uint32_t lb,
                                           uint32_t diag, uint32_t flip, uint32_t lo = 0u, uint32_t hi = ~0u) {
    if (diag > lb && lo < diag - lb) lo = diag - lb;
    if (hi > diag) hi = diag;
    if (hi > la) hi = la;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (key_le(A[mid], B[diag - 1u - mid], flip)) lo = mid + 1u;
        else hi = mid;
    }
    return lo;
}

// 16-B aligned: the full-tile path reads and writes sm.out / sm.vout as uint4
#ifndef LABSORT_MG_PAD
#define LABSORT_MG_PAD 1
#endif
constexpr bool MG_PAD = LABSORT_MG_PAD != 0;  // keys-only merge pass: +inf pads after both runs in LDS
constexpr uint32_t MG_PADW = 8;
template <bool KV = false>
struct alignas(16) MgSmem {
    uint32_t in[MG_TILE + 2 * MG_PADW];
    alignas(16) uint32_t out[MG_TILE + MG_TILE / 32];
    uint32_t vin[KV ? MG_TILE : 1];  // key/value: payloads of sm.in
    alignas(16) uint32_t vout[KV ? MG_TILE + MG_TILE / 32 : 1];
};
static_assert(offsetof(MgSmem<false>, out) % 16 == 0 && offsetof(MgSmem<true>, vout) % 16 == 0, "uint4 LDS rows");

// merge A[a0,a1) and B[b0,b1) (a1-a0 + b1-b0 <= MG_TILE) into out[0 ..)
template <int BLOCK, int KPT>
__device__ __forceinline__ void merge_tile(const uint32_t *__restrict__ A, uint32_t a0, uint32_t a1,
                                           const uint32_t *__restrict__ B, uint32_t b0, uint32_t b1,
                                           uint32_t *__restrict__ out, uint32_t flip, MgSmem<> &sm) {
    const uint32_t tid = threadIdx.x;
    const uint32_t la = a1 - a0, lb = b1 - b0, tot = la + lb;
    for (uint32_t i = tid; i < la; i += BLOCK) sm.in[i] = A[a0 + i];
    for (uint32_t i = tid; i < lb; i += BLOCK) sm.in[la + i] = B[b0 + i];
    __syncthreads();
    const uint32_t *sa = sm.in, *sb = sm.in + la;
    const uint32_t d = tid * KPT < tot ? tid * KPT : tot;
    uint32_t ai = corank(sa, la, sb, lb, d, flip);
    uint32_t bi = d - ai;
    uint32_t va = ai < la ? sa[ai] : 0u;
    uint32_t vb = bi < lb ? sb[bi] : 0u;
    uint32_t r[KPT];
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const bool takeA = (bi >= lb) || (ai < la && key_le(va, vb, flip));
        r[j] = takeA ? va : vb;
        if (takeA) {
            ++ai;
            va = ai < la ? sa[ai] : 0u;
        } else {
            ++bi;
            vb = bi < lb ? sb[bi] : 0u;
        }
    }
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t idx = tid * KPT + j;
        if (idx < tot) sm.out[idx + (idx >> 5)] = r[j];
    }
    __syncthreads();
    for (uint32_t i = tid; i < tot; i += BLOCK) out[i] = sm.out[i + (i >> 5)];
}

struct PairGeom {
    uint32_t pb, la, lb;
};
__device__ __forceinline__ PairGeom pair_of(uint32_t o, uint32_t n, uint32_t run, const MgPairs &pr) {
    PairGeom g;
    if (pr.np) {  // explicit pairs: the one holding output position o
        uint32_t i = 0;
#pragma unroll
        for (int q = 1; q < MG_MAX_PAIRS; ++q)
            if ((uint32_t)q < pr.np && o >= pr.pb[q]) i = (uint32_t)q;
        g.pb = pr.pb[i];
        g.la = pr.la[i];
        g.lb = pr.pb[i + 1] - pr.pb[i] - pr.la[i];
        return g;
    }
    g.pb = (o / (2u * run)) * (2u * run);
    const uint32_t rest = n - g.pb;
    g.la = rest < run ? rest : run;
    const uint32_t restb = rest - g.la;
    g.lb = restb < run ? restb : run;
    return g;
}

// Persistent, software-pipelined merge pass.  Workgroup b merges the consecutive
// output tiles [b*m, (b+1)*m): it first finds the co-ranks at all their starts with
// concurrent binary searches (one per thread, their latencies overlapping; no
// separate partition launch), then merges tile after tile, the keys of the next
// tile loading into registers while the current one is merged in LDS.
// KV: key/value pairs; each output takes the payload of the key it took (vsrc/vdst).
// Keys only: at most 64 VGPRs (8 waves per SIMD, four 512-thread workgroups per CU: the
// network merge below needs 71 unbounded, which would leave three).
template <int BLOCK, int KPT, bool KV = false>
__global__ __launch_bounds__(BLOCK, KV ? 4 : 8) void k_merge_pass_p(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                                        uint32_t n, uint32_t run, uint32_t flip, uint32_t ntiles,
                                                        uint32_t m, MgPairs pr, const uint32_t *__restrict__ vsrc = nullptr,
                                                        uint32_t *__restrict__ vdst = nullptr,
                                                        uint32_t *__restrict__ samp_out = nullptr) {
    constexpr uint32_t T = (uint32_t)(BLOCK * KPT);
    static_assert(T == (uint32_t)MG_TILE, "tile granularity");
    __shared__ MgSmem<KV> sm;
    __shared__ uint32_t s_part[MG_MAX_TPB + 1];
    const uint32_t tid = threadIdx.x;
    const uint32_t t0 = blockIdx.x * m;
    if (t0 >= ntiles) return;
    const uint32_t t1 = t0 + m < ntiles ? t0 + m : ntiles;
    // A-side co-rank at the start of every tile of this workgroup (and of the next one),
    // in two rounds: every MG_BRACKET-th tile over its whole pair of runs, then the
    // others inside the bracket of their round-1 neighbours (co-ranks are monotone
    // within a pair and move by at most one per output key), which keeps the second
    // round's probes in a few cached lines instead of the whole run.  (A third level
    // measured slower: each level adds a chain of dependent loads.)
    const uint32_t nb = t1 - t0;
    // co-rank of tile i, bracketed by the tiles il = i - i % S and min(il + S, nb) when S > 0
    auto search = [&](uint32_t i, uint32_t S) {
        const uint32_t o = (t0 + i) * T;
        if (o >= n) return 0u;
        const PairGeom g = pair_of(o, n, run, pr);
        uint32_t lo = 0u, hi = ~0u;
        if (S) {
            const uint32_t il = i - i % S, ih = il + S < nb ? il + S : nb;
            const uint32_t ol = (t0 + il) * T, oh = (t0 + ih) * T;
            if (pair_of(ol, n, run, pr).pb == g.pb) {
                lo = s_part[il];
                hi = lo + (o - ol);
            }
            if (oh < n && pair_of(oh, n, run, pr).pb == g.pb) {
                const uint32_t ah = s_part[ih];
                hi = hi < ah ? hi : ah;
                if (ah > oh - o && lo < ah - (oh - o)) lo = ah - (oh - o);
            }
        }
        return corank(src + g.pb, g.la, src + g.pb + g.la, g.lb, o - g.pb, flip, lo, hi);
    };
    for (uint32_t i = tid * MG_BRACKET; i <= nb; i += BLOCK * MG_BRACKET) s_part[i] = search(i, 0);
    if (tid == 0 && nb % MG_BRACKET) s_part[nb] = search(nb, 0);
    __syncthreads();
    for (uint32_t i = tid; i < nb; i += BLOCK)
        if (i % MG_BRACKET) s_part[i] = search(i, MG_BRACKET);
    __syncthreads();
    struct Geo {
        uint32_t o0, tot, la, sa, sb;  // output start, keys, A keys, A start, B start (absolute)
    };
    auto geo = [&](uint32_t t) {
        Geo q;
        q.o0 = t * T;
        const uint32_t o1 = (n - q.o0) < T ? n : q.o0 + T;
        const PairGeom g = pair_of(q.o0, n, run, pr);
        const uint32_t a0 = s_part[t - t0];
        const uint32_t a1 = (o1 - g.pb == g.la + g.lb) ? g.la : s_part[t + 1 - t0];
        const uint32_t b0 = (q.o0 - g.pb) - a0;
        q.tot = o1 - q.o0;
        q.la = a1 - a0;
        q.sa = g.pb + a0;
        q.sb = g.pb + g.la + b0;
        return q;
    };
    auto load = [&](const Geo &q, uint32_t (&v)[KPT], uint32_t (&vv)[KV ? KPT : 1]) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t k = tid + (uint32_t)j * BLOCK;
            const uint32_t a = k < q.la ? q.sa + k : q.sb + (k - q.la);
            v[j] = k < q.tot ? ld_stream<NT_MERGE>(src + a) : 0u;
            if constexpr (KV) vv[j] = k < q.tot ? vsrc[a] : 0u;
        }
    };
    uint32_t nx[KPT];
    uint32_t nv[KV ? KPT : 1];
    Geo cur = geo(t0);
    load(cur, nx, nv);
    for (uint32_t t = t0; t < t1; ++t) {
        __syncthreads();  // previous tile's merge no longer reads sm.in
        if constexpr (!KV && MG_PAD) {
            // keys only: A | MG_PADW words of +inf | B | MG_PADW words of +inf, so the network's
            // windows need no bounds checks (the keys-only merge is VALU-bound: r29)
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t i = tid + (uint32_t)j * BLOCK;
                if (i < cur.tot) sm.in[i + (i >= cur.la ? MG_PADW : 0u)] = nx[j];  // (not over B's pads)
            }
            if (tid < 2u * MG_PADW)
                sm.in[(tid < MG_PADW ? cur.la : cur.tot + MG_PADW) + tid % MG_PADW] = ~flip;  // +inf in key order
        } else {
#pragma unroll
            for (int j = 0; j < KPT; ++j) sm.in[tid + (uint32_t)j * BLOCK] = nx[j];
        }
        if constexpr (KV) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) sm.vin[tid + (uint32_t)j * BLOCK] = nv[j];
        }
        // next tile: geometry from the co-ranks, keys into registers
        Geo nxt = cur;
        if (t + 1 < t1) {
            nxt = geo(t + 1);
            load(nxt, nx, nv);
        }
        __syncthreads();  // sm.in holds the current tile
        const uint32_t la = cur.la, lb = cur.tot - cur.la, tot = cur.tot;
        const uint32_t *sa = sm.in, *sb = sm.in + la;
        const uint32_t d = tid * KPT < tot ? tid * KPT : tot;
        uint32_t r[KPT];
        uint32_t from[KV ? KPT : 1];  // key/value: LDS slot (sm.in) of each output
        if constexpr (!KV) {
            // keys only: the thread's KPT outputs are the KPT smallest of A[ai, ai+KPT) and
            // B[bi, bi+KPT) (equal keys are identical words, so the order among them does not
            // matter): both windows read at once, merged by a bitonic network in registers
            // (A ascending, B reversed), instead of KPT dependent LDS reads with a branch
            // each: 0.458 -> 0.437 ms per pass at 2^28 (r28, profiles/r28_ab_merge_network.txt;
            // a copy in place of any merge: 0.424)
            const uint32_t pb = la + (MG_PAD ? MG_PADW : 0u);  // B's LDS offset
            const uint32_t ai = corank(sa, la, sm.in + pb, lb, d, flip), bi = d - ai;
            uint32_t x[2 * KPT];
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t ia = ai + (uint32_t)j, ib = bi + (uint32_t)j;
                if constexpr (MG_PAD) {  // the pads end both windows
                    x[j] = sm.in[ia] ^ flip;
                    x[2 * KPT - 1 - j] = sm.in[pb + ib] ^ flip;
                } else {
                    const uint32_t va = sm.in[min(ia, T - 1u)] ^ flip;       // sa = sm.in
                    const uint32_t vb = sm.in[min(la + ib, T - 1u)] ^ flip;  // sb = sm.in + la
                    x[j] = ia < la ? va : 0xFFFFFFFFu;
                    x[2 * KPT - 1 - j] = ib < lb ? vb : 0xFFFFFFFFu;
                }
            }
#pragma unroll
            for (int s = KPT; s >= 1; s >>= 1) {
#pragma unroll
                for (int i = 0; i < 2 * KPT; ++i) {
                    if ((i & s) == 0) {
                        const uint32_t lo = min(x[i], x[i + s]), hi = max(x[i], x[i + s]);
                        x[i] = lo;
                        x[i + s] = hi;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < KPT; ++j) r[j] = x[j] ^ flip;
        } else {
            // key/value: stable, A before B on equal keys, each output's LDS slot kept (the
            // network on 64-bit (key, slot) words measured equal, 13.87-13.94 vs 13.94-13.96
            // ms per 2^28-pair merge sort: profiles/r28_ab_kv_network.txt)
            uint32_t ai = corank(sa, la, sb, lb, d, flip);
            uint32_t bi = d - ai;
            uint32_t va = ai < la ? sa[ai] : 0u;
            uint32_t vb = bi < lb ? sb[bi] : 0u;
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const bool takeA = (bi >= lb) || (ai < la && key_le(va, vb, flip));
                r[j] = takeA ? va : vb;
                if constexpr (KV) from[j] = takeA ? ai : la + bi;
                if (takeA) {
                    ++ai;
                    va = ai < la ? sa[ai] : 0u;
                } else {
                    ++bi;
                    vb = bi < lb ? sb[bi] : 0u;
                }
            }
        }
        uint32_t pv[KV ? KPT : 1];  // key/value: the payloads, all read before any store (as k_tile_sort)
        if constexpr (KV) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) pv[j] = sm.vin[from[j]];
        }
        if (KPT % 4 == 0 && tot == T && (((uintptr_t)dst) & 15u) == 0 && (!KV || (((uintptr_t)vdst) & 15u) == 0)) {
            // a full tile: each thread's KPT outputs are consecutive.  They go to HBM through
            // a wave-private transpose in sm.out (sm.vout for the payloads; both unused by
            // full tiles): written as each lane's KPT words, read back lane-contiguous,
            // stored as 16-B nontemporal stores that each cover 1 KB -- no barrier.  Stored
            // straight from the registers, each lane's two 16-B stores at a 32-B lane stride
            // leave every wave-store half of each line: 0.486 ms per pass at 2^28 against
            // 0.464 (r28; the A/B launcher is in git history, commit 402e9ea).
            const uint32_t lane = tid & 63u, w = tid >> 6;
            uint32_t *wo = sm.out + w * 64u * KPT;
#pragma unroll
            for (int j = 0; j < KPT / 4; ++j)
                *reinterpret_cast<uint4 *>(wo + lane * KPT + 4 * j) = make_uint4(r[4 * j], r[4 * j + 1], r[4 * j + 2], r[4 * j + 3]);
            if constexpr (KV) {
                uint32_t *wv = sm.vout + w * 64u * KPT;
#pragma unroll
                for (int j = 0; j < KPT / 4; ++j)
                    *reinterpret_cast<uint4 *>(wv + lane * KPT + 4 * j) =
                        make_uint4(pv[4 * j], pv[4 * j + 1], pv[4 * j + 2], pv[4 * j + 3]);
            }
            // the read-back takes other lanes' words: order the wave's LDS writes before it
            // (a wave's LDS operations complete in order on gfx950; this states it)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            u32x4 *o4 = reinterpret_cast<u32x4 *>(dst + cur.o0 + w * 64u * KPT);
#pragma unroll
            for (int j = 0; j < KPT / 4; ++j) {
                const uint4 v = *reinterpret_cast<const uint4 *>(wo + 4u * (lane + 64u * j));
                __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, o4 + lane + 64u * j);
            }
            // samp_out: every M4_S-th output key for a four-way pass next (merge4.hip): the
            // wave's 64 KPT outputs hold 64 KPT / M4_S of them, one store by as many lanes
            {
                static_assert((64 * KPT) % M4_S == 0 && (uint32_t)MG_TILE % M4_S == 0, "samples per wave");
                if (samp_out && lane < 64u * KPT / M4_S)
                    samp_out[(cur.o0 + w * 64u * KPT) / M4_S + lane] = wo[M4_S * lane];
            }
            if constexpr (KV) {
                const uint32_t *wv = sm.vout + w * 64u * KPT;
                u32x4 *ov4 = reinterpret_cast<u32x4 *>(vdst + cur.o0 + w * 64u * KPT);
#pragma unroll
                for (int j = 0; j < KPT / 4; ++j) {
                    const uint4 v = *reinterpret_cast<const uint4 *>(wv + 4u * (lane + 64u * j));
                    __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, ov4 + lane + 64u * j);
                }
            }
            cur = nxt;
            continue;
        }
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t idx = tid * KPT + j;
            if (idx < tot) {
                sm.out[idx + (idx >> 5)] = r[j];
                if constexpr (KV) sm.vout[idx + (idx >> 5)] = pv[j];
            }
        }
        __syncthreads();
        uint32_t *__restrict__ o = dst + cur.o0;
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t i = tid + (uint32_t)j * BLOCK;
            if (i < tot) {
                o[i] = sm.out[i + (i >> 5)];
                if (samp_out && ((cur.o0 + i) & (M4_S - 1u)) == 0u) samp_out[(cur.o0 + i) / M4_S] = sm.out[i + (i >> 5)];
            }
        }
        if constexpr (KV) {
            uint32_t *__restrict__ ov = vdst + cur.o0;
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t i = tid + (uint32_t)j * BLOCK;
                if (i < tot) ov[i] = sm.vout[i + (i >> 5)];
            }
        }
        cur = nxt;
    }
}

// two separate arrays, diagonal range [d0, d1): part has ntiles+1 entries
__global__ __launch_bounds__(256) void k_merge_part_ab(const uint32_t *__restrict__ A, uint32_t la,
                                                       const uint32_t *__restrict__ B, uint32_t lb, uint32_t d0,
                                                       uint32_t d1, uint32_t flip, uint32_t *__restrict__ part,
                                                       uint32_t ntiles) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > ntiles) return;
    uint32_t o = d0 + i * (uint32_t)MG_TILE;
    if (o > d1 || i == ntiles) o = d1;
    part[i] = corank(A, la, B, lb, o, flip);
}

template <int BLOCK, int KPT>
__global__ __launch_bounds__(BLOCK) void k_merge_ab(const uint32_t *__restrict__ A, const uint32_t *__restrict__ B,
                                                    uint32_t *__restrict__ out, uint32_t d0, uint32_t d1,
                                                    uint32_t flip, const uint32_t *__restrict__ part) {
    __shared__ MgSmem<> sm;
    const uint32_t i = blockIdx.x;
    const uint32_t o0 = d0 + i * (uint32_t)MG_TILE;
    const uint32_t o1 = (d1 - o0) < (uint32_t)MG_TILE ? d1 : o0 + (uint32_t)MG_TILE;
    const uint32_t a0 = part[i], a1 = part[i + 1];
    merge_tile<BLOCK, KPT>(A, a0, a1, B, o0 - a0, o1 - a1, out + (o0 - d0), flip, sm);
}

// ---------------------------------------------------------------------------------
// streaming copy: the practical ceiling of a read-once / write-once pass (bench.py's
// copy_ceiling).  16384-word tiles per 1024-thread workgroup, 4 x 16 B per lane,
// nontemporal loads and stores, persistent grid of one workgroup per CU (the layout of
// harness/exp/lsweep_probe.hip's fastest copy: 0.389 ms for 2^28 words, 5.5 TB/s).
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_stream_copy(const u32x4 *__restrict__ a, u32x4 *__restrict__ b, size_t n4) {
    const size_t ntiles = n4 / 4096;
    const uint32_t tid = threadIdx.x;
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const u32x4 *s = a + t * 4096 + tid;
        u32x4 k[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) k[j] = __builtin_nontemporal_load(s + j * 1024);
        u32x4 *d = b + t * 4096 + tid;
#pragma unroll
        for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(k[j], d + j * 1024);
    }
    for (size_t i = ntiles * 4096 + (size_t)blockIdx.x * 1024 + tid; i < n4; i += (size_t)gridDim.x * 1024) b[i] = a[i];
}
__global__ __launch_bounds__(256) void k_word_copy(const uint32_t *__restrict__ a, uint32_t *__restrict__ b, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}

// ---------------------------------------------------------------------------------
// verification helper
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_count_descents(const uint32_t *__restrict__ keys, size_t n, uint32_t flip,
                                                        uint32_t *__restrict__ count) {
    __shared__ uint32_t ws[4];
    uint32_t c = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += stride)
        c += ((keys[i] ^ flip) > (keys[i + 1] ^ flip)) ? 1u : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63u) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t s = ws[0] + ws[1] + ws[2] + ws[3];
        if (s) atomicAdd(count, s);
    }
}

// ---------------------------------------------------------------------------------
// splitter partition of a sorted run: out[i] = number of keys <= values[i]
// (upper bound, key order), one thread per value -- the multi-GPU exchange cuts
// each rank's sorted shard at the common splitters with it.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_upper_bound(const uint32_t *__restrict__ keys, uint32_t n, uint32_t flip,
                                                    const uint32_t *__restrict__ values, uint32_t nv,
                                                    uint32_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nv) return;
    const uint32_t v = values[i] ^ flip;
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if ((keys[mid] ^ flip) <= v) lo = mid + 1;
        else hi = mid;
    }
    out[i] = lo;
}

// =================================================================================
// host launchers
// =================================================================================
static inline unsigned blocks_for(size_t work, unsigned per, unsigned cap) {
    size_t b = (work + per - 1) / per;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (unsigned)b;
}

hipError_t launch_fill(uint32_t *out, size_t n, uint64_t seed, int dist, uint64_t param, uint64_t first,
                       hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_fill<<<blocks_for(n, 256 * 8, 8192), 256, 0, s>>>(out, n, seed, dist, param, first);
    return hipGetLastError();
}

hipError_t launch_histogram(const uint32_t *keys, size_t n, uint32_t flip, int bits, uint32_t *hist,
                            hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned g = blocks_for(n, 16384, 256);
    if (bits == 8) k_histogram<8><<<g, HIST_BLOCK, 0, s>>>(keys, n, flip, hist);
    else if (bits == 1) k_histogram<1><<<g, HIST_BLOCK, 0, s>>>(keys, n, flip, hist);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_plan(const uint32_t *hist, size_t n, int bits, int in_is_out, Plan *plan, hipStream_t s) {
    k_plan<<<1, 256, 0, s>>>(hist, (uint32_t)n, bits, in_is_out, plan);
    return hipGetLastError();
}

hipError_t launch_onesweep(Bufs b, const Plan *plan, int pass, int bits, size_t n, uint32_t flip,
                           const uint32_t *hist, uint32_t *lookback, uint32_t *counter, uint32_t *err,
                           hipStream_t s) {
    if (bits != 1) return hipErrorInvalidValue;  // 8-bit digits: the persistent pass
    const unsigned g = (unsigned)((n + OS_TILE - 1) / OS_TILE);
    k_onesweep<1, OS_BLOCK, OS_KPT><<<g, OS_BLOCK, 0, s>>>(b, plan, pass, (uint32_t)n, flip, hist, lookback, counter,
                                                           err);
    return hipGetLastError();
}

static int cu_count() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus;
}

hipError_t launch_onesweep_p(Bufs b, const Plan *plan, int pass, size_t n, uint32_t flip, const SegPlan *sp,
                             uint32_t *lookback, uint32_t *counter, uint32_t *err, hipStream_t s, const Bufs *vb) {
    if (n > RADIX_MAX_N) return hipErrorInvalidValue;  // buffer descriptors: 4 n bytes < 2^32 (osp_rsrc)
    const size_t ntiles = (n + OSP_TILE - 1) / OSP_TILE + NSEG;
    const size_t want = (size_t)cu_count();  // one workgroup per CU (LDS-bound)
    const unsigned g = (unsigned)(ntiles < want ? ntiles : want);
    if (vb)
        k_onesweep_p<true><<<g, OSP_KV_BLOCK, 0, s>>>(b, plan, pass, (uint32_t)n, flip, sp, lookback, counter, err, *vb);
    else
        k_onesweep_p<false><<<g, OSP_BLOCK, 0, s>>>(b, plan, pass, (uint32_t)n, flip, sp, lookback, counter, err, b);
    return hipGetLastError();
}


hipError_t launch_hist_seg(const uint32_t *keys, size_t n, uint32_t flip, uint32_t *hps, uint32_t *joint,
                           hipStream_t s) {
    if (n == 0) return hipSuccess;
    // workgroups per position segment: HS_BPS at large n; at small n at least
    // HS_MIN_KEYS keys each, since every workgroup flushes ~13 K counters with global
    // atomics (512 workgroups at 2^20: 97 us, contended on the same 48 KB)
    size_t bps = n / ((size_t)NSEG * HS_MIN_KEYS);
    bps = bps < 1 ? 1 : bps > (size_t)HS_BPS ? (size_t)HS_BPS : bps;
    k_hist_seg<<<NSEG * (unsigned)bps, HIST_BLOCK, 0, s>>>(keys, n, flip, hps, joint, (uint32_t)bps);
    return hipGetLastError();
}

hipError_t launch_plan8(const uint32_t *hps, const uint32_t *joint, size_t n, int in_is_out, Plan *plan,
                        SegPlan *segplans, uint32_t *hist, void *zero_p, size_t zero_bytes, hipStream_t s) {
    // the look-back clear rides in the plan launch (workgroups 1..): one launch fewer (r27)
    const bool fold = zero_bytes % 16 == 0;
    if (!fold && zero_bytes) {
        const hipError_t z = launch_zero(zero_p, zero_bytes, s);
        if (z != hipSuccess) return z;
    }
    const size_t zn4 = fold ? zero_bytes / 16 : 0;
    const unsigned g = 4u + (zn4 ? blocks_for(zn4, 256 * 4, 2048) : 0u);
    k_plan8<<<g, 256, 0, s>>>(hps, joint, (uint32_t)n, in_is_out, 1, plan, segplans, hist,
                              static_cast<uint4 *>(zero_p), zn4);
    return hipGetLastError();
}


// Zero a workspace range with a kernel instead of hipMemsetAsync: the sorts' zeroing must
// replay inside captured HIP graphs (tests/test_gpu_graph.py), which a kernel node does.
__global__ __launch_bounds__(256) void k_zero(uint4 *__restrict__ p4, size_t n4, uint32_t *__restrict__ tail,
                                             uint32_t ntail) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) p4[i] = make_uint4(0, 0, 0, 0);
    if (blockIdx.x == 0 && threadIdx.x < ntail) tail[threadIdx.x] = 0u;
}

hipError_t launch_zero(void *p, size_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    // callers pass 4-byte multiples starting 16-byte aligned
    const size_t n4 = bytes / 16;
    uint32_t *tail = reinterpret_cast<uint32_t *>(static_cast<char *>(p) + n4 * 16);
    const uint32_t ntail = (uint32_t)((bytes - n4 * 16) / 4);
    k_zero<<<blocks_for(n4 ? n4 : 1, 256 * 4, 2048), 256, 0, s>>>(static_cast<uint4 *>(p), n4, tail, ntail);
    return hipGetLastError();
}

hipError_t launch_final_copy(Bufs b, const Plan *plan, size_t n, hipStream_t s) {
    k_final_copy<<<blocks_for(n, 256 * 16, 4096), 256, 0, s>>>(b, plan, n);
    return hipGetLastError();
}

hipError_t launch_tile_sort(const uint32_t *in, uint32_t *out, size_t n, uint32_t flip, hipStream_t s,
                            uint32_t *samp_out) {
    if (n == 0) return hipSuccess;
    const size_t nt = (n + TS_TILE - 1) / TS_TILE;
    k_tile_sort<TS_KBLOCK, TS_KPT><<<(unsigned)nt, TS_KBLOCK, 0, s>>>(in, out, nullptr, nullptr, (uint32_t)n, flip,
                                                                     samp_out);
    return hipGetLastError();
}

hipError_t launch_wave_tile_sort(uint32_t *keys, size_t n, uint32_t flip, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned g = (unsigned)((n + 255) / 256);
    k_wave_split<<<g, 256, 0, s>>>(keys, (uint32_t)n, flip);
    return hipGetLastError();
}

hipError_t launch_merge_pass(const uint32_t *in, uint32_t *out, size_t n, size_t run, uint32_t flip,
                             uint32_t *part, hipStream_t s, const uint32_t *vin, uint32_t *vout, const MgPairs *pairs,
                             uint32_t *samp_out) {
    MgPairs pr{};
    if (pairs) pr = *pairs;
    if (n == 0) return hipSuccess;
    (void)part;  // co-ranks are found inside k_merge_pass_p
    const uint32_t ntiles = (uint32_t)((n + MG_TILE - 1) / MG_TILE);
    const uint32_t want = (uint32_t)(MG_BLOCKS_PER_CU * cu_count());
    uint32_t m = (ntiles + want - 1) / want;  // consecutive tiles per workgroup
    if (m > (uint32_t)MG_MAX_TPB) m = MG_MAX_TPB;
    const uint32_t g = (ntiles + m - 1) / m;
    if (vin)
        k_merge_pass_p<MG_BLOCK, MG_KPT, true>
            <<<g, MG_BLOCK, 0, s>>>(in, out, (uint32_t)n, (uint32_t)run, flip, ntiles, m, pr, vin, vout, samp_out);
    else
        k_merge_pass_p<MG_BLOCK, MG_KPT><<<g, MG_BLOCK, 0, s>>>(in, out, (uint32_t)n, (uint32_t)run, flip, ntiles, m, pr,
                                                                nullptr, nullptr, samp_out);
    return hipGetLastError();
}

hipError_t launch_tile_sort_kv(const uint32_t *in, uint32_t *out, const uint32_t *vin, uint32_t *vout, size_t n,
                               uint32_t flip, hipStream_t s, uint32_t *samp_out) {
    if (n == 0) return hipSuccess;
    const unsigned g = (unsigned)((n + TS_TILE_KV - 1) / TS_TILE_KV);
    k_tile_sort<TS_BLOCK, TS_KPT_KV, true><<<g, TS_BLOCK, 0, s>>>(in, out, vin, vout, (uint32_t)n, flip, samp_out);
    return hipGetLastError();
}

hipError_t launch_merge_ab(const uint32_t *a, size_t la, const uint32_t *b, size_t lb, uint32_t *out, size_t d0,
                           size_t d1, uint32_t flip, uint32_t *part, hipStream_t s) {
    if (d1 <= d0) return hipSuccess;
    const uint32_t ntiles = (uint32_t)((d1 - d0 + MG_TILE - 1) / MG_TILE);
    k_merge_part_ab<<<(ntiles + 1 + 255) / 256, 256, 0, s>>>(a, (uint32_t)la, b, (uint32_t)lb, (uint32_t)d0,
                                                              (uint32_t)d1, flip, part, ntiles);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    k_merge_ab<MG_BLOCK, MG_KPT><<<ntiles, MG_BLOCK, 0, s>>>(a, b, out, (uint32_t)d0, (uint32_t)d1, flip, part);
    return hipGetLastError();
}

hipError_t launch_upper_bound(const uint32_t *keys, size_t n, uint32_t flip, const uint32_t *values, size_t nv,
                              uint32_t *out, hipStream_t s) {
    if (nv == 0) return hipSuccess;
    k_upper_bound<<<(unsigned)((nv + 63) / 64), 64, 0, s>>>(keys, (uint32_t)n, flip, values, (uint32_t)nv, out);
    return hipGetLastError();
}

hipError_t launch_stream_copy(const uint32_t *in, uint32_t *out, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (((((uintptr_t)in) | ((uintptr_t)out)) & 15u) == 0) {
        const size_t n4 = n / 4;
        if (n4) k_stream_copy<<<(unsigned)cu_count(), 1024, 0, s>>>(reinterpret_cast<const u32x4 *>(in), reinterpret_cast<u32x4 *>(out), n4);
        if (n % 4) k_word_copy<<<1, 256, 0, s>>>(in + n4 * 4, out + n4 * 4, n % 4);
    } else {
        k_word_copy<<<blocks_for(n, 256 * 16, 4096), 256, 0, s>>>(in, out, n);
    }
    return hipGetLastError();
}

hipError_t launch_count_descents(const uint32_t *keys, size_t n, uint32_t flip, uint32_t *count, hipStream_t s) {
    if (n < 2) return hipSuccess;
    k_count_descents<<<blocks_for(n, 256 * 16, 4096), 256, 0, s>>>(keys, n, flip, count);
    return hipGetLastError();
}

}  // namespace labsort

