// lsweep_exp.hip -- EXPERIMENT, not in the product (r28): the local first pass of the 8-bit
// LSD radix sort (keys only, onesweep path).  It ran in the product for one build with the
// gathering first onesweep pass (kernels.hip at commit 4cccab1): correct on 479 radix GPU
// tests, but 2.417 ms per 2^28 sort against 2.127 ms for the histogram path (k_lsweep
// 0.642 ms, the gathering pass 0.785 ms), so the histogram path was
// restored.  Kept for harness/exp/lsweep_probe.hip.
//
// The onesweep pass (kernels.hip, k_onesweep_p) needs every digit's global offset before
// it scatters, so the classic design reads the keys once more up front (k_hist_seg:
// 4 B/key, 0.24 ms of a 2.1 ms sort at 2^28).  The first pass does not need them: it can
// leave its output in a LOGICAL order instead (as the gathered radix of gsweep.hip does):
//
//   k_lsweep   each 16384-key tile is sorted by digit 0 in LDS (the stable wave rank of
//              the onesweep pass) and written back CONTIGUOUSLY at its own position
//              (whole 16-B lanes, no partial granules, no look-back).  Its digit counts
//              and local offsets go to a 1-KB row; the same read of the keys counts the
//              three 12-bit joint fields (top nibble of digit p, digit p + 1) that size
//              the later passes' look-back segments, and the digit-0 totals -- what
//              k_hist_seg counted, without a read of its own.
//   k_lscan    from the rows: the logical start and source address of every (digit, tile)
//              run in digit-major order and, for every TILE-aligned logical tile, the
//              first run it covers (the global exclusive scan of letra.pdf's split over
//              counts only; decoupled look-back over 64-tile groups).
//   pass 1     the first active onesweep pass GATHERS its tiles through those tables
//              (k_onesweep_p<..., GATHER>) and scatters by its digit as before.
//
// The reference's counterpart is the split of radix_sort_kernel (lab.cu:47-87: a
// block-local stable split by one bit, exlusiveScan lab.cu:11-41) followed by letra.pdf's
// global scan and scatter; here a tile is split by 8 bits at once and the scatter of the
// first pass is deferred to the second pass's gather.
#include "../../include/labsort.h"
#include "../../radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/csrc/common.h"
#include "../../radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/csrc/devutil.h"

namespace labsort {

constexpr int LS_BLOCK = 1024, LS_KPT = 16, LS_TILE = LS_BLOCK * LS_KPT;
constexpr int LS_GROUP = 64;  // tiles per k_lscan workgroup
struct GthTables {            // k_lscan's run tables (ls, sr: digit-major; first: per tile)
    uint32_t *ls, *sr, *first;
};

namespace {

constexpr int LB = LS_BLOCK, LK = LS_KPT, LT = LS_TILE, LW = LS_BLOCK / WAVE;
constexpr int LJF = 4096;  // 12-bit joint fields
static_assert(LT == OSP_TILE, "pass 1 reads the local pass's tiles as its logical tiles");

// LDS word of tile slot i in the reorder buffer: 4 pad words per 32 slots, so slots
// 4m .. 4m+3 are one 16-B aligned LDS word group (the write-out reads them with
// ds_read_b128) and a wave's stores to slots 64 apart (sorted input: every digit of a
// tile has the same count) spread over 4 banks
__device__ __forceinline__ uint32_t ls_pad(uint32_t i) { return i + ((i >> 5) << 2); }

struct LsSmem {
    uint32_t keys[LT + LT / 8];
    uint32_t wh[LW * 256];
    uint32_t jh[3 * LJF];
    uint32_t probe[WAVE];
    uint32_t wsum[8];
    uint32_t ordered;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ls_rsrc(const uint32_t *p, uint32_t n) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0, (int)(n * 4u), 0x00020000);
}

// Joint fields of one key slot of a wave, counted into jh (3 x 4096 counters): fields
// f_p = (key ^ flip) >> (8p + 4), 12 bits (the top nibble of digit p and digit p + 1).
// Random keys: one LDS add per lane and field.  A wave whose keys repeat a field (sorted,
// clustered or small keys: many lanes on one counter would serialise) adds each run of
// equal values in consecutive lanes once instead: lane-run leaders by one shuffle and
// one ballot, the run length from the next leader.  The choice is made per wave and
// tile from its first slot (another lane sharing lane 0's value: 1 in 64 for uniform
// 12-bit fields).  ok: the lane holds a real key (partial last tile).
__device__ __forceinline__ void ls_count_runs(uint32_t *jh, uint32_t f, bool ok, uint32_t lane) {
    const uint32_t fp = __shfl_up(f, 1);
    const bool lead = ok && (lane == 0 || f != fp);
    const uint64_t L = __ballot(lead);
    // (both ballots with the whole wave active: a ballot inside the select below would be
    // compiled into its divergent arm and count only the lanes that take it)
    const uint32_t nok = (uint32_t)__popcll(__ballot(ok));
    const uint64_t after = L & ~((2ull << lane) - 1ull);  // leaders after this lane (lane 63: none)
    const uint32_t next = after ? (uint32_t)__builtin_ctzll(after) : nok;
    if (lead) atomicAdd(jh + f, next - lane);
}
__device__ __forceinline__ bool ls_repeats(uint32_t f) {
    const uint32_t f0 = __builtin_amdgcn_readfirstlane(f);
    return __popcll(__ballot(f == f0)) > 1;
}

}  // namespace

// Persistent: workgroup b sorts tiles b, b + G, b + 2G, ... (G = grid), the next tile's
// keys loading into registers while the current one is ranked, reordered and written.
// rows[t * 256 + d] = local offset of digit d in tile t | count << 16.  tot0[d] += the
// digit-0 counts, joint[((p + 1) * NSEG + nibble) * 256 + digit] += the joint fields
// (both zeroed by the caller).
__global__ __launch_bounds__(LB, 4) void k_lsweep(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint32_t n,
                                                 uint32_t flip, uint32_t *__restrict__ rows, uint32_t *__restrict__ tot0,
                                                 uint32_t *__restrict__ joint) {
    __shared__ LsSmem sm;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t ntiles = (n + (uint32_t)LT - 1u) / (uint32_t)LT;
    for (uint32_t i = tid; i < (uint32_t)(LW * 256); i += LB) sm.wh[i] = 0u;
    for (uint32_t i = tid; i < (uint32_t)(3 * LJF); i += LB) sm.jh[i] = 0u;
    if (wid == 0) {
        const bool ord = lds_lane_ordered(sm.probe, lane);
        if (lane == 0) sm.ordered = ord ? 1u : 0u;
    }
    const __amdgpu_buffer_rsrc_t rin = ls_rsrc(in, n), rout = ls_rsrc(out, n);
    const uint32_t sentinel = ~flip;  // digit 255: ranks after every real key of the tile
    const uint32_t woff = wid * (LK * WAVE) + lane;
    constexpr int NT = (NT_LOADS & NT_OSP) ? 2 : 0;  // streamed (read once)
    auto load = [&](uint32_t t, uint32_t (&k)[LK]) {
        const uint32_t beg = t * (uint32_t)LT, nv = n - beg < (uint32_t)LT ? n - beg : (uint32_t)LT;
        const uint32_t o = (beg + woff) * 4u;
        if (nv == (uint32_t)LT) {
#pragma unroll
            for (int j = 0; j < LK; ++j) k[j] = __builtin_amdgcn_raw_buffer_load_b32(rin, o + j * WAVE * 4, 0, NT);
        } else {  // out-of-range buffer loads return 0: replaced by the sentinel
#pragma unroll
            for (int j = 0; j < LK; ++j) {
                const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rin, o + j * WAVE * 4, 0, NT);
                k[j] = woff + j * WAVE < nv ? v : sentinel;
            }
        }
    };
    uint32_t t = blockIdx.x;
    uint32_t kN[LK], kB[LK];
    if (t < ntiles) load(t, kN);
    __syncthreads();
    const bool atomic_rank = __builtin_amdgcn_readfirstlane(sm.ordered) != 0u;
    uint32_t *wh = sm.wh + wid * 256;
    uint32_t ctot = 0;  // thread d < 256: digit d's count over this workgroup's tiles
    for (; t < ntiles; t += gridDim.x) {
#pragma unroll
        for (int j = 0; j < LK; ++j) kB[j] = kN[j];
        const uint32_t beg = t * (uint32_t)LT, nvalid = n - beg < (uint32_t)LT ? n - beg : (uint32_t)LT;
        if (t + gridDim.x < ntiles) load(t + gridDim.x, kN);
        // stable wave rank by digit 0 (slot-major order = position order)
        uint32_t rk[LK / 2];
#pragma unroll
        for (int j = 0; j < LK; ++j) {
            const uint32_t d = (kB[j] ^ flip) & 255u;
            uint32_t r;
            if (atomic_rank) {
                r = wave_atomic_rank(wh, d, lane);
            } else {
                const uint64_t m = match8(d);
                const uint32_t pre = mbcnt64(m), old = wh[d];
                if (pre == 0) wh[d] = old + (uint32_t)__popcll(m);
                r = old + pre;
            }
            rk[j / 2] = (j & 1) ? rk[j / 2] | (r << 16) : r;
        }
        // the joint fields (3 per key), plain adds unless this wave's keys repeat them
        {
            bool rep = false;
#pragma unroll
            for (int p = 0; p < 3; ++p) rep |= ls_repeats(((kB[0] ^ flip) >> (8 * p + 4)) & (LJF - 1u));
            if (!rep && nvalid == (uint32_t)LT) {
#pragma unroll
                for (int j = 0; j < LK; ++j) {
                    const uint32_t x = kB[j] ^ flip;
#pragma unroll
                    for (int p = 0; p < 3; ++p) atomicAdd(sm.jh + p * LJF + ((x >> (8 * p + 4)) & (LJF - 1u)), 1u);
                }
            } else {
#pragma unroll
                for (int j = 0; j < LK; ++j) {
                    const uint32_t x = kB[j] ^ flip;
                    const bool ok = woff + j * WAVE < nvalid;
#pragma unroll
                    for (int p = 0; p < 3; ++p) ls_count_runs(sm.jh + p * LJF, (x >> (8 * p + 4)) & (LJF - 1u), ok, lane);
                }
            }
        }
        __syncthreads();  // (1) wave counts
        uint32_t tot = 0;
        if (tid < 256u) {
#pragma unroll
            for (int w = 0; w < LW; ++w) tot += sm.wh[w * 256 + tid];
        }
        const uint32_t ds = block_excl_scan<LB, 256>(tot, sm.wsum);  // (barrier)
        if (tid < 256u) {
            uint32_t run = ds;
#pragma unroll
            for (int w = 0; w < LW; ++w) {
                const uint32_t c = sm.wh[w * 256 + tid];
                sm.wh[w * 256 + tid] = run;
                run += c;
            }
            const uint32_t cnt = tid == 255u ? tot - ((uint32_t)LT - nvalid) : tot;  // drop the sentinels
            rows[(size_t)t * 256 + tid] = ds | (cnt << 16);
            ctot += cnt;
        }
        __syncthreads();  // (2) per-wave digit offsets
#pragma unroll
        for (int j = 0; j < LK; ++j) {
            const uint32_t d = (kB[j] ^ flip) & 255u;
            sm.keys[ls_pad(wh[d] + ((rk[j / 2] >> ((j & 1) * 16)) & 0xFFFFu))] = kB[j];
        }
        __syncthreads();  // (3) the tile sorted by digit 0 in LDS
        if (nvalid == (uint32_t)LT) {
#pragma unroll
            for (int g = 0; g < LK / 4; ++g) {
                const uint32_t q = (uint32_t)g * LB + tid;  // slots 4q .. 4q + 3
                const uint4 v = *reinterpret_cast<const uint4 *>(sm.keys + ls_pad(4u * q));
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, rout, (beg + 4u * q) * 4u, 0, 0);
            }
        } else {
#pragma unroll
            for (int j = 0; j < LK; ++j) {
                const uint32_t i = (uint32_t)j * LB + tid;
                if (i < nvalid) __builtin_amdgcn_raw_buffer_store_b32(sm.keys[ls_pad(i)], rout, (beg + i) * 4u, 0, 0);
            }
        }
        // each wave clears its own counters (read by no other wave before barrier (1))
        for (uint32_t i = lane; i < 256u; i += WAVE) wh[i] = 0u;
    }
    if (tid < 256u && ctot) atomicAdd(tot0 + tid, ctot);
    {
        __syncthreads();
        // field f = (digit p+1) << 4 | (top nibble of digit p) -> joint[p+1][nibble][digit];
        // each workgroup starts its flush at a different place, so the atomics of
        // workgroups that finish together do not queue on the same lines
        const uint32_t rot = (blockIdx.x * (uint32_t)LB) % (3u * LJF);
        for (uint32_t i0 = tid; i0 < 3u * LJF; i0 += LB) {
            uint32_t i = i0 + rot;
            i = i >= 3u * LJF ? i - 3u * LJF : i;
            const uint32_t c = sm.jh[i];
            const uint32_t p = i / LJF, f = i % LJF;
            if (c) atomicAdd(&joint[((p + 1) * NSEG + (f & 15u)) * 256 + (f >> 4)], c);
        }
    }
}

// ---------------------------------------------------------------------------------
// k_lscan: the run tables of the local pass's logical order.  Run e = d * ntp + t (digit
// d of tile t: rows[t][d] = loc | count << 16) starts at logical position
//   ls[e] = G0[d] + sum_{t' < t} count(t', d)       (G0 = exclusive scan of the totals)
// and at address sr[e] = t * TILE + loc in the local pass's output; ls[256 ntp] = n.
// first[T] = the run holding logical position T * TILE, first[ntp] = the run holding n - 1.
// One workgroup per LG-tile group (acquired in order from gctr; the groups' column sums
// are chained by decoupled look-back over flags, every wait bounded: an expired spin sets
// the error word); 4 threads per digit, 16 tiles each.  The digit-major writes go through
// LDS so each is a 256-B line segment.
// ---------------------------------------------------------------------------------
constexpr int LG = LS_GROUP;
__global__ __launch_bounds__(1024) void k_lscan(const uint32_t *__restrict__ rows, const uint32_t *__restrict__ tot0,
                                                uint32_t *flags, uint32_t *gctr, uint32_t *err, uint32_t *__restrict__ ls,
                                                uint32_t *__restrict__ sr, uint32_t *__restrict__ first, uint32_t ntp,
                                                uint32_t n) {
    constexpr int TPQ = LG / 4;
    __shared__ uint32_t lsb[LG][257], srb[LG][257];
    __shared__ uint32_t part[4][256], gbase[256], wsum[16], gid;
    const uint32_t tid = threadIdx.x, d = tid & 255u, q = tid >> 8;
    if (tid == 0) gid = atomicAdd(gctr, 1u);
    __syncthreads();
    const uint32_t g = gid;
    const uint32_t t0 = g * LG + q * TPQ;
    uint32_t w[TPQ], h = 0;
#pragma unroll
    for (int i = 0; i < TPQ; ++i) {
        w[i] = t0 + i < ntp ? rows[(size_t)(t0 + i) * 256 + d] : 0u;
        h += w[i] >> 16;
    }
    part[q][d] = h;
    // global digit-0 offsets from the totals (the local pass accumulated them)
    const uint32_t gx = block_excl_scan<1024, 256>(q == 0 ? tot0[d] : 0u, wsum);
    __syncthreads();  // part[][] complete
    if (q == 0) {
        const uint32_t agg = part[0][d] + part[1][d] + part[2][d] + part[3][d];
        uint32_t *fl = flags + (size_t)g * 256 + d;
        st_agent(fl, (g == 0 ? LB_INC : LB_AGG) | agg);
        uint32_t excl = 0;
        if (g > 0) {
            uint32_t t = g - 1, spins = 0;
            for (;;) {
                const uint32_t v = ld_agent(flags + (size_t)t * 256 + d);
                if ((v & ~LB_VAL) == 0u) {
                    if (++spins > SPIN_LIMIT) {
                        atomicOr(err, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += v & LB_VAL;
                if (v & LB_INC) break;
                --t;
            }
            st_agent(fl, LB_INC | (excl + agg));
        }
        gbase[d] = gx + excl;
    }
    __syncthreads();
    uint32_t run = gbase[d];
    for (uint32_t r = 0; r < q; ++r) run += part[r][d];
#pragma unroll
    for (int i = 0; i < TPQ; ++i) {
        const uint32_t t = t0 + i;
        const uint32_t hh = w[i] >> 16, l = run;
        run += hh;
        lsb[q * TPQ + i][d] = l;
        srb[q * TPQ + i][d] = t * (uint32_t)LT + (w[i] & 0xFFFFu);
        if (hh && t < ntp) {
            const uint32_t e = d * ntp + t;
            for (uint32_t T = (l + LT - 1) / LT; T < ntp && T * (uint32_t)LT < l + hh; ++T) first[T] = e;
            if (l <= n - 1 && n - 1 < l + hh) first[ntp] = e;
        }
    }
    if (g == 0 && tid == 0) ls[(size_t)256 * ntp] = n;  // the sentinel start after the last run
    __syncthreads();
    // digit-major writes: lane ti of every wave writes tile g*LG + ti of its digits
    const uint32_t lane = tid & 63u, wv = tid >> 6, tg = g * LG + lane;
    if (tg < ntp) {
        for (uint32_t dd = wv; dd < 256u; dd += 16u) {
            ls[(size_t)dd * ntp + tg] = lsb[lane][dd];
            sr[(size_t)dd * ntp + tg] = srb[lane][dd];
        }
    }
}

hipError_t launch_lsweep(const uint32_t *in, uint32_t *out, size_t n, uint32_t flip, uint32_t *rows, uint32_t *tot0,
                         uint32_t *joint, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const size_t ntiles = (n + LT - 1) / LT;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    const unsigned g = (unsigned)(ntiles < (size_t)cus ? ntiles : (size_t)cus);  // one workgroup per CU (LDS-bound)
    k_lsweep<<<g, LB, 0, s>>>(in, out, (uint32_t)n, flip, rows, tot0, joint);
    return hipGetLastError();
}

hipError_t launch_lscan(const uint32_t *rows, const uint32_t *tot0, uint32_t *flags, uint32_t *gctr, uint32_t *err,
                        GthTables tb, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t ntp = (uint32_t)((n + LT - 1) / LT), ng = (ntp + LG - 1) / LG;
    k_lscan<<<ng, 1024, 0, s>>>(rows, tot0, flags, gctr, err, const_cast<uint32_t *>(tb.ls), const_cast<uint32_t *>(tb.sr),
                                const_cast<uint32_t *>(tb.first), ntp, (uint32_t)n);
    return hipGetLastError();
}

}  // namespace labsort
