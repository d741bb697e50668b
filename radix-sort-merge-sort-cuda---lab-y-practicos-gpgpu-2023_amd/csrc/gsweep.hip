// gsweep.hip -- LSD radix sort whose passes gather their reads and write whole tiles.
//
// The onesweep pass (kernels.hip, k_onesweep_p) reads its tile contiguously and
// scatters it: every (tile, digit) run of ~64 keys lands at an arbitrary word offset,
// so the 64-B granules at run edges are written partially by two tiles.  On MI355X
// that write shape caps a pass at ~0.55 ms for 2^28 keys (harness/exp/bw_probe.hip:
// abutting misaligned 64-word runs 0.55 ms, the same runs read instead of written
// 0.44 ms, a tiled copy 0.39 ms).  Here every pass reverses the shape:
//
//   pass p (k_gsweep): tile T of the pass's LOGICAL input -- the keys in the order
//     the previous pass defines -- is gathered run by run from the previous pass's
//     output, sorted by digit p in LDS (stable wave rank, as the onesweep pass), and
//     written back CONTIGUOUSLY at T's own position: whole lines, no partial granules.
//     The tile's digit counts and local offsets go to a row of `rt`.
//   scan (k_gsum, k_gout): from the rows, the logical start of every
//     (tile, digit) run (global digit offset + counts of earlier tiles) in digit-major
//     order, its source address, and for every next-pass tile the first run it covers.
//     This is the global exclusive scan of letra.pdf's split (lab.cu's per-bit
//     "totalFalses" generalised to 256 digits) done once per pass over counts only.
//   final (k_gcopy): the logical order after the last pass is the sorted array; one
//     gathered read + contiguous write produces it.
//
// Pass 0 reads the input contiguously and also records every tile's digit min/max, so
// passes whose digit is the same for every key are skipped on the device (the
// deterministic counterpart of the reference's "stop when sorted", lab.cu:61).
// Tiles of a pass are independent; the only look-back is k_gsum's over the groups of
// GS_GROUP tiles (at most 128 of them), and only above GS_SMALL_NG groups.
//
// Logical input of pass p >= 1 (previous pass q wrote buffer X): run (t, d) = the keys
// of digit d in tile t of X, at X[t*TILE + lo(t,d)], length h(t,d); runs in the order
// (d, t) are the keys in order.  Tables per buffer, digit-major, e = d*ntp + t:
//   ls[e]     logical start of run e (ls[256*ntp] = n)
//   sr[e]     source address t*TILE + lo(t,d)
//   first[T]  e of the run holding logical position T*TILE; first[ntp]: position n-1
#include <algorithm>

#include "../../include/labsort.h"
#include "common.h"
#include "devutil.h"

namespace labsort {

namespace {

constexpr int GB = GS_BLOCK, GK = GS_KPT, GT = GS_TILE, GW = GS_BLOCK / WAVE;
// launch bounds: at least this many waves per SIMD (a VGPR cap).  k_gsweep needs 77
// VGPRs, k_gcopy 54, so 6 waves per SIMD fit: 3 workgroups of 512 per CU.
constexpr int GS_WAVES_PER_EU = 3;
static_assert(GT == GB * GK && GW * WAVE == GB, "tile shape");

struct GsTables {
    uint32_t *ls, *sr, *first;
};

// Workspace header (first 512 B; word 0 is the labsort error word, never set here)
struct GsState {
    uint32_t err;       // labsort's device error word (a scan look-back spin expired)
    uint32_t pad;
    uint32_t dmin[4];   // per digit, min / max over all keys (flipped digit values), from pass 0
    uint32_t dmax[4];
    uint32_t gctr[4];   // per pass: scan groups acquired (k_gsum's dynamic group ids)
};
constexpr uint32_t GS_SPIN_LIMIT = 1u << 22;

// digit min / max: GsState (written by the scan after pass 0), or GsMM in LDS (the fused
// small path: every workgroup reduces the tiles' pairs itself)
struct GsMM {
    uint32_t dmin[4], dmax[4];
};
template <class S>
__device__ __forceinline__ bool gs_active(const S *st, int pass) {
    return pass == 0 || st->dmin[pass] != st->dmax[pass];
}

// The buffer holding the logical order before pass p (0: the input, 1: A, 2: B): pass 0
// always runs and writes A, every later active pass writes the other buffer.  A
// function of the digit min / max only (written once, by pass 0's scan), so no kernel
// ever updates shared "current buffer" state while others read it.
template <class S>
__device__ __forceinline__ uint32_t gs_cur(const S *st, int p) {
    if (p == 0) return 0u;
    uint32_t nact = 1;
    for (int q = 1; q < p; ++q) nact += st->dmin[q] != st->dmax[q] ? 1u : 0u;
    return (nact & 1u) ? 1u : 2u;
}
template <class S>
__device__ __forceinline__ uint32_t gs_dst(const S *st, int p) { return gs_cur(st, p) == 1u ? 2u : 1u; }

// tiles dealt per XCD: blocks b, b+8, b+16, ... (one XCD) take consecutive tiles, so a
// run's neighbouring reads meet in one L2 (bw_probe: gather 0.49 -> 0.44 ms)
__device__ __forceinline__ uint32_t gs_tile(uint32_t b, uint32_t ntp) {
    const uint32_t per = (ntp + 7u) >> 3;
    return (b & 7u) * per + (b >> 3);
}

// ---- digit min / max of the tile pairs ------------------------------------------------
// bytewise min / max of packed digit words (byte q = digit q of key ^ flip)
__device__ __forceinline__ uint32_t bmin4(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t x = (a >> (8 * q)) & 255u, y = (b >> (8 * q)) & 255u;
        r |= (x < y ? x : y) << (8 * q);
    }
    return r;
}
__device__ __forceinline__ uint32_t bmax4(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t x = (a >> (8 * q)) & 255u, y = (b >> (8 * q)) & 255u;
        r |= (x > y ? x : y) << (8 * q);
    }
    return r;
}
// Wave-wide bytewise min / max of (mn, mx) pairs, result in every lane.
__device__ __forceinline__ void wave_minmax4(uint32_t &mn, uint32_t &mx) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        mn = bmin4(mn, __shfl_xor(mn, off));
        mx = bmax4(mx, __shfl_xor(mx, off));
    }
}
// Digit min / max over `cnt` packed (min, max) pairs into st->dmin / dmax.  Whole
// block, block-uniform call (barrier).
template <int BLOCK, class S>
__device__ __forceinline__ void gs_reduce_minmax(const uint32_t *pairs, uint32_t cnt, uint32_t (*red)[2], S *st) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    uint32_t mn = 0xFFFFFFFFu, mx = 0u;
    for (uint32_t i = tid; i < cnt; i += BLOCK) {
        mn = bmin4(mn, pairs[2 * i]);
        mx = bmax4(mx, pairs[2 * i + 1]);
    }
    wave_minmax4(mn, mx);
    if (lane == 0) {
        red[wid][0] = mn;
        red[wid][1] = mx;
    }
    __syncthreads();
    if (tid < 4u) {
        uint32_t a = 255u, b = 0u;
#pragma unroll
        for (int w = 0; w < BLOCK / WAVE; ++w) {
            const uint32_t x = (red[w][0] >> (8 * tid)) & 255u, y = (red[w][1] >> (8 * tid)) & 255u;
            a = x < a ? x : a;
            b = y > b ? y : b;
        }
        st->dmin[tid] = a;
        st->dmax[tid] = b;
    }
}

struct GsRuns {
    uint32_t bits[GT / 32];     // run-start bitmap over the tile's positions
    uint32_t wpre[GT / 32];     // exclusive prefix of the bitmap words' popcounts
    int32_t delta[GS_KMAX];     // per nonempty run, in order: source address - logical position
    uint32_t wsum[8];
};

// Keys of tile T (positions L0 + wid*GK*64 + j*64 + lane) of the logical order held in
// `src` with tables tb; sentinel past nvalid.  Block-uniform control flow (barriers).
// The run of position p = (number of nonempty runs starting at or before p) - 1, read
// off a start bitmap with one popcount, so the 16 slots of a lane are independent and
// their loads issue back to back.
__device__ __forceinline__ void gs_gather(const uint32_t *__restrict__ src, const GsTables &tb, uint32_t T,
                                          uint32_t L0, uint32_t nvalid, uint32_t sentinel, GsRuns &g,
                                          uint32_t (&k)[GK], uint32_t tid, uint32_t lane, uint32_t wid) {
    const uint32_t e0 = tb.first[T], e1 = tb.first[T + 1];
    const uint32_t K = e1 - e0 + 1;  // runs of the tile, empty ones included
    const uint32_t pw = wid * (GK * WAVE) + lane;
    if (K <= (uint32_t)GS_KMAX) {
        constexpr int RPT = GS_KMAX / GB;  // run entries per thread
        uint32_t rel[RPT], sr[RPT];
        bool ne[RPT];
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
            const uint32_t i = tid + (uint32_t)r * GB;
            ne[r] = false;
            rel[r] = sr[r] = 0;
            if (i < K) {
                const uint32_t a = tb.ls[e0 + i], b = tb.ls[e0 + i + 1];  // e0 + K <= 256 * ntp (sentinel)
                sr[r] = tb.sr[e0 + i] - a;  // delta (mod 2^32)
                ne[r] = b > a && a < L0 + nvalid;  // the bracket's last run may start at the next tile
                rel[r] = a > L0 ? a - L0 : 0u;
            }
        }
        if (tid < (uint32_t)(GT / 32)) g.bits[tid] = 0u;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RPT; ++r)
            if (ne[r]) atomicOr(&g.bits[rel[r] >> 5], 1u << (rel[r] & 31u));
        __syncthreads();
        const uint32_t pc = tid < (uint32_t)(GT / 32) ? (uint32_t)__popc(g.bits[tid]) : 0u;
        const uint32_t ex = block_excl_scan<GB, GT / 32>(pc, g.wsum);
        if (tid < (uint32_t)(GT / 32)) g.wpre[tid] = ex;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
            if (ne[r]) {
                const uint32_t w = rel[r] >> 5;
                g.delta[g.wpre[w] + (uint32_t)__popc(g.bits[w] & ((1u << (rel[r] & 31u)) - 1u))] = (int32_t)sr[r];
            }
        }
        __syncthreads();
        uint32_t addr[GK];
#pragma unroll
        for (int j = 0; j < GK; ++j) {
            const uint32_t p = pw + (uint32_t)j * WAVE;
            const uint32_t w = p >> 5, b = p & 31u;
            const uint32_t m = b == 31u ? 0xFFFFFFFFu : (2u << b) - 1u;
            const uint32_t idx = g.wpre[w] + (uint32_t)__popc(g.bits[w] & m) - 1u;
            addr[j] = L0 + p + (uint32_t)g.delta[idx < (uint32_t)GS_KMAX ? idx : 0u];
        }
        if (nvalid == (uint32_t)GT) {
#pragma unroll
            for (int j = 0; j < GK; ++j) k[j] = ld_stream<NT_GS>(src + addr[j]);
        } else {
#pragma unroll
            for (int j = 0; j < GK; ++j) k[j] = pw + (uint32_t)j * WAVE < nvalid ? ld_stream<NT_GS>(src + addr[j]) : sentinel;
        }
    } else {
        // many (mostly empty) runs: each lane searches the tables directly
#pragma unroll 1
        for (int j = 0; j < GK; ++j) {
            const uint32_t p = pw + (uint32_t)j * WAVE;
            if (p < nvalid) {
                const uint32_t P = L0 + p;
                uint32_t lo = e0, hi = e1 + 1;  // ls[lo] <= P < ls[hi]
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (tb.ls[mid] <= P) lo = mid;
                    else hi = mid;
                }
                k[j] = ld_stream<NT_GS>(src + tb.sr[lo] + (P - tb.ls[lo]));
            } else {
                k[j] = sentinel;
            }
        }
    }
}

// ---- fused small path ------------------------------------------------------------------
// Up to GS_SMALL_NG scan groups (2^20 keys, 128 tiles: fewer tiles than CUs) the passes
// are bound by launches, not bytes (r26: ten launches, 0.073-0.080 ms at 2^20).  There
// the scan is not launched at all: each workgroup of pass p derives the runs of its own
// tile from the previous pass's tile rows (L2-resident, 1 KB per tile), so a pass is one
// launch -- sweep 0, sweeps 1-3 and the gathered copy: five launches, no memset.  The
// rows of a buffer are kept beside it (rt for A, rt2 for B), since the pass that reads
// A's rows writes B's.
//
// LDS of the prologue (aliases the reorder buffer, as GsRuns): run-start bitmap, its
// popcount prefix, one delta per nonempty run overlapping the tile (at most GT).
struct GsRunsF {
    uint32_t bits[GT / 32];
    uint32_t wpre[GT / 32];
    int32_t delta[GT];
    uint32_t tot[256];  // digit totals of the logical order
    uint32_t wsum[8];
};

// Fused small path: each active pass q adds its tiles' digit counts into acc[q], spread
// over GS_FSLOTS copies (tile T into copy T % GS_FSLOTS: 8 atomics per address at 128
// tiles, where one copy serialised 128 and cost ~5 us a pass).
constexpr int GS_FSLOTS = 16;
// after the copies: per copy one 256-B line of pass 0's digit min / max atomics, words
// 0-3 = 255 - min of digit q, 4-7 = max (zero-initialised maxima)
constexpr size_t GS_FACC_WORDS = (size_t)4 * GS_FSLOTS * 256, GS_FWORDS = GS_FACC_WORDS + GS_FSLOTS * 64;
// Start of pass p >= 1 (p = 4: the final copy), one round trip and one barrier: the
// digit min / max of pass 0 (every thread gets them, in mm) and the digit totals of the
// logical order before p, for thread tid < 256's digit.  The totals are always read from
// acc[p - 1]: an active pass accumulates its own there, a skipped pass forwards the
// totals it received (gs_forward), so no pass has to know which earlier pass wrote them.
// part: 272 words of LDS.  Block-uniform.
__device__ __forceinline__ uint32_t gs_fused_prologue(const uint32_t *acc, int p, GsMM &mm, uint32_t *part,
                                                      uint32_t tid) {
    static_assert(GB == 512, "two threads per digit");
    const uint32_t d = tid & 255u, h = tid >> 8, lane = tid & 63u;
    const uint32_t *a = acc + ((size_t)(p - 1) * GS_FSLOTS + h * (GS_FSLOTS / 2)) * 256 + d;
    uint32_t v[GS_FSLOTS / 2], c = 0;
#pragma unroll
    for (int i = 0; i < GS_FSLOTS / 2; ++i) v[i] = ld_agent(a + i * 256);
    static_assert(GS_FSLOTS * 8 == 128, "min / max slots: waves 0 and 1");
    uint32_t m = tid < 128u ? ld_agent(acc + GS_FACC_WORDS + (tid >> 3) * 64u + (tid & 7u)) : 0u;
#pragma unroll
    for (int off = 8; off < 64; off <<= 1) {
        const uint32_t o = __shfl_xor(m, off);
        m = o > m ? o : m;
    }
    if (tid < 128u && lane < 8u) part[256u + (tid >> 6) * 8u + lane] = m;
#pragma unroll
    for (int i = 0; i < GS_FSLOTS / 2; ++i) c += v[i];
    if (h) part[d] = c;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t x = part[256 + q], y = part[264 + q], u = part[260 + q], w = part[268 + q];
        mm.dmin[q] = 255u - (x > y ? x : y);
        mm.dmax[q] = u > w ? u : w;
    }
    return h ? 0u : c + part[d];
}

// Pass 1 of the fused path (no memset runs): pass 0 accumulated nothing, so the
// digit min / max come from its per-tile pairs and the totals from its 128 tile rows
// (every workgroup sums them: 128 KB from L2), and workgroup 0 publishes the min / max
// in line 0 of the min / max lines for the passes after it.  part: 288 words.
__device__ __forceinline__ uint32_t gs_fused_prologue1(const uint32_t *rows, const uint32_t *mmp, uint32_t ntp,
                                                       uint32_t *acc, GsMM &mm, uint32_t *part, uint32_t tid) {
    const uint32_t d = tid & 255u, h = tid >> 8;
    uint32_t c = 0;
#pragma unroll 8
    for (uint32_t t = h; t < ntp; t += 2u) c += rows[(size_t)t * 256 + d] >> 16;
    GsMM *lmm = reinterpret_cast<GsMM *>(part + 256);
    gs_reduce_minmax<GB>(mmp, ntp, reinterpret_cast<uint32_t (*)[2]>(part + 264), lmm);
    if (h) part[d] = c;
    __syncthreads();
    mm = *lmm;
    if (blockIdx.x == 0 && tid < 4u) {
        acc[GS_FACC_WORDS + tid] = 255u - mm.dmin[tid];
        acc[GS_FACC_WORDS + 4u + tid] = mm.dmax[tid];
    }
    return h ? 0u : c + part[d];
}

// A skipped pass p: workgroup 0 forwards the totals it received to acc[p] (copy 0; the
// other copies stay zero), where pass p + 1 (or the final copy) reads them.
__device__ __forceinline__ void gs_forward(uint32_t *acc, int p, uint32_t tot, uint32_t tid) {
    if (blockIdx.x == 0 && tid < 256u) acc[(size_t)p * GS_FSLOTS * 256 + tid] = tot;
}

// Keys of logical tile T (positions L0 + wid*GK*64 + j*64 + lane) of the order that the
// pass which wrote `src` defines, from that pass's digit totals (tot: thread tid < 256's
// digit) and that buffer's tile rows (row t, digit d: local offset lo | count << 16).  In that order the runs (d, t) follow each other digit-major;
// the tile overlaps the runs of the digits [dlo, dhi] whose logical range meets it.
// Block-uniform (barriers).  Matches gs_gather on the tables k_gout would have written.
__device__ __forceinline__ void gs_gather_f(const uint32_t *__restrict__ src, const uint32_t *__restrict__ rows,
                                            uint32_t tot, uint32_t ntp, uint32_t n, uint32_t L0, uint32_t nvalid, uint32_t sentinel,
                                            GsRunsF &g, uint32_t (&k)[GK], uint32_t tid, uint32_t lane,
                                            uint32_t wid) {
    // the digit totals to LDS; every wave then scans them itself (4 digits per lane) for
    // the digits [dlo, dhi] whose logical range meets the tile and the logical start of
    // dlo: no block scan, no barrier
    if (tid < 256u) g.tot[tid] = tot;
    if (tid < (uint32_t)(GT / 32)) g.bits[tid] = 0u;
    __syncthreads();
    const uint32_t L1 = L0 + nvalid;
    uint32_t dlo = 1, dhi = 0, base0 = 0;
    {
        const uint4 t4 = *reinterpret_cast<const uint4 *>(&g.tot[4u * lane]);
        const uint32_t tv[4] = {t4.x, t4.y, t4.z, t4.w};
        const uint32_t sum = t4.x + t4.y + t4.z + t4.w;
        uint32_t x = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(x, off);
            if (lane >= (uint32_t)off) x += y;
        }
        uint32_t gd = x - sum, first = 4u, last = 0u, gfirst = 0u;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            if (tv[q] != 0u && gd < L1 && gd + tv[q] > L0) {
                if (first == 4u) {
                    first = q;
                    gfirst = gd;
                }
                last = q;
            }
            gd += tv[q];
        }
        const uint64_t b = __ballot(first != 4u);
        if (b) {
            const int fl = __builtin_ctzll(b), ll = 63 - __builtin_clzll(b);
            dlo = 4u * (uint32_t)fl + (uint32_t)__shfl((int)first, fl);
            dhi = 4u * (uint32_t)ll + (uint32_t)__shfl((int)last, ll);
            base0 = (uint32_t)__shfl((int)gfirst, fl);
        }
    }
    const uint32_t E = dhi >= dlo ? (dhi - dlo + 1u) * ntp : 0u;  // runs (d, t), digit-major
    constexpr uint32_t CW = 8;  // runs per lane of the one-wave path
    if (E <= WAVE * CW) {  // block-uniform: the usual case (a tile meets ~3 digits), wave 0 alone
        if (wid == 0) {
            uint32_t w[CW], sr[CW], s = 0;
#pragma unroll
            for (uint32_t j = 0; j < CW; ++j) {
                const uint32_t e = lane * CW + j;
                w[j] = 0u;
                sr[j] = 0u;
                if (e < E) {
                    const uint32_t dd = dlo + e / ntp, t = e % ntp;
                    w[j] = rows[(size_t)t * 256 + dd];
                    sr[j] = t * (uint32_t)GT + (w[j] & 0xFFFFu);
                }
                s += w[j] >> 16;
            }
            uint32_t x = s;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(x, off);
                if (lane >= (uint32_t)off) x += y;
            }
            const uint32_t ls0 = base0 + x - s;
            uint32_t ls = ls0;
#pragma unroll
            for (uint32_t j = 0; j < CW; ++j) {
                const uint32_t cnt = w[j] >> 16;
                if (cnt != 0u && ls < L1 && ls + cnt > L0) {
                    const uint32_t rel = ls > L0 ? ls - L0 : 0u;
                    atomicOr(&g.bits[rel >> 5], 1u << (rel & 31u));
                }
                ls += cnt;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            // popcount prefix of the 256 bitmap words, 4 per lane
            const uint4 b4 = *reinterpret_cast<const uint4 *>(&g.bits[4u * lane]);
            const uint32_t p0 = (uint32_t)__popc(b4.x), p1 = (uint32_t)__popc(b4.y), p2 = (uint32_t)__popc(b4.z),
                           p3 = (uint32_t)__popc(b4.w), ps = p0 + p1 + p2 + p3;
            uint32_t y = ps;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t z = __shfl_up(y, off);
                if (lane >= (uint32_t)off) y += z;
            }
            const uint32_t e0 = y - ps;
            *reinterpret_cast<uint4 *>(&g.wpre[4u * lane]) = make_uint4(e0, e0 + p0, e0 + p0 + p1, e0 + p0 + p1 + p2);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            ls = ls0;
#pragma unroll
            for (uint32_t j = 0; j < CW; ++j) {
                const uint32_t cnt = w[j] >> 16;
                if (cnt != 0u && ls < L1 && ls + cnt > L0) {
                    const uint32_t rel = ls > L0 ? ls - L0 : 0u, wd = rel >> 5, bb = rel & 31u;
                    g.delta[g.wpre[wd] + (uint32_t)__popc(g.bits[wd] & ((1u << bb) - 1u))] = (int32_t)(sr[j] - ls);
                }
                ls += cnt;
            }
        }
        __syncthreads();
    } else {
    constexpr uint32_t C = 4, CH = GB * C;
    // two sweeps over the runs: (0) mark the start of every nonempty run inside the tile,
    // (1) store its delta (source address - logical position) at its rank among them.
    // One chunk (the usual case: a tile meets ~3 digits): sweep 1 reuses sweep 0's loads.
    const bool one = E <= CH;
    uint32_t w[C], sr[C], ex1 = 0;
#pragma unroll 1
    for (int sweep = 0; sweep < 2; ++sweep) {
        if (sweep == 1) {
            const uint32_t pc = tid < (uint32_t)(GT / 32) ? (uint32_t)__popc(g.bits[tid]) : 0u;
            const uint32_t ex = block_excl_scan<GB, GT / 32>(pc, g.wsum);
            if (tid < (uint32_t)(GT / 32)) g.wpre[tid] = ex;
            __syncthreads();
        }
        uint32_t base = base0;
#pragma unroll 1
        for (uint32_t c0 = 0; c0 < E; c0 += CH) {
            uint32_t ex = ex1, chunk = 0;
            if (!(one && sweep == 1)) {  // block-uniform
                uint32_t s = 0;
#pragma unroll
                for (uint32_t j = 0; j < C; ++j) {
                    const uint32_t e = c0 + tid * C + j;
                    w[j] = 0u;
                    sr[j] = 0u;
                    if (e < E) {
                        const uint32_t dd = dlo + e / ntp, t = e % ntp;
                        w[j] = rows[(size_t)t * 256 + dd];
                        sr[j] = t * (uint32_t)GT + (w[j] & 0xFFFFu);
                    }
                    s += w[j] >> 16;
                }
                ex = ex1 = block_excl_scan<GB, GB>(s, g.wsum);
#pragma unroll
                for (int q = 0; q < GB / 64; ++q) chunk += g.wsum[q];
            }
            uint32_t ls = base + ex;
#pragma unroll
            for (uint32_t j = 0; j < C; ++j) {
                const uint32_t cnt = w[j] >> 16;
                if (cnt != 0u && ls < L1 && ls + cnt > L0) {
                    const uint32_t rel = ls > L0 ? ls - L0 : 0u, wd = rel >> 5, b = rel & 31u;
                    if (sweep == 0) atomicOr(&g.bits[wd], 1u << b);
                    else g.delta[g.wpre[wd] + (uint32_t)__popc(g.bits[wd] & ((1u << b) - 1u))] = (int32_t)(sr[j] - ls);
                }
                ls += cnt;
            }
            base += chunk;
            __syncthreads();  // g.wsum reused by the next chunk's scan
        }
    }
    }  // (many runs: the whole block, in chunks)
    const uint32_t pw = wid * (GK * WAVE) + lane;
    uint32_t addr[GK];
#pragma unroll
    for (int j = 0; j < GK; ++j) {
        const uint32_t p = pw + (uint32_t)j * WAVE;
        const uint32_t w = (p >> 5) & (uint32_t)(GT / 32 - 1), b = p & 31u;
        const uint32_t m = b == 31u ? 0xFFFFFFFFu : (2u << b) - 1u;
        const uint32_t idx = g.wpre[w] + (uint32_t)__popc(g.bits[w] & m) - 1u;
        const uint32_t a = L0 + p + (uint32_t)g.delta[idx < (uint32_t)GT ? idx : 0u];
        addr[j] = a < n ? a : n - 1u;  // (never past the buffer, whatever the rows say)
    }
    if (nvalid == (uint32_t)GT) {
#pragma unroll
        for (int j = 0; j < GK; ++j) k[j] = ld_stream<NT_GS>(src + addr[j]);
    } else {
#pragma unroll
        for (int j = 0; j < GK; ++j) k[j] = pw + (uint32_t)j * WAVE < nvalid ? ld_stream<NT_GS>(src + addr[j]) : sentinel;
    }
}

// LDS word of tile slot i in the reorder buffer: 4 pad words per 32 slots (16-B
// aligned, for the uint4 write-out).  In a sorted tile every digit holds 32 keys, so a
// wave's reorder stores land 32 slots apart: one bank unpadded, 8 banks padded.
__device__ __forceinline__ uint32_t gs_pad(uint32_t i) { return i + ((i >> 5) << 2); }

struct GsSmem {
    union {  // the run tables are only read while the tile is gathered, before the reorder
        uint32_t keys[GT + GT / 8];
        GsRuns g;
        GsRunsF f;  // fused small path
    };
    uint32_t fpart[288];  // fused small path: the prologues' scratch
    uint32_t wh[GW * 256];
    uint32_t probe[WAVE];
    uint32_t wsum[8];
    uint32_t mm[GW][8];
    uint32_t ordered;
};

// One pass: gather (or, for the input, load) tile T, sort it by digit `pass` in LDS,
// write it contiguously to the other buffer, record its digit counts and offsets.
// FUSED (small path): no scan launches; rt holds A's tile rows and rt2 B's, the tile's
// runs come from gs_gather_f, the skip test from the tiles' digit min / max pairs.
template <bool FUSED>
__global__ __launch_bounds__(GB, GS_WAVES_PER_EU) void k_gsweep(const uint32_t *__restrict__ in, uint32_t *bufA, uint32_t *bufB,
                                                  GsTables tA, GsTables tB, uint32_t *__restrict__ rt,
                                                  uint32_t *__restrict__ rt2, uint32_t *__restrict__ mm, GsState *st,
                                                  uint32_t *__restrict__ acc, int pass, uint32_t n, uint32_t ntp,
                                                  uint32_t flip, int nozero) {
    if (!FUSED && !gs_active(st, pass)) return;
    const uint32_t T = gs_tile(blockIdx.x, ntp);
    if (T >= ntp) return;
    __shared__ GsSmem sm;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    uint32_t ftot = 0;  // fused: this thread's digit total of the previous active pass
    GsMM fmm;           // fused: digit min / max (pass > 0)
    if (FUSED && pass > 0) {
        ftot = (nozero && pass == 1) ? gs_fused_prologue1(rt, mm, ntp, acc, fmm, sm.fpart, tid)
                                     : gs_fused_prologue(acc, pass, fmm, sm.fpart, tid);
        if (!gs_active(&fmm, pass)) {  // block-uniform
            gs_forward(acc, pass, ftot, tid);
            return;
        }
    }
    const uint32_t cur = FUSED ? gs_cur(&fmm, pass) : gs_cur(st, pass);
    if (FUSED && nozero && pass == 0 && T == 0) {  // what the memset would have cleared
        if (tid == 0) st->err = 0u;
        uint4 *z = reinterpret_cast<uint4 *>(acc + (size_t)GS_FSLOTS * 256);  // acc[1..3], min / max lines
        for (uint32_t i = tid; i < (uint32_t)((GS_FWORDS - GS_FSLOTS * 256) / 4); i += GB) z[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    const uint32_t *src = cur == 0 ? in : cur == 1 ? bufA : bufB;
    uint32_t *dst = cur == 1 ? bufB : bufA;
    const uint32_t L0 = T * (uint32_t)GT;
    const uint32_t nvalid = (n - L0) < (uint32_t)GT ? (n - L0) : (uint32_t)GT;
    const uint32_t sentinel = ~flip;  // digit 255 in every pass: ranks after all real keys
    const uint32_t shift = (uint32_t)pass * 8u;

    for (uint32_t i = tid; i < (uint32_t)(GW * 256); i += GB) sm.wh[i] = 0u;
    if (wid == 0) {
        const bool ord = lds_lane_ordered(sm.probe, lane);
        if (lane == 0) sm.ordered = ord ? 1u : 0u;
    }
    uint32_t k[GK];
    if (cur == 0) {
        const uint32_t *s = src + L0 + wid * (GK * WAVE) + lane;
        const uint32_t woff = wid * (GK * WAVE) + lane;
        if (nvalid == (uint32_t)GT) {
#pragma unroll
            for (int j = 0; j < GK; ++j) k[j] = s[j * WAVE];
        } else {
#pragma unroll
            for (int j = 0; j < GK; ++j) k[j] = woff + j * WAVE < nvalid ? s[j * WAVE] : sentinel;
        }
        __syncthreads();
    } else {
        if constexpr (FUSED) gs_gather_f(src, cur == 1 ? rt : rt2, ftot, ntp, n, L0, nvalid, sentinel, sm.f, k, tid, lane, wid);
        else gs_gather(src, cur == 1 ? tA : tB, T, L0, nvalid, sentinel, sm.g, k, tid, lane, wid);
        __syncthreads();
    }
    const bool atomic_rank = __builtin_amdgcn_readfirstlane(sm.ordered) != 0u;

    // stable wave rank (slot-major order = position order), two 16-bit ranks per register
    uint32_t *wh = sm.wh + wid * 256;
    uint32_t rk[GK / 2];
#pragma unroll
    for (int j = 0; j < GK; ++j) {
        const uint32_t d = ((k[j] ^ flip) >> shift) & 255u;
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
        rk[j / 2] = (j & 1) ? rk[j / 2] | (r << 16) : r;
    }
    // pass 0: digit min / max over the valid keys (for the later passes' skip test)
    if (pass == 0) {
        uint32_t mn = 0xFFFFFFFFu, mx = 0u;  // bytes: digits 0..3 of (key ^ flip)
        uint32_t mnb[4] = {255u, 255u, 255u, 255u}, mxb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < GK; ++j) {
            if (wid * (GK * WAVE) + j * WAVE + lane < nvalid) {
                const uint32_t v = k[j] ^ flip;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t b = (v >> (8 * q)) & 255u;
                    mnb[q] = b < mnb[q] ? b : mnb[q];
                    mxb[q] = b > mxb[q] ? b : mxb[q];
                }
            }
        }
        mn = mnb[0] | (mnb[1] << 8) | (mnb[2] << 16) | (mnb[3] << 24);
        mx = mxb[0] | (mxb[1] << 8) | (mxb[2] << 16) | (mxb[3] << 24);
        // per-byte min / max across the wave
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint32_t omn = __shfl_xor(mn, off), omx = __shfl_xor(mx, off);
            uint32_t a = 0, b = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t x = (mn >> (8 * q)) & 255u, y = (omn >> (8 * q)) & 255u;
                const uint32_t u = (mx >> (8 * q)) & 255u, w = (omx >> (8 * q)) & 255u;
                a |= (x < y ? x : y) << (8 * q);
                b |= (u > w ? u : w) << (8 * q);
            }
            mn = a;
            mx = b;
        }
        if (lane == 0) {
            sm.mm[wid][0] = mn;
            sm.mm[wid][1] = mx;
        }
    }
    __syncthreads();  // (1) wave counts

    // tile histogram, local digit offsets, per-wave offsets
    uint32_t tot = 0;
    if (tid < 256u) {
#pragma unroll
        for (int w = 0; w < GW; ++w) tot += sm.wh[w * 256 + tid];
    }
    const uint32_t ds = block_excl_scan<GB, 256>(tot, sm.wsum);
    if (tid < 256u) {
        uint32_t run = ds;
#pragma unroll
        for (int w = 0; w < GW; ++w) {
            const uint32_t c = sm.wh[w * 256 + tid];
            sm.wh[w * 256 + tid] = run;
            run += c;
        }
        const uint32_t cnt = tid == 255u ? tot - ((uint32_t)GT - nvalid) : tot;  // drop sentinels
        (FUSED && dst == bufB ? rt2 : rt)[(size_t)T * 256 + tid] = ds | (cnt << 16);
        if (FUSED && cnt && !(nozero && pass == 0))
            atomicAdd(acc + ((size_t)pass * GS_FSLOTS + T % GS_FSLOTS) * 256 + tid, cnt);  // next pass's totals
    }
    if (pass == 0 && tid == 0) {
        uint32_t mn = sm.mm[0][0], mx = sm.mm[0][1];
        for (int w = 1; w < GW; ++w) {
            uint32_t a = 0, b = 0;
            for (int q = 0; q < 4; ++q) {
                const uint32_t x = (mn >> (8 * q)) & 255u, y = (sm.mm[w][0] >> (8 * q)) & 255u;
                const uint32_t u = (mx >> (8 * q)) & 255u, v = (sm.mm[w][1] >> (8 * q)) & 255u;
                a |= (x < y ? x : y) << (8 * q);
                b |= (u > v ? u : v) << (8 * q);
            }
            mn = a;
            mx = b;
        }
        mm[2 * T] = mn;
        mm[2 * T + 1] = mx;
        if (FUSED && !nozero) {
            uint32_t *f = acc + GS_FACC_WORDS + (T % GS_FSLOTS) * 64u;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                atomicMax(f + q, 255u - ((mn >> (8 * q)) & 255u));
                atomicMax(f + 4 + q, (mx >> (8 * q)) & 255u);
            }
        }
    }
    __syncthreads();  // (2) wave offsets

    // reorder into LDS, then write the tile contiguously (whole lines)
#pragma unroll
    for (int j = 0; j < GK; ++j) {
        const uint32_t d = ((k[j] ^ flip) >> shift) & 255u;
        sm.keys[gs_pad(wh[d] + ((rk[j / 2] >> ((j & 1) * 16)) & 0xFFFFu))] = k[j];
    }
    __syncthreads();  // (3) tile sorted in LDS
    if (nvalid == (uint32_t)GT) {
        const uint4 *s4 = reinterpret_cast<const uint4 *>(sm.keys);
        uint4 *d4 = reinterpret_cast<uint4 *>(dst + L0);
#pragma unroll
        for (int j = 0; j < GK / 4; ++j) {
            const uint32_t q = (uint32_t)j * GB + tid;  // uint4 q = slots 4q..4q+3, one 32-slot row
            d4[q] = s4[q + (q >> 3)];
        }
    } else {
#pragma unroll
        for (int j = 0; j < GK; ++j) {
            const uint32_t i = (uint32_t)j * GB + tid;
            if (i < nvalid) dst[L0 + i] = sm.keys[gs_pad(i)];
        }
    }
}

// k_gsum: column sums of GS_GROUP consecutive tiles' counts, and their exclusive prefix
// over the groups by decoupled look-back (groups taken in order from a counter, so a
// group only waits on groups already running; every wait bounded: an expired spin sets
// the error word that labsort_workspace_status reports).  The last group writes the
// digit totals.  After pass 0 it also reduces its tiles' digit min / max.
__global__ __launch_bounds__(256) void k_gsum(const uint32_t *__restrict__ rt, const uint32_t *__restrict__ mm,
                                              uint32_t *__restrict__ gsx, uint32_t *__restrict__ tot,
                                              uint32_t *__restrict__ gmm, uint32_t *flags, GsState *st, int pass,
                                              uint32_t ntp, uint32_t ngroups) {
    if (!gs_active(st, pass)) return;
    __shared__ uint32_t gid;
    const uint32_t d = threadIdx.x;
    if (d == 0) gid = atomicAdd(&st->gctr[pass], 1u);
    __syncthreads();
    const uint32_t g = gid;
    const uint32_t t0 = g * GS_GROUP, t1 = t0 + GS_GROUP < ntp ? t0 + GS_GROUP : ntp;
    uint32_t h = 0;
#pragma unroll 8
    for (uint32_t t = t0; t < t1; ++t) h += rt[(size_t)t * 256 + d] >> 16;
    uint32_t *fl = flags + (size_t)pass * ngroups * 256;
    st_agent(fl + (size_t)g * 256 + d, (g == 0 ? LB_INC : LB_AGG) | h);
    uint32_t excl = 0;
    if (g > 0) {
        uint32_t t = g - 1, spins = 0;
        for (;;) {
            const uint32_t w = ld_agent(fl + (size_t)t * 256 + d);
            if ((w & ~LB_VAL) == 0u) {
                if (++spins > GS_SPIN_LIMIT) {
                    atomicOr(&st->err, 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            excl += w & LB_VAL;
            if (w & LB_INC) break;
            --t;
        }
        st_agent(fl + (size_t)g * 256 + d, LB_INC | (excl + h));
    }
    gsx[(size_t)g * 256 + d] = excl;
    if (g + 1 == ngroups) tot[d] = excl + h;
    if (pass == 0 && d < 64u) {  // the group's tiles' digit min / max, one tile per lane
        static_assert(GS_GROUP == WAVE, "one tile per lane of wave 0");
        uint32_t mn = 0xFFFFFFFFu, mx = 0u;
        if (t0 + d < t1) {
            mn = mm[2 * (t0 + d)];
            mx = mm[2 * (t0 + d) + 1];
        }
        wave_minmax4(mn, mx);
        if (d == 0) {
            gmm[2 * g] = mn;
            gmm[2 * g + 1] = mx;
        }
    }
}

// k_gout: the tables of this pass's output buffer, GS_GROUP tiles per workgroup (4
// threads per digit, 16 tiles each); digit-major writes go through LDS so each is a line
// segment.  Workgroup 0 writes the sentinel and, after pass 0, the digit min / max.
__global__ __launch_bounds__(1024) void k_gout(const uint32_t *__restrict__ rt, const uint32_t *__restrict__ gsx,
                                               const uint32_t *__restrict__ tot, const uint32_t *__restrict__ gmm,
                                               GsTables tA, GsTables tB, GsState *st, int pass, uint32_t ntp,
                                               uint32_t n) {
    if (!gs_active(st, pass)) return;
    constexpr int G = GS_GROUP, TPQ = G / 4;
    __shared__ uint32_t lsb[G][257], srb[G][257];
    __shared__ uint32_t part[4][256];
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t red[16][2];
    const GsTables tb = gs_dst(st, pass) == 1u ? tA : tB;
    const uint32_t g = blockIdx.x, tid = threadIdx.x, d = tid & 255u, q = tid >> 8;
    const uint32_t t0 = g * G + q * TPQ;
    uint32_t w[TPQ], h = 0;
#pragma unroll
    for (int i = 0; i < TPQ; ++i) {
        w[i] = t0 + i < ntp ? rt[(size_t)(t0 + i) * 256 + d] : 0u;
        h += w[i] >> 16;
    }
    part[q][d] = h;
    const uint32_t total = tot[d], before = gsx[(size_t)g * 256 + d];
    if (g == 0) {
        if (tid == 0) tb.ls[(size_t)256 * ntp] = n;  // sentinel start after the last run
        if (pass == 0)  // per scan group: packed digit min / max pairs
            gs_reduce_minmax<1024>(gmm, (ntp + GS_GROUP - 1) / GS_GROUP, red, st);
    }
    // global exclusive digit offsets from the digit totals
    const uint32_t gx = block_excl_scan<1024, 256>(q == 0 ? total : 0u, wsum);
    __shared__ uint32_t gxs[256];
    if (q == 0) gxs[d] = gx;
    __syncthreads();
    uint32_t run = gxs[d] + before;
    for (uint32_t r = 0; r < q; ++r) run += part[r][d];
#pragma unroll
    for (int i = 0; i < TPQ; ++i) {
        const uint32_t t = t0 + i;
        const uint32_t hh = w[i] >> 16, ls = run;
        run += hh;
        lsb[q * TPQ + i][d] = ls;
        srb[q * TPQ + i][d] = t * (uint32_t)GT + (w[i] & 0xFFFFu);
        if (hh && t < ntp) {
            const uint32_t e = d * ntp + t;
            for (uint32_t T = (ls + GT - 1) / GT; T < ntp && (uint64_t)T * GT < (uint64_t)ls + hh; ++T) tb.first[T] = e;
            if (ls <= n - 1 && n - 1 < ls + hh) tb.first[ntp] = e;
        }
    }
    __syncthreads();
    // digit-major writes: G consecutive tiles of one digit per lane group
    constexpr uint32_t LPD = (uint32_t)G, DPW = WAVE / LPD;  // lanes per digit, digits per wave pass
    const uint32_t lane = tid & 63u, wv = tid >> 6;
    const uint32_t ti = lane % LPD, tg = g * G + ti;
    if (tg < ntp) {
        for (uint32_t dd = wv * DPW + lane / LPD; dd < 256u; dd += 16u * DPW) {
            tb.ls[(size_t)dd * ntp + tg] = lsb[ti][dd];
            tb.sr[(size_t)dd * ntp + tg] = srb[ti][dd];
        }
    }
}

// Final pass: the logical order after the last pass, gathered and written to `out`.
template <bool FUSED>
__global__ __launch_bounds__(GB, GS_WAVES_PER_EU) void k_gcopy(const uint32_t *__restrict__ bufA, const uint32_t *__restrict__ bufB,
                                                 GsTables tA, GsTables tB, const uint32_t *__restrict__ rt,
                                                 const uint32_t *__restrict__ rt2, const GsState *st,
                                                 const uint32_t *__restrict__ acc, uint32_t *__restrict__ out, uint32_t n,
                                                 uint32_t ntp) {
    const uint32_t T = gs_tile(blockIdx.x, ntp);
    if (T >= ntp) return;
    __shared__ union {
        GsRuns g;
        GsRunsF f;
    } u;
    __shared__ uint32_t fpart[272];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    uint32_t ftot = 0;
    GsMM fmm;
    if constexpr (FUSED) ftot = gs_fused_prologue(acc, 4, fmm, fpart, tid);
    const uint32_t cur = FUSED ? gs_cur(&fmm, 4) : gs_cur(st, 4);
    const uint32_t L0 = T * (uint32_t)GT;
    const uint32_t nvalid = (n - L0) < (uint32_t)GT ? (n - L0) : (uint32_t)GT;
    uint32_t k[GK];
    if constexpr (FUSED) gs_gather_f(cur == 1 ? bufA : bufB, cur == 1 ? rt : rt2, ftot, ntp, n, L0, nvalid, 0u, u.f, k, tid, lane, wid);
    else gs_gather(cur == 1 ? bufA : bufB, cur == 1 ? tA : tB, T, L0, nvalid, 0u, u.g, k, tid, lane, wid);
    uint32_t *o = out + L0 + wid * (GK * WAVE) + lane;
    const uint32_t woff = wid * (GK * WAVE) + lane;
#pragma unroll
    for (int j = 0; j < GK; ++j)
        if (woff + j * WAVE < nvalid) o[j * WAVE] = k[j];
}

inline size_t al(size_t x) { return (x + 65535) / 65536 * 65536; }

}  // namespace

// ---- host side -------------------------------------------------------------------------
GsLayout gs_layout(size_t n) {
    GsLayout L{};
    const size_t ntp = (n + GT - 1) / GT, ng = (ntp + GS_GROUP - 1) / GS_GROUP, ne = 256 * ntp;
    size_t o = 0;
    // state, then the scan look-back flags of the 4 passes, or (fused small path) the 4 x
    // GS_FSLOTS copies of the digit totals: zeroed together
    L.off_state = o;
    o = al(o + 512 + std::max<size_t>(4 * ng * 256 * 4, ng <= (size_t)GS_SMALL_NG ? GS_FWORDS * 4 : 0));
    L.off_a = o;
    o = al(o + n * 4);
    L.off_b = o;
    o = al(o + n * 4);
    L.off_rt = o;
    o = al(o + ne * 4);
    L.off_rt2 = o;  // B's tile rows (fused small path only)
    if (ng <= (size_t)GS_SMALL_NG) o = al(o + ne * 4);
    L.off_mm = o;
    o = al(o + ntp * 8);
    L.off_gsx = o;
    o = al(o + ng * 256 * 4);
    L.off_gx = o;
    o = al(o + 257 * 4);
    L.off_gmm = o;
    o = al(o + ng * 2 * 4);
    for (int s = 0; s < 2; ++s) {
        L.off_ls[s] = o;
        o = al(o + (ne + 1) * 4);
        L.off_sr[s] = o;
        o = al(o + ne * 4);
        L.off_first[s] = o;
        o = al(o + (ntp + 1) * 4);
    }
    L.total = o;
    return L;
}

hipError_t launch_gsweep_sort(const uint32_t *in, uint32_t *out, size_t n, uint32_t flip, char *ws, hipStream_t s,
                              const GsHooks &hooks) {
    const GsLayout L = gs_layout(n);
    const uint32_t ntp = (uint32_t)((n + GT - 1) / GT), ng = (ntp + GS_GROUP - 1) / GS_GROUP;
    GsState *st = reinterpret_cast<GsState *>(ws + L.off_state);
    uint32_t *A = reinterpret_cast<uint32_t *>(ws + L.off_a), *B = reinterpret_cast<uint32_t *>(ws + L.off_b);
    uint32_t *rt = reinterpret_cast<uint32_t *>(ws + L.off_rt), *mm = reinterpret_cast<uint32_t *>(ws + L.off_mm);
    uint32_t *gsx = reinterpret_cast<uint32_t *>(ws + L.off_gsx);
    uint32_t *gx = reinterpret_cast<uint32_t *>(ws + L.off_gx), *gmm = reinterpret_cast<uint32_t *>(ws + L.off_gmm);
    GsTables t[2];
    for (int i = 0; i < 2; ++i)
        t[i] = GsTables{reinterpret_cast<uint32_t *>(ws + L.off_ls[i]), reinterpret_cast<uint32_t *>(ws + L.off_sr[i]),
                        reinterpret_cast<uint32_t *>(ws + L.off_first[i])};
    uint32_t *flags = reinterpret_cast<uint32_t *>(ws + L.off_state + 512);
    uint32_t *rt2 = reinterpret_cast<uint32_t *>(ws + L.off_rt2);
    const unsigned grid = 8u * ((ntp + 7u) / 8u);
    hipError_t e;
    if (ng <= (uint32_t)GS_SMALL_NG) {  // fused small path: sweeps 0-3 and the gathered copy, no memset
        uint32_t *acc = flags;
        for (int p = 0; p < 4; ++p) {
            if (hooks.begin) hooks.begin(hooks.ctx, LABSORT_K_GSWEEP, s);
            k_gsweep<true><<<grid, GB, 0, s>>>(in, A, B, t[0], t[1], rt, rt2, mm, st, acc, p, (uint32_t)n, ntp, flip, 1);
            if (hooks.end) hooks.end(hooks.ctx, LABSORT_K_GSWEEP, s);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        if (hooks.begin) hooks.begin(hooks.ctx, LABSORT_K_GCOPY, s);
        k_gcopy<true><<<grid, GB, 0, s>>>(A, B, t[0], t[1], rt, rt2, st, acc, out, (uint32_t)n, ntp);
        if (hooks.end) hooks.end(hooks.ctx, LABSORT_K_GCOPY, s);
        return hipGetLastError();
    }
    e = launch_zero(ws + L.off_state, 512 + (size_t)4 * ng * 256 * 4, s);
    if (e != hipSuccess) return e;
    for (int p = 0; p < 4; ++p) {
        if (hooks.begin) hooks.begin(hooks.ctx, LABSORT_K_GSWEEP, s);
        k_gsweep<false><<<grid, GB, 0, s>>>(in, A, B, t[0], t[1], rt, rt2, mm, st, flags, p, (uint32_t)n, ntp, flip, 0);
        if (hooks.end) hooks.end(hooks.ctx, LABSORT_K_GSWEEP, s);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        k_gsum<<<ng, 256, 0, s>>>(rt, mm, gsx, gx, gmm, flags, st, p, ntp, ng);
        k_gout<<<ng, 1024, 0, s>>>(rt, gsx, gx, gmm, t[0], t[1], st, p, ntp, (uint32_t)n);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (hooks.begin) hooks.begin(hooks.ctx, LABSORT_K_GCOPY, s);
    k_gcopy<false><<<grid, GB, 0, s>>>(A, B, t[0], t[1], rt, rt2, st, flags, out, (uint32_t)n, ntp);
    if (hooks.end) hooks.end(hooks.ctx, LABSORT_K_GCOPY, s);
    return hipGetLastError();
}

}  // namespace labsort
