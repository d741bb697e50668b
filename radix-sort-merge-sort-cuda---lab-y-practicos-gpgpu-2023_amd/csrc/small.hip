// small.hip -- LSD radix sort in ONE launch for TS_TILE < n <= SR_MAX_N (config 2's 2^20).
//
// Below a few million keys the multi-launch radix paths are bound by launch count, not
// bytes: at 2^20 the gathered passes spend 4 x (k_gsweep 9.3 us + k_gout 7.3 us) +
// k_gcopy 6.1 us = 72 us on 4 MB of keys that live in the Infinity Cache
// (profiles/r25_kernel_stats.csv).  Here one cooperative launch of G = ceil(n / 16384)
// workgroups (one 16384-key tile each, G <= 256, all co-resident) runs every pass, with
// grid barriers between the phases that need all tiles:
//
//   load tile t, AND/OR of its keys -> andor[t]            | barrier: every WG knows
//                                                          |   which digits vary
//   per active pass (digit p):                             |
//     (load tile t of the pass input)                      |
//     stable wave rank of digit p (lane-ordered LDS         |
//       atomics, as k_onesweep_p), tile histogram -> cnt[t]|
//     per-wave offsets in LDS                              | barrier: all histograms
//     read the G rows of cnt: digit totals (-> digit        |
//       bases by a scan) and the rows of tiles < t          |
//     reorder the tile in LDS, scatter it                  | barrier (unless last)
//
// That is the split of lab.cu:47-87 generalised to 8-bit digits (the digit bases are
// the reference's "totalFalses" scan, the rows of earlier tiles its exclusive scan),
// with the reference's "stop when sorted" (lab.cu:61) as the skip of digits that are
// the same for every key.  The cnt matrix is read whole by every workgroup (G x 1 KB),
// which at G <= 256 costs less than another barrier.
//
// Grid barrier: one 64-bit word, [63:20] a launch tag the host makes unique per launch,
// [19:0] the arrivals.  Each workgroup first swaps a stale tag for its own (count 0), so
// the workspace needs no clearing launch; the last workgroup to leave resets the count,
// so a graph replay of the same launch finds it at 0.  Arrival = release (L2 writeback
// of the scatter), the spin = acquire loads; every spin is bounded (the error word).
#include <unistd.h>

#include <atomic>
#include <chrono>

#include "../../include/labsort.h"
#include "common.h"
#include "devutil.h"

namespace labsort {

namespace {

constexpr int SB = SR_BLOCK, SK = SR_KPT, ST = SR_TILE, SW = SR_BLOCK / WAVE, SRR = 256;
constexpr uint32_t SR_SPIN_LIMIT = 1u << 22;
constexpr unsigned long long SR_CNT_MASK = (1ull << 20) - 1ull;
// LABSORT_SR_SC1: the key loads and scatter stores are agent-coherent themselves (sc1:
// the cache policy bit 4 of the buffer ops), so the barriers need no L2 writeback /
// invalidate; else plain ops and release / acquire barriers.  LABSORT_SR_COOP: launch
// with hipLaunchCooperativeKernel (co-residency checked by the runtime), else <<<>>>.
#ifndef LABSORT_SR_SC1
#define LABSORT_SR_SC1 1  // r26: 2^20 0.094 ms (sc1) vs 0.102 (fences), 2^22 0.183 vs 0.226
#endif
#ifndef LABSORT_SR_COOP
#define LABSORT_SR_COOP 1  // <<<>>> is 13-16 us faster but can deadlock beside concurrent kernels
#endif
constexpr int SR_CPOL = LABSORT_SR_SC1 ? 16 : 0;

__device__ __forceinline__ uint32_t sr_pad(uint32_t i) { return i + (i >> 5); }  // as osp_pad

// buffer descriptor over n keys (32-bit lane offsets; out-of-range loads read 0 and
// out-of-range stores are dropped), as k_onesweep_p's
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sr_rsrc(const uint32_t *p, uint32_t n) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0, (int)(n * 4u), 0x00020000);
}

struct SrSmem {
    uint32_t keys[ST + ST / 32];
    uint32_t wh[SW * SRR];
    uint32_t red[4 * SRR];
    uint32_t delta[SRR];
    uint32_t wsum[SW];
    uint32_t probe[WAVE];
    uint32_t misc[4];
};

// grid barrier number `idx` (0-based): every workgroup arrives once per barrier
__device__ __forceinline__ bool sr_sync(unsigned long long *bar, uint32_t target, uint32_t *err) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's stores have reached the L2
    __syncthreads();
    __shared__ uint32_t ok_s;
    if (threadIdx.x == 0) {
        uint32_t ok = 1u, spins = 0;
        __hip_atomic_fetch_add(bar, 1ull, LABSORT_SR_SC1 ? __ATOMIC_RELAXED : __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        while ((uint32_t)(__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & SR_CNT_MASK) < target) {
            if (++spins > SR_SPIN_LIMIT) {
                atomicOr(err, 1u);
                ok = 0u;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (!LABSORT_SR_SC1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (one L2 invalidate, after the spin)
        ok_s = ok;
    }
    __syncthreads();
    return ok_s != 0u;
}

__global__ __launch_bounds__(SB) void k_small_radix(const uint32_t *__restrict__ in, uint32_t *out, uint32_t *tmp,
                                                     uint32_t n, uint32_t flip, uint32_t *err,
                                                     unsigned long long *bar, uint32_t *andor, uint32_t *cnt,
                                                     unsigned long long tag) {
    __shared__ SrSmem sm;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t G = gridDim.x, t = blockIdx.x;
    const uint32_t base = t * (uint32_t)ST;
    const uint32_t nvalid = n - base < (uint32_t)ST ? n - base : (uint32_t)ST;
    const uint32_t woff = wid * (SK * WAVE) + lane;  // wave-blocked load layout (as k_onesweep_p)
    const uint32_t sentinel = ~flip;

    if (tid == 0) {
        if (t == 0) st_agent(err, 0u);
        // adopt this launch's tag (count 0) unless another workgroup already has
        unsigned long long old = __hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while ((old >> 20) != tag) {
            if (__hip_atomic_compare_exchange_strong(bar, &old, tag << 20, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT))
                break;
        }
    }
    if (wid == 0) {
        const bool ord = lds_lane_ordered(sm.probe, lane);
        if (lane == 0) sm.misc[0] = ord ? 1u : 0u;
    }
    const __amdgpu_buffer_rsrc_t rin = sr_rsrc(in, n), rout = sr_rsrc(out, n), rtmp = sr_rsrc(tmp, n);
    uint32_t k[SK];
    uint32_t a = ~0u, o = 0u;
#pragma unroll
    for (int j = 0; j < SK; ++j) {
        const uint32_t i = woff + (uint32_t)j * WAVE;
        const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rin, (base + i) * 4u, 0, 0);
        const bool ok = i < nvalid;
        k[j] = ok ? v : sentinel;
        a &= ok ? v ^ flip : ~0u;
        o |= ok ? v ^ flip : 0u;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a &= __shfl_xor(a, off);
        o |= __shfl_xor(o, off);
    }
    if (lane == 0) {
        sm.red[wid] = a;
        sm.red[SW + wid] = o;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t aa = ~0u, oo = 0u;
        for (int w = 0; w < SW; ++w) {
            aa &= sm.red[w];
            oo |= sm.red[SW + w];
        }
        st_agent(andor + 2 * t, aa);  // agent-coherent: read by every workgroup
        st_agent(andor + 2 * t + 1, oo);
    }
    uint32_t nb = 0;  // barriers passed
    if (!sr_sync(bar, ++nb * G, err)) return;
    // digits that vary over the whole input
    {
        uint32_t aa = ~0u, oo = 0u;
        for (uint32_t r = tid; r < G; r += SB) {
            aa &= ld_agent(andor + 2 * r);
            oo |= ld_agent(andor + 2 * r + 1);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            aa &= __shfl_xor(aa, off);
            oo |= __shfl_xor(oo, off);
        }
        if (lane == 0) {
            sm.red[wid] = aa;
            sm.red[SW + wid] = oo;
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t x = ~0u, y = 0u;
            for (int w = 0; w < SW; ++w) {
                x &= sm.red[w];
                y |= sm.red[SW + w];
            }
            sm.misc[1] = x ^ y;
        }
        __syncthreads();
    }
    const uint32_t diff = sm.misc[1];
    const bool atomic_rank = __builtin_amdgcn_readfirstlane(sm.misc[0]) != 0u;
    uint32_t amask = 0;  // bit p: digit p varies
#pragma unroll
    for (int p = 0; p < 4; ++p) amask |= ((diff >> (8 * p)) & 0xFFu) ? 1u << p : 0u;
    const int na = __builtin_popcount(amask);
    // destination of active pass i: the last one writes `out`, they alternate with tmp
    // before it; in place (in == out) with an odd count, pass 0 would read and write one
    // buffer, so tmp, out, tmp, ... and a final copy
    const bool shifted = in == out && (na & 1);
    auto dst_is_tmp = [&](int i) -> bool { return shifted ? !(i & 1) : ((na - 1 - i) & 1) != 0; };
    if (na == 0) {  // every key equal: the input is sorted
        if (in != out)
#pragma unroll
            for (int j = 0; j < SK; ++j) {
                const uint32_t i = woff + (uint32_t)j * WAVE;
                if (i < nvalid) out[base + i] = k[j];
            }
    }
    uint32_t *wh = sm.wh + wid * SRR;
    uint32_t rem = amask;
    for (int ip = 0; ip < na; ++ip) {
        const uint32_t shift = 8u * (uint32_t)__builtin_ctz(rem);
        rem &= rem - 1u;
        // per-pass copies the compiler cannot hoist: otherwise it keeps every slot's
        // bounds mask and LDS address live across the pass loop (44 SGPRs spilled)
        uint32_t tid_ = tid, nv_ = nvalid;
        asm volatile("" : "+v"(tid_), "+s"(nv_));
        const uint32_t woff_ = (tid_ >> 6) * (SK * WAVE) + (tid_ & 63u);
        if (ip > 0) {
            const __amdgpu_buffer_rsrc_t rsrc = dst_is_tmp(ip - 1) ? rtmp : rout;
#pragma unroll
            for (int j = 0; j < SK; ++j) {
                const uint32_t i = woff_ + (uint32_t)j * WAVE;
                const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rsrc, (base + i) * 4u, 0, SR_CPOL);
                k[j] = i < nv_ ? v : sentinel;
            }
        }
        for (uint32_t i = lane; i < (uint32_t)SRR; i += WAVE) wh[i] = 0u;
        uint32_t rank[SK / 2];
#pragma unroll
        for (int j = 0; j < SK; ++j) {
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
            rank[j / 2] = (j & 1) ? rank[j / 2] | (r << 16) : r;
        }
        __syncthreads();
        uint32_t h = 0;
        if (tid < (uint32_t)SRR) {
#pragma unroll
            for (int w = 0; w < SW; ++w) h += sm.wh[w * SRR + tid];
            if (tid == (uint32_t)SRR - 1) h -= (uint32_t)ST - nvalid;  // sentinels
            st_agent(cnt + t * SRR + tid, h);
        }
        const uint32_t hs = tid == (uint32_t)SRR - 1 ? h + ((uint32_t)ST - nvalid) : h;  // with sentinels
        const uint32_t ds = block_excl_scan<SB, SRR>(hs, sm.wsum);                   // tile-local digit start
        if (tid < (uint32_t)SRR) {
            uint32_t run = ds;
#pragma unroll
            for (int w = 0; w < SW; ++w) {
                const uint32_t c = sm.wh[w * SRR + tid];
                sm.wh[w * SRR + tid] = run;
                run += c;
            }
        }
        if (!sr_sync(bar, ++nb * G, err)) return;
        // digit totals and the counts of earlier tiles, from all G histogram rows
        {
            const uint32_t d = tid & (SRR - 1), g = tid >> 8;
            uint32_t tot = 0, pre = 0;
            for (uint32_t r = g; r < G; r += (uint32_t)(SB / SRR)) {
                const uint32_t v = ld_agent(cnt + r * SRR + d);
                tot += v;
                pre += r < t ? v : 0u;
            }
            sm.red[tid] = tot;
            __syncthreads();
            uint32_t T = 0;
            if (tid < (uint32_t)SRR)
#pragma unroll
                for (int q = 0; q < SB / SRR; ++q) T += sm.red[q * SRR + tid];
            __syncthreads();
            sm.red[tid] = pre;
            __syncthreads();
            uint32_t P = 0;
            if (tid < (uint32_t)SRR)
#pragma unroll
                for (int q = 0; q < SB / SRR; ++q) P += sm.red[q * SRR + tid];
            __syncthreads();  // (block_excl_scan reuses wsum)
            const uint32_t gb = block_excl_scan<SB, SRR>(T, sm.wsum);  // digit base
            if (tid < (uint32_t)SRR) sm.delta[tid] = gb + P - ds;
        }
        // reorder by digit in LDS (sentinels last), then scatter in slot order
#pragma unroll
        for (int j = 0; j < SK; ++j) {
            const uint32_t d = ((k[j] ^ flip) >> shift) & 255u;
            sm.keys[sr_pad(wh[d] + ((rank[j / 2] >> ((j & 1) * 16)) & 0xFFFFu))] = k[j];
        }
        __syncthreads();
        const __amdgpu_buffer_rsrc_t rdst = dst_is_tmp(ip) ? rtmp : rout;
#pragma unroll
        for (int j = 0; j < SK; ++j) {
            const uint32_t i = (uint32_t)j * SB + tid_;
            const uint32_t key = sm.keys[sr_pad(i)];
            // a partial tile's sentinels (i >= nvalid) go past the array's end: dropped
            const uint32_t at = i < nv_ ? sm.delta[((key ^ flip) >> shift) & 255u] + i : n;
            __builtin_amdgcn_raw_buffer_store_b32(key, rdst, at * 4u, 0, SR_CPOL);
        }
        if (ip + 1 < na)
            if (!sr_sync(bar, ++nb * G, err)) return;
    }
    if (shifted) {  // in place, odd number of passes: the result is in tmp
        if (!sr_sync(bar, ++nb * G, err)) return;
        const uint32_t *src = tmp;
#pragma unroll
        for (int j = 0; j < SK; ++j) {
            const uint32_t i = woff + (uint32_t)j * WAVE;
            if (i < nvalid) out[base + i] = LABSORT_SR_SC1 ? ld_agent(src + base + i) : src[base + i];
        }
    }
    // leave: the last workgroup out resets the arrival count (graph replays)
    if (tid == 0) {
        const unsigned long long old = __hip_atomic_fetch_add(bar, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(old & SR_CNT_MASK) + 1u == (nb + 1u) * G)
            __hip_atomic_store(bar, tag << 20, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

std::atomic<unsigned long long> g_sr_tag{0};

}  // namespace

static inline size_t sr_align(size_t x, size_t a) { return (x + a - 1) / a * a; }

SrLayout sr_layout(size_t n) {
    SrLayout L{};
    const size_t G = (n + SR_TILE - 1) / SR_TILE;
    size_t o = 0;
    L.off_err = o;  // word 0: labsort's device error word
    L.off_bar = 64;
    o = 256;
    L.off_andor = o;
    o = sr_align(o + G * 2 * 4, 256);
    L.off_cnt = o;
    o = sr_align(o + G * 256 * 4, 256);
    L.off_tmp = sr_align(o, 65536);
    L.total = sr_align(L.off_tmp + n * 4, 256);
    return L;
}

hipError_t launch_small_radix(const uint32_t *in, uint32_t *out, size_t n, uint32_t flip, char *ws, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (n > SR_MAX_N) return hipErrorInvalidValue;
    const SrLayout L = sr_layout(n);
    if (g_sr_tag.load() == 0) {
        // a per-process start: tags of two processes sharing a workspace never meet
        const unsigned long long seed =
            ((unsigned long long)getpid() << 24) ^ (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count();
        unsigned long long z = 0;
        g_sr_tag.compare_exchange_strong(z, (seed & ((1ull << 43) - 1)) | (1ull << 43));
    }
    unsigned long long tag = g_sr_tag.fetch_add(1) & ((1ull << 44) - 1);
    const unsigned G = (unsigned)((n + SR_TILE - 1) / SR_TILE);
    const uint32_t *in_ = in;
    uint32_t *out_ = out;
    uint32_t *tmp = reinterpret_cast<uint32_t *>(ws + L.off_tmp);
    uint32_t n_ = (uint32_t)n;
    uint32_t *err = reinterpret_cast<uint32_t *>(ws + L.off_err);
    unsigned long long *bar = reinterpret_cast<unsigned long long *>(ws + L.off_bar);
    uint32_t *andor = reinterpret_cast<uint32_t *>(ws + L.off_andor);
    uint32_t *cnt = reinterpret_cast<uint32_t *>(ws + L.off_cnt);
    void *args[] = {&in_, &out_, &tmp, &n_, &flip, &err, &bar, &andor, &cnt, &tag};
    if (!LABSORT_SR_COOP) {
        k_small_radix<<<G, SB, 0, s>>>(in_, out_, tmp, n_, flip, err, bar, andor, cnt, tag);
        return hipGetLastError();
    }
    return hipLaunchCooperativeKernel(reinterpret_cast<const void *>(k_small_radix), dim3(G), dim3(SB), args, 0, s);
}

}  // namespace labsort
