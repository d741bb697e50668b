// harness/exp/onesweep_exp.hip -- diagnostic experiment (not part of the product):
// times variants and ablations of one LSD onesweep pass at n = 2^28 on one MI355X
// to find what bounds the pass.  Build: hipcc --offload-arch=gfx950 -O3 -o exp onesweep_exp.hip
// Outputs of the non-ablated variants are compared word for word against variant 0.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr uint32_t LB_AGG = 1u << 30, LB_INC = 2u << 30, LB_VAL = (1u << 30) - 1u;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ void k_fill(uint32_t *o, size_t n, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        o[i] = (uint32_t)(mix64(seed ^ (i * 0x9E3779B97F4A7C15ull)) >> 32);
}
__global__ void k_hist(const uint32_t *k, size_t n, uint32_t shift, uint32_t *h) {
    __shared__ uint32_t s[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s[i] = 0;
    __syncthreads();
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        atomicAdd(&s[(k[i] >> shift) & 255], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += blockDim.x) atomicAdd(&h[i], s[i]);
}
__global__ void k_scan256(const uint32_t *h, uint32_t *g) {
    if (threadIdx.x == 0) { uint32_t s = 0; for (int i = 0; i < 256; ++i) { g[i] = s; s += h[i]; } }
}
__global__ void k_copy(const uint4 *a, uint4 *b, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_agent(uint32_t *p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// match: RM=0 select form (current library), RM=1 xor/or3 form
template <int RM>
__device__ __forceinline__ uint64_t match8(uint32_t d) {
    if constexpr (RM == 0) {
        uint64_t m = ~0ull;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bal = __ballot(bit);
            m &= bit ? bal : ~bal;
        }
        return m;
    } else if constexpr (RM == 2) {
        const uint64_t bal = __ballot(d & 1u);
        return (d & 1u) ? bal : ~bal;
    } else {
        uint32_t xlo = 0, xhi = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const int32_t s = ((int32_t)(d << (31 - b))) >> 31;
            const uint64_t bal = __ballot(s != 0);
            xlo |= (uint32_t)bal ^ (uint32_t)s;
            xhi |= (uint32_t)(bal >> 32) ^ (uint32_t)s;
        }
        return ((uint64_t)~xhi << 32) | (uint64_t)~xlo;
    }
}

// ABL bits: 1 = no look-back, 2 = trivial rank, 4 = coalesced (unscattered) store, 8 = skip LDS reorder
template <int BLOCK, int KPT, int RM, int CM, int ABL>
__global__ __launch_bounds__(BLOCK) void k_os(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint32_t n,
                                              uint32_t shift, const uint32_t *__restrict__ gscan, uint32_t *lookback,
                                              uint32_t *counter, unsigned long long *stamps) {
    constexpr int R = 256, W = BLOCK / 64, TILE = BLOCK * KPT;
    unsigned long long T[8];
#define STAMP(i) do { if constexpr (ABL & 32) { __builtin_amdgcn_sched_barrier(0); T[i] = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } } while (0)
    STAMP(0);
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_wh[W * R];
    __shared__ uint32_t s_delta[R];
    __shared__ uint32_t s_wsum[W];
    __shared__ uint32_t s_tile;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(counter, 1u);
    for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLOCK) s_wh[i] = 0u;
    __syncthreads();
    const uint32_t tile = s_tile;
    STAMP(1);
    const uint32_t base = tile * (uint32_t)TILE;
    uint32_t k[KPT];
    const uint32_t wbase = base + wid * (KPT * 64) + lane;
#pragma unroll
    for (int j = 0; j < KPT; ++j) k[j] = in[wbase + j * 64];
    uint32_t dig[KPT], rank[KPT];
    uint32_t *wh = s_wh + wid * R;
#pragma unroll
    for (int j = 0; j < KPT; ++j) dig[j] = (k[j] >> shift) & 255u;
    STAMP(2);
    if constexpr (ABL & 2) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) rank[j] = j * 64 + lane;
        if (lane == 0) wh[0] = KPT * 64;
    } else if constexpr (CM == 0) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t d = dig[j];
            const uint64_t m = match8<RM>(d);
            const uint32_t pre = mbcnt64(m);
            const uint32_t old = wh[d];
            if (pre == 0) wh[d] = old + (uint32_t)__popcll(m);
            rank[j] = old + pre;
        }
    } else {
        // leader ds_add_rtn + bpermute of the returned base
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t d = dig[j];
            const uint64_t m = match8<RM>(d);
            const uint32_t pre = mbcnt64(m);
            uint32_t old = 0;
            if (pre == 0) old = atomicAdd(&wh[d], (uint32_t)__popcll(m));
            const uint32_t lo = (uint32_t)m;
            const uint32_t leader = lo ? __builtin_ctz(lo) : 32u + __builtin_ctz((uint32_t)(m >> 32));
            rank[j] = pre | (leader << 16);
            dig[j] |= old << 8;  // stash (old < 2^24)
        }
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t old = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((rank[j] >> 16) << 2), (int)(dig[j] >> 8));
            rank[j] = old + (rank[j] & 0xFFFFu);
            dig[j] &= 255u;
        }
    }
    STAMP(3);
    __syncthreads();
    uint32_t tot = 0;
    if (tid < (uint32_t)R) {
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint32_t c = s_wh[w * R + tid];
            s_wh[w * R + tid] = tot;
            tot += c;
        }
    }
    uint32_t *lb_mine = lookback + (size_t)tile * R + tid;
    if (!(ABL & 1) && !(ABL & 16) && tid < (uint32_t)R) st_agent(lb_mine, (tile == 0 ? LB_INC : LB_AGG) | tot);
    // block exclusive scan of tot over 256 digits (4 waves)
    uint32_t x = tot;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(x, off);
        if (lane >= (uint32_t)off) x += t;
    }
    if (lane == 63 && wid < 4) s_wsum[wid] = x;
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) if ((uint32_t)w < wid) add += s_wsum[w];
    const uint32_t dstart = x + add - tot;
    if (tid < (uint32_t)R) s_delta[tid] = dstart;
    __syncthreads();
    STAMP(4);
    if constexpr (!(ABL & 8)) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) s_keys[(s_delta[dig[j]] + wh[dig[j]] + rank[j]) & (TILE - 1)] = k[j];
    } else {
#pragma unroll
        for (int j = 0; j < KPT; ++j) s_keys[j * BLOCK + tid] = k[j];
    }
    STAMP(5);
    if (tid < (uint32_t)R) {
        uint32_t excl = 0;
        if constexpr ((ABL & 64) != 0) {
            constexpr int LBW = 8;
            int32_t hi = (int32_t)tile - 1;
            uint32_t spins = 0;
            while (hi >= 0) {
                uint32_t w[LBW];
#pragma unroll
                for (int i = 0; i < LBW; ++i) w[i] = (hi - i >= 0) ? ld_agent(lookback + (size_t)(hi - i) * R + tid) : LB_INC;
                int consumed = 0;
                bool done = false, stall = false;
#pragma unroll
                for (int i = 0; i < LBW; ++i) {
                    if (!done && !stall) {
                        if ((w[i] & ~LB_VAL) == 0u) stall = true;
                        else { excl += w[i] & LB_VAL; ++consumed; done = (w[i] & LB_INC) != 0; }
                    }
                }
                if (done) break;
                hi -= consumed;
                if (stall) { if (++spins > (1u << 22)) { atomicAdd(counter + 1, 1u); break; } __builtin_amdgcn_s_sleep(1); }
            }
            if (tile > 0) st_agent(lb_mine, LB_INC | (excl + tot));
        } else if (!(ABL & 1) && !(ABL & 16) && tile > 0) {
            uint32_t t = tile - 1, spins = 0;
            for (;;) {
                const uint32_t w = ld_agent(lookback + (size_t)t * R + tid);
                if ((w & ~LB_VAL) == 0u) { if (++spins > (1u << 22)) { atomicAdd(counter + 1, 1u); break; } __builtin_amdgcn_s_sleep(1); continue; }
                excl += w & LB_VAL;
                if (w & LB_INC) break;
                --t;
            }
            st_agent(lb_mine, LB_INC | (excl + tot));
        }
        if (ABL & 1) excl = tile * (TILE / R);  // fake
        if constexpr (ABL & 16) s_delta[tid] = lookback[(size_t)tile * R + tid] - dstart;
        else s_delta[tid] = gscan[tid] + excl - dstart;
    }
    __syncthreads();
    STAMP(6);
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t i = (uint32_t)j * BLOCK + tid;
        const uint32_t key = s_keys[i];
        if constexpr (ABL & 4) out[base + i] = key;
        else {
            const uint32_t d = (key >> shift) & 255u;
            out[(s_delta[d] + i) & (n - 1)] = key;  // mask only matters for ablations
        }
    }
    if constexpr (ABL & 32) {
        STAMP(7);
        if (tid == 0 || tid == 256) {
            unsigned long long *o = stamps + ((size_t)tile * 2 + (tid ? 1 : 0)) * 8;
            for (int i = 0; i < 8; ++i) o[i] = T[i];
        }
    }
}

template <int TILE>
__global__ void k_tilehist(const uint32_t *k, uint32_t shift, uint32_t *cnt) {
    __shared__ uint32_t s[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < TILE; i += blockDim.x) atomicAdd(&s[(k[(size_t)blockIdx.x * TILE + i] >> shift) & 255], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += blockDim.x) cnt[(size_t)blockIdx.x * 256 + i] = s[i];
}
__global__ void k_colscan(uint32_t *cnt, uint32_t ntiles, const uint32_t *gscan) {
    const uint32_t d = threadIdx.x;
    uint32_t s = gscan[d];
    for (uint32_t t = 0; t < ntiles; ++t) { uint32_t c = cnt[(size_t)t * 256 + d]; cnt[(size_t)t * 256 + d] = s; s += c; }
}

// v4: tile histogram first (LDS atomics), AGG published before ranking, look-back
// window loads issued before ranking and completed after it.
template <int BLOCK, int KPT, int LBW, int ABL>
__global__ __launch_bounds__(BLOCK) void k_os4(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint32_t n,
                                               uint32_t shift, const uint32_t *__restrict__ gscan, uint32_t *lookback,
                                               uint32_t *counter, unsigned long long *stamps) {
    constexpr int R = 256, W = BLOCK / 64, TILE = BLOCK * KPT;
    static_assert(BLOCK >= 256, "");
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_wh[W * R];
    __shared__ uint32_t s_hist[R];
    __shared__ uint32_t s_delta[R];
    __shared__ uint32_t s_wsum[4];
    __shared__ uint32_t s_tile;
    unsigned long long T[8];
    unsigned long long RT[4] = {0, 0, 0, 0};
    uint32_t nsteps = 0, nstall = 0;
    STAMP(0);
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(counter, 1u);
    for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLOCK) s_wh[i] = 0u;
    if (tid < (uint32_t)R) s_hist[tid] = 0u;
    __syncthreads();
    const uint32_t tile = s_tile;
    if constexpr (ABL & 128) RT[0] = __builtin_amdgcn_s_memrealtime();
    STAMP(1);
    const uint32_t base = tile * (uint32_t)TILE;
    uint32_t k[KPT], dig[KPT], rank[KPT];
    const uint32_t wbase = base + wid * (KPT * 64) + lane;
#pragma unroll
    for (int j = 0; j < KPT; ++j) k[j] = in[wbase + j * 64];
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        dig[j] = (k[j] >> shift) & 255u;
        atomicAdd(&s_hist[dig[j]], 1u);
    }
    __syncthreads();
    STAMP(2);
    // digit threads: publish the tile aggregate, scan it, start the look-back
    uint32_t h = 0, x = 0;
    uint32_t *lb_mine = lookback + (size_t)tile * R + tid;
    if (tid < (uint32_t)R) {
        h = s_hist[tid];
        st_agent(lb_mine, (tile == 0 ? LB_INC : LB_AGG) | h);
        if constexpr (ABL & 128) RT[1] = __builtin_amdgcn_s_memrealtime();
        x = h;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t t = __shfl_up(x, off);
            if (lane >= (uint32_t)off) x += t;
        }
        if (lane == 63) s_wsum[wid] = x;
    }
    uint32_t lw[LBW];
    int32_t hi = (int32_t)tile - 1;
    if (tid < (uint32_t)R) {
#pragma unroll
        for (int i = 0; i < LBW; ++i) lw[i] = (hi - i >= 0) ? ld_agent(lookback + (size_t)(hi - i) * R + tid) : LB_INC;
    }
    // wave-level stable rank
    uint32_t *wh = s_wh + wid * R;
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t d = dig[j];
        const uint64_t m = match8<1>(d);
        const uint32_t pre = mbcnt64(m);
        const uint32_t old = wh[d];
        if (pre == 0) wh[d] = old + (uint32_t)__popcll(m);
        rank[j] = old + pre;
    }
    STAMP(3);
    __syncthreads();
    if (tid < (uint32_t)R) {
        uint32_t excl = 0, spins = 0;
        for (;;) {
            int consumed = 0;
            bool done = false, stall = false;
#pragma unroll
            for (int i = 0; i < LBW; ++i) {
                if (!done && !stall) {
                    if ((lw[i] & ~LB_VAL) == 0u) stall = true;
                    else { excl += lw[i] & LB_VAL; ++consumed; done = (lw[i] & LB_INC) != 0; }
                }
            }
            ++nsteps;
            if (done) break;
            hi -= consumed;
            if (stall) {
                ++nstall;
                if (++spins > (1u << 22)) { atomicAdd(counter + 1, 1u); break; }
                __builtin_amdgcn_s_sleep(1);
            }
#pragma unroll
            for (int i = 0; i < LBW; ++i) lw[i] = (hi - i >= 0) ? ld_agent(lookback + (size_t)(hi - i) * R + tid) : LB_INC;
        }
        if (tile > 0) st_agent(lb_mine, LB_INC | (excl + h));
        if constexpr (ABL & 128) RT[2] = __builtin_amdgcn_s_memrealtime();
        uint32_t add = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) if ((uint32_t)w < wid) add += s_wsum[w];
        const uint32_t dstart = x + add - h;
        s_delta[tid] = gscan[tid] + excl - dstart;
        // per-digit exclusive prefix over waves, offset by the digit's tile start
        uint32_t run = dstart;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint32_t c = s_wh[w * R + tid];
            s_wh[w * R + tid] = run;
            run += c;
        }
    }
    __syncthreads();
    STAMP(4);
#pragma unroll
    for (int j = 0; j < KPT; ++j) s_keys[(wh[dig[j]] + rank[j]) & (TILE - 1)] = k[j];
    STAMP(5);
    __syncthreads();
    STAMP(6);
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t i = (uint32_t)j * BLOCK + tid;
        const uint32_t key = s_keys[i];
        const uint32_t d = (key >> shift) & 255u;
        out[(s_delta[d] + i) & (n - 1)] = key;  // mask: a bug shows as a mismatch, not a fault
    }
    if constexpr (ABL & 128) {
        RT[3] = __builtin_amdgcn_s_memrealtime();
        if (tid == 0) {
            unsigned long long *o = stamps + (size_t)tile * 8;
            o[0] = RT[0]; o[1] = RT[1]; o[2] = RT[2]; o[3] = RT[3]; o[4] = nsteps; o[5] = nstall;
        }
    }
    if constexpr (ABL & 32) {
        STAMP(7);
        if (tid == 0 || tid == 256) {
            unsigned long long *o = stamps + ((size_t)tile * 2 + (tid ? 1 : 0)) * 8;
            for (int i = 0; i < 8; ++i) o[i] = T[i];
        }
    }
}

// v5: v4 + optional LDS atomic-OR match (MT=1) + helping INC publication (ABL&256)
template <int BLOCK, int KPT, int LBW, int ABL, int MT, int OCC = 1>
__global__ __launch_bounds__(BLOCK, OCC) void k_os5(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint32_t n,
                                               uint32_t shift, const uint32_t *__restrict__ gscan, uint32_t *lookback,
                                               uint32_t *counter, unsigned long long *stamps, const uint32_t *segoff) {
    constexpr uint32_t P = (ABL >> 16) ? (uint32_t)(ABL >> 16) : 1u;
    constexpr int R = 256, W = BLOCK / 64, TILE = BLOCK * KPT;
    static_assert(BLOCK >= 256, "");
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_wh[W * R];
    __shared__ uint32_t s_hist[R];
    __shared__ uint32_t s_delta[R];
    __shared__ uint32_t s_wsum[4];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_match[MT ? W * R : 1];
    unsigned long long T[8];
    unsigned long long RT[4] = {0, 0, 0, 0};
    uint32_t nsteps = 0, nstall = 0;
    STAMP(0);
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(counter, 1u);
    for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLOCK) s_wh[i] = 0u;
    if constexpr (MT) for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLOCK) s_match[i] = 0ull;
    if (tid < (uint32_t)R) s_hist[tid] = 0u;
    __syncthreads();
    const uint32_t ntiles_ = n / (BLOCK * KPT), tps = ntiles_ / P;
    const uint32_t tile = (s_tile % P) * tps + s_tile / P;
    const int32_t lo = (int32_t)((tile / tps) * tps);
    if constexpr (ABL & 128) RT[0] = __builtin_amdgcn_s_memrealtime();
    STAMP(1);
    const uint32_t base = tile * (uint32_t)TILE;
    uint32_t k[KPT], dig[KPT], rank[KPT];
    const uint32_t wbase = base + wid * (KPT * 64) + lane;
#pragma unroll
    for (int j = 0; j < KPT; ++j) k[j] = in[wbase + j * 64];
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        dig[j] = (k[j] >> shift) & 255u;
        atomicAdd(&s_hist[dig[j]], 1u);
    }
    __syncthreads();
    STAMP(2);
    // digit threads: publish the tile aggregate, scan it, start the look-back
    uint32_t h = 0, x = 0;
    uint32_t *lb_mine = lookback + (size_t)tile * R + tid;
    if (tid < (uint32_t)R) {
        h = s_hist[tid];
        st_agent(lb_mine, (tile % tps == 0 ? LB_INC : LB_AGG) | h);
        if constexpr (ABL & 128) RT[1] = __builtin_amdgcn_s_memrealtime();
        x = h;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t t = __shfl_up(x, off);
            if (lane >= (uint32_t)off) x += t;
        }
        if (lane == 63) s_wsum[wid] = x;
    }
    uint32_t lw[LBW];
    int32_t hi = (int32_t)tile - 1;
    if (tid < (uint32_t)R) {
#pragma unroll
        for (int i = 0; i < LBW; ++i) lw[i] = (hi - i >= lo) ? ld_agent(lookback + (size_t)(hi - i) * R + tid) : LB_INC;
    }
    // wave-level stable rank
    uint32_t *wh = s_wh + wid * R;
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t d = dig[j];
        uint64_t m;
        if constexpr (MT) {
            uint64_t *slot = s_match + wid * R + d;
            __hip_atomic_fetch_or(slot, 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            m = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            __hip_atomic_store(slot, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        } else {
            m = match8<1>(d);
        }
        const uint32_t pre = mbcnt64(m);
        const uint32_t old = wh[d];
        if (pre == 0) wh[d] = old + (uint32_t)__popcll(m);
        rank[j] = old + pre;
    }
    STAMP(3);
    __syncthreads();
    if (tid < (uint32_t)R) {
        uint32_t excl = 0, spins = 0;
        for (;;) {
            int consumed = 0;
            bool done = false, stall = false;
#pragma unroll
            for (int i = 0; i < LBW; ++i) {
                if (!done && !stall) {
                    if ((lw[i] & ~LB_VAL) == 0u) stall = true;
                    else { excl += lw[i] & LB_VAL; ++consumed; done = (lw[i] & LB_INC) != 0; }
                }
            }
            ++nsteps;
            if constexpr ((ABL & 256) != 0) {
                if (done && nsteps > 1) {
                    // help: publish INC for the tiles of this window newer than the found INC
                    uint32_t run = 0;
                    bool seen = false;
#pragma unroll
                    for (int i = LBW - 1; i >= 0; --i) {
                        if (i < consumed) {
                            if (!seen) { if (lw[i] & LB_INC) { seen = true; run = lw[i] & LB_VAL; } }
                            else { run += lw[i] & LB_VAL; if (!(lw[i] & LB_INC)) st_agent(lookback + (size_t)(hi - i) * R + tid, LB_INC | run); }
                        }
                    }
                }
            }
            if (done) break;
            hi -= consumed;
            if (stall) {
                ++nstall;
                if (++spins > (1u << 22)) { atomicAdd(counter + 1, 1u); break; }
                __builtin_amdgcn_s_sleep(1);
            }
#pragma unroll
            for (int i = 0; i < LBW; ++i) lw[i] = (hi - i >= lo) ? ld_agent(lookback + (size_t)(hi - i) * R + tid) : LB_INC;
        }
        if (tile % tps) st_agent(lb_mine, LB_INC | (excl + h));
        if constexpr (ABL & 128) RT[2] = __builtin_amdgcn_s_memrealtime();
        uint32_t add = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) if ((uint32_t)w < wid) add += s_wsum[w];
        const uint32_t dstart = x + add - h;
        s_delta[tid] = ((P > 1) ? segoff[(size_t)(tile / tps) * tps * R + tid] : gscan[tid]) + excl - dstart;
        // per-digit exclusive prefix over waves, offset by the digit's tile start
        uint32_t run = dstart;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint32_t c = s_wh[w * R + tid];
            s_wh[w * R + tid] = run;
            run += c;
        }
    }
    __syncthreads();
    STAMP(4);
#pragma unroll
    for (int j = 0; j < KPT; ++j) s_keys[(wh[dig[j]] + rank[j]) & (TILE - 1)] = k[j];
    STAMP(5);
    __syncthreads();
    STAMP(6);
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t i = (uint32_t)j * BLOCK + tid;
        const uint32_t key = s_keys[i];
        const uint32_t d = (key >> shift) & 255u;
        out[(s_delta[d] + i) & (n - 1)] = key;  // mask: a bug shows as a mismatch, not a fault
    }
    if constexpr (ABL & 128) {
        RT[3] = __builtin_amdgcn_s_memrealtime();
        if (tid == 0) {
            unsigned long long *o = stamps + (size_t)tile * 8;
            o[0] = RT[0]; o[1] = RT[1]; o[2] = RT[2]; o[3] = RT[3]; o[4] = nsteps; o[5] = nstall;
        }
    }
    if constexpr (ABL & 32) {
        STAMP(7);
        if (tid == 0 || tid == 256) {
            unsigned long long *o = stamps + ((size_t)tile * 2 + (tid ? 1 : 0)) * 8;
            for (int i = 0; i < 8; ++i) o[i] = T[i];
        }
    }
}

// v6: persistent, software-pipelined onesweep.  Each block loops over dynamically
// acquired tiles; tile A waits (keys in registers, scatter order) for its look-back
// while the block loads, histograms, publishes and ranks tile B.
template <int BLOCK, int KPT, int LBW, int ABL, int MT, int OCC = 1>
__global__ __launch_bounds__(BLOCK, OCC) void k_os6(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint32_t n,
                                                    uint32_t shift, const uint32_t *__restrict__ gscan, uint32_t *lookback,
                                                    uint32_t *counter, unsigned long long *stamps, const uint32_t *segoff) {
    constexpr int R = 256, W = BLOCK / 64, TILE = BLOCK * KPT;
    constexpr uint32_t P = (ABL >> 16) ? (uint32_t)(ABL >> 16) : 1u;
    static_assert(BLOCK >= 256, "");
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_wh[W * R];
    __shared__ uint32_t s_hist[R];
    __shared__ uint32_t s_delta[R];
    __shared__ uint32_t s_wsum[4];
    __shared__ uint32_t s_next;
    __shared__ uint64_t s_match[MT ? W * R : 1];
    constexpr bool SEGH = (ABL & 1024) != 0;
    __shared__ uint32_t s_seg[SEGH ? P * R : 1];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t ntiles = n / TILE;
    if constexpr (SEGH) for (uint32_t i = tid; i < P * R; i += BLOCK) s_seg[i] = 0u;
    const uint32_t tps = ntiles / P;  // tiles per segment (P divides ntiles here)
    const uint32_t segshift = 31u - __builtin_clz(tps * TILE);  // tps * TILE is a power of two here
    const uint32_t tsh = 31u - __builtin_clz(tps);  // tps is a power of two in this experiment
    auto map = [&](uint32_t c) { return ((c % P) << tsh) + c / P; };
    for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLOCK) s_wh[i] = 0u;
    if constexpr (MT) for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLOCK) s_match[i] = 0ull;
    if (tid < (uint32_t)R) s_hist[tid] = 0u;
    if (tid == 0) s_next = atomicAdd(counter, 1u);
    __syncthreads();
    uint32_t tileB = s_next < ntiles ? map(s_next) : ntiles;
    // carried state of tile A
    uint32_t tileA = 0xFFFFFFFFu;
    uint32_t kA[KPT];
    uint32_t lwA[LBW];
    int32_t hiA = -1, loA = 0;
    uint32_t hA = 0, dstartA = 0, exclA = 0;
    bool doneA = false;
    constexpr bool EARLY = (ABL & 512) != 0;
    uint32_t *wh = s_wh + wid * R;
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tprev = 0, tnow = 0;
    uint32_t iters = 0;
#define PH(i) do { if constexpr (ABL & 32) { __builtin_amdgcn_sched_barrier(0); tnow = __builtin_amdgcn_s_memtime(); ph[i] += tnow - tprev; tprev = tnow; __builtin_amdgcn_sched_barrier(0); } } while (0)
    if constexpr (ABL & 32) tprev = __builtin_amdgcn_s_memtime();
    for (;;) {
        ++iters;
        const bool haveB = tileB < ntiles;
        uint32_t kB[KPT], rB[KPT];
        uint32_t hB = 0, xB = 0;
        bool doneB = false;
        uint32_t exclB = 0;
        if (tileA != 0xFFFFFFFFu && !doneA && tid < (uint32_t)R) {
#pragma unroll
            for (int i = 0; i < LBW; ++i) lwA[i] = (hiA - i >= loA) ? ld_agent(lookback + (size_t)(hiA - i) * R + tid) : LB_INC;
        }
        if (haveB) {
            const uint32_t wbase = tileB * (uint32_t)TILE + wid * (KPT * 64) + lane;
#pragma unroll
            for (int j = 0; j < KPT; ++j) kB[j] = in[wbase + j * 64];
#pragma unroll
            for (int j = 0; j < KPT; ++j) atomicAdd(&s_hist[(kB[j] >> shift) & 255u], 1u);
        }
        PH(0);
        __syncthreads();  // (1) histogram of B complete
        PH(1);
        if (haveB) {
            if (tid < (uint32_t)R) {
                hB = s_hist[tid];
                st_agent(lookback + (size_t)tileB * R + tid, ((tileB & (tps - 1)) == 0 ? LB_INC : LB_AGG) | hB);
                xB = hB;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const uint32_t t = __shfl_up(xB, off);
                    if (lane >= (uint32_t)off) xB += t;
                }
                if (lane == 63) s_wsum[wid] = xB;
            }
            uint32_t lwB[EARLY ? LBW : 1];
            const int32_t loB = (int32_t)((tileB / tps) * tps);
            if constexpr (EARLY) {
                if (tid < (uint32_t)R) {
#pragma unroll
                    for (int i = 0; i < LBW; ++i) lwB[i] = ((int32_t)tileB - 1 - i >= loB) ? ld_agent(lookback + (size_t)(tileB - 1 - i) * R + tid) : LB_INC;
                }
            }
            // stable wave rank of B
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t d = (kB[j] >> shift) & 255u;
                uint64_t m;
                if constexpr (MT) {
                    uint64_t *slot = s_match + wid * R + d;
                    __hip_atomic_fetch_or(slot, 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                    m = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                    __hip_atomic_store(slot, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                } else {
                    m = match8<1>(d);
                }
                const uint32_t pre = mbcnt64(m);
                const uint32_t old = wh[d];
                if (pre == 0) wh[d] = old + (uint32_t)__popcll(m);
                rB[j] = ((old + pre) << 8) | d;
            }
            if constexpr (EARLY) {
                if (tid < (uint32_t)R) {
                    bool stall = false;
#pragma unroll
                    for (int i = 0; i < LBW; ++i) {
                        if (!doneB && !stall) {
                            if ((lwB[i] & ~LB_VAL) == 0u) stall = true;
                            else { exclB += lwB[i] & LB_VAL; doneB = (lwB[i] & LB_INC) != 0; }
                        }
                    }
                    if (doneB) { if (tileB % tps) st_agent(lookback + (size_t)tileB * R + tid, LB_INC | (exclB + hB)); }
                    else exclB = 0;
                }
            }
        }
        PH(2);
        // complete the look-back of A
        if (tileA != 0xFFFFFFFFu && tid < (uint32_t)R) {
            uint32_t excl = exclA, spins = 0;
            int32_t hi = hiA;
            if (!doneA) for (;;) {
                int consumed = 0;
                bool done = false, stall = false;
#pragma unroll
                for (int i = 0; i < LBW; ++i) {
                    if (!done && !stall) {
                        if ((lwA[i] & ~LB_VAL) == 0u) stall = true;
                        else { excl += lwA[i] & LB_VAL; ++consumed; done = (lwA[i] & LB_INC) != 0; }
                    }
                }
                if (done) break;
                hi -= consumed;
                if (stall) {
                    if (++spins > (1u << 22)) { atomicAdd(counter + 1, 1u); break; }
                    __builtin_amdgcn_s_sleep(1);
                }
#pragma unroll
                for (int i = 0; i < LBW; ++i) lwA[i] = (hi - i >= loA) ? ld_agent(lookback + (size_t)(hi - i) * R + tid) : LB_INC;
            }
            if (!doneA && (tileA & (tps - 1))) st_agent(lookback + (size_t)tileA * R + tid, LB_INC | (excl + hA));
            const uint32_t base = (P > 1) ? segoff[(size_t)((tileA >> tsh) << tsh) * R + tid] : gscan[tid];
            s_delta[tid] = base + excl - dstartA;
        }
        PH(3);
        __syncthreads();  // (2) delta of A, wave counts of B, s_wsum of B
        PH(4);
        if (tileA != 0xFFFFFFFFu) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t i = (uint32_t)j * BLOCK + tid;
                const uint32_t pos = s_delta[(kA[j] >> shift) & 255u] + i;
                out[pos] = kA[j];
                if constexpr (SEGH) atomicAdd(&s_seg[(pos >> segshift) * R + ((kA[j] >> (shift + 8)) & 255u)], 1u);
            }
        }
        if (!haveB) break;
        if (tid < (uint32_t)R) {
            uint32_t add = 0;
#pragma unroll
            for (int w = 0; w < 4; ++w) if ((uint32_t)w < wid) add += s_wsum[w];
            const uint32_t ds = xB + add - hB;
            uint32_t run = ds;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint32_t c = s_wh[w * R + tid];
                s_wh[w * R + tid] = run;
                run += c;
            }
            s_hist[tid] = 0u;
            dstartA = ds;
        }
        if (tid == 0) s_next = atomicAdd(counter, 1u);
        PH(5);
        __syncthreads();  // (3) wave offsets of B
        PH(6);
#pragma unroll
        for (int j = 0; j < KPT; ++j) s_keys[wh[rB[j] & 255u] + (rB[j] >> 8)] = kB[j];
        __syncthreads();  // (4) B reordered in LDS
        PH(7);
#pragma unroll
        for (int j = 0; j < KPT; ++j) kA[j] = s_keys[j * BLOCK + tid];
        for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLOCK) s_wh[i] = 0u;
        tileA = tileB;
        hA = hB;
        hiA = (int32_t)tileB - 1;
        doneA = doneB;
        exclA = exclB;
        loA = (int32_t)((tileB >> tsh) << tsh);
        tileB = s_next < ntiles ? map(s_next) : ntiles;
    }
    if constexpr (SEGH) {
        __syncthreads();
        uint32_t *gseg = reinterpret_cast<uint32_t *>(stamps);
        for (uint32_t i = tid; i < P * R; i += BLOCK) if (s_seg[i]) atomicAdd(&gseg[i], s_seg[i]);
    }
    if constexpr (ABL & 32) {
        if (tid == 0 || tid == 256) {
            unsigned long long *o = stamps + ((size_t)blockIdx.x * 2 + (tid ? 1 : 0)) * 10;
            for (int i = 0; i < 8; ++i) o[i] = ph[i];
            o[8] = iters;
        }
    }
}

// v7: two-level look-back.  Tiles are grouped S at a time.  Each tile publishes its
// digit counts (AGG) for the tiles of its own group and adds them into the group's
// aggregate (device atomics); the last wave to arrive publishes the group aggregate
// (GAGG).  A tile's exclusive prefix = prefix of all earlier groups (a decoupled
// look-back over group words: GAGG / GINC, window WG) + the AGGs of its group's
// earlier tiles.  Walkers publish GINC for the group before theirs.
constexpr uint32_t G_AGG = 1u << 30, G_INC = 2u << 30;
template <int BLOCK, int KPT, int S, int WG, int MT>
__global__ __launch_bounds__(BLOCK) void k_os7(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint32_t n,
                                               uint32_t shift, const uint32_t *__restrict__ gscan, uint32_t *lbt,
                                               uint32_t *counter, uint32_t *gagg, uint32_t *garr, uint32_t *gst) {
    constexpr int R = 256, W = BLOCK / 64, TILE = BLOCK * KPT;
    static_assert(BLOCK == 512, "waves 0-3: in-group part, waves 4-7: group walk");
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_wh[W * R];
    __shared__ uint32_t s_hist[R];
    __shared__ uint32_t s_delta[R];
    __shared__ uint32_t s_pg[R];
    __shared__ uint32_t s_wsum[4];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_match[MT ? W * R : 1];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t ntiles = n / TILE;
    if (tid == 0) s_tile = atomicAdd(counter, 1u);
    for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLOCK) s_wh[i] = 0u;
    if constexpr (MT) for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLOCK) s_match[i] = 0ull;
    if (tid < (uint32_t)R) s_hist[tid] = 0u;
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint32_t g = tile / S, q = tile % S;
    const uint32_t gsize = (g + 1) * S <= ntiles ? S : ntiles - g * S;
    uint32_t k[KPT], rk[KPT];
    const uint32_t wbase = tile * (uint32_t)TILE + wid * (KPT * 64) + lane;
#pragma unroll
    for (int j = 0; j < KPT; ++j) k[j] = in[wbase + j * 64];
#pragma unroll
    for (int j = 0; j < KPT; ++j) atomicAdd(&s_hist[(k[j] >> shift) & 255u], 1u);
    __syncthreads();
    uint32_t h = 0, x = 0;
    uint32_t lw[S > 1 ? S - 1 : 1];
    uint32_t gw[WG];
    if (tid < (uint32_t)R) {
        h = s_hist[tid];
        st_agent(lbt + (size_t)tile * R + tid, G_AGG | h);
        atomicAdd(gagg + (size_t)g * R + tid, h);
        x = h;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t t = __shfl_up(x, off);
            if (lane >= (uint32_t)off) x += t;
        }
        if (lane == 63) s_wsum[wid] = x;
        // arrival: this wave's 64 group atomics are complete before it counts itself
        __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
        uint32_t old = 0;
        if (lane == 0) old = atomicAdd(garr + g, 1u);
        old = __shfl(old, 0);
        if (old == 4u * gsize - 1u) {  // last wave of the group: publish the group aggregate
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t d = u * 64 + lane;
                st_agent(gst + (size_t)g * R + d, G_AGG | ld_agent(gagg + (size_t)g * R + d));
            }
        }
        // in-group predecessors' AGGs (issued now, consumed after ranking)
#pragma unroll
        for (int i = 0; i < S - 1; ++i) lw[i] = ((uint32_t)i < q) ? ld_agent(lbt + (size_t)(g * S + i) * R + tid) : G_AGG;
    } else if (tid < 2u * R) {
        const uint32_t d = tid - R;
#pragma unroll
        for (int i = 0; i < WG; ++i) gw[i] = ((int32_t)g - 1 - i >= 0) ? ld_agent(gst + (size_t)(g - 1 - i) * R + d) : G_INC;
    }
    // stable wave rank
    uint32_t *wh = s_wh + wid * R;
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t d = (k[j] >> shift) & 255u;
        uint64_t m;
        if constexpr (MT) {
            uint64_t *slot = s_match + wid * R + d;
            __hip_atomic_fetch_or(slot, 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            m = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            __hip_atomic_store(slot, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        } else {
            m = match8<1>(d);
        }
        const uint32_t pre = mbcnt64(m);
        const uint32_t old = wh[d];
        if (pre == 0) wh[d] = old + (uint32_t)__popcll(m);
        rk[j] = ((old + pre) << 8) | d;
    }
    // complete the look-back parts
    if (tid < (uint32_t)R) {
        uint32_t spins = 0;
        for (;;) {
            bool ready = true;
#pragma unroll
            for (int i = 0; i < S - 1; ++i) ready &= (lw[i] & G_AGG) != 0u;
            if (ready) break;
            if (++spins > (1u << 22)) { atomicAdd(counter + 1, 1u); break; }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int i = 0; i < S - 1; ++i)
                if (!(lw[i] & G_AGG)) lw[i] = ld_agent(lbt + (size_t)(g * S + i) * R + tid);
        }
        uint32_t within = 0;
#pragma unroll
        for (int i = 0; i < S - 1; ++i) within += lw[i] & LB_VAL;
        s_delta[tid] = within;
    } else if (tid < 2u * R) {
        const uint32_t d = tid - R;
        uint32_t pg = 0, spins = 0;
        int32_t gh = (int32_t)g - 1;
        if (g > 0) {
            for (;;) {
                int consumed = 0;
                bool done = false, stall = false;
#pragma unroll
                for (int i = 0; i < WG; ++i) {
                    if (!done && !stall) {
                        if ((gw[i] & ~LB_VAL) == 0u) stall = true;
                        else { pg += gw[i] & LB_VAL; ++consumed; done = (gw[i] & G_INC) != 0; }
                    }
                }
                if (done) break;
                gh -= consumed;
                if (stall) {
                    if (++spins > (1u << 22)) { atomicAdd(counter + 1, 1u); break; }
                    __builtin_amdgcn_s_sleep(1);
                }
#pragma unroll
                for (int i = 0; i < WG; ++i) gw[i] = (gh - i >= 0) ? ld_agent(gst + (size_t)(gh - i) * R + d) : G_INC;
            }
            st_agent(gst + (size_t)(g - 1) * R + d, G_INC | pg);
        }
        s_pg[d] = pg;
    }
    __syncthreads();
    if (tid < (uint32_t)R) {
        uint32_t add = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) if ((uint32_t)w < wid) add += s_wsum[w];
        const uint32_t ds = x + add - h;
        s_delta[tid] = gscan[tid] + s_pg[tid] + s_delta[tid] - ds;
        uint32_t run = ds;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint32_t c = s_wh[w * R + tid];
            s_wh[w * R + tid] = run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < KPT; ++j) s_keys[wh[rk[j] & 255u] + (rk[j] >> 8)] = k[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t i = (uint32_t)j * BLOCK + tid;
        const uint32_t key = s_keys[i];
        out[(s_delta[(key >> shift) & 255u] + i) & (n - 1)] = key;
    }
}

// v9: persistent onesweep, raw tiles prefetched into LDS by DMA (global_load_lds),
// sorted tile A kept in LDS (not registers) while its look-back completes.
// LDS ping-pong X/Y: X = raw B (DMA) then raw C; Y = sorted A then sorted B.
template <int BLOCK, int KPT, int LBW, int ABL>
__global__ __launch_bounds__(BLOCK) void k_os9(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint32_t n,
                                               uint32_t shift, const uint32_t *__restrict__ gscan, uint32_t *lookback,
                                               uint32_t *counter, unsigned long long *stamps, const uint32_t *segoff) {
    constexpr int R = 256, W = BLOCK / 64, TILE = BLOCK * KPT;
    constexpr uint32_t P = (ABL >> 16) ? (uint32_t)(ABL >> 16) : 1u;
    static_assert(BLOCK >= 256 && KPT % 4 == 0, "");
    __shared__ __attribute__((aligned(16))) uint32_t s_buf[2][TILE];
    __shared__ uint32_t s_wh[W * R];
    __shared__ uint32_t s_hist[R];
    __shared__ uint32_t s_delta[R];
    __shared__ uint32_t s_wsum[4];
    __shared__ uint32_t s_next;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t ntiles = n / TILE;
    const uint32_t tps = ntiles / P;
    auto map = [&](uint32_t c) { return (c % P) * tps + c / P; };
    // DMA of one tile into an LDS buffer: KPT/4 wave-instructions of 1 KiB per wave
    auto dma = [&](uint32_t t, uint32_t *buf) {
        const uint32_t *src = in + (size_t)t * TILE + wid * (KPT * 64);
        uint32_t *dst = buf + wid * (KPT * 64);
#pragma unroll
        for (int u = 0; u < KPT / 4; ++u)
            __builtin_amdgcn_global_load_lds(src + u * 256 + lane * 4, dst + u * 256, 16, 0, 0);
    };
    for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLOCK) s_wh[i] = 0u;
    if (tid < (uint32_t)R) s_hist[tid] = 0u;
    if (tid == 0) s_next = atomicAdd(counter, 1u);
    __syncthreads();
    uint32_t tileB = s_next < ntiles ? map(s_next) : ntiles;
    constexpr int xb = 0;  // X = s_buf[0] (raw, DMA target), Y = s_buf[1] (sorted)
    if (tileB < ntiles) dma(tileB, s_buf[xb]);
    if (tid == 0) s_next = atomicAdd(counter, 1u);
    uint32_t tileA = 0xFFFFFFFFu;
    int32_t hiA = -1, loA = 0;
    uint32_t hA = 0, dstartA = 0;
    uint32_t *wh = s_wh + wid * R;
    for (;;) {
        __syncthreads();  // I1: raw B landed in X (the barrier drains the DMA), s_next visible
        const bool haveB = tileB < ntiles;
        const uint32_t tileC = s_next < ntiles ? map(s_next) : ntiles;
        uint32_t kB[KPT], rB[KPT];
        uint32_t lwA[LBW];
        uint32_t hB = 0, xB = 0;
        if (haveB) {
            const uint32_t *X = s_buf[xb] + wid * (KPT * 64) + lane;
#pragma unroll
            for (int j = 0; j < KPT; ++j) kB[j] = X[j * 64];
        }
        if (tileA != 0xFFFFFFFFu && tid < (uint32_t)R) {
#pragma unroll
            for (int i = 0; i < LBW; ++i) lwA[i] = (hiA - i >= loA) ? ld_agent(lookback + (size_t)(hiA - i) * R + tid) : LB_INC;
        }
        if (haveB) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) atomicAdd(&s_hist[(kB[j] >> shift) & 255u], 1u);
        }
        __syncthreads();  // I2: X free, histogram of B complete
        if (tileC < ntiles) dma(tileC, s_buf[xb]);
        if (tid == 0 && tileC < ntiles) s_next = atomicAdd(counter, 1u);
        if (haveB) {
            if (tid < (uint32_t)R) {
                hB = s_hist[tid];
                st_agent(lookback + (size_t)tileB * R + tid, (tileB % tps == 0 ? LB_INC : LB_AGG) | hB);
                xB = hB;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const uint32_t t = __shfl_up(xB, off);
                    if (lane >= (uint32_t)off) xB += t;
                }
                if (lane == 63) s_wsum[wid] = xB;
            }
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t d = (kB[j] >> shift) & 255u;
                const uint64_t m = match8<1>(d);
                const uint32_t pre = mbcnt64(m);
                const uint32_t old = wh[d];
                if (pre == 0) wh[d] = old + (uint32_t)__popcll(m);
                rB[j] = ((old + pre) << 8) | d;
            }
        }
        if (tileA != 0xFFFFFFFFu && tid < (uint32_t)R) {
            uint32_t excl = 0, spins = 0;
            int32_t hi = hiA;
            for (;;) {
                int consumed = 0;
                bool done = false, stall = false;
#pragma unroll
                for (int i = 0; i < LBW; ++i) {
                    if (!done && !stall) {
                        if ((lwA[i] & ~LB_VAL) == 0u) stall = true;
                        else { excl += lwA[i] & LB_VAL; ++consumed; done = (lwA[i] & LB_INC) != 0; }
                    }
                }
                if (done) break;
                hi -= consumed;
                if (stall) {
                    if (++spins > (1u << 22)) { atomicAdd(counter + 1, 1u); break; }
                    __builtin_amdgcn_s_sleep(1);
                }
#pragma unroll
                for (int i = 0; i < LBW; ++i) lwA[i] = (hi - i >= loA) ? ld_agent(lookback + (size_t)(hi - i) * R + tid) : LB_INC;
            }
            if (tileA % tps) st_agent(lookback + (size_t)tileA * R + tid, LB_INC | (excl + hA));
            const uint32_t base = (P > 1) ? segoff[(size_t)(tileA / tps) * tps * R + tid] : gscan[tid];
            s_delta[tid] = base + excl - dstartA;
        }
        __syncthreads();  // I5: delta of A, wave counts of B, s_wsum of B
        if (tileA != 0xFFFFFFFFu) {
            const uint32_t *Y = s_buf[xb ^ 1];
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t i = (uint32_t)j * BLOCK + tid;
                const uint32_t key = Y[i];
                out[s_delta[(key >> shift) & 255u] + i] = key;
            }
        }
        if (!haveB) break;
        if (tid < (uint32_t)R) {
            uint32_t add = 0;
#pragma unroll
            for (int w = 0; w < 4; ++w) if ((uint32_t)w < wid) add += s_wsum[w];
            const uint32_t ds = xB + add - hB;
            uint32_t run = ds;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const uint32_t c = s_wh[w * R + tid];
                s_wh[w * R + tid] = run;
                run += c;
            }
            s_hist[tid] = 0u;
            dstartA = ds;
        }
        __syncthreads();  // I7: Y free (A scattered), wave offsets of B
        {
            uint32_t *Y = s_buf[xb ^ 1];
#pragma unroll
            for (int j = 0; j < KPT; ++j) Y[wh[rB[j] & 255u] + (rB[j] >> 8)] = kB[j];
        }
        __syncthreads();  // I8: wave offsets consumed before zeroing
        for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLOCK) s_wh[i] = 0u;
        tileA = tileB;
        hA = hB;
        hiA = (int32_t)tileB - 1;
        loA = (int32_t)((tileB / tps) * tps);
        tileB = tileC;
    }
}

struct Ctx {
    uint32_t *in, *out, *gscan, *lb, *cnt;
    unsigned long long *st;
    size_t n;
};

template <int BLOCK, int KPT, int RM, int CM, int ABL, int V = 0, int OCC = 1>
float run(Ctx &c, const char *name, const uint32_t *ref, int reps = 10) {
    constexpr int TILE = BLOCK * KPT;
    const uint32_t ntiles = (uint32_t)(c.n / TILE);
    std::vector<float> ts;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int r = 0; r < reps + 2; ++r) {
        if ((V == 6 || V == 5 || V == 9) && (ABL >> 16) > 1 && r == 0) {
            k_tilehist<TILE><<<ntiles, 256>>>(c.in, 0, c.lb + 2 * (size_t)ntiles * 256);
            k_colscan<<<1, 256>>>(c.lb + 2 * (size_t)ntiles * 256, ntiles, c.gscan);
        }
        if (ABL & 16) {
            k_tilehist<TILE><<<ntiles, 256>>>(c.in, 0, c.lb);
            k_colscan<<<1, 256>>>(c.lb, ntiles, c.gscan);
        } else CK(hipMemset(c.lb, 0, (size_t)ntiles * 256 * 4 * (V == 7 ? 3 : 1)));
        if (V == 7) CK(hipMemset(c.st, 0, (size_t)ntiles * 4));
        if (ABL & 1024) CK(hipMemset(c.st, 0, 1 << 20));
        CK(hipMemset(c.cnt, 0, 8));
        CK(hipEventRecord(a));
        if constexpr (V == 9) k_os9<BLOCK, KPT, RM, ABL><<<std::min<uint32_t>(ntiles, 512), BLOCK>>>(c.in, c.out, (uint32_t)c.n, 0, c.gscan, c.lb, c.cnt, c.st, c.lb + 2 * (size_t)ntiles * 256);
        else if constexpr (V == 7) k_os7<BLOCK, KPT, (ABL >> 16), RM, CM><<<ntiles, BLOCK>>>(c.in, c.out, (uint32_t)c.n, 0, c.gscan, c.lb, c.cnt, c.lb + (size_t)ntiles * 256, (uint32_t *)c.st, c.lb + (size_t)ntiles * 256 + (size_t)ntiles * 256);
        else if constexpr (V == 6) k_os6<BLOCK, KPT, RM, ABL, CM, OCC><<<std::min<uint32_t>(ntiles, 256 * (OCC > 1 ? OCC * 256 / BLOCK : 2)), BLOCK>>>(c.in, c.out, (uint32_t)c.n, 0, c.gscan, c.lb, c.cnt, c.st, c.lb + 2 * (size_t)ntiles * 256);
        else if constexpr (V == 5) k_os5<BLOCK, KPT, RM, ABL, CM, OCC><<<ntiles, BLOCK>>>(c.in, c.out, (uint32_t)c.n, 0, c.gscan, c.lb, c.cnt, c.st, c.lb + 2 * (size_t)ntiles * 256);
        else if constexpr (V == 4) k_os4<BLOCK, KPT, RM, ABL><<<ntiles, BLOCK>>>(c.in, c.out, (uint32_t)c.n, 0, c.gscan, c.lb, c.cnt, c.st);
        else k_os<BLOCK, KPT, RM, CM, ABL><<<ntiles, BLOCK>>>(c.in, c.out, (uint32_t)c.n, 0, c.gscan, c.lb, c.cnt, c.st);
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    float med = ts[ts.size() / 2];
    uint32_t hc[2];
    CK(hipMemcpy(hc, c.cnt, 8, hipMemcpyDeviceToHost));
    if (hc[1]) printf("   !! spin limit hit %u times\n", hc[1]);
    const char *ok = "";
    if (ref && ((ABL & 0xFFFF) & ~(16 | 32 | 64 | 128 | 256 | 512 | 1024)) == 0 && TILE * ntiles == c.n) {
        std::vector<uint32_t> h(c.n);
        CK(hipMemcpy(h.data(), c.out, c.n * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < c.n; ++i) bad += h[i] != ref[i];
        static char buf[64];
        snprintf(buf, sizeof buf, bad ? " [MISMATCH %zu]" : " [match]", bad);
        ok = buf;
    }
    printf("%-44s B%4d K%2d  %.4f ms  %7.1f GB/s (8B/key)%s\n", name, BLOCK, KPT, med, 8.0 * c.n / med / 1e6, ok);
    if ((ABL & 128) && V != 7) {
        std::vector<unsigned long long> st((size_t)ntiles * 8);
        CK(hipMemcpy(st.data(), c.st, st.size() * 8, hipMemcpyDeviceToHost));
        double pub = 0, lbk = 0, rest = 0, steps = 0, stalls = 0, predlate = 0; int npl = 0;
        unsigned long long t0 = ~0ull, t1 = 0;
        for (uint32_t t = 0; t < ntiles; ++t) {
            unsigned long long *o = &st[(size_t)t * 8];
            pub += o[1] - o[0]; lbk += o[2] - o[1]; rest += o[3] - o[2]; steps += o[4]; stalls += o[5];
            t0 = std::min(t0, o[0]); t1 = std::max(t1, o[3]);
            if (t > 0 && st[(size_t)(t - 1) * 8 + 1] > o[1]) { predlate += st[(size_t)(t - 1) * 8 + 1] - o[1]; ++npl; }
        }
        printf("   realtime (100MHz ticks)/tile: acquire->agg %.1f  agg->lookback-done %.1f  ->end %.1f | steps %.2f stalls %.2f | pred AGG later than mine: %d tiles, avg %.1f | span %.3f ms\n",
               pub / ntiles, lbk / ntiles, rest / ntiles, steps / ntiles, stalls / ntiles, npl, npl ? predlate / npl : 0.0, (t1 - t0) / 1e5);
        // in-flight estimate: tiles acquired but not ended at the midpoint
        unsigned long long mid = (t0 + t1) / 2; int inflight = 0;
        for (uint32_t t = 0; t < ntiles; ++t) inflight += st[(size_t)t * 8] <= mid && st[(size_t)t * 8 + 3] >= mid;
        printf("   tiles in flight at midpoint: %d\n", inflight);
    }
    if (ABL & 1024) {
        constexpr uint32_t P = (ABL >> 16);
        std::vector<uint32_t> h(c.n), gs(P * 256), ex(P * 256, 0);
        CK(hipMemcpy(h.data(), c.out, c.n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(gs.data(), c.st, P * 256 * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < c.n; ++i) ex[(i / (c.n / P)) * 256 + ((h[i] >> 8) & 255)]++;
        printf("   next-pass segment histograms: %s\n", gs == ex ? "match" : "MISMATCH");
    }
    if ((ABL & 32) && V == 6) {
        const uint32_t nb = std::min<uint32_t>(ntiles, 512);
        std::vector<unsigned long long> st((size_t)nb * 20);
        CK(hipMemcpy(st.data(), c.st, st.size() * 8, hipMemcpyDeviceToHost));
        for (int w = 0; w < 2; ++w) {
            double acc[9] = {0};
            for (uint32_t b = 0; b < nb; ++b) for (int i = 0; i < 9; ++i) acc[i] += (double)st[(b * 2 + w) * 10 + i];
            printf("   %s cycles/iter: load+hist %.0f bar1 %.0f publish+rank %.0f lbA %.0f bar2 %.0f scatA+prefix %.0f bar3 %.0f reorder+bar4 %.0f (iters/block %.1f)\n",
                   w ? "wave4" : "wave0", acc[0] / acc[8], acc[1] / acc[8], acc[2] / acc[8], acc[3] / acc[8], acc[4] / acc[8], acc[5] / acc[8], acc[6] / acc[8], acc[7] / acc[8], acc[8] / nb);
        }
    }
    if ((ABL & 32) && V != 7 && V != 6) {
        std::vector<unsigned long long> st((size_t)ntiles * 16);
        CK(hipMemcpy(st.data(), c.st, st.size() * 8, hipMemcpyDeviceToHost));
        for (int w = 0; w < 2; ++w) {
            double acc[8] = {0};
            for (uint32_t t = 0; t < ntiles; ++t)
                for (int i = 1; i < 8; ++i) acc[i] += (double)(st[(t * 2 + w) * 8 + i] - st[(t * 2 + w) * 8 + i - 1]);
            printf("   %s phase cycles/tile: tileid %.0f load %.0f rank %.0f scan %.0f ldsscat %.0f lookback %.0f store %.0f\n",
                   w ? "wave4" : "wave0", acc[1] / ntiles, acc[2] / ntiles, acc[3] / ntiles, acc[4] / ntiles, acc[5] / ntiles, acc[6] / ntiles, acc[7] / ntiles);
        }
    }
    return med;
}

int main() {
    Ctx c;
    c.n = (size_t)1 << 28;
    CK(hipMalloc(&c.in, c.n * 4));
    CK(hipMalloc(&c.out, c.n * 4));
    CK(hipMalloc(&c.gscan, 256 * 4));
    CK(hipMalloc(&c.lb, (c.n / 1024) * 256 * 4));
    CK(hipMalloc(&c.cnt, 8));
    CK(hipMalloc(&c.st, (c.n / 1024) * 16 * 8));
    uint32_t *h;
    CK(hipMalloc(&h, 256 * 4));
    k_fill<<<4096, 256>>>(c.in, c.n, 0x5EED0003);
    CK(hipMemset(h, 0, 1024));
    k_hist<<<2048, 256>>>(c.in, c.n, 0, h);
    k_scan256<<<1, 64>>>(h, c.gscan);
    CK(hipDeviceSynchronize());
    {   // copy roofline
        std::vector<float> ts;
        hipEvent_t a, b;
        hipEventCreate(&a); hipEventCreate(&b);
        for (int r = 0; r < 12; ++r) {
            hipEventRecord(a);
            k_copy<<<8192, 256>>>((const uint4 *)c.in, (uint4 *)c.out, c.n / 4);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); if (r >= 2) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-44s            %.4f ms  %7.1f GB/s\n", "copy uint4 (read+write 8B/key)", ts[5], 8.0 * c.n / ts[5] / 1e6);
    }
    run<512, 16, 0, 0, 0>(c, "v0 select-match, RMW counters", nullptr);
    std::vector<uint32_t> ref(c.n);
    {
        std::vector<uint32_t> hin(c.n);
        CK(hipMemcpy(hin.data(), c.in, c.n * 4, hipMemcpyDeviceToHost));
        std::vector<size_t> off(257, 0);
        for (size_t i = 0; i < c.n; ++i) off[(hin[i] & 255) + 1]++;
        for (int d = 0; d < 256; ++d) off[d + 1] += off[d];
        for (size_t i = 0; i < c.n; ++i) ref[off[hin[i] & 255]++] = hin[i];
        std::vector<uint32_t> h0(c.n);
        CK(hipMemcpy(h0.data(), c.out, c.n * 4, hipMemcpyDeviceToHost));
        printf("v0 vs host stable counting sort: %s\n", memcmp(h0.data(), ref.data(), c.n * 4) ? "MISMATCH" : "match");
    }
    run<512, 16, 4, 1, 0, 6>(c, "v6 (shift mapping)", ref.data());
    run<512, 16, 4, 1, 16 << 16, 6>(c, "v8 16 segments (shift mapping)", ref.data());
    run<512, 16, 4, 1, 64 << 16, 6>(c, "v8 64 segments (shift mapping)", ref.data());
    run<512, 16, 8, 1, 16 << 16, 6>(c, "v8 W8 16 segments (shift mapping)", ref.data());
    return 0;
}
