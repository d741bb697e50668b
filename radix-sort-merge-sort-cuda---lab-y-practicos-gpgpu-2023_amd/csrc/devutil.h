// devutil.h -- wave64 / LDS device helpers shared by the labsort kernels (gfx950).
#pragma once
#include "common.h"

namespace labsort {

// ---------------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t ld_agent(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Streamed key loads (NT_LOADS, one bit per kernel family, NT_*): a pass reads
// each key once, so its loads are issued nontemporal and the L2 keeps its capacity for
// the lines being written.  For the onesweep scatter that matters: the partial 64-B
// granules two consecutive tiles write at a digit-run boundary meet in the L2 before
// write-back instead of reaching HBM as read-modify-writes.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int BIT>
__device__ __forceinline__ uint32_t ld_stream(const uint32_t *p) {
    if constexpr ((NT_LOADS & BIT) != 0) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int BIT>
__device__ __forceinline__ uint4 ld_stream4(const uint4 *p) {
    if constexpr ((NT_LOADS & BIT) != 0) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}

// Lanes whose digit equals mine (all 64 lanes active): BITS ballots.
template <int BITS>
__device__ __forceinline__ uint64_t match_digit(uint32_t d) {
    uint64_t m = ~0ull;
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        m &= bit ? bal : ~bal;
    }
    return m;
}

// Lanes whose 8-bit digit equals mine, XOR form (v_xor / v_or3 per ballot).
__device__ __forceinline__ uint64_t match8(uint32_t d) {
    uint32_t xlo = 0, xhi = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const int32_t sgn = ((int32_t)(d << (31 - b))) >> 31;  // 0 or -1: bit b of d
        const uint64_t bal = __ballot(sgn != 0);
        xlo |= (uint32_t)bal ^ (uint32_t)sgn;
        xhi |= (uint32_t)(bal >> 32) ^ (uint32_t)sgn;
    }
    return ((uint64_t)~xhi << 32) | (uint64_t)~xlo;
}

// Lanes of this wave whose digit selects the same LDS slot as mine, by an atomic XOR
// of lane bits: the slot changes by exactly the peers' bits whatever it held, so it
// needs no clearing (a read before and after instead of an OR, a read and a 64-bit
// clearing store).  LDS operations of one wave complete in issue order.
__device__ __forceinline__ uint64_t lds_peers(uint64_t *slot, uint32_t lane) {
    const uint64_t before = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __hip_atomic_fetch_xor(slot, 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    return before ^ __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// True (in every lane) if one returning LDS atomic add instruction services the lanes
// that hit one address in ascending lane order, on five sharing patterns (all lanes,
// contiguous groups, strided groups, two scrambled ones).  Call with the whole wave
// active; `scratch` = 64 words of LDS private to the wave.
__device__ __forceinline__ bool lds_lane_ordered(uint32_t *scratch, uint32_t lane) {
    bool ok = true;
#pragma unroll
    for (int p = 0; p < 5; ++p) {
        const uint32_t a = p == 0 ? 0u
                         : p == 1 ? lane >> 3
                         : p == 2 ? lane & 7u
                         : p == 3 ? ((lane * 37u) ^ (lane >> 2)) & 15u
                                  : ((lane * 0x9E37u) >> 5) & 3u;
        __hip_atomic_store(scratch + lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        const uint32_t got = __hip_atomic_fetch_add(scratch + a, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        ok &= got == mbcnt64(match_digit<6>(a));
    }
    return __ballot(!ok) == 0ull;
}

// Stable rank of digit d among this wave's keys so far, by one returning LDS atomic
// add on the wave's counter wh[d] (lane-ordered: see lds_lane_ordered).  A digit the
// whole wave shares (sorted or nearly sorted input: the high digits of 64 consecutive
// keys) takes one add of 64 instead of 64 adds serialised on one address.  All 64
// lanes active.
__device__ __forceinline__ uint32_t wave_atomic_rank(uint32_t *wh, uint32_t d, uint32_t lane) {
    const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
    if (__ballot(d != d0) == 0ull) {
        uint32_t b = 0;
        if (lane == 0) b = __hip_atomic_fetch_add(wh + d0, 64u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        return __builtin_amdgcn_readfirstlane(b) + lane;
    }
    return __hip_atomic_fetch_add(wh + d, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// Exclusive scan over the first R threads of the block (value v in thread tid < R,
// others pass 0).  Must be called by every thread (contains a barrier when R > 64).
template <int BLOCK, int R>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *wsum) {
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(x, off);
        if (lane >= (uint32_t)off) x += t;
    }
    if constexpr (R > 64) {
        constexpr int NW = R / 64;
        if (lane == 63 && wid < (uint32_t)NW) wsum[wid] = x;
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w)
            if ((uint32_t)w < wid) add += wsum[w];
        x += add;
    }
    return x - v;
}

// Stable rank of KPT digits per lane inside one wave (slot-major order: slot j of
// lane l is element j*64+l of the wave's stripe).  `wh` = this wave's R counters
// (zeroed); on return wh[d] = count of digit d in the wave.
template <int BITS, int KPT>
__device__ __forceinline__ void wave_rank(const uint32_t (&dig)[KPT], uint32_t (&rank)[KPT], uint32_t *wh) {
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t d = dig[j];
        const uint64_t m = match_digit<BITS>(d);
        const uint32_t pre = mbcnt64(m);
        const uint32_t old = wh[d];  // peers read the same word (broadcast)
        if (pre == 0) wh[d] = old + (uint32_t)__popcll(m);  // one leader per digit
        rank[j] = old + pre;
    }
}

}  // namespace labsort
