// kmerge.hip -- K-way merge passes (K = 2, 4, 8) for gfx950.
//
// The reference's stage 3 (lab.cu:348-391) merges pairs of sorted runs, one doubling
// per iteration, with separators every 256 keys (separators_kernel :209-270) and a
// shared-memory merge per segment (merge_segments_kernel :272-300).  Here one pass
// merges K runs at once, so the 2^28-key merge sort needs 5 passes over HBM instead
// of 13, and the multi-GPU exchange merges the p received runs in one pass.
//
// Same separator idea, generalised to K runs and made exact:
//   k_km_samples  every KM_S-th key of every run (the reference's separators every
//                 256 keys) into a compact sample array;
//   k_km_split    each sample's rank among all samples of its K runs (binary
//                 searches in the other runs' samples, busquedaPorBiparticion
//                 :102-132); every KM_M-th sample becomes a block boundary and gets
//                 its exact cut in every run (a binary search inside one sample
//                 chunk of that run);
//   k_km_blocks   one workgroup per block: its K slices (<= (KM_M + K) * KM_S keys
//                 in total) into LDS, log2(K) levels of pairwise merge-path merges
//                 in LDS, one coalesced store of the merged block.
// Order: (key, run, position), i.e. equal keys keep run order (A before B, as
// deviceOrderedJoin :144-182 places the left run first) -- a stable merge.
#include "common.h"

namespace labsort {

__device__ __forceinline__ bool km_le(uint32_t a, uint32_t b, uint32_t flip) { return (a ^ flip) <= (b ^ flip); }
__device__ __forceinline__ bool km_lt(uint32_t a, uint32_t b, uint32_t flip) { return (a ^ flip) < (b ^ flip); }

__device__ __forceinline__ uint32_t km_rb(const KmRuns &rs, uint32_t job, uint32_t q) {
    if (rs.explicit_runs) return rs.offs[q];
    const uint64_t b = ((uint64_t)job * rs.K + q) * rs.run;
    return (uint32_t)(b < rs.n ? b : rs.n);
}
__device__ __forceinline__ uint32_t km_re(const KmRuns &rs, uint32_t job, uint32_t q) {
    if (rs.explicit_runs) return rs.offs[q + 1];
    const uint64_t e = ((uint64_t)job * rs.K + q + 1) * rs.run;
    return (uint32_t)(e < rs.n ? e : rs.n);
}
__device__ __forceinline__ uint32_t km_pad(uint32_t i) { return i + (i >> 5); }  // LDS bank padding
__device__ __forceinline__ uint32_t km_ns(uint32_t len) { return (len + KM_S - 1) / KM_S; }  // samples of a run
// first sample slot of run q of `job`
__device__ __forceinline__ uint32_t km_sbase(const KmRuns &rs, uint32_t job, uint32_t q) {
    if (!rs.explicit_runs) return (job * rs.K + q) * (rs.run / KM_S);
    uint32_t b = 0;
    for (uint32_t r = 0; r < q; ++r) b += km_ns(rs.offs[r + 1] - rs.offs[r]);
    return b;
}
// sample slot -> (job, run, sample index); false if the slot holds no sample
__device__ __forceinline__ bool km_slot(const KmRuns &rs, uint32_t slot, uint32_t &job, uint32_t &q, uint32_t &j) {
    if (!rs.explicit_runs) {
        const uint32_t spr = rs.run / KM_S, gr = slot / spr;
        job = gr / rs.K;
        q = gr % rs.K;
        j = slot % spr;
        return job < rs.njobs && j < km_ns(km_re(rs, job, q) - km_rb(rs, job, q));
    }
    job = 0;
    uint32_t b = 0;
    for (q = 0; q < rs.K; ++q) {
        const uint32_t ns = km_ns(rs.offs[q + 1] - rs.offs[q]);
        if (slot < b + ns) {
            j = slot - b;
            return true;
        }
        b += ns;
    }
    return false;
}

__global__ __launch_bounds__(256) void k_km_samples(const uint32_t *__restrict__ keys, KmRuns rs,
                                                   uint32_t *__restrict__ samp, uint32_t nslots) {
    for (uint32_t s = blockIdx.x * 256u + threadIdx.x; s < nslots; s += gridDim.x * 256u) {
        uint32_t job, q, j;
        if (km_slot(rs, s, job, q, j)) samp[s] = keys[km_rb(rs, job, q) + j * KM_S];
    }
}

// number of elements of sorted a[0, len) that precede key v of a run after (upper
// = false: elements < v) or before (upper = true: elements <= v) a's run
__device__ __forceinline__ uint32_t km_count(const uint32_t *a, uint32_t lo, uint32_t hi, uint32_t v, bool upper,
                                             uint32_t flip) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const bool pre = upper ? km_le(a[mid], v, flip) : km_lt(a[mid], v, flip);
        if (pre) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// cuts[(job * rs.nspl_max + s) * K + q'] = keys of run q' preceding splitter s of `job`
template <int K>
__global__ __launch_bounds__(256) void k_km_split(const uint32_t *__restrict__ keys, KmRuns rs,
                                                 const uint32_t *__restrict__ samp, uint32_t nslots,
                                                 uint32_t *__restrict__ cuts, uint32_t flip) {
    for (uint32_t s = blockIdx.x * 256u + threadIdx.x; s < nslots; s += gridDim.x * 256u) {
        uint32_t job, q, j;
        if (!km_slot(rs, s, job, q, j)) continue;
        const uint32_t v = samp[s];
        uint32_t c[K];
        uint32_t r = 0;
#pragma unroll
        for (uint32_t q2 = 0; q2 < (uint32_t)K; ++q2) {
            if (q2 == q) {
                c[q2] = j;
            } else {
                const uint32_t b = km_sbase(rs, job, q2), ns = km_ns(km_re(rs, job, q2) - km_rb(rs, job, q2));
                c[q2] = km_count(samp + b, 0, ns, v, q2 < q, flip);
            }
            r += c[q2];
        }
        if (r % KM_M) continue;
        uint32_t *cw = cuts + ((size_t)job * rs.nspl_max + r / KM_M) * K;
#pragma unroll
        for (uint32_t q2 = 0; q2 < (uint32_t)K; ++q2) {
            if (q2 == q) {
                cw[q2] = j * KM_S;
                continue;
            }
            const uint32_t rb = km_rb(rs, job, q2), len = km_re(rs, job, q2) - rb;
            // samples 0 .. c-1 of run q2 precede, sample c (if any) does not
            const uint32_t lo = c[q2] ? (c[q2] - 1u) * KM_S + 1u : 0u;
            const uint32_t hi = c[q2] * KM_S < len ? c[q2] * KM_S : len;
            cw[q2] = km_count(keys + rb, lo, hi, v, q2 < q, flip);
        }
    }
}

// one workgroup per block (job, b): block b = keys between boundaries b and b + 1,
// boundary 0 = the runs' starts, boundary nspl + 1 = their ends, boundary s + 1 =
// splitter s
template <int K>
__global__ __launch_bounds__(KM_BLOCK) void k_km_blocks(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                      KmRuns rs, const uint32_t *__restrict__ cuts, uint32_t flip) {
    __shared__ uint32_t buf[2][KM_BMAX(K) + KM_BMAX(K) / 32];
    __shared__ uint32_t s_len[K], s_src[K];
    const uint32_t tid = threadIdx.x;
    const uint32_t bpj = rs.nspl_max + 1u;
    const uint32_t job = blockIdx.x / bpj, b = blockIdx.x % bpj;
    if (job >= rs.njobs) return;
    if (tid < (uint32_t)K) {
        // lane q: run q's slice of this block (the K cut loads issue in parallel)
        uint32_t ts = 0;  // samples of this job -> ceil(ts / KM_M) splitters
#pragma unroll
        for (int r = 0; r < K; ++r) ts += km_ns(km_re(rs, job, r) - km_rb(rs, job, r));
        const uint32_t nspl = (ts + KM_M - 1) / KM_M;
        const uint32_t q = tid, rb = km_rb(rs, job, q), len = km_re(rs, job, q) - rb;
        const uint32_t lo = b == 0 ? 0u : b > nspl ? len : cuts[((size_t)job * rs.nspl_max + b - 1) * K + q];
        const uint32_t hi = b >= nspl ? len : cuts[((size_t)job * rs.nspl_max + b) * K + q];
        s_src[q] = rb + lo;
        s_len[q] = hi > lo ? hi - lo : 0u;
    }
    __syncthreads();
    // slice prefix (pk) and source shift (sh: LDS index i of run q <- in[i + sh[q]]),
    // uniform over the workgroup, in registers
    uint32_t pk[K + 1], sh[K];
    uint32_t obase = km_rb(rs, job, 0);  // output position of the block's first key
    pk[0] = 0;
#pragma unroll
    for (int q = 0; q < K; ++q) {
        const uint32_t sq = s_src[q];
        pk[q + 1] = pk[q] + s_len[q];
        sh[q] = sq - pk[q];
        obase += sq - km_rb(rs, job, q);
    }
    const uint32_t B = pk[K];
    if (B == 0) return;
    // K slices into LDS: every load issued before the first store (coalesced within
    // each slice)
    constexpr int LPT = (KM_BMAX(K) + KM_BLOCK - 1) / KM_BLOCK;
    {
        uint32_t v[LPT];
#pragma unroll
        for (int j = 0; j < LPT; ++j) {
            const uint32_t i = tid + (uint32_t)j * KM_BLOCK;
            uint32_t s0 = sh[0];
#pragma unroll
            for (int r = 1; r < K; ++r) s0 = i >= pk[r] ? sh[r] : s0;
            v[j] = i < B ? in[i + s0] : 0u;
        }
#pragma unroll
        for (int j = 0; j < LPT; ++j) {
            const uint32_t i = tid + (uint32_t)j * KM_BLOCK;
            if (i < B) buf[0][km_pad(i)] = v[j];
        }
    }
    __syncthreads();
    // log2(K) levels of pairwise merges: segments of w runs -> segments of 2w runs.
    // Thread t produces outputs [t E, t E + E) of each level in chunks of 8: a
    // merge-path co-rank search, then the 8 outputs by a bitonic merge of 8 + 8
    // candidates (or a sequential merge, KM_SEQ).  E is a multiple of 8, so a chunk is split only where it
    // crosses a segment end.  LDS index i is stored at km_pad(i): the 8-key chunks of
    // neighbouring lanes (stride 8 words) then fall on distinct banks.
    const uint32_t E = ((B + KM_BLOCK - 1) / KM_BLOCK + 7u) & ~7u;
    int cur = 0;
#pragma unroll
    for (int w = 1; w < K; w <<= 1) {
        const uint32_t *s = buf[cur];
        uint32_t *d = buf[cur ^ 1];
        uint32_t pos = tid * E;
        const uint32_t p1 = pos + E < B ? pos + E : B;
        while (pos < p1) {
            // this level's segment holding pos: [pk[2w pr], pk[2w (pr + 1)])
            uint32_t xs = 0, xm = pk[w], ye = pk[2 * w];
#pragma unroll
            for (int r = 1; r < K / (2 * w); ++r)
                if (pos >= pk[r * 2 * w]) {
                    xs = pk[r * 2 * w];
                    xm = pk[r * 2 * w + w];
                    ye = pk[(r + 1) * 2 * w];
                }
            const uint32_t lx = xm - xs, ly = ye - xm;
            const uint32_t end = p1 < ye ? p1 : ye;
            for (; pos < end; pos += 8) {
                const uint32_t diag = pos - xs, cnt = end - pos < 8 ? end - pos : 8;
                uint32_t lo = diag > ly ? diag - ly : 0u, hi = diag < lx ? diag : lx;
                while (lo < hi) {  // merge path: X before Y on equal keys
                    const uint32_t mid = (lo + hi) >> 1;
                    if (km_le(s[km_pad(xs + mid)], s[km_pad(xm + diag - mid - 1)], flip)) lo = mid + 1;
                    else hi = mid;
                }
                uint32_t r8[8];
                if (KM_SEQ) {
                    uint32_t ai = xs + lo, bi = xm + (diag - lo);
                    uint32_t va = ai < xm ? s[km_pad(ai)] : 0u, vb = bi < ye ? s[km_pad(bi)] : 0u;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const bool takeA = bi >= ye || (ai < xm && km_le(va, vb, flip));
                        r8[k] = takeA ? va : vb;
                        if (takeA) {
                            ++ai;
                            va = ai < xm ? s[km_pad(ai)] : 0u;
                        } else {
                            ++bi;
                            vb = bi < ye ? s[km_pad(bi)] : 0u;
                        }
                    }
                } else {
                    // 8 + 8 candidates; the 8 smallest by a bitonic merge (keys only: equal
                    // keys are interchangeable, so +inf padding and the network's tie order
                    // cannot change the output)
                    const uint32_t i = lo, jj = diag - lo;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const uint32_t xv = i + k < lx ? s[km_pad(xs + i + k)] ^ flip : 0xFFFFFFFFu;
                        const uint32_t yv = jj + 7 - k < ly ? s[km_pad(xm + jj + 7 - k)] ^ flip : 0xFFFFFFFFu;
                        r8[k] = xv < yv ? xv : yv;  // bitonic sequence
                    }
#pragma unroll
                    for (int dd = 4; dd >= 1; dd >>= 1)
#pragma unroll
                        for (int k = 0; k < 8; ++k)
                            if ((k & dd) == 0) {
                                const uint32_t a = r8[k], b2 = r8[k + dd];
                                r8[k] = a < b2 ? a : b2;
                                r8[k + dd] = a < b2 ? b2 : a;
                            }
#pragma unroll
                    for (int k = 0; k < 8; ++k) r8[k] ^= flip;
                }
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if ((uint32_t)k < cnt) d[km_pad(pos + k)] = r8[k];
            }
            pos = end;
        }
        __syncthreads();
        cur ^= 1;
    }
    for (uint32_t i = tid; i < B; i += KM_BLOCK) out[obase + i] = buf[cur][km_pad(i)];
}

// Persistent, software-pipelined form of k_km_blocks: workgroup g merges blocks g,
// g + G, g + 2G, ...  While block i merges in LDS, the keys of block i + G are
// already loading into registers and the slice header (K cuts) of block i + 2G is
// in flight, so HBM latency overlaps the LDS merge instead of idling the CU.
template <int K>
__device__ __forceinline__ void km_hdr(const KmRuns &rs, const uint32_t *__restrict__ cuts, uint32_t blk, uint32_t q,
                                       uint32_t &src, uint32_t &len) {
    const uint32_t bpj = rs.nspl_max + 1u;
    const uint32_t job = blk / bpj, b = blk % bpj;
    uint32_t ts = 0;  // samples of this job -> ceil(ts / KM_M) splitters
#pragma unroll
    for (int r = 0; r < K; ++r) ts += km_ns(km_re(rs, job, r) - km_rb(rs, job, r));
    const uint32_t nspl = (ts + KM_M - 1) / KM_M;
    const uint32_t rb = km_rb(rs, job, q), rl = km_re(rs, job, q) - rb;
    const uint32_t lo = b == 0 ? 0u : b > nspl ? rl : cuts[((size_t)job * rs.nspl_max + b - 1) * K + q];
    const uint32_t hi = b >= nspl ? rl : cuts[((size_t)job * rs.nspl_max + b) * K + q];
    src = rb + lo;
    len = hi > lo ? hi - lo : 0u;
}

template <int K>
struct KmGeo {
    uint32_t pk[K + 1], sh[K], obase;
};
template <int K>
__device__ __forceinline__ void km_geo(const KmRuns &rs, uint32_t blk, const uint32_t *hs, const uint32_t *hl,
                                       KmGeo<K> &g) {
    const uint32_t job = blk / (rs.nspl_max + 1u);
    g.obase = km_rb(rs, job, 0);
    g.pk[0] = 0;
#pragma unroll
    for (int q = 0; q < K; ++q) {
        const uint32_t sq = hs[q];
        g.pk[q + 1] = g.pk[q] + hl[q];
        g.sh[q] = sq - g.pk[q];
        g.obase += sq - km_rb(rs, job, q);
    }
}

template <int K, int LPT>
__device__ __forceinline__ void km_load(const uint32_t *__restrict__ in, const KmGeo<K> &g, uint32_t tid,
                                        uint32_t (&v)[LPT]) {
    const uint32_t B = g.pk[K];
#pragma unroll
    for (int j = 0; j < LPT; ++j) {
        const uint32_t i = tid + (uint32_t)j * KM_BLOCK;
        uint32_t s0 = g.sh[0];
#pragma unroll
        for (int r = 1; r < K; ++r) s0 = i >= g.pk[r] ? g.sh[r] : s0;
        v[j] = i < B ? in[i + s0] : 0u;
    }
}

template <int K>
__global__ __launch_bounds__(KM_BLOCK) void k_km_blocks_p(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                        KmRuns rs, const uint32_t *__restrict__ cuts, uint32_t flip,
                                                        uint32_t nblk) {
    constexpr int LPT = (KM_BMAX(K) + KM_BLOCK - 1) / KM_BLOCK;
    __shared__ uint32_t buf[2][KM_BMAX(K) + KM_BMAX(K) / 32];
    __shared__ uint32_t s_hs[2][K], s_hl[2][K];  // slice headers of the next two blocks
    const uint32_t tid = threadIdx.x, G = gridDim.x;
    uint32_t blk = blockIdx.x;
    if (blk >= nblk) return;
    if (tid < (uint32_t)K) {
        uint32_t a, l;
        km_hdr<K>(rs, cuts, blk, tid, a, l);
        s_hs[0][tid] = a;
        s_hl[0][tid] = l;
        if (blk + G < nblk) {
            km_hdr<K>(rs, cuts, blk + G, tid, a, l);
            s_hs[1][tid] = a;
            s_hl[1][tid] = l;
        }
    }
    __syncthreads();
    KmGeo<K> g;
    km_geo<K>(rs, blk, s_hs[0], s_hl[0], g);
    uint32_t v[LPT];
    km_load<K, LPT>(in, g, tid, v);
    int slot = 0;  // header slot of blk; blk + G's is slot ^ 1
    for (;;) {
        const uint32_t B = g.pk[K];
#pragma unroll
        for (int j = 0; j < LPT; ++j) {
            const uint32_t i = tid + (uint32_t)j * KM_BLOCK;
            if (i < B) buf[0][km_pad(i)] = v[j];
        }
        __syncthreads();  // buf[0] holds blk; s_hs/s_hl[slot ^ 1] hold blk + G
        const uint32_t nb = blk + G;
        const bool has_next = nb < nblk;
        KmGeo<K> gn = g;
        if (has_next) {
            km_geo<K>(rs, nb, s_hs[slot ^ 1], s_hl[slot ^ 1], gn);
            km_load<K, LPT>(in, gn, tid, v);  // in flight during the merge below
        }
        uint32_t ha = 0, hl = 0;
        const bool hh = tid < (uint32_t)K && nb + G < nblk;
        if (hh) km_hdr<K>(rs, cuts, nb + G, tid, ha, hl);
        // log2(K) LDS merge levels (as in k_km_blocks)
        const uint32_t E = ((B + KM_BLOCK - 1) / KM_BLOCK + 7u) & ~7u;
        int cur = 0;
#pragma unroll
        for (int w = 1; w < K; w <<= 1) {
            const uint32_t *s = buf[cur];
            uint32_t *d = buf[cur ^ 1];
            uint32_t pos = tid * E;
            const uint32_t p1 = pos + E < B ? pos + E : B;
            while (pos < p1) {
                uint32_t xs = 0, xm = g.pk[w], ye = g.pk[2 * w];
#pragma unroll
                for (int r = 1; r < K / (2 * w); ++r)
                    if (pos >= g.pk[r * 2 * w]) {
                        xs = g.pk[r * 2 * w];
                        xm = g.pk[r * 2 * w + w];
                        ye = g.pk[(r + 1) * 2 * w];
                    }
                const uint32_t lx = xm - xs, ly = ye - xm;
                const uint32_t end = p1 < ye ? p1 : ye;
                for (; pos < end; pos += 8) {
                    const uint32_t diag = pos - xs, cnt = end - pos < 8 ? end - pos : 8;
                    uint32_t lo = diag > ly ? diag - ly : 0u, hi = diag < lx ? diag : lx;
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (km_le(s[km_pad(xs + mid)], s[km_pad(xm + diag - mid - 1)], flip)) lo = mid + 1;
                        else hi = mid;
                    }
                    const uint32_t i = lo, jj = diag - lo;
                    uint32_t r8[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const uint32_t xv = i + k < lx ? s[km_pad(xs + i + k)] ^ flip : 0xFFFFFFFFu;
                        const uint32_t yv = jj + 7 - k < ly ? s[km_pad(xm + jj + 7 - k)] ^ flip : 0xFFFFFFFFu;
                        r8[k] = xv < yv ? xv : yv;
                    }
#pragma unroll
                    for (int dd = 4; dd >= 1; dd >>= 1)
#pragma unroll
                        for (int k = 0; k < 8; ++k)
                            if ((k & dd) == 0) {
                                const uint32_t a = r8[k], b2 = r8[k + dd];
                                r8[k] = a < b2 ? a : b2;
                                r8[k + dd] = a < b2 ? b2 : a;
                            }
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if ((uint32_t)k < cnt) d[km_pad(pos + k)] = r8[k] ^ flip;
                }
                pos = end;
            }
            __syncthreads();
            cur ^= 1;
        }
        if (hh) {  // blk's header slot is free: its geometry is in registers
            s_hs[slot][tid] = ha;
            s_hl[slot][tid] = hl;
        }
        {
            uint32_t *__restrict__ o = out + g.obase;
            const uint32_t *f = buf[cur];
#pragma unroll 4
            for (uint32_t i = tid; i < B; i += KM_BLOCK) o[i] = f[km_pad(i)];
        }
        if (!has_next) break;
        __syncthreads();  // the output reads are done before buf[0] is refilled
        g = gn;
        blk = nb;
        slot ^= 1;
    }
}

// ---------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------
size_t km_sample_slots(const KmRuns &rs) {
    if (!rs.explicit_runs) return (size_t)rs.njobs * rs.K * (rs.run / KM_S);
    size_t t = 0;
    for (uint32_t q = 0; q < rs.K; ++q) t += (rs.offs[q + 1] - rs.offs[q] + KM_S - 1) / KM_S;
    return t;
}

// splitters of the job with the most samples (uniform: a full job)
static uint32_t km_nspl_max(const KmRuns &rs) {
    size_t ts = 0;
    if (!rs.explicit_runs) {
        ts = (size_t)rs.K * (rs.run / KM_S);
    } else {
        ts = km_sample_slots(rs);
    }
    return (uint32_t)((ts + KM_M - 1) / KM_M);
}

size_t km_workspace_words(size_t n) {
    // sample slots: uniform passes njobs * K * run / KM_S <= n / KM_S + K * run / KM_S
    // <= 3 n / KM_S (K * run < 2 n); explicit runs <= n / KM_S + K.
    // cuts: njobs * nspl_max * K <= (3 n / (KM_S * KM_M) + n / KM_S + 1) * 8
    const size_t slots = 3 * (n / KM_S) + 64;
    return slots + (4 * (n / (KM_S * KM_M)) + n / KM_S + 64) * 8;
}

hipError_t launch_kmerge(const uint32_t *in, uint32_t *out, KmRuns rs, uint32_t flip, uint32_t *ws, hipStream_t s) {
    if (rs.K != 2 && rs.K != 4 && rs.K != 8) return hipErrorInvalidValue;
    if (!rs.explicit_runs && (rs.run % KM_S) != 0) return hipErrorInvalidValue;
    rs.nspl_max = km_nspl_max(rs);
    const size_t slots = km_sample_slots(rs);
    uint32_t *samp = ws, *cuts = ws + slots;
    const unsigned gs = (unsigned)((slots + 255) / 256 < 8192 ? (slots + 255) / 256 : 8192);
    if (slots) {
        k_km_samples<<<gs ? gs : 1, 256, 0, s>>>(in, rs, samp, (uint32_t)slots);
        switch (rs.K) {
        case 2: k_km_split<2><<<gs ? gs : 1, 256, 0, s>>>(in, rs, samp, (uint32_t)slots, cuts, flip); break;
        case 4: k_km_split<4><<<gs ? gs : 1, 256, 0, s>>>(in, rs, samp, (uint32_t)slots, cuts, flip); break;
        default: k_km_split<8><<<gs ? gs : 1, 256, 0, s>>>(in, rs, samp, (uint32_t)slots, cuts, flip); break;
        }
    }
    const size_t grid = (size_t)rs.njobs * (rs.nspl_max + 1);
    if (grid == 0) return hipGetLastError();
    if (KM_PERSIST) {
        // persistent grid: as many workgroups as fit on the chip (LDS-bound), at most one per block
        static int cus = 0;
        if (!cus) {
            int dev = 0;
            if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        }
        static int fit[9] = {0};
        if (!fit[rs.K]) {
            hipError_t e = hipSuccess;
            switch (rs.K) {
            case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&fit[2], k_km_blocks_p<2>, KM_BLOCK, 0); break;
            case 4: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&fit[4], k_km_blocks_p<4>, KM_BLOCK, 0); break;
            default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&fit[8], k_km_blocks_p<8>, KM_BLOCK, 0); break;
            }
            if (e != hipSuccess || fit[rs.K] <= 0) fit[rs.K] = 1;
        }
        size_t g = (size_t)cus * (size_t)fit[rs.K] * (size_t)KM_PERSIST_OVER;
        if (g > grid) g = grid;
        switch (rs.K) {
        case 2: k_km_blocks_p<2><<<(unsigned)g, KM_BLOCK, 0, s>>>(in, out, rs, cuts, flip, (uint32_t)grid); break;
        case 4: k_km_blocks_p<4><<<(unsigned)g, KM_BLOCK, 0, s>>>(in, out, rs, cuts, flip, (uint32_t)grid); break;
        default: k_km_blocks_p<8><<<(unsigned)g, KM_BLOCK, 0, s>>>(in, out, rs, cuts, flip, (uint32_t)grid); break;
        }
        return hipGetLastError();
    }
    switch (rs.K) {
    case 2: k_km_blocks<2><<<(unsigned)grid, KM_BLOCK, 0, s>>>(in, out, rs, cuts, flip); break;
    case 4: k_km_blocks<4><<<(unsigned)grid, KM_BLOCK, 0, s>>>(in, out, rs, cuts, flip); break;
    default: k_km_blocks<8><<<(unsigned)grid, KM_BLOCK, 0, s>>>(in, out, rs, cuts, flip); break;
    }
    return hipGetLastError();
}

}  // namespace labsort
