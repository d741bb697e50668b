// bw_probe.hip -- HBM ceilings for the onesweep pass's access pattern on one MI355X.
// Standalone (no labsort code): times, for n = 2^28 uint32 words (1 GiB in, 1 GiB out),
//   copy-gs     grid-stride uint4 copy
//   copy-tile   16384-word tiles per 1024-thread workgroup, dword loads/stores in the
//               onesweep pass's blocked layout (16 slots per thread)
//   read        read-only reduction (uint4)
//   write       write-only fill (uint4)
//   runs-al     tile t writes 256 runs of 64 words, run d to region d at t*64 (256-B
//               aligned): the ideal onesweep scatter
//   runs-mis    the same with every run shifted by a per-(t,d) word offset, so runs
//               straddle lines as the real scatter's do
//   runs-var    run lengths vary (uniform-key multinomial-like: 32..96 words) per tile
// Build: hipcc --offload-arch=gfx950 -O3 -o bw_probe bw_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_copy_gs(const uint4 *a, uint4 *b, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ __launch_bounds__(1024) void k_copy_tile(const uint32_t *a, uint32_t *b, uint32_t ntiles) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t *s = a + (size_t)t * 16384 + wid * 1024 + lane;
        uint32_t k[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) k[j] = s[j * 64];
        uint32_t *d = b + (size_t)t * 16384 + wid * 1024 + lane;
#pragma unroll
        for (int j = 0; j < 16; ++j) d[j * 64] = k[j];
    }
}
// copy-tile with the destination shifted by SH words: every wave store straddles
// granules (partial granules written by two stores of one workgroup, not across tiles)
template <int SH>
__global__ __launch_bounds__(1024) void k_copy_tile_sh(const uint32_t *a, uint32_t *b, uint32_t ntiles) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t *s = a + (size_t)t * 16384 + wid * 1024 + lane;
        uint32_t k[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) k[j] = s[j * 64];
        uint32_t *d = b + SH + (size_t)t * 16384 + wid * 1024 + lane;
#pragma unroll
        for (int j = 0; j < 16; ++j) d[j * 64] = k[j];
    }
}
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
// copy with U uint4 per thread per step in flight (grid-stride), optionally nontemporal
template <int U, int NT>
__global__ __launch_bounds__(256) void k_copy_u(const v4u *a, v4u *b, size_t n4) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(a + i + u * stride) : a[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], b + i + u * stride);
            else b[i + u * stride] = v[u];
        }
    }
    for (; i < n4; i += stride) b[i] = a[i];
}
// tiled copy (16384 words per 1024-thread tile) with uint4 per lane: 4 x uint4 per thread
template <int NT>
__global__ __launch_bounds__(1024) void k_copy_tile4(const v4u *a, v4u *b, uint32_t ntiles) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const v4u *s = a + (size_t)t * 4096 + tid;
        v4u k[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) k[j] = NT ? __builtin_nontemporal_load(s + j * 1024) : s[j * 1024];
        v4u *d = b + (size_t)t * 4096 + tid;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (NT) __builtin_nontemporal_store(k[j], d + j * 1024);
            else d[j * 1024] = k[j];
        }
    }
}
__global__ __launch_bounds__(256) void k_read(const uint4 *a, size_t n4, uint32_t *sink) {
    uint32_t x = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x12345678u) sink[0] = x;
}
__global__ __launch_bounds__(256) void k_write(uint4 *b, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        b[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
// abutting runs of RUN words: tile t's run for region d = [d*stride + sh_d + t*RUN, +RUN), sh_d
// a fixed per-region word shift, so consecutive tiles share each boundary line as the
// real scatter's do (SH = 0: aligned)
// XL: tiles dealt per XCD group (blockIdx % 8 = group): group g takes the g-th
// contiguous eighth of the tiles, so consecutive tiles share one L2
// SEL: stores whose 64-B granule lies inside the run are nontemporal, the run's edge
// granules (shared with the neighbouring tiles) use the default policy
// HO: handoff pattern -- each tile's run shifted down to the granule boundary, so every
// tile writes whole granules (its tail granule's words are written by the next tile)
template <int RUN, int SH, int XL = 0, int NTL = 0, int SEL = 0, int HO = 0>
__global__ __launch_bounds__(1024) void k_abut(const uint32_t *a, uint32_t *b, uint32_t ntiles) {
    const uint32_t tid = threadIdx.x;
    const size_t stride = (size_t)ntiles * RUN + 64;
    const uint32_t g = blockIdx.x & 7u, per = ntiles / 8u;
    for (uint32_t q = XL ? blockIdx.x >> 3 : blockIdx.x; q < (XL ? per : ntiles); q += XL ? gridDim.x >> 3 : gridDim.x) {
        const uint32_t t = XL ? g * per + q : q;
        uint32_t k[16];
#pragma unroll
        for (int j = 0; j < 16; ++j)
            k[j] = NTL ? __builtin_nontemporal_load(a + (size_t)t * 16384 + j * 1024 + tid) : a[(size_t)t * 16384 + j * 1024 + tid];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t i = j * 1024 + tid, d = i / RUN;
            const uint32_t sh = SH == 1 ? (d * 5u + 3u) & 31u : SH == 2 ? ((d * 5u + 3u) & 1u) * 16u : 0u;
            const size_t rs = d * stride + sh + (size_t)t * RUN, pos = rs + (i % RUN) - (HO ? (rs & 15) : 0);
            const size_t gs = pos & ~(size_t)15;
            if (SEL && gs >= rs && gs + 16 <= rs + RUN) __builtin_nontemporal_store(k[j], b + pos);
            else b[pos] = k[j];
        }
    }
}
// abutting misaligned runs (as k_abut<RUN, 1, XL>) with each granule shared by two
// tiles written once, whole, by the earlier tile (a carry handoff's store pattern):
// the head granule is skipped, the tail granule written as 4 x uint4
template <int RUN, int XL>
__global__ __launch_bounds__(1024) void k_abut_own(const uint32_t *a, uint32_t *b, uint32_t ntiles) {
    const uint32_t tid = threadIdx.x;
    const size_t stride = (size_t)ntiles * RUN + 64;
    const uint32_t g = blockIdx.x & 7u, per = ntiles / 8u;
    for (uint32_t q = XL ? blockIdx.x >> 3 : blockIdx.x; q < (XL ? per : ntiles); q += XL ? gridDim.x >> 3 : gridDim.x) {
        const uint32_t t = XL ? g * per + q : q;
        uint32_t k[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) k[j] = a[(size_t)t * 16384 + j * 1024 + tid];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t i = j * 1024 + tid, d = i / RUN;
            const uint32_t sh = (d * 5u + 3u) & 31u;
            const size_t rs = d * stride + sh + (size_t)t * RUN, pos = rs + (i % RUN);
            const size_t gs = pos & ~(size_t)15;
            if (t > 0 && gs < rs) continue;
            if (t + 1 < ntiles && gs + 16 > rs + RUN) {
                if (pos == (gs > rs ? gs : rs)) {
                    uint4 *p4 = reinterpret_cast<uint4 *>(b + gs);
                    const uint4 v = make_uint4(k[j], k[j], k[j], k[j]);
                    p4[0] = v; p4[1] = v; p4[2] = v; p4[3] = v;
                }
                continue;
            }
            b[pos] = k[j];
        }
    }
}
// runs of K consecutive tiles per workgroup (tiles dealt per XCD group as XL): the
// onesweep shape where one workgroup scatters K consecutive tiles of a chain in turn.
// CARRY: inside a workgroup's run of tiles, the granule a tile shares with the next
// tile is written once, whole, by the next tile (the tail keys carried in LDS); only
// the first tile's head and the last tile's tail granules are shared across workgroups.
// VEC: tile keys loaded as uint4 per lane (4 consecutive keys) instead of 4-B lanes.
template <int RUN, int K, int CARRY, int VEC = 0>
__global__ __launch_bounds__(1024) void k_abut_run(const uint32_t *a, uint32_t *b, uint32_t ntiles) {
    const uint32_t tid = threadIdx.x;
    const size_t stride = (size_t)ntiles * RUN + 64;
    const uint32_t g = blockIdx.x & 7u, per = ntiles / 8u, runs = per / K;
    for (uint32_t q = blockIdx.x >> 3; q < runs; q += gridDim.x >> 3) {
        for (uint32_t kk = 0; kk < (uint32_t)K; ++kk) {
            const uint32_t t = g * per + q * K + kk;
            uint32_t k[16];
            if (VEC) {
                const uint4 *src = reinterpret_cast<const uint4 *>(a + (size_t)t * 16384);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint4 v = src[j * 1024 + tid];
                    k[4 * j] = v.x; k[4 * j + 1] = v.y; k[4 * j + 2] = v.z; k[4 * j + 3] = v.w;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 16; ++j) k[j] = a[(size_t)t * 16384 + j * 1024 + tid];
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t i = j * 1024 + tid, d = i / RUN, u = i % RUN;
                const uint32_t sh = (d * 5u + 3u) & 31u;
                const size_t rs = d * stride + sh + (size_t)t * RUN, re = rs + RUN, pos = rs + u;
                if (CARRY) {
                    const size_t hi = kk + 1 < (uint32_t)K ? (re & ~(size_t)15) : re;
                    if (kk > 0 && u < (rs & 15)) b[(rs & ~(size_t)15) + u] = k[j];  // the carried head words
                    if (pos < hi) b[pos] = k[j];
                } else {
                    b[pos] = k[j];
                }
            }
        }
    }
}
// gather: the reverse shape -- output tile T is written contiguously (whole lines) and
// its keys are read as runs of RUN words from the locally sorted source tiles: logical
// position L = T*16384 + i lies in bucket d = L / (ntiles*RUN), run t (source tile t),
// word u; the run starts at a misaligned word offset inside source tile t
template <int RUN, int XL, int VEC = 0>
__global__ __launch_bounds__(1024) void k_gather(const uint32_t *a, uint32_t *b, uint32_t ntiles) {
    const uint32_t tid = threadIdx.x;
    const size_t bucket = (size_t)ntiles * RUN, tstride = 16384 + 32;
    const uint32_t g = blockIdx.x & 7u, per = ntiles / 8u;
    for (uint32_t q = XL ? blockIdx.x >> 3 : blockIdx.x; q < (XL ? per : ntiles); q += XL ? gridDim.x >> 3 : gridDim.x) {
        const uint32_t T = XL ? g * per + q : q;
        uint32_t k[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const size_t L = (size_t)T * 16384 + (VEC ? (j >> 2) * 4096 + tid * 4 + (j & 3) : j * 1024 + tid);
            const size_t d = L / bucket, r = L % bucket, t = r / RUN, u = r % RUN;
            const uint32_t sh = (uint32_t)((t * 37u + d * 11u) & 31u);
            k[j] = a[t * tstride + d * RUN + sh + u];
        }
        if (VEC) {
            uint4 *dst = reinterpret_cast<uint4 *>(b + (size_t)T * 16384);
#pragma unroll
            for (int j = 0; j < 4; ++j) dst[j * 1024 + tid] = make_uint4(k[4 * j], k[4 * j + 1], k[4 * j + 2], k[4 * j + 3]);
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) b[(size_t)T * 16384 + j * 1024 + tid] = k[j];
        }
    }
}
// padded scatter: tile t writes 256 runs of RUN words, run (t, d) at a 16-word-aligned
// slot of SLOT words (SLOT - RUN words of padding nobody writes); GATHER: the tile's
// keys are also read as runs of RUN words from such a padded layout (the next pass of
// a padded design), else read contiguously
template <int RUN, int SLOT, int GATHER>
__global__ __launch_bounds__(1024) void k_padded(const uint32_t *a, uint32_t *b, uint32_t ntiles) {
    const uint32_t tid = threadIdx.x;
    const size_t region = (size_t)ntiles * SLOT;
    const uint32_t g = blockIdx.x & 7u, per = ntiles / 8u;
    constexpr uint32_t TK = 256 * RUN;  // keys per tile
    for (uint32_t q = blockIdx.x >> 3; q < per; q += gridDim.x >> 3) {
        const uint32_t t = g * per + q;
        uint32_t k[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t i = j * 1024 + tid;
            if (i < TK) {
                if (GATHER) {
                    // logical position L = t*TK + i: bucket d = L / (ntiles*RUN), run tt, word u
                    const size_t L = (size_t)t * TK + i, d = L / ((size_t)ntiles * RUN), r = L % ((size_t)ntiles * RUN);
                    k[j] = a[d * region + (r / RUN) * SLOT + r % RUN];
                } else {
                    k[j] = a[(size_t)t * TK + i];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t i = j * 1024 + tid;
            if (i < TK) b[(i / RUN) * region + (size_t)t * SLOT + i % RUN] = k[j];
        }
    }
}
// MODE 0: aligned runs of 64; 1: runs shifted by a per-(t,d) offset (region stride has
// 64 words of slack per tile); 2: variable run lengths (lens[t*256+d], prefix offs).
template <int MODE>
__global__ __launch_bounds__(1024) void k_runs(const uint32_t *a, uint32_t *b, uint32_t ntiles,
                                              const uint32_t *offs, const uint32_t *lens) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        uint32_t k[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) k[j] = a[(size_t)t * 16384 + j * 1024 + tid];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t i = j * 1024 + tid;  // position within the tile's sorted order
            size_t dst;
            if constexpr (MODE == 0) {
                dst = (size_t)(i >> 6) * ntiles * 64 + (size_t)t * 64 + (i & 63);
            } else if constexpr (MODE == 1) {
                const uint32_t d = i >> 6;
                const uint32_t sh = (t * 37u + d * 11u) & 63u;
                dst = (size_t)d * (ntiles * 64 + 64) + (size_t)t * 64 + sh + (i & 63);
            } else {
                // run boundaries from offs (tile-local exclusive prefix of lens): binary search
                const uint32_t *o = offs + (size_t)t * 257;
                uint32_t lo = 0, hi = 256;
                while (hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if (o[m] <= i) lo = m; else hi = m; }
                dst = (size_t)lens[(size_t)t * 256 + lo] + (i - o[lo]);  // lens holds the global base here
            }
            b[dst] = k[j];
        }
    }
}

template <class F>
static float timeit(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    std::vector<float> ts;
    for (int r = 0; r < 12; ++r) {
        hipEventRecord(a);
        f();
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (r >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    const size_t n = (size_t)1 << 28;
    const uint32_t ntiles = (uint32_t)(n / 16384);
    uint32_t *in, *out, *sink, *offs, *bases;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4 + ((size_t)1 << 20)));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&offs, (size_t)ntiles * 257 * 4));
    CK(hipMalloc(&bases, (size_t)ntiles * 256 * 4));
    CK(hipMemset(in, 1, n * 4));
    // variable runs: lengths 32..96 (pseudo-random, each tile sums to 16384), bases = regions
    {
        std::vector<uint32_t> len((size_t)ntiles * 256), off((size_t)ntiles * 257), base((size_t)ntiles * 256);
        uint64_t s = 0x9E3779B97F4A7C15ull;
        for (uint32_t t = 0; t < ntiles; ++t) {
            for (int d = 0; d < 256; d += 2) {
                s = s * 6364136223846793005ull + 1442695040888963407ull;
                const uint32_t r = (uint32_t)(s >> 33) % 65;  // 0..64
                len[(size_t)t * 256 + d] = 32 + r;
                len[(size_t)t * 256 + d + 1] = 96 - r;
            }
            off[(size_t)t * 257] = 0;
            for (int d = 0; d < 256; ++d) off[(size_t)t * 257 + d + 1] = off[(size_t)t * 257 + d] + len[(size_t)t * 256 + d];
        }
        std::vector<uint64_t> tot(256, 0);
        for (uint32_t t = 0; t < ntiles; ++t)
            for (int d = 0; d < 256; ++d) tot[d] += len[(size_t)t * 256 + d];
        std::vector<uint64_t> rb(257, 0);
        for (int d = 0; d < 256; ++d) rb[d + 1] = rb[d] + tot[d];
        std::vector<uint64_t> cur(rb.begin(), rb.end() - 1);
        for (uint32_t t = 0; t < ntiles; ++t)
            for (int d = 0; d < 256; ++d) {
                base[(size_t)t * 256 + d] = (uint32_t)cur[d];
                cur[d] += len[(size_t)t * 256 + d];
            }
        CK(hipMemcpy(offs, off.data(), off.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(bases, base.data(), base.size() * 4, hipMemcpyHostToDevice));
    }
    const double gb = 8.0 * n / 1e9;
    float t;
    t = timeit([&] { k_copy_gs<<<8192, 256>>>((const uint4 *)in, (uint4 *)out, n / 4); });
    printf("copy-gs    %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    for (int g : {256, 512, 1024}) {
        t = timeit([&] { k_copy_tile<<<g, 1024>>>(in, out, ntiles); });
        printf("copy-tile  %.4f ms  %7.1f GB/s  (grid %d)\n", t, gb / t * 1e3, g);
    }
    for (int g : {1024, 2048, 4096, 8192}) {
        t = timeit([&] { k_copy_u<4, 0><<<g, 256>>>((const v4u *)in, (v4u *)out, n / 4); });
        printf("copy-u4    %.4f ms  %7.1f GB/s  (grid %d)\n", t, gb / t * 1e3, g);
        t = timeit([&] { k_copy_u<4, 1><<<g, 256>>>((const v4u *)in, (v4u *)out, n / 4); });
        printf("copy-u4nt  %.4f ms  %7.1f GB/s  (grid %d)\n", t, gb / t * 1e3, g);
    }
    t = timeit([&] { k_copy_u<8, 0><<<2048, 256>>>((const v4u *)in, (v4u *)out, n / 4); });
    printf("copy-u8    %.4f ms  %7.1f GB/s  (grid 2048)\n", t, gb / t * 1e3);
    for (int g : {256, 512, 1024}) {
        t = timeit([&] { k_copy_tile4<0><<<g, 1024>>>((const v4u *)in, (v4u *)out, ntiles); });
        printf("copy-tile4   %.4f ms  %7.1f GB/s  (grid %d)\n", t, gb / t * 1e3, g);
        t = timeit([&] { k_copy_tile4<1><<<g, 1024>>>((const v4u *)in, (v4u *)out, ntiles); });
        printf("copy-tile4nt %.4f ms  %7.1f GB/s  (grid %d)\n", t, gb / t * 1e3, g);
    }
    t = timeit([&] { k_copy_tile_sh<7><<<256, 1024>>>(in, out, ntiles); });
    printf("copy-tile+7  %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_copy_tile_sh<16><<<256, 1024>>>(in, out, ntiles); });
    printf("copy-tile+16 %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_read<<<8192, 256>>>((const uint4 *)in, n / 4, sink); });
    printf("read       %.4f ms  %7.1f GB/s\n", t, gb / 2 / t * 1e3);
    t = timeit([&] { k_write<<<8192, 256>>>((uint4 *)out, n / 4); });
    printf("write      %.4f ms  %7.1f GB/s\n", t, gb / 2 / t * 1e3);
    for (int g : {256}) {
        t = timeit([&] { k_runs<0><<<g, 1024>>>(in, out, ntiles, offs, bases); });
        printf("runs-al    %.4f ms  %7.1f GB/s  (grid %d)\n", t, gb / t * 1e3, g);
        t = timeit([&] { k_runs<1><<<g, 1024>>>(in, out, ntiles, offs, bases); });
        printf("runs-mis   %.4f ms  %7.1f GB/s  (grid %d)\n", t, gb / t * 1e3, g);
        t = timeit([&] { k_runs<2><<<g, 1024>>>(in, out, ntiles, offs, bases); });
        printf("runs-var   %.4f ms  %7.1f GB/s  (grid %d)\n", t, gb / t * 1e3, g);
    }
    t = timeit([&] { k_abut<64, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64    %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<64, 1, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64xl  %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<64, 1, 1, 0, 0, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64xl-ho %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<32, 1, 1, 0, 0, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-32xl-ho %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<64, 1, 0, 0, 0, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64-ho %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut_own<64, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64xl-own %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut_own<64, 0><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64-own %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut_own<32, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-32xl-own %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<64, 1, 1, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64xlnt %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<64, 1, 0, 0, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64sel %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<64, 1, 1, 0, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64xlsel %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<64, 1, 1, 1, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64xlselnt %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<64, 1, 0, 1, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64selnt %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<64, 2, 0><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64h   %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<64, 2, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64hxl %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<128, 1, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-128xl %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<32, 1, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-32xl  %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<64, 0><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-64al  %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<128, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-128   %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<256, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-256   %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<32, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-32    %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<16, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-16    %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<8, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-8     %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<16, 1, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-16xl  %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut<8, 1, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("abut-8xl   %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut_run<64, 1, 0><<<256, 1024>>>(in, out, ntiles); });
    printf("run-64 K1     %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut_run<64, 4, 0><<<256, 1024>>>(in, out, ntiles); });
    printf("run-64 K4     %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut_run<64, 4, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("run-64 K4c    %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut_run<64, 8, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("run-64 K8c    %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut_run<64, 16, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("run-64 K16c   %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut_run<64, 8, 0><<<256, 1024>>>(in, out, ntiles); });
    printf("run-64 K8     %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut_run<64, 1, 0, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("run-64 K1v    %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut_run<64, 8, 1, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("run-64 K8cv   %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    t = timeit([&] { k_abut_run<64, 16, 1, 1><<<256, 1024>>>(in, out, ntiles); });
    printf("run-64 K16cv  %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
    {
        uint32_t *pa, *pb;
        const size_t words = (size_t)ntiles * 256 * 80 + 4096;
        CK(hipMalloc(&pa, words * 4));
        CK(hipMalloc(&pb, words * 4));
        CK(hipMemset(pa, 1, words * 4));
        auto rate = [&](double keys, float ms) { return 8.0 * keys / 1e9 / ms * 1e3; };
        t = timeit([&] { k_padded<64, 64, 0><<<256, 1024>>>(pa, pb, ntiles); });
        printf("pad-64/64      %.4f ms  %7.1f GB/s (aligned runs, no padding)\n", t, rate(256.0 * 64 * ntiles, t));
        t = timeit([&] { k_padded<56, 64, 0><<<256, 1024>>>(pa, pb, ntiles); });
        printf("pad-56/64      %.4f ms  %7.1f GB/s (aligned runs, unshared partial tails)\n", t, rate(256.0 * 56 * ntiles, t));
        t = timeit([&] { k_padded<60, 64, 0><<<256, 1024>>>(pa, pb, ntiles); });
        printf("pad-60/64      %.4f ms  %7.1f GB/s\n", t, rate(256.0 * 60 * ntiles, t));
        t = timeit([&] { k_padded<56, 64, 1><<<256, 1024>>>(pa, pb, ntiles); });
        printf("pad-56/64 gath %.4f ms  %7.1f GB/s (padded runs gathered + padded scatter)\n", t, rate(256.0 * 56 * ntiles, t));
        t = timeit([&] { k_padded<60, 64, 1><<<256, 1024>>>(pa, pb, ntiles); });
        printf("pad-60/64 gath %.4f ms  %7.1f GB/s\n", t, rate(256.0 * 60 * ntiles, t));
        CK(hipFree(pa));
        CK(hipFree(pb));
    }
    {
        uint32_t *src2;
        CK(hipMalloc(&src2, (size_t)ntiles * (16384 + 32) * 4 + 4096));
        CK(hipMemset(src2, 1, (size_t)ntiles * (16384 + 32) * 4));
        t = timeit([&] { k_gather<64, 0><<<256, 1024>>>(src2, out, ntiles); });
        printf("gather-64     %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
        t = timeit([&] { k_gather<64, 1><<<256, 1024>>>(src2, out, ntiles); });
        printf("gather-64xl   %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
        t = timeit([&] { k_gather<64, 0, 1><<<256, 1024>>>(src2, out, ntiles); });
        printf("gather-64v    %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
        t = timeit([&] { k_gather<64, 0><<<512, 1024>>>(src2, out, ntiles); });
        printf("gather-64 g512 %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
        t = timeit([&] { k_gather<32, 0><<<256, 1024>>>(src2, out, ntiles); });
        printf("gather-32     %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
        t = timeit([&] { k_gather<32, 1><<<256, 1024>>>(src2, out, ntiles); });
        printf("gather-32xl   %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
        t = timeit([&] { k_gather<16, 1><<<256, 1024>>>(src2, out, ntiles); });
        printf("gather-16xl   %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
        t = timeit([&] { k_gather<8, 1><<<256, 1024>>>(src2, out, ntiles); });
        printf("gather-8xl    %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
        t = timeit([&] { k_gather<8, 1><<<512, 1024>>>(src2, out, ntiles); });
        printf("gather-8xl g512 %.4f ms  %7.1f GB/s\n", t, gb / t * 1e3);
        CK(hipFree(src2));
    }
    CK(hipDeviceSynchronize());
    return 0;
}
