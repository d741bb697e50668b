// mg_probe.hip -- the merge pass's memory shape without its merge (r4 experiment).
// Standalone: n = 2^28 uint32 words, pairs of runs of RUN words.  Each 4096-word output
// tile reads two 2048-word segments (A at pb + (o-pb)/2, B at pb + RUN + (o-pb)/2: the
// co-ranks of a balanced merge of uniform keys) and writes 4096 words.  Skeleton of
// k_merge_pass_p: 512 threads, 32 consecutive tiles per workgroup, the next tile's keys
// prefetched into registers, the current tile staged through LDS, each thread's 8
// consecutive outputs stored as two 16-B stores.  The merge itself is replaced by reading
// the thread's 8 consecutive staged words, so the time is the memory shape alone.
//   LD4   4-B loads (as the product)      LD16  16-B loads (segments 16-B aligned here)
//   NOLDS no LDS round trip: loads go straight to the stores (pure two-stream copy)
// Build: hipcc --offload-arch=gfx950 -O3 -o mg_probe mg_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);             \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

constexpr uint32_t BLOCK = 512, KPT = 8, T = BLOCK * KPT, HALF = T / 2;

// VEC: 0 = 4-B loads, 1 = 16-B loads; STAGE: stage through LDS; NT: nontemporal loads
template <int VEC, int STAGE, int NT>
__global__ __launch_bounds__(BLOCK) void k_shape(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                                 uint32_t ntiles, uint32_t m, uint32_t run) {
    __shared__ uint32_t sm[T];
    const uint32_t tid = threadIdx.x;
    const uint32_t t0 = blockIdx.x * m;
    if (t0 >= ntiles) return;
    const uint32_t t1 = min(t0 + m, ntiles);
    auto seg = [&](uint32_t t, uint32_t &sa, uint32_t &sb) {
        const uint32_t o = t * T, pb = (o / (2u * run)) * (2u * run), h = (o - pb) / 2u;
        sa = pb + h;
        sb = pb + run + h;
    };
    uint32_t nx[KPT];
    auto load = [&](uint32_t t) {
        uint32_t sa, sb;
        seg(t, sa, sb);
        if constexpr (VEC) {
            // 1024 uint4: the first 512 from A, the rest from B; thread tid takes uint4 tid and tid + 512
            const uint4 *a4 = reinterpret_cast<const uint4 *>(src + sa), *b4 = reinterpret_cast<const uint4 *>(src + sb);
            uint4 x, y;
            if constexpr (NT) {
                typedef uint32_t v4 __attribute__((ext_vector_type(4)));
                const v4 p = __builtin_nontemporal_load(reinterpret_cast<const v4 *>(a4 + tid));
                const v4 q = __builtin_nontemporal_load(reinterpret_cast<const v4 *>(b4 + tid));
                x = make_uint4(p.x, p.y, p.z, p.w);
                y = make_uint4(q.x, q.y, q.z, q.w);
            } else {
                x = a4[tid];
                y = b4[tid];
            }
            nx[0] = x.x; nx[1] = x.y; nx[2] = x.z; nx[3] = x.w;
            nx[4] = y.x; nx[5] = y.y; nx[6] = y.z; nx[7] = y.w;
        } else {
#pragma unroll
            for (int j = 0; j < (int)KPT; ++j) {
                const uint32_t k = tid + (uint32_t)j * BLOCK;
                const uint32_t a = k < HALF ? sa + k : sb + (k - HALF);
                nx[j] = NT ? __builtin_nontemporal_load(src + a) : src[a];
            }
        }
    };
    load(t0);
    for (uint32_t t = t0; t < t1; ++t) {
        uint32_t r[KPT];
        if constexpr (STAGE) {
            __syncthreads();
            if constexpr (VEC) {
                // uint4 tid -> words 4*tid..; uint4 tid+512 -> words 2048 + 4*tid..
                reinterpret_cast<uint4 *>(sm)[tid] = make_uint4(nx[0], nx[1], nx[2], nx[3]);
                reinterpret_cast<uint4 *>(sm)[tid + BLOCK] = make_uint4(nx[4], nx[5], nx[6], nx[7]);
            } else {
#pragma unroll
                for (int j = 0; j < (int)KPT; ++j) sm[tid + (uint32_t)j * BLOCK] = nx[j];
            }
            if (t + 1 < t1) load(t + 1);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < (int)KPT; ++j) r[j] = sm[tid * KPT + (uint32_t)j];
        } else {
#pragma unroll
            for (int j = 0; j < (int)KPT; ++j) r[j] = nx[j];
            if (t + 1 < t1) load(t + 1);
        }
        uint4 *o4 = reinterpret_cast<uint4 *>(dst + (size_t)t * T + tid * KPT);
        o4[0] = make_uint4(r[0], r[1], r[2], r[3]);
        o4[1] = make_uint4(r[4], r[5], r[6], r[7]);
    }
}

// k_merge_pass_p's loop with the merge replaced by a dependent chain of 20 LDS reads
// (COMPUTE, a stand-in for its co-rank search and 8-step merge) and three store timings:
//   DEFER 0: the tile's two 16-B stores at the end of its iteration, as the product: the
//            next iteration's wait for its prefetched keys (vmcnt(0)) also waits for them
//   DEFER 1: results kept in registers, stored right after the next iteration's wait, so
//            each store has a whole iteration to complete
//   DEFER 2: results staged in a second LDS buffer, stored (coalesced) after that wait
template <int DEFER, int COMPUTE>
__global__ __launch_bounds__(BLOCK) void k_defer(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                                 uint32_t ntiles, uint32_t m, uint32_t run) {
    __shared__ uint32_t sm[T];
    __shared__ uint32_t so[DEFER == 2 ? T + T / 32 : 1];
    const uint32_t tid = threadIdx.x;
    const uint32_t t0 = blockIdx.x * m;
    if (t0 >= ntiles) return;
    const uint32_t t1 = min(t0 + m, ntiles);
    uint32_t nx[KPT];
    auto load = [&](uint32_t t) {
        const uint32_t o = t * T, pb = (o / (2u * run)) * (2u * run), h = (o - pb) / 2u;
        const uint32_t sa = pb + h, sb = pb + run + h;
#pragma unroll
        for (int j = 0; j < (int)KPT; ++j) {
            const uint32_t k = tid + (uint32_t)j * BLOCK;
            nx[j] = src[k < HALF ? sa + k : sb + (k - HALF)];
        }
    };
    load(t0);
    uint32_t r[KPT];
    uint32_t prev = ~0u;  // tile whose results wait to be stored (DEFER)
    for (uint32_t t = t0; t < t1; ++t) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < (int)KPT; ++j) sm[tid + (uint32_t)j * BLOCK] = nx[j];
        if (DEFER == 1 && prev != ~0u) {
            uint4 *o4 = reinterpret_cast<uint4 *>(dst + (size_t)prev * T + tid * KPT);
            o4[0] = make_uint4(r[0], r[1], r[2], r[3]);
            o4[1] = make_uint4(r[4], r[5], r[6], r[7]);
        }
        if (DEFER == 2 && prev != ~0u) {
#pragma unroll
            for (int j = 0; j < (int)KPT; ++j) {
                const uint32_t i = tid + (uint32_t)j * BLOCK;
                dst[(size_t)prev * T + i] = so[i + (i >> 5)];
            }
        }
        if (t + 1 < t1) load(t + 1);
        __syncthreads();
        uint32_t x = tid;
        if (COMPUTE) {
#pragma unroll
            for (int i = 0; i < 20; ++i) x = sm[(x * 2654435761u + (uint32_t)i) & (T - 1)];
        }
#pragma unroll
        for (int j = 0; j < (int)KPT; ++j) r[j] = sm[tid * KPT + (uint32_t)j];
        r[0] += (x == 0xFFFFFFFFu);
        if (DEFER == 0) {
            uint4 *o4 = reinterpret_cast<uint4 *>(dst + (size_t)t * T + tid * KPT);
            o4[0] = make_uint4(r[0], r[1], r[2], r[3]);
            o4[1] = make_uint4(r[4], r[5], r[6], r[7]);
        }
        if (DEFER == 2) {
#pragma unroll
            for (int j = 0; j < (int)KPT; ++j) {
                const uint32_t idx = tid * KPT + (uint32_t)j;
                so[idx + (idx >> 5)] = r[j];
            }
        }
        prev = t;
    }
    if (DEFER == 1 && prev != ~0u) {
        uint4 *o4 = reinterpret_cast<uint4 *>(dst + (size_t)prev * T + tid * KPT);
        o4[0] = make_uint4(r[0], r[1], r[2], r[3]);
        o4[1] = make_uint4(r[4], r[5], r[6], r[7]);
    }
    if (DEFER == 2 && prev != ~0u) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < (int)KPT; ++j) {
            const uint32_t i = tid + (uint32_t)j * BLOCK;
            dst[(size_t)prev * T + i] = so[i + (i >> 5)];
        }
    }
}

// store shapes of the merge tile (4-B loads, LDS staging as k_shape<0,1,0>):
//   ST 0: thread tid stores its 8 consecutive outputs as two 16-B stores at 32-B lane
//         stride (each wave-store covers every other 16 B of 2 KB)
//   ST 1: lane-contiguous 16-B stores: wave-store j of a wave writes 1 KB contiguously
//         (outputs 4*(tid + 512 j) .. +3, read from LDS in that order)
//   NTS: nontemporal stores
template <int ST, int NTS>
__global__ __launch_bounds__(BLOCK) void k_store(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                                 uint32_t ntiles, uint32_t m, uint32_t run) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    __shared__ uint32_t sm[T];
    const uint32_t tid = threadIdx.x;
    const uint32_t t0 = blockIdx.x * m;
    if (t0 >= ntiles) return;
    const uint32_t t1 = min(t0 + m, ntiles);
    uint32_t nx[KPT];
    auto load = [&](uint32_t t) {
        const uint32_t o = t * T, pb = (o / (2u * run)) * (2u * run), h = (o - pb) / 2u;
        const uint32_t sa = pb + h, sb = pb + run + h;
#pragma unroll
        for (int j = 0; j < (int)KPT; ++j) {
            const uint32_t k = tid + (uint32_t)j * BLOCK;
            nx[j] = src[k < HALF ? sa + k : sb + (k - HALF)];
        }
    };
    load(t0);
    for (uint32_t t = t0; t < t1; ++t) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < (int)KPT; ++j) sm[tid + (uint32_t)j * BLOCK] = nx[j];
        if (t + 1 < t1) load(t + 1);
        __syncthreads();
        v4 w[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint32_t base = ST == 0 ? tid * KPT + 4u * (uint32_t)q : 4u * (tid + (uint32_t)q * BLOCK);
            w[q] = v4{sm[base], sm[base + 1], sm[base + 2], sm[base + 3]};
        }
        v4 *o4 = reinterpret_cast<v4 *>(dst + (size_t)t * T);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint32_t at = ST == 0 ? 2u * tid + (uint32_t)q : tid + (uint32_t)q * BLOCK;
            if (NTS) __builtin_nontemporal_store(w[q], o4 + at);
            else o4[at] = w[q];
        }
    }
}
// the library's streaming copy (k_stream_copy: 16-B nontemporal, 4096 uint4 per tile,
// one 1024-thread workgroup per CU)
__global__ __launch_bounds__(1024) void k_libcopy(const uint4 *a, uint4 *b, size_t n4) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    const size_t ntiles = n4 / 4096;
    const v4 *a4 = reinterpret_cast<const v4 *>(a);
    v4 *b4 = reinterpret_cast<v4 *>(b);
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        v4 k[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) k[j] = __builtin_nontemporal_load(a4 + t * 4096 + threadIdx.x + j * 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(k[j], b4 + t * 4096 + threadIdx.x + j * 1024);
    }
}

template <class F>
static float timeit(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::vector<float> ts;
    for (int r = 0; r < 12; ++r) {
        hipEventRecord(a);
        f();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (r >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    const size_t n = (size_t)1 << 28;
    const uint32_t ntiles = (uint32_t)(n / T);
    uint32_t *in, *out;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMemset(in, 1, n * 4));
    const double gb = 8.0 * n / 1e9;
    {
        float t = timeit([&] { k_libcopy<<<256, 1024>>>((const uint4 *)in, (uint4 *)out, n / 4); });
        printf("libcopy               %.4f ms %7.1f GB/s\n", t, gb / t * 1e3);
        for (uint32_t grid : {2048u, 1024u}) {
            const uint32_t m = (ntiles + grid - 1) / grid, run = 1u << 20;
#define STO(S, N)                                                                                     \
    t = timeit([&] { k_store<S, N><<<grid, BLOCK>>>(in, out, ntiles, m, run); });                    \
    printf("store %d nt %d grid %4u   %.4f ms %7.1f GB/s\n", S, N, grid, t, gb / t * 1e3);
            STO(0, 0) STO(1, 0) STO(0, 1) STO(1, 1)
        }
    }
    if (getenv("MG_ALL") == nullptr) {
        CK(hipDeviceSynchronize());
        return 0;
    }
    for (uint32_t grid : {2048u, 1024u}) {
        const uint32_t m = (ntiles + grid - 1) / grid, run = 1u << 20;
        float t;
#define DEF(D, C)                                                                                     \
    t = timeit([&] { k_defer<D, C><<<grid, BLOCK>>>(in, out, ntiles, m, run); });                    \
    printf("defer %d compute %d grid %4u  %.4f ms %7.1f GB/s\n", D, C, grid, t, gb / t * 1e3);
        DEF(0, 0) DEF(1, 0) DEF(2, 0) DEF(0, 1) DEF(1, 1) DEF(2, 1)
    }
    for (uint32_t run : {1u << 15, 1u << 20, 1u << 27}) {
        for (uint32_t grid : {1024u, 2048u, 4096u}) {
            const uint32_t m = (ntiles + grid - 1) / grid;
            float t;
            t = timeit([&] { k_shape<0, 1, 0><<<grid, BLOCK>>>(in, out, ntiles, m, run); });
            printf("run 2^%-2d grid %4u  ld4  lds    %.4f ms %7.1f GB/s\n", __builtin_ctz(run), grid, t, gb / t * 1e3);
            t = timeit([&] { k_shape<0, 1, 1><<<grid, BLOCK>>>(in, out, ntiles, m, run); });
            printf("run 2^%-2d grid %4u  ld4nt lds    %.4f ms %7.1f GB/s\n", __builtin_ctz(run), grid, t, gb / t * 1e3);
            t = timeit([&] { k_shape<1, 1, 0><<<grid, BLOCK>>>(in, out, ntiles, m, run); });
            printf("run 2^%-2d grid %4u  ld16 lds     %.4f ms %7.1f GB/s\n", __builtin_ctz(run), grid, t, gb / t * 1e3);
            t = timeit([&] { k_shape<1, 1, 1><<<grid, BLOCK>>>(in, out, ntiles, m, run); });
            printf("run 2^%-2d grid %4u  ld16nt lds   %.4f ms %7.1f GB/s\n", __builtin_ctz(run), grid, t, gb / t * 1e3);
            t = timeit([&] { k_shape<0, 0, 0><<<grid, BLOCK>>>(in, out, ntiles, m, run); });
            printf("run 2^%-2d grid %4u  ld4  nolds   %.4f ms %7.1f GB/s\n", __builtin_ctz(run), grid, t, gb / t * 1e3);
            t = timeit([&] { k_shape<1, 0, 0><<<grid, BLOCK>>>(in, out, ntiles, m, run); });
            printf("run 2^%-2d grid %4u  ld16 nolds   %.4f ms %7.1f GB/s\n", __builtin_ctz(run), grid, t, gb / t * 1e3);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
