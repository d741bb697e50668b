// write_probe.hip -- the store side of the headline pass: can a
// streaming 1 GiB fill reach the guide's 6.0-6.2 TB/s plain-store figure
// (MI355X_MICROARCH.md, "plain stores of the same shape") on this pool, and which store
// form gets closest?  Standalone, no labsort code.  For n = 2^28 uint32 words (1 GiB) it
// times (median of 7 event-timed launches, after 2 warm-ups):
//   fill  W B per lane (4 / 8 / 16), flavour plain / nt (__builtin_nontemporal_store) /
//         agent-scope relaxed atomic store (sc1; 4-B only), U stores in flight per thread
//         (1 / 2 / 4 / 8), grid-stride or tiled (each workgroup writes contiguous 64 KiB
//         tiles, the onesweep pass's output shape), workgroups per CU 1..8
//   copy  the tiled 16-B copy (read + write, labsort_copy's shape) and a tiled 16-B
//         read-only reduction beside them, for the same launch geometry
// Output: one line per variant, "name ms GB/s".
// Build: hipcc --offload-arch=gfx950 -O3 -o write_probe write_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);       \
            return 1;                                                              \
        }                                                                          \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

enum { PLAIN = 0, NT = 1, SC1 = 2 };

template <typename T>
__device__ __forceinline__ T mk(uint32_t v);
template <>
__device__ __forceinline__ uint32_t mk<uint32_t>(uint32_t v) { return v; }
template <>
__device__ __forceinline__ u32x2 mk<u32x2>(uint32_t v) { return u32x2{v, v + 1u}; }
template <>
__device__ __forceinline__ u32x4 mk<u32x4>(uint32_t v) { return u32x4{v, v + 1u, v + 2u, v + 3u}; }

template <int F, typename T>
__device__ __forceinline__ void st(T *p, T v) {
    if constexpr (F == NT) __builtin_nontemporal_store(v, p);
    else if constexpr (F == SC1 && sizeof(T) == 4) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

// grid-stride: U elements of type T per thread per step, the U stores of a step one grid
// stride apart
template <typename T, int F, int U>
__global__ __launch_bounds__(256) void k_fill_gs(T *b, size_t ne, uint32_t seed) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < ne; i += U * stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) st<F>(b + i + u * stride, mk<T>(seed ^ (uint32_t)(i + u * stride)));
    }
    for (; i < ne; i += stride) st<F>(b + i, mk<T>(seed ^ (uint32_t)i));
}

// tiled: each workgroup of NT_ threads writes whole 65536-B tiles in turn (tile t of
// gridDim-strided tiles), each thread TPT elements of T per tile at thread + j * NT_
template <typename T, int F, int NTH>
__global__ __launch_bounds__(NTH) void k_fill_tile(T *b, uint32_t ntiles, uint32_t seed) {
    constexpr int PER = 65536 / (int)sizeof(T) / NTH;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        T *d = b + (size_t)t * (65536 / sizeof(T)) + threadIdx.x;
#pragma unroll
        for (int j = 0; j < PER; ++j) st<F>(d + j * NTH, mk<T>(seed ^ (t * 65536u + threadIdx.x + j * NTH)));
    }
}

template <int F, int NTH>
__global__ __launch_bounds__(NTH) void k_copy_tile(const u32x4 *a, u32x4 *b, uint32_t ntiles) {
    constexpr int PER = 4096 / NTH;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const u32x4 *s = a + (size_t)t * 4096 + threadIdx.x;
        u32x4 k[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) k[j] = F == NT ? __builtin_nontemporal_load(s + j * NTH) : s[j * NTH];
        u32x4 *d = b + (size_t)t * 4096 + threadIdx.x;
#pragma unroll
        for (int j = 0; j < PER; ++j) st<F>(d + j * NTH, k[j]);
    }
}

template <int NTH>
__global__ __launch_bounds__(NTH) void k_read_tile(const u32x4 *a, uint32_t ntiles, uint32_t *sink) {
    constexpr int PER = 4096 / NTH;
    uint32_t acc = 0;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const u32x4 *s = a + (size_t)t * 4096 + threadIdx.x;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const u32x4 v = __builtin_nontemporal_load(s + j * NTH);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const size_t n = (size_t)1 << 28, bytes = n * 4;
    const uint32_t ntiles = (uint32_t)(bytes / 65536);
    uint32_t *a = nullptr, *b = nullptr, *sink = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, bytes));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const std::function<void()> &f) {
        f();
        f();
        std::vector<float> ts;
        for (int r = 0; r < 7; ++r) {
            (void)hipEventRecord(e0, 0);
            f();
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        return ts[3];
    };
    auto line = [&](const char *name, float ms, double moved) {
        printf("%-34s %.4f ms %8.1f GB/s\n", name, ms, moved / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    char nm[96];
    printf("CUs %d, fill 1 GiB / copy 1 GiB in + 1 GiB out\n", cus);
    // grid-stride fills: width x flavour x stores in flight, 8 x 256-thread workgroups per CU
    const unsigned g8 = 8u * cus;
#define GS(T, F, U, FN)                                                                          \
    snprintf(nm, sizeof nm, "fill-gs w%zu %s u%d", sizeof(T), FN, U);                            \
    line(nm, timeit([&] { k_fill_gs<T, F, U><<<g8, 256>>>((T *)b, bytes / sizeof(T), 7u); }), (double)bytes);
    GS(uint32_t, PLAIN, 1, "plain") GS(uint32_t, PLAIN, 4, "plain") GS(uint32_t, NT, 4, "nt") GS(uint32_t, SC1, 4, "sc1")
    GS(u32x2, PLAIN, 4, "plain") GS(u32x2, NT, 4, "nt")
    GS(u32x4, PLAIN, 1, "plain") GS(u32x4, PLAIN, 2, "plain") GS(u32x4, PLAIN, 4, "plain") GS(u32x4, PLAIN, 8, "plain")
    GS(u32x4, NT, 1, "nt") GS(u32x4, NT, 4, "nt") GS(u32x4, NT, 8, "nt")
    // grid-stride 16-B fills at other occupancies
    for (unsigned per : {1u, 2u, 4u, 16u, 32u}) {
        snprintf(nm, sizeof nm, "fill-gs w16 plain u4 wg/CU %u", per);
        line(nm, timeit([&] { k_fill_gs<u32x4, PLAIN, 4><<<per * cus, 256>>>((u32x4 *)b, bytes / 16, 7u); }), (double)bytes);
        snprintf(nm, sizeof nm, "fill-gs w16 nt u4 wg/CU %u", per);
        line(nm, timeit([&] { k_fill_gs<u32x4, NT, 4><<<per * cus, 256>>>((u32x4 *)b, bytes / 16, 7u); }), (double)bytes);
    }
    // tiled fills (contiguous 64 KiB per workgroup and step), 1024 / 256 threads
#define TL(T, F, NTH, PER, FN)                                                                          \
    snprintf(nm, sizeof nm, "fill-tile w%zu %s t%d wg/CU %d", sizeof(T), FN, NTH, PER);                 \
    line(nm, timeit([&] { k_fill_tile<T, F, NTH><<<PER * cus, NTH>>>((T *)b, ntiles, 7u); }), (double)bytes);
    TL(uint32_t, PLAIN, 1024, 1, "plain") TL(uint32_t, NT, 1024, 1, "nt")
    TL(u32x4, PLAIN, 1024, 1, "plain") TL(u32x4, NT, 1024, 1, "nt") TL(u32x4, PLAIN, 1024, 2, "plain")
    TL(u32x4, NT, 1024, 2, "nt") TL(u32x4, PLAIN, 256, 4, "plain") TL(u32x4, NT, 256, 4, "nt")
    TL(u32x4, PLAIN, 256, 8, "plain") TL(u32x4, NT, 256, 8, "nt")
    // copies and reads of the same tile shape
#define CP(F, NTH, PER, FN)                                                                             \
    snprintf(nm, sizeof nm, "copy-tile w16 %s t%d wg/CU %d", FN, NTH, PER);                            \
    line(nm, timeit([&] { k_copy_tile<F, NTH><<<PER * cus, NTH>>>((const u32x4 *)a, (u32x4 *)b, ntiles); }), 2.0 * bytes);
    CP(PLAIN, 1024, 1, "plain") CP(NT, 1024, 1, "nt") CP(NT, 1024, 2, "nt") CP(NT, 256, 4, "nt") CP(NT, 256, 8, "nt")
    for (int per : {1, 2, 4}) {
        snprintf(nm, sizeof nm, "read-tile w16 nt t1024 wg/CU %d", per);
        line(nm, timeit([&] { k_read_tile<1024><<<per * cus, 1024>>>((const u32x4 *)a, ntiles, sink); }), (double)bytes);
    }
    snprintf(nm, sizeof nm, "hipMemsetD32 1 GiB");
    line(nm, timeit([&] { (void)hipMemsetD32((hipDeviceptr_t)b, 7u, n); }), (double)bytes);
    snprintf(nm, sizeof nm, "hipMemcpy D2D 1 GiB");
    line(nm, timeit([&] { (void)hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); }), 2.0 * bytes);
    CK(hipDeviceSynchronize());
    return 0;
}
