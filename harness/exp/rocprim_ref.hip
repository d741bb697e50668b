// rocprim_ref.hip -- library baseline on the same box (not product code): rocPRIM's
// device radix sort (onesweep) and merge sort of n uniform uint32 keys, device-resident,
// timed with HIP events, plus a device-to-device memcpy of the same bytes for scale.
//   rocprim_ref [log2n=28] [reps=10]
// Output: one JSON line.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 rocprim_ref.hip -o ../bin/rocprim_ref
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_merge_sort.hpp>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

__global__ void k_gen(uint32_t *out, size_t n, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        out[i] = (uint32_t)((z ^ (z >> 31)) >> 32);
    }
}
__global__ void k_desc(const uint32_t *a, size_t n, unsigned long long *cnt) {
    unsigned long long c = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i + 1 < n; i += (size_t)gridDim.x * blockDim.x)
        c += a[i] > a[i + 1];
    if (c) atomicAdd(cnt, c);
}

template <class F>
static float time_ms(F f, int reps, hipStream_t s) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();  // warm-up
    f();
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char **argv) {
    const int lg = argc > 1 ? std::atoi(argv[1]) : 28;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 10;
    const size_t n = (size_t)1 << lg;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    uint32_t *in, *out;
    unsigned long long *cnt;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&cnt, 8));
    k_gen<<<4096, 256, 0, s>>>(in, n, 0x5EED0003ull);
    CK(hipGetLastError());

    size_t tb = 0;
    CK(rocprim::radix_sort_keys(nullptr, tb, in, out, n, 0, 32, s));
    void *tmp;
    size_t tbm = 0;
    CK(rocprim::merge_sort(nullptr, tbm, in, out, n, rocprim::less<uint32_t>(), s));
    CK(hipMalloc(&tmp, tb > tbm ? tb : tbm));
    auto check = [&](const char *who) {
        CK(hipMemsetAsync(cnt, 0, 8, s));
        k_desc<<<4096, 256, 0, s>>>(out, n, cnt);
        unsigned long long h = 1;
        CK(hipMemcpyAsync(&h, cnt, 8, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        if (h) {
            std::fprintf(stderr, "%s: %llu descents\n", who, h);
            std::exit(2);
        }
    };
    const float t_radix = time_ms([&] { (void)rocprim::radix_sort_keys(tmp, tb, in, out, n, 0, 32, s); }, reps, s);
    check("radix_sort_keys");
    const float t_merge = time_ms([&] { (void)rocprim::merge_sort(tmp, tbm, in, out, n, rocprim::less<uint32_t>(), s); },
                                  reps, s);
    check("merge_sort");
    const float t_copy = time_ms([&] { CK(hipMemcpyAsync(out, in, n * 4, hipMemcpyDeviceToDevice, s)); }, reps, s);
    std::printf("{\"n\": %zu, \"rocprim_version\": %d, \"radix_sort_keys_ms\": %.4f, \"radix_Mkeys_s\": %.1f, "
                "\"merge_sort_ms\": %.4f, \"merge_Mkeys_s\": %.1f, \"d2d_copy_ms\": %.4f, \"d2d_copy_GBs\": %.1f}\n",
                n, ROCPRIM_VERSION, t_radix, n / t_radix / 1e3, t_merge, n / t_merge / 1e3, t_copy,
                2.0 * n * 4 / t_copy / 1e6);
    return 0;
}
