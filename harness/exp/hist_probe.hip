// hist_probe.hip -- variants of the upfront histogram (k_hist_seg's counting) on one
// MI355X, n = 2^28 uniform uint32 keys.  Standalone (no labsort code).
//   MODE 0: loads only (read floor of this loop shape)
//   MODE 1: digit-0 counters replicated 32x only
//   MODE 2: + the three 12-bit joint fields (k_hist_seg's work)
// PIPE: next batch of 4 uint4 loaded while the current one is counted
// grid: workgroups (1024 threads), LDS 80 KB each
// Build: hipcc --offload-arch=gfx950 -O3 -o hist_probe hist_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int HB = 1024;

template <int MODE, int PIPE, int JREP>
__global__ __launch_bounds__(HB) void k_hist(const uint32_t *__restrict__ keys, size_t n, uint32_t *__restrict__ out) {
    constexpr int SL = 32, JF = 4096;
    __shared__ uint32_t h[256 * SL];
    __shared__ uint32_t hj[3 * JF * JREP];
    for (int i = threadIdx.x; i < 256 * SL; i += HB) h[i] = 0u;
    if (MODE >= 2)
        for (int i = threadIdx.x; i < 3 * JF * JREP; i += HB) hj[i] = 0u;
    __syncthreads();
    const uint32_t slot = threadIdx.x & (SL - 1);
    const uint32_t jr = JREP > 1 ? (threadIdx.x >> 6) & (JREP - 1) : 0u;  // joint replica per wave
    uint32_t x_ = 0;
    auto count = [&](uint32_t k) {
        if (MODE == 0) { x_ ^= k; return; }
        atomicAdd(&h[(k & 255u) * SL + slot], 1u);
        if (MODE >= 2) {
#pragma unroll
            for (int p = 0; p < 3; ++p) atomicAdd(&hj[(p * JF + ((k >> (8 * p + 4)) & (JF - 1))) * JREP + jr], 1u);
        }
    };
    const size_t per = n / gridDim.x;
    const uint4 *v = reinterpret_cast<const uint4 *>(keys + (size_t)blockIdx.x * per);
    const size_t nv = per / 4;
    size_t i = threadIdx.x;
    if (PIPE) {
        uint4 c[4], x[4];
        if (i + 3 * HB < nv)
#pragma unroll
            for (int u = 0; u < 4; ++u) c[u] = v[i + u * HB];
        for (; i + 3 * HB < nv; i += 4 * HB) {
            const size_t in = i + 4 * HB;
            if (in + 3 * HB < nv) {
#pragma unroll
                for (int u = 0; u < 4; ++u) x[u] = v[in + u * HB];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) { count(c[u].x); count(c[u].y); count(c[u].z); count(c[u].w); }
#pragma unroll
            for (int u = 0; u < 4; ++u) c[u] = x[u];
        }
    } else {
        for (; i + 3 * HB < nv; i += 4 * HB) {
            uint4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = v[i + u * HB];
#pragma unroll
            for (int u = 0; u < 4; ++u) { count(x[u].x); count(x[u].y); count(x[u].z); count(x[u].w); }
        }
    }
    for (; i < nv; i += HB) { const uint4 x = v[i]; count(x.x); count(x.y); count(x.z); count(x.w); }
    __syncthreads();
    if (MODE == 0) { if (x_ == 0x12345u) out[0] = x_; return; }
    for (int d = threadIdx.x; d < 256; d += HB) {
        uint32_t c = 0;
        for (int q = 0; q < SL; ++q) c += h[d * SL + ((q + d) & (SL - 1))];
        if (c) atomicAdd(&out[d], c);
    }
    if (MODE >= 2)
        for (int f = threadIdx.x; f < 3 * JF; f += HB) {
            uint32_t c = 0;
            for (int r = 0; r < JREP; ++r) c += hj[f * JREP + r];
            if (c) atomicAdd(&out[256 + f], c);
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
    uint32_t *keys, *out;
    CK(hipMalloc(&keys, n * 4));
    CK(hipMalloc(&out, (256 + 3 * 4096) * 4));
    {
        std::vector<uint32_t> h(n);
        uint64_t s = 0x9E3779B97F4A7C15ull;
        for (size_t i = 0; i < n; ++i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h[i] = (uint32_t)(s >> 16); }
        CK(hipMemcpy(keys, h.data(), n * 4, hipMemcpyHostToDevice));
    }
    const double gb = 4.0 * n / 1e9;
    float t;
#define RUN(M, P, J, G) \
    t = timeit([&] { k_hist<M, P, J><<<G, HB>>>(keys, n, out); }); \
    printf("mode %d pipe %d jrep %d grid %4d  %.4f ms  %7.1f GB/s\n", M, P, J, G, t, gb / t * 1e3);
    RUN(0, 0, 1, 256) RUN(0, 1, 1, 256) RUN(0, 0, 1, 1024)
    RUN(1, 0, 1, 256) RUN(1, 1, 1, 256)
    RUN(2, 0, 1, 256) RUN(2, 1, 1, 256) RUN(2, 1, 1, 512)
    RUN(2, 1, 2, 256)
    CK(hipDeviceSynchronize());
    return 0;
}
