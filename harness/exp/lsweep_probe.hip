// lsweep_probe.hip -- times the local first pass (csrc/lsweep.hip, k_lsweep) at 2^28 keys
// against a tiled 16-B copy of the same bytes (joint-field counting included),
// for uniform / sorted / %100 / %1000 keys, and checks a few tiles on the host.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o lsweep_probe lsweep_probe.hip
#include "lsweep_exp.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace labsort;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);               \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

__global__ void k_fillp(uint32_t *o, size_t n, int dist) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = 0x5EED0003ull ^ (i * 0x9E3779B97F4A7C15ull);
        z += 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const uint32_t hi = (uint32_t)(z >> 32);
        o[i] = dist == 0 ? hi : dist == 1 ? (uint32_t)i : dist == 2 ? hi % 100u : hi % 1000u;
    }
}
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
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
            if (NT & 2) __builtin_nontemporal_store(k[j], d + j * 1024);
            else d[j * 1024] = k[j];
        }
    }
}

template <class F>
float timeit(F f, int reps = 10) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    f();
    (void)hipDeviceSynchronize();
    std::vector<float> v;
    for (int r = 0; r < reps; ++r) {
        (void)hipEventRecord(a);
        f();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const size_t n = (size_t)1 << lg;
    const uint32_t ntiles = (uint32_t)((n + LS_TILE - 1) / LS_TILE);
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *in, *out, *rows, *tot0, *joint;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&rows, (size_t)ntiles * 256 * 4));
    CK(hipMalloc(&tot0, 256 * 4));
    CK(hipMalloc(&joint, 4 * NSEG * 256 * 4));
    const double gb = 8.0 * n / 1e9;
    for (int nt : {0, 1, 3}) {
        float t = timeit([&] {
            if (nt == 0) k_copy_tile4<0><<<cus, 1024>>>((const v4u *)in, (v4u *)out, (uint32_t)(n / 16384));
            else if (nt == 1) k_copy_tile4<1><<<cus, 1024>>>((const v4u *)in, (v4u *)out, (uint32_t)(n / 16384));
            else k_copy_tile4<3><<<cus, 1024>>>((const v4u *)in, (v4u *)out, (uint32_t)(n / 16384));
        });
        printf("copy-tile4 nt=%d        %.4f ms  %7.1f GB/s\n", nt, t, gb / t * 1e3);
    }
    const char *dn[] = {"uniform", "sorted", "mod100", "mod1000"};
    for (int dist = 0; dist < 4; ++dist) {
        k_fillp<<<8192, 256>>>(in, n, dist);
        CK(hipDeviceSynchronize());
        {
            float t = timeit([&] {
                (void)hipMemsetAsync(tot0, 0, 1024, 0);
                (void)hipMemsetAsync(joint, 0, 4 * NSEG * 256 * 4, 0);
                (void)launch_lsweep(in, out, n, 0u, rows, tot0, joint, 0);
            });
            printf("lsweep %-8s %.4f ms  %7.1f GB/s\n", dn[dist], t, gb / t * 1e3);
        }
        // host check: every tile sorted by digit 0 (stably) and the counts
        std::vector<uint32_t> hi(n), ho(n), hr((size_t)ntiles * 256), ht(256), hj(4 * NSEG * 256);
        CK(hipMemset(tot0, 0, 1024));
        CK(hipMemset(joint, 0, 4 * NSEG * 256 * 4));
        CK(launch_lsweep(in, out, n, 0u, rows, tot0, joint, 0));
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(hi.data(), in, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ho.data(), out, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hr.data(), rows, hr.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ht.data(), tot0, 1024, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hj.data(), joint, hj.size() * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        std::vector<uint64_t> tot(256, 0), jt(4 * NSEG * 256, 0);
        for (uint32_t t = 0; t < ntiles; ++t) {
            const size_t b = (size_t)t * LS_TILE, e = std::min(n, b + LS_TILE);
            std::vector<uint32_t> x(hi.begin() + b, hi.begin() + e);
            std::stable_sort(x.begin(), x.end(), [](uint32_t a, uint32_t c) { return (a & 255u) < (c & 255u); });
            if (!std::equal(x.begin(), x.end(), ho.begin() + b)) ++bad;
            std::vector<uint32_t> c(256, 0);
            for (uint32_t v : x) c[v & 255u]++;
            uint32_t off = 0;
            for (int d = 0; d < 256; ++d) {
                if (hr[(size_t)t * 256 + d] != (off | (c[d] << 16))) ++bad;
                off += c[d];
                tot[d] += c[d];
            }
        }
        for (size_t i = 0; i < n; ++i)
            for (int p = 0; p < 3; ++p) {
                const uint32_t f = (hi[i] >> (8 * p + 4)) & 4095u;
                jt[((p + 1) * NSEG + (f & 15u)) * 256 + (f >> 4)]++;
            }
        for (int d = 0; d < 256; ++d) bad += tot[d] != ht[d];
        for (size_t i = 0; i < jt.size(); ++i) bad += jt[i] != hj[i];
        printf("check %-8s: %zu mismatches\n", dn[dist], bad);
    }
    return 0;
}
