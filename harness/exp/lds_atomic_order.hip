// Diagnostic: in which lane order does one ds_add_rtn_u32 instruction service lanes
// that hit the same LDS address?  Each wave ranks 64 keys per step by an atomic add
// of 1 on a per-wave counter table and records the returned values; the host checks
// whether, for every address, the returns increase with the lane index (a stable
// rank) or follow some other order.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int BLOCK = 1024, KPT = 16, R = 256, W = BLOCK / 64;

__global__ __launch_bounds__(BLOCK) void k_rank(const uint32_t *keys, uint32_t *ret, int mode) {
    __shared__ uint32_t cnt[W * R];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    for (uint32_t i = tid; i < (uint32_t)(W * R); i += BLOCK) cnt[i] = 0u;
    __syncthreads();
    uint32_t *wc = cnt + wid * R;
    const size_t base = (size_t)blockIdx.x * BLOCK * KPT + wid * (KPT * 64) + lane;
    uint32_t r[KPT];
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t d = keys[base + j * 64] & 255u;
        if (mode == 0) r[j] = atomicAdd(&wc[d], 1u);
        else r[j] = __hip_atomic_fetch_add(&wc[d], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
#pragma unroll
    for (int j = 0; j < KPT; ++j) ret[base + j * 64] = r[j];
}

static uint64_t sm(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main() {
    const int blocks = 4096;
    const size_t n = (size_t)blocks * BLOCK * KPT;
    std::vector<uint32_t> h(n), out(n);
    uint32_t *dk, *dr;
    hipMalloc(&dk, n * 4);
    hipMalloc(&dr, n * 4);
    const char *names[] = {"uniform256", "uniform4", "const", "mixed", "skew"};
    long bad_total = 0;
    for (int dist = 0; dist < 5; ++dist) {
        uint64_t s = 0x1234 + dist;
        for (size_t i = 0; i < n; ++i) {
            uint64_t x = sm(s);
            uint32_t d;
            switch (dist) {
                case 0: d = x & 255; break;
                case 1: d = x & 3; break;
                case 2: d = 7; break;
                case 3: d = ((x >> 8) & 1) ? (x & 255) : (x & 1); break;
                default: d = (uint32_t)(__builtin_clzll(x | 1) * 4) & 255; break;
            }
            h[i] = d;
        }
        hipMemcpy(dk, h.data(), n * 4, hipMemcpyHostToDevice);
        for (int mode = 0; mode < 2; ++mode) {
            hipLaunchKernelGGL(k_rank, dim3(blocks), dim3(BLOCK), 0, 0, dk, dr, mode);
            hipDeviceSynchronize();
            hipMemcpy(out.data(), dr, n * 4, hipMemcpyDeviceToHost);
            // replay: per wave, stable rank = count of earlier (step, lane) with same digit
            long bad = 0, perm_ok = 0;
            for (size_t w = 0; w < n / (KPT * 64); ++w) {
                uint32_t c[R] = {0};
                for (int j = 0; j < KPT; ++j) {
                    for (int l = 0; l < 64; ++l) {
                        const size_t i = w * KPT * 64 + j * 64 + l;
                        const uint32_t d = h[i];
                        if (out[i] != c[d]) ++bad;
                        ++c[d];
                    }
                }
                ++perm_ok;
            }
            printf("%-10s mode %d: %ld of %zu returns differ from the lane-order rank\n", names[dist], mode, bad, n);
            bad_total += bad;
        }
    }
    printf("total mismatches %ld\n", bad_total);
    return 0;
}
