// digit_probe.hip -- timing probe for the digit width of the LSD radix pass (VERDICT r4 item 1:
// would a 3-pass 11/11/10-bit sort beat the 4-pass 8-bit one?).
//
// One scatter pass over 2^28 uniform uint32 keys with B-bit digits (B = 8, 10, 11), in the
// onesweep pass's shape minus its look-back: 16384-key tiles, one 1024-thread workgroup per
// CU looping over tiles, tiles dealt to the 8 XCDs as contiguous eighths in order (each XCD
// takes its eighth's tiles from its own counter, as k_onesweep_p's XCD-grouped chains), each
// tile ranked by LDS atomics on 2^B tile-wide counters, reordered by digit in LDS, read back
// and scattered to its (tile, digit) run's global offset.  The offsets come from a setup
// count + scan (not timed): the probe pays no look-back, so it bounds a real pass from below.
// The 8-bit row calibrates it against the shipped pass (bench: 0.466-0.472 ms).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 digit_probe.hip -o ../bin/digit_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

constexpr int BLK = 1024, KPT = 16, TILE = BLK * KPT;

__global__ void k_gen(uint32_t *k, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = 0x5EED0003ull ^ (i * 0x9E3779B97F4A7C15ull);
        z += 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        k[i] = (uint32_t)((z ^ (z >> 31)) >> 32);
    }
}

// per-tile digit counts, digit-major: cnt[d * ntiles + t]
template <int B>
__global__ __launch_bounds__(BLK) void k_count(const uint32_t *k, uint32_t *cnt, uint32_t ntiles, int shift) {
    constexpr int R = 1 << B;
    __shared__ uint32_t h[R];
    for (int i = threadIdx.x; i < R; i += BLK) h[i] = 0;
    __syncthreads();
    const uint32_t t = blockIdx.x;
    for (int j = 0; j < KPT; ++j) atomicAdd(&h[(k[(size_t)t * TILE + j * BLK + threadIdx.x] >> shift) & (R - 1)], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < R; i += BLK) cnt[(size_t)i * ntiles + t] = h[i];
}

// exclusive scan of cnt (single workgroup, serial chunks: setup only)
__global__ __launch_bounds__(1024) void k_scan(uint32_t *cnt, size_t m) {
    __shared__ uint32_t part[1024];
    const size_t per = (m + 1023) / 1024, b = threadIdx.x * per, e = b + per < m ? b + per : m;
    uint32_t s = 0;
    for (size_t i = b; i < e; ++i) s += cnt[i];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int i = 0; i < 1024; ++i) {
            const uint32_t v = part[i];
            part[i] = run;
            run += v;
        }
    }
    __syncthreads();
    uint32_t run = part[threadIdx.x];
    for (size_t i = b; i < e; ++i) {
        const uint32_t v = cnt[i];
        cnt[i] = run;
        run += v;
    }
}

__device__ __forceinline__ uint32_t pad(uint32_t i) { return i + (i >> 5); }

template <int B>
struct Sm {
    static constexpr int R = 1 << B;
    uint32_t keys[TILE + TILE / 32];
    uint32_t cnt[R];    // counts, then tile-local digit starts
    uint32_t delta[R];  // global offset of the digit's run minus its tile-local start
    uint32_t wsum[16];
    uint32_t next;
};

// SCATTER = false: the same work, but the reordered tile is written back contiguously at
// its own position (whole lines): separates the scatter's write shape from the LDS work
template <int B, bool SCATTER = true>
__global__ __launch_bounds__(BLK) void k_pass(const uint32_t *in, uint32_t *out, const uint32_t *off, uint32_t ntiles,
                                              int shift, uint32_t *ctr) {
    constexpr int R = 1 << B, PER = R / BLK > 0 ? R / BLK : 1;
    __shared__ Sm<B> sm;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t g = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u;  // HW_REG_XCC_ID
    const uint32_t per = ntiles / 8u;
    const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)(ntiles * (uint32_t)TILE * 4u), 0x00020000);
    for (;;) {
        if (tid == 0) {
            const uint32_t q = atomicAdd(ctr + g, 1u);
            sm.next = q < per ? g * per + q : 0xFFFFFFFFu;
        }
        for (int i = tid; i < R; i += BLK) sm.cnt[i] = 0;
        __syncthreads();
        const uint32_t t = sm.next;
        if (t == 0xFFFFFFFFu) break;
        uint32_t k[KPT], r[KPT];
#pragma unroll
        for (int j = 0; j < KPT; ++j) k[j] = __builtin_nontemporal_load(in + (size_t)t * TILE + wid * (KPT * 64) + j * 64 + lane);
#pragma unroll
        for (int j = 0; j < KPT; ++j) r[j] = atomicAdd(&sm.cnt[(k[j] >> shift) & (R - 1)], 1u);
        __syncthreads();
        // tile-local digit starts: each thread scans PER consecutive digits, block scan on top
        uint32_t c[PER], s = 0;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint32_t d = tid * PER + q;
            c[q] = d < (uint32_t)R ? sm.cnt[d] : 0u;
            s += c[q];
        }
        uint32_t x = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= (uint32_t)o) x += y;
        }
        if (lane == 63) sm.wsum[wid] = x;
        __syncthreads();
        uint32_t add = 0;
        for (uint32_t w = 0; w < wid; ++w) add += sm.wsum[w];
        uint32_t run = x - s + add;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint32_t d = tid * PER + q;
            if (d < (uint32_t)R) {
                sm.cnt[d] = run;
                sm.delta[d] = off[(size_t)d * ntiles + t] - run;
            }
            run += c[q];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < KPT; ++j) sm.keys[pad(sm.cnt[(k[j] >> shift) & (R - 1)] + r[j])] = k[j];
        __syncthreads();
        // scatter in slot order: 4 consecutive slots per lane, one 16-B store inside a run
#pragma unroll
        for (int gq = 0; gq < KPT / 4; ++gq) {
            const uint32_t i0 = 4u * (gq * BLK + tid);
            uint32_t v[4], d[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                v[q] = sm.keys[pad(i0 + q)];
                d[q] = (v[q] >> shift) & (R - 1);
            }
            if (!SCATTER) {
                typedef uint32_t u4 __attribute__((ext_vector_type(4)));
                const u4 w = {v[0], v[1], v[2], v[3]};
                __builtin_amdgcn_raw_buffer_store_b128(w, rout, (t * (uint32_t)TILE + i0) * 4u, 0, 0);
                continue;
            }
            if (d[0] == d[3]) {  // (as k_onesweep_p: dword-aligned 16-B buffer store)
                typedef uint32_t u4 __attribute__((ext_vector_type(4)));
                const u4 w = {v[0], v[1], v[2], v[3]};
                __builtin_amdgcn_raw_buffer_store_b128(w, rout, (sm.delta[d[0]] + i0) * 4u, 0, 0);
                continue;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) __builtin_amdgcn_raw_buffer_store_b32(v[q], rout, (sm.delta[d[q]] + i0 + q) * 4u, 0, 0);
        }
        __syncthreads();
    }
}

template <int B, bool SCATTER = true>
void run(const uint32_t *in, uint32_t *out, uint32_t *cnt, uint32_t *ctr, size_t n, int cus) {
    const uint32_t ntiles = (uint32_t)(n / TILE);
    const int shift = 0;
    k_count<B><<<ntiles, BLK>>>(in, cnt, ntiles, shift);
    k_scan<<<1, 1024>>>(cnt, (size_t)ntiles << B);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int rep = 0; rep < 12; ++rep) {
        CK(hipMemsetAsync(ctr, 0, 64));
        CK(hipEventRecord(a));
        k_pass<B, SCATTER><<<cus, BLK>>>(in, out, cnt, ntiles, shift, ctr);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    // check: out sorted by the digit (stable order not required), a permutation (sum)
    std::vector<uint32_t> h(n);
    CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 1; SCATTER && i < n; ++i) bad += (h[i] & ((1u << B) - 1)) < (h[i - 1] & ((1u << B) - 1));
    printf("{\"write\": \"%s\", \"digit_bits\": %d, \"runs_per_tile\": %d, \"avg_run_keys\": %.1f, \"pass_ms_median\": %.4f, \"pass_ms_min\": %.4f, "
           "\"GBps\": %.1f, \"digit_order_violations\": %zu}\n",
           SCATTER ? "scatter" : "contiguous", B, 1 << B, (double)TILE / (1 << B), ts[ts.size() / 2], ts[0], 8.0 * n / (ts[ts.size() / 2] * 1e6), bad);
    fflush(stdout);
}

int main(int argc, char **argv) {
    const size_t n = (size_t)1 << 28;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    uint32_t *in, *out, *cnt, *ctr;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&cnt, (n / TILE) * 2048 * 4));
    CK(hipMalloc(&ctr, 64));
    k_gen<<<4096, 256>>>(in, n);
    CK(hipDeviceSynchronize());
    // argv[1]: digit bits (0: all); argv[2] = "c": the contiguous-write variant only
    const int which = argc > 1 ? atoi(argv[1]) : 0;
    const bool contig = argc > 2 && argv[2][0] == 'c', both = argc <= 2;
    if ((!which || which == 8) && !contig) run<8>(in, out, cnt, ctr, n, cus);
    if ((!which || which == 10) && !contig) run<10>(in, out, cnt, ctr, n, cus);
    if ((!which || which == 11) && !contig) run<11>(in, out, cnt, ctr, n, cus);
    if ((!which || which == 8) && (contig || both)) run<8, false>(in, out, cnt, ctr, n, cus);
    if ((!which || which == 11) && (contig || both)) run<11, false>(in, out, cnt, ctr, n, cus);
    return 0;
}
