// pmc_cal.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the
// exact access widths the labsort kernels use (MI355X_MICROARCH.md §HBM: only the
// 16-B/lane streaming read is calibrated there, at 1/2).  Each kernel moves a KNOWN byte
// count (2^28 words = 1 GiB read and/or written, far past the 256 MiB Infinity Cache)
// with one access shape; profiles/pmc_summary.py divides the counters by these bytes
// and corrects each product kernel by the factors of its own shapes.
//   cal_rd_dword     16 dword loads per lane in the onesweep/tile-sort blocked layout
//                    (1024-thread workgroups, 16384-word tiles), plain
//   cal_rd_dword_nt  the same, nontemporal (k_onesweep_p's r25 key loads)
//   cal_rd_buf_nt    buffer_load_dword nt (k_onesweep_p's key loads from r26)
//   cal_rd_x4_nt     16-B/lane nontemporal loads (k_hist_seg)
//   cal_rd_x4        16-B/lane plain loads (the guide's reference shape)
//   cal_wr_dword     16 dword stores per lane, blocked layout (tile sort, merge stores)
//   cal_wr_buf       buffer_store_dword, blocked layout (k_onesweep_p's scatter from r26)
//   cal_wr_x4        16-B/lane stores
// Each kernel runs 3 times.  Build: hipcc --offload-arch=gfx950 -O3 -o ../bin/pmc_cal pmc_cal.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);    \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr unsigned TILE = 16384;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}

__global__ __launch_bounds__(1024) void cal_rd_dword(const unsigned *a, unsigned ntiles, unsigned *sink) {
    const unsigned tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    unsigned acc = 0;
    for (unsigned t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const unsigned *s = a + (size_t)t * TILE + wid * 1024 + lane;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc += s[j * 64];
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
__global__ __launch_bounds__(1024) void cal_rd_dword_nt(const unsigned *a, unsigned ntiles, unsigned *sink) {
    const unsigned tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    unsigned acc = 0;
    for (unsigned t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const unsigned *s = a + (size_t)t * TILE + wid * 1024 + lane;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc += __builtin_nontemporal_load(s + j * 64);
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
__global__ __launch_bounds__(1024) void cal_rd_buf_nt(const unsigned *a, unsigned ntiles, unsigned *sink) {
    const unsigned tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const __amdgpu_buffer_rsrc_t r = rsrc(a, ntiles * TILE * 4u);
    unsigned acc = 0;
    for (unsigned t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const unsigned o = (t * TILE + wid * 1024 + lane) * 4u;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc += __builtin_amdgcn_raw_buffer_load_b32(r, o + j * 256, 0, 2);
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
__global__ __launch_bounds__(256) void cal_rd_x4_nt(const v4u *a, size_t n4, unsigned *sink) {
    v4u acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        acc += __builtin_nontemporal_load(a + i);
    if (acc.x + acc.y + acc.z + acc.w == 0x12345678u) sink[0] = 1;
}
__global__ __launch_bounds__(256) void cal_rd_x4(const v4u *a, size_t n4, unsigned *sink) {
    v4u acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        acc += a[i];
    if (acc.x + acc.y + acc.z + acc.w == 0x12345678u) sink[0] = 1;
}
__global__ __launch_bounds__(1024) void cal_wr_dword(unsigned *b, unsigned ntiles) {
    const unsigned tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (unsigned t = blockIdx.x; t < ntiles; t += gridDim.x) {
        unsigned *d = b + (size_t)t * TILE + wid * 1024 + lane;
#pragma unroll
        for (int j = 0; j < 16; ++j) d[j * 64] = t + j;
    }
}
__global__ __launch_bounds__(1024) void cal_wr_buf(unsigned *b, unsigned ntiles) {
    const unsigned tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const __amdgpu_buffer_rsrc_t r = rsrc(b, ntiles * TILE * 4u);
    for (unsigned t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const unsigned o = (t * TILE + wid * 1024 + lane) * 4u;
#pragma unroll
        for (int j = 0; j < 16; ++j) __builtin_amdgcn_raw_buffer_store_b32(t + j, r, o + j * 256, 0, 0);
    }
}
__global__ __launch_bounds__(256) void cal_wr_x4(v4u *b, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const unsigned x = (unsigned)i;
        b[i] = v4u{x, x + 1, x + 2, x + 3};
    }
}

int main() {
    const size_t n = (size_t)1 << 28;  // words: 1 GiB per buffer
    const unsigned ntiles = (unsigned)(n / TILE);
    unsigned *a, *b, *sink;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, n * 4));
    CK(hipMemset(b, 0, n * 4));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](const char *name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float ms = 0, tot = 0;
        for (int r = 0; r < 3; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
        }
        std::printf("%-16s %8.4f ms  %7.1f GB/s (1 GiB moved per launch)\n", name, tot / 3, (double)n * 4 / (tot / 3) / 1e6);
    };
    timed("cal_rd_dword", [&] { cal_rd_dword<<<cus, 1024>>>(a, ntiles, sink); });
    timed("cal_rd_dword_nt", [&] { cal_rd_dword_nt<<<cus, 1024>>>(a, ntiles, sink); });
    timed("cal_rd_buf_nt", [&] { cal_rd_buf_nt<<<cus, 1024>>>(a, ntiles, sink); });
    timed("cal_rd_x4_nt", [&] { cal_rd_x4_nt<<<cus * 8, 256>>>((const v4u *)a, n / 4, sink); });
    timed("cal_rd_x4", [&] { cal_rd_x4<<<cus * 8, 256>>>((const v4u *)a, n / 4, sink); });
    timed("cal_wr_dword", [&] { cal_wr_dword<<<cus, 1024>>>(b, ntiles); });
    timed("cal_wr_buf", [&] { cal_wr_buf<<<cus, 1024>>>(b, ntiles); });
    timed("cal_wr_x4", [&] { cal_wr_x4<<<cus * 8, 256>>>((v4u *)b, n / 4); });
    CK(hipDeviceSynchronize());
    return 0;
}
