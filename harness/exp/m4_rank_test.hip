// Diagnostic: k_m4_rank on 4 sorted runs of 65536 (keys = positions): prints the boundary
// rows around the A/B transition and the device's view of sample (k=1, q=20).
#include "../../radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/csrc/merge4.hip"
#include <cstdio>
#include <vector>
using namespace labsort;
__global__ void k_probe(const uint32_t *src, M4Geo G, const uint32_t *samp) {
    const uint32_t spr = G.r / M4_S, sid = 1 * spr + 20;
    printf("dev: spr %u spg %u bpg %u samp[sid] %u src[r+2560] %u samp[A,511] %u len? n %u r %u\n", spr, G.spg, G.bpg,
           samp[sid], src[G.r + 2560], samp[511], G.n, G.r);
}
int main() {
    const uint32_t r = 65536, n = 4 * r;
    std::vector<uint32_t> h(n);
    for (uint32_t i = 0; i < n; ++i) h[i] = i;
    uint32_t *d, *o, *ws;
    hipMalloc(&d, n * 4); hipMalloc(&o, n * 4);
    const size_t bw = merge4_bnd_words(n, r);
    hipMalloc(&ws, bw * 4 + 4096);
    hipMemset(ws, 0, bw * 4 + 4096);
    hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
    hipError_t e = launch_merge4_pass(d, o, n, r, 0, ws, nullptr, nullptr, 0);
    hipDeviceSynchronize();
    printf("launch %d\n", (int)e);
    const M4Geo G = m4_geo(n, r);
    k_probe<<<1, 1>>>(d, G, ws + (size_t)G.ngroups * G.bpg * 4);
    hipDeviceSynchronize();
    std::vector<uint32_t> b(G.ngroups * G.bpg * 4);
    hipMemcpy(b.data(), ws, b.size() * 4, hipMemcpyDeviceToHost);
    for (uint32_t i = 17; i < 21; ++i) printf("row %u: %u %u %u %u\n", i, b[4 * i], b[4 * i + 1], b[4 * i + 2], b[4 * i + 3]);
    std::vector<uint32_t> out(n);
    hipMemcpy(out.data(), o, n * 4, hipMemcpyDeviceToHost);
    size_t bad = 0; for (uint32_t i = 0; i < n; ++i) bad += out[i] != i;
    printf("wrong %zu\n", bad);
}
