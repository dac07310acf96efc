// Random 16-byte reads inside per-block 1 MB regions: spread over a large
// allocation (one region per block, like view rows) vs folded into a small
// one.  Same access count and pattern; differs only in pages touched.
// build: hipcc -O3 --offload-arch=gfx950 tools/micro/tlb_probe.hip -o tools/micro/tlb_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_rand(const uint4* __restrict__ buf, uint64_t region_elems, uint32_t nregions, uint32_t per_block,
                       unsigned long long* sink) {
    const uint64_t base = (uint64_t)(blockIdx.x % nregions) * region_elems;
    uint32_t x = blockIdx.x * 2654435761u + threadIdx.x * 40503u + 1u;
    uint32_t acc = 0;
    for (uint32_t i = threadIdx.x; i < per_block; i += blockDim.x) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        const uint4 v = buf[base + (x % region_elems)];
        acc += v.x ^ v.w;
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

__global__ void k_stream(const uint2* __restrict__ buf, uint64_t region_elems, uint32_t nregions, uint32_t per_block,
                         unsigned long long* sink) {
    const uint64_t base = (uint64_t)(blockIdx.x % nregions) * region_elems;
    uint32_t acc = 0;
    for (uint32_t i = threadIdx.x; i < per_block; i += blockDim.x) {
        const uint2 v = buf[base + i];
        acc += v.x ^ v.y;
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

int main() {
    const size_t total = 64ull << 30;  // 64 GB
    void* p = nullptr;
    if (hipMalloc(&p, total) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(p, 1, total);
    unsigned long long* sink;
    hipMalloc(&sink, 8);
    const uint32_t blocks = 65536;
    const uint64_t region = (1ull << 20) / 16;  // 1 MB of 16-byte cells
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    struct Cfg { const char* name; uint32_t nregions; };
    // 65536 regions = 64 GB spread; 64 regions = 64 MB (fits the 256 MB MALL); 1024 regions = 1 GB
    Cfg cfgs[] = {{"spread 64 GB", 65536}, {"folded 1 GB", 1024}, {"folded 64 MB", 64}};
    for (int rep = 0; rep < 2; rep++)
        for (auto& c : cfgs) {
            for (uint32_t per : {400u, 4000u}) {
                hipLaunchKernelGGL(k_rand, dim3(blocks), dim3(256), 0, 0, (const uint4*)p, region, c.nregions, per, sink);
                hipEventRecord(a);
                hipLaunchKernelGGL(k_rand, dim3(blocks), dim3(256), 0, 0, (const uint4*)p, region, c.nregions, per, sink);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms; hipEventElapsedTime(&ms, a, b);
                double acc = (double)blocks * per;
                if (rep) printf("rand16  %-14s %5u/block: %.3f ms, %.2f G accesses/s, %.0f GB/s at 64 B/access\n", c.name, per, ms,
                       acc / ms / 1e6, acc * 64 / ms / 1e6);
            }
            const uint32_t per = 8192;  // 64 KB streamed per block
            hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(256), 0, 0, (const uint2*)p, region * 2, c.nregions, per, sink);
            hipEventRecord(a);
            hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(256), 0, 0, (const uint2*)p, region * 2, c.nregions, per, sink);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            if (rep) printf("stream8 %-14s 64 KB/block: %.3f ms, %.0f GB/s\n", c.name, ms, (double)blocks * per * 8 / ms / 1e6);
        }
    hipFree(p);
    return 0;
}
