// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access kinds of the
// merge and issue kernels (MI355X_MICROARCH.md: only wide streaming reads are
// calibrated -- "double it" -- other widths are not).  Each kernel makes a
// known number of accesses over a 32 GB allocation (no reuse, nothing
// resident in the 256 MB Infinity Cache):
//   rand16     random 16-byte reads (a view cell, random in a 1 MB row)
//   rand16rmw  random 16-byte read + 8-byte write back into it (an applied change)
//   rand4      random 4-byte reads (a log slot, a seen word)
//   stream16   16 B per lane, coalesced (the guide's calibrated case)
//   stream4    4 B per lane, coalesced (an issue's log scan)
// Run under `rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc WRITE_SIZE`;
// tools/fetch_cal.py divides the counters by the access counts printed here.
// build: hipcc -O3 --offload-arch=gfx950 tools/micro/fetch_cal.hip -o tools/micro/fetch_cal
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr uint32_t BLOCKS = 32768, THREADS = 256, PER = 64;  // 537 M accesses per random kernel
constexpr uint64_t REGION = (1ull << 20) / 16;                // 1 MB rows of 16-byte cells

__device__ inline uint32_t xs(uint32_t& x) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    return x;
}
__global__ void rand16(const uint4* __restrict__ buf, uint32_t nrows, unsigned long long* sink) {
    const uint64_t base = (uint64_t)(blockIdx.x % nrows) * REGION;
    uint32_t x = blockIdx.x * 2654435761u + threadIdx.x * 40503u + 1u, acc = 0;
    for (uint32_t i = 0; i < PER; i++) {
        const uint4 v = buf[base + xs(x) % REGION];
        acc += v.x ^ v.w;
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}
__global__ void rand16rmw(uint4* __restrict__ buf, uint32_t nrows, unsigned long long* sink) {
    const uint64_t base = (uint64_t)(blockIdx.x % nrows) * REGION;
    uint32_t x = blockIdx.x * 2654435761u + threadIdx.x * 40503u + 7u, acc = 0;
    for (uint32_t i = 0; i < PER; i++) {
        uint4* p = &buf[base + xs(x) % REGION];
        const uint4 v = *p;
        acc += v.x;
        *(uint2*)p = make_uint2(v.x + 1u, v.y);
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}
__global__ void rand4(const uint32_t* __restrict__ buf, uint32_t nrows, unsigned long long* sink) {
    const uint64_t base = (uint64_t)(blockIdx.x % nrows) * REGION * 4;
    uint32_t x = blockIdx.x * 2654435761u + threadIdx.x * 40503u + 3u, acc = 0;
    for (uint32_t i = 0; i < PER; i++) acc += buf[base + xs(x) % (REGION * 4)];
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}
__global__ void stream16(const uint4* __restrict__ buf, unsigned long long* sink) {
    const uint64_t base = (uint64_t)blockIdx.x * THREADS * PER;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < PER; i++) {
        const uint4 v = buf[base + i * THREADS + threadIdx.x];
        acc += v.x ^ v.w;
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}
__global__ void stream4(const uint32_t* __restrict__ buf, unsigned long long* sink) {
    const uint64_t base = (uint64_t)blockIdx.x * THREADS * PER;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < PER; i++) acc += buf[base + i * THREADS + threadIdx.x];
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

int main() {
    const size_t total = 32ull << 30;
    void* p = nullptr;
    if (hipMalloc(&p, total) != hipSuccess) { printf("alloc failed\n"); return 1; }
    if (hipMemset(p, 1, total) != hipSuccess) return 1;
    unsigned long long* sink;
    if (hipMalloc(&sink, 8) != hipSuccess) return 1;
    const uint32_t nrows = (uint32_t)(total / (1ull << 20));  // 32,768 rows of 1 MB
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const double acc = (double)BLOCKS * THREADS * PER;
    auto timed = [&](const char* name, double bytes_per_access, auto launch) {
        launch();
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        printf("{\"kernel\": \"%s\", \"accesses_per_launch\": %.0f, \"launches\": 2, \"ms\": %.4f, "
               "\"G_accesses_per_s\": %.2f, \"requested_bytes_per_access\": %.0f}\n",
               name, acc, ms, acc / ms / 1e6, bytes_per_access);
    };
    timed("rand16", 16, [&] { hipLaunchKernelGGL(rand16, dim3(BLOCKS), dim3(THREADS), 0, 0, (const uint4*)p, nrows, sink); });
    timed("rand16rmw", 16, [&] { hipLaunchKernelGGL(rand16rmw, dim3(BLOCKS), dim3(THREADS), 0, 0, (uint4*)p, nrows, sink); });
    timed("rand4", 4, [&] { hipLaunchKernelGGL(rand4, dim3(BLOCKS), dim3(THREADS), 0, 0, (const uint32_t*)p, nrows, sink); });
    timed("stream16", 16, [&] { hipLaunchKernelGGL(stream16, dim3(BLOCKS), dim3(THREADS), 0, 0, (const uint4*)p, sink); });
    timed("stream4", 4, [&] { hipLaunchKernelGGL(stream4, dim3(BLOCKS), dim3(THREADS), 0, 0, (const uint32_t*)p, sink); });
    hipFree(p);
    hipFree(sink);
    return 0;
}
