// Workgroup-level primitives for 256-thread (4 x wave64) blocks.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rp {

constexpr int BLOCK = 256;
constexpr int NWAVE = BLOCK / 64;

struct BlockScratch {
    uint32_t w32[NWAVE];
    uint64_t w64[NWAVE];
    uint32_t bcast[4];
    uint64_t bcast64[2];
};

__device__ inline int lane_id() { return threadIdx.x & 63; }
__device__ inline int wave_id() { return threadIdx.x >> 6; }

// Exclusive rank of `flag` among the block's threads (thread order) and the
// block total.  Contains two barriers: call from uniform control flow.
__device__ inline uint32_t block_rank(bool flag, BlockScratch& sc, uint32_t& total) {
    uint64_t m = __ballot(flag);
    int lane = lane_id(), w = wave_id();
    uint32_t r = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) sc.w32[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NWAVE; i++) {
        uint32_t c = sc.w32[i];
        off += (i < w) ? c : 0u;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return off + r;
}

__device__ inline uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ inline uint32_t wave_min32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { uint32_t t = __shfl_xor(v, o); v = t < v ? t : v; }
    return v;
}

__device__ inline uint64_t block_sum64(uint64_t v, BlockScratch& sc) {
    v = wave_sum64(v);
    if (lane_id() == 0) sc.w64[wave_id()] = v;
    __syncthreads();
    uint64_t t = 0;
#pragma unroll
    for (int i = 0; i < NWAVE; i++) t += sc.w64[i];
    __syncthreads();
    return t;
}
__device__ inline uint32_t block_min32(uint32_t v, BlockScratch& sc) {
    v = wave_min32(v);
    if (lane_id() == 0) sc.w32[wave_id()] = v;
    __syncthreads();
    uint32_t t = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < NWAVE; i++) t = sc.w32[i] < t ? sc.w32[i] : t;
    __syncthreads();
    return t;
}
__device__ inline bool block_any(bool f, BlockScratch& sc) {
    uint32_t tot;
    block_rank(f, sc, tot);
    return tot != 0;
}

}  // namespace rp
