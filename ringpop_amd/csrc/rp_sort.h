// Device-wide primitives for the ring build and the request grouping,
// written for gfx950 (256-thread blocks of 4 x wave64):
//   exclusive_scan      tile reduce -> one-block scan of the tile sums ->
//                       tile scan with carry-in (three launches)
//   radix_sort_pairs    stable LSD radix sort of u32 keys (+ u32 values) over
//                       bits [0, kb), <= 8 bits per pass: a per-tile digit
//                       histogram (LDS atomics), an exclusive scan of the
//                       digit-major histogram matrix, and a scatter whose
//                       in-tile ranks come from wave ballots (the lanes of a
//                       row holding the same digit, popcount below) and
//                       per-wave running counters in LDS -- rows are taken in
//                       input order, so equal keys keep their order
// Replaces the rbtree's ordered insert (lib/rbtree.js:70-137) for batched
// addRemoveServers and underscore's groupBy (index.js:636-645).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rp_block.h"
#include "rp_internal.h"

namespace rp {

constexpr uint32_t PS_IPT = 16;                 // items per thread
constexpr uint32_t PS_TILE = BLOCK * PS_IPT;    // 4,096 items per block

// ------------------------------------------------------------------ scan
// exclusive scan of one value per thread over the block; *total = the sum
template <class T>
__device__ inline T block_excl_scan(T x, T* lds, T& total) {
    const int lane = lane_id(), w = wave_id();
    T incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) lds[w] = incl;
    __syncthreads();
    T before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NWAVE; i++) {
        const T c = lds[i];
        before += i < w ? c : T(0);
        tot += c;
    }
    __syncthreads();
    total = tot;
    return before + incl - x;
}

template <class T>
__global__ void __launch_bounds__(BLOCK) k_scan_reduce(const T* in, uint64_t n, T* part) {
    __shared__ T lds[NWAVE];
    const uint64_t base = (uint64_t)blockIdx.x * PS_TILE;
    T s = 0;
#pragma unroll
    for (uint32_t k = 0; k < PS_IPT; k++) {
        const uint64_t i = base + k * BLOCK + threadIdx.x;
        if (i < n) s += in[i];
    }
    T tot;
    block_excl_scan<T>(s, lds, tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// one block: part[0..nt) -> exclusive prefix sums
template <class T>
__global__ void __launch_bounds__(BLOCK) k_scan_partials(T* part, uint32_t nt) {
    __shared__ T lds[NWAVE];
    T carry = 0;
    for (uint32_t c0 = 0; c0 < nt; c0 += PS_TILE) {
        // thread t: the PS_IPT consecutive entries c0 + t * PS_IPT ...
        T v[PS_IPT];
        T s = 0;
        const uint32_t b = c0 + threadIdx.x * PS_IPT;
#pragma unroll
        for (uint32_t k = 0; k < PS_IPT; k++) {
            v[k] = b + k < nt ? part[b + k] : T(0);
            s += v[k];
        }
        T tot;
        T run = carry + block_excl_scan<T>(s, lds, tot);
#pragma unroll
        for (uint32_t k = 0; k < PS_IPT; k++) {
            if (b + k < nt) part[b + k] = run;
            run += v[k];
        }
        carry += tot;
    }
}

template <class T>
__global__ void __launch_bounds__(BLOCK) k_scan_tiles(const T* in, uint64_t n, const T* part, T* out) {
    __shared__ T lds[NWAVE];
    const uint64_t b = (uint64_t)blockIdx.x * PS_TILE + (uint64_t)threadIdx.x * PS_IPT;
    T v[PS_IPT];
    T s = 0;
#pragma unroll
    for (uint32_t k = 0; k < PS_IPT; k++) {
        v[k] = b + k < n ? in[b + k] : T(0);
        s += v[k];
    }
    T tot;
    T run = part[blockIdx.x] + block_excl_scan<T>(s, lds, tot);
#pragma unroll
    for (uint32_t k = 0; k < PS_IPT; k++) {
        if (b + k < n) out[b + k] = run;
        run += v[k];
    }
}

struct ScanWork {
    DevBuf<uint64_t> part;  // (u32 scans use its words)
};

// out[i] = in[0] + ... + in[i - 1] for i < n (in == out allowed)
template <class T>
inline void exclusive_scan(const T* in, T* out, uint64_t n, ScanWork& w, hipStream_t st) {
    if (!n) return;
    const uint64_t nt = (n + PS_TILE - 1) / PS_TILE;
    if (nt > 0xFFFFFFFFull) throw Error(RP_ERR_INVALID, "scan too long");
    w.part.reserve((nt * sizeof(T) + 7) / 8 + 1);
    T* part = (T*)w.part.p;
    hipLaunchKernelGGL(k_scan_reduce<T>, dim3((unsigned)nt), dim3(BLOCK), 0, st, in, n, part);
    hipLaunchKernelGGL(k_scan_partials<T>, dim3(1), dim3(BLOCK), 0, st, part, (uint32_t)nt);
    hipLaunchKernelGGL(k_scan_tiles<T>, dim3((unsigned)nt), dim3(BLOCK), 0, st, in, n, (const T*)part, out);
    RP_HIP(hipGetLastError());
}

// ------------------------------------------------------------------ radix sort
__global__ void __launch_bounds__(BLOCK) k_rs_upsweep(const uint32_t* key, uint32_t n, uint32_t shift, uint32_t bits,
                                                      uint32_t* hist, uint32_t ntiles) {
    __shared__ uint32_t cnt[256];
    const uint32_t bins = 1u << bits, mask = bins - 1u, tile = blockIdx.x;
    cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)tile * PS_TILE;
#pragma unroll
    for (uint32_t k = 0; k < PS_IPT; k++) {
        const uint64_t i = base + k * BLOCK + threadIdx.x;
        if (i < n) atomicAdd(&cnt[(key[i] >> shift) & mask], 1u);
    }
    __syncthreads();
    if (threadIdx.x < bins) hist[(size_t)threadIdx.x * ntiles + tile] = cnt[threadIdx.x];
}

// Wave w of a tile owns its items w * 1024 ... + 1023, in rows of 64 (row k:
// items + 64 k + lane, read coalesced).  A lane's rank among the earlier
// items of its digit = (the wave's running count of that digit before the
// row) + (lanes of the row below it with the same digit: a ballot per digit
// bit); the lowest such lane moves the running count on.  After the rows, the
// waves' counts are turned into per-wave prefixes, and the tile's base per
// digit comes from the scanned histogram.
template <bool VALS>
__global__ void __launch_bounds__(BLOCK) k_rs_downsweep(const uint32_t* kin, const uint32_t* vin, uint32_t* kout,
                                                        uint32_t* vout, uint32_t n, uint32_t shift, uint32_t bits,
                                                        const uint32_t* hist, uint32_t ntiles) {
    __shared__ uint32_t cw[NWAVE][256];
    __shared__ uint32_t gb[256];
    const uint32_t bins = 1u << bits, mask = bins - 1u, tile = blockIdx.x;
    const int lane = lane_id(), w = wave_id();
    const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
    for (int q = 0; q < NWAVE; q++) cw[q][threadIdx.x] = 0;
    if (threadIdx.x < bins) gb[threadIdx.x] = hist[(size_t)threadIdx.x * ntiles + tile];
    __syncthreads();
    const uint64_t base = (uint64_t)tile * PS_TILE + (uint64_t)w * (64 * PS_IPT);
    uint32_t key[PS_IPT], val[PS_IPT], rk[PS_IPT];
#pragma unroll
    for (uint32_t k = 0; k < PS_IPT; k++) {
        const uint64_t i = base + k * 64 + lane;
        key[k] = i < n ? kin[i] : 0u;
        if (VALS) val[k] = i < n ? vin[i] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < PS_IPT; k++) {
        const uint64_t i = base + k * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = (key[k] >> shift) & mask;
        uint64_t peers = __ballot(valid);
        for (uint32_t b = 0; b < bits; b++) {
            const uint64_t m = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        const uint32_t before = valid ? cw[w][d] : 0u;
        rk[k] = before + (uint32_t)__popcll(peers & below);
        if (valid && (peers & below) == 0) cw[w][d] = before + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    if (threadIdx.x < bins) {
        uint32_t run = 0;
#pragma unroll
        for (int q = 0; q < NWAVE; q++) {
            const uint32_t c = cw[q][threadIdx.x];
            cw[q][threadIdx.x] = run + gb[threadIdx.x];
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < PS_IPT; k++) {
        const uint64_t i = base + k * 64 + lane;
        if (i >= n) continue;
        const uint32_t pos = cw[w][(key[k] >> shift) & mask] + rk[k];
        kout[pos] = key[k];
        if (VALS) vout[pos] = val[k];
    }
}

// The same passes with the keys computed on the fly (KeyFn: key of item i)
// and, without VIN, the item's index as its value; KOUT = false drops the
// keys of a last pass (its caller keeps only the values).
struct KeysIn {
    const uint32_t* k;
    __device__ inline uint32_t operator()(uint64_t i) const { return k[i]; }
};
template <class KeyFn>
__global__ void __launch_bounds__(BLOCK) k_rs_upsweep_f(KeyFn kf, uint32_t n, uint32_t shift, uint32_t bits,
                                                        uint32_t* hist, uint32_t ntiles) {
    __shared__ uint32_t cnt[256];
    const uint32_t bins = 1u << bits, mask = bins - 1u, tile = blockIdx.x;
    cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)tile * PS_TILE;
    uint32_t key[PS_IPT];
#pragma unroll
    for (uint32_t k = 0; k < PS_IPT; k++) {
        const uint64_t i = base + k * BLOCK + threadIdx.x;
        key[k] = i < n ? kf(i) : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < PS_IPT; k++) {
        const uint64_t i = base + k * BLOCK + threadIdx.x;
        if (i < n) atomicAdd(&cnt[(key[k] >> shift) & mask], 1u);
    }
    __syncthreads();
    if (threadIdx.x < bins) hist[(size_t)threadIdx.x * ntiles + tile] = cnt[threadIdx.x];
}
// The tile is first sorted by digit in LDS, then written out in that order:
// consecutive threads store consecutive positions of one digit's run, so the
// scatter leaves the block as whole lines instead of one lane per line.
template <class KeyFn, bool VIN, bool KOUT>
__global__ void __launch_bounds__(BLOCK) k_rs_downsweep_f(KeyFn kf, const uint32_t* vin, uint32_t* kout,
                                                          uint32_t* vout, uint32_t n, uint32_t shift, uint32_t bits,
                                                          const uint32_t* hist, uint32_t ntiles) {
    __shared__ uint32_t cw[NWAVE][256];
    __shared__ uint32_t lsd[256], gbs[256], scan_tmp[NWAVE];
    __shared__ uint32_t sk[PS_TILE], sv[PS_TILE];
    const uint32_t bins = 1u << bits, mask = bins - 1u, tile = blockIdx.x;
    const int lane = lane_id(), w = wave_id();
    const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
    for (int q = 0; q < NWAVE; q++) cw[q][threadIdx.x] = 0;
    uint32_t gbv = threadIdx.x < bins ? hist[(size_t)threadIdx.x * ntiles + tile] : 0u;
    __syncthreads();
    const uint64_t base = (uint64_t)tile * PS_TILE + (uint64_t)w * (64 * PS_IPT);
    uint32_t key[PS_IPT], val[PS_IPT], rk[PS_IPT];
#pragma unroll
    for (uint32_t k = 0; k < PS_IPT; k++) {
        const uint64_t i = base + k * 64 + lane;
        key[k] = i < n ? kf(i) : 0u;
        val[k] = VIN ? (i < n ? vin[i] : 0u) : (uint32_t)i;
    }
#pragma unroll
    for (uint32_t k = 0; k < PS_IPT; k++) {
        const uint64_t i = base + k * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = (key[k] >> shift) & mask;
        uint64_t peers = __ballot(valid);
        for (uint32_t b = 0; b < bits; b++) {
            const uint64_t m = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        const uint32_t before = valid ? cw[w][d] : 0u;
        rk[k] = before + (uint32_t)__popcll(peers & below);
        if (valid && (peers & below) == 0) cw[w][d] = before + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // per digit: the waves' prefixes, the tile's total, its start in the
    // tile's digit order (a block scan) and its base in the output
    uint32_t run = 0;
    if (threadIdx.x < bins) {
#pragma unroll
        for (int q = 0; q < NWAVE; q++) {
            const uint32_t c = cw[q][threadIdx.x];
            cw[q][threadIdx.x] = run;
            run += c;
        }
    }
    uint32_t tot;
    const uint32_t start = block_excl_scan<uint32_t>(threadIdx.x < bins ? run : 0u, scan_tmp, tot);
    if (threadIdx.x < bins) { lsd[threadIdx.x] = start; gbs[threadIdx.x] = gbv; }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < PS_IPT; k++) {
        const uint64_t i = base + k * 64 + lane;
        if (i >= n) continue;
        const uint32_t d = (key[k] >> shift) & mask;
        const uint32_t lp = lsd[d] + cw[w][d] + rk[k];
        sk[lp] = key[k];
        sv[lp] = val[k];
    }
    __syncthreads();
    const uint64_t t0 = (uint64_t)tile * PS_TILE;
    const uint32_t cnt = (uint32_t)min<uint64_t>(PS_TILE, n - t0);
    for (uint32_t j = threadIdx.x; j < cnt; j += BLOCK) {
        const uint32_t kk = sk[j], d = (kk >> shift) & mask;
        const uint32_t pos = gbs[d] + (j - lsd[d]);
        if (KOUT) kout[pos] = kk;
        vout[pos] = sv[j];
    }
}

struct SortWork {
    DevBuf<uint32_t> hist;
    ScanWork scan;
};

// Stable sort of the indices 0 .. n-1 by the keys kf(i), bits [0, kb): the
// sorted indices land in `out`; ka/va/kb_/vb are scratch of n entries (the
// middle passes' keys and values).  The first pass computes the keys, the
// last writes values only.
template <class KeyFn>
inline void radix_sort_indices(KeyFn kf, uint32_t n, int kb, uint32_t* out, uint32_t* ka, uint32_t* va,
                               uint32_t* kb_, uint32_t* vb, SortWork& w, hipStream_t st) {
    if (n == 0) return;
    const uint32_t ntiles = (n + PS_TILE - 1) / PS_TILE;
    const int passes = std::max(1, (kb + 7) / 8);
    const uint32_t per = (uint32_t)((std::max(kb, 1) + passes - 1) / passes);
    w.hist.reserve((size_t)256 * ntiles);
    uint32_t *kin = nullptr, *vin = nullptr;
    for (int p = 0; p < passes; p++) {
        const uint32_t shift = (uint32_t)p * per;
        const uint32_t bits = std::min<uint32_t>(per, (uint32_t)std::max(kb, 1) - shift);
        const bool last = p == passes - 1;
        uint32_t* ko = (p % 2 == 0) ? ka : kb_;
        uint32_t* vo = last ? out : ((p % 2 == 0) ? va : vb);
        if (p == 0)
            hipLaunchKernelGGL(k_rs_upsweep_f<KeyFn>, dim3(ntiles), dim3(BLOCK), 0, st, kf, n, shift, bits, w.hist.p,
                               ntiles);
        else
            hipLaunchKernelGGL(k_rs_upsweep_f<KeysIn>, dim3(ntiles), dim3(BLOCK), 0, st, KeysIn{kin}, n, shift, bits,
                               w.hist.p, ntiles);
        exclusive_scan<uint32_t>(w.hist.p, w.hist.p, (uint64_t)ntiles << bits, w.scan, st);
        if (p == 0 && last)
            hipLaunchKernelGGL((k_rs_downsweep_f<KeyFn, false, false>), dim3(ntiles), dim3(BLOCK), 0, st, kf,
                               (const uint32_t*)nullptr, (uint32_t*)nullptr, vo, n, shift, bits,
                               (const uint32_t*)w.hist.p, ntiles);
        else if (p == 0)
            hipLaunchKernelGGL((k_rs_downsweep_f<KeyFn, false, true>), dim3(ntiles), dim3(BLOCK), 0, st, kf,
                               (const uint32_t*)nullptr, ko, vo, n, shift, bits, (const uint32_t*)w.hist.p, ntiles);
        else if (last)
            hipLaunchKernelGGL((k_rs_downsweep_f<KeysIn, true, false>), dim3(ntiles), dim3(BLOCK), 0, st,
                               KeysIn{kin}, (const uint32_t*)vin, (uint32_t*)nullptr, vo, n, shift, bits,
                               (const uint32_t*)w.hist.p, ntiles);
        else
            hipLaunchKernelGGL((k_rs_downsweep_f<KeysIn, true, true>), dim3(ntiles), dim3(BLOCK), 0, st,
                               KeysIn{kin}, (const uint32_t*)vin, ko, vo, n, shift, bits, (const uint32_t*)w.hist.p,
                               ntiles);
        RP_HIP(hipGetLastError());
        kin = ko;
        vin = vo;
    }
}

// Stable sort of n (key, value) pairs by key bits [0, kb).  The pairs are in
// (k0, v0); (k1, v1) is scratch of the same size.  Returns true when the
// sorted pairs ended in (k1, v1).  v0 == nullptr: keys only.
inline bool radix_sort_pairs(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint32_t n, int kb,
                             SortWork& w, hipStream_t st) {
    if (n <= 1 || kb <= 0) return false;
    const uint32_t ntiles = (n + PS_TILE - 1) / PS_TILE;
    const int passes = (kb + 7) / 8;
    const uint32_t per = (uint32_t)((kb + passes - 1) / passes);  // bits per pass (<= 8)
    w.hist.reserve((size_t)256 * ntiles);
    bool flip = false;
    for (uint32_t shift = 0; shift < (uint32_t)kb; shift += per) {
        const uint32_t bits = std::min<uint32_t>(per, (uint32_t)kb - shift);
        uint32_t *ki = flip ? k1 : k0, *vi = flip ? v1 : v0, *ko = flip ? k0 : k1, *vo = flip ? v0 : v1;
        hipLaunchKernelGGL(k_rs_upsweep, dim3(ntiles), dim3(BLOCK), 0, st, (const uint32_t*)ki, n, shift, bits,
                           w.hist.p, ntiles);
        exclusive_scan<uint32_t>(w.hist.p, w.hist.p, (uint64_t)ntiles << bits, w.scan, st);
        if (v0)
            hipLaunchKernelGGL(k_rs_downsweep<true>, dim3(ntiles), dim3(BLOCK), 0, st, (const uint32_t*)ki,
                               (const uint32_t*)vi, ko, vo, n, shift, bits, (const uint32_t*)w.hist.p, ntiles);
        else
            hipLaunchKernelGGL(k_rs_downsweep<false>, dim3(ntiles), dim3(BLOCK), 0, st, (const uint32_t*)ki,
                               (const uint32_t*)nullptr, ko, (uint32_t*)nullptr, n, shift, bits,
                               (const uint32_t*)w.hist.p, ntiles);
        RP_HIP(hipGetLastError());
        flip = !flip;
    }
    return flip;
}

}  // namespace rp
