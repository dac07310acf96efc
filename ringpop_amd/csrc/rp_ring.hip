// ringpop_amd — batched farmhash32 and the consistent-hash ring on the device.
//
// HashRing (lib/ring.js) keeps replica points hash32(server + i), i < 100, in
// a red-black tree (lib/rbtree.js).  Here the ring is a sorted array of
// distinct point hashes with their owner; lookup is an inclusive lower bound
// (rbtree.upperBound returns the first key >= h, lib/rbtree.js:263-271) with
// wrap to the minimum (lib/ring.js:138-147), answered for a whole batch of
// keys per launch through a 64K-bucket index on the top 16 hash bits.
#include <hip/hip_runtime.h>
#include "rp_common.h"
#include "rp_ring.h"
#include "rp_whash.h"

namespace rp {

// ------------------------------------------------------------- batch hash
// one lane per string; strings of long_min bytes or more are left to
// k_hash_long
__global__ void k_hash_batch(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t* out,
                             uint32_t long_min) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t o = off[i];
    const uint32_t len = (uint32_t)(off[i + 1] - o);
    if (len < long_min) out[i] = farmhash32(bytes + o, len);
}

// one wave (a 64-thread block) per listed string (rp_whash.h)
__global__ void __launch_bounds__(64) k_hash_long(const uint8_t* bytes, const uint64_t* off, const uint32_t* idx,
                                                  uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[WH_BUF_WORDS];
    const uint32_t i = idx[blockIdx.x];
    const uint64_t o = off[i];
    const uint32_t h = wave_farmhash32(bytes + o, (uint32_t)(off[i + 1] - o), buf);
    if (lane_id() == 0) out[i] = h;
}

// one string of any length by one wave (the ring checksum, lib/ring.js:96-105)
__global__ void __launch_bounds__(64) k_hash_one(const uint8_t* bytes, uint32_t len, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[WH_BUF_WORDS];
    const uint32_t h = wave_farmhash32(bytes, len, buf);
    if (lane_id() == 0) *out = h;
}

// The same for a string in pinned host memory (the ring checksum's server
// string, up to HASH_HOST_MAX bytes): the block's four waves pull it over
// PCIe into LDS with 16-byte loads, all in flight together, then the first
// wave hashes it from there -- instead of a staging copy and its launch
// ahead of k_hash_one.  `host` is coherent (uncached) pinned memory holding
// at least len rounded up to 16 bytes.
__global__ void __launch_bounds__(256) k_hash_host(const uint4* host, uint32_t len, uint32_t* out) {
    __shared__ uint4 str[HASH_HOST_MAX / 16];
    __shared__ __attribute__((aligned(16))) uint32_t buf[WH_BUF_WORDS];
    for (uint32_t i = threadIdx.x; i < (len + 15) / 16; i += blockDim.x) str[i] = host[i];
    __syncthreads();
    if (threadIdx.x >= 64) return;
    const uint32_t h = wave_farmhash32((const uint8_t*)str, len, buf);
    if (lane_id() == 0) *out = h;
}

// replica point hashes hash32(name + decimal(r)) for r < replicas
// (lib/ring.js:50-58).  The string is never materialised: words of
// name ++ digits are fetched from the name in global memory and the decimal
// digits held in two registers, so names of any length hash the same way.
__global__ void k_replica_hashes(const uint8_t* names, const uint64_t* off, uint32_t nserv, int replicas,
                                 uint32_t* out) {
    uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)nserv * replicas) return;
    uint32_t s = (uint32_t)(t / replicas), r = (uint32_t)(t % replicas);
    const uint8_t* nm = names + off[s];
    const uint32_t L = (uint32_t)(off[s + 1] - off[s]);
    uint64_t dig = 0;  // decimal digits of r, first digit in the low byte (at most 8 for r < 10^8)
    uint32_t nd = 0;
    {
        uint8_t d[12];
        uint32_t x = r;
        do { d[nd++] = (uint8_t)('0' + x % 10); x /= 10; } while (x);
        for (uint32_t k = 0; k < nd; k++) dig |= (uint64_t)d[nd - 1 - k] << (8 * k);
    }
    auto byte_at = [&](uint32_t i) -> uint32_t { return i < L ? nm[i] : (uint32_t)(dig >> (8 * (i - L))) & 0xffu; };
    const uint32_t len = L + nd;
    out[t] = farmhash32_f(len, [&](uint32_t q) -> uint32_t {
        if (q + 4 <= L) return fetch32(nm + q);
        uint32_t w = 0;
        for (uint32_t k = 0; k < 4 && q + k < len; k++) w |= byte_at(q + k) << (8 * k);
        return w;
    });
}

// ------------------------------------------------------------- ring build
// An incremental update (rp_capi.hip rp_ring::apply_delta): the host knows the
// exact delta from its mirror of the ring -- `ins` points (hash, owner) whose
// hashes were absent, `del` hashes that were present, both sorted and
// disjoint -- so one pass builds the new sorted point array: a kept old point
// i goes to i - #(del < h_i) + #(ins < h_i), inserted point j to
// j + #(old < x_j) - #(del < x_j).  The delta is small (a few servers'
// replicas): its binary searches stay in L1/L2; the old array streams once.
__device__ inline uint32_t lower_bound_u32(const uint32_t* a, uint32_t m, uint32_t x) {
    uint32_t lo = 0, hi = m;
    while (lo < hi) { const uint32_t mid = (lo + hi) >> 1; if (a[mid] < x) lo = mid + 1; else hi = mid; }
    return lo;
}
// (p < nout always holds when the delta matches the points -- the host
// mirror's invariant; the bound keeps a broken one from writing past them)
__device__ inline void ring_merge_one(uint64_t t, const uint32_t* h, const int32_t* own, uint32_t n,
                                      const uint32_t* ins_h, const int32_t* ins_o, uint32_t nins,
                                      const uint32_t* del_h, uint32_t ndel, uint32_t* ho, int32_t* oo, uint32_t nout) {
    if (t < n) {
        const uint32_t x = h[t];
        const uint32_t d = lower_bound_u32(del_h, ndel, x);
        if (d < ndel && del_h[d] == x) return;  // erased (rbtree.remove by hash, lib/rbtree.js:152)
        const uint32_t p = (uint32_t)t - d + lower_bound_u32(ins_h, nins, x);
        if (p >= nout) return;
        ho[p] = x;
        oo[p] = own[t];
    } else if (t < (uint64_t)n + nins) {
        const uint32_t j = (uint32_t)(t - n), x = ins_h[j];
        const uint32_t p = j + lower_bound_u32(h, n, x) - lower_bound_u32(del_h, ndel, x);
        if (p >= nout) return;
        ho[p] = x;
        oo[p] = ins_o[j];
    }
}
__global__ void k_ring_merge(const uint32_t* h, const int32_t* own, uint32_t n, const uint32_t* ins_h,
                             const int32_t* ins_o, uint32_t nins, const uint32_t* del_h, uint32_t ndel, uint32_t* ho,
                             int32_t* oo, uint32_t nout) {
    ring_merge_one((uint64_t)blockIdx.x * blockDim.x + threadIdx.x, h, own, n, ins_h, ins_o, nins, del_h, ndel, ho,
                   oo, nout);
}
// The same merge with a small delta (a server's replicas: addServer /
// removeServer) in the kernel arguments: no staging copy before the launch.
// Each block copies it to LDS once for its binary searches.  The first 65,537
// threads also move the 16-bit bucket index (k_bucket_index) by the delta in
// place: bucket[b] counts the points below b << 16, so it gains the inserted
// hashes below that key and loses the erased ones; and they reset the
// 16-bit directory's verdict (bad, if any) for k_dir_both.  (bucket null:
// the index is stale, k_bucket_index rebuilds it.)
__global__ void __launch_bounds__(256) k_ring_merge_small(const uint32_t* h, const int32_t* own, uint32_t n,
                                                          RingDelta d, uint32_t* ho, int32_t* oo, uint32_t nout,
                                                          uint32_t* bucket, uint32_t* bad) {
    __shared__ uint32_t w[RING_DELTA_WORDS];
    const uint32_t m = 2 * d.nins + d.ndel;
    for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) w[i] = d.w[i];
    __syncthreads();
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    ring_merge_one(t, h, own, n, w, (const int32_t*)(w + d.nins), d.nins, w + 2 * d.nins, d.ndel, ho, oo, nout);
    if (!bucket) return;
    if (t < 65536u) {
        const uint32_t key = (uint32_t)t << 16;
        bucket[t] = bucket[t] + lower_bound_u32(w, d.nins, key) - lower_bound_u32(w + 2 * d.nins, d.ndel, key);
    } else if (t == 65536u) {
        bucket[t] = nout;
        if (bad) *bad = 0;
    }
}

// Points are kept sorted by hash, one per distinct hash value.
// Adding (rp_capi.hip rp_ring::add): existing points, then the new ones in
// insertion order, stably radix-sorted by hash (rp_sort.h), so the first
// entry of every hash run is the rbtree's surviving inserter.
__global__ void k_bucket_index(const uint32_t* h, uint32_t n, uint32_t* bucket, uint32_t* bad) {
    // bucket[b] = first point with (hash >> 16) >= b, for b in [0, 65536];
    // also resets the 16-bit directory's verdict for k_dir_both (bad, if any)
    uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > 65536u) return;
    uint32_t key = b << 16;
    if (b == 65536u) {
        bucket[b] = n;
        if (bad) *bad = 0;
        return;
    }
    uint32_t lo = 0, hi = n;
    while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (h[m] < key) lo = m + 1; else hi = m; }
    bucket[b] = lo;
}

__device__ inline int32_t ring_find(uint32_t x, const uint32_t* h, const int32_t* own, uint32_t n,
                                    const uint32_t* bucket) {
    if (n == 0) return -1;
    uint32_t top = x >> 16;
    uint32_t lo = bucket[top], hi = bucket[top + 1];
    while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (h[m] < x) lo = m + 1; else hi = m; }
    if (lo == n) lo = 0;  // past the largest point: wrap to rbtree.min()
    return own[lo];
}

// Direct lookup table over the top DIR_BITS hash bits.  Entry for bucket b
// (keys [b << s, (b + 1) << s), s = 32 - DIR_BITS): the owner itself when one
// point answers every key of the bucket (the first point >= the bucket start
// lies at or past its last key, or none does and the lookup wraps to the
// minimum), else DIR_ESCAPE | index of the first point >= the bucket start,
// from which a lookup scans the packed (owner << 32 | hash) points.  With
// 1M points and 2^21 buckets ~38% of keys take the scan (1-2 steps).
// (built by k_dir_both below, or k_index_build for large rings)

// The 16-bit directory: 2^D16_BITS buckets of 2^D16_SHIFT hash values.  A
// bucket without a point boundary inside holds its owner (< 0x8000: rings of
// fewer than 32,768 servers); one with a point inside holds 0x8000 | (index
// of its first point - coarse[bucket >> 6]), the base of its group of 64
// buckets (an offset < 2^15).  Half the bytes of the 32-bit directory at the
// same resolution: 4 MB + 128 KB at 21 bits (config 3, 100 M keys: 1.78 ms
// against 2.15 ms; 20 bits, 2 MB: 1.91 ms, more keys escape to the points).
// *bad != 0: not representable (the host keeps the 32-bit directory).
// (built by k_dir_both below, or k_index_build for large rings)

// The two directories in one launch, a thread per bucket, each first-point
// search narrowed by the 16-bit bucket index (k_bucket_index or
// k_ring_merge_small, launched first): a bucket's first point lies in
// [bucket[top], bucket[top + 1]] of its top-16-bit bucket -- ~1.5 points at
// a 1,000-server ring -- so up to 3 of them are compared from 4 loads issued
// together (one dependent step: index, points, owner), and only fuller
// buckets binary-search.  The 16-bit directory's coarse base (the first
// point of each group of 64 buckets) is the search result of the wave's
// first lane: a wave is one group.
static_assert(D16_GROUP_LOG == 6, "a wave of 64 buckets is one coarse group");
__global__ void __launch_bounds__(256) k_dir_both(const uint32_t* h, const int32_t* own, uint32_t n,
                                                  const uint32_t* bucket, uint32_t* dir, uint64_t* packed,
                                                  uint16_t* dir16, uint32_t* coarse, uint32_t* bad, int do16) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < n) packed[b] = ((uint64_t)(uint32_t)own[b] << 32) | h[b];
    // first point >= key (n: none) and its hash
    auto first_ge = [&](uint32_t key, uint32_t& hv) {
        const uint32_t lo = bucket[key >> 16], hi = bucket[(key >> 16) + 1];
        if (hi - lo <= 3) {
            uint32_t x[4];
#pragma unroll
            for (int j = 0; j < 4; j++) x[j] = lo + j < n ? h[lo + j] : 0xFFFFFFFFu;
            uint32_t c = 0;
#pragma unroll
            for (int j = 0; j < 3; j++) c += ((uint32_t)j < hi - lo && x[j] < key) ? 1u : 0u;
            hv = c == 0 ? x[0] : c == 1 ? x[1] : c == 2 ? x[2] : x[3];
            return lo + c;
        }
        uint32_t l = lo, r = hi;
        while (l < r) { const uint32_t m = (l + r) >> 1; if (h[m] < key) l = m + 1; else r = m; }
        hv = l < n ? h[l] : 0u;
        return l;
    };
    uint32_t hv = 0, lo = 0;
    if (b < DIR_SIZE) {
        const uint32_t start = b << DIR_SHIFT, last = start + ((1u << DIR_SHIFT) - 1u);
        lo = first_ge(start, hv);
        if (lo == n) dir[b] = (uint32_t)own[0];  // past the largest point: rbtree.min()
        else if (hv >= last) dir[b] = (uint32_t)own[lo];
        else dir[b] = DIR_ESCAPE | lo;
    }
    if (!do16 || b >= D16_SIZE) return;
    const uint32_t start = b << D16_SHIFT, last = start + ((1u << D16_SHIFT) - 1u);
    if (D16_SHIFT != DIR_SHIFT || b >= DIR_SIZE) lo = first_ge(start, hv);
    // (every lane of the wave is here: the directory sizes are multiples of 64)
    const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane((int)lo);
    if ((b & ((1u << D16_GROUP_LOG) - 1u)) == 0) coarse[b >> D16_GROUP_LOG] = lo;
    uint32_t e;
    if (lo == n) e = (uint32_t)own[0];
    else if (hv >= last) e = (uint32_t)own[lo];
    else e = 0x8000u | (lo - base);
    if ((e & 0x8000u) ? (lo - base) >= 0x8000u : e >= 0x8000u) atomicOr(bad, 1u);
    dir16[b] = (uint16_t)e;
}

// The three lookup indexes above (k_bucket_index, then k_dir_both)
// in one launch, a thread per point and one past the last: point i is the
// first point >= the start of exactly the buckets (B(h[i-1]), B(h[i])] of
// each directory (B = the hash's top bits), so it writes those entries --
// the owner, or for its own bucket (unless it is that bucket's last hash) an
// escape to itself -- instead of every bucket binary-searching the points;
// the thread past the last writes the buckets after it (wrap to the minimum).
// Rings of at least INDEX_SCATTER_MIN points (fewer: the per-bucket kernels).
__global__ void k_index_build(const uint32_t* h, const int32_t* own, uint32_t n, uint32_t* bucket, uint32_t* dir,
                              uint64_t* packed, uint16_t* dir16, uint32_t* coarse, uint32_t* bad, int do16) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n || n == 0) return;
    const bool last = i == n;
    const uint32_t x = last ? 0u : h[i];
    const uint32_t prev = i ? h[i - 1] : 0u;
    const uint32_t o = (uint32_t)(last ? own[0] : own[i]);
    if (!last) packed[i] = ((uint64_t)o << 32) | x;
    // [b0, b1]: this point's buckets of a directory of 2^(32 - shift) buckets
    auto range = [&](uint32_t shift, uint32_t size, uint32_t& b0, uint32_t& b1) {
        b0 = i ? (prev >> shift) + 1u : 0u;
        b1 = last ? size - 1u : (x >> shift);
    };
    uint32_t b0, b1;
    range(16, 65536u, b0, b1);
    for (uint32_t b = b0; b <= b1 && b0 <= b1; b++) bucket[b] = i;
    if (last) bucket[65536] = n;
    range(DIR_SHIFT, DIR_SIZE, b0, b1);
    const uint32_t lastkey = (1u << DIR_SHIFT) - 1u;
    for (uint32_t b = b0; b <= b1 && b0 <= b1; b++)
        dir[b] = (last || b < b1 || (x & lastkey) == lastkey) ? o : (DIR_ESCAPE | i);
    if (!do16) return;
    range(D16_SHIFT, D16_SIZE, b0, b1);
    const uint32_t lastk16 = (1u << D16_SHIFT) - 1u;
    bool b16 = false;
    for (uint32_t b = b0; b <= b1 && b0 <= b1; b++) {
        if ((b & ((1u << D16_GROUP_LOG) - 1u)) == 0) coarse[b >> D16_GROUP_LOG] = i;
        uint32_t e;
        if (last || b < b1 || (x & lastk16) == lastk16) {
            e = o;
            b16 |= o >= 0x8000u;
        } else {
            // the escape's base: the first point of its group of buckets
            const uint32_t g0 = b & ~((1u << D16_GROUP_LOG) - 1u);
            uint32_t base = i;
            if (g0 < b0) {  // (an earlier point is the group's first)
                uint32_t lo = 0, hi = i;
                const uint32_t key = g0 << D16_SHIFT;
                while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (h[m] < key) lo = m + 1; else hi = m; }
                base = lo;
            }
            e = 0x8000u | (i - base);
            b16 |= (i - base) >= 0x8000u;
        }
        dir16[b] = (uint16_t)e;
    }
    if (b16) atomicOr(bad, 1u);
}

__device__ inline int32_t dir_find(uint32_t x, const uint32_t* dir, const uint64_t* packed, uint32_t n) {
    const uint32_t e = dir[x >> DIR_SHIFT];
    if (!(e & DIR_ESCAPE)) return (int32_t)e;
    for (uint32_t p = e & ~DIR_ESCAPE;; p++) {
        if (p == n) return (int32_t)(uint32_t)(packed[0] >> 32);  // wrap to rbtree.min()
        const uint64_t q = packed[p];
        if ((uint32_t)q >= x) return (int32_t)(uint32_t)(q >> 32);
    }
}

// Scalar calls (rp_hash32, a one-key lookup): the key travels in the kernel
// arguments and the result is written straight to pinned host memory, so a
// call is one launch and one stream synchronisation (no copies).
__device__ inline uint32_t small_key_hash(const SmallKey& k, uint32_t* buf) {
    for (uint32_t w = threadIdx.x; w < (k.len + 3) / 4; w += blockDim.x) buf[w] = k.w[w];
    __syncthreads();
    return wave_farmhash32((const uint8_t*)buf, k.len, buf + SMALL_KEY_WORDS);
}
__global__ void __launch_bounds__(64) k_hash_small(SmallKey k, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[SMALL_KEY_WORDS + WH_BUF_WORDS];
    const uint32_t h = small_key_hash(k, buf);
    if (threadIdx.x == 0) *out = h;
}
__global__ void __launch_bounds__(64) k_lookup_small(SmallKey k, const uint32_t* dir, const uint64_t* packed,
                                                     uint32_t n, int32_t* out) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[SMALL_KEY_WORDS + WH_BUF_WORDS];
    const uint32_t h = small_key_hash(k, buf);
    if (threadIdx.x == 0) *out = n ? dir_find(h, dir, packed, n) : -1;
}

// ring.lookup(key) for a batch of keys (lib/ring.js:138-147): farmhash32 of
// the key string, then the first point >= it.  A block's 256 * LK_KPT keys
// are one contiguous byte span: it is staged in LDS with 16-byte loads and
// each lane hashes its LK_KPT keys from there (unaligned words via
// alignbyte); spans longer than the stage (long keys) hash straight from
// global memory.  The kernel is latency-bound (one dependent chain of
// offsets -> bytes -> directory -> point per key), so each lane keeps its
// LK_KPT chains in flight together: offsets, directory entries and first
// point reads are issued as batches.
#ifndef RP_LK_STAGE256
#define RP_LK_STAGE256 8192
#endif
constexpr uint32_t LK_STAGE = RP_LK_STAGE256 * LK_KPT;  // bytes staged per 256 keys: 32 on average
__global__ void __launch_bounds__(256) k_lookup_keys(const uint8_t* bytes, const uint64_t* off, uint64_t nk,
                                                     const uint32_t* dir, const uint64_t* packed, uint32_t n,
                                                     int32_t* out, uint32_t* hout, const uint16_t* dir16,
                                                     const uint32_t* coarse, const uint32_t* d16_bad) {
    // (the directory build's verdict, read here rather than by the host: a ring
    // update needs no synchronisation before its lookups)
    if (dir16 && *d16_bad) dir16 = nullptr;
    __shared__ __attribute__((aligned(16))) uint8_t stage[LK_STAGE + 16];
    constexpr uint32_t TILE = 256 * LK_KPT;
    const uint64_t i0 = (uint64_t)blockIdx.x * TILE;
    const uint32_t cnt = (uint32_t)min<uint64_t>(TILE, nk - i0);
    const uint64_t first = off[i0], last = off[i0 + cnt], limit = off[nk];
    const uint64_t abase = first & ~15ull;
    const uint64_t span = last - abase;
    // (keys, offsets and owners stream through once: non-temporal, so that
    // the L2 keeps the directory lines the lookups share)
    uint64_t o[LK_KPT], e[LK_KPT];
#pragma unroll
    for (uint32_t j = 0; j < LK_KPT; j++) {
        const uint32_t t = threadIdx.x + 256 * j;
        o[j] = 0; e[j] = 0;
        if (t < cnt) { o[j] = __builtin_nontemporal_load(off + i0 + t); e[j] = __builtin_nontemporal_load(off + i0 + t + 1); }
    }
    uint32_t x[LK_KPT];
    if (span <= LK_STAGE) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const uint32_t nchunk = (uint32_t)((span + 15) >> 4);
        for (uint32_t c = threadIdx.x; c < nchunk; c += 256) {
            const uint64_t g = abase + ((uint64_t)c << 4);
            if (g + 16 <= limit) {
                *(u32x4*)&stage[c << 4] = __builtin_nontemporal_load((const u32x4*)(bytes + g));
            } else {
                for (uint32_t k = 0; k < 16; k++) stage[(c << 4) + k] = g + k < limit ? bytes[g + k] : 0;
            }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < LK_KPT; j++) {
            const uint32_t p0 = (uint32_t)(o[j] - abase);
            auto f = [&](uint32_t q) -> uint32_t {
                const uint32_t a = p0 + q, al = a & ~3u;
                const uint32_t w0 = *(const uint32_t*)&stage[al], w1 = *(const uint32_t*)&stage[al + 4];
                return __builtin_amdgcn_alignbyte(w1, w0, a & 3u);
            };
            x[j] = farmhash32_f((uint32_t)(e[j] - o[j]), f);
        }
    } else {
#pragma unroll
        for (uint32_t j = 0; j < LK_KPT; j++) x[j] = farmhash32(bytes + o[j], (uint32_t)(e[j] - o[j]));
    }
    if (hout) {  // pass 1 of the split lookup: hashes only
#pragma unroll
        for (uint32_t j = 0; j < LK_KPT; j++) {
            const uint32_t t = threadIdx.x + 256 * j;
            if (t < cnt) hout[i0 + t] = x[j];
        }
        return;
    }
    if (n == 0) {
#pragma unroll
        for (uint32_t j = 0; j < LK_KPT; j++) {
            const uint32_t t = threadIdx.x + 256 * j;
            if (t < cnt) out[i0 + t] = -1;
        }
        return;
    }
    // dir_find, batched: every directory entry, then every escape's first point
    uint32_t ent[LK_KPT];
    if (dir16) {  // (the L2-resident directory: escapes rebased to absolute point indices)
        uint32_t e16[LK_KPT];
#pragma unroll
        for (uint32_t j = 0; j < LK_KPT; j++) e16[j] = dir16[x[j] >> D16_SHIFT];
#pragma unroll
        for (uint32_t j = 0; j < LK_KPT; j++)
            ent[j] = (e16[j] & 0x8000u) ? DIR_ESCAPE | (coarse[x[j] >> (D16_SHIFT + D16_GROUP_LOG)] + (e16[j] & 0x7FFFu))
                                        : e16[j];
    } else {
#pragma unroll
        for (uint32_t j = 0; j < LK_KPT; j++) ent[j] = dir[x[j] >> DIR_SHIFT];
    }
    uint64_t q[LK_KPT];
#pragma unroll
    for (uint32_t j = 0; j < LK_KPT; j++) {
        const uint32_t p = ent[j] & ~DIR_ESCAPE;
        q[j] = ((ent[j] & DIR_ESCAPE) && p < n) ? packed[p] : 0;
    }
#pragma unroll
    for (uint32_t j = 0; j < LK_KPT; j++) {
        const uint32_t t = threadIdx.x + 256 * j;
        int32_t r = (int32_t)ent[j];
        if (ent[j] & DIR_ESCAPE) {
            uint32_t p = ent[j] & ~DIR_ESCAPE;
            uint64_t qq = q[j];
            for (;;) {
                if (p == n) { r = (int32_t)(uint32_t)(packed[0] >> 32); break; }  // wrap to rbtree.min()
                if ((uint32_t)qq >= x[j]) { r = (int32_t)(uint32_t)(qq >> 32); break; }
                if (++p < n) qq = packed[p];
            }
        }
        if (t < cnt) __builtin_nontemporal_store(r, out + i0 + t);
    }
}
// Pass 2 of the split lookup.  Resolving hashes in input order makes every
// key one random 128-byte line fetch from an 8 MB directory that no XCD's
// 4 MB L2 holds (PMC: 1.3 L2 misses per key, 16 GB of line traffic per 100 M
// keys).  Here block b resolves only the keys of chunk b / 8 whose hash lies
// in eighth b % 8 of the hash space; dispatch places block b on XCD b % 8, so
// each XCD's L2 sees one eighth of the directory and of the points (1 MB +
// 1 MB).  Correctness does not depend on that placement: every key is
// resolved by exactly one block.
__global__ void __launch_bounds__(256) k_lookup_split(const uint32_t* keyh, uint64_t nk, const uint32_t* dir,
                                                      const uint64_t* packed, uint32_t n, int32_t* out) {
    const uint32_t r = blockIdx.x & 7u;
    const uint64_t c0 = (uint64_t)(blockIdx.x >> 3) * LK_SPLIT_CHUNK;
    uint32_t x[LK_SPLIT_CHUNK / 256];
#pragma unroll
    for (uint32_t j = 0; j < LK_SPLIT_CHUNK / 256; j++) {
        const uint64_t i = c0 + j * 256 + threadIdx.x;
        x[j] = i < nk ? keyh[i] : 0;
    }
#pragma unroll
    for (uint32_t j = 0; j < LK_SPLIT_CHUNK / 256; j++) {
        const uint64_t i = c0 + j * 256 + threadIdx.x;
        if (i < nk && (x[j] >> 29) == r) out[i] = n ? dir_find(x[j], dir, packed, n) : -1;
    }
}
__global__ void k_lookup_hashes(const uint32_t* keyh, uint64_t nk, const uint32_t* dir, const uint64_t* packed,
                                uint32_t n, int32_t* out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nk) return;
    out[i] = n ? dir_find(keyh[i], dir, packed, n) : -1;
}

// decimal strings of seeded u64 keys (config 3): lengths, then bytes
__global__ void k_keygen_len(uint64_t seed, uint64_t nk, uint64_t* len) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nk) return;
    uint64_t s = seed + i * 0x9E3779B97F4A7C15ULL;
    uint64_t v = splitmix_next(s);
    uint32_t nd = 1;
    uint64_t x = v;
    while (x >= 10) { x /= 10; nd++; }
    len[i] = nd;
}
__global__ void k_keygen_bytes(uint64_t seed, uint64_t nk, const uint64_t* off, uint8_t* bytes) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nk) return;
    uint64_t s = seed + i * 0x9E3779B97F4A7C15ULL;
    uint64_t v = splitmix_next(s);
    uint64_t e = off[i + 1];
    do { bytes[--e] = (uint8_t)('0' + v % 10); v /= 10; } while (v);
}

}  // namespace rp
