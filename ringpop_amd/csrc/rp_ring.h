// ringpop_amd — ring / hashing kernels shared by the C-ABI host code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rp {
__global__ void k_hash_batch(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t* out,
                             uint32_t long_min);
__global__ void k_hash_long(const uint8_t* bytes, const uint64_t* off, const uint32_t* idx, uint32_t* out);
__global__ void k_hash_one(const uint8_t* bytes, uint32_t len, uint32_t* out);
constexpr uint32_t HASH_HOST_MAX = 48 * 1024;  // k_hash_host's LDS copy of the string (+ 13 KB of hash buffer)
__global__ void k_hash_host(const uint4* host, uint32_t len, uint32_t* out);
constexpr uint32_t HASH_LONG_MIN = 1024;  // strings at least this long: one wave each (k_hash_long)
// a scalar call's key, passed by value in the kernel arguments
constexpr uint32_t SMALL_KEY_WORDS = 768;
struct SmallKey {
    uint32_t len;
    uint32_t w[SMALL_KEY_WORDS];
};
__global__ void k_hash_small(SmallKey k, uint32_t* out);
__global__ void k_replica_hashes(const uint8_t* names, const uint64_t* off, uint32_t nserv, int replicas,
                                 uint32_t* out);
__global__ void k_bucket_index(const uint32_t* h, uint32_t n, uint32_t* bucket, uint32_t* bad);
#ifndef RP_DIR_BITS
#define RP_DIR_BITS 21
#endif
constexpr uint32_t DIR_BITS = RP_DIR_BITS;
constexpr uint32_t DIR_SHIFT = 32 - DIR_BITS;
constexpr uint32_t DIR_SIZE = 1u << DIR_BITS;
constexpr uint32_t DIR_ESCAPE = 0x80000000u;
#ifndef RP_LK_KPT
#define RP_LK_KPT 1
#endif
constexpr uint32_t LK_KPT = RP_LK_KPT;  // keys per thread of k_lookup_keys (block tile 256 * LK_KPT)
// The L2-resident directory (rings of < 32,768 servers): 2^D16_BITS 16-bit
// entries (4 MB at 21 bits) -- an owner, or 0x8000 | the bucket's first point
// relative to a per-64-bucket base (coarse, 64 KB).  See rp_ring.hip.
#ifndef RP_D16_BITS
#define RP_D16_BITS 21
#endif
constexpr uint32_t D16_BITS = RP_D16_BITS;
constexpr uint32_t D16_SHIFT = 32 - D16_BITS;
constexpr uint32_t D16_SIZE = 1u << D16_BITS;
constexpr uint32_t D16_GROUP_LOG = 6;  // buckets per coarse base: 64
// rings of at least this many points (at most 4 buckets of each directory per
// point) build their indexes with k_index_build; below it a point owns long
// runs of buckets and the per-bucket kernels' coalesced stores win (a
// 1,000-server ring, 100 k points: 73 us of device time against 148)
constexpr uint32_t INDEX_SCATTER_MIN = DIR_SIZE / 4;
__global__ void k_dir_both(const uint32_t* h, const int32_t* own, uint32_t n, const uint32_t* bucket, uint32_t* dir,
                           uint64_t* packed, uint16_t* dir16, uint32_t* coarse, uint32_t* bad, int do16);
__global__ void k_index_build(const uint32_t* h, const int32_t* own, uint32_t n, uint32_t* bucket, uint32_t* dir,
                              uint64_t* packed, uint16_t* dir16, uint32_t* coarse, uint32_t* bad, int do16);
__global__ void k_lookup_keys(const uint8_t* bytes, const uint64_t* off, uint64_t nk, const uint32_t* dir,
                              const uint64_t* packed, uint32_t n, int32_t* out, uint32_t* hout,
                              const uint16_t* dir16, const uint32_t* coarse, const uint32_t* d16_bad);
__global__ void k_ring_merge(const uint32_t* h, const int32_t* own, uint32_t n, const uint32_t* ins_h,
                             const int32_t* ins_o, uint32_t nins, const uint32_t* del_h, uint32_t ndel, uint32_t* ho,
                             int32_t* oo, uint32_t nout);
// a small delta passed by value: ins hashes | ins owners | del hashes
constexpr uint32_t RING_DELTA_WORDS = 768;  // (3 KB of kernel arguments, as SmallKey)
struct RingDelta {
    uint32_t nins, ndel;
    uint32_t w[RING_DELTA_WORDS];
};
__global__ void k_ring_merge_small(const uint32_t* h, const int32_t* own, uint32_t n, RingDelta d, uint32_t* ho,
                                   int32_t* oo, uint32_t nout, uint32_t* bucket, uint32_t* bad);
#ifndef RP_LK_SPLIT_MIN
#define RP_LK_SPLIT_MIN 0xFFFFFFFFFFFFFFFFull  // off: measured slower
#endif
constexpr uint64_t LK_SPLIT_MIN = RP_LK_SPLIT_MIN;  // batches at least this large take the split lookup
constexpr uint32_t LK_SPLIT_CHUNK = 2048;           // keys read per k_lookup_split block
__global__ void k_lookup_split(const uint32_t* keyh, uint64_t nk, const uint32_t* dir, const uint64_t* packed,
                               uint32_t n, int32_t* out);
__global__ void k_lookup_small(SmallKey k, const uint32_t* dir, const uint64_t* packed, uint32_t n, int32_t* out);
__global__ void k_lookup_hashes(const uint32_t* keyh, uint64_t nk, const uint32_t* dir, const uint64_t* packed,
                                uint32_t n, int32_t* out);
__global__ void k_keygen_len(uint64_t seed, uint64_t nk, uint64_t* len);
__global__ void k_keygen_bytes(uint64_t seed, uint64_t nk, const uint64_t* off, uint8_t* bytes);
}  // namespace rp
