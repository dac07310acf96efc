// ringpop_amd — shared device definitions (gfx950 / CDNA4).
//
// Encodings used everywhere on the device:
//   status      0 absent, 1 alive, 2 suspect, 3 faulty, 4 leave  (lib/member.js:35-40)
//   view entry  u64 = incarnation << 3 | status   (incarnations are JS integers < 2^53)
//   change      16 B {u32 addr, u32 origin, u64 inc_status}
//   origin      index into a table of {source addr, source incarnation}; the pair is
//               what lib/dissemination.js:91-98 compares, the index is only storage.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rp {

enum : uint32_t { ST_ABSENT = 0, ST_ALIVE = 1, ST_SUSPECT = 2, ST_FAULTY = 3, ST_LEAVE = 4 };

constexpr uint64_t INC0 = 1434401518824ULL;   // node i starts at INC0 + i
constexpr uint64_t T0 = 1500000000000ULL;     // virtual time of round 0
constexpr uint64_t PERIOD_MS = 200;           // lib/swim/gossip.js:127-129
constexpr int REPLICAS = 100;                 // lib/ring.js:28
constexpr int PIGGYBACK_FACTOR = 15;          // lib/dissemination.js:133-136
constexpr uint32_t NONE = 0xFFFFFFFFu;

__host__ __device__ inline uint64_t pack_view(uint64_t inc, uint32_t st) { return (inc << 3) | st; }
__host__ __device__ inline uint32_t v_status(uint64_t v) { return (uint32_t)(v & 7); }
__host__ __device__ inline uint64_t v_inc(uint64_t v) { return v >> 3; }

struct Change {
    uint32_t addr;
    uint32_t origin;
    uint64_t vs;  // inc << 3 | status
};
static_assert(sizeof(Change) == 16, "change record is 16 bytes");

struct Origin {
    uint32_t source;      // NONE: undefined
    uint32_t round;       // makeAlive origins: round of the update (its incarnation is that round's now)
    uint64_t source_inc;  // 0: undefined (JS falsy)
};

// ------------------------------------------------------------- farmhash32
// farmhashmk::Hash32 (npm farmhash ^0.2.0 -> util::Hash32 on default x86-64
// flags).  Same algorithm as oracle/farmhash32.c; see its header for what is
// pinned.
constexpr uint32_t FH_C1 = 0xcc9e2d51u;
constexpr uint32_t FH_C2 = 0x1b873593u;

__host__ __device__ inline uint32_t rotr32(uint32_t v, int s) {
    return s == 0 ? v : (v >> s) | (v << (32 - s));
}
__host__ __device__ inline uint32_t fh_fmix(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}
__host__ __device__ inline uint32_t fh_mur(uint32_t a, uint32_t h) {
    a *= FH_C1; a = rotr32(a, 17); a *= FH_C2;
    h ^= a; h = rotr32(h, 19);
    return h * 5u + 0xe6546b64u;
}

// Fetch a little-endian u32 from a byte pointer without alignment assumptions.
__host__ __device__ inline uint32_t fetch32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// farmhash32 of a len-byte string whose little-endian u32 at byte offset q
// is fetch(q) (q + 4 <= len) and whose byte q is fetch(q) & 0xff.
template <class F>
__host__ __device__ inline uint32_t farmhash32_f(uint32_t len, const F& fetch) {
    if (len <= 4) {
        uint32_t b = 0, c = 9;
        for (uint32_t i = 0; i < len; i++) {
            int32_t v = (int8_t)(fetch(i) & 0xffu);
            b = b * FH_C1 + (uint32_t)v;
            c ^= b;
        }
        return fh_fmix(fh_mur(b, fh_mur(len, c)));
    }
    if (len <= 12) {
        uint32_t a = len, b = len * 5u, c = 9, d = b;
        a += fetch(0);
        b += fetch(len - 4);
        c += fetch((len >> 1) & 4);
        return fh_fmix(fh_mur(c, fh_mur(b, fh_mur(a, d))));
    }
    if (len <= 24) {
        uint32_t a = fetch((len >> 1) - 4), b = fetch(4), c = fetch(len - 8);
        uint32_t d = fetch(len >> 1), e = fetch(0), f = fetch(len - 4);
        uint32_t h = d * FH_C1 + len;
        a = rotr32(a, 12) + f;
        h = fh_mur(c, h) + a;
        a = rotr32(a, 3) + c;
        h = fh_mur(e, h) + a;
        a = rotr32(a + f, 12) + d;
        h = fh_mur(b, h) + a;
        return fh_fmix(h);
    }
    uint32_t h = len, g = FH_C1 * len, f = g;
    uint32_t a0 = rotr32(fetch(len - 4) * FH_C1, 17) * FH_C2;
    uint32_t a1 = rotr32(fetch(len - 8) * FH_C1, 17) * FH_C2;
    uint32_t a2 = rotr32(fetch(len - 16) * FH_C1, 17) * FH_C2;
    uint32_t a3 = rotr32(fetch(len - 12) * FH_C1, 17) * FH_C2;
    uint32_t a4 = rotr32(fetch(len - 20) * FH_C1, 17) * FH_C2;
    h ^= a0; h = rotr32(h, 19); h = h * 5u + 0xe6546b64u;
    h ^= a2; h = rotr32(h, 19); h = h * 5u + 0xe6546b64u;
    g ^= a1; g = rotr32(g, 19); g = g * 5u + 0xe6546b64u;
    g ^= a3; g = rotr32(g, 19); g = g * 5u + 0xe6546b64u;
    f += a4; f = rotr32(f, 19) + 113u;
    uint32_t iters = (len - 1) / 20, s = 0;
    do {
        uint32_t a = fetch(s), b = fetch(s + 4), c = fetch(s + 8);
        uint32_t d = fetch(s + 12), e = fetch(s + 16);
        h += a; g += b; f += c;
        h = fh_mur(d, h) + e;
        g = fh_mur(c, g) + a;
        f = fh_mur(b + e * FH_C1, f) + d;
        f += g; g += f;
        s += 20;
    } while (--iters != 0);
    g = rotr32(g, 11) * FH_C1; g = rotr32(g, 17) * FH_C1;
    f = rotr32(f, 11) * FH_C1; f = rotr32(f, 17) * FH_C1;
    h = rotr32(h + g, 19); h = h * 5u + 0xe6546b64u; h = rotr32(h, 17) * FH_C1;
    h = rotr32(h + f, 19); h = h * 5u + 0xe6546b64u; h = rotr32(h, 17) * FH_C1;
    return h;
}

// Hash of a string held in (possibly unaligned) memory; used for replica
// names, batch hashing and short checksum strings.
__host__ __device__ inline uint32_t farmhash32(const uint8_t* s, uint32_t len) {
    return farmhash32_f(len, [s, len](uint32_t q) -> uint32_t {
        return q + 4 <= len ? fetch32(s + q) : (uint32_t)s[q];
    });
}

// Streaming state for the >24-byte branch once (len, last 20 bytes) are known.
struct FhStream {
    uint32_t h, g, f;
    uint32_t blocks_left;
};
__host__ __device__ inline FhStream fh_stream_begin5(uint32_t len, uint32_t t0, uint32_t t1, uint32_t t2,
                                                     uint32_t t3, uint32_t t4) {
    // t_k = Fetch(s + len - 20 + 4k)
    const uint32_t tail[5] = {t0, t1, t2, t3, t4};
    FhStream st;
    uint32_t h = len, g = FH_C1 * len, f = g;
    uint32_t a0 = rotr32(tail[4] * FH_C1, 17) * FH_C2;  // len-4
    uint32_t a1 = rotr32(tail[3] * FH_C1, 17) * FH_C2;  // len-8
    uint32_t a2 = rotr32(tail[1] * FH_C1, 17) * FH_C2;  // len-16
    uint32_t a3 = rotr32(tail[2] * FH_C1, 17) * FH_C2;  // len-12
    uint32_t a4 = rotr32(tail[0] * FH_C1, 17) * FH_C2;  // len-20
    h ^= a0; h = rotr32(h, 19); h = h * 5u + 0xe6546b64u;
    h ^= a2; h = rotr32(h, 19); h = h * 5u + 0xe6546b64u;
    g ^= a1; g = rotr32(g, 19); g = g * 5u + 0xe6546b64u;
    g ^= a3; g = rotr32(g, 19); g = g * 5u + 0xe6546b64u;
    f += a4; f = rotr32(f, 19) + 113u;
    st.h = h; st.g = g; st.f = f;
    st.blocks_left = (len - 1) / 20;
    return st;
}
__host__ __device__ inline void fh_stream_block(FhStream& st, uint32_t a, uint32_t b, uint32_t c,
                                                uint32_t d, uint32_t e) {
    uint32_t h = st.h, g = st.g, f = st.f;
    h += a; g += b; f += c;
    h = fh_mur(d, h) + e;
    g = fh_mur(c, g) + a;
    f = fh_mur(b + e * FH_C1, f) + d;
    f += g; g += f;
    st.h = h; st.g = g; st.f = f;
}
// fh_stream_block split in two: fh_stream_pre computes everything that
// depends on the block's words only (12-word record, lane-parallel), and
// fh_stream_block_pre runs the part on the h/g/f chain (sequential).
//   h' = rotr((h + a) ^ X(d), 19) * 5 + K + e
//   g' = rotr((g + b) ^ X(c), 19) * 5 + K + a
//   f' = rotr((f + c) ^ X(b + e c1), 19) * 5 + K + d;  f' += g'; g' += f'
// with X(x) = rotr(x c1, 17) c2 and K = 0xe6546b64 (fh_mur)
__host__ __device__ inline void fh_stream_pre(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e,
                                              uint32_t* r) {
    auto X = [](uint32_t x) { return rotr32(x * FH_C1, 17) * FH_C2; };
    r[0] = a; r[1] = b; r[2] = c; r[3] = 0;
    r[4] = X(d); r[5] = X(c); r[6] = X(b + e * FH_C1); r[7] = 0;
    r[8] = 0xe6546b64u + e; r[9] = 0xe6546b64u + a; r[10] = 0xe6546b64u + d; r[11] = 0;
}
// fh_stream_pre with the record sliced by chain: words 4k..4k+2 are what the
// h (k = 0), g (k = 1) or f (k = 2) step adds, xors and adds (word 4k+3 unused)
__host__ __device__ inline void fh_stream_pre_sliced(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e,
                                                     uint32_t* r) {
    auto X = [](uint32_t x) { return rotr32(x * FH_C1, 17) * FH_C2; };
    r[0] = a; r[1] = X(d); r[2] = 0xe6546b64u + e; r[3] = 0;
    r[4] = b; r[5] = X(c); r[6] = 0xe6546b64u + a; r[7] = 0;
    r[8] = c; r[9] = X(b + e * FH_C1); r[10] = 0xe6546b64u + d; r[11] = 0;
}
__host__ __device__ inline void fh_stream_block_pre(FhStream& st, const uint32_t* r) {
    uint32_t h = st.h + r[0], g = st.g + r[1], f = st.f + r[2];
    h = rotr32(h ^ r[4], 19) * 5u + r[8];
    g = rotr32(g ^ r[5], 19) * 5u + r[9];
    f = rotr32(f ^ r[6], 19) * 5u + r[10];
    f += g; g += f;
    st.h = h; st.g = g; st.f = f;
}
__host__ __device__ inline uint32_t fh_stream_end(const FhStream& st) {
    uint32_t h = st.h, g = st.g, f = st.f;
    g = rotr32(g, 11) * FH_C1; g = rotr32(g, 17) * FH_C1;
    f = rotr32(f, 11) * FH_C1; f = rotr32(f, 17) * FH_C1;
    h = rotr32(h + g, 19); h = h * 5u + 0xe6546b64u; h = rotr32(h, 17) * FH_C1;
    h = rotr32(h + f, 19); h = h * 5u + 0xe6546b64u; h = rotr32(h, 17) * FH_C1;
    return h;
}

// ------------------------------------------------------------- PRNG
// Per-node Math.random (harness definition, oracle/harness/common.js):
// splitmix64, top 53 bits as an exact double.
__host__ __device__ inline uint64_t splitmix_next(uint64_t& s) {
    s += 0x9E3779B97F4A7C15ULL;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__host__ __device__ inline double js_math_random(uint64_t& s) {
    return (double)(splitmix_next(s) >> 11) * 0x1p-53;
}
// underscore random(min, max) = min + floor(Math.random() * (max - min + 1))
__host__ __device__ inline int js_random_int(uint64_t& s, int min, int max) {
    double x = js_math_random(s);
    double p = __dmul_rn(x, (double)(max - min + 1));
    return min + (int)floor(p);
}
__host__ __device__ inline uint64_t node_rng_seed(uint64_t seed, uint32_t i) {
    return seed ^ ((uint64_t)(i + 1) * 0xD1B54A32D192ED03ULL);
}
constexpr uint64_t CHURN_XOR = 0x5851F42D4C957F2DULL;
constexpr uint64_t STORM_XOR = 0x2545F4914F6CDD1DULL;  // false-suspicion storm stream (config 5)

// Content fingerprint of one view entry; a view's fingerprint is the sum over
// its addresses (mod 2^64), kept incrementally.  Used only to skip work:
// equal fingerprints are taken as equal views (collision odds 2^-64).
__host__ __device__ inline uint64_t entry_mix(uint32_t a, uint64_t vs) {
    uint64_t x = vs ^ ((uint64_t)(a + 1) * 0x9E3779B97F4A7C15ULL);
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

// Dissemination.adjustMaxPiggybackCount (lib/dissemination.js:38-55):
// 15 * ceil(log10(serverCount + 1)) as an exact integer rule.
__host__ __device__ inline int max_piggyback(int server_count) {
    uint64_t x = (uint64_t)server_count + 1, p = 1;
    int digits = 0;
    for (uint64_t t = x; t; t /= 10) digits++;
    for (int i = 1; i < digits; i++) p *= 10;
    return PIGGYBACK_FACTOR * (x == p ? digits - 1 : digits);
}

}  // namespace rp
