/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle.  Never linked into the product
 * library (ringpop_amd/csrc); only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.
 *
 * Restatement of the 32-bit FarmHash used by the reference:
 *   lib/membership.js:24,57 and lib/ring.js:21,29 call `farmhash.hash32`
 *   from the npm package `farmhash` ^0.2.0 (package.json:30), a node-gyp
 *   addon over Google FarmHash.  Built with default x86-64 flags (no
 *   __SSE4_1__/__SSE4_2__), `util::Hash32` dispatches to
 *   `farmhashmk::Hash32` (== util::Fingerprint32).  The npm package is NOT
 *   vendored in /root/reference and is absent from this image, so this is a
 *   restatement of the published algorithm.
 *
 * Parity status: PARTIALLY PINNED.  Two upstream known answers are
 * reproduced (see tests/test_oracle.py, the known-answer tests at its top):
 *   Hash32("")                         == 0xdc56d17a (3696677242)
 *   Hash32WithSeed("", CreateSeed(0,-1)) == 4223616069
 * which pin c1/c2, Mur, fmix, Rotate, the len<=4 branch and the test-data
 * seed schedule.  The 5..12, 13..24 and >24 branches are unpinned: no
 * reference test or fixture records a farmhash value.
 */
#include "farmhash32.h"

#include <string.h>

static const uint32_t c1 = 0xcc9e2d51u;
static const uint32_t c2 = 0x1b873593u;

static inline uint32_t fetch32(const uint8_t *p) {
    uint32_t r;
    memcpy(&r, p, 4); /* little-endian host */
    return r;
}

static inline uint32_t rotr32(uint32_t v, int s) {
    return s == 0 ? v : (v >> s) | (v << (32 - s));
}

static inline uint32_t fmix(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

static inline uint32_t mur(uint32_t a, uint32_t h) {
    a *= c1;
    a = rotr32(a, 17);
    a *= c2;
    h ^= a;
    h = rotr32(h, 19);
    return h * 5u + 0xe6546b64u;
}

static uint32_t len0to4(const uint8_t *s, size_t len, uint32_t seed) {
    uint32_t b = seed, c = 9;
    for (size_t i = 0; i < len; i++) {
        int8_t v = (int8_t)s[i]; /* upstream: signed char */
        b = b * c1 + (uint32_t)(int32_t)v;
        c ^= b;
    }
    return fmix(mur(b, mur((uint32_t)len, c)));
}

static uint32_t len5to12(const uint8_t *s, size_t len, uint32_t seed) {
    uint32_t a = (uint32_t)len, b = (uint32_t)len * 5u, c = 9, d = b + seed;
    a += fetch32(s);
    b += fetch32(s + len - 4);
    c += fetch32(s + ((len >> 1) & 4));
    return fmix(seed ^ mur(c, mur(b, mur(a, d))));
}

static uint32_t len13to24(const uint8_t *s, size_t len, uint32_t seed) {
    uint32_t a = fetch32(s - 4 + (len >> 1));
    uint32_t b = fetch32(s + 4);
    uint32_t c = fetch32(s + len - 8);
    uint32_t d = fetch32(s + (len >> 1));
    uint32_t e = fetch32(s);
    uint32_t f = fetch32(s + len - 4);
    uint32_t h = d * c1 + (uint32_t)len + seed;
    a = rotr32(a, 12) + f;
    h = mur(c, h) + a;
    a = rotr32(a, 3) + c;
    h = mur(e, h) + a;
    a = rotr32(a + f, 12) + d;
    h = mur(b ^ seed, h) + a;
    return fmix(h);
}

uint32_t oracle_farmhash32(const uint8_t *s, size_t len) {
    if (len <= 24) {
        if (len <= 12) return len <= 4 ? len0to4(s, len, 0) : len5to12(s, len, 0);
        return len13to24(s, len, 0);
    }
    uint32_t h = (uint32_t)len, g = c1 * (uint32_t)len, f = g;
    uint32_t a0 = rotr32(fetch32(s + len - 4) * c1, 17) * c2;
    uint32_t a1 = rotr32(fetch32(s + len - 8) * c1, 17) * c2;
    uint32_t a2 = rotr32(fetch32(s + len - 16) * c1, 17) * c2;
    uint32_t a3 = rotr32(fetch32(s + len - 12) * c1, 17) * c2;
    uint32_t a4 = rotr32(fetch32(s + len - 20) * c1, 17) * c2;
    h ^= a0; h = rotr32(h, 19); h = h * 5u + 0xe6546b64u;
    h ^= a2; h = rotr32(h, 19); h = h * 5u + 0xe6546b64u;
    g ^= a1; g = rotr32(g, 19); g = g * 5u + 0xe6546b64u;
    g ^= a3; g = rotr32(g, 19); g = g * 5u + 0xe6546b64u;
    f += a4; f = rotr32(f, 19) + 113u;
    size_t iters = (len - 1) / 20;
    do {
        uint32_t a = fetch32(s), b = fetch32(s + 4), c = fetch32(s + 8);
        uint32_t d = fetch32(s + 12), e = fetch32(s + 16);
        h += a; g += b; f += c;
        h = mur(d, h) + e;
        g = mur(c, g) + a;
        f = mur(b + e * c1, f) + d;
        f += g; g += f;
        s += 20;
    } while (--iters != 0);
    g = rotr32(g, 11) * c1; g = rotr32(g, 17) * c1;
    f = rotr32(f, 11) * c1; f = rotr32(f, 17) * c1;
    h = rotr32(h + g, 19); h = h * 5u + 0xe6546b64u; h = rotr32(h, 17) * c1;
    h = rotr32(h + f, 19); h = h * 5u + 0xe6546b64u; h = rotr32(h, 17) * c1;
    return h;
}

uint32_t oracle_farmhash32_seed(const uint8_t *s, size_t len, uint32_t seed) {
    if (len <= 24) {
        if (len >= 13) return len13to24(s, len, seed * c1);
        if (len >= 5) return len5to12(s, len, seed);
        return len0to4(s, len, seed);
    }
    uint32_t h = len13to24(s, 24, seed ^ (uint32_t)len);
    return mur(oracle_farmhash32(s + 24, len - 24) + seed, h);
}

/* farmhash-test.cc's per-offset seed schedule (used only by the KAT test). */
uint32_t oracle_farmhash_test_seed(int offset, int salt) {
    uint32_t h = (uint32_t)salt;
    h = h * c1; h ^= h >> 17;
    h = h * c1; h ^= h >> 17;
    h = h * c1; h ^= h >> 17;
    h += (uint32_t)offset;
    h = h * c1; h ^= h >> 17;
    h = h * c1; h ^= h >> 17;
    h = h * c1; h ^= h >> 17;
    return h;
}

void oracle_farmhash32_batch(const uint8_t *bytes, const uint64_t *offsets,
                             size_t n, uint32_t *out) {
    for (size_t i = 0; i < n; i++)
        out[i] = oracle_farmhash32(bytes + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
}
