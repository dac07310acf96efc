// Device generation + hashing of a view's checksum string.
//
// lib/membership.js:41-93: members sorted by address (view rows are indexed
// by address rank, so a row already is in that order), each rendered as
// address + status + String(incarnationNumber), joined by ';', then
// farmhash.hash32.  The string is never materialised: one pass measures it,
// a short pass renders the last 20 bytes (farmhash's >24 branch starts from
// the tail), and a streaming pass feeds 20-byte blocks straight into the hash.
#pragma once
#include "rp_common.h"

namespace rp {

constexpr uint32_t ADDR_WORDS = 8;  // little-endian words per address: addresses of up to 32 bytes
struct AddrTable {
    const uint32_t* words;  // ADDR_WORDS words per address
    const uint8_t* len;
};

__device__ __host__ inline uint32_t status_len(uint32_t st) {
    return st == ST_SUSPECT ? 7u : st == ST_FAULTY ? 6u : 5u;
}
// "alive" "suspect" "faulty" "leave" as (first word, second word, second len)
__device__ __host__ inline void status_words(uint32_t st, uint32_t& w0, uint32_t& w1, int& n1) {
    switch (st) {
    case ST_ALIVE: w0 = 0x76696c61u; w1 = 0x65u; n1 = 1; break;      // "aliv" "e"
    case ST_SUSPECT: w0 = 0x70737573u; w1 = 0x746365u; n1 = 3; break; // "susp" "ect"
    case ST_FAULTY: w0 = 0x6c756166u; w1 = 0x7974u; n1 = 2; break;    // "faul" "ty"
    default: w0 = 0x7661656cu; w1 = 0x65u; n1 = 1; break;             // "leav" "e"
    }
}

__device__ __host__ inline uint32_t dec_len(uint64_t v) {
    // incarnations are integers < 2^53 < 10^16
    uint32_t n = 1;
    n += v >= 10ull; n += v >= 100ull; n += v >= 1000ull; n += v >= 10000ull; n += v >= 100000ull;
    n += v >= 1000000ull; n += v >= 10000000ull; n += v >= 100000000ull; n += v >= 1000000000ull;
    n += v >= 10000000000ull; n += v >= 100000000000ull; n += v >= 1000000000000ull;
    n += v >= 10000000000000ull; n += v >= 100000000000000ull; n += v >= 1000000000000000ull;
    n += v >= 10000000000000000ull; n += v >= 100000000000000000ull; n += v >= 1000000000000000000ull;
    n += v >= 10000000000000000000ull;
    return n;
}

// 4 decimal digits of g (< 10000) as ASCII, most significant first in the low byte.
__device__ __host__ inline uint32_t dec4(uint32_t g) {
    uint32_t a = g / 100u, b = g - a * 100u;
    uint32_t d0 = a / 10u, d1 = a - d0 * 10u, d2 = b / 10u, d3 = b - d2 * 10u;
    return (0x30u + d0) | ((0x30u + d1) << 8) | ((0x30u + d2) << 16) | ((0x30u + d3) << 24);
}

// Appends bytes to a 64-bit accumulator and emits whole little-endian words.
template <class Emit>
struct WordSink {
    uint64_t acc = 0;
    uint32_t bits = 0;
    Emit emit;
    __device__ __host__ inline void put(uint32_t w, uint32_t nbytes) {
        uint64_t m = nbytes >= 4 ? 0xFFFFFFFFull : ((1ull << (8 * nbytes)) - 1ull);
        acc |= ((uint64_t)w & m) << bits;
        bits += 8 * nbytes;
        if (bits >= 32) {
            emit((uint32_t)acc);
            acc >>= 32;
            bits -= 32;
        }
    }
};

template <class Sink>
__device__ __host__ inline void put_dec(Sink& s, uint64_t v) {
    // split into 4-digit groups without arrays (keeps everything in registers)
    const uint32_t nd = dec_len(v);
    const uint64_t hi = v / 100000000ull;
    const uint32_t lo = (uint32_t)(v - hi * 100000000ull);
    const uint32_t hi32 = (uint32_t)(hi > 0xFFFFFFFFull ? 0xFFFFFFFFull : hi);
    const uint32_t w0 = dec4(hi32 / 10000u), w1 = dec4(hi32 % 10000u), w2 = dec4(lo / 10000u), w3 = dec4(lo % 10000u);
    const uint32_t ng = (nd + 3) / 4;          // groups used (1..4 for v < 10^16)
    const uint32_t lead = nd - 4 * (ng - 1);   // digits in the leading group
    const uint32_t sh = 8 * (4 - lead);
    if (ng == 4) { s.put(w0 >> sh, lead); s.put(w1, 4); s.put(w2, 4); s.put(w3, 4); }
    else if (ng == 3) { s.put(w1 >> sh, lead); s.put(w2, 4); s.put(w3, 4); }
    else if (ng == 2) { s.put(w2 >> sh, lead); s.put(w3, 4); }
    else { s.put(w3 >> sh, lead); }
}

template <class Sink>
__device__ __host__ inline void put_member(Sink& s, const AddrTable& at, uint32_t a, uint64_t vs) {
    uint32_t L = at.len[a];
    const uint32_t* w = at.words + (size_t)a * ADDR_WORDS;
    for (uint32_t k = 0; k * 4 < L; k++) s.put(w[k], L - 4 * k >= 4 ? 4 : L - 4 * k);
    uint32_t w0, w1; int n1;
    status_words(v_status(vs), w0, w1, n1);
    s.put(w0, 4);
    s.put(w1, (uint32_t)n1);
    put_dec(s, v_inc(vs));
}

// put_member with the address already in registers (L bytes in words wa, wb)
template <class Sink>
__device__ __host__ inline void put_member_regs(Sink& s, uint32_t L, const uint4& wa, const uint4& wb, uint64_t vs) {
    const uint32_t w[ADDR_WORDS] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
    for (uint32_t k = 0; k < ADDR_WORDS; k++)
        if (k * 4 < L) s.put(w[k], L - 4 * k >= 4 ? 4 : L - 4 * k);
    uint32_t w0, w1; int n1;
    status_words(v_status(vs), w0, w1, n1);
    s.put(w0, 4);
    s.put(w1, (uint32_t)n1);
    put_dec(s, v_inc(vs));
}

__device__ __host__ inline uint32_t member_len(const AddrTable& at, uint32_t a, uint64_t vs) {
    return at.len[a] + status_len(v_status(vs)) + dec_len(v_inc(vs));
}

struct TailEmit {
    uint32_t skip_words;  // words to drop before the 5 kept
    uint32_t seen = 0;
    uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    __device__ __host__ inline void operator()(uint32_t w) {
        if (seen >= skip_words) {
            uint32_t k = seen - skip_words;
            if (k == 0) t0 = w; else if (k == 1) t1 = w; else if (k == 2) t2 = w;
            else if (k == 3) t3 = w; else if (k == 4) t4 = w;
        }
        seen++;
    }
};

struct SmallEmit {  // whole string <= 24 bytes: keep 6 words
    uint32_t n = 0;
    uint32_t w[7] = {0, 0, 0, 0, 0, 0, 0};
    __device__ __host__ inline void operator()(uint32_t x) { if (n < 7) w[n] = x; n++; }
};

struct StreamEmit {
    FhStream st;
    uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0, b4 = 0;
    uint32_t nw = 0;
    __device__ __host__ inline void operator()(uint32_t w) {
        b0 = b1; b1 = b2; b2 = b3; b3 = b4; b4 = w;
        if (++nw == 5) {
            nw = 0;
            if (st.blocks_left) {
                fh_stream_block(st, b0, b1, b2, b3, b4);
                st.blocks_left--;
            }
        }
    }
};

// Whole string <= 24 bytes (a view with a single member): render it, hash it.
template <class RowFn>
__device__ __host__ __attribute__((noinline)) uint32_t small_view_checksum(RowFn row, uint32_t n, const AddrTable& at,
                                                                          uint32_t len) {
    WordSink<SmallEmit> s;
    bool first = true;
    for (uint32_t a = 0; a < n; a++) {
        uint64_t vs = row(a);
        if (v_status(vs) == ST_ABSENT) continue;
        if (!first) s.put(0x3Bu, 1);
        first = false;
        put_member(s, at, a, vs);
    }
    s.put(0, 4);  // flush
    uint8_t buf[28];
    for (int k = 0; k < 7; k++) {
        buf[4 * k] = (uint8_t)s.emit.w[k]; buf[4 * k + 1] = (uint8_t)(s.emit.w[k] >> 8);
        buf[4 * k + 2] = (uint8_t)(s.emit.w[k] >> 16); buf[4 * k + 3] = (uint8_t)(s.emit.w[k] >> 24);
    }
    return farmhash32(buf, len);
}

// farmhash32 of the checksum string of one view row (row[a] = inc<<3|status).
template <class RowFn>
__device__ __host__ inline uint32_t view_checksum(RowFn row, uint32_t n, const AddrTable& at) {
    uint64_t len = 0;
    uint32_t cnt = 0, last = 0;
    for (uint32_t a = 0; a < n; a++) {
        uint64_t vs = row(a);
        if (v_status(vs) == ST_ABSENT) continue;
        len += member_len(at, a, vs);
        cnt++;
        last = a;
    }
    if (cnt == 0) return farmhash32(nullptr, 0);
    len += cnt - 1;
    if (len <= 24) return small_view_checksum(row, n, at, (uint32_t)len);
    // Tail: walk back from the last member until >= 20 bytes are covered.
    uint32_t j = last;
    uint64_t T = member_len(at, j, row(j));
    while (T < 20) {
        uint32_t p = j;
        do { p--; } while (v_status(row(p)) == ST_ABSENT);
        j = p;
        T += member_len(at, j, row(j)) + 1;
    }
    // bytes from member j to the end = T; we need bytes [T-20, T).  Pad the
    // front so that T-20 falls on a word boundary.
    uint32_t pad = (uint32_t)((4 - ((T - 20) & 3)) & 3);
    WordSink<TailEmit> ts;
    ts.emit.skip_words = (uint32_t)((T - 20 + pad) / 4);
    if (pad) ts.put(0, pad);
    for (uint32_t a = j; a < n; a++) {
        uint64_t vs = row(a);
        if (v_status(vs) == ST_ABSENT) continue;
        if (a != j) ts.put(0x3Bu, 1);
        put_member(ts, at, a, vs);
    }
    WordSink<StreamEmit> ss;
    ss.emit.st = fh_stream_begin5((uint32_t)len, ts.emit.t0, ts.emit.t1, ts.emit.t2, ts.emit.t3, ts.emit.t4);
    bool first = true;
    for (uint32_t a = 0; a < n && ss.emit.st.blocks_left; a++) {
        uint64_t vs = row(a);
        if (v_status(vs) == ST_ABSENT) continue;
        if (!first) ss.put(0x3Bu, 1);
        first = false;
        put_member(ss, at, a, vs);
    }
    return fh_stream_end(ss.emit.st);
}

// Incremental form for callers that feed members themselves (in address
// order) and know the string length (SimDev::slen) and the last 20 bytes:
// begin(len, tail) / member(a, vs) ... / end().  Requires len > 24.
struct ChecksumStream {
    WordSink<StreamEmit> ss;
    bool first = true;
    __device__ __host__ inline void begin(uint64_t len, const TailEmit& t) {
        ss.emit.st = fh_stream_begin5((uint32_t)len, t.t0, t.t1, t.t2, t.t3, t.t4);
    }
    __device__ __host__ inline void member(const AddrTable& at, uint32_t a, uint64_t vs) {
        if (!ss.emit.st.blocks_left || v_status(vs) == ST_ABSENT) return;
        if (!first) ss.put(0x3Bu, 1);
        first = false;
        put_member(ss, at, a, vs);
    }
    __device__ __host__ inline uint32_t end() const { return fh_stream_end(ss.emit.st); }
};

// The last 20 bytes of a view's checksum string (members from the end until
// >= 20 bytes are covered).
template <class RowFn>
__device__ __host__ inline TailEmit checksum_tail(RowFn row, uint32_t n, const AddrTable& at) {
    uint32_t j = n;
    do { j--; } while (j > 0 && v_status(row(j)) == ST_ABSENT);
    const uint32_t last = j;
    uint64_t T = member_len(at, j, row(j));
    while (T < 20) {
        uint32_t p = j;
        do { p--; } while (v_status(row(p)) == ST_ABSENT);
        j = p;
        T += member_len(at, j, row(j)) + 1;
    }
    uint32_t pad = (uint32_t)((4 - ((T - 20) & 3)) & 3);
    WordSink<TailEmit> ts;
    ts.emit.skip_words = (uint32_t)((T - 20 + pad) / 4);
    if (pad) ts.put(0, pad);
    for (uint32_t a = j; a <= last; a++) {
        uint64_t vs = row(a);
        if (v_status(vs) == ST_ABSENT) continue;
        if (a != j) ts.put(0x3Bu, 1);
        put_member(ts, at, a, vs);
    }
    return ts.emit;
}

}  // namespace rp
