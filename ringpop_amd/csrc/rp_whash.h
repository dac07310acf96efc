// ringpop_amd — farmhash32 of one long string by one wave.
//
// farmhashmk::Hash32 (rp_common.h) is a single dependent chain over 20-byte
// blocks, so a long string (a membership checksum string: ~35 bytes per
// member, 2.3 MB at 65,536 members) cannot be split across lanes.  What one
// lane cannot do fast is fetch: byte loads from global memory put a memory
// round trip into every block.  Here the wave stages the string through LDS
// in spans of 192 blocks (3,840 bytes, 60 per lane as 16 aligned dword loads
// shifted with alignbyte), loads span i + 1 into registers while it hashes
// span i from LDS, and every lane runs the same chain (the result is
// wave-uniform).  The chain itself bounds it: ~40 dependent instructions per
// 20-byte block (six of them quarter-rate 32-bit multiplies), ~200 cycles,
// about 0.25 GB/s per wave (measured 9.8 ms for 2.3 MB, copy included).  Bytes are read only from aligned dwords that start inside
// the string, so no load crosses into a page the string does not touch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rp_block.h"
#include "rp_common.h"

namespace rp {

constexpr uint32_t WH_BLOCKS = 192;                // 20-byte blocks per span
constexpr uint32_t WH_WORDS = WH_BLOCKS * 5;       // 960 words = 3,840 bytes of LDS
constexpr uint32_t WH_LANE_WORDS = WH_WORDS / 64;  // 15 words per lane
// LDS a caller gives wave_farmhash32: the span, then its blocks' records
// (fh_stream_pre_sliced: 12 words per block) for the chain (FhLanes)
constexpr uint32_t WH_BUF_WORDS = WH_WORDS + 12 * WH_BLOCKS;  // 3,264 words

// x * 5 + r as v_lshl_add_u32 + add (left to itself the compiler picks a
// 64-bit multiply-add, a quarter-rate instruction, on the checksum chain)
__device__ inline uint32_t x5_add(uint32_t x, uint32_t r) {
    uint32_t y;
    asm("v_lshl_add_u32 %0, %1, 2, %1" : "=v"(y) : "v"(x));
    return y + r;
}
// The farmhash chain over block records in the sliced layout
// (fh_stream_pre_sliced), one VALU instruction per step for all three of
// h, g, f: the wave holds h in lane 0, g in lane 4 and f in lane 8 (each
// lane reads its slice, slot = min(lane / 4, 2)); f += g and g += f are
// DPP row shifts by 4 lanes that write one bank (lanes 8-11, then 4-7) of
// each row.  7 VALU per 20-byte block instead of 17, on one dependency chain.
struct FhLanes {
    uint32_t s;     // h | g | f by lane slot
    uint32_t slot;  // min(lane / 4, 2)
    __device__ inline void init(const FhStream& st) {
        slot = min(lane_id() >> 2, 2u);
        s = slot == 0 ? st.h : slot == 1 ? st.g : st.f;
    }
    __device__ inline void step(const uint4& r) {
        uint32_t x = s + r.x;
        x = x5_add(rotr32(x ^ r.y, 19), r.z);
        x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0x4, false);  // row_shr:4 into bank 2: f += g
        x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x104, 0xF, 0x2, false);  // row_shl:4 into bank 1: g += f
        s = x;
    }
    // records [j0, j1) of rec (3 x uint4 per block).  An LDS read's latency
    // is longer than a step's 7 dependent instructions, so reads run 4 to 8
    // blocks ahead: two sets of 4 registers, one read while the other is
    // hashed (no register moves on the way); reads past j1 - 1 re-read it.
    __device__ inline void run(const uint4* rec, uint32_t j0, uint32_t j1) {
        if (j0 >= j1) return;
        const uint32_t jl = j1 - 1;
        auto ld = [&](uint32_t j) { return rec[3 * min(j, jl) + slot]; };
        uint4 a0 = ld(j0), a1 = ld(j0 + 1), a2 = ld(j0 + 2), a3 = ld(j0 + 3);
        uint32_t j = j0;
        for (; j + 8 <= j1; j += 8) {
            const uint4 b0 = ld(j + 4), b1 = ld(j + 5), b2 = ld(j + 6), b3 = ld(j + 7);
            step(a0); step(a1); step(a2); step(a3);
            a0 = ld(j + 8); a1 = ld(j + 9); a2 = ld(j + 10); a3 = ld(j + 11);
            step(b0); step(b1); step(b2); step(b3);
        }
        const uint4 b0 = ld(j + 4), b1 = ld(j + 5), b2 = ld(j + 6);
        if (j < j1) step(a0);
        if (j + 1 < j1) step(a1);
        if (j + 2 < j1) step(a2);
        if (j + 3 < j1) step(a3);
        if (j + 4 < j1) step(b0);
        if (j + 5 < j1) step(b1);
        if (j + 6 < j1) step(b2);
    }
    __device__ inline FhStream get(uint32_t blocks_left) const {
        FhStream st;
        st.h = (uint32_t)__builtin_amdgcn_readlane((int)s, 0);
        st.g = (uint32_t)__builtin_amdgcn_readlane((int)s, 4);
        st.f = (uint32_t)__builtin_amdgcn_readlane((int)s, 8);
        st.blocks_left = blocks_left;
        return st;
    }
};

__device__ inline void wh_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// The 16 aligned dwords covering this lane's 60 bytes of span `span`.
__device__ inline void wh_load(const uint8_t* s, uint32_t len, uint32_t span, uint32_t d[16]) {
    const uintptr_t first = (uintptr_t)s + (uintptr_t)span * (WH_WORDS * 4) + (uintptr_t)lane_id() * 60u;
    const uint32_t* a = (const uint32_t*)(first & ~(uintptr_t)3);
    const uintptr_t end = (uintptr_t)s + len;
#pragma unroll
    for (int k = 0; k < 16; k++) d[k] = (uintptr_t)(a + k) < end ? __builtin_nontemporal_load(a + k) : 0u;
}

// farmhash32(s, len) computed by the calling wave (all 64 lanes, uniform
// control flow); buf: WH_BUF_WORDS words of LDS owned by the wave.  Per span,
// the blocks' data-only mixing runs one block per lane, then the chain one
// VALU step per block for h, g and f together (FhLanes).
__device__ inline uint32_t wave_farmhash32(const uint8_t* s, uint32_t len, uint32_t* buf) {
    if (len <= 24) return farmhash32(s, len);
    const FhStream st0 = fh_stream_begin5(len, fetch32(s + len - 20), fetch32(s + len - 16), fetch32(s + len - 12),
                                          fetch32(s + len - 8), fetch32(s + len - 4));
    uint32_t left = st0.blocks_left;
    FhLanes fl;
    fl.init(st0);
    const uint32_t shift = (uint32_t)((uintptr_t)s & 3u);
    const uint32_t lane = lane_id();
    uint32_t* const pre = buf + WH_WORDS;
    uint32_t d[16];
    wh_load(s, len, 0, d);
    for (uint32_t span = 0; left; span++) {
#pragma unroll
        for (int k = 0; k < 15; k++) buf[lane * WH_LANE_WORDS + k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], shift);
        wh_lds_sync();
        const uint32_t nb = min(WH_BLOCKS, left);
        if (nb < left) wh_load(s, len, span + 1, d);  // in flight while this span hashes
        for (uint32_t j = lane; j < nb; j += 64)
            fh_stream_pre_sliced(buf[5 * j], buf[5 * j + 1], buf[5 * j + 2], buf[5 * j + 3], buf[5 * j + 4], pre + 12 * j);
        wh_lds_sync();
        fl.run((const uint4*)pre, 0, nb);
        left -= nb;
        wh_lds_sync();
    }
    return fh_stream_end(fl.get(0));
}

}  // namespace rp
