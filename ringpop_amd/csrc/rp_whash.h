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
// control flow); buf: WH_WORDS words of LDS owned by the wave.
__device__ inline uint32_t wave_farmhash32(const uint8_t* s, uint32_t len, uint32_t* buf) {
    if (len <= 24) return farmhash32(s, len);
    FhStream st = fh_stream_begin5(len, fetch32(s + len - 20), fetch32(s + len - 16), fetch32(s + len - 12),
                                   fetch32(s + len - 8), fetch32(s + len - 4));
    const uint32_t shift = (uint32_t)((uintptr_t)s & 3u);
    const uint32_t lane = lane_id();
    uint32_t d[16];
    wh_load(s, len, 0, d);
    for (uint32_t span = 0; st.blocks_left; span++) {
#pragma unroll
        for (int k = 0; k < 15; k++) buf[lane * WH_LANE_WORDS + k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], shift);
        wh_lds_sync();
        const uint32_t nb = min(WH_BLOCKS, st.blocks_left);
        if (nb < st.blocks_left) wh_load(s, len, span + 1, d);  // in flight while this span hashes
        for (uint32_t j = 0; j < nb; j++)
            fh_stream_block(st, buf[5 * j], buf[5 * j + 1], buf[5 * j + 2], buf[5 * j + 3], buf[5 * j + 4]);
        st.blocks_left -= nb;
        wh_lds_sync();
    }
    return fh_stream_end(st);
}

}  // namespace rp
