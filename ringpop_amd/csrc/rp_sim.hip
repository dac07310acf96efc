// ringpop_amd — device-resident gossip simulation of N ringpop instances.
//
// One gossip round (mirrors oracle/harness/sim.js which runs the
// reference JS) is a fixed sequence of kernels on one HIP stream:
//
//   k_churn     membership.makeAlive(self, now) on the round's churn set
//               (lib/membership.js:141-144,324-352)
//   k_phase1    MembershipIterator.next + Dissemination.issueAsSender for every
//               live node (index.js:458-481, lib/membership-iterator.js:29-52,
//               lib/dissemination.js:78-84,138-182) -> ping messages
//   k_inbox_*   group pings by receiver, in sender-id order
//   k_checksums farmhash snapshots the receivers may compare against
//   k_phase2    per receiver, in sender order: Membership.update(ping.changes)
//               then Dissemination.issueAsReceiver (server/ping-handler.js:22-40)
//   k_pending   resolve full-sync decisions (lib/dissemination.js:102-117)
//   k_phase3    per sender: Membership.update(response.changes)
//               (lib/swim/ping-sender.js:36-39; the second application at
//               index.js:488 is provably a no-op)
//   k_round_end all live views equal? (and the round's counters)
//
// Every node is processed by one 256-thread workgroup; a change batch is
// evaluated 256 changes at a time (all changes of a batch carry distinct
// addresses, so they are independent), and order-dependent side effects
// (dissemination key order, ring insert order) are resolved with block-wide
// ballot/prefix ranks in batch order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "rp_block.h"
#include "rp_checksum.h"
#include "rp_common.h"
#include "rp_sim.h"
#include "rp_whash.h"

namespace rp {

// Log entry: ONE 32-bit word, stamp << 24 | LOG_ALIVE | origin id (23 bits).
// Piggyback counts are implicit: a node's issue counter I advances by one per
// issue, and an entry records I mod 128 when (re)written, so count = (I -
// stamp) mod 128 without any per-issue write (counts never exceed
// maxPiggybackCount + 1 <= 121).  A filtered issue leaves the count where it
// was by bumping the stamp, and sets bit 7: count 0 with bit 7 clear is the
// reference's `undefined` count.  The entry's address and value follow from a
// makeAlive origin (the origin's source, alive at the origin's round); other
// entries keep them in SimDev::dad / dvs, read only when the entry is written
// out, so an issue scans 4 bytes per entry.
constexpr uint32_t ADDR_MASK = 0x00FFFFFFu;
// Origin word carried by changes: table index | flag bits.
constexpr uint32_t ORIGIN_ID_MASK = 0x007FFFFFu;
constexpr uint32_t ORIGIN_ALIVE = 0x80000000u;  // created by makeAlive: all its changes are that one alive update
constexpr uint32_t LOG_ALIVE = ORIGIN_ALIVE >> 8;  // the flag's bit in a log word
constexpr uint32_t LOG_ORIGIN_MASK = ORIGIN_ID_MASK | LOG_ALIVE;
// deleted: the id field all ones without LOG_ALIVE (table slots stay below
// ORIGIN_ID_MASK, makeAlive sequence numbers carry LOG_ALIVE)
constexpr uint32_t TOMB_WORD = 0xFF000000u | ORIGIN_ID_MASK;
constexpr uint32_t STAMP_MASK = 0x7Fu;
constexpr uint32_t STAMP_DEFINED = 0x80u;
__device__ __host__ inline uint32_t log_word(uint32_t origin, uint32_t stamp24) {
    return (origin & ORIGIN_ID_MASK) | ((origin >> 8) & LOG_ALIVE) | stamp24;
}
__device__ __host__ inline uint32_t log_origin(uint32_t w) { return (w & ORIGIN_ID_MASK) | ((w & LOG_ALIVE) << 8); }
// Messages in the arena are written once and read once: they are stored
// non-temporally (streamed past L2) and read with plain loads -- reading
// them non-temporally too measured slower in the box's slow mode (DESIGN
// §6.11: k_p2_apply 487-500 against 447-455 us, the round 4.67 against
// 4.51-4.58 ms) and the same in its fast mode
// (profiles/r06/kstats_msg_loads_modes_r06ak.txt).
#ifndef RP_MSG_NT
#define RP_MSG_NT 1  // bit 0: non-temporal message stores, bit 1: non-temporal loads
#endif
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ inline void store_msg(Change* dst, const Change& c) {
    u32x4 v = {c.addr, c.origin, (uint32_t)c.vs, (uint32_t)(c.vs >> 32)};
    if (RP_MSG_NT & 1) __builtin_nontemporal_store(v, (u32x4*)dst);
    else *(u32x4*)dst = v;
}
template <bool NT = (RP_MSG_NT & 2) != 0>
__device__ inline Change load_msg(const Change* src) {
    u32x4 v = NT ? __builtin_nontemporal_load((const u32x4*)src) : *(const u32x4*)src;
    Change c;
    c.addr = v.x; c.origin = v.y; c.vs = (uint64_t)v.z | ((uint64_t)v.w << 32);
    return c;
}

__device__ __host__ inline bool is_tomb(uint32_t w) { return (w & LOG_ORIGIN_MASK) == ORIGIN_ID_MASK; }
// Table slot of an origin word: a makeAlive origin word carries its sequence
// number (SimDev::alive_base); other words carry their slot (fullSync origins
// 0 .. n-1, the undefined origin n, local suspect/faulty origins from
// lorigin_base).
__device__ __host__ inline uint32_t origin_slot(const SimDev& S, uint32_t w) {
    return (w & ORIGIN_ALIVE) ? S.alive_base + ((w & ORIGIN_ID_MASK) & S.alive_mask) : (w & ORIGIN_ID_MASK);
}
// A makeAlive origin determines its change: {address = source, alive,
// incarnation = now of its round}; log entries and messages with such an
// origin carry no value of their own (SimDev::dvs is not written for them).
__device__ __host__ inline uint64_t alive_value(const Origin& o) { return pack_view(T0 + PERIOD_MS * o.round, ST_ALIVE); }
// The address of the live log entry w at slot i (arow: the log row's dad row).
// (Keeping the address row for makeAlive entries too, so that a merge's
// log-position check reads it beside the word instead of the origin table,
// measured slower in round 5: the origin table is L2-resident, a dad line is not.)
__device__ inline uint32_t entry_addr(const SimDev& S, uint32_t w, const uint32_t* arow, uint32_t i) {
    return (w & LOG_ALIVE) ? S.origins[origin_slot(S, log_origin(w))].source : arow[i];
}
// The change of the live log entry w at slot i (vrow, arow: the log row's dvs, dad rows)
__device__ inline Change log_change(const SimDev& S, uint32_t w, const uint64_t* vrow, const uint32_t* arow, uint32_t i) {
    Change o;
    o.origin = log_origin(w);
    if (w & LOG_ALIVE) {
        const Origin r = S.origins[origin_slot(S, o.origin)];
        o.addr = r.source;
        o.vs = alive_value(r);
    } else {
        o.addr = arow[i];
        o.vs = vrow[i];
    }
    return o;
}
// An entry of a cross-shard message (SimDev::rxw): makeAlive origin word or
// escape index.  (An escape's origin is already in this shard's table: see
// Esc and k_origin_install.)
__device__ inline Change wire_change(const SimDev& S, uint32_t w, const Esc* esc) {
    if (!(w & ORIGIN_ALIVE)) return load_msg(&esc[w].c);
    const Origin o = S.origins[origin_slot(S, w)];
    Change c;
    c.addr = o.source; c.origin = w; c.vs = alive_value(o);
    return c;
}
// Message offsets of ping-req bodies and relay pings (SimDev::pq_off,
// rl_off): the arena, or with RX_MSG set the decoded buffer rxc (the body
// arrived from another shard).
constexpr uint64_t RX_MSG = 1ull << 63;
__device__ inline const Change* slot_msg(const SimDev& S, uint64_t off) {
    return (off & RX_MSG) ? S.rxc + (off & ~RX_MSG) : S.arena + off;
}
__device__ __host__ inline uint32_t entry_count(uint32_t w, uint32_t icount) {
    return (icount - (w >> 24)) & STAMP_MASK;
}
constexpr uint32_t ARENA_SHARDS = 64;
#ifndef RP_SETTLED_GROUP_LOG
#define RP_SETTLED_GROUP_LOG 3  // nodes per gathered settled mask: up to 8
#endif
#ifndef RP_ISSUE_STASH
#define RP_ISSUE_STASH 256  // wg_issue: written entries per wave kept in LDS between the passes
#endif

struct Shared {
    BlockScratch sc;
    uint64_t red[3][NWAVE];
    uint32_t wc[4][4][NWAVE];
    uint32_t u[12];
    uint64_t q[4];
    uint64_t aoff;  // wg_issue: the arena offset of the issue's output
    uint32_t ahead; // wg_apply: the log head at batch start
    // the node scalars the prologue loads and the epilogue updates, kept here
    // rather than in thread 0's registers across the batch / the log scan
    uint64_t a_fp0;
    uint32_t a_dt0, a_dl0, a_th0, i_dl0, a_m0;
    uint32_t i_keep, i_keep_pos;  // wg_issue: identical views at the destination (see there)
    uint32_t i_settled;           // wg_issue: suspect/faulty origins exist (settled members possible)
    // wg_issue: compact the log after the issue.  A slot of its own: waves read
    // it after the issue's last barrier, when wave 0 may already be in the
    // next wg_apply, whose thread 0 writes u[] before that call's first barrier
    uint32_t i_compact;
    uint32_t ims[NWAVE];          // wg_issue's epilogue: per wave, the smallest safe count
    uint64_t itop[2][NWAVE];      // ... and the top-2 keys
    int32_t a_np0;
    // wg_apply: the words of the staged seen bitset its batch changed (bit j
    // of word i: seen word 32 i + j), so only those are written back
    uint32_t seen_dirty[32];
    // wg_issue: the destination's seen bitset; wg_apply: the node's own
    // (SEEN_STAGE_WORDS; staged with one coalesced read)
    alignas(16) uint32_t seen[1024];
    // (everything a full-view merge uses ends with ring: the merge-only
    // kernels allocate the struct only up to there, APPLY_LDS_BYTES)
    union {
        uint32_t ring[1024];  // wg_apply: one chunk's ring adds of servers with colliding replica hashes (batch order)
        struct {
            uint32_t gbase[512];   // wg_issue: per group, the output index of its first written entry (wg_compact: scratch)
            uint64_t imask[512];   // wg_issue: per 64-entry log group, the entries written out (ISSUE_SEG groups)
            // wg_issue: per wave, the written entries of pass 1 in group order
            // (key|origin word; group << 6 | lane), so pass 2 neither re-reads
            // the log nor walks groups with nothing to write
            uint32_t st_kv[NWAVE][RP_ISSUE_STASH];
            uint16_t st_m[NWAVE][RP_ISSUE_STASH];
        };
    };
    uint64_t glm[512];  // wg_issue: the live entries of each 64-entry group of the first segment (prefix packing)
};
// A merge kernel's LDS: the whole struct when it may splice (JOIN), else the
// prefix through `ring`
#define RP_MERGE_SHARED(JOIN_)                                                                    \
    __shared__ __attribute__((aligned(16))) uint8_t sh_raw_[(JOIN_) ? sizeof(Shared) : APPLY_LDS_BYTES_]; \
    Shared& sh = *reinterpret_cast<Shared*>(sh_raw_)
// LDS of a kernel that only merges full views (no issue, no splice): the
// struct up to the end of `ring` (its other users -- wg_compact's gbase -- lie inside)
constexpr size_t APPLY_LDS_BYTES_ = offsetof(Shared, ring) + sizeof(uint32_t) * 1024;
static_assert(offsetof(Shared, gbase) + sizeof(uint32_t) * 512 <= APPLY_LDS_BYTES_, "wg_compact scratch inside the merge LDS");
constexpr uint32_t SEEN_STAGE_WORDS = 1024;  // seen windows up to 32,768 ids are staged in LDS
static_assert(SEEN_STAGE_WORDS == 4 * BLOCK, "stage_seen: one 16-byte load per thread");
// Stage a seen bitset (seen_words words) in LDS: one 16-byte load per thread
// when rows are 16-byte multiples (windows >= 128 ids), so the copy costs one
// memory round trip (a plain loop is compiled to two, load -> wait -> store)
__device__ inline void stage_seen(uint32_t* dst, const uint32_t* src, uint32_t sw) {
    if ((sw & 3u) == 0) {
        if (threadIdx.x < sw / 4) ((uint4*)dst)[threadIdx.x] = ((const uint4*)src)[threadIdx.x];
    } else {
        for (uint32_t w = threadIdx.x; w < sw; w += BLOCK) dst[w] = src[w];
    }
}
constexpr uint32_t ISSUE_SEG = 512;          // 64-entry log groups per wg_issue segment (32,768 entries)
constexpr uint32_t ISSUE_STASH = RP_ISSUE_STASH;
#ifndef RP_ISSUE_UNR
#define RP_ISSUE_UNR 8  // wg_issue pass 1: groups in flight per wave (respond, k_phase2)
#endif
#ifndef RP_SETTLED_PF
#define RP_SETTLED_PF 1  // k_phase1 / k_p2_respond, fault runs: the settled-member checks' loads prefetched (wg_issue SPF)
#endif
#ifndef RP_ISSUE_UNR_P1
#define RP_ISSUE_UNR_P1 8  // the same for issueAsSender in k_phase1 (rocprof means at 65,536: 1.38 ms at 8, 1.49 at 4, 1.56 at 6)
#endif
#ifndef RP_ISSUE_P2U
#define RP_ISSUE_P2U 2  // wg_issue pass 2: groups gathered per step
#endif

// Per-round counters: one column per counter, one row per block index; the
// block's lane 0 owns its cells (no same-address atomics -- those serialise
// at one L2 channel).  k_round_end folds them into S.stats.
__device__ inline void stat_add(const SimDev& S, int i, unsigned long long x) {
    atomicAdd(&S.bstats[(size_t)i * S.bstride + blockIdx.x], x);  // uncontended, no return: no wait
}

// RP_DIAG builds: shader-clock stamps of thread 0, summed per section into the
// STAT_DIAG* counters (tools/diag.py); compiled out otherwise.
#ifndef RP_DIAG_PHASE
#define RP_DIAG_PHASE 2  // the issue whose sections are stamped: 1 = issueAsSender (k_phase1), 2 = issueAsReceiver
#endif
#ifndef RP_DIAG_FINE
#define RP_DIAG_FINE 0  // 1: finer wg_issue sections (prologue and epilogue split; tools/diag.py)
#endif
#ifdef RP_DIAG
__device__ inline uint64_t diag_clock() { return __builtin_amdgcn_s_memtime(); }
#define DIAG_ADD(S_, i_, v_) do { if (threadIdx.x == 0) stat_add(S_, STAT_DIAG0 + (i_), (v_)); } while (0)
#else
__device__ inline uint64_t diag_clock() { return 0; }
#define DIAG_ADD(S_, i_, v_) do { } while (0)
#endif

__device__ inline bool rule_applies(uint32_t ms, uint64_t mi, uint32_t cs, uint64_t ci) {
    // lib/membership-update-rules.js:25-59
    switch (cs) {
    case ST_ALIVE: return ci > mi;
    case ST_SUSPECT: return (ms == ST_SUSPECT && ci > mi) || (ms == ST_FAULTY && ci > mi) ||
                            (ms == ST_ALIVE && ci >= mi);
    case ST_FAULTY: return (ms == ST_SUSPECT && ci >= mi) || (ms == ST_FAULTY && ci > mi) ||
                           (ms == ST_ALIVE && ci >= mi);
    case ST_LEAVE: return ms != ST_LEAVE && ci >= mi;
    default: return false;
    }
}

__device__ inline bool is_pingable_status(uint32_t st) { return st == ST_ALIVE || st == ST_SUSPECT; }

// Workgroup barrier for exchanges through LDS only: waits for this wave's LDS
// traffic, not for its outstanding global stores (__syncthreads would).
__device__ inline void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Three block-wide reductions in one LDS exchange (2 barriers), results to
// every thread.  op 0 = sum, 1 = min (per value, compile-time).
template <int OA, int OB, int OC>
__device__ inline void block_reduce3(uint64_t& a, uint64_t& b, uint64_t& c, Shared& sh) {
    auto comb = [](int op, uint64_t x, uint64_t y) { return op == 0 ? x + y : (x < y ? x : y); };
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a = comb(OA, a, __shfl_xor(a, o));
        b = comb(OB, b, __shfl_xor(b, o));
        c = comb(OC, c, __shfl_xor(c, o));
    }
    const int w = wave_id();
    if (lane_id() == 0) { sh.red[0][w] = a; sh.red[1][w] = b; sh.red[2][w] = c; }
    lds_barrier();
    a = sh.red[0][0]; b = sh.red[1][0]; c = sh.red[2][0];
#pragma unroll
    for (int i = 1; i < NWAVE; i++) {
        a = comb(OA, a, sh.red[0][i]);
        b = comb(OB, b, sh.red[1][i]);
        c = comb(OC, c, sh.red[2][i]);
    }
    lds_barrier();
}

// Four block-wide sums in one LDS exchange (2 barriers), results to every thread.
__device__ inline void block_sum4(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, Shared& sh) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o); b += __shfl_xor(b, o); c += __shfl_xor(c, o); d += __shfl_xor(d, o);
    }
    const int w = wave_id();
    if (lane_id() == 0) { sh.red[0][w] = a; sh.red[1][w] = b; sh.red[2][w] = c; sh.q[w] = d; }
    lds_barrier();
    a = sh.red[0][0]; b = sh.red[1][0]; c = sh.red[2][0]; d = sh.q[0];
#pragma unroll
    for (int i = 1; i < NWAVE; i++) { a += sh.red[0][i]; b += sh.red[1][i]; c += sh.red[2][i]; d += sh.q[i]; }
    lds_barrier();
}

// ---------------------------------------------------------------- ring
// HashRing.addRemoveServers(add, remove) of one applied batch (lib/ring.js:
// 60-94, lib/rbtree.js:70-232) without a serial epilogue.  A view's ring is
// its in-ring server set plus, for each replica hash shared by several
// servers, the owner of that rbtree node (first inserter; erased by hash on
// any owner's removal).  Servers of one batch are distinct, so in-ring bits
// are set/cleared by their own threads.  Collision groups keep the reference
// order (all adds in batch order, then all removes): a removal writes the
// batch's mark (-2 - batch number) into its groups, which adds of the same
// batch treat as occupied and later batches as empty; adds of servers with
// colliding replicas are applied per chunk by one lane in batch order.
__device__ inline int32_t ring_mark(uint32_t batch) { return -2 - (int32_t)(batch & 0x3FFFFFFFu); }
__device__ inline bool coll_free(int32_t owner, int32_t mark) { return owner == -1 || (owner <= -2 && owner != mark); }

// ---------------------------------------------------------------- compaction
// Squeeze tombstones out of node v's dissemination log, keeping key order
// (positions are absolute counters; slot = position mod n).
// Chunks of CK * BLOCK entries: each thread loads its CK entries together
// (one memory round trip), ranks come from per-wave ballots combined in LDS
// (two barriers per chunk).  Entries only move towards the head, and a chunk
// is loaded whole before any of it is written.
#ifndef RP_COMPACT_MUL
#define RP_COMPACT_MUL 4u  // an issue compacts a log whose span exceeds MUL x its live keys + ADD (A/B vs 2x + 1,024: 5.92 vs 5.93-6.17 ms/round)
#endif
#ifndef RP_COMPACT_ADD
#define RP_COMPACT_ADD 8192u
#endif
constexpr int COMPACT_CK = 4;
__device__ void wg_compact(const SimDev& S, uint32_t v, Shared& sh) {
    constexpr int CK = COMPACT_CK;
    static_assert(CK * NWAVE <= 512, "wave counts live in Shared::gbase");
    const size_t base = S.row(v);
    uint32_t* const lrow = S.dko + base;
    uint64_t* const lvrow = S.dvs + base;
    uint32_t* const larow = S.dad + base;
    VEnt* const vrow = S.view + base;
    const uint32_t n = S.n;
    if (threadIdx.x == 0) { sh.u[0] = S.dhead[v]; sh.u[1] = S.dtail[v]; }
    __syncthreads();
    const uint32_t head = sh.u[0], tail = sh.u[1];
    const int lane = lane_id(), wv = wave_id();
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t out = head;  // next output position (block-uniform)
    for (uint32_t p0 = head; p0 < tail; p0 += CK * BLOCK) {
        uint32_t ko[CK], ad[CK];
        uint64_t vs[CK];
#pragma unroll
        for (int k = 0; k < CK; k++) {
            const uint32_t p = p0 + k * BLOCK + threadIdx.x;
            ko[k] = p < tail ? lrow[p % n] : TOMB_WORD;
        }
        uint32_t rk[CK];
#pragma unroll
        for (int k = 0; k < CK; k++) {
            const bool live = !is_tomb(ko[k]);
            vs[k] = 0;
            ad[k] = 0;
            if (live) ad[k] = entry_addr(S, ko[k], larow, (p0 + k * BLOCK + threadIdx.x) % n);
            if (live && !(ko[k] & LOG_ALIVE)) vs[k] = lvrow[(p0 + k * BLOCK + threadIdx.x) % n];
            const uint64_t m = __ballot(live);
            rk[k] = live ? (uint32_t)__popcll(m & below) : NONE;
            if (lane == 0) sh.gbase[k * NWAVE + wv] = (uint32_t)__popcll(m);
        }
        lds_barrier();
        uint32_t before = 0, tot = 0;  // live entries ahead of (k, this wave); in the chunk
#pragma unroll
        for (int k = 0; k < CK; k++) {
#pragma unroll
            for (int w = 0; w < NWAVE; w++) {
                const uint32_t c = sh.gbase[k * NWAVE + w];
                if (rk[k] != NONE && w < wv) rk[k] += c;
                tot += c;
            }
            if (rk[k] != NONE) rk[k] += out + before;
            before = tot;
        }
#pragma unroll
        for (int k = 0; k < CK; k++) {
            const uint32_t q = rk[k], i = q % n;
            if (q == NONE || q == p0 + k * BLOCK + threadIdx.x) continue;  // (dead, or not moving)
            lrow[i] = ko[k];
            if (!(ko[k] & LOG_ALIVE)) { lvrow[i] = vs[k]; larow[i] = ad[k]; }
            vrow[ad[k]].dpos = q;
        }
        out += tot;
        lds_barrier();  // (the next chunk's wave counts reuse gbase)
    }
    if (threadIdx.x == 0) S.dtail[v] = out;
    __syncthreads();
}

#ifndef RP_SEEN_GROUP_LOG
#define RP_SEEN_GROUP_LOG 0  // cross-shard seen masks: per destination node (see DEST_REMOTE)
#endif
#ifndef RP_SEEN_GROUP_LOG_RCCL
#define RP_SEEN_GROUP_LOG_RCCL 2  // the same with one shard per process (RCCL): groups of 4 nodes
#endif
#ifndef RP_SEEN_ROUNDS
#define RP_SEEN_ROUNDS 40
#endif
#ifndef RP_KPT
#define RP_KPT 1  // (2 in round 1; with the merges in launches of their own, 1 measured 5.79-5.83 vs 5.84-5.85 ms/round)
#endif
constexpr int KPT = RP_KPT;                  // changes per thread per chunk
constexpr uint32_t CHUNK = KPT * BLOCK;  // element e of a chunk: k = e / BLOCK, thread = e % BLOCK

// Exclusive ranks (chunk order) of up to NF (3 or 4) flags carried by each of
// a thread's KPT elements, plus the chunk totals; one LDS exchange.
template <int NF>
__device__ inline void multi_rank(const uint32_t (&flags)[KPT], uint32_t (&rank)[KPT][NF], uint32_t (&total)[NF],
                                  Shared& sh) {
    const int lane = lane_id(), w = wave_id();
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t lr[KPT][NF];
#pragma unroll
    for (int k = 0; k < KPT; k++) {
#pragma unroll
        for (int f = 0; f < NF; f++) {
            uint64_t m = __ballot((flags[k] >> f) & 1u);
            lr[k][f] = (uint32_t)__popcll(m & lt);
            if (lane == 0) sh.wc[f][k][w] = (uint32_t)__popcll(m);
        }
    }
    lds_barrier();
#pragma unroll
    for (int f = 0; f < NF; f++) {
        uint32_t run = 0;
#pragma unroll
        for (int k = 0; k < KPT; k++) {
            uint32_t before = 0, tk = 0;
#pragma unroll
            for (int ww = 0; ww < NWAVE; ww++) {
                uint32_t c = sh.wc[f][k][ww];
                before += ww < w ? c : 0u;
                tk += c;
            }
            rank[k][f] = run + before + lr[k][f];
            run += tk;
        }
        total[f] = run;
    }
    lds_barrier();
}

// ---------------------------------------------------------------- seen window
struct SeenWin {
    uint32_t smask, olo, ohi;
};
__device__ inline SeenWin seen_window(const SimDev& S) {
    SeenWin w;
    w.smask = S.seen_words * 32u - 1u;
    w.ohi = S.oc_snap[S.round & 1];
    w.olo = w.ohi > w.smask ? w.ohi - w.smask : 0u;  // W - 1 sequence numbers below ohi
    return w;
}
// Is change (origin o, view value vs) a makeAlive update that node `dest`
// has already evaluated?  Then it is a no-op there (SimDev::seen).  Only
// origins of makeAlive updates qualify: a suspect/faulty origin also labels
// local-override reassertions with varying incarnations.
// A destination on another shard (dest | DEST_REMOTE): the mask of makeAlive
// origins every live node of its group (1 << gsz_log consecutive ids; one
// node by default) had evaluated by the end of the previous round
// (SimDev::gseen; stale is safe: evaluated stays evaluated).  The masks of
// all groups travel once per round: at config 4 on 4 shards per-node masks
// (N x W/8 = 256 MB all-gathered) cut the ping/response all-to-alls from 550
// to 172 MB per round against groups of 32 (8 MB of masks), and the merge
// kernels' time by 13 %.
// Both are staged in LDS by wg_issue (the window is at most SEEN_STAGE_WORDS).
constexpr uint32_t DEST_REMOTE = 0x80000000u;

// ---------------------------------------------------------------- pingable bits
// Per local node, one bit per address: the member is pingable (alive or
// suspect) in the node's view.  Kept next to the seen rows (in SimDev::seen,
// so the merge kernels need no new kernel-argument fields) by the merges'
// status changes and rebuilt from the view by k_init_fp.  The ping-req member
// selection walks the member order against these bits (8 KB per node at
// 65,536, L2-resident) instead of one random view-cell line per member.
__device__ inline uint32_t* ping_bits(const SimDev& S, uint32_t v) {
    return S.seen + (size_t)S.nl * S.seen_words + (size_t)(v - S.lo) * ((S.n + 31) / 32);
}
__device__ inline bool ping_bit(const uint32_t* b, uint32_t a) { return (b[a >> 5] >> (a & 31)) & 1u; }

// ---------------------------------------------------------------- settled bits
// Per local node, one bit per address a != v: the node's view holds a as
// faulty at a's first incarnation INC0 + a.  A change for a with
// incarnation <= INC0 + a that is not a leave is then a no-op there: its
// (incarnation, status) key cannot exceed (INC0 + a, faulty) -- and a's own
// view is excluded (the local override reasserts it whatever the key).  The
// reference value is fixed, so a bit goes stale only through the node's own
// merges, which keep it (wg_apply), or through bulk view writes, after which
// k_init_fp rebuilds it.  A mass failure's faulty updates (config 5) are
// nearly all of this kind: once settled, a receiver drops them without
// reading the view cell (one L2-resident word of an n/8-byte row instead of
// a random line of the n x 16-byte view row).  Stored after the pingable bits.
__device__ inline uint32_t* settled_bits(const SimDev& S, uint32_t v) {
    const size_t pw = (S.n + 31) / 32;
    return S.seen + (size_t)S.nl * S.seen_words + (size_t)S.nl * pw + (size_t)(v - S.lo) * pw;
}
__device__ inline bool settles(uint32_t v, uint32_t a, uint64_t vs) {
    return a != v && v_status(vs) == ST_FAULTY && v_inc(vs) == INC0 + a;
}

// ---------------------------------------------------------------- splices
// New members of a batch (absent from v's view) are spliced into the member
// list at getJoinPosition() = floor(Math.random() * members.length)
// (lib/membership.js:99-101, 285-298), one after the other in batch order:
// the j-th drew x_j (v's Math.random stream, draw j of the batch) and went to
// floor(x_j * (M + j)) of the list as it then was.  The batch's addresses
// wait at ord[M + j] (free: a view holds at most n members); groups of up to
// SPLICE_G inserts are applied in turn (sequential splices compose).  Within
// a group the final slot of insert t is p_t shifted right once per later
// insert at or before it; old member r then lands at r + #{final slots -
// rank <= r}.  Old members only move right, so they move in place from the
// top down.
constexpr uint32_t SPLICE_G = 1024;
__device__ void wg_splice(const SimDev& S, uint32_t v, uint32_t M, uint32_t J, Shared& sh) {
    uint32_t* ord = S.order + S.row(v);
    uint32_t* la = sh.ring;  // the group's addresses (the whole 12 KB union)
    uint32_t* lp = la + SPLICE_G;       // positions drawn, then final slots
    uint32_t* lh = lp + SPLICE_G;       // final slots ascending, minus their rank
    const uint64_t s0 = S.rng[v];
    for (uint32_t g0 = 0; g0 < J; g0 += SPLICE_G) {
        const uint32_t G = min(SPLICE_G, J - g0), Mg = M + g0;
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < G; t += BLOCK) {
            const uint32_t j = g0 + t;
            la[t] = ord[M + j];
            uint64_t st = s0 + (uint64_t)j * 0x9E3779B97F4A7C15ull;
            lp[t] = (uint32_t)floor(js_math_random(st) * (double)(M + j));
        }
        __syncthreads();
        uint32_t fin[SPLICE_G / BLOCK];
#pragma unroll
        for (uint32_t q = 0; q < SPLICE_G / BLOCK; q++) {
            const uint32_t t = threadIdx.x + q * BLOCK;
            uint32_t f = t < G ? lp[t] : 0u;
            if (t < G)
                for (uint32_t i = t + 1; i < G; i++) f += lp[i] <= f;
            fin[q] = f;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t q = 0; q < SPLICE_G / BLOCK; q++)
            if (threadIdx.x + q * BLOCK < G) lp[threadIdx.x + q * BLOCK] = fin[q];
        __syncthreads();
#pragma unroll
        for (uint32_t q = 0; q < SPLICE_G / BLOCK; q++) {
            const uint32_t t = threadIdx.x + q * BLOCK;
            if (t < G) {
                const uint32_t f = lp[t];
                uint32_t r = 0;
                for (uint32_t i = 0; i < G; i++) r += lp[i] < f;
                lh[r] = f - r;
            }
        }
        __syncthreads();
        for (int64_t c0 = (int64_t)((Mg + BLOCK - 1) / BLOCK) * BLOCK - BLOCK; c0 >= 0; c0 -= BLOCK) {
            const uint32_t r = (uint32_t)c0 + threadIdx.x;
            uint32_t a = 0, np = 0;
            if (r < Mg) {
                a = ord[r];
                uint32_t lo = 0, hi = G;
                while (lo < hi) {
                    const uint32_t m = (lo + hi) >> 1;
                    if (lh[m] <= r) lo = m + 1; else hi = m;
                }
                np = r + lo;
            }
            __syncthreads();
            if (r < Mg) ord[np] = a;
            __syncthreads();
        }
        for (uint32_t t = threadIdx.x; t < G; t += BLOCK) ord[lp[t]] = la[t];
    }
    __syncthreads();
}

// ---------------------------------------------------------------- apply
// Membership.update(changes) for node v followed by the update listener
// (lib/membership.js:208-313, lib/membership-update-listener.js:24-75).
// src(i) yields the i-th change of the batch (distinct addresses, so the
// rule evaluations are independent); order-dependent effects (new
// dissemination keys, suspicion timers, ring inserts) take chunk-order ranks.
// L = entries present in src; Llog = length of the reference's change list
// (the sender left out entries that were provably no-ops here).
// JOIN: members absent from the view are taken wholesale and spliced in
// (wg_splice); without it (the full-view hot kernels of a cluster that has
// no absent members) such a change is an error.
// The node scalars wg_apply's prologue reads (thread 0).  A caller that knows
// the node before it knows the batch (k_phase3: the node is the block's, the
// batch comes with the response record) loads them -- and stages the seen
// bitset -- in the same round trip as that record (PRE).
struct ApplyPro {
    uint32_t dh, tt, ic, dt0, th0, dl0, rb, m0;
    uint64_t fp0;
    int32_t np0;
};
__device__ inline ApplyPro load_apply_pro(const SimDev& S, uint32_t v, bool join) {
    ApplyPro p;
    p.dh = S.dhead[v]; p.tt = S.ttail[v]; p.ic = S.icount[v]; p.dt0 = S.dtail[v]; p.th0 = S.thead[v];
    p.dl0 = S.dlive[v]; p.fp0 = S.fp[v]; p.np0 = S.npingable[v]; p.rb = S.rbatch[v];
    p.m0 = join ? S.mcount[v] : 0u;
    return p;
}
template <bool JOIN = true, bool PRE = false, class Src>
__device__ uint32_t wg_apply(const SimDev& S, uint32_t v, const Src& src, uint32_t L, uint32_t Llog, uint64_t now,
                             uint32_t eval_weight, int phase, Shared& sh, const ApplyPro* pre = nullptr) {
    if (L == 0) {
        if (threadIdx.x == 0 && Llog) {
            stat_add(S, STAT_EVALUATED, (unsigned long long)Llog * eval_weight);
            if (phase == 2) stat_add(S, STAT_EVAL_P2, (unsigned long long)Llog);
            if (phase == 3) stat_add(S, STAT_EVAL_P3, (unsigned long long)Llog);
        }
        return 0;
    }
    const uint32_t n = S.n;
    const size_t base = S.row(v);
    // the node's rows as uniform base pointers: per-change addresses are then
    // a scalar base plus a 32-bit lane offset
    VEnt* const vrow = S.view + base;
    uint32_t* const lrow = S.dko + base;
    uint64_t* const lvrow = S.dvs + base;
    uint32_t* const larow = S.dad + base;
    uint8_t* const rrow = S.in_ring + base;
    uint32_t* const srow = S.seen + S.srow(v);
    uint32_t* const fbits = settled_bits(S, v);
    // the node's seen bitset is staged in LDS, in flight with its scalars: a
    // change's seen check is then no global round trip (a batch holds
    // distinct addresses, hence distinct makeAlive origins, so the copy needs
    // no updates within the batch; only this block writes v's bitset)
    if (!PRE) stage_seen(sh.seen, srow, S.seen_words);
    // the first chunk's changes are in flight with them (the batch is
    // written before this call, and no step below rewrites it)
    Change c[KPT];
    auto load_chunk = [&](uint32_t c0) {
#pragma unroll
        for (int k = 0; k < KPT; k++) {
            const uint32_t i = c0 + k * BLOCK + threadIdx.x;
            if (i < L) c[k] = src(i);
            else { c[k].addr = NONE; c[k].origin = 0; c[k].vs = 0; }
        }
    };
    load_chunk(0);
    if (threadIdx.x < 32) sh.seen_dirty[threadIdx.x] = 0;
    // lane 0 loads the node's scalars once; the epilogue only stores
    if (threadIdx.x == 0) {
        const ApplyPro p = PRE ? *pre : load_apply_pro(S, v, JOIN);
        sh.a_dt0 = p.dt0; sh.a_dl0 = p.dl0; sh.a_th0 = p.th0; sh.a_fp0 = p.fp0; sh.a_np0 = p.np0;
        sh.u[3] = (p.dt0 - p.dh) + L > n;
        sh.u[9] = p.rb;
        sh.u[4] = p.dt0; sh.u[8] = p.tt; sh.u[10] = p.ic; sh.u[11] = p.tt != p.th0;
        sh.ahead = p.dh;
        if (JOIN) sh.a_m0 = p.m0;
    }
    __syncthreads();
    if (sh.u[3]) {
        wg_compact(S, v, sh);
        if (threadIdx.x == 0) { sh.a_dt0 = S.dtail[v]; sh.u[4] = sh.a_dt0; stat_add(S, STAT_COMPACT_APPLY, 1); }
        __syncthreads();
    }
    uint32_t tail = sh.u[4], ttail = sh.u[8];
    const uint32_t head = sh.ahead;
    const int32_t mark = ring_mark(sh.u[9]);
    const bool timers_live = sh.u[11] != 0;  // suspicion timers pending at batch start
    const uint32_t stamp = (sh.u[10] & STAMP_MASK) << 24;  // count undefined until the next issue
    const SeenWin win = seen_window(S);
    const uint32_t smask = win.smask, olo = win.olo, ohi = win.ohi;

    uint64_t fp_delta = 0;
    uint32_t napplied = 0, ntouched = 0;
    int32_t dping = 0, dslen = 0;  // pingable members, checksum string length + members (SimDev::slen)
    const AddrTable at{S.addr_words, S.addr_len};
    uint64_t ringops = 0;  // adds | removes << 32
    uint32_t ins = 0;      // JOIN: new members so far (batch order)
    constexpr int NF = JOIN ? 4 : 3;
    for (uint32_t c0 = 0; c0 < L; c0 += CHUNK) {
        if (c0) load_chunk(c0);
        uint64_t cur[KPT];
        uint32_t seen_bit[KPT];  // 0: untracked; else the bit to set once evaluated
#pragma unroll
        for (int k = 0; k < KPT; k++) {
            seen_bit[k] = 0;
            // only origins of makeAlive updates: a suspect/faulty origin can
            // also label local-override reassertions with varying incarnations
            const uint32_t o = c[k].origin & ORIGIN_ID_MASK;
            if (c[k].addr != NONE && (c[k].origin & ORIGIN_ALIVE) && ((o - olo) & ORIGIN_ID_MASK) < ohi - olo) {
                const uint32_t wi = (o & smask) >> 5;
                const uint32_t w = sh.seen[wi];
                if ((w >> (o & 31)) & 1u) c[k].addr = NONE;  // already evaluated here: a no-op
                else seen_bit[k] = 1u << (o & 31);
            }
        }
        // settled faulty members (settled_bits): a key at or below (INC0 + a,
        // faulty) is a no-op without a view-cell read (never true for a
        // makeAlive origin's change, whose incarnation is a round's now)
#pragma unroll
        for (int k = 0; k < KPT; k++) {
            const uint32_t a = c[k].addr & ADDR_MASK;
            if (c[k].addr != NONE && a != v && v_status(c[k].vs) != ST_LEAVE && v_inc(c[k].vs) <= INC0 + a &&
                ((fbits[a >> 5] >> (a & 31)) & 1u))
                c[k].addr = NONE;
        }
        uint32_t cpos[KPT];  // the cell's log position comes with the value (same 16 B)
        uint32_t ctst[KPT];  // and its timer stamp (the cell is rewritten whole)
#pragma unroll
        for (int k = 0; k < KPT; k++) {
            cur[k] = 0;
            cpos[k] = NONE;
            ctst[k] = 0;
            if (c[k].addr != NONE) {
                ntouched++;
                const u32x4 cell = *(const u32x4*)&vrow[c[k].addr & ADDR_MASK];
                cur[k] = (uint64_t)cell.x | ((uint64_t)cell.y << 32);
                cpos[k] = cell.z;
                ctst[k] = cell.w;
            }
        }
        uint32_t flags[KPT];
        // (the value to store is c[k].vs: overwritten for a local override)
#pragma unroll
        for (int k = 0; k < KPT; k++) {
            flags[k] = 0;
            // (set in the staged copy; its changed words are written back after the batch)
            if (seen_bit[k]) {
                const uint32_t wi = ((c[k].origin & ORIGIN_ID_MASK) & smask) >> 5;
                atomicOr(&sh.seen[wi], seen_bit[k]);
                atomicOr(&sh.seen_dirty[wi >> 5], 1u << (wi & 31));
            }
            if (c[k].addr == NONE) continue;
            const uint32_t a = c[k].addr & ADDR_MASK;
            const uint32_t cs = v_status(cur[k]), st = v_status(c[k].vs);
            bool ap = false;
            if (cs == ST_ABSENT) {
                if (JOIN) {
                    ap = true;  // first time seen: taken wholesale (lib/membership.js:237-240)
                    flags[k] |= 8u;
                } else {
                    atomicOr(S.err, SIMERR_ABSENT_MEMBER);
                }
            } else if (a == v && (st == ST_SUSPECT || st == ST_FAULTY)) {
                ap = true;  // local override: reassert alive (lib/membership.js:244-254)
                c[k].vs = pack_view(now, ST_ALIVE);
            } else {
                ap = rule_applies(cs, v_inc(cur[k]), st, v_inc(c[k].vs));
            }
            if (!ap) continue;
            const uint64_t nv = c[k].vs;
            flags[k] |= 16u;  // the cell is stored after the ranks
            fp_delta += entry_mix(a, nv) - entry_mix(a, cur[k]);
            // a cell's log position goes stale when its entry expires (the
            // issue does not clear it): valid iff the slot, inside the live
            // window, still holds this address's key
            uint32_t pos = cpos[k];
#ifdef RP_DIAG_APPLY
            // (diagnostic builds: how the applied changes' log-position checks go)
            uint32_t dg_inwin = 0, dg_alive = 0, dg_tomb = 0;
#endif
            if (pos != NONE) {
                if (pos - head >= tail - head) {
                    pos = NONE;
                } else {
                    const uint32_t w = lrow[pos % n];
#ifdef RP_DIAG_APPLY
                    dg_inwin = 1; dg_alive = (w & LOG_ALIVE) && !is_tomb(w); dg_tomb = is_tomb(w);
#endif
                    if (is_tomb(w) || entry_addr(S, w, larow, pos % n) != a) pos = NONE;
                }
            }
#ifdef RP_DIAG_APPLY
            atomicAdd(&S.stats[STAT_DIAG0], 1ull);
            if (cpos[k] != NONE) atomicAdd(&S.stats[STAT_DIAG0 + 1], 1ull);
            if (dg_inwin) atomicAdd(&S.stats[STAT_DIAG0 + 2], 1ull);
            if (dg_tomb) atomicAdd(&S.stats[STAT_DIAG0 + 3], 1ull);
            if (dg_alive) atomicAdd(&S.stats[STAT_DIAG0 + 4], 1ull);
            if (pos != NONE) atomicAdd(&S.stats[STAT_DIAG0 + 5], 1ull);
#endif
            if (pos != NONE) {  // overwrite keeps key order
                const uint32_t i = pos % n;
                lrow[i] = log_word(c[k].origin, stamp);
                if (!(c[k].origin & ORIGIN_ALIVE)) { lvrow[i] = nv; larow[i] = a; }
            } else {
                flags[k] |= 1u;  // new dissemination key
            }
            const uint32_t ns = v_status(nv);
            if (ns == ST_SUSPECT) {
                if (a != v) flags[k] |= 2u;               // suspicion.start (self is skipped)
            } else {
                if (timers_live) ctst[k] = 0;
            }
            // an alive member is always in the ring (added by every alive update,
            // removed only by faulty/leave): skip the lookup then
            const bool inr = cs == ST_ALIVE || rrow[a] != 0;
            if (ns == ST_ALIVE && !inr) {
                rrow[a] = 1;
                ringops += 1;
                if (S.coll_off[a + 1] != S.coll_off[a]) flags[k] |= 4u;  // group owners: in batch order below
            }
            if ((ns == ST_FAULTY || ns == ST_LEAVE) && inr) {
                rrow[a] = 0;
                ringops += 1ull << 32;
                for (uint32_t q = S.coll_off[a], qe = S.coll_off[a + 1]; q < qe; q++)
                    S.coll_owner[S.crow(v) + S.coll_ids[q]] = mark;  // erased after this batch's adds
            }
            if (is_pingable_status(ns) != is_pingable_status(cs)) {
                uint32_t* const pb = ping_bits(S, v) + (a >> 5);
                if (is_pingable_status(ns)) atomicOr(pb, 1u << (a & 31));
                else atomicAnd(pb, ~(1u << (a & 31)));
                if (a != v) dping += is_pingable_status(ns) ? 1 : -1;
            }
            if (settles(v, a, nv) != settles(v, a, cur[k])) {
                if (settles(v, a, nv)) atomicOr(&fbits[a >> 5], 1u << (a & 31));
                else atomicAnd(&fbits[a >> 5], ~(1u << (a & 31)));
            }
            // (a new member adds its string and a ';' separator)
            dslen += (int32_t)member_len(at, a, nv) - (cs == ST_ABSENT ? -1 : (int32_t)member_len(at, a, cur[k]));
            napplied++;
        }
        uint32_t rank[KPT][NF], total[NF];
        multi_rank<NF>(flags, rank, total, sh);
#pragma unroll
        for (int k = 0; k < KPT; k++) {
            if (!flags[k]) continue;
            const uint32_t a = c[k].addr & ADDR_MASK;
            uint32_t dpos = cpos[k], tst = ctst[k];
            if (flags[k] & 1u) {
                const uint32_t p = tail + rank[k][0];
                const uint32_t i = p % n;
                lrow[i] = log_word(c[k].origin, stamp);
                if (!(c[k].origin & ORIGIN_ALIVE)) { lvrow[i] = c[k].vs; larow[i] = a; }
                dpos = p;
            }
            if (flags[k] & 2u) {  // timers are created in listener (batch) order
                const uint32_t p = ttail + rank[k][1];
                S.tfifo[S.trow(v) + p % S.tcap] = make_uint2(a, S.round);
                tst = p + 1;
            }
            if (flags[k] & 16u) {
                u32x4 cell;
                cell.x = (uint32_t)c[k].vs; cell.y = (uint32_t)(c[k].vs >> 32); cell.z = dpos; cell.w = tst;
                *(u32x4*)&vrow[a] = cell;
            }
            if (flags[k] & 4u) sh.ring[rank[k][2]] = a;
            if (JOIN && (flags[k] & 8u)) S.order[base + sh.a_m0 + ins + rank[k][NF - 1]] = a;  // spliced below
        }
        if (total[2]) {  // rbtree inserts of colliding replica hashes, in batch order
            lds_barrier();
            if (threadIdx.x == 0) {
                for (uint32_t j = 0; j < total[2]; j++) {
                    const uint32_t s = sh.ring[j];
                    for (uint32_t q = S.coll_off[s], qe = S.coll_off[s + 1]; q < qe; q++) {
                        int32_t* o = &S.coll_owner[S.crow(v) + S.coll_ids[q]];
                        if (coll_free(*o, mark)) *o = (int32_t)s;
                    }
                }
            }
            lds_barrier();
        }
        tail += total[0];
        ttail += total[1];
        if (JOIN) ins += total[NF - 1];
    }
    if (JOIN && ins) wg_splice(S, v, sh.a_m0, ins, sh);
    // applied and touched share a sum (each < 2^32); so do pingable and
    // length deltas: dping * 2^32 + dslen (|dslen| < 2^31)
    uint64_t fp_tot = fp_delta, ap_tot = napplied | ((uint64_t)ntouched << 32),
             dp_tot = (uint64_t)((int64_t)dping * 4294967296ll + dslen), rg_tot = ringops;
    block_sum4(fp_tot, ap_tot, dp_tot, rg_tot, sh);
    const uint32_t touched_tot = (uint32_t)(ap_tot >> 32);
    // the node's seen bitset, updated in LDS: the changed words back to its row
    // (16 bytes per thread where any of the four changed; only a touched change
    // can have set a bit, and a batch's makeAlive origins are mostly a few
    // rounds' contiguous id ranges, so a few dozen of the 1,024 words)
    if (touched_tot) {
        const uint32_t sw = S.seen_words;
        if ((sw & 3u) == 0) {
            const uint32_t w0 = 4 * threadIdx.x;
            if (w0 < sw && ((sh.seen_dirty[w0 >> 5] >> (w0 & 31)) & 0xFu))
                ((uint4*)srow)[threadIdx.x] = ((const uint4*)sh.seen)[threadIdx.x];
        } else {
            for (uint32_t w = threadIdx.x; w < sw; w += BLOCK)
                if ((sh.seen_dirty[w >> 5] >> (w & 31)) & 1u) srow[w] = sh.seen[w];
        }
    }
    ap_tot &= 0xFFFFFFFFull;
    const int32_t sl_tot = (int32_t)(uint32_t)dp_tot;
    dp_tot = (uint64_t)(((int64_t)dp_tot - sl_tot) >> 32);
    if (threadIdx.x == 0) {
        const uint32_t dt0 = sh.a_dt0;
        if (tail != dt0) { S.dlive[v] = sh.a_dl0 + (tail - dt0); S.dtail[v] = tail; }
        S.ttail[v] = ttail;
        if (ttail - sh.a_th0 > S.tcap) atomicOr(S.err, SIMERR_TIMERS_FULL);
        if (fp_tot) S.fp[v] = sh.a_fp0 + fp_tot;
        if (dp_tot) S.npingable[v] = sh.a_np0 + (int32_t)(int64_t)dp_tot;
        if (sl_tot) S.slen[v] += (int64_t)sl_tot;
        if (ap_tot) S.csum_valid[v] = 0;
        if (JOIN && ins) {
            S.mcount[v] = sh.a_m0 + ins;
            S.rng[v] += (uint64_t)ins * 0x9E3779B97F4A7C15ull;  // one getJoinPosition draw per new member
        }
        stat_add(S, STAT_EVALUATED, (unsigned long long)Llog * eval_weight);
        stat_add(S, STAT_APPLIED, (unsigned long long)ap_tot);
        if (touched_tot) stat_add(S, STAT_TOUCHED, (unsigned long long)touched_tot);
        if (phase == 2) {
            stat_add(S, STAT_EVAL_P2, (unsigned long long)Llog);
            stat_add(S, STAT_APPLIED_P2, (unsigned long long)ap_tot);
            if (touched_tot) stat_add(S, STAT_TOUCHED_P2, (unsigned long long)touched_tot);
        }
        if (phase == 3) { stat_add(S, STAT_EVAL_P3, (unsigned long long)Llog); stat_add(S, STAT_APPLIED_P3, (unsigned long long)ap_tot); }
        if (rg_tot) {  // 'ringChanged' (lib/ring.js:93) -> adjustMaxPiggybackCount
            const int32_t rc = S.ring_count[v] + (int32_t)(uint32_t)rg_tot - (int32_t)(rg_tot >> 32);
            S.ring_count[v] = rc;
            S.max_pb[v] = max_piggyback(rc);
            S.rbatch[v] = sh.u[9] + 1;
        }
    }
    __syncthreads();
    return (uint32_t)ap_tot;
}

// ---------------------------------------------------------------- prefix packing
// A key overwritten in place keeps its log position (lib/dissemination.js:
// 125-127: an object key keeps its insertion slot), so an entry re-recorded
// while still live pins the log head for another maxPiggybackCount issues,
// and the window an issue scans fills with tombstones behind it (config 4:
// ~12.6 k words per sender issue for ~4.7 k live keys).  After an issue,
// when the first groups of the window hold few live entries, those entries
// move -- in order -- to the end of that prefix, and the head jumps past the
// dead part: the relative order of all live keys is unchanged, so every
// later list is the reference's.  At most PREFIX_CAP entries move (one per
// thread, each a word, its side rows for a non-makeAlive entry and the
// address's view-cell log position), and only when the window shrinks by
// at least PREFIX_MIN.  glm[q]: the live entries of group q after this issue
// (its tombstones are written).
constexpr uint32_t PREFIX_CAP = BLOCK;
#ifndef RP_PREFIX_MIN
#define RP_PREFIX_MIN 512  // the default of rp_sim_config.prefix_min
#endif
__device__ void wg_pack_prefix(const SimDev& S, uint32_t v, Shared& sh, uint32_t head, uint32_t tail, uint32_t base,
                               uint32_t ngroups) {
    // head: the head after the issue (its first live entry; glm has no live
    // entry before it)
    const int lane = lane_id();
    const uint32_t n = S.n;
    // groups lying wholly inside [base, tail): the longest prefix with at
    // most PREFIX_CAP live entries, and each group's first live rank (gbase:
    // free once the issue's pass 2 is done)
    if (wave_id() == 0) {
        const uint32_t full = tail - base >= 64 ? min(ngroups, (tail - base) / 64) : 0u;
        uint32_t run = 0, g = 0;
        for (uint32_t c0 = 0; c0 < full; c0 += 64) {
            const uint32_t q = c0 + lane;
            const uint32_t x = q < full ? (uint32_t)__popcll(sh.glm[q]) : 0xFFFFu;
            uint32_t incl = x;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            const bool in = q < full && run + incl <= PREFIX_CAP;
            if (in) sh.gbase[q] = run + incl - x;
            const uint64_t ok = __ballot(in);
            const uint32_t c = (uint32_t)__popcll(ok);  // (a prefix of the lanes: counts are >= 0)
            if (c) run += __shfl(incl, (int)c - 1);
            g += c;
            if (c < 64) break;
        }
        if (lane == 0) { sh.u[0] = g; sh.u[1] = run; }
    }
    lds_barrier();
    const uint32_t G = sh.u[0], X = base + 64 * G, k = sh.u[1];
    // (uniform) worth it: k >= 1 live entries before X (else the issue's head
    // is already past X) and the window shrinks by at least PREFIX_MIN
    if (k == 0 || X - head > tail - head || X - head < k + S.prefix_min) return;
    uint32_t* const lrow = S.dko + S.row(v);
    uint64_t* const lvrow = S.dvs + S.row(v);
    uint32_t* const larow = S.dad + S.row(v);
    VEnt* const vrow = S.view + S.row(v);
    const uint32_t hs = head % n;
    auto slot = [&](uint32_t p) { const uint32_t sl = hs + (p - head); return sl >= n ? sl - n : sl; };
    // thread r < k: the r-th live entry, found from the masks (its group by
    // a binary search over the first ranks, its lane by halving the mask),
    // so all k words are read in one round trip
    const uint32_t r = threadIdx.x;
    uint32_t w = 0, pold = 0, a = NONE;
    uint64_t vs = 0;
    const uint32_t P = X - k + r;
    bool mv = false;
    if (r < k) {
        uint32_t lo = 0, hi = G;  // the last group whose first rank is <= r
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (sh.gbase[mid] <= r) lo = mid; else hi = mid;
        }
        uint64_t m = sh.glm[lo];
        uint32_t j = r - sh.gbase[lo], pos = 0;
#pragma unroll
        for (int h = 32; h > 0; h >>= 1) {
            const uint32_t c = (uint32_t)__popcll(m & ((1ull << h) - 1ull));
            if (j >= c) { j -= c; m >>= h; pos += h; }
        }
        pold = base + 64 * lo + pos;
        mv = pold != P;
    }
    __syncthreads();  // this issue's tombstones and stamp bumps (any wave) are visible
    if (mv) {
        w = lrow[slot(pold)];
        a = entry_addr(S, w, larow, slot(pold));
        if (!(w & LOG_ALIVE)) vs = lvrow[slot(pold)];
    }
    __syncthreads();  // every source read before any write
    if (mv) {
        const uint32_t i = slot(P);
        lrow[i] = w;
        if (!(w & LOG_ALIVE)) { lvrow[i] = vs; larow[i] = a; }
        vrow[a].dpos = P;
    }
    if (threadIdx.x == 0) { S.dhead[v] = X - k; stat_add(S, STAT_PREFIX_PACKS, 1); }
    __syncthreads();
}

// ---------------------------------------------------------------- issue
// The two smallest piggyback counts left in a log with distinct update
// sources, as (count << 32 | source) keys: k_need_checksums takes the second
// when the first's source is the pinging sender (whose issueAsReceiver
// filter could skip that entry).  Mergeable by inserting the other's pair.
__device__ inline void top2_insert(uint64_t& a1, uint64_t& a2, uint64_t x) {
    if ((uint32_t)x == (uint32_t)a1) { a1 = x < a1 ? x : a1; }
    else if (x < a1) { a2 = a1; a1 = x; }
    else { a2 = x < a2 ? x : a2; }
}

// Dissemination.issueAs (lib/dissemination.js:138-182) over node v's log, in
// key order; filter = issueAsReceiver's sender filter (:91-98).  Returns the
// length of the reference's change list.  Its entries are written to `out` in
// key order, except -- when `dest` names the node that will apply the list --
// those that are provably no-ops at dest (its seen bitset); *phys = entries written.
// ESC: also count the written entries without a makeAlive origin (*phys_esc;
// sharded runs only, where they become wire escapes)
//
// dfp: a fingerprint the destination's view had at some point before it
// applies the list (FP_NONE: unknown).  When it equals v's own, the two views
// were identical then; every log entry of v holds the change v last applied to
// that member (its view cell is that change or a later one, and a member's
// cell only moves up the rules' (incarnation, status) order except through
// the node's own local override), so at the destination every entry is a
// no-op except the one about the destination itself (lib/membership.js:
// 244-254 reasserts it).  Only that entry is written then; the list's
// length, counts and expiries are unchanged (the fingerprint is the one
// k_need_checksums and respond_as_receiver already take for view
// identity).
constexpr uint64_t FP_NONE = ~0ull;
// The decision as a word: keep << 32 | kpos, keep 0 = every entry, 1 = only
// the entry at kpos, 2 = none (SV_NONE: not precomputed).  Node v's issue
// to node d (d's fingerprint dfp); *hit: the views were identical.
constexpr uint64_t SV_NONE = ~0ull;
__device__ inline uint64_t same_view_word(const SimDev& S, uint32_t v, uint32_t d, uint64_t dfp, bool* hit) {
    *hit = false;
    if (dfp == FP_NONE) return 0;
    // one round of independent loads, then the slot's word and address
    const uint32_t n = S.n, dh = S.dhead[v], dt = S.dtail[v];
    const uint64_t fpv = S.fp[v];
    const uint32_t kp = S.view[S.row(v) + d].dpos;  // (may be stale: checked)
    if (fpv != dfp) return 0;
    *hit = true;
    bool ok = kp != NONE && kp - dh < dt - dh;
    if (ok) {
        const uint32_t sl = kp % n;
        const uint32_t w = S.dko[S.row(v) + sl], aa = S.dad[S.row(v) + sl];  // (the address row read alongside)
        ok = !is_tomb(w) && ((w & LOG_ALIVE) ? S.origins[origin_slot(S, log_origin(w))].source : aa) == d;
    }
    return ((uint64_t)(ok ? 1u : 2u) << 32) | kp;
}
// k_phase1's same-view decision for node v pinging T (wg_issue): taken where
// the target is chosen (k_iterate, k_shuffle), one thread per node, so that the chain of loads it needs (fingerprints, the
// target's view cell, the log slot it names) leaves the issue's prologue
__device__ inline void set_same_view(const SimDev& S, uint32_t v, uint32_t T) {
    bool hit;
    S.sv_word[v] = same_view_word(S, v, T, S.local(T) ? S.fp[T] : S.snd_fp[T], &hit);
    if (hit) stat_add(S, STAT_SAME_VIEW, 1ull);
}

// A load through the scalar cache (constant address space: s_load into SGPRs)
// of a value at a wave-uniform address that no block changes before this
// block reads it: a node's scalars read by its own block ahead of its own
// stores, a record written by an earlier kernel.
// (readfirstlane pins the value in an SGPR where it is loaded: without it the
// compiler sinks such loads past the caller's early returns and turns them
// into vector loads whose VGPRs it then keeps, or spills, across the issue)
__device__ inline uint32_t sload32(const uint32_t* p) {
    return __builtin_amdgcn_readfirstlane(*(const __attribute__((address_space(4))) uint32_t*)p);
}
// a wave-uniform 64-bit value pinned to SGPRs (readfirstlane is 32-bit and
// returns int: each half is zero-extended here)
__device__ inline uint64_t rfl64(uint64_t x) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
}
__device__ inline uint64_t sload64(const uint64_t* p) {
    return rfl64(*(const __attribute__((address_space(4))) uint64_t*)p);
}
// N words at p (16-byte aligned)
template <int N>
__device__ inline void sload_words(const void* p, uint32_t (&w)[N]) {
    // (word loads at consecutive uniform addresses: merged into s_load_dwordx4 / x8 / x16)
#pragma unroll
    for (int i = 0; i < N; i++) w[i] = __builtin_amdgcn_readfirstlane(*((const __attribute__((address_space(4))) uint32_t*)p + i));
}

// The seen bitset an issue to `dest` stages (DEST_REMOTE: the destination's
// shard mask), and the origin range it is valid for.
__device__ inline const uint32_t* seen_stage_src(const SimDev& S, uint32_t dest, const SeenWin& win, uint32_t& s_lo,
                                                 uint32_t& s_hi) {
    if (dest & DEST_REMOTE) {
        s_lo = S.gs_range[0]; s_hi = S.gs_range[1];
        return S.gseen + (size_t)((dest & ~DEST_REMOTE) >> S.gsz_log) * S.seen_words;
    }
    s_lo = win.olo; s_hi = win.ohi;
    return S.seen + S.srow(dest);
}
// SET: the settled-member filter at the destination (fault runs; the hot
// kernels of runs without faults are instantiated without it, at no cost).
// (Taking the node scalars and the arena room from a thread-per-node pre-pass
// instead, with the first log words loaded before the prologue's barrier,
// measured slower: DESIGN §6.8.)
// SPF (with SET): the settled-member checks of pass 1 prefetched per UNR / 2
// groups (k_phase1, k_p2_respond; the other callers' registers do not fit it).
// FAST (k_phase1, k_p2_respond): pass 1 on 64-aligned rows as lane masks
// (pass1_fast); in k_phase2 its extra code made the fused kernel
// spill more (+19 % there), so it keeps the general pass.
template <bool ESC = false, int UNR = RP_ISSUE_UNR, bool SET = true, bool SPF = false, bool FAST = false>
__device__ uint32_t wg_issue(const SimDev& S, uint32_t v, bool filter, uint32_t fsrc, uint64_t finc,
                             uint64_t* arena_off, int phase, Shared& sh, uint32_t dest, uint32_t* phys,
                             uint32_t* phys_esc, uint64_t dfp = FP_NONE, uint64_t sv = SV_NONE) {
    const uint64_t dg_e = diag_clock();
    const uint32_t n = S.n;
    uint32_t* const lrow = S.dko + S.row(v);  // the log row (uniform base, 32-bit slot offsets)
    const uint64_t* const lvrow = S.dvs + S.row(v);
    const uint32_t* const larow = S.dad + S.row(v);
    const SeenWin win = seen_window(S);
    // the destination's seen bitset (or its shard's mask) is staged in LDS:
    // one coalesced 4 KB read instead of a dependent global lookup per entry;
    // its loads, the node's scalars and the arena reservation are in flight
    // together before the prologue's LDS barrier
    // (a full barrier: the caller's writes to this node's log and view, by
    // any wave, are visible from here on)
    __syncthreads();
    const bool staged = dest != NONE;
    uint32_t s_lo = 0, s_hi = 0;
    const uint32_t* ssrc = staged ? seen_stage_src(S, dest, win, s_lo, s_hi) : nullptr;
    uint32_t a_res = 0;  // thread 0: the slice offset of the arena reservation
    const uint32_t a_shard = blockIdx.x % ARENA_SHARDS;
    // the issue's scalars (uniform): log head and tail, maxPiggybackCount,
    // issue count, live keys, the receiver filter, suspect/faulty origins
    // exist, and the same-view decision (0: every entry; 1: only the entry at
    // keep_pos; 2: none)
    uint32_t head, tail, maxpb, icount, dl0, keep, keep_pos;
    bool do_filter, any_settled;
    // groups start at `base`: the head rounded down to 64 entries (256 B,
    // two cache lines) when slots are 64-aligned with positions (n % 64 == 0),
    // so a group's words never straddle a third line; lanes before the head
    // read nothing
    uint32_t base = 0, base_slot = 0;
    auto slot_of = [&](uint32_t p) { uint32_t sl = base_slot + (p - base); return sl >= n ? sl - n : sl; };
    // (the wave index as a uniform value: group indices and their positions stay scalar)
    const int lane = lane_id(), wv = __builtin_amdgcn_readfirstlane(wave_id());
    {
        if (staged) stage_seen(sh.seen, ssrc, S.seen_words);
        if (threadIdx.x == 0) {
            // one round of independent loads (the same-view candidates with them)
            const uint32_t dh = S.dhead[v], dt = S.dtail[v];
            sh.u[0] = dh; sh.u[1] = dt; sh.u[6] = (uint32_t)S.max_pb[v]; sh.u[10] = S.icount[v];
            const uint32_t dlv = S.dlive[v];
            sh.i_dl0 = dlv;
            // ARENA_SHARDS cursors on lines of their own, each owning a slice
            // (< 2^32 changes, checked at setup; the cursor's low word); an issue
            // emits at most the live keys.  The returned offset is first needed
            // after pass 1 (the prologue's barrier does not wait for it), so its
            // latency hides behind the log scan.
            a_res = atomicAdd((uint32_t*)&S.arena_cursor[a_shard * 16], dlv);
            // the sender filter can only match origins created by makeSuspect /
            // makeFaulty (source at its current incarnation); without any, skip it
            const bool dang = *S.dangerous != 0;
            sh.u[9] = filter && fsrc != NONE && finc != 0 && dang;
            // (a member is settled only once a faulty update exists, and every
            // faulty update has a suspect/faulty origin)
            sh.i_settled = dang;
            // 0: every entry; 1: only the entry at i_keep_pos; 2: none (precomputed
            // when sv is given: k_iterate, for k_phase1)
            if (sv == SV_NONE && dest != NONE) {
                bool hit;
                sv = same_view_word(S, v, dest & ~DEST_REMOTE, dfp, &hit);
                if (hit) stat_add(S, STAT_SAME_VIEW, 1ull);
            }
            sh.i_keep = dest == NONE ? 0u : (uint32_t)(sv >> 32);
            sh.i_keep_pos = (uint32_t)sv;
        }
        const uint64_t dg_pb = diag_clock();
        // (the staged words and thread 0's scalars are in LDS; the arena
        // reservation may still be in flight)
        lds_barrier();
        if (RP_DIAG_FINE && phase == RP_DIAG_PHASE) { DIAG_ADD(S, 0, dg_pb - dg_e); DIAG_ADD(S, 1, diag_clock() - dg_pb); }
        (void)dg_pb;
        head = sh.u[0]; tail = sh.u[1]; maxpb = sh.u[6]; icount = sh.u[10]; dl0 = sh.i_dl0;
        do_filter = filter && sh.u[9] != 0;  // (issueAsSender: no filter loop compiled)
        any_settled = sh.i_settled != 0;
        keep = sh.i_keep; keep_pos = sh.i_keep_pos;
        base = ((n & 63u) == 0) ? (head & ~63u) : head;
        base_slot = base % n;
    }
    auto publish_off = [&] {
        if (threadIdx.x == 0) {
            const uint64_t a_part = S.arena_cap / ARENA_SHARDS;
            uint64_t o = a_res;
            if (o + dl0 > a_part) { atomicOr(S.err, SIMERR_ARENA_FULL); o = 0; }
            sh.aoff = a_shard * a_part + o;
        }
    };
    // (uniform) every entry may be written, or only the one at kpos (head - 1: none)
    const bool kall = keep == 0;
    const uint32_t kpos = keep == 1 ? keep_pos : head - 1u;
    auto noop_at_dest = [&](uint32_t oword) -> bool {
        if (dest == NONE) return false;
        (void)win;
        const uint32_t o = oword & ORIGIN_ID_MASK;
        if (!(oword & ORIGIN_ALIVE) || ((o - s_lo) & ORIGIN_ID_MASK) >= s_hi - s_lo) return false;
        return (sh.seen[(o & win.smask) >> 5] >> (o & 31)) & 1u;
    };
    // a local destination's settled faulty members (settled_bits): an entry
    // without a makeAlive origin whose key cannot exceed (INC0 + a, faulty)
    // is a no-op there.  (A bit read while the destination merges other
    // messages is safe either way: once its view held that key, every such
    // entry stays a no-op, keys never decrease.)
    // A destination on another shard: the AND over its group of the bits
    // gathered at the end of an earlier round (SimDev::gsettled).
    const uint32_t dnode = dest & ~DEST_REMOTE;
    const uint32_t* const fdest =
        (!SET || dest == NONE || !any_settled) ? nullptr
        : !(dest & DEST_REMOTE)       ? settled_bits(S, dest)
        : S.gsettled                  ? S.gsettled + (size_t)(dnode >> S.fs_log) * ((n + 31) / 32)
                                      : nullptr;
    auto settled_at_dest = [&](uint32_t w, uint32_t sl) -> bool {
        if (!fdest || (w & LOG_ALIVE)) return false;
        const uint32_t a = larow[sl];
        if (a == dnode) return false;
        const uint64_t vs = lvrow[sl];
        return v_status(vs) != ST_LEAVE && v_inc(vs) <= INC0 + a && ((fdest[a >> 5] >> (a & 31)) & 1u);
    };
    // Two passes per segment of up to ISSUE_SEG 64-entry groups, group q
    // handled by wave q % NWAVE (no workgroup barrier inside a pass):
    //  1. stream the key|origin words (UNR groups in flight per wave): counts,
    //     expiries (tombstones), filtered stamp bumps, and a ballot mask per
    //     group of the entries to write out;
    //  2. after one barrier, per 64 groups a wave scan of the written counts
    //     gives every group's output base; gather the written entries (a few
    //     per group) and store them at their ranks.
    // Interleaving matters: the entries written out are mostly the freshest,
    // at the log's tail, so every wave gets its share of pass 2.
    uint32_t first_live = NONE, min_left = NONE, deleted = 0, emitted = 0, escapes = 0, wbase = 0;
    // phase 1: the smallest count among entries no receiver filter can skip
    // (makeAlive and fullSync origins), and the top-2 by distinct source of
    // the others (local suspect/faulty origins), for k_need_checksums
    uint32_t min_safe = NONE;
    uint64_t top1 = ~0ull, top2 = ~0ull;
    const uint64_t below = (1ull << lane) - 1ull;
    const uint32_t ngroups = (tail - base + 63) / 64;
    uint64_t dg_p1 = 0, dg_x = 0, dg_p2 = 0, dg_pro = diag_clock() - dg_e;
    for (uint32_t s0 = 0; s0 < ngroups; s0 += ISSUE_SEG) {
        const uint32_t sg = min(ISSUE_SEG, ngroups - s0);
        uint64_t dg_t = diag_clock();
        uint32_t st_n = 0, st_full = NONE;  // this wave's stash fill; its first group not stashed
        // pass 1 as two loops: with the receiver filter, and without (the
        // common case, straight-line: the issue is bound by instructions per
        // scanned word)
        auto pass1 = [&](auto filt) {
        constexpr bool FILTER = decltype(filt)::value;
        for (uint32_t q0 = wv; q0 < sg; q0 += NWAVE * UNR) {
            // every lane loads (a lane outside the window loads the head's
            // word, dropped below): no branch between the UNR loads, so all
            // are in flight before the first use
            uint32_t ko[UNR];
            bool inw[UNR];
#pragma unroll
            for (int u = 0; u < UNR; u++) {
                const uint32_t q = q0 + u * NWAVE, p = base + (s0 + q) * 64 + lane;
                inw[u] = q < sg && p - head < tail - head;
                ko[u] = lrow[slot_of(inw[u] ? p : head)];
            }
#pragma unroll
            for (int u = 0; u < UNR; u++) ko[u] = inw[u] ? ko[u] : TOMB_WORD;
            // settled_at_dest for the UNR groups at once (bit u of stl), its
            // dependent loads -- address, the destination's settled word, the
            // value -- in flight for all groups together rather than one
            // group after another
            // (in halves of UNR / 2 groups: the registers of all UNR at once spill)
            uint32_t stl = 0;
            if constexpr (SPF) {
                if (fdest) {  // (wave-uniform)
                    constexpr int H = UNR / 2;
#pragma unroll
                    for (int h = 0; h < UNR; h += H) {
                        uint32_t sa[H], sb[H];
#pragma unroll
                        for (int u = 0; u < H; u++) {
                            const uint32_t p = base + (s0 + q0 + (h + u) * NWAVE) * 64 + lane;
                            sa[u] = (!(ko[h + u] & LOG_ALIVE) && !is_tomb(ko[h + u])) ? larow[slot_of(p)] : dnode;
                        }
#pragma unroll
                        for (int u = 0; u < H; u++) sb[u] = sa[u] != dnode ? fdest[sa[u] >> 5] : 0u;
                        uint32_t cm = 0;
#pragma unroll
                        for (int u = 0; u < H; u++) cm |= ((sb[u] >> (sa[u] & 31)) & 1u) << u;
                        if (cm) {  // (per lane)
                            uint64_t sv[H];
#pragma unroll
                            for (int u = 0; u < H; u++) {
                                const uint32_t p = base + (s0 + q0 + (h + u) * NWAVE) * 64 + lane;
                                sv[u] = ((cm >> u) & 1u) ? lvrow[slot_of(p)] : 0ull;
                            }
#pragma unroll
                            for (int u = 0; u < H; u++)
                                if (((cm >> u) & 1u) && v_status(sv[u]) != ST_LEAVE && v_inc(sv[u]) <= INC0 + sa[u])
                                    stl |= 1u << (h + u);
                        }
                    }
                }
            }
            auto settled_u = [&](int u, uint32_t w, uint32_t sl) -> bool {
                if constexpr (SPF) { (void)w; (void)sl; return (stl >> u) & 1u; }
                else return settled_at_dest(w, sl);
            };
#pragma unroll
            for (int u = 0; u < UNR; u++) {
                const uint32_t q = q0 + u * NWAVE, p = base + (s0 + q) * 64 + lane;
                if (q >= sg) break;  // wave-uniform
                const uint32_t w = ko[u], org = log_origin(w);
                bool wr = false, alive = false;
                bool f_ex = false, f_em = false, f_esc = false;  // (issueAsSender: counted by ballots below)
                if constexpr (!FILTER) {
                    // no receiver filter can match
                    const bool nt = !is_tomb(w);
                    const uint32_t c2 = entry_count(w, icount) + 1u;  // an undefined count counts as 0 (:149-151)
                    const bool ex = nt && c2 > maxpb;                  // lib/dissemination.js:162-165
                    alive = nt && !ex;
                    // (the address's cell keeps its stale log position: wg_apply checks it)
                    if (ex) lrow[slot_of(p)] = TOMB_WORD;
                    const uint32_t o = w & ORIGIN_ID_MASK;
                    const uint32_t sw = sh.seen[(o & win.smask) >> 5];
                    const bool seen = staged && (w & LOG_ALIVE) && ((o - s_lo) & ORIGIN_ID_MASK) < s_hi - s_lo &&
                                      ((sw >> (o & 31)) & 1u);
                    wr = alive && !seen && (kall || p == kpos) && !settled_u(u, w, slot_of(p));
                    f_ex = ex;
                    f_em = alive;
                    f_esc = ESC && wr && !(w & LOG_ALIVE);  // an escape on the wire
                    min_left = min(min_left, alive ? c2 : NONE);
                    if (phase == 1) {
                        const bool safe = (w & LOG_ALIVE) || o < S.lorigin_base;
                        min_safe = min(min_safe, alive && safe ? c2 : NONE);
                        if (__ballot(alive && !safe) && alive && !safe)
                            top2_insert(top1, top2, ((uint64_t)c2 << 32) | S.origins[o].source);
                    }
                } else if (!is_tomb(w)) {
                    uint32_t c2 = entry_count(w, icount);  // an undefined count counts as 0 (:149-151)
                    bool live = true;
                    const Origin o = S.origins[origin_slot(S, org)];
                    const bool filtered = o.source != NONE && o.source_inc != 0 && o.source == fsrc && o.source_inc == finc;
                    if (filtered) {  // count stays: bump the stamp along with the issue counter
                        lrow[slot_of(p)] = (w & LOG_ORIGIN_MASK) | (((((w >> 24) + 1) & STAMP_MASK) | STAMP_DEFINED) << 24);
                    } else {
                        c2 += 1;
                        if (c2 > maxpb) {  // lib/dissemination.js:162-165
                            f_ex = true;
                            live = false;
                            // (the address's cell keeps its stale log position: wg_apply checks it)
                            lrow[slot_of(p)] = TOMB_WORD;
                        } else {
                            f_em = true;
                            wr = !noop_at_dest(org) && (kall || p == kpos) && !settled_u(u, w, slot_of(p));
                            f_esc = ESC && wr && !(org & ORIGIN_ALIVE);  // an escape on the wire
                        }
                    }
                    alive = live;
                    if (live) {
                        min_left = min(min_left, c2);
                        if (phase == 1) {
                            const uint32_t oid = org & ORIGIN_ID_MASK;
                            if ((org & ORIGIN_ALIVE) || oid < S.lorigin_base) min_safe = min(min_safe, c2);
                            else top2_insert(top1, top2, ((uint64_t)c2 << 32) | S.origins[oid].source);
                        }
                    }
                }
                if (phase == 1) {  // (wave-uniform counts: no per-lane adds, no shuffles at the end)
                    deleted += (uint32_t)__popcll(__ballot(f_ex));
                    emitted += (uint32_t)__popcll(__ballot(f_em));
                    if (ESC) escapes += (uint32_t)__popcll(__ballot(f_esc));
                } else {
                    deleted += f_ex;
                    emitted += f_em;
                    if (ESC) escapes += f_esc;
                }
                const uint64_t m = __ballot(wr);
                if (lane == 0) sh.imask[q] = m;
                {
                    // live entries (this issue's expiries excluded): the
                    // wave's first one (its groups come in increasing order)
                    // and, in the first segment, the group's count
                    const uint64_t lm = __ballot(alive);
                    if (lm && first_live == NONE) first_live = base + (s0 + q) * 64 + (uint32_t)__builtin_ctzll(lm);
                    if (s0 == 0 && lane == 0) sh.glm[q] = lm;
                }
                if (m) {  // (wave-uniform) stash the group's written entries while they fit
                    const uint32_t c = (uint32_t)__popcll(m);
                    if (st_full == NONE && st_n + c <= ISSUE_STASH) {
                        if (wr) {
                            const uint32_t e = st_n + (uint32_t)__popcll(m & below);
                            sh.st_kv[wv][e] = ko[u];
                            sh.st_m[wv][e] = (uint16_t)((q << 6) | (uint32_t)lane);
                        }
                        st_n += c;
                    } else if (st_full == NONE) {
                        st_full = q;  // this and later groups of the wave: gathered from the log in pass 2
                    }
                }
            }
        }
        };
        // Pass 1 without the receiver filter on 64-aligned rows (n % 64 == 0,
        // groups start at head & ~63): a group's 64 slots are contiguous, so
        // its address is a uniform row pointer plus the lane's offset, and the
        // entries' tests become lane masks combined on the scalar unit.  The
        // same decisions as pass1(false_type) (instructions per scanned word:
        // DESIGN §6.9).
        // KALL: every entry may be written (the same-view decision keeps one
        // or none only when the destination's view equals the sender's: rare)
        auto pass1_fast = [&](auto kall_t) {
            constexpr bool KALL = decltype(kall_t)::value;
            const uint32_t lane4 = (uint32_t)lane << 2;
            const uint32_t hlo = head - base, span = tail - base;  // the window, relative to base
            const uint32_t sspan = s_hi - s_lo;
            const uint32_t smhi = win.smask & ~31u;  // the staged seen word's byte offset: (w & smhi) >> 3
            const uint32_t rowb = n * 4u;            // the log row's bytes
            uint32_t ud = 0, ue = 0, uesc = 0;       // expired, emitted, escapes (wave sums)
            uint32_t ml1 = NONE, ms1 = NONE;         // the smallest count c1 = c2 - 1 (left, safe)
            // the log row as a buffer resource: a group's word is one buffer
            // load at the lane's offset plus the group's (scalar) byte offset
            // (past the row -- a group beyond the segment -- reads 0, dropped)
            const __amdgpu_buffer_rsrc_t rrow = __builtin_amdgcn_make_buffer_rsrc(lrow, (short)0, (int)rowb, 0x00020000);
            const uint32_t tomb = TOMB_WORD, none = NONE, one = 1u, zero = 0u;
            // v_cndmask with a lane mask held in SGPRs (ballots combined on the
            // scalar unit; as per-lane booleans the compiler would re-derive
            // them with vector compares); volatile: inside a branch taken by few
            // groups, not hoisted out of it
            auto sel = [](uint64_t mask, uint32_t t, uint32_t f) {
                const uint64_t ms = rfl64(mask);
                uint32_t r;
                asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(ms));
                return r;
            };
            auto bit = [&](uint64_t mask) { return sel(mask, one, zero) != 0u; };
            // (the same on every group's path: a mask the scalar unit made)
            auto sel_s = [](uint64_t mask, uint32_t t, uint32_t f) {
                uint32_t r;
                asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(mask));
                return r;
            };
            // the byte offset of group s0 + wv's first slot (one wrap at most);
            // a wave's groups are NWAVE apart: 1 KB of slots
            uint32_t off0 = (base_slot + (s0 + (uint32_t)wv) * 64u) << 2;
            if (off0 >= rowb) off0 -= rowb;
            // the groups the window does not cut: g_lo <= g < g_lo + g_n (the
            // head lies in group 0, hlo < 64), tested as one unsigned compare
            const uint32_t g_lo = hlo ? 1u : 0u, g_hi = span >> 6;
            const uint32_t g_n = g_hi > g_lo ? g_hi - g_lo : 0u;
            // the stash takes groups while they fit; from the first that does
            // not (st_full), none: lim drops to 0
            uint32_t lim = st_full == NONE ? ISSUE_STASH : 0u;
            for (uint32_t q0 = wv; q0 < sg; q0 += NWAVE * UNR) {
                uint32_t ko[UNR];
#pragma unroll
                for (int u = 0; u < UNR; u++) {
                    uint32_t o = off0 + (uint32_t)u * (NWAVE * 256u);
                    if (o >= rowb) o -= rowb;
                    ko[u] = __builtin_amdgcn_raw_buffer_load_b32(rrow, lane4, o, 0);
                }
#pragma unroll
                for (int u = 0; u < UNR; u++) {
                    const uint32_t q = q0 + u * NWAVE;
                    if (q >= sg) break;  // wave-uniform
                    const uint32_t g = s0 + q, gp = g * 64u;
                    uint32_t w = ko[u];
                    if (__builtin_expect(g - g_lo >= g_n, 0)) {  // (gp < hlo || gp + 64 > span)
                        // the window's lanes of a group it cuts (its first or its last)
                        const uint32_t lo = gp < hlo ? hlo - gp : 0u, hi = min(span - gp, 64u);
                        w = sel((hi >= 64u ? ~0ull : ((1ull << hi) - 1ull)) & ~((1ull << lo) - 1ull), w, tomb);
                    }
                    const uint32_t c1 = (icount - (w >> 24)) & STAMP_MASK;  // an undefined count counts as 0
                    const uint64_t mnt = __ballot((w & LOG_ORIGIN_MASK) != ORIGIN_ID_MASK);
                    const uint64_t mge = __ballot(c1 >= maxpb);               // c1 + 1 > maxpb: lib/dissemination.js:162-165
                    const uint64_t mex = mnt & mge, lm = mnt & ~mge;          // expire now / stay live
                    if (mex && bit(mex)) {  // (the cell keeps its stale log position: wg_apply checks it)
                        uint32_t o = off0 + (uint32_t)u * (NWAVE * 256u);
                        if (o >= rowb) o -= rowb;
                        __builtin_amdgcn_raw_buffer_store_b32(TOMB_WORD, rrow, lane4, o, 0);
                    }
                    const uint64_t mla = __ballot((w & LOG_ALIVE) != 0);
                    const uint32_t sw = *(const uint32_t*)((const char*)sh.seen + ((w & smhi) >> 3));
                    uint64_t m = lm & ~(mla & __ballot(((w - s_lo) & ORIGIN_ID_MASK) < sspan) &
                                        __ballot(__builtin_amdgcn_ubfe(sw, w, 1u) != 0));
                    if constexpr (!KALL) {  // only the entry at kpos may be written
                        const uint32_t kl = kpos - (base + gp);
                        m &= kl < 64u ? (1ull << kl) : 0ull;
                    }
                    ud += (uint32_t)__popcll(mex);
                    ue += (uint32_t)__popcll(lm);
                    if (ESC) uesc += (uint32_t)__popcll(m & ~mla);
                    ml1 = min(ml1, sel_s(lm, c1, none));
                    if (phase == 1) {
                        const uint64_t mu = lm & ~(mla | __ballot((w & ORIGIN_ID_MASK) < S.lorigin_base));
                        ms1 = min(ms1, sel_s(lm & ~mu, c1, none));
                        if (mu && bit(mu))  // (fault runs: unsafe live entries)
                            top2_insert(top1, top2, ((uint64_t)(c1 + 1u) << 32) | S.origins[w & ORIGIN_ID_MASK].source);
                    }
                    if (lane == 0) {
                        sh.imask[q] = m;
                        if (s0 == 0) sh.glm[q] = lm;
                    }
                    if (__builtin_expect(first_live == NONE, 0) && lm)
                        first_live = base + gp + (uint32_t)__builtin_ctzll(lm);
                    if (m) {  // (wave-uniform) stash the group's written entries while they fit
                        const uint32_t c = (uint32_t)__popcll(m), e0 = st_n;
                        if (st_n + c <= lim) {
                            st_n += c;
                            if (bit(m)) {
                                const uint32_t e = e0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                                sh.st_kv[wv][e] = w;
                                sh.st_m[wv][e] = (uint16_t)((q << 6) | (uint32_t)lane);
                            }
                        } else if (lim) {
                            st_full = q;  // this and later groups of the wave: gathered from the log in pass 2
                            lim = 0;
                        }
                    }
                }
                off0 += NWAVE * UNR * 256u;
                if (off0 >= rowb) off0 -= rowb;
            }
            // into the general path's accumulators: per lane c2 = c1 + 1;
            // phase 1 keeps wave-uniform counts, the others per-lane sums (lane 0)
            min_left = min(min_left, ml1 == NONE ? NONE : ml1 + 1u);
            if (phase == 1) {
                min_safe = min(min_safe, ms1 == NONE ? NONE : ms1 + 1u);
                deleted += ud; emitted += ue; escapes += uesc;
            } else if (lane == 0) {
                deleted += ud; emitted += ue; escapes += uesc;
            }
        };
        if (do_filter) pass1(std::true_type{});
        else if (FAST && !SET && staged && (n & 63u) == 0) {
            if (kall) pass1_fast(std::true_type{});
            else pass1_fast(std::false_type{});
        } else pass1(std::false_type{});
        {
            const uint64_t t = diag_clock();
            dg_p1 += t - dg_t;
            dg_t = t;
        }
        publish_off();
        lds_barrier();
        Change* const out = S.arena + sh.aoff;
        {
            const uint64_t t = diag_clock();
            dg_x += t - dg_t;
            dg_t = t;
        }
        uint32_t run = wbase;
        for (uint32_t c0 = 0; c0 < sg; c0 += 64) {
            // output bases of groups c0 .. c0 + 63 (lane l: group c0 + l)
            const uint64_t mq = c0 + lane < sg ? sh.imask[c0 + lane] : 0ull;
            const uint32_t x = (uint32_t)__popcll(mq);
            uint32_t incl = x;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            const uint32_t excl = run + incl - x;
            run += __shfl(incl, 63);
            const uint32_t lim = min(64u, sg - c0);
            if (c0 + lane < sg && ((c0 + lane) % NWAVE) == (uint32_t)wv) sh.gbase[c0 + lane] = excl;
            if (st_full == NONE || c0 + lim <= st_full) continue;  // all of this wave's groups here are stashed
            constexpr int U2 = RP_ISSUE_P2U;
            for (uint32_t l0 = wv; l0 < lim; l0 += NWAVE * U2) {  // this wave's groups of the chunk
                uint64_t mk[U2];
                uint32_t sl[U2], bs[U2], kv[U2];
#pragma unroll
                for (int u = 0; u < U2; u++) {
                    const uint32_t l = l0 + u * NWAVE;
                    const uint32_t ls = l < lim ? l : 0u;
                    mk[u] = (l < lim && c0 + l >= st_full) ? __shfl(mq, (int)ls) : 0ull;
                    bs[u] = __shfl(excl, (int)ls);
                    sl[u] = slot_of(base + (s0 + c0 + ls) * 64 + lane);
                    kv[u] = ((mk[u] >> lane) & 1ull) ? lrow[sl[u]] : 0u;
                }
#pragma unroll
                for (int u = 0; u < U2; u++) {
                    if ((mk[u] >> lane) & 1ull) {
                        const uint32_t pos = bs[u] + (uint32_t)__popcll(mk[u] & below);
                        if (pos < dl0) store_msg(out + pos, log_change(S, kv[u], lvrow, larow, sl[u]));
                        else atomicOr(S.err, SIMERR_ARENA_FULL);  // (cannot happen: written <= live keys)
                    }
                }
            }
        }
        // the stashed entries: output index = group base + rank in the group
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (this wave's gbase writes)
        for (uint32_t e0 = 0; e0 < st_n; e0 += 64) {
            const uint32_t e = e0 + lane;
            if (e < st_n) {
                const uint32_t kv = sh.st_kv[wv][e];
                const uint32_t mt = sh.st_m[wv][e], q = mt >> 6, ln = mt & 63u;
                const uint32_t pos = sh.gbase[q] + (uint32_t)__popcll(sh.imask[q] & ((1ull << ln) - 1ull));
                if (pos < dl0) store_msg(out + pos, log_change(S, kv, lvrow, larow, slot_of(base + (s0 + q) * 64 + ln)));
                else atomicOr(S.err, SIMERR_ARENA_FULL);  // (the reservation is the live keys: never past it)
            }
        }
        wbase = run;
        dg_p2 += diag_clock() - dg_t;
        if (s0 + ISSUE_SEG < ngroups) lds_barrier();  // the next segment reuses imask
    }
    if (!RP_DIAG_FINE && phase == RP_DIAG_PHASE) { DIAG_ADD(S, 0, dg_p1); DIAG_ADD(S, 1, dg_x + dg_p2); DIAG_ADD(S, 2, dg_pro); }
    if (RP_DIAG_FINE && phase == RP_DIAG_PHASE) DIAG_ADD(S, 5, dg_p1 + dg_x + dg_p2);
    (void)dg_p1; (void)dg_x; (void)dg_p2; (void)dg_pro;
    const uint32_t written = wbase;
    const uint64_t dg_ep = diag_clock();
    publish_off();  // (an empty log has no segment)
    // deleted, emitted and escapes are each < 2^21 (a log spans < 2n + 1024 entries)
    // the block's reductions in one LDS exchange (one barrier): first live
    // position, smallest count left, the three counts packed, and in phase 1
    // the smallest safe count and the top-2 keys
    uint64_t fl64 = first_live, ml64 = min_left,
             cnt = deleted | ((uint64_t)emitted << 21) | ((uint64_t)escapes << 42);
    uint32_t ms32 = min_safe;
    if (phase == 1) {
        // first_live and the counts are the same in every lane of a wave
        // (ballot-derived); min_left / min_safe are per lane, 32-bit; the
        // top-2 keys only when some lane holds one (unsafe entries: fault runs)
        uint32_t ml32 = min_left;
        const bool tops = phase == 1 && __ballot(top1 != ~0ull) != 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            ml32 = min(ml32, (uint32_t)__shfl_xor(ml32, o));
            if (phase == 1) ms32 = min(ms32, (uint32_t)__shfl_xor(ms32, o));
            if (tops) {
                const uint64_t b1 = __shfl_xor(top1, o), b2 = __shfl_xor(top2, o);
                top2_insert(top1, top2, b1);
                top2_insert(top1, top2, b2);
            }
        }
        ml64 = ml32;
    } else {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            fl64 = min(fl64, (uint64_t)__shfl_xor(fl64, o));
            ml64 = min(ml64, (uint64_t)__shfl_xor(ml64, o));
            cnt += __shfl_xor(cnt, o);
            if (phase == 1) {
                ms32 = min(ms32, (uint32_t)__shfl_xor(ms32, o));
                const uint64_t b1 = __shfl_xor(top1, o), b2 = __shfl_xor(top2, o);
                top2_insert(top1, top2, b1);
                top2_insert(top1, top2, b2);
            }
        }
    }
    if (lane == 0) {
        sh.red[0][wv] = fl64; sh.red[1][wv] = ml64; sh.red[2][wv] = cnt;
        if (phase == 1) { sh.ims[wv] = ms32; sh.itop[0][wv] = top1; sh.itop[1][wv] = top2; }
    }
    lds_barrier();
    fl64 = sh.red[0][0]; ml64 = sh.red[1][0]; cnt = sh.red[2][0];
#pragma unroll
    for (int i = 1; i < NWAVE; i++) { fl64 = min(fl64, sh.red[0][i]); ml64 = min(ml64, sh.red[1][i]); cnt += sh.red[2][i]; }
    if (phase == 1 && threadIdx.x == 0) {  // (thread 0 stores them)
        ms32 = sh.ims[0];
        top1 = top2 = ~0ull;
#pragma unroll
        for (int i = 0; i < NWAVE; i++) {
            if (i) ms32 = min(ms32, sh.ims[i]);
            top2_insert(top1, top2, sh.itop[0][i]);
            top2_insert(top1, top2, sh.itop[1][i]);
        }
        min_safe = ms32;
    }
    const uint64_t dg_r = diag_clock();
    if (RP_DIAG_FINE && phase == RP_DIAG_PHASE) DIAG_ADD(S, 2, dg_r - dg_ep);
    (void)dg_r;
    if (ESC) escapes = (uint32_t)(cnt >> 42);
    const uint32_t ndel = (uint32_t)(cnt & 0x1FFFFFu);
    emitted = (uint32_t)((cnt >> 21) & 0x1FFFFFu);
    const uint32_t fl = (uint32_t)fl64, ml = (uint32_t)ml64;
    if (threadIdx.x == 0) {
        S.icount[v] = icount + 1;
        const uint32_t nh = fl == NONE ? tail : fl, nl = dl0 - (uint32_t)ndel;
        if (nh != head) S.dhead[v] = nh;
        if (ndel) S.dlive[v] = nl;
        sh.i_compact = (tail - nh) > S.compact_mul * nl + S.compact_add;  // mostly tombstones: compact
        if (phase == 1) { S.min_cnt[v] = ml; S.min_safe[v] = min_safe; S.min_l1[v] = top1; S.min_l2[v] = top2; }
        stat_add(S, phase == 1 ? STAT_SCANNED_P1 : STAT_SCANNED_P2, (unsigned long long)(tail - head));
        stat_add(S, phase == 1 ? STAT_EMITTED_P1 : STAT_EMITTED_P2, (unsigned long long)emitted);
        stat_add(S, phase == 1 ? STAT_WRITTEN_P1 : STAT_WRITTEN_P2, (unsigned long long)written);
        if (sh.i_compact) stat_add(S, STAT_COMPACT_ISSUE, 1);
    }
    // (the prefix packing's barrier publishes sh.i_compact and keeps sh.red from
    // being reused before every wave has read it)
    const uint64_t dg_s = diag_clock();
    if (RP_DIAG_FINE && phase == RP_DIAG_PHASE) DIAG_ADD(S, 3, dg_s - dg_r);
    (void)dg_s;
    *arena_off = sh.aoff;
    wg_pack_prefix(S, v, sh, fl == NONE ? tail : fl, tail, base, min(ISSUE_SEG, ngroups));
    if (phase == RP_DIAG_PHASE) DIAG_ADD(S, 4, diag_clock() - (RP_DIAG_FINE ? dg_s : dg_ep));
    (void)dg_ep;
    if (sh.i_compact) {
        __syncthreads();  // pass 1's tombstones (any wave) are visible to the compaction
        wg_compact(S, v, sh);
    }
    *phys = written;
    *phys_esc = escapes;
    return emitted;
}

// ---------------------------------------------------------------- init
__global__ void k_init_rows(SimDev S) {
    const uint64_t total = (uint64_t)S.nl * S.n;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t a = (uint32_t)(i % S.n);
        VEnt c;
        c.vs = pack_view(INC0 + a, ST_ALIVE);  // makeAlive(self) + set(): every member alive
        c.dpos = NONE;
        c.tstamp = 0;
        S.view[i] = c;
        S.in_ring[i] = 1;
    }
}

// bootstrap per node (index.js:233-267 with a full-membership join result,
// then lib/swim/gossip.js:85 shuffle): members = [self, others in id order],
// one Math.random for getJoinPosition on the empty list, then _.shuffle
// (done by k_shuffle).
__global__ void k_init_order(SimDev S) {
    const uint32_t v = S.lo + blockIdx.x, n = S.n;
    uint32_t* ord = S.order + S.row(v);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) ord[i] = i == 0 ? v : (i <= v ? i - 1 : i);
}
// per-node scalars of every node (remote entries are overwritten by exchanges)
__global__ void k_init_scalars(SimDev S, uint64_t seed, uint8_t* need_shuffle) {
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x, n = S.n;
    if (v >= n) return;
    {
        uint64_t s = node_rng_seed(seed, v);
        (void)js_math_random(s);  // getJoinPosition() for the local member (lib/membership.js:99-101)
        S.rng[v] = s;
        S.iter_index[v] = -1;
        S.iter_round[v] = 0;
        S.dhead[v] = 0;
        S.dtail[v] = 0;
        S.dlive[v] = 0;
        S.icount[v] = 0;
        S.max_pb[v] = max_piggyback(1);  // ringChanged after the local member joined the ring
        S.ring_count[v] = (int32_t)n;
        S.csum_valid[v] = 0;
        S.npingable[v] = (int32_t)n - 1;
        S.mcount[v] = n;
        S.dead[v] = 0;
        S.self_inc[v] = INC0 + v;
        need_shuffle[v] = S.local(v) ? 1 : 0;
    }
}

// Membership.shuffle -> _.shuffle (underscore 1.13): for i in [0, L):
// swap(a[i], a[random(i, L-1)]).  The draws of a counter-based splitmix
// stream are independent, so a block computes 256 swap targets at a time in
// parallel and one lane applies them to the row held in LDS (16-bit ids).
// With find_target, the iterator then continues at index 0 of the new order
// (lib/membership-iterator.js:37-47).
// list != nullptr: the nodes to shuffle are list[0 .. *count) (k_iterate's
// wrapped iterators); else every local node with need_shuffle set.
__global__ void __launch_bounds__(BLOCK) k_shuffle(SimDev S, uint8_t* need_shuffle, int find_target,
                                                   const uint32_t* list, const uint32_t* count) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    __shared__ Shared sh;
    __shared__ uint32_t tgt[BLOCK];
    uint16_t* a = (uint16_t*)dyn;
    // grid-stride over the candidates: only the few whose iterator wrapped do any work
    const uint32_t nc = list ? *count : S.nl;
    for (uint32_t c = blockIdx.x; c < nc; c += gridDim.x) {
        const uint32_t v = list ? list[c] : S.lo + c;
        if (!need_shuffle[v]) continue;
        uint32_t* ord = S.order + S.row(v);
        const uint32_t M = S.mcount[v];  // the members (a view need not hold all n)
        for (uint32_t i = threadIdx.x; i < M; i += BLOCK) a[i] = (uint16_t)ord[i];
        const uint64_t s0 = S.rng[v];
        for (uint32_t c0 = 0; c0 < M; c0 += BLOCK) {
            uint32_t i = c0 + threadIdx.x;
            if (i < M) {
                uint64_t s = s0 + (uint64_t)i * 0x9E3779B97F4A7C15ULL;
                tgt[threadIdx.x] = (uint32_t)js_random_int(s, (int)i, (int)M - 1);
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                uint32_t m = min((uint32_t)BLOCK, M - c0);
                for (uint32_t j = 0; j < m; j++) {
                    uint32_t x = c0 + j, r = tgt[j];
                    uint16_t t = a[x]; a[x] = a[r]; a[r] = t;
                }
            }
            __syncthreads();
        }
        for (uint32_t i = threadIdx.x; i < M; i += BLOCK) ord[i] = a[i];
        uint32_t first = NONE;
        if (find_target) {
            const VEnt* row = S.view + S.row(v);
            for (uint32_t i = threadIdx.x; i < M; i += BLOCK) {
                uint32_t m = a[i];
                if (m != v && is_pingable_status(v_status(row[m].vs))) { first = i; break; }
            }
        }
        first = block_min32(first, sh.sc);  // also orders the LDS row reuse
        if (threadIdx.x == 0) {
            S.rng[v] = s0 + (uint64_t)M * 0x9E3779B97F4A7C15ULL;
            need_shuffle[v] = 0;
            if (find_target) {
                S.iter_index[v] = (int32_t)first;
                S.target[v] = first == NONE ? -1 : (int32_t)a[first];
                if (first != NONE) set_same_view(S, v, a[first]);
            }
        }
    }
}

__global__ void k_init_owner(SimDev S, const int32_t* coll_min) {
    const uint64_t total = (uint64_t)S.nl * S.ncoll;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x)
        S.coll_owner[i] = coll_min[i % S.ncoll];
}
__global__ void k_init_owner_self(SimDev S) {
    // the local member is added to its own ring before set() adds the others
    uint32_t v = S.lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= S.lo + S.nl) return;
    for (int r = 0; r < REPLICAS; r++) {
        int32_t cid = S.coll_of[(size_t)v * REPLICAS + r];
        if (cid >= 0) S.coll_owner[S.crow(v) + cid] = (int32_t)v;
    }
}

// fingerprint and checksum-string length of views v0 + block (or ids[block])
__global__ void __launch_bounds__(BLOCK) k_init_fp(SimDev S, uint32_t v0, const uint32_t* ids) {
    __shared__ Shared sh;
    uint32_t v = ids ? ids[blockIdx.x] : v0 + blockIdx.x;
    if (!S.local(v)) return;
    const size_t base = S.row(v);
    const AddrTable at{S.addr_words, S.addr_len};
    uint64_t acc = 0, len = 0, cnt = 0;
    uint32_t* const pb = ping_bits(S, v);
    uint32_t* const fb = settled_bits(S, v);
    for (uint32_t a0 = 0; a0 < S.n; a0 += BLOCK) {
        const uint32_t a = a0 + threadIdx.x;
        bool pg = false, fs = false;
        if (a < S.n) {
            const uint64_t vs = S.view[base + a].vs;
            acc += entry_mix(a, vs);
            if (v_status(vs) != ST_ABSENT) { len += member_len(at, a, vs); cnt++; }
            pg = is_pingable_status(v_status(vs));
            fs = settles(v, a, vs);
        }
        const uint64_t m = __ballot(pg);  // (the pingable and settled bits, rebuilt: 64 addresses per wave)
        const uint64_t mf = __ballot(fs);
        if ((lane_id() & 31) == 0 && a < S.n) {
            pb[a >> 5] = (uint32_t)(m >> (lane_id() & 32));
            fb[a >> 5] = (uint32_t)(mf >> (lane_id() & 32));
        }
    }
    acc = block_sum64(acc, sh.sc);
    len = block_sum64(len, sh.sc);
    cnt = block_sum64(cnt, sh.sc);
    if (threadIdx.x == 0) { S.fp[v] = acc; S.slen[v] = len + cnt; }  // (SimDev::slen)
}

// ---------------------------------------------------------------- set_views
// rp_sim_set_views: the bootstrap of nodes [v0, v0 + count) redone with
// arbitrary full views (status / incarnation per member; the node's own
// entry alive): makeAlive(self) then set() of the others in id order
// (lib/membership.js:162-206), whose listener (lib/membership-set-listener.js:
// 24-48) adds the alive ones to the ring and starts a suspicion timer per
// suspect; then shuffle() and clearChanges() as in k_init_*.  The bootstrap
// clock lies more than one suspicion period before round 0, so those timers
// are due at round 0: their start round is -25 (k_timers).
constexpr uint32_t BOOT_TIMER_ROUND = 0xFFFFFFE7u;  // (uint32)-25
// One block per node of the range (every shard: the per-node scalars of all
// of them; the node's own shard: its rows).  st/inc: count x n, this range.
// member_map (rp_sim_join): instead of st/inc, the view of the members in the
// map, everyone alive at INC0 + id.
__global__ void __launch_bounds__(BLOCK) k_set_views(SimDev S, uint32_t v0, const uint8_t* st, const uint64_t* inc,
                                                     uint64_t seed, uint8_t* need_shuffle, const uint8_t* member_map) {
    __shared__ Shared sh;
    const uint32_t v = v0 + blockIdx.x, n = S.n;
    const uint8_t* srow = member_map ? member_map : st + (size_t)blockIdx.x * n;
    const uint64_t* irow = member_map ? nullptr : inc + (size_t)blockIdx.x * n;
    auto inc_of = [&](uint32_t a) { return irow ? irow[a] : INC0 + a; };
    const bool local = S.local(v);
    VEnt* vrow = local ? S.view + S.row(v) : nullptr;
    uint8_t* rrow = local ? S.in_ring + S.row(v) : nullptr;
    uint32_t ring = 0, ping = 0;
    uint32_t tpos = 0, mpos = 1;  // timers, members so far (block-wide; the node itself is member 0)
    for (uint32_t c0 = 0; c0 < n; c0 += BLOCK) {
        const uint32_t a = c0 + threadIdx.x;
        uint32_t stt = ST_ABSENT;  // (status 0: not a member of this view)
        if (a < n) stt = a == v ? ST_ALIVE : srow[a];
        const bool susp = a < n && a != v && stt == ST_SUSPECT;
        const bool other = a < n && a != v && stt != ST_ABSENT;
        uint32_t tot, mtot;
        const uint32_t r = block_rank(susp, sh.sc, tot);
        const uint32_t mr = block_rank(other, sh.sc, mtot);
        if (a < n) {
            ring += stt == ST_ALIVE;
            ping += a != v && is_pingable_status(stt);
            if (local) {
                VEnt c;
                c.vs = stt == ST_ABSENT ? 0ull : pack_view(inc_of(a), stt);
                c.dpos = NONE;
                c.tstamp = 0;
                if (susp) {
                    const uint32_t p = tpos + r;
                    if (p < S.tcap) S.tfifo[S.trow(v) + p] = make_uint2(a, BOOT_TIMER_ROUND);
                    c.tstamp = p + 1;
                }
                vrow[a] = c;
                rrow[a] = stt == ST_ALIVE;
                if (a == v) S.order[S.row(v)] = a;
                else if (other) S.order[S.row(v) + mpos + mr] = a;  // set(): the others in id order
            }
        }
        tpos += tot;
        mpos += mtot;
        __syncthreads();
    }
    const uint64_t rt = block_sum64(((uint64_t)ring << 32) | ping, sh.sc);
    if (threadIdx.x == 0) {
        uint64_t s = node_rng_seed(seed, v);
        (void)js_math_random(s);  // getJoinPosition() for the local member (lib/membership.js:99-101)
        S.rng[v] = s;
        S.iter_index[v] = -1;
        S.iter_round[v] = 0;
        S.dhead[v] = 0; S.dtail[v] = 0; S.dlive[v] = 0; S.icount[v] = 0;
        S.max_pb[v] = max_piggyback(1);  // ringChanged after the local member joined the ring; set() emits none
        S.ring_count[v] = (int32_t)(rt >> 32);
        S.npingable[v] = (int32_t)(uint32_t)rt;
        S.mcount[v] = mpos;
        S.csum_valid[v] = 0;
        S.dead[v] = 0;
        S.self_inc[v] = inc_of(v);
        S.thead[v] = 0;
        S.ttail[v] = min(tpos, S.tcap);
        if (tpos > S.tcap) atomicOr(S.err, SIMERR_TIMERS_FULL);
        S.rbatch[v] = 0;
        need_shuffle[v] = local ? 1 : 0;
    }
}
// Ring owners of the colliding replica hashes in a re-bootstrapped view: the
// local member's own (inserted first), else the smallest alive server of the
// group (set() inserts in id order; first inserter wins, lib/rbtree.js:112-117).
__global__ void k_set_owners(SimDev S, uint32_t v0, uint32_t count) {
    const uint64_t total = (uint64_t)count * S.ncoll;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = v0 + (uint32_t)(i / S.ncoll), g = (uint32_t)(i % S.ncoll);
        int32_t own = -1;
        for (uint32_t q = S.cmem_off[g]; q < S.cmem_off[g + 1]; q++) {
            const uint32_t sv = S.cmem[q];
            if (sv == v) { own = (int32_t)v; break; }
            if (own < 0 && S.in_ring[S.row(v) + sv]) own = (int32_t)sv;
        }
        S.coll_owner[S.crow(v) + g] = own;
    }
}

// ---------------------------------------------------------------- round
// The round's makeAlive updates (membership.makeAlive(self, now),
// lib/membership.js:141-144), one block per churn slot j, on every shard:
// the update gets sequence number base + j, base = origin_count at the
// round's start (k_round_start's snapshot; only churn allocates makeAlive
// origins), stored in ring slot alive_base + seq mod ring (makeUpdate: source
// = the node, sourceIncarnationNumber = its incarnation before the update,
// :327-337); the node's own shard then applies it.
__global__ void __launch_bounds__(BLOCK) k_churn(SimDev S, uint32_t k, uint32_t round_slot, uint64_t now) {
    __shared__ Shared sh;
    const uint32_t base = S.oc_snap[S.round & 1];
    if (blockIdx.x == 0 && threadIdx.x == 0) *S.origin_count = base + k;
    const int32_t vi = S.churn_ids[(size_t)round_slot * k + blockIdx.x];
    if (vi < 0) return;
    const uint32_t v = (uint32_t)vi, seq = base + blockIdx.x;
    if (threadIdx.x == 0) {
        const uint32_t id = S.alive_base + (seq & S.alive_mask);
        S.origins[id].source = v;
        S.origins[id].source_inc = S.local(v) ? v_inc(S.view[S.row(v) + v].vs) : S.self_inc[v];
        S.origins[id].round = S.round;
        S.self_inc[v] = now;
    }
    if (!S.local(v)) return;
    __syncthreads();  // (the origin record before the merge)
    Change c;
    c.addr = v; c.origin = (seq & ORIGIN_ID_MASK) | ORIGIN_ALIVE; c.vs = pack_view(now, ST_ALIVE);
    auto src = [&](uint32_t) { return c; };
    wg_apply(S, v, src, 1, 1, now, 1, 0, sh);
}

// Start of round r: snapshot origin_count and clear every node's seen bits for
// the ids allocated during round r-1 (they become trackable this round).
// blk: this block's index among the seen-clearing blocks (k_round_start).
__device__ inline void seen_clear(const SimDev& S, uint32_t blk) {
    // 4 nodes per block, one wave per node
    const uint32_t prev = S.oc_snap[(S.round + 1) & 1], now = *S.origin_count;
    if (blk == 0 && threadIdx.x == 0) S.oc_snap[S.round & 1] = now;
    const uint32_t v = S.lo + blk * 4 + (threadIdx.x >> 6);
    if (now == prev || v >= S.lo + S.nl) return;
    const uint32_t wlo = prev >> 5, whi = (now + 31) >> 5;  // words holding ids [prev, now)
    const uint32_t nw = min(whi - wlo, S.seen_words);     // all of them: the window turned over
    uint32_t* row = S.seen + S.srow(v);
    for (uint32_t j = threadIdx.x & 63; j < nw; j += 64) {
        const uint32_t word = wlo + j, b0 = word * 32u;
        uint32_t m = 0xFFFFFFFFu;
        if (nw < S.seen_words) {
            if (prev > b0) m &= ~((1u << (prev - b0)) - 1u);
            if (now < b0 + 32u) m &= (1u << (now - b0)) - 1u;
        }
        row[word & (S.seen_words - 1u)] &= ~m;
    }
}

// MembershipIterator.next (lib/membership-iterator.js:29-52): advance to the
// next pingable member; reaching the end of the list reshuffles it (k_shuffle)
// and the scan continues from its start.
__global__ void k_iterate(SimDev S, uint8_t* need_shuffle, uint32_t* shuf_list, uint32_t* shuf_count) {
    uint32_t v = S.lo + blockIdx.x * blockDim.x + threadIdx.x;
    const bool mine = v < S.lo + S.nl;
    bool found = false;
    if (mine) {
        S.target[v] = -1;
        S.min_cnt[v] = NONE;
        S.min_safe[v] = NONE;
        S.min_l1[v] = ~0ull;
        S.min_l2[v] = ~0ull;
        S.need_csum[v] = 0;
    }
    if (mine && !S.dead[v]) {
        if (S.npingable[v] <= 0) {
            atomicOr(S.err, SIMERR_PING_FAILED);  // "no usable nodes" path not modelled yet
        } else {
            const uint32_t* ord = S.order + S.row(v);
            const VEnt* row = S.view + S.row(v);
            const int32_t M = (int32_t)S.mcount[v];
            for (int32_t idx = S.iter_index[v] + 1; idx < M; idx++) {
                uint32_t a = ord[idx];
                if (a != v && is_pingable_status(v_status(row[a].vs))) {
                    S.iter_index[v] = idx;
                    S.target[v] = (int32_t)a;
                    set_same_view(S, v, a);
                    found = true;
                    break;
                }
            }
            if (!found) {
                S.iter_round[v]++;
                need_shuffle[v] = 1;
                shuf_list[atomicAdd(shuf_count, 1u)] = v;  // (rare: an iterator wraps once per ~n pings)
            }
        }
    }
}

// occupancy targets (waves per SIMD) chosen as the most the register
// allocator reaches without spilling: the round kernels are latency-bound
// chains of dependent loads, so resident waves are what hides them
#ifndef RP_P1_WAVES
#define RP_P1_WAVES 7
#endif
#ifndef RP_P2_WAVES
#define RP_P2_WAVES 6
#endif
#ifndef RP_P3_WAVES
#define RP_P3_WAVES 7
#endif
template <bool ESC, bool SET>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(RP_P1_WAVES, RP_P1_WAVES))) k_phase1(SimDev S) {
    __shared__ Shared sh;
    const uint32_t v = S.lo + blockIdx.x;
    const int32_t T = S.target[v];
    // (the sender's incarnation and fingerprint, which the issue does not
    // change, read with the target rather than after the issue)
    // (uniform addresses: scalar loads, kept in SGPRs across the issue)
    const uint64_t svs = S.view[S.row(v) + v].vs, sfp = S.fp[v];
    // the same-view decision, in the same round trip as the target
    const uint64_t sv = sload64(S.sv_word + v);
    if (T < 0) return;
    // one shard: this round's grouping of the pings by target counts here
    // (Shard::group without its k_group_count launch)
    if (S.nranks == 1 && threadIdx.x == 0) atomicAdd(&S.g_cnt[T], 1u);
    uint64_t off;
    uint32_t pm, pe;
    // the seen filter: the target's own bitset on this shard, else the cluster-wide mask
    // (the same-view decision against the target's fingerprint -- now, or on
    // another shard at its last ping -- was taken when the target was chosen:
    // nothing it reads changes before this block's issue)
    const bool tl = S.local((uint32_t)T);
    __builtin_assume(T < 0x7FFFFFFF);  // (the destination is never NONE: its seen bitset is staged)
    uint32_t m = wg_issue<ESC, RP_ISSUE_UNR_P1, SET, SET && RP_SETTLED_PF, true>(S, v, false, NONE, 0, &off, 1, sh,
                                                     tl ? (uint32_t)T : ((uint32_t)T | DEST_REMOTE), &pm, &pe,
                                                     FP_NONE, sv);  // issueAsSender (ping-sender.js:70)
    if (threadIdx.x == 0) {
        S.msg_off[v] = off;
        S.msg_len[v] = m;
        S.msg_plen[v] = pm;
        S.msg_nesc[v] = pe;
        S.snd_inc[v] = v_inc(svs);  // getIncarnationNumber()
        S.snd_fp[v] = sfp;
        stat_add(S, STAT_PINGS, 1ull);
        stat_add(S, STAT_MESSAGES, 1ull);
    }
}

// ---------------------------------------------------------------- grouping
// Messages of a wave live in "slots" (a sender id, or 3*A+i for the i-th
// ping-req relay of A).  A wave is delivered per destination in slot order,
// which is the harness's queue order.
__global__ void k_group_count(const int32_t* dest, uint32_t nslots, uint32_t* cnt) {
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nslots) return;
    int32_t t = dest[s];
    if (t >= 0) atomicAdd(&cnt[t], 1u);
}
// single-block exclusive scan of cnt[n] -> base[n+1]
// Exclusive scan of the per-destination counts (base[n] = total) in two
// launches of coalesced 1,024-element tiles: each tile's local scan and total
// (k_group_scan), then every tile adds the sum of the tiles before it
// (k_group_scan_add).  A single block walking strided 64-element ranges took
// 63-90 us per round at 65,536 nodes.
__device__ inline uint32_t block_scan_incl_1024(uint32_t x, uint32_t* wsum) {
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if ((int)lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t q = 0; q < w; q++) before += wsum[q];
    return x + before;
}
__global__ void __launch_bounds__(1024) k_group_scan(const uint32_t* cnt, uint32_t* base, uint32_t n, uint32_t* tile) {
    __shared__ uint32_t wsum[16];
    const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
    const uint32_t x = i < n ? cnt[i] : 0u;
    const uint32_t incl = block_scan_incl_1024(x, wsum);
    if (i < n) base[i] = incl - x;
    if (threadIdx.x == 1023) tile[blockIdx.x] = incl;
}
__global__ void __launch_bounds__(1024) k_group_scan_add(uint32_t* base, uint32_t n, const uint32_t* tile) {
    __shared__ uint32_t wsum[16];
    // the sum of the tiles before this one (tiles = gridDim.x <= 1024 ... any)
    uint32_t part = 0;
    for (uint32_t t = threadIdx.x; t < blockIdx.x; t += 1024) part += tile[t];
    const uint32_t off = block_scan_incl_1024(part, wsum);  // (thread 1023: the whole sum)
    __shared__ uint32_t tot;
    if (threadIdx.x == 1023) tot = off;
    __syncthreads();
    const uint32_t o = tot, i = blockIdx.x * 1024 + threadIdx.x;
    if (i < n) base[i] += o;
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) base[n] = o + tile[blockIdx.x];
}
// With the tiles' totals prefix-summed in each block (pre[j]: the counts of
// tiles before j), fill and sort read the tile-local bases of k_group_scan
// directly and the sort writes the final bases: no k_group_scan_add launch.
constexpr uint32_t GROUP_FUSE_TILES = 1024;  // (n <= 2^20; larger clusters take the three-launch scan)
__device__ inline void group_tile_prefix(const uint32_t* tile, uint32_t tiles, uint32_t* pre) {
    if (threadIdx.x < 64) {  // one wave: 16 tiles per lane, then a wave scan of the lane sums
        const uint32_t l = threadIdx.x;
        uint32_t v[16], sum = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) { v[k] = 16 * l + k < tiles ? tile[16 * l + k] : 0u; sum += v[k]; }
        uint32_t incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if ((int)l >= o) incl += y;
        }
        uint32_t run = incl - sum;
#pragma unroll
        for (int k = 0; k < 16; k++) { pre[16 * l + k] = run; run += v[k]; }
        if (l == 63) pre[GROUP_FUSE_TILES] = incl;  // (all of them)
    }
    __syncthreads();
}
__global__ void __launch_bounds__(256) k_group_fill2(const int32_t* dest, uint32_t nslots, const uint32_t* bloc,
                                                     const uint32_t* tile, uint32_t tiles, uint32_t* fill,
                                                     uint32_t* list) {
    __shared__ uint32_t pre[GROUP_FUSE_TILES + 1];
    group_tile_prefix(tile, tiles, pre);
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nslots) return;
    const int32_t t = dest[s];
    if (t >= 0) list[bloc[t] + pre[(uint32_t)t >> 10] + atomicAdd(&fill[t], 1u)] = s;
}
__global__ void __launch_bounds__(256) k_group_sort2(const uint32_t* bloc, const uint32_t* tile, uint32_t tiles,
                                                     uint32_t* list, uint32_t n, uint32_t* base) {
    __shared__ uint32_t pre[GROUP_FUSE_TILES + 1];
    group_tile_prefix(tile, tiles, pre);
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > n) return;
    const uint32_t total = pre[GROUP_FUSE_TILES];
    if (b == n) { base[n] = total; return; }
    const uint32_t lo = bloc[b] + pre[b >> 10], hi = b + 1 < n ? bloc[b + 1] + pre[(b + 1) >> 10] : total;
    base[b] = lo;
    for (uint32_t i = lo + 1; i < hi; i++) {
        uint32_t x = list[i], j = i;
        while (j > lo && list[j - 1] > x) { list[j] = list[j - 1]; j--; }
        list[j] = x;
    }
}
__global__ void k_group_fill(const int32_t* dest, uint32_t nslots, const uint32_t* base, uint32_t* fill,
                             uint32_t* list) {
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nslots) return;
    int32_t t = dest[s];
    if (t >= 0) list[base[t] + atomicAdd(&fill[t], 1u)] = s;
}
__global__ void k_group_sort(const uint32_t* base, uint32_t* list, uint32_t n) {
    uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n) return;
    uint32_t lo = base[b], hi = base[b + 1];
    for (uint32_t i = lo + 1; i < hi; i++) {
        uint32_t x = list[i], j = i;
        while (j > lo && list[j - 1] > x) { list[j] = list[j - 1]; j--; }
        list[j] = x;
    }
}

__device__ inline uint32_t node_checksum(const SimDev& S, uint32_t v) {
    AddrTable at{S.addr_words, S.addr_len};
    const VEnt* row = S.view + S.row(v);
    return view_checksum([&](uint32_t a) { return row[a].vs; }, S.n, at);
}
__device__ inline uint32_t cached_checksum(const SimDev& S, uint32_t v) {
    if (!S.csum_valid[v]) { S.csum[v] = node_checksum(S, v); S.csum_valid[v] = 1; }
    return S.csum[v];
}

__device__ inline bool cut(const SimDev& S, uint32_t a, uint32_t b) {
    return S.part_split > 0 && S.round >= S.part_start && S.round < S.part_end &&
           ((a < S.part_split) != (b < S.part_split));
}
__device__ inline bool unreachable(const SimDev& S, uint32_t from, uint32_t to) {
    return S.dead[to] || cut(S, from, to);
}
__device__ inline void note_wave(const SimDev& S, uint32_t w) {
    // (no return: the block does not wait on it)
    atomicMax(&S.bstats[(size_t)STAT_WAVES * S.bstride + blockIdx.x], (unsigned long long)w);
}

// Which senders' checksum snapshots can a receiver need?  A receiver B
// compares checksums only when its issueAsReceiver list for sender A_j (its
// j-th ping this round) comes out empty (lib/dissemination.js:102-117).  That
// cannot happen when B's log still holds an entry that A_j's filter cannot
// skip (:91-98: makeAlive and fullSync origins never match; a local
// suspect/faulty origin matches only its own source) whose piggyback count c
// satisfies c + j <= the smallest maxPiggybackCount B can have this phase
// (an overwrite only resets c), and B's ring cannot empty (more
// servers than inbound changes).  Pings to unreachable receivers get a
// transport error, never a comparison.  Only the remaining senders get the
// (sequential, per-view) farmhash snapshot.
// (fd[0..nfd): the shards' counts of members declared faulty (k_fdecl_share;
// one shard: its fdecl_count), which bound the members any node knows as
// faulty or leave, so b's ring loses at most min(inbound, their sum) servers
// before it answers its pings; see k_pr_need.  nullptr: no such bound.)
// The local senders that need a snapshot are listed for k_checksums as they
// are found (membership.checksum in the ping body, lib/swim/ping-sender.js:71;
// a sender pings one receiver, so it is listed at most once).
__global__ void k_need_checksums(SimDev S, const uint32_t* fd, uint32_t nfd, uint32_t* list, uint32_t* count) {
    uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= S.n) return;
    const uint32_t lo = S.g_base[b], hi = S.g_base[b + 1];
    if (lo == hi) return;
    uint64_t inbound = 0;
    for (uint32_t j = lo; j < hi; j++) inbound += S.msg_len[S.g_list[j]];
    if (fd) {
        uint64_t F = 0;
        for (uint32_t i = 0; i < nfd; i++) F += fd[i];
        inbound = min(inbound, F);
    }
    const bool safe = (uint64_t)S.ring_count[b] > inbound;
    // maxPiggybackCount changes only on ringChanged, to the rule's value for
    // the new server count (it starts below that: lib/dissemination.js:38-55)
    const uint32_t maxpb_lo =
        safe ? min((uint32_t)S.max_pb[b], (uint32_t)max_piggyback((int)((uint64_t)S.ring_count[b] - inbound))) : 0u;
    const uint32_t ms = S.min_safe[b];
    const uint64_t l1 = S.min_l1[b], l2 = S.min_l2[b];
    for (uint32_t j = lo; j < hi; j++) {
        const uint32_t A = S.g_list[j];
        if (unreachable(S, A, b)) continue;
        const uint64_t l = (uint32_t)l1 != A ? l1 : l2;
        const uint32_t mc = min(ms, l == ~0ull ? NONE : (uint32_t)(l >> 32));
        const bool p = safe && mc != NONE && mc + (j - lo + 1) <= maxpb_lo;
        if (!p) {
            S.need_csum[A] = 1;
            if (S.local(A)) list[atomicAdd(count, 1u)] = A;
        }
    }
}

// Checksum of one view by a whole wave (lib/membership.js:41-93).  farmhash
// is one sequential chain per string, but rendering the string is not: per
// chunk of 64 members each lane renders its member (and the ';' before it)
// into a per-wave LDS buffer at its prefix-sum offset, then every lane runs
// the same hash steps over the buffer's whole 20-byte blocks (broadcast LDS
// reads; no divergence) and the leftover bytes move to the buffer's front.
// One view costs one hash chain plus 1/64 of its rendering, instead of a
// lane's whole rendering, and a handful of views fill as many waves as there
// are views (a lane per view left most of the GPU idle: config 5).
constexpr uint32_t CKW_TEXT = 3712;  // < 20 carried + 64 x (1 + 32 + 7 + 16) rendered bytes
constexpr uint32_t CKW_PRE = 184;    // >= the 20-byte blocks of one chunk (CKW_TEXT / 20)
constexpr uint32_t CKW_BUF = CKW_TEXT + CKW_PRE * 48;  // + their fh_stream_pre records
struct LdsByteEmit {
    uint8_t* p;
    __device__ inline void operator()(uint32_t w) {
        p[0] = (uint8_t)w; p[1] = (uint8_t)(w >> 8); p[2] = (uint8_t)(w >> 16); p[3] = (uint8_t)(w >> 24);
        p += 4;
    }
};
__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
}
// the same for LDS only (s_waitcnt lgkmcnt(0)): loads from global memory
// issued before it -- the next chunk's prefetch -- stay in flight
__device__ inline void wave_lds_fence() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // vmcnt and expcnt at their maxima, lgkmcnt 0
    __builtin_amdgcn_wave_barrier();
}
template <class RowFn>
__device__ uint32_t wave_view_checksum(RowFn row, uint32_t n, const AddrTable& at, uint8_t* buf) {
    const uint32_t lane = lane_id();
    // pass 1 (parallel): string length and present-member count (8 rows in
    // flight per lane)
    uint64_t len = 0, cnt = 0;
    constexpr uint32_t P1 = 8;
    for (uint32_t a0 = lane; a0 < n; a0 += 64 * P1) {
        uint64_t vs[P1];
        uint32_t L[P1];
#pragma unroll
        for (uint32_t k = 0; k < P1; k++) {
            const uint32_t a = a0 + 64 * k;
            vs[k] = a < n ? row(a) : 0ull;
            L[k] = a < n ? at.len[a] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < P1; k++) {
            if (v_status(vs[k]) == ST_ABSENT) continue;  // (also rows past n)
            len += L[k] + status_len(v_status(vs[k])) + dec_len(v_inc(vs[k]));
            cnt++;
        }
    }
    len = wave_sum64(len);
    cnt = wave_sum64(cnt);
    if (cnt == 0) return farmhash32(nullptr, 0);
    len += cnt - 1;
    if (len <= 24) return small_view_checksum(row, n, at, (uint32_t)len);
    FhStream st;
    {
        const TailEmit t = checksum_tail(row, n, at);  // (every lane, same values)
        st = fh_stream_begin5((uint32_t)len, t.t0, t.t1, t.t2, t.t3, t.t4);
    }
    FhLanes fl;
    fl.init(st);
    uint32_t carry = 0;
    bool any_before = false;
    // software pipeline: the next chunk's view values and addresses are in
    // flight while this chunk renders and hashes (each chunk otherwise waits
    // a full memory round trip before its sequential hash blocks)
    uint64_t vs_n = 0;
    uint32_t L_n = 0;
    uint4 wa_n = make_uint4(0, 0, 0, 0), wb_n = wa_n;
    auto fetch = [&](uint32_t a) {
        if (a < n) {
            vs_n = row(a);
            L_n = at.len[a];
            const uint4* p = (const uint4*)(at.words + (size_t)a * ADDR_WORDS);
            wa_n = p[0];
            wb_n = p[1];
        } else {
            vs_n = 0;
        }
    };
    fetch(lane);
    for (uint32_t c0 = 0; c0 < n && st.blocks_left; c0 += 64) {
        const uint32_t a = c0 + lane;
        const uint64_t vs = vs_n;
        const uint32_t L = L_n;
        const uint4 aw0 = wa_n, aw1 = wb_n;
        fetch(c0 + 64 + lane);
        const bool present = a < n && v_status(vs) != ST_ABSENT;
        const uint64_t m = __ballot(present);
        const bool sep = present && (any_before || (m & ((1ull << lane) - 1ull)) != 0);
        const uint32_t b = present ? L + status_len(v_status(vs)) + dec_len(v_inc(vs)) + (sep ? 1u : 0u) : 0u;
        uint32_t incl = b;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if ((int)lane >= o) incl += y;
        }
        const uint32_t total = __shfl(incl, 63);
        if (present) {
            WordSink<LdsByteEmit> w;
            w.emit.p = buf + carry + (incl - b);
            if (sep) w.put(0x3Bu, 1);
            put_member_regs(w, L, aw0, aw1, vs);
            for (uint32_t i = 0; i < w.bits / 8; i++) w.emit.p[i] = (uint8_t)(w.acc >> (8 * i));
        }
        any_before |= m != 0;
        wave_lds_fence();
        const uint32_t avail = carry + total;
        const uint32_t nb = min(avail / 20u, st.blocks_left);
        const uint32_t* wb = (const uint32_t*)buf;
        // the blocks' data-only mixing, one block per lane; then the
        // sequential chain over the 48-byte records (three 16-byte LDS reads
        // per block, the next block's in flight)
        uint32_t* const pre = (uint32_t*)(buf + CKW_TEXT);
        for (uint32_t j = lane; j < nb; j += 64)
            fh_stream_pre_sliced(wb[5 * j], wb[5 * j + 1], wb[5 * j + 2], wb[5 * j + 3], wb[5 * j + 4], pre + 12 * j);
        wave_lds_fence();
        fl.run((const uint4*)pre, 0, nb);  // (the chain: FhLanes)
        st.blocks_left -= nb;
        const uint32_t left = avail - 20u * nb;
        // (while blocks remain, left < 20 <= 20 nb or nb = 0: no overlapping move)
        uint8_t mv = 0;
        if (nb && st.blocks_left && lane < left) mv = buf[20u * nb + lane];
        wave_lds_fence();
        if (nb && st.blocks_left && lane < left) buf[lane] = mv;
        wave_lds_fence();
        carry = left;
    }
    return fh_stream_end(fl.get(0));
}

// Checksums of a list of local views, one wave per view (grid-stride).
// Writes the cache (csum, csum_valid) and out[node].
// run_min: the list is left alone unless it holds at least run_min views
// (the round's sender checksums with a side stream: the live views only when
// the leaders outnumber the snapshot rows, k_ck_snapcopy)
__global__ void __launch_bounds__(BLOCK) k_checksums(SimDev S, const uint32_t* list, const uint32_t* count,
                                                     uint32_t* out, uint32_t run_min = 0) {
    __shared__ __attribute__((aligned(16))) uint8_t bufs[NWAVE][CKW_BUF];
    const uint32_t cnt = *count;
    if (cnt >= S.ck_lane_min || cnt < run_min) return;  // (k_checksums_pc takes the list)
    const AddrTable at{S.addr_words, S.addr_len};
    for (uint32_t i = blockIdx.x * NWAVE + wave_id(); i < cnt; i += gridDim.x * NWAVE) {
        const uint32_t v = list[i];
        if (S.csum_valid[v]) {
            if (lane_id() == 0) out[v] = S.csum[v];
            continue;
        }
        const VEnt* row = S.view + S.row(v);
        const uint32_t c = wave_view_checksum([&](uint32_t a) { return row[a].vs; }, S.n, at, bufs[wave_id()]);
        if (lane_id() == 0) {
            S.csum[v] = c;
            S.csum_valid[v] = 1;
            out[v] = c;
            stat_add(S, STAT_CK_VIEWS, 1ull);  // (a view row of n cells rendered and hashed)
        }
    }
}

// Checksums of a long list of views, one LANE per view (a wave hashes 64
// views at once).  wave_view_checksum spreads one view's rendering over a
// wave but runs its farmhash chain -- 115 k dependent 20-byte blocks for a
// 65,536-member view -- on all 64 lanes at once, so a list of thousands of
// views is bound by (views / resident waves) chain latencies (~1.8 ms each:
// 400 ms for every view of config 4).  Here every lane runs its own view's
// chain: the lanes of a wave walk the members in the same order, so each
// member's address is one uniform (scalar) load for the whole wave, while the
// status and incarnation, the byte offsets and the hash state are per lane.
// A lane renders its member's text as whole little-endian words into its own
// LDS ring and hashes every complete 20-byte block; the string length comes
// from SimDev::slen and the last 20 bytes from a short walk back from the end,
// as farmhash's > 24-byte branch needs both before the first block.  Used
// when the list outnumbers what wave-per-view keeps in flight (SimDev::
// ck_lane_min); short lists (a round's senders) stay on k_checksums.
#ifndef RP_CK_LANE_MIN
#define RP_CK_LANE_MIN 12288  // the default of rp_sim_config.ck_lane_min (measured crossover)
#endif
// A lane's byte stream into its LDS buffer, by whole words.  `acc` holds the
// nb (0-3) bytes of the incomplete word; appending a piece of K bytes given as
// little-endian words c[] writes the words (acc | c << 8 nb, then
// alignbyte(c[i], c[i - 1], 4 - nb)) unconditionally at the write position and
// advances it by the number completed (a word written past it is garbage that
// a later append overwrites before the hash reads it).  No branches: a piece
// is a handful of funnel shifts and LDS writes (at immediate offsets from the
// write position) whatever its length.  The buffer is linear: after each hash
// drain the < 5 words left are moved to its front.
struct LaneStream {
    uint32_t* buf;
    uint32_t acc, nb, wpos;
    __device__ inline void w(uint32_t i, uint32_t x) { buf[wpos + i] = x; }
    __device__ static inline uint32_t low_bytes(uint32_t x, uint32_t k) { return x & ((1u << (8 * k)) - 1u); }
    __device__ inline uint32_t fun(uint32_t hi, uint32_t lo) const {  // bytes [4 - nb, 8 - nb) of lo|hi
        // (one byte permute: selector byte m = 4 - nb + m; 4..7 name hi's bytes, 0..3 lo's)
        return __builtin_amdgcn_perm(hi, lo, 0x07060504u - nb * 0x01010101u);
    }
    // the state after appending K bytes (0 when off) whose words from the
    // write position on are o_lo (word (nb + K) >> 2 when that is W - 1) / o_hi
    __device__ inline void advance(uint32_t K, uint32_t o_lo, uint32_t o_hi, uint32_t W) {
        const uint32_t tot = nb + K, nout = tot >> 2;
        acc = K ? low_bytes(nout == W ? o_hi : o_lo, tot & 3) : acc;
        wpos += nout;
        nb = tot & 3;
    }
    __device__ inline void byte(uint32_t b, bool on) {
        const uint32_t x = acc | (b << (8 * nb));
        w(0, x);
        advance(on ? 1u : 0u, x, 0u, 1u);  // (nb + 1 < 4: the acc is x; = 4: word 1, i.e. empty)
    }
    // K uniform bytes in uniform words c[0 .. W), W = ceil(K / 4) <= MAXW (K >= 1)
    template <uint32_t MAXW = 8>
    __device__ inline void uniform_piece(const uint32_t* c, uint32_t K, uint32_t W, bool on) {
        uint32_t prev = acc | (c[0] << (8 * nb)), cur = prev;
        w(0, prev);
#pragma unroll
        for (uint32_t i = 1; i <= MAXW; i++) {
            if (i > W) break;  // (uniform)
            const uint32_t ci = i < W ? c[i] : 0u;
            prev = cur;
            cur = fun(ci, c[i - 1]);
            w(i, cur);
        }
        advance(on ? K : 0u, prev, cur, W);
    }
    // The same append without a loop: all MAXW + 1 output words are computed
    // (compile-time register indices) and written whatever K is.  The new
    // partial word is output word nout = (nb + K) >> 2, which is Q or Q + 1
    // for the wave-uniform Q = K >> 2: two uniformly indexed register reads
    // and a select.  c[0 .. MAXW] are read (values past K are don't-care);
    // K (wave-uniform) in 1 .. 4 MAXW.
    template <uint32_t MAXW>
    __device__ inline void uniform_piece_flat(const uint32_t* c, uint32_t K, bool on) {
        uint32_t o[MAXW + 1];
        o[0] = acc | (c[0] << (8 * nb));
#pragma unroll
        for (uint32_t i = 1; i <= MAXW; i++) o[i] = fun(c[i], c[i - 1]);
#pragma unroll
        for (uint32_t i = 0; i <= MAXW; i++) w(i, o[i]);
        const uint32_t Q = __builtin_amdgcn_readfirstlane(K >> 2);
        const uint32_t oq = o[min(Q, MAXW)], oq1 = o[min(Q + 1, MAXW)];
        const uint32_t tot = nb + (on ? K : 0u), nout = tot >> 2, r = tot & 3;
        acc = on ? low_bytes(nout == Q ? oq : oq1, r) : acc;
        wpos += nout;
        nb = r;
    }
};
// String(incarnationNumber) as four 4-digit groups right-aligned in 16 bytes
// D[0..3], and its digit count
__device__ inline void dec16(uint64_t v, uint32_t D[4], uint32_t& nd) {
    const uint64_t hi = v / 100000000ull;
    const uint32_t lo = (uint32_t)(v - hi * 100000000ull);
    const uint32_t h32 = (uint32_t)hi;  // (< 2^53 / 10^8 < 2^27)
    auto len32 = [](uint32_t x) {
        return 1u + (x >= 10u) + (x >= 100u) + (x >= 1000u) + (x >= 10000u) + (x >= 100000u) + (x >= 1000000u) +
               (x >= 10000000u) + (x >= 100000000u);
    };
    nd = h32 ? 8u + len32(h32) : len32(lo);
    D[0] = dec4(h32 / 10000u); D[1] = dec4(h32 % 10000u); D[2] = dec4(lo / 10000u); D[3] = dec4(lo % 10000u);
}
// status and String(incarnationNumber) of one member (lib/membership.js:
// 84-90) appended to a lane's stream; on = the member is rendered.
__device__ inline void lane_status_inc(LaneStream& ls, uint64_t vs, bool on) {
    const uint32_t stt = v_status(vs);
    const uint32_t w0 = stt == ST_SUSPECT ? 0x70737573u : stt == ST_FAULTY ? 0x6c756166u : stt == ST_ALIVE ? 0x76696c61u : 0x7661656cu;
    const uint32_t w1 = stt == ST_SUSPECT ? 0x746365u : stt == ST_FAULTY ? 0x7974u : 0x65u;
    const uint32_t sl = stt == ST_SUSPECT ? 7u : stt == ST_FAULTY ? 6u : 5u;
    {  // the status: 5-7 bytes in two words
        const uint32_t o0 = ls.acc | (w0 << (8 * ls.nb));
        const uint32_t o1 = ls.fun(w1, w0), o2 = ls.fun(0u, w1);
        ls.w(0, o0);
        ls.w(1, o1);
        ls.advance(on ? sl : 0u, o1, o2, 2u);
    }
    const uint64_t v = v_inc(vs);
    uint32_t D[4], nd;
    dec16(v, D, nd);
    // stream byte p (p >= nb) is digit byte p + d of D, d = (16 - nd) - nb in
    // [-3, 15]: word i of the output is bytes [4i + d, 4i + d + 4) of D
    // (zeros outside), i.e. E[i + 1] : E[i] shifted by d & 3, E[k] = D[k + (d >> 2)]
    const int32_t d = (int32_t)(16u - nd) - (int32_t)ls.nb;
    const int32_t j0 = d >> 2;  // -1 .. 3
    const uint32_t s = (uint32_t)d & 3u;
    auto Dx = [&](int32_t k) -> uint32_t {
        return k == 0 ? D[0] : k == 1 ? D[1] : k == 2 ? D[2] : k == 3 ? D[3] : 0u;
    };
    uint32_t E[6];
#pragma unroll
    for (int k = 0; k < 6; k++) E[k] = Dx(j0 + k);
    uint32_t o[5];
#pragma unroll
    for (int i = 0; i < 5; i++) o[i] = s ? __builtin_amdgcn_alignbyte(E[i + 1], E[i], s) : E[i];
    // word 0: the acc's bytes below nb (the leading '0' digits that land there are dropped)
    o[0] = ls.acc | (o[0] & ~((1u << (8 * ls.nb)) - 1u));
#pragma unroll
    for (int i = 0; i < 5; i++) ls.w((uint32_t)i, o[i]);
    const uint32_t tot = ls.nb + (on ? nd : 0u), nout = tot >> 2;  // 0 .. 4
    const uint32_t last = nout == 0 ? o[0] : nout == 1 ? o[1] : nout == 2 ? o[2] : nout == 3 ? o[3] : o[4];
    ls.acc = on ? LaneStream::low_bytes(last, tot & 3) : ls.acc;
    ls.wpos += nout;
    ls.nb = tot & 3;
}

constexpr uint32_t CKL_TEXT = 16;  // words per member text (';' + text: <= 56 bytes)
// The lane path: two waves per 64 views (one view per lane): the render
// wave walks the members and writes each lane's byte stream into one of two
// LDS buffers, the hash wave runs the lanes' farmhash chains over the buffer
// the render wave filled one phase (CKP_GRP members) before; a block barrier
// ends each phase.  The hash wave also loads the cells the render wave reads
// (two phases ahead, handed over in LDS), so the render path has no global
// load but the canonical refresh every 64 members.  With one view per lane
// the 65,536 views of config 4 are 1,024 view groups: one wave each (the
// single-wave k_checksums_lanes) was latency-bound, a drain every 4 members
// stalling the render for its dependent LDS reads and the hash chain; two
// waves per group overlap the render and the chains.
// A uniform load through the scalar cache (constant address space: s_load),
// for read-only tables at wave-uniform addresses: it waits on lgkmcnt, not
// behind the vector loads in flight.
typedef __attribute__((address_space(4))) const uint32_t kconst_u32;
__device__ inline uint32_t kload(const uint32_t* p) { return *(kconst_u32*)p; }
#ifndef RP_CKP_GRP
#define RP_CKP_GRP 4
#endif
constexpr uint32_t CKP_GRP = RP_CKP_GRP;           // members per phase
// words per lane buffer (odd): the last member of a phase starts at < 5 +
// (CKP_GRP - 1) x 14 complete words and writes <= 15 from there
constexpr uint32_t CKP_STRIDE = (4 + (CKP_GRP - 1) * 14 + 15) | 1u;
constexpr uint32_t CKP_THREADS = 128;              // wave 0 renders, wave 1 hashes
static_assert(4 + (CKP_GRP - 1) * 14 + 15 <= CKP_STRIDE, "lane buffer too short");
static_assert(64 % CKP_GRP == 0, "a phase's members lie in one chunk of 64");
static_assert(CKP_GRP == 4, "the shared-stream phase is written for 4 members");
#ifndef RP_DIAG_CKSPLIT
#define RP_DIAG_CKSPLIT 0  // (RP_DIAG builds: k_checksums_pc's refresh and shared-phase clocks in diag1 / diag3)
#endif
#ifndef RP_CKP_SHARED
#define RP_CKP_SHARED 1  // k_checksums_pc: shared-stream phases (see below)
#endif
__global__ void __launch_bounds__(CKP_THREADS) k_checksums_pc(SimDev S, const uint32_t* list, const uint32_t* count,
                                                             uint32_t* out) {
    __shared__ uint32_t bufs[2][64 * CKP_STRIDE];
    __shared__ __attribute__((aligned(16))) uint32_t text[64][CKL_TEXT];
    __shared__ uint32_t nbk_sh[2][64];
    __shared__ uint32_t sbuf[2][64];  // a shared-stream phase's words (all hashing lanes')
    __shared__ uint32_t uni_sh[2];    // the phase was shared
    __shared__ uint64_t vs_sh[2][CKP_GRP][64];  // a phase's cells, loaded by the hash wave
    const uint32_t cnt = *count;
    if (cnt < S.ck_lane_min) return;  // (k_checksums takes the list)
    const uint32_t n = S.n, lane = lane_id();
    const bool render = wave_id() == 0;
    const AddrTable at{S.addr_words, S.addr_len};
    const uint32_t NP = (n + CKP_GRP - 1) / CKP_GRP;  // render phases
    for (uint32_t i0 = blockIdx.x * 64; i0 < cnt; i0 += gridDim.x * 64) {
        const uint32_t i = i0 + lane;
        uint32_t v = 0;
        bool act = i < cnt;
        if (act) {
            v = list[i];
            if (S.csum_valid[v]) {
                if (!render) out[v] = S.csum[v];
                act = false;
            }
        }
        const VEnt* const row = S.view + S.row(act ? v : list[i0]);
        auto rowfn = [&](uint32_t a) { return row[a].vs; };
        const int64_t sl = act ? S.slen[v] : 0;
        const uint32_t len = sl > 0 ? (uint32_t)(sl - 1) : 0u;
        const bool run = act && len > 24;
        uint32_t res = 0;
        FhStream st;
        st.h = st.g = st.f = 0;
        st.blocks_left = 0;
        if (!render && act) {
            if (len == 0) {
                res = farmhash32(nullptr, 0);
            } else if (len <= 24) {
                res = small_view_checksum(rowfn, n, at, len);
            } else {
                const TailEmit t = checksum_tail(rowfn, n, at);
                st = fh_stream_begin5(len, t.t0, t.t1, t.t2, t.t3, t.t4);
            }
        }
        const uint64_t runm = __ballot(run);  // (the same in both waves: same views)
        if (runm) {
            // render wave state
            LaneStream ls;
            ls.acc = 0;
            ls.nb = 0;
            ls.wpos = 0;
            bool first = true;
            uint32_t pbl = run ? (len - 1) / 20 : 0u;  // blocks the chain still takes (fh_stream_begin5)
            const uint32_t cl = (uint32_t)__builtin_ctzll(runm);
            const VEnt* const crow = S.view + S.row(__shfl(v, (int)cl));
            uint64_t cvs = 0;   // lane j: the canonical value of member c0 + j
            uint32_t clen = 0;  // ... and its text's length (0: absent)
            // The cells go through LDS: the hash wave (idle most of a phase)
            // loads those of phase p + 2 in phase p into register set (p & 1)
            // -- unconditional loads (clamped index; lanes that do not hash
            // never look at the value: a masked load plus a masked zero into
            // one register makes the zero wait for the load), no register
            // holding a load in flight copied -- and stores them to vs_sh in
            // phase p + 1; the render wave reads them in phase p + 2 with no
            // global load on its path.
            uint64_t vs_a[CKP_GRP], vs_b[CKP_GRP];
            uint32_t lq0 = 0, lq1 = 0, lq2 = 0, lq3 = 0, lq4 = 0;  // the words the last drain left
            bool prev_uni = false;  // the last phase was shared ...
            uint64_t prev_am = 0;   // ... with these lanes active
            if (!render) {
#pragma unroll
                for (uint32_t k = 0; k < CKP_GRP; k++) vs_sh[0][k][lane] = row[min(k, n - 1)].vs;
#pragma unroll
                for (uint32_t k = 0; k < CKP_GRP; k++) {
                    vs_b[k] = row[min(CKP_GRP + k, n - 1)].vs;
                    vs_a[k] = row[min(2 * CKP_GRP + k, n - 1)].vs;
                }
            }
            __syncthreads();  // (phase 0's cells)
            // (RP_DIAG builds: clocks of work and of barrier waits, per role)
            uint64_t dg_work = 0, dg_wait = 0;
            // (RP_DIAG_CKSPLIT: a shared phase's clocks to its decision, to its
            // words written, and from there to the phase's end)
            uint64_t dg_s1 = 0, dg_s2 = 0, dg_s3 = 0;
            auto phase = [&](uint32_t ph, uint64_t (&vsx)[CKP_GRP]) {
                const uint64_t dg_0 = diag_clock();
                uint64_t dg_t1 = dg_0, dg_t2 = dg_0;
                if (render && ph < NP) {
                    uint32_t* const cur = bufs[ph & 1] + lane * CKP_STRIDE;
                    uint64_t vs[CKP_GRP];
#pragma unroll
                    for (uint32_t k = 0; k < CKP_GRP; k++) vs[k] = vs_sh[ph & 1][k][lane];
                    const uint32_t a0 = ph * CKP_GRP;
                    if ((a0 & 63u) == 0) {
                        // canonical texts of members a0 .. a0 + 63 (lane j: member a0 + j)
                        const uint32_t b = a0 + lane;
                        cvs = b < n ? crow[b].vs : 0ull;
                        clen = 0;
                        if (b < n && v_status(cvs) != ST_ABSENT) {
                            const uint32_t L = at.len[b];
                            const uint32_t* aw = at.words + (size_t)b * ADDR_WORDS;
                            uint32_t w[ADDR_WORDS];
#pragma unroll
                            for (uint32_t q = 0; q < ADDR_WORDS; q++) w[q] = aw[q];
                            LaneStream ts;
                            ts.buf = text[lane];
                            ts.acc = 0;
                            ts.nb = 0;
                            ts.wpos = 0;
                            ts.byte(0x3Bu, true);
                            ts.uniform_piece(w, L, (L + 3) >> 2, true);
                            lane_status_inc(ts, cvs, true);
                            ts.buf[ts.wpos] = ts.acc;
                            clen = 4 * ts.wpos + ts.nb;
                        }
                        wave_lds_sync();
                    }
                    // A shared-stream phase: every lane still hashing (active)
                    // holds the same stream state -- write position, partial
                    // word, carried words, its first member behind it -- and
                    // agrees with the canonical value of each of the phase's
                    // members (config 4's views: most phases).  Then all of
                    // them append the same bytes, the canonical texts, and the
                    // wave renders them once: lane i builds word i of the
                    // phase's stream into sbuf (one or two pieces' words
                    // funnel-shifted), instead of every lane appending every
                    // member into its own buffer.  Other phases: per lane.
                    const bool active = run && pbl != 0;
                    const uint64_t am = __ballot(active);
                    bool uni = RP_CKP_SHARED && am != 0;
                    uint32_t word = 0, w0 = 0, c0 = 0, c1 = 0, c2 = 0, c3 = 0;  // (a shared phase's, for its tail)
                    if (uni) {
                        const int fl = (int)__builtin_ctzll(am);
                        w0 = __builtin_amdgcn_readlane(ls.wpos, fl);
                        const uint32_t nb0 = __builtin_amdgcn_readlane(ls.nb, fl);
                        const uint32_t ac0 = __builtin_amdgcn_readlane(ls.acc, fl);
                        c0 = __builtin_amdgcn_readlane(lq0, fl); c1 = __builtin_amdgcn_readlane(lq1, fl);
                        c2 = __builtin_amdgcn_readlane(lq2, fl); c3 = __builtin_amdgcn_readlane(lq3, fl);
                        // (carried words past the write position are stale: not
                        // compared; after a shared phase with the same lanes
                        // active the states are equal by construction)
                        bool differ = !(prev_uni && am == prev_am) &&
                                      (first || ls.wpos != w0 || ls.nb != nb0 || ls.acc != ac0 || (w0 > 0 && lq0 != c0) ||
                                       (w0 > 1 && lq1 != c1) || (w0 > 2 && lq2 != c2) || (w0 > 3 && lq3 != c3));
                        // the members' text lengths (0: absent or past n)
                        auto len_of = [&](uint32_t k, const uint64_t& v) -> uint32_t {
                            const uint32_t a = a0 + k, j = a & 63u;
                            if (a >= n) return 0u;  // (uniform)
                            const uint32_t cvl = __builtin_amdgcn_readlane((uint32_t)cvs, (int)j);
                            const uint32_t cvh = __builtin_amdgcn_readlane((uint32_t)(cvs >> 32), (int)j);
                            differ = differ || v != (((uint64_t)cvh << 32) | cvl);
                            return __builtin_amdgcn_readlane(clen, (int)j);
                        };
                        const uint32_t K0 = len_of(0, vs[0]), K1 = len_of(1, vs[1]), K2 = len_of(2, vs[2]),
                                       K3 = len_of(3, vs[3]);
                        uni = __ballot(active && differ) == 0;
                        dg_t1 = diag_clock();
                        if (uni) {
                            // the phase's stream: the partial word's nb0 bytes, then
                            // the texts; piece k spans bytes [Pk, Pk+1) (P0 = nb0, P4 = T)
                            const uint32_t P1 = nb0 + K0, P2 = P1 + K1, P3 = P2 + K2, T = P3 + K3;
                            // the non-empty piece holding byte x < T
                            auto piece_at = [&](uint32_t x) { return (x >= P1 ? 1u : 0u) + (x >= P2 ? 1u : 0u) + (x >= P3 ? 1u : 0u); };
                            auto start_of = [&](uint32_t k) { return k == 0 ? nb0 : k == 1 ? P1 : k == 2 ? P2 : P3; };
                            auto end_of = [&](uint32_t k) { return k == 0 ? P1 : k == 1 ? P2 : k == 2 ? P3 : T; };
                            // lane i: stream word i, from the piece holding its
                            // first byte (k0, at offset d) and the first word of
                            // the next piece (when the word runs past k0's end):
                            // the three reads are independent, issued together
                            // (lanes past T compute garbage they do not store)
                            const uint32_t bi = 4u * lane;
                            const uint32_t bx = max(bi, nb0);
                            const uint32_t k0 = piece_at(min(bx, T - 1u)), st0 = start_of(k0), d = bx - st0;
                            const uint32_t e = end_of(k0);  // the piece's end
                            const uint32_t* tx = text[(a0 + k0) & 63u];
                            const uint32_t wl = tx[min(d >> 2, CKL_TEXT - 1u)], wh = tx[min((d >> 2) + 1u, CKL_TEXT - 1u)];
                            const uint32_t t1 = text[(a0 + piece_at(min(e, T - 1u))) & 63u][0];
                            if (bi < nb0) {  // (lane 0) the partial word, then the first text's bytes
                                word = ac0 | (wl << (8 * nb0));
                            } else {
                                word = __builtin_amdgcn_alignbyte(wh, wl, d & 3u);
                                if (bi + 4u > e && e < T) {  // (the rest from the next piece)
                                    const uint32_t r = e - bi;  // 1 .. 3 bytes of this one
                                    word = LaneStream::low_bytes(word, r) | (t1 << (8 * r));
                                }
                            }
                            uint32_t* const sb = sbuf[ph & 1];
                            if (lane < w0) sb[lane] = lane == 0 ? c0 : lane == 1 ? c1 : lane == 2 ? c2 : c3;  // (w0 < 5)
                            if (bi < T) sb[w0 + lane] = word;
                            const uint32_t nout = T >> 2;
                            const uint32_t accn = LaneStream::low_bytes(__builtin_amdgcn_readlane(word, (int)nout), T & 3u);
                            if (active) {
                                ls.wpos = w0 + nout;
                                ls.nb = T & 3u;
                                ls.acc = accn;
                            }
                            dg_t2 = diag_clock();
                        }
                    }
                    if (lane == 0) uni_sh[ph & 1] = uni ? 1u : 0u;
#if RP_DIAG
                    if (lane == 0 && uni) stat_add(S, STAT_DIAG0 + 5, 1ull);  // (RP_DIAG builds: shared phases)
#endif
                    if (!uni) {
                    // the < 5 words the last drain left, to the front
                    cur[0] = lq0; cur[1] = lq1; cur[2] = lq2; cur[3] = lq3; cur[4] = lq4;
                    ls.buf = cur;
#pragma unroll
                    for (uint32_t k = 0; k < CKP_GRP; k++) {
                        const uint32_t a = ph * CKP_GRP + k;
                        if (a >= n) break;  // (uniform)
                        const uint32_t j = a & 63u;
                        const bool present = run && pbl && v_status(vs[k]) != ST_ABSENT;
                        const bool lead = present && first;
                        first = first && !present;
                        const uint32_t cvl = __builtin_amdgcn_readlane((uint32_t)cvs, (int)j);
                        const uint32_t cvh = __builtin_amdgcn_readlane((uint32_t)(cvs >> 32), (int)j);
                        const uint64_t cv = ((uint64_t)cvh << 32) | cvl;
                        if (__ballot(present && (vs[k] != cv || lead)) == 0) {  // (uniform)
                            const uint32_t K = __builtin_amdgcn_readlane(clen, (int)j);
                            if (K) {
                                uint32_t tw[CKL_TEXT];
                                const uint4* tp = (const uint4*)text[j];
#pragma unroll
                                for (uint32_t q = 0; q < CKL_TEXT / 4; q++) {
                                    const uint4 x = tp[q];
                                    tw[4 * q] = x.x; tw[4 * q + 1] = x.y; tw[4 * q + 2] = x.z; tw[4 * q + 3] = x.w;
                                }
                                ls.uniform_piece_flat<CKL_TEXT - 2>(tw, K, present);
                            }
                        } else {
                            ls.byte(0x3Bu, present && !lead);  // ';' between members
                            // the address: scalar loads (not behind the cells in flight)
                            const uint32_t L = (kload((const uint32_t*)at.len + (a >> 2)) >> (8 * (a & 3u))) & 0xFFu;
                            const uint32_t* aw = at.words + (size_t)a * ADDR_WORDS;
                            uint32_t w[ADDR_WORDS];
#pragma unroll
                            for (uint32_t q = 0; q < ADDR_WORDS; q++) w[q] = kload(aw + q);
                            ls.uniform_piece(w, L, (L + 3) >> 2, present);
                            lane_status_inc(ls, vs[k], present);
                        }
                    }
                    }
                    // the complete blocks of this phase go to the hash wave
                    const uint32_t nbk = run ? min(ls.wpos / 5u, pbl) : 0u;
                    nbk_sh[ph & 1][lane] = nbk;
                    pbl -= nbk;
                    ls.wpos -= 5 * nbk;
                    bool same = false;  // (a shared phase whose active lanes drained alike)
                    if (!uni) {
                        const uint32_t* q = cur + 5 * nbk;
                        lq0 = q[0]; lq1 = q[1]; lq2 = q[2]; lq3 = q[3]; lq4 = q[4];
                    } else {
                        // the words after the drained blocks: stream words of lanes
                        // 5 nbk - w0 ... when every active lane drained the same
                        // blocks (one or more), else (an inactive lane of a shared
                        // phase keeps its words) from sbuf
                        const uint32_t nbu = __builtin_amdgcn_readlane(nbk, (int)__builtin_ctzll(am));
                        if (nbu != 0 && __ballot(active && nbk != nbu) == 0) {
                            const int p = (int)(5 * nbu - w0);
                            const uint32_t x0 = __builtin_amdgcn_readlane(word, p), x1 = __builtin_amdgcn_readlane(word, p + 1);
                            const uint32_t x2 = __builtin_amdgcn_readlane(word, p + 2), x3 = __builtin_amdgcn_readlane(word, p + 3);
                            const uint32_t x4 = __builtin_amdgcn_readlane(word, p + 4);
                            if (active) { lq0 = x0; lq1 = x1; lq2 = x2; lq3 = x3; lq4 = x4; }
                            same = true;
                        } else {
                            wave_lds_sync();
                            if (active) {
                                const uint32_t* q = sbuf[ph & 1] + 5 * nbk;
                                lq0 = q[0]; lq1 = q[1]; lq2 = q[2]; lq3 = q[3]; lq4 = q[4];
                            }
                        }
                    }
                    prev_uni = same;
                    prev_am = am;

                }
                if (!render && ph + 1 < NP) {  // the next phase's cells to LDS, then the set reloaded
#pragma unroll
                    for (uint32_t k = 0; k < CKP_GRP; k++) vs_sh[(ph + 1) & 1][k][lane] = vsx[k];
#pragma unroll
                    for (uint32_t k = 0; k < CKP_GRP; k++) vsx[k] = row[min((ph + 3) * CKP_GRP + k, n - 1)].vs;
                }
                if (!render && ph > 0) {
                    const uint32_t* const b = uni_sh[(ph - 1) & 1] ? sbuf[(ph - 1) & 1] : bufs[(ph - 1) & 1] + lane * CKP_STRIDE;
                    const uint32_t nbk = nbk_sh[(ph - 1) & 1][lane];
                    uint32_t q0 = b[0], q1 = b[1], q2 = b[2], q3 = b[3], q4 = b[4];
                    for (uint32_t jb = 0; __ballot(jb < nbk) != 0; jb++) {
                        const uint32_t* q = b + 5 * (jb + 1);
                        const uint32_t r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4];
                        if (jb < nbk) {
                            fh_stream_block(st, q0, q1, q2, q3, q4);
                            q0 = r0; q1 = r1; q2 = r2; q3 = r3; q4 = r4;
                        }
                    }
                    st.blocks_left -= nbk;
                }
                const uint64_t dg_1 = diag_clock();
                __syncthreads();
                dg_work += dg_1 - dg_0;
                dg_wait += diag_clock() - dg_1;
                if (render && ph < NP && uni_sh[ph & 1]) { dg_s1 += dg_t1 - dg_0; dg_s2 += dg_t2 - dg_t1; dg_s3 += dg_1 - dg_t2; }
            };
            for (uint32_t ph = 0; ph <= NP; ph += 2) {
                phase(ph, vs_b);  // (phase p stores the cells of p + 1: set B holds odd phases', A even ones')
                if (ph + 1 <= NP) phase(ph + 1, vs_a);  // (uniform)
            }
#if RP_DIAG
            if (lane == 0) {
#if RP_DIAG_CKSPLIT
                if (render) {
                    stat_add(S, STAT_DIAG0, dg_work);
                    stat_add(S, STAT_DIAG0 + 1, dg_s1); stat_add(S, STAT_DIAG0 + 2, dg_s2); stat_add(S, STAT_DIAG0 + 3, dg_s3);
                }
#else
                stat_add(S, STAT_DIAG0 + (render ? 0 : 2), dg_work);
                stat_add(S, STAT_DIAG0 + (render ? 1 : 3), dg_wait);
#endif
                if (render) stat_add(S, STAT_DIAG0 + 4, (unsigned long long)n);
            }
#endif
            (void)dg_work; (void)dg_wait; (void)dg_s1; (void)dg_s2; (void)dg_s3;
            if (!render && run) res = fh_stream_end(st);
        }
        if (!render && act) {
            S.csum[v] = res;
            S.csum_valid[v] = 1;
            out[v] = res;
            stat_add(S, STAT_CK_VIEWS, 1ull);
        }
        __syncthreads();  // (the next group's canonical texts and buffers)
    }
}

// Views with equal content fingerprints have equal checksums (DESIGN.md §3
// fact 2), so a list of views to checksum is reduced to one leader per
// distinct fingerprint: an open-addressing table of fingerprints (claimed by
// atomicCAS), the winners listed for k_checksums, the rest copy their
// leader's value in k_ck_store_follow.  Converging clusters (config 5's late
// rounds) have few distinct views.
constexpr unsigned long long FP_EMPTY = ~0ull;
// Checksums computed in earlier rounds, by view fingerprint (the same 2^-64
// assumption as the per-call dedupe): a direct-mapped cache of {fingerprint,
// check word | checksum}.  Entries are written without locks; the check word
// (a mix of both halves) rejects an entry torn between two writers.
struct CkEntry { unsigned long long key, val; };
__device__ inline uint32_t ck_slot(unsigned long long f, uint32_t mask) {
    return (uint32_t)((f * 0x9E3779B97F4A7C15ull) >> 32) & mask;
}
__device__ inline unsigned long long ck_pack(unsigned long long f, uint32_t cs) {
    const uint32_t chk = (uint32_t)(f ^ (f >> 32)) ^ (cs * 0x9E3779B1u);
    return ((unsigned long long)chk << 32) | cs;
}
__device__ inline bool ck_lookup(const CkEntry* cache, uint32_t mask, unsigned long long f, uint32_t& cs) {
    const CkEntry e = cache[ck_slot(f, mask)];
    if (e.key != f) return false;
    cs = (uint32_t)e.val;
    return e.val == ck_pack(f, cs);
}
// snap_out (the side-stream path, k_ck_snapcopy): entries resolved here get
// their value in snap_out at once; every other entry, its leader included,
// gets its fingerprint slot in slot_of and hlead[slot] = the leader's index
__global__ void k_ck_dedupe(SimDev S, const uint32_t* list, const uint32_t* count, unsigned long long* hkey,
                            uint32_t* hval, uint32_t hmask, uint32_t* leaders, uint32_t* nleaders, uint32_t* slot_of,
                            const CkEntry* cache, uint32_t cmask, uint32_t* snap_out = nullptr,
                            uint32_t* hlead = nullptr) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *count) return;
    const uint32_t v = list[i];
    slot_of[i] = NONE;
    if (S.csum_valid[v]) {
        if (snap_out) snap_out[v] = S.csum[v];
        return;
    }
    {
        uint32_t cs;
        if (ck_lookup(cache, cmask, S.fp[v], cs)) {  // computed in an earlier round
            S.csum[v] = cs;
            S.csum_valid[v] = 1;
            if (snap_out) snap_out[v] = cs;
            return;
        }
    }
    unsigned long long f = S.fp[v];
    if (f == FP_EMPTY) f = FP_EMPTY - 1;  // (the empty marker; any stand-in works, fingerprints only select leaders)
    for (uint32_t h = (uint32_t)(f ^ (f >> 32)) & hmask;; h = (h + 1) & hmask) {
        const unsigned long long old = atomicCAS(&hkey[h], FP_EMPTY, f);
        if (old == FP_EMPTY) {  // leader
            hval[h] = v;
            const uint32_t li = atomicAdd(nleaders, 1u);
            leaders[li] = v;
            if (hlead) { hlead[h] = li; slot_of[i] = h; }
            return;
        }
        if (old == f) { slot_of[i] = h; return; }
    }
}

// after k_checksums: the leaders' checksums into the cache, and every
// follower's from its leader (independent halves: the followers read the
// leaders' checksums, which neither half writes)
__global__ void k_ck_store_follow(SimDev S, const uint32_t* leaders, const uint32_t* nleaders, CkEntry* cache,
                                  uint32_t mask, const uint32_t* list, const uint32_t* count, const uint32_t* hval,
                                  const uint32_t* slot_of, uint32_t* out, uint32_t run_min = 0) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nl = *nleaders;
    if (nl < run_min) return;
    if (i < nl) {
        const uint32_t v = leaders[i];
        const unsigned long long f = S.fp[v];
        CkEntry e;
        e.key = f; e.val = ck_pack(f, S.csum[v]);
        cache[ck_slot(f, mask)] = e;
    }
    if (i >= *count) return;
    const uint32_t v = list[i], h = slot_of[i];
    if (h != NONE) {
        const uint32_t c = S.csum[hval[h]];
        S.csum[v] = c;
        S.csum_valid[v] = 1;
    }
    out[v] = S.csum[v];
}

// The round's sender checksums beside the ping merge (one shard): the
// checksum stage is a few hundred farmhash chains of ~115 k dependent steps
// (config 5: ~1.6 ms per stage whatever runs it, on a handful of waves), and
// nothing before the fullSync decisions (k_pending) reads the values.  So the
// main stream copies each leader's view (k_ck_snapcopy: its values, n x 8 B,
// and its fingerprint) before the merges change it, and a side stream hashes
// the copies (k_checksums_snap) and hands the results out (k_ck_finish_snap)
// while the ping merge runs.  Nothing on the side stream writes a node's
// csum / csum_valid (the merges clear those concurrently); results go to
// snd_csum and to the fingerprint-keyed cache, which is content-addressed.
// When the leaders outnumber the snapshot rows, the live path runs instead
// (k_checksums / k_ck_store_follow with run_min = cap + 1) before the
// merges.  Leader i's result goes to hres[slot of its fingerprint].
__global__ void __launch_bounds__(256) k_ck_snapcopy(SimDev S, const uint32_t* leaders, const uint32_t* nleaders,
                                                      uint64_t* rows, unsigned long long* lfp, uint32_t cap) {
    const uint32_t nl = *nleaders;
    if (nl > cap) return;  // (the live path)
    for (uint32_t i = blockIdx.x; i < nl; i += gridDim.x) {
        const uint32_t v = leaders[i];
        const VEnt* src = S.view + S.row(v);
        uint64_t* dst = rows + (size_t)i * S.n;
        for (uint32_t a = threadIdx.x; a < S.n; a += blockDim.x) dst[a] = src[a].vs;
        if (threadIdx.x == 0) lfp[i] = S.fp[v];
    }
}
__global__ void __launch_bounds__(BLOCK) k_checksums_snap(SimDev S, const uint64_t* rows, const uint32_t* nleaders,
                                                          uint32_t cap, uint32_t* lres) {
    __shared__ __attribute__((aligned(16))) uint8_t bufs[NWAVE][CKW_BUF];
    const uint32_t cnt = *nleaders;
    if (cnt > cap) return;
    const AddrTable at{S.addr_words, S.addr_len};
    for (uint32_t i = blockIdx.x * NWAVE + wave_id(); i < cnt; i += gridDim.x * NWAVE) {
        const uint64_t* row = rows + (size_t)i * S.n;
        const uint32_t c = wave_view_checksum([&](uint32_t a) { return row[a]; }, S.n, at, bufs[wave_id()]);
        if (lane_id() == 0) {
            lres[i] = c;
            stat_add(S, STAT_CK_VIEWS, 1ull);
        }
    }
}
// every entry of the list: its checksum from its leader (hval: the leader's
// node id by fingerprint slot; the leader's index from lslot), the cache
// entries of the leaders
__global__ void k_ck_finish_snap(SimDev S, const uint32_t* list, const uint32_t* count, const uint32_t* nleaders,
                                 uint32_t cap, const uint32_t* slot_of, const uint32_t* hlead, const uint32_t* lres,
                                 const unsigned long long* lfp, CkEntry* cache, uint32_t cmask, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nl = *nleaders;
    if (nl > cap) return;
    if (i < nl) {
        CkEntry e;
        e.key = lfp[i]; e.val = ck_pack(lfp[i], lres[i]);
        cache[ck_slot(lfp[i], cmask)] = e;
    }
    if (i >= *count) return;
    const uint32_t h = slot_of[i];
    if (h != NONE) out[list[i]] = lres[hlead[h]];  // (entries resolved by the dedupe have their value already)
}


// Dissemination.issueAsReceiver for `requester` (filter = its source and
// incarnation) and the response record: a list, an empty list, or a pending
// fullSync decision (view snapshot; k_pending compares real checksums).
// sv: the same-view decision when the caller has it (k_p2_pre), else SV_NONE.
// A ping's response (slot = the sender A, req_csum = snd_csum[A]): a pending
// fullSync decision names the slot with PEND_SND, and k_pending compares with
// snd_csum[A] itself -- the round's sender checksums may still be in flight on
// the side stream while the ping merge runs (k_checksums_snap).
constexpr uint32_t PEND_SND = 0x80000000u;
template <bool ESC = false, bool SET = true, bool SPF = false, bool FAST = false>
__device__ void respond_as_receiver(const SimDev& S, uint32_t b, uint32_t requester, uint64_t req_inc,
                                    uint64_t req_fp, uint32_t req_csum, bool csum_known, uint32_t slot,
                                    uint32_t ping_status, Shared& sh, uint64_t sv = SV_NONE,
                                    bool csum_of_sender = false) {
    const uint32_t n = S.n;
    uint64_t off;
    uint32_t pm, pe;
    // (the seen filter: the requester's own bitset on this shard, else the cluster-wide mask)
    // (req_fp: the requester's fingerprint when it sent the ping)
    uint32_t m = wg_issue<ESC, RP_ISSUE_UNR, SET, SPF, FAST>(S, b, true, requester, req_inc, &off, 2, sh,
                               S.local(requester) ? requester : (requester | DEST_REMOTE), &pm, &pe, req_fp, sv);
    if (threadIdx.x == 0) {
        Resp r;
        r.kind = RESP_LIST; r.from = b; r.off = off; r.len = m; r.snap = NONE; r.ping_status = ping_status;
        r.plen = pm;
        r.nesc = pe;
        r.eoff = 0;
        if (m == 0) {
            if (S.fp[b] == req_fp) {
                r.kind = RESP_EMPTY;  // identical views: identical checksums
            } else if (!csum_known) {
                atomicOr(S.err, SIMERR_PREDICATE);
                r.kind = RESP_EMPTY;
            } else {
                uint32_t k = atomicAdd(S.snap_count, 1u);
                if (k >= S.snap_cap) { atomicOr(S.err, SIMERR_SNAP_FULL); r.kind = RESP_EMPTY; }
                else {
                    r.kind = RESP_FS_PENDING; r.snap = k;
                    S.pend_slot[k] = csum_of_sender ? (slot | PEND_SND) : slot;
                    S.pend_csum[k] = req_csum;
                }
            }
        }
        S.resp[slot] = r;
        sh.u[7] = r.kind == RESP_FS_PENDING ? r.snap : NONE;
        stat_add(S, STAT_MESSAGES, 1ull);
    }
    lds_barrier();
    if (sh.u[7] != NONE) {  // snapshot the view for a possible fullSync() (read in later kernels)
        uint64_t* dst = S.snaps + (size_t)sh.u[7] * n;
        const VEnt* srow = S.view + S.row(b);
        for (uint32_t a = threadIdx.x; a < n; a += BLOCK) dst[a] = srow[a].vs;
        // ... with the member order it lists them in (later batches may splice)
        const uint32_t M = S.mcount[b];
        uint32_t* dord = S.snap_ord + (size_t)sh.u[7] * n;
        const uint32_t* sord = S.order + S.row(b);
        for (uint32_t i = threadIdx.x; i < M; i += BLOCK) dord[i] = sord[i];
        if (threadIdx.x == 0) S.snap_m[sh.u[7]] = M;
    }
    lds_barrier();
}

// Apply a response record to node x (lib/swim/ping-sender.js:36-39 etc.):
// `weight` = how many times the reference calls update() with it.
// A response from another shard (RESP_LIST_RX): with XS merged straight from
// its wire words (rx2w, rx2e); without, from its decoded copy in rxc (k_w5,
// whose registers do not fit a third merge loop; k_xs_unpack<5> decodes).
template <bool JOIN = true, bool PRE = false, bool XS = true>
__device__ void apply_response(const SimDev& S, uint32_t x, const Resp& r, uint64_t now, uint32_t weight,
                               int phase, Shared& sh, const ApplyPro* pre = nullptr) {
    const uint32_t n = S.n;
    if (r.kind == RESP_LIST || (!XS && r.kind == RESP_LIST_RX)) {
        const Change* msg = (r.kind == RESP_LIST ? S.arena : S.rxc) + r.off;
        auto src = [&](uint32_t i) { return load_msg(msg + i); };
        wg_apply<JOIN, PRE>(S, x, src, r.plen, r.len, now, weight, phase, sh, pre);
    } else if (XS && r.kind == RESP_LIST_RX) {
        const uint32_t* w = S.rx2w + r.off;
        const Esc* e = S.rx2e + r.eoff;
        auto src = [&](uint32_t i) { return wire_change(S, w[i], e); };
        wg_apply<JOIN, PRE>(S, x, src, r.plen, r.len, now, weight, phase, sh, pre);
    } else if (r.kind == RESP_FS) {
        const uint32_t B = r.from;
        const uint32_t* ord = S.snap_ord + (size_t)r.snap * n;
        const uint64_t* snap = S.snaps + (size_t)r.snap * n;
        const uint32_t M = S.snap_m[r.snap];
        auto src = [&](uint32_t i) {
            Change c;
            c.addr = ord[i];
            c.origin = B;  // fullSync origin: source = B, no sourceIncarnationNumber
            c.vs = snap[c.addr];
            return c;
        };
        wg_apply<JOIN, PRE>(S, x, src, M, M, now, weight, phase, sh, pre);
    }
}

// W1: receivers handle pings in sender-id order (server/ping-handler.js:22-40).
// JOIN: a cluster whose views may lack members (rp_sim_join); the full-view
// instantiations keep the hot path free of the splice code.
// The first P2_SPLIT pings of every receiver run as separate merge and respond
// launches (k_p2_apply / k_p2_respond, one pair per ping rank): each half
// alone fits its registers at 7 waves per SIMD without scratch, where the
// fused loop spills.  k_phase2 then handles the remaining pings of receivers
// with more (from rank P2_SPLIT on), in order.  Receivers are independent
// within the wave (another receiver's seen bitset is only read, and a stale
// read only lets a provable no-op through), so the per-receiver order is all
// that matters.  Each launch walks a list of the receivers it has work for
// (k_p2_lists), one block per entry (a grid of its bound, p2_grid).
#ifndef RP_P2_SPLIT
#define RP_P2_SPLIT 2
#endif
constexpr uint32_t P2_SPLIT = RP_P2_SPLIT;
constexpr uint32_t P2_DEAD = 0x80000000u;  // k_p2_lists: the receiver is down (node ids < 2^31)
// Launch grid for the receivers with more than k pings: a wave carries at most
// one ping per node of the cluster (n), so at most n / (k + 1) of a shard's nl
// receivers have more than k
__host__ __device__ inline uint32_t p2_grid(uint32_t nl, uint32_t n, uint32_t k) {
    const uint32_t b = n / (k + 1);
    return b < nl ? (b ? b : 1u) : nl;
}
// lists[k * nl ..]: local receivers with more than k pings (k < P2_SPLIT);
// lists[P2_SPLIT * nl ..]: those with more than P2_SPLIT; lens[k] their counts.
// lists[(P2_SPLIT + 1 + k) * nl ..] (k < P2_SPLIT): the sender of each entry's
// k-th ping, so that k_p2_apply / k_p2_respond have both ids after one read
// (not list -> g_base -> g_list, two more dependent round trips per block),
// with P2_DEAD set when the receiver is down (S.dead is fixed within a round)
// msgs[(k * nl + e) * 2 ..] (k < P2_SPLIT): that ping's body for k_p2_apply --
// its offset in the arena, or P2_RX | its offset in rxc (a sender on another
// shard), then plen | len << 32 -- read with the entry instead of after it
constexpr uint64_t P2_RX = 1ull << 63;
__global__ void __launch_bounds__(256) k_p2_lists(SimDev S, uint32_t* lists, uint32_t* lens, uint64_t* msgs) {
    __shared__ uint32_t wbase[P2_SPLIT + 1][4], bbase[P2_SPLIT + 1];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = S.lo + i;
    const uint32_t c = i < S.nl ? S.g_base[b + 1] - S.g_base[b] : 0u;
    const uint64_t below = (1ull << lane_id()) - 1ull;
    const int w = threadIdx.x >> 6;
    uint64_t m[P2_SPLIT + 1];
    // one atomic per block and list: wave counts -> block offsets in LDS
#pragma unroll
    for (uint32_t k = 0; k <= P2_SPLIT; k++) {
        m[k] = __ballot(c > k);
        if (lane_id() == 0) wbase[k][w] = (uint32_t)__popcll(m[k]);
    }
    __syncthreads();
    if (threadIdx.x <= P2_SPLIT) {
        const uint32_t k = threadIdx.x;
        uint32_t t = 0;
        for (int q = 0; q < 4; q++) { const uint32_t x = wbase[k][q]; wbase[k][q] = t; t += x; }
        bbase[k] = t ? atomicAdd(&lens[k], t) : 0u;
        if (bbase[k] + t > p2_grid(S.nl, S.n, k)) atomicOr(S.err, SIMERR_P2_LIST);  // (cannot happen)
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k <= P2_SPLIT; k++) {
        if (c > k) {
            const uint32_t e = bbase[k] + wbase[k][w] + (uint32_t)__popcll(m[k] & below);
            lists[(size_t)k * S.nl + e] = b;
            if (k < P2_SPLIT) {
                const uint32_t A = S.g_list[S.g_base[b] + k];
                lists[(size_t)(P2_SPLIT + 1 + k) * S.nl + e] = A | (S.dead[b] ? P2_DEAD : 0u);
                uint64_t* mp = msgs + ((size_t)k * S.nl + e) * 2;
                mp[0] = S.local(A) ? S.msg_off[A] : (S.rx_off[A] | P2_RX);
                mp[1] = S.msg_plen[A] | ((uint64_t)S.msg_len[A] << 32);
            }
        }
    }
}
template <bool JOIN>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(RP_P3_WAVES, 8)))
k_p2_apply(SimDev S, uint64_t now, uint32_t k, const uint32_t* list, const uint32_t* len, const uint64_t* msgs) {
    RP_MERGE_SHARED(JOIN);
    // (uniform values: kept in SGPRs; the entry is read with its count -- the
    // grid never exceeds the list's allocation -- in one round trip)
    const uint32_t b = __builtin_amdgcn_readfirstlane(list[blockIdx.x]);
    const uint32_t Ad = __builtin_amdgcn_readfirstlane(list[(size_t)(P2_SPLIT + 1) * S.nl + blockIdx.x]);  // (k_p2_lists)
    const uint64_t mo = msgs[2 * blockIdx.x], ml = msgs[2 * blockIdx.x + 1];  // (k_p2_lists)
    if (blockIdx.x >= *len) return;
    if (k == 0 && threadIdx.x == 0) note_wave(S, 1);
    const uint32_t A = Ad & ~P2_DEAD;
    if ((Ad & P2_DEAD) || cut(S, A, b)) return;  // unreachable (k_p2_respond records the transport error)
    // (a sender on another shard: its body decoded into rxc by k_expand_pings;
    // merged from the wire words instead it measured slower)
    const Change* msg = (mo & P2_RX) ? S.rxc + (mo & ~P2_RX) : S.arena + mo;
    auto src = [&](uint32_t e) { return load_msg(msg + e); };
    wg_apply<JOIN>(S, b, src, (uint32_t)ml, (uint32_t)(ml >> 32), now, 1, 2, sh);  // server/ping-handler.js:34
}
// What k_p2_respond's block for list entry e needs before its issue, packed
// by k_p2_pre (one thread per entry, after k_p2_apply of the same rank) into
// one 32-byte record: the receiver b and requester A (P2_DEAD: down or cut
// off), the same-view decision against A's fingerprint at its ping
// (same_view_word: a chain of three dependent loads, taken here rather than
// by the block's thread 0), and A's ping metadata.
// (the requester's need_csum rides in Ad: P2_NEED; a ping's pending fullSync
// decision compares with snd_csum[A] in k_pending, PEND_SND)
constexpr uint32_t P2_NEED = 0x40000000u;
struct alignas(16) P2Rec {  // (k_p2_respond reads it as 8 words: keep the layout)
    uint32_t b, Ad;
    uint64_t sv;
    uint64_t req_inc, req_fp;
};
static_assert(sizeof(P2Rec) == 32 && offsetof(P2Rec, sv) == 8 && offsetof(P2Rec, req_fp) == 24,
              "k_p2_pre record: 32 bytes, read as words by k_p2_respond");
__global__ void __launch_bounds__(256) k_p2_pre(SimDev S, const uint32_t* list, const uint32_t* len, P2Rec* rec) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t cnt = *len;
    bool hit = false;
    P2Rec r{};
    const bool mine = e < cnt;
    if (mine) {
        r.b = list[e];
        r.Ad = list[(size_t)(P2_SPLIT + 1) * S.nl + e];  // (k_p2_lists)
        const uint32_t A = r.Ad & ~P2_DEAD;
        if (!(r.Ad & P2_DEAD) && cut(S, A, r.b)) r.Ad |= P2_DEAD;
        if (!(r.Ad & P2_DEAD)) {
            r.req_inc = S.snd_inc[A];
            r.req_fp = S.snd_fp[A];
            if (S.need_csum[A]) r.Ad |= P2_NEED;
            r.sv = same_view_word(S, r.b, A, r.req_fp, &hit);
        }
    }
    if (mine) {
        const uint4* src = (const uint4*)&r;
        uint4* dst = (uint4*)(rec + e);
#pragma unroll
        for (int i = 0; i < 2; i++) dst[i] = src[i];
    }
    const uint64_t hits = __ballot(hit);
    if (lane_id() == 0 && hits) stat_add(S, STAT_SAME_VIEW, (unsigned long long)__popcll(hits));
}
template <bool ESC, bool SET>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(RP_P1_WAVES, 8)))
k_p2_respond(SimDev S, uint32_t k, const P2Rec* rec, const uint32_t* len) {
    __shared__ Shared sh;
    // (uniform values: the record in SGPRs, read with the count)
    uint32_t w[8];
    sload_words(rec + blockIdx.x, w);
    const uint32_t b = w[0], Ad = w[1];
    const uint64_t sv = ((uint64_t)w[3] << 32) | w[2];
    const uint64_t req_inc = ((uint64_t)w[5] << 32) | w[4], req_fp = ((uint64_t)w[7] << 32) | w[6];
    if (blockIdx.x >= *len) return;
    (void)k;
    const uint32_t A = Ad & ~(P2_DEAD | P2_NEED);
    const bool need = (Ad & P2_NEED) != 0;
    if (Ad & P2_DEAD) {  // down or cut off: transport error one wave later
        if (threadIdx.x == 0) {
            Resp rr{};
            rr.kind = RESP_ERR; rr.from = b; rr.snap = NONE;
            S.resp[A] = rr;
            stat_add(S, STAT_MESSAGES, 1ull);
        }
        return;
    }
    respond_as_receiver<ESC, SET, SET && RP_SETTLED_PF, true>(S, b, A, req_inc, req_fp, 0u, need, A, 0, sh, sv, true);
}

template <bool ESC, bool JOIN, bool SET>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(RP_P2_WAVES, 8))) k_phase2(SimDev S, uint64_t now, const uint32_t* list, const uint32_t* len) {
    __shared__ Shared sh;
    if (blockIdx.x >= *len) return;
    {
        const uint32_t b = __builtin_amdgcn_readfirstlane(list[blockIdx.x]);
        const uint32_t lo = S.g_base[b], hi = S.g_base[b + 1];
        const bool down = S.dead[b] != 0;  // (fixed within the round: read once)
        // the next sender is read while the current ping is merged and answered
        uint32_t An = lo + P2_SPLIT < hi ? S.g_list[lo + P2_SPLIT] : 0u;
        for (uint32_t j = lo + P2_SPLIT; j < hi; j++) {
            const uint32_t A = __builtin_amdgcn_readfirstlane(An);
            if (j + 1 < hi) An = S.g_list[j + 1];
            if (down || cut(S, A, b)) {  // unreachable: transport error one wave later
                if (threadIdx.x == 0) {
                    Resp r{};
                    r.kind = RESP_ERR; r.from = b; r.snap = NONE;
                    S.resp[A] = r;
                    stat_add(S, STAT_MESSAGES, 1ull);
                }
                __syncthreads();
                continue;
            }
            const uint64_t d0 = diag_clock();
            // ping bodies of senders on other shards: decoded into rxc (k_expand_pings)
            const Change* msg = S.local(A) ? S.arena + S.msg_off[A] : S.rxc + S.rx_off[A];
            auto src = [&](uint32_t e) { return load_msg(msg + e); };
            wg_apply<JOIN>(S, b, src, S.msg_plen[A], S.msg_len[A], now, 1, 2, sh);  // :34
            const uint64_t d1 = diag_clock();
            respond_as_receiver<ESC, SET, SET && RP_SETTLED_PF>(S, b, A, S.snd_inc[A], S.snd_fp[A], 0u, S.need_csum[A] != 0, A, 0, sh, SV_NONE,
                                          true);
            if (!RP_DIAG_FINE && RP_DIAG_PHASE == 2) { DIAG_ADD(S, 3, d1 - d0); DIAG_ADD(S, 5, diag_clock() - d1); }
        }
    }
}

// Resolve pending fullSync decisions with real farmhash values.
__device__ inline void pending_verdict(const SimDev& S, uint32_t k, uint32_t cs) {
    S.pend_done[k] = 1;
    const uint32_t ps = S.pend_slot[k], slot = ps & ~PEND_SND;
    if (cs != ((ps & PEND_SND) ? S.snd_csum[slot] : S.pend_csum[k])) {
        S.resp[slot].kind = RESP_FS;  // Dissemination.fullSync (lib/dissemination.js:61-76)
        atomicAdd(&S.stats[STAT_FULLSYNC], 1ull);  // one per snapshot: rare
    } else {
        S.resp[slot].kind = RESP_EMPTY;
    }
}
__global__ void __launch_bounds__(BLOCK) k_pending(SimDev S) {
    __shared__ __attribute__((aligned(16))) uint8_t bufs[NWAVE][CKW_BUF];
    const uint32_t cnt = min(*S.snap_count, S.snap_cap);
    const AddrTable at{S.addr_words, S.addr_len};
    for (uint32_t k = blockIdx.x * NWAVE + wave_id(); k < cnt; k += gridDim.x * NWAVE) {  // one wave per snapshot
        if (S.pend_done[k]) continue;
        const uint64_t* row = S.snaps + (size_t)k * S.n;
        const uint32_t cs = wave_view_checksum([&](uint32_t a) { return row[a]; }, S.n, at, bufs[wave_id()]);
        if (lane_id() == 0) pending_verdict(S, k, cs);
    }
}

// The members at positions pos[0 .. np) (np <= 8) of x's list of pingable
// members other than x and `excl`, in member order -> out[] (LDS, valid after
// the call).  One pass: each wave counts a contiguous quarter of the list per
// 64 members (ballots, counts kept in LDS); then each position is located from
// the counts and resolved by reloading its 64 members.
constexpr uint32_t SEL_MAX = 8;
__device__ void select_pingable_at(const SimDev& S, uint32_t x, uint32_t excl, const uint32_t* pos, uint32_t np,
                                   uint32_t* out, Shared& sh) {
    const uint32_t n = S.mcount[x];  // the member list's length
    const uint32_t* ord = S.order + S.row(x);
    const uint32_t* pb = ping_bits(S, x);
    const int lane = lane_id(), wv = wave_id();
    const uint32_t nch = (n + 63) / 64, cpw = (nch + NWAVE - 1) / NWAVE;  // 64-member chunks, per wave
    const uint32_t c_lo = min(nch, wv * cpw), c_hi = min(nch, c_lo + cpw);
    uint32_t* ccount = sh.ring;  // nch <= 1024 chunk counts
    auto flag_of = [&](uint32_t i, uint32_t& a) {
        a = i < n ? ord[i] : NONE;
        return a != NONE && a != x && a != excl && ping_bit(pb, a);
    };
    uint32_t run = 0;
    constexpr int U = 4;
    for (uint32_t c0 = c_lo; c0 < c_hi; c0 += U) {
        uint32_t am[U];
#pragma unroll
        for (int u = 0; u < U; u++) am[u] = c0 + u < c_hi && (c0 + u) * 64 + lane < n ? ord[(c0 + u) * 64 + lane] : NONE;
        bool pg[U];
#pragma unroll
        for (int u = 0; u < U; u++) pg[u] = am[u] != NONE && ping_bit(pb, am[u]);
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (c0 + u >= c_hi) break;  // wave-uniform
            const bool f = pg[u] && am[u] != x && am[u] != excl;
            const uint32_t c = (uint32_t)__popcll(__ballot(f));
            if (lane == 0) ccount[c0 + u] = c;
            run += c;
        }
    }
    if (lane == 0) sh.wc[0][0][wv] = run;
    lds_barrier();
    // position j -> wave j % NWAVE: find its chunk, reload it, pick the member
    for (uint32_t j = wv; j < np; j += NWAVE) {
        uint32_t p = pos[j], c = 0;
        for (int w = 0; w < NWAVE; w++) {
            const uint32_t t = sh.wc[0][0][w];
            if (p < t) { c = min(nch, w * cpw); break; }
            p -= t;
        }
        while (c < nch && p >= ccount[c]) { p -= ccount[c]; c++; }  // wave-uniform LDS walk
        uint32_t a;
        const bool f = c < nch && flag_of(c * 64 + lane, a);
        const uint64_t m = __ballot(f);
        const uint64_t below = (1ull << lane) - 1ull;
        if (f && (uint32_t)__popcll(m & below) == p) out[j] = a;
    }
    lds_barrier();
}

// W2: senders handle their ping response.  Success: Membership.update twice
// (the second call is a no-op, counted); failure: ping-req fan-out
// (lib/swim/ping-req-sender.js:153-199): up to 3 random pingable members
// (lib/membership.js:111-120, underscore 1.13 sample), one issueAsSender each.
// W2, answered pings: the sender merges the response.
// pass 0: every sender; with the fullSync decisions on the side stream
// (k_pending beside this kernel), pass 1 takes the responses without a
// pending snapshot and pass 2, after k_pending, those with one (r.snap is
// set when the response is made and k_pending leaves it alone).
template <bool JOIN, bool XS>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(RP_P3_WAVES, 8))) k_phase3(SimDev S, uint64_t now,
                                                                                                    int pass) {
    RP_MERGE_SHARED(JOIN);
    const uint32_t A = S.lo + blockIdx.x;
    // the response record, the target, A's seen bitset (staged in LDS) and
    // A's node scalars: one round trip (the merge's prologue then waits for
    // nothing but its first chunk of changes)
    const int32_t T = S.target[A];
    const Resp r = S.resp[A];
    if (pass == 2 && (T < 0 || r.snap == NONE)) return;  // (before staging: most blocks of pass 2 end here)
    stage_seen(sh.seen, S.seen + S.srow(A), S.seen_words);
    ApplyPro pro;
    if (threadIdx.x == 0) pro = load_apply_pro(S, A, JOIN);
    if (T < 0 || (pass == 1 && r.snap != NONE)) return;
    if (threadIdx.x == 0) note_wave(S, 2);
    if (r.kind != RESP_ERR) apply_response<JOIN, true, XS>(S, A, r, now, 2, 3, sh, &pro);
}

// W2, failed pings (fault runs only): the sender starts the ping-req fan-out.
template <bool ESC>
__global__ void __launch_bounds__(BLOCK) k_phase3_err(SimDev S, uint64_t now, int list_all) {
    __shared__ Shared sh;
    const uint32_t A = S.lo + blockIdx.x, n = S.n;
    if (S.target[A] < 0) return;
    if (S.resp[A].kind != RESP_ERR) return;
    if (threadIdx.x == 0) note_wave(S, 2);
    const uint32_t T = (uint32_t)S.target[A];
    // L = pingable members other than A and the target (npingable counts A's
    // pingable members other than itself)
    __shared__ uint32_t pos[2 * 3], val[2 * 3], pick[3], sel_k;
    if (threadIdx.x == 0) {
        const uint32_t L = (uint32_t)S.npingable[A] - (is_pingable_status(v_status(S.view[S.row(A) + T].vs)) ? 1u : 0u);
        const uint32_t k = L < 3 ? L : 3;
        // forward partial Fisher-Yates over the filtered list (underscore 1.13
        // sample): the draws fix which positions are touched
        uint64_t s = S.rng[A];
        for (uint32_t i = 0; i < k; i++) { pos[i] = i; pos[k + i] = (uint32_t)js_random_int(s, (int)i, (int)L - 1); }
        S.rng[A] = s;
        sel_k = k;
    }
    __syncthreads();
    const uint32_t k = sel_k;
    select_pingable_at(S, A, T, pos, 2 * k, val, sh);
    if (threadIdx.x == 0) {
        // the swaps on the (at most 2k) touched positions
        uint32_t p[6], v[6], m = 0;
        auto slot = [&](uint32_t q) -> uint32_t {
            for (uint32_t t = 0; t < m; t++) if (p[t] == q) return t;
            for (uint32_t t = 0; t < 2 * k; t++) if (pos[t] == q) { p[m] = q; v[m] = val[t]; return m++; }
            return 0;  // unreachable: every swapped position was resolved
        };
        for (uint32_t i = 0; i < k; i++) {
            const uint32_t a = slot(i), b = slot(pos[k + i]);
            const uint32_t t = v[a]; v[a] = v[b]; v[b] = t;
        }
        for (uint32_t i = 0; i < k; i++) pick[i] = v[slot(i)];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        S.pr_n[A] = k;
        S.pr_errors[A] = 0;
        S.pr_bad[A] = 0;
        S.pr_done[A] = k == 0 ? 1u : 0u;  // NoMembersError ends the protocol period
        S.pr_inc[A] = v_inc(S.view[S.row(A) + A].vs);
        S.pr_fp[A] = S.fp[A];
        S.pr_csum[A] = 0u;
        S.pr_ckv[A] = 0;
        // its checksum: k_checksums after this kernel (single shard: only if
        // k_pr_need finds a relay that could compare it)
        if (k && list_all) { S.ck_list[atomicAdd(S.ck_count, 1u)] = A; S.pr_ckv[A] = 1; }
    }
    __syncthreads();
    for (uint32_t i = 0; i < k; i++) {   // PingReqSender.send per member (:57-99)
        uint64_t off;
        uint32_t pm, pe;
        uint32_t m = wg_issue<ESC>(S, A, false, NONE, 0, &off, 1, sh, NONE, &pm, &pe);
        if (threadIdx.x == 0) {
            uint32_t slot = 3 * A + i;
            S.w3_dest[slot] = (int32_t)pick[i];
            S.pq_off[slot] = off;
            S.pq_len[slot] = m;
            S.pq_nesc[slot] = pe;
            stat_add(S, STAT_MESSAGES, 1ull);
        }
        __syncthreads();
    }
}

// Which ping-req initiators' checksums can a relay compare?  Relay K answers
// initiator A in W5 with issueAsReceiver(A, ...), which compares checksums
// only when its list comes out empty (lib/dissemination.js:102-117).  K's
// log after its phase-1 issue held an entry A's filter cannot skip with
// count c (k_need_checksums' per-source minima); every later issue of K adds
// at most 1: its phase-2 responses (pings it received), a relay ping and a W5
// response per ping-req it relays, and W4 responses as the target of other
// relays' pings (at most 3 per failed ping aimed at K).  While c + that bound
// <= 15 (maxPiggybackCount never drops below 15: a node is always in its own
// ring) the list is non-empty.  Each shard counts its own initiators' ping-
// reqs and failed pings; a cluster sums the counts (one all-reduce) before
// k_pr_need.  A relay that cannot be reached never answers.
// this shard's members declared faulty (all n when unbounded), for fdecl_all
__global__ void k_fdecl_share(SimDev S, uint32_t* out, uint32_t unbounded) {
    *out = unbounded ? S.n : min(*S.fdecl_count, S.n);
}
__global__ void k_pr_hist(SimDev S, uint32_t* w3cnt, uint32_t* w4b, uint32_t unbounded) {
    const uint32_t A = S.lo + blockIdx.x * blockDim.x + threadIdx.x;
    // w3cnt[n]: members this shard ever declared faulty (summed over the
    // shards with the counts: an upper bound of the cluster's distinct ones;
    // all n when a view may hold faulty or leave members from elsewhere)
    if (A == S.lo) atomicAdd(&w3cnt[S.n], unbounded ? S.n : min(*S.fdecl_count, S.n));
    if (A >= S.lo + S.nl || S.target[A] < 0 || S.resp[A].kind != RESP_ERR) return;
    atomicAdd(&w4b[S.target[A]], 3u);
    for (uint32_t i = 0; i < S.pr_n[A]; i++) atomicAdd(&w3cnt[S.w3_dest[3 * A + i]], 1u);
}
// (a relay K answers A with a non-empty list -- so A's checksum is never read
// -- when an entry K must send A stays live through K's U issues before that
// answer: its count c + U within K's maxPiggybackCount then.  That count
// changes only with K's ring, and the ring shrinks only by members with a
// faulty (or leave) update, which no node can know of before some node
// declared them (k_timers; k_pr_hist counts them): so it stays at least the
// rule's value for ring_count - F.)
__global__ void k_pr_need(SimDev S, const uint32_t* w3cnt, const uint32_t* w4b) {
    const uint32_t A = S.lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (A >= S.lo + S.nl || S.target[A] < 0 || S.resp[A].kind != RESP_ERR) return;
    const uint32_t F = w3cnt[S.n];
    bool need = false;
    for (uint32_t i = 0; i < S.pr_n[A] && !need; i++) {
        const uint32_t K = (uint32_t)S.w3_dest[3 * A + i];
        if (unreachable(S, A, K)) continue;
        const uint64_t U = (uint64_t)(S.g_base[K + 1] - S.g_base[K]) + 2ull * w3cnt[K] + w4b[K];
        const uint64_t l1 = S.min_l1[K], l2 = S.min_l2[K];
        const uint64_t l = (uint32_t)l1 != A ? l1 : l2;
        const uint32_t c = min(S.min_safe[K], l == ~0ull ? NONE : (uint32_t)(l >> 32));
        const uint32_t rc = (uint32_t)S.ring_count[K];
        const uint32_t maxpb_lo = min((uint32_t)S.max_pb[K], (uint32_t)max_piggyback((int)(rc > F ? rc - F : 0u)));
        need = c == NONE || (uint64_t)c + U > (uint64_t)max(maxpb_lo, (uint32_t)PIGGYBACK_FACTOR);
    }
    if (need) { S.ck_list[atomicAdd(S.ck_count, 1u)] = A; S.pr_ckv[A] = 1; }
}

// W3: relays handle ping-reqs (server/ping-req-handler.js:24-46): update, then
// ping the target (their own issueAsSender).
template <bool ESC>
__global__ void __launch_bounds__(BLOCK) k_w3(SimDev S, uint64_t now) {
    __shared__ Shared sh;
    const uint32_t K = S.lo + blockIdx.x, n = S.n;
    const uint32_t lo = S.g_base[K], hi = S.g_base[K + 1];
    if (lo < hi && threadIdx.x == 0) note_wave(S, 3);
    for (uint32_t j = lo; j < hi; j++) {
        const uint32_t slot = S.g_list[j], A = slot / 3;
        const uint32_t T = (uint32_t)S.target[A];
        if (unreachable(S, A, K)) {  // PingReqPingError for A, delivered in W4
            if (threadIdx.x == 0) {
                S.w4_dest[slot] = (int32_t)A;
                S.w4_err[slot] = 1;
                stat_add(S, STAT_MESSAGES, 1ull);
            }
            __syncthreads();
            continue;
        }
        const Change* msg = slot_msg(S, S.pq_off[slot]);
        auto src = [&](uint32_t i) { return load_msg(msg + i); };
        wg_apply(S, K, src, S.pq_len[slot], S.pq_len[slot], now, 1, 2, sh);  // :37
        uint64_t off;
        uint32_t pm, pe;
        uint32_t m = wg_issue<ESC>(S, K, false, NONE, 0, &off, 1, sh, NONE, &pm, &pe);  // sendPing -> issueAsSender
        if (threadIdx.x == 0) {
            S.w4_dest[slot] = (int32_t)T;
            S.w4_err[slot] = 0;
            S.rl_off[slot] = off;
            S.rl_len[slot] = m;
            S.rl_nesc[slot] = pe;
            S.rl_inc[slot] = v_inc(S.view[S.row(K) + K].vs);
            S.rl_fp[slot] = S.fp[K];
            // the body checksum matters only if T can answer
            S.rl_csum[slot] = unreachable(S, K, T) ? 0u : cached_checksum(S, K);
            stat_add(S, STAT_MESSAGES, 1ull);
        }
        __syncthreads();
    }
}


// Origin of a suspect/faulty update made locally by node v (makeSuspect /
// makeFaulty: source = v, sourceIncarnationNumber = v's incarnation,
// lib/membership.js:327-337).  Such origins are only ever compared by value
// (the receiver filter, lib/dissemination.js:91-98; they are not seen-tracked),
// so all of v's local updates at one incarnation share one table entry.
__device__ inline uint32_t local_origin(const SimDev& S, uint32_t v, uint64_t self_inc) {
    uint32_t id = S.self_origin[v];
    if (id != NONE && S.origins[id].source == v && S.origins[id].source_inc == self_inc) return id;
    // this shard's range is a ring as well: a slot is reused long after the
    // log entries and messages naming its previous origin have expired
    const uint32_t k = atomicAdd(S.lorigin_count, 1u);
    id = S.lorigin_base + S.rank * S.lorigin_per + k % S.lorigin_per;
    S.origins[id].source = v;
    S.origins[id].source_inc = self_inc;
    S.self_origin[v] = id;
    return id;
}

__device__ void pingreq_done(const SimDev& S, uint32_t A, int kind, uint64_t now, Shared& sh);

// W4: targets answer relay pings; A counts PingReqPingErrors.
template <bool ESC>
__global__ void __launch_bounds__(BLOCK) k_w4(SimDev S, uint64_t now) {
    __shared__ Shared sh;
    const uint32_t d = S.lo + blockIdx.x;
    const uint32_t lo = S.g_base[d], hi = S.g_base[d + 1];
    if (lo < hi && threadIdx.x == 0) note_wave(S, 4);
    for (uint32_t j = lo; j < hi; j++) {
        const uint32_t slot = S.g_list[j], A = slot / 3;
        const uint32_t K = (uint32_t)S.w3_dest[slot];
        if (S.w4_err[slot]) {
            pingreq_done(S, A, 1, now, sh);
            continue;
        }
        const uint32_t R4 = S.n + slot;
        if (unreachable(S, K, d)) {
            if (threadIdx.x == 0) {
                Resp r{};
                r.kind = RESP_ERR; r.from = d; r.snap = NONE;
                S.resp[R4] = r;
                stat_add(S, STAT_MESSAGES, 1ull);
            }
            __syncthreads();
            continue;
        }
        const Change* msg = slot_msg(S, S.rl_off[slot]);
        auto src = [&](uint32_t i) { return load_msg(msg + i); };
        wg_apply(S, d, src, S.rl_len[slot], S.rl_len[slot], now, 1, 2, sh);
        respond_as_receiver<ESC>(S, d, K, S.rl_inc[slot], S.rl_fp[slot], S.rl_csum[slot], true, R4, 0, sh);
    }
}

// W5: relays get the target's answer (ping-sender.js:30-44 + ping-req-handler.js:47-58):
// on success update twice, then answer A with issueAsReceiver and pingStatus.
template <bool ESC>
__global__ void __launch_bounds__(BLOCK) k_w5(SimDev S, uint64_t now) {
    __shared__ Shared sh;
    const uint32_t K = S.lo + blockIdx.x;
    const uint32_t lo = S.g_base[K], hi = S.g_base[K + 1];
    if (lo < hi && threadIdx.x == 0) note_wave(S, 5);
    for (uint32_t j = lo; j < hi; j++) {
        const uint32_t slot = S.g_list[j], A = slot / 3;
        const Resp r = S.resp[S.n + slot];
        const bool ok = r.kind != RESP_ERR;
        if (ok) apply_response<true, false, false>(S, K, r, now, 2, 2, sh);
        respond_as_receiver<ESC>(S, K, A, S.pr_inc[A], S.pr_fp[A], S.pr_csum[A], S.pr_ckv[A] != 0, 4 * S.n + slot,
                                 ok ? 1u : 0u,
                            sh);
    }
}

// ping-req aggregation at A (lib/swim/ping-req-sender.js:176-281); kind 0 ok,
// 1 PingReqPingError, 2 BadPingReqPingStatusError
__device__ void pingreq_done(const SimDev& S, uint32_t A, int kind, uint64_t now, Shared& sh) {
    if (threadIdx.x == 0) {
        sh.u[7] = 0;
        if (!S.pr_done[A]) {
            if (kind == 0) {
                S.pr_done[A] = 1;
            } else {
                S.pr_errors[A]++;
                if (kind == 2) S.pr_bad[A]++;
                if (S.pr_errors[A] >= S.pr_n[A]) {
                    S.pr_done[A] = 1;
                    if (S.pr_bad[A] > 0) sh.u[7] = 1;  // makeSuspect
                }
            }
        }
    }
    __syncthreads();
    if (sh.u[7]) {
        const uint32_t n = S.n, T = (uint32_t)S.target[A];
        if (threadIdx.x == 0) {
            // makeSuspect(target, target.incarnationNumber): source = A at its
            // current incarnation -> a receiver filter can match this origin
            const uint32_t id = local_origin(S, A, v_inc(S.view[S.row(A) + A].vs));
            *S.dangerous = 1;
            sh.u[6] = id;
            sh.q[1] = pack_view(v_inc(S.view[S.row(A) + T].vs), ST_SUSPECT);
        }
        __syncthreads();
        Change c;
        c.addr = T; c.origin = sh.u[6]; c.vs = sh.q[1];
        auto src = [&](uint32_t) { return c; };
        wg_apply(S, A, src, 1, 1, now, 1, 0, sh);
    }
    __syncthreads();
}

// W6: A applies ping-req responses (ping-req-sender.js:138) and aggregates.
template <bool ESC>
__global__ void __launch_bounds__(BLOCK) k_w6(SimDev S, uint64_t now) {
    __shared__ Shared sh;
    const uint32_t A = S.lo + blockIdx.x;
    const uint32_t lo = S.g_base[A], hi = S.g_base[A + 1];
    if (lo < hi && threadIdx.x == 0) note_wave(S, 6);
    for (uint32_t j = lo; j < hi; j++) {
        const uint32_t slot = S.g_list[j];
        const Resp r = S.resp[4 * S.n + slot];
        apply_response<true, false, ESC>(S, A, r, now, 1, 3, sh);
        pingreq_done(S, A, r.ping_status ? 0 : 2, now, sh);
    }
}

// W5/W6 destination maps from the slot state, for the messages this shard
// sends (W5 from a local target, W6 from a local relay); messages from other
// shards set their destination when they are unpacked (k_xs_unpack)
__global__ void k_dest_w5(SimDev S) {
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= 3 * S.n) return;
    const int32_t d4 = S.w4_dest[s];
    S.w5_dest[s] = (S.w3_dest[s] >= 0 && d4 >= 0 && !S.w4_err[s] && S.local((uint32_t)d4)) ? S.w3_dest[s] : -1;
}
__global__ void k_dest_w6(SimDev S) {
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= 3 * S.n) return;
    const int32_t d5 = S.w5_dest[s];
    S.w6_dest[s] = (d5 >= 0 && S.local((uint32_t)d5)) ? (int32_t)(s / 3) : -1;
}

// Suspicion timers due this round (lib/swim/suspicion.js:66-68): fired in
// creation order, each a separate makeFaulty(address, incarnation).  A timer is
// live iff its stamp is still the one stored for the address (stop/restart
// overwrite it); dead nodes' timers are dropped.  The live due timers of a node
// are applied as one batch per chunk of the queue: each makeFaulty's update
// concerns its own address (live timers name distinct addresses), a faulty
// update only stops its own timer, and the batch's ring removals, recorded
// changes and counters equal those of the calls one by one (no issue or read
// of the view happens between them).  The queue is in creation order, so the
// due timers are a prefix; chunks of TIMER_CHUNK are scanned in parallel.
constexpr uint32_t TIMER_CHUNK = 1024;
__global__ void __launch_bounds__(BLOCK) k_timers(SimDev S, uint32_t round, uint64_t now) {
    __shared__ Shared sh;
    __shared__ uint32_t due[TIMER_CHUNK];  // the chunk's live due timers' addresses, in queue order
    const uint32_t v = S.lo + blockIdx.x;
    const size_t tb = S.trow(v);
    const bool dead = S.dead[v] != 0;
    for (;;) {
        if (threadIdx.x == 0) { sh.u[0] = S.thead[v]; sh.u[1] = S.ttail[v]; }
        __syncthreads();
        const uint32_t head = sh.u[0], tail = sh.u[1];
        if (head >= tail) break;
        const uint32_t m = min(tail - head, TIMER_CHUNK);
        uint32_t first_not_due = NONE, cnt = 0;
        for (uint32_t c0 = 0; c0 < m; c0 += BLOCK) {
            const uint32_t i = c0 + threadIdx.x, p = head + i;
            bool live = false;
            uint32_t a = 0;
            if (i < m) {
                const uint2 e = S.tfifo[tb + p % S.tcap];
                if (e.y + 25 > round) first_not_due = min(first_not_due, i);  // 5000 ms = 25 rounds of 200 ms
                else { a = e.x; live = !dead && S.view[S.row(v) + a].tstamp == p + 1; }
            }
            uint32_t tot;
            const uint32_t r = block_rank(live, sh.sc, tot);
            if (live) due[cnt + r] = a;
            cnt += tot;
            __syncthreads();
        }
        // (due entries are a prefix of the queue: every live one lies before the first not-due one)
        const uint32_t ndue = min(m, block_min32(first_not_due, sh.sc));
        const uint32_t fire = cnt;
        // (distinct members ever declared faulty: k_pr_need's bound)
        for (uint32_t k = threadIdx.x; k < fire; k += BLOCK) {
            const uint32_t a = due[k], bit = 1u << (a & 31);
            if (!(atomicOr(&S.fdecl_bits[a >> 5], bit) & bit)) atomicAdd(S.fdecl_count, 1u);
        }
        if (threadIdx.x == 0) {
            S.thead[v] = head + ndue;
            if (fire) {
                sh.u[5] = local_origin(S, v, v_inc(S.view[S.row(v) + v].vs));
                *S.dangerous = 1;
            }
        }
        __syncthreads();
        if (fire) {
            const uint32_t id = sh.u[5];
            const VEnt* row = S.view + S.row(v);
            auto src = [&](uint32_t k) {
                Change c;
                c.addr = due[k]; c.origin = id; c.vs = pack_view(v_inc(row[c.addr].vs), ST_FAULTY);
                return c;
            };
            wg_apply(S, v, src, fire, fire, now, 1, 0, sh);
        }
        if (ndue < m || ndue == 0) break;
    }
}

// False-suspicion storm: accuser A
// calls membership.makeSuspect(victim, its view's incarnation of the victim)
// (lib/membership.js:154-156 -> makeUpdate :324-352), the victim refutes once
// the suspect reaches it (local override, :244-254).  The round's (accuser,
// victim) pairs come sorted by accuser, draw order kept within an accuser;
// the first block of each accuser's run applies its makeSuspects in order.
__global__ void __launch_bounds__(BLOCK) k_storm(SimDev S, const int32_t* acc, const int32_t* vic, uint32_t K,
                                                 uint64_t now) {
    __shared__ Shared sh;
    const uint32_t b = blockIdx.x;
    const int32_t A = acc[b];
    if ((b > 0 && acc[b - 1] == A) || !S.local((uint32_t)A)) return;
    for (uint32_t i = b; i < K && acc[i] == A; i++) {
        if (threadIdx.x == 0) {
            const uint32_t T = (uint32_t)vic[i];
            // source = A at its current incarnation: a receiver filter can match it
            sh.u[6] = local_origin(S, (uint32_t)A, v_inc(S.view[S.row(A) + A].vs));
            *S.dangerous = 1;
            sh.u[5] = T;
            sh.q[1] = pack_view(v_inc(S.view[S.row(A) + T].vs), ST_SUSPECT);
        }
        __syncthreads();
        Change c;
        c.addr = sh.u[5]; c.origin = sh.u[6]; c.vs = sh.q[1];
        auto src = [&](uint32_t) { return c; };
        wg_apply(S, (uint32_t)A, src, 1, 1, now, 1, 0, sh);
    }
}

// ---------------------------------------------------------------- join path
// SURVEY.md §8(f)4; DESIGN.md §3.  A node outside the cluster (dead = 2: no
// view, not pinging, unknown to the others) joins at the start of a round,
// after the due suspicion timers and before churn, as index.js:233-292 and
// lib/swim/join-sender.js do with the round's clock:
//   1. makeAlive(self, now) (index.js:235): source = itself at the new
//      incarnation (no local member yet), spliced into its empty member list
//      (one getJoinPosition draw);
//   2. each seed, in the given order, handles the join (server/join-handler.js:
//      76-98): makeAlive(joiner, its incarnation) -- an update with the seed
//      as source at its current incarnation, a local origin since its address
//      is not its source -- then replies with its checksum and fullSync();
//   3. the joiner merges the replies (lib/swim/join-response-merge.js:40-56:
//      all checksums equal and non-zero -> the first reply's members, else
//      mergeMembershipChangesets over all of them, lib/membership-changeset-
//      merge.js:22-51: first-appearance order, the largest incarnation wins,
//      the first of equals), update() stashes them (evaluated, none applied),
//      set() pushes them after itself (lib/membership.js:162-206) and its
//      listener adds the alive ones to the ring, starts a suspicion timer per
//      suspect and records every one (source = the replying seed), then
//      shuffle() (gossip.start).
// A node that has not joined yet: empty view, fresh RNG, Dissemination's
// default maxPiggybackCount (1).
__global__ void __launch_bounds__(BLOCK) k_join_reset(SimDev S, const uint32_t* ids, uint32_t count, uint64_t seed) {
    const uint32_t v = ids[blockIdx.x], n = S.n;
    if (threadIdx.x == 0) {
        S.rng[v] = node_rng_seed(seed, v);
        S.iter_index[v] = -1; S.iter_round[v] = 0;
        S.dhead[v] = 0; S.dtail[v] = 0; S.dlive[v] = 0; S.icount[v] = 0;
        S.max_pb[v] = 1;
        S.ring_count[v] = 0; S.npingable[v] = 0; S.mcount[v] = 0;
        S.csum_valid[v] = 0; S.fp[v] = 0; S.slen[v] = 0;
        S.dead[v] = 2;
        S.self_inc[v] = 0;
        S.thead[v] = 0; S.ttail[v] = 0; S.rbatch[v] = 0;
    }
    if (!S.local(v)) return;
    for (uint32_t a = threadIdx.x; a < n; a += BLOCK) {
        VEnt c;
        c.vs = 0; c.dpos = NONE; c.tstamp = 0;
        S.view[S.row(v) + a] = c;
        S.in_ring[S.row(v) + a] = 0;
    }
    for (uint32_t w = threadIdx.x; w < S.seen_words; w += BLOCK) S.seen[S.srow(v) + w] = 0;
    for (uint32_t w = threadIdx.x; w < (n + 31) / 32; w += BLOCK) settled_bits(S, v)[w] = 0;  // (empty view)
    for (uint32_t g = threadIdx.x; g < S.ncoll; g += BLOCK) S.coll_owner[S.crow(v) + g] = -1;
}
// Step 1.  makeUpdate without a local member yet (lib/membership.js:323-337):
// source = the joiner, sourceIncarnationNumber = the new incarnation -- the
// value a receiver filter compares, so a local origin (not a makeAlive
// origin, whose source incarnation is always an older one).
__global__ void __launch_bounds__(BLOCK) k_join_self(SimDev S, const uint32_t* joiners, uint64_t now) {
    __shared__ Shared sh;
    const uint32_t v = joiners[blockIdx.x];
    if (!S.local(v)) return;
    if (threadIdx.x == 0) {
        sh.u[6] = local_origin(S, v, now);
        *S.dangerous = 1;
    }
    __syncthreads();
    Change c;
    c.addr = v; c.origin = sh.u[6]; c.vs = pack_view(now, ST_ALIVE);
    auto src = [&](uint32_t) { return c; };
    wg_apply<true>(S, v, src, 1, 1, now, 1, 0, sh);
}
// Step 2: pairs sorted by seed (schedule order kept within a seed); the first
// block of each seed's run handles its joins in order and snapshots each
// reply: the view (jvs), the member order (jord) and count (jm).
__global__ void __launch_bounds__(BLOCK) k_join_seed(SimDev S, const int32_t* pseed, const uint32_t* pidx,
                                                     const uint32_t* pjoin, uint32_t P, uint64_t now, uint64_t* jvs,
                                                     uint32_t* jord, uint32_t* jm) {
    __shared__ Shared sh;
    const uint32_t b = blockIdx.x, n = S.n;
    const int32_t sd = pseed[b];
    if ((b > 0 && pseed[b - 1] == sd) || !S.local((uint32_t)sd)) return;
    const uint32_t s = (uint32_t)sd;
    for (uint32_t i = b; i < P && pseed[i] == sd; i++) {
        if (threadIdx.x == 0) {
            sh.u[6] = local_origin(S, s, v_inc(S.view[S.row(s) + s].vs));
            *S.dangerous = 1;
        }
        __syncthreads();
        Change c;
        c.addr = pjoin[i]; c.origin = sh.u[6]; c.vs = pack_view(now, ST_ALIVE);  // the joiner's incarnation
        auto src = [&](uint32_t) { return c; };
        wg_apply<true>(S, s, src, 1, 1, now, 1, 0, sh);
        const size_t slot = pidx[i];
        const VEnt* row = S.view + S.row(s);
        for (uint32_t a = threadIdx.x; a < n; a += BLOCK) jvs[slot * n + a] = row[a].vs;
        const uint32_t M = S.mcount[s];
        for (uint32_t q = threadIdx.x; q < M; q += BLOCK) jord[slot * n + q] = S.order[S.row(s) + q];
        if (threadIdx.x == 0) {
            jm[slot] = M;
            stat_add(S, STAT_FULLSYNC, 1ull);  // the reply's dissemination.fullSync()
        }
        __syncthreads();
    }
}
// The replies' checksums (membership.checksum after the seed's update): one
// wave per reply whose seed lives on this shard.
__global__ void __launch_bounds__(BLOCK) k_join_csum(SimDev S, const uint32_t* seed_of, uint32_t P, const uint64_t* jvs,
                                                     uint32_t* jcs) {
    __shared__ __attribute__((aligned(16))) uint8_t bufs[NWAVE][CKW_BUF];
    const AddrTable at{S.addr_words, S.addr_len};
    for (uint32_t p = blockIdx.x * NWAVE + wave_id(); p < P; p += gridDim.x * NWAVE) {
        if (!S.local(seed_of[p])) continue;
        const uint64_t* row = jvs + (size_t)p * S.n;
        const uint32_t cs = wave_view_checksum([&](uint32_t a) { return row[a]; }, S.n, at, bufs[wave_id()]);
        if (lane_id() == 0) jcs[p] = cs;
    }
}
// Step 3, one block per joiner of this shard: its replies are pairs
// [poff[t], poff[t+1]) (seed_of: the replying seed).
__global__ void __launch_bounds__(BLOCK) k_join_merge(SimDev S, const uint32_t* joiners, const uint32_t* poff,
                                                      const uint32_t* seed_of, const uint64_t* jvs, const uint32_t* jord,
                                                      const uint32_t* jm, const uint32_t* jcs, uint8_t* need_shuffle) {
    __shared__ Shared sh;
    const uint32_t t = blockIdx.x, v = joiners[t], n = S.n;
    if (!S.local(v)) return;
    const uint32_t p0 = poff[t], p1 = poff[t + 1];
    bool same = p1 > p0;  // hasSameChecksums (join-response-merge.js:22-37)
    for (uint32_t p = p0; p < p1; p++) same = same && jcs[p] != 0 && jcs[p] == jcs[p0];
    const uint32_t pe = same ? p0 + 1 : p1;  // the changesets merged
    VEnt* vrow = S.view + S.row(v);
    uint32_t* lrow = S.dko + S.row(v);
    uint64_t* lvrow = S.dvs + S.row(v);
    uint32_t* larow = S.dad + S.row(v);
    uint32_t* ord = S.order + S.row(v);
    const uint32_t dt0 = S.dtail[v], M0 = S.mcount[v];  // (after step 1: the joiner alone)
    const uint32_t stamp = (S.icount[v] & STAMP_MASK) << 24;  // a recorded change's count is undefined
    uint32_t U = 0;
    for (uint32_t p = p0; p < pe; p++) {
        const uint32_t M = jm[p], src = seed_of[p];
        const uint64_t* snap = jvs + (size_t)p * n;
        const uint32_t* sord = jord + (size_t)p * n;
        for (uint32_t c0 = 0; c0 < M; c0 += BLOCK) {
            const uint32_t i = c0 + threadIdx.x;
            uint32_t a = NONE;
            uint64_t val = 0, cur = 0;
            if (i < M) {
                a = sord[i];
                if (a == v) a = NONE;  // the local member is skipped (changeset-merge.js:31-33)
                else { val = snap[a]; cur = vrow[a].vs; }
            }
            const bool isnew = a != NONE && v_status(cur) == ST_ABSENT;
            uint32_t tot;
            const uint32_t r = block_rank(isnew, sh.sc, tot);
            if (isnew) {
                const uint32_t pos = dt0 + U + r;  // set() pushes in merge order; recordChange in that order
                VEnt c;
                c.vs = val; c.dpos = pos; c.tstamp = 0;
                vrow[a] = c;
                ord[M0 + U + r] = a;
                lrow[pos % n] = log_word(src, stamp);  // fullSync origin: source = the seed
                lvrow[pos % n] = val;
                larow[pos % n] = a;
            } else if (a != NONE && v_inc(val) > v_inc(cur)) {  // a later changeset's larger incarnation wins
                vrow[a].vs = val;
                const uint32_t pos = vrow[a].dpos;
                lrow[pos % n] = log_word(src, stamp);
                lvrow[pos % n] = val;
                larow[pos % n] = a;
            }
            U += tot;
            __syncthreads();
        }
    }
    // the set listener over the U updates in order (lib/membership-set-listener.js:24-48)
    uint32_t ring = 0, ping = 0, tt = S.ttail[v];
    for (uint32_t c0 = 0; c0 < U; c0 += BLOCK) {
        const uint32_t i = c0 + threadIdx.x;
        uint32_t a = 0, st = ST_ABSENT;
        if (i < U) { a = ord[M0 + i]; st = v_status(vrow[a].vs); }
        const bool susp = i < U && st == ST_SUSPECT;
        uint32_t tot;
        const uint32_t r = block_rank(susp, sh.sc, tot);
        if (i < U) {
            ring += st == ST_ALIVE;
            ping += is_pingable_status(st);
            S.in_ring[S.row(v) + a] = st == ST_ALIVE;
            if (susp) {
                S.tfifo[S.trow(v) + (tt + r) % S.tcap] = make_uint2(a, S.round);
                vrow[a].tstamp = tt + r + 1;
            }
        }
        tt += tot;
        __syncthreads();
    }
    const uint64_t rt = block_sum64(((uint64_t)ring << 32) | ping, sh.sc);
    if (threadIdx.x == 0) {
        const uint64_t evaluated = same ? jm[p0] : U;  // update(mergeJoinResponses(...)) while not ready
        stat_add(S, STAT_EVALUATED, (unsigned long long)evaluated);
        S.mcount[v] = M0 + U;
        S.dtail[v] = dt0 + U;
        S.dlive[v] += U;
        if (tt - S.thead[v] > S.tcap) atomicOr(S.err, SIMERR_TIMERS_FULL);
        S.ttail[v] = tt;
        S.ring_count[v] += (int32_t)(rt >> 32);
        S.npingable[v] += (int32_t)(uint32_t)rt;
        S.csum_valid[v] = 0;
        need_shuffle[v] = 1;  // gossip.start() -> shuffle()
    }
}
// Ring owners of colliding replica hashes in a joiner's ring: the server of
// the group inserted first -- itself (makeAlive), then set()'s alive
// servers in update order, which is their log order (dpos).
__global__ void k_join_owners(SimDev S, const uint32_t* joiners, uint32_t J) {
    const uint64_t total = (uint64_t)J * S.ncoll;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = joiners[i / S.ncoll], g = (uint32_t)(i % S.ncoll);
        if (!S.local(v)) continue;
        int32_t own = -1;
        uint32_t best = NONE;
        for (uint32_t q = S.cmem_off[g]; q < S.cmem_off[g + 1]; q++) {
            const uint32_t sv = S.cmem[q];
            if (!S.in_ring[S.row(v) + sv]) continue;
            const uint32_t d = S.view[S.row(v) + sv].dpos;
            if (d < best) { best = d; own = (int32_t)sv; }
        }
        S.coll_owner[S.crow(v) + g] = own;
    }
}
// a list of nodes joined at `now` (every shard)
__global__ void k_mark_joined(SimDev S, const uint32_t* ids, uint32_t k, uint64_t now) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) { S.dead[ids[i]] = 0; S.self_inc[ids[i]] = now; }
}

// every local node's own incarnation into self_inc (all-gathered by sharded fault runs)
__global__ void k_self_inc(SimDev S) {
    const uint32_t v = S.lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (v < S.lo + S.nl) S.self_inc[v] = v_inc(S.view[S.row(v) + v].vs);
}

// In-process exchanges: every segment copy of one collective in one launch
// (blockIdx.y = segment) instead of a copy launch per (source, destination)
// pair -- G (G - 1) of them per all-to-all or all-gather, a few hundred per
// sharded round, each costing a launch on the cluster stream.
struct CopyDesc {
    const void* src;
    void* dst;
    uint64_t bytes;
};
constexpr uint32_t COPY_BATCH = 128;  // (the batch travels as a 3 KB kernel argument)
struct CopyBatch {
    uint32_t n, pad;
    CopyDesc d[COPY_BATCH];
};
__global__ void __launch_bounds__(256) k_copy_batch(CopyBatch b) {
    const CopyDesc c = b.d[blockIdx.y];
    const uint64_t stride = (uint64_t)gridDim.x * 256, t0 = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uintptr_t al = (uintptr_t)c.src | (uintptr_t)c.dst | (uintptr_t)c.bytes;
    if ((al & 15u) == 0) {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const u4* s = (const u4*)c.src;
        u4* d = (u4*)c.dst;
        for (uint64_t i = t0; i < c.bytes / 16; i += stride) d[i] = s[i];
    } else if ((al & 3u) == 0) {
        const uint32_t* s = (const uint32_t*)c.src;
        uint32_t* d = (uint32_t*)c.dst;
        for (uint64_t i = t0; i < c.bytes / 4; i += stride) d[i] = s[i];
    } else {
        const uint8_t* s = (const uint8_t*)c.src;
        uint8_t* d = (uint8_t*)c.dst;
        for (uint64_t i = t0; i < c.bytes; i += stride) d[i] = s[i];
    }
}
// The round's buffer resets in one launch (blockIdx.y = buffer) instead of a
// fill launch per buffer: a sharded round is a chain of short launches per
// shard, and each memset was one more.
struct FillDesc {
    void* dst;
    uint64_t bytes;  // a multiple of 4
    uint32_t word;   // the byte value repeated
    uint32_t pad;
};
constexpr uint32_t FILL_BATCH = 16;
struct FillBatch {
    uint32_t n, pad;
    FillDesc d[FILL_BATCH];
};
__device__ inline void fill_desc(const FillDesc& f, uint32_t x, uint32_t gx) {
    uint32_t* d = (uint32_t*)f.dst;
    for (uint64_t i = (uint64_t)x * 256 + threadIdx.x; i < f.bytes / 4; i += (uint64_t)gx * 256) d[i] = f.word;
}
__global__ void __launch_bounds__(256) k_fill_batch(FillBatch b) { fill_desc(b.d[blockIdx.y], blockIdx.x, gridDim.x); }
// The round's start in one launch: blocks [0, gx * b.n) are a fill batch (gx
// blocks per buffer), the rest clear the seen bits of 4 nodes each.
__global__ void __launch_bounds__(256) k_round_start(FillBatch b, uint32_t gx, SimDev S) {
    const uint32_t nf = gx * b.n;
    if (blockIdx.x < nf) fill_desc(b.d[blockIdx.x / gx], blockIdx.x % gx, gx);
    else seen_clear(S, blockIdx.x - nf);
}
__global__ void k_add_u32(uint32_t* dst, const uint32_t* src, uint32_t count) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) dst[i] += src[i];
}

__global__ void k_mark_dead(SimDev S, const int32_t* ids, uint32_t k) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) S.dead[ids[i]] = 1;
}

// Per-block counters are folded into S.stats, and the live fingerprints'
// min and max taken (all live views equal <=> min == max; fp_mm = {min, max},
// reset to {~0, 0} at the round's start), by k_round_end.
// The round's end: blocks [0, ncv) take the live
// fingerprints' bounds, the next 64 x STAT_NSTATS fold a 1/64 slice of one
// counter column each; one launch instead of two.  (Finishing the round in
// its last block, behind a device-scope fence per block, cost 128 us per
// round on gfx950 -- each fence writes back the XCD's L2 -- so a single shard
// still finishes in k_converge_done.)
__global__ void __launch_bounds__(BLOCK) k_round_end(SimDev S, unsigned long long* fp_mm, uint32_t ncv) {
    __shared__ BlockScratch sc;
    if (blockIdx.x < ncv) {
        uint64_t lo = ~0ull, hi = 0;
        for (uint32_t v = S.lo + blockIdx.x * BLOCK + threadIdx.x; v < S.lo + S.nl; v += ncv * BLOCK) {
            if (S.dead[v]) continue;
            const uint64_t f = S.fp[v];
            lo = f < lo ? f : lo;
            hi = f > hi ? f : hi;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t a = __shfl_xor(lo, o), b = __shfl_xor(hi, o);
            lo = a < lo ? a : lo;
            hi = b > hi ? b : hi;
        }
        if (lane_id() == 0) {
            atomicMin(&fp_mm[0], (unsigned long long)lo);
            atomicMax(&fp_mm[1], (unsigned long long)hi);
        }
    } else {
        const uint32_t x = (blockIdx.x - ncv) % 64u, i = (blockIdx.x - ncv) / 64u;
        const uint32_t per = (S.bstride + 63u) / 64u;
        const uint32_t lo = x * per, hi = min(lo + per, S.bstride);
        unsigned long long* col = S.bstats + (size_t)i * S.bstride;
        unsigned long long acc = 0;
        for (uint32_t r = lo + threadIdx.x; r < hi; r += BLOCK) {
            const unsigned long long v = col[r];
            if (v) {
                acc = i == STAT_WAVES ? (v > acc ? v : acc) : acc + v;
                col[r] = 0;
            }
        }
        if (i == STAT_WAVES) {
            const uint32_t m = block_min32(~(uint32_t)acc, sc);  // max via min of complements
            if (threadIdx.x == 0 && ~m) atomicMax(&S.stats[i], (unsigned long long)~m);
        } else {
            const unsigned long long t = block_sum64(acc, sc);
            if (threadIdx.x == 0 && t) atomicAdd(&S.stats[i], t);
        }
    }
}
__global__ void k_converge_done(SimDev S, const unsigned long long* fp_mm, unsigned long long* totals) {
    if (threadIdx.x != 0) return;
    const bool conv = fp_mm[0] >= fp_mm[1];  // also true when no node is live
    *S.conv = conv ? 1u : 0u;
    for (int i = 0; i < STAT_NSTATS; i++) totals[i] += S.stats[i];
    totals[STAT_NSTATS] += conv ? 1ull : 0ull;  // converged rounds
}

// The origin record of every slot of node v's dissemination log, and the
// address of entries with a makeAlive origin (host reads; addr holds the dad row)
__global__ void k_log_origins(SimDev S, uint32_t v, Origin* out, uint32_t* addr) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S.n) return;
    const uint32_t ko = S.dko[S.row(v) + i];
    Origin o{};
    // (slots outside the live window [head, tail) hold stale words)
    const uint32_t head = S.dhead[v], tail = S.dtail[v], n = S.n;
    const uint32_t p = head + (i + n - head % n) % n;  // the position of slot i in the window's span
    if (p < tail && !is_tomb(ko)) {
        o = S.origins[origin_slot(S, log_origin(ko))];
        if (ko & LOG_ALIVE) addr[i] = o.source;
    }
    out[i] = o;
}

// Per local view: members by status (absent .. leave) and ring server count
// (test and bench invariants over every view without copying views out).
__global__ void __launch_bounds__(BLOCK) k_view_counts(SimDev S, uint32_t* out) {
    __shared__ BlockScratch sc;
    const uint32_t v = S.lo + blockIdx.x;
    const VEnt* row = S.view + S.row(v);
    uint32_t c[5] = {0, 0, 0, 0, 0};
    for (uint32_t a = threadIdx.x; a < S.n; a += BLOCK) {
        const uint32_t st = v_status(row[a].vs);
        c[0] += st == 0; c[1] += st == 1; c[2] += st == 2; c[3] += st == 3; c[4] += st == 4;
    }
    for (int i = 0; i < 5; i++) {
        const uint64_t t = block_sum64(c[i], sc);
        if (threadIdx.x == 0) out[(size_t)v * 6 + i] = (uint32_t)t;
    }
    if (threadIdx.x == 0) out[(size_t)v * 6 + 5] = (uint32_t)S.ring_count[v];
}

__global__ void k_list_local(SimDev S, uint32_t* list, uint32_t* count) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < S.nl) list[i] = S.lo + i;
    if (i == 0) *count = S.nl;
}

// ring lookup in view v for a batch of key hashes (lib/ring.js:138-147)
__global__ void k_view_lookup(SimDev S, uint32_t v, const uint32_t* pt_hash, const int32_t* pt_server,
                              const int32_t* pt_coll, uint32_t npts, const uint32_t* h, uint32_t nk,
                              int32_t* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nk) return;
    uint32_t lo = 0, hi = npts, key = h[i];
    while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (pt_hash[m] < key) lo = m + 1; else hi = m; }
    int32_t res = -1;
    for (uint32_t k = 0; k < npts; k++) {
        uint32_t p = lo + k;
        if (p >= npts) p -= npts;
        int32_t o;
        if (pt_coll[p] >= 0) o = S.coll_owner[S.crow(v) + pt_coll[p]];
        else o = S.in_ring[S.row(v) + pt_server[p]] ? pt_server[p] : -1;
        if (o >= 0) { res = o; break; }
    }
    out[i] = res;
}

// ---------------------------------------------------------------- wire bridge
// Node-level ping path between rounds (rp_sim_ping_body / rp_sim_handle_ping /
// rp_sim_update): the reference's JSON ping bodies and
// responses, as rows (address, status, incarnation, source, source
// incarnation) the host codec (ringpop_amd/wire.py, js/) turns into JSON.
// One workgroup each; they run on the node's shard between rounds, with the
// clock of the next round.
struct WireRow {
    int64_t addr, status, inc, source, source_inc;  // source -1 / source_inc 0: undefined
};
// Changes from the wire: each gets a local origin with its (source,
// sourceIncarnationNumber) -- the receiver filter compares them by value.
__global__ void k_bridge_origins(SimDev S, const WireRow* rows, uint32_t n, Change* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const WireRow r = rows[i];
    const uint32_t k = atomicAdd(S.lorigin_count, 1u);
    uint32_t id;
    {
        id = S.lorigin_base + S.rank * S.lorigin_per + k % S.lorigin_per;
        S.origins[id].source = r.source < 0 ? NONE : (uint32_t)r.source;
        S.origins[id].source_inc = (uint64_t)r.source_inc;
        S.origins[id].round = S.round;
        if (r.source >= 0 && r.source_inc != 0) *S.dangerous = 1;
    }
    Change c;
    c.addr = (uint32_t)r.addr; c.origin = id; c.vs = pack_view((uint64_t)r.inc, (uint32_t)r.status);
    out[i] = c;
}
// Membership.update(changes) at node v (lib/membership.js:208-313)
__global__ void __launch_bounds__(BLOCK) k_bridge_apply(SimDev S, uint32_t v, const Change* c, uint32_t n, uint64_t now,
                                                        uint32_t* applied) {
    __shared__ Shared sh;
    auto src = [&](uint32_t i) { return c[i]; };
    const uint32_t a = wg_apply(S, v, src, n, n, now, 1, 0, sh);
    if (threadIdx.x == 0) *applied = a;
}
// issueAsSender (filter 0) / issueAsReceiver's list (filter 1) of node v;
// res = {arena offset, list length}
__global__ void __launch_bounds__(BLOCK) k_bridge_issue(SimDev S, uint32_t v, int filter, uint32_t fsrc, uint64_t finc,
                                                        uint64_t* res) {
    __shared__ Shared sh;
    uint64_t off;
    uint32_t pm, pe;
    const uint32_t m = wg_issue<false>(S, v, filter != 0, fsrc, finc, &off, filter ? 2 : 1, sh, NONE, &pm, &pe);
    if (threadIdx.x == 0) { res[0] = off; res[1] = m; }
}
// issued changes -> rows (the issueAs copy, lib/dissemination.js:170-177)
__global__ void k_bridge_rows(SimDev S, const Change* msg, uint32_t m, WireRow* rows) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const Change c = msg[i];
    const Origin o = S.origins[origin_slot(S, c.origin)];
    WireRow r;
    r.addr = c.addr & ADDR_MASK; r.status = v_status(c.vs); r.inc = (int64_t)v_inc(c.vs);
    r.source = o.source == NONE ? -1 : (int64_t)o.source; r.source_inc = (int64_t)o.source_inc;
    rows[i] = r;
}
// Dissemination.fullSync (lib/dissemination.js:61-76): every member in
// member order, source = v, no sourceIncarnationNumber
__global__ void k_bridge_fullsync(SimDev S, uint32_t v, WireRow* rows) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S.mcount[v]) return;
    const uint32_t a = S.order[S.row(v) + i];
    const uint64_t vs = S.view[S.row(v) + a].vs;
    WireRow r;
    r.addr = a; r.status = v_status(vs); r.inc = (int64_t)v_inc(vs); r.source = v; r.source_inc = 0;
    rows[i] = r;
}
// membership.checksum and getIncarnationNumber() of node v
__global__ void k_bridge_checksum(SimDev S, uint32_t v, uint64_t* out) {
    if (threadIdx.x != 0) return;
    out[0] = cached_checksum(S, v);
    out[1] = v_inc(S.view[S.row(v) + v].vs);
}

// =====================================================================
// Sharding: nodes [lo, lo + nl) per shard.  One round of a G-shard cluster
// exchanges: the senders' ping metadata (all-gather), their
// checksum snapshots (all-gather), ping bodies (all-to-all, shard -> the
// target's shard), response records and response changes (all-to-all back),
// and the round statistics (all-gather).  Every buffer of an all-to-all is
// laid out as one segment per partner shard in partner order, each segment
// in ascending sender id, so both sides derive the same offsets from the
// replicated metadata and no count exchange is needed for pings.
// =====================================================================
struct PingMeta {
    int32_t target;
    uint32_t len, plen, min_cnt;
    int32_t ring_count;
    uint32_t nesc;
    uint64_t inc, fp;
    uint64_t min_l1, min_l2;
    uint32_t min_safe;
    int32_t max_pb;
};
static_assert(sizeof(PingMeta) == 64, "ping metadata is 64 bytes");
struct RespRec {  // a response crossing shards: kind, reference list length, words and escapes shipped
    int32_t kind;
    uint32_t len, psize, pesc;
};
// Exchange counts per partner shard (XC_NCAT x G, entries of the segment):
// ping words / escapes, response records, response words / escapes.
enum {
    XC_PING_SEND = 0, XC_PING_RECV, XC_PESC_SEND, XC_PESC_RECV, XC_REC_SEND, XC_REC_RECV,
    XC_PAY_SEND, XC_PAY_RECV, XC_RESC_SEND, XC_RESC_RECV,
    // ping-req waves (k_xs_*): records, words, escapes
    XS_REC_SEND, XS_REC_RECV, XS_W_SEND, XS_W_RECV, XS_E_SEND, XS_E_RECV, XC_NCAT
};

__global__ void k_meta_pack(SimDev S, PingMeta* meta) {
    const uint32_t v = S.lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= S.lo + S.nl) return;
    PingMeta m;
    m.target = S.target[v]; m.len = S.msg_len[v]; m.plen = S.msg_plen[v]; m.min_cnt = S.min_cnt[v];
    m.ring_count = S.ring_count[v]; m.nesc = S.msg_nesc[v]; m.inc = S.snd_inc[v]; m.fp = S.snd_fp[v];
    m.min_l1 = S.min_l1[v]; m.min_l2 = S.min_l2[v]; m.min_safe = S.min_safe[v]; m.max_pb = S.max_pb[v];
    meta[v] = m;
}
__global__ void k_meta_unpack(SimDev S, const PingMeta* meta) {
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= S.n || S.local(v)) return;
    const PingMeta m = meta[v];
    S.target[v] = m.target; S.msg_len[v] = m.len; S.msg_plen[v] = m.plen; S.min_cnt[v] = m.min_cnt;
    S.ring_count[v] = m.ring_count; S.msg_nesc[v] = m.nesc; S.snd_inc[v] = m.inc; S.snd_fp[v] = m.fp;
    S.min_l1[v] = m.min_l1; S.min_l2[v] = m.min_l2; S.min_safe[v] = m.min_safe; S.max_pb[v] = m.max_pb;
    S.need_csum[v] = 0;
}

// Planning.  Every all-to-all buffer holds one segment per partner shard in
// partner order, senders ascending inside a segment.  A planning kernel runs
// one 1024-thread block per partner (grid.y: 0 = outgoing, the local senders
// whose target lives on that partner; 1 = incoming, the partner's senders
// whose target lives here), each scanning its senders in coalesced tiles
// with three counters at once; offsets come out relative to the segment and
// k_plan_fix adds the segment bases once every partner's total is known.
constexpr int XB = 1024;
constexpr uint32_t MAXG = 64;  // shards per cluster
struct U3 { uint64_t a, b, c; };

// Exclusive tile-wise scan of get(i) (three counters; zero for non-members)
// over i in [0, L): put(i, prefix) for members, returns the totals.
template <class Get, class Put>
__device__ U3 tile_scan3(uint32_t L, const Get& get, const Put& put) {
    __shared__ uint64_t wsum[3][XB / 64];
    const int lane = lane_id(), w = wave_id();
    U3 run = {0, 0, 0};
    for (uint32_t t0 = 0; t0 < L; t0 += XB) {
        const uint32_t i = t0 + threadIdx.x;
        bool member = false;
        U3 v = {0, 0, 0};
        if (i < L) member = get(i, v);
        uint64_t x[3] = {v.a, v.b, v.c};
#pragma unroll
        for (int f = 0; f < 3; f++) {
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint64_t y = __shfl_up(x[f], o);
                if (lane >= o) x[f] += y;
            }
            if (lane == 63) wsum[f][w] = x[f];
        }
        __syncthreads();
        uint64_t before[3] = {0, 0, 0}, tot[3] = {0, 0, 0};
#pragma unroll
        for (int f = 0; f < 3; f++)
            for (int ww = 0; ww < XB / 64; ww++) {
                const uint64_t c = wsum[f][ww];
                before[f] += ww < w ? c : 0;
                tot[f] += c;
            }
        if (member) put(i, U3{run.a + before[0] + x[0] - v.a, run.b + before[1] + x[1] - v.b, run.c + before[2] + x[2] - v.c});
        run.a += tot[0]; run.b += tot[1]; run.c += tot[2];
        __syncthreads();
    }
    return run;
}

// Ping words / escapes / response-record slots of both directions.
__global__ void __launch_bounds__(XB) k_plan_pings(SimDev S, uint64_t* soff, uint64_t* seoff, uint32_t* rr_idx,
                                                  uint32_t* rs_idx, unsigned long long* cnt) {
    const uint32_t q = blockIdx.x, me = S.rank, G = S.nranks;
    if (blockIdx.y == 0) {  // outgoing to q
        U3 t = {0, 0, 0};
        if (q != me)
            t = tile_scan3(S.nl, [&](uint32_t i, U3& v) {
                const uint32_t A = S.lo + i;
                const int32_t T = S.target[A];
                if (T < 0 || S.owner((uint32_t)T) != q) return false;
                v = U3{S.msg_plen[A], S.msg_nesc[A], 1};
                return true;
            }, [&](uint32_t i, const U3& p) { soff[S.lo + i] = p.a; seoff[S.lo + i] = p.b; rr_idx[S.lo + i] = (uint32_t)p.c; });
        if (threadIdx.x == 0) { cnt[XC_PING_SEND * G + q] = t.a; cnt[XC_PESC_SEND * G + q] = t.b; cnt[XC_REC_RECV * G + q] = t.c; }
    } else {  // incoming from q
        U3 t = {0, 0, 0};
        if (q != me)
            t = tile_scan3(S.nl, [&](uint32_t i, U3& v) {
                const uint32_t A = q * S.nl + i;
                const int32_t T = S.target[A];
                if (T < 0 || !S.local((uint32_t)T)) return false;
                v = U3{S.msg_plen[A], S.msg_nesc[A], 1};
                return true;
            }, [&](uint32_t i, const U3& p) { const uint32_t A = q * S.nl + i; S.rx_off[A] = p.a; S.rx_eoff[A] = p.b; rs_idx[A] = (uint32_t)p.c; });
        if (threadIdx.x == 0) { cnt[XC_PING_RECV * G + q] = t.a; cnt[XC_PESC_RECV * G + q] = t.b; cnt[XC_REC_SEND * G + q] = t.c; }
    }
}
__device__ inline uint64_t seg_base(const unsigned long long* cnt, int cat, uint32_t G, uint32_t q) {
    uint64_t b = 0;
    for (uint32_t r = 0; r < q; r++) b += cnt[cat * G + r];
    return b;
}
// Segment bases into the planned offsets (one thread per sender).
__global__ void k_plan_fix_pings(SimDev S, uint64_t* soff, uint64_t* seoff, uint32_t* rr_idx, uint32_t* rs_idx,
                                 const unsigned long long* cnt) {
    const uint32_t A = blockIdx.x * blockDim.x + threadIdx.x, G = S.nranks;
    if (A >= S.n) return;
    const int32_t T = S.target[A];
    if (T < 0) return;
    if (S.local(A) && !S.local((uint32_t)T)) {
        const uint32_t q = S.owner((uint32_t)T);
        soff[A] += seg_base(cnt, XC_PING_SEND, G, q);
        seoff[A] += seg_base(cnt, XC_PESC_SEND, G, q);
        rr_idx[A] += (uint32_t)seg_base(cnt, XC_REC_RECV, G, q);
    } else if (!S.local(A) && S.local((uint32_t)T)) {
        const uint32_t r = S.owner(A);
        S.rx_off[A] += seg_base(cnt, XC_PING_RECV, G, r);
        S.rx_eoff[A] += seg_base(cnt, XC_PESC_RECV, G, r);
        rs_idx[A] += (uint32_t)seg_base(cnt, XC_REC_SEND, G, r);
    }
}

// A message of `len` changes -> wire words + escapes (one block).
__device__ inline void store_esc(const SimDev& S, Esc* dst, const Change& c) {
    (void)S;
    store_msg(&dst->c, c);
}

// Local (suspect / faulty) origins allocated since this shard's last
// all-gather, as one block of og: header {source = ring position of the
// first, round = count}, then the records (one block of 1024 threads).  The
// all-gather runs before every exchange that can carry an origin created
// since the previous one (the pings: round-start timers, storms, joins and
// the previous round's ping-req verdicts; wave W5: W4's verdicts).
__global__ void __launch_bounds__(1024) k_origin_pack(SimDev S, Origin* og, uint32_t cap) {
    Origin* blk = og + (size_t)S.rank * (cap + 1);
    const uint32_t prev = *S.lorigin_sent, cnt = *S.lorigin_count - prev;
    if (cnt > cap || cnt > S.lorigin_per) {
        if (threadIdx.x == 0) { atomicOr(S.err, SIMERR_ORIGIN_FULL); blk[0].source = prev; blk[0].round = 0; }
        return;
    }
    const uint32_t base = S.lorigin_base + S.rank * S.lorigin_per;
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) blk[1 + i] = S.origins[base + (prev + i) % S.lorigin_per];
    __syncthreads();
    if (threadIdx.x == 0) { blk[0].source = prev; blk[0].round = cnt; blk[0].source_inc = 0; *S.lorigin_sent = prev + cnt; }
}
// ... installed under their cluster-wide ids on every other shard (grid G);
// such origins make the receiver filter live here too (SimDev::dangerous)
__global__ void __launch_bounds__(256) k_origin_install(SimDev S, const Origin* og, uint32_t cap) {
    const uint32_t r = blockIdx.x;
    if (r == S.rank) return;
    const Origin* blk = og + (size_t)r * (cap + 1);
    const uint32_t prev = blk[0].source, cnt = blk[0].round;
    const uint32_t base = S.lorigin_base + r * S.lorigin_per;
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) S.origins[base + (prev + i) % S.lorigin_per] = blk[1 + i];
    if (cnt && threadIdx.x == 0) *S.dangerous = 1;
}
__device__ inline void pack_wire(const SimDev& S, const Change* src, uint32_t len, uint32_t* w, Esc* esc, Shared& sh) {
    if (threadIdx.x == 0) sh.u[5] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < len; i += BLOCK) {
        const Change c = load_msg(src + i);
        uint32_t word = c.origin;
        if (!(c.origin & ORIGIN_ALIVE)) {
            word = atomicAdd(&sh.u[5], 1u);  // escape order is immaterial: the word names it
            store_esc(S, esc + word, c);
        }
        w[i] = word;
    }
    __syncthreads();
}

// Outgoing ping bodies: one block per local sender with a remote target.
__global__ void __launch_bounds__(BLOCK) k_pack_pings(SimDev S, const uint64_t* soff, const uint64_t* seoff,
                                                      uint32_t* sendw, Esc* sende) {
    __shared__ Shared sh;
    const uint32_t A = S.lo + blockIdx.x;
    const int32_t T = S.target[A];
    if (T < 0 || S.local((uint32_t)T)) return;
    pack_wire(S, S.arena + S.msg_off[A], S.msg_plen[A], sendw + soff[A], sende + seoff[A], sh);
}

// Response records for remote senders (their targets are on this shard) and
// the words / escapes each carries: a list as written, a fullSync expanded in
// the responder's member order (lib/dissemination.js:61-76; all escapes).
// One block per partner; k_plan_fix_resp adds the segment bases.
__global__ void __launch_bounds__(XB) k_plan_resp(SimDev S, const uint32_t* rs_idx, RespRec* rsend, uint64_t* psoff,
                                                 uint64_t* pseoff, unsigned long long* cnt) {
    const uint32_t r = blockIdx.x, G = S.nranks;
    U3 t = {0, 0, 0};
    if (r != S.rank)
        t = tile_scan3(S.nl, [&](uint32_t i, U3& v) {
            const uint32_t A = r * S.nl + i;
            const int32_t T = S.target[A];
            if (T < 0 || !S.local((uint32_t)T)) return false;
            const Resp& x = S.resp[A];
            const uint32_t fsm = x.kind == RESP_FS ? S.snap_m[x.snap] : 0u;  // a fullSync: all the members
            v.a = x.kind == RESP_LIST ? x.plen : fsm;
            v.b = x.kind == RESP_LIST ? x.nesc : fsm;
            v.c = 0;
            RespRec rec;
            rec.kind = x.kind; rec.len = x.kind == RESP_FS ? fsm : x.len;
            rec.psize = (uint32_t)v.a; rec.pesc = (uint32_t)v.b;
            rsend[rs_idx[A]] = rec;
            return true;
        }, [&](uint32_t i, const U3& p) { const uint32_t A = r * S.nl + i; psoff[A] = p.a; pseoff[A] = p.b; });
    if (threadIdx.x == 0) { cnt[XC_PAY_SEND * G + r] = t.a; cnt[XC_RESC_SEND * G + r] = t.b; }
}
__global__ void k_plan_fix_resp(SimDev S, uint64_t* psoff, uint64_t* pseoff, const unsigned long long* cnt) {
    const uint32_t A = blockIdx.x * blockDim.x + threadIdx.x, G = S.nranks;
    if (A >= S.n || S.local(A)) return;
    const int32_t T = S.target[A];
    if (T < 0 || !S.local((uint32_t)T)) return;
    const uint32_t r = S.owner(A);
    psoff[A] += seg_base(cnt, XC_PAY_SEND, G, r);
    pseoff[A] += seg_base(cnt, XC_RESC_SEND, G, r);
}
__global__ void __launch_bounds__(BLOCK) k_pack_resp(SimDev S, const uint64_t* psoff, const uint64_t* pseoff,
                                                     uint32_t* psendw, Esc* psende) {
    __shared__ Shared sh;
    const uint32_t b = S.lo + blockIdx.x, n = S.n;
    for (uint32_t j = S.g_base[b]; j < S.g_base[b + 1]; j++) {
        const uint32_t A = S.g_list[j];
        if (S.local(A)) continue;
        const Resp r = S.resp[A];
        if (r.kind == RESP_LIST) {
            pack_wire(S, S.arena + r.off, r.plen, psendw + psoff[A], psende + pseoff[A], sh);
        } else if (r.kind == RESP_FS) {
            const uint32_t* ord = S.snap_ord + (size_t)r.snap * n;
            const uint64_t* snap = S.snaps + (size_t)r.snap * n;
            const uint32_t M = S.snap_m[r.snap];
            uint32_t* w = psendw + psoff[A];
            Esc* e = psende + pseoff[A];
            for (uint32_t i = threadIdx.x; i < M; i += BLOCK) {
                Change c;
                c.addr = ord[i]; c.origin = b; c.vs = snap[c.addr];  // fullSync origin: source b
                store_esc(S, e + i, c);
                w[i] = i;
            }
        }
    }
}
// Incoming response records -> resp[A] of local senders with a remote target;
// one block per partner q (segment bases from the all-gathered G x 2 x G
// payload counts, xrow[r][0 words | 1 escapes][receiver]).
__global__ void __launch_bounds__(XB) k_unpack_resp(SimDev S, const uint32_t* rr_idx, const RespRec* rrecv,
                                                   const unsigned long long* xrow) {
    const uint32_t q = blockIdx.x, me = S.rank, G = S.nranks;
    if (q == me) return;
    uint64_t wbase = 0, ebase = 0;
    for (uint32_t r = 0; r < q; r++) { wbase += xrow[(size_t)r * 2 * G + me]; ebase += xrow[(size_t)r * 2 * G + G + me]; }
    tile_scan3(S.nl, [&](uint32_t i, U3& v) {
        const uint32_t A = S.lo + i;
        const int32_t T = S.target[A];
        if (T < 0 || S.owner((uint32_t)T) != q) return false;
        const RespRec rec = rrecv[rr_idx[A]];
        v = U3{rec.psize, rec.pesc, 0};
        return true;
    }, [&](uint32_t i, const U3& p) {
        const uint32_t A = S.lo + i;
        const RespRec rec = rrecv[rr_idx[A]];
        Resp r{};
        r.from = (uint32_t)S.target[A]; r.snap = NONE; r.ping_status = 0;
        r.len = rec.len; r.plen = rec.psize; r.nesc = rec.pesc;
        r.kind = (rec.kind == RESP_LIST || rec.kind == RESP_FS) ? RESP_LIST_RX : rec.kind;
        r.off = wbase + p.a;
        r.eoff = (uint32_t)(ebase + p.b);
        S.resp[A] = r;
    });
}

// Wire words -> changes, once per received ping body (the ping merges read
// every body in one format; the responses merge from the wire words).
__global__ void __launch_bounds__(BLOCK) k_expand_pings(SimDev S) {
    const uint32_t A = blockIdx.x;
    const int32_t T = S.target[A];
    if (S.local(A) || T < 0 || !S.local((uint32_t)T)) return;
    const uint32_t* w = S.rxw + S.rx_off[A];
    const Esc* e = S.rxe + S.rx_eoff[A];
    Change* out = S.rxc + S.rx_off[A];
    for (uint32_t i = threadIdx.x; i < S.msg_plen[A]; i += BLOCK) store_msg(out + i, wire_change(S, w[i], e));
}

// ---------------------------------------------------------------- ping-req waves across shards
// W3..W6 deliver one message per slot 3A+i (A's i-th ping-req): W3 A -> relay
// K (ping-req body), W4 K -> target T (relay ping) or K -> A (PingReqPingError),
// W5 T -> K (response to the relay ping), W6 K -> A (ping-req response).  A
// message whose destination lives on another shard travels as a SlotRec (the
// slot state its handler reads) plus its change list in wire format; the
// receiver installs the slot state and decodes the list into rxc (W3, W4,
// W5; W6 responses are merged from rx2w).  Unlike pings, the receiver cannot
// derive which slots will arrive, so the per-partner counts are all-gathered
// first.
struct SlotRec {
    uint32_t slot;
    int32_t dest;
    int32_t kind;         // W3: 0; W4: 1 = PingReqPingError back to A; W5/W6: Resp kind
    uint32_t len;         // the reference's list length
    uint32_t plen, nesc;  // entries shipped, and of those escapes
    uint32_t aux;         // W4: the relay K; W5/W6: the responder
    uint32_t csum;        // W3: A's checksum (its ping-req body); W4: K's
    uint32_t ping_status;
    uint32_t woff, eoff;  // payload offsets inside the partner segment
    uint32_t pad;
    uint64_t inc, fp;     // W3: A's incarnation / fingerprint; W4: K's
};
static_assert(sizeof(SlotRec) == 64, "slot record is 64 bytes");

// Does slot s carry a wave-W message from this shard to another?  Its
// destination, and the words / escapes of its list.
template <int W>
__device__ inline bool xs_out(const SimDev& S, uint32_t s, uint32_t& dest, uint32_t& words, uint32_t& esc) {
    const uint32_t n = S.n;
    int32_t d = -1;
    words = esc = 0;
    if (W == 3) {
        if (!S.local(s / 3)) return false;
        d = S.w3_dest[s];
        if (d >= 0) { words = S.pq_len[s]; esc = S.pq_nesc[s]; }
    } else if (W == 4) {
        const int32_t K = S.w3_dest[s];
        if (K < 0 || !S.local((uint32_t)K)) return false;
        d = S.w4_dest[s];
        if (d >= 0 && !S.w4_err[s]) { words = S.rl_len[s]; esc = S.rl_nesc[s]; }
    } else {
        d = W == 5 ? S.w5_dest[s] : S.w6_dest[s];
        if (d >= 0) {
            const Resp& r = S.resp[(W == 5 ? n : 4 * n) + s];
            if (r.kind == RESP_LIST) { words = r.plen; esc = r.nesc; }
            else if (r.kind == RESP_FS) { words = S.snap_m[r.snap]; esc = words; }
        }
    }
    if (d < 0 || S.local((uint32_t)d)) return false;
    dest = (uint32_t)d;
    return true;
}

// Record / word / escape offsets of the outgoing slots inside their
// partner's segments, and the segment totals (cnt's XS_*_SEND rows, zeroed by
// k_xs_zero).  One thread per slot; a block takes its partner ranges with one
// global atomic per (partner, counter) and hands them out through LDS
// atomics.  Placement inside a segment is therefore in no particular order:
// a record names its slot and its payload offsets, and the receiver handles
// each record on its own (k_xs_unpack).
template <int W>
__global__ void __launch_bounds__(256) k_xs_plan(SimDev S, uint32_t* xs_rec, uint32_t* xs_w, uint32_t* xs_e,
                                               unsigned long long* cnt) {
    __shared__ uint32_t lc[3][MAXG];
    __shared__ unsigned long long lb[3][MAXG];
    const uint32_t G = S.nranks, s = blockIdx.x * 256 + threadIdx.x;
    for (uint32_t i = threadIdx.x; i < 3 * G; i += 256) lc[i / G][i % G] = 0;
    __syncthreads();
    uint32_t d, w = 0, e = 0, q = NONE, r0 = 0, r1 = 0, r2 = 0;
    if (s < 3 * S.n && xs_out<W>(S, s, d, w, e)) {
        q = S.owner(d);
        r0 = atomicAdd(&lc[0][q], 1u);
        r1 = w ? atomicAdd(&lc[1][q], w) : 0u;
        r2 = e ? atomicAdd(&lc[2][q], e) : 0u;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 3 * G; i += 256) {
        const uint32_t c = i / G, qq = i % G, x = lc[c][qq];
        lb[c][qq] = x ? atomicAdd(&cnt[(XS_REC_SEND + 2 * c) * G + qq], (unsigned long long)x) : 0ull;
    }
    __syncthreads();
    if (q != NONE) {
        xs_rec[s] = (uint32_t)(lb[0][q] + r0);
        xs_w[s] = (uint32_t)(lb[1][q] + r1);
        xs_e[s] = (uint32_t)(lb[2][q] + r2);
    }
}
__global__ void k_xs_zero(unsigned long long* cnt, uint32_t G, uint32_t* nlist) {
    const uint32_t i = threadIdx.x;
    if (i < 3 * G) cnt[(XS_REC_SEND + 2 * (i / G)) * G + i % G] = 0;
    if (i == 0) *nlist = 0;
}

// One thread per slot: the outgoing records (at their segment positions) and
// the list of slots whose payload k_xs_pack writes; the shard's send counts
// go to its row of the all-gathered count matrix.
template <int W>
__global__ void k_xs_fill(SimDev S, const uint32_t* xs_rec, const uint32_t* xs_w, const uint32_t* xs_e,
                          const unsigned long long* cnt, SlotRec* xsend, uint64_t* xs_wabs, uint64_t* xs_eabs,
                          uint32_t* xs_list, uint32_t* xs_nlist, unsigned long long* xsrow) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x, n = S.n, G = S.nranks;
    if (s == 0)
        for (uint32_t q = 0; q < G; q++)
            for (int c = 0; c < 3; c++)
                xsrow[((size_t)S.rank * 3 + c) * G + q] = cnt[(XS_REC_SEND + 2 * c) * G + q];
    if (s >= 3 * n) return;
    uint32_t d, words, esc;
    if (!xs_out<W>(S, s, d, words, esc)) return;
    const uint32_t q = S.owner(d);
    SlotRec r{};
    r.slot = s; r.dest = (int32_t)d; r.plen = words; r.nesc = esc; r.woff = xs_w[s]; r.eoff = xs_e[s];
    if (W == 3) {
        const uint32_t A = s / 3;
        r.len = S.pq_len[s]; r.inc = S.pr_inc[A]; r.fp = S.pr_fp[A]; r.csum = S.pr_csum[A];
    } else if (W == 4) {
        r.kind = S.w4_err[s]; r.aux = (uint32_t)S.w3_dest[s];
        if (!r.kind) { r.len = S.rl_len[s]; r.inc = S.rl_inc[s]; r.fp = S.rl_fp[s]; r.csum = S.rl_csum[s]; }
    } else {
        const Resp& x = S.resp[(W == 5 ? n : 4 * n) + s];
        r.kind = x.kind; r.aux = x.from; r.len = x.kind == RESP_FS ? S.snap_m[x.snap] : x.len; r.ping_status = x.ping_status;
    }
    xsend[xs_rec[s] + seg_base(cnt, XS_REC_SEND, G, q)] = r;
    xs_wabs[s] = xs_w[s] + seg_base(cnt, XS_W_SEND, G, q);
    xs_eabs[s] = xs_e[s] + seg_base(cnt, XS_E_SEND, G, q);
    if (words) xs_list[atomicAdd(xs_nlist, 1u)] = s;
}

// Payloads of the outgoing slots with a list (one block per listed slot).
template <int W>
__global__ void __launch_bounds__(BLOCK) k_xs_pack(SimDev S, const uint32_t* xs_list, const uint64_t* xs_wabs,
                                                   const uint64_t* xs_eabs, uint32_t* sendw, Esc* sende) {
    __shared__ Shared sh;
    const uint32_t s = xs_list[blockIdx.x], n = S.n;
    uint32_t* w = sendw + xs_wabs[s];
    Esc* e = sende + xs_eabs[s];
    if (W == 3) {
        pack_wire(S, S.arena + S.pq_off[s], S.pq_len[s], w, e, sh);
    } else if (W == 4) {
        pack_wire(S, S.arena + S.rl_off[s], S.rl_len[s], w, e, sh);
    } else {
        const Resp r = S.resp[(W == 5 ? n : 4 * n) + s];
        if (r.kind == RESP_LIST) {
            pack_wire(S, S.arena + r.off, r.plen, w, e, sh);
        } else {  // RESP_FS: the responder's snapshot in its member order (lib/dissemination.js:61-76)
            const uint32_t b = r.from;
            const uint32_t* ord = S.snap_ord + (size_t)r.snap * n;
            const uint64_t* snap = S.snaps + (size_t)r.snap * n;
            const uint32_t M = S.snap_m[r.snap];
            for (uint32_t i = threadIdx.x; i < M; i += BLOCK) {
                Change c;
                c.addr = ord[i]; c.origin = b; c.vs = snap[c.addr];
                store_esc(S, e + i, c);
                w[i] = i;
            }
        }
    }
}

// Received records (one block each): install the slot state for the wave's
// handler and decode the list.  xsrow = the all-gathered send counts
// [shard][record | words | escapes][partner].
template <int W>
__global__ void __launch_bounds__(BLOCK) k_xs_unpack(SimDev S, const SlotRec* xrecv, const unsigned long long* xsrow,
                                                     const uint32_t* rxw, const Esc* rxe, Change* dec) {
    const uint32_t i = blockIdx.x, me = S.rank, G = S.nranks, n = S.n;
    uint64_t rb = 0, wb = 0, eb = 0;
    for (uint32_t r = 0; r < G; r++) {
        if (r == me) continue;
        const uint64_t c = xsrow[((size_t)r * 3 + 0) * G + me];
        if (i < rb + c) break;
        rb += c;
        wb += xsrow[((size_t)r * 3 + 1) * G + me];
        eb += xsrow[((size_t)r * 3 + 2) * G + me];
    }
    const SlotRec x = xrecv[i];
    const uint64_t woff = wb + x.woff, eoff = eb + x.eoff;
    const uint32_t s = x.slot;
    if (threadIdx.x == 0) {
        if (W == 3) {
            const uint32_t A = s / 3;
            S.w3_dest[s] = x.dest; S.pq_off[s] = RX_MSG | woff; S.pq_len[s] = x.len;
            S.pr_inc[A] = x.inc; S.pr_fp[A] = x.fp; S.pr_csum[A] = x.csum; S.pr_ckv[A] = 1;
        } else if (W == 4) {
            S.w4_dest[s] = x.dest; S.w4_err[s] = (uint8_t)x.kind; S.w3_dest[s] = (int32_t)x.aux;
            if (!x.kind) { S.rl_off[s] = RX_MSG | woff; S.rl_len[s] = x.len; S.rl_inc[s] = x.inc; S.rl_fp[s] = x.fp; S.rl_csum[s] = x.csum; }
        } else {
            Resp r{};
            r.kind = (x.kind == RESP_LIST || x.kind == RESP_FS) ? RESP_LIST_RX : x.kind;
            r.from = x.aux; r.off = woff; r.len = x.len; r.plen = x.plen; r.nesc = x.nesc; r.eoff = (uint32_t)eoff;
            r.snap = NONE; r.ping_status = x.ping_status;
            S.resp[(W == 5 ? n : 4 * n) + s] = r;
            if (W == 5) S.w5_dest[s] = x.dest; else S.w6_dest[s] = x.dest;
        }
    }
    // (W6 responses are merged from their wire words: apply_response)
    if (W <= 5)
        for (uint32_t j = threadIdx.x; j < x.plen; j += BLOCK) store_msg(dec + woff + j, wire_change(S, rxw[woff + j], rxe + eoff));
}

// Seen masks for other shards, step 1: per group of 1 << gsz_log local nodes,
// the AND of its live nodes' seen bitsets (valid for the ids the round
// tracked) into gseen[group].  grid (seen_words / 256, local groups)
__global__ void __launch_bounds__(256) k_seen_and(SimDev S, uint32_t* gseen) {
    const uint32_t w = blockIdx.x * 256 + threadIdx.x;
    if (w >= S.seen_words) return;
    const uint32_t g = (S.lo >> S.gsz_log) + blockIdx.y, v0 = g << S.gsz_log, v1 = v0 + (1u << S.gsz_log);
    uint32_t acc = 0xFFFFFFFFu;
    // (fail-stopped nodes receive nothing; a node still outside the cluster,
    // dead = 2, counts with its empty bitset: it may join before the mask is used)
    for (uint32_t v = v0; v < v1; v++)
        if (S.dead[v] != 1) acc &= S.seen[S.srow(v) + w];
    gseen[(size_t)g * S.seen_words + w] = acc;
}
// Settled masks for other shards (fault runs): per group of 1 << fs_log local
// nodes, the AND of their settled bits (fail-stopped nodes receive nothing; a
// node outside the cluster counts with its empty view).  A bit stays a valid
// filter after the round it was gathered in (view keys never decrease).
// grid (n/32 / 256, local groups)
__global__ void __launch_bounds__(256) k_settled_and(SimDev S, uint32_t* out) {
    const uint32_t pw = (S.n + 31) / 32, w = blockIdx.x * 256 + threadIdx.x;
    if (w >= pw) return;
    const uint32_t g = (S.lo >> S.fs_log) + blockIdx.y, v0 = g << S.fs_log, v1 = v0 + (1u << S.fs_log);
    uint32_t acc = 0xFFFFFFFFu;
    for (uint32_t v = v0; v < v1; v++)
        if (S.dead[v] != 1) acc &= settled_bits(S, v)[w];
    out[(size_t)g * pw + w] = acc;
}
// step 2 (after the all-gather of every shard's part into gseen): the masks
// are valid for the ids [olo, ohi) tracked this round
__global__ void k_seen_range(SimDev S) {
    const SeenWin win = seen_window(S);
    S.gs_range[0] = win.olo;
    S.gs_range[1] = win.ohi;
}

// Round statistics of every shard: [STAT_NSTATS counters, fp min, fp max] per
// shard -> global counters (waves: max), convergence, totals.
__global__ void k_stats_pack(SimDev S, const unsigned long long* fp_mm, unsigned long long* g,
                             unsigned long long* ltotals) {
    unsigned long long* mine = g + (size_t)S.rank * (STAT_NSTATS + 2);
    for (int i = threadIdx.x; i < STAT_NSTATS; i += blockDim.x) { mine[i] = S.stats[i]; ltotals[i] += S.stats[i]; }
    if (threadIdx.x == 0) { mine[STAT_NSTATS] = fp_mm[0]; mine[STAT_NSTATS + 1] = fp_mm[1]; }
}
__global__ void k_stats_combine(SimDev S, const unsigned long long* g, unsigned long long* totals) {
    if (threadIdx.x != 0) return;
    unsigned long long lo = ~0ull, hi = 0;
    for (int i = 0; i < STAT_NSTATS; i++) {
        unsigned long long acc = 0;
        for (uint32_t r = 0; r < S.nranks; r++) {
            const unsigned long long x = g[(size_t)r * (STAT_NSTATS + 2) + i];
            acc = i == STAT_WAVES ? (x > acc ? x : acc) : acc + x;
        }
        S.stats[i] = acc;
        totals[i] += acc;
    }
    for (uint32_t r = 0; r < S.nranks; r++) {
        const unsigned long long a = g[(size_t)r * (STAT_NSTATS + 2) + STAT_NSTATS];
        const unsigned long long b = g[(size_t)r * (STAT_NSTATS + 2) + STAT_NSTATS + 1];
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    const bool conv = lo >= hi;
    *S.conv = conv ? 1u : 0u;
    totals[STAT_NSTATS] += conv ? 1ull : 0ull;
}

}  // namespace rp

// =====================================================================
// Host side: rp_sim objects and their C ABI.
// =====================================================================
#include <rccl/rccl.h>

#include <map>
#include <memory>

#include "rp_internal.h"

namespace {

using rp::Change;
using rp::DevBuf;
using rp::Error;

constexpr int NCAT = 7;  // churn, issue, merge_ping, merge_resp, checksum, other, exchange
#ifndef RP_CK_SIDE
#define RP_CK_SIDE 1  // one shard: the round's sender checksums and fullSync decisions on a side stream
#endif
#ifndef RP_CK_SIDE_MB
#define RP_CK_SIDE_MB 4096  // the side stream's leader view copies (config 5 at 65,536: 8,192 rows of 512 KB,
                           // enough for the mass failure's first rounds)
#endif
constexpr uint32_t CHURN_SLOTS = 1024;  // rounds of churn ids staged per copy

struct TimedSpan {
    int cat;
    hipEvent_t a, b;
};


struct Shard {
    rp_sim_config cfg{};
    uint32_t n = 0, k = 0;
    uint32_t lo = 0, nl = 0, rank = 0, G = 1;  // this shard holds nodes [lo, lo + nl) of G shards
    bool one_per_process = false;  // exchanges over RCCL (rp_sim_create_rank)
    hipStream_t st = nullptr;
    bool own_stream = false;
    hipEvent_t xev = nullptr;  // in-process clusters: this shard's stream reached an exchange step
    rp::SimDev d{};
    DevBuf<rp::VEnt> view;
    DevBuf<uint64_t> fp, rng, snd_inc, snd_fp, msg_off, snaps, pr_inc, pr_fp, pq_off, rl_off, rl_inc, rl_fp;
    DevBuf<uint32_t> mcount, snap_ord, snap_m;
    DevBuf<uint32_t> order, dhead, dtail, csum, csum_valid, addr_words, msg_len, msg_plen, snd_csum, g_cnt, g_fill, g_base,
        g_list, snap_count, pend_slot, pend_csum, origin_count, err, conv, pr_n, pr_errors, pr_bad, pr_done, pr_csum,
        pq_len, rl_len, rl_csum, thead, ttail;
    DevBuf<Change> arena;
    DevBuf<uint32_t> dko;
    DevBuf<uint32_t> dad;
    DevBuf<uint32_t> p2_list, p2_len;  // k_p2_lists: receivers per ping rank
    DevBuf<uint64_t> p2_msg;           // ... and their pings' bodies (k_p2_apply)
    DevBuf<rp::P2Rec> p2_rec;          // k_p2_pre: one rank's respond records (k_p2_respond)
    DevBuf<uint64_t> dvs;
    DevBuf<rp::Resp> resp;
    DevBuf<uint2> tfifo;
    DevBuf<int32_t> storm;  // CHURN_SLOTS x 2 x storm_kmax: per round, accusers then victims (k_storm)
    uint32_t storm_kmax = 0;
    DevBuf<int32_t> max_pb, ring_count, coll_owner, coll_of, iter_index, iter_round, npingable, target, churn_ids,
        pt_server, pt_coll, w3_dest, w4_dest, w5_dest, w6_dest, dead_ids;
    DevBuf<uint64_t> sv_word;  // k_phase1: same-view decisions
    DevBuf<uint8_t> in_ring, dead, addr_len, need_shuffle, need_csum, pend_done, w4_err;
    DevBuf<uint32_t> shuf_list, shuf_count, g_tile, g_bloc;  // k_iterate: nodes whose iterator wrapped this round
    DevBuf<uint64_t> min_l1, min_l2;
    DevBuf<uint32_t> min_safe, min_cnt, dangerous, dlive, icount, seen, oc_snap, coll_off, coll_ids, rbatch, self_origin;
    DevBuf<uint32_t> cmem_off, cmem;  // per collision group, its servers (ascending): rp_sim_set_views' ring owners
    DevBuf<uint64_t> self_inc;
    DevBuf<int64_t> slen;
    DevBuf<uint32_t> ck_list, ck_count;  // views queued for k_checksums
    DevBuf<unsigned long long> hkey;       // Shard::checksums: fingerprint table
    DevBuf<uint32_t> hval, ck_lead, ck_nlead, ck_slot;
    DevBuf<rp::CkEntry> ck_cache;
    // the round's sender checksums and fullSync decisions on a side stream
    // (one shard: k_ck_snapcopy, k_checksums_snap beside the ping merge,
    // k_pending beside the response merge's pass 1)
    bool ck_side = false;                      // the side stream exists (one shard)
    // ... and this round uses it: fault runs (fail-stops, storms, partitions),
    // whose distinct views make the checksum stage a few hundred long chains;
    // without faults the stage is a handful of short ones and splitting the
    // response merge around k_pending costs more than it hides
    bool side_round() const { return ck_side && fault_mode; }
    hipStream_t st2 = nullptr;
    hipEvent_t ev_ck_copy = nullptr, ev_ck_done = nullptr, ev_merge_done = nullptr, ev_pend_done = nullptr;
    uint32_t ck_cap = 0;                       // leader rows of the snapshot
    DevBuf<uint64_t> ck_rows;                  // ck_cap x n view values
    DevBuf<unsigned long long> ck_lfp;         // the leaders' fingerprints
    DevBuf<uint32_t> ck_lres, ck_hlead;        // their checksums; leader index by fingerprint slot
    double side_ms = 0;                        // device time of the side stream's work (timing on)
    std::vector<TimedSpan> side_spans;
    DevBuf<rp::Origin> origins;
    DevBuf<unsigned long long> arena_cursor, stats, totals, fp_mm, bstats;
    DevBuf<uint32_t> pt_hash;
    // exchange (G > 1)
    DevBuf<rp::PingMeta> meta;
    DevBuf<uint64_t> soff, seoff, psoff, pseoff, rx_off, rx_eoff;
    DevBuf<uint32_t> rr_idx, rs_idx, msg_nesc;
    DevBuf<rp::RespRec> rsend, rrecv;
    DevBuf<uint32_t> sendw, rxw, psendw, rx2w;  // cross-shard messages: words ...
    DevBuf<rp::Esc> sende, rxe, psende, rx2e;  // ... and escapes (SimDev::rxw)
    DevBuf<Change> rxc;                         // received pings, W3-W5 lists decoded (responses, W6: from rx2w)
    DevBuf<unsigned long long> xcnt, sgather, xrow, ltotals;  // ltotals: this shard's own counters
    DevBuf<uint32_t> gseen, gs_range, gsettled;
    // ping-req waves across shards (k_xs_*)
    DevBuf<uint8_t> pr_ckv;
    DevBuf<uint32_t> w3cnt, w4b;  // k_pr_need's per-relay bounds
    DevBuf<uint32_t> fdecl_bits, fdecl_count;
    DevBuf<uint32_t> fdecl_all;  // G: every shard's k_fdecl_share, all-gathered (sharded fault rounds)
    bool fd_shared = false;      // fdecl_all holds this round's counts
    // a view may hold faulty or leave members no k_timers declared (views set
    // from given statuses, changes applied through the node bridge): k_pr_need
    // then bounds its relays' ring shrink by all n (k_pr_hist)
    bool faulty_unbounded = false;
    DevBuf<uint32_t> pq_nesc, rl_nesc, xs_rec, xs_w, xs_e, xs_list, xs_nlist, lorigin_count, lorigin_sent;
    DevBuf<rp::Origin> og;  // origin all-gather: G blocks of 1 + og_cap records (k_origin_pack)
    uint32_t og_cap = 0;
    DevBuf<uint64_t> xs_wabs, xs_eabs;
    DevBuf<rp::SlotRec> xsend, xrecv;
    DevBuf<unsigned long long> xsrow;
    unsigned long long* h_xsrow = nullptr;  // pinned: the all-gathered G x 3 x G send counts, then the pack count
    unsigned long long* h_xcnt = nullptr;  // pinned: XC_NCAT x G counts of the round
    unsigned long long* h_xrow = nullptr;  // pinned: G x 2 x G response payload counts (words, escapes)
    uint32_t npts = 0, ncoll = 0, seen_words = 0;
    bool join_mode = false;  // views may lack members: the JOIN merge kernels
    bool fault_mode = false;  // fail-stops, storms or partitions scheduled: the settled-filter issue kernels
    // join replies of a round (rp_sim_join): per pair its seed's view, member
    // order / count and checksum (filled on the seed's shard, then shared)
    DevBuf<uint64_t> jvs;
    DevBuf<uint32_t> jord, jm, jcs, j_ids, j_poff, j_pidx, j_pjoin, j_seedof;
    DevBuf<int32_t> j_pseed;
    std::vector<std::string> addrs;  // in sort order; preset by rp_sim_load_addresses, else the sim scheme
    uint32_t timing = 0;  // bit cat: stage cat's spans are timed (rp_sim_enable_timing_stages)
    uint64_t xsent = 0;  // bytes this shard sent to other shards (all-gathers, all-to-alls, all-reduces) since enable_timing
    std::vector<TimedSpan> spans;
    std::vector<hipEvent_t> ev_pool;  // recorded and collected events, reused (an event create costs a driver call)
    double kms[NCAT] = {0, 0, 0, 0, 0, 0, 0};
    uint64_t klaunch[NCAT] = {0, 0, 0, 0, 0, 0, 0};

    ~Shard() {
        for (auto& s : spans) { (void)hipEventDestroy(s.a); (void)hipEventDestroy(s.b); }
        for (auto e : ev_pool) (void)hipEventDestroy(e);
        if (h_xcnt) (void)hipHostFree(h_xcnt);
        if (h_xrow) (void)hipHostFree(h_xrow);
        if (h_xsrow) (void)hipHostFree(h_xsrow);
        if (xev) (void)hipEventDestroy(xev);
        for (hipEvent_t e : {ev_ck_copy, ev_ck_done, ev_merge_done, ev_pend_done})
            if (e) (void)hipEventDestroy(e);
        for (auto& sp : side_spans) { (void)hipEventDestroy(sp.a); (void)hipEventDestroy(sp.b); }
        if (st2) (void)hipStreamDestroy(st2);
        if (st && own_stream) (void)hipStreamDestroy(st);
    }
    // side-stream work, timed on its own stream (kernel_ms "checksum_side")
    template <class F>
    void side_timed(F&& launch) {
        if (!((timing >> 4) & 1u)) { launch(); return; }
        TimedSpan sp{4, take_event(), take_event()};
        RP_HIP(hipEventRecord(sp.a, st2));
        launch();
        RP_HIP(hipEventRecord(sp.b, st2));
        side_spans.push_back(sp);
    }

    template <class F>
    void timed(int cat, F&& launch) {
        if (!((timing >> cat) & 1u)) { launch(); return; }
        TimedSpan s{cat, take_event(), take_event()};
        RP_HIP(hipEventRecord(s.a, st));
        launch();
        RP_HIP(hipEventRecord(s.b, st));
        spans.push_back(s);
    }
    void collect_timing() {
        for (auto& s : spans) {
            float ms = 0;
            RP_HIP(hipEventElapsedTime(&ms, s.a, s.b));
            kms[s.cat] += ms;
            klaunch[s.cat]++;
            ev_pool.push_back(s.a);
            ev_pool.push_back(s.b);
        }
        spans.clear();
        for (auto& sp : side_spans) {
            float ms = 0;
            RP_HIP(hipEventElapsedTime(&ms, sp.a, sp.b));
            side_ms += ms;
            ev_pool.push_back(sp.a);
            ev_pool.push_back(sp.b);
        }
        side_spans.clear();
    }
    // buffer resets queued for one k_fill_batch launch (fill_flush)
    std::vector<rp::FillDesc> fills;
    void fill(void* dst, uint64_t bytes, uint8_t byte) {
        if (bytes % 4) throw Error(RP_ERR_STATE, "fill: size not a multiple of 4");
        if (bytes) fills.push_back(rp::FillDesc{dst, bytes, byte * 0x01010101u, 0});
    }
    // seen_clear: the last batch also clears the round's seen bits (k_round_start)
    void fill_flush(bool seen_clear = false) {
        for (size_t i0 = 0; i0 < fills.size() || (seen_clear && i0 == 0); i0 += rp::FILL_BATCH) {
            rp::FillBatch b{};
            b.n = (uint32_t)std::min<size_t>(rp::FILL_BATCH, fills.size() - i0);
            uint64_t mx = 0;
            for (uint32_t j = 0; j < b.n; j++) { b.d[j] = fills[i0 + j]; mx = std::max<uint64_t>(mx, b.d[j].bytes); }
            const uint32_t gx = (uint32_t)std::min<uint64_t>(256, std::max<uint64_t>(1, (mx / 4 + 255) / 256));
            if (seen_clear && i0 + rp::FILL_BATCH >= fills.size())
                hipLaunchKernelGGL(rp::k_round_start, dim3(gx * b.n + (nl + 3) / 4), dim3(256), 0, st, b, gx, d);
            else
                hipLaunchKernelGGL(rp::k_fill_batch, dim3(gx, b.n), dim3(256), 0, st, b);
        }
        fills.clear();
    }
    hipEvent_t take_event() {
        hipEvent_t e = nullptr;
        if (!ev_pool.empty()) { e = ev_pool.back(); ev_pool.pop_back(); return e; }
        RP_HIP(hipEventCreate(&e));
        return e;
    }

    void setup();
    // prefilled: counts reset by stage_start; counted: and counted already (k_phase1, one shard)
    void group(const int32_t* dest, uint32_t nslots, bool prefilled = false, bool counted = false);
    // the pending fullSync decisions (k_pending)
    void launch_pending(hipStream_t s) {
        hipLaunchKernelGGL(rp::k_pending, dim3(std::min(rp::grid_for(d.snap_cap, rp::NWAVE), 8192u)), dim3(rp::BLOCK), 0,
                           s, d);
    }
    // one round = these stages in order; a cluster exchanges between them
    void stage_start(uint32_t round, bool churn_active, uint32_t slot, const std::vector<int32_t>& dead_now,
                     bool faults, const uint32_t part[3], uint32_t storm_k);
    void stage_churn(bool churn_active, uint32_t slot, uint32_t storm_k, uint64_t now);
    // the set() bootstrap of nodes [node_lo, node_lo + count) from views (st/inc
    // rows, or every member of member_map alive at INC0 + id) (rp_sim_set_views)
    void bootstrap_views(uint32_t node_lo, uint32_t count, const uint8_t* st, const uint64_t* inc,
                         const uint8_t* member_map, uint64_t seed);
    void stage_issue();
    void stage_checksums();
    void stage_ping_merge(uint64_t now);
    void stage_resp_merge(uint64_t now, bool faults);
    void stage_pr_need();
    void stage_wave(int w, uint64_t now);  // ping-req waves W3..W6 (faults)
    void checksums(uint32_t* out, bool prefilled = false);  // ck_list's views -> out[v] (and the cache), one per distinct view
    void ensure_ck_side();                 // the side stream's leader rows (allocated when faults are scheduled)
    void checksums_side(uint32_t* out, bool prefilled = false);  // the same, the chains on st2 (ck_side; ready at ev_ck_done)
    // exchange buffers sized to a round's traffic (escapes dominate once
    // suspect/faulty updates circulate); direction 0: pings and W3/W4,
    // 1: responses and W5/W6
    void fit_exchange(int dir, uint64_t send_w, uint64_t send_e, uint64_t recv_w, uint64_t recv_e);
    // every exchange buffer to at least e elements (rp_sim::presize_exchange)
    void presize(uint64_t e) {
        for (auto* b : {&sendw, &rxw, &psendw, &rx2w}) b->reserve(e);
        for (auto* b : {&sende, &rxe, &psende, &rx2e}) b->reserve(e);
        rxc.reserve(e);
        d.rxw = rxw.p; d.rxe = rxe.p; d.rx2w = rx2w.p; d.rx2e = rx2e.p; d.rxc = rxc.p;
    }
    uint64_t xsum(int cat) const {
        uint64_t t = 0;
        for (uint32_t q = 0; q < G; q++) t += h_xcnt[(size_t)cat * G + q];
        return t;
    }
    void stage_end();
    uint32_t read_err();
};

// Every device pointer the round kernels dereference unconditionally, checked
// on the host before the first launch: a field added to SimDev and never
// assigned is an error here, not a fault on the device.
static void check_simdev(const rp::SimDev& d) {
    const struct { const char* name; const void* p; } req[] = {
        {"view", d.view},
        {"order", d.order},
        {"dko", d.dko},
        {"dvs", d.dvs},
        {"dad", d.dad},
        {"dhead", d.dhead},
        {"dtail", d.dtail},
        {"dlive", d.dlive},
        {"icount", d.icount},
        {"max_pb", d.max_pb},
        {"in_ring", d.in_ring},
        {"ring_count", d.ring_count},
        {"rbatch", d.rbatch},
        {"fp", d.fp},
        {"slen", d.slen},
        {"csum", d.csum},
        {"csum_valid", d.csum_valid},
        {"iter_index", d.iter_index},
        {"iter_round", d.iter_round},
        {"npingable", d.npingable},
        {"mcount", d.mcount},
        {"rng", d.rng},
        {"dead", d.dead},
        {"origins", d.origins},
        {"origin_count", d.origin_count},
        {"self_origin", d.self_origin},
        {"lorigin_count", d.lorigin_count},
        {"lorigin_sent", d.lorigin_sent},
        {"self_inc", d.self_inc},
        {"ck_list", d.ck_list},
        {"ck_count", d.ck_count},
        {"seen", d.seen},
        {"oc_snap", d.oc_snap},
        {"gseen", d.gseen},
        {"gs_range", d.gs_range},
        {"addr_words", d.addr_words},
        {"addr_len", d.addr_len},
        {"arena", d.arena},
        {"arena_cursor", d.arena_cursor},
        {"msg_off", d.msg_off},
        {"msg_nesc", d.msg_nesc},
        {"msg_len", d.msg_len},
        {"msg_plen", d.msg_plen},
        {"target", d.target},
        {"sv_word", d.sv_word},
        {"snd_inc", d.snd_inc},
        {"snd_fp", d.snd_fp},
        {"snd_csum", d.snd_csum},
        {"need_csum", d.need_csum},
        {"min_cnt", d.min_cnt},
        {"min_safe", d.min_safe},
        {"min_l1", d.min_l1},
        {"min_l2", d.min_l2},
        {"dangerous", d.dangerous},
        {"g_cnt", d.g_cnt},
        {"g_fill", d.g_fill},
        {"g_base", d.g_base},
        {"g_list", d.g_list},
        {"resp", d.resp},
        {"snaps", d.snaps},
        {"snap_ord", d.snap_ord},
        {"snap_m", d.snap_m},
        {"snap_count", d.snap_count},
        {"pend_slot", d.pend_slot},
        {"pend_csum", d.pend_csum},
        {"pend_done", d.pend_done},
        {"pr_n", d.pr_n},
        {"pr_errors", d.pr_errors},
        {"pr_bad", d.pr_bad},
        {"pr_done", d.pr_done},
        {"pr_inc", d.pr_inc},
        {"pr_fp", d.pr_fp},
        {"pr_csum", d.pr_csum},
        {"pr_ckv", d.pr_ckv},
        {"fdecl_bits", d.fdecl_bits},
        {"fdecl_count", d.fdecl_count},
        {"w3_dest", d.w3_dest},
        {"w4_dest", d.w4_dest},
        {"w5_dest", d.w5_dest},
        {"w6_dest", d.w6_dest},
        {"w4_err", d.w4_err},
        {"pq_off", d.pq_off},
        {"pq_len", d.pq_len},
        {"pq_nesc", d.pq_nesc},
        {"rl_off", d.rl_off},
        {"rl_len", d.rl_len},
        {"rl_nesc", d.rl_nesc},
        {"rl_inc", d.rl_inc},
        {"rl_fp", d.rl_fp},
        {"rl_csum", d.rl_csum},
        {"tfifo", d.tfifo},
        {"thead", d.thead},
        {"ttail", d.ttail},
        {"stats", d.stats},
        {"bstats", d.bstats},
        {"err", d.err},
        {"conv", d.conv},
    };
    for (const auto& r : req)
        if (!r.p) throw Error(RP_ERR_STATE, std::string("SimDev.") + r.name + " not allocated");
}

void Shard::setup() {
    using namespace rp;
    n = cfg.n;
    k = std::min(cfg.churn_k, n);
    RP_HIP(hipSetDevice(rp::current_device()));
    if (!st) { RP_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking)); own_stream = true; }
    if (!xev) RP_HIP(hipEventCreateWithFlags(&xev, hipEventDisableTiming));

    // addresses 10.<b2>.<b1>.<b0>:<3000+i%7> unless loaded (rp_sim_load_addresses);
    // ids = ranks in sort order, so a view row indexed by id is in checksum order
    if (addrs.empty()) {
        addrs.resize(n);
        for (uint32_t i = 0; i < n; i++) {
            char b[40];
            snprintf(b, sizeof b, "10.%u.%u.%u:%u", (i >> 16) & 255u, (i >> 8) & 255u, i & 255u, 3000u + i % 7u);
            addrs[i] = b;
        }
        std::sort(addrs.begin(), addrs.end());
    }
    if (addrs.size() != n) throw Error(RP_ERR_INVALID, "address count differs from the cluster size");
    std::vector<uint32_t> words((size_t)n * rp::ADDR_WORDS, 0);
    std::vector<uint8_t> lens(n);
    std::string blob;
    std::vector<uint64_t> off{0};
    for (uint32_t i = 0; i < n; i++) {
        const std::string& a = addrs[i];
        if (a.empty() || a.size() > 4 * rp::ADDR_WORDS) throw Error(RP_ERR_INVALID, "address length must be 1..32 bytes");
        lens[i] = (uint8_t)a.size();
        memcpy(&words[(size_t)i * rp::ADDR_WORDS], a.data(), a.size());
        blob += a;
        off.push_back(blob.size());
    }

    // replica points hash32(address + i) and the hash values shared by more
    // than one server (rbtree collisions, lib/rbtree.js:112-117)
    std::vector<uint32_t> rep;
    rp::device_replica_hashes(blob, off, REPLICAS, rep, st);
    if (cfg.replica_hash_shift)
        for (auto& h : rep) h = (h >> cfg.replica_hash_shift) << cfg.replica_hash_shift;
    struct P { uint32_t h, s, r; };
    std::vector<P> pts((size_t)n * REPLICAS);
    for (size_t t = 0; t < pts.size(); t++) pts[t] = {rep[t], (uint32_t)(t / REPLICAS), (uint32_t)(t % REPLICAS)};
    std::sort(pts.begin(), pts.end(), [](const P& a, const P& b) {
        return a.h != b.h ? a.h < b.h : a.s != b.s ? a.s < b.s : a.r < b.r;
    });
    std::vector<int32_t> h_coll_of(pts.size(), -1), coll_min;
    std::vector<uint32_t> h_pt_hash;
    std::vector<int32_t> h_pt_server, h_pt_coll;
    for (size_t i = 0; i < pts.size();) {
        size_t j = i;
        bool multi = false;
        while (j < pts.size() && pts[j].h == pts[i].h) { multi |= pts[j].s != pts[i].s; j++; }
        int32_t cid = -1;
        if (multi) {
            cid = (int32_t)coll_min.size();
            coll_min.push_back((int32_t)pts[i].s);  // smallest server id generating it
            for (size_t q = i; q < j; q++) h_coll_of[(size_t)pts[q].s * REPLICAS + pts[q].r] = cid;
        }
        h_pt_hash.push_back(pts[i].h);
        h_pt_server.push_back((int32_t)pts[i].s);
        h_pt_coll.push_back(cid);
        i = j;
    }
    ncoll = (uint32_t)coll_min.size();
    std::vector<uint32_t> h_coll_off(n + 1, 0), h_coll_ids;
    std::vector<uint32_t> h_cmem_off(ncoll + 1, 0), h_cmem;
    for (uint32_t sv = 0; sv < n; sv++) {
        for (int r = 0; r < REPLICAS; r++)
            if (h_coll_of[(size_t)sv * REPLICAS + r] >= 0) {
                h_coll_ids.push_back((uint32_t)h_coll_of[(size_t)sv * REPLICAS + r]);
                h_cmem_off[h_coll_of[(size_t)sv * REPLICAS + r] + 1]++;
            }
        h_coll_off[sv + 1] = (uint32_t)h_coll_ids.size();
    }
    for (uint32_t g = 0; g < ncoll; g++) h_cmem_off[g + 1] += h_cmem_off[g];
    {
        // servers of each group in ascending id (a server with two replicas in
        // one group is listed twice: harmless for a minimum)
        std::vector<uint32_t> fill(h_cmem_off.begin(), h_cmem_off.end() - 1);
        h_cmem.resize(h_cmem_off[ncoll]);
        for (uint32_t sv = 0; sv < n; sv++)
            for (uint32_t q = h_coll_off[sv]; q < h_coll_off[sv + 1]; q++) h_cmem[fill[h_coll_ids[q]]++] = sv;
    }
    npts = (uint32_t)h_pt_hash.size();

    const uint64_t nn = (uint64_t)nl * n;  // rows of this shard's nodes
    view.alloc(nn); order.alloc(nn); dko.alloc(nn); dvs.alloc(nn); dad.alloc(nn); in_ring.alloc(nn);
    RP_HIP(hipMemsetD32Async((hipDeviceptr_t)dko.p, rp::TOMB_WORD, nn, st));  // every log slot starts deleted
    dhead.alloc(n); dtail.alloc(n); max_pb.alloc(n); ring_count.alloc(n);
    coll_owner.alloc(std::max<uint64_t>((uint64_t)nl * ncoll, 1)); coll_of.alloc(h_coll_of.size());
    coll_off.alloc(n + 1); coll_ids.alloc(std::max<size_t>(h_coll_ids.size(), 1)); rbatch.alloc(n);
    self_origin.alloc(n);
    RP_HIP(hipMemsetAsync(self_origin.p, 0xFF, n * 4, st));
    RP_HIP(hipMemsetAsync(rbatch.p, 0, n * 4, st));
    RP_HIP(hipMemcpyAsync(coll_off.p, h_coll_off.data(), (n + 1) * 4, hipMemcpyHostToDevice, st));
    if (!h_coll_ids.empty())
        RP_HIP(hipMemcpyAsync(coll_ids.p, h_coll_ids.data(), h_coll_ids.size() * 4, hipMemcpyHostToDevice, st));
    cmem_off.alloc(ncoll + 1); cmem.alloc(std::max<size_t>(h_cmem.size(), 1));
    RP_HIP(hipMemcpyAsync(cmem_off.p, h_cmem_off.data(), (ncoll + 1) * 4, hipMemcpyHostToDevice, st));
    if (!h_cmem.empty()) RP_HIP(hipMemcpyAsync(cmem.p, h_cmem.data(), h_cmem.size() * 4, hipMemcpyHostToDevice, st));
    fp.alloc(n); csum.alloc(n); csum_valid.alloc(n); iter_index.alloc(n); iter_round.alloc(n); npingable.alloc(n); mcount.alloc(n);
    rng.alloc(n); dead.alloc(n);
    // (table slots stay below ORIGIN_ID_MASK, the log's tombstone id)
    uint32_t ocap = cfg.origin_slots ? cfg.origin_slots : rp::ORIGIN_ID_MASK;
    if (ocap > rp::ORIGIN_ID_MASK) throw Error(RP_ERR_INVALID, "origin_slots must be < 2^23");
    if (ocap < n + 16) ocap = n + 16;
    origins.alloc(ocap); origin_count.alloc(1);
    // the top quarter of the table: local suspect/faulty origins, one range per
    // shard; below it from n + 1: the ring of makeAlive origins (a power of two)
    const uint32_t lper = (ocap / 4) / G;
    if (lper < 16) throw Error(RP_ERR_INVALID, "origin_slots too small");
    const uint32_t lbase = ocap - lper * G;
    if (lbase < n + 1 + 64) throw Error(RP_ERR_INVALID, "origin_slots too small");
    uint32_t alive_cap = 64;
    while (alive_cap * 2 <= lbase - (n + 1)) alive_cap *= 2;
    lorigin_count.alloc(1); lorigin_sent.alloc(1);
    RP_HIP(hipMemsetAsync(lorigin_count.p, 0, 4, st));
    RP_HIP(hipMemsetAsync(lorigin_sent.p, 0, 4, st));
    if (G > 1) {
        // at most a few local origins per node between two all-gathers (one
        // per incarnation; a churn between a round's timers and its storm
        // makes two)
        og_cap = 2 * nl + 64;
        og.alloc((size_t)G * (og_cap + 1));
    }
    addr_words.alloc(words.size()); addr_len.alloc(((size_t)n + 3) & ~(size_t)3);  // (whole words: k_checksums_pc reads lengths by the word)
    uint64_t acap = cfg.arena_entries ? cfg.arena_entries : std::max<uint64_t>(1ull << 22, (uint64_t)nl * 16384);
    if (acap / rp::ARENA_SHARDS >= (1ull << 32)) throw Error(RP_ERR_CAPACITY, "message arena slice above 2^32 changes");
    arena.alloc(acap); arena_cursor.alloc(16 * rp::ARENA_SHARDS);
    bstats.alloc((size_t)rp::STAT_NSTATS * n);
    RP_HIP(hipMemsetAsync(bstats.p, 0, bstats.bytes(), st));
    msg_off.alloc(n); msg_len.alloc(n); msg_plen.alloc(n); target.alloc(n); sv_word.alloc(n); snd_inc.alloc(n); snd_fp.alloc(n); snd_csum.alloc(n);
    RP_HIP(hipMemsetAsync(snd_fp.p, 0xFF, snd_fp.bytes(), st));  // FP_NONE until a node's first ping
    g_cnt.alloc(n); g_fill.alloc(n); g_base.alloc(n + 1); g_list.alloc(3 * (size_t)n); g_tile.alloc((n + 1023) / 1024); g_bloc.alloc(n + 1);
    p2_list.alloc((size_t)(2 * rp::P2_SPLIT + 1) * nl); p2_msg.alloc((size_t)2 * rp::P2_SPLIT * nl); p2_len.alloc(rp::P2_SPLIT + 1);
    p2_rec.alloc(nl);
    resp.alloc(7 * (size_t)n);
    // full-sync snapshots: a shard's share of 4,096 (fullSync replies are rare)
    uint32_t scap = cfg.snapshot_slots ? cfg.snapshot_slots : std::min<uint32_t>(n, std::max<uint32_t>(4096 / G, 512));
    snaps.alloc((uint64_t)scap * n); snap_ord.alloc((uint64_t)scap * n); snap_m.alloc(scap); snap_count.alloc(1); pend_slot.alloc(scap); pend_csum.alloc(scap);
    pend_done.alloc((scap + 3u) & ~3u);  // (whole words: the round's fill batch clears it)
    pr_n.alloc(n); pr_errors.alloc(n); pr_bad.alloc(n); pr_done.alloc(n); pr_inc.alloc(n); pr_fp.alloc(n);
    pr_csum.alloc(n);
    const size_t n3 = 3 * (size_t)n;
    w3_dest.alloc(n3); w4_dest.alloc(n3); w5_dest.alloc(n3); w6_dest.alloc(n3); w4_err.alloc(n3);
    pq_nesc.alloc(n3); rl_nesc.alloc(n3);
    pr_ckv.alloc(n); w3cnt.alloc(n + 1); w4b.alloc(n);  // (w3cnt[n]: k_pr_hist's faulty count)
    fdecl_bits.alloc((n + 31) / 32); fdecl_count.alloc(1); fdecl_all.alloc(G);
    RP_HIP(hipMemsetAsync(fdecl_bits.p, 0, fdecl_bits.bytes(), st));
    RP_HIP(hipMemsetAsync(fdecl_count.p, 0, 4, st));
    pq_off.alloc(n3); pq_len.alloc(n3); rl_off.alloc(n3); rl_len.alloc(n3); rl_inc.alloc(n3); rl_fp.alloc(n3);
    rl_csum.alloc(n3);
    const uint32_t tcap = std::min<uint32_t>(n, 16384);
    tfifo.alloc((size_t)nl * tcap); thead.alloc(n); ttail.alloc(n);
    RP_HIP(hipMemsetAsync(thead.p, 0, n * 4, st));
    RP_HIP(hipMemsetAsync(ttail.p, 0, n * 4, st));
    dead_ids.alloc(n);
    churn_ids.alloc((size_t)CHURN_SLOTS * std::max<uint32_t>(k, 1));
    stats.alloc(rp::STAT_NSTATS); totals.alloc(rp::STAT_NSTATS + 1); fp_mm.alloc(2);
    err.alloc(1); conv.alloc(1);
    need_csum.alloc(n); min_cnt.alloc(n); min_safe.alloc(n); min_l1.alloc(n); min_l2.alloc(n); dangerous.alloc(1); dlive.alloc(n); icount.alloc(n);
    {
        // seen-origin window: a power of two covering RP_SEEN_ROUNDS rounds of
        // churn ids (entries expire after about maxPiggybackCount / 2 rounds;
        // older origins are merely unfiltered, never wrong)
        uint64_t W = 4096;
        while (W < (uint64_t)RP_SEEN_ROUNDS * std::max<uint32_t>(k, 1) && W < (1ull << 20)) W <<= 1;
        W = std::min<uint64_t>(W, alive_cap / 2);  // the window must lie inside the makeAlive ring
        W = std::min<uint64_t>(W, (uint64_t)rp::SEEN_STAGE_WORDS * 32);  // staged whole in LDS by the merges
        if (cfg.seen_window) {
            W = cfg.seen_window;
            if (W < 32 || (W & (W - 1)) || W > alive_cap / 2 || W > (uint64_t)rp::SEEN_STAGE_WORDS * 32)
                throw Error(RP_ERR_INVALID, "seen_window: power of two in [32, min(32768, half the makeAlive origin ring)]");
        }
        seen_words = (uint32_t)(W / 32);
        seen.alloc((size_t)nl * (seen_words + 2 * ((n + 31) / 32)));  // + pingable and settled bits (rp::ping_bits, rp::settled_bits)
        RP_HIP(hipMemsetAsync(seen.p, 0, seen.bytes(), st));
        oc_snap.alloc(2);
    }
    RP_HIP(hipMemsetAsync(need_csum.p, 0, n, st));
    RP_HIP(hipMemsetAsync(dangerous.p, 0, 4, st));
    pt_hash.alloc(npts); pt_server.alloc(npts); pt_coll.alloc(npts);
    DevBuf<int32_t> dcoll_min(std::max<size_t>(coll_min.size(), 1));

    RP_HIP(hipMemcpyAsync(addr_words.p, words.data(), words.size() * 4, hipMemcpyHostToDevice, st));
    RP_HIP(hipMemcpyAsync(addr_len.p, lens.data(), n, hipMemcpyHostToDevice, st));
    RP_HIP(hipMemcpyAsync(coll_of.p, h_coll_of.data(), h_coll_of.size() * 4, hipMemcpyHostToDevice, st));
    if (ncoll) RP_HIP(hipMemcpyAsync(dcoll_min.p, coll_min.data(), ncoll * 4, hipMemcpyHostToDevice, st));
    RP_HIP(hipMemcpyAsync(pt_hash.p, h_pt_hash.data(), npts * 4, hipMemcpyHostToDevice, st));
    RP_HIP(hipMemcpyAsync(pt_server.p, h_pt_server.data(), npts * 4, hipMemcpyHostToDevice, st));
    RP_HIP(hipMemcpyAsync(pt_coll.p, h_pt_coll.data(), npts * 4, hipMemcpyHostToDevice, st));
    // origins 0..n-1: fullSync from node v (source v, no sourceIncarnationNumber)
    std::vector<rp::Origin> o0(n + 1);
    for (uint32_t v = 0; v < n; v++) o0[v] = {v, 0, 0};
    o0[n] = {rp::NONE, 0, 0};
    RP_HIP(hipMemcpyAsync(origins.p, o0.data(), o0.size() * sizeof(rp::Origin), hipMemcpyHostToDevice, st));
    const uint32_t oc[2] = {0, 0};
    RP_HIP(hipMemcpy(origin_count.p, oc, 4, hipMemcpyHostToDevice));
    RP_HIP(hipMemcpy(oc_snap.p, oc, 8, hipMemcpyHostToDevice));
    RP_HIP(hipMemsetAsync(err.p, 0, 4, st));
    RP_HIP(hipMemsetAsync(totals.p, 0, totals.bytes(), st));

    self_inc.alloc(n); ck_list.alloc(n); ck_count.alloc(1); slen.alloc(n);
    {
        size_t hs = 1024;
        while (hs < 2 * (size_t)nl) hs <<= 1;
        hkey.alloc(hs); hval.alloc(hs); ck_lead.alloc(nl); ck_nlead.alloc(1); ck_slot.alloc(nl);
        // checksums of earlier rounds by fingerprint: 2^20 entries (16 MB), empty = key ~0
        ck_cache.alloc(1u << 20);
        RP_HIP(hipMemsetAsync(ck_cache.p, 0xFF, ck_cache.bytes(), st));
    }
    if (G > 1) {
        // exchange buffers (the ping and response traffic of one round fits the arena)
        meta.alloc(n); soff.alloc(n); seoff.alloc(n); psoff.alloc(n); pseoff.alloc(n); rx_off.alloc(n);
        rx_eoff.alloc(n); rr_idx.alloc(n); rs_idx.alloc(n);
        rsend.alloc(n); rrecv.alloc(n);
        // entries per direction and round: words for all, escapes for the
        // few without a makeAlive origin (full syncs are all escapes)
        // (a start: fit_exchange grows them to a round's actual traffic, so
        // the footprint follows the traffic rather than the arena's size)
        const uint64_t xcap = 1ull << 20, ecap = 1ull << 18;
        sendw.alloc(xcap); rxw.alloc(xcap); psendw.alloc(xcap); rx2w.alloc(xcap);
        sende.alloc(ecap); rxe.alloc(ecap); psende.alloc(ecap); rx2e.alloc(ecap);
        rxc.alloc(xcap);
        xcnt.alloc((size_t)rp::XC_NCAT * G); sgather.alloc((size_t)G * (rp::STAT_NSTATS + 2));
        xrow.alloc((size_t)2 * G * G);
        ltotals.alloc(rp::STAT_NSTATS + 1);
        RP_HIP(hipMemsetAsync(ltotals.p, 0, ltotals.bytes(), st));
        RP_HIP(hipHostMalloc((void**)&h_xcnt, (size_t)rp::XC_NCAT * G * 8));
        RP_HIP(hipHostMalloc((void**)&h_xrow, (size_t)2 * G * G * 8));
        xs_rec.alloc(n3); xs_w.alloc(n3); xs_e.alloc(n3); xs_list.alloc(n3); xs_nlist.alloc(1);
        xs_wabs.alloc(n3); xs_eabs.alloc(n3); xsend.alloc(n3); xrecv.alloc(n3);
        xsrow.alloc((size_t)3 * G * G);
        RP_HIP(hipHostMalloc((void**)&h_xsrow, ((size_t)3 * G * G + 1) * 8));
    }
    d.n = n; d.ncoll = ncoll; d.lo = lo; d.nl = nl; d.rank = rank; d.nranks = G;
    d.self_inc = self_inc.p; d.slen = slen.p; d.ck_list = ck_list.p; d.ck_count = ck_count.p;
    msg_nesc.alloc(n);
    RP_HIP(hipMemsetAsync(msg_nesc.p, 0, n * 4, st));
    d.rxw = rxw.p; d.rxe = rxe.p; d.rx_off = rx_off.p; d.rx_eoff = rx_eoff.p; d.rx2w = rx2w.p; d.rx2e = rx2e.p;
    d.rxc = rxc.p;
    d.msg_nesc = msg_nesc.p;
    d.view = view.p; d.order = order.p; d.dko = dko.p; d.dvs = dvs.p; d.dad = dad.p; d.dhead = dhead.p; d.dtail = dtail.p;
    d.max_pb = max_pb.p; d.in_ring = in_ring.p; d.ring_count = ring_count.p; d.coll_owner = coll_owner.p;
    d.coll_of = coll_of.p; d.coll_off = coll_off.p; d.coll_ids = coll_ids.p; d.cmem_off = cmem_off.p; d.cmem = cmem.p; d.rbatch = rbatch.p; d.self_origin = self_origin.p; d.fp = fp.p; d.csum = csum.p; d.csum_valid = csum_valid.p; d.iter_index = iter_index.p;
    d.iter_round = iter_round.p; d.npingable = npingable.p; d.rng = rng.p; d.dead = dead.p;
    d.origins = origins.p; d.origin_count = origin_count.p; d.origin_cap = ocap;
    d.lorigin_count = lorigin_count.p; d.lorigin_sent = lorigin_sent.p; d.lorigin_base = lbase; d.lorigin_per = lper;
    d.alive_base = n + 1; d.alive_mask = alive_cap - 1;
    d.pq_nesc = pq_nesc.p; d.rl_nesc = rl_nesc.p; d.pr_ckv = pr_ckv.p;
    d.fdecl_bits = fdecl_bits.p; d.fdecl_count = fdecl_count.p;
    d.addr_words = addr_words.p; d.addr_len = addr_len.p;
    d.arena = arena.p; d.arena_cursor = arena_cursor.p; d.bstats = bstats.p; d.bstride = n; d.arena_cap = acap;
    d.msg_off = msg_off.p; d.msg_len = msg_len.p; d.msg_plen = msg_plen.p; d.target = target.p; d.sv_word = sv_word.p; d.snd_inc = snd_inc.p; d.snd_fp = snd_fp.p;
    d.snd_csum = snd_csum.p; d.g_cnt = g_cnt.p; d.g_fill = g_fill.p; d.g_base = g_base.p; d.g_list = g_list.p;
    d.resp = resp.p; d.snaps = snaps.p; d.snap_ord = snap_ord.p; d.snap_m = snap_m.p; d.mcount = mcount.p; d.snap_count = snap_count.p; d.snap_cap = scap; d.pend_slot = pend_slot.p;
    d.pend_csum = pend_csum.p; d.pend_done = pend_done.p;
    d.pr_n = pr_n.p; d.pr_errors = pr_errors.p; d.pr_bad = pr_bad.p; d.pr_done = pr_done.p; d.pr_inc = pr_inc.p;
    d.pr_fp = pr_fp.p; d.pr_csum = pr_csum.p; d.w3_dest = w3_dest.p; d.w4_dest = w4_dest.p; d.w5_dest = w5_dest.p;
    d.w6_dest = w6_dest.p; d.w4_err = w4_err.p; d.pq_off = pq_off.p; d.pq_len = pq_len.p; d.rl_off = rl_off.p;
    d.rl_len = rl_len.p; d.rl_inc = rl_inc.p; d.rl_fp = rl_fp.p; d.rl_csum = rl_csum.p;
    d.tfifo = tfifo.p; d.thead = thead.p; d.ttail = ttail.p; d.tcap = tcap;
    d.churn_ids = churn_ids.p; d.stats = stats.p;
    d.err = err.p; d.conv = conv.p;
    d.need_csum = need_csum.p; d.min_cnt = min_cnt.p; d.min_safe = min_safe.p; d.min_l1 = min_l1.p; d.min_l2 = min_l2.p; d.dangerous = dangerous.p; d.dlive = dlive.p; d.icount = icount.p;
    d.seen = seen.p; d.seen_words = seen_words; d.oc_snap = oc_snap.p;
    if (cfg.compact_mul || cfg.compact_add) { d.compact_mul = cfg.compact_mul; d.compact_add = cfg.compact_add; }
    else { d.compact_mul = RP_COMPACT_MUL; d.compact_add = RP_COMPACT_ADD; }
    d.prefix_min = cfg.prefix_min ? cfg.prefix_min : RP_PREFIX_MIN;
    d.ck_lane_min = cfg.ck_lane_min ? cfg.ck_lane_min : RP_CK_LANE_MIN;
    {
        // seen groups: the largest power of two up to 2^cap dividing the shard
        // size.  In process the mask all-gather is a device copy and per-node
        // masks filter best; over RCCL every rank receives (G-1)/G of the
        // masks, so groups of 4 trade them for all-to-all bytes (config 4 on 8
        // in-process shards: masks 256 / 64 / 32 / 8 MB and all-to-alls 201 /
        // 428 / 510 / 642 MB per round for groups of 1 / 4 / 8 / 32, merge
        // and issue kernels 8.1 / 8.8 / 9.0 / 9.4 ms per round summed)
        const uint32_t cap = one_per_process ? RP_SEEN_GROUP_LOG_RCCL : RP_SEEN_GROUP_LOG;
        uint32_t lg = 0;
        while (lg < cap && nl % (2u << lg) == 0) lg++;
        d.gsz_log = G > 1 ? lg : 0;
    }
    gseen.alloc(G > 1 ? (size_t)(n >> d.gsz_log) * seen_words : 1); gs_range.alloc(2);
    RP_HIP(hipMemsetAsync(gs_range.p, 0, 8, st));
    d.gseen = gseen.p; d.gs_range = gs_range.p;
    {
        // settled groups: the largest power of two up to 2^RP_SETTLED_GROUP_LOG
        // dividing the shard size (config 5 at 65,536 nodes on 4 shards: 64 MB
        // of masks per shard, 16 MB sent per rank and round)
        uint32_t lg = 0;
        while (lg < RP_SETTLED_GROUP_LOG && nl % (2u << lg) == 0) lg++;
        d.fs_log = lg;
        const size_t pw = (n + 31) / 32;
        if (G > 1) {
            gsettled.alloc((size_t)(n >> lg) * pw);
            RP_HIP(hipMemsetAsync(gsettled.p, 0, gsettled.bytes(), st));
        }
        d.gsettled = gsettled.p;  // (null: one shard, every destination local)
    }

    check_simdev(d);
    const unsigned gfill = 4096;
    hipLaunchKernelGGL(rp::k_init_rows, dim3(gfill), dim3(256), 0, st, d);
    need_shuffle.alloc(n); shuf_list.alloc(nl); shuf_count.alloc(1);
    RP_HIP(hipFuncSetAttribute((const void*)rp::k_shuffle, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(n * 2)));
    hipLaunchKernelGGL(rp::k_init_scalars, dim3(rp::grid_for(n, 256)), dim3(256), 0, st, d, cfg.seed, need_shuffle.p);
    hipLaunchKernelGGL(rp::k_init_order, dim3(nl), dim3(256), 0, st, d);
    hipLaunchKernelGGL(rp::k_shuffle, dim3(nl), dim3(rp::BLOCK), (size_t)n * 2, st, d, need_shuffle.p, 0,
                       (const uint32_t*)nullptr, (const uint32_t*)nullptr);
    if (ncoll) {
        hipLaunchKernelGGL(rp::k_init_owner, dim3(gfill), dim3(256), 0, st, d, (const int32_t*)dcoll_min.p);
        hipLaunchKernelGGL(rp::k_init_owner_self, dim3(rp::grid_for(nl, 256)), dim3(256), 0, st, d);
    }
    hipLaunchKernelGGL(rp::k_init_fp, dim3(nl), dim3(rp::BLOCK), 0, st, d, lo, (const uint32_t*)nullptr);
    // the side stream of the round's checksums (one shard; a list that could
    // take the lane path keeps the live path: ck_cap < ck_lane_min)
    {
        const size_t budget = (size_t)RP_CK_SIDE_MB << 20;
        ck_cap = (uint32_t)std::min<size_t>(nl, std::max<size_t>(64, budget / ((size_t)n * 8)));
        ck_side = RP_CK_SIDE && G == 1 && ck_cap < d.ck_lane_min;
        if (ck_side) {
            RP_HIP(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
            for (hipEvent_t* e : {&ev_ck_copy, &ev_ck_done, &ev_merge_done, &ev_pend_done})
                RP_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
            // (the leader rows -- up to RP_CK_SIDE_MB -- are allocated once a
            // fault, partition or storm is scheduled, ensure_ck_side: runs
            // without them never use the side stream)
        }
    }
    RP_HIP(hipGetLastError());
    RP_HIP(hipStreamSynchronize(st));
}


void Shard::bootstrap_views(uint32_t node_lo, uint32_t count, const uint8_t* vst, const uint64_t* vinc,
                            const uint8_t* member_map, uint64_t seed) {
    using namespace rp;
    if (vst) faulty_unbounded = true;
    RP_HIP(hipMemsetAsync(need_shuffle.p, 0, n, st));
    hipLaunchKernelGGL(k_set_views, dim3(count), dim3(BLOCK), 0, st, d, node_lo, vst, vinc, seed, need_shuffle.p,
                       member_map);
    // this shard's nodes of the range
    const uint32_t l0 = std::max(node_lo, lo), l1 = std::min(node_lo + count, lo + nl);
    if (l0 < l1) {
        hipLaunchKernelGGL(k_shuffle, dim3(std::min<uint32_t>(l1 - l0, 2048)), dim3(BLOCK), (size_t)n * 2, st, d,
                           need_shuffle.p, 0, (const uint32_t*)nullptr, (const uint32_t*)nullptr);
        if (ncoll)
            hipLaunchKernelGGL(k_set_owners, dim3(grid_for((uint64_t)(l1 - l0) * ncoll, 256)), dim3(256), 0, st, d, l0,
                               l1 - l0);
        hipLaunchKernelGGL(k_init_fp, dim3(l1 - l0), dim3(BLOCK), 0, st, d, l0, (const uint32_t*)nullptr);
    }
    RP_HIP(hipGetLastError());
}

void Shard::fit_exchange(int dir, uint64_t send_w, uint64_t send_e, uint64_t recv_w, uint64_t recv_e) {
    // grow to twice the need (whole MiB-multiples of elements): a mass
    // failure's traffic ramps up over its first rounds, and every growth is a
    // free + malloc (a device synchronisation; slow near a full device)
#if RP_DIAG
    static const bool dbg = getenv("RP_DEBUG_GROW") != nullptr;  // (diagnostic builds: growth events on stderr)
#else
    constexpr bool dbg = false;
#endif
    auto grow = [&](auto& b, uint64_t need) {
        if (need <= b.n) return;
        const uint64_t want = std::max<uint64_t>(2 * need, b.n + b.n / 2);
        const auto t0 = std::chrono::steady_clock::now();
        b.reserve((want + (1u << 20) - 1) & ~(uint64_t)((1u << 20) - 1));
        if (dbg)
            fprintf(stderr, "grow shard %u dir %d: %.3f GB in %.2f ms\n", rank, dir, b.bytes() / 1e9,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    };
    if (dir == 0) {
        grow(sendw, send_w); grow(sende, send_e); grow(rxw, recv_w); grow(rxe, recv_e); grow(rxc, recv_w);
    } else {
        grow(psendw, send_w); grow(psende, send_e); grow(rx2w, recv_w); grow(rx2e, recv_e);
    }
    d.rxw = rxw.p; d.rxe = rxe.p; d.rx2w = rx2w.p; d.rx2e = rx2e.p; d.rxc = rxc.p;
}

// The round's sender checksums with the side stream (ck_side): the dedupe
// and the leaders' view copies on the main stream (then the merges may
// change the views), the chains and the hand-out on st2, the live path on the
// main stream only for a list of more leaders than copy rows.
void Shard::ensure_ck_side() {
    if (!ck_side || ck_rows.p) return;
    ck_rows.alloc((size_t)ck_cap * n);
    ck_lfp.alloc(ck_cap);
    ck_lres.alloc(ck_cap);
    ck_hlead.alloc(hkey.n);
}

void Shard::checksums_side(uint32_t* out, bool prefilled) {
    using namespace rp;
    ensure_ck_side();  // (already done when the faults were scheduled)
    if (!prefilled) {
        fill(hkey.p, hkey.bytes(), 0xFF);
        fill(ck_nlead.p, 4, 0);
        fill_flush();
    }
    const uint32_t cmask = (uint32_t)(ck_cache.n - 1);
    hipLaunchKernelGGL(k_ck_dedupe, dim3(grid_for(nl, 256)), dim3(256), 0, st, d, (const uint32_t*)ck_list.p,
                       (const uint32_t*)ck_count.p, hkey.p, hval.p, (uint32_t)(hkey.n - 1), ck_lead.p, ck_nlead.p,
                       ck_slot.p, (const CkEntry*)ck_cache.p, cmask, out, ck_hlead.p);
    hipLaunchKernelGGL(k_ck_snapcopy, dim3(std::min<uint32_t>(ck_cap, 1024)), dim3(256), 0, st, d,
                       (const uint32_t*)ck_lead.p, (const uint32_t*)ck_nlead.p, ck_rows.p, ck_lfp.p, ck_cap);
    // (the live path: a no-op unless more than ck_cap leaders)
    hipLaunchKernelGGL(k_checksums, dim3(std::min(grid_for(nl, NWAVE), 8192u)), dim3(BLOCK), 0, st, d,
                       (const uint32_t*)ck_lead.p, (const uint32_t*)ck_nlead.p, out, ck_cap + 1);
    if (d.ck_lane_min <= nl)  // (its own guard: ck_lane_min > ck_cap leaders)
        hipLaunchKernelGGL(k_checksums_pc, dim3(std::min(grid_for(nl, 64), 16384u)), dim3(CKP_THREADS), 0, st, d,
                           (const uint32_t*)ck_lead.p, (const uint32_t*)ck_nlead.p, out);
    hipLaunchKernelGGL(k_ck_store_follow, dim3(grid_for(nl, 256)), dim3(256), 0, st, d, (const uint32_t*)ck_lead.p,
                       (const uint32_t*)ck_nlead.p, (CkEntry*)ck_cache.p, cmask, (const uint32_t*)ck_list.p,
                       (const uint32_t*)ck_count.p, (const uint32_t*)hval.p, (const uint32_t*)ck_slot.p, out,
                       ck_cap + 1);
    RP_HIP(hipEventRecord(ev_ck_copy, st));
    RP_HIP(hipStreamWaitEvent(st2, ev_ck_copy, 0));
    side_timed([&] {
        hipLaunchKernelGGL(k_checksums_snap, dim3(std::max<uint32_t>(1, std::min<uint32_t>(ck_cap / NWAVE + 1, 2048))),
                           dim3(BLOCK), 0, st2, d, (const uint64_t*)ck_rows.p, (const uint32_t*)ck_nlead.p, ck_cap,
                           ck_lres.p);

        hipLaunchKernelGGL(k_ck_finish_snap, dim3(grid_for(nl, 256)), dim3(256), 0, st2, d, (const uint32_t*)ck_list.p,
                           (const uint32_t*)ck_count.p, (const uint32_t*)ck_nlead.p, ck_cap, (const uint32_t*)ck_slot.p,
                           (const uint32_t*)ck_hlead.p, (const uint32_t*)ck_lres.p,
                           (const unsigned long long*)ck_lfp.p, ck_cache.p, cmask, out);
    });
    RP_HIP(hipEventRecord(ev_ck_done, st2));
}

void Shard::checksums(uint32_t* out, bool prefilled) {
    using namespace rp;
    if (!prefilled) {
        fill(hkey.p, hkey.bytes(), 0xFF);
        fill(ck_nlead.p, 4, 0);
        fill_flush();
    }
    hipLaunchKernelGGL(k_ck_dedupe, dim3(grid_for(nl, 256)), dim3(256), 0, st, d, (const uint32_t*)ck_list.p,
                       (const uint32_t*)ck_count.p, hkey.p, hval.p, (uint32_t)(hkey.n - 1), ck_lead.p, ck_nlead.p,
                       ck_slot.p, (const CkEntry*)ck_cache.p, (uint32_t)(ck_cache.n - 1));
    hipLaunchKernelGGL(k_checksums, dim3(std::min(grid_for(nl, NWAVE), 8192u)), dim3(BLOCK), 0, st, d,
                       (const uint32_t*)ck_lead.p,
                       (const uint32_t*)ck_nlead.p, out);
    if (d.ck_lane_min <= nl)  // (only a list of >= ck_lane_min leaders runs it)
        hipLaunchKernelGGL(k_checksums_pc, dim3(std::min(grid_for(nl, 64), 16384u)), dim3(CKP_THREADS), 0, st, d,
                           (const uint32_t*)ck_lead.p, (const uint32_t*)ck_nlead.p, out);
    hipLaunchKernelGGL(k_ck_store_follow, dim3(grid_for(nl, 256)), dim3(256), 0, st, d, (const uint32_t*)ck_lead.p,
                       (const uint32_t*)ck_nlead.p, (CkEntry*)ck_cache.p, (uint32_t)(ck_cache.n - 1),
                       (const uint32_t*)ck_list.p, (const uint32_t*)ck_count.p, (const uint32_t*)hval.p,
                       (const uint32_t*)ck_slot.p, out, 0u);
}

void Shard::group(const int32_t* dest, uint32_t nslots, bool prefilled, bool counted) {
    using namespace rp;
    if (!prefilled) {
        fill(g_cnt.p, (size_t)n * 4, 0);
        fill(g_fill.p, (size_t)n * 4, 0);
        fill_flush();
    }
    if (!counted)
        hipLaunchKernelGGL(k_group_count, dim3(grid_for(nslots, 256)), dim3(256), 0, st, dest, nslots, g_cnt.p);
    const uint32_t tiles = (n + 1023) / 1024;
    if (tiles <= GROUP_FUSE_TILES) {
        hipLaunchKernelGGL(k_group_scan, dim3(tiles), dim3(1024), 0, st, g_cnt.p, g_bloc.p, n, g_tile.p);
        hipLaunchKernelGGL(k_group_fill2, dim3(grid_for(nslots, 256)), dim3(256), 0, st, dest, nslots,
                           (const uint32_t*)g_bloc.p, (const uint32_t*)g_tile.p, tiles, g_fill.p, g_list.p);
        hipLaunchKernelGGL(k_group_sort2, dim3(grid_for(n + 1, 256)), dim3(256), 0, st, (const uint32_t*)g_bloc.p,
                           (const uint32_t*)g_tile.p, tiles, g_list.p, n, g_base.p);
        return;
    }
    hipLaunchKernelGGL(k_group_scan, dim3(tiles), dim3(1024), 0, st, g_cnt.p, g_base.p, n, g_tile.p);
    hipLaunchKernelGGL(k_group_scan_add, dim3(tiles), dim3(1024), 0, st, g_base.p, n, (const uint32_t*)g_tile.p);
    hipLaunchKernelGGL(k_group_fill, dim3(grid_for(nslots, 256)), dim3(256), 0, st, dest, nslots, g_base.p,
                       g_fill.p, g_list.p);
    hipLaunchKernelGGL(k_group_sort, dim3(grid_for(n, 256)), dim3(256), 0, st, g_base.p, g_list.p, n);
}

void Shard::stage_start(uint32_t round, bool churn_active, uint32_t slot, const std::vector<int32_t>& dead_now,
                        bool faults, const uint32_t part[3], uint32_t storm_k) {
    using namespace rp;
    const uint64_t now = T0 + PERIOD_MS * round;
    d.round = round;
    d.part_start = part[0]; d.part_end = part[1]; d.part_split = part[2];
    // every per-round reset of the stages below, in one launch
    fill(stats.p, stats.bytes(), 0);
    fill(arena_cursor.p, arena_cursor.bytes(), 0);
    fill(snap_count.p, 4, 0);
    fill(pend_done.p, (d.snap_cap + 3u) & ~3u, 0);  // (pend_done holds a multiple of 4 bytes: setup)
    fill(shuf_count.p, 4, 0);                       // k_iterate
    fill(p2_len.p, p2_len.bytes(), 0);              // k_p2_lists
    fill(fp_mm.p, 8, 0xFF);                         // k_round_end: min, max
    fill(fp_mm.p + 1, 8, 0);
    if (faults) {
        fill(w3_dest.p, w3_dest.bytes(), 0xFF);     // k_phase3_err, k_w3
        fill(w4_dest.p, w4_dest.bytes(), 0xFF);
        fill(w3cnt.p, w3cnt.bytes(), 0);            // k_pr_hist
        fill(w4b.p, w4b.bytes(), 0);
    }
    // the checksum stage's resets (group counts, the dedupe table, the lists)
    fill(g_cnt.p, (size_t)n * 4, 0);
    fill(g_fill.p, (size_t)n * 4, 0);
    fill(hkey.p, hkey.bytes(), 0xFF);
    fill(ck_nlead.p, 4, 0);
    fill(ck_count.p, 4, 0);
    fill_flush(true);  // (+ the seen bits of the ids allocated last round)
    if (faults) {
        if (!dead_now.empty()) {
            RP_HIP(hipMemcpyAsync(dead_ids.p, dead_now.data(), dead_now.size() * 4, hipMemcpyHostToDevice, st));
            RP_HIP(hipStreamSynchronize(st));  // dead_now is a host temporary
            hipLaunchKernelGGL(k_mark_dead, dim3(grid_for(dead_now.size(), 256)), dim3(256), 0, st, d,
                               (const int32_t*)dead_ids.p, (uint32_t)dead_now.size());
        }
        timed(0, [&] { hipLaunchKernelGGL(k_timers, dim3(nl), dim3(BLOCK), 0, st, d, round, now); });
    }
}

void Shard::stage_churn(bool churn_active, uint32_t slot, uint32_t storm_k, uint64_t now) {
    using namespace rp;
    if (churn_active && k)
        timed(0, [&] {
            hipLaunchKernelGGL(k_churn, dim3(k), dim3(BLOCK), 0, st, d, k, slot, now);
        });
    if (storm_k) {
        const int32_t* pairs = storm.p + (size_t)slot * 2 * storm_kmax;
        timed(0, [&] {
            hipLaunchKernelGGL(k_storm, dim3(storm_k), dim3(BLOCK), 0, st, d, pairs, pairs + storm_kmax, storm_k, now);
        });
    }
}

void Shard::stage_issue() {
    using namespace rp;
    timed(1, [&] {
        hipLaunchKernelGGL(k_iterate, dim3(grid_for(nl, 64)), dim3(64), 0, st, d, need_shuffle.p, shuf_list.p,
                           shuf_count.p);
        // (a block holds the n * 2 bytes of LDS, one per CU at 65,536 nodes;
        // iterators wrap once per view length, a few nodes a round: a small
        // grid strides over them and leaves the CUs to the other shards' work)
        hipLaunchKernelGGL(k_shuffle, dim3(std::min<uint32_t>(nl, 32)), dim3(BLOCK), (size_t)n * 2, st, d,
                           need_shuffle.p, 1, (const uint32_t*)shuf_list.p, (const uint32_t*)shuf_count.p);
        if (fault_mode) {
            if (G > 1) hipLaunchKernelGGL((k_phase1<true, true>), dim3(nl), dim3(BLOCK), 0, st, d);
            else hipLaunchKernelGGL((k_phase1<false, true>), dim3(nl), dim3(BLOCK), 0, st, d);
        } else {
            if (G > 1) hipLaunchKernelGGL((k_phase1<true, false>), dim3(nl), dim3(BLOCK), 0, st, d);
            else hipLaunchKernelGGL((k_phase1<false, false>), dim3(nl), dim3(BLOCK), 0, st, d);
        }
    });
}

void Shard::stage_checksums() {
    using namespace rp;
    // (the group counts, ck_count and the dedupe table were reset by stage_start's launch)
    timed(5, [&] { group(target.p, n, true, G == 1); });
    timed(4, [&] {
        // (one shard: its own count is the cluster's; a shard of several
        // uses the counts all-gathered at this round's start, fd_shared)
        const uint32_t* fd = G == 1 ? (faulty_unbounded ? nullptr : (const uint32_t*)fdecl_count.p)
                                    : (fd_shared ? (const uint32_t*)fdecl_all.p : nullptr);
        hipLaunchKernelGGL(k_need_checksums, dim3(grid_for(n, 256)), dim3(256), 0, st, d, fd, G == 1 ? 1u : G,
                           ck_list.p, ck_count.p);
        if (side_round()) checksums_side(snd_csum.p, true);
        else checksums(snd_csum.p, true);
    });
}

void Shard::stage_ping_merge(uint64_t now) {
    using namespace rp;
    timed(2, [&] {
        hipLaunchKernelGGL(k_p2_lists, dim3(grid_for(nl, 256)), dim3(256), 0, st, d, p2_list.p, p2_len.p, p2_msg.p);
        for (uint32_t k = 0; k < P2_SPLIT; k++) {
            const uint32_t* lk = p2_list.p + (size_t)k * nl;
            const dim3 grid(p2_grid(nl, n, k));
            const uint64_t* mk = p2_msg.p + (size_t)k * nl * 2;
            if (join_mode) hipLaunchKernelGGL(k_p2_apply<true>, grid, dim3(BLOCK), 0, st, d, now, k, lk, p2_len.p + k, mk);
            else hipLaunchKernelGGL(k_p2_apply<false>, grid, dim3(BLOCK), 0, st, d, now, k, lk, p2_len.p + k, mk);
            hipLaunchKernelGGL(k_p2_pre, dim3(grid_for(grid.x, 256)), dim3(256), 0, st, d, lk, p2_len.p + k, p2_rec.p);
            const P2Rec* rk = p2_rec.p;
            if (fault_mode) {
                if (G > 1) hipLaunchKernelGGL((k_p2_respond<true, true>), grid, dim3(BLOCK), 0, st, d, k, rk, p2_len.p + k);
                else hipLaunchKernelGGL((k_p2_respond<false, true>), grid, dim3(BLOCK), 0, st, d, k, rk, p2_len.p + k);
            } else {
                if (G > 1) hipLaunchKernelGGL((k_p2_respond<true, false>), grid, dim3(BLOCK), 0, st, d, k, rk, p2_len.p + k);
                else hipLaunchKernelGGL((k_p2_respond<false, false>), grid, dim3(BLOCK), 0, st, d, k, rk, p2_len.p + k);
            }
        }
        const uint32_t* lt = p2_list.p + (size_t)P2_SPLIT * nl;
        const uint32_t* nt = p2_len.p + P2_SPLIT;
        const dim3 gt(p2_grid(nl, n, P2_SPLIT));
        // (joins and fault runs: the splice and settled-filter variants)
        if (join_mode) {
            if (G > 1) hipLaunchKernelGGL((k_phase2<true, true, true>), gt, dim3(BLOCK), 0, st, d, now, lt, nt);
            else hipLaunchKernelGGL((k_phase2<false, true, true>), gt, dim3(BLOCK), 0, st, d, now, lt, nt);
        } else if (fault_mode) {
            if (G > 1) hipLaunchKernelGGL((k_phase2<true, false, true>), gt, dim3(BLOCK), 0, st, d, now, lt, nt);
            else hipLaunchKernelGGL((k_phase2<false, false, true>), gt, dim3(BLOCK), 0, st, d, now, lt, nt);
        } else {
            if (G > 1) hipLaunchKernelGGL((k_phase2<true, false, false>), gt, dim3(BLOCK), 0, st, d, now, lt, nt);
            else hipLaunchKernelGGL((k_phase2<false, false, false>), gt, dim3(BLOCK), 0, st, d, now, lt, nt);
        }
    });
    if (side_round()) {
        // the fullSync decisions beside the response merge's pass 1 (after
        // the sender checksums, which they compare against, on the same stream)
        RP_HIP(hipEventRecord(ev_merge_done, st));
        RP_HIP(hipStreamWaitEvent(st2, ev_merge_done, 0));
        side_timed([&] {
            launch_pending(st2);
        });
        RP_HIP(hipEventRecord(ev_pend_done, st2));
    } else {
        timed(4, [&] { launch_pending(st); });
    }
}

void Shard::stage_resp_merge(uint64_t now, bool faults) {
    using namespace rp;
    timed(3, [&] {
        auto p3 = [&](int pass) {
            if (join_mode) {
                if (G > 1) hipLaunchKernelGGL((k_phase3<true, true>), dim3(nl), dim3(BLOCK), 0, st, d, now, pass);
                else hipLaunchKernelGGL((k_phase3<true, false>), dim3(nl), dim3(BLOCK), 0, st, d, now, pass);
            } else {
                if (G > 1) hipLaunchKernelGGL((k_phase3<false, true>), dim3(nl), dim3(BLOCK), 0, st, d, now, pass);
                else hipLaunchKernelGGL((k_phase3<false, false>), dim3(nl), dim3(BLOCK), 0, st, d, now, pass);
            }
        };
        if (side_round()) {
            p3(1);  // (beside k_pending on st2)
            RP_HIP(hipStreamWaitEvent(st, ev_pend_done, 0));
            p3(2);  // the responses whose fullSync decision k_pending took
        } else {
            p3(0);
        }
        if (faults) {
            RP_HIP(hipMemsetAsync(ck_count.p, 0, 4, st));
            if (G > 1) hipLaunchKernelGGL(k_phase3_err<true>, dim3(nl), dim3(BLOCK), 0, st, d, now, 0);
            else hipLaunchKernelGGL(k_phase3_err<false>, dim3(nl), dim3(BLOCK), 0, st, d, now, 0);
            hipLaunchKernelGGL(k_pr_hist, dim3(grid_for(nl, 256)), dim3(256), 0, st, d, w3cnt.p, w4b.p,
                               faulty_unbounded ? 1u : 0u);
        }
    });
}

// (after a cluster summed w3cnt / w4b) the ping-req initiators whose checksum
// a relay can compare, and those checksums (the body of PingReqSender.send)
void Shard::stage_pr_need() {
    using namespace rp;
    timed(3, [&] {
        hipLaunchKernelGGL(k_pr_need, dim3(grid_for(nl, 256)), dim3(256), 0, st, d, (const uint32_t*)w3cnt.p,
                           (const uint32_t*)w4b.p);
        checksums(pr_csum.p);
    });
}

// Ping-req wave w (lib/swim/ping-req-sender.js, server/ping-req-handler.js):
// handlers of the messages addressed to this shard's nodes, in slot order;
// a cluster exchanges each wave's cross-shard messages before it (k_xs_*).
void Shard::stage_wave(int w, uint64_t now) {
    using namespace rp;
    const uint32_t n3 = 3 * n;
    const bool esc = G > 1;
    timed(5, [&] {
        if (w == 3) {
            group(w3_dest.p, n3);
            if (esc) hipLaunchKernelGGL(k_w3<true>, dim3(nl), dim3(BLOCK), 0, st, d, now);
            else hipLaunchKernelGGL(k_w3<false>, dim3(nl), dim3(BLOCK), 0, st, d, now);
        } else if (w == 4) {
            group(w4_dest.p, n3);
            if (esc) hipLaunchKernelGGL(k_w4<true>, dim3(nl), dim3(BLOCK), 0, st, d, now);
            else hipLaunchKernelGGL(k_w4<false>, dim3(nl), dim3(BLOCK), 0, st, d, now);
            launch_pending(st);
            hipLaunchKernelGGL(k_dest_w5, dim3(grid_for(n3, 256)), dim3(256), 0, st, d);
        } else if (w == 5) {
            group(w5_dest.p, n3);
            if (esc) hipLaunchKernelGGL(k_w5<true>, dim3(nl), dim3(BLOCK), 0, st, d, now);
            else hipLaunchKernelGGL(k_w5<false>, dim3(nl), dim3(BLOCK), 0, st, d, now);
            launch_pending(st);
            hipLaunchKernelGGL(k_dest_w6, dim3(grid_for(n3, 256)), dim3(256), 0, st, d);
        } else {
            group(w6_dest.p, n3);
            if (esc) hipLaunchKernelGGL(k_w6<true>, dim3(nl), dim3(BLOCK), 0, st, d, now);
            else hipLaunchKernelGGL(k_w6<false>, dim3(nl), dim3(BLOCK), 0, st, d, now);
        }
    });
}

// local statistics and this shard's fingerprint range; a single shard also
// finishes the round (k_converge_done)
void Shard::stage_end() {
    using namespace rp;
    timed(5, [&] {
        const uint32_t ncv = grid_for(nl, BLOCK * 4);
        hipLaunchKernelGGL(k_round_end, dim3(ncv + 64 * STAT_NSTATS), dim3(BLOCK), 0, st, d, fp_mm.p, ncv);
        if (G == 1)
            hipLaunchKernelGGL(k_converge_done, dim3(1), dim3(64), 0, st, d, (const unsigned long long*)fp_mm.p,
                               totals.p);
    });
    RP_HIP(hipGetLastError());
}

uint32_t Shard::read_err() {
    uint32_t e = 0;
    RP_HIP(hipMemcpyAsync(&e, err.p, 4, hipMemcpyDeviceToHost, st));
    RP_HIP(hipStreamSynchronize(st));
    if (timing) collect_timing();
    return e;
}

}  // namespace


// ---------------------------------------------------------------- rank transports
// A process that holds one shard of a G-rank cluster exchanges with the other
// ranks through a transport: RCCL (one process per GPU, rp_sim_create_rank),
// or a loopback among the host threads of one process on one device
// (rp_sim_create_rank_loop): the same rank code -- plans, counts, offsets,
// buffer sizes -- with the collectives done as device copies, so that the
// rank path runs and is compared with the in-process shards where one GPU is
// all there is.
namespace rp {
struct Xfer {
    uint32_t peer;
    void* ptr;
    size_t bytes;
};
struct Xport {
    virtual ~Xport() = default;
    // in place: this rank's chunk is base + rank * bytes, the others arrive
    virtual void allgather(uint8_t* base, size_t bytes, uint32_t rank, hipStream_t st) = 0;
    virtual void allreduce_u32(uint32_t* buf, size_t count, hipStream_t st) = 0;
    // matching pairs: this rank's send to q is q's receive from this rank
    virtual void sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t st) = 0;
    virtual void broadcast(uint8_t* p, size_t bytes, uint32_t root, hipStream_t st) = 0;
};
}  // namespace rp

#define RP_NCCL(expr)                                                                               \
    do {                                                                                            \
        ncclResult_t r_ = (expr);                                                                   \
        if (r_ != ncclSuccess) throw Error(RP_ERR_HIP, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

namespace rp {
struct NcclXport : Xport {
    ncclComm_t comm = nullptr;
    ~NcclXport() override { if (comm) (void)ncclCommDestroy(comm); }
    void allgather(uint8_t* base, size_t bytes, uint32_t rank, hipStream_t st) override {
        RP_NCCL(ncclAllGather(base + (size_t)rank * bytes, base, bytes, ncclUint8, comm, st));
    }
    void allreduce_u32(uint32_t* buf, size_t count, hipStream_t st) override {
        RP_NCCL(ncclAllReduce(buf, buf, count, ncclUint32, ncclSum, comm, st));
    }
    void sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t st) override {
        RP_NCCL(ncclGroupStart());
        for (const Xfer& x : sends) RP_NCCL(ncclSend(x.ptr, x.bytes, ncclUint8, (int)x.peer, comm, st));
        for (const Xfer& x : recvs) RP_NCCL(ncclRecv(x.ptr, x.bytes, ncclUint8, (int)x.peer, comm, st));
        RP_NCCL(ncclGroupEnd());
    }
    void broadcast(uint8_t* p, size_t bytes, uint32_t root, hipStream_t st) override {
        RP_NCCL(ncclBroadcast(p, p, bytes, ncclUint8, (int)root, comm, st));
    }
};

// The loopback group: every collective is a rendezvous of all G rank threads.
// Each rank posts its transfers and records an event after its earlier work;
// the last rank to arrive leads: on the group's own stream it waits for every
// rank's event, moves all G x (G - 1) segments with batched copy launches
// (k_copy_batch, as the in-process exchanges do) and records one done event,
// then releases the others; every rank's stream waits on that one event.  Per
// collective that is 2 API calls per rank plus G + 2 for the leader, where a
// copy and two waits per segment (~180 calls at G = 8, with eight threads
// contending for the runtime) left the GPU idle a third of each round.
struct LoopGroup {
    uint32_t G;
    std::mutex m;
    std::condition_variable cv;
    uint32_t arrived = 0;
    uint64_t gen = 0;
    bool broken = false;  // a rank threw: the others stop waiting
    struct Post {
        std::vector<Xfer> sends, recvs;
        hipEvent_t ready = nullptr;
    };
    std::vector<Post> post;
    hipStream_t xs = nullptr;    // the leader's copies (created by the first leader)
    hipEvent_t done = nullptr;   // recorded on xs after each collective's copies
    explicit LoopGroup(uint32_t g) : G(g), post(g) {}
    ~LoopGroup() {
        if (xs) (void)hipStreamSynchronize(xs);
        if (done) (void)hipEventDestroy(done);
        if (xs) (void)hipStreamDestroy(xs);
    }
    // true for the last rank to arrive, which then leads and calls release()
    bool arrive() {
        std::unique_lock<std::mutex> l(m);
        if (broken) throw Error(RP_ERR_STATE, "loopback cluster: another rank failed");
        const uint64_t g0 = gen;
        if (++arrived == G) {
            arrived = 0;
            return true;
        }
        if (!cv.wait_for(l, std::chrono::seconds(120), [&] { return gen != g0 || broken; }) || broken) {
            broken = true;
            cv.notify_all();
            throw Error(RP_ERR_STATE, "loopback cluster: a rank did not reach the collective");
        }
        return false;
    }
    void release() {
        std::lock_guard<std::mutex> l(m);
        gen++;
        cv.notify_all();
    }
    void fail() {
        std::lock_guard<std::mutex> l(m);
        broken = true;
        cv.notify_all();
    }
    // (the leader, all posts in) every receive matched to its send, the
    // segments copied on xs once every rank's earlier work is done
    void lead() {
        if (!xs) {
            RP_HIP(hipStreamCreateWithFlags(&xs, hipStreamNonBlocking));
            RP_HIP(hipEventCreateWithFlags(&done, hipEventDisableTiming));
        }
        for (const Post& p : post) RP_HIP(hipStreamWaitEvent(xs, p.ready, 0));
        CopyBatch b{};
        uint64_t mx = 0;
        auto flush = [&] {
            if (!b.n) return;
            const uint32_t gx = (uint32_t)std::min<uint64_t>(1024, std::max<uint64_t>(1, (mx + 65535) / 65536));
            hipLaunchKernelGGL(k_copy_batch, dim3(gx, b.n), dim3(256), 0, xs, b);
            b.n = 0;
            mx = 0;
        };
        size_t nsend = 0, nrecv = 0;
        for (const Post& p : post) nsend += p.sends.size();
        for (uint32_t r = 0; r < G; r++) {
            for (const Xfer& x : post[r].recvs) {
                const Xfer* src = nullptr;
                for (const Xfer& y : post[x.peer].sends)
                    if (y.peer == r) { src = &y; break; }
                if (!src || src->bytes != x.bytes)
                    throw Error(RP_ERR_STATE, "loopback cluster: a receive has no matching send");
                nrecv++;
                if (!x.bytes) continue;
                b.d[b.n++] = CopyDesc{src->ptr, x.ptr, (uint64_t)x.bytes};
                mx = std::max<uint64_t>(mx, x.bytes);
                if (b.n == COPY_BATCH) flush();
            }
        }
        if (nrecv != nsend) throw Error(RP_ERR_STATE, "loopback cluster: a send has no matching receive");
        flush();
        RP_HIP(hipGetLastError());
        RP_HIP(hipEventRecord(done, xs));
    }
};

struct LoopXport : Xport {
    LoopGroup* g;
    uint32_t rank;
    hipEvent_t ready = nullptr;
    DevBuf<uint32_t> stage, tmp;  // all-reduce: this rank's input, then every other rank's
    LoopXport(LoopGroup* grp, uint32_t r) : g(grp), rank(r) {
        RP_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    }
    ~LoopXport() override {
        if (ready) (void)hipEventDestroy(ready);
    }
    void exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t st) {
        try {
            RP_HIP(hipEventRecord(ready, st));
            g->post[rank].sends = sends;
            g->post[rank].recvs = recvs;
            g->post[rank].ready = ready;
            if (g->arrive()) {
                try {
                    g->lead();
                } catch (...) {
                    g->fail();
                    throw;
                }
                g->release();
            }
            // (the posts are read by the leader before its release: this
            // rank may post again once it is past here)
            RP_HIP(hipStreamWaitEvent(st, g->done, 0));
        } catch (...) {
            g->fail();
            throw;
        }
    }
    void allgather(uint8_t* base, size_t bytes, uint32_t r, hipStream_t st) override {
        std::vector<Xfer> sends, recvs;
        for (uint32_t q = 0; q < g->G; q++)
            if (q != r) {
                sends.push_back(Xfer{q, base + (size_t)r * bytes, bytes});
                recvs.push_back(Xfer{q, base + (size_t)q * bytes, bytes});
            }
        exchange(sends, recvs, st);
    }
    void allreduce_u32(uint32_t* buf, size_t count, hipStream_t st) override {
        stage.reserve(count);
        tmp.reserve(count * g->G);
        RP_HIP(hipMemcpyAsync(stage.p, buf, count * 4, hipMemcpyDeviceToDevice, st));
        std::vector<Xfer> sends, recvs;
        for (uint32_t q = 0; q < g->G; q++)
            if (q != rank) {
                sends.push_back(Xfer{q, stage.p, count * 4});
                recvs.push_back(Xfer{q, tmp.p + (size_t)q * count, count * 4});
            }
        exchange(sends, recvs, st);
        for (uint32_t q = 0; q < g->G; q++)
            if (q != rank)
                hipLaunchKernelGGL(k_add_u32, dim3(grid_for(count, 256)), dim3(256), 0, st, buf,
                                   (const uint32_t*)(tmp.p + (size_t)q * count), (uint32_t)count);
    }
    void sendrecv(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t st) override {
        exchange(sends, recvs, st);
    }
    void broadcast(uint8_t* p, size_t bytes, uint32_t root, hipStream_t st) override {
        std::vector<Xfer> sends, recvs;
        if (rank == root) {
            for (uint32_t q = 0; q < g->G; q++)
                if (q != root) sends.push_back(Xfer{q, p, bytes});
        } else {
            recvs.push_back(Xfer{root, p, bytes});
        }
        exchange(sends, recvs, st);
    }
};
}  // namespace rp

struct rp_loop {
    rp::LoopGroup grp;
    explicit rp_loop(uint32_t g) : grp(g) {}
};

// A simulated cluster: G shards of N/G nodes each.  Either all shards live in
// this process on one device (exchanges are device copies; used by the tests
// and for single-GPU runs, G = 1), or this process holds one shard of a
// G-process cluster and exchanges over RCCL (one process per GPU).
struct rp_sim {
    rp_sim_config cfg{};
    uint32_t n = 0, k = 0, G = 1;
    int dev = 0;  // the HIP device it lives on (entry points may come from any host thread)
    std::vector<std::unique_ptr<Shard>> sh;  // local shards (all G, or one)
    std::unique_ptr<rp::Xport> comm;         // RCCL (or loopback): this process holds shard `rank` only
    uint32_t rank = 0;
    hipStream_t st = nullptr;                // shared by in-process shards
    std::vector<int32_t> fail_round;         // per node: round of its fail-stop, -1 none
    struct JoinEv { uint32_t round, joiner; std::vector<int32_t> seeds; };
    std::vector<JoinEv> joins;               // rp_sim_join's schedule, in order
    std::vector<int32_t> join_round;         // per node: round it joins at, -1 = a member from the start
    bool live_at(uint32_t i, uint32_t r) const {  // neither failed nor still outside the cluster at round r
        return (fail_round[i] < 0 || (uint32_t)fail_round[i] > r) && (join_round[i] < 0 || (uint32_t)join_round[i] <= r);
    }
    void join_step(uint32_t r, uint64_t now);
    bool faults = false;
    bool views_set = false;                  // rp_sim_set_views ran (rp_sim_load_addresses must come first)
    uint32_t part[3] = {0, 0, 0};
    uint64_t churn_rng = 0;
    uint32_t round = 0;
    int32_t* h_churn = nullptr;              // pinned staging for churn ids
    // false-suspicion storm: rounds [start, end), ceil(live * ppm / 1e6) victims per round
    uint32_t storm_start = 0, storm_end = 0, storm_ppm = 0, storm_kmax = 0;
    uint64_t storm_rng = 0;
    int32_t* h_storm = nullptr;              // pinned staging: CHURN_SLOTS x 2 x storm_kmax
    std::vector<uint32_t> storm_k;           // pairs per staged round
    uint64_t xbytes = 0, xcalls = 0;         // bytes this process sent in exchanges

    // f(shard) for every shard this process holds, in shard order.  (One host
    // thread per in-process shard was measured: no faster, and it varied
    // more -- 39.6-75 against 39.1-39.3 ms/round at 65,536 nodes on 4 shards.)
    template <class F>
    void each(F&& f) {
        for (auto& s : sh) f(*s);
    }

    ~rp_sim() {
        sh.clear();
        if (xdone) (void)hipEventDestroy(xdone);
        comm.reset();
        if (h_churn) (void)hipHostFree(h_churn);
        if (h_storm) (void)hipHostFree(h_storm);
        if (st) (void)hipStreamDestroy(st);
    }
    Shard& owner_of(uint32_t node) {
        for (auto& s : sh)
            if (node - s->lo < s->nl) return *s;
        throw Error(RP_ERR_INVALID, "node " + std::to_string(node) + " is not held by this process");
    }
    void choose_churn(int32_t* out, uint32_t r);
    uint32_t choose_storm(int32_t* out, uint32_t r);
    void enqueue_round(bool churn_active, uint32_t slot);
    void run(int k_rounds, bool churn_active);
    void check_errors();
    // exchanges
    template <class T>
    void allgather_nodes(DevBuf<T> Shard::*buf, size_t per_node);
    template <class T>
    void allgather_block(DevBuf<T> Shard::*buf, size_t per_shard);
    void allreduce_sum(DevBuf<uint32_t> Shard::*buf, size_t count);
    void alltoallv(DevBuf<Change> Shard::*sendb, DevBuf<Change> Shard::*recvb, int cat_send, int cat_recv,
                   size_t elem);
    template <class T>
    void alltoallv_t(DevBuf<T> Shard::*sendb, DevBuf<T> Shard::*recvb, int cat_send, int cat_recv);
    void read_counts();
    void origin_exchange();
    template <int W>
    void slot_exchange();
    void sync_all() { for (auto& s : sh) RP_HIP(hipStreamSynchronize(s->st)); }
    bool presized = false;
    bool loop_rank = false;  // a loopback rank: its G - 1 peers share this device
    void presize_exchange();
    // In-process clusters run each shard on a stream of its own, so that the
    // shards' kernels overlap as one-GPU-per-shard ranks would; an exchange
    // step (device copies on the cluster stream st) starts after every
    // shard's earlier work (xbegin) and every shard's later work waits for it
    // (xend).  One shard per process (RCCL): the shard's stream orders both.
    hipEvent_t xdone = nullptr;
    // segment copies of the current in-process exchange (k_copy_batch at xend)
    std::vector<rp::CopyDesc> cbatch;
    void copy(void* dst, const void* src, size_t bytes) {
        if (bytes) cbatch.push_back(rp::CopyDesc{src, dst, (uint64_t)bytes});
    }
    void copy_flush() {
        for (size_t i0 = 0; i0 < cbatch.size(); i0 += rp::COPY_BATCH) {
            rp::CopyBatch b{};
            b.n = (uint32_t)std::min<size_t>(rp::COPY_BATCH, cbatch.size() - i0);
            uint64_t mx = 0;
            for (uint32_t j = 0; j < b.n; j++) { b.d[j] = cbatch[i0 + j]; mx = std::max<uint64_t>(mx, b.d[j].bytes); }
            const uint32_t gx = (uint32_t)std::min<uint64_t>(1024, std::max<uint64_t>(1, (mx + 65535) / 65536));
            hipLaunchKernelGGL(rp::k_copy_batch, dim3(gx, b.n), dim3(256), 0, st, b);
        }
        cbatch.clear();
    }
    bool overlap() const { return !comm && sh.size() > 1 && sh.front()->st != st; }
    // (nested scopes: consecutive collectives with no shard work between
    // them share one ordering step and one copy launch)
    int xdepth = 0;
    void xbegin() {
        if (xdepth++ > 0 || !overlap()) return;
        for (auto& s : sh) {
            RP_HIP(hipEventRecord(s->xev, s->st));
            RP_HIP(hipStreamWaitEvent(st, s->xev, 0));
        }
    }
    void xend() {
        if (--xdepth > 0) return;
        copy_flush();
        if (!overlap()) return;
        RP_HIP(hipEventRecord(xdone, st));
        for (auto& s : sh) RP_HIP(hipStreamWaitEvent(s->st, xdone, 0));
    }
};

// Every shard's slice [lo, lo + nl) of a per-node array -> every shard.
template <class T>
void rp_sim::allgather_nodes(DevBuf<T> Shard::*buf, size_t per_node) {
    const size_t nl = n / G, bytes = nl * per_node * sizeof(T);
    if (comm) {
        Shard& s = *sh[0];
        T* base = (s.*buf).p;
        comm->allgather((uint8_t*)base, bytes, s.rank, s.st);  // (the slice of rank r starts at r * bytes)
        xbytes += bytes * (G - 1);
        s.xsent += bytes * (G - 1);
        return;
    }
    xbegin();
    for (auto& dst : sh)
        for (auto& src : sh)
            if (dst != src) {
                copy((dst.get()->*buf).p + (size_t)src->lo * per_node, (src.get()->*buf).p + (size_t)src->lo * per_node,
                     bytes);
                src->xsent += bytes;
            }
    xend();
}
// Every shard's block [rank * per, (rank + 1) * per) -> every shard.
template <class T>
void rp_sim::allgather_block(DevBuf<T> Shard::*buf, size_t per_shard) {
    const size_t bytes = per_shard * sizeof(T);
    if (comm) {
        Shard& s = *sh[0];
        T* base = (s.*buf).p;
        comm->allgather((uint8_t*)base, bytes, s.rank, s.st);
        s.xsent += bytes * (G - 1);
        return;
    }
    xbegin();
    for (auto& dst : sh)
        for (auto& src : sh)
            if (dst != src) {
                copy((dst.get()->*buf).p + (size_t)src->rank * per_shard,
                     (src.get()->*buf).p + (size_t)src->rank * per_shard, bytes);
                src->xsent += bytes;
            }
    xend();
}

// Element-wise sum of a u32 buffer over the shards, result on every shard.
void rp_sim::allreduce_sum(DevBuf<uint32_t> Shard::*buf, size_t count) {
    if (comm) {
        Shard& s = *sh[0];
        comm->allreduce_u32((s.*buf).p, count, s.st);
        s.xsent += 2 * (uint64_t)count * 4 * (G - 1) / G;  // (a ring all-reduce's share)
        return;
    }
    Shard& s0 = *sh[0];
    xbegin();
    for (size_t i = 1; i < sh.size(); i++)
        hipLaunchKernelGGL(rp::k_add_u32, dim3(rp::grid_for(count, 256)), dim3(256), 0, st, (s0.*buf).p,
                           (const uint32_t*)(sh[i].get()->*buf).p, (uint32_t)count);
    for (size_t i = 1; i < sh.size(); i++) {
        copy((sh[i].get()->*buf).p, (s0.*buf).p, count * 4);
        sh[i]->xsent += count * 4;  // (its part in, the sum back)
        s0.xsent += count * 4;
    }
    xend();
}

// Newly allocated local origins of every shard -> every shard (before an
// exchange that may name them; Esc).
void rp_sim::origin_exchange() {
    using namespace rp;
    each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_origin_pack, dim3(1), dim3(1024), 0, s->st, s->d, s->og.p, s->og_cap); });
    allgather_block(&Shard::og, (size_t)sh.front()->og_cap + 1);
    each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_origin_install, dim3(G), dim3(256), 0, s->st, s->d, (const Origin*)s->og.p, s->og_cap); });
}

// Counts staged by the planning kernels -> host (one sync).
void rp_sim::read_counts() {
    each([&](Shard& sr) { Shard* const s = &sr; RP_HIP(hipMemcpyAsync(s->h_xcnt, s->xcnt.p, (size_t)rp::XC_NCAT * G * 8, hipMemcpyDeviceToHost, s->st)); });
    sync_all();
}

// All-to-all of variable segments: shard s sends h_xcnt[cat_send][q] elements
// to shard q (segments in partner order) and receives h_xcnt[cat_recv][r]
// from shard r.
template <class T>
void rp_sim::alltoallv_t(DevBuf<T> Shard::*sendb, DevBuf<T> Shard::*recvb, int cat_send, int cat_recv) {
    const size_t E = sizeof(T);
    if (comm) {
        Shard& s = *sh[0];
        const unsigned long long* sc = s.h_xcnt + (size_t)cat_send * G;
        const unsigned long long* rc = s.h_xcnt + (size_t)cat_recv * G;
        uint64_t so = 0, ro = 0, st_ = 0, rt = 0;
        for (uint32_t q = 0; q < G; q++) { st_ += sc[q]; rt += rc[q]; }
        if (st_ > (s.*sendb).n || rt > (s.*recvb).n)
            throw Error(RP_ERR_CAPACITY, "exchange buffer too small for this round's traffic");
        std::vector<rp::Xfer> sends, recvs;
        for (uint32_t q = 0; q < G; q++) {
            if (q == s.rank) continue;
            if (sc[q]) sends.push_back(rp::Xfer{q, (void*)((s.*sendb).p + so), sc[q] * E});
            if (rc[q]) recvs.push_back(rp::Xfer{q, (void*)((s.*recvb).p + ro), rc[q] * E});
            so += sc[q];
            ro += rc[q];
        }
        comm->sendrecv(sends, recvs, s.st);
        xbytes += so * E;
        s.xsent += so * E;
        return;
    }
    // in process: segment (s -> d) sits at s's send offset for d and d's
    // receive offset for s; both sides must agree on its length
    xbegin();
    for (auto& src : sh) {
        const unsigned long long* sc = src->h_xcnt + (size_t)cat_send * G;
        uint64_t so = 0;
        for (uint32_t q = 0; q < G; q++) {
            if (q != src->rank && sc[q]) {
                Shard& dst = *sh[q];
                const unsigned long long* rc = dst.h_xcnt + (size_t)cat_recv * G;
                if (rc[src->rank] != sc[q]) throw Error(RP_ERR_STATE, "exchange plan mismatch between shards");
                uint64_t ro = 0;
                for (uint32_t r = 0; r < src->rank; r++) ro += rc[r];
                if (so + sc[q] > (src.get()->*sendb).n || ro + sc[q] > (dst.*recvb).n)
                    throw Error(RP_ERR_CAPACITY, "exchange buffer too small for this round's traffic");
                copy((dst.*recvb).p + ro, (src.get()->*sendb).p + so, sc[q] * E);
                xbytes += sc[q] * E;
                src->xsent += sc[q] * E;
            }
            so += sc[q];
        }
    }
    xend();
}

// One ping-req wave's cross-shard messages (k_xs_*): plan, all-gather of the
// per-partner counts (one host sync), pack, all-to-all of records, words and
// escapes, unpack.
template <int W>
void rp_sim::slot_exchange() {
    using namespace rp;
    const uint32_t n3 = 3 * n;
    each([&](Shard& sr) {
            Shard* const s = &sr;
        hipLaunchKernelGGL(k_xs_zero, dim3(1), dim3(256), 0, s->st, s->xcnt.p, G, s->xs_nlist.p);
        hipLaunchKernelGGL(k_xs_plan<W>, dim3(grid_for(n3, 256)), dim3(256), 0, s->st, s->d, s->xs_rec.p, s->xs_w.p,
                           s->xs_e.p, s->xcnt.p);
        hipLaunchKernelGGL(k_xs_fill<W>, dim3(grid_for(n3, 256)), dim3(256), 0, s->st, s->d,
                           (const uint32_t*)s->xs_rec.p, (const uint32_t*)s->xs_w.p, (const uint32_t*)s->xs_e.p,
                           (const unsigned long long*)s->xcnt.p, s->xsend.p, s->xs_wabs.p, s->xs_eabs.p,
                           s->xs_list.p, s->xs_nlist.p, s->xsrow.p);
    });
    allgather_block(&Shard::xsrow, 3 * G);
    each([&](Shard& sr) {
            Shard* const s = &sr;
        RP_HIP(hipMemcpyAsync(s->h_xsrow, s->xsrow.p, (size_t)3 * G * G * 8, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipMemcpyAsync((uint32_t*)(s->h_xsrow + (size_t)3 * G * G), s->xs_nlist.p, 4, hipMemcpyDeviceToHost,
                              s->st));
    });
    sync_all();
    each([&](Shard& sr) {
            Shard* const s = &sr;
        const unsigned long long* m = s->h_xsrow;
        for (uint32_t q = 0; q < G; q++)
            for (int c = 0; c < 3; c++) {
                s->h_xcnt[(size_t)(XS_REC_SEND + 2 * c) * G + q] = m[((size_t)s->rank * 3 + c) * G + q];
                s->h_xcnt[(size_t)(XS_REC_RECV + 2 * c) * G + q] = m[((size_t)q * 3 + c) * G + s->rank];
            }
        s->fit_exchange(W <= 4 ? 0 : 1, s->xsum(XS_W_SEND), s->xsum(XS_E_SEND), s->xsum(XS_W_RECV),
                        s->xsum(XS_E_RECV));
        const uint32_t npack = *(const uint32_t*)(m + (size_t)3 * G * G);
        if (npack)
            hipLaunchKernelGGL(k_xs_pack<W>, dim3(npack), dim3(BLOCK), 0, s->st, s->d, (const uint32_t*)s->xs_list.p,
                               (const uint64_t*)s->xs_wabs.p, (const uint64_t*)s->xs_eabs.p,
                               W <= 4 ? s->sendw.p : s->psendw.p, W <= 4 ? s->sende.p : s->psende.p);
    });
    xbegin();
    alltoallv_t(&Shard::xsend, &Shard::xrecv, XS_REC_SEND, XS_REC_RECV);
    if (W <= 4) {
        alltoallv_t(&Shard::sendw, &Shard::rxw, XS_W_SEND, XS_W_RECV);
        alltoallv_t(&Shard::sende, &Shard::rxe, XS_E_SEND, XS_E_RECV);
    } else {
        alltoallv_t(&Shard::psendw, &Shard::rx2w, XS_W_SEND, XS_W_RECV);
        alltoallv_t(&Shard::psende, &Shard::rx2e, XS_E_SEND, XS_E_RECV);
    }
    xend();
    each([&](Shard& sr) {
            Shard* const s = &sr;
        uint64_t nrec = 0, nw = 0;
        for (uint32_t r = 0; r < G; r++) {
            nrec += s->h_xcnt[(size_t)XS_REC_RECV * G + r];
            nw += s->h_xcnt[(size_t)XS_W_RECV * G + r];
        }
        if (nw > (W <= 4 ? s->rxw.n : s->rx2w.n)) throw Error(RP_ERR_CAPACITY, "exchange buffer too small for this round's traffic");
        if (W == 5 && nw > s->rxc.n) {  // (W5 lists are decoded into rxc, free once k_w4 has run)
            s->rxc.reserve((nw + (1u << 20) - 1) & ~(uint64_t)((1u << 20) - 1));
            s->d.rxc = s->rxc.p;
        }
        if (nrec)
            hipLaunchKernelGGL(k_xs_unpack<W>, dim3((uint32_t)nrec), dim3(BLOCK), 0, s->st, s->d,
                               (const SlotRec*)s->xrecv.p, (const unsigned long long*)s->xsrow.p,
                               (const uint32_t*)(W <= 4 ? s->rxw.p : s->rx2w.p), (const Esc*)(W <= 4 ? s->rxe.p : s->rx2e.p),
                               W <= 5 ? s->rxc.p : nullptr);
    });
}

void rp_sim::choose_churn(int32_t* out, uint32_t r) {
    // oracle/harness/common.js chooseChurn: partial Fisher-Yates over the ids
    // alive in round r, in id order
    std::vector<int32_t> cand;
    cand.reserve(n);
    for (uint32_t i = 0; i < n; i++)
        if (live_at(i, r)) cand.push_back((int32_t)i);
    uint32_t L = (uint32_t)cand.size(), kk = std::min(k, L);
    for (uint32_t j = 0; j < kk; j++) {
        double x = rp::js_math_random(churn_rng);
        uint32_t rr = j + (uint32_t)floor(x * (double)(L - j));
        std::swap(cand[j], cand[rr]);
    }
    for (uint32_t j = 0; j < k; j++) out[j] = j < kk ? cand[j] : -1;
}

// The round's false suspicions (oracle/harness/common.js chooseStorm): K =
// ceil(live * ppm / 10^6) victims by partial Fisher-Yates over the live ids in
// id order, then per victim an accuser drawn uniformly from the other live
// ids.  out = K accusers then K victims, sorted stably by accuser (k_storm).
uint32_t rp_sim::choose_storm(int32_t* out, uint32_t r) {
    if (!storm_ppm || r < storm_start || r >= storm_end) return 0;
    std::vector<int32_t> live;
    live.reserve(n);
    for (uint32_t i = 0; i < n; i++)
        if (live_at(i, r)) live.push_back((int32_t)i);
    const uint64_t L = live.size();
    if (L < 2) return 0;
    const uint32_t K = (uint32_t)std::min<uint64_t>((L * storm_ppm + 999999) / 1000000, L);
    std::vector<int32_t> cand = live;
    for (uint32_t j = 0; j < K; j++) {
        const double x = rp::js_math_random(storm_rng);
        const uint32_t rr = j + (uint32_t)floor(x * (double)(L - j));
        std::swap(cand[j], cand[rr]);
    }
    std::vector<std::pair<int32_t, int32_t>> pr(K);
    for (uint32_t j = 0; j < K; j++) {
        const int32_t v = cand[j];
        const uint64_t pos = (uint64_t)(std::lower_bound(live.begin(), live.end(), v) - live.begin());
        const uint64_t idx = (uint64_t)floor(rp::js_math_random(storm_rng) * (double)(L - 1));
        pr[j] = {live[idx < pos ? idx : idx + 1], v};
    }
    std::stable_sort(pr.begin(), pr.end(), [](const std::pair<int32_t, int32_t>& a, const std::pair<int32_t, int32_t>& b) {
        return a.first < b.first;
    });
    for (uint32_t j = 0; j < K; j++) { out[j] = pr[j].first; out[storm_kmax + j] = pr[j].second; }
    return K;
}

// The round's joins (rp_sim_join; the kernels' comment, "join path").  Every
// shard stages the same lists; a reply is made on its seed's shard and
// shared before the joiners merge.
void rp_sim::join_step(uint32_t r, uint64_t now) {
    using namespace rp;
    std::vector<uint32_t> ids, poff{0}, pidx, pjoin, seed_of;
    std::vector<int32_t> pseed;
    for (const JoinEv& e : joins) {
        if (e.round != r) continue;
        if (fail_round[e.joiner] >= 0 && (uint32_t)fail_round[e.joiner] <= r) continue;  // fail-stopped first: never joins
        ids.push_back(e.joiner);
        for (int32_t sd : e.seeds) {
            if (fail_round[sd] >= 0 && (uint32_t)fail_round[sd] <= r)
                throw Error(RP_ERR_STATE, "a join seed has fail-stopped");
            seed_of.push_back((uint32_t)sd);
        }
        poff.push_back((uint32_t)seed_of.size());
    }
    if (ids.empty()) return;
    const uint32_t J = (uint32_t)ids.size(), P = (uint32_t)seed_of.size();
    // pairs grouped by seed, schedule order kept within a seed (k_join_seed)
    std::vector<uint32_t> perm(P);
    for (uint32_t p = 0; p < P; p++) perm[p] = p;
    std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) { return seed_of[a] < seed_of[b]; });
    {
        std::vector<uint32_t> joiner_of(P);
        for (uint32_t t = 0; t < J; t++)
            for (uint32_t p = poff[t]; p < poff[t + 1]; p++) joiner_of[p] = ids[t];
        for (uint32_t q : perm) { pseed.push_back((int32_t)seed_of[q]); pidx.push_back(q); pjoin.push_back(joiner_of[q]); }
    }
    for (auto& s : sh) {
        auto up = [&](DevBuf<uint32_t>& b, const std::vector<uint32_t>& v) {
            b.reserve(std::max<size_t>(v.size(), 1));
            if (!v.empty()) RP_HIP(hipMemcpyAsync(b.p, v.data(), v.size() * 4, hipMemcpyHostToDevice, s->st));
        };
        up(s->j_ids, ids); up(s->j_poff, poff); up(s->j_pidx, pidx); up(s->j_pjoin, pjoin); up(s->j_seedof, seed_of);
        s->j_pseed.reserve(std::max<size_t>(P, 1));
        if (P) RP_HIP(hipMemcpyAsync(s->j_pseed.p, pseed.data(), P * 4, hipMemcpyHostToDevice, s->st));
        s->jvs.reserve((size_t)std::max(P, 1u) * n); s->jord.reserve((size_t)std::max(P, 1u) * n);
        s->jm.reserve(std::max(P, 1u)); s->jcs.reserve(std::max(P, 1u));
        RP_HIP(hipStreamSynchronize(s->st));  // (the host vectors are temporaries)
        SimDev& d = s->d;
        s->timed(0, [&] {
            hipLaunchKernelGGL(k_join_self, dim3(J), dim3(BLOCK), 0, s->st, d, (const uint32_t*)s->j_ids.p, now);
            if (P) {
                hipLaunchKernelGGL(k_join_seed, dim3(P), dim3(BLOCK), 0, s->st, d, (const int32_t*)s->j_pseed.p,
                                   (const uint32_t*)s->j_pidx.p, (const uint32_t*)s->j_pjoin.p, P, now, s->jvs.p,
                                   s->jord.p, s->jm.p);
                hipLaunchKernelGGL(k_join_csum, dim3(grid_for(P, NWAVE)), dim3(BLOCK), 0, s->st, d,
                                   (const uint32_t*)s->j_seedof.p, P, (const uint64_t*)s->jvs.p, s->jcs.p);
            }
        });
    }
    if (G > 1 && P) {
        // each reply from its seed's shard to every shard
        for (uint32_t p = 0; p < P; p++) {
            const uint32_t root = seed_of[p] / (n / G);
            if (comm) {
                Shard& s0 = *sh[0];
                comm->broadcast((uint8_t*)(s0.jvs.p + (size_t)p * n), (size_t)n * 8, root, s0.st);
                comm->broadcast((uint8_t*)(s0.jord.p + (size_t)p * n), (size_t)n * 4, root, s0.st);
                comm->broadcast((uint8_t*)(s0.jm.p + p), 4, root, s0.st);
                comm->broadcast((uint8_t*)(s0.jcs.p + p), 4, root, s0.st);
            } else {
                Shard& src = *sh[root];
                xbegin();
                for (auto& dst : sh) {
                    if (dst.get() == &src) continue;
                    copy(dst->jvs.p + (size_t)p * n, src.jvs.p + (size_t)p * n, (size_t)n * 8);
                    copy(dst->jord.p + (size_t)p * n, src.jord.p + (size_t)p * n, (size_t)n * 4);
                    copy(dst->jm.p + p, src.jm.p + p, 4);
                    copy(dst->jcs.p + p, src.jcs.p + p, 4);
                }
                xend();
            }
        }
    }
    for (auto& s : sh) {
        SimDev& d = s->d;
        s->timed(0, [&] {
            hipLaunchKernelGGL(k_join_merge, dim3(J), dim3(BLOCK), 0, s->st, d, (const uint32_t*)s->j_ids.p,
                               (const uint32_t*)s->j_poff.p, (const uint32_t*)s->j_seedof.p, (const uint64_t*)s->jvs.p,
                               (const uint32_t*)s->jord.p, (const uint32_t*)s->jm.p, (const uint32_t*)s->jcs.p,
                               s->need_shuffle.p);
            if (s->ncoll)
                hipLaunchKernelGGL(k_join_owners, dim3(grid_for((uint64_t)J * s->ncoll, 256)), dim3(256), 0, s->st, d,
                                   (const uint32_t*)s->j_ids.p, J);
            hipLaunchKernelGGL(k_init_fp, dim3(J), dim3(BLOCK), 0, s->st, d, 0u, (const uint32_t*)s->j_ids.p);
            hipLaunchKernelGGL(k_shuffle, dim3(std::min<uint32_t>(s->nl, 2048)), dim3(BLOCK), (size_t)n * 2, s->st, d,
                               s->need_shuffle.p, 0, (const uint32_t*)nullptr, (const uint32_t*)nullptr);
            hipLaunchKernelGGL(k_mark_joined, dim3(grid_for(J, 256)), dim3(256), 0, s->st, d, (const uint32_t*)s->j_ids.p, J, now);
        });
    }
}

void rp_sim::enqueue_round(bool churn_active, uint32_t slot) {
    using namespace rp;
    const uint64_t now = T0 + PERIOD_MS * round;
    std::vector<int32_t> dead_now;
    if (faults)
        for (uint32_t i = 0; i < n; i++) if (fail_round[i] == (int32_t)round) dead_now.push_back((int32_t)i);
    if (faults && G > 1 && churn_active && k) {
        // refutes change a node's incarnation on its own shard only; churn
        // origins record the re-asserting node's previous incarnation
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_self_inc, dim3(grid_for(s->nl, 256)), dim3(256), 0, s->st, s->d); });
        allgather_nodes(&Shard::self_inc, 1);
    }
    const uint32_t sk = slot < storm_k.size() ? storm_k[slot] : 0;
    for (auto& s : sh) s->fault_mode = faults || part[1] > part[0];
    each([&](Shard& sr) { Shard* const s = &sr; s->stage_start(round, churn_active, slot, dead_now, faults, part, sk); });
    join_step(round, now);
    each([&](Shard& sr) { Shard* const s = &sr; s->stage_churn(churn_active, slot, sk, now); });
    each([&](Shard& sr) { Shard* const s = &sr; s->stage_issue(); });
    if (G > 1) {
        sh.front()->timed(6, [&] {
        // local origins made at this round's start and in the previous round's waves
        if (faults || !joins.empty()) origin_exchange();
        // members declared faulty per shard, for the sender-checksum predicate
        for (auto& s : sh) s->fd_shared = faults;
        if (faults) {
            each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_fdecl_share, dim3(1), dim3(1), 0, s->st, s->d, s->fdecl_all.p + s->rank,
                                   s->faulty_unbounded ? 1u : 0u); });
            allgather_block(&Shard::fdecl_all, 1);
        }
        // ping metadata: every shard learns every sender's target, list
        // lengths, incarnation, fingerprint and the receivers' log state
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_meta_pack, dim3(grid_for(s->nl, 256)), dim3(256), 0, s->st, s->d, s->meta.p); });
        allgather_nodes(&Shard::meta, 1);
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_meta_unpack, dim3(grid_for(n, 256)), dim3(256), 0, s->st, s->d,
                               (const PingMeta*)s->meta.p); });
        });
    }
    each([&](Shard& sr) { Shard* const s = &sr; s->stage_checksums(); });
    if (G > 1) {
        sh.front()->timed(6, [&] {
        allgather_nodes(&Shard::snd_csum, 1);
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_plan_pings, dim3(G, 2), dim3(XB), 0, s->st, s->d, s->soff.p, s->seoff.p, s->rr_idx.p,
                               s->rs_idx.p, s->xcnt.p); });
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_plan_fix_pings, dim3(grid_for(n, 256)), dim3(256), 0, s->st, s->d, s->soff.p,
                               s->seoff.p, s->rr_idx.p, s->rs_idx.p, (const unsigned long long*)s->xcnt.p); });
        read_counts();
        each([&](Shard& sr) { Shard* const s = &sr; s->fit_exchange(0, s->xsum(XC_PING_SEND), s->xsum(XC_PESC_SEND), s->xsum(XC_PING_RECV),
                            s->xsum(XC_PESC_RECV)); });
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_pack_pings, dim3(s->nl), dim3(BLOCK), 0, s->st, s->d, (const uint64_t*)s->soff.p,
                               (const uint64_t*)s->seoff.p, s->sendw.p, s->sende.p); });
        xbegin();
        alltoallv_t(&Shard::sendw, &Shard::rxw, XC_PING_SEND, XC_PING_RECV);
        alltoallv_t(&Shard::sende, &Shard::rxe, XC_PESC_SEND, XC_PESC_RECV);
        xend();
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_expand_pings, dim3(n), dim3(BLOCK), 0, s->st, s->d); });
        });
    }
    each([&](Shard& sr) { Shard* const s = &sr; s->stage_ping_merge(now); });
    if (G > 1) {
        sh.front()->timed(6, [&] {
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_plan_resp, dim3(G), dim3(XB), 0, s->st, s->d, (const uint32_t*)s->rs_idx.p,
                               s->rsend.p, s->psoff.p, s->pseoff.p, s->xcnt.p); });
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_plan_fix_resp, dim3(grid_for(n, 256)), dim3(256), 0, s->st, s->d, s->psoff.p,
                               s->pseoff.p, (const unsigned long long*)s->xcnt.p); });
        // response payload sizes (words, escapes): each shard's outgoing rows -> everyone
        each([&](Shard& sr) {
            Shard* const s = &sr;
            RP_HIP(hipMemcpyAsync(s->xrow.p + (size_t)s->rank * 2 * G, s->xcnt.p + (size_t)XC_PAY_SEND * G, G * 8,
                                  hipMemcpyDeviceToDevice, s->st));
            RP_HIP(hipMemcpyAsync(s->xrow.p + (size_t)s->rank * 2 * G + G, s->xcnt.p + (size_t)XC_RESC_SEND * G, G * 8,
                                  hipMemcpyDeviceToDevice, s->st));
        });
        allgather_block(&Shard::xrow, 2 * G);
        each([&](Shard& sr) { Shard* const s = &sr; RP_HIP(hipMemcpyAsync(s->h_xrow, s->xrow.p, (size_t)2 * G * G * 8, hipMemcpyDeviceToHost, s->st)); });
        read_counts();
        each([&](Shard& sr) {
            Shard* const s = &sr;
            for (uint32_t r = 0; r < G; r++) {
                s->h_xcnt[(size_t)XC_PAY_RECV * G + r] = s->h_xrow[(size_t)r * 2 * G + s->rank];
                s->h_xcnt[(size_t)XC_RESC_RECV * G + r] = s->h_xrow[(size_t)r * 2 * G + G + s->rank];
            }
            s->fit_exchange(1, s->xsum(XC_PAY_SEND), s->xsum(XC_RESC_SEND), s->xsum(XC_PAY_RECV),
                            s->xsum(XC_RESC_RECV));
            hipLaunchKernelGGL(k_pack_resp, dim3(s->nl), dim3(BLOCK), 0, s->st, s->d, (const uint64_t*)s->psoff.p,
                               (const uint64_t*)s->pseoff.p, s->psendw.p, s->psende.p);
        });
        xbegin();
        alltoallv_t(&Shard::rsend, &Shard::rrecv, XC_REC_SEND, XC_REC_RECV);
        alltoallv_t(&Shard::psendw, &Shard::rx2w, XC_PAY_SEND, XC_PAY_RECV);
        alltoallv_t(&Shard::psende, &Shard::rx2e, XC_RESC_SEND, XC_RESC_RECV);
        xend();
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_unpack_resp, dim3(G), dim3(XB), 0, s->st, s->d, (const uint32_t*)s->rr_idx.p,
                               (const RespRec*)s->rrecv.p, (const unsigned long long*)s->xrow.p); });
        });
    }
    each([&](Shard& sr) { Shard* const s = &sr; s->stage_resp_merge(now, faults); });
    if (faults) {
        if (G > 1) sh.front()->timed(6, [&] {
            xbegin();
            allreduce_sum(&Shard::w3cnt, n + 1);
            allreduce_sum(&Shard::w4b, n);
            xend();
        });
        each([&](Shard& sr) { Shard* const s = &sr; s->stage_pr_need(); });
        if (G > 1) sh.front()->timed(6, [&] { slot_exchange<3>(); });
        each([&](Shard& sr) { Shard* const s = &sr; s->stage_wave(3, now); });
        if (G > 1) sh.front()->timed(6, [&] { slot_exchange<4>(); });
        each([&](Shard& sr) { Shard* const s = &sr; s->stage_wave(4, now); });
        if (G > 1) sh.front()->timed(6, [&] { origin_exchange(); slot_exchange<5>(); });  // (W4's verdicts)
        each([&](Shard& sr) { Shard* const s = &sr; s->stage_wave(5, now); });
        if (G > 1) sh.front()->timed(6, [&] { slot_exchange<6>(); });
        each([&](Shard& sr) { Shard* const s = &sr; s->stage_wave(6, now); });
    }
    each([&](Shard& sr) { Shard* const s = &sr; s->stage_end(); });
    if (G > 1) {
        // cluster-wide seen mask for the next round's issues to other shards
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_seen_and, dim3((s->seen_words + 255) / 256, s->nl >> s->d.gsz_log), dim3(256), 0,
                               s->st, s->d, s->gseen.p); });
        allgather_block(&Shard::gseen, (size_t)(sh.front()->nl >> sh.front()->d.gsz_log) * sh.front()->seen_words);
        if (faults) {  // settled masks for the next round's issues to other shards
            const uint32_t pw = (n + 31) / 32;
            each([&](Shard& s) {
                hipLaunchKernelGGL(k_settled_and, dim3((pw + 255) / 256, s.nl >> s.d.fs_log), dim3(256), 0, s.st, s.d,
                                   s.gsettled.p);
            });
            allgather_block(&Shard::gsettled, (size_t)(sh.front()->nl >> sh.front()->d.fs_log) * pw);
        }
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_seen_range, dim3(1), dim3(1), 0, s->st, s->d); });
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_stats_pack, dim3(1), dim3(64), 0, s->st, s->d, (const unsigned long long*)s->fp_mm.p,
                               s->sgather.p, s->ltotals.p); });
        allgather_block(&Shard::sgather, STAT_NSTATS + 2);
        each([&](Shard& sr) { Shard* const s = &sr; hipLaunchKernelGGL(k_stats_combine, dim3(1), dim3(64), 0, s->st, s->d,
                               (const unsigned long long*)s->sgather.p, s->totals.p); });
        xcalls++;
    }
    RP_HIP(hipGetLastError());
    round++;
}

void rp_sim::run(int k_rounds, bool churn_active) {
    RP_HIP(hipSetDevice(dev));
    int done = 0;
    while (done < k_rounds) {
        int batch = std::min<int>(k_rounds - done, (int)CHURN_SLOTS);
        if (churn_active && k) {
            // the staging buffer may still feed the previous batch's copy
            sync_all();
            for (int b = 0; b < batch; b++) choose_churn(h_churn + (size_t)b * k, round + (uint32_t)b);
            for (auto& s : sh)
                RP_HIP(hipMemcpyAsync(s->churn_ids.p, h_churn, (size_t)batch * k * 4, hipMemcpyHostToDevice, s->st));
        }
        storm_k.assign(batch, 0);
        if (storm_kmax && round < storm_end && round + (uint32_t)batch > storm_start) {
            sync_all();
            for (int b = 0; b < batch; b++)
                storm_k[b] = choose_storm(h_storm + (size_t)b * 2 * storm_kmax, round + (uint32_t)b);
            for (auto& s : sh)
                RP_HIP(hipMemcpyAsync(s->storm.p, h_storm, (size_t)batch * 2 * storm_kmax * 4, hipMemcpyHostToDevice,
                                      s->st));
        }
        for (int b = 0; b < batch; b++) enqueue_round(churn_active, (uint32_t)b);
        done += batch;
    }
}

// Fault runs on shards: every suspect and faulty update crosses shards as a
// 16-byte escape and the traffic ramps up within a few rounds; growing the
// exchange buffers then is a free + malloc on a nearly full device (measured:
// one 2.1 GB growth took 568 ms at 65,536 nodes on 4 in-process shards).  So
// once faults are scheduled (before the first round), the buffers are
// presized, split over a shard's ten buffers (4-byte words, 16-byte escapes
// and decoded changes: 112 bytes per element of each).  The budget is a fixed
// share of the device -- 3/8 of its total memory, never more than half of
// what is free now -- divided over every shard that lives on this device (all
// G for in-process shards and for loopback ranks, whose threads presize one
// after the other; one for an RCCL rank), at most 16 GB per shard and n^2/8G
// elements: later simulations, rings and buffer growth keep the rest.
void rp_sim::presize_exchange() {
    for (auto& s : sh) s->ensure_ck_side();  // (one shard: the side stream's rows, used in fault rounds only)
    if (presized || G < 2 || round > 0) return;
    presized = true;
    sync_all();
    size_t fr = 0, tot = 0;
    RP_HIP(hipMemGetInfo(&fr, &tot));
    const uint64_t on_device = loop_rank ? G : (uint64_t)sh.size();
    const uint64_t budget = std::min<uint64_t>((uint64_t)fr / 2, (uint64_t)tot / 8 * 3);
    const uint64_t per = std::min<uint64_t>(budget / on_device, 16ull << 30);
    // (config 5 at 65,536 nodes on 4 shards peaked at ~67 M escapes per
    // buffer; small test clusters need little)
    const uint64_t e = std::min<uint64_t>(per / 112, std::max<uint64_t>((uint64_t)n * n / (8ull * G), 1ull << 20));
    for (auto& s : sh) s->presize(e);
    sync_all();
}

void rp_sim::check_errors() {
    uint32_t e = 0;
    for (auto& s : sh) e |= s->read_err();
    if (!e) return;
    std::string m = "simulation kernel error flags 0x" + std::to_string(e) + ":";
    if (e & rp::SIMERR_ABSENT_MEMBER) m += " change for an absent member (full views only);";
    if (e & rp::SIMERR_TIMERS_FULL) m += " suspicion timer FIFO full;";
    if (e & rp::SIMERR_ORIGIN_FULL) m += " origin table full;";
    if (e & rp::SIMERR_ARENA_FULL) m += " message arena full;";
    if (e & rp::SIMERR_SNAP_FULL) m += " full-sync snapshot slots exhausted;";
    if (e & rp::SIMERR_RINGOPS) m += " too many ring changes in one batch;";
    if (e & rp::SIMERR_PING_FAILED) m += " a node has no pingable member (not modelled on device);";
    if (e & rp::SIMERR_PREDICATE) m += " internal: checksum-snapshot predicate violated;";
    if (e & rp::SIMERR_P2_LIST) m += " internal: a ping-rank receiver list outgrew its launch grid;";
    int code = (e & (rp::SIMERR_ORIGIN_FULL | rp::SIMERR_ARENA_FULL | rp::SIMERR_SNAP_FULL | rp::SIMERR_RINGOPS |
                     rp::SIMERR_TIMERS_FULL))
                   ? RP_ERR_CAPACITY
                   : RP_ERR_UNSUPPORTED;
    throw Error(code, m);
}


extern "C" {

static rp_sim* make_cluster(const rp_sim_config* cfg, uint32_t G, int only_rank, std::unique_ptr<rp::Xport> comm) {
    if (!cfg) throw Error(RP_ERR_INVALID, "null pointer");
    if (cfg->n < 2 || cfg->n > 65536) throw Error(RP_ERR_INVALID, "n must be in [2, 65536]");
    if (cfg->replica_hash_shift >= 32) throw Error(RP_ERR_INVALID, "rp_sim_config.replica_hash_shift must be < 32");
    if (G < 1 || G > rp::MAXG || cfg->n % G) throw Error(RP_ERR_INVALID, "shards must divide n (and be <= 64)");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        throw Error(RP_ERR_HIP, "no HIP device available (ringpop_amd requires an MI355X / gfx950 GPU)");
    RP_HIP(hipSetDevice(rp::current_device()));
    std::unique_ptr<rp_sim> c(new rp_sim());
    c->dev = rp::current_device();
    c->cfg = *cfg;
    c->n = cfg->n;
    c->k = std::min(cfg->churn_k, cfg->n);
    c->G = G;
    c->comm = std::move(comm);
    c->rank = only_rank < 0 ? 0 : (uint32_t)only_rank;
    if (only_rank < 0 && G > 1) {
        RP_HIP(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
        RP_HIP(hipEventCreateWithFlags(&c->xdone, hipEventDisableTiming));
    }
    const uint32_t nl = c->n / G;
    for (uint32_t r = 0; r < G; r++) {
        if (only_rank >= 0 && r != (uint32_t)only_rank) continue;
        std::unique_ptr<Shard> sh(new Shard());
        sh->cfg = *cfg;
        sh->lo = r * nl; sh->nl = nl; sh->rank = r; sh->G = G;
        sh->one_per_process = only_rank >= 0 && G > 1;
        // a stream of its own (setup); exchanges order them (rp_sim::xbegin / xend)
        sh->st = nullptr;
        sh->setup();
        c->sh.push_back(std::move(sh));
    }
    c->fail_round.assign(c->n, -1);
    c->join_round.assign(c->n, -1);
    c->churn_rng = cfg->seed ^ rp::CHURN_XOR;
    RP_HIP(hipHostMalloc((void**)&c->h_churn, (size_t)CHURN_SLOTS * std::max<uint32_t>(c->k, 1) * 4));
    return c.release();
}

int rp_sim_create(const rp_sim_config* cfg, rp_sim** out) {
    return rp::guarded([&] {
        if (!out) throw Error(RP_ERR_INVALID, "null pointer");
        *out = make_cluster(cfg, 1, -1, std::unique_ptr<rp::Xport>());
    });
}

int rp_sim_create_shards(const rp_sim_config* cfg, int nshards, rp_sim** out) {
    return rp::guarded([&] {
        if (!out || nshards < 1) throw Error(RP_ERR_INVALID, "bad argument");
        *out = make_cluster(cfg, (uint32_t)nshards, -1, std::unique_ptr<rp::Xport>());
    });
}

int rp_comm_unique_id(uint8_t* id, size_t cap) {
    return rp::guarded([&] {
        if (!id || cap < sizeof(ncclUniqueId)) throw Error(RP_ERR_INVALID, "id buffer must hold 128 bytes");
        ncclUniqueId u;
        RP_NCCL(ncclGetUniqueId(&u));
        memcpy(id, &u, sizeof u);
    });
}

int rp_sim_create_rank(const rp_sim_config* cfg, int nranks, int rank, const uint8_t* id, rp_sim** out) {
    return rp::guarded([&] {
        if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) throw Error(RP_ERR_INVALID, "bad argument");
        std::unique_ptr<rp::NcclXport> x;
        if (nranks > 1) {
            RP_HIP(hipSetDevice(rp::current_device()));
            ncclUniqueId u;
            memcpy(&u, id, sizeof u);
            x.reset(new rp::NcclXport());
            RP_NCCL(ncclCommInitRank(&x->comm, nranks, u, rank));
        }
        *out = make_cluster(cfg, (uint32_t)nranks, nranks > 1 ? rank : -1, std::move(x));
    });
}

// The RCCL transport on its own (rp::NcclXport, the four calls the rank path
// makes), on small buffers whose contents every rank can predict: rank r's
// all-gather chunk, all-reduce input and sends are functions of (r, peer, i).
// nranks = 1 runs every call on one GPU (the sends and receives go to the
// rank itself), so the library's RCCL linkage, communicator set-up and call
// arguments are exercised where only one GPU is available.
static uint32_t selftest_word(uint32_t from, uint32_t to, uint32_t i) {
    return 0x9E3779B1u * (from + 1) ^ 0x85EBCA6Bu * (to + 7) ^ (i * 2654435761u);
}
int rp_comm_selftest(int nranks, int rank, const uint8_t* id, uint32_t words, uint32_t* failures) {
    return rp::guarded([&] {
        if (!id || !failures || nranks < 1 || rank < 0 || rank >= nranks || words == 0 || words > (1u << 24))
            throw Error(RP_ERR_INVALID, "bad argument");
        RP_HIP(hipSetDevice(rp::current_device()));
        rp::NcclXport x;
        ncclUniqueId u;
        memcpy(&u, id, sizeof u);
        RP_NCCL(ncclCommInitRank(&x.comm, nranks, u, rank));
        const uint32_t G = (uint32_t)nranks, r = (uint32_t)rank, W = words;
        struct StreamGuard {  // (destroyed on every exit, a throw included)
            hipStream_t s = nullptr;
            ~StreamGuard() { if (s) (void)hipStreamDestroy(s); }
        } sg;
        RP_HIP(hipStreamCreateWithFlags(&sg.s, hipStreamNonBlocking));
        const hipStream_t st = sg.s;
        DevBuf<uint32_t> ag, ar, sb, rb;
        ag.alloc((size_t)G * W); ar.alloc(W); sb.alloc((size_t)G * W); rb.alloc((size_t)G * W);
        std::vector<uint32_t> h((size_t)G * W, 0u);
        // all-gather in place: this rank's chunk at base + r * bytes
        for (uint32_t i = 0; i < W; i++) h[(size_t)r * W + i] = selftest_word(r, rp::NONE, i);
        RP_HIP(hipMemcpyAsync(ag.p, h.data(), h.size() * 4, hipMemcpyHostToDevice, st));
        x.allgather((uint8_t*)ag.p, (size_t)W * 4, r, st);
        // all-reduce (sum) of u32
        std::vector<uint32_t> a(W);
        for (uint32_t i = 0; i < W; i++) a[i] = selftest_word(r, 0, i) & 0xFFFFu;
        RP_HIP(hipMemcpyAsync(ar.p, a.data(), (size_t)W * 4, hipMemcpyHostToDevice, st));
        x.allreduce_u32(ar.p, W, st);
        // one grouped send/recv with every rank (itself included), a
        // different length per pair as the exchanges have
        std::vector<uint32_t> sbh((size_t)G * W);
        std::vector<rp::Xfer> sends, recvs;
        for (uint32_t q = 0; q < G; q++) {
            const uint32_t len_s = W - (r + 2 * q) % W, len_r = W - (q + 2 * r) % W;
            for (uint32_t i = 0; i < W; i++) sbh[(size_t)q * W + i] = selftest_word(r, q, i);
            sends.push_back(rp::Xfer{q, sb.p + (size_t)q * W, (size_t)len_s * 4});
            recvs.push_back(rp::Xfer{q, rb.p + (size_t)q * W, (size_t)len_r * 4});
        }
        RP_HIP(hipMemcpyAsync(sb.p, sbh.data(), sbh.size() * 4, hipMemcpyHostToDevice, st));
        RP_HIP(hipMemsetAsync(rb.p, 0, (size_t)G * W * 4, st));
        x.sendrecv(sends, recvs, st);
        std::vector<uint32_t> hag((size_t)G * W), har(W), hrb((size_t)G * W), hbc(W);
        RP_HIP(hipMemcpyAsync(hag.data(), ag.p, hag.size() * 4, hipMemcpyDeviceToHost, st));
        RP_HIP(hipMemcpyAsync(har.data(), ar.p, har.size() * 4, hipMemcpyDeviceToHost, st));
        RP_HIP(hipMemcpyAsync(hrb.data(), rb.p, hrb.size() * 4, hipMemcpyDeviceToHost, st));
        // broadcast from the last rank (reuses ar on the device; the payload
        // has a host vector of its own, so the pageable all-reduce input
        // copied above is never rewritten while that copy may be pending)
        const uint32_t root = G - 1;
        std::vector<uint32_t> bc(W, 0u);
        if (r == root)
            for (uint32_t i = 0; i < W; i++) bc[i] = selftest_word(root, root, i);
        RP_HIP(hipMemcpyAsync(ar.p, bc.data(), (size_t)W * 4, hipMemcpyHostToDevice, st));
        x.broadcast((uint8_t*)ar.p, (size_t)W * 4, root, st);
        RP_HIP(hipMemcpyAsync(hbc.data(), ar.p, hbc.size() * 4, hipMemcpyDeviceToHost, st));
        RP_HIP(hipStreamSynchronize(st));
        uint32_t bad = 0;
        for (uint32_t q = 0; q < G; q++)
            for (uint32_t i = 0; i < W; i++) {
                bad += hag[(size_t)q * W + i] != selftest_word(q, rp::NONE, i);
                const uint32_t len_r = W - (q + 2 * r) % W;
                bad += hrb[(size_t)q * W + i] != (i < len_r ? selftest_word(q, r, i) : 0u);
            }
        for (uint32_t i = 0; i < W; i++) {
            uint32_t want = 0;
            for (uint32_t q = 0; q < G; q++) want += selftest_word(q, 0, i) & 0xFFFFu;
            bad += har[i] != want;
            bad += hbc[i] != selftest_word(root, root, i);
        }
        *failures = bad;
    });
}

int rp_loop_create(int nranks, rp_loop** out) {
    return rp::guarded([&] {
        if (!out || nranks < 2 || nranks > (int)rp::MAXG) throw Error(RP_ERR_INVALID, "nranks must be in [2, 64]");
        *out = new rp_loop((uint32_t)nranks);
    });
}
int rp_loop_destroy(rp_loop* g) {
    delete g;
    return RP_OK;
}
int rp_sim_create_rank_loop(const rp_sim_config* cfg, rp_loop* group, int rank, rp_sim** out) {
    return rp::guarded([&] {
        if (!out || !group || rank < 0 || rank >= (int)group->grp.G) throw Error(RP_ERR_INVALID, "bad argument");
        RP_HIP(hipSetDevice(rp::current_device()));
        std::unique_ptr<rp::Xport> x(new rp::LoopXport(&group->grp, (uint32_t)rank));
        *out = make_cluster(cfg, group->grp.G, rank, std::move(x));
        (*out)->loop_rank = true;
    });
}

int rp_sim_shard_range(rp_sim* s, uint32_t* lo, uint32_t* hi) {
    if (!s || !lo || !hi) return RP_ERR_INVALID;
    *lo = s->sh.front()->lo;
    *hi = s->sh.back()->lo + s->sh.back()->nl;
    return RP_OK;
}

int rp_sim_destroy(rp_sim* s) {
    delete s;
    return RP_OK;
}

int rp_sim_run(rp_sim* s, int k_rounds, int churn_active) {
    return rp::guarded([&] {
        if (!s || k_rounds < 0) throw Error(RP_ERR_INVALID, "bad argument");
        s->run(k_rounds, churn_active != 0);
    });
}

int rp_sim_fail(rp_sim* s, uint32_t node, uint32_t round) {
    return rp::guarded([&] {
        if (!s || node >= s->n) throw Error(RP_ERR_INVALID, "bad node");
        if (round < s->round) throw Error(RP_ERR_INVALID, "round already simulated");
        s->fail_round[node] = (int32_t)round;
        s->faults = true;
        s->presize_exchange();
    });
}

// Arbitrary clusters: the cluster's addresses, then the
// full-view set() bootstrap from given views.  Both before the first round;
// in a multi-process cluster every rank makes the same calls.
int rp_sim_load_addresses(rp_sim* s, const uint8_t* bytes, const uint64_t* off, uint32_t n) {
    return rp::guarded([&] {
        if (!s || !bytes || !off) throw Error(RP_ERR_INVALID, "null pointer");
        if (s->round != 0) throw Error(RP_ERR_STATE, "addresses can only be loaded before the first round");
        if (n != s->n) throw Error(RP_ERR_INVALID, "address count differs from the cluster size");
        // the shards are rebuilt from scratch (full views): views or a join
        // schedule set before would be silently dropped
        if (s->views_set || !s->joins.empty())
            throw Error(RP_ERR_STATE, "addresses must be loaded before rp_sim_set_views / rp_sim_join");
        std::vector<std::string> a(n);
        for (uint32_t i = 0; i < n; i++) {
            if (off[i + 1] < off[i]) throw Error(RP_ERR_INVALID, "offsets must be non-decreasing");
            a[i].assign((const char*)bytes + off[i], (size_t)(off[i + 1] - off[i]));
            if (a[i].empty() || a[i].size() > 4 * rp::ADDR_WORDS) throw Error(RP_ERR_INVALID, "address length must be 1..32 bytes");
            for (unsigned char ch : a[i])
                if (ch < 0x21 || ch > 0x7e) throw Error(RP_ERR_INVALID, "addresses must be printable ASCII");
            // ids are ranks in the reference's sort order (JS string order = byte order for ASCII)
            if (i && !(a[i - 1] < a[i])) throw Error(RP_ERR_INVALID, "addresses must be distinct and sorted");
        }
        RP_HIP(hipSetDevice(s->dev));
        s->sync_all();
        for (auto& old : s->sh) {
            const uint32_t lo = old->lo, nl = old->nl, rank = old->rank, G = old->G;
            const bool opp = old->one_per_process;
            hipStream_t st = old->own_stream ? nullptr : old->st;
            old.reset();  // free the views before the new ones are allocated
            std::unique_ptr<Shard> sh(new Shard());
            sh->cfg = s->cfg;
            sh->lo = lo; sh->nl = nl; sh->rank = rank; sh->G = G;
            sh->one_per_process = opp;
            sh->st = st;
            sh->addrs = a;
            sh->setup();
            if (s->storm_kmax) { sh->storm.alloc((size_t)CHURN_SLOTS * 2 * s->storm_kmax); sh->storm_kmax = s->storm_kmax; }
            old = std::move(sh);
        }
    });
}

int rp_sim_set_views(rp_sim* s, uint32_t node_lo, uint32_t count, const int32_t* status, const int64_t* incarnation) {
    return rp::guarded([&] {
        if (!s || (count && (!status || !incarnation))) throw Error(RP_ERR_INVALID, "null pointer");
        if (s->round != 0) throw Error(RP_ERR_STATE, "views can only be set before the first round");
        if ((uint64_t)node_lo + count > s->n) throw Error(RP_ERR_INVALID, "node range outside the cluster");
        if (!count) return;
        const uint32_t n = s->n;
        std::vector<uint8_t> st((size_t)count * n);
        std::vector<uint64_t> inc((size_t)count * n);
        bool any_suspect = false, any_absent = false;
        for (uint32_t r = 0; r < count; r++)
            for (uint32_t a = 0; a < n; a++) {
                const size_t i = (size_t)r * n + a;
                const int32_t x = status[i];
                if (x < rp::ST_ABSENT || x > rp::ST_LEAVE)
                    throw Error(RP_ERR_INVALID, "view status must be 0..4 (absent, alive, suspect, faulty, leave)");
                any_absent |= x == rp::ST_ABSENT;
                if (node_lo + r == a && x != rp::ST_ALIVE) throw Error(RP_ERR_INVALID, "a node's own entry must be alive");
                if (incarnation[i] < 0 || (uint64_t)incarnation[i] >= (1ull << 53))
                    throw Error(RP_ERR_INVALID, "incarnation must be in [0, 2^53)");
                st[i] = (uint8_t)x;
                inc[i] = (uint64_t)incarnation[i];
                any_suspect |= x == rp::ST_SUSPECT;
            }
        RP_HIP(hipSetDevice(s->dev));
        s->sync_all();
        for (auto& sh : s->sh) {
            DevBuf<uint8_t> dst;
            DevBuf<uint64_t> dinc;
            dst.alloc(st.size()); dinc.alloc(inc.size());
            RP_HIP(hipMemcpyAsync(dst.p, st.data(), st.size(), hipMemcpyHostToDevice, sh->st));
            RP_HIP(hipMemcpyAsync(dinc.p, inc.data(), inc.size() * 8, hipMemcpyHostToDevice, sh->st));
            sh->bootstrap_views(node_lo, count, dst.p, dinc.p, nullptr, s->cfg.seed);
            RP_HIP(hipStreamSynchronize(sh->st));  // (the staging buffers die here)
        }
        s->views_set = true;
        if (any_suspect) {  // bootstrap suspicion timers fire at round 0 (k_timers)
            s->faults = true;
            s->presize_exchange();
        }
        if (any_absent)
            for (auto& sh : s->sh) sh->join_mode = true;  // partial views: the merges splice new members
        s->check_errors();
    });
}

int rp_sim_join(rp_sim* s, const uint32_t* joiners, const uint32_t* rounds, const int32_t* seeds, uint32_t count,
                uint32_t seeds_per) {
    return rp::guarded([&] {
        if (!s || (count && (!joiners || !rounds || (seeds_per && !seeds)))) throw Error(RP_ERR_INVALID, "null pointer");
        if (s->round != 0) throw Error(RP_ERR_STATE, "joins can only be scheduled before the first round");
        if (!s->joins.empty()) throw Error(RP_ERR_STATE, "the join schedule is already set");
        const uint32_t n = s->n;
        std::vector<int32_t> jr(n, -1);
        for (uint32_t i = 0; i < count; i++) {
            if (joiners[i] >= n) throw Error(RP_ERR_INVALID, "joiner id out of range");
            if (jr[joiners[i]] >= 0) throw Error(RP_ERR_INVALID, "a node joins once");
            if (rounds[i] > (1u << 30)) throw Error(RP_ERR_INVALID, "join round out of range");
            jr[joiners[i]] = (int32_t)rounds[i];
        }
        std::vector<rp_sim::JoinEv> ev;
        for (uint32_t i = 0; i < count; i++) {
            rp_sim::JoinEv e{rounds[i], joiners[i], {}};
            for (uint32_t q = 0; q < seeds_per; q++) {
                const int32_t sd = seeds[(size_t)i * seeds_per + q];
                if (sd < 0) continue;
                if ((uint32_t)sd >= n || (uint32_t)sd == joiners[i]) throw Error(RP_ERR_INVALID, "bad join seed");
                // a seed is in the cluster before the joiner's round (a member from the start, or joined earlier)
                if (jr[sd] >= 0 && (uint32_t)jr[sd] >= rounds[i])
                    throw Error(RP_ERR_INVALID, "a join seed must have joined in an earlier round");
                e.seeds.push_back(sd);
            }
            ev.push_back(std::move(e));
        }
        RP_HIP(hipSetDevice(s->dev));
        s->sync_all();
        std::vector<uint8_t> map(n);
        std::vector<uint32_t> ids;
        for (uint32_t a = 0; a < n; a++) { map[a] = jr[a] < 0; if (jr[a] >= 0) ids.push_back(a); }
        for (auto& sh : s->sh) {
            DevBuf<uint8_t> dmap;
            DevBuf<uint32_t> dids;
            dmap.alloc(n); dids.alloc(std::max<size_t>(ids.size(), 1));
            RP_HIP(hipMemcpyAsync(dmap.p, map.data(), n, hipMemcpyHostToDevice, sh->st));
            if (!ids.empty()) RP_HIP(hipMemcpyAsync(dids.p, ids.data(), ids.size() * 4, hipMemcpyHostToDevice, sh->st));
            // the members from the start: bootstrapped with each other only
            sh->bootstrap_views(0, n, nullptr, nullptr, dmap.p, s->cfg.seed);
            if (!ids.empty())
                hipLaunchKernelGGL(rp::k_join_reset, dim3((uint32_t)ids.size()), dim3(rp::BLOCK), 0, sh->st, sh->d,
                                   (const uint32_t*)dids.p, (uint32_t)ids.size(), s->cfg.seed);
            RP_HIP(hipGetLastError());
            RP_HIP(hipStreamSynchronize(sh->st));
            sh->join_mode = true;
        }
        s->joins = std::move(ev);
        s->join_round = jr;
        s->check_errors();
    });
}

int rp_sim_storm(rp_sim* s, uint32_t start, uint32_t end, uint32_t ppm) {
    return rp::guarded([&] {
        if (!s) throw Error(RP_ERR_INVALID, "null sim");
        if (ppm > 1000000) throw Error(RP_ERR_INVALID, "ppm must be <= 10^6");
        if (s->round > start) throw Error(RP_ERR_INVALID, "storm must start at a round not yet simulated");
        s->sync_all();
        s->storm_start = start; s->storm_end = end; s->storm_ppm = ppm;
        s->storm_rng = s->cfg.seed ^ rp::STORM_XOR;
        const uint32_t kmax = ppm && end > start ? (uint32_t)std::min<uint64_t>(((uint64_t)s->n * ppm + 999999) / 1000000, s->n) : 0;
        if (kmax > s->storm_kmax) {
            if (s->h_storm) (void)hipHostFree(s->h_storm);
            s->h_storm = nullptr;
            RP_HIP(hipHostMalloc((void**)&s->h_storm, (size_t)CHURN_SLOTS * 2 * kmax * 4));
            for (auto& sh : s->sh) { sh->storm.alloc((size_t)CHURN_SLOTS * 2 * kmax); sh->storm_kmax = kmax; }
            s->storm_kmax = kmax;
        }
        if (kmax) { s->faults = true; s->presize_exchange(); }  // suspicion timers, ping-req waves
    });
}

int rp_sim_partition(rp_sim* s, uint32_t start, uint32_t end, uint32_t split) {
    return rp::guarded([&] {
        if (!s) throw Error(RP_ERR_INVALID, "null sim");
        s->part[0] = start; s->part[1] = end; s->part[2] = split;
        if (split > 0 && end > start) { s->faults = true; s->presize_exchange(); }
    });
}

int rp_sim_sync(rp_sim* s) {
    return rp::guarded([&] {
        if (!s) throw Error(RP_ERR_INVALID, "null sim");
        RP_HIP(hipSetDevice(s->dev));
        s->check_errors();
    });
}

static void read_stats(rp_sim* c, const unsigned long long* src, rp_round_stats* out, bool with_conv) {
    Shard* s = c->sh.front().get();
    unsigned long long h[rp::STAT_NSTATS + 1] = {0};
    RP_HIP(hipMemcpyAsync(h, src, (rp::STAT_NSTATS + (with_conv ? 0 : 1)) * 8, hipMemcpyDeviceToHost, s->st));
    uint32_t conv = 0;
    if (with_conv) RP_HIP(hipMemcpyAsync(&conv, s->conv.p, 4, hipMemcpyDeviceToHost, s->st));
    RP_HIP(hipStreamSynchronize(s->st));
    out->evaluated = h[rp::STAT_EVALUATED];
    out->applied = h[rp::STAT_APPLIED];
    out->full_syncs = h[rp::STAT_FULLSYNC];
    out->messages = h[rp::STAT_MESSAGES];
    out->waves = h[rp::STAT_WAVES];
    out->pings = h[rp::STAT_PINGS];
    out->converged = with_conv ? conv : h[rp::STAT_NSTATS];
}

int rp_sim_round(rp_sim* s, int churn_active, rp_round_stats* stats) {
    return rp::guarded([&] {
        if (!s) throw Error(RP_ERR_INVALID, "null sim");
        s->run(1, churn_active != 0);
        s->check_errors();
        if (stats) read_stats(s, s->sh.front()->stats.p, stats, true);
    });
}

int rp_sim_totals(rp_sim* s, rp_round_stats* totals) {
    return rp::guarded([&] {
        if (!s || !totals) throw Error(RP_ERR_INVALID, "null pointer");
        RP_HIP(hipSetDevice(s->dev));
        s->check_errors();
        read_stats(s, s->sh.front()->totals.p, totals, false);
    });
}

int rp_sim_counters(rp_sim* c, uint64_t* out, int cap, int* n) {
    return rp::guarded([&] {
        if (!c || !out || !n) throw Error(RP_ERR_INVALID, "null pointer");
        c->check_errors();
        Shard* s = c->sh.front().get();
        unsigned long long h[rp::STAT_NSTATS + 1];
        RP_HIP(hipMemcpyAsync(h, s->totals.p, sizeof h, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipStreamSynchronize(s->st));
        int m = std::min(cap, (int)rp::STAT_NSTATS + 1);
        for (int i = 0; i < m; i++) out[i] = h[i];
        *n = rp::STAT_NSTATS + 1;
    });
}

int rp_sim_local_counters(rp_sim* c, uint64_t* out, int cap, int* n) {
    return rp::guarded([&] {
        if (!c || !out || !n) throw Error(RP_ERR_INVALID, "null pointer");
        if (c->G == 1) {
            int rc = rp_sim_counters(c, out, cap, n);
            if (rc) throw Error(rc, rp_last_error());
            return;
        }
        c->check_errors();
        std::vector<unsigned long long> acc(rp::STAT_NSTATS + 1, 0), h(rp::STAT_NSTATS + 1);
        for (auto& s : c->sh) {
            RP_HIP(hipMemcpyAsync(h.data(), s->ltotals.p, h.size() * 8, hipMemcpyDeviceToHost, s->st));
            RP_HIP(hipStreamSynchronize(s->st));
            for (size_t i = 0; i < h.size(); i++) acc[i] += h[i];
        }
        int m = std::min(cap, (int)rp::STAT_NSTATS + 1);
        for (int i = 0; i < m; i++) out[i] = acc[i];
        *n = rp::STAT_NSTATS + 1;
    });
}

int rp_sim_rounds(rp_sim* s, uint32_t* rounds) {
    if (!s || !rounds) return RP_ERR_INVALID;
    *rounds = s->round;
    return RP_OK;
}

int rp_sim_size(rp_sim* c, uint32_t* n) {
    if (!c || !n) return RP_ERR_INVALID;
    *n = c->n;
    return RP_OK;
}

int rp_sim_view_counts(rp_sim* c, uint32_t* out, size_t cap) {
    return rp::guarded([&] {
        if (!c || !out) throw Error(RP_ERR_INVALID, "null pointer");
        if (cap < (size_t)c->n * 6) throw Error(RP_ERR_INVALID, "counts buffer holds fewer than 6 n entries");
        memset(out, 0, (size_t)c->n * 6 * 4);
        for (auto& sp : c->sh) {
            Shard* s = sp.get();
            DevBuf<uint32_t> d((size_t)s->n * 6);
            hipLaunchKernelGGL(rp::k_view_counts, dim3(s->nl), dim3(rp::BLOCK), 0, s->st, s->d, d.p);
            RP_HIP(hipGetLastError());
            RP_HIP(hipMemcpyAsync(out + (size_t)s->lo * 6, d.p + (size_t)s->lo * 6, (size_t)s->nl * 24,
                                  hipMemcpyDeviceToHost, s->st));
            RP_HIP(hipStreamSynchronize(s->st));
        }
    });
}

int rp_sim_read_checksums(rp_sim* c, uint32_t* out, size_t cap) {
    return rp::guarded([&] {
        if (!c || !out) throw Error(RP_ERR_INVALID, "null pointer");
        if (cap < c->n) throw Error(RP_ERR_INVALID, "checksum buffer holds fewer than n entries");
        memset(out, 0, (size_t)c->n * 4);  // nodes of other processes' shards stay 0
        for (auto& sp : c->sh) {
            Shard* s = sp.get();
            DevBuf<uint32_t> d(s->n);
            // every local view, one wave per distinct view (Shard::checksums)
            hipLaunchKernelGGL(rp::k_list_local, dim3(rp::grid_for(s->nl, 256)), dim3(256), 0, s->st, s->d,
                               s->ck_list.p, s->ck_count.p);
            s->checksums(d.p);
            RP_HIP(hipGetLastError());
            RP_HIP(hipMemcpyAsync(out + s->lo, d.p + s->lo, s->nl * 4, hipMemcpyDeviceToHost, s->st));
            RP_HIP(hipStreamSynchronize(s->st));
        }
    });
}

// ---- wire bridge (node-level ping path between rounds) ----------------------
static Shard& bridge_shard(rp_sim* c, uint32_t v) {
    if (!c || v >= c->n) throw Error(RP_ERR_INVALID, "bad node");
    Shard& s = c->owner_of(v);
    s.d.round = c->round;  // the clock of the next round (local overrides, timers)
    s.faulty_unbounded = true;
    return s;
}
// the bridge's counters are not a round's: clear them; surface kernel errors
static void bridge_done(rp_sim* c, Shard& s) {
    RP_HIP(hipMemsetAsync(s.bstats.p, 0, s.bstats.bytes(), s.st));
    RP_HIP(hipGetLastError());
    c->check_errors();
}
static void check_rows(Shard& s, const rp_change* rows, uint32_t n) {
    if (n && !rows) throw Error(RP_ERR_INVALID, "null changes");
    for (uint32_t i = 0; i < n; i++) {
        const rp_change& r = rows[i];
        if (r.address < 0 || r.address >= (int64_t)s.n || r.status < rp::ST_ALIVE || r.status > rp::ST_LEAVE ||
            r.source < -1 || r.source >= (int64_t)s.n || r.incarnation < 0 || r.incarnation >= (1ll << 53) ||
            r.source_incarnation < 0)
            throw Error(RP_ERR_INVALID, "change " + std::to_string(i) + ": address, status or incarnation out of range");
    }
}
static uint32_t bridge_apply(Shard& s, uint32_t v, const rp_change* rows, uint32_t n, uint64_t now) {
    if (n == 0) return 0;
    check_rows(s, rows, n);
    static_assert(sizeof(rp_change) == sizeof(rp::WireRow), "rp_change is the wire row");
    DevBuf<rp::WireRow> dr(n);
    DevBuf<Change> dc(n);
    DevBuf<uint32_t> da(1);
    RP_HIP(hipMemcpyAsync(dr.p, rows, n * sizeof(rp_change), hipMemcpyHostToDevice, s.st));
    hipLaunchKernelGGL(rp::k_bridge_origins, dim3(rp::grid_for(n, 256)), dim3(256), 0, s.st, s.d, (const rp::WireRow*)dr.p,
                       n, dc.p);
    hipLaunchKernelGGL(rp::k_bridge_apply, dim3(1), dim3(rp::BLOCK), 0, s.st, s.d, v, (const Change*)dc.p, n, now, da.p);
    uint32_t applied = 0;
    RP_HIP(hipMemcpyAsync(&applied, da.p, 4, hipMemcpyDeviceToHost, s.st));
    RP_HIP(hipStreamSynchronize(s.st));
    return applied;
}
static std::vector<rp::WireRow> bridge_issue(Shard& s, uint32_t v, bool filter, int64_t fsrc, uint64_t finc) {
    DevBuf<uint64_t> res(2);
    RP_HIP(hipMemsetAsync(s.arena_cursor.p, 0, s.arena_cursor.bytes(), s.st));  // the last round's messages are dead
    hipLaunchKernelGGL(rp::k_bridge_issue, dim3(1), dim3(rp::BLOCK), 0, s.st, s.d, v, filter ? 1 : 0,
                       fsrc < 0 ? rp::NONE : (uint32_t)fsrc, finc, res.p);
    uint64_t h[2] = {0, 0};
    RP_HIP(hipMemcpyAsync(h, res.p, 16, hipMemcpyDeviceToHost, s.st));
    RP_HIP(hipStreamSynchronize(s.st));
    std::vector<rp::WireRow> out(h[1]);
    if (h[1]) {
        DevBuf<rp::WireRow> dr(h[1]);
        hipLaunchKernelGGL(rp::k_bridge_rows, dim3(rp::grid_for(h[1], 256)), dim3(256), 0, s.st, s.d,
                           (const Change*)(s.arena.p + h[0]), (uint32_t)h[1], dr.p);
        RP_HIP(hipMemcpyAsync(out.data(), dr.p, h[1] * sizeof(rp::WireRow), hipMemcpyDeviceToHost, s.st));
        RP_HIP(hipStreamSynchronize(s.st));
    }
    return out;
}
static void bridge_checksum(Shard& s, uint32_t v, uint32_t* checksum, uint64_t* inc) {
    DevBuf<uint64_t> d(2);
    hipLaunchKernelGGL(rp::k_bridge_checksum, dim3(1), dim3(64), 0, s.st, s.d, v, d.p);
    uint64_t h[2];
    RP_HIP(hipMemcpyAsync(h, d.p, 16, hipMemcpyDeviceToHost, s.st));
    RP_HIP(hipStreamSynchronize(s.st));
    if (checksum) *checksum = (uint32_t)h[0];
    if (inc) *inc = h[1];
}
static void rows_out(const std::vector<rp::WireRow>& r, rp_change* out, uint32_t cap, uint32_t* count) {
    if (count) *count = (uint32_t)r.size();
    if (r.size() > cap || (!out && !r.empty())) throw Error(RP_ERR_INVALID, "changes buffer too small");
    if (!r.empty()) memcpy(out, r.data(), r.size() * sizeof(rp_change));
}

int rp_sim_ping_body(rp_sim* c, uint32_t node, rp_change* out, uint32_t cap, uint32_t* count, uint32_t* checksum,
                     uint64_t* incarnation) {
    return rp::guarded([&] {
        Shard& s = bridge_shard(c, node);
        // a list never exceeds the n live keys of the log: check the buffer
        // before the issue consumes piggyback counts
        if (!out || cap < c->n) throw Error(RP_ERR_INVALID, "changes buffer must hold n entries");
        const std::vector<rp::WireRow> r = bridge_issue(s, node, false, -1, 0);
        bridge_checksum(s, node, checksum, incarnation);
        bridge_done(c, s);
        rows_out(r, out, cap, count);
    });
}

int rp_sim_handle_ping(rp_sim* c, uint32_t node, int64_t source, uint64_t source_incarnation, uint32_t checksum,
                       const rp_change* changes, uint32_t n, rp_change* out, uint32_t cap, uint32_t* count,
                       uint32_t* applied, int* full_sync) {
    return rp::guarded([&] {
        Shard& s = bridge_shard(c, node);
        if (source < -1 || source >= (int64_t)c->n) throw Error(RP_ERR_INVALID, "bad source");
        // the response (a list or a fullSync) holds at most n changes: check
        // the buffer before the update and the issue change any state
        if (!out || cap < c->n) throw Error(RP_ERR_INVALID, "changes buffer must hold n entries");
        check_rows(s, changes, n);
        const uint64_t now = rp::T0 + rp::PERIOD_MS * c->round;
        const uint32_t a = bridge_apply(s, node, changes, n, now);
        std::vector<rp::WireRow> r = bridge_issue(s, node, true, source, source_incarnation);
        int fs = 0;
        if (r.empty()) {  // lib/dissemination.js:102-117
            uint32_t mine = 0;
            bridge_checksum(s, node, &mine, nullptr);
            if (mine != checksum) {
                fs = 1;
                uint32_t m = 0;
                RP_HIP(hipMemcpyAsync(&m, s.mcount.p + node, 4, hipMemcpyDeviceToHost, s.st));
                RP_HIP(hipStreamSynchronize(s.st));
                DevBuf<rp::WireRow> dr(std::max(m, 1u));
                hipLaunchKernelGGL(rp::k_bridge_fullsync, dim3(rp::grid_for(std::max(m, 1u), 256)), dim3(256), 0, s.st, s.d, node, dr.p);
                r.resize(m);
                if (m) RP_HIP(hipMemcpyAsync(r.data(), dr.p, m * sizeof(rp::WireRow), hipMemcpyDeviceToHost, s.st));
                RP_HIP(hipStreamSynchronize(s.st));
            }
        }
        bridge_done(c, s);
        if (applied) *applied = a;
        if (full_sync) *full_sync = fs;
        rows_out(r, out, cap, count);
    });
}

int rp_sim_update(rp_sim* c, uint32_t node, const rp_change* changes, uint32_t n, uint32_t* applied) {
    return rp::guarded([&] {
        Shard& s = bridge_shard(c, node);
        const uint32_t a = bridge_apply(s, node, changes, n, rp::T0 + rp::PERIOD_MS * c->round);
        bridge_done(c, s);
        if (applied) *applied = a;
    });
}

int rp_sim_read_view(rp_sim* c, uint32_t node, uint8_t* status, uint64_t* inc, size_t cap) {
    return rp::guarded([&] {
        if (!c || node >= c->n) throw Error(RP_ERR_INVALID, "bad node");
        if (cap < c->n) throw Error(RP_ERR_INVALID, "view buffers hold fewer than n entries");
        Shard* s = &c->owner_of(node);
        std::vector<rp::VEnt> row(s->n);
        RP_HIP(hipMemcpyAsync(row.data(), s->view.p + s->d.row(node), s->n * sizeof(rp::VEnt),
                              hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipStreamSynchronize(s->st));
        for (uint32_t a = 0; a < s->n; a++) {
            if (status) status[a] = (uint8_t)rp::v_status(row[a].vs);
            if (inc) inc[a] = rp::v_inc(row[a].vs);
        }
    });
}

int rp_sim_read_members(rp_sim* c, uint32_t node, uint32_t* out, size_t cap, uint32_t* count) {
    return rp::guarded([&] {
        if (!c || node >= c->n || !out) throw Error(RP_ERR_INVALID, "bad argument");
        if (cap < c->n) throw Error(RP_ERR_INVALID, "members buffer holds fewer than n entries");
        Shard* s = &c->owner_of(node);
        uint32_t m = 0;
        RP_HIP(hipMemcpyAsync(&m, s->mcount.p + node, 4, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipStreamSynchronize(s->st));
        if (m) RP_HIP(hipMemcpyAsync(out, s->order.p + s->d.row(node), (size_t)m * 4, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipStreamSynchronize(s->st));
        if (count) *count = m;
    });
}

int rp_sim_read_changes(rp_sim* c, uint32_t node, int64_t* rows, uint32_t cap, uint32_t* count) {
    return rp::guarded([&] {
        if (!c || node >= c->n) throw Error(RP_ERR_INVALID, "bad node");
        Shard* s = &c->owner_of(node);
        const uint32_t n = s->n;
        std::vector<uint32_t> ko(n), ad(n);
        std::vector<uint64_t> vs(n);
        std::vector<rp::Origin> org(n);
        uint32_t head = 0, tail = 0, ic = 0;
        const size_t row = s->d.row(node);
        DevBuf<rp::Origin> dorg(n);
        DevBuf<uint32_t> dad(n);
        RP_HIP(hipMemcpyAsync(dad.p, s->dad.p + row, n * 4, hipMemcpyDeviceToDevice, s->st));
        hipLaunchKernelGGL(rp::k_log_origins, dim3(rp::grid_for(n, 256)), dim3(256), 0, s->st, s->d, node, dorg.p, dad.p);
        RP_HIP(hipGetLastError());
        RP_HIP(hipMemcpyAsync(ko.data(), s->dko.p + row, n * 4, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipMemcpyAsync(ad.data(), dad.p, n * 4, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipMemcpyAsync(vs.data(), s->dvs.p + row, n * 8, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipMemcpyAsync(org.data(), dorg.p, n * sizeof(rp::Origin), hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipMemcpyAsync(&ic, s->icount.p + node, 4, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipMemcpyAsync(&head, s->dhead.p + node, 4, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipMemcpyAsync(&tail, s->dtail.p + node, 4, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipStreamSynchronize(s->st));
        uint32_t kk = 0;
        for (uint32_t p = head; p < tail; p++) {
            const uint32_t slot = p % n, key = ko[slot], ow = rp::log_origin(key);
            if (rp::is_tomb(key)) continue;
            const uint32_t cnt = rp::entry_count(key, ic);
            const bool undef = cnt == 0 && !((key >> 24) & rp::STAMP_DEFINED);
            if (rows && kk < cap) {
                int64_t* r = rows + 6 * (size_t)kk;
                const rp::Origin& o = org[slot];
                r[0] = ad[slot];
                r[1] = undef ? -1 : (int64_t)cnt;
                r[2] = o.source == rp::NONE ? -1 : (int64_t)o.source;
                r[3] = (int64_t)o.source_inc;
                const uint64_t val = (ow & rp::ORIGIN_ALIVE) ? rp::alive_value(o) : vs[slot];
                r[4] = rp::v_status(val);
                r[5] = (int64_t)rp::v_inc(val);
            }
            kk++;
        }
        if (count) *count = kk;
        if (rows && kk > cap) throw Error(RP_ERR_INVALID, "rows buffer too small");
    });
}

int rp_sim_node_info(rp_sim* c, uint32_t node, int64_t* info) {
    return rp::guarded([&] {
        if (!c || node >= c->n || !info) throw Error(RP_ERR_INVALID, "bad argument");
        Shard* s = &c->owner_of(node);
        int32_t mpb = 0, rc = 0, ii = 0, ir = 0;
        uint8_t dd = 0;
        uint64_t rs = 0;
        std::vector<uint8_t> inr(s->n);
        RP_HIP(hipMemcpyAsync(&mpb, s->max_pb.p + node, 4, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipMemcpyAsync(&rc, s->ring_count.p + node, 4, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipMemcpyAsync(&ii, s->iter_index.p + node, 4, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipMemcpyAsync(&ir, s->iter_round.p + node, 4, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipMemcpyAsync(&dd, s->dead.p + node, 1, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipMemcpyAsync(&rs, s->rng.p + node, 8, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipMemcpyAsync(inr.data(), s->in_ring.p + s->d.row(node), s->n, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipStreamSynchronize(s->st));
        // ring checksum: hash32(sorted server names joined by ';') (lib/ring.js:96-105)
        std::string str;
        for (uint32_t a = 0; a < s->n; a++) {
            if (!inr[a]) continue;
            if (!str.empty()) str += ';';
            str += s->addrs[a];
        }
        uint32_t rcs = 0;
        int e = rp_hash32((const uint8_t*)str.data(), str.size(), &rcs);
        if (e) throw Error(e, rp_last_error());
        info[0] = mpb; info[1] = rc; info[2] = rcs; info[3] = ii; info[4] = ir; info[5] = dd;
        info[6] = (int64_t)rs; info[7] = 0;
    });
}

int rp_sim_ring_lookup(rp_sim* c, uint32_t node, const uint32_t* key_hashes, size_t nk, int32_t* owners) {
    return rp::guarded([&] {
        if (!c || node >= c->n) throw Error(RP_ERR_INVALID, "bad node");
        if (nk == 0) return;
        Shard* s = &c->owner_of(node);
        DevBuf<uint32_t> dh(nk);
        DevBuf<int32_t> dout(nk);
        RP_HIP(hipMemcpyAsync(dh.p, key_hashes, nk * 4, hipMemcpyHostToDevice, s->st));
        hipLaunchKernelGGL(rp::k_view_lookup, dim3(rp::grid_for(nk, 256)), dim3(256), 0, s->st, s->d, node,
                           s->pt_hash.p, s->pt_server.p, s->pt_coll.p, s->npts, dh.p, (uint32_t)nk, dout.p);
        RP_HIP(hipGetLastError());
        RP_HIP(hipMemcpyAsync(owners, dout.p, nk * 4, hipMemcpyDeviceToHost, s->st));
        RP_HIP(hipStreamSynchronize(s->st));
    });
}

int rp_sim_address(rp_sim* c, uint32_t node, char* buf, size_t cap) {
    if (!c || node >= c->n || !buf) return RP_ERR_INVALID;
    const std::string& a = c->sh.front()->addrs[node];
    if (cap < a.size() + 1) return RP_ERR_INVALID;
    memcpy(buf, a.c_str(), a.size() + 1);
    return RP_OK;
}

int rp_sim_enable_timing(rp_sim* c, int enable) {
    return rp_sim_enable_timing_stages(c, enable ? (1u << NCAT) - 1u : 0u);
}

int rp_sim_enable_timing_stages(rp_sim* c, uint32_t mask) {
    return rp::guarded([&] {
        if (!c) throw Error(RP_ERR_INVALID, "null sim");
        for (auto& s : c->sh) {
            RP_HIP(hipStreamSynchronize(s->st));
            s->collect_timing();
            if (s->st2) RP_HIP(hipStreamSynchronize(s->st2));
            s->collect_timing();
            s->timing = mask & ((1u << NCAT) - 1u);
            for (int i = 0; i < NCAT; i++) { s->kms[i] = 0; s->klaunch[i] = 0; }
            s->side_ms = 0;
        }
        c->xbytes = 0; c->xcalls = 0;
        for (auto& s : c->sh) s->xsent = 0;
    });
}

int rp_sim_kernel_times(rp_sim* c, double* ms6, uint64_t* launches6) {
    return rp::guarded([&] {
        if (!c) throw Error(RP_ERR_INVALID, "null sim");
        for (int i = 0; i < 6; i++) {
            if (ms6) ms6[i] = 0;
            if (launches6) launches6[i] = 0;
        }
        for (auto& s : c->sh) {
            RP_HIP(hipStreamSynchronize(s->st));
            if (s->st2) RP_HIP(hipStreamSynchronize(s->st2));
            s->collect_timing();
            for (int i = 0; i < 6; i++) {
                if (ms6) ms6[i] += s->kms[i];
                if (launches6) launches6[i] += s->klaunch[i];
            }
        }
    });
}

int rp_sim_side_ms(rp_sim* c, double* ms) {
    return rp::guarded([&] {
        if (!c || !ms) throw Error(RP_ERR_INVALID, "null pointer");
        *ms = 0;
        for (auto& s : c->sh) {
            RP_HIP(hipStreamSynchronize(s->st));
            if (s->st2) RP_HIP(hipStreamSynchronize(s->st2));
            s->collect_timing();
            *ms += s->side_ms;
        }
    });
}

int rp_sim_exchange_shard_bytes(rp_sim* c, uint64_t* out, int cap, int* count) {
    if (!c || !out || !count || cap < 0) return RP_ERR_INVALID;
    *count = (int)c->sh.size();
    for (size_t i = 0; i < c->sh.size() && (int)i < cap; i++) out[i] = c->sh[i]->xsent;
    return RP_OK;
}

int rp_sim_exchange_stats(rp_sim* c, double* ms, uint64_t* bytes_sent, uint64_t* rounds) {
    if (!c) return RP_ERR_INVALID;
    int rc = rp::guarded([&] {
        RP_HIP(hipStreamSynchronize(c->sh.front()->st));
        c->sh.front()->collect_timing();
    });
    if (rc) return rc;
    if (ms) *ms = c->sh.front()->kms[6];
    if (bytes_sent) *bytes_sent = c->xbytes;
    if (rounds) *rounds = c->xcalls;
    return RP_OK;
}

}  // extern "C"
