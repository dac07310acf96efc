// Device-resident simulation of N ringpop instances (host-side declarations).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "rp_common.h"

namespace rp {

// Error bits raised by kernels (rp_sim_* returns them as RP_ERR_*)
enum : uint32_t {
    SIMERR_ABSENT_MEMBER = 1u << 0,  // change for an address missing from a full view
    SIMERR_TIMERS_FULL = 1u << 1,    // suspicion timer FIFO full
    SIMERR_ORIGIN_FULL = 1u << 2,
    SIMERR_ARENA_FULL = 1u << 3,
    SIMERR_SNAP_FULL = 1u << 4,
    SIMERR_RINGOPS = 1u << 5,
    SIMERR_PING_FAILED = 1u << 6,
    SIMERR_PREDICATE = 1u << 7,      // internal: a response the predicate proved non-empty was empty
    SIMERR_P2_LIST = 1u << 8,        // internal: a ping-rank receiver list outgrew its launch grid
};

// RESP_LIST_RX: a list (or an expanded fullSync) that arrived from another
// shard; its changes are in SimDev::rx2 at `off`.
enum : int32_t { RESP_NONE = 0, RESP_LIST = 1, RESP_EMPTY = 2, RESP_FS_PENDING = 3, RESP_FS = 4, RESP_ERR = 5,
                 RESP_LIST_RX = 6 };

// A response message: a change list in the arena, an empty list, a fullSync
// (snapshot of the responder's view) or a transport error.
struct Resp {
    int32_t kind;
    uint32_t from;
    uint64_t off;
    uint32_t len;
    uint32_t snap;
    uint32_t ping_status;
    uint32_t plen;  // RESP_LIST entries actually written (len = the reference's list length)
    uint32_t nesc;  // of those, entries without a makeAlive origin (RESP_LIST_RX: they are in rx2e)
    uint32_t eoff;  // RESP_LIST_RX: offset of the message's escapes in rx2e
};

// One view cell: what a merge of a change for this (node, address) touches,
// on one line: the view value, the address's position in the node's
// dissemination log, and its suspicion-timer stamp.
struct VEnt {
    uint64_t vs;      // inc << 3 | status
    uint32_t dpos;    // absolute log position of the address's key, NONE: not in the log
    uint32_t tstamp;  // FIFO position + 1 of the live suspicion timer, 0: none
};
static_assert(sizeof(VEnt) == 16, "view cell is 16 bytes");

// An escape on the wire between shards: a change without a makeAlive origin,
// as is.  Its origin is known to the receiver already: fullSync origins are
// fixed, and a local suspect/faulty origin (an id in the sending shard's
// range of the origin table) was installed on every shard by the all-gather
// of each shard's newly allocated local origins (k_origin_pack /
// k_origin_install) before any message could name it.
struct Esc {
    Change c;
};
static_assert(sizeof(Esc) == 16, "wire escape is 16 bytes");

struct SimDev {
    uint32_t n;
    uint32_t ncoll;
    // shard: this object holds the rows (views, member orders, logs, ring
    // state, seen bitsets, timers) of nodes [lo, lo + nl); per-node scalar
    // arrays are indexed by global node id (remote entries hold exchanged
    // message metadata).  One shard: lo = 0, nl = n.
    uint32_t lo, nl;
    uint32_t rank, nranks;  // shard index / count (nodes per shard = nl)
    __host__ __device__ size_t row(uint32_t v) const { return (size_t)(v - lo) * n; }
    __host__ __device__ size_t srow(uint32_t v) const { return (size_t)(v - lo) * seen_words; }
    __host__ __device__ size_t trow(uint32_t v) const { return (size_t)(v - lo) * tcap; }
    __host__ __device__ size_t crow(uint32_t v) const { return (size_t)(v - lo) * ncoll; }
    __host__ __device__ bool local(uint32_t v) const { return v - lo < nl; }
    __host__ __device__ uint32_t owner(uint32_t v) const { return v / nl; }
    // views, member order
    VEnt* view;          // n*n
    uint32_t* order;     // n*n
    // dissemination: per-node log ring buffer (capacity n) + position index
    // (structure of arrays: an issue scans one 4-byte word per entry, values
    // and addresses only for the entries it writes out)
    uint32_t* dko;       // n*n  stamp << 24 | LOG_ALIVE | origin id (rp_sim.hip: implicit piggyback
                         //      counts; a makeAlive origin determines the entry's address and value)
    uint64_t* dvs;       // n*n  inc << 3 | status   (entries without a makeAlive origin)
    uint32_t* dad;       // n*n  address             (entries without a makeAlive origin)
    uint32_t* dhead;     // n
    uint32_t* dtail;     // n
    uint32_t* dlive;     // n  live keys in the log
    uint32_t compact_mul, compact_add;  // an issue compacts a log spanning > mul x live + add entries
    uint32_t prefix_min;  // wg_pack_prefix: the window must shrink by >= moved entries + prefix_min
    uint32_t ck_lane_min; // checksum lists of at least this many views: one lane per view (k_checksums_lanes)
    uint32_t* icount;    // n  issues so far (implicit piggyback counts, see rp_sim.hip)
    int32_t* max_pb;     // n
    // ring
    uint8_t* in_ring;    // n*n
    int32_t* ring_count; // n
    int32_t* coll_owner; // n*ncoll
    const int32_t* coll_of;  // n*REPLICAS
    const uint32_t* coll_off;  // n+1: server s's colliding replica groups are coll_ids[coll_off[s] .. coll_off[s+1])
    const uint32_t* coll_ids;
    const uint32_t* cmem_off;  // ncoll+1: group g's servers (ascending) are cmem[cmem_off[g] .. cmem_off[g+1])
    const uint32_t* cmem;
    uint32_t* rbatch;          // n  ring batches applied (collision-group erase marks)
    // per node scalars
    uint64_t* fp;
    // n  the node's checksum string length + its member count (every member
    // adds its text and a ';', so increments need no first-member case):
    // the string (lib/membership.js:70-93) is slen - 1 bytes, or empty at 0
    int64_t* slen;
    uint32_t* csum;
    uint32_t* csum_valid;
    int32_t* iter_index;
    int32_t* iter_round;
    int32_t* npingable;
    uint32_t* mcount;     // members in the node's view (its order row's first mcount entries)
    uint64_t* rng;
    uint8_t* dead;
    // origins
    Origin* origins;
    uint32_t* origin_count;  // makeAlive origins allocated so far (sequence numbers)
    uint32_t origin_cap;
    uint32_t* self_origin;  // n  origin of the node's local suspect/faulty updates at its incarnation
    // local (makeSuspect / makeFaulty) origins: ids [lorigin_base + rank * lorigin_per, + lorigin_per)
    // per shard, so that ids are unique cluster-wide; the shared counter
    // origin_count allocates makeAlive / fullSync origins (identically on every shard)
    uint32_t* lorigin_count;
    uint32_t* lorigin_sent;  // [1] lorigin_count at this shard's last origin all-gather
    uint32_t lorigin_base, lorigin_per;
    // makeAlive origins: a ring of alive_mask + 1 slots from alive_base; their
    // origin words carry the allocation sequence number (mod 2^23), and a
    // slot is reused once every live reference to its previous origin has
    // expired (log entries live at most maxPiggybackCount + 1 issues)
    uint32_t alive_base, alive_mask;
    uint64_t* self_inc;     // n  every node's own incarnation as known from churn (all shards)
    uint32_t* ck_list;      // n  views queued for k_checksums
    uint32_t* ck_count;     // [1]
    // seen-origin bitsets: bit (v, o mod W) set once node v has evaluated an
    // alive change of origin o, which from then on can never apply at v
    // (alive applies iff its incarnation exceeds the view's, and view
    // incarnations never decrease).  Valid for o in [oc_snap[round&1] - W,
    // oc_snap[round&1]) (ids created before this round); ranges are cleared
    // one round after their ids were allocated.
    uint32_t* seen;       // n * seen_words
    uint32_t seen_words;  // W / 32
    uint32_t* oc_snap;    // [2] origin_count at the start of even / odd rounds
    uint32_t* gseen;      // (n / gsz) x seen_words: makeAlive origins every live node of group g had evaluated
    uint32_t gsz_log;     // nodes per seen group: 1 << gsz_log consecutive ids (divides the shard size)
    uint32_t* gs_range;   // [2] ids [lo, hi) for which gseen is valid (empty: none)
    uint32_t* gsettled;   // (n >> fs_log) x n/32 (fault runs on G > 1 shards): settled bits every live node
                          // of group g had at the end of some earlier round (rp_sim.hip settled_bits); else null
    uint32_t fs_log;      // nodes per settled group: 1 << fs_log consecutive ids
    // address strings for checksums
    const uint32_t* addr_words;
    const uint8_t* addr_len;
    // round scratch
    uint32_t round;
    uint32_t part_start, part_end, part_split;  // partition injection
    Change* arena;
    unsigned long long* arena_cursor;
    unsigned long long arena_cap;
    uint64_t* msg_off;    // n   ping bodies (W0)
    // Messages crossing shards travel as one 4-byte word per entry: a
    // makeAlive origin word (the change is a function of the origin,
    // alive_change) or, bit 31 clear, the index of the entry in the message's
    // escape list of full 16-byte changes.
    uint32_t* rxw;        // ping bodies from senders on other shards (words)
    Esc* rxe;             //   and their escapes
    uint64_t* rx_off;     // n   offset of a remote sender's ping words in rxw
    uint64_t* rx_eoff;    // n   offset of its escapes in rxe
    uint32_t* rx2w;       // response lists from receivers on other shards (RESP_LIST_RX), words
    Esc* rx2e;            //   and escapes
    uint32_t* msg_nesc;   // n   ping entries written without a makeAlive origin
    Change* rxc;          // rxw (pings, W3, W4) and W5's rx2w lists decoded (same offsets); responses merge from rx2w
    uint32_t* msg_len;    // n   reference list length
    uint32_t* msg_plen;   // n   entries written (no-ops at the receiver left out)
    int32_t* target;      // n
    uint64_t* sv_word;    // n   the ping's same-view decision (k_iterate / k_shuffle, read by k_phase1)
    uint64_t* snd_inc;    // n   sender incarnation at send time
    uint64_t* snd_fp;     // n
    uint32_t* snd_csum;   // n
    uint8_t* need_csum;   // n  sender checksum snapshot required this round
    uint32_t* min_cnt;    // n  smallest piggyback count left in the log after phase 1
    uint32_t* min_safe;   // n  ... among entries no receiver filter can skip
    uint64_t* min_l1;     // n  ... among the others: (count << 32 | source), smallest
    uint64_t* min_l2;     // n  ... and smallest with a different source
    uint32_t* dangerous;  // origins that a receiver filter could match exist (suspect/faulty by their source)
    // wave grouping (per destination, slot order)
    uint32_t* g_cnt;      // n
    uint32_t* g_fill;     // n
    uint32_t* g_base;     // n+1
    uint32_t* g_list;     // 3n
    // responses: [0,n) ping responses by sender, [n,4n) relay-ping responses,
    // [4n,7n) ping-req responses, by slot 3A+i
    Resp* resp;
    uint64_t* snaps;      // snap_cap * n
    uint32_t* snap_ord;   // snap_cap * n: the responder's member order at the snapshot ...
    uint32_t* snap_m;     // snap_cap: ... and its member count (a fullSync lists exactly those)
    uint32_t* snap_count;
    uint32_t snap_cap;
    uint32_t* pend_slot;  // snap_cap
    uint32_t* pend_csum;  // snap_cap
    uint8_t* pend_done;   // snap_cap
    // ping-req state per initiator A and per slot 3A+i
    uint32_t* pr_n;
    uint32_t* pr_errors;
    uint32_t* pr_bad;
    uint32_t* pr_done;
    uint64_t* pr_inc;
    uint64_t* pr_fp;
    uint32_t* pr_csum;
    uint8_t* pr_ckv;      // pr_csum computed (else a relay must not need it: SIMERR_PREDICATE)
    uint32_t* fdecl_bits; // n bits: members some node of this shard declared faulty (k_timers), ever
    uint32_t* fdecl_count; // 1: how many bits of fdecl_bits are set (k_pr_need's ring-shrink bound)
    int32_t* w3_dest;
    int32_t* w4_dest;
    int32_t* w5_dest;
    int32_t* w6_dest;
    uint8_t* w4_err;
    uint64_t* pq_off;     // ping-req bodies: arena offset, or RX_MSG | offset in rxc (from another shard)
    uint32_t* pq_len;
    uint32_t* pq_nesc;    // entries without a makeAlive origin (sharded runs: wire escapes)
    uint64_t* rl_off;     // relay pings: arena offset, or RX_MSG | offset in rxc
    uint32_t* rl_len;
    uint32_t* rl_nesc;
    uint64_t* rl_inc;
    uint64_t* rl_fp;
    uint32_t* rl_csum;
    // suspicion timers: per-node FIFO of {address, creation round}; stamp per
    // (node, address) = FIFO position + 1 of the live timer, 0 = none
    uint2* tfifo;         // n*tcap
    uint32_t* thead;
    uint32_t* ttail;
    uint32_t tcap;
    int32_t* churn_ids;   // rounds_cap * churn_k
    unsigned long long* stats;  // per-round counters (see STAT_*)
    unsigned long long* bstats; // STAT_NSTATS x bstride per-block partial counters
    uint32_t bstride;           // rows = largest grid of a counting kernel (n)
    uint32_t* err;
    uint32_t* conv;       // converged flag for the last round
};

enum {
    STAT_EVALUATED = 0, STAT_APPLIED, STAT_FULLSYNC, STAT_MESSAGES, STAT_WAVES, STAT_PINGS,
    // per-kernel unit counts for the roofline (not part of the reference's stats)
    STAT_EVAL_P2, STAT_APPLIED_P2, STAT_EVAL_P3, STAT_APPLIED_P3, STAT_SCANNED_P1, STAT_EMITTED_P1,
    STAT_SCANNED_P2, STAT_EMITTED_P2, STAT_WRITTEN_P1, STAT_WRITTEN_P2,
    // changes whose view cell a merge actually read (the rest of `evaluated`
    // never reached it: left out by the sender or dropped by the seen filter)
    STAT_TOUCHED, STAT_TOUCHED_P2,
    // views whose checksum k_checksums computed (farmhash over the rendered row)
    STAT_CK_VIEWS,
    // dissemination-log compactions: issue-time (span > compact_mul x live +
    // compact_add) and apply-time (the batch would overrun the n-slot ring)
    STAT_COMPACT_ISSUE, STAT_COMPACT_APPLY,
    STAT_PREFIX_PACKS,  // issues that moved the window's live prefix forward (wg_pack_prefix)
    STAT_SAME_VIEW,     // issues to a destination with an identical view (wg_issue: its own entry only)
    // diagnostics (RP_DIAG builds only): shader-clock cycles by code section
    STAT_DIAG0, STAT_DIAG1, STAT_DIAG2, STAT_DIAG3, STAT_DIAG4, STAT_DIAG5,
    STAT_NSTATS
};

}  // namespace rp
