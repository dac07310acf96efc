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
    SIMERR_SUSPICION = 1u << 1,      // suspect applied / ping failure (needs failure support)
    SIMERR_ORIGIN_FULL = 1u << 2,
    SIMERR_ARENA_FULL = 1u << 3,
    SIMERR_SNAP_FULL = 1u << 4,
    SIMERR_RINGOPS = 1u << 5,
    SIMERR_PING_FAILED = 1u << 6,
    SIMERR_PREDICATE = 1u << 7,      // internal: a response the predicate proved non-empty was empty
};

enum : int32_t { RESP_NONE = 0, RESP_LIST = 1, RESP_EMPTY = 2, RESP_FS_PENDING = 3, RESP_FS = 4 };

struct SimDev {
    uint32_t n;
    uint32_t ncoll;
    // views, member order
    uint64_t* view;      // n*n
    uint32_t* order;     // n*n
    // dissemination: per-node log ring buffer (capacity n) + position index
    Change* dlog;        // n*n, addr field = addr | cnt << 24
    uint32_t* dpos;      // n*n
    uint32_t* dhead;     // n
    uint32_t* dtail;     // n
    uint32_t* dlive;     // n  live keys in the log
    int32_t* max_pb;     // n
    // ring
    uint8_t* in_ring;    // n*n
    int32_t* ring_count; // n
    int32_t* coll_owner; // n*ncoll
    const int32_t* coll_of;  // n*REPLICAS
    // per node scalars
    uint64_t* fp;
    uint32_t* csum;
    uint32_t* csum_valid;
    int32_t* iter_index;
    int32_t* iter_round;
    int32_t* npingable;
    uint64_t* rng;
    uint8_t* dead;
    // origins
    Origin* origins;
    uint32_t* origin_count;
    uint32_t origin_cap;
    // address strings for checksums
    const uint32_t* addr_words;
    const uint8_t* addr_len;
    // round scratch
    Change* arena;
    unsigned long long* arena_cursor;
    unsigned long long arena_cap;
    uint64_t* msg_off;    // n
    uint32_t* msg_len;    // n
    int32_t* target;      // n
    uint64_t* snd_inc;    // n   sender incarnation at send time
    uint64_t* snd_fp;     // n
    uint32_t* snd_csum;   // n
    uint8_t* need_csum;   // n  sender checksum snapshot required this round
    uint32_t* min_cnt;    // n  smallest piggyback count left in the log after phase 1
    uint32_t* dangerous;  // origins that a receiver filter could match exist (suspect/faulty/leave by their source)
    uint32_t* in_count;   // n
    uint32_t* in_fill;    // n
    uint32_t* in_base;    // n+1
    uint32_t* inbox;      // n
    uint64_t* resp_off;   // n (indexed by sender)
    uint32_t* resp_len;   // n
    int32_t* resp_kind;   // n
    int32_t* resp_from;   // n
    uint32_t* resp_snap;  // n
    uint64_t* snaps;      // snap_cap * n
    uint32_t* snap_count;
    uint32_t snap_cap;
    uint32_t* pend_sender;  // snap_cap
    int32_t* churn_ids;   // rounds_cap * churn_k
    unsigned long long* stats;  // per-round counters (see STAT_*)
    uint32_t* err;
    uint32_t* conv;       // converged flag for the last round
};

enum {
    STAT_EVALUATED = 0, STAT_APPLIED, STAT_FULLSYNC, STAT_MESSAGES, STAT_WAVES, STAT_PINGS,
    // per-kernel unit counts for the roofline (not part of the reference's stats)
    STAT_EVAL_P2, STAT_APPLIED_P2, STAT_EVAL_P3, STAT_APPLIED_P3, STAT_SCANNED_P1, STAT_EMITTED_P1,
    STAT_SCANNED_P2, STAT_EMITTED_P2,
    STAT_NSTATS
};

}  // namespace rp
