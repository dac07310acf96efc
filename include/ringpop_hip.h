/*
 * ringpop_hip.h — C ABI of the MI355X-native ringpop membership-convergence
 * path (libringpop_hip.so, gfx950).
 *
 * Drop-in boundary: these entry points are what the reference's JavaScript
 * would bind through a thin N-API addon.  Each block
 * names the reference interface it replaces (paths relative to the
 * reference repository).  Plain pointers and sizes only; every function
 * returns RP_OK (0) or a negative RP_ERR_* code, with a message available from
 * rp_last_error().  Host buffers are copied; *_device variants take device
 * pointers and a hipStream_t (passed as void *).
 */
#ifndef RINGPOP_HIP_H
#define RINGPOP_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RP_OK 0
#define RP_ERR_INVALID (-1)     /* bad argument */
#define RP_ERR_HIP (-2)         /* HIP runtime error (no GPU, launch failure, ...) */
#define RP_ERR_NOMEM (-3)       /* device allocation failed */
#define RP_ERR_UNSUPPORTED (-4) /* configuration outside what the device path models */
#define RP_ERR_CAPACITY (-5)    /* a device arena overflowed; recreate with more capacity */
#define RP_ERR_STATE (-6)       /* a kernel raised an error flag */

const char *rp_last_error(void);
int rp_abi_version(void);
/* select the HIP device used by objects created afterwards (default 0) */
int rp_set_device(int device);

/* ---- device utilities --------------------------------------------------------
 * Buffers, streams and events of the HIP runtime this library links, for
 * callers of the *_device entry points that have no runtime handle of their
 * own (bench.py, tests).  memcpy kind: 1 host->device, 2 device->host,
 * 3 device->device. */
int rp_device_malloc(size_t bytes, void **out);
int rp_device_free(void *ptr);
int rp_device_memcpy(void *dst, const void *src, size_t bytes, int kind);
int rp_device_synchronize(void);
/* free / total bytes of the current device (hipMemGetInfo): the footprint report of bench.py */
int rp_device_memory(size_t *free_bytes, size_t *total_bytes);
int rp_stream_create(void **out);
int rp_stream_destroy(void *stream);
int rp_stream_synchronize(void *stream);
int rp_event_create(void **out);
int rp_event_record(void *event, void *stream);
int rp_event_elapsed_ms(void *start, void *end, float *ms);
int rp_event_destroy(void *event);
/* this box's memory ceilings for the round kernels' access kinds (bench.py's
 * box_ceiling; measurement infrastructure, no reference counterpart): over a
 * fresh device allocation of `bytes` (>= 1 GiB, past the Infinity Cache),
 * out[0..4] = accesses per second of random 16-byte reads, random 16-byte
 * read + 8-byte write-backs, random 4-byte reads, 16-byte-per-lane streaming
 * reads and 4-byte-per-lane streaming reads (nout >= 5) */
int rp_calibrate(size_t bytes, double *out, int nout);
/* the current device's PCI bus id ("0000:xx:yy.z"), to find its sysfs clocks */
int rp_device_pci_bus_id(char *buf, int len);

/* ---- farmhash.hash32 -------------------------------------------------------
 * Replaces npm `farmhash` ^0.2.0 `hash32(string)` (package.json:30), called at
 * lib/membership.js:57 and as HashRing's default hashFunc at lib/ring.js:29.
 * Strings are given as one byte buffer plus n+1 offsets (string i is
 * bytes[offsets[i] .. offsets[i+1])). Computed on the device. */
int rp_hash32(const uint8_t *bytes, size_t len, uint32_t *out);
int rp_hash32_batch(const uint8_t *bytes, const uint64_t *offsets, size_t n, uint32_t *out);
int rp_hash32_batch_device(const uint8_t *d_bytes, const uint64_t *d_offsets, size_t n, uint32_t *d_out,
                           void *stream);

/* ---- HashRing ----------------------------------------------------------------
 * Replaces lib/ring.js:25-184 (HashRing) and its lib/rbtree.js index.
 * Servers are identified by the index of their first appearance
 * (rp_ring_server_name maps back).  add/remove follow addRemoveServers
 * (lib/ring.js:60-94): adds in order (insert-if-absent per replica point),
 * then removes (erase by hash).  add_hashes / rm_hashes, when non-NULL, give
 * the replica hashes [n * replica_points] instead of farmhash32(name + i):
 * the reference's `hashFunc` option (lib/ring.js:29). */
typedef struct rp_ring rp_ring;
int rp_ring_create(int replica_points, rp_ring **out);
int rp_ring_destroy(rp_ring *ring);
int rp_ring_add_remove(rp_ring *ring, const uint8_t *add_bytes, const uint64_t *add_offsets, size_t nadd,
                       const uint32_t *add_hashes, const uint8_t *rm_bytes, const uint64_t *rm_offsets,
                       size_t nrm, const uint32_t *rm_hashes, int *changed);
/* device time of the last rp_ring_add_remove that changed the ring: replica
 * hashing, the stable radix sort of the points, first-inserter dedupe and
 * compaction, the lookup directories (HIP events around the device work;
 * names cross PCIe inside it) */
int rp_ring_build_ms(rp_ring *ring, double *device_ms);
/* host microseconds of the last rp_ring_add_remove by phase and of the last
 * computed rp_ring_checksum (measurement): us[i] for
 * i < n, indexed by RP_RING_PROF_*; phases a bulk call skips are 0 */
#define RP_RING_PROF_SELECT 0   /* name interning, present / duplicate checks */
#define RP_RING_PROF_HASH 1     /* replica hashes (incremental path: on the host) */
#define RP_RING_PROF_MERGE 2    /* host mirror delta, staging copy, k_ring_merge launch */
#define RP_RING_PROF_INDEX 3    /* lookup-index rebuild launches and events */
#define RP_RING_PROF_TOTAL 4    /* the whole call */
#define RP_RING_PROF_CK_BUILD 5 /* checksum: the sorted, ';'-joined server string */
#define RP_RING_PROF_CK_HASH 6  /* checksum: copy, hash kernel, synchronisation */
#define RP_RING_PROF_N 7
int rp_ring_profile(rp_ring *ring, double *us, int n);
int rp_ring_server_count(rp_ring *ring, int *out);                                  /* :107-109 */
int rp_ring_has_server(rp_ring *ring, const uint8_t *name, size_t len, int *out);   /* :111-113 */
int rp_ring_checksum(rp_ring *ring, uint32_t *out);                                 /* :96-105 */
int rp_ring_server_name(rp_ring *ring, int index, char *buf, size_t cap, size_t *len);
/* lookup (lib/ring.js:138-147): owner server index per key, -1 on an empty ring */
int rp_ring_lookup_batch(rp_ring *ring, const uint8_t *bytes, const uint64_t *offsets, size_t n,
                         int32_t *owners);
int rp_ring_lookup_batch_device(rp_ring *ring, const uint8_t *d_bytes, const uint64_t *d_offsets, size_t n,
                                int32_t *d_owners, void *stream);
/* lookup for precomputed key hashes (custom hashFunc) */
int rp_ring_lookup_hashes(rp_ring *ring, const uint32_t *key_hashes, size_t n, int32_t *owners);
/* lookupN (lib/ring.js:150-182): up to n distinct owners per key hash; out is
 * [nkeys * n], unused slots -1; counts[k] = owners found */
int rp_ring_lookup_n_hashes(rp_ring *ring, const uint32_t *key_hashes, size_t nkeys, int n, int32_t *out,
                            int32_t *counts);
/* handleOrProxyAll's grouping (index.js:636-645: _.groupBy(keys, this.lookup),
 * then Object.keys): groups in first-appearance order of their owner, keys of
 * a group in input order.  dests[g] = owner server index (-1: empty ring, the
 * reference's "null" group); the keys of group g are
 * key_index[group_off[g] .. group_off[g + 1]).  Arrays: dests and key_index
 * [n], group_off [n + 1]; *ngroups receives the group count (n < 2^31 - 1). */
int rp_ring_group_keys(rp_ring *ring, const uint8_t *bytes, const uint64_t *offsets, size_t n, int32_t *dests,
                       uint32_t *group_off, uint32_t *key_index, size_t *ngroups);
/* the same for precomputed key hashes (custom hashFunc) */
int rp_ring_group_hashes(rp_ring *ring, const uint32_t *key_hashes, size_t n, int32_t *dests, uint32_t *group_off,
                         uint32_t *key_index, size_t *ngroups);
/* device arrays: owners from rp_ring_lookup_batch_device; synchronises `stream` */
int rp_ring_group_device(rp_ring *ring, const int32_t *d_owners, size_t n, int32_t *d_dests, uint32_t *d_group_off,
                         uint32_t *d_key_index, size_t *ngroups, void *stream);
/* sorted distinct points (rbtree in-order walk) */
int rp_ring_points(rp_ring *ring, uint32_t *hashes, int32_t *owners, size_t cap, size_t *count);
/* device-generated synthetic keys: decimal strings of splitmix64(seed + i*golden)
 * (benchmark config 3); returns device pointers owned by the ring object */
int rp_ring_make_keys_device(rp_ring *ring, uint64_t seed, size_t n, const uint8_t **d_bytes,
                             const uint64_t **d_offsets, uint64_t *total_bytes);

/* ---- Simulation of N ringpop instances ---------------------------------------
 * Each simulated node runs the reference's Membership (lib/membership.js),
 * Dissemination (lib/dissemination.js), HashRing and MembershipIterator
 * state; a round is one protocol period for every live node
 * (index.js:458-515) under the synchronous semantics of DESIGN.md §3. */
typedef struct rp_sim rp_sim;
typedef struct {
    uint32_t n;               /* simulated nodes (<= 65536) */
    uint32_t churn_k;         /* alive re-assertions per churning round */
    uint64_t seed;
    uint64_t arena_entries;   /* message arena capacity (16-byte changes); 0 = auto */
    uint32_t snapshot_slots;  /* full-sync snapshots per round; 0 = auto */
    uint32_t origin_slots;    /* update-origin table capacity (0 = auto = 2^23 - 1, the maximum): n + 1 fixed slots, a ring of
                                 makeAlive origins (a power of two) and per-shard rings of local
                                 suspect/faulty origins in the top quarter; slots are reused once
                                 every reference to their previous origin has expired */
    uint32_t seen_window;     /* ids per node in the seen-origin bitset (power of two in [32, 32768]); 0 = auto */
    uint32_t replica_hash_shift; /* testing: clear this many low bits of every replica hash (forces
                                    rbtree collisions; 0 = the reference's hashes, < 32) */
    uint32_t compact_mul;     /* an issue squeezes the tombstones out of a dissemination log whose span */
    uint32_t compact_add;     /* exceeds compact_mul x its live keys + compact_add (0, 0 = auto: 4, 8192);
                                 a layout choice with no observable effect (tests force it with tiny values) */
    uint32_t prefix_min;      /* after an issue, the live entries of the window's first groups move forward to the
                                 end of that prefix when that shrinks the window by >= (entries moved) + prefix_min
                                 (0 = auto: 512; never below 1); a layout choice with no observable effect */
    uint32_t ck_lane_min;     /* a list of at least this many distinct views to checksum is hashed one view per
                                 lane (k_checksums_lanes), shorter ones one view per wave (0 = auto: 12288;
                                 1 = always per lane, 0xFFFFFFFF = never); same checksums either way */
} rp_sim_config;

typedef struct {
    uint64_t evaluated;   /* changes passed to Membership.update() */
    uint64_t applied;     /* changes applied */
    uint64_t full_syncs;  /* Dissemination.fullSync() responses */
    uint64_t messages;    /* requests + responses */
    uint64_t waves;
    uint64_t pings;
    uint64_t converged;   /* all live views identical after the round */
} rp_round_stats;

int rp_sim_create(const rp_sim_config *cfg, rp_sim **out);
int rp_sim_destroy(rp_sim *sim);

/* ---- Sharded simulations -------------------------------------
 * The N nodes are split into G shards of N/G consecutive ids (G divides N,
 * G <= 64).  Each round the shards exchange ping metadata, checksum
 * snapshots, ping bodies and responses, and with fail-stops or partitions
 * the ping-req waves (ping-req bodies, relay pings, their responses; the
 * suspect/faulty update origins travel with them).  Results equal the
 * single-shard run's bit for bit.
 *   rp_sim_create_shards: all G shards in this process on the current device
 *     (exchanges are device copies); results equal rp_sim_create's.
 *   rp_sim_create_rank: this process holds shard `rank` of `nranks`, one
 *     process per GPU; exchanges are RCCL all-gathers and send/recv groups
 *     over the communicator named by `unique_id` (from rp_comm_unique_id on
 *     one rank, 128 bytes, distributed by the caller).  Per-node reads
 *     (read_view, read_changes, ...) only reach this process's nodes;
 *     rp_sim_read_checksums leaves other nodes' entries 0. */
int rp_sim_create_shards(const rp_sim_config *cfg, int nshards, rp_sim **out);
int rp_comm_unique_id(uint8_t *unique_id, size_t cap);
int rp_sim_create_rank(const rp_sim_config *cfg, int nranks, int rank, const uint8_t *unique_id, rp_sim **out);
/* The RCCL transport the rank path uses (in-place all-gather, u32 sum
 * all-reduce, a grouped send/recv with every rank, broadcast), run on small
 * buffers of `words` u32 with predictable contents over the communicator
 * named by `unique_id`; *failures = words that differ from the expectation.
 * Every rank calls it; nranks = 1 exercises every call on one GPU (sends to
 * itself).  Replaces nothing in the reference: a check of the transport that
 * carries lib/swim/ping-sender.js:81-99's traffic between GPUs. */
int rp_comm_selftest(int nranks, int rank, const uint8_t *unique_id, uint32_t words, uint32_t *failures);
/* The rank path without RCCL, for one GPU: the ranks of an nranks-rank
 * cluster as host threads of this process on the current device (each rank
 * its own rp_sim, its calls made from its own thread, every rank making the
 * same calls in the same order).  The collectives are device copies after a
 * rendezvous of the rank threads; everything else is rp_sim_create_rank's
 * code.  A rank that fails or stalls for 120 s fails the others'
 * collectives.  Destroy the loop after its ranks. */
typedef struct rp_loop rp_loop;
int rp_loop_create(int nranks, rp_loop **out);
int rp_loop_destroy(rp_loop *loop);
int rp_sim_create_rank_loop(const rp_sim_config *cfg, rp_loop *loop, int rank, rp_sim **out);
/* nodes [lo, hi) held by this process */
int rp_sim_shard_range(rp_sim *sim, uint32_t *lo, uint32_t *hi);
/* rp_sim_counters restricted to the work of this process's shards (the
 * per-kernel unit counts behind its own kernel times); converged rounds 0 */
int rp_sim_local_counters(rp_sim *sim, uint64_t *out, int cap, int *n);
/* since rp_sim_enable_timing: device time of the exchange steps (planning and
 * packing kernels, copies / RCCL collectives, host waits for their counts;
 * ms, timing enabled only), bytes this process sent, rounds exchanged */
int rp_sim_exchange_stats(rp_sim *sim, double *ms, uint64_t *bytes_sent, uint64_t *rounds);
/* since rp_sim_enable_timing: bytes each of this process's shards sent to
 * other shards (all-gathers, all-to-alls, all-reduces; in-process shards
 * count the device copies a shard's data is the source of), out[i] for its
 * i-th local shard; *count = the local shards */
int rp_sim_exchange_shard_bytes(rp_sim *sim, uint64_t *out, int cap, int *count);
/* Arbitrary clusters; both before the first round, and in a
 * multi-process cluster every rank makes the same calls.
 * rp_sim_load_addresses: the cluster's n address strings (bytes[off[i] ..
 * off[i+1]), 1..32 printable ASCII bytes, distinct, in ascending sort order:
 * node i is the i-th address, so a view indexed by id is in the order
 * generateChecksumString sorts members, lib/membership.js:62-93).  Replaces
 * the 10.x.x.x:300x scheme; every view is re-bootstrapped as rp_sim_create does,
 * so it must come FIRST: after rp_sim_set_views or rp_sim_join it fails with
 * RP_ERR_STATE.  Call order: create, load_addresses, set_views / join, rounds.
 * rp_sim_set_views: re-bootstrap nodes [node_lo, node_lo + count) from
 * views -- status[r * n + a] (0 absent, 1 alive, 2 suspect, 3 faulty, 4 leave) and
 * incarnation[r * n + a] of member a in node node_lo + r's view, its own
 * entry alive -- as the reference's bootstrap does with that join result:
 * makeAlive(self, inc), set() (lib/membership.js:162-206) whose listener adds
 * the alive members to the ring and starts a suspicion timer per suspect
 * (lib/membership-set-listener.js:24-48; due at round 0), shuffle(),
 * clearChanges().  Replaces the full-alive views of rp_sim_create (index.js:
 * 233-267 with a full-membership join result). */
int rp_sim_load_addresses(rp_sim *sim, const uint8_t *bytes, const uint64_t *offsets, uint32_t n);
/* Join path, before the first round: node joiners[i]
 * stays outside the cluster (no view, not pinging, absent from every view)
 * until the start of round rounds[i] (after the due suspicion timers, before
 * churn), when it joins through seeds[i * seeds_per ..] (-1 = none; each
 * seed a member from the start or joined in an earlier round) as the
 * reference bootstraps: makeAlive(self, now) (index.js:235), each seed's
 * handleJoin -- makeAlive(joiner) then its checksum and fullSync()
 * (server/join-handler.js:76-98) --, mergeJoinResponses (lib/swim/
 * join-response-merge.js:40-56), update() + set() (lib/membership.js:162-206)
 * and shuffle().  The other nodes are re-bootstrapped with views of each
 * other (everyone alive at 1434401518824 + id); the merges then splice
 * members they learn of at getJoinPosition (lib/membership.js:99-101,
 * 285-298).  Once per simulation. */
int rp_sim_join(rp_sim *sim, const uint32_t *joiners, const uint32_t *rounds, const int32_t *seeds, uint32_t count,
                uint32_t seeds_per);
int rp_sim_set_views(rp_sim *sim, uint32_t node_lo, uint32_t count, const int32_t *status,
                     const int64_t *incarnation);
/* fail-stop `node` at the start of `round` (it stops pinging and answering;
 * requests to it come back as transport errors one wave later) */
int rp_sim_fail(rp_sim *sim, uint32_t node, uint32_t round);
/* requests between ids on different sides of `split` fail during rounds
 * [start, end) (partition injection; split = 0 disables) */
int rp_sim_partition(rp_sim *sim, uint32_t start, uint32_t end, uint32_t split);
/* false-suspicion storm (config 5): in rounds [start, end),
 * after churn, ceil(live * ppm / 10^6) seeded live victims are each suspected
 * by a seeded live accuser through Membership.makeSuspect(victim, the
 * accuser's incarnation of it) (lib/membership.js:154-156); victims refute
 * through the local override (:244-254).  ppm = 0 disables. */
int rp_sim_storm(rp_sim *sim, uint32_t start, uint32_t end, uint32_t ppm);
/* run one round and return its statistics (synchronous) */
int rp_sim_round(rp_sim *sim, int churn_active, rp_round_stats *stats);
/* enqueue k rounds on the simulation's stream (asynchronous); totals accumulate */
int rp_sim_run(rp_sim *sim, int k_rounds, int churn_active);
int rp_sim_sync(rp_sim *sim);
int rp_sim_totals(rp_sim *sim, rp_round_stats *totals);
int rp_sim_rounds(rp_sim *sim, uint32_t *rounds);
/* cumulative device counters: evaluated, applied, full_syncs, messages, waves,
 * pings, then per kernel: ping-merge evaluated/applied, response-merge
 * evaluated/applied, sender-issue scanned/emitted, receiver-issue
 * scanned/emitted and written, touched (all merges / ping merge), views
 * checksummed by k_checksums, six diagnostic counters, then converged
 * rounds (ringpop_amd/sim.py Sim.COUNTERS); returns the count in *n */
int rp_sim_counters(rp_sim *sim, uint64_t *out, int cap, int *n);
/* simulated node count */
int rp_sim_size(rp_sim *sim, uint32_t *n);
/* Membership.checksum of every node (farmhash32 of the checksum string);
 * out holds cap >= n entries */
int rp_sim_read_checksums(rp_sim *sim, uint32_t *out, size_t cap);
/* status (0 absent,1 alive,2 suspect,3 faulty,4 leave) and incarnation per address */
/* ---- Wire-format bridge (node-level ping path, between rounds) -------------
 * The reference's ping wire surface for one simulated node, so that a host
 * codec can speak the JSON bodies of lib/swim/ping-sender.js:70-76 and
 * server/ping-handler.js:36-39 (ringpop_amd/wire.py, js/index.js).  A change
 * is 5 int64: address and source are member ids (rp_sim_address; source -1 =
 * undefined), status 1 alive 2 suspect 3 faulty 4 leave, source_incarnation 0
 * = undefined.  Each call runs on the node's shard with the next round's
 * clock; changes from the wire get update origins of their own (the receiver
 * filter compares origins by value), so round results stay the reference's.
 *   rp_sim_ping_body    PingSender.send (ping-sender.js:70-76): issueAsSender
 *                       (advances piggyback counts), membership.checksum,
 *                       getIncarnationNumber()
 *   rp_sim_handle_ping  handlePing (server/ping-handler.js:22-40):
 *                       Membership.update(changes), then issueAsReceiver(source,
 *                       source_incarnation, checksum); *full_sync = 1 when the
 *                       response is Dissemination.fullSync() (:102-117)
 *   rp_sim_update       PingSender.onPing's Membership.update (ping-sender.js:36-39)
 * Output buffers must hold cap >= n changes (a fullSync is n of them; the
 * call is refused before any state changes otherwise); *count is the list
 * length. */
typedef struct {
    int64_t address;
    int64_t status;
    int64_t incarnation;
    int64_t source;
    int64_t source_incarnation;
} rp_change;
int rp_sim_ping_body(rp_sim *sim, uint32_t node, rp_change *out, uint32_t cap, uint32_t *count, uint32_t *checksum,
                     uint64_t *incarnation);
int rp_sim_handle_ping(rp_sim *sim, uint32_t node, int64_t source, uint64_t source_incarnation, uint32_t checksum,
                       const rp_change *changes, uint32_t n, rp_change *out, uint32_t cap, uint32_t *count,
                       uint32_t *applied, int *full_sync);
int rp_sim_update(rp_sim *sim, uint32_t node, const rp_change *changes, uint32_t n, uint32_t *applied);

/* per node, 6 counts: members absent / alive / suspect / faulty / leave in its
 * view and its ring's server count (nodes of other processes: 0); out holds
 * cap >= 6 n entries */
int rp_sim_view_counts(rp_sim *sim, uint32_t *out, size_t cap);
/* status / inc hold cap >= n entries (either may be NULL) */
int rp_sim_read_view(rp_sim *sim, uint32_t node, uint8_t *status, uint64_t *inc, size_t cap);
/* Membership.members order; out holds cap >= n entries */
int rp_sim_read_members(rp_sim *sim, uint32_t node, uint32_t *out, size_t cap, uint32_t *count);
/* Dissemination.changes in key order: rows of 6 int64 {address, piggybackCount
 * (-1 undefined), source (-1), sourceIncarnationNumber (0 undefined), status,
 * incarnationNumber} */
int rp_sim_read_changes(rp_sim *sim, uint32_t node, int64_t *rows, uint32_t cap, uint32_t *count);
/* {maxPiggybackCount, ring server count, ring checksum, iterator index,
 *  iterator round, dead, rng state, pending suspicion timers} */
int rp_sim_node_info(rp_sim *sim, uint32_t node, int64_t *info8);
/* ring.lookup in one node's view, for precomputed key hashes */
int rp_sim_ring_lookup(rp_sim *sim, uint32_t node, const uint32_t *key_hashes, size_t n, int32_t *owners);
int rp_sim_address(rp_sim *sim, uint32_t node, char *buf, size_t cap);
/* per-kernel device time (HIP events on the simulation stream), ms, summed
 * since enable; names: churn, issue(phase1), merge_ping(phase2),
 * merge_resp(phase3), checksum, other */
int rp_sim_enable_timing(rp_sim *sim, int enable);
/* the same for some stages only: bit i of mask times stage i (the order of
 * rp_sim_kernel_times, then 6 = the exchange steps); every timed stage adds
 * two events per launch to the simulation stream, which the timed rounds pay
 * for (bench.py times only the ping merge inside its timed region) */
int rp_sim_enable_timing_stages(rp_sim *sim, uint32_t mask);
int rp_sim_kernel_times(rp_sim *sim, double *ms6, uint64_t *launches6);
/* device time (ms, summed since enable) of the work one shard runs on its
 * side stream beside the round kernels: the round's sender checksum chains
 * (beside the ping merge) and the fullSync decisions (beside the response
 * merge); the "checksum" category above counts only the checksum work left
 * on the simulation stream */
int rp_sim_side_ms(rp_sim *sim, double *ms);

/* ---- One ringpop instance: Membership + Dissemination ------------------------
 * Replaces lib/membership.js:31-354 (Membership) and lib/dissemination.js:
 * 27-184 (Dissemination) for one ringpop process; js/index.js and
 * ringpop_amd/node.py wrap it with the reference's classes, methods and
 * events.  Address strings are interned to dense ids in first-seen order
 * (rp_node_intern; the local address is id 0).  Math.random, read by
 * getJoinPosition (lib/membership.js:99-101), shuffle and sample, is the
 * instance's splitmix64 stream, settable for replay.
 * A change is 48 bytes; incarnations are integers < 2^53.  */
typedef struct {
    int64_t address;            /* address id; -1: undefined (update() only) */
    int64_t incarnation;        /* -1: undefined */
    int64_t source;             /* address id; -1: undefined */
    int64_t source_incarnation; /* -1: undefined */
    int32_t status;             /* 1 alive, 2 suspect, 3 faulty, 4 leave */
    int32_t piggyback;          /* piggybackCount in rp_dissemination_changes (-1: undefined) */
    int64_t reserved;
} rp_member_change;
typedef struct rp_node rp_node;
int rp_node_create(const uint8_t *self_address, size_t len, uint64_t rng_state, rp_node **out);
int rp_node_destroy(rp_node *node);
/* ids[i] = id of address i (interning unknown ones) */
int rp_node_intern(rp_node *node, const uint8_t *bytes, const uint64_t *offsets, size_t n, uint32_t *ids);
int rp_node_address(rp_node *node, uint32_t id, char *buf, size_t cap, size_t *len);
/* read (get) and/or replace (set) the Math.random state */
int rp_node_rng(rp_node *node, uint64_t *get, const uint64_t *set);
/* Membership.update(changes) once ringpop is ready (lib/membership.js:208-313):
 * rules (lib/membership-update-rules.js:25-59), unknown members taken
 * wholesale and spliced at getJoinPosition(), the local suspect/faulty
 * override rewritten in place to {alive, now} (_.extend, :246-251).
 * applied[i] = 1 for every change on the returned list; when any applied the
 * checksum is recomputed (:266-268) and returned. */
int rp_membership_update(rp_node *node, rp_member_change *changes, uint32_t n, uint64_t now, uint8_t *applied,
                         uint32_t *napplied, uint32_t *checksum);
/* Membership.set() (:162-206) over the flattened stashed changesets:
 * mergeMembershipChangesets (lib/membership-changeset-merge.js:22-51), then
 * each update pushed at the end of members; winners[k] = index into `stash`
 * of the k-th update (the set listener's list). */
int rp_membership_set(rp_node *node, const rp_member_change *stash, uint32_t n, uint32_t *winners,
                      uint32_t *nwinners, uint32_t *checksum);
int rp_membership_checksum(rp_node *node, uint32_t *checksum);                       /* computeChecksum :41-64 */
int rp_membership_checksum_string(rp_node *node, char *buf, size_t cap, size_t *len); /* :70-93 */
/* members in order: ids / status / incarnation (any may be NULL) */
int rp_membership_members(rp_node *node, uint32_t *ids, uint8_t *status, uint64_t *inc, size_t cap,
                          uint32_t *count);
int rp_membership_shuffle(rp_node *node);                                         /* :315-317 */
/* replace the member order with a permutation of it (ids, count = the member
 * count): getStats() sorts `members` in place with localeCompare
 * (lib/membership.js:122-129), which the JS host computes and writes back */
int rp_membership_set_order(rp_node *node, const uint32_t *ids, uint32_t count);
int rp_membership_random(rp_node *node, uint32_t k, double *out);                 /* k Math.random() draws */
/* set a member's status / incarnation directly (what tests do to Member objects) */
int rp_membership_force(rp_node *node, uint32_t id, int status, uint64_t incarnation);
/* Dissemination.recordChange for a batch, in order (:125-127) */
int rp_dissemination_record(rp_node *node, const rp_member_change *changes, uint32_t n);
/* issueAsSender (:78-84): the list; cap must cover every recorded change */
int rp_dissemination_issue(rp_node *node, int32_t max_piggyback, rp_member_change *out, size_t cap, uint32_t *count);
/* issueAsReceiver (:86-119) with its fullSync fallback (*full_sync = 1);
 * sender -1 / sender_incarnation -1 = undefined, has_checksum 0 = undefined */
int rp_dissemination_issue_as_receiver(rp_node *node, int64_t sender, int64_t sender_incarnation,
                                       uint32_t sender_checksum, int has_checksum, int32_t max_piggyback,
                                       rp_member_change *out, size_t cap, uint32_t *count, int *full_sync);
int rp_dissemination_full_sync(rp_node *node, rp_member_change *out, size_t cap, uint32_t *count); /* :61-76 */
int rp_dissemination_clear(rp_node *node);                                                        /* :57-59 */
/* Dissemination.changes in key order, with piggybackCount */
int rp_dissemination_changes(rp_node *node, rp_member_change *out, size_t cap, uint32_t *count);

#ifdef __cplusplus
}
#endif
#endif
