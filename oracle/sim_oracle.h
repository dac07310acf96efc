/* TEST INFRASTRUCTURE ONLY — CPU restatement (oracle) of ringpop's
 * membership-convergence path and of the build's simulation semantics.
 * See sim_oracle.c for the reference citations.  Loaded only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg. */
#ifndef RINGPOP_ORACLE_SIM_H
#define RINGPOP_ORACLE_SIM_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_sim orc_sim;

typedef struct {
    int64_t evaluated;   /* changes passed to Membership.update() */
    int64_t applied;     /* changes it applied */
    int64_t full_syncs;  /* Dissemination.fullSync() calls */
    int64_t messages;    /* requests + responses queued */
    int64_t waves;
    int64_t converged;   /* all live checksums equal after the round */
} orc_stats;

orc_sim *orc_sim_new(int n, uint64_t seed, int churn_k, int eager_checksums);
orc_sim *orc_sim_new2(int n, uint64_t seed, int churn_k, int eager_checksums, int replica_hash_shift);
/* arbitrary clusters: addresses in sort order (NULL: the sim scheme) and n x n
 * bootstrap views (status 1..4, incarnation; NULL: all alive at INC0 + id) */
orc_sim *orc_sim_new3(int n, uint64_t seed, int churn_k, int eager_checksums, int replica_hash_shift,
                      const uint8_t *addr_bytes, const uint64_t *addr_off, const uint8_t *vstatus,
                      const uint64_t *vinc);
void orc_sim_free(orc_sim *s);
/* schedule a fail-stop of `node` at the start of round `round` */
int orc_sim_fail(orc_sim *s, int node, int round);
/* requests between ids on different sides of `split` fail during rounds
 * [start, end) */
int orc_sim_partition(orc_sim *s, int start, int end, int split);
/* false-suspicion storm in rounds [start, end): ceil(live * ppm / 10^6)
 * makeSuspects per round after churn */
int orc_sim_storm(orc_sim *s, int start, int end, int ppm);
/* join schedule (before the first round): joiners[i] joins at rounds[i]
 * through seeds[i * seeds_per ..] (-1 = none) */
int orc_sim_join(orc_sim *s, const int32_t *joiners, const int32_t *rounds, const int32_t *seeds, int count,
                 int seeds_per);
/* run the next round; churn is applied when churn_active != 0 */
int orc_sim_round(orc_sim *s, int churn_active, orc_stats *st, int32_t *churned_out, int *nchurned);
int orc_sim_rounds_done(const orc_sim *s);

uint32_t orc_sim_checksum(orc_sim *s, int v);
int orc_sim_is_dead(const orc_sim *s, int v);
void orc_sim_dump_view(orc_sim *s, int v, uint8_t *status, uint64_t *inc);
int orc_sim_dump_members(orc_sim *s, int v, int32_t *out);
/* rows of 6 int64: addr, piggybackCount(-1 undef), source(-1), sourceInc(0 undef), status, inc */
int orc_sim_dump_changes(orc_sim *s, int v, int64_t *out);
/* max_pb, ring_servers, ring_checksum, iter_index, iter_round, dead, rng_state, n_timers */
void orc_sim_node_info(orc_sim *s, int v, int64_t *info);
/* addresses with live suspicion timers (sorted); returns count */
int orc_sim_dump_timers(orc_sim *s, int v, int32_t *out);
/* ring owner for a key hash in view v (-1 on empty ring) */
int orc_sim_ring_lookup(orc_sim *s, int v, uint32_t h);
/* address string of node i (sim address scheme) */
int orc_sim_address(const orc_sim *s, int i, char *buf, int cap);

/* ---- wire bridge: node-level ping path between rounds -------------------
 * rows of 5 int64: address, status, incarnation, source (-1 undefined),
 * sourceIncarnationNumber (0 undefined) */
int orc_sim_ping_body(orc_sim *s, int v, int64_t *out, int cap, uint32_t *checksum, uint64_t *incarnation);
int orc_sim_handle_ping(orc_sim *s, int v, int source, uint64_t source_inc, uint32_t checksum, const int64_t *rows,
                        int n, int64_t *out, int cap, int *applied, int *full_sync);
int orc_sim_update(orc_sim *s, int v, const int64_t *rows, int n);

/* ---- standalone single-instance HashRing (lib/ring.js) ------------------ */
typedef struct orc_ring orc_ring;
orc_ring *orc_ring_new(int replica_points);
void orc_ring_free(orc_ring *r);
/* names are passed as one byte buffer + n+1 offsets; hashes may be given
 * (custom hashFunc seam, lib/ring.js:29) as replica_hashes[n*replica_points],
 * or NULL to use farmhash32(name + i). returns 1 if the ring changed */
int orc_ring_add_remove(orc_ring *r, const uint8_t *add_bytes, const uint64_t *add_off, int nadd,
                        const uint32_t *add_hashes, const uint8_t *rm_bytes, const uint64_t *rm_off,
                        int nrm, const uint32_t *rm_hashes);
int orc_ring_server_count(const orc_ring *r);
uint32_t orc_ring_checksum(orc_ring *r);
/* owner server index (into the order servers were first named) for each key
 * hash; -1 for an empty ring */
void orc_ring_lookup_hashes(orc_ring *r, const uint32_t *h, size_t n, int32_t *owner);
/* number of distinct points and their (hash, owner) in ascending hash order */
size_t orc_ring_points(orc_ring *r, uint32_t *hashes, int32_t *owners);
int orc_ring_server_name(const orc_ring *r, int idx, char *buf, int cap);
/* lookupN (lib/ring.js:150-182) for one key hash; returns count */
int orc_ring_lookup_n(orc_ring *r, uint32_t h, int n, int32_t *out);

/* ---- single view update rules (lib/membership.js:208-313) --------------- */
/* Evaluates a batch against a view of `nmem` addresses (status 0 = absent);
 * self = local address index. Mutates status/inc, writes applied flags and the
 * (possibly rewritten) change status/inc. returns the number applied. */
int orc_view_update(int self, uint64_t now, uint8_t *status, uint64_t *inc,
                    int nchanges, const int32_t *addr, uint8_t *cstatus, uint64_t *cinc,
                    uint8_t *applied);

/* checksum string / checksum of a view given address strings in sorted order */
size_t orc_checksum_string(const uint8_t *addr_bytes, const uint64_t *addr_off, int naddr,
                           const uint8_t *status, const uint64_t *inc, uint8_t *out, size_t cap);
uint32_t orc_view_checksum(const uint8_t *addr_bytes, const uint64_t *addr_off, int naddr,
                           const uint8_t *status, const uint64_t *inc);
/* Dissemination.adjustMaxPiggybackCount formula (lib/dissemination.js:38-55) */
int orc_max_piggyback(int server_count, int factor);

#ifdef __cplusplus
}
#endif
#endif
