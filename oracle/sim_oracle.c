/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle.  Plain-C restatement of the
 * reference's membership-convergence path, driven by the build's
 * simulation semantics (mirrored by oracle/harness/sim.js
 * which runs the UNMODIFIED reference JS).  Never linked into the product
 * library; loaded only by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.
 *
 * Restated reference code (paths relative to /root/reference):
 *   Membership.update / applyUpdate .......... lib/membership.js:208-313
 *   update rules ............................. lib/membership-update-rules.js:25-59
 *   makeUpdate / makeAlive / ... ............. lib/membership.js:141-156,324-352
 *   set() + changeset merge + set listener ... lib/membership.js:162-206,
 *                                              lib/membership-changeset-merge.js:22-51,
 *                                              lib/membership-set-listener.js:24-48
 *   computeChecksum / generateChecksumString . lib/membership.js:41-93
 *   getJoinPosition / shuffle / random members lib/membership.js:99-120,315-317
 *   update listener .......................... lib/membership-update-listener.js:24-75
 *   Dissemination issueAs / fullSync / ....... lib/dissemination.js:38-182
 *   HashRing add/remove/checksum/lookup ...... lib/ring.js:25-182, lib/rbtree.js:70-285
 *   MembershipIterator.next .................. lib/membership-iterator.js:29-52
 *   Suspicion start/stop ..................... lib/swim/suspicion.js:45-84
 *   pingMemberNow ............................ index.js:458-515
 *   ping sender / ping-req sender ............ lib/swim/ping-sender.js:30-107,
 *                                              lib/swim/ping-req-sender.js:57-296
 *   ping / ping-req handlers + endpoint checks server/ping-handler.js:22-40,
 *                                              server/ping-req-handler.js:24-60,
 *                                              server/index.js:175-215
 *   underscore 1.13 shuffle/sample ........... (npm underscore ^1.5.2, package.json:37)
 */
#include "sim_oracle.h"
#include "farmhash32.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { ST_ABSENT = 0, ST_ALIVE = 1, ST_SUSPECT = 2, ST_FAULTY = 3, ST_LEAVE = 4 };
static const char *STATUS_STR[5] = {"", "alive", "suspect", "faulty", "leave"};
static const int STATUS_LEN[5] = {0, 5, 7, 6, 5};

#define INC0 1434401518824ULL
#define T0 1500000000000ULL
#define PERIOD 200ULL
#define SUSPICION_MS 5000ULL
#define REPLICAS 100
#define PIGGYBACK_FACTOR 15

/* ------------------------------------------------------------------ util */
static void *xmalloc(size_t n) {
    void *p = malloc(n ? n : 1);
    if (!p) { fprintf(stderr, "oracle: out of memory (%zu)\n", n); abort(); }
    return p;
}
static void *xcalloc(size_t n, size_t s) {
    void *p = calloc(n ? n : 1, s ? s : 1);
    if (!p) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    return p;
}

typedef struct { uint64_t s; } rng_t;
static uint64_t rng_next(rng_t *r) {
    r->s += 0x9E3779B97F4A7C15ULL;
    uint64_t z = r->s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
/* Math.random() */
static double rng_random(rng_t *r) { return (double)(rng_next(r) >> 11) * 0x1p-53; }
/* underscore random(min, max) = min + floor(Math.random() * (max - min + 1)) */
static int js_random(rng_t *r, int min, int max) {
    double x = rng_random(r);
    volatile double p = x * (double)(max - min + 1);
    return min + (int)floor(p);
}

static int u64_to_dec(uint64_t v, char *out) {
    char tmp[24];
    int n = 0;
    do { tmp[n++] = (char)('0' + v % 10); v /= 10; } while (v);
    for (int i = 0; i < n; i++) out[i] = tmp[n - 1 - i];
    return n;
}

int orc_max_piggyback(int server_count, int factor) {
    /* factor * Math.ceil(Math.log(serverCount + 1) / LOG_10): exact integer
     * form, verified against V8 for serverCount+1 <= 2e7. */
    uint64_t x = (uint64_t)server_count + 1, p = 1;
    int digits = 0;
    for (uint64_t t = x; t; t /= 10) digits++;
    for (int i = 1; i < digits; i++) p *= 10;
    return factor * (x == p ? digits - 1 : digits);
}

/* ------------------------------------------------------------- changes */
typedef struct {
    int32_t addr;
    int32_t status;
    uint64_t inc;
    int32_t source;       /* -1: undefined */
    uint64_t source_inc;  /* 0: undefined (JS falsy) */
} change_t;

typedef struct { change_t *v; int n, cap; } clist;
static void cl_push(clist *l, change_t c) {
    if (l->n == l->cap) {
        l->cap = l->cap ? l->cap * 2 : 16;
        l->v = (change_t *)realloc(l->v, (size_t)l->cap * sizeof(change_t));
        if (!l->v) abort();
    }
    l->v[l->n++] = c;
}
static void cl_free(clist *l) { free(l->v); l->v = NULL; l->n = l->cap = 0; }

/* ------------------------------------------------------------- sim types */
typedef struct {
    int id;
    int dead, ready, pinging, has_local;
    /* membership */
    int32_t *members; int nmembers;
    uint8_t *status; uint64_t *inc;
    uint32_t checksum; int checksum_dirty;
    /* dissemination: insertion-ordered dict keyed by address */
    int32_t *d_prev, *d_next; int d_head, d_tail, d_size;
    uint8_t *d_present, *d_status;
    int32_t *d_count, *d_source;
    uint64_t *d_inc, *d_source_inc;
    int max_pb;
    /* ring: server set + owners of colliding replica hashes */
    uint8_t *in_ring; int ring_count; int32_t *coll_owner;
    uint32_t ring_checksum; int ring_dirty;
    /* suspicion: timer index per address (-1 none) */
    int32_t *timer;
    /* iterator */
    int iter_index, iter_round;
    uint32_t *visit_stamp; uint32_t visit_epoch;
    rng_t rng;
} node_t;

typedef struct { uint64_t due; int node, addr; uint64_t inc; int cancelled, fired; } timer_t_;

enum { M_REQ_PING = 1, M_REQ_PINGREQ = 2, M_RESP = 3 };
enum { C_PM = 1, C_RELAY_PING = 2, C_PINGREQ = 3 };
typedef struct {
    int kind, from, to;
    /* request body */
    uint32_t checksum; int source; uint64_t source_inc; int target;
    clist changes;
    /* continuation at the requester */
    int cont, cont_ref;
    /* response */
    int err, ok, ping_status, has_changes;
} msg_t;
typedef struct { msg_t *v; int n, cap; } mqueue;

typedef struct { int a, target, nmembers, nerrors, nbad, called_back; } pingreq_t;
typedef struct { int k, a, target, agg; uint64_t source_inc; uint32_t checksum; } relay_t;

struct orc_sim {
    int n, churn_k, eager, round;
    uint64_t now, seed;
    char *addr_bytes; uint64_t *addr_off;
    node_t *nodes;
    /* replica hashes and collision table */
    uint32_t *rep_hash;                 /* n*REPLICAS */
    int32_t *coll_of;                   /* n*REPLICAS: collision id or -1 */
    int ncoll; uint32_t *coll_hash;
    uint32_t *pt_hash; int32_t *pt_server; int32_t *pt_coll; int npts; /* sorted distinct points */
    timer_t_ *timers; int ntimers, timers_cap, timer_head;
    mqueue cur, next;
    pingreq_t *pr; int npr, pr_cap;
    relay_t *rl; int nrl, rl_cap;
    int32_t *fail_round;
    rng_t churn_rng;
    int part_start, part_end, part_split;
    int storm_start, storm_end, storm_ppm;  /* false-suspicion storm (config 5) */
    /* join schedule (orc_sim_join): in processing order */
    int njoins; int32_t *join_round, *join_node, *join_nseeds, *join_seeds; int join_sp;
    rng_t storm_rng;
    orc_stats st;
};

static const char *addr_of(const orc_sim *S, int i, int *len) {
    *len = (int)(S->addr_off[i + 1] - S->addr_off[i]);
    return S->addr_bytes + S->addr_off[i];
}

/* --------------------------------------------------------- checksum */
static size_t view_string(const orc_sim *S, const node_t *X, uint8_t *out) {
    /* lib/membership.js:70-93: members sorted by address (ids are sorted-address
     * ranks), address + status + incarnationNumber joined by ';'. */
    size_t p = 0; int first = 1;
    for (int a = 0; a < S->n; a++) {
        if (X->status[a] == ST_ABSENT) continue;
        if (!first) out[p++] = ';';
        first = 0;
        int al; const char *as = addr_of(S, a, &al);
        memcpy(out + p, as, (size_t)al); p += (size_t)al;
        memcpy(out + p, STATUS_STR[X->status[a]], (size_t)STATUS_LEN[X->status[a]]);
        p += (size_t)STATUS_LEN[X->status[a]];
        p += (size_t)u64_to_dec(X->inc[a], (char *)out + p);
    }
    return p;
}
static uint8_t *g_strbuf; static size_t g_strcap;
static uint8_t *strbuf(size_t need) {
    if (need > g_strcap) { free(g_strbuf); g_strcap = need * 2; g_strbuf = (uint8_t *)xmalloc(g_strcap); }
    return g_strbuf;
}
static void compute_checksum(orc_sim *S, node_t *X) {
    uint8_t *buf = strbuf((size_t)S->n * 48 + 64);
    size_t len = view_string(S, X, buf);
    X->checksum = oracle_farmhash32(buf, len);
    X->checksum_dirty = 0;
}
static uint32_t get_checksum(orc_sim *S, node_t *X) {
    if (X->checksum_dirty) compute_checksum(S, X);
    return X->checksum;
}
static void compute_ring_checksum(orc_sim *S, node_t *X) {
    /* lib/ring.js:96-105: hash32(Object.keys(servers).sort().join(';')) */
    uint8_t *buf = strbuf((size_t)S->n * 48 + 64);
    size_t p = 0; int first = 1;
    for (int a = 0; a < S->n; a++) {
        if (!X->in_ring[a]) continue;
        if (!first) buf[p++] = ';';
        first = 0;
        int al; const char *as = addr_of(S, a, &al);
        memcpy(buf + p, as, (size_t)al); p += (size_t)al;
    }
    X->ring_checksum = oracle_farmhash32(buf, p);
    X->ring_dirty = 0;
}

/* ------------------------------------------------------------- ring */
static int ring_add_remove(orc_sim *S, node_t *X, const int *add, int nadd, const int *rm, int nrm) {
    /* lib/ring.js:60-94: adds first (insert-if-absent per replica, in call
     * order), then removes (erase by hash).  Points hashed by only one server
     * are present iff that server is in the set; colliding hashes keep an
     * explicit owner (lib/rbtree.js:112-117 keeps the first inserter,
     * lib/ring.js:134 / rbtree.js:152 erase by hash only). */
    int added = 0, removed = 0;
    for (int i = 0; i < nadd; i++) {
        int s = add[i];
        if (X->in_ring[s]) continue;
        X->in_ring[s] = 1; X->ring_count++;
        for (int r = 0; r < REPLICAS; r++) {
            int c = S->coll_of[(size_t)s * REPLICAS + r];
            if (c >= 0 && X->coll_owner[c] < 0) X->coll_owner[c] = s;
        }
        added = 1;
    }
    for (int i = 0; i < nrm; i++) {
        int s = rm[i];
        if (!X->in_ring[s]) continue;
        X->in_ring[s] = 0; X->ring_count--;
        for (int r = 0; r < REPLICAS; r++) {
            int c = S->coll_of[(size_t)s * REPLICAS + r];
            if (c >= 0) X->coll_owner[c] = -1;
        }
        removed = 1;
    }
    int changed = added || removed;
    if (changed) {
        X->ring_dirty = 1;
        if (S->eager) compute_ring_checksum(S, X);
    }
    return changed;
}

static int point_owner(const orc_sim *S, const node_t *X, int p) {
    if (S->pt_coll[p] >= 0) return X->coll_owner[S->pt_coll[p]];
    int s = S->pt_server[p];
    return X->in_ring[s] ? s : -1;
}

int orc_sim_ring_lookup(orc_sim *S, int v, uint32_t h) {
    /* lib/ring.js:138-147: first point >= h (rbtree.upperBound is an
     * inclusive lower bound, lib/rbtree.js:263-271), else the minimum */
    node_t *X = &S->nodes[v];
    int lo = 0, hi = S->npts;
    while (lo < hi) { int mid = (lo + hi) / 2; if (S->pt_hash[mid] < h) lo = mid + 1; else hi = mid; }
    for (int k = 0; k < S->npts; k++) {
        int p = (lo + k) % S->npts;
        int o = point_owner(S, X, p);
        if (o >= 0) return o;
    }
    return -1;
}

/* ------------------------------------------------------------- dissemination */
static void d_record(node_t *X, const change_t *c) {
    /* lib/dissemination.js:125-127: changes[address] = change (overwrite keeps
     * the key's position; the new object has no piggybackCount). */
    int a = c->addr;
    if (!X->d_present[a]) {
        X->d_present[a] = 1;
        X->d_prev[a] = X->d_tail; X->d_next[a] = -1;
        if (X->d_tail >= 0) X->d_next[X->d_tail] = a; else X->d_head = a;
        X->d_tail = a; X->d_size++;
    }
    X->d_count[a] = -1;
    X->d_status[a] = (uint8_t)c->status; X->d_inc[a] = c->inc;
    X->d_source[a] = c->source; X->d_source_inc[a] = c->source_inc;
}
static void d_delete(node_t *X, int a) {
    int p = X->d_prev[a], q = X->d_next[a];
    if (p >= 0) X->d_next[p] = q; else X->d_head = q;
    if (q >= 0) X->d_prev[q] = p; else X->d_tail = p;
    X->d_present[a] = 0; X->d_size--;
}
static void d_clear(node_t *X) {
    for (int a = X->d_head; a >= 0;) { int q = X->d_next[a]; X->d_present[a] = 0; a = q; }
    X->d_head = X->d_tail = -1; X->d_size = 0;
}
static void adjust_max_pb(node_t *X) {
    X->max_pb = orc_max_piggyback(X->ring_count, PIGGYBACK_FACTOR);
}

/* lib/dissemination.js:138-182; filter_src < 0 means issueAsSender */
static void issue_as(node_t *X, int filter_src, uint64_t filter_inc, clist *out) {
    int a = X->d_head;
    while (a >= 0) {
        int nxt = X->d_next[a];
        if (X->d_count[a] < 0) X->d_count[a] = 0;
        int filtered = filter_src >= 0 && filter_inc != 0 && X->d_source[a] >= 0 &&
                       X->d_source_inc[a] != 0 && X->d_source[a] == filter_src &&
                       X->d_source_inc[a] == filter_inc;
        if (!filtered) {
            X->d_count[a] += 1;
            if (X->d_count[a] > X->max_pb) {
                d_delete(X, a);
            } else {
                change_t c = {a, X->d_status[a], X->d_inc[a], X->d_source[a], X->d_source_inc[a]};
                cl_push(out, c);
            }
        }
        a = nxt;
    }
}
static void full_sync(orc_sim *S, node_t *X, clist *out) {
    /* lib/dissemination.js:61-76: every member in `members` order, source=self,
     * no sourceIncarnationNumber. */
    S->st.full_syncs++;
    for (int i = 0; i < X->nmembers; i++) {
        int a = X->members[i];
        change_t c = {a, X->status[a], X->inc[a], X->id, 0};
        cl_push(out, c);
    }
}
static void issue_as_receiver(orc_sim *S, node_t *X, int sender, uint64_t sender_inc,
                              uint32_t sender_checksum, clist *out) {
    issue_as(X, sender, sender_inc, out);
    if (out->n > 0) return;
    if (get_checksum(S, X) != sender_checksum) full_sync(S, X, out);
}

/* ------------------------------------------------------------- suspicion */
static void suspicion_stop(orc_sim *S, node_t *X, int addr) {
    int t = X->timer[addr];
    if (t >= 0) S->timers[t].cancelled = 1;
    X->timer[addr] = -1;
}
static void suspicion_start(orc_sim *S, node_t *X, const change_t *u) {
    if (u->addr == X->id) return;  /* lib/swim/suspicion.js:56-62 */
    if (X->timer[u->addr] >= 0) suspicion_stop(S, X, u->addr);
    if (S->ntimers == S->timers_cap) {
        S->timers_cap = S->timers_cap ? S->timers_cap * 2 : 1024;
        S->timers = (timer_t_ *)realloc(S->timers, (size_t)S->timers_cap * sizeof(timer_t_));
        if (!S->timers) abort();
    }
    timer_t_ t = {S->now + SUSPICION_MS, X->id, u->addr, u->inc, 0, 0};
    S->timers[S->ntimers] = t;
    X->timer[u->addr] = S->ntimers++;
}

/* ------------------------------------------------------------- membership */
static void members_splice(node_t *X, int pos, int a) {
    memmove(X->members + pos + 1, X->members + pos, (size_t)(X->nmembers - pos) * sizeof(int32_t));
    X->members[pos] = a;
    X->nmembers++;
}

#ifdef ORC_TRACE_APPLY
/* (diagnostic builds only, tools/apply_lines.c: every applied (node, address)
 * with the delivery wave it happened in) */
void orc_trace_apply(int wave, int node, int addr);
#endif

static void apply_update(orc_sim *S, node_t *X, const change_t *c) {
    (void)S;
#ifdef ORC_TRACE_APPLY
    orc_trace_apply(S->st.waves, X->id, c->addr);
#endif
    /* lib/membership.js:273-312 (address / incarnation are always defined in
     * the simulation) */
    if (X->status[c->addr] == ST_ABSENT) {
        if (c->addr == X->id) X->has_local = 1;
        int pos = (int)floor(rng_random(&X->rng) * (double)X->nmembers); /* :99-101 */
        members_splice(X, pos, c->addr);
    }
    X->status[c->addr] = (uint8_t)c->status;
    X->inc[c->addr] = c->inc;
}

static void update_listener(orc_sim *S, node_t *X, const clist *applied) {
    /* lib/membership-update-listener.js:24-75 */
    int *add = (int *)xmalloc((size_t)applied->n * sizeof(int) + 4);
    int *rm = (int *)xmalloc((size_t)applied->n * sizeof(int) + 4);
    int nadd = 0, nrm = 0;
    for (int i = 0; i < applied->n; i++) {
        const change_t *u = &applied->v[i];
        if (u->status == ST_ALIVE) { add[nadd++] = u->addr; suspicion_stop(S, X, u->addr); }
        else if (u->status == ST_SUSPECT) { suspicion_start(S, X, u); }
        else if (u->status == ST_FAULTY) { rm[nrm++] = u->addr; suspicion_stop(S, X, u->addr); }
        else if (u->status == ST_LEAVE) { rm[nrm++] = u->addr; suspicion_stop(S, X, u->addr); }
        d_record(X, u);
    }
    if (nadd > 0 || nrm > 0) {
        if (ring_add_remove(S, X, add, nadd, rm, nrm)) adjust_max_pb(X); /* 'ringChanged' */
    }
    free(add); free(rm);
}

static int override_rules(const node_t *X, int a, const change_t *c) {
    /* lib/membership-update-rules.js:25-59 */
    int ms = X->status[a]; uint64_t mi = X->inc[a];
    switch (c->status) {
    case ST_ALIVE: return c->inc > mi;
    case ST_SUSPECT: return (ms == ST_SUSPECT && c->inc > mi) || (ms == ST_FAULTY && c->inc > mi) ||
                            (ms == ST_ALIVE && c->inc >= mi);
    case ST_FAULTY: return (ms == ST_SUSPECT && c->inc >= mi) || (ms == ST_FAULTY && c->inc > mi) ||
                           (ms == ST_ALIVE && c->inc >= mi);
    case ST_LEAVE: return ms != ST_LEAVE && c->inc >= mi;
    default: return 0;
    }
}

/* Membership.update: mutates `changes` in place like _.extend does (:251). */
static int membership_update(orc_sim *S, node_t *X, change_t *changes, int nchanges) {
    S->st.evaluated += nchanges;
    if (nchanges == 0) return 0;
    clist applied = {0};
    for (int i = 0; i < nchanges; i++) {
        change_t *c = &changes[i];
        if (X->status[c->addr] == ST_ABSENT) {
            apply_update(S, X, c); cl_push(&applied, *c); continue;
        }
        if (c->addr == X->id && (c->status == ST_SUSPECT || c->status == ST_FAULTY)) {
            c->status = ST_ALIVE; c->inc = S->now;  /* :244-254 local override */
            apply_update(S, X, c); cl_push(&applied, *c); continue;
        }
        if (override_rules(X, c->addr, c)) { apply_update(S, X, c); cl_push(&applied, *c); }
    }
    int napplied = applied.n;
    if (napplied > 0) {
        X->checksum_dirty = 1;
        if (S->eager) compute_checksum(S, X);
        update_listener(S, X, &applied);
    }
    S->st.applied += napplied;
    cl_free(&applied);
    return napplied;
}

static void make_update(orc_sim *S, node_t *X, int addr, uint64_t inc, int status) {
    /* lib/membership.js:324-352 */
    change_t c;
    c.addr = addr; c.status = status; c.inc = inc;
    if (X->has_local) { c.source = X->id; c.source_inc = X->inc[X->id]; }
    else { c.source = addr; c.source_inc = inc; }
    membership_update(S, X, &c, 1);
}

static int is_pingable(const node_t *X, int a) {
    return a != X->id && (X->status[a] == ST_ALIVE || X->status[a] == ST_SUSPECT);
}

static void shuffle_members(node_t *X) {
    /* _.shuffle (underscore 1.13): sample(list, Infinity) */
    int L = X->nmembers;
    for (int i = 0; i < L; i++) {
        int r = js_random(&X->rng, i, L - 1);
        int32_t t = X->members[i]; X->members[i] = X->members[r]; X->members[r] = t;
    }
}

static int iterator_next(node_t *X) {
    /* lib/membership-iterator.js:29-52 */
    X->visit_epoch++;
    if (X->visit_epoch == 0) { memset(X->visit_stamp, 0, (size_t)X->nmembers * 4); X->visit_epoch = 1; }
    int visited = 0, max = X->nmembers;
    while (visited < max) {
        X->iter_index++;
        if (X->iter_index >= X->nmembers) { X->iter_index = 0; X->iter_round++; shuffle_members(X); }
        int a = X->members[X->iter_index];
        if (X->visit_stamp[a] != X->visit_epoch) { X->visit_stamp[a] = X->visit_epoch; visited++; }
        if (is_pingable(X, a)) return a;
    }
    return -1;
}

static int random_pingable(node_t *X, int n, int exclude, int *out) {
    /* lib/membership.js:111-120 with underscore 1.13 sample(list, n) */
    int *f = (int *)xmalloc((size_t)X->nmembers * sizeof(int) + 4);
    int L = 0;
    for (int i = 0; i < X->nmembers; i++) {
        int a = X->members[i];
        if (a == exclude) continue;
        if (is_pingable(X, a)) f[L++] = a;
    }
    int k = n < L ? n : L;
    for (int i = 0; i < k; i++) {
        int r = js_random(&X->rng, i, L - 1);
        int t = f[i]; f[i] = f[r]; f[r] = t;
    }
    memcpy(out, f, (size_t)k * sizeof(int));
    free(f);
    return k;
}

/* ------------------------------------------------------------- transport */
static void enqueue(orc_sim *S, msg_t m) {
    mqueue *q = &S->next;
    if (q->n == q->cap) {
        q->cap = q->cap ? q->cap * 2 : 1024;
        q->v = (msg_t *)realloc(q->v, (size_t)q->cap * sizeof(msg_t));
        if (!q->v) abort();
    }
    q->v[q->n++] = m;
    S->st.messages++;
}

static void send_ping(orc_sim *S, node_t *X, int target, int cont, int ref) {
    /* lib/swim/ping-sender.js:57-99 */
    msg_t m; memset(&m, 0, sizeof m);
    m.kind = M_REQ_PING; m.from = X->id; m.to = target;
    issue_as(X, -1, 0, &m.changes);
    m.checksum = get_checksum(S, X);
    m.source = X->id; m.source_inc = X->has_local ? X->inc[X->id] : 0;
    m.cont = cont; m.cont_ref = ref;
    enqueue(S, m);
}

static void respond(orc_sim *S, const msg_t *req, int err, int ok, clist *changes, int has_changes, int ping_status) {
    msg_t r; memset(&r, 0, sizeof r);
    r.kind = M_RESP; r.from = req->to; r.to = req->from;
    r.cont = req->cont; r.cont_ref = req->cont_ref;
    r.err = err; r.ok = ok; r.ping_status = ping_status; r.has_changes = has_changes;
    if (changes) { r.changes = *changes; changes->v = NULL; changes->n = changes->cap = 0; }
    enqueue(S, r);
}

static void ping_member_now(orc_sim *S, node_t *A) {
    /* index.js:458-515 */
    if (A->pinging || !A->ready) return;
    int m = iterator_next(A);
    if (m < 0) return;
    A->pinging = 1;
    send_ping(S, A, m, C_PM, m);
}

static void send_ping_req(orc_sim *S, node_t *A, int target) {
    /* lib/swim/ping-req-sender.js:153-296 */
    int members[3];
    int k = random_pingable(A, 3, target, members);
    if (k == 0) { A->pinging = 0; return; } /* NoMembersError -> pingMemberNow callback */
    if (S->npr == S->pr_cap) {
        S->pr_cap = S->pr_cap ? S->pr_cap * 2 : 256;
        S->pr = (pingreq_t *)realloc(S->pr, (size_t)S->pr_cap * sizeof(pingreq_t));
        if (!S->pr) abort();
    }
    pingreq_t g = {A->id, target, k, 0, 0, 0};
    int gi = S->npr++;
    S->pr[gi] = g;
    for (int i = 0; i < k; i++) {
        msg_t m; memset(&m, 0, sizeof m);
        m.kind = M_REQ_PINGREQ; m.from = A->id; m.to = members[i];
        m.checksum = get_checksum(S, A);
        issue_as(A, -1, 0, &m.changes);
        m.source = A->id; m.source_inc = A->has_local ? A->inc[A->id] : 0;
        m.target = target;
        m.cont = C_PINGREQ; m.cont_ref = gi;
        enqueue(S, m);
    }
}

static void pingreq_done(orc_sim *S, int gi, int kind /* 0 ok, 1 ping error, 2 bad status */) {
    pingreq_t *g = &S->pr[gi];
    node_t *A = &S->nodes[g->a];
    if (g->called_back) return;
    if (kind == 0) { g->called_back = 1; A->pinging = 0; return; }
    g->nerrors++;
    if (kind == 2) g->nbad++;
    if (g->nerrors < g->nmembers) return;
    if (g->nbad > 0) make_update(S, A, g->target, A->inc[g->target], ST_SUSPECT); /* makeSuspect */
    g->called_back = 1;
    A->pinging = 0;
}

/* partition injection (harness fault model): requests across `split` fail
 * during rounds [start, end) like requests to a dead node */
static int cut(const orc_sim *S, int a, int b) {
    return S->part_split > 0 && S->round >= S->part_start && S->round < S->part_end &&
           ((a < S->part_split) != (b < S->part_split));
}

static void deliver(orc_sim *S, msg_t *m) {
    if (m->kind == M_REQ_PING || m->kind == M_REQ_PINGREQ) {
        node_t *B = &S->nodes[m->to];
        if (B->dead || cut(S, m->from, m->to)) { respond(S, m, 1, 0, NULL, 0, 0); return; }
        /* server/index.js:175-215: body checks (checksum 0 is falsy) */
        if (m->checksum == 0) { respond(S, m, 0, 0, NULL, 0, 0); return; }
        membership_update(S, B, m->changes.v, m->changes.n);
        if (m->kind == M_REQ_PING) {
            clist out = {0};
            issue_as_receiver(S, B, m->source, m->source_inc, m->checksum, &out);
            respond(S, m, 0, 1, &out, 1, 0);
        } else {
            if (S->nrl == S->rl_cap) {
                S->rl_cap = S->rl_cap ? S->rl_cap * 2 : 256;
                S->rl = (relay_t *)realloc(S->rl, (size_t)S->rl_cap * sizeof(relay_t));
                if (!S->rl) abort();
            }
            relay_t r = {B->id, m->from, m->target, m->cont_ref, m->source_inc, m->checksum};
            int ri = S->nrl++;
            S->rl[ri] = r;
            send_ping(S, B, m->target, C_RELAY_PING, ri);
        }
        return;
    }
    /* response at the requester */
    node_t *X = &S->nodes[m->to];
    int is_ok = !m->err && m->ok && m->has_changes;
    if (m->cont == C_PM) {
        if (is_ok) {
            membership_update(S, X, m->changes.v, m->changes.n);  /* ping-sender.js:36-39 */
            X->pinging = 0;
            membership_update(S, X, m->changes.v, m->changes.n);  /* index.js:488 */
        } else {
            send_ping_req(S, X, m->cont_ref);
        }
    } else if (m->cont == C_RELAY_PING) {
        relay_t *r = &S->rl[m->cont_ref];
        if (is_ok) {
            membership_update(S, X, m->changes.v, m->changes.n);
            membership_update(S, X, m->changes.v, m->changes.n);  /* ping-req-handler.js:50 */
        }
        clist out = {0};
        issue_as_receiver(S, X, r->a, r->source_inc, r->checksum, &out);
        msg_t req; memset(&req, 0, sizeof req);
        req.from = r->a; req.to = X->id; req.cont = C_PINGREQ; req.cont_ref = r->agg;
        respond(S, &req, 0, 1, &out, 1, is_ok);
    } else if (m->cont == C_PINGREQ) {
        if (m->err || !m->ok) { pingreq_done(S, m->cont_ref, 1); return; }
        membership_update(S, X, m->changes.v, m->changes.n);  /* ping-req-sender.js:138 */
        pingreq_done(S, m->cont_ref, m->ping_status ? 0 : 2);
    }
}

static void run_waves(orc_sim *S) {
    while (S->next.n > 0) {
        mqueue w = S->next;
        S->next = S->cur; S->next.n = 0;
        for (int i = 0; i < w.n; i++) { deliver(S, &w.v[i]); cl_free(&w.v[i].changes); }
        S->cur = w; S->cur.n = 0;
        S->st.waves++;
    }
}

/* ------------------------------------------------------------- setup */
static int cmp_str(const void *a, const void *b) { return strcmp(*(char *const *)a, *(char *const *)b); }

typedef struct { uint32_t h; int32_t s, r; } pt_t;
static int cmp_pt(const void *a, const void *b) {
    const pt_t *x = (const pt_t *)a, *y = (const pt_t *)b;
    if (x->h != y->h) return x->h < y->h ? -1 : 1;
    if (x->s != y->s) return x->s < y->s ? -1 : 1;
    return x->r - y->r;
}

orc_sim *orc_sim_new(int n, uint64_t seed, int churn_k, int eager) { return orc_sim_new2(n, seed, churn_k, eager, 0); }

/* hash_shift > 0 (testing): clear that many low bits of every replica hash, so
 * that many replica points collide (exercises lib/rbtree.js:112-117,152) */
orc_sim *orc_sim_new2(int n, uint64_t seed, int churn_k, int eager, int hash_shift) {
    return orc_sim_new3(n, seed, churn_k, eager, hash_shift, NULL, NULL, NULL, NULL);
}

/* addr_bytes/addr_off: the cluster's addresses in sort order (NULL: the sim
 * scheme); vstatus/vinc: n x n full views for the bootstrap (NULL: every
 * member alive at INC0 + id) -- the harness's cfg.addresses / cfg.views */
orc_sim *orc_sim_new3(int n, uint64_t seed, int churn_k, int eager, int hash_shift, const uint8_t *addr_bytes,
                      const uint64_t *addr_off, const uint8_t *vstatus, const uint64_t *vinc) {
    orc_sim *S = (orc_sim *)xcalloc(1, sizeof(orc_sim));
    S->n = n; S->churn_k = churn_k; S->eager = eager;
    /* addresses: 10.<b2>.<b1>.<b0>:<3000+i%7>, ids = sorted ranks */
    char **raw = (char **)xmalloc((size_t)n * sizeof(char *));
    for (int i = 0; i < n; i++) {
        raw[i] = (char *)xmalloc(40);
        if (addr_bytes) {
            size_t l = (size_t)(addr_off[i + 1] - addr_off[i]);
            if (l > 32) l = 32;
            memcpy(raw[i], addr_bytes + addr_off[i], l);
            raw[i][l] = 0;
        } else {
            snprintf(raw[i], 40, "10.%d.%d.%d:%d", (i >> 16) & 255, (i >> 8) & 255, i & 255, 3000 + i % 7);
        }
    }
    qsort(raw, (size_t)n, sizeof(char *), cmp_str);
    S->addr_off = (uint64_t *)xmalloc((size_t)(n + 1) * 8);
    S->addr_bytes = (char *)xmalloc((size_t)n * 40);
    uint64_t p = 0;
    for (int i = 0; i < n; i++) {
        S->addr_off[i] = p;
        size_t l = strlen(raw[i]);
        memcpy(S->addr_bytes + p, raw[i], l); p += l;
        free(raw[i]);
    }
    S->addr_off[n] = p;
    free(raw);

    /* replica points hash32(server + i) (lib/ring.js:50-58) and the table of
     * hash values produced by more than one server */
    S->rep_hash = (uint32_t *)xmalloc((size_t)n * REPLICAS * 4);
    pt_t *pts = (pt_t *)xmalloc((size_t)n * REPLICAS * sizeof(pt_t));
    char buf[64];
    for (int s = 0; s < n; s++) {
        int al; const char *as = addr_of(S, s, &al);
        memcpy(buf, as, (size_t)al);
        for (int r = 0; r < REPLICAS; r++) {
            int l = al + u64_to_dec((uint64_t)r, buf + al);
            uint32_t h = oracle_farmhash32((const uint8_t *)buf, (size_t)l);
            if (hash_shift > 0) h = (h >> hash_shift) << hash_shift;
            S->rep_hash[(size_t)s * REPLICAS + r] = h;
            pt_t t = {h, s, r};
            pts[(size_t)s * REPLICAS + r] = t;
        }
    }
    size_t np = (size_t)n * REPLICAS;
    qsort(pts, np, sizeof(pt_t), cmp_pt);
    S->coll_of = (int32_t *)xmalloc(np * 4);
    for (size_t i = 0; i < np; i++) S->coll_of[i] = -1;
    S->pt_hash = (uint32_t *)xmalloc(np * 4);
    S->pt_server = (int32_t *)xmalloc(np * 4);
    S->pt_coll = (int32_t *)xmalloc(np * 4);
    S->coll_hash = (uint32_t *)xmalloc(np * 4);
    for (size_t i = 0; i < np;) {
        size_t j = i;
        int multi = 0;
        while (j < np && pts[j].h == pts[i].h) { if (pts[j].s != pts[i].s) multi = 1; j++; }
        int cid = -1;
        if (multi) {
            cid = S->ncoll++;
            S->coll_hash[cid] = pts[i].h;
            for (size_t k = i; k < j; k++) S->coll_of[(size_t)pts[k].s * REPLICAS + pts[k].r] = cid;
        }
        S->pt_hash[S->npts] = pts[i].h; S->pt_server[S->npts] = pts[i].s; S->pt_coll[S->npts] = cid;
        S->npts++;
        i = j;
    }
    free(pts);

    S->nodes = (node_t *)xcalloc((size_t)n, sizeof(node_t));
    S->fail_round = (int32_t *)xmalloc((size_t)n * 4);
    for (int i = 0; i < n; i++) S->fail_round[i] = -1;
    S->churn_rng.s = seed ^ 0x5851F42D4C957F2DULL;
    S->seed = seed;

    for (int i = 0; i < n; i++) {
        node_t *X = &S->nodes[i];
        X->id = i;
        X->members = (int32_t *)xmalloc((size_t)n * 4);
        X->status = (uint8_t *)xcalloc((size_t)n, 1);
        X->inc = (uint64_t *)xcalloc((size_t)n, 8);
        X->d_prev = (int32_t *)xmalloc((size_t)n * 4);
        X->d_next = (int32_t *)xmalloc((size_t)n * 4);
        X->d_present = (uint8_t *)xcalloc((size_t)n, 1);
        X->d_status = (uint8_t *)xcalloc((size_t)n, 1);
        X->d_count = (int32_t *)xmalloc((size_t)n * 4);
        X->d_source = (int32_t *)xmalloc((size_t)n * 4);
        X->d_inc = (uint64_t *)xcalloc((size_t)n, 8);
        X->d_source_inc = (uint64_t *)xcalloc((size_t)n, 8);
        X->d_head = X->d_tail = -1;
        X->in_ring = (uint8_t *)xcalloc((size_t)n, 1);
        X->coll_owner = (int32_t *)xmalloc((size_t)(S->ncoll + 1) * 4);
        for (int c = 0; c < S->ncoll; c++) X->coll_owner[c] = -1;
        X->timer = (int32_t *)xmalloc((size_t)n * 4);
        for (int a = 0; a < n; a++) X->timer[a] = -1;
        X->visit_stamp = (uint32_t *)xcalloc((size_t)n, 4);
        X->iter_index = -1;
        X->max_pb = 1;  /* Dissemination.Defaults.maxPiggybackCount */
        X->checksum_dirty = 1; X->ring_dirty = 1;
        X->rng.s = seed ^ ((uint64_t)(i + 1) * 0xD1B54A32D192ED03ULL);

        /* bootstrap (index.js:233-267 with a full-membership join result) */
        S->now = INC0 + (uint64_t)i;
        const uint8_t *rs = vstatus ? vstatus + (size_t)i * n : NULL;
        const uint64_t *ri = vinc ? vinc + (size_t)i * n : NULL;
        make_update(S, X, i, ri ? ri[i] : INC0 + (uint64_t)i, ST_ALIVE);  /* makeAlive(self) */
        /* set(): merge skips self, keeps max incarnation, insertion order */
        clist set_updates = {0};
        for (int j = 0; j < n; j++) {
            if (j == i || (rs && rs[j] == ST_ABSENT)) continue;  /* (absent: not in the join result) */
            change_t c = {j, rs ? rs[j] : ST_ALIVE, ri ? ri[j] : INC0 + (uint64_t)j, -1, 0};
            cl_push(&set_updates, c);
        }
        for (int k = 0; k < set_updates.n; k++) {
            const change_t *c = &set_updates.v[k];
            X->members[X->nmembers++] = c->addr;
            X->status[c->addr] = (uint8_t)c->status;
            X->inc[c->addr] = c->inc;
        }
        X->checksum_dirty = 1;
        if (S->eager) compute_checksum(S, X);
        /* set listener (lib/membership-set-listener.js:24-48) */
        int *add = (int *)xmalloc((size_t)set_updates.n * 4 + 4);
        int nadd = 0;
        for (int k = 0; k < set_updates.n; k++) {
            const change_t *c = &set_updates.v[k];
            if (c->status == ST_ALIVE) add[nadd++] = c->addr;
            else if (c->status == ST_SUSPECT) suspicion_start(S, X, c);
            d_record(X, c);
        }
        if (nadd > 0) ring_add_remove(S, X, add, nadd, NULL, 0);  /* no ringChanged */
        free(add);
        cl_free(&set_updates);
        shuffle_members(X);   /* lib/swim/gossip.js:85 */
        X->ready = 1;
        d_clear(X);           /* harness: dissemination cleared after set() */
    }
    S->st.evaluated = S->st.applied = 0;
    return S;
}

void orc_sim_free(orc_sim *S) {
    if (!S) return;
    for (int i = 0; i < S->n; i++) {
        node_t *X = &S->nodes[i];
        free(X->members); free(X->status); free(X->inc); free(X->d_prev); free(X->d_next);
        free(X->d_present); free(X->d_status); free(X->d_count); free(X->d_source); free(X->d_inc);
        free(X->d_source_inc); free(X->in_ring); free(X->coll_owner); free(X->timer); free(X->visit_stamp);
    }
    free(S->nodes); free(S->addr_bytes); free(S->addr_off); free(S->rep_hash); free(S->coll_of);
    free(S->coll_hash); free(S->pt_hash); free(S->pt_server); free(S->pt_coll); free(S->timers);
    free(S->cur.v); free(S->next.v); free(S->pr); free(S->rl); free(S->fail_round);
    free(S->join_round); free(S->join_node); free(S->join_nseeds); free(S->join_seeds);
    free(S);
}

int orc_sim_fail(orc_sim *S, int node, int round) {
    if (node < 0 || node >= S->n) return -1;
    S->fail_round[node] = round;
    return 0;
}

int orc_sim_storm(orc_sim *S, int start, int end, int ppm) {
    S->storm_start = start; S->storm_end = end; S->storm_ppm = ppm;
    S->storm_rng.s = S->seed ^ 0x2545F4914F6CDD1DULL;
    return 0;
}

int orc_sim_partition(orc_sim *S, int start, int end, int split) {
    S->part_start = start; S->part_end = end; S->part_split = split;
    return 0;
}

/* ------------------------------------------------------------- join path */
/* Node e of the schedule joins (index.js:233-292, lib/swim/join-sender.js):
 * makeAlive(self, now) (index.js:235); each seed in order handles the join
 * (server/join-handler.js:76-98): makeAlive(joiner, its incarnation), reply =
 * {checksum, fullSync()}; mergeJoinResponses (lib/swim/join-response-merge.js:
 * 22-56) -> update() while not ready (stashed: evaluated, none applied) ->
 * set() (lib/membership.js:162-206, changeset merge :22-51) with its listener
 * (lib/membership-set-listener.js:24-48) -> shuffle() (gossip.start). */
static void join_node(orc_sim *S, int e) {
    node_t *X = &S->nodes[S->join_node[e]];
    const int n = S->n, ns = S->join_nseeds[e];
    const int32_t *seeds = S->join_seeds + (size_t)e * S->join_sp;
    make_update(S, X, X->id, S->now, ST_ALIVE);  /* no local member yet: source = itself, sourceInc = now */
    uint32_t *cs = (uint32_t *)xmalloc((size_t)ns * 4 + 4);
    int32_t **mem = (int32_t **)xmalloc((size_t)ns * sizeof(int32_t *) + 8);
    uint8_t **mst = (uint8_t **)xmalloc((size_t)ns * sizeof(uint8_t *) + 8);
    uint64_t **minc = (uint64_t **)xmalloc((size_t)ns * sizeof(uint64_t *) + 8);
    int *mcnt = (int *)xmalloc((size_t)ns * 4 + 4);
    for (int k = 0; k < ns; k++) {
        node_t *D = &S->nodes[seeds[k]];
        make_update(S, D, X->id, X->inc[X->id], ST_ALIVE);  /* handleJoin's makeAlive(source, incarnation) */
        cs[k] = get_checksum(S, D);
        S->st.full_syncs++;  /* the reply's dissemination.fullSync() */
        mcnt[k] = D->nmembers;
        mem[k] = (int32_t *)xmalloc((size_t)D->nmembers * 4 + 4);
        memcpy(mem[k], D->members, (size_t)D->nmembers * 4);
        mst[k] = (uint8_t *)xmalloc((size_t)n);
        memcpy(mst[k], D->status, (size_t)n);
        minc[k] = (uint64_t *)xmalloc((size_t)n * 8);
        memcpy(minc[k], D->inc, (size_t)n * 8);
    }
    int same = ns > 0;  /* hasSameChecksums: every checksum truthy and equal */
    for (int k = 0; k < ns; k++) same = same && cs[k] != 0 && cs[k] == cs[0];
    const int K = same ? 1 : ns;
    /* mergeMembershipChangesets: first-appearance order, largest incarnation
     * (the first of equals), the local member skipped */
    int32_t *pos = (int32_t *)xmalloc((size_t)n * 4);
    for (int a = 0; a < n; a++) pos[a] = -1;
    clist ups = {0};
    for (int k = 0; k < K; k++)
        for (int i = 0; i < mcnt[k]; i++) {
            int a = mem[k][i];
            if (a == X->id) continue;
            change_t c = {a, mst[k][a], minc[k][a], seeds[k], 0};  /* fullSync: source = the seed */
            if (pos[a] < 0) { pos[a] = ups.n; cl_push(&ups, c); }
            else if (ups.v[pos[a]].inc < c.inc) ups.v[pos[a]] = c;
        }
    S->st.evaluated += same ? mcnt[0] : ups.n;  /* update(updates) before ready */
    for (int k = 0; k < ups.n; k++) {           /* set(): pushed after the local member */
        const change_t *c = &ups.v[k];
        X->members[X->nmembers++] = c->addr;
        X->status[c->addr] = (uint8_t)c->status;
        X->inc[c->addr] = c->inc;
    }
    X->checksum_dirty = 1;
    if (S->eager) compute_checksum(S, X);
    int *add = (int *)xmalloc((size_t)ups.n * 4 + 4);
    int nadd = 0;
    for (int k = 0; k < ups.n; k++) {
        const change_t *c = &ups.v[k];
        if (c->status == ST_ALIVE) add[nadd++] = c->addr;
        else if (c->status == ST_SUSPECT) suspicion_start(S, X, c);
        d_record(X, c);
    }
    if (nadd > 0) ring_add_remove(S, X, add, nadd, NULL, 0);  /* no ringChanged */
    shuffle_members(X);
    X->ready = 1;
    X->dead = 0;
    free(add); free(pos); cl_free(&ups);
    for (int k = 0; k < ns; k++) { free(mem[k]); free(mst[k]); free(minc[k]); }
    free(cs); free(mem); free(mst); free(minc); free(mcnt);
}

/* Before the first round: schedule joins; the joiners start outside the
 * cluster (empty views, a fresh RNG, not pinging).  The other nodes' views
 * must not hold them (orc_sim_new3 with status 0 for them). */
int orc_sim_join(orc_sim *S, const int32_t *joiners, const int32_t *rounds, const int32_t *seeds, int count,
                 int seeds_per) {
    if (S->round != 0 || S->njoins) return -1;
    S->njoins = count;
    S->join_sp = seeds_per > 0 ? seeds_per : 1;
    S->join_round = (int32_t *)xmalloc((size_t)count * 4 + 4);
    S->join_node = (int32_t *)xmalloc((size_t)count * 4 + 4);
    S->join_nseeds = (int32_t *)xmalloc((size_t)count * 4 + 4);
    S->join_seeds = (int32_t *)xmalloc((size_t)count * S->join_sp * 4 + 4);
    for (int e = 0; e < count; e++) {
        S->join_round[e] = rounds[e]; S->join_node[e] = joiners[e];
        int k = 0;
        for (int q = 0; q < seeds_per; q++)
            if (seeds[(size_t)e * seeds_per + q] >= 0) S->join_seeds[(size_t)e * S->join_sp + k++] = seeds[(size_t)e * seeds_per + q];
        S->join_nseeds[e] = k;
        node_t *X = &S->nodes[joiners[e]];
        for (int a = 0; a < S->n; a++) {
            X->status[a] = 0; X->inc[a] = 0; X->in_ring[a] = 0;
            if (X->timer[a] >= 0) { S->timers[X->timer[a]].cancelled = 1; X->timer[a] = -1; }
        }
        X->nmembers = 0;
        d_clear(X);
        X->ring_count = 0;
        for (int c = 0; c < S->ncoll; c++) X->coll_owner[c] = -1;
        X->iter_index = -1; X->iter_round = 0; X->visit_epoch = 0;
        X->max_pb = 1;
        X->checksum_dirty = 1; X->ring_dirty = 1;
        X->rng.s = S->seed ^ ((uint64_t)(joiners[e] + 1) * 0xD1B54A32D192ED03ULL);
        X->ready = 0; X->has_local = 0; X->pinging = 0;
        X->dead = 2;
    }
    return 0;
}

int orc_sim_round(orc_sim *S, int churn_active, orc_stats *st, int32_t *churned_out, int *nchurned) {
    memset(&S->st, 0, sizeof S->st);
    int r = S->round;
    S->now = T0 + PERIOD * (uint64_t)r;
    for (int i = 0; i < S->n; i++) if (S->fail_round[i] == r) S->nodes[i].dead = 1;

    /* due suspicion timers, creation order (constant 5000 ms delay keeps the
     * array sorted by due time) */
    while (S->timer_head < S->ntimers && S->timers[S->timer_head].due <= S->now) {
        timer_t_ *t = &S->timers[S->timer_head++];
        if (t->cancelled || S->nodes[t->node].dead) continue;
        t->fired = 1;
        node_t *X = &S->nodes[t->node];
        make_update(S, X, t->addr, t->inc, ST_FAULTY);   /* lib/swim/suspicion.js:66-68 */
    }

    /* joins of this round, in schedule order (join path) */
    for (int e = 0; e < S->njoins; e++)  /* (a node that fail-stopped before its round never joins) */
        if (S->join_round[e] == r && S->nodes[S->join_node[e]].dead != 1) join_node(S, e);

    int nc = 0;
    if (churn_active) {
        int *cand = (int *)xmalloc((size_t)S->n * 4);
        int L = 0;
        for (int i = 0; i < S->n; i++) if (!S->nodes[i].dead) cand[L++] = i;
        int k = S->churn_k < L ? S->churn_k : L;
        for (int j = 0; j < k; j++) {
            int rr = j + (int)floor(rng_random(&S->churn_rng) * (double)(L - j));
            int t = cand[j]; cand[j] = cand[rr]; cand[rr] = t;
        }
        for (int j = 0; j < k; j++) {
            node_t *X = &S->nodes[cand[j]];
            make_update(S, X, X->id, S->now, ST_ALIVE);
            if (churned_out) churned_out[j] = cand[j];
        }
        nc = k;
        free(cand);
    }
    if (nchurned) *nchurned = nc;

    /* false-suspicion storm (harness common.js chooseStorm): K victims by
     * partial Fisher-Yates over the live ids, then per victim an accuser drawn
     * from the other live ids; in draw order, accuser.makeSuspect(victim, its
     * view's incarnation of the victim) (lib/membership.js:154-156) */
    if (S->storm_ppm > 0 && r >= S->storm_start && r < S->storm_end) {
        int *live = (int *)xmalloc((size_t)S->n * 4), *cand = (int *)xmalloc((size_t)S->n * 4);
        int L = 0;
        for (int i = 0; i < S->n; i++) if (!S->nodes[i].dead) live[L++] = i;
        if (L >= 2) {
            int K = (int)(((int64_t)L * S->storm_ppm + 999999) / 1000000);
            if (K > L) K = L;
            memcpy(cand, live, (size_t)L * 4);
            for (int j = 0; j < K; j++) {
                int rr = j + (int)floor(rng_random(&S->storm_rng) * (double)(L - j));
                int t = cand[j]; cand[j] = cand[rr]; cand[rr] = t;
            }
            int *acc = (int *)xmalloc((size_t)K * 4 + 4);
            for (int j = 0; j < K; j++) {
                int v = cand[j], lo = 0, hi = L;
                while (lo < hi) { int m = (lo + hi) / 2; if (live[m] < v) lo = m + 1; else hi = m; }
                int idx = (int)floor(rng_random(&S->storm_rng) * (double)(L - 1));
                acc[j] = live[idx < lo ? idx : idx + 1];
            }
            for (int j = 0; j < K; j++) {
                node_t *X = &S->nodes[acc[j]];
                make_update(S, X, cand[j], X->inc[cand[j]], ST_SUSPECT);
            }
            free(acc);
        }
        free(live); free(cand);
    }

    for (int i = 0; i < S->n; i++) {
        if (S->nodes[i].dead) continue;
        ping_member_now(S, &S->nodes[i]);
    }
    run_waves(S);

    int conv = 1; uint32_t first = 0; int have = 0;
    for (int i = 0; i < S->n; i++) {
        if (S->nodes[i].dead) continue;
        uint32_t c = get_checksum(S, &S->nodes[i]);
        if (!have) { first = c; have = 1; } else if (c != first) { conv = 0; }
    }
    S->st.converged = conv;
    if (st) *st = S->st;
    S->round++;
    return 0;
}

int orc_sim_rounds_done(const orc_sim *S) { return S->round; }
uint32_t orc_sim_checksum(orc_sim *S, int v) { return get_checksum(S, &S->nodes[v]); }
int orc_sim_is_dead(const orc_sim *S, int v) { return S->nodes[v].dead; }

void orc_sim_dump_view(orc_sim *S, int v, uint8_t *status, uint64_t *inc) {
    memcpy(status, S->nodes[v].status, (size_t)S->n);
    memcpy(inc, S->nodes[v].inc, (size_t)S->n * 8);
}
int orc_sim_dump_members(orc_sim *S, int v, int32_t *out) {
    memcpy(out, S->nodes[v].members, (size_t)S->nodes[v].nmembers * 4);
    return S->nodes[v].nmembers;
}
int orc_sim_dump_changes(orc_sim *S, int v, int64_t *out) {
    node_t *X = &S->nodes[v];
    int k = 0;
    for (int a = X->d_head; a >= 0; a = X->d_next[a]) {
        int64_t *row = out + 6 * k++;
        row[0] = a; row[1] = X->d_count[a]; row[2] = X->d_source[a];
        row[3] = (int64_t)X->d_source_inc[a]; row[4] = X->d_status[a]; row[5] = (int64_t)X->d_inc[a];
    }
    return k;
}
void orc_sim_node_info(orc_sim *S, int v, int64_t *info) {
    node_t *X = &S->nodes[v];
    if (X->ring_dirty) compute_ring_checksum(S, X);
    int nt = 0;
    for (int a = 0; a < S->n; a++) if (X->timer[a] >= 0) nt++;
    info[0] = X->max_pb; info[1] = X->ring_count; info[2] = X->ring_checksum;
    info[3] = X->iter_index; info[4] = X->iter_round; info[5] = X->dead;
    info[6] = (int64_t)X->rng.s; info[7] = nt;
}
int orc_sim_dump_timers(orc_sim *S, int v, int32_t *out) {
    node_t *X = &S->nodes[v];
    int k = 0;
    for (int a = 0; a < S->n; a++) if (X->timer[a] >= 0) out[k++] = a;
    return k;
}
int orc_sim_address(const orc_sim *S, int i, char *buf, int cap) {
    int l; const char *a = addr_of(S, i, &l);
    if (l + 1 > cap) return -1;
    memcpy(buf, a, (size_t)l); buf[l] = 0;
    return l;
}

/* ---------------------------------------------- single view rules (tests) */
int orc_view_update(int self, uint64_t now, uint8_t *status, uint64_t *inc,
                    int nchanges, const int32_t *addr, uint8_t *cstatus, uint64_t *cinc,
                    uint8_t *applied) {
    int n = 0;
    for (int i = 0; i < nchanges; i++) {
        int a = addr[i];
        applied[i] = 0;
        int ap = 0;
        if (status[a] == ST_ABSENT) ap = 1;
        else if (a == self && (cstatus[i] == ST_SUSPECT || cstatus[i] == ST_FAULTY)) {
            cstatus[i] = ST_ALIVE; cinc[i] = now; ap = 1;
        } else {
            node_t X; memset(&X, 0, sizeof X);
            X.status = status; X.inc = inc;
            change_t c = {a, cstatus[i], cinc[i], -1, 0};
            ap = override_rules(&X, a, &c);
        }
        if (ap) { status[a] = cstatus[i]; inc[a] = cinc[i]; applied[i] = 1; n++; }
    }
    return n;
}

size_t orc_checksum_string(const uint8_t *addr_bytes, const uint64_t *addr_off, int naddr,
                           const uint8_t *status, const uint64_t *inc, uint8_t *out, size_t cap) {
    size_t p = 0; int first = 1;
    for (int a = 0; a < naddr; a++) {
        if (status[a] == ST_ABSENT) continue;
        size_t al = (size_t)(addr_off[a + 1] - addr_off[a]);
        if (p + al + 32 > cap) return (size_t)-1;
        if (!first) out[p++] = ';';
        first = 0;
        memcpy(out + p, addr_bytes + addr_off[a], al); p += al;
        memcpy(out + p, STATUS_STR[status[a]], (size_t)STATUS_LEN[status[a]]);
        p += (size_t)STATUS_LEN[status[a]];
        p += (size_t)u64_to_dec(inc[a], (char *)out + p);
    }
    return p;
}

uint32_t orc_view_checksum(const uint8_t *addr_bytes, const uint64_t *addr_off, int naddr,
                           const uint8_t *status, const uint64_t *inc) {
    size_t cap = (size_t)(addr_off[naddr] - addr_off[0]) + (size_t)naddr * 32 + 16;
    uint8_t *buf = (uint8_t *)xmalloc(cap);
    size_t l = orc_checksum_string(addr_bytes, addr_off, naddr, status, inc, buf, cap);
    uint32_t h = oracle_farmhash32(buf, l);
    free(buf);
    return h;
}

/* ---------------------------------------------- standalone HashRing */
typedef struct { uint32_t h; int32_t owner; } rpt_t;
struct orc_ring {
    int replicas;
    /* server names ever seen, index = first-seen order */
    char **names; int nnames, names_cap;
    uint8_t *present; int count;
    /* point map hash -> owner, kept as a sorted array (insert-if-absent,
     * erase-by-key; lib/rbtree.js semantics) */
    rpt_t *pts; size_t npts, pts_cap;
    uint32_t checksum; int checksum_dirty;
};

orc_ring *orc_ring_new(int replica_points) {
    orc_ring *r = (orc_ring *)xcalloc(1, sizeof(orc_ring));
    r->replicas = replica_points > 0 ? replica_points : 100;
    r->checksum_dirty = 1;
    return r;
}
void orc_ring_free(orc_ring *r) {
    if (!r) return;
    for (int i = 0; i < r->nnames; i++) free(r->names[i]);
    free(r->names); free(r->present); free(r->pts); free(r);
}
static int ring_name_index(orc_ring *r, const uint8_t *b, size_t l) {
    for (int i = 0; i < r->nnames; i++)
        if (strlen(r->names[i]) == l && memcmp(r->names[i], b, l) == 0) return i;
    if (r->nnames == r->names_cap) {
        r->names_cap = r->names_cap ? r->names_cap * 2 : 64;
        r->names = (char **)realloc(r->names, (size_t)r->names_cap * sizeof(char *));
        r->present = (uint8_t *)realloc(r->present, (size_t)r->names_cap);
        if (!r->names || !r->present) abort();
    }
    r->names[r->nnames] = (char *)xmalloc(l + 1);
    memcpy(r->names[r->nnames], b, l); r->names[r->nnames][l] = 0;
    r->present[r->nnames] = 0;
    return r->nnames++;
}
static size_t rpt_lb(const orc_ring *r, uint32_t h) {
    size_t lo = 0, hi = r->npts;
    while (lo < hi) { size_t m = (lo + hi) / 2; if (r->pts[m].h < h) lo = m + 1; else hi = m; }
    return lo;
}
static void rpt_insert(orc_ring *r, uint32_t h, int owner) {
    size_t p = rpt_lb(r, h);
    if (p < r->npts && r->pts[p].h == h) return;  /* duplicate: first inserter kept */
    if (r->npts == r->pts_cap) {
        r->pts_cap = r->pts_cap ? r->pts_cap * 2 : 1024;
        r->pts = (rpt_t *)realloc(r->pts, r->pts_cap * sizeof(rpt_t));
        if (!r->pts) abort();
    }
    memmove(r->pts + p + 1, r->pts + p, (r->npts - p) * sizeof(rpt_t));
    r->pts[p].h = h; r->pts[p].owner = owner; r->npts++;
}
static void rpt_erase(orc_ring *r, uint32_t h) {
    size_t p = rpt_lb(r, h);
    if (p < r->npts && r->pts[p].h == h) {
        memmove(r->pts + p, r->pts + p + 1, (r->npts - p - 1) * sizeof(rpt_t));
        r->npts--;
    }
}
static uint32_t replica_hash(const orc_ring *r, const char *name, int i) {
    char buf[512];
    size_t l = strlen(name);
    if (l > 480) l = 480;
    memcpy(buf, name, l);
    l += (size_t)u64_to_dec((uint64_t)i, buf + l);
    (void)r;
    return oracle_farmhash32((const uint8_t *)buf, l);
}
int orc_ring_add_remove(orc_ring *r, const uint8_t *add_bytes, const uint64_t *add_off, int nadd,
                        const uint32_t *add_hashes, const uint8_t *rm_bytes, const uint64_t *rm_off,
                        int nrm, const uint32_t *rm_hashes) {
    int added = 0, removed = 0;
    for (int i = 0; i < nadd; i++) {
        int s = ring_name_index(r, add_bytes + add_off[i], (size_t)(add_off[i + 1] - add_off[i]));
        if (r->present[s]) continue;
        r->present[s] = 1; r->count++;
        for (int k = 0; k < r->replicas; k++) {
            uint32_t h = add_hashes ? add_hashes[(size_t)i * r->replicas + k] : replica_hash(r, r->names[s], k);
            rpt_insert(r, h, s);
        }
        added = 1;
    }
    for (int i = 0; i < nrm; i++) {
        int s = ring_name_index(r, rm_bytes + rm_off[i], (size_t)(rm_off[i + 1] - rm_off[i]));
        if (!r->present[s]) continue;
        r->present[s] = 0; r->count--;
        for (int k = 0; k < r->replicas; k++) {
            uint32_t h = rm_hashes ? rm_hashes[(size_t)i * r->replicas + k] : replica_hash(r, r->names[s], k);
            rpt_erase(r, h);
        }
        removed = 1;
    }
    if (added || removed) r->checksum_dirty = 1;
    return added || removed;
}
int orc_ring_server_count(const orc_ring *r) { return r->count; }
static int cmp_name(const void *a, const void *b) { return strcmp(*(char *const *)a, *(char *const *)b); }
uint32_t orc_ring_checksum(orc_ring *r) {
    if (!r->checksum_dirty) return r->checksum;
    char **v = (char **)xmalloc((size_t)(r->nnames + 1) * sizeof(char *));
    int k = 0; size_t tot = 0;
    for (int i = 0; i < r->nnames; i++) if (r->present[i]) { v[k++] = r->names[i]; tot += strlen(r->names[i]) + 1; }
    qsort(v, (size_t)k, sizeof(char *), cmp_name);
    uint8_t *buf = (uint8_t *)xmalloc(tot + 1);
    size_t p = 0;
    for (int i = 0; i < k; i++) {
        if (i) buf[p++] = ';';
        size_t l = strlen(v[i]); memcpy(buf + p, v[i], l); p += l;
    }
    r->checksum = oracle_farmhash32(buf, p);
    r->checksum_dirty = 0;
    free(buf); free(v);
    return r->checksum;
}
void orc_ring_lookup_hashes(orc_ring *r, const uint32_t *h, size_t n, int32_t *owner) {
    for (size_t i = 0; i < n; i++) {
        if (r->npts == 0) { owner[i] = -1; continue; }
        size_t p = rpt_lb(r, h[i]);
        if (p == r->npts) p = 0;
        owner[i] = r->pts[p].owner;
    }
}
size_t orc_ring_points(orc_ring *r, uint32_t *hashes, int32_t *owners) {
    for (size_t i = 0; i < r->npts; i++) {
        if (hashes) hashes[i] = r->pts[i].h;
        if (owners) owners[i] = r->pts[i].owner;
    }
    return r->npts;
}
int orc_ring_server_name(const orc_ring *r, int idx, char *buf, int cap) {
    if (idx < 0 || idx >= r->nnames) return -1;
    int l = (int)strlen(r->names[idx]);
    if (l + 1 > cap) return -1;
    memcpy(buf, r->names[idx], (size_t)l + 1);
    return l;
}
int orc_ring_lookup_n(orc_ring *r, uint32_t h, int n, int32_t *out) {
    /* lib/ring.js:150-182: walk successors from the inclusive lower bound,
     * wrapping once, collecting distinct owners */
    if (n > r->count) n = r->count;
    int k = 0;
    if (r->npts == 0 || n <= 0) return 0;
    size_t start = rpt_lb(r, h);
    for (size_t j = 0; j < r->npts && k < n; j++) {
        size_t p = (start + j) % r->npts;
        int o = r->pts[p].owner, dup = 0;
        for (int q = 0; q < k; q++) if (out[q] == o) { dup = 1; break; }
        if (!dup) out[k++] = o;
    }
    return k;
}

/* ------------------------------------------------------------- wire bridge
 * Node-level ping path between rounds: rows of
 * 5 int64 = address, status, incarnation, source (-1 undefined),
 * sourceIncarnationNumber (0 undefined).  `now` = the next round's virtual
 * clock (local overrides, suspicion timers). */
static void bridge_now(orc_sim *S) { S->now = T0 + PERIOD * (uint64_t)S->round; }
static int rows_out(const clist *l, int64_t *out, int cap) {
    for (int i = 0; i < l->n && i < cap; i++) {
        int64_t *r = out + 5 * i;
        r[0] = l->v[i].addr; r[1] = l->v[i].status; r[2] = (int64_t)l->v[i].inc;
        r[3] = l->v[i].source; r[4] = (int64_t)l->v[i].source_inc;
    }
    return l->n;
}
static change_t *rows_in(const int64_t *rows, int n) {
    change_t *c = (change_t *)xmalloc((size_t)n * sizeof(change_t) + 1);
    for (int i = 0; i < n; i++) {
        const int64_t *r = rows + 5 * i;
        c[i].addr = (int32_t)r[0]; c[i].status = (int32_t)r[1]; c[i].inc = (uint64_t)r[2];
        c[i].source = (int32_t)r[3]; c[i].source_inc = (uint64_t)r[4];
    }
    return c;
}
/* PingSender.send (lib/swim/ping-sender.js:70-76): issueAsSender + the body's
 * checksum and sourceIncarnationNumber */
int orc_sim_ping_body(orc_sim *S, int v, int64_t *out, int cap, uint32_t *checksum, uint64_t *incarnation) {
    bridge_now(S);
    node_t *X = &S->nodes[v];
    clist l = {0};
    issue_as(X, -1, 0, &l);
    int k = rows_out(&l, out, cap);
    cl_free(&l);
    *checksum = get_checksum(S, X);
    *incarnation = X->inc[X->id];
    return k;
}
/* handlePing (server/ping-handler.js:22-40): update, then issueAsReceiver */
int orc_sim_handle_ping(orc_sim *S, int v, int source, uint64_t source_inc, uint32_t checksum, const int64_t *rows,
                        int n, int64_t *out, int cap, int *applied, int *full_sync) {
    bridge_now(S);
    node_t *X = &S->nodes[v];
    change_t *c = rows_in(rows, n);
    *applied = membership_update(S, X, c, n);
    free(c);
    int64_t fs0 = S->st.full_syncs;
    clist l = {0};
    issue_as_receiver(S, X, source, source_inc, checksum, &l);
    *full_sync = S->st.full_syncs != fs0;
    int k = rows_out(&l, out, cap);
    cl_free(&l);
    return k;
}
/* PingSender.onPing's Membership.update (lib/swim/ping-sender.js:36-39) */
int orc_sim_update(orc_sim *S, int v, const int64_t *rows, int n) {
    bridge_now(S);
    change_t *c = rows_in(rows, n);
    int a = membership_update(S, &S->nodes[v], c, n);
    free(c);
    return a;
}
