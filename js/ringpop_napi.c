/*
 * ringpop_hip.node — N-API addon over the C ABI in include/ringpop_hip.h.
 *
 * This is the thin binding a ringpop maintainer adds to reach the MI355X
 * path from JavaScript: `hash32` replaces the npm farmhash addon
 * (package.json:30), the ring functions back HashRing (lib/ring.js), and the
 * sim functions drive the device-resident simulation.  All work happens in
 * libringpop_hip.so; this file only converts JS values.
 */
#define NAPI_VERSION 4
#include <node_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ringpop_hip.h"

#define CHECK_NAPI(call)                                   \
    do {                                                   \
        if ((call) != napi_ok) {                           \
            napi_throw_error(env, NULL, "N-API call failed"); \
            return NULL;                                   \
        }                                                  \
    } while (0)

static napi_value throw_rp(napi_env env, int rc) {
    char code[16];
    snprintf(code, sizeof code, "%d", rc);
    napi_throw_error(env, code, rp_last_error());
    return NULL;
}
#define CHECK_RP(call)                 \
    do {                               \
        int rc_ = (call);              \
        if (rc_ != RP_OK) return throw_rp(env, rc_); \
    } while (0)

static napi_value num(napi_env env, double v) {
    napi_value r;
    napi_create_double(env, v, &r);
    return r;
}

/* string array -> (bytes, offsets) */
typedef struct { uint8_t *bytes; uint64_t *off; uint32_t n; } strbuf;
static int read_strings(napi_env env, napi_value arr, strbuf *sb) {
    uint32_t n = 0;
    bool is_arr = false;
    napi_is_array(env, arr, &is_arr);
    memset(sb, 0, sizeof *sb);
    if (!is_arr) return 0;
    napi_get_array_length(env, arr, &n);
    sb->n = n;
    sb->off = (uint64_t *)calloc(n + 1, 8);
    size_t cap = 64 + (size_t)n * 24, used = 0;
    sb->bytes = (uint8_t *)malloc(cap);
    for (uint32_t i = 0; i < n; i++) {
        napi_value e, s;
        napi_get_element(env, arr, i, &e);
        napi_coerce_to_string(env, e, &s);  /* lookup(key + '') coerces (index.js:412) */
        size_t len = 0;
        napi_get_value_string_utf8(env, s, NULL, 0, &len);
        if (used + len + 1 > cap) {
            cap = (used + len + 1) * 2;
            sb->bytes = (uint8_t *)realloc(sb->bytes, cap);
        }
        napi_get_value_string_utf8(env, s, (char *)sb->bytes + used, len + 1, &len);
        used += len;
        sb->off[i + 1] = used;
    }
    return 1;
}
static void free_strings(strbuf *sb) { free(sb->bytes); free(sb->off); }

static napi_value typed(napi_env env, napi_typedarray_type t, size_t elems, size_t esz, void **data) {
    napi_value ab, ta;
    napi_create_arraybuffer(env, elems * esz, data, &ab);
    napi_create_typedarray(env, t, elems, ab, 0, &ta);
    return ta;
}

static void *get_external(napi_env env, napi_value v) {
    void *p = NULL;
    napi_get_value_external(env, v, &p);
    return p;
}

/* ---------------------------------------------------------------- farmhash */
static napi_value js_hash32(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], s;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    CHECK_NAPI(napi_coerce_to_string(env, argv[0], &s));
    size_t len = 0;
    napi_get_value_string_utf8(env, s, NULL, 0, &len);
    char *buf = (char *)malloc(len + 1);
    napi_get_value_string_utf8(env, s, buf, len + 1, &len);
    uint32_t h = 0;
    int rc = rp_hash32((const uint8_t *)buf, len, &h);
    free(buf);
    if (rc) return throw_rp(env, rc);
    return num(env, (double)h);
}

static napi_value js_hash32_batch(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    strbuf sb;
    read_strings(env, argv[0], &sb);
    void *out;
    napi_value ta = typed(env, napi_uint32_array, sb.n, 4, &out);
    int rc = sb.n ? rp_hash32_batch(sb.bytes, sb.off, sb.n, (uint32_t *)out) : RP_OK;
    free_strings(&sb);
    if (rc) return throw_rp(env, rc);
    return ta;
}

/* ---------------------------------------------------------------- ring */
static void ring_finalize(napi_env env, void *data, void *hint) {
    (void)env; (void)hint;
    rp_ring_destroy((rp_ring *)data);
}

static napi_value js_ring_create(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], ext;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    int32_t rp = 100;
    if (argc > 0) napi_get_value_int32(env, argv[0], &rp);
    rp_ring *r = NULL;
    CHECK_RP(rp_ring_create(rp, &r));
    CHECK_NAPI(napi_create_external(env, r, ring_finalize, NULL, &ext));
    return ext;
}

/* a Uint32Array argument; *n = its length.  Anything else (or undefined)
 * gives NULL and *n = 0, so a NULL pointer never travels with a length. */
static const uint32_t *opt_u32(napi_env env, napi_value v, size_t *n) {
    bool is_ta = false;
    *n = 0;
    napi_is_typedarray(env, v, &is_ta);
    if (!is_ta) return NULL;
    napi_typedarray_type t;
    void *data;
    napi_value ab;
    size_t off, len = 0;
    napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off);
    if (t != napi_uint32_array) return NULL;
    *n = len;
    return (const uint32_t *)data;
}
static bool is_typed(napi_env env, napi_value v) {
    bool is_ta = false;
    napi_is_typedarray(env, v, &is_ta);
    return is_ta;
}

/* ringAddRemove(ring, add[], remove[], addHashes?, rmHashes?, replicaPoints) -> changed */
static napi_value js_ring_add_remove(napi_env env, napi_callback_info info) {
    size_t argc = 6;
    napi_value argv[6];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_ring *r = (rp_ring *)get_external(env, argv[0]);
    strbuf a, b;
    read_strings(env, argv[1], &a);
    read_strings(env, argv[2], &b);
    size_t na = 0, nb = 0;
    const uint32_t *ah = argc > 3 ? opt_u32(env, argv[3], &na) : NULL;
    const uint32_t *bh = argc > 4 ? opt_u32(env, argv[4], &nb) : NULL;
    /* custom replica hashes (hashFunc seam): exactly names x replicaPoints */
    int32_t R = 0;
    if (argc > 5) napi_get_value_int32(env, argv[5], &R);
    if ((argc > 3 && is_typed(env, argv[3]) && (!ah || na != (size_t)a.n * (size_t)R)) ||
        (argc > 4 && is_typed(env, argv[4]) && (!bh || nb != (size_t)b.n * (size_t)R))) {
        free_strings(&a);
        free_strings(&b);
        napi_throw_range_error(env, NULL, "replica hashes must be a Uint32Array of names.length * replicaPoints");
        return NULL;
    }
    int changed = 0;
    int rc = rp_ring_add_remove(r, a.bytes, a.off, a.n, ah, b.bytes, b.off, b.n, bh, &changed);
    free_strings(&a);
    free_strings(&b);
    if (rc) return throw_rp(env, rc);
    napi_value res;
    napi_get_boolean(env, changed != 0, &res);
    return res;
}

static napi_value js_ring_count(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    int c = 0;
    CHECK_RP(rp_ring_server_count((rp_ring *)get_external(env, argv[0]), &c));
    return num(env, c);
}

static napi_value js_ring_checksum(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint32_t c = 0;
    CHECK_RP(rp_ring_checksum((rp_ring *)get_external(env, argv[0]), &c));
    return num(env, c);
}

static napi_value js_ring_server_name(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], s;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    int32_t idx = -1;
    napi_get_value_int32(env, argv[1], &idx);
    if (idx < 0) {
        napi_get_null(env, &s);
        return s;
    }
    char buf[512];
    size_t len = 0;
    CHECK_RP(rp_ring_server_name((rp_ring *)get_external(env, argv[0]), idx, buf, sizeof buf, &len));
    napi_create_string_utf8(env, buf, len, &s);
    return s;
}

/* ringLookup(ring, keys[]) -> Int32Array of server indices (-1: empty ring) */
static napi_value js_ring_lookup(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    strbuf sb;
    read_strings(env, argv[1], &sb);
    void *out;
    napi_value ta = typed(env, napi_int32_array, sb.n, 4, &out);
    int rc = sb.n ? rp_ring_lookup_batch((rp_ring *)get_external(env, argv[0]), sb.bytes, sb.off, sb.n,
                                         (int32_t *)out)
                  : RP_OK;
    free_strings(&sb);
    if (rc) return throw_rp(env, rc);
    return ta;
}

/* ringLookupHashes(ring, Uint32Array) -> Int32Array */
static napi_value js_ring_lookup_hashes(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    size_t n = 0;
    const uint32_t *h = opt_u32(env, argv[1], &n);
    if (!h && is_typed(env, argv[1])) {
        napi_throw_type_error(env, NULL, "key hashes must be a Uint32Array");
        return NULL;
    }
    void *out;
    napi_value ta = typed(env, napi_int32_array, n, 4, &out);
    if (n) CHECK_RP(rp_ring_lookup_hashes((rp_ring *)get_external(env, argv[0]), h, n, (int32_t *)out));
    return ta;
}

/* ringGroup(ring, keys[] | Uint32Array hashes) -> [Int32Array dests, Uint32Array groupOff,
 * Uint32Array keyIndex]: handleOrProxyAll's _.groupBy(keys, lookup) (index.js:636-645) */
static napi_value js_ring_group(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], res;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_ring *ring = (rp_ring *)get_external(env, argv[0]);
    bool is_ta = false;
    napi_is_typedarray(env, argv[1], &is_ta);
    strbuf sb = {0};
    size_t n = 0;
    const uint32_t *h = NULL;
    if (is_ta) {
        h = opt_u32(env, argv[1], &n);
        if (!h) { napi_throw_type_error(env, NULL, "key hashes must be a Uint32Array"); return NULL; }
    } else {
        read_strings(env, argv[1], &sb);
        n = sb.n;
    }
    int32_t *dests = (int32_t *)calloc(n ? n : 1, 4);
    uint32_t *goff = (uint32_t *)calloc(n + 1, 4), *kidx = (uint32_t *)calloc(n ? n : 1, 4);
    size_t ng = 0;
    int rc = is_ta ? rp_ring_group_hashes(ring, h, n, dests, goff, kidx, &ng)
                   : rp_ring_group_keys(ring, sb.bytes, sb.off, n, dests, goff, kidx, &ng);
    if (!is_ta) free_strings(&sb);
    if (rc) { free(dests); free(goff); free(kidx); return throw_rp(env, rc); }
    void *d;
    napi_create_array_with_length(env, 3, &res);
    napi_value a0 = typed(env, napi_int32_array, ng, 4, &d);
    memcpy(d, dests, ng * 4);
    napi_value a1 = typed(env, napi_uint32_array, ng + 1, 4, &d);
    memcpy(d, goff, (ng + 1) * 4);
    napi_value a2 = typed(env, napi_uint32_array, n, 4, &d);
    memcpy(d, kidx, n * 4);
    napi_set_element(env, res, 0, a0);
    napi_set_element(env, res, 1, a1);
    napi_set_element(env, res, 2, a2);
    free(dests); free(goff); free(kidx);
    return res;
}

/* ringLookupN(ring, Uint32Array hashes, n) -> Array of Int32Array */
static napi_value js_ring_lookup_n(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], res;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    size_t nk = 0;
    const uint32_t *h = opt_u32(env, argv[1], &nk);
    if (!h && is_typed(env, argv[1])) {
        napi_throw_type_error(env, NULL, "key hashes must be a Uint32Array");
        return NULL;
    }
    int32_t n = 0;
    napi_get_value_int32(env, argv[2], &n);
    if (n < 0) n = 0;
    int32_t *out = (int32_t *)calloc(nk * (size_t)(n ? n : 1), 4);
    int32_t *cnt = (int32_t *)calloc(nk ? nk : 1, 4);
    int rc = nk ? rp_ring_lookup_n_hashes((rp_ring *)get_external(env, argv[0]), h, nk, n, out, cnt) : RP_OK;
    if (rc) { free(out); free(cnt); return throw_rp(env, rc); }
    napi_create_array_with_length(env, nk, &res);
    for (size_t k = 0; k < nk; k++) {
        void *d;
        napi_value ta = typed(env, napi_int32_array, (size_t)cnt[k], 4, &d);
        memcpy(d, out + k * n, (size_t)cnt[k] * 4);
        napi_set_element(env, res, (uint32_t)k, ta);
    }
    free(out);
    free(cnt);
    return res;
}

/* ---------------------------------------------------------------- sim */
static void sim_finalize(napi_env env, void *data, void *hint) {
    (void)env; (void)hint;
    rp_sim_destroy((rp_sim *)data);
}

static double get_num_prop(napi_env env, napi_value o, const char *k, double dflt) {
    bool has = false;
    napi_has_named_property(env, o, k, &has);
    if (!has) return dflt;
    napi_value v;
    double d = dflt;
    napi_get_named_property(env, o, k, &v);
    napi_get_value_double(env, v, &d);
    return d;
}

static napi_value js_sim_create(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], ext;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_sim_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.n = (uint32_t)get_num_prop(env, argv[0], "n", 64);
    cfg.seed = (uint64_t)get_num_prop(env, argv[0], "seed", 1);
    double k = get_num_prop(env, argv[0], "churnK", -1);
    cfg.churn_k = k < 0 ? (cfg.n + 99) / 100 : (uint32_t)k;
    rp_sim *s = NULL;
    CHECK_RP(rp_sim_create(&cfg, &s));
    CHECK_NAPI(napi_create_external(env, s, sim_finalize, NULL, &ext));
    return ext;
}

static napi_value stats_obj(napi_env env, const rp_round_stats *st) {
    napi_value o;
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "evaluated", num(env, (double)st->evaluated));
    napi_set_named_property(env, o, "applied", num(env, (double)st->applied));
    napi_set_named_property(env, o, "fullSyncs", num(env, (double)st->full_syncs));
    napi_set_named_property(env, o, "messages", num(env, (double)st->messages));
    napi_set_named_property(env, o, "waves", num(env, (double)st->waves));
    napi_set_named_property(env, o, "pings", num(env, (double)st->pings));
    napi_value b;
    napi_get_boolean(env, st->converged != 0, &b);
    napi_set_named_property(env, o, "converged", b);
    return o;
}

static napi_value js_sim_round(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    bool churn = true;
    if (argc > 1) napi_get_value_bool(env, argv[1], &churn);
    rp_round_stats st;
    CHECK_RP(rp_sim_round((rp_sim *)get_external(env, argv[0]), churn ? 1 : 0, &st));
    return stats_obj(env, &st);
}

static napi_value js_sim_run(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    int32_t k = 1;
    bool churn = true;
    napi_get_value_int32(env, argv[1], &k);
    if (argc > 2) napi_get_value_bool(env, argv[2], &churn);
    rp_sim *s = (rp_sim *)get_external(env, argv[0]);
    CHECK_RP(rp_sim_run(s, k, churn ? 1 : 0));
    CHECK_RP(rp_sim_sync(s));
    rp_round_stats st;
    CHECK_RP(rp_sim_totals(s, &st));
    return stats_obj(env, &st);
}

/* simRunAsync(sim, k, churn) -> Promise<stats>: the rounds run as
 * napi_async_work on a libuv worker thread, so the event loop keeps serving
 * (SURVEY §8(b)); the handle must not be used by other calls until the
 * promise settles (the JS wrapper enforces this). */
typedef struct {
    napi_async_work work;
    napi_deferred deferred;
    napi_ref sim_ref;  /* keeps the handle alive while the worker runs */
    rp_sim *sim;
    int32_t k;
    int churn;
    int rc;
    char err[512];
    rp_round_stats st;
} run_job;

static void run_execute(napi_env env, void *data) {
    (void)env;
    run_job *j = (run_job *)data;
    j->rc = rp_sim_run(j->sim, j->k, j->churn);
    if (!j->rc) j->rc = rp_sim_sync(j->sim);
    if (!j->rc) j->rc = rp_sim_totals(j->sim, &j->st);
    if (j->rc) snprintf(j->err, sizeof j->err, "%s", rp_last_error());  /* the error text is per thread */
}

static void run_complete(napi_env env, napi_status status, void *data) {
    run_job *j = (run_job *)data;
    if (status != napi_ok && !j->rc) {
        j->rc = RP_ERR_STATE;
        snprintf(j->err, sizeof j->err, "async work cancelled");
    }
    if (j->rc) {
        napi_value msg, code, e;
        char cs[16];
        snprintf(cs, sizeof cs, "%d", j->rc);
        napi_create_string_utf8(env, j->err, NAPI_AUTO_LENGTH, &msg);
        napi_create_string_utf8(env, cs, NAPI_AUTO_LENGTH, &code);
        napi_create_error(env, code, msg, &e);
        napi_reject_deferred(env, j->deferred, e);
    } else {
        napi_resolve_deferred(env, j->deferred, stats_obj(env, &j->st));
    }
    napi_delete_reference(env, j->sim_ref);
    napi_delete_async_work(env, j->work);
    free(j);
}

static napi_value js_sim_run_async(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], promise, name;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    run_job *j = (run_job *)calloc(1, sizeof *j);
    if (!j) { napi_throw_error(env, NULL, "out of memory"); return NULL; }
    bool churn = true;
    j->k = 1;
    napi_get_value_int32(env, argv[1], &j->k);
    if (argc > 2) napi_get_value_bool(env, argv[2], &churn);
    j->churn = churn ? 1 : 0;
    j->sim = (rp_sim *)get_external(env, argv[0]);
    CHECK_NAPI(napi_create_reference(env, argv[0], 1, &j->sim_ref));
    CHECK_NAPI(napi_create_promise(env, &j->deferred, &promise));
    CHECK_NAPI(napi_create_string_utf8(env, "ringpop_hip.simRunAsync", NAPI_AUTO_LENGTH, &name));
    CHECK_NAPI(napi_create_async_work(env, NULL, name, run_execute, run_complete, j, &j->work));
    CHECK_NAPI(napi_queue_async_work(env, j->work));
    return promise;
}

/* simFail(sim, node, round) -> rp_sim_fail; simPartition(sim, start, end, split) -> rp_sim_partition */
static napi_value js_sim_fail(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint32_t node = 0, round = 0;
    napi_get_value_uint32(env, argv[1], &node);
    napi_get_value_uint32(env, argv[2], &round);
    CHECK_RP(rp_sim_fail((rp_sim *)get_external(env, argv[0]), node, round));
    return NULL;
}

static napi_value js_sim_partition(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint32_t a = 0, b = 0, c = 0;
    napi_get_value_uint32(env, argv[1], &a);
    napi_get_value_uint32(env, argv[2], &b);
    napi_get_value_uint32(env, argv[3], &c);
    CHECK_RP(rp_sim_partition((rp_sim *)get_external(env, argv[0]), a, b, c));
    return NULL;
}

/* the node count of a sim handle: output buffers are sized from the
 * library's own n, never from a JavaScript argument */
static int sim_size(napi_env env, napi_value ext, rp_sim **sim, uint32_t *n) {
    *sim = (rp_sim *)get_external(env, ext);
    *n = 0;
    return *sim ? rp_sim_size(*sim, n) : RP_ERR_INVALID;
}

static napi_value js_sim_checksums(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_sim *sim;
    uint32_t n;
    CHECK_RP(sim_size(env, argv[0], &sim, &n));
    void *out;
    napi_value ta = typed(env, napi_uint32_array, (size_t)n, 4, &out);
    CHECK_RP(rp_sim_read_checksums(sim, (uint32_t *)out, n));
    return ta;
}

/* simView(sim, n, node) -> {status: Uint8Array, inc: Float64Array} */
static napi_value js_sim_view(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], o;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_sim *sim;
    uint32_t n;
    int32_t node = 0;
    CHECK_RP(sim_size(env, argv[0], &sim, &n));
    napi_get_value_int32(env, argv[2], &node);
    void *st, *incd;
    napi_value sta = typed(env, napi_uint8_array, (size_t)n, 1, &st);
    napi_value inca = typed(env, napi_float64_array, (size_t)n, 8, &incd);
    uint64_t *tmp = (uint64_t *)malloc((size_t)(n ? n : 1) * 8);
    int rc = rp_sim_read_view(sim, (uint32_t)node, (uint8_t *)st, tmp, n);
    for (uint32_t i = 0; i < n && !rc; i++) ((double *)incd)[i] = (double)tmp[i];  /* incarnations < 2^53 */
    free(tmp);
    if (rc) return throw_rp(env, rc);
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "status", sta);
    napi_set_named_property(env, o, "inc", inca);
    return o;
}

static napi_value js_sim_members(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_sim *sim;
    uint32_t n;
    int32_t node = 0;
    CHECK_RP(sim_size(env, argv[0], &sim, &n));
    napi_get_value_int32(env, argv[2], &node);
    void *out;
    napi_value ta = typed(env, napi_uint32_array, (size_t)n, 4, &out);
    uint32_t cnt = 0;
    CHECK_RP(rp_sim_read_members(sim, (uint32_t)node, (uint32_t *)out, n, &cnt));
    return ta;
}

/* simChanges(sim, node) -> Float64Array of rows of 6 */
static napi_value js_sim_changes(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    int32_t node = 0;
    napi_get_value_int32(env, argv[1], &node);
    rp_sim *s = (rp_sim *)get_external(env, argv[0]);
    uint32_t cnt = 0;
    CHECK_RP(rp_sim_read_changes(s, (uint32_t)node, NULL, 0, &cnt));
    int64_t *rows = (int64_t *)malloc((size_t)(cnt ? cnt : 1) * 6 * 8);
    int rc = rp_sim_read_changes(s, (uint32_t)node, rows, cnt, &cnt);
    if (rc) { free(rows); return throw_rp(env, rc); }
    void *out;
    napi_value ta = typed(env, napi_float64_array, (size_t)cnt * 6, 8, &out);
    for (size_t i = 0; i < (size_t)cnt * 6; i++) ((double *)out)[i] = (double)rows[i];
    free(rows);
    return ta;
}

static napi_value js_sim_info(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], o;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    int32_t node = 0;
    napi_get_value_int32(env, argv[1], &node);
    int64_t v[8];
    CHECK_RP(rp_sim_node_info((rp_sim *)get_external(env, argv[0]), (uint32_t)node, v));
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "maxPiggybackCount", num(env, (double)v[0]));
    napi_set_named_property(env, o, "ringServerCount", num(env, (double)v[1]));
    napi_set_named_property(env, o, "ringChecksum", num(env, (double)(uint32_t)v[2]));
    napi_set_named_property(env, o, "iteratorIndex", num(env, (double)v[3]));
    napi_set_named_property(env, o, "iteratorRound", num(env, (double)v[4]));
    return o;
}

static napi_value js_sim_address(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], s;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    int32_t node = 0;
    napi_get_value_int32(env, argv[1], &node);
    char buf[64];
    CHECK_RP(rp_sim_address((rp_sim *)get_external(env, argv[0]), (uint32_t)node, buf, sizeof buf));
    napi_create_string_utf8(env, buf, NAPI_AUTO_LENGTH, &s);
    return s;
}


/* ---- wire bridge: rows of 5 (address, status, incarnation, source, source
 * incarnation) as Float64Array (values < 2^53) */
static int64_t *rows_from(napi_env env, napi_value v, uint32_t *n) {
    void *data = NULL;
    size_t len = 0;
    napi_typedarray_type t;
    napi_value ab;
    size_t off;
    *n = 0;
    if (napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off) != napi_ok || t != napi_float64_array) return NULL;
    *n = (uint32_t)(len / 5);
    int64_t *r = (int64_t *)malloc((size_t)(*n ? *n : 1) * 5 * 8);
    for (size_t i = 0; i < (size_t)*n * 5; i++) r[i] = (int64_t)((double *)data)[i];
    return r;
}
static napi_value rows_to(napi_env env, const rp_change *rows, uint32_t n) {
    void *out;
    napi_value ta = typed(env, napi_float64_array, (size_t)n * 5, 8, &out);
    for (uint32_t i = 0; i < n; i++) {
        double *d = (double *)out + 5 * (size_t)i;
        d[0] = (double)rows[i].address; d[1] = (double)rows[i].status; d[2] = (double)rows[i].incarnation;
        d[3] = (double)rows[i].source; d[4] = (double)rows[i].source_incarnation;
    }
    return ta;
}

/* simPingBody(sim, n, node) -> {changes, checksum, incarnation} (PingSender.send) */
static napi_value js_sim_ping_body(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], o;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_sim *sim;
    uint32_t n;
    int32_t node = 0;
    CHECK_RP(sim_size(env, argv[0], &sim, &n));
    napi_get_value_int32(env, argv[2], &node);
    rp_change *rows = (rp_change *)malloc((size_t)(n ? n : 1) * sizeof(rp_change));
    uint32_t cnt = 0, cs = 0;
    uint64_t inc = 0;
    int rc = rp_sim_ping_body(sim, (uint32_t)node, rows, n, &cnt, &cs, &inc);
    if (rc) { free(rows); return throw_rp(env, rc); }
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "changes", rows_to(env, rows, cnt));
    napi_set_named_property(env, o, "checksum", num(env, (double)cs));
    napi_set_named_property(env, o, "incarnation", num(env, (double)inc));
    free(rows);
    return o;
}

/* simHandlePing(sim, n, node, source, sourceInc, checksum, rows) -> {changes, applied, fullSync} (handlePing) */
static napi_value js_sim_handle_ping(napi_env env, napi_callback_info info) {
    size_t argc = 7;
    napi_value argv[7], o;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_sim *sim;
    uint32_t n;
    int32_t node = 0;
    double src = -1, sinc = 0, cs = 0;
    CHECK_RP(sim_size(env, argv[0], &sim, &n));
    napi_get_value_int32(env, argv[2], &node);
    napi_get_value_double(env, argv[3], &src);
    napi_get_value_double(env, argv[4], &sinc);
    napi_get_value_double(env, argv[5], &cs);
    uint32_t k = 0;
    int64_t *in = rows_from(env, argv[6], &k);
    if (!in) { napi_throw_type_error(env, NULL, "changes must be a Float64Array of rows of 5"); return NULL; }
    rp_change *out = (rp_change *)malloc((size_t)(n ? n : 1) * sizeof(rp_change));
    uint32_t cnt = 0, applied = 0;
    int fs = 0;
    int rc = rp_sim_handle_ping(sim, (uint32_t)node, (int64_t)src, (uint64_t)sinc, (uint32_t)cs, (const rp_change *)in, k,
                                out, n, &cnt, &applied, &fs);
    free(in);
    if (rc) { free(out); return throw_rp(env, rc); }
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "changes", rows_to(env, out, cnt));
    napi_set_named_property(env, o, "applied", num(env, (double)applied));
    napi_value b;
    napi_get_boolean(env, fs != 0, &b);
    napi_set_named_property(env, o, "fullSync", b);
    free(out);
    return o;
}

/* typed array of a given element type -> data, element count (NULL otherwise) */
static void *typed_data(napi_env env, napi_value v, napi_typedarray_type want, size_t *n) {
    bool is_ta = false;
    *n = 0;
    napi_is_typedarray(env, v, &is_ta);
    if (!is_ta) return NULL;
    napi_typedarray_type t;
    void *data;
    napi_value ab;
    size_t off, len = 0;
    napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off);
    if (t != want) return NULL;
    *n = len;
    return data;
}

/* simLoadAddresses(sim, [address, ...]) -> rp_sim_load_addresses (sorted, before round 0) */
static napi_value js_sim_load_addresses(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    strbuf sb;
    if (!read_strings(env, argv[1], &sb)) { napi_throw_type_error(env, NULL, "addresses must be an array"); return NULL; }
    int rc = rp_sim_load_addresses((rp_sim *)get_external(env, argv[0]), sb.bytes, sb.off, sb.n);
    free_strings(&sb);
    if (rc) return throw_rp(env, rc);
    return NULL;
}

/* simSetViews(sim, nodeLo, Int32Array status, Float64Array incarnation): rows of n -> rp_sim_set_views */
static napi_value js_sim_set_views(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_sim *sim;
    uint32_t n, lo = 0;
    CHECK_RP(sim_size(env, argv[0], &sim, &n));
    napi_get_value_uint32(env, argv[1], &lo);
    size_t ns = 0, ni = 0;
    const int32_t *st = (const int32_t *)typed_data(env, argv[2], napi_int32_array, &ns);
    const double *inc = (const double *)typed_data(env, argv[3], napi_float64_array, &ni);
    if (!st || !inc || ns != ni || ns % n) {
        napi_throw_type_error(env, NULL, "status: Int32Array, incarnation: Float64Array, rows of n");
        return NULL;
    }
    int64_t *inc64 = (int64_t *)malloc(ni * 8 + 8);
    for (size_t i = 0; i < ni; i++) inc64[i] = (int64_t)inc[i];
    int rc = rp_sim_set_views(sim, lo, (uint32_t)(ns / n), st, inc64);
    free(inc64);
    if (rc) return throw_rp(env, rc);
    return NULL;
}

/* simJoin(sim, Uint32Array joiners, Uint32Array rounds, Int32Array seeds, seedsPer) -> rp_sim_join */
static napi_value js_sim_join(napi_env env, napi_callback_info info) {
    size_t argc = 5;
    napi_value argv[5];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    size_t nj = 0, nr = 0, nsd = 0;
    uint32_t sp = 0;
    const uint32_t *j = (const uint32_t *)typed_data(env, argv[1], napi_uint32_array, &nj);
    const uint32_t *r = (const uint32_t *)typed_data(env, argv[2], napi_uint32_array, &nr);
    const int32_t *sd = (const int32_t *)typed_data(env, argv[3], napi_int32_array, &nsd);
    napi_get_value_uint32(env, argv[4], &sp);
    if (!j || !r || !sd || nj != nr || nsd != nj * sp) {
        napi_throw_type_error(env, NULL, "joiners, rounds: Uint32Array; seeds: Int32Array of joiners x seedsPer");
        return NULL;
    }
    CHECK_RP(rp_sim_join((rp_sim *)get_external(env, argv[0]), j, r, sd, (uint32_t)nj, sp));
    return NULL;
}

/* simUpdate(sim, node, rows) -> applied (Membership.update) */
static napi_value js_sim_update(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    int32_t node = 0;
    napi_get_value_int32(env, argv[1], &node);
    uint32_t k = 0, applied = 0;
    int64_t *in = rows_from(env, argv[2], &k);
    if (!in) { napi_throw_type_error(env, NULL, "changes must be a Float64Array of rows of 5"); return NULL; }
    int rc = rp_sim_update((rp_sim *)get_external(env, argv[0]), (uint32_t)node, (const rp_change *)in, k, &applied);
    free(in);
    if (rc) return throw_rp(env, rc);
    return num(env, (double)applied);
}


/* ---------------------------------------------------------------- one instance
 * rp_node: Membership + Dissemination of one ringpop process.  Changes cross
 * as Float64Array rows of 6: address id, incarnation, source id,
 * source incarnation, status, piggybackCount (-1 = undefined; values < 2^53). */
static void node_finalize(napi_env env, void *data, void *hint) {
    (void)env; (void)hint;
    rp_node_destroy((rp_node *)data);
}

/* nodeCreate(selfAddress, rngHi, rngLo) -> external */
static napi_value js_node_create(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], s, ext;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    CHECK_NAPI(napi_coerce_to_string(env, argv[0], &s));
    size_t len = 0;
    napi_get_value_string_utf8(env, s, NULL, 0, &len);
    char *buf = (char *)malloc(len + 1);
    napi_get_value_string_utf8(env, s, buf, len + 1, &len);
    uint32_t hi = 0, lo = 0;
    if (argc > 1) napi_get_value_uint32(env, argv[1], &hi);
    if (argc > 2) napi_get_value_uint32(env, argv[2], &lo);
    rp_node *n = NULL;
    int rc = rp_node_create((const uint8_t *)buf, len, ((uint64_t)hi << 32) | lo, &n);
    free(buf);
    if (rc) return throw_rp(env, rc);
    CHECK_NAPI(napi_create_external(env, n, node_finalize, NULL, &ext));
    return ext;
}

/* nodeIntern(node, [addresses]) -> Uint32Array ids */
static napi_value js_node_intern(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    strbuf sb;
    read_strings(env, argv[1], &sb);
    void *out;
    napi_value ta = typed(env, napi_uint32_array, sb.n, 4, &out);
    int rc = sb.n ? rp_node_intern((rp_node *)get_external(env, argv[0]), sb.bytes, sb.off, sb.n, (uint32_t *)out) : RP_OK;
    free_strings(&sb);
    if (rc) return throw_rp(env, rc);
    return ta;
}

/* nodeRng(node[, hi, lo]) -> [hi, lo] of the state before any replacement */
static napi_value js_node_rng(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], res;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_node *n = (rp_node *)get_external(env, argv[0]);
    uint64_t cur = 0;
    CHECK_RP(rp_node_rng(n, &cur, NULL));
    if (argc > 2) {
        uint32_t hi = 0, lo = 0;
        napi_get_value_uint32(env, argv[1], &hi);
        napi_get_value_uint32(env, argv[2], &lo);
        uint64_t v = ((uint64_t)hi << 32) | lo;
        CHECK_RP(rp_node_rng(n, NULL, &v));
    }
    napi_create_array_with_length(env, 2, &res);
    napi_set_element(env, res, 0, num(env, (double)(uint32_t)(cur >> 32)));
    napi_set_element(env, res, 1, num(env, (double)(uint32_t)cur));
    return res;
}

static rp_member_change *mrows_from(napi_env env, napi_value v, uint32_t *n) {
    void *data = NULL;
    size_t len = 0, off;
    napi_typedarray_type t;
    napi_value ab;
    *n = 0;
    if (napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off) != napi_ok || t != napi_float64_array) return NULL;
    *n = (uint32_t)(len / 6);
    rp_member_change *r = (rp_member_change *)calloc(*n ? *n : 1, sizeof(rp_member_change));
    const double *d = (const double *)data;
    for (uint32_t i = 0; i < *n; i++) {
        r[i].address = (int64_t)d[6 * i]; r[i].incarnation = (int64_t)d[6 * i + 1];
        r[i].source = (int64_t)d[6 * i + 2]; r[i].source_incarnation = (int64_t)d[6 * i + 3];
        r[i].status = (int32_t)d[6 * i + 4]; r[i].piggyback = (int32_t)d[6 * i + 5];
    }
    return r;
}
static napi_value mrows_to(napi_env env, const rp_member_change *r, uint32_t n) {
    void *out;
    napi_value ta = typed(env, napi_float64_array, (size_t)n * 6, 8, &out);
    double *d = (double *)out;
    for (uint32_t i = 0; i < n; i++) {
        d[6 * i] = (double)r[i].address; d[6 * i + 1] = (double)r[i].incarnation;
        d[6 * i + 2] = (double)r[i].source; d[6 * i + 3] = (double)r[i].source_incarnation;
        d[6 * i + 4] = (double)r[i].status; d[6 * i + 5] = (double)r[i].piggyback;
    }
    return ta;
}
#define MROWS_ARG(i, var, n)                                                                 \
    uint32_t n = 0;                                                                          \
    rp_member_change *var = mrows_from(env, argv[i], &n);                                    \
    if (!var) { napi_throw_type_error(env, NULL, "changes must be a Float64Array of rows of 6"); return NULL; }

/* memberUpdate(node, rows, now) -> {applied: Uint8Array, rows, checksum} (Membership.update) */
static napi_value js_member_update(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], o;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    MROWS_ARG(1, rows, n)
    double now = 0;
    napi_get_value_double(env, argv[2], &now);
    void *ap;
    napi_value apa = typed(env, napi_uint8_array, n, 1, &ap);
    uint32_t na = 0, cs = 0;
    int rc = rp_membership_update((rp_node *)get_external(env, argv[0]), rows, n, (uint64_t)now, (uint8_t *)ap, &na, &cs);
    if (rc) { free(rows); return throw_rp(env, rc); }
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "applied", apa);
    napi_set_named_property(env, o, "rows", mrows_to(env, rows, n));
    napi_set_named_property(env, o, "count", num(env, na));
    napi_set_named_property(env, o, "checksum", num(env, cs));
    free(rows);
    return o;
}

/* memberSet(node, rows) -> {winners: Uint32Array, checksum} (Membership.set) */
static napi_value js_member_set(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], o;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    MROWS_ARG(1, rows, n)
    uint32_t *w = (uint32_t *)calloc(n ? n : 1, 4), nw = 0, cs = 0;
    int rc = rp_membership_set((rp_node *)get_external(env, argv[0]), rows, n, w, &nw, &cs);
    free(rows);
    if (rc) { free(w); return throw_rp(env, rc); }
    void *out;
    napi_value wa = typed(env, napi_uint32_array, nw, 4, &out);
    memcpy(out, w, (size_t)nw * 4);
    free(w);
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "winners", wa);
    napi_set_named_property(env, o, "checksum", num(env, cs));
    return o;
}

static napi_value js_member_checksum(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint32_t cs = 0;
    CHECK_RP(rp_membership_checksum((rp_node *)get_external(env, argv[0]), &cs));
    return num(env, cs);
}

static napi_value js_member_checksum_string(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], s;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_node *n = (rp_node *)get_external(env, argv[0]);
    size_t len = 0;
    CHECK_RP(rp_membership_checksum_string(n, NULL, 0, &len));
    char *buf = (char *)malloc(len + 1);
    int rc = rp_membership_checksum_string(n, buf, len + 1, &len);
    if (rc) { free(buf); return throw_rp(env, rc); }
    napi_create_string_utf8(env, buf, len, &s);
    free(buf);
    return s;
}

/* memberMembers(node) -> {ids: Uint32Array, status: Uint8Array, inc: Float64Array} */
static napi_value js_member_members(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], o;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_node *n = (rp_node *)get_external(env, argv[0]);
    uint32_t cnt = 0;
    CHECK_RP(rp_membership_members(n, NULL, NULL, NULL, 0, &cnt));
    void *ids, *st, *incd;
    napi_value a = typed(env, napi_uint32_array, cnt, 4, &ids);
    napi_value b = typed(env, napi_uint8_array, cnt, 1, &st);
    napi_value c = typed(env, napi_float64_array, cnt, 8, &incd);
    uint64_t *tmp = (uint64_t *)malloc((size_t)(cnt ? cnt : 1) * 8);
    int rc = cnt ? rp_membership_members(n, (uint32_t *)ids, (uint8_t *)st, tmp, cnt, &cnt) : RP_OK;
    for (uint32_t i = 0; i < cnt && !rc; i++) ((double *)incd)[i] = (double)tmp[i];
    free(tmp);
    if (rc) return throw_rp(env, rc);
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "ids", a);
    napi_set_named_property(env, o, "status", b);
    napi_set_named_property(env, o, "inc", c);
    return o;
}

static napi_value js_member_shuffle(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    CHECK_RP(rp_membership_shuffle((rp_node *)get_external(env, argv[0])));
    return NULL;
}

/* memberSetOrder(node, Uint32Array ids): the member order replaced by a
 * permutation of it (getStats' in-place sort, lib/membership.js:122-129) */
static napi_value js_member_set_order(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    size_t n = 0;
    const uint32_t *ids = argc > 1 ? opt_u32(env, argv[1], &n) : NULL;
    napi_typedarray_type t = napi_int8_array;
    if (argc > 1 && is_typed(env, argv[1])) {
        void *data;
        napi_value ab;
        size_t len, off;
        napi_get_typedarray_info(env, argv[1], &t, &len, &data, &ab, &off);
    }
    if (t != napi_uint32_array) {
        napi_throw_type_error(env, NULL, "member ids must be a Uint32Array");
        return NULL;
    }
    CHECK_RP(rp_membership_set_order((rp_node *)get_external(env, argv[0]), ids, (uint32_t)n));
    return NULL;
}

/* memberRandom(node, k) -> Float64Array of k Math.random() draws */
static napi_value js_member_random(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint32_t k = 0;
    napi_get_value_uint32(env, argv[1], &k);
    void *out;
    napi_value ta = typed(env, napi_float64_array, k, 8, &out);
    if (k) CHECK_RP(rp_membership_random((rp_node *)get_external(env, argv[0]), k, (double *)out));
    return ta;
}

static napi_value js_member_force(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint32_t id = 0;
    int32_t st = 0;
    double inc = 0;
    napi_get_value_uint32(env, argv[1], &id);
    napi_get_value_int32(env, argv[2], &st);
    napi_get_value_double(env, argv[3], &inc);
    CHECK_RP(rp_membership_force((rp_node *)get_external(env, argv[0]), id, st, (uint64_t)inc));
    return NULL;
}

/* dissRecord(node, rows): Dissemination.recordChange for a batch */
static napi_value js_diss_record(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    MROWS_ARG(1, rows, n)
    int rc = rp_dissemination_record((rp_node *)get_external(env, argv[0]), rows, n);
    free(rows);
    if (rc) return throw_rp(env, rc);
    return NULL;
}

static uint32_t diss_cap(rp_node *n) {
    uint32_t live = 0, mem = 0;
    rp_dissemination_changes(n, NULL, 0, &live);
    rp_membership_members(n, NULL, NULL, NULL, 0, &mem);
    return (live > mem ? live : mem) + 1;
}

/* dissIssue(node, maxPiggybackCount) -> rows (issueAsSender) */
static napi_value js_diss_issue(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_node *n = (rp_node *)get_external(env, argv[0]);
    int32_t maxpb = 1;
    napi_get_value_int32(env, argv[1], &maxpb);
    uint32_t cap = diss_cap(n), cnt = 0;
    rp_member_change *out = (rp_member_change *)calloc(cap, sizeof(rp_member_change));
    int rc = rp_dissemination_issue(n, maxpb, out, cap, &cnt);
    if (rc) { free(out); return throw_rp(env, rc); }
    napi_value r = mrows_to(env, out, cnt);
    free(out);
    return r;
}

/* dissIssueReceiver(node, senderId, senderInc, checksum|undefined, maxPiggybackCount)
 * -> {rows, fullSync} (issueAsReceiver) */
static napi_value js_diss_issue_receiver(napi_env env, napi_callback_info info) {
    size_t argc = 5;
    napi_value argv[5], o;
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_node *n = (rp_node *)get_external(env, argv[0]);
    double src = -1, sinc = -1, cs = 0;
    int32_t maxpb = 1;
    napi_get_value_double(env, argv[1], &src);
    napi_get_value_double(env, argv[2], &sinc);
    napi_valuetype t;
    napi_typeof(env, argv[3], &t);
    int has = t == napi_number;
    if (has) napi_get_value_double(env, argv[3], &cs);
    napi_get_value_int32(env, argv[4], &maxpb);
    uint32_t cap = diss_cap(n), cnt = 0;
    int fs = 0;
    rp_member_change *out = (rp_member_change *)calloc(cap, sizeof(rp_member_change));
    int rc = rp_dissemination_issue_as_receiver(n, (int64_t)src, (int64_t)sinc, (uint32_t)cs, has, maxpb, out, cap, &cnt, &fs);
    if (rc) { free(out); return throw_rp(env, rc); }
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "rows", mrows_to(env, out, cnt));
    napi_value b;
    napi_get_boolean(env, fs != 0, &b);
    napi_set_named_property(env, o, "fullSync", b);
    free(out);
    return o;
}

static napi_value js_diss_full_sync(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_node *n = (rp_node *)get_external(env, argv[0]);
    uint32_t cap = diss_cap(n), cnt = 0;
    rp_member_change *out = (rp_member_change *)calloc(cap, sizeof(rp_member_change));
    int rc = rp_dissemination_full_sync(n, out, cap, &cnt);
    if (rc) { free(out); return throw_rp(env, rc); }
    napi_value r = mrows_to(env, out, cnt);
    free(out);
    return r;
}

static napi_value js_diss_clear(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    CHECK_RP(rp_dissemination_clear((rp_node *)get_external(env, argv[0])));
    return NULL;
}

static napi_value js_diss_changes(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    CHECK_NAPI(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    rp_node *n = (rp_node *)get_external(env, argv[0]);
    uint32_t cnt = 0;
    CHECK_RP(rp_dissemination_changes(n, NULL, 0, &cnt));
    rp_member_change *out = (rp_member_change *)calloc(cnt ? cnt : 1, sizeof(rp_member_change));
    int rc = cnt ? rp_dissemination_changes(n, out, cnt, &cnt) : RP_OK;
    if (rc) { free(out); return throw_rp(env, rc); }
    napi_value r = mrows_to(env, out, cnt);
    free(out);
    return r;
}

#define EXPORT(name, fn)                                              \
    do {                                                              \
        napi_value f_;                                                \
        napi_create_function(env, name, NAPI_AUTO_LENGTH, fn, NULL, &f_); \
        napi_set_named_property(env, exports, name, f_);              \
    } while (0)

static napi_value init(napi_env env, napi_value exports) {
    EXPORT("hash32", js_hash32);
    EXPORT("hash32Batch", js_hash32_batch);
    EXPORT("ringCreate", js_ring_create);
    EXPORT("ringAddRemove", js_ring_add_remove);
    EXPORT("ringServerCount", js_ring_count);
    EXPORT("ringChecksum", js_ring_checksum);
    EXPORT("ringServerName", js_ring_server_name);
    EXPORT("ringLookup", js_ring_lookup);
    EXPORT("ringLookupHashes", js_ring_lookup_hashes);
    EXPORT("ringLookupN", js_ring_lookup_n);
    EXPORT("ringGroup", js_ring_group);
    EXPORT("simCreate", js_sim_create);
    EXPORT("simRound", js_sim_round);
    EXPORT("simRun", js_sim_run);
    EXPORT("simRunAsync", js_sim_run_async);
    EXPORT("simLoadAddresses", js_sim_load_addresses);
    EXPORT("simSetViews", js_sim_set_views);
    EXPORT("simJoin", js_sim_join);
    EXPORT("simFail", js_sim_fail);
    EXPORT("simPartition", js_sim_partition);
    EXPORT("simChecksums", js_sim_checksums);
    EXPORT("simView", js_sim_view);
    EXPORT("simMembers", js_sim_members);
    EXPORT("simChanges", js_sim_changes);
    EXPORT("simInfo", js_sim_info);
    EXPORT("simAddress", js_sim_address);
    EXPORT("simPingBody", js_sim_ping_body);
    EXPORT("simHandlePing", js_sim_handle_ping);
    EXPORT("simUpdate", js_sim_update);
    EXPORT("nodeCreate", js_node_create);
    EXPORT("nodeIntern", js_node_intern);
    EXPORT("nodeRng", js_node_rng);
    EXPORT("memberUpdate", js_member_update);
    EXPORT("memberSet", js_member_set);
    EXPORT("memberChecksum", js_member_checksum);
    EXPORT("memberChecksumString", js_member_checksum_string);
    EXPORT("memberMembers", js_member_members);
    EXPORT("memberShuffle", js_member_shuffle);
    EXPORT("memberSetOrder", js_member_set_order);
    EXPORT("memberRandom", js_member_random);
    EXPORT("memberForce", js_member_force);
    EXPORT("dissRecord", js_diss_record);
    EXPORT("dissIssue", js_diss_issue);
    EXPORT("dissIssueReceiver", js_diss_issue_receiver);
    EXPORT("dissFullSync", js_diss_full_sync);
    EXPORT("dissClear", js_diss_clear);
    EXPORT("dissChanges", js_diss_changes);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
