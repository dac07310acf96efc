// TEST INFRASTRUCTURE ONLY (oracle harness; runs here under Node, never on
// the GPU box).  Drives the UNMODIFIED reference ringpop modules from
// /root/reference (index.js RingPop, lib/*, lib/swim/*, server/index.js
// endpoint wiring) as N in-process instances over a build-owned synchronous
// transport, under the simulation semantics defined in DESIGN.md:
//
//   round r, virtual now = T0 + 200 r:
//     0a. fail-stop nodes scheduled for round r
//     0b. fire due suspicion timers, (due, creation) order, in their node's context
//     0c. churn: k seeded live nodes call membership.makeAlive(self, now)
//     0d. storm (config 5): seeded live accusers call makeSuspect(victim, inc)
//     1.  every live node, in id order, runs RingPop.pingMemberNow() (index.js:458)
//     2+. message waves: every request/response queued while a wave is
//         delivered goes to the next wave; a wave is delivered in queue order.
//         Requests to dead nodes (or across an injected partition) come back
//         as transport errors one wave later.
//
// The driven code is the reference's own: pingMemberNow, ping-sender,
// ping-req-sender, server/ping-handler, server/ping-req-handler, Membership,
// Dissemination, HashRing, listeners, Suspicion, MembershipIterator.
// Only npm dependencies are shimmed (oracle/harness/shims, NODE_PATH).
'use strict';

var path = require('path');
var common = require('./common.js');
var REF = process.env.RINGPOP_REFERENCE || '/root/reference';

var STATUS_CODE = { alive: 1, suspect: 2, faulty: 3, leave: 4 };

function runSim(cfg) {
    var RingPop = require(path.join(REF, 'index.js'));
    var createServer = require(path.join(REF, 'server/index.js'));
    var handleJoin = require(path.join(REF, 'server/join-handler.js'));
    var mergeJoinResponses = require(path.join(REF, 'lib/swim/join-response-merge.js'));
    var uuid = require('node-uuid');
    uuid._reset();

    var n = cfg.n;
    // cfg.addresses: the cluster's addresses in sort order (default: the sim
    // scheme); cfg.views[i][j] = [status code, incarnation] of j in node i's
    // bootstrap view (default: everyone alive at INC0 + j)
    var addr = cfg.addresses || common.simAddresses(n);
    var STATUS_NAME = [null, 'alive', 'suspect', 'faulty', 'leave'];
    var idOf = {};
    addr.forEach(function (a, i) { idOf[a] = i; });
    var seed = cfg.seed;
    var rngs = [];
    for (var i = 0; i < n; i++) rngs.push(common.nodeRng(seed, i));
    var crng = common.churnRng(seed);
    var srng = common.stormRng(seed);
    var ctx = { node: -1, now: 0 };
    var timers = new common.TimerQueue();

    var saved = { now: Date.now, random: Math.random, st: global.setTimeout, ct: global.clearTimeout };
    Date.now = function () { return ctx.now; };
    Math.random = function () {
        if (ctx.node < 0) throw new Error('Math.random outside a node context');
        return rngs[ctx.node].random();
    };
    global.setTimeout = function (fn, ms) { return timers.add(ctx.now + ms, ctx.node, fn); };
    global.clearTimeout = function (t) { if (t && typeof t === 'object' && 'cancelled' in t) t.cancelled = true; };

    var dead = new Array(n).fill(false);
    // cfg.joins: [[round, joiner, [seeds]], ...] (join path): the joiners stay
    // outside the cluster until their round; the others bootstrap with each other
    var joinsAt = {}, joined = new Array(n).fill(true);
    (cfg.joins || []).forEach(function (e) {
        (joinsAt[e[0]] = joinsAt[e[0]] || []).push(e);
        joined[e[1]] = false;
    });
    var next = [];
    var handlers = [];
    var stats = { evaluated: 0, applied: 0, fullSyncs: 0, messages: 0 };

    function enqueue(m) { next.push(m); stats.messages++; }

    var rps = [];
    var tBoot = saved.now();
    try {
        for (i = 0; i < n; i++) {
            (function (me) {
                handlers.push({});
                var channel = {
                    waitForIdentified: function (opts, cb) { cb(); },
                    request: function (opts) {
                        return {
                            send: function (endpoint, head, body, cb) {
                                enqueue({ type: 'req', from: me, to: idOf[opts.host], endpoint: endpoint,
                                          head: head, body: body, cb: cb });
                            }
                        };
                    }
                };
                var tchannel = { register: function (url, h) { handlers[me][url] = h; } };
                ctx.node = me;
                ctx.now = common.INC0 + me;
                var rp = new RingPop({ app: 'sim', hostPort: addr[me], channel: channel });
                // Logging-only subsystem (lib/membership-update-rollup.js), out of scope.
                rp.membershipUpdateRollup = { trackUpdates: function () {}, destroy: function () {} };
                createServer(rp, tchannel);

                // Bootstrap as index.js:200-292 does, with a full-membership join result
                // (joiners: later, through the join path below).
                if (joined[me]) {
                    var row = cfg.views ? cfg.views[me] : null;
                    rp.membership.makeAlive(addr[me], row ? row[me][1] : common.INC0 + me);
                    var stash = [];
                    for (var j = 0; j < n; j++) {
                        if (row ? row[j][0] === 0 : !joined[j]) continue;  // not in the join result
                        stash.push(row ? { address: addr[j], status: STATUS_NAME[row[j][0]], incarnationNumber: row[j][1] }
                                       : { address: addr[j], status: 'alive', incarnationNumber: common.INC0 + j });
                    }
                    rp.membership.stashedUpdates = [stash];
                    rp.membership.set();
                    rp.membership.shuffle();            // lib/swim/gossip.js:85 (gossip.start)
                    rp.isReady = true;
                    rp.dissemination.clearChanges();    // config: dissemination cleared after set()
                }

                var upd = rp.membership.update;
                rp.membership.update = function (changes, isLocal) {
                    var c = Array.isArray(changes) ? changes.length : 1;
                    var res = upd.apply(this, arguments);
                    stats.evaluated += c;
                    stats.applied += res.length;
                    return res;
                };
                var fs = rp.dissemination.fullSync;
                rp.dissemination.fullSync = function () { stats.fullSyncs++; return fs.apply(this, arguments); };
                rps.push(rp);
            })(i);
        }

        // Partition injection: during rounds [start, end) requests between ids
        // on different sides of `split` fail like requests to a dead node.
        var part = cfg.partition || null;
        var curRound = 0;
        function cut(a, b) {
            return !!part && curRound >= part.start && curRound < part.end &&
                ((a < part.split) !== (b < part.split));
        }

        function deliver(m) {
            if (m.type === 'req') {
                if (dead[m.to] || cut(m.from, m.to)) {
                    enqueue({ type: 'resp', to: m.from, cb: m.cb, err: new Error('request timed out') });
                    return;
                }
                ctx.node = m.to;
                var res = {
                    headers: {},
                    sendOk: function (r1, r2) { enqueue({ type: 'resp', to: m.from, cb: m.cb, err: null, ok: true, r1: r1, r2: r2 }); },
                    sendNotOk: function (r1, r2) { enqueue({ type: 'resp', to: m.from, cb: m.cb, err: null, ok: false, r1: r1, r2: r2 }); }
                };
                handlers[m.to][m.endpoint]({ remoteAddr: addr[m.from] }, res, m.head, m.body);
            } else {
                ctx.node = m.to;
                if (m.err) m.cb(m.err);
                else m.cb(null, { ok: m.ok }, m.r1, m.r2);
            }
        }

        var rounds = [];
        var convergedAt = -1;
        // optional wall-clock timing of rounds >= cfg.timeFrom (CPU baseline:
        // the reference's own code path, oracle/time_reference.py)
        var timing = cfg.timeFrom === undefined ? undefined :
            { bootstrapSeconds: 0, seconds: 0, evaluated: 0, applied: 0, rounds: 0 };
        var wall = saved.now;
        var failAt = cfg.failures || {};   // {round: [ids]}
        var churnK = cfg.churnK === undefined ? Math.ceil(0.01 * n) : cfg.churnK;
        var dumpRounds = cfg.dumpRounds || [];
        var dumps = {};
        if (timing) timing.bootstrapSeconds = (wall() - tBoot) / 1000;
        for (var r = 0; r < cfg.maxRounds; r++) {
            var tRound = wall();
            ctx.now = common.T0 + common.PERIOD * r;
            curRound = r;
            stats.evaluated = 0; stats.applied = 0; stats.fullSyncs = 0; stats.messages = 0;
            (failAt[r] || []).forEach(function (v) { dead[v] = true; });

            var due = timers.due(ctx.now);
            for (var t = 0; t < due.length; t++) {
                if (dead[due[t].node]) continue;
                ctx.node = due[t].node;
                due[t].fn();
            }

            // 0b'. joins (join path): the joiner's makeAlive(self) (index.js:235),
            // each seed's handleJoin (server/join-handler.js:76-98: makeAlive +
            // fullSync reply), mergeJoinResponses (lib/swim/join-response-merge.js),
            // update() while not ready (stashed), set(), gossip.start's shuffle
            (joinsAt[r] || []).forEach(function (e) {
                var jn = e[1], rpj = rps[jn];
                if (dead[jn]) return;  // a node that fail-stopped before its round never joins
                ctx.node = jn;
                rpj.membership.makeAlive(addr[jn], ctx.now);
                var jinc = rpj.membership.localMember.incarnationNumber;
                var responses = e[2].map(function (sd) {
                    if (dead[sd] || !joined[sd]) throw new Error('join seed ' + sd + ' is not a live member');
                    ctx.node = sd;
                    var body = null;
                    handleJoin({ ringpop: rps[sd], source: addr[jn], incarnationNumber: jinc, app: 'sim' },
                               function (err, res) { if (err) throw err; body = res; });
                    // (as join-sender.js:437-440 reads the reply off the wire)
                    return JSON.parse(JSON.stringify({ checksum: body.membershipChecksum, members: body.membership }));
                });
                ctx.node = jn;
                rpj.membership.update(mergeJoinResponses(rpj, responses));
                rpj.membership.set();
                rpj.membership.shuffle();
                rpj.isReady = true;
                joined[jn] = true;
            });

            var live = [];
            for (i = 0; i < n; i++) if (!dead[i] && joined[i]) live.push(i);
            var churned = [];
            if (r < cfg.churnRounds) {
                churned = common.chooseChurn(crng, live, churnK);
                churned.forEach(function (v) {
                    ctx.node = v;
                    rps[v].membership.makeAlive(addr[v], ctx.now);
                });
            }
            // 0d. false-suspicion storm: accuser.makeSuspect(victim, its incarnation of the victim)
            var storm = cfg.storm;
            if (storm && r >= storm.start && r < storm.end) {
                common.chooseStorm(srng, live, storm.ppm).forEach(function (p) {
                    ctx.node = p[0];
                    var mem = rps[p[0]].membership;
                    mem.makeSuspect(addr[p[1]], mem.findMemberByAddress(addr[p[1]]).incarnationNumber);
                });
            }

            for (i = 0; i < n; i++) {
                if (dead[i] || !joined[i]) continue;
                ctx.node = i;
                rps[i].pingMemberNow();
            }
            var waves = 0;
            while (next.length) {
                var wave = next; next = [];
                for (var w = 0; w < wave.length; w++) deliver(wave[w]);
                waves++;
            }
            ctx.node = -1;

            if (timing && r >= cfg.timeFrom) {
                timing.seconds += (wall() - tRound) / 1000;
                timing.evaluated += stats.evaluated; timing.applied += stats.applied; timing.rounds++;
            }
            var sums = rps.map(function (rp, v) { return dead[v] || !joined[v] ? null : rp.membership.checksum; });
            var liveSums = sums.filter(function (s) { return s !== null; });
            var converged = liveSums.every(function (s) { return s === liveSums[0]; });
            rounds.push({ round: r, churned: churned, checksums: sums, evaluated: stats.evaluated,
                          applied: stats.applied, fullSyncs: stats.fullSyncs, messages: stats.messages,
                          waves: waves, converged: converged });
            if (dumpRounds.indexOf(r) >= 0) dumps[r] = dumpAll();
            if (converged && r >= cfg.churnRounds && convergedAt < 0) {
                convergedAt = r;
                if (cfg.stopAtConvergence) break;
            }
        }
        var bridge = cfg.bridge ? runBridge(cfg.bridge, common.T0 + common.PERIOD * rounds.length) : undefined;
        return { config: cfg, addresses: addr, rounds: rounds, convergedAt: convergedAt, dumps: dumps,
                 final: cfg.noFinal ? undefined : dumpAll(), bridge: bridge, timing: timing };
    } finally {
        Date.now = saved.now; Math.random = saved.random;
        global.setTimeout = saved.st; global.clearTimeout = saved.ct;
    }

    function dumpNode(rp, v) {
        var m = rp.membership;
        var view = new Array(n).fill(null);
        m.members.forEach(function (mem) { view[idOf[mem.address]] = [STATUS_CODE[mem.status], mem.incarnationNumber]; });
        var d = rp.dissemination;
        var keys = Object.keys(d.changes).map(function (a) {
            var c = d.changes[a];
            return [idOf[a], c.piggybackCount === undefined ? -1 : c.piggybackCount,
                    c.source === undefined ? -1 : idOf[c.source],
                    c.sourceIncarnationNumber === undefined ? 0 : c.sourceIncarnationNumber,
                    STATUS_CODE[c.status], c.incarnationNumber];
        });
        var suspects = Object.keys(rp.suspicion.timers).map(function (a) { return idOf[a]; });
        return {
            dead: dead[v], checksum: m.checksum, members: m.members.map(function (x) { return idOf[x.address]; }),
            view: view, changes: keys, maxPiggyback: d.maxPiggybackCount,
            ringServers: rp.ring.getServerCount(), ringChecksum: rp.ring.checksum,
            iterIndex: rp.memberIterator.currentIndex, iterRound: rp.memberIterator.currentRound,
            timers: suspects, rng: rngs[v].s.toString()
        };
    }
    function dumpAll() { return rps.map(dumpNode); }

    // Wire-format bridge fixture (DESIGN.md §8(f) 2): after the rounds, the
    // reference's own ping path between two instances with the JSON bodies
    // as they go over the wire -- PingSender.send's body (lib/swim/
    // ping-sender.js:70-76), the /protocol/ping handler's response
    // (server/index.js:175-192, server/ping-handler.js:22-40) and
    // PingSender.onPing's membership.update (ping-sender.js:36-39) -- or a
    // foreign body injected into a handler.
    function runBridge(ops, now) {
        ctx.now = now;
        return ops.map(function (op) {
            var body, resp = null;
            if (op.op === 'ping') {
                ctx.node = op.from;
                var a = rps[op.from];
                body = JSON.stringify({
                    checksum: a.membership.checksum,
                    changes: a.dissemination.issueAsSender(),
                    source: a.whoami(),
                    sourceIncarnationNumber: a.membership.getIncarnationNumber()
                });
            } else {
                body = JSON.stringify(op.body);
            }
            ctx.node = op.to;
            var res = { headers: {}, sendOk: function (r1, r2) { resp = r2; }, sendNotOk: function (r1, r2) { resp = null; } };
            handlers[op.to]['/protocol/ping']({ remoteAddr: op.op === 'ping' ? addr[op.from] : '0.0.0.0:0' }, res, null, body);
            var out = { op: op, body: JSON.parse(body), response: resp === null ? null : JSON.parse(resp) };
            if (op.op === 'ping') {
                ctx.node = op.from;
                // (a fresh parse: the instance records the objects it applies
                // and later issues mutate them; the fixture keeps the wire body)
                out.applied = rps[op.from].membership.update(JSON.parse(resp).changes).length;
                out.fromDump = dumpNode(rps[op.from], op.from);
            }
            out.toDump = dumpNode(rps[op.to], op.to);
            ctx.node = -1;
            return out;
        });
    }
}

module.exports = { runSim: runSim, STATUS_CODE: STATUS_CODE };

if (require.main === module) {
    var cfg = JSON.parse(process.argv[2]);
    var res = runSim(cfg);
    process.stdout.write(JSON.stringify(res));
}
