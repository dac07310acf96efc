// TEST INFRASTRUCTURE ONLY.  Generates the committed golden fixtures in
// tests/golden/ by running the UNMODIFIED reference modules from
// /root/reference under the build-owned harness (shims on NODE_PATH).
//
//   NODE_PATH=oracle/harness/shims node oracle/harness/gen_golden.js tests/golden
//
// farmhash values inside the fixtures come from the harness's farmhash
// restatement (the npm addon is absent): they pin everything AROUND the hash
// (string construction, ordering, collision history, protocol), while the
// hash function itself is only partially pinned (see oracle/farmhash32.c).
'use strict';

var fs = require('fs');
var path = require('path');
var zlib = require('zlib');
var REF = process.env.RINGPOP_REFERENCE || '/root/reference';
var sim = require('./sim.js');
var common = require('./common.js');
var farmhash = require('farmhash');

var outDir = process.argv[2] || 'tests/golden';
var only = process.argv[3] || '';
fs.mkdirSync(outDir, { recursive: true });

function write(name, obj) {
    var p = path.join(outDir, name);
    var s = JSON.stringify(obj);
    if (name.endsWith('.gz')) fs.writeFileSync(p, zlib.gzipSync(Buffer.from(s), { level: 9 }));
    else fs.writeFileSync(p, s);
    console.log('wrote', p, fs.statSync(p).size, 'bytes');
}

function want(name) { return !only || only.split(',').indexOf(name) >= 0; }

// ---------------------------------------------------------------- farmhash
if (want('farmhash')) {
    var strs = [''];
    var s = '';
    for (var i = 0; i < 200; i++) { s += String.fromCharCode(32 + ((i * 37) % 95)); strs.push(s); }
    strs.push('10.28.5.35:2080099', '127.0.0.1:3000', '127.0.0.1:30000', 'localhost:3000alive1414142122274');
    write('farmhash_vectors.json', { note: 'harness farmhash restatement (JS); cross-check of the C/HIP transcriptions',
        strings: strs, hash32: strs.map(function (x) { return farmhash.hash32(x); }) });
}

// ---------------------------------------------------------------- rules
function freshRingpop(hostPort) {
    var RingPop = require(path.join(REF, 'index.js'));
    var rp = new RingPop({ app: 'golden', hostPort: hostPort || '127.0.0.1:3000' });
    rp.membershipUpdateRollup = { trackUpdates: function () {}, destroy: function () {} };
    return rp;
}

function withDeterminism(seed, fn) {
    var saved = { now: Date.now, random: Math.random };
    var rng = new common.Rng(BigInt(seed));
    var now = 1500000000000;
    Date.now = function () { return now; };
    Math.random = function () { return rng.random(); };
    try { return fn(); } finally { Date.now = saved.now; Math.random = saved.random; }
}

if (want('rules')) {
    // Every (current status) x (change status) x (inc relation) x (self/other),
    // evaluated by the reference Membership.update (lib/membership.js:208-313).
    var STAT = ['alive', 'suspect', 'faulty', 'leave'];
    var cases = [];
    withDeterminism(1, function () {
        STAT.forEach(function (cur) {
            STAT.forEach(function (chg) {
                [-1, 0, 1].forEach(function (rel) {
                    [false, true].forEach(function (isSelf) {
                        var rp = freshRingpop('127.0.0.1:3000');
                        rp.isReady = true;
                        rp.membership.makeAlive(rp.whoami(), 1000);
                        var target = isSelf ? rp.whoami() : '127.0.0.1:3001';
                        if (!isSelf) rp.membership.makeAlive(target, 1000);
                        var m = rp.membership.findMemberByAddress(target);
                        m.status = cur; m.incarnationNumber = 1000;  // force the current state
                        var applied = rp.membership.update([{ address: target, status: chg,
                            incarnationNumber: 1000 + rel, source: '127.0.0.1:3009', sourceIncarnationNumber: 7 }]);
                        cases.push({ current: cur, change: chg, rel: rel, self: isSelf,
                            applied: applied.length, status: m.status, inc: m.incarnationNumber });
                        rp.destroy();
                    });
                });
            });
        });
    });
    write('rules_truth_table.json', { now: 1500000000000, cases: cases });
}

// ---------------------------------------------------------------- config 1
if (want('config1')) {
    var large = require(path.join(REF, 'benchmarks/large-membership.json'));
    var res = {};
    [100, 1000, 1332].forEach(function (size) {
        withDeterminism(42 + size, function () {
            var rp = freshRingpop('127.0.0.1:3000');
            rp.isReady = true;   // benchmarks/*.js forget this (SURVEY.md §0.4)
            var applied = rp.membership.update(JSON.parse(JSON.stringify(large.slice(0, size))));
            var str = rp.membership.generateChecksumString();
            res[size] = {
                applied: applied.length,
                members_order: rp.membership.members.map(function (m) { return m.address; }),
                checksum_string_len: Buffer.byteLength(str),
                checksum_string_sha: require('crypto').createHash('sha256').update(str).digest('hex'),
                checksum: rp.membership.checksum,
                ring_servers: rp.ring.getServerCount(),
                ring_checksum: rp.ring.checksum,
                max_piggyback: rp.dissemination.maxPiggybackCount,
                changes: Object.keys(rp.dissemination.changes)
            };
            rp.destroy();
        });
    });
    write('config1_large_membership.json', { seed_base: 42, results: res });
}

// ---------------------------------------------------------------- node ops
// One ringpop instance driven through Membership / Dissemination / HashRing
// by a seeded random operation sequence (the drop-in surface, SURVEY.md
// §8(b)): update batches with unknown members (getJoinPosition splices),
// duplicates inside a batch, self suspects (local override), rule ties;
// makeSuspect / makeFaulty; issueAsSender; issueAsReceiver with matching and
// mismatching senders and checksums (filter, fullSync fallback); shuffle;
// clearChanges.  The reference's own listeners feed the ring and the
// dissemination table.  After every op: its result and the instance state.
if (want('node_ops') || want('node_stats')) {
    var STATUSES = ['alive', 'suspect', 'faulty', 'leave'];
    // stats: also getStats() (lib/membership.js:122-129, an in-place sort by
    // localeCompare) between ops, over addresses whose localeCompare order
    // differs from their byte order ('10.0.0.1:3000' vs '10.0.0.11:3002')
    var nodeOpsFn = nodeOps;  // (node_stats below)
    function nodeOps(seed, nops, stats) {
        var g = new common.Rng(BigInt(seed) * 7919n + 13n);
        function ri(n) { return Number(g.next64() % BigInt(n)); }
        var self = '10.0.0.1:3001';
        var rp = freshRingpop(self);
        rp.isReady = true;
        var addrs = [];
        for (var i = 0; i < 24; i++) {
            if (stats) addrs.push('10.0.0.' + (1 + 5 * i) + ':' + (3000 + (i % 5)));
            else addrs.push('10.0.' + (i >> 3) + '.' + (i & 7) + ':' + (3000 + (i % 5)));
        }
        var ops = [];
        var nextId = 0;
        function snapshot() {
            var d = rp.dissemination;
            return {
                checksum: rp.membership.checksum,
                members: rp.membership.members.map(function (m) { return [m.address, m.status, m.incarnationNumber]; }),
                changes: Object.keys(d.changes).map(function (a) {
                    var c = d.changes[a];
                    return [a, c.status, c.incarnationNumber, c.source === undefined ? null : c.source,
                            c.sourceIncarnationNumber === undefined ? null : c.sourceIncarnationNumber,
                            c.piggybackCount === undefined ? null : c.piggybackCount];
                }),
                maxPiggybackCount: d.maxPiggybackCount,
                ringServers: rp.ring.getServerCount(), ringChecksum: rp.ring.checksum
            };
        }
        function strip(list) {
            return list.map(function (c) {
                var o = {};
                ['source', 'sourceIncarnationNumber', 'address', 'status', 'incarnationNumber'].forEach(function (k) {
                    if (c[k] !== undefined) o[k] = c[k];
                });
                return o;
            });
        }
        var first = { op: 'makeAlive', address: self, incarnationNumber: 1000 };
        first.result = strip(rp.membership.makeAlive(self, 1000));
        first.state = snapshot();
        ops.push(first);
        for (var s = 0; s < nops; s++) {
            if (stats && ri(5) === 0) {
                var gs = rp.membership.getStats();
                op = { op: 'getStats', result: { checksum: gs.checksum, members: gs.members.map(function (m) {
                    return [m.address, m.status, m.incarnationNumber]; }) } };
                op.state = snapshot();
                ops.push(op);
            }
            var kind = ri(100), op;
            Date.now = (function (t) { return function () { return t; }; })(1500000000000 + s);
            if (kind < 45) {
                var k = 1 + ri(10), batch = [];
                for (var j = 0; j < k; j++) {
                    var a = ri(8) === 0 ? self : addrs[ri(addrs.length)];
                    var c = { id: 'u' + (nextId++), address: a, status: STATUSES[ri(4)], incarnationNumber: 1000 + ri(4) };
                    if (ri(3)) { c.source = addrs[ri(addrs.length)]; c.sourceIncarnationNumber = 1000 + ri(3); }
                    batch.push(c);
                }
                op = { op: 'update', changes: JSON.parse(JSON.stringify(batch)) };
                op.result = strip(rp.membership.update(batch));
            } else if (kind < 55) {
                var mem = rp.membership.members[ri(rp.membership.members.length)];
                var which = ri(2) ? 'makeSuspect' : 'makeFaulty';
                op = { op: which, address: mem.address, incarnationNumber: mem.incarnationNumber };
                op.result = strip(rp.membership[which](mem.address, mem.incarnationNumber));
            } else if (kind < 70) {
                op = { op: 'issueAsSender' };
                op.result = strip(rp.dissemination.issueAsSender());
            } else if (kind < 90) {
                var snd = addrs[ri(addrs.length)], sinc = 1000 + ri(3);
                var cs = ri(2) ? rp.membership.checksum : 12345;
                op = { op: 'issueAsReceiver', sender: snd, senderIncarnationNumber: sinc, senderChecksum: cs };
                op.result = strip(rp.dissemination.issueAsReceiver(snd, sinc, cs));
            } else if (kind < 95) {
                op = { op: 'shuffle' };
                rp.membership.shuffle();
            } else if (kind < 97) {
                op = { op: 'clearChanges' };
                rp.dissemination.clearChanges();
            } else {
                op = { op: 'fullSync' };
                op.result = strip(rp.dissemination.fullSync());
            }
            if (stats) op.now = 1500000000000 + s;
            op.state = snapshot();
            ops.push(op);
        }
        rp.destroy();
        return { seed: seed, self: self, ops: ops };
    }
    if (want('node_ops')) {
        var ncases = [];
        [1, 2, 3, 4].forEach(function (seed) {
            ncases.push(withDeterminism(1000 + seed, function () { return nodeOps(seed, 150); }));
        });
        write('node_ops.json.gz', { note: 'Math.random = splitmix64(seed = 1000 + case seed), Date.now = 1.5e12 + op index',
                                    cases: ncases });
    }
}
if (want('node_stats')) {
    var scases = [];
    [5, 6, 7].forEach(function (seed) {
        scases.push(withDeterminism(1000 + seed, function () { return nodeOpsFn(seed, 150, true); }));
    });
    write('node_stats.json.gz', { note: 'as node_ops, with getStats() (in-place localeCompare sort) between ops; ' +
                                        'node ' + process.version + ', ICU ' + process.versions.icu, cases: scases });
}

// ---------------------------------------------------------------- ring
if (want('ring')) {
    var HashRing = require(path.join(REF, 'lib/ring.js'));
    // (a) farmhash ring: test/ring-test.js servers 127.0.0.1:3000+i
    var servers = [];
    for (var k = 0; k < 1000; k++) servers.push('127.0.0.1:' + (3000 + k));
    var ring = new HashRing();
    ring.addRemoveServers(servers, null);
    var keys = [], owners = [];
    var rng = new common.Rng(99n);
    for (k = 0; k < 5000; k++) keys.push(String(rng.next64()));
    servers.forEach(function (sv) { keys.push(sv + '0'); });
    keys.push('', 'a', 'abcd', 'abcde', 'hello world', '127.0.0.1:3000');
    keys.forEach(function (key) { owners.push(ring.lookup(key)); });
    var removed = servers.filter(function (_, j) { return j % 3 === 0; });
    ring.addRemoveServers(null, removed);
    var owners2 = keys.map(function (key) { return ring.lookup(key); });
    var lookupN = keys.slice(0, 200).map(function (key) { return ring.lookupN(key, 3); });
    write('ring_farmhash.json', { servers: servers, keys: keys, owners: owners, removed: removed,
        owners_after_remove: owners2, checksum_after_remove: ring.checksum, server_count: ring.getServerCount(),
        lookupN3_after_remove: lookupN });

    // (b) forced collisions through the reference's hashFunc seam (lib/ring.js:29):
    // 8 servers x 4 replicas with colliding replica hashes; a scripted history of
    // add/remove batches; after each step the rbtree contents and lookups.
    var R = 4;
    var table = {};
    var crng = new common.Rng(7n);
    var snames = ['A', 'B', 'C', 'D', 'E', 'F', 'G', 'H'];
    snames.forEach(function (sv) {
        for (var i = 0; i < R; i++) table[sv + i] = Number(crng.next64() % 40n) * 100;  // many collisions
    });
    function hf(str) { return table[str] !== undefined ? table[str] : Number(str.slice(4)); }
    var ops = [
        [['A', 'B', 'C'], []], [['D'], ['B']], [['B', 'E', 'F'], ['A']], [[], ['C', 'D']],
        [['A', 'G', 'H', 'C'], ['E']], [['D', 'E'], ['H', 'A']], [['A', 'B'], ['B', 'A']], [['H'], []]
    ];
    var cring = new HashRing({ hashFunc: hf, replicaPoints: R });
    var probes = [];
    for (k = 0; k <= 4100; k += 37) probes.push('key:' + k);
    var steps = ops.map(function (op) {
        var changed = cring.addRemoveServers(op[0], op[1]);
        var pts = [];
        var it = cring.rbtree.iterator();
        for (var v = it.next(); v !== null; v = it.next()) pts.push([v, it.str()]);
        return { add: op[0], remove: op[1], changed: changed, points: pts,
            servers: Object.keys(cring.servers).sort(),
            lookups: probes.map(function (p) { return cring.lookup(p); }),
            lookupN: probes.slice(0, 40).map(function (p) { return cring.lookupN(p, 3); }) };
    });
    write('ring_collisions.json', { replica_points: R, table: table, probes: probes, steps: steps });
}

// ---------------------------------------------------------------- piggyback
if (want('piggyback')) {
    var Dissemination = require(path.join(REF, 'lib/dissemination.js'));
    var EventEmitter = require('events').EventEmitter;
    var counts = [0, 1, 2, 8, 9, 10, 11, 98, 99, 100, 101, 999, 1000, 1023, 1024, 9999, 10000, 65535, 65536, 99999, 100000, 999999];
    var table2 = counts.map(function (c) {
        var fake = new EventEmitter();
        fake.ring = { getServerCount: function () { return c; } };
        fake.stat = function () {};
        fake.logger = { debug: function () {} };
        var d = new Dissemination(fake);
        d.adjustMaxPiggybackCount();
        return [c, d.maxPiggybackCount];
    });
    write('max_piggyback.json', { table: table2 });
}

// ---------------------------------------------------------------- sim
function simFixture(cfg, full) {
    var t = Date.now();
    var r = sim.runSim(cfg);
    var out = { config: cfg, convergedAt: r.convergedAt, rounds: r.rounds.map(function (x) {
        return { round: x.round, churned: x.churned, evaluated: x.evaluated, applied: x.applied,
                 fullSyncs: x.fullSyncs, messages: x.messages, waves: x.waves, converged: x.converged,
                 checksums: x.checksums };
    }) };
    if (full) out.final = r.final;
    else out.final_checksums = r.final.map(function (f) { return f.checksum; });
    console.log('sim', JSON.stringify(cfg), 'converged at', r.convergedAt, 'in', (Date.now() - t), 'ms');
    return out;
}

if (want('sim_small')) {
    write('sim_small.json.gz', { cases: [
        simFixture({ n: 64, seed: 1, maxRounds: 40, churnRounds: 10, churnK: 2 }, true),
        simFixture({ n: 48, seed: 5, maxRounds: 90, churnRounds: 60, churnK: 3 }, true),      // iterator wraps + shuffles
        simFixture({ n: 64, seed: 3, maxRounds: 60, churnRounds: 5, churnK: 1, failures: { 0: [5, 17, 40], 7: [3] } }, true),
        simFixture({ n: 32, seed: 1, maxRounds: 80, churnRounds: 20, churnK: 2, partition: { start: 3, end: 25, split: 16 } }, true),
        simFixture({ n: 40, seed: 11, maxRounds: 120, churnRounds: 100, churnK: 4, failures: { 0: [1, 2, 3, 4, 5, 6, 7, 8] } }, true)
    ] });
}

if (want('sim_medium')) {
    write('sim_medium.json.gz', { cases: [
        simFixture({ n: 256, seed: 2, maxRounds: 60, churnRounds: 20, churnK: 3, stopAtConvergence: true }, false),
        simFixture({ n: 200, seed: 7, maxRounds: 70, churnRounds: 20, churnK: 2, failures: { 2: [11, 150] },
                     partition: { start: 4, end: 26, split: 90 } }, false)
    ] });
}

if (want('sim_storm')) {
    // Config 5's refute storm (SURVEY.md §8(d)): seeded false suspicions
    // (makeSuspect by a live accuser, lib/membership.js:154-156) refuted by the
    // victims (:244-254), alone and on top of fail-stops, timers and churn.
    write('sim_storm.json.gz', { cases: [
        simFixture({ n: 48, seed: 9, maxRounds: 60, churnRounds: 0, churnK: 0, storm: { start: 0, end: 30, ppm: 1000 } }, true),
        simFixture({ n: 64, seed: 4, maxRounds: 80, churnRounds: 5, churnK: 2, failures: { 0: [3, 30] },
                     storm: { start: 0, end: 30, ppm: 20000 } }, true),
        simFixture({ n: 200, seed: 12, maxRounds: 90, churnRounds: 0, churnK: 0,
                     failures: { 0: [0, 9, 17, 33, 41, 50, 66, 71, 88, 99, 104, 120, 131, 142, 150, 163, 177, 181, 190, 199] },
                     storm: { start: 0, end: 25, ppm: 1000 } }, false)
    ] });
}

if (want('sim_views')) {
    // Arbitrary clusters (rp_sim_load_addresses / rp_sim_set_views, SURVEY.md
    // §8(b)): addresses of 4-32 bytes, and full bootstrap views that differ per
    // node (statuses alive/suspect/faulty/leave, incarnations around INC0) --
    // suspects start suspicion timers in set() (due at round 0), faulty/leave
    // members stay out of the ring, and gossip has to reconcile the views.
    // RingPop accepts hostPorts matching /^(\d+.\d+.\d+.\d+):\d+$/ (index.js:52;
    // the dots match any character)
    function addresses(n, seed) {
        var r = common.nodeRng(seed, 0), set = {}, out = [];
        function d(k) { return Math.floor(r.random() * k); }
        while (out.length < n) {
            var k = d(5), a;
            if (k === 0) a = d(10) + '.' + d(10) + '.' + d(10) + '.' + d(10) + ':' + (1 + d(9));
            else if (k === 1) a = (100000 + d(900000)) + '.' + (100000 + d(900000)) + '.' + (100000 + d(900000)) + '.' +
                                  (100000 + d(900000)) + ':' + (1000 + d(9000));
            else if (k === 2) a = '192.168.' + d(256) + '.' + d(256) + ':' + (20000 + d(1000));
            else if (k === 3) a = '10-' + d(256) + '-' + d(256) + '-' + d(256) + ':' + (8000 + d(100));
            else a = '172.' + (16 + d(16)) + '.' + d(256) + '.' + d(256) + ':' + (30000 + d(5000));
            if (a.length > 32 || set[a]) continue;
            set[a] = 1;
            out.push(a);
        }
        return out.sort(function (x, y) { return x < y ? -1 : x > y ? 1 : 0; });
    }
    function views(n, seed, pNoise) {
        var r = common.nodeRng(seed, 1), base = [], out = [];
        for (var j = 0; j < n; j++) {
            var u = r.random();
            base.push([u < 0.8 ? 1 : u < 0.88 ? 2 : u < 0.95 ? 3 : 4, common.INC0 + j + Math.floor(r.random() * 4) * 1000]);
        }
        for (var i = 0; i < n; i++) {
            var row = [];
            for (j = 0; j < n; j++) {
                var e = base[j].slice();
                if (r.random() < pNoise) {  // this node's view of j differs
                    var v = r.random();
                    e = [v < 0.5 ? 1 : v < 0.75 ? 2 : v < 0.9 ? 3 : 4, e[1] + (r.random() < 0.5 ? 0 : 1000)];
                }
                if (i === j) e = [1, e[1]];
                row.push(e);
            }
            out.push(row);
        }
        return out;
    }
    write('sim_views.json.gz', { cases: [
        simFixture({ n: 40, seed: 21, maxRounds: 40, churnRounds: 10, churnK: 2, addresses: addresses(40, 77) }, true),
        simFixture({ n: 48, seed: 22, maxRounds: 90, churnRounds: 10, churnK: 2, addresses: addresses(48, 78),
                     views: views(48, 79, 0.15) }, true),
        simFixture({ n: 32, seed: 23, maxRounds: 90, churnRounds: 5, churnK: 1, views: views(32, 80, 0.3),
                     failures: { 0: [4, 19], 6: [25] } }, true),
        simFixture({ n: 96, seed: 24, maxRounds: 120, churnRounds: 20, churnK: 2, addresses: addresses(96, 81),
                     views: views(96, 82, 0.05) }, false)
    ] });
}

if (want('sim_join')) {
    // The join path (SURVEY.md §8(f)4): nInit nodes start as a cluster, the
    // rest join perRound per round, each through nSeeds seeds drawn from the
    // nodes that were members before its round (handleJoin + mergeJoinResponses
    // + set()); gossip then spreads them (new members spliced at
    // getJoinPosition everywhere).
    function joinSchedule(n, nInit, seed, perRound, nSeeds, every, failed) {
        var r = common.nodeRng(seed, 2), ids = [];
        for (var i = 0; i < n; i++) ids.push(i);
        for (i = n - 1; i > 0; i--) { var k = Math.floor(r.random() * (i + 1)); var t = ids[i]; ids[i] = ids[k]; ids[k] = t; }
        var members = ids.slice(0, nInit).filter(function (v) { return !(failed || []).includes(v); }), out = [], round = 0;
        for (var q = nInit; q < n; q += perRound) {
            var batch = ids.slice(q, q + perRound), add = [];
            batch.forEach(function (j) {
                var pool = members.slice(), seeds = [];
                for (var z = 0; z < nSeeds && pool.length; z++) seeds.push(pool.splice(Math.floor(r.random() * pool.length), 1)[0]);
                out.push([round, j, seeds]);
                add.push(j);
            });
            members = members.concat(add.filter(function (v) { return !(failed || []).includes(v); }));
            round += every;
        }
        return out;
    }
    write('sim_join.json.gz', { cases: [
        simFixture({ n: 32, seed: 41, maxRounds: 60, churnRounds: 0, churnK: 0, joins: joinSchedule(32, 4, 41, 4, 3, 2) }, true),
        simFixture({ n: 48, seed: 42, maxRounds: 80, churnRounds: 30, churnK: 2, joins: joinSchedule(48, 8, 42, 5, 2, 3) }, true),
        simFixture({ n: 40, seed: 43, maxRounds: 90, churnRounds: 10, churnK: 1, joins: joinSchedule(40, 10, 43, 6, 3, 4, [5]),
                     failures: { 9: [5] } }, true),
        simFixture({ n: 128, seed: 44, maxRounds: 80, churnRounds: 20, churnK: 2, joins: joinSchedule(128, 16, 44, 16, 3, 2) }, false)
    ] });
}

if (want('sim_config2')) {
    // Config 2 (SURVEY.md §8(d)): 1,024 nodes, ceil(1% N) = 11 alive re-assertions
    // per round for 20 rounds, then gossip until every live checksum agrees.
    write('sim_config2_n1024.json.gz', { cases: [
        simFixture({ n: 1024, seed: 2024, maxRounds: 80, churnRounds: 20, churnK: 11, stopAtConvergence: true }, false)
    ] });
}

// ---------------------------------------------------------------- wire bridge
// The reference's ping path as JSON bodies between instances after a few
// rounds (churn + a fail-stop: alive, suspect and faulty updates in flight),
// and foreign bodies injected into /protocol/ping: a suspect about a live
// member, a suspect about the receiver itself (refuted), a higher-incarnation
// alive, and empty change lists with a matching / mismatching checksum
// (issueAsReceiver's fullSync fallback, lib/dissemination.js:102-117).
if (want('bridge')) {
    var cases = [];
    function bridgeCase(cfg, mkOps) {
        var probe = sim.runSim(Object.assign({}, cfg));
        cfg.bridge = mkOps(probe);
        cases.push(sim.runSim(cfg));
    }
    bridgeCase({ n: 48, seed: 5, churnK: 2, churnRounds: 12, maxRounds: 12, failures: { 3: [7] } }, function (p) {
        var A = p.addresses, f9 = p.final[9];
        return [
            { op: 'ping', from: 0, to: 5 }, { op: 'ping', from: 5, to: 0 }, { op: 'ping', from: 12, to: 30 },
            { op: 'ping', from: 30, to: 12 },
            { op: 'inject', to: 9, body: { checksum: 12345, source: A[20], sourceIncarnationNumber: f9.view[20][1],
              changes: [
                { address: A[3], status: 'suspect', incarnationNumber: f9.view[3][1], source: A[20],
                  sourceIncarnationNumber: f9.view[20][1] },
                { address: A[9], status: 'suspect', incarnationNumber: f9.view[9][1], source: A[20],
                  sourceIncarnationNumber: f9.view[20][1] },
                { address: A[11], status: 'alive', incarnationNumber: f9.view[11][1] + 1000, source: A[11],
                  sourceIncarnationNumber: f9.view[11][1] },
                { address: A[14], status: 'faulty', incarnationNumber: f9.view[14][1], source: A[20],
                  sourceIncarnationNumber: f9.view[20][1] } ] } },
            { op: 'ping', from: 9, to: 20 }
        ];
    });
    bridgeCase({ n: 40, seed: 8, churnK: 2, churnRounds: 4, maxRounds: 90 }, function (p) {
        var A = p.addresses;
        return [
            { op: 'inject', to: 4, body: { checksum: p.final[4].checksum, source: A[17], sourceIncarnationNumber: p.final[17].view[17][1], changes: [] } },
            { op: 'inject', to: 4, body: { checksum: 1, source: A[17], sourceIncarnationNumber: p.final[17].view[17][1], changes: [] } },
            { op: 'ping', from: 6, to: 4 }
        ];
    });
    write('wire_bridge.json', { note: 'reference ping path as JSON bodies (ids are the harness uuid shim\'s)', cases: cases });
}
