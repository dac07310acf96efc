// GPU parity of the JS drop-in Membership / Dissemination / HashRing (one
// ringpop instance on the device) against fixtures the reference produced
// (oracle/harness/gen_golden.js): the seeded operation sequences, config 1
// and the rules truth table.  The RingPop wiring the classes rely on -- the
// update / set listeners (lib/membership-update-listener.js:24-75,
// lib/membership-set-listener.js:24-48) and 'ringChanged' -- is restated here,
// since the reference does not travel to the GPU box.
'use strict';
var assert = require('assert');
var EventEmitter = require('events').EventEmitter;
var fs = require('fs');
var path = require('path');
var util = require('util');
var zlib = require('zlib');
var ROOT = path.join(__dirname, '..', '..');
var rp = require(path.join(ROOT, 'js', 'index.js'));

function golden(name) {
    var b = fs.readFileSync(path.join(ROOT, 'tests', 'golden', name));
    return JSON.parse(name.endsWith('.gz') ? zlib.gunzipSync(b) : b);
}

function FakeRingpop(whoami, seed) {
    EventEmitter.call(this);
    this.hostPort = whoami;
    this.isReady = true;
    this.membershipSeed = [0, seed];
    this.logger = { debug: function () {}, info: function () {}, warn: function () {}, error: function () {} };
    this.stat = function () {};
    this.suspicion = { start: function () {}, stop: function () {} };
    this.ring = new rp.HashRing();
    this.dissemination = new rp.Dissemination(this);
    this.membership = new rp.Membership(this);
    var self = this;
    this.membership.on('updated', function (updates) {
        var add = [], rm = [];
        updates.forEach(function (u) {
            if (u.status === 'alive') { add.push(u.address); self.suspicion.stop(u); }
            else if (u.status === 'suspect') self.suspicion.start(u);
            else if (u.status === 'faulty' || u.status === 'leave') { rm.push(u.address); self.suspicion.stop(u); }
            self.dissemination.recordChange(u);
        });
        if (add.length || rm.length) {
            if (self.ring.addRemoveServers(add, rm)) self.emit('ringChanged');
        }
    });
    this.membership.on('set', function (updates) {
        var add = [];
        updates.forEach(function (u) {
            if (u.status === 'alive') add.push(u.address);
            else if (u.status === 'suspect') self.suspicion.start(u);
            self.dissemination.recordChange(u);
        });
        if (add.length) self.ring.addRemoveServers(add);
    });
}
util.inherits(FakeRingpop, EventEmitter);
FakeRingpop.prototype.whoami = function () { return this.hostPort; };

function strip(list) {
    return list.map(function (c) {
        var o = {};
        ['source', 'sourceIncarnationNumber', 'address', 'status', 'incarnationNumber'].forEach(function (k) {
            if (c[k] !== undefined) o[k] = c[k];
        });
        return o;
    });
}
function snapshot(r) {
    var d = r.dissemination;
    return {
        checksum: r.membership.checksum,
        members: r.membership.members.map(function (m) { return [m.address, m.status, m.incarnationNumber]; }),
        changes: Object.keys(d.changes).map(function (a) {
            var c = d.changes[a];
            return [a, c.status, c.incarnationNumber, c.source === undefined ? null : c.source,
                    c.sourceIncarnationNumber === undefined ? null : c.sourceIncarnationNumber,
                    c.piggybackCount === undefined ? null : c.piggybackCount];
        }),
        maxPiggybackCount: d.maxPiggybackCount, ringServers: r.ring.getServerCount(), ringChecksum: r.ring.checksum
    };
}

var savedNow = Date.now;
// (1) seeded operation sequences
// node_stats: the same with getStats() between ops (an in-place sort of
// `members` by localeCompare, lib/membership.js:122-129, seen by every later op)
golden('node_ops.json.gz').cases.concat(golden('node_stats.json.gz').cases).forEach(function (c) {
    var r = new FakeRingpop(c.self, 1000 + c.seed);
    c.ops.forEach(function (op, k) {
        var now = op.now !== undefined ? op.now : 1500000000000 + Math.max(k - 1, 0);
        Date.now = (function (t) { return function () { return t; }; })(now);
        var res;
        if (op.op === 'getStats') {
            var gs = r.membership.getStats();
            assert.strictEqual(gs.members, r.membership.members, 'getStats returns the members array itself');
            assert.deepStrictEqual({ checksum: gs.checksum, members: gs.members.map(function (m) {
                return [m.address, m.status, m.incarnationNumber]; }) }, op.result, 'case ' + c.seed + ' op ' + k);
        }
        if (op.op === 'update') res = r.membership.update(JSON.parse(JSON.stringify(op.changes)));
        else if (op.op === 'makeAlive' || op.op === 'makeSuspect' || op.op === 'makeFaulty') {
            res = r.membership[op.op](op.address, op.incarnationNumber);
        } else if (op.op === 'issueAsSender') res = r.dissemination.issueAsSender();
        else if (op.op === 'issueAsReceiver') {
            res = r.dissemination.issueAsReceiver(op.sender, op.senderIncarnationNumber, op.senderChecksum);
        } else if (op.op === 'fullSync') res = r.dissemination.fullSync();
        else if (op.op === 'shuffle') r.membership.shuffle();
        else if (op.op === 'clearChanges') r.dissemination.clearChanges();
        if (op.result && op.op !== 'getStats') assert.deepStrictEqual(strip(res), op.result, 'case ' + c.seed + ' op ' + k + ' ' + op.op);
        assert.deepStrictEqual(snapshot(r), op.state, 'case ' + c.seed + ' op ' + k + ' ' + op.op + ' state');
    });
});
Date.now = savedNow;

// (2) config 1: large-membership.json into a ready instance
var c1 = golden('config1_large_membership.json'), recs = golden('large_membership_input.json');
[100, 1000, 1332].forEach(function (size) {
    var want = c1.results[String(size)];
    var r = new FakeRingpop('127.0.0.1:3000', c1.seed_base + size);
    var applied = r.membership.update(JSON.parse(JSON.stringify(recs.slice(0, size))));
    assert.strictEqual(applied.length, want.applied);
    assert.deepStrictEqual(r.membership.members.map(function (m) { return m.address; }), want.members_order);
    var str = r.membership.generateChecksumString();
    assert.strictEqual(Buffer.byteLength(str), want.checksum_string_len);
    assert.strictEqual(require('crypto').createHash('sha256').update(str).digest('hex'), want.checksum_string_sha);
    assert.strictEqual(r.membership.checksum, want.checksum);
    assert.strictEqual(r.ring.getServerCount(), want.ring_servers);
    assert.strictEqual(r.ring.checksum, want.ring_checksum);
    assert.strictEqual(r.dissemination.maxPiggybackCount, want.max_piggyback);
    assert.deepStrictEqual(Object.keys(r.dissemination.changes), want.changes);
});

// (3) the rules truth table through the device merge
var tt = golden('rules_truth_table.json');
Date.now = function () { return tt.now; };
tt.cases.forEach(function (t) {
    var r = new FakeRingpop('127.0.0.1:3000', 1);
    r.membership.makeAlive('127.0.0.1:3000', 1000);
    var target = t.self ? '127.0.0.1:3000' : '127.0.0.1:3001';
    if (!t.self) r.membership.makeAlive(target, 1000);
    var dev = r.__rpDeviceNode;
    rp.addon.memberForce(dev.h, dev.ids.get(target), { alive: 1, suspect: 2, faulty: 3, leave: 4 }[t.current], 1000);
    r.membership._cache = null;
    var applied = r.membership.update([{ address: target, status: t.change, incarnationNumber: 1000 + t.rel,
                                         source: '127.0.0.1:3009', sourceIncarnationNumber: 7 }]);
    var m = r.membership.findMemberByAddress(target);
    assert.deepStrictEqual([applied.length, m.status, m.incarnationNumber], [t.applied, t.status, t.inc], JSON.stringify(t));
});
Date.now = savedNow;
console.log('js membership/dissemination ok');
