// GPU parity of the JS drop-in HashRing (js/index.js) against the reference's
// own ring test expectations (test/ring-test.js, test/hashring_test.js) and the
// golden fixtures produced by the reference (tests/golden/ring_*.json).
'use strict';
var assert = require('assert');
var path = require('path');
var ROOT = path.join(__dirname, '..', '..');
var rp = require(path.join(ROOT, 'js', 'index.js'));
var golden = function (n) { return require(path.join(ROOT, 'tests', 'golden', n)); };

function servers(size) { var s = []; for (var i = 0; i < size; i++) s.push('127.0.0.1:' + (3000 + i)); return s; }
function extractPort(server) { return parseInt(server.substr(server.lastIndexOf(':') + 1)); }

// test/ring-test.js: server counts on add/remove
(function () {
    var ring = new rp.HashRing();
    var s = servers(1000);
    ring.addRemoveServers(s, null);
    assert.strictEqual(ring.getServerCount(), 1000);
    ring.addRemoveServers(null, s);
    assert.strictEqual(ring.getServerCount(), 0);
    ring.addRemoveServers(s, s);
    assert.strictEqual(ring.getServerCount(), 0);
})();

// test/ring-test.js: checksum computed once per addRemoveServers
(function () {
    var ring = new rp.HashRing(), n = 0;
    ring.on('checksumComputed', function () { n++; });
    ring.addRemoveServers(servers(1000), servers(1000));
    assert.strictEqual(n, 1);
})();

// test/ring-test.js: lookup(server + '0') === server for 1000 servers
(function () {
    var ring = new rp.HashRing();
    var s = servers(1000);
    ring.addRemoveServers(s, null);
    var got = ring.lookupBatch(s.map(function (x) { return x + '0'; }));
    for (var i = 0; i < s.length; i++) assert.strictEqual(got[i], s[i]);
})();

// test/ring-test.js: lookupN with hashFunc = extractPort
(function () {
    var ring = new rp.HashRing({ hashFunc: extractPort });
    var s = servers(1000);
    ring.addRemoveServers(s, null);
    for (var i = 0; i < s.length; i += 7) {
        assert.deepStrictEqual(ring.lookupN(s[i] + '0', 3), [s[i], s[(i + 1) % 1000], s[(i + 2) % 1000]]);
    }
    var one = new rp.HashRing({ hashFunc: extractPort });
    one.addRemoveServers([s[0]], null);
    assert.deepStrictEqual(one.lookupN(s[0] + '0', 3), [s[0]]);
    var empty = new rp.HashRing({ hashFunc: extractPort });
    assert.deepStrictEqual(empty.lookupN(s[0] + '0', 3), []);
})();

// test/hashring_test.js: checksum changes on add/remove and does not depend on order
(function () {
    var a = new rp.HashRing(), b = new rp.HashRing();
    a.addServer('server1'); var c1 = a.checksum;
    a.addServer('server2'); assert.notStrictEqual(a.checksum, c1);
    b.addServer('server2'); b.addServer('server1');
    assert.strictEqual(a.checksum, b.checksum);
    a.removeServer('server2'); assert.strictEqual(a.checksum, c1);
})();

// golden: reference ring with real (restated) farmhash
(function () {
    var g = golden('ring_farmhash.json');
    var ring = new rp.HashRing();
    ring.addRemoveServers(g.servers, null);
    assert.deepStrictEqual(ring.lookupBatch(g.keys), g.owners);
    ring.addRemoveServers(null, g.removed);
    assert.deepStrictEqual(ring.lookupBatch(g.keys), g.owners_after_remove);
    assert.strictEqual(ring.checksum, g.checksum_after_remove);
})();

// golden: forced collisions through the hashFunc seam
(function () {
    var g = golden('ring_collisions.json');
    var hf = function (s) { return g.table[s] !== undefined ? g.table[s] : Number(s.slice(4)); };
    var ring = new rp.HashRing({ hashFunc: hf, replicaPoints: g.replica_points });
    g.steps.forEach(function (st) {
        assert.strictEqual(ring.addRemoveServers(st.add, st.remove), st.changed);
        assert.deepStrictEqual(ring.lookupBatch(g.probes), st.lookups);
        for (var i = 0; i < 40; i++) assert.deepStrictEqual(ring.lookupN(g.probes[i], 3), st.lookupN[i]);
    });
})();

// handleOrProxyAll's grouping (index.js:642): _.groupBy(keys, ring.lookup),
// expected result built from the reference fixture's owners
(function () {
    var g = golden('ring_farmhash.json');
    var ring = new rp.HashRing();
    assert.deepStrictEqual(ring.groupByOwner(g.keys.slice(0, 5)), { 'null': g.keys.slice(0, 5) });
    assert.deepStrictEqual(ring.groupByOwner([]), {});
    ring.addRemoveServers(g.servers, null);
    var want = {};
    g.keys.forEach(function (k, i) { (want[g.owners[i]] = want[g.owners[i]] || []).push(k); });
    var got = ring.groupByOwner(g.keys);
    assert.deepStrictEqual(Object.keys(got), Object.keys(want));
    assert.deepStrictEqual(got, want);
    var pr = new rp.HashRing({ hashFunc: extractPort });
    pr.addRemoveServers(servers(10), null);
    var keys = ['a:3003', 'b:3001', 'c:3003', 'd:9999', 'e:3001'];
    var exp = {};
    keys.forEach(function (k) { var o = pr.lookup(k); (exp[o] = exp[o] || []).push(k); });
    assert.deepStrictEqual(pr.groupByOwner(keys), exp);
})();

// lookupAsync: the keys of one tick in one device batch, the same owners as
// the reference fixture, callbacks in call order and never inside the call's
// tick; a resolve by size mid-tick; a ring change after a call does not change
// its answer; a throwing callback does not skip the others
function asyncLookups(done) {
    var g = golden('ring_farmhash.json');
    var ring = new rp.HashRing();
    ring.addRemoveServers(g.servers, null);
    var got = new Array(g.keys.length), order = [];
    g.keys.forEach(function (k, i) {
        ring.lookupAsync(k, function (err, owner) { assert.ifError(err); got[i] = owner; order.push(i); });
    });
    assert.strictEqual(order.length, 0);  // nothing answered inside the tick
    setImmediate(function () {
        assert.strictEqual(ring.lookupBatches, 1);
        assert.deepStrictEqual(got, g.owners);
        for (var i = 0; i < order.length; i++) assert.strictEqual(order[i], i);
        var keep = rp.HashRing.LOOKUP_FLUSH_KEYS, n = 0;
        rp.HashRing.LOOKUP_FLUSH_KEYS = 3;
        for (var j = 0; j < 7; j++) ring.lookupAsync(g.keys[j], function () { n++; });
        rp.HashRing.LOOKUP_FLUSH_KEYS = keep;
        assert.strictEqual(n, 0);  // two batches resolved, none answered in this tick
        assert.strictEqual(ring.lookupBatches, 3);
        setImmediate(function () {
            assert.strictEqual(n, 7);  // the two early batches, then the last at its own setImmediate
            assert.strictEqual(ring.lookupBatches, 4);
            assert.throws(function () { ring.lookupAsync('x'); }, TypeError);
            ringChangeAfterCall(ring, g, done);
        });
    });
}

function ringChangeAfterCall(ring, g, done) {
    // the owner of key 0, then that owner removed in the same tick: the
    // queued lookup still answers with the ring as of its call
    var k0 = g.keys[0], before = ring.lookup(k0), ans = null, after = null;
    ring.lookupAsync(k0, function (err, o) { assert.ifError(err); ans = o; });
    ring.removeServer(before);
    ring.lookupAsync(k0, function (err, o) { assert.ifError(err); after = o; });
    var calls = [];
    ring.lookupAsync(k0, function () { calls.push(1); throw new Error('cb boom'); });
    ring.lookupAsync(k0, function () { calls.push(2); });
    process.once('uncaughtException', function (e) {
        assert.strictEqual(e.message, 'cb boom');
        assert.strictEqual(ans, before);
        assert.notStrictEqual(after, before);
        assert.strictEqual(after, ring.lookup(k0));
        assert.deepStrictEqual(calls, [1, 2]);  // the second ran although the first threw
        ring.addServer(before);
        done();
    });
}

asyncLookups(function () { console.log('js hashring ok'); });
