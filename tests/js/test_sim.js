// GPU parity of the JS SimCluster against the reference-generated simulation
// fixture (tests/golden/sim_small.json.gz, case 0: 64 nodes, churn).
'use strict';
var assert = require('assert');
var path = require('path');
var zlib = require('zlib');
var fs = require('fs');
var ROOT = path.join(__dirname, '..', '..');
var rp = require(path.join(ROOT, 'js', 'index.js'));

var g = JSON.parse(zlib.gunzipSync(fs.readFileSync(path.join(ROOT, 'tests', 'golden', 'sim_small.json.gz'))));
var c = g.cases[0], cfg = c.config;
var sim = new rp.SimCluster({ n: cfg.n, seed: cfg.seed, churnK: cfg.churnK });
c.rounds.forEach(function (jr, r) {
    var st = sim.round(r < cfg.churnRounds);
    assert.strictEqual(st.evaluated, jr.evaluated);
    assert.strictEqual(st.applied, jr.applied);
    assert.strictEqual(st.converged, jr.converged);
    assert.deepStrictEqual(Array.from(sim.checksums()), jr.checksums);
});
var STATUS = [null, 'alive', 'suspect', 'faulty', 'leave'];
for (var v = 0; v < cfg.n; v += 9) {
    var node = sim.node(v), f = c.final[v];
    assert.strictEqual(node.membership.checksum, f.checksum);
    assert.deepStrictEqual(node.membership.members.map(function (m) { return g.cases[0].final ? m.address : m; }).length, f.members.length);
    f.view.forEach(function (e, a) {
        var m = node.membership.findMemberByAddress(sim.addresses()[a]);
        assert.strictEqual(m.status, STATUS[e[0]]);
        assert.strictEqual(m.incarnationNumber, e[1]);
    });
    var keys = Object.keys(node.dissemination.changes);
    assert.deepStrictEqual(keys, f.changes.map(function (row) { return sim.addresses()[row[0]]; }));
    assert.strictEqual(node.dissemination.maxPiggybackCount, f.maxPiggyback);
    assert.strictEqual(node.ring.getServerCount(), f.ringServers);
}
console.log('js sim ok');
