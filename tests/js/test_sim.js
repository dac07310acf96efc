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
// arbitrary clusters and the join path through SimCluster's options, against
// the reference fixtures (loaded addresses + per-node views; joins)
function fixtureRun(name, idx) {
    var fc = JSON.parse(zlib.gunzipSync(fs.readFileSync(path.join(ROOT, 'tests', 'golden', name)))).cases[idx];
    var cf = fc.config, opts = { n: cf.n, seed: cf.seed, churnK: cf.churnK };
    if (cf.addresses) opts.addresses = cf.addresses;
    if (cf.joins) opts.joins = cf.joins;
    if (cf.views) {
        var st = new Int32Array(cf.n * cf.n), inc = new Float64Array(cf.n * cf.n);
        cf.views.forEach(function (row, v) { row.forEach(function (e, a) { st[v * cf.n + a] = e[0]; inc[v * cf.n + a] = e[1]; }); });
        opts.views = { status: st, incarnation: inc };
    }
    var c2 = new rp.SimCluster(opts);
    fc.rounds.forEach(function (jr, r) {
        var st2 = c2.round(r < cf.churnRounds);
        assert.strictEqual(st2.evaluated, jr.evaluated, name + ' round ' + r);
        assert.strictEqual(st2.applied, jr.applied, name + ' round ' + r);
        var got = Array.from(c2.checksums());
        jr.checksums.forEach(function (x, v) { if (x !== null) assert.strictEqual(got[v], x, name + ' round ' + r); });
    });
    if (cf.addresses) assert.deepStrictEqual(c2.addresses(), cf.addresses);
}
fixtureRun('sim_views.json.gz', 1);
fixtureRun('sim_join.json.gz', 0);

// the same cluster through runAsync (napi_async_work): the cluster is busy
// until the promise settles, then its totals and checksums equal the fixture's
var sim2 = new rp.SimCluster({ n: cfg.n, seed: cfg.seed, churnK: cfg.churnK });
var R = c.rounds.length, CR = Math.min(cfg.churnRounds, R);
var p1 = sim2.runAsync(CR, true);
assert.throws(function () { sim2.checksums(); }, /in flight/);
var ticks = 0;
var timer = setInterval(function () { ticks++; }, 0);
p1.then(function () { return sim2.runAsync(R - CR, false); }).then(function (tot) {
    clearInterval(timer);
    var ev = 0, ap = 0;
    c.rounds.forEach(function (jr) { ev += jr.evaluated; ap += jr.applied; });
    assert.strictEqual(tot.evaluated, ev);
    assert.strictEqual(tot.applied, ap);
    assert.deepStrictEqual(Array.from(sim2.checksums()), c.rounds[R - 1].checksums);
    console.log('js sim ok (async: ' + ticks + ' event-loop ticks during the runs)');
}).catch(function (e) {
    console.error(e);
    process.exit(1);
});
