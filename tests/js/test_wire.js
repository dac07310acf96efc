// GPU: the JS wire facade (SimCluster.prototype.wire) against the reference's
// own JSON ping bodies and responses (tests/golden/wire_bridge.json, made by
// oracle/harness/gen_golden.js); the reference's uuid `id` fields are not
// modelled and are dropped before comparing.
'use strict';
var assert = require('assert');
var path = require('path');
var fs = require('fs');
var ROOT = path.join(__dirname, '..', '..');
var rp = require(path.join(ROOT, 'js', 'index.js'));

function noIds(changes) {
    return changes.map(function (c) {
        var o = {};
        Object.keys(c).forEach(function (k) { if (k !== 'id') o[k] = c[k]; });
        return o;
    });
}

var g = JSON.parse(fs.readFileSync(path.join(ROOT, 'tests', 'golden', 'wire_bridge.json')));
g.cases.forEach(function (c, ci) {
    var cfg = c.config;
    var sim = new rp.SimCluster({ n: cfg.n, seed: cfg.seed, churnK: cfg.churnK });
    Object.keys(cfg.failures || {}).forEach(function (r) {
        cfg.failures[r].forEach(function (v) { sim.fail(v, Number(r)); });
    });
    for (var r = 0; r < cfg.maxRounds; r++) sim.round(r < cfg.churnRounds);
    assert.deepStrictEqual(sim.addresses(), c.addresses);
    c.bridge.forEach(function (op, k) {
        var o = op.op, body;
        if (o.op === 'ping') {
            body = sim.wire(o.from).pingBody();
            var want = Object.assign({}, op.body, { changes: noIds(op.body.changes) });
            assert.strictEqual(body, JSON.stringify(want), 'case ' + ci + ' op ' + k + ' body');
        } else {
            body = JSON.stringify(o.body);
        }
        var resp = sim.wire(o.to).handlePing(body);
        assert.strictEqual(resp, JSON.stringify({ changes: noIds(op.response.changes) }), 'case ' + ci + ' op ' + k + ' response');
        if (o.op === 'ping') {
            assert.strictEqual(sim.wire(o.from).onPingResponse(JSON.stringify(op.response)), op.applied);
        }
        assert.strictEqual(sim.checksums()[o.to], op.toDump.checksum);
    });
    assert.throws(function () { sim.wire(0).handlePing('{"source":"x","changes":[]}'); }, /need req body/);
});
console.log('js wire ok');
