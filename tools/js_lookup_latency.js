// Per-request cost of the drop-in ring lookup from JS (INTEGRATION.md §5):
// scalar ring.lookup (one launch + sync each) against lookupAsync (the keys of
// one tick in one launch), 1,000-server ring, on the GPU box:
//   node tools/js_lookup_latency.js > gpurun_out/js_lookup_latency.json
'use strict';
var path = require('path');
var rp = require(path.join(__dirname, '..', 'js', 'index.js'));

var servers = [];
for (var i = 0; i < 1000; i++) servers.push('10.0.' + (i >> 8) + '.' + (i & 255) + ':3000');
var ring = new rp.HashRing();
ring.addRemoveServers(servers, null);
var keys = [];
for (var k = 0; k < 200000; k++) keys.push('key-' + k);

function now() { var t = process.hrtime(); return t[0] * 1e9 + t[1]; }
for (var w = 0; w < 200; w++) ring.lookup(keys[w]);
var n1 = 5000, t0 = now();
for (var j = 0; j < n1; j++) ring.lookup(keys[j]);
var scalar_ns = (now() - t0) / n1;

function ticks(per, nticks, done) {
    var t = now(), left = nticks, answered = 0;
    (function tick() {
        for (var q = 0; q < per; q++) ring.lookupAsync(keys[(left * per + q) % keys.length], function () { answered++; });
        setImmediate(function () {
            if (--left > 0) return tick();
            done((now() - t) / (per * nticks), answered);
        });
    })();
}
var out = { servers: 1000, scalar_lookup_ns: Math.round(scalar_ns), async: [] };
var sizes = [1, 16, 256, 4096, 65536], si = 0;
(function next() {
    if (si === sizes.length) { console.log(JSON.stringify(out)); return; }
    var per = sizes[si++];
    ticks(per, per >= 4096 ? 20 : 200, function (ns, answered) {
        out.async.push({ keys_per_tick: per, ns_per_lookup: Math.round(ns), answered: answered });
        next();
    });
})();
