// benchmarks/add-remove-hashring.js's two patterns (1,000 servers of
// large-membership.json: addServer / removeServer one at a time, and one
// addRemoveServers(servers, servers) call) through a HashRing, per call:
//   node tools/js_ring_addremove.js gpu        -- js/index.js (the drop-in; on the GPU box)
//   NODE_PATH=oracle/harness/shims node tools/js_ring_addremove.js reference
//                                              -- /root/reference/lib/ring.js (build container only;
//                                                 farmhash = the harness's JS transcription)
// Prints one JSON line.
'use strict';
var path = require('path');
var impl = process.argv[2] || 'gpu';
var reps = +(process.argv[3] || 10);
var HashRing = impl === 'reference' ? require('/root/reference/lib/ring.js')
                                    : require(path.join(__dirname, '..', 'js', 'index.js')).HashRing;
var members = require(path.join(__dirname, '..', 'tests', 'golden', 'large_membership_input.json')).slice(0, 1000);
var servers = members.map(function (m) { return m.address; });

function now() { var t = process.hrtime(); return t[0] * 1e9 + t[1]; }

function individual(ring) {
    for (var i = 0; i < servers.length; i++) ring.addServer(servers[i]);
    for (var j = 0; j < servers.length; j++) ring.removeServer(servers[j]);
}
function bulk(ring) { ring.addRemoveServers(servers, servers); }

function time(fn, n) {
    var ring = new HashRing();
    fn(ring);  // (warm-up pass: code paths, device buffers)
    var t0 = now();
    for (var r = 0; r < n; r++) fn(ring);
    return (now() - t0) / n;
}
var ind = time(individual, reps), blk = time(bulk, reps);
// a probe after the last removal: the ring is empty again
var check = new HashRing();
individual(check);
console.log(JSON.stringify({
    impl: impl, node: process.version, servers: servers.length, reps: reps,
    individual_ms_per_pass: +(ind / 1e6).toFixed(3),
    individual_us_per_call: +(ind / 1e3 / (2 * servers.length)).toFixed(2),
    bulk_ms_per_call: +(blk / 1e6).toFixed(3),
    empty_after: check.getServerCount() === 0
}));
