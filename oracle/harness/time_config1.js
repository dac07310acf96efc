// TEST INFRASTRUCTURE ONLY.  Times config 1 on the reference JavaScript, in
// the build container (the reference cannot travel to the GPU box):
//
//   NODE_PATH=oracle/harness/shims node oracle/harness/time_config1.js > bench_data/reference_js_config1.json
//
// Task A: membership.update() of benchmarks/large-membership.json's 1,332
//         records into a fresh READY instance (benchmarks/large-membership-
//         update.js:37-47 with isReady set, SURVEY.md §0.4: the script as
//         published stashes the batch and measures nothing).  The update
//         listener's ring.addRemoveServers (100 farmhash32 per alive server)
//         and the one computeChecksum() are inside the timed call, as in the
//         reference.
// Task B: membership.computeChecksum() on 1,000 members
//         (benchmarks/compute-checksum.js:46-62, again with a ready instance).
// farmhash is the harness's JavaScript transcription (shims/farmhash): the npm
// native addon is absent, so hashing runs slower than the addon would.
'use strict';

var path = require('path');
var REF = process.env.RINGPOP_REFERENCE || '/root/reference';

function freshRingpop(hostPort) {
    var RingPop = require(path.join(REF, 'index.js'));
    var rp = new RingPop({ app: 'time', hostPort: hostPort });
    rp.membershipUpdateRollup = { trackUpdates: function () {}, destroy: function () {} };
    rp.isReady = true;
    return rp;
}

function ms(t0) { return Number(process.hrtime.bigint() - t0) / 1e6; }
function median(a) { var s = a.slice().sort(function (x, y) { return x - y; }); return s[s.length >> 1]; }

var large = require(path.join(REF, 'benchmarks/large-membership.json'));
var out = { node: process.version, what: 'reference ringpop JS, build container, one core',
            farmhash: 'harness JS transcription (npm addon absent)' };

// warm the JIT on a few untimed runs, then time
var A = [];
for (var it = 0; it < 40; it++) {
    var rp = freshRingpop('127.0.0.1:3000');
    var batch = JSON.parse(JSON.stringify(large));
    var t0 = process.hrtime.bigint();
    var applied = rp.membership.update(batch);
    var t = ms(t0);
    if (it >= 10) A.push(t);
    if (applied.length !== 1332) throw new Error('applied ' + applied.length);
    rp.destroy();
}
out.update_1332 = { median_ms: median(A), min_ms: Math.min.apply(null, A), iterations: A.length,
                    task: 'membership.update(1,332 records) into a fresh ready instance, listeners included' };

var rp2 = freshRingpop('127.0.0.1:3000');
rp2.membership.update(JSON.parse(JSON.stringify(large.slice(0, 1000))));
if (rp2.membership.getMemberCount() !== 1000) throw new Error('members ' + rp2.membership.getMemberCount());
var B = [];
for (var j = 0; j < 300; j++) {
    var t1 = process.hrtime.bigint();
    rp2.membership.computeChecksum();
    var tb = ms(t1);
    if (j >= 50) B.push(tb);
}
out.compute_checksum_1000 = { median_ms: median(B), min_ms: Math.min.apply(null, B), iterations: B.length,
                              checksum: rp2.membership.checksum,
                              string_bytes: Buffer.byteLength(rp2.membership.generateChecksumString()),
                              task: 'membership.computeChecksum() on 1,000 members' };
rp2.destroy();
console.log(JSON.stringify(out, null, 1));
