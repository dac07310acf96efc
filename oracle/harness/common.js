// TEST INFRASTRUCTURE ONLY (oracle harness, runs in this container under
// Node; never shipped to the GPU box).  Deterministic environment the
// build-owned harness injects around the reference modules:
//   * per-node seeded Math.random (reference reads it at
//     lib/membership.js:100, lib/swim/gossip.js:44 and through underscore at
//     lib/membership.js:115-119,316),
//   * a virtual Date.now (index.js:235, lib/membership.js:248,340),
//   * a virtual setTimeout/clearTimeout queue (lib/swim/suspicion.js:66).
// The same definitions are restated in C in oracle/sim_oracle.c and in the
// product (ringpop_amd/csrc/rp_sim.hip); DESIGN.md §"Simulation semantics".
'use strict';

var MASK = (1n << 64n) - 1n;
var GOLDEN = 0x9E3779B97F4A7C15n;
var NODE_MUL = 0xD1B54A32D192ED03n;
var CHURN_XOR = 0x5851F42D4C957F2Dn;
var STORM_XOR = 0x2545F4914F6CDD1Dn;
var TWO_M53 = Math.pow(2, -53);

// splitmix64: state += golden; z = mix(state).
function Rng(state) { this.s = BigInt.asUintN(64, state); }
Rng.prototype.next64 = function next64() {
    this.s = (this.s + GOLDEN) & MASK;
    var z = this.s;
    z = ((z ^ (z >> 30n)) * 0xBF58476D1CE4E5B9n) & MASK;
    z = ((z ^ (z >> 27n)) * 0x94D049BB133111EBn) & MASK;
    return z ^ (z >> 31n);
};
// Math.random() replacement: top 53 bits as an exact double in [0,1).
Rng.prototype.random = function random() { return Number(this.next64() >> 11n) * TWO_M53; };

function nodeRng(seed, i) { return new Rng(BigInt.asUintN(64, BigInt(seed)) ^ ((BigInt(i + 1) * NODE_MUL) & MASK)); }
function churnRng(seed) { return new Rng(BigInt.asUintN(64, BigInt(seed)) ^ CHURN_XOR); }
function stormRng(seed) { return new Rng(BigInt.asUintN(64, BigInt(seed)) ^ STORM_XOR); }

// Config-2/4 address scheme (SURVEY.md §8(d)): 10.<b2>.<b1>.<b0>:<3000+i%7>,
// node ids are the ranks of these strings in JS (`<`) sort order so that a
// view indexed by node id is already in checksum order
// (lib/membership.js:70-93).
function simAddresses(n) {
    var raw = [];
    for (var i = 0; i < n; i++) {
        raw.push('10.' + ((i >> 16) & 255) + '.' + ((i >> 8) & 255) + '.' + (i & 255) + ':' + (3000 + (i % 7)));
    }
    raw.sort(function (a, b) { return a < b ? -1 : a > b ? 1 : 0; });
    return raw;
}

var INC0 = 1434401518824;      // initial incarnation of node i is INC0 + i
var T0 = 1500000000000;        // virtual time of round 0
var PERIOD = 200;              // lib/swim/gossip.js:127-129 minProtocolPeriod

// Churn choice for one round: partial Fisher-Yates over the live ids.
function chooseChurn(rng, liveIds, k) {
    var cand = liveIds.slice();
    var L = cand.length;
    k = Math.min(k, L);
    for (var j = 0; j < k; j++) {
        var r = j + Math.floor(rng.random() * (L - j));
        var t = cand[j]; cand[j] = cand[r]; cand[r] = t;
    }
    return cand.slice(0, k);
}

// False-suspicion storm for one round (config 5): K = ceil(L * ppm / 1e6)
// victims by partial Fisher-Yates over the live ids (ascending), then per
// victim an accuser drawn uniformly from the other live ids.  Returns
// [accuser, victim] pairs in draw order.
function chooseStorm(rng, liveIds, ppm) {
    var L = liveIds.length;
    if (L < 2) return [];
    var K = Math.min(Math.floor((L * ppm + 999999) / 1000000), L);
    var cand = liveIds.slice();
    for (var j = 0; j < K; j++) {
        var r = j + Math.floor(rng.random() * (L - j));
        var t = cand[j]; cand[j] = cand[r]; cand[r] = t;
    }
    var pairs = [];
    for (j = 0; j < K; j++) {
        var v = cand[j], lo = 0, hi = L;
        while (lo < hi) { var m = (lo + hi) >> 1; if (liveIds[m] < v) lo = m + 1; else hi = m; }
        var idx = Math.floor(rng.random() * (L - 1));
        pairs.push([liveIds[idx < lo ? idx : idx + 1], v]);
    }
    return pairs;
}

// Virtual timers: fire in (due, creation seq) order, each in its node context.
function TimerQueue() { this.items = []; this.seq = 0; }
TimerQueue.prototype.add = function add(due, node, fn) {
    var t = { due: due, seq: this.seq++, node: node, fn: fn, cancelled: false };
    this.items.push(t);
    return t;
};
TimerQueue.prototype.due = function due(now) {
    var d = this.items.filter(function (t) { return !t.cancelled && t.due <= now; });
    d.sort(function (a, b) { return a.due - b.due || a.seq - b.seq; });
    this.items = this.items.filter(function (t) { return !t.cancelled && t.due > now; });
    return d;
};

module.exports = {
    Rng: Rng, nodeRng: nodeRng, churnRng: churnRng, stormRng: stormRng, simAddresses: simAddresses,
    chooseChurn: chooseChurn, chooseStorm: chooseStorm, TimerQueue: TimerQueue, INC0: INC0, T0: T0, PERIOD: PERIOD
};
