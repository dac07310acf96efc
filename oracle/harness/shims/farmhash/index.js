// TEST INFRASTRUCTURE ONLY (oracle harness).  Stands in for the npm
// `farmhash` ^0.2.0 native addon (package.json:30), which is absent from
// this image.  A JavaScript transcription of the same farmhashmk::Hash32
// restatement as oracle/farmhash32.c; the two are cross-checked by
// tests/test_oracle_farmhash.py (parity of the algorithm itself: see the
// header of oracle/farmhash32.c).
'use strict';

var C1 = 0xcc9e2d51 | 0;
var C2 = 0x1b873593 | 0;

function rotr(v, s) { return s === 0 ? v | 0 : ((v >>> s) | (v << (32 - s))) | 0; }
function fmix(h) {
    h ^= h >>> 16; h = Math.imul(h, 0x85ebca6b | 0);
    h ^= h >>> 13; h = Math.imul(h, 0xc2b2ae35 | 0);
    h ^= h >>> 16; return h | 0;
}
function mur(a, h) {
    a = Math.imul(a, C1); a = rotr(a, 17); a = Math.imul(a, C2);
    h ^= a; h = rotr(h, 19);
    return (Math.imul(h, 5) + (0xe6546b64 | 0)) | 0;
}

function hashBuf(s) {
    var len = s.length;
    function f(o) { return s.readInt32LE(o); }
    var a, b, c, d, e, h, g, fv;
    if (len <= 4) {
        b = 0; c = 9;
        for (var i = 0; i < len; i++) {
            var v = s.readInt8(i);
            b = (Math.imul(b, C1) + v) | 0; c ^= b;
        }
        return fmix(mur(b, mur(len, c))) >>> 0;
    }
    if (len <= 12) {
        a = len; b = len * 5; c = 9; d = b;
        a = (a + f(0)) | 0; b = (b + f(len - 4)) | 0; c = (c + f((len >>> 1) & 4)) | 0;
        return fmix(mur(c, mur(b, mur(a, d)))) >>> 0;
    }
    if (len <= 24) {
        a = f(-4 + (len >>> 1)); b = f(4); c = f(len - 8); d = f(len >>> 1); e = f(0); fv = f(len - 4);
        h = (Math.imul(d, C1) + len) | 0;
        a = (rotr(a, 12) + fv) | 0; h = (mur(c, h) + a) | 0;
        a = (rotr(a, 3) + c) | 0; h = (mur(e, h) + a) | 0;
        a = (rotr((a + fv) | 0, 12) + d) | 0; h = (mur(b, h) + a) | 0;
        return fmix(h) >>> 0;
    }
    h = len | 0; g = Math.imul(C1, len); fv = g;
    var a0 = Math.imul(rotr(Math.imul(f(len - 4), C1), 17), C2);
    var a1 = Math.imul(rotr(Math.imul(f(len - 8), C1), 17), C2);
    var a2 = Math.imul(rotr(Math.imul(f(len - 16), C1), 17), C2);
    var a3 = Math.imul(rotr(Math.imul(f(len - 12), C1), 17), C2);
    var a4 = Math.imul(rotr(Math.imul(f(len - 20), C1), 17), C2);
    var K = 0xe6546b64 | 0;
    h ^= a0; h = rotr(h, 19); h = (Math.imul(h, 5) + K) | 0;
    h ^= a2; h = rotr(h, 19); h = (Math.imul(h, 5) + K) | 0;
    g ^= a1; g = rotr(g, 19); g = (Math.imul(g, 5) + K) | 0;
    g ^= a3; g = rotr(g, 19); g = (Math.imul(g, 5) + K) | 0;
    fv = (fv + a4) | 0; fv = (rotr(fv, 19) + 113) | 0;
    var iters = Math.floor((len - 1) / 20);
    var o = 0;
    do {
        a = f(o); b = f(o + 4); c = f(o + 8); d = f(o + 12); e = f(o + 16);
        h = (h + a) | 0; g = (g + b) | 0; fv = (fv + c) | 0;
        h = (mur(d, h) + e) | 0;
        g = (mur(c, g) + a) | 0;
        fv = (mur((b + Math.imul(e, C1)) | 0, fv) + d) | 0;
        fv = (fv + g) | 0; g = (g + fv) | 0;
        o += 20;
    } while (--iters !== 0);
    g = Math.imul(rotr(g, 11), C1); g = Math.imul(rotr(g, 17), C1);
    fv = Math.imul(rotr(fv, 11), C1); fv = Math.imul(rotr(fv, 17), C1);
    h = rotr((h + g) | 0, 19); h = (Math.imul(h, 5) + K) | 0; h = Math.imul(rotr(h, 17), C1);
    h = rotr((h + fv) | 0, 19); h = (Math.imul(h, 5) + K) | 0; h = Math.imul(rotr(h, 17), C1);
    return h >>> 0;
}

function hash32(input) {
    return hashBuf(Buffer.isBuffer(input) ? input : Buffer.from(String(input), 'utf8'));
}

module.exports = { hash32: hash32, hashBuf: hashBuf };
