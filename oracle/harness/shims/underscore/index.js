// TEST INFRASTRUCTURE ONLY: minimal stand-in for npm underscore, which the
// reference pins only as ^1.5.2 (package.json:37) and does not vendor.  The
// harness pins the algorithms of underscore 1.13.x (what that range resolves
// to today): `random(min,max) = min + floor(Math.random()*(max-min+1))`,
// `sample(list, n)` = forward partial Fisher-Yates over a copy with
// `random(index, last)` per step, `shuffle(list) = sample(list, Infinity)`.
// Only the functions the hot path touches are provided
// (lib/membership.js:115-119,251,316,320).
'use strict';

function random(min, max) {
    if (max == null) { max = min; min = 0; }
    return min + Math.floor(Math.random() * (max - min + 1));
}

function values(obj) { return Object.keys(obj).map(function (k) { return obj[k]; }); }

function sample(obj, n, guard) {
    var arr = Array.isArray(obj) ? obj.slice() : values(obj);
    if (n == null || guard) return arr[random(arr.length - 1)];
    var length = arr.length;
    n = Math.max(Math.min(n, length), 0);
    var last = length - 1;
    for (var index = 0; index < n; index++) {
        var rand = random(index, last);
        var temp = arr[index];
        arr[index] = arr[rand];
        arr[rand] = temp;
    }
    return arr.slice(0, n);
}

function shuffle(obj) { return sample(obj, Infinity); }

function extend(obj) {
    for (var i = 1; i < arguments.length; i++) {
        var src = arguments[i];
        if (src) Object.keys(src).forEach(function (k) { obj[k] = src[k]; });
    }
    return obj;
}

function defaults(obj) {
    for (var i = 1; i < arguments.length; i++) {
        var src = arguments[i];
        if (src) Object.keys(src).forEach(function (k) { if (obj[k] === undefined) obj[k] = src[k]; });
    }
    return obj;
}

function pluck(list, key) { return list.map(function (o) { return o[key]; }); }
function times(n, fn) { var r = []; for (var i = 0; i < n; i++) r.push(fn(i)); return r; }
function groupBy(list, fn) {
    var r = {};
    list.forEach(function (x) { var k = fn(x); (r[k] = r[k] || []).push(x); });
    return r;
}

function Chain(v) { this._v = v; }
Chain.prototype.reject = function (fn) { return new Chain(this._v.filter(function (x) { return !fn(x); })); };
Chain.prototype.filter = function (fn) { return new Chain(this._v.filter(fn)); };
Chain.prototype.sample = function (n) { return new Chain(sample(this._v, n)); };
Chain.prototype.value = function () { return this._v; };

module.exports = {
    random: random, sample: sample, shuffle: shuffle, extend: extend, defaults: defaults,
    pluck: pluck, times: times, groupBy: groupBy, values: values,
    chain: function (v) { return new Chain(v); }
};
