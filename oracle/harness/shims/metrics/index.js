// TEST INFRASTRUCTURE ONLY: stand-in for npm metrics (stats only, no state effect).
'use strict';
function Rate() {} Rate.prototype.stop = function () {};
function Meter() { this.m1Rate = new Rate(); this.m5Rate = new Rate(); this.m15Rate = new Rate(); }
Meter.prototype.mark = function () {};
function Histogram() { this.v = []; }
Histogram.prototype.update = function (x) { this.v.push(x); if (this.v.length > 64) this.v.shift(); };
Histogram.prototype.percentiles = function (ps) {
    var s = this.v.slice().sort(function (a, b) { return a - b; }), r = {};
    ps.forEach(function (p) { r[p] = s.length ? s[Math.floor(p * (s.length - 1))] : 0; });
    return r;
};
module.exports = { Meter: Meter, Histogram: Histogram };
