// ringpop_amd JavaScript host: drop-in surfaces for ringpop's hot path backed
// by the MI355X library through the N-API addon (js/ringpop_hip.node).
//
//   farmhash   -> replaces require('farmhash') (package.json:30): hash32(str)
//   HashRing   -> lib/ring.js:25-184 API (addServer, removeServer,
//                 addRemoveServers, computeChecksum, getServerCount,
//                 hasServer, lookup, lookupN, groupByOwner; events added / removed /
//                 checksumComputed) + lookupBatch for batched device lookups
//   SimCluster -> N simulated ringpop instances on the device, with per-node
//                 read facades named after Membership / Dissemination / ring
//
// There is no JavaScript fallback: loading fails if the addon or the HIP
// library is missing, and calls throw when no GPU is available.
'use strict';

var EventEmitter = require('events').EventEmitter;
var path = require('path');
var util = require('util');

var addon = require(path.join(__dirname, 'ringpop_hip.node'));

var STATUS = [null, 'alive', 'suspect', 'faulty', 'leave'];

var farmhash = {
    hash32: function hash32(input) { return addon.hash32(String(input)); },
    hash32Batch: function hash32Batch(list) { return addon.hash32Batch(list); }
};

function HashRing(options) {
    if (!(this instanceof HashRing)) return new HashRing(options);
    EventEmitter.call(this);
    this.options = options || {};
    this.replicaPoints = this.options.replicaPoints || 100;   // lib/ring.js:28
    this.hashFunc = this.options.hashFunc || null;            // lib/ring.js:29 (device farmhash by default)
    this.servers = {};
    this.checksum = null;
    this._ring = addon.ringCreate(this.replicaPoints);
}
util.inherits(HashRing, EventEmitter);

HashRing.prototype._replicaHashes = function (names) {
    if (!this.hashFunc || names.length === 0) return undefined;
    var out = new Uint32Array(names.length * this.replicaPoints);
    for (var s = 0; s < names.length; s++) {
        for (var i = 0; i < this.replicaPoints; i++) out[s * this.replicaPoints + i] = this.hashFunc(names[s] + i) >>> 0;
    }
    return out;
};

HashRing.prototype.addRemoveServers = function addRemoveServers(serversToAdd, serversToRemove) {
    var add = serversToAdd || [], rm = serversToRemove || [];
    var changed = addon.ringAddRemove(this._ring, add, rm, this._replicaHashes(add), this._replicaHashes(rm),
                                      this.replicaPoints);
    var self = this;
    add.forEach(function (s) { self.servers[s] = true; });
    rm.forEach(function (s) { delete self.servers[s]; });
    if (changed) this.computeChecksum();
    return changed;
};

HashRing.prototype.addServer = function addServer(name) {
    if (this.hasServer(name)) return;
    addon.ringAddRemove(this._ring, [name], [], this._replicaHashes([name]), undefined, this.replicaPoints);
    this.servers[name] = true;
    this.computeChecksum();
    this.emit('added', name);
};

HashRing.prototype.removeServer = function removeServer(name) {
    if (!this.hasServer(name)) return;
    addon.ringAddRemove(this._ring, [], [name], undefined, this._replicaHashes([name]), this.replicaPoints);
    delete this.servers[name];
    this.computeChecksum();
    this.emit('removed', name);
};

HashRing.prototype.computeChecksum = function computeChecksum() {
    if (this.hashFunc) this.checksum = this.hashFunc(Object.keys(this.servers).sort().join(';'));
    else this.checksum = addon.ringChecksum(this._ring);
    this.emit('checksumComputed');
};

HashRing.prototype.getServerCount = function getServerCount() { return addon.ringServerCount(this._ring); };
HashRing.prototype.hasServer = function hasServer(name) { return !!this.servers[name]; };

HashRing.prototype.lookupBatch = function lookupBatch(keys) {
    var idx;
    if (this.hashFunc) {
        var h = new Uint32Array(keys.length);
        for (var i = 0; i < keys.length; i++) h[i] = this.hashFunc(keys[i]) >>> 0;
        idx = addon.ringLookupHashes(this._ring, h);
    } else {
        idx = addon.ringLookup(this._ring, keys);
    }
    var out = new Array(idx.length);
    for (var j = 0; j < idx.length; j++) out[j] = addon.ringServerName(this._ring, idx[j]);
    return out;
};

HashRing.prototype.lookup = function lookup(str) { return this.lookupBatch([str])[0]; };

HashRing.prototype.lookupN = function lookupN(str, n) {
    var h = new Uint32Array([this.hashFunc ? this.hashFunc(str) >>> 0 : addon.hash32(String(str))]);
    var ring = this._ring;
    return Array.prototype.map.call(addon.ringLookupN(ring, h, n)[0], function (i) {
        return addon.ringServerName(ring, i);
    });
};

// handleOrProxyAll's keysByDest (index.js:642): _.groupBy(keys, ring.lookup) on
// the device -- dest keys in first-appearance order, keys in input order
// within a group, 'null' for an empty ring.
HashRing.prototype.groupByOwner = function groupByOwner(keys) {
    var arg = keys;
    if (this.hashFunc) {
        arg = new Uint32Array(keys.length);
        for (var i = 0; i < keys.length; i++) arg[i] = this.hashFunc(keys[i]) >>> 0;
    } else {
        arg = keys.map(String);
    }
    var g = addon.ringGroup(this._ring, arg), out = {};
    for (var q = 0; q < g[0].length; q++) {
        var dest = addon.ringServerName(this._ring, g[0][q]), list = [];
        for (var j = g[1][q]; j < g[1][q + 1]; j++) list.push(keys[g[2][j]]);
        out[dest] = list;
    }
    return out;
};

function SimCluster(opts) {
    if (!(this instanceof SimCluster)) return new SimCluster(opts);
    this.n = opts.n;
    this._sim = addon.simCreate({ n: opts.n, seed: opts.seed || 1,
                                  churnK: opts.churnK === undefined ? -1 : opts.churnK });
    this._addr = null;
}

// fail-stop `node` at the start of `round`; requests across `split` fail in [start, end)
SimCluster.prototype.fail = function fail(node, round) { addon.simFail(this._sim, node, round); };
SimCluster.prototype.partition = function partition(start, end, split) {
    addon.simPartition(this._sim, start, end, split);
};
SimCluster.prototype.round = function round(churn) { return addon.simRound(this._sim, churn !== false); };
SimCluster.prototype.run = function run(k, churn) { return addon.simRun(this._sim, k, churn !== false); };
SimCluster.prototype.checksums = function checksums() { return addon.simChecksums(this._sim, this.n); };
SimCluster.prototype.addresses = function addresses() {
    if (!this._addr) {
        this._addr = [];
        for (var i = 0; i < this.n; i++) this._addr.push(addon.simAddress(this._sim, i));
    }
    return this._addr;
};

// Read facade for node i, named after the reference objects it mirrors.
SimCluster.prototype.node = function node(i) {
    var sim = this._sim, n = this.n, addrs = this.addresses();
    var view = addon.simView(sim, n, i);
    var order = addon.simMembers(sim, n, i);
    var info = addon.simInfo(sim, i);
    var members = Array.prototype.map.call(order, function (a) {
        return { address: addrs[a], status: STATUS[view.status[a]], incarnationNumber: view.inc[a] };
    });
    var byAddr = {};
    members.forEach(function (m) { byAddr[m.address] = m; });
    var rows = addon.simChanges(sim, i);
    var changes = {};
    for (var r = 0; r < rows.length; r += 6) {
        var c = { source: rows[r + 2] < 0 ? undefined : addrs[rows[r + 2]],
                  sourceIncarnationNumber: rows[r + 3] === 0 ? undefined : rows[r + 3],
                  address: addrs[rows[r]], status: STATUS[rows[r + 4]], incarnationNumber: rows[r + 5] };
        if (rows[r + 1] >= 0) c.piggybackCount = rows[r + 1];
        changes[addrs[rows[r]]] = c;
    }
    var checksum = this.checksums()[i];
    return {
        address: addrs[i],
        membership: {
            checksum: checksum,
            members: members,
            findMemberByAddress: function (a) { return byAddr[a]; },
            getMemberCount: function () { return members.length; },
            generateChecksumString: function () {   // lib/membership.js:70-93
                return members.slice().sort(function (a, b) { return a.address < b.address ? -1 : a.address > b.address ? 1 : 0; })
                    .map(function (m) { return m.address + m.status + m.incarnationNumber; }).join(';');
            }
        },
        dissemination: { changes: changes, maxPiggybackCount: info.maxPiggybackCount },
        ring: { getServerCount: function () { return info.ringServerCount; }, checksum: info.ringChecksum },
        memberIterator: { currentIndex: info.iteratorIndex, currentRound: info.iteratorRound }
    };
};

// Wire-format bridge for node i: the JSON bodies ringpop puts on the wire
// (lib/swim/ping-sender.js:70-76, server/ping-handler.js:36-39), so a real
// ringpop process can gossip with simulated nodes.  Changes carry the issueAs
// copy's fields (lib/dissemination.js:170-177) minus the uuid `id`, which
// nothing on this path reads.
var STATUS_CODE = { alive: 1, suspect: 2, faulty: 3, leave: 4 };
SimCluster.prototype.wire = function wire(i) {
    var self = this, addrs = this.addresses(), index = {};
    addrs.forEach(function (a, k) { index[a] = k; });
    function toJson(rows) {
        var out = [];
        for (var r = 0; r < rows.length; r += 5) {
            var c = {};
            if (rows[r + 3] >= 0) c.source = addrs[rows[r + 3]];
            if (rows[r + 4]) c.sourceIncarnationNumber = rows[r + 4];
            c.address = addrs[rows[r]];
            c.status = STATUS[rows[r + 1]];
            c.incarnationNumber = rows[r + 2];
            out.push(c);
        }
        return out;
    }
    function toRows(changes) {
        var rows = new Float64Array(changes.length * 5);
        changes.forEach(function (c, k) {
            rows[5 * k] = index[c.address]; rows[5 * k + 1] = STATUS_CODE[c.status];
            rows[5 * k + 2] = c.incarnationNumber;
            rows[5 * k + 3] = c.source ? index[c.source] : -1;
            rows[5 * k + 4] = c.sourceIncarnationNumber || 0;
        });
        return rows;
    }
    return {
        // PingSender.send's body
        pingBody: function pingBody() {
            var b = addon.simPingBody(self._sim, self.n, i);
            return JSON.stringify({ checksum: b.checksum, changes: toJson(b.changes), source: addrs[i],
                                    sourceIncarnationNumber: b.incarnation });
        },
        // /protocol/ping (server/index.js:175-192 -> server/ping-handler.js:22-40)
        handlePing: function handlePing(body) {
            var b;
            try { b = JSON.parse(body); } catch (e) { b = null; }
            if (b === null || !b.source || !b.changes || !b.checksum) {
                throw new Error('need req body with source, changes, and checksum');
            }
            var src = index[b.source] === undefined ? -1 : index[b.source];
            var r = addon.simHandlePing(self._sim, self.n, i, src, b.sourceIncarnationNumber || 0, b.checksum,
                                        toRows(b.changes));
            return JSON.stringify({ changes: toJson(r.changes) });
        },
        // PingSender.onPing: Membership.update with the response's changes
        onPingResponse: function onPingResponse(res) {
            var b;
            try { b = JSON.parse(res); } catch (e) { b = null; }
            if (!b || !b.changes) return null;
            return addon.simUpdate(self._sim, i, toRows(b.changes));
        }
    };
};

module.exports = { farmhash: farmhash, HashRing: HashRing, SimCluster: SimCluster, addon: addon };
