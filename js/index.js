// ringpop_amd JavaScript host: drop-in surfaces for ringpop's hot path backed
// by the MI355X library through the N-API addon (js/ringpop_hip.node).
//
//   farmhash   -> replaces require('farmhash') (package.json:30): hash32(str)
//   HashRing   -> lib/ring.js:25-184 API (addServer, removeServer,
//                 addRemoveServers, computeChecksum, getServerCount,
//                 hasServer, lookup, lookupN, groupByOwner; events added / removed /
//                 checksumComputed) + lookupBatch for batched device lookups
//   Membership -> lib/membership.js:31-354 API (update, set, computeChecksum,
//                 generateChecksumString, make{Alive,Suspect,Faulty,Leave},
//                 findMemberByAddress, getMemberAt, getMemberCount,
//                 getIncarnationNumber, getJoinPosition, getRandomPingableMembers,
//                 hasMember, isPingable, shuffle, getStats, toString; fields
//                 members, membersByAddress, checksum, localMember,
//                 stashedUpdates; events checksumComputed / updated / set)
//   Dissemination -> lib/dissemination.js:27-184 API (issueAsSender,
//                 issueAsReceiver, fullSync, recordChange, clearChanges,
//                 adjustMaxPiggybackCount, resetMaxPiggybackCount,
//                 onRingChanged; fields changes, maxPiggybackCount,
//                 piggybackFactor; Defaults; event maxPiggybackCountAdjusted)
//                 -- one instance's state on the device (rp_node_*)
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
    if (this._lookupQ) this._resolveLookups(false);  // queued lookupAsync keys see the ring as it was
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
    if (this._lookupQ) this._resolveLookups(false);
    addon.ringAddRemove(this._ring, [name], [], this._replicaHashes([name]), undefined, this.replicaPoints);
    this.servers[name] = true;
    this.computeChecksum();
    this.emit('added', name);
};

HashRing.prototype.removeServer = function removeServer(name) {
    if (!this.hasServer(name)) return;
    if (this._lookupQ) this._resolveLookups(false);
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

// Scalar lookups coalesced per event-loop tick: every key asked for before
// the next setImmediate goes to the device in one lookupBatch launch, and each
// callback gets (err, owner) in call order, always on a later tick than the
// call.  For request routing (handleOrProxy, index.js:409-426) whose answer is
// asynchronous anyway: one launch per tick instead of one per request
// (INTEGRATION.md §5).  Answers are the ring's as of the lookupAsync call,
// like the reference's synchronous lookup: a ring change (addServer,
// removeServer, addRemoveServers) first resolves the keys queued before it.
HashRing.LOOKUP_FLUSH_KEYS = 65536;  // a batch this long is resolved at once
HashRing.prototype.lookupAsync = function lookupAsync(key, cb) {
    if (typeof cb !== 'function') throw new TypeError('lookupAsync needs a callback');
    var q = this._lookupQ;
    if (!q) {
        q = this._lookupQ = { keys: [], cbs: [] };
        var self = this;
        // (a later tick than every call of the batch: the callbacks run at once)
        setImmediate(function () { if (self._lookupQ === q) self._resolveLookups(true); });
    }
    q.keys.push(key);
    q.cbs.push(cb);
    if (q.keys.length >= HashRing.LOOKUP_FLUSH_KEYS) this._resolveLookups(false);
};
// Resolve the queued keys against the ring as it is now (one device batch);
// the callbacks run in call order, from setImmediate unless deliverNow (the
// batch's own setImmediate).  A callback that throws does not keep the others
// of its batch from running; the first error is rethrown after all of them.
HashRing.prototype._resolveLookups = function _resolveLookups(deliverNow) {
    var q = this._lookupQ;
    this._lookupQ = null;
    if (!q || !q.keys.length) return 0;
    var owners, err = null;
    try { owners = this.lookupBatch(q.keys); } catch (e) { err = e; }
    this.lookupBatches = (this.lookupBatches || 0) + 1;
    function deliver() {
        var thrown = null;
        for (var i = 0; i < q.cbs.length; i++) {
            try { q.cbs[i](err, err ? undefined : owners[i]); } catch (e) { if (thrown === null) thrown = e; }
        }
        if (thrown !== null) throw thrown;
    }
    if (deliverNow) deliver();
    else setImmediate(deliver);
    return q.keys.length;
};
// resolve the pending batch now (its callbacks still run on a later tick)
HashRing.prototype.flushLookups = function flushLookups() { return this._resolveLookups(false); };

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


// ---------------------------------------------------------------- one instance
// The device state of one ringpop process (rp_node): shared by its Membership
// and Dissemination, created on first use with ringpop.whoami().  Math.random
// for getJoinPosition / shuffle / sample is the instance's splitmix64 stream
// (DESIGN.md §3), seeded by options.seed (ringpop.membershipSeed) or from
// Math.random once.
var STATUS_CODE_M = { alive: 1, suspect: 2, faulty: 3, leave: 4 };
function DeviceNode(whoami, seed) {
    if (seed === undefined) seed = [Math.floor(Math.random() * 4294967296), Math.floor(Math.random() * 4294967296)];
    if (typeof seed === 'number') seed = [Math.floor(seed / 4294967296), seed >>> 0];
    this.h = addon.nodeCreate(whoami, seed[0] >>> 0, seed[1] >>> 0);
    this.names = [whoami];
    this.ids = new Map([[whoami, 0]]);
}
DeviceNode.of = function of(ringpop) {
    if (!ringpop.__rpDeviceNode) ringpop.__rpDeviceNode = new DeviceNode(ringpop.whoami(), ringpop.membershipSeed);
    return ringpop.__rpDeviceNode;
};
DeviceNode.prototype.intern = function intern(list) {
    var fresh = [], seen = new Set();
    for (var i = 0; i < list.length; i++) {
        var a = list[i];
        if (!this.ids.has(a) && !seen.has(a)) { seen.add(a); fresh.push(a); }
    }
    if (fresh.length) {
        var ids = addon.nodeIntern(this.h, fresh);
        for (var k = 0; k < fresh.length; k++) {
            if (ids[k] !== this.names.length) throw new Error('address interning out of step');
            this.ids.set(fresh[k], ids[k]);
            this.names.push(fresh[k]);
        }
    }
};
function incOf(x) {
    if (x === undefined || x === null) return -1;
    if (typeof x !== 'number' || !Number.isInteger(x) || x < 0 || x > 9007199254740991) {
        throw new TypeError('incarnation numbers must be non-negative integers: ' + x);
    }
    return x;
}
DeviceNode.prototype.rows = function rows(changes) {
    var need = [];
    changes.forEach(function (c) {
        if (c.address !== undefined && c.address !== null) need.push(String(c.address));
        if (c.source) need.push(String(c.source));
    });
    this.intern(need);
    var r = new Float64Array(changes.length * 6);
    for (var i = 0; i < changes.length; i++) {
        var c = changes[i];
        if (!STATUS_CODE_M[c.status]) throw new TypeError('unsupported member status: ' + c.status);
        r[6 * i] = c.address === undefined || c.address === null ? -1 : this.ids.get(String(c.address));
        r[6 * i + 1] = incOf(c.incarnationNumber);
        r[6 * i + 2] = c.source ? this.ids.get(String(c.source)) : -1;
        r[6 * i + 3] = incOf(c.sourceIncarnationNumber);
        r[6 * i + 4] = STATUS_CODE_M[c.status];
        r[6 * i + 5] = -1;
    }
    return r;
};
DeviceNode.prototype.change = function change(r, i) {
    var c = {};
    if (r[6 * i + 2] >= 0) c.source = this.names[r[6 * i + 2]];
    if (r[6 * i + 3] >= 0) c.sourceIncarnationNumber = r[6 * i + 3];
    c.address = this.names[r[6 * i]];
    c.status = STATUS[r[6 * i + 4]];
    c.incarnationNumber = r[6 * i + 1];
    return c;
};

function Member(address, status, incarnationNumber) {  // lib/member.js:22-33
    this.address = address;
    this.status = status;
    this.incarnationNumber = incarnationNumber;
}

function Membership(ringpop) {
    if (!(this instanceof Membership)) return new Membership(ringpop);
    EventEmitter.call(this);
    this.ringpop = ringpop;
    this.checksum = null;
    this.stashedUpdates = [];
    this._hasLocal = false;
    this._cache = null;
}
util.inherits(Membership, EventEmitter);
Membership.prototype._dev = function _dev() { return DeviceNode.of(this.ringpop); };
// members / membersByAddress are read from the device when they changed
Membership.prototype._view = function _view() {
    if (!this._cache) {
        var dev = this._dev(), m = addon.memberMembers(dev.h), list = new Array(m.ids.length), by = {};
        for (var i = 0; i < m.ids.length; i++) {
            var mem = new Member(dev.names[m.ids[i]], STATUS[m.status[i]], m.inc[i]);
            list[i] = mem;
            by[mem.address] = mem;
        }
        this._cache = { members: list, byAddress: by };
    }
    return this._cache;
};
Object.defineProperty(Membership.prototype, 'members', { get: function () { return this._view().members; } });
Object.defineProperty(Membership.prototype, 'membersByAddress', { get: function () { return this._view().byAddress; } });
Object.defineProperty(Membership.prototype, 'localMember', {
    get: function () { return this._hasLocal ? this.findMemberByAddress(this.ringpop.whoami()) : undefined; }
});

Membership.prototype.computeChecksum = function computeChecksum() {      // :41-64
    var start = new Date();
    this.checksum = addon.memberChecksum(this._dev().h);
    this.emit('checksumComputed');
    this.ringpop.stat('timing', 'compute-checksum', start);
    this.ringpop.stat('gauge', 'checksum', this.checksum);
    return this.checksum;
};
Membership.prototype.findMemberByAddress = function findMemberByAddress(address) { return this.membersByAddress[address]; };
Membership.prototype.generateChecksumString = function generateChecksumString() {  // :70-93
    return addon.memberChecksumString(this._dev().h);
};
Membership.prototype.getIncarnationNumber = function getIncarnationNumber() {
    return this.localMember && this.localMember.incarnationNumber;
};
Membership.prototype.getJoinPosition = function getJoinPosition() {     // :99-101, the instance's stream
    return Math.floor(addon.memberRandom(this._dev().h, 1)[0] * this.members.length);
};
Membership.prototype.getMemberAt = function getMemberAt(index) { return this.members[index]; };
Membership.prototype.getMemberCount = function getMemberCount() { return this.members.length; };
// :111-120 -- _.chain(members).reject(excluded).filter(isPingable).sample(n),
// sample as underscore 1.13 (partial Fisher-Yates) on the instance's stream
Membership.prototype.getRandomPingableMembers = function getRandomPingableMembers(n, excluding) {
    var self = this;
    var f = this.members.filter(function (m) { return excluding.indexOf(m.address) < 0 && self.isPingable(m); });
    var k = Math.max(Math.min(n, f.length), 0);
    var draws = addon.memberRandom(this._dev().h, k);
    for (var i = 0; i < k; i++) {
        var r = i + Math.floor(draws[i] * (f.length - i));
        var t = f[i]; f[i] = f[r]; f[r] = t;
    }
    return f.slice(0, k);
};
// :122-129 -- sorts `members` IN PLACE (later getMemberAt / iteration / shuffle
// see the sorted order), so the new order goes back to the device
Membership.prototype.getStats = function getStats() {
    var members = this.members, dev = this._dev();
    members.sort(function (a, b) { return a.address.localeCompare(b.address); });
    var ids = new Uint32Array(members.length);
    for (var i = 0; i < members.length; i++) ids[i] = dev.ids.get(members[i].address);
    addon.memberSetOrder(dev.h, ids);
    return { checksum: this.checksum, members: members };
};
Membership.prototype.hasMember = function hasMember(member) { return !!this.findMemberByAddress(member.address); };
Membership.prototype.isPingable = function isPingable(member) {
    return member.address !== this.ringpop.whoami() && (member.status === 'alive' || member.status === 'suspect');
};
Membership.prototype.makeAlive = function makeAlive(address, incarnationNumber) {
    return makeUpdate(this, address, incarnationNumber, 'alive', address === this.ringpop.whoami());
};
Membership.prototype.makeFaulty = function makeFaulty(address, incarnationNumber) {
    return makeUpdate(this, address, incarnationNumber, 'faulty');
};
Membership.prototype.makeLeave = function makeLeave(address, incarnationNumber) {
    return makeUpdate(this, address, incarnationNumber, 'leave');
};
Membership.prototype.makeSuspect = function makeSuspect(address, incarnationNumber) {
    return makeUpdate(this, address, incarnationNumber, 'suspect');
};

// :162-206 with mergeMembershipChangesets on the device
Membership.prototype.set = function set() {
    if (this.ringpop.isReady || this.stashedUpdates === null) return;
    if (!Array.isArray(this.stashedUpdates) || this.stashedUpdates.length === 0) return;
    var flat = [];
    this.stashedUpdates.forEach(function (cs) { flat.push.apply(flat, cs); });
    var dev = this._dev();
    var r = addon.memberSet(dev.h, dev.rows(flat));
    var updates = Array.prototype.map.call(r.winners, function (i) { return flat[i]; });
    this.stashedUpdates = null;
    this._cache = null;
    var start = new Date();  // (computeChecksum, :199 -> :41-64, ran inside memberSet)
    this.checksum = r.checksum;
    this.emit('checksumComputed');
    this.ringpop.stat('timing', 'compute-checksum', start);
    this.ringpop.stat('gauge', 'checksum', this.checksum);
    this.emit('set', updates);
};

// :208-313 on the device: rules, local override, unknown members spliced at
// getJoinPosition(); the returned list holds the caller's change objects,
// the local override rewritten in place as _.extend does (:246-251)
Membership.prototype.update = function update(changes, isLocal) {
    changes = Array.isArray(changes) ? changes : [changes];
    this.ringpop.stat('gauge', 'changes.apply', changes.length);
    if (changes.length === 0) return [];
    if (!isLocal && !this.ringpop.isReady) {
        if (Array.isArray(this.stashedUpdates)) this.stashedUpdates.push(changes);
        return [];
    }
    var dev = this._dev(), whoami = this.ringpop.whoami(), start = new Date();
    var res = addon.memberUpdate(dev.h, dev.rows(changes), Date.now());
    var updates = [];
    for (var i = 0; i < changes.length; i++) {
        if (!res.applied[i]) continue;
        var c = changes[i], st = STATUS[res.rows[6 * i + 4]], inc = res.rows[6 * i + 1];
        if (st !== c.status || (inc >= 0 && inc !== c.incarnationNumber)) {
            c.status = st;
            c.incarnationNumber = inc;
        }
        if (c.address === whoami && inc >= 0) this._hasLocal = true;
        updates.push(c);
    }
    this._cache = null;
    if (updates.length > 0) {
        this.checksum = res.checksum;  // computeChecksum (:266-268), done on the device with the merge
        this.emit('checksumComputed');
        this.ringpop.stat('timing', 'compute-checksum', start);
        this.ringpop.stat('gauge', 'checksum', this.checksum);
        this.emit('updated', updates);
    }
    return updates;
};
Membership.prototype.shuffle = function shuffle() {                     // :315-317
    addon.memberShuffle(this._dev().h);
    this._cache = null;
};
Membership.prototype.toString = function toString() {
    return JSON.stringify(this.members.map(function (m) { return m.address; }));
};

var uuid;
try { uuid = require('node-uuid'); } catch (e) {
    uuid = { v4: function () {
        var b = require('crypto').randomBytes(16);
        b[6] = (b[6] & 0x0f) | 0x40; b[8] = (b[8] & 0x3f) | 0x80;
        var h = b.toString('hex');
        return h.slice(0, 8) + '-' + h.slice(8, 12) + '-' + h.slice(12, 16) + '-' + h.slice(16, 20) + '-' + h.slice(20);
    } };
}
function makeUpdate(membership, address, incarnationNumber, status, isLocal) {  // :324-352
    var localMember = membership.localMember || { address: address, incarnationNumber: incarnationNumber };
    return membership.update({
        id: uuid.v4(), source: localMember.address, sourceIncarnationNumber: localMember.incarnationNumber,
        address: address, status: status, incarnationNumber: incarnationNumber, timestamp: Date.now()
    }, isLocal);
}

var LOG_10 = Math.log(10);
function Dissemination(ringpop) {
    if (!(this instanceof Dissemination)) return new Dissemination(ringpop);
    EventEmitter.call(this);
    this.ringpop = ringpop;
    this.ringpop.on('ringChanged', this.onRingChanged.bind(this));
    this.maxPiggybackCount = Dissemination.Defaults.maxPiggybackCount;
    this.piggybackFactor = Dissemination.Defaults.piggybackFactor;
    this._pending = [];   // recordChange calls not yet on the device (one batch per flush)
    this._ids = {};       // address -> id of its recorded change (the issueAs copy carries it)
}
util.inherits(Dissemination, EventEmitter);
Dissemination.Defaults = { maxPiggybackCount: 1, piggybackFactor: 15 };
Dissemination.prototype._dev = function _dev() { return DeviceNode.of(this.ringpop); };
Dissemination.prototype._flush = function _flush() {
    if (this._pending.length) {
        var dev = this._dev(), p = this._pending;
        this._pending = [];
        addon.dissRecord(dev.h, dev.rows(p));
    }
};
Dissemination.prototype.adjustMaxPiggybackCount = function adjustMaxPiggybackCount() {  // :38-55
    var serverCount = this.ringpop.ring.getServerCount();
    var prev = this.maxPiggybackCount;
    var next = this.piggybackFactor * Math.ceil(Math.log(serverCount + 1) / LOG_10);
    if (this.maxPiggybackCount !== next) {
        this.maxPiggybackCount = next;
        this.ringpop.stat('gauge', 'max-piggyback', this.maxPiggybackCount);
        this.ringpop.logger.debug('adjusted max piggyback count', {
            newPiggybackCount: next, oldPiggybackCount: prev, piggybackFactor: this.piggybackFactor,
            serverCount: serverCount });
        this.emit('maxPiggybackCountAdjusted');
    }
};
Dissemination.prototype.clearChanges = function clearChanges() {
    this._pending = [];
    this._ids = {};
    addon.dissClear(this._dev().h);
};
Dissemination.prototype._list = function _list(rows) {
    var dev = this._dev(), out = new Array(rows.length / 6);
    for (var i = 0; i < out.length; i++) {
        var c = dev.change(rows, i), o = { id: this._ids[c.address] };
        o.source = c.source; o.sourceIncarnationNumber = c.sourceIncarnationNumber;
        o.address = c.address; o.status = c.status; o.incarnationNumber = c.incarnationNumber;
        out[i] = o;
    }
    return out;
};
Dissemination.prototype.fullSync = function fullSync() {               // :61-76
    var dev = this._dev(), rows = addon.dissFullSync(dev.h), out = new Array(rows.length / 6);
    for (var i = 0; i < out.length; i++) {
        out[i] = { source: this.ringpop.whoami(), address: dev.names[rows[6 * i]], status: STATUS[rows[6 * i + 4]],
                   incarnationNumber: rows[6 * i + 1] };
    }
    return out;
};
Dissemination.prototype.issueAsSender = function issueAsSender() {     // :78-84
    this._flush();
    var list = this._list(addon.dissIssue(this._dev().h, this.maxPiggybackCount));
    this.ringpop.stat('gauge', 'changes.disseminate', list.length);
    return list;
};
Dissemination.prototype.issueAsReceiver = function issueAsReceiver(senderAddr, senderIncarnationNumber, senderChecksum) {
    this._flush();                                                      // :86-119
    var dev = this._dev();
    if (senderAddr) dev.intern([String(senderAddr)]);
    var src = senderAddr ? dev.ids.get(String(senderAddr)) : -1;
    var sinc = senderIncarnationNumber ? incOf(senderIncarnationNumber) : -1;
    var cs = typeof senderChecksum === 'number' ? senderChecksum : undefined;
    var r = addon.dissIssueReceiver(dev.h, src, sinc, cs, this.maxPiggybackCount);
    if (!r.fullSync) {
        var list = this._list(r.rows);
        this.ringpop.stat('gauge', 'changes.disseminate', list.length);
        return list;
    }
    this.ringpop.stat('gauge', 'changes.disseminate', 0);
    this.ringpop.stat('increment', 'full-sync');
    this.ringpop.logger.info('full sync', { local: this.ringpop.whoami(), localChecksum: this.ringpop.membership.checksum,
                                            dest: senderAddr, destChecksum: senderChecksum });
    var out = new Array(r.rows.length / 6);
    for (var i = 0; i < out.length; i++) {
        out[i] = { source: this.ringpop.whoami(), address: dev.names[r.rows[6 * i]], status: STATUS[r.rows[6 * i + 4]],
                   incarnationNumber: r.rows[6 * i + 1] };
    }
    return out;
};
Dissemination.prototype.onRingChanged = function onRingChanged() { this.adjustMaxPiggybackCount(); };
Dissemination.prototype.recordChange = function recordChange(change) {  // :125-127, batched to the device
    this._pending.push(change);
    this._ids[change.address] = change.id;
};
Dissemination.prototype.resetMaxPiggybackCount = function resetMaxPiggybackCount() {
    this.maxPiggybackCount = Dissemination.Defaults.maxPiggybackCount;
};
// Dissemination.changes: {address: change} in key order, with piggybackCount
Object.defineProperty(Dissemination.prototype, 'changes', {
    get: function () {
        this._flush();
        var dev = this._dev(), rows = addon.dissChanges(dev.h), out = {};
        for (var i = 0; i < rows.length / 6; i++) {
            var c = dev.change(rows, i), o = { id: this._ids[c.address] };
            o.source = c.source; o.sourceIncarnationNumber = c.sourceIncarnationNumber;
            o.address = c.address; o.status = c.status; o.incarnationNumber = c.incarnationNumber;
            if (rows[6 * i + 5] >= 0) o.piggybackCount = rows[6 * i + 5];
            out[c.address] = o;
        }
        return out;
    }
});

// opts.addresses: the instances' hostPorts (sorted; rp_sim_load_addresses);
// opts.views: {status: Int32Array, incarnation: Float64Array} rows of n, the
// join result each instance bootstraps from (rp_sim_set_views; status 0 = not
// a member); opts.joins: [[round, node, [seed, ...]], ...] (rp_sim_join)
function SimCluster(opts) {
    if (!(this instanceof SimCluster)) return new SimCluster(opts);
    this.n = opts.n;
    this._sim = addon.simCreate({ n: opts.n, seed: opts.seed || 1,
                                  churnK: opts.churnK === undefined ? -1 : opts.churnK });
    this._addr = null;
    if (opts.addresses) addon.simLoadAddresses(this._sim, opts.addresses);
    if (opts.joins && opts.joins.length) {
        var sp = Math.max.apply(null, opts.joins.map(function (e) { return e[2].length; }).concat([1]));
        var js = new Uint32Array(opts.joins.length), rs = new Uint32Array(opts.joins.length);
        var sd = new Int32Array(opts.joins.length * sp).fill(-1);
        opts.joins.forEach(function (e, k) {
            rs[k] = e[0]; js[k] = e[1];
            e[2].forEach(function (x, q) { sd[k * sp + q] = x; });
        });
        addon.simJoin(this._sim, js, rs, sd, sp);
    }
    if (opts.views) addon.simSetViews(this._sim, 0, opts.views.status, opts.views.incarnation);
}

// fail-stop `node` at the start of `round`; requests across `split` fail in [start, end)
SimCluster.prototype.fail = function fail(node, round) { addon.simFail(this._sim, node, round); };
SimCluster.prototype.partition = function partition(start, end, split) {
    addon.simPartition(this._sim, start, end, split);
};
SimCluster.prototype.round = function round(churn) { return addon.simRound(this._sim, churn !== false); };
SimCluster.prototype.run = function run(k, churn) { return addon.simRun(this._sim, k, churn !== false); };
// the same rounds off the event loop (napi_async_work): resolves with the
// cluster totals; the cluster is busy (every other call throws) until then
SimCluster.prototype.runAsync = function runAsync(k, churn) {
    if (this._busy) return Promise.reject(new Error('SimCluster: a runAsync is in flight'));
    var self = this;
    self._busy = true;
    return addon.simRunAsync(this._sim, k, churn !== false).then(function (st) {
        self._busy = false;
        return st;
    }, function (e) {
        self._busy = false;
        throw e;
    });
};
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

// while a runAsync is in flight the device cluster belongs to the worker
Object.keys(SimCluster.prototype).forEach(function (name) {
    if (name === 'runAsync') return;
    var f = SimCluster.prototype[name];
    SimCluster.prototype[name] = function () {
        if (this._busy) throw new Error('SimCluster.' + name + ': a runAsync is in flight');
        return f.apply(this, arguments);
    };
});

module.exports = { farmhash: farmhash, HashRing: HashRing, Membership: Membership, Dissemination: Dissemination,
                   Member: Member, SimCluster: SimCluster, addon: addon };
