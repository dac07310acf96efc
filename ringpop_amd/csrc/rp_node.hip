// ringpop_amd — one ringpop instance's Membership and Dissemination on the
// device (the drop-in surface of lib/membership.js and lib/dissemination.js;
// js/index.js and ringpop_amd/node.py wrap it with the reference's classes).
//
// Unlike the simulation (rp_sim.hip: N instances over one fixed address
// scheme, full views), an instance here holds arbitrary address strings,
// interned to dense ids in first-seen order, and starts from an empty member
// list: changes for unknown members are taken wholesale and spliced into
// `members` at getJoinPosition() (lib/membership.js:99-101,237-240,285-298).
//
// Kernels run as one 1024-thread workgroup (one instance, batches of tens to
// thousands of changes; the work is latency-bound, not bandwidth-bound):
//   k_node_update    Membership.update: rules + local override in parallel
//                    over runs of distinct addresses (host-split), new members'
//                    getJoinPosition draws in parallel (counter-based
//                    splitmix), then the splices resolved at once: in reverse
//                    insertion order each new member claims the p-th free slot
//                    of the final list (Fenwick tree in LDS), the old members
//                    fill the rest in order.
//   k_node_checksum  computeChecksum: the checksum string rendered in
//                    parallel (prefix sums over the address-sorted members),
//                    farmhash32 over it.
//   k_node_set       Membership.set: mergeMembershipChangesets (max
//                    incarnation per address, first appearance order).
//   k_node_record / k_node_issue / k_node_fullsync / k_node_clear:
//                    Dissemination's insertion-ordered change table.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "rp_block.h"
#include "rp_checksum.h"
#include "rp_whash.h"
#include "rp_common.h"
#include "rp_internal.h"

namespace rp {

constexpr int NB = 1024;        // threads of a node kernel
constexpr int NBW = NB / 64;
constexpr uint32_t FEN_LDS = 16384;  // Fenwick tree in LDS up to this many member slots

// rp_member_change with device-friendly names (same layout)
struct NChange {
    int64_t address, inc, source, source_inc;
    int32_t status, piggyback;
    int64_t reserved;
};
static_assert(sizeof(NChange) == 48, "rp_member_change is 48 bytes");

struct NodeDev {
    uint32_t cap;        // address ids
    uint64_t* vs;        // [cap] inc << 3 | status, 0 = not a member
    uint32_t* order;     // [cap] Membership.members (ids)
    uint32_t* tmp;       // [cap] scratch: the new member order
    uint32_t* fen;       // [cap + 1] scratch: Fenwick tree (lists > FEN_LDS)
    uint32_t* ins;       // [cap] ids inserted by the batch, in order
    uint32_t* pos;       // [cap] their join positions, then their final slots
    uint32_t* st;        // [8] members, log head, log tail, log live, checksum, string length, new members
    uint64_t* rng;       // [1] Math.random state (splitmix64)
    uint32_t* dpos;      // [cap] position of the address's key in the change log, NONE: no key
    NChange* dlog;       // [dcap] Dissemination.changes in key order (address -1: deleted)
    uint32_t dcap;
    const uint8_t* abytes;   // interned address strings
    const uint64_t* aoff;    // [nids + 1]
    const uint32_t* sorted;  // ids in JS string order (lib/membership.js:72-80)
    uint32_t nids;
    uint8_t* str;            // checksum string scratch
};
enum { NS_MEMBERS = 0, NS_HEAD, NS_TAIL, NS_LIVE, NS_CHECKSUM, NS_STRLEN, NS_NEW };

__device__ inline uint64_t nvalue(const NChange& c) { return pack_view((uint64_t)c.inc, (uint32_t)c.status); }

__device__ inline bool rules_apply(uint32_t ms, uint64_t mi, uint32_t cs, uint64_t ci) {
    // lib/membership-update-rules.js:25-59
    switch (cs) {
    case ST_ALIVE: return ci > mi;
    case ST_SUSPECT: return (ms == ST_SUSPECT && ci > mi) || (ms == ST_FAULTY && ci > mi) || (ms == ST_ALIVE && ci >= mi);
    case ST_FAULTY: return (ms == ST_SUSPECT && ci >= mi) || (ms == ST_FAULTY && ci > mi) || (ms == ST_ALIVE && ci >= mi);
    case ST_LEAVE: return ms != ST_LEAVE && ci >= mi;
    default: return false;
    }
}

// Exclusive rank of `flag` in thread order across the 1024-thread block and
// the block total (two barriers).
__device__ inline uint32_t nb_rank(bool flag, uint32_t* wc, uint32_t& total) {
    const uint64_t m = __ballot(flag);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t r = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wc[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NBW; i++) { const uint32_t c = wc[i]; off += i < w ? c : 0u; tot += c; }
    __syncthreads();
    total = tot;
    return off + r;
}
// Exclusive prefix sum of a per-thread value (thread order) and the total.
__device__ inline uint64_t nb_scan(uint64_t x, uint64_t* ws, uint64_t& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    uint64_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NBW; i++) { const uint64_t c = ws[i]; off += i < w ? c : 0ull; tot += c; }
    __syncthreads();
    total = tot;
    return off + incl - x;
}

// Membership.update(changes) (lib/membership.js:208-313) after the host's
// isReady / empty-batch checks.  seg[0..nseg] splits the batch into runs of
// distinct addresses (a later duplicate sees the earlier one's result, as the
// reference's sequential loop does).  Changes are rewritten in place by the
// local override (_.extend(change, assertion), :246-251); applied[i] = 1 for
// every change pushed onto the returned list.
__global__ void __launch_bounds__(NB) k_node_update(NodeDev D, NChange* ch, const uint32_t* seg, uint32_t nseg,
                                                    int64_t self, uint64_t now, uint8_t* applied) {
    __shared__ uint32_t wc[NBW];
    __shared__ uint32_t fen_lds[FEN_LDS + 1];
    const uint32_t L0 = D.st[NS_MEMBERS];
    const uint64_t rng0 = *D.rng;
    uint32_t m = 0;  // members inserted so far (uniform)
    for (uint32_t s = 0; s < nseg; s++) {
        const uint32_t lo = seg[s], hi = seg[s + 1];
        for (uint32_t c0 = lo; c0 < hi; c0 += NB) {
            const uint32_t i = c0 + threadIdx.x;
            bool ap = false, isnew = false;
            uint32_t id = NONE;
            if (i < hi) {
                NChange c = ch[i];
                if (c.address < 0) {
                    ap = true;  // undefined address: applyUpdate ignores it, update() still returns it (:237-240,277-283)
                } else {
                    id = (uint32_t)c.address;
                    const uint64_t cur = D.vs[id];
                    const uint32_t cs = v_status(cur), st = (uint32_t)c.status;
                    const bool inc_def = c.inc >= 0;
                    if (cs == ST_ABSENT) {  // first time seeing the member: take the change wholesale
                        ap = true;
                        if (inc_def) { isnew = true; D.vs[id] = nvalue(c); }
                    } else if ((int64_t)id == self && (st == ST_SUSPECT || st == ST_FAULTY)) {
                        ap = true;  // local override: reassert alive with Date.now() (:244-254)
                        c.status = ST_ALIVE;
                        c.inc = (int64_t)now;
                        ch[i].status = c.status;
                        ch[i].inc = c.inc;
                        D.vs[id] = nvalue(c);
                    } else if (inc_def && rules_apply(cs, v_inc(cur), st, (uint64_t)c.inc)) {
                        ap = true;
                        D.vs[id] = nvalue(c);
                    }
                }
                applied[i] = ap ? 1 : 0;
            }
            uint32_t tot;
            const uint32_t r = nb_rank(isnew, wc, tot);
            if (isnew) {
                // getJoinPosition(): floor(Math.random() * members.length), the
                // (m + r)-th draw of the instance's stream, members.length = L0 + m + r
                const uint32_t j = m + r;
                uint64_t s2 = rng0 + (uint64_t)j * 0x9E3779B97F4A7C15ULL;
                const double x = js_math_random(s2);
                D.ins[j] = id;
                D.pos[j] = (uint32_t)floor(__dmul_rn(x, (double)(L0 + j)));
            }
            m += tot;
        }
    }
    if (threadIdx.x == 0) { *D.rng = rng0 + (uint64_t)m * 0x9E3779B97F4A7C15ULL; D.st[NS_NEW] = m; }
    if (m == 0) return;
    // The splices, resolved at once.  Walking the insertions backwards, the
    // j-th new member sits at free slot pos[j] of the final list (later
    // inserts only shift it); claim it.  Old members fill the free slots left.
    const uint32_t T = L0 + m;
    uint32_t* fen = T <= FEN_LDS ? fen_lds : D.fen;
    for (uint32_t k = 1 + threadIdx.x; k <= T; k += NB) fen[k] = k & (0u - k);  // every slot free
    for (uint32_t k = threadIdx.x; k < T; k += NB) D.tmp[k] = NONE;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t top = 1;
        while (top * 2 <= T) top *= 2;
        for (uint32_t j = m; j-- > 0;) {
            uint32_t rem = D.pos[j], idx = 0;  // the (rem + 1)-th free slot
            for (uint32_t b = top; b; b >>= 1) {
                const uint32_t nx = idx + b;
                if (nx <= T && fen[nx] <= rem) { idx = nx; rem -= fen[nx]; }
            }
            for (uint32_t k = idx + 1; k <= T; k += k & (0u - k)) fen[k]--;
            D.tmp[idx] = D.ins[j];
        }
    }
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t c0 = 0; c0 < T; c0 += NB) {
        const uint32_t k = c0 + threadIdx.x;
        const bool fr = k < T && D.tmp[k] == NONE;
        uint32_t tot;
        const uint32_t r = nb_rank(fr, wc, tot);
        if (fr) D.tmp[k] = D.order[base + r];
        base += tot;
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < T; k += NB) D.order[k] = D.tmp[k];
    if (threadIdx.x == 0) D.st[NS_MEMBERS] = T;
}

// Membership.computeChecksum / generateChecksumString (lib/membership.js:
// 41-93): members in address order, address + status + incarnation joined by
// ';', rendered in parallel into D.str, then farmhash32 (one chain).
__device__ inline uint32_t nmember_len(const NodeDev& D, uint32_t id, uint64_t vs) {
    return (uint32_t)(D.aoff[id + 1] - D.aoff[id]) + status_len(v_status(vs)) + dec_len(v_inc(vs));
}
struct ByteEmit {
    uint8_t* p;
    __device__ inline void operator()(uint32_t w) {
        p[0] = (uint8_t)w; p[1] = (uint8_t)(w >> 8); p[2] = (uint8_t)(w >> 16); p[3] = (uint8_t)(w >> 24);
        p += 4;
    }
};
__global__ void __launch_bounds__(NB) k_node_checksum(NodeDev D) {
    __shared__ uint64_t ws[NBW];
    __shared__ __attribute__((aligned(16))) uint32_t hbuf[WH_BUF_WORDS];
    uint64_t run = 0, cnt = 0;
    for (uint32_t c0 = 0; c0 < D.nids; c0 += NB) {
        const uint32_t k = c0 + threadIdx.x;
        uint32_t id = NONE, len = 0;
        uint64_t vs = 0;
        if (k < D.nids) {
            id = D.sorted[k];
            vs = D.vs[id];
            if (v_status(vs) != ST_ABSENT) len = nmember_len(D, id, vs);
        }
        const bool present = len != 0;
        uint64_t tl, tc;
        // member q (q-th present) starts at sum(len of earlier) + q: one ';' after each earlier member
        const uint64_t bl = nb_scan(len, ws, tl), bc = nb_scan(present ? 1 : 0, ws, tc);
        if (present) {
            const uint64_t q = cnt + bc, o = run + bl + q;
            uint8_t* p = D.str + o;
            if (q) p[-1] = ';';
            const uint32_t L = (uint32_t)(D.aoff[id + 1] - D.aoff[id]);
            const uint8_t* a = D.abytes + D.aoff[id];
            for (uint32_t b = 0; b < L; b++) p[b] = a[b];
            WordSink<ByteEmit> w;
            w.emit.p = p + L;
            uint32_t w0, w1;
            int n1;
            status_words(v_status(vs), w0, w1, n1);
            w.put(w0, 4);
            w.put(w1, (uint32_t)n1);
            put_dec(w, v_inc(vs));
            for (uint32_t b = 0; b < w.bits / 8; b++) w.emit.p[b] = (uint8_t)(w.acc >> (8 * b));
        }
        run += tl;
        cnt += tc;
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // one wave hashes the string (rp_whash.h)
        const uint64_t total = cnt ? run + cnt - 1 : 0;
        const uint32_t h = wave_farmhash32(D.str, (uint32_t)total, hbuf);
        if (threadIdx.x == 0) {
            D.st[NS_STRLEN] = (uint32_t)total;
            D.st[NS_CHECKSUM] = h;
        }
    }
}

// Membership.set (lib/membership.js:162-206) with mergeMembershipChangesets
// (lib/membership-changeset-merge.js:22-51): per address (self skipped) the
// change with the largest incarnation, the first of equals; updates in the
// order addresses first appeared; each pushed at the end of `members`.
// win[id] / first[id] scratch: NONE-initialised by the host.  out[k] = index
// (into the flattened stash) of the k-th update.
__global__ void __launch_bounds__(NB) k_node_set(NodeDev D, const NChange* ch, uint32_t n, int64_t self,
                                                 unsigned long long* best, uint32_t* first, uint32_t* out,
                                                 uint32_t* nout) {
    __shared__ uint32_t wc[NBW];
    for (uint32_t i = threadIdx.x; i < n; i += NB) {
        const NChange c = ch[i];
        if (c.address < 0 || c.address == self) continue;
        atomicMin(&first[c.address], i);
        atomicMax(&best[c.address], (unsigned long long)c.inc);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += NB) {  // the first change carrying the best incarnation wins
        const NChange c = ch[i];
        if (c.address < 0 || c.address == self) continue;
        if ((unsigned long long)c.inc == best[c.address]) atomicMin(&D.tmp[c.address], i);
    }
    __syncthreads();
    const uint32_t L0 = D.st[NS_MEMBERS];
    uint32_t base = 0;
    for (uint32_t c0 = 0; c0 < n; c0 += NB) {
        const uint32_t i = c0 + threadIdx.x;
        bool head = false;
        int64_t a = -1;
        if (i < n) {
            a = ch[i].address;
            head = a >= 0 && a != self && first[a] == i;
        }
        uint32_t tot;
        const uint32_t r = nb_rank(head, wc, tot);
        if (head) {
            const uint32_t w = D.tmp[a];
            out[base + r] = w;
            D.order[L0 + base + r] = (uint32_t)a;
            D.vs[a] = nvalue(ch[w]);
        }
        base += tot;
    }
    if (threadIdx.x == 0) { D.st[NS_MEMBERS] = L0 + base; *nout = base; }
}

// Dissemination.recordChange (lib/dissemination.js:125-127) for a batch, in
// order: an existing key is overwritten in place (the new change object has
// no piggybackCount), a new key is appended.  seg: runs of distinct addresses.
__global__ void __launch_bounds__(NB) k_node_record(NodeDev D, const NChange* ch, const uint32_t* seg, uint32_t nseg) {
    __shared__ uint32_t wc[NBW];
    uint32_t tail = D.st[NS_TAIL], live = D.st[NS_LIVE];
    for (uint32_t s = 0; s < nseg; s++) {
        const uint32_t lo = seg[s], hi = seg[s + 1];
        for (uint32_t c0 = lo; c0 < hi; c0 += NB) {
            const uint32_t i = c0 + threadIdx.x;
            bool app = false;
            NChange c{};
            if (i < hi) {
                c = ch[i];
                c.piggyback = -1;
                const uint32_t p = D.dpos[c.address];
                if (p != NONE) D.dlog[p] = c;
                else app = true;
            }
            uint32_t tot;
            const uint32_t r = nb_rank(app, wc, tot);
            if (app) {
                D.dlog[tail + r] = c;
                D.dpos[c.address] = tail + r;
            }
            tail += tot;
            live += tot;
            __syncthreads();
        }
    }
    if (threadIdx.x == 0) { D.st[NS_TAIL] = tail; D.st[NS_LIVE] = live; }
}

// Squeeze deleted keys out of the log, keeping key order.
__global__ void __launch_bounds__(NB) k_node_compact(NodeDev D) {
    __shared__ uint32_t wc[NBW];
    const uint32_t head = D.st[NS_HEAD], tail = D.st[NS_TAIL];
    uint32_t out = 0;
    for (uint32_t c0 = head; c0 < tail; c0 += NB) {
        const uint32_t p = c0 + threadIdx.x;
        NChange e{};
        bool live = false;
        if (p < tail) { e = D.dlog[p]; live = e.address >= 0; }
        __syncthreads();  // (reads of this chunk before writes below it: out <= c0 - head + threadIdx)
        uint32_t tot;
        const uint32_t r = nb_rank(live, wc, tot);
        if (live) { D.dlog[out + r] = e; D.dpos[e.address] = out + r; }
        out += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) { D.st[NS_HEAD] = 0; D.st[NS_TAIL] = out; D.st[NS_LIVE] = out; }
}

// issueAs (lib/dissemination.js:138-182) in key order: an undefined count
// becomes 0; a change the receiver filter matches (:91-98) is skipped
// uncounted; otherwise counted, deleted past maxPiggybackCount, or copied out.
__global__ void __launch_bounds__(NB) k_node_issue(NodeDev D, int filter, int64_t fsrc, int64_t finc,
                                                   int32_t maxpb, NChange* out, uint32_t* nout) {
    __shared__ uint32_t wc[NBW];
    const uint32_t head = D.st[NS_HEAD], tail = D.st[NS_TAIL];
    uint32_t emitted = 0, deleted = 0, first_live = NONE;
    const bool do_filter = filter && fsrc >= 0 && finc > 0;
    for (uint32_t c0 = head; c0 < tail; c0 += NB) {
        const uint32_t p = c0 + threadIdx.x;
        bool em = false;
        NChange e{};
        if (p < tail) {
            e = D.dlog[p];
            if (e.address >= 0) {
                int32_t pc = e.piggyback < 0 ? 0 : e.piggyback;
                const bool filtered = do_filter && e.source >= 0 && e.source_inc > 0 && e.source == fsrc &&
                                      e.source_inc == finc;
                if (!filtered) {
                    pc += 1;
                    if (pc > maxpb) {  // :162-165 delete
                        D.dlog[p].address = -1;
                        D.dpos[e.address] = NONE;
                        deleted++;
                    } else {
                        em = true;
                    }
                }
                if (em || filtered) {
                    D.dlog[p].piggyback = pc;
                    first_live = min(first_live, p);
                }
            }
        }
        uint32_t tot;
        const uint32_t r = nb_rank(em, wc, tot);
        if (em) { e.piggyback = -1; out[emitted + r] = e; }
        emitted += tot;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) deleted += __shfl_xor(deleted, o);
    first_live = wave_min32(first_live);
    __shared__ uint32_t dl[NBW], fl[NBW];
    if ((threadIdx.x & 63) == 0) { dl[threadIdx.x >> 6] = deleted; fl[threadIdx.x >> 6] = first_live; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t d = 0, f = NONE;
        for (int i = 0; i < NBW; i++) { d += dl[i]; f = min(f, fl[i]); }
        D.st[NS_LIVE] -= d;
        D.st[NS_HEAD] = f == NONE ? tail : f;
        *nout = emitted;
    }
}

// Dissemination.fullSync (lib/dissemination.js:61-76): every member in
// `members` order, source = self, no sourceIncarnationNumber.
__global__ void k_node_fullsync(NodeDev D, int64_t self, NChange* out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= D.st[NS_MEMBERS]) return;
    const uint32_t id = D.order[k];
    const uint64_t vs = D.vs[id];
    NChange c{};
    c.address = id; c.status = (int32_t)v_status(vs); c.inc = (int64_t)v_inc(vs);
    c.source = self; c.source_inc = -1; c.piggyback = -1;
    out[k] = c;
}

// clearChanges (:57-59)
__global__ void k_node_clear(NodeDev D) {
    const uint32_t head = D.st[NS_HEAD], tail = D.st[NS_TAIL];
    for (uint32_t p = head + blockIdx.x * blockDim.x + threadIdx.x; p < tail; p += gridDim.x * blockDim.x) {
        const int64_t a = D.dlog[p].address;
        if (a >= 0) D.dpos[a] = NONE;
    }
}

// Membership.shuffle (lib/membership.js:315-317) -> _.shuffle (underscore
// 1.13, as the simulation's): swap(a[i], a[random(i, L-1)]) for i < L; draws
// computed in parallel from the counter-based stream, swaps applied in order.
__global__ void __launch_bounds__(NB) k_node_shuffle(NodeDev D) {
    __shared__ uint32_t tgt[NB];
    const uint32_t L = D.st[NS_MEMBERS];
    const uint64_t s0 = *D.rng;
    for (uint32_t c0 = 0; c0 < L; c0 += NB) {
        const uint32_t i = c0 + threadIdx.x;
        if (i < L) {
            uint64_t s = s0 + (uint64_t)i * 0x9E3779B97F4A7C15ULL;
            tgt[threadIdx.x] = (uint32_t)js_random_int(s, (int)i, (int)L - 1);
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (uint32_t j = 0; j < min((uint32_t)NB, L - c0); j++) {
                const uint32_t x = c0 + j, r = tgt[j];
                const uint32_t t = D.order[x];
                D.order[x] = D.order[r];
                D.order[r] = t;
            }
        __syncthreads();
    }
    if (threadIdx.x == 0) *D.rng = s0 + (uint64_t)L * 0x9E3779B97F4A7C15ULL;
}

// k Math.random() draws from the instance's stream (getRandomPingableMembers'
// _.sample and other host-side consumers share the stream with the device).
__global__ void k_node_random(NodeDev D, uint32_t k, double* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t s0 = *D.rng;
    if (i < k) {
        uint64_t s = s0 + (uint64_t)i * 0x9E3779B97F4A7C15ULL;
        out[i] = js_math_random(s);
    }
}
__global__ void k_node_rng_advance(NodeDev D, uint32_t k) { *D.rng += (uint64_t)k * 0x9E3779B97F4A7C15ULL; }

}  // namespace rp

// ===================================================================== host
using rp::DevBuf;
using rp::Error;
using rp::NChange;

struct rp_node {
    std::vector<std::string> names;
    std::unordered_map<std::string, uint32_t> index;
    std::vector<uint32_t> sorted;  // ids by JS `<` (bytewise for the addresses ringpop uses)
    std::string blob;
    std::vector<uint64_t> offs{0};
    int64_t self = -1;
    bool names_dirty = true;
    uint32_t cap = 0;
    hipStream_t st = nullptr;
    DevBuf<uint64_t> vs, rng;
    DevBuf<uint32_t> order, tmp, fen, ins, pos, stt, dpos, sorted_d;
    DevBuf<NChange> dlog;
    DevBuf<uint8_t> abytes, str;
    DevBuf<uint64_t> aoff;
    uint32_t members = 0, checksum = 0, strlen_ = 0;
    bool checksum_known = false;  // Membership.checksum: null until the first computeChecksum
    uint64_t str_cap = 0;

    ~rp_node() {
        if (st) (void)hipStreamDestroy(st);
    }

    rp::NodeDev dev() {
        rp::NodeDev D{};
        D.cap = cap; D.vs = vs.p; D.order = order.p; D.tmp = tmp.p; D.fen = fen.p; D.ins = ins.p; D.pos = pos.p;
        D.st = stt.p; D.rng = rng.p; D.dpos = dpos.p; D.dlog = dlog.p; D.dcap = (uint32_t)dlog.n;
        D.abytes = abytes.p; D.aoff = aoff.p; D.sorted = sorted_d.p; D.nids = (uint32_t)names.size(); D.str = str.p;
        return D;
    }

    // capacity for `need` ids: device arrays are reallocated and copied
    void grow(uint32_t need) {
        if (need <= cap) return;
        uint32_t nc = std::max<uint32_t>(1024, cap);
        while (nc < need) nc *= 2;
        auto regrow32 = [&](DevBuf<uint32_t>& b, uint32_t fill_byte, bool keep) {
            DevBuf<uint32_t> nb(nc + 1);
            RP_HIP(hipMemsetAsync(nb.p, fill_byte, nb.bytes(), st));
            if (keep && b.p) RP_HIP(hipMemcpyAsync(nb.p, b.p, b.bytes(), hipMemcpyDeviceToDevice, st));
            b = std::move(nb);
        };
        DevBuf<uint64_t> nvs(nc);
        RP_HIP(hipMemsetAsync(nvs.p, 0, nvs.bytes(), st));
        if (vs.p) RP_HIP(hipMemcpyAsync(nvs.p, vs.p, vs.bytes(), hipMemcpyDeviceToDevice, st));
        vs = std::move(nvs);
        regrow32(order, 0, true);
        regrow32(dpos, 0xFF, true);
        regrow32(tmp, 0xFF, false);
        regrow32(fen, 0, false);
        regrow32(ins, 0, false);
        regrow32(pos, 0, false);
        // the change log holds at most one live key per address; 2 x ids
        // leaves room for deleted keys between compactions
        DevBuf<NChange> nl((size_t)2 * nc);
        if (dlog.p) RP_HIP(hipMemcpyAsync(nl.p, dlog.p, dlog.bytes(), hipMemcpyDeviceToDevice, st));
        dlog = std::move(nl);
        cap = nc;
    }

    uint32_t intern(const char* b, size_t l) {
        // the checksum string orders members bytewise; the reference compares
        // with JS `<` (UTF-16 code units, lib/membership.js:72-80).  The two
        // agree on ASCII, which is all RingPop's host:port addresses hold.
        for (size_t i = 0; i < l; i++)
            if ((unsigned char)b[i] < 0x20 || (unsigned char)b[i] > 0x7E)
                throw Error(RP_ERR_INVALID, "addresses must be printable ASCII");
        std::string s(b, l);
        auto it = index.find(s);
        if (it != index.end()) return it->second;
        const uint32_t id = (uint32_t)names.size();
        names.push_back(s);
        index.emplace(std::move(s), id);
        blob.append(b, l);
        offs.push_back(blob.size());
        names_dirty = true;
        return id;
    }

    // the address table and its sort order on the device (after interning)
    void sync_names() {
        if (!names_dirty) return;
        grow((uint32_t)names.size());
        const size_t old = sorted.size();
        for (size_t i = old; i < names.size(); i++) sorted.push_back((uint32_t)i);
        auto lt = [&](uint32_t a, uint32_t b) { return names[a] < names[b]; };
        std::sort(sorted.begin() + old, sorted.end(), lt);
        std::inplace_merge(sorted.begin(), sorted.begin() + old, sorted.end(), lt);
        abytes.alloc(blob.size() + 8);
        aoff.alloc(offs.size());
        sorted_d.alloc(std::max<size_t>(sorted.size(), 1));
        if (!blob.empty()) RP_HIP(hipMemcpyAsync(abytes.p, blob.data(), blob.size(), hipMemcpyHostToDevice, st));
        RP_HIP(hipMemcpyAsync(aoff.p, offs.data(), offs.size() * 8, hipMemcpyHostToDevice, st));
        if (!sorted.empty())
            RP_HIP(hipMemcpyAsync(sorted_d.p, sorted.data(), sorted.size() * 4, hipMemcpyHostToDevice, st));
        // the checksum string: every name once plus "suspect" + 16 digits + ';' per member
        const uint64_t need = blob.size() + 24 * (uint64_t)names.size() + 64;
        if (need > str_cap) { str.alloc(need * 2); str_cap = need * 2; }
        RP_HIP(hipStreamSynchronize(st));  // host vectors may change before the copies run
        names_dirty = false;
    }

    void check_ids(const NChange* c, uint32_t n, bool allow_undefined) {
        for (uint32_t i = 0; i < n; i++) {
            if (c[i].address >= (int64_t)names.size() || (c[i].address < 0 && !allow_undefined))
                throw Error(RP_ERR_INVALID, "change " + std::to_string(i) + ": address id not interned");
            if (c[i].status < rp::ST_ALIVE || c[i].status > rp::ST_LEAVE)
                throw Error(RP_ERR_UNSUPPORTED, "change " + std::to_string(i) + ": status must be alive, suspect, "
                                                "faulty or leave");
            if (c[i].inc >= (1ll << 53) || c[i].source >= (int64_t)names.size())
                throw Error(RP_ERR_INVALID, "change " + std::to_string(i) + ": incarnation or source out of range");
        }
    }

    // runs of distinct addresses (NONE-free ids), as segment starts + end
    std::vector<uint32_t> segments(const NChange* c, uint32_t n) {
        std::vector<uint32_t> seg{0};
        std::vector<uint32_t> mark(names.size(), NONE_U32);
        uint32_t cur = 0;
        for (uint32_t i = 0; i < n; i++) {
            if (c[i].address < 0) continue;
            uint32_t& m = mark[(size_t)c[i].address];
            if (m == cur) { seg.push_back(i); cur++; }
            m = cur;
        }
        seg.push_back(n);
        return seg;
    }
    static constexpr uint32_t NONE_U32 = 0xFFFFFFFFu;

    // distinct addresses of a batch (ids already checked)
    uint32_t distinct(const NChange* c, uint32_t n) {
        std::vector<uint8_t> seen(names.size(), 0);
        uint32_t k = 0;
        for (uint32_t i = 0; i < n; i++) {
            if (c[i].address < 0) continue;
            uint8_t& s = seen[(size_t)c[i].address];
            k += s == 0;
            s = 1;
        }
        return k;
    }

    void read_state() {
        uint32_t h[8];
        RP_HIP(hipMemcpyAsync(h, stt.p, sizeof h, hipMemcpyDeviceToHost, st));
        RP_HIP(hipStreamSynchronize(st));
        members = h[rp::NS_MEMBERS];
    }

    void compute_checksum() {
        sync_names();
        hipLaunchKernelGGL(rp::k_node_checksum, dim3(1), dim3(rp::NB), 0, st, dev());
        RP_HIP(hipGetLastError());
        uint32_t h[8];
        RP_HIP(hipMemcpyAsync(h, stt.p, sizeof h, hipMemcpyDeviceToHost, st));
        RP_HIP(hipStreamSynchronize(st));
        checksum = h[rp::NS_CHECKSUM];
        strlen_ = h[rp::NS_STRLEN];
        members = h[rp::NS_MEMBERS];
        checksum_known = true;
    }

    // the log has room for n appends (compacting when needed)
    void reserve_log(uint32_t n) {
        uint32_t h[8];
        RP_HIP(hipMemcpyAsync(h, stt.p, sizeof h, hipMemcpyDeviceToHost, st));
        RP_HIP(hipStreamSynchronize(st));
        if ((uint64_t)h[rp::NS_TAIL] + n <= dlog.n) return;
        hipLaunchKernelGGL(rp::k_node_compact, dim3(1), dim3(rp::NB), 0, st, dev());
        RP_HIP(hipGetLastError());
        RP_HIP(hipMemcpyAsync(h, stt.p, sizeof h, hipMemcpyDeviceToHost, st));
        RP_HIP(hipStreamSynchronize(st));
        if ((uint64_t)h[rp::NS_TAIL] + n > dlog.n) throw Error(RP_ERR_STATE, "change log overflow");
    }
};

static rp_node* node_of(rp_node* m) {
    if (!m) throw Error(RP_ERR_INVALID, "null node");
    RP_HIP(hipSetDevice(rp::current_device()));
    return m;
}

extern "C" {

int rp_node_create(const uint8_t* self, size_t len, uint64_t rng_state, rp_node** out) {
    return rp::guarded([&] {
        if (!out || (!self && len)) throw Error(RP_ERR_INVALID, "null pointer");
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
            throw Error(RP_ERR_HIP, "no HIP device available (ringpop_amd requires an MI355X / gfx950 GPU)");
        RP_HIP(hipSetDevice(rp::current_device()));
        std::unique_ptr<rp_node> m(new rp_node());
        RP_HIP(hipStreamCreateWithFlags(&m->st, hipStreamNonBlocking));
        m->stt.alloc(8);
        m->rng.alloc(1);
        RP_HIP(hipMemsetAsync(m->stt.p, 0, 32, m->st));
        RP_HIP(hipMemcpyAsync(m->rng.p, &rng_state, 8, hipMemcpyHostToDevice, m->st));
        m->self = (int64_t)m->intern((const char*)self, len);
        m->sync_names();
        *out = m.release();
    });
}

int rp_node_destroy(rp_node* m) {
    delete m;
    return RP_OK;
}

int rp_node_intern(rp_node* m, const uint8_t* bytes, const uint64_t* offsets, size_t n, uint32_t* ids) {
    return rp::guarded([&] {
        node_of(m);
        if (n && (!bytes || !offsets || !ids)) throw Error(RP_ERR_INVALID, "null pointer");
        for (size_t i = 0; i < n; i++)  // (all or none interned)
            for (uint64_t j = offsets[i]; j < offsets[i + 1]; j++)
                if (bytes[j] < 0x20 || bytes[j] > 0x7E) throw Error(RP_ERR_INVALID, "addresses must be printable ASCII");
        for (size_t i = 0; i < n; i++)
            ids[i] = m->intern((const char*)bytes + offsets[i], offsets[i + 1] - offsets[i]);
        if (m->names.size() >= 0x7FFFFFFFu) throw Error(RP_ERR_CAPACITY, "too many addresses");
    });
}

int rp_node_address(rp_node* m, uint32_t id, char* buf, size_t cap, size_t* len) {
    if (!m || id >= m->names.size()) return RP_ERR_INVALID;
    const std::string& s = m->names[id];
    if (len) *len = s.size();
    if (buf) {
        if (cap < s.size() + 1) return RP_ERR_INVALID;
        memcpy(buf, s.c_str(), s.size() + 1);
    }
    return RP_OK;
}

int rp_node_rng(rp_node* m, uint64_t* get, const uint64_t* set) {
    return rp::guarded([&] {
        node_of(m);
        if (set) RP_HIP(hipMemcpyAsync(m->rng.p, set, 8, hipMemcpyHostToDevice, m->st));
        if (get) RP_HIP(hipMemcpyAsync(get, m->rng.p, 8, hipMemcpyDeviceToHost, m->st));
        RP_HIP(hipStreamSynchronize(m->st));
    });
}

int rp_membership_update(rp_node* m, rp_member_change* changes, uint32_t n, uint64_t now, uint8_t* applied,
                         uint32_t* napplied, uint32_t* checksum) {
    return rp::guarded([&] {
        node_of(m);
        if (n && (!changes || !applied)) throw Error(RP_ERR_INVALID, "null pointer");
        NChange* c = (NChange*)changes;
        m->check_ids(c, n, true);
        m->sync_names();
        uint32_t na = 0;
        if (n) {
            const std::vector<uint32_t> seg = m->segments(c, n);
            DevBuf<NChange> dc(n);
            DevBuf<uint32_t> ds(seg.size());
            DevBuf<uint8_t> da(n);
            RP_HIP(hipMemcpyAsync(dc.p, c, n * sizeof(NChange), hipMemcpyHostToDevice, m->st));
            RP_HIP(hipMemcpyAsync(ds.p, seg.data(), seg.size() * 4, hipMemcpyHostToDevice, m->st));
            hipLaunchKernelGGL(rp::k_node_update, dim3(1), dim3(rp::NB), 0, m->st, m->dev(), dc.p, (const uint32_t*)ds.p,
                               (uint32_t)(seg.size() - 1), m->self, now, da.p);
            RP_HIP(hipGetLastError());
            RP_HIP(hipMemcpyAsync(c, dc.p, n * sizeof(NChange), hipMemcpyDeviceToHost, m->st));
            RP_HIP(hipMemcpyAsync(applied, da.p, n, hipMemcpyDeviceToHost, m->st));
            RP_HIP(hipStreamSynchronize(m->st));
            for (uint32_t i = 0; i < n; i++) na += applied[i] != 0;
        }
        // computeChecksum when anything applied (lib/membership.js:266-268)
        if (na) m->compute_checksum();
        else m->read_state();
        if (napplied) *napplied = na;
        if (checksum) *checksum = m->checksum;
    });
}

int rp_membership_set(rp_node* m, const rp_member_change* stash, uint32_t n, uint32_t* winners, uint32_t* nwinners,
                      uint32_t* checksum) {
    return rp::guarded([&] {
        node_of(m);
        if (n && (!stash || !winners)) throw Error(RP_ERR_INVALID, "null pointer");
        const NChange* c = (const NChange*)stash;
        m->check_ids(c, n, true);
        for (uint32_t i = 0; i < n; i++)
            if (c[i].inc < 0) throw Error(RP_ERR_UNSUPPORTED, "set(): changes need an incarnation number");
        m->sync_names();
        m->read_state();
        {
            // set() pushes every merged address; one already a member would be
            // listed twice by the reference -- not modelled
            std::vector<uint32_t> ids(m->members);
            if (m->members) RP_HIP(hipMemcpy(ids.data(), m->order.p, m->members * 4, hipMemcpyDeviceToHost));
            std::vector<uint8_t> present(m->names.size(), 0);
            for (uint32_t id : ids) present[id] = 1;
            for (uint32_t i = 0; i < n; i++)
                if (c[i].address >= 0 && c[i].address != m->self && present[(size_t)c[i].address])
                    throw Error(RP_ERR_UNSUPPORTED, "set(): an update for an existing member");
        }
        uint32_t nw = 0;
        if (n) {
            DevBuf<NChange> dc(n);
            DevBuf<unsigned long long> best(m->cap);
            DevBuf<uint32_t> first(m->cap), out(n), dn(1);
            RP_HIP(hipMemcpyAsync(dc.p, c, n * sizeof(NChange), hipMemcpyHostToDevice, m->st));
            RP_HIP(hipMemsetAsync(best.p, 0, best.bytes(), m->st));
            RP_HIP(hipMemsetAsync(first.p, 0xFF, first.bytes(), m->st));
            RP_HIP(hipMemsetAsync(m->tmp.p, 0xFF, m->tmp.bytes(), m->st));
            hipLaunchKernelGGL(rp::k_node_set, dim3(1), dim3(rp::NB), 0, m->st, m->dev(), (const NChange*)dc.p, n, m->self,
                               best.p, first.p, out.p, dn.p);
            RP_HIP(hipGetLastError());
            RP_HIP(hipMemcpyAsync(&nw, dn.p, 4, hipMemcpyDeviceToHost, m->st));
            RP_HIP(hipStreamSynchronize(m->st));
            if (nw) RP_HIP(hipMemcpy(winners, out.p, nw * 4, hipMemcpyDeviceToHost));
        }
        m->compute_checksum();
        if (nwinners) *nwinners = nw;
        if (checksum) *checksum = m->checksum;
    });
}

int rp_membership_checksum(rp_node* m, uint32_t* checksum) {
    return rp::guarded([&] {
        node_of(m);
        if (!checksum) throw Error(RP_ERR_INVALID, "null pointer");
        m->compute_checksum();
        *checksum = m->checksum;
    });
}

int rp_membership_checksum_string(rp_node* m, char* buf, size_t cap, size_t* len) {
    return rp::guarded([&] {
        node_of(m);
        m->compute_checksum();
        if (len) *len = m->strlen_;
        if (!buf) return;
        if (cap < (size_t)m->strlen_ + 1) throw Error(RP_ERR_INVALID, "buffer too small");
        if (m->strlen_) RP_HIP(hipMemcpy(buf, m->str.p, m->strlen_, hipMemcpyDeviceToHost));
        buf[m->strlen_] = 0;
    });
}

int rp_membership_members(rp_node* m, uint32_t* ids, uint8_t* status, uint64_t* inc, size_t cap, uint32_t* count) {
    return rp::guarded([&] {
        node_of(m);
        m->read_state();
        if (count) *count = m->members;
        if (!ids && !status && !inc) return;
        if (cap < m->members) throw Error(RP_ERR_INVALID, "buffers hold fewer entries than members");
        std::vector<uint32_t> ord(m->members);
        std::vector<uint64_t> v(m->cap);
        if (m->members) RP_HIP(hipMemcpy(ord.data(), m->order.p, m->members * 4, hipMemcpyDeviceToHost));
        RP_HIP(hipMemcpy(v.data(), m->vs.p, (size_t)m->cap * 8, hipMemcpyDeviceToHost));
        for (uint32_t k = 0; k < m->members; k++) {
            if (ids) ids[k] = ord[k];
            if (status) status[k] = (uint8_t)rp::v_status(v[ord[k]]);
            if (inc) inc[k] = rp::v_inc(v[ord[k]]);
        }
    });
}

int rp_membership_force(rp_node* m, uint32_t id, int status, uint64_t inc) {
    return rp::guarded([&] {
        node_of(m);
        if (id >= m->names.size() || status < rp::ST_ALIVE || status > rp::ST_LEAVE)
            throw Error(RP_ERR_INVALID, "bad member or status");
        m->sync_names();
        uint64_t cur = 0;
        RP_HIP(hipMemcpy(&cur, m->vs.p + id, 8, hipMemcpyDeviceToHost));
        if (rp::v_status(cur) == rp::ST_ABSENT) throw Error(RP_ERR_INVALID, "not a member");
        const uint64_t v = rp::pack_view(inc, (uint32_t)status);
        RP_HIP(hipMemcpy(m->vs.p + id, &v, 8, hipMemcpyHostToDevice));  // (checksum untouched, as for a mutated Member)
    });
}

int rp_membership_shuffle(rp_node* m) {
    return rp::guarded([&] {
        node_of(m);
        m->sync_names();
        hipLaunchKernelGGL(rp::k_node_shuffle, dim3(1), dim3(rp::NB), 0, m->st, m->dev());
        RP_HIP(hipGetLastError());
        RP_HIP(hipStreamSynchronize(m->st));
    });
}

int rp_membership_set_order(rp_node* m, const uint32_t* ids, uint32_t count) {
    return rp::guarded([&] {
        node_of(m);
        m->read_state();
        if (count != m->members) throw Error(RP_ERR_INVALID, "the order must list every member once");
        if (!count) return;
        if (!ids) throw Error(RP_ERR_INVALID, "null pointer");
        std::vector<uint32_t> cur(count);
        RP_HIP(hipMemcpy(cur.data(), m->order.p, count * 4, hipMemcpyDeviceToHost));
        std::vector<uint8_t> mark(m->names.size(), 0);
        for (uint32_t id : cur) mark[id] = 1;
        for (uint32_t k = 0; k < count; k++) {
            if (ids[k] >= m->names.size() || mark[ids[k]] != 1)
                throw Error(RP_ERR_INVALID, "the order must be a permutation of the members");
            mark[ids[k]] = 2;
        }
        RP_HIP(hipMemcpy(m->order.p, ids, count * 4, hipMemcpyHostToDevice));
    });
}

int rp_membership_random(rp_node* m, uint32_t k, double* out) {
    return rp::guarded([&] {
        node_of(m);
        if (k && !out) throw Error(RP_ERR_INVALID, "null pointer");
        if (!k) return;
        DevBuf<double> d(k);
        hipLaunchKernelGGL(rp::k_node_random, dim3(rp::grid_for(k, 256)), dim3(256), 0, m->st, m->dev(), k, d.p);
        hipLaunchKernelGGL(rp::k_node_rng_advance, dim3(1), dim3(1), 0, m->st, m->dev(), k);
        RP_HIP(hipGetLastError());
        RP_HIP(hipMemcpyAsync(out, d.p, k * 8, hipMemcpyDeviceToHost, m->st));
        RP_HIP(hipStreamSynchronize(m->st));
    });
}

int rp_dissemination_record(rp_node* m, const rp_member_change* changes, uint32_t n) {
    return rp::guarded([&] {
        node_of(m);
        if (!n) return;
        if (!changes) throw Error(RP_ERR_INVALID, "null pointer");
        const NChange* c = (const NChange*)changes;
        m->check_ids(c, n, false);
        m->sync_names();
        const std::vector<uint32_t> seg = m->segments(c, n);
        // room for the batch's new keys: at most one per distinct address
        // (recordChange upserts by address, lib/dissemination.js:125-127), so
        // a batch that repeats a few addresses never outgrows the log
        m->reserve_log(m->distinct(c, n));
        DevBuf<NChange> dc(n);
        DevBuf<uint32_t> ds(seg.size());
        RP_HIP(hipMemcpyAsync(dc.p, c, n * sizeof(NChange), hipMemcpyHostToDevice, m->st));
        RP_HIP(hipMemcpyAsync(ds.p, seg.data(), seg.size() * 4, hipMemcpyHostToDevice, m->st));
        hipLaunchKernelGGL(rp::k_node_record, dim3(1), dim3(rp::NB), 0, m->st, m->dev(), (const NChange*)dc.p,
                           (const uint32_t*)ds.p, (uint32_t)(seg.size() - 1));
        RP_HIP(hipGetLastError());
        RP_HIP(hipStreamSynchronize(m->st));
    });
}

static void node_issue(rp_node* m, int filter, int64_t src, int64_t src_inc, int32_t maxpb, NChange* out, size_t cap,
                       uint32_t* count) {
    m->sync_names();
    uint32_t h[8];
    RP_HIP(hipMemcpyAsync(h, m->stt.p, sizeof h, hipMemcpyDeviceToHost, m->st));
    RP_HIP(hipStreamSynchronize(m->st));
    // a list never exceeds the live keys: check the buffer before counts move
    if (h[rp::NS_LIVE] && (!out || cap < h[rp::NS_LIVE])) throw Error(RP_ERR_INVALID, "changes buffer too small");
    DevBuf<NChange> dout(std::max<uint32_t>(h[rp::NS_LIVE], 1));
    DevBuf<uint32_t> dn(1);
    hipLaunchKernelGGL(rp::k_node_issue, dim3(1), dim3(rp::NB), 0, m->st, m->dev(), filter, src, src_inc, maxpb, dout.p,
                       dn.p);
    RP_HIP(hipGetLastError());
    uint32_t k = 0;
    RP_HIP(hipMemcpyAsync(&k, dn.p, 4, hipMemcpyDeviceToHost, m->st));
    RP_HIP(hipStreamSynchronize(m->st));
    if (k) RP_HIP(hipMemcpy(out, dout.p, k * sizeof(NChange), hipMemcpyDeviceToHost));
    *count = k;
}

int rp_dissemination_issue(rp_node* m, int32_t max_piggyback, rp_member_change* out, size_t cap, uint32_t* count) {
    return rp::guarded([&] {
        node_of(m);
        if (!count) throw Error(RP_ERR_INVALID, "null pointer");
        node_issue(m, 0, -1, -1, max_piggyback, (NChange*)out, cap, count);
    });
}

int rp_dissemination_full_sync(rp_node* m, rp_member_change* out, size_t cap, uint32_t* count) {
    return rp::guarded([&] {
        node_of(m);
        if (!count) throw Error(RP_ERR_INVALID, "null pointer");
        m->read_state();
        *count = m->members;
        if (!m->members) return;
        if (!out || cap < m->members) throw Error(RP_ERR_INVALID, "changes buffer too small");
        DevBuf<NChange> d(m->members);
        hipLaunchKernelGGL(rp::k_node_fullsync, dim3(rp::grid_for(m->members, 256)), dim3(256), 0, m->st, m->dev(),
                           m->self, d.p);
        RP_HIP(hipGetLastError());
        RP_HIP(hipMemcpyAsync(out, d.p, m->members * sizeof(NChange), hipMemcpyDeviceToHost, m->st));
        RP_HIP(hipStreamSynchronize(m->st));
    });
}

int rp_dissemination_issue_as_receiver(rp_node* m, int64_t sender, int64_t sender_inc, uint32_t sender_checksum,
                                       int has_checksum, int32_t max_piggyback, rp_member_change* out, size_t cap,
                                       uint32_t* count, int* full_sync) {
    return rp::guarded([&] {
        node_of(m);
        if (!count) throw Error(RP_ERR_INVALID, "null pointer");
        if (sender >= (int64_t)m->names.size()) throw Error(RP_ERR_INVALID, "sender id not interned");
        m->read_state();
        uint32_t h[8];
        RP_HIP(hipMemcpy(h, m->stt.p, sizeof h, hipMemcpyDeviceToHost));
        // the response is a list or a fullSync: check the buffer before any state moves
        if (!out || cap < std::max<size_t>(std::max(m->members, h[rp::NS_LIVE]), 1))
            throw Error(RP_ERR_INVALID, "changes buffer must hold every member and every recorded change");
        node_issue(m, 1, sender, sender_inc, max_piggyback, (NChange*)out, cap, count);
        int fs = 0;
        if (*count == 0) {  // lib/dissemination.js:102-117 (membership.checksum: the last computed one)
            if (!m->checksum_known || !has_checksum || m->checksum != sender_checksum) {
                fs = 1;
                if (rp_dissemination_full_sync(m, out, cap, count) != RP_OK) throw Error(RP_ERR_HIP, rp_last_error());
            }
        }
        if (full_sync) *full_sync = fs;
    });
}

int rp_dissemination_clear(rp_node* m) {
    return rp::guarded([&] {
        node_of(m);
        m->sync_names();
        hipLaunchKernelGGL(rp::k_node_clear, dim3(64), dim3(256), 0, m->st, m->dev());
        RP_HIP(hipGetLastError());
        RP_HIP(hipMemsetAsync(m->stt.p + rp::NS_HEAD, 0, 12, m->st));
        RP_HIP(hipStreamSynchronize(m->st));
    });
}

int rp_dissemination_changes(rp_node* m, rp_member_change* out, size_t cap, uint32_t* count) {
    return rp::guarded([&] {
        node_of(m);
        if (!count) throw Error(RP_ERR_INVALID, "null pointer");
        uint32_t h[8];
        RP_HIP(hipMemcpyAsync(h, m->stt.p, sizeof h, hipMemcpyDeviceToHost, m->st));
        RP_HIP(hipStreamSynchronize(m->st));
        *count = h[rp::NS_LIVE];
        if (!out) return;
        if (cap < h[rp::NS_LIVE]) throw Error(RP_ERR_INVALID, "changes buffer too small");
        const uint32_t span = h[rp::NS_TAIL] - h[rp::NS_HEAD];
        std::vector<NChange> v(span);
        if (span) RP_HIP(hipMemcpy(v.data(), m->dlog.p + h[rp::NS_HEAD], span * sizeof(NChange), hipMemcpyDeviceToHost));
        uint32_t k = 0;
        for (const NChange& e : v)
            if (e.address >= 0) memcpy(out + k++, &e, sizeof e);
    });
}

}  // extern "C"
