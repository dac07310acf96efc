// ringpop_amd — C ABI: error state, farmhash.hash32 and HashRing on the device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "rp_common.h"
#include "rp_internal.h"
#include "rp_pointmap.h"
#include "rp_ring.h"
#include "rp_sort.h"

namespace rp {
struct GroupWork;

static thread_local std::string g_last_error;
static int g_device = 0;

void set_last_error(const std::string& msg) { g_last_error = msg; }
int current_device() { return g_device; }

static void ensure_device() {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0)
        throw Error(RP_ERR_HIP, "no HIP device available (ringpop_amd requires an MI355X / gfx950 GPU)");
    RP_HIP(hipSetDevice(g_device));
}

// ------------------------------------------------------------- hashing
static void hash_batch_device(const uint8_t* d_bytes, const uint64_t* d_off, size_t n, uint32_t* d_out,
                              hipStream_t st) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_hash_batch, dim3(grid_for(n, 256)), dim3(256), 0, st, d_bytes, d_off, (uint64_t)n, d_out,
                       0xFFFFFFFFu);
    RP_HIP(hipGetLastError());
}

// Scalar calls: a stream of their own and a pinned result slot the kernel
// writes directly (k_hash_small / k_lookup_small), one per process.
struct SmallCall {
    std::mutex m;
    hipStream_t st = nullptr;
    void* hout = nullptr;
    void init() {
        if (st) return;
        RP_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        RP_HIP(hipHostMalloc(&hout, 64, hipHostMallocCoherent));
    }
};
static SmallCall& small_call() {
    static SmallCall* c = new SmallCall();  // (never destroyed: no HIP calls at process exit)
    return *c;
}
static bool small_key(const uint8_t* b, size_t len, SmallKey& k) {
    if (len > SMALL_KEY_WORDS * 4) return false;
    k.len = (uint32_t)len;
    if (len) memcpy(k.w, b, len);
    return true;
}

static void hash_batch_host(const uint8_t* bytes, const uint64_t* offsets, size_t n, uint32_t* out) {
    ensure_device();
    if (n == 0) return;
    uint64_t base = offsets[0], total = offsets[n] - base;
    std::vector<uint64_t> off(offsets, offsets + n + 1);
    std::vector<uint32_t> lng;  // strings hashed one wave each
    for (size_t i = 0; i < n; i++)
        if (off[i + 1] - off[i] >= HASH_LONG_MIN) lng.push_back((uint32_t)i);
    for (auto& o : off) o -= base;
    DevBuf<uint8_t> db(total + 8);
    DevBuf<uint64_t> doff(n + 1);
    DevBuf<uint32_t> dout(n), dl(std::max<size_t>(lng.size(), 1));
    if (total) RP_HIP(hipMemcpy(db.p, bytes + base, total, hipMemcpyHostToDevice));
    RP_HIP(hipMemcpy(doff.p, off.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    if (lng.size() < n)
        hipLaunchKernelGGL(k_hash_batch, dim3(grid_for(n, 256)), dim3(256), 0, 0, db.p, doff.p, (uint64_t)n, dout.p,
                           HASH_LONG_MIN);
    if (!lng.empty()) {
        RP_HIP(hipMemcpy(dl.p, lng.data(), lng.size() * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_hash_long, dim3((uint32_t)lng.size()), dim3(64), 0, 0, db.p, doff.p, dl.p, dout.p);
    }
    RP_HIP(hipGetLastError());
    RP_HIP(hipMemcpy(out, dout.p, n * 4, hipMemcpyDeviceToHost));
}

static uint32_t hash_one(const uint8_t* bytes, size_t len) {
    ensure_device();
    SmallKey k;
    if (!small_key(bytes, len, k)) {
        uint64_t off[2] = {0, len};
        uint32_t h = 0;
        hash_batch_host(bytes, off, 1, &h);
        return h;
    }
    SmallCall& c = small_call();
    std::lock_guard<std::mutex> g(c.m);
    c.init();
    hipLaunchKernelGGL(k_hash_small, dim3(1), dim3(64), 0, c.st, k, (uint32_t*)c.hout);
    RP_HIP(hipGetLastError());
    RP_HIP(hipStreamSynchronize(c.st));
    return *(volatile uint32_t*)c.hout;
}

void device_replica_hashes(const std::string& names, const std::vector<uint64_t>& offsets, int replicas,
                           std::vector<uint32_t>& out, hipStream_t st) {
    size_t ns = offsets.size() - 1;
    out.assign(ns * replicas, 0);
    if (ns == 0) return;
    DevBuf<uint8_t> db(names.size() + 8);
    DevBuf<uint64_t> doff(ns + 1);
    DevBuf<uint32_t> dh(ns * replicas);
    if (!names.empty()) RP_HIP(hipMemcpyAsync(db.p, names.data(), names.size(), hipMemcpyHostToDevice, st));
    RP_HIP(hipMemcpyAsync(doff.p, offsets.data(), (ns + 1) * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_replica_hashes, dim3(grid_for((uint64_t)ns * replicas, 256)), dim3(256), 0, st, db.p,
                       doff.p, (uint32_t)ns, replicas, dh.p);
    RP_HIP(hipGetLastError());
    RP_HIP(hipMemcpyAsync(out.data(), dh.p, ns * replicas * 4, hipMemcpyDeviceToHost, st));
    RP_HIP(hipStreamSynchronize(st));
}

// the same hashes left on the device (the ring build sorts them there)
static void device_replica_hashes_dev(const std::string& names, const std::vector<uint64_t>& offsets, int replicas,
                                      DevBuf<uint32_t>& out, hipStream_t st) {
    const size_t ns = offsets.size() - 1;
    out.alloc(ns * replicas);
    if (ns == 0) return;
    DevBuf<uint8_t> db(names.size() + 8);
    DevBuf<uint64_t> doff(ns + 1);
    if (!names.empty()) RP_HIP(hipMemcpyAsync(db.p, names.data(), names.size(), hipMemcpyHostToDevice, st));
    RP_HIP(hipMemcpyAsync(doff.p, offsets.data(), (ns + 1) * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_replica_hashes, dim3(grid_for((uint64_t)ns * replicas, 256)), dim3(256), 0, st, db.p,
                       doff.p, (uint32_t)ns, replicas, out.p);
    RP_HIP(hipGetLastError());
    RP_HIP(hipStreamSynchronize(st));  // (the staging buffers die here)
}

// ring build helpers: new points as (hash, owner) pairs; the first point of
// each run of equal hashes (rbtree.insert keeps the first inserter,
// lib/rbtree.js:112-117); points whose hash is in a sorted removal set
// (rbtree.remove erases by hash, :152); stream compaction by flags
__global__ void k_new_points(const uint32_t* h, const int32_t* owner_of_server, uint32_t nserv, int replicas,
                             uint32_t* key, uint32_t* val) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)nserv * replicas) return;
    key[t] = h[t];
    val[t] = (uint32_t)owner_of_server[t / replicas];
}
__global__ void k_first_of_run32(const uint32_t* key, uint32_t n, uint32_t* flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    flag[i] = i < n && (i == 0 || key[i] != key[i - 1]) ? 1u : 0u;  // (flag[n] = 0: the scan's total slot)
}
__global__ void k_keep_unless_removed(const uint32_t* h, uint32_t n, const uint32_t* rm, uint32_t nrm, uint32_t* keep) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    if (i == n) { keep[i] = 0; return; }
    uint32_t lo = 0, hi = nrm;
    const uint32_t x = h[i];
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (rm[m] < x) lo = m + 1; else hi = m; }
    keep[i] = (lo < nrm && rm[lo] == x) ? 0u : 1u;
}
// after an in-place exclusive scan of the flags: point i was flagged iff
// pos[i + 1] != pos[i]
__global__ void k_compact_kept(const uint32_t* k, const uint32_t* v, const uint32_t* pos, uint32_t n, uint32_t* ko,
                               int32_t* vo) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = pos[i];
    if (pos[i + 1] == p) return;
    ko[p] = k[i];
    vo[p] = (int32_t)v[i];
}

}  // namespace rp

// ----------------------------------------------------------------- ring
#ifndef RP_RING_INCR_MAX_POINTS
#define RP_RING_INCR_MAX_POINTS 8192  // add_remove calls touching at most this many replica points: incremental (host hashing ~100 ns a point)
#endif
constexpr size_t RING_INCR_MAX_POINTS = RP_RING_INCR_MAX_POINTS;
#ifndef RP_LOOKUP_DIR16
#define RP_LOOKUP_DIR16 1  // batched lookups through the 16-bit L2-resident directory when representable
#endif
struct rp_ring {
    int replicas = 100;
    std::vector<std::string> names;
    std::unordered_map<std::string, int> index;
    std::vector<uint8_t> present;
    int count = 0;
    rp::DevBuf<uint32_t> h;
    rp::DevBuf<int32_t> own;
    rp::DevBuf<uint32_t> bucket;  // first point per top-16-bit bucket (lookupN)
    rp::DevBuf<uint32_t> dir;     // direct lookup table (rp_ring.hip k_dir_both / k_index_build)
    rp::DevBuf<uint64_t> packed;  // owner << 32 | hash per point
    rp::DevBuf<uint16_t> dir16;   // the L2-resident 16-bit directory, when representable
    rp::DevBuf<uint32_t> coarse, d16bad;
    bool use16 = false;
    // key hashes between the passes of a split lookup: scratch of this ring,
    // so device lookups on one ring are ordered on one stream at a time
    rp::DevBuf<uint32_t> keyh;
    uint32_t npts = 0;
    uint32_t checksum = 0;
    bool checksum_valid = false;
    // the present servers' ids in name order (Object.keys(servers).sort(),
    // lib/ring.js:96-105), kept across single adds and removes; a bulk change
    // re-sorts once when the checksum is next asked for
    std::vector<int> sorted;
    bool sorted_valid = true;
    // the checksum string's staging (pinned host, device) and its result slot,
    // kept between calls: one copy, one launch and one sync per checksum
    uint8_t* ck_host = nullptr;
    size_t ck_cap = 0;
    rp::DevBuf<uint8_t> ck_dev;
    uint32_t* ck_out = nullptr;
    hipStream_t ck_st = nullptr;
    // host microseconds of the last rp_ring_add_remove by phase, and of the
    // last checksum (rp_ring_profile)
    double prof[RP_RING_PROF_N] = {};
    void set_present(int id, bool on, bool bulk) {
        if (present[id] == (on ? 1 : 0)) return;
        present[id] = on ? 1 : 0;
        count += on ? 1 : -1;
        checksum_valid = false;
        ck_inflight = false;  // (a queued hash is of the previous server set)
        if (bulk || !sorted_valid) { sorted_valid = false; return; }
        auto less = [&](int a, int b) { return names[a] < names[b]; };
        auto it = std::lower_bound(sorted.begin(), sorted.end(), id, less);
        if (on) sorted.insert(it, id);
        else if (it != sorted.end() && *it == id) sorted.erase(it);
        else sorted_valid = false;  // (cannot happen: re-sorted on the next checksum)
    }
    rp::DevBuf<uint8_t> kbytes;
    rp::DevBuf<uint64_t> koff;
    std::shared_ptr<rp::GroupWork> gwork;  // handleOrProxyAll grouping workspace (rp_ring_group_*)

    int intern(const uint8_t* b, size_t l) {
        std::string s((const char*)b, l);
        auto it = index.find(s);
        if (it != index.end()) return it->second;
        int id = (int)names.size();
        names.push_back(s);
        index.emplace(std::move(s), id);
        present.push_back(0);
        return id;
    }

    // The lookup indexes of the current points (null stream).  Whether the
    // 16-bit directory can represent them is the build's flag (d16bad), which
    // the lookup kernel reads itself: no synchronisation here.
    // bucket_valid: the bucket index describes the current points;
    // bucket_ready: k_ring_merge_small moved it to them and reset d16bad, so
    // the next rebuild skips k_bucket_index.
    bool bucket_valid = false, bucket_ready = false;
    void ensure_index_bufs() {
        if (!bucket.p) bucket.alloc(65537);
        if (!dir.p) dir.alloc(rp::DIR_SIZE);
        if (RP_LOOKUP_DIR16 && !dir16.p) { dir16.alloc(rp::D16_SIZE); coarse.alloc(rp::D16_SIZE >> rp::D16_GROUP_LOG); d16bad.alloc(1); }
    }
    void rebuild_index() {
        ensure_index_bufs();
        packed.reserve(std::max<uint32_t>(npts, 1));
        const bool ready = bucket_ready;
        bucket_ready = false;
        bucket_valid = true;  // (both paths below rebuild it)
        if (npts >= rp::INDEX_SCATTER_MIN) {  // (one launch, a thread per point)
            if (RP_LOOKUP_DIR16) RP_HIP(hipMemsetAsync(d16bad.p, 0, 4, 0));
            hipLaunchKernelGGL(rp::k_index_build, dim3(rp::grid_for((uint64_t)npts + 1, 256)), dim3(256), 0, 0, h.p,
                               own.p, npts, bucket.p, dir.p, packed.p, dir16.p, coarse.p, d16bad.p, RP_LOOKUP_DIR16);
            use16 = RP_LOOKUP_DIR16 != 0;
            RP_HIP(hipGetLastError());
            return;
        }
        // (fewer points: the bucket index, then both directories a thread per
        // bucket with searches the bucket index narrows)
        const int do16 = RP_LOOKUP_DIR16 && npts;
        if (!ready)
            hipLaunchKernelGGL(rp::k_bucket_index, dim3(rp::grid_for(65537, 256)), dim3(256), 0, 0, h.p, npts,
                               bucket.p, do16 ? d16bad.p : nullptr);
        use16 = do16 != 0;
        if (npts) {
            const uint32_t nb = std::max<uint32_t>(std::max<uint32_t>(npts, rp::DIR_SIZE), do16 ? rp::D16_SIZE : 0u);
            hipLaunchKernelGGL(rp::k_dir_both, dim3(rp::grid_for(nb, 256)), dim3(256), 0, 0, h.p, own.p, npts,
                               (const uint32_t*)bucket.p, dir.p, packed.p, dir16.p, coarse.p, d16bad.p, do16);
        }
        RP_HIP(hipGetLastError());
    }

    // ---- incremental updates (lib/ring.js addServer / removeServer, small
    // addRemoveServers): a host mirror of the points (hash -> owner) gives a
    // call's exact delta in the reference's order -- inserts that find their
    // hash taken keep the first inserter (lib/rbtree.js:112-117), removals
    // erase by hash whoever owns it (:152) -- and k_ring_merge applies it on
    // the device in one pass into the other buffer of (h, own).  No device
    // allocation on the way (buffers grow by reserve), no host
    // synchronisation: lookups are ordered after the update on the null
    // stream, or wait for ev_done on their own stream.
    PointMap pmap;
    bool pmap_valid = true;  // (false after a bulk build: rebuilt from the device points when next needed)
    rp::DevBuf<uint32_t> h2;
    rp::DevBuf<int32_t> own2;
    rp::DevBuf<uint32_t> dstage;           // the delta on the device: ins hashes | ins owners | del hashes
    uint32_t* hstage = nullptr;            // ... and its pinned host staging
    size_t hstage_n = 0;
    hipEvent_t ev_stage = nullptr;         // the last staging copy has left hstage
    hipEvent_t ev_done = nullptr;          // the last update's device work

    // replica hashes on the host: hashFunc(server + i) (lib/ring.js:52-57)
    void host_replica_hashes(const std::vector<int>& ids, std::vector<uint32_t>& out) {
        out.resize(ids.size() * (size_t)replicas);
        std::string str;
        for (size_t k = 0; k < ids.size(); k++) {
            const std::string& nm = names[ids[k]];
            for (int i = 0; i < replicas; i++) {
                str.assign(nm);
                str += std::to_string(i);
                out[k * replicas + i] = rp::farmhash32((const uint8_t*)str.data(), (uint32_t)str.size());
            }
        }
    }

    void ensure_events() {
        if (ev_stage) return;
        RP_HIP(hipEventCreateWithFlags(&ev_stage, hipEventDisableTiming));
        RP_HIP(hipEventCreateWithFlags(&ev_done, hipEventDisableTiming));
    }

    void mirror_from_device() {
        std::vector<uint32_t> hh(npts);
        std::vector<int32_t> oo(npts);
        if (npts) {
            RP_HIP(hipMemcpy(hh.data(), h.p, (size_t)npts * 4, hipMemcpyDeviceToHost));
            RP_HIP(hipMemcpy(oo.data(), own.p, (size_t)npts * 4, hipMemcpyDeviceToHost));
        }
        pmap.reset(npts + 16);
        for (uint32_t i = 0; i < npts; i++) pmap.insert(hh[i], oo[i]);
        pmap_valid = true;
    }

    // adds (in order), then removes: ah / rh are their replica hashes
    void apply_delta(const std::vector<int>& adds, const std::vector<uint32_t>& ah, const std::vector<int>& rms,
                     const std::vector<uint32_t>& rh) {
        if (!pmap_valid) mirror_from_device();
        PointMap ins;               // inserted by this call (and still there)
        ins.reset(adds.size() * (size_t)replicas);
        std::vector<uint32_t> del;  // erased hashes that were points before the call
        for (size_t k = 0; k < adds.size(); k++)
            for (int i = 0; i < replicas; i++) {
                const uint32_t x = ah[k * replicas + i];
                if (pmap.insert(x, adds[k])) ins.insert(x, adds[k]);
            }
        for (size_t k = 0; k < rms.size(); k++)
            for (int i = 0; i < replicas; i++) {
                const uint32_t x = rh[k * replicas + i];
                if (!pmap.erase(x)) continue;
                if (!ins.erase(x)) del.push_back(x);
            }
        std::vector<std::pair<uint32_t, int32_t>> iv;
        iv.reserve(ins.n);
        ins.each([&](uint32_t x, int32_t o) { iv.emplace_back(x, o); });
        std::sort(iv.begin(), iv.end());
        std::sort(del.begin(), del.end());
        const uint32_t nins = (uint32_t)iv.size(), ndel = (uint32_t)del.size();
        if (nins == 0 && ndel == 0) return;  // (servers whose replicas all collided or were already erased)
        // The mirror already holds this call's points; the device ones change
        // only at the swap below.  If a step before it fails, the mirror is
        // rebuilt from the device points on the next call, so a failed call
        // leaves the ring (and every later delta) as it was.
        try {
            merge_delta(iv, del);
        } catch (...) {
            pmap_valid = false;
            throw;
        }
    }

    void merge_delta(const std::vector<std::pair<uint32_t, int32_t>>& iv, const std::vector<uint32_t>& del) {
        const uint32_t nins = (uint32_t)iv.size(), ndel = (uint32_t)del.size();
        const size_t m = 2 * (size_t)nins + ndel;
        const uint32_t nnew = npts + nins - ndel;
        h2.reserve(std::max<uint32_t>(nnew, 1));
        own2.reserve(std::max<uint32_t>(nnew, 1));
        const uint64_t work = (uint64_t)npts + nins;
        if (m <= rp::RING_DELTA_WORDS) {  // (one server's replicas: the delta rides in the kernel arguments)
            ensure_index_bufs();
            uint32_t* bk = bucket_valid ? bucket.p : nullptr;
            rp::RingDelta d;
            d.nins = nins;
            d.ndel = ndel;
            for (uint32_t j = 0; j < nins; j++) { d.w[j] = iv[j].first; d.w[nins + j] = (uint32_t)iv[j].second; }
            for (uint32_t j = 0; j < ndel; j++) d.w[2 * nins + j] = del[j];
            const uint64_t threads = std::max<uint64_t>(work, 65537);  // (and one per bucket-index entry)
            hipLaunchKernelGGL(rp::k_ring_merge_small, dim3(rp::grid_for(threads, 256)), dim3(256), 0, 0, h.p,
                               own.p, npts, d, h2.p, own2.p, nnew, bk, RP_LOOKUP_DIR16 ? d16bad.p : nullptr);
            bucket_ready = bk != nullptr;
        } else {
            stage_merge(iv, del, work, nnew);
            bucket_valid = false;
        }
        RP_HIP(hipGetLastError());
        std::swap(h, h2);
        std::swap(own, own2);
        npts = nnew;
    }

    void stage_merge(const std::vector<std::pair<uint32_t, int32_t>>& iv, const std::vector<uint32_t>& del,
                     uint64_t work, uint32_t nnew) {
        const uint32_t nins = (uint32_t)iv.size(), ndel = (uint32_t)del.size();
        const size_t m = 2 * (size_t)nins + ndel;
        ensure_events();
        RP_HIP(hipEventSynchronize(ev_stage));  // (the previous delta's copy: long done)
        if (hstage_n < m) {
            if (hstage) RP_HIP(hipHostFree(hstage));
            hstage = nullptr;
            hstage_n = std::max(m, hstage_n + hstage_n / 2);
            RP_HIP(hipHostMalloc((void**)&hstage, hstage_n * 4, hipHostMallocDefault));
        }
        for (uint32_t j = 0; j < nins; j++) { hstage[j] = iv[j].first; hstage[nins + j] = (uint32_t)iv[j].second; }
        for (uint32_t j = 0; j < ndel; j++) hstage[2 * nins + j] = del[j];
        dstage.reserve(m);
        RP_HIP(hipMemcpyAsync(dstage.p, hstage, m * 4, hipMemcpyHostToDevice, 0));
        RP_HIP(hipEventRecord(ev_stage, 0));
        hipLaunchKernelGGL(rp::k_ring_merge, dim3(rp::grid_for(work, 256)), dim3(256), 0, 0, h.p, own.p, npts,
                           dstage.p, (const int32_t*)(dstage.p + nins), nins, dstage.p + 2 * nins, ndel, h2.p,
                           own2.p, nnew);
    }

    void replica_hashes_for(const std::vector<int>& ids, const std::vector<uint32_t>& custom, bool use_custom,
                            rp::DevBuf<uint32_t>& out) {
        size_t m = ids.size() * (size_t)replicas;
        out.alloc(m);
        if (use_custom) {
            RP_HIP(hipMemcpy(out.p, custom.data(), m * 4, hipMemcpyHostToDevice));
            return;
        }
        std::string blob;
        std::vector<uint64_t> off{0};
        for (int id : ids) { blob += names[id]; off.push_back(blob.size()); }
        std::vector<uint32_t> hv;
        rp::device_replica_hashes(blob, off, replicas, hv, 0);
        RP_HIP(hipMemcpy(out.p, hv.data(), m * 4, hipMemcpyHostToDevice));
    }

    // Device part of the last add_remove (HIP events on the null stream):
    // replica hashing, the stable point sort, dedupe, compaction, directories.
    hipEvent_t ev_build[2] = {nullptr, nullptr};
    float build_ms = 0.0f;
    bool build_pending = false;  // ev_build[1] recorded, build_ms not yet read
    rp::SortWork sortw;
    ~rp_ring() {
        for (hipEvent_t e : ev_build)
            if (e) (void)hipEventDestroy(e);
        if (ev_stage) (void)hipEventDestroy(ev_stage);
        if (ev_done) (void)hipEventDestroy(ev_done);
        for (auto& p : lk_ev) (void)hipEventDestroy(p.second);
        if (hstage) (void)hipHostFree(hstage);
        if (ck_st) (void)hipStreamSynchronize(ck_st);  // (a checksum launched by an update may be reading ck_host)
        if (ck_host) (void)hipHostFree(ck_host);
        if (ck_out) (void)hipHostFree(ck_out);
        if (ck_st) (void)hipStreamDestroy(ck_st);
    }
    // The ring checksum (lib/ring.js:96-105): hash32 of the sorted server
    // names joined by ';'.  launch_checksum() builds the string and queues its
    // hash on the ring's own stream; finish_checksum() waits for the value.
    // An incremental update launches it at once (HashRing.addServer /
    // removeServer recompute it after every change, lib/ring.js:39-58), so
    // the hash runs beside the update's own device work and the caller's
    // checksum read only waits for what is left of it.
    bool ck_inflight = false;  // the hash of the current server set is queued on ck_st
    void launch_checksum() {
        const auto t0 = std::chrono::steady_clock::now();
        if (!sorted_valid) {
            sorted.clear();
            for (size_t i = 0; i < names.size(); i++) if (present[i]) sorted.push_back((int)i);
            std::sort(sorted.begin(), sorted.end(), [&](int a, int b) { return names[a] < names[b]; });
            sorted_valid = true;
        }
        size_t len = 0;
        for (size_t i = 0; i < sorted.size(); i++) len += names[sorted[i]].size() + (i ? 1 : 0);
        if (!ck_st) {
            RP_HIP(hipStreamCreateWithFlags(&ck_st, hipStreamNonBlocking));
            RP_HIP(hipHostMalloc((void**)&ck_out, 64, hipHostMallocCoherent));
        }
        // (the previous hash, if still running, reads ck_host: it is long done
        // or nearly, a single 20 KB chain)
        RP_HIP(hipStreamSynchronize(ck_st));
        ck_inflight = false;
        if (ck_cap < len + 16) {
            if (ck_host) RP_HIP(hipHostFree(ck_host));
            ck_host = nullptr;
            ck_cap = std::max(len + 16, ck_cap * 2);
            // (coherent: k_hash_host reads it in place, uncached)
            RP_HIP(hipHostMalloc((void**)&ck_host, ck_cap, hipHostMallocCoherent));
            if (ck_cap > rp::HASH_HOST_MAX) ck_dev.alloc(ck_cap);
        }
        uint8_t* p = ck_host;
        for (size_t i = 0; i < sorted.size(); i++) {
            if (i) *p++ = ';';
            const std::string& nm = names[sorted[i]];
            memcpy(p, nm.data(), nm.size());
            p += nm.size();
        }
        // one wave on the ring's own stream, reading the string over PCIe
        // (longer ones: a copy first); the result lands in pinned memory
        if (len <= rp::HASH_HOST_MAX) {
            hipLaunchKernelGGL(rp::k_hash_host, dim3(1), dim3(256), 0, ck_st, (const uint4*)ck_host, (uint32_t)len,
                               ck_out);
        } else {
            RP_HIP(hipMemcpyAsync(ck_dev.p, ck_host, len, hipMemcpyHostToDevice, ck_st));
            hipLaunchKernelGGL(rp::k_hash_one, dim3(1), dim3(64), 0, ck_st, (const uint8_t*)ck_dev.p, (uint32_t)len,
                               ck_out);
        }
        RP_HIP(hipGetLastError());
        ck_inflight = true;
        prof[RP_RING_PROF_CK_BUILD] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
    void finish_checksum() {
        const auto t1 = std::chrono::steady_clock::now();
        RP_HIP(hipStreamSynchronize(ck_st));
        ck_inflight = false;
        checksum = *(volatile uint32_t*)ck_out;
        checksum_valid = true;
        prof[RP_RING_PROF_CK_HASH] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count();
    }
    // lookups on a stream other than the null stream wait for the last update
    void order_after_update(hipStream_t st) {
        if (st && ev_done) RP_HIP(hipStreamWaitEvent(st, ev_done, 0));
    }
    // ... and an update waits for the device lookups still reading the
    // points and directories it rewrites in place: each caller stream's last
    // lookup records an event the next update's null-stream work waits on
    // (the callers' streams are non-blocking: rp_stream_create)
    std::vector<std::pair<hipStream_t, hipEvent_t>> lk_ev;
    void note_lookup(hipStream_t st) {
        if (!st) return;  // (the null stream: already in order with the updates)
        for (auto& p : lk_ev)
            if (p.first == st) { RP_HIP(hipEventRecord(p.second, st)); return; }
        if (lk_ev.size() >= 64) {  // (streams come and go: start over once the device is idle)
            RP_HIP(hipDeviceSynchronize());
            for (auto& p : lk_ev) (void)hipEventDestroy(p.second);
            lk_ev.clear();
        }
        hipEvent_t e;
        RP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        lk_ev.emplace_back(st, e);
        RP_HIP(hipEventRecord(e, st));
    }
    void order_after_lookups() {
        for (auto& p : lk_ev) RP_HIP(hipStreamWaitEvent(0, p.second, 0));
    }

    void replica_hashes_dev(const std::vector<int>& ids, const std::vector<uint32_t>& custom, bool use_custom,
                            rp::DevBuf<uint32_t>& out) {
        if (use_custom) {
            out.alloc(ids.size() * (size_t)replicas);
            RP_HIP(hipMemcpy(out.p, custom.data(), out.n * 4, hipMemcpyHostToDevice));
            return;
        }
        std::string blob;
        std::vector<uint64_t> off{0};
        for (int id : ids) { blob += names[id]; off.push_back(blob.size()); }
        rp::device_replica_hashes_dev(blob, off, replicas, out, 0);
    }

    // (hash, owner) pairs in k/v, flags[0..n] -> the ring's points
    void compact_points(const uint32_t* k, const uint32_t* v, rp::DevBuf<uint32_t>& flag, uint32_t n) {
        rp::exclusive_scan<uint32_t>(flag.p, flag.p, (uint64_t)n + 1, sortw.scan, 0);  // in place: positions
        uint32_t m = 0;
        RP_HIP(hipMemcpy(&m, flag.p + n, 4, hipMemcpyDeviceToHost));
        rp::DevBuf<uint32_t> nh(std::max<uint32_t>(m, 1));
        rp::DevBuf<int32_t> no(std::max<uint32_t>(m, 1));
        // the flags are now positions: a point is kept iff the next position differs
        if (n)
            hipLaunchKernelGGL(rp::k_compact_kept, dim3(rp::grid_for(n, 256)), dim3(256), 0, 0, k, v,
                               (const uint32_t*)flag.p, n, nh.p, no.p);
        RP_HIP(hipGetLastError());
        h = std::move(nh);
        own = std::move(no);
        npts = m;
        pmap_valid = false;
        bucket_valid = false;
    }

    void add(const std::vector<int>& ids, const std::vector<uint32_t>& custom, bool use_custom) {
        rp::DevBuf<uint32_t> nh;
        replica_hashes_dev(ids, custom, use_custom, nh);
        const uint32_t nnew = (uint32_t)(ids.size() * replicas), total = npts + nnew;
        // existing points first (already sorted and distinct), then the new
        // ones in insertion order: a stable sort by hash leaves the first
        // inserter of every hash at the head of its run
        rp::DevBuf<uint32_t> k0(total), k1(total), v0(total), v1(total), flag(total + 1);
        rp::DevBuf<int32_t> owners(ids.size());
        RP_HIP(hipMemcpy(owners.p, ids.data(), ids.size() * 4, hipMemcpyHostToDevice));
        if (npts) {
            RP_HIP(hipMemcpyAsync(k0.p, h.p, (size_t)npts * 4, hipMemcpyDeviceToDevice, 0));
            RP_HIP(hipMemcpyAsync(v0.p, own.p, (size_t)npts * 4, hipMemcpyDeviceToDevice, 0));
        }
        hipLaunchKernelGGL(rp::k_new_points, dim3(rp::grid_for(nnew, 256)), dim3(256), 0, 0, nh.p, owners.p,
                           (uint32_t)ids.size(), replicas, k0.p + npts, v0.p + npts);
        RP_HIP(hipGetLastError());
        const bool in1 = rp::radix_sort_pairs(k0.p, v0.p, k1.p, v1.p, total, 32, sortw, 0);
        const uint32_t* ks = in1 ? k1.p : k0.p;
        const uint32_t* vs = in1 ? v1.p : v0.p;
        hipLaunchKernelGGL(rp::k_first_of_run32, dim3(rp::grid_for(total + 1, 256)), dim3(256), 0, 0, ks, total,
                           flag.p);
        compact_points(ks, vs, flag, total);
    }

    void remove(const std::vector<int>& ids, const std::vector<uint32_t>& custom, bool use_custom) {
        rp::DevBuf<uint32_t> rh;
        replica_hashes_dev(ids, custom, use_custom, rh);
        const uint32_t nr = (uint32_t)(ids.size() * replicas);
        rp::DevBuf<uint32_t> rs(nr);
        const bool in1 = rp::radix_sort_pairs(rh.p, nullptr, rs.p, nullptr, nr, 32, sortw, 0);
        if (!npts) return;
        rp::DevBuf<uint32_t> keep(npts + 1);
        hipLaunchKernelGGL(rp::k_keep_unless_removed, dim3(rp::grid_for(npts + 1, 256)), dim3(256), 0, 0, h.p, npts,
                           (const uint32_t*)(in1 ? rs.p : rh.p), nr, keep.p);
        RP_HIP(hipGetLastError());
        rp::DevBuf<uint32_t> k(npts), v(npts);
        RP_HIP(hipMemcpyAsync(k.p, h.p, (size_t)npts * 4, hipMemcpyDeviceToDevice, 0));
        RP_HIP(hipMemcpyAsync(v.p, own.p, (size_t)npts * 4, hipMemcpyDeviceToDevice, 0));
        compact_points(k.p, v.p, keep, npts);
    }
};

static double us_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

extern "C" {

const char* rp_last_error(void) { return rp::g_last_error.c_str(); }
int rp_abi_version(void) { return 2; }
int rp_set_device(int device) {
    return rp::guarded([&] {
        int count = 0;
        RP_HIP(hipGetDeviceCount(&count));
        if (device < 0 || device >= count) throw rp::Error(RP_ERR_INVALID, "device index out of range");
        rp::g_device = device;
        RP_HIP(hipSetDevice(device));
    });
}

// ---- device utilities: the runtime this library links, for *_device callers
int rp_device_malloc(size_t bytes, void** out) {
    return rp::guarded([&] {
        if (!out) throw rp::Error(RP_ERR_INVALID, "null pointer");
        rp::ensure_device();
        RP_HIP(hipMalloc(out, bytes ? bytes : 1));
    });
}
int rp_device_free(void* p) {
    return rp::guarded([&] { if (p) RP_HIP(hipFree(p)); });
}
int rp_device_memcpy(void* dst, const void* src, size_t bytes, int kind) {
    return rp::guarded([&] {
        if (kind < 1 || kind > 3) throw rp::Error(RP_ERR_INVALID, "kind: 1 host->device, 2 device->host, 3 device->device");
        const hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice : kind == 2 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
        if (bytes) RP_HIP(hipMemcpy(dst, src, bytes, k));
    });
}
int rp_device_synchronize(void) {
    return rp::guarded([&] { RP_HIP(hipDeviceSynchronize()); });
}
int rp_device_memory(size_t* free_bytes, size_t* total_bytes) {
    return rp::guarded([&] {
        if (!free_bytes || !total_bytes) throw rp::Error(RP_ERR_INVALID, "null pointer");
        rp::ensure_device();
        RP_HIP(hipMemGetInfo(free_bytes, total_bytes));
    });
}
int rp_stream_create(void** out) {
    return rp::guarded([&] {
        if (!out) throw rp::Error(RP_ERR_INVALID, "null pointer");
        rp::ensure_device();
        RP_HIP(hipStreamCreateWithFlags((hipStream_t*)out, hipStreamNonBlocking));
    });
}
int rp_stream_destroy(void* s) {
    return rp::guarded([&] { if (s) RP_HIP(hipStreamDestroy((hipStream_t)s)); });
}
int rp_stream_synchronize(void* s) {
    return rp::guarded([&] { RP_HIP(hipStreamSynchronize((hipStream_t)s)); });
}
int rp_event_create(void** out) {
    return rp::guarded([&] {
        if (!out) throw rp::Error(RP_ERR_INVALID, "null pointer");
        rp::ensure_device();
        RP_HIP(hipEventCreate((hipEvent_t*)out));
    });
}
int rp_event_record(void* ev, void* stream) {
    return rp::guarded([&] { RP_HIP(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream)); });
}
int rp_event_elapsed_ms(void* start, void* end, float* ms) {
    return rp::guarded([&] {
        if (!ms) throw rp::Error(RP_ERR_INVALID, "null pointer");
        RP_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end));
    });
}
int rp_event_destroy(void* ev) {
    return rp::guarded([&] { if (ev) RP_HIP(hipEventDestroy((hipEvent_t)ev)); });
}

int rp_hash32(const uint8_t* bytes, size_t len, uint32_t* out) {
    return rp::guarded([&] {
        if (!out || (!bytes && len)) throw rp::Error(RP_ERR_INVALID, "null pointer");
        static const uint8_t empty = 0;
        *out = rp::hash_one(bytes ? bytes : &empty, len);
    });
}

int rp_hash32_batch(const uint8_t* bytes, const uint64_t* offsets, size_t n, uint32_t* out) {
    return rp::guarded([&] {
        if (n && (!bytes || !offsets || !out)) throw rp::Error(RP_ERR_INVALID, "null pointer");
        rp::hash_batch_host(bytes, offsets, n, out);
    });
}

int rp_hash32_batch_device(const uint8_t* d_bytes, const uint64_t* d_offsets, size_t n, uint32_t* d_out,
                           void* stream) {
    return rp::guarded([&] { rp::hash_batch_device(d_bytes, d_offsets, n, d_out, (hipStream_t)stream); });
}

int rp_ring_create(int replica_points, rp_ring** out) {
    return rp::guarded([&] {
        if (!out) throw rp::Error(RP_ERR_INVALID, "null out");
        rp::ensure_device();
        auto* r = new rp_ring();
        if (replica_points > 100000000) throw rp::Error(RP_ERR_INVALID, "replica_points must be <= 10^8");
        r->replicas = replica_points > 0 ? replica_points : 100;  // lib/ring.js:28
        *out = r;
    });
}

int rp_ring_destroy(rp_ring* ring) {
    delete ring;
    return RP_OK;
}

int rp_ring_add_remove(rp_ring* r, const uint8_t* add_bytes, const uint64_t* add_off, size_t nadd,
                       const uint32_t* add_hashes, const uint8_t* rm_bytes, const uint64_t* rm_off, size_t nrm,
                       const uint32_t* rm_hashes, int* changed) {
    return rp::guarded([&] {
        if (!r) throw rp::Error(RP_ERR_INVALID, "null ring");
        if ((nadd && (!add_bytes || !add_off)) || (nrm && (!rm_bytes || !rm_off)))
            throw rp::Error(RP_ERR_INVALID, "null server name arrays");
        rp::ensure_device();
        const auto t_call = std::chrono::steady_clock::now();
        auto t_last = t_call;
        for (int i = 0; i < RP_RING_PROF_CK_BUILD; i++) r->prof[i] = 0.0;
        auto prof_mark = [&](int phase) {
            const auto t = std::chrono::steady_clock::now();
            r->prof[phase] = std::chrono::duration<double, std::micro>(t - t_last).count();
            t_last = t;
        };
        const int R = r->replicas;
        // lib/ring.js:60-94: the adds (skipping servers already present,
        // :72), then the removes (skipping absent ones, :81).  The ring's own
        // state changes only once a step's replica points are in place, so a
        // failed call leaves the ring as it was before that step.
        std::vector<int> added, removed;
        std::vector<uint32_t> ah, rh;
        std::vector<uint8_t> in_batch;
        if (!r->ev_build[0]) {
            RP_HIP(hipEventCreate(&r->ev_build[0]));
            RP_HIP(hipEventCreate(&r->ev_build[1]));
        }
        r->order_after_lookups();  // (device lookups queued on callers' streams read what this call rewrites)
        bool timed = false;
        auto tick = [&] {
            if (!timed) RP_HIP(hipEventRecord(r->ev_build[0], 0));
            timed = true;
        };
        auto mark = [&](int id) {
            if ((size_t)id >= in_batch.size()) in_batch.resize(r->names.size(), 0);
            if (in_batch[id]) return false;
            in_batch[id] = 1;
            return true;
        };
        for (size_t i = 0; i < nadd; i++) {
            int id = r->intern(add_bytes + add_off[i], add_off[i + 1] - add_off[i]);
            if (r->present[id] || !mark(id)) continue;  // hasServer (lib/ring.js:72)
            added.push_back(id);
            if (add_hashes) ah.insert(ah.end(), add_hashes + i * R, add_hashes + (i + 1) * R);
        }
        // A few servers (addServer / removeServer, a gossip batch's ring
        // changes): the incremental path, whose device work is one merge and
        // the index rebuild, with no synchronisation.  Many (a bulk build):
        // replica hashing and a radix sort on the device.
        std::vector<int> rm_ids;
        std::vector<uint32_t> rm_h;
        {
            std::vector<uint8_t> seen_rm(r->names.size() + nrm, 0);
            for (size_t i = 0; i < nrm; i++) {
                // (adds first: a server added by this call may be removed by it)
                auto it = r->index.find(std::string((const char*)rm_bytes + rm_off[i], rm_off[i + 1] - rm_off[i]));
                if (it == r->index.end()) continue;
                const int id = it->second;
                const bool present = r->present[id] || (id < (int)in_batch.size() && in_batch[id]);
                if (!present || seen_rm[id]) continue;  // lib/ring.js:81
                seen_rm[id] = 1;
                rm_ids.push_back(id);
                if (rm_hashes) rm_h.insert(rm_h.end(), rm_hashes + i * R, rm_hashes + (i + 1) * R);
            }
        }
        if ((added.size() + rm_ids.size()) * (size_t)R <= RING_INCR_MAX_POINTS && !(added.empty() && rm_ids.empty())) {
            prof_mark(RP_RING_PROF_SELECT);
            if (!add_hashes) r->host_replica_hashes(added, ah);
            if (!rm_hashes) r->host_replica_hashes(rm_ids, rm_h);
            prof_mark(RP_RING_PROF_HASH);
            r->ensure_events();
            // the new server set first: its checksum's hash then runs while
            // the host builds the delta (launch_checksum); a failed delta
            // puts the set back
            for (int id : added) r->set_present(id, true, false);
            for (int id : rm_ids) r->set_present(id, false, false);
            r->launch_checksum();
            tick();
            try {
                r->apply_delta(added, ah, rm_ids, rm_h);
            } catch (...) {
                for (int id : rm_ids) r->set_present(id, true, false);
                for (int id : added) r->set_present(id, false, false);
                throw;
            }
            prof_mark(RP_RING_PROF_MERGE);
            r->rebuild_index();
            RP_HIP(hipEventRecord(r->ev_build[1], 0));
            RP_HIP(hipEventRecord(r->ev_done, 0));
            prof_mark(RP_RING_PROF_INDEX);
            r->build_pending = true;
            if (changed) *changed = 1;
            r->prof[RP_RING_PROF_TOTAL] = us_since(t_call);
            return;
        }
        if (!added.empty()) {
            tick();
            r->add(added, ah, add_hashes != nullptr);
            for (int id : added) r->set_present(id, true, true);
            r->rebuild_index();
        }
        in_batch.assign(r->names.size(), 0);
        for (size_t i = 0; i < nrm; i++) {
            int id = r->intern(rm_bytes + rm_off[i], rm_off[i + 1] - rm_off[i]);
            if (!r->present[id] || !mark(id)) continue;  // lib/ring.js:81
            removed.push_back(id);
            if (rm_hashes) rh.insert(rh.end(), rm_hashes + i * R, rm_hashes + (i + 1) * R);
        }
        if (!removed.empty()) {
            tick();
            r->remove(removed, rh, rm_hashes != nullptr);
            for (int id : removed) r->set_present(id, false, true);
            r->rebuild_index();
        }
        if (timed) RP_HIP(hipEventRecord(r->ev_build[1], 0));
        RP_HIP(hipDeviceSynchronize());
        if (timed) RP_HIP(hipEventElapsedTime(&r->build_ms, r->ev_build[0], r->ev_build[1]));
        r->build_pending = false;
        if (changed) *changed = (!added.empty() || !removed.empty()) ? 1 : 0;
        r->prof[RP_RING_PROF_TOTAL] = us_since(t_call);
    });
}

int rp_ring_build_ms(rp_ring* r, double* device_ms) {
    if (!r || !device_ms) return RP_ERR_INVALID;
    return rp::guarded([&] {
        if (r->build_pending) {  // (an incremental update: timed when asked)
            RP_HIP(hipEventSynchronize(r->ev_build[1]));
            RP_HIP(hipEventElapsedTime(&r->build_ms, r->ev_build[0], r->ev_build[1]));
            r->build_pending = false;
        }
        *device_ms = r->build_ms;
    });
}

int rp_ring_server_count(rp_ring* r, int* out) {
    if (!r || !out) return RP_ERR_INVALID;
    *out = r->count;
    return RP_OK;
}

int rp_ring_has_server(rp_ring* r, const uint8_t* name, size_t len, int* out) {
    if (!r || !out || (!name && len)) return RP_ERR_INVALID;
    auto it = r->index.find(std::string((const char*)name, len));
    *out = it != r->index.end() && r->present[it->second];
    return RP_OK;
}

int rp_ring_checksum(rp_ring* r, uint32_t* out) {
    return rp::guarded([&] {
        if (!r || !out) throw rp::Error(RP_ERR_INVALID, "null pointer");
        if (!r->checksum_valid) {
            // hash32(Object.keys(servers).sort().join(';')) (lib/ring.js:96-105)
            rp::ensure_device();
            if (!r->ck_inflight) r->launch_checksum();  // (an update may have queued it already)
            r->finish_checksum();
        }
        *out = r->checksum;
    });
}

int rp_ring_profile(rp_ring* r, double* us, int n) {
    if (!r || !us || n < 1) return RP_ERR_INVALID;
    for (int i = 0; i < n; i++) us[i] = i < RP_RING_PROF_N ? r->prof[i] : 0.0;
    return RP_OK;
}

int rp_ring_server_name(rp_ring* r, int idx, char* buf, size_t cap, size_t* len) {
    if (!r || idx < 0 || (size_t)idx >= r->names.size()) return RP_ERR_INVALID;
    const std::string& s = r->names[idx];
    if (len) *len = s.size();
    if (buf) {
        if (cap < s.size() + 1) return RP_ERR_INVALID;
        memcpy(buf, s.c_str(), s.size() + 1);
    }
    return RP_OK;
}

int rp_ring_lookup_batch_device(rp_ring* r, const uint8_t* d_bytes, const uint64_t* d_off, size_t n,
                                int32_t* d_owners, void* stream) {
    return rp::guarded([&] {
        if (!r) throw rp::Error(RP_ERR_INVALID, "null ring");
        if (n == 0) return;
        if (!r->bucket.p) r->rebuild_index();
        r->order_after_update((hipStream_t)stream);
        if (n >= rp::LK_SPLIT_MIN && r->npts) {
            r->keyh.reserve(n);
            hipLaunchKernelGGL(rp::k_lookup_keys, dim3(rp::grid_for(n, 256 * rp::LK_KPT)), dim3(256), 0,
                               (hipStream_t)stream, d_bytes, d_off, (uint64_t)n, r->dir.p, r->packed.p, r->npts,
                               d_owners, r->keyh.p, (const uint16_t*)nullptr, (const uint32_t*)nullptr,
                               (const uint32_t*)nullptr);
            hipLaunchKernelGGL(rp::k_lookup_split, dim3(8 * rp::grid_for(n, rp::LK_SPLIT_CHUNK)), dim3(256), 0,
                               (hipStream_t)stream, r->keyh.p, (uint64_t)n, r->dir.p, r->packed.p, r->npts, d_owners);
        } else {
            hipLaunchKernelGGL(rp::k_lookup_keys, dim3(rp::grid_for(n, 256 * rp::LK_KPT)), dim3(256), 0,
                               (hipStream_t)stream, d_bytes, d_off, (uint64_t)n, r->dir.p, r->packed.p, r->npts,
                               d_owners, (uint32_t*)nullptr, r->use16 ? (const uint16_t*)r->dir16.p : nullptr,
                               (const uint32_t*)r->coarse.p, (const uint32_t*)r->d16bad.p);
        }
        RP_HIP(hipGetLastError());
        r->note_lookup((hipStream_t)stream);
    });
}

int rp_ring_lookup_batch(rp_ring* r, const uint8_t* bytes, const uint64_t* offsets, size_t n, int32_t* owners) {
    return rp::guarded([&] {
        if (!r) throw rp::Error(RP_ERR_INVALID, "null ring");
        if (n && (!bytes || !offsets || !owners)) throw rp::Error(RP_ERR_INVALID, "null key arrays or owners");
        rp::ensure_device();
        if (n == 0) return;
        rp::SmallKey k;
        if (n == 1 && r->npts && rp::small_key(bytes + offsets[0], offsets[1] - offsets[0], k)) {  // ring.lookup(key)
            if (!r->bucket.p) {
                r->rebuild_index();
                RP_HIP(hipStreamSynchronize(0));  // (index builds run on the null stream)
            }
            rp::SmallCall& c = rp::small_call();
            std::lock_guard<std::mutex> g(c.m);
            c.init();
            r->order_after_update(c.st);
            hipLaunchKernelGGL(rp::k_lookup_small, dim3(1), dim3(64), 0, c.st, k, r->dir.p, r->packed.p, r->npts,
                               (int32_t*)c.hout);
            RP_HIP(hipGetLastError());
            RP_HIP(hipStreamSynchronize(c.st));
            owners[0] = *(volatile int32_t*)c.hout;
            return;
        }
        uint64_t base = offsets[0], total = offsets[n] - base;
        std::vector<uint64_t> off(offsets, offsets + n + 1);
        for (auto& o : off) o -= base;
        rp::DevBuf<uint8_t> db(total + 8);
        rp::DevBuf<uint64_t> doff(n + 1);
        rp::DevBuf<int32_t> dout(n);
        if (total) RP_HIP(hipMemcpy(db.p, bytes + base, total, hipMemcpyHostToDevice));
        RP_HIP(hipMemcpy(doff.p, off.data(), (n + 1) * 8, hipMemcpyHostToDevice));
        int rc = rp_ring_lookup_batch_device(r, db.p, doff.p, n, dout.p, 0);
        if (rc) throw rp::Error(rc, rp_last_error());
        RP_HIP(hipMemcpy(owners, dout.p, n * 4, hipMemcpyDeviceToHost));
    });
}

int rp_ring_lookup_hashes(rp_ring* r, const uint32_t* key_hashes, size_t n, int32_t* owners) {
    return rp::guarded([&] {
        if (!r) throw rp::Error(RP_ERR_INVALID, "null ring");
        if (n && (!key_hashes || !owners)) throw rp::Error(RP_ERR_INVALID, "null key hashes or owners");
        rp::ensure_device();
        if (n == 0) return;
        if (!r->bucket.p) r->rebuild_index();
        rp::DevBuf<uint32_t> dk(n);
        rp::DevBuf<int32_t> dout(n);
        RP_HIP(hipMemcpy(dk.p, key_hashes, n * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(rp::k_lookup_hashes, dim3(rp::grid_for(n, 256)), dim3(256), 0, 0, dk.p, (uint64_t)n,
                           r->dir.p, r->packed.p, r->npts, dout.p);
        RP_HIP(hipGetLastError());
        RP_HIP(hipMemcpy(owners, dout.p, n * 4, hipMemcpyDeviceToHost));
    });
}

}  // extern "C"

namespace rp {
// lookupN walk (lib/ring.js:150-182): from the inclusive lower bound, one full
// circle over the points, collecting distinct owners until n are found.
__global__ void k_lookup_n(const uint32_t* keyh, uint64_t nk, const uint32_t* h, const int32_t* own, uint32_t npts,
                           const uint32_t* bucket, int n, int32_t* out, int32_t* counts) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nk) return;
    int32_t* o = out + i * n;
    for (int k = 0; k < n; k++) o[k] = -1;
    int got = 0;
    if (npts && n > 0) {
        uint32_t x = keyh[i], top = x >> 16;
        uint32_t lo = bucket[top], hi = bucket[top + 1];
        while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (h[m] < x) lo = m + 1; else hi = m; }
        for (uint32_t s = 0; s < npts && got < n; s++) {
            uint32_t p = lo + s;
            if (p >= npts) p -= npts;
            int32_t w = own[p];
            bool dup = false;
            for (int k = 0; k < got; k++) dup |= o[k] == w;
            if (!dup) o[got++] = w;
        }
    }
    counts[i] = got;
}
}  // namespace rp

extern "C" int rp_ring_lookup_n_hashes(rp_ring* r, const uint32_t* key_hashes, size_t nkeys, int n, int32_t* out,
                                       int32_t* counts) {
    return rp::guarded([&] {
        if (!r || n < 0) throw rp::Error(RP_ERR_INVALID, "bad argument");
        if (nkeys && (!key_hashes || !out || !counts)) throw rp::Error(RP_ERR_INVALID, "null pointer");
        rp::ensure_device();
        if (nkeys == 0) return;
        int nn = std::min(n, r->count);  // "can't return more than the number of servers"
        if (!r->bucket.p) r->rebuild_index();
        rp::DevBuf<uint32_t> dk(nkeys);
        rp::DevBuf<int32_t> dout(nkeys * (size_t)std::max(nn, 1));
        rp::DevBuf<int32_t> dc(nkeys);
        RP_HIP(hipMemcpy(dk.p, key_hashes, nkeys * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(rp::k_lookup_n, dim3(rp::grid_for(nkeys, 256)), dim3(256), 0, 0, dk.p, (uint64_t)nkeys,
                           r->h.p, r->own.p, r->npts, r->bucket.p, nn, dout.p, dc.p);
        RP_HIP(hipGetLastError());
        std::vector<int32_t> tmp(nkeys * (size_t)std::max(nn, 1));
        RP_HIP(hipMemcpy(tmp.data(), dout.p, tmp.size() * 4, hipMemcpyDeviceToHost));
        RP_HIP(hipMemcpy(counts, dc.p, nkeys * 4, hipMemcpyDeviceToHost));
        for (size_t k = 0; k < nkeys; k++)
            for (int j = 0; j < n; j++) out[k * n + j] = j < nn ? tmp[k * nn + j] : -1;
    });
}

extern "C" int rp_ring_points(rp_ring* r, uint32_t* hashes, int32_t* owners, size_t cap, size_t* count) {
    return rp::guarded([&] {
        if (!r || !count) throw rp::Error(RP_ERR_INVALID, "null pointer");
        *count = r->npts;
        if (!hashes && !owners) return;
        if (cap < r->npts) throw rp::Error(RP_ERR_INVALID, "buffer too small");
        if (r->npts && hashes) RP_HIP(hipMemcpy(hashes, r->h.p, r->npts * 4, hipMemcpyDeviceToHost));
        if (r->npts && owners) RP_HIP(hipMemcpy(owners, r->own.p, r->npts * 4, hipMemcpyDeviceToHost));
    });
}

extern "C" int rp_ring_make_keys_device(rp_ring* r, uint64_t seed, size_t n, const uint8_t** d_bytes,
                                        const uint64_t** d_offsets, uint64_t* total_bytes) {
    return rp::guarded([&] {
        if (!r || !d_bytes || !d_offsets) throw rp::Error(RP_ERR_INVALID, "null pointer");
        rp::ensure_device();
        r->koff.alloc(n + 1);
        rp::DevBuf<uint64_t> len(n + 1);
        RP_HIP(hipMemset(len.p, 0, (n + 1) * 8));
        hipLaunchKernelGGL(rp::k_keygen_len, dim3(rp::grid_for(n, 256)), dim3(256), 0, 0, seed, (uint64_t)n, len.p);
        rp::ScanWork sw;
        rp::exclusive_scan<uint64_t>(len.p, r->koff.p, (uint64_t)n + 1, sw, 0);
        uint64_t total = 0;
        RP_HIP(hipMemcpy(&total, r->koff.p + n, 8, hipMemcpyDeviceToHost));
        r->kbytes.alloc(total + 8);
        hipLaunchKernelGGL(rp::k_keygen_bytes, dim3(rp::grid_for(n, 256)), dim3(256), 0, 0, seed, (uint64_t)n,
                           r->koff.p, r->kbytes.p);
        RP_HIP(hipGetLastError());
        RP_HIP(hipDeviceSynchronize());
        *d_bytes = r->kbytes.p;
        *d_offsets = r->koff.p;
        if (total_bytes) *total_bytes = total;
    });
}

// ------------------------------------------------- handleOrProxyAll grouping
// index.js:636-645: keysByDest = _.groupBy(keys, this.lookup); dests =
// Object.keys(keysByDest).  Groups come in first-appearance order of their
// owner (string keys keep insertion order), keys within a group in input
// order; an empty ring puts every key in one group (owner -1, the
// reference's "null" key).  On the device, for owners o = owner + 1 in
// [0, nserv]:
//  1. per owner its key count and first key index (LDS-aggregated per block:
//     an atomicAdd / atomicMin per key on the block's copy, one global atomic
//     per owner and block);
//  2. the present owners, listed and sorted by first index (the hand-written
//     radix sort of rp_sort.h), are the groups in order: dests, and the
//     group offsets by an exclusive scan of their counts;
//  3. every key gets its group's rank as a sort key, and a stable radix sort
//     of (rank, key index) over ceil(log2 groups) bits leaves the key indices
//     grouped, each group in input order.
namespace rp {
constexpr uint32_t GK_LDS_BINS = 12288;  // owners aggregated in LDS per block (96 KB); more: global atomics
__global__ void __launch_bounds__(BLOCK) k_gk_count(const int32_t* own, uint32_t n, uint32_t nb, uint32_t* cnt,
                                                    uint32_t* first, uint32_t* err) {
    extern __shared__ uint32_t lds[];
    const bool local = nb <= GK_LDS_BINS;
    uint32_t* lc = lds;
    uint32_t* lf = lds + (local ? nb : 0u);
    if (local) {
        for (uint32_t o = threadIdx.x; o < nb; o += BLOCK) { lc[o] = 0; lf[o] = 0xFFFFFFFFu; }
        __syncthreads();
    }
    const uint32_t ntiles = (n + PS_TILE - 1) / PS_TILE;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
#pragma unroll 4
        for (uint32_t k = 0; k < PS_IPT; k++) {
            const uint32_t i = t * PS_TILE + k * BLOCK + threadIdx.x;
            if (i >= n) break;
            const uint32_t o = (uint32_t)(own[i] + 1);
            if (o >= nb) { atomicOr(err, 1u); continue; }
            if (local) { atomicAdd(&lc[o], 1u); atomicMin(&lf[o], i); }
            else { atomicAdd(&cnt[o], 1u); atomicMin(&first[o], i); }
        }
    }
    if (!local) return;
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < nb; o += BLOCK)
        if (lc[o]) { atomicAdd(&cnt[o], lc[o]); atomicMin(&first[o], lf[o]); }
}
__global__ void k_gk_present(const uint32_t* cnt, uint32_t nb, uint32_t* flag) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o <= nb) flag[o] = o < nb && cnt[o] ? 1u : 0u;
}
// after the flags' in-place exclusive scan: present owner o -> list slot pos[o]
__global__ void k_gk_list(const uint32_t* pos, const uint32_t* first, uint32_t nb, uint32_t* fk, uint32_t* fv) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= nb || pos[o + 1] == pos[o]) return;
    fk[pos[o]] = first[o];
    fv[pos[o]] = o;
}
__global__ void k_gk_groups(const uint32_t* fv, uint32_t G, const uint32_t* cnt, int32_t* dests, uint32_t* rank,
                            uint32_t* gcnt) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= G) return;
    const uint32_t o = fv[q];
    dests[q] = (int32_t)o - 1;
    rank[o] = q;
    gcnt[q] = cnt[o];
}
// key i of the final sort: the rank of key i's group
struct GroupKey {
    const int32_t* own;
    const uint32_t* rank;
    __device__ inline uint32_t operator()(uint64_t i) const { return rank[own[i] + 1]; }
};
inline int key_bits(uint32_t maxv) { return maxv ? 32 - __builtin_clz(maxv) : 1; }

// Workspace kept by the ring between calls (grows to the largest batch).
struct GroupWork {
    DevBuf<uint32_t> k0, v0, k1, v1, cnt, first, flag, fk, fv, fk1, fv1, rank, gcnt, err;
    SortWork sort;
};

// owners -> (dests[ngroups], goff[ngroups + 1], key_index[n]), all on the device
static void group_owners(GroupWork& w, const int32_t* d_own, uint32_t n, uint32_t nserv, int32_t* d_dests,
                         uint32_t* d_goff, uint32_t* d_kidx, size_t* ngroups, hipStream_t st) {
    const uint32_t nb = nserv + 1;
    w.cnt.reserve(nb); w.first.reserve(nb); w.flag.reserve(nb + 1); w.err.reserve(1);
    RP_HIP(hipMemsetAsync(w.cnt.p, 0, (size_t)nb * 4, st));
    RP_HIP(hipMemsetAsync(w.first.p, 0xFF, (size_t)nb * 4, st));
    RP_HIP(hipMemsetAsync(w.err.p, 0, 4, st));
    const uint32_t ntiles = (n + PS_TILE - 1) / PS_TILE;
    const size_t lds = nb <= GK_LDS_BINS ? (size_t)nb * 8 : 0;
    // (LDS copies are zeroed and flushed per block: a few tiles per block)
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(ntiles, nb <= GK_LDS_BINS ? 1024u : 8192u));
    hipLaunchKernelGGL(k_gk_count, dim3(blocks), dim3(BLOCK), lds, st, d_own, n, nb, w.cnt.p, w.first.p, w.err.p);
    hipLaunchKernelGGL(k_gk_present, dim3(grid_for(nb + 1, 256)), dim3(256), 0, st, (const uint32_t*)w.cnt.p, nb,
                       w.flag.p);
    exclusive_scan<uint32_t>(w.flag.p, w.flag.p, (uint64_t)nb + 1, w.sort.scan, st);
    uint32_t hb[2] = {0, 0};
    RP_HIP(hipMemcpyAsync(&hb[0], w.flag.p + nb, 4, hipMemcpyDeviceToHost, st));
    RP_HIP(hipMemcpyAsync(&hb[1], w.err.p, 4, hipMemcpyDeviceToHost, st));
    RP_HIP(hipStreamSynchronize(st));
    if (hb[1]) throw Error(RP_ERR_INVALID, "an owner outside [-1, server count) in the batch");
    const uint32_t G = hb[0];  // >= 1 (n >= 1), <= nb
    w.fk.reserve(G); w.fv.reserve(G); w.fk1.reserve(G); w.fv1.reserve(G); w.rank.reserve(nb); w.gcnt.reserve(G);
    hipLaunchKernelGGL(k_gk_list, dim3(grid_for(nb, 256)), dim3(256), 0, st, (const uint32_t*)w.flag.p,
                       (const uint32_t*)w.first.p, nb, w.fk.p, w.fv.p);
    const bool f1 = radix_sort_pairs(w.fk.p, w.fv.p, w.fk1.p, w.fv1.p, G, key_bits(n - 1), w.sort, st);
    hipLaunchKernelGGL(k_gk_groups, dim3(grid_for(G, 256)), dim3(256), 0, st, (const uint32_t*)(f1 ? w.fv1.p : w.fv.p),
                       G, (const uint32_t*)w.cnt.p, d_dests, w.rank.p, w.gcnt.p);
    exclusive_scan<uint32_t>(w.gcnt.p, d_goff, G, w.sort.scan, st);
    RP_HIP(hipMemcpyAsync(d_goff + G, &n, 4, hipMemcpyHostToDevice, st));
    // the stable sort of the key indices by group rank: the first pass
    // computes the ranks from the owners, the last writes only the indices,
    // straight into d_kidx
    const int kb = key_bits(G - 1);
    if ((kb + 7) / 8 > 1) { w.k0.reserve(n); w.v0.reserve(n); }
    if ((kb + 7) / 8 > 2) { w.k1.reserve(n); w.v1.reserve(n); }
    radix_sort_indices(GroupKey{d_own, w.rank.p}, n, kb, d_kidx, w.k0.p, w.v0.p, w.k1.p, w.v1.p, w.sort, st);
    RP_HIP(hipGetLastError());
    RP_HIP(hipStreamSynchronize(st));
    *ngroups = G;
}
}  // namespace rp

static rp::GroupWork& group_work(rp_ring* r) {
    if (!r->gwork) r->gwork = std::make_shared<rp::GroupWork>();
    return *r->gwork;
}

static void check_group_args(rp_ring* r, size_t n, const void* dests, const void* goff, const void* kidx,
                             const size_t* ngroups) {
    if (!r || !ngroups) throw rp::Error(RP_ERR_INVALID, "null pointer");
    if (n && (!dests || !goff || !kidx)) throw rp::Error(RP_ERR_INVALID, "null output array");
    if (n >= 0x7FFFFFFFull) throw rp::Error(RP_ERR_INVALID, "more than 2^31 - 2 keys in one batch");
}

extern "C" int rp_ring_group_device(rp_ring* r, const int32_t* d_owners, size_t n, int32_t* d_dests,
                                    uint32_t* d_group_off, uint32_t* d_key_index, size_t* ngroups, void* stream) {
    return rp::guarded([&] {
        check_group_args(r, n, d_dests, d_group_off, d_key_index, ngroups);
        *ngroups = 0;
        if (n == 0) return;
        rp::group_owners(group_work(r), d_owners, (uint32_t)n, (uint32_t)r->names.size(), d_dests, d_group_off,
                         d_key_index, ngroups, (hipStream_t)stream);
    });
}

// host arrays: owners from device lookups of the keys (or key hashes), grouped on the device
static void group_to_host(rp_ring* r, const int32_t* d_own, size_t n, int32_t* dests, uint32_t* group_off,
                          uint32_t* key_index, size_t* ngroups) {
    rp::DevBuf<int32_t> dd(n);
    rp::DevBuf<uint32_t> dg(n + 1), dk(n);
    rp::group_owners(group_work(r), d_own, (uint32_t)n, (uint32_t)r->names.size(), dd.p, dg.p, dk.p, ngroups, 0);
    RP_HIP(hipMemcpy(dests, dd.p, *ngroups * 4, hipMemcpyDeviceToHost));
    RP_HIP(hipMemcpy(group_off, dg.p, (*ngroups + 1) * 4, hipMemcpyDeviceToHost));
    RP_HIP(hipMemcpy(key_index, dk.p, n * 4, hipMemcpyDeviceToHost));
}

extern "C" int rp_ring_group_keys(rp_ring* r, const uint8_t* bytes, const uint64_t* offsets, size_t n,
                                  int32_t* dests, uint32_t* group_off, uint32_t* key_index, size_t* ngroups) {
    return rp::guarded([&] {
        check_group_args(r, n, dests, group_off, key_index, ngroups);
        if (n && (!bytes || !offsets)) throw rp::Error(RP_ERR_INVALID, "null key arrays");
        rp::ensure_device();
        *ngroups = 0;
        if (n == 0) { if (group_off) group_off[0] = 0; return; }
        uint64_t base = offsets[0], total = offsets[n] - base;
        std::vector<uint64_t> off(offsets, offsets + n + 1);
        for (auto& o : off) o -= base;
        rp::DevBuf<uint8_t> db(total + 8);
        rp::DevBuf<uint64_t> doff(n + 1);
        rp::DevBuf<int32_t> down(n);
        if (total) RP_HIP(hipMemcpy(db.p, bytes + base, total, hipMemcpyHostToDevice));
        RP_HIP(hipMemcpy(doff.p, off.data(), (n + 1) * 8, hipMemcpyHostToDevice));
        int rc = rp_ring_lookup_batch_device(r, db.p, doff.p, n, down.p, 0);
        if (rc) throw rp::Error(rc, rp_last_error());
        group_to_host(r, down.p, n, dests, group_off, key_index, ngroups);
    });
}

extern "C" int rp_ring_group_hashes(rp_ring* r, const uint32_t* key_hashes, size_t n, int32_t* dests,
                                    uint32_t* group_off, uint32_t* key_index, size_t* ngroups) {
    return rp::guarded([&] {
        check_group_args(r, n, dests, group_off, key_index, ngroups);
        if (n && !key_hashes) throw rp::Error(RP_ERR_INVALID, "null key hashes");
        rp::ensure_device();
        *ngroups = 0;
        if (n == 0) { if (group_off) group_off[0] = 0; return; }
        if (!r->bucket.p) r->rebuild_index();
        rp::DevBuf<uint32_t> dkh(n);
        rp::DevBuf<int32_t> down(n);
        RP_HIP(hipMemcpy(dkh.p, key_hashes, n * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(rp::k_lookup_hashes, dim3(rp::grid_for(n, 256)), dim3(256), 0, 0, dkh.p, (uint64_t)n,
                           r->dir.p, r->packed.p, r->npts, down.p);
        RP_HIP(hipGetLastError());
        group_to_host(r, down.p, n, dests, group_off, key_index, ngroups);
    });
}
