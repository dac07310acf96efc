// ringpop_amd -- host-side hash -> owner map of the drop-in ring's points.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

// hash -> owner for the incremental ring path (rp_ring::apply_delta): open
// addressing over a power-of-two table, linear probing, deletion by backward
// shift (no tombstones).  A single addServer touches 100 keys of a
// 100,000-point map; std::unordered_map's node allocations cost several
// microseconds of that call.
struct PointMap {
    std::vector<uint32_t> key;
    std::vector<int32_t> val;
    std::vector<uint8_t> used;
    size_t n = 0, mask = 0;
    static size_t home(uint32_t x, size_t m) {
        x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
        return x & m;
    }
    void reset(size_t cap) {
        size_t sz = 16;
        while (sz < 2 * cap) sz <<= 1;
        key.assign(sz, 0); val.assign(sz, 0); used.assign(sz, 0);
        n = 0; mask = sz - 1;
    }
    bool insert(uint32_t k, int32_t v) {  // (false: the key is present, its owner kept)
        if (key.empty() || 2 * (n + 1) > key.size()) grow();
        size_t i = home(k, mask);
        for (; used[i]; i = (i + 1) & mask)
            if (key[i] == k) return false;
        used[i] = 1; key[i] = k; val[i] = v; n++;
        return true;
    }
    bool erase(uint32_t k) {
        if (key.empty()) return false;
        size_t i = home(k, mask);
        for (; used[i] && key[i] != k; i = (i + 1) & mask) {}
        if (!used[i]) return false;
        // refill the hole from the run after it: an entry stays when its home
        // lies cyclically in (hole, its slot]
        for (size_t j = i;;) {
            j = (j + 1) & mask;
            if (!used[j]) break;
            const size_t h = home(key[j], mask);
            const bool stays = i <= j ? (i < h && h <= j) : (i < h || h <= j);
            if (stays) continue;
            key[i] = key[j]; val[i] = val[j];
            i = j;
        }
        used[i] = 0; n--;
        return true;
    }
    void grow() {
        std::vector<uint32_t> k0 = std::move(key);
        std::vector<int32_t> v0 = std::move(val);
        std::vector<uint8_t> u0 = std::move(used);
        reset(std::max<size_t>(2 * n + 16, u0.size()));
        for (size_t i = 0; i < u0.size(); i++) if (u0[i]) insert(k0[i], v0[i]);
    }
    template <class F> void each(F&& f) const {
        for (size_t i = 0; i < used.size(); i++) if (used[i]) f(key[i], val[i]);
    }
};
