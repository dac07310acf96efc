"""The drop-in ring's host map of points (ringpop_amd/csrc/rp_pointmap.h:
open addressing, backward-shift deletion), fuzzed against std::unordered_map
with g++ on the host: random inserts (first inserter kept), erases of
present and absent keys, clustered keys that share home slots, growth from
empty, and the iteration order-independent contents after every batch."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = r"""
#include <cstdio>
#include <random>
#include <unordered_map>
#include "rp_pointmap.h"
int main() {
    std::mt19937_64 rng(7);
    for (int trial = 0; trial < 40; trial++) {
        PointMap pm;
        std::unordered_map<uint32_t, int32_t> ref;
        if (trial % 2) pm.reset(1000);
        // a narrow key space makes collisions, home-slot clusters and re-inserts common
        const uint32_t space = trial % 3 == 0 ? 64u : trial % 3 == 1 ? 5000u : 0xFFFFFFFFu;
        for (int step = 0; step < 20000; step++) {
            const uint32_t k = (uint32_t)(rng() % ((uint64_t)space + 1)) * (trial % 4 == 3 ? 1024u : 1u);
            if (rng() % 3) {
                const int32_t v = (int32_t)(rng() % 1000);
                const bool a = pm.insert(k, v), b = ref.emplace(k, v).second;
                if (a != b) { printf("insert mismatch %d %d\n", trial, step); return 1; }
            } else {
                const bool a = pm.erase(k), b = ref.erase(k) > 0;
                if (a != b) { printf("erase mismatch %d %d\n", trial, step); return 1; }
            }
            if (pm.n != ref.size()) { printf("size mismatch %d %d\n", trial, step); return 1; }
            if (step % 997 == 0) {
                size_t seen = 0;
                bool ok = true;
                pm.each([&](uint32_t key, int32_t val) {
                    auto it = ref.find(key);
                    ok = ok && it != ref.end() && it->second == val;
                    seen++;
                });
                if (!ok || seen != ref.size()) { printf("contents mismatch %d %d\n", trial, step); return 1; }
            }
        }
    }
    printf("ok\n");
    return 0;
}
"""


def test_pointmap_against_unordered_map(tmp_path):
    src = tmp_path / "pm.cc"
    src.write_text(DRIVER)
    exe = tmp_path / "pm"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "ringpop_amd", "csrc"), str(src), "-o",
                    str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
