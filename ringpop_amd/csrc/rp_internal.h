// ringpop_amd — host-side helpers shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ringpop_hip.h"

namespace rp {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);
int current_device();

#define RP_HIP(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            throw ::rp::Error(e_ == hipErrorOutOfMemory ? RP_ERR_NOMEM : RP_ERR_HIP,        \
                              std::string(#expr) + ": " + hipGetErrorString(e_));            \
    } while (0)

// Runs `body`, converting exceptions to status codes.
template <class F>
int guarded(F&& body) {
    try {
        body();
        return RP_OK;
    } catch (const Error& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc&) {
        set_last_error("host allocation failed");
        return RP_ERR_NOMEM;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return RP_ERR_INVALID;
    }
}

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    explicit DevBuf(size_t count) { alloc(count); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
        return *this;
    }
    ~DevBuf() { release(); }
    void alloc(size_t count) {
        release();
        if (count) RP_HIP(hipMalloc(&p, count * sizeof(T)));
        n = count;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    size_t bytes() const { return n * sizeof(T); }
    // at least `count` elements (contents are not kept); grows by 1.5x steps
    bool reserve(size_t count) {
        if (count <= n) return false;
        alloc(std::max(count, n + n / 2));
        return true;
    }
};

inline unsigned grid_for(uint64_t n, unsigned block) {
    uint64_t g = (n + block - 1) / block;
    if (g == 0) g = 1;
    if (g > 0x7FFFFFFFull) g = 0x7FFFFFFFull;
    return (unsigned)g;
}

// one-time device hashing helper used by the sim setup
void device_replica_hashes(const std::string& names, const std::vector<uint64_t>& offsets, int replicas,
                           std::vector<uint32_t>& out, hipStream_t stream);

}  // namespace rp
