// growbuf.hpp — the growth policy of the library's grow-only buffers (DevBuf in
// ctx.hpp), free of HIP so that tests/cpp/growbuf_test.cpp can drive it with an
// allocator that runs out of memory.  Internal.
#pragma once

#include <stddef.h>

#include <algorithm>
#include <vector>

namespace lsmb {

// Alloc: void* alloc(size_t) (nullptr when out of memory), void free(void*).
//
// Growing never frees on the common path: ROCm's hipFree waits for every
// stream of the device, so a free on the build path would stall every other
// context (a flush next to a background compaction,
// src/compaction/scheduler.rs:37).  An outgrown buffer is retired instead —
// kernels queued on other streams may still read it — and freed by release()
// at teardown.  Growth is at least 1.5x, so the retired buffers never add up to
// more than twice the live one.
//
// Out of memory, the fallbacks free in order of cost: first try exactly `want`
// instead of the 1.5x capacity, then free the retired buffers, then free the
// live buffer too (ensure never keeps contents: every caller rewrites or zeroes
// a buffer it grew) and try `want` once more.  Each free is a device-wide wait,
// not a failure, so a growth that fits once the old buffers are gone succeeds.
template <class Alloc>
struct GrowBuf {
    void* p = nullptr;
    size_t bytes = 0;
    std::vector<void*> retired;
    Alloc al;

    bool ensure(size_t want) {
        if (want <= bytes) return true;
        size_t cap = std::max(want, bytes + bytes / 2);
        void* q = al.alloc(cap);
        if (!q && cap != want) q = al.alloc(cap = want);
        if (!q && !retired.empty()) {
            free_retired();
            q = al.alloc(cap = want);
        }
        if (!q && p) {
            al.free(p);  // out of memory only
            p = nullptr;
            bytes = 0;
            q = al.alloc(cap = want);
        }
        if (!q) return false;
        if (p) retired.push_back(p);
        p = q;
        bytes = cap;
        return true;
    }
    void free_retired() {
        for (void* r : retired) al.free(r);  // teardown / out-of-memory only
        retired.clear();
    }
    void release() {
        free_retired();
        if (p) al.free(p);  // teardown
        p = nullptr;
        bytes = 0;
    }
};

}  // namespace lsmb
