// ctx.hpp — the per-GPU context behind lsmb_ctx and the host plumbing shared by
// capi.hip (single GPU) and multi.hip (one process, several GPUs).  Internal.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/lsmbloom.h"
#include "growbuf.hpp"
#include "kernels.hpp"

namespace lsmb {

// A grow-only device buffer: GrowBuf's policy (growbuf.hpp) over hipMalloc.
// Outgrown buffers are retired, not freed, and freed by release() at teardown
// (lsmb_close and the handles' close functions, after their streams are
// synchronised); out of memory, the retired and then the live buffer are freed
// before the last try.
struct HipAlloc {
    hipError_t last = hipSuccess;
    void* alloc(size_t n) {
        void* q = nullptr;
        last = hipMalloc(&q, n);
        if (last != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        return q;
    }
    void free(void* q) { (void)hipFree(q); }  // teardown / out-of-memory only
};
struct DevBuf : GrowBuf<HipAlloc> {
    hipError_t ensure(size_t want) {
        if (GrowBuf<HipAlloc>::ensure(want)) return hipSuccess;
        return al.last != hipSuccess ? al.last : hipErrorOutOfMemory;
    }
};

// Pinned host staging with the same policy (hipHostFree waits for the device
// too): outgrown blocks are retired and freed at teardown.
struct PinnedPool {
    std::vector<void*> retired;
    void retire(void* p) {
        if (p) retired.push_back(p);
    }
    void release() {
        for (void* r : retired) (void)hipHostFree(r);  // teardown
        retired.clear();
    }
};

struct DevGuard {
    int prev = -1;
    explicit DevGuard(int dev) {
        hipGetDevice(&prev);
        if (prev != dev) hipSetDevice(dev);
    }
    ~DevGuard() {
        int cur = -1;
        hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) hipSetDevice(prev);
    }
};

// Thread-local error message (lsmb_last_error) and the error returns.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int hip_fail(hipError_t e, const char* what);
const std::string& last_error();
void set_last_error(const std::string& s);

#define HIP_TRY(expr)                                           \
    do {                                                        \
        hipError_t e_ = (expr);                                 \
        if (e_ != hipSuccess) return ::lsmb::hip_fail(e_, #expr); \
    } while (0)

inline uint64_t nwords64(uint32_t num_bits) { return ((uint64_t)num_bits + 63) / 64; }

// Reference arguments that would panic (% by zero in get_position, mod.rs:195).
int check_filter(uint32_t num_bits, uint32_t k);

// Builds of at most this many keys run the library's host loop (the
// reference's own per-key insert, src/bloom/mod.rs:70-78) instead of a device
// round trip; see lsmb_host_max_keys().
uint64_t host_max_keys();
void set_host_max_keys(uint64_t n);
constexpr uint64_t kDefaultHostMaxKeys = 2048;  // SST-sized flush latency

}  // namespace lsmb

struct lsmb_ctx {
    int dev = 0;
    int num_cus = 256;
    hipStream_t st = nullptr;
    lsmb::BuildTimers tm;
    lsmb::DevBuf ws_regions, ws_counts;  // partition / tiled workspace
    lsmb::DevBuf crc_parts;              // CRC-32 workgroup partials (crc32.hip)
    lsmb::DevBuf ws_hashes;              // k_hash records (var-len / odd-length keys)
    lsmb::DevBuf err;                    // LSMB_STATS builds: pass A's overflow counters
    lsmb::DevBuf ws_ovf, ws_dirty;       // partition: overflow words + unit marks (all-zero between builds)
    lsmb::DevBuf ws_ovl, ws_ovn;         // fresh partition builds: overflow position lists + lengths
    // The workspace above is shared by every build on this context, whatever
    // stream it is issued on: ws_done marks the last build that used it, and a
    // build on another stream waits for it first (build_dev).
    hipEvent_t ws_done = nullptr;
    hipStream_t ws_stream = nullptr;     // stream of the last workspace user (nullptr: none yet)
    lsmb::DevBuf keys, offs, words, out; // staging for the host-memory entry points
    lsmb::DevBuf filt_words;             // probe: device copies of host filters
    lsmb::DevBuf filt_desc;              // probe: ProbeFilter array
    std::vector<lsmb::ProbeFilter> hfilt;
    std::vector<lsmb::ProbeFilter> desc_uploaded;  // what filt_desc currently holds
    lsmb::ProbeFilter* desc_pinned = nullptr;      // pinned staging for descriptor uploads
    hipEvent_t desc_done = nullptr;                // last kernel that read filt_desc
    std::vector<uint64_t> offs_tmp;
    bool timing = true;                  // per-build HIP events (lsmb_set_timing)
    // host-memory builds: two staging slots, H2D on `cst` overlapping the
    // kernels of the previous chunk on `st` (host_build_dev)
    hipStream_t cst = nullptr;
    hipEvent_t ev_copy[2] = {nullptr, nullptr}, ev_built[2] = {nullptr, nullptr};
    lsmb::DevBuf kslot[2], oslot[2];
    uint64_t* offs_pin[2] = {nullptr, nullptr};  // pinned rebased offsets per slot
    uint64_t offs_pin_cap[2] = {0, 0};
    uint8_t* pin_small = nullptr;  // pinned staging of small host builds (host_build_small)
    uint64_t pin_small_cap = 0;
    lsmb::PinnedPool pinned_retired;  // outgrown pinned staging, freed by lsmb_close
};

namespace lsmb {

// `stream` of an entry point, NULL = the context's own build stream.
hipStream_t pick_stream(lsmb_ctx* c, void* stream);

// Device build of one batch on `st` into d_words (OR-accumulate; fresh =
// BloomFilter::new + inserts: d_words is output-only), chunked so the
// partition workspace stays bounded.  Asynchronous.
int build_dev(lsmb_ctx* c, const KeyBatch& kb, uint32_t num_bits, uint32_t k, uint32_t* d_words, hipStream_t st,
              int sweep = -1, bool fresh = false);

// Keys in host memory -> OR-accumulated into the device words dw (already
// zeroed or loaded by the caller) on c->st: chunked H2D through the two
// staging slots, overlapped with the build.  Returns once everything is
// enqueued; the caller synchronises c->st.
int host_build_dev(lsmb_ctx* c, const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                   uint32_t num_bits, uint32_t k, uint32_t* dw);

// Host build (the library's native per-key loop) into words (OR-accumulate).
void host_insert_batch(const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                       uint32_t num_bits, uint32_t k, uint64_t* words);

// LSMB_STATS builds only: prints and clears pass A's overflow counters
// (ring overflow, full regions).  Requires the builds to have completed.
void report_stats(lsmb_ctx* c);
// CRC-32 (crc32fast::hash / zlib crc32) of device bytes appended to `crc`
// (crc32.hip); synchronises `st`.
int crc32_dev(lsmb_ctx* c, const uint8_t* d, uint64_t len, uint32_t crc, hipStream_t st, uint32_t* out);
uint32_t crc32_host(const uint8_t* p, uint64_t len, uint32_t crc);
uint32_t crc32_combine_host(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

}  // namespace lsmb
