// capi.hip — the C ABI (include/lsmbloom.h) over the HIP kernels.
//
// Host-side plumbing only: argument validation with the reference's error
// behaviour, the per-GPU context (stream, events, grow-only device arenas),
// chunking of large builds, and the format functions of src/bloom/mod.rs.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "ctx.hpp"

using namespace lsmb;

namespace lsmb {

namespace {
thread_local std::string g_err;
}  // namespace

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(LSMB_EHIP, "%s: %s", what, hipGetErrorString(e));
}

const std::string& last_error() { return g_err; }
void set_last_error(const std::string& s) { g_err = s; }

int check_filter(uint32_t num_bits, uint32_t k) {
    if (num_bits == 0 && k > 0)
        return fail(LSMB_EINVAL, "num_bits == 0 with num_hashes > 0 (reference panics: %% by zero)");
    return LSMB_OK;
}

namespace {
std::atomic<uint64_t> g_host_max_keys{~0ull};  // ~0: not yet read from the environment

uint32_t rd32le(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

uint64_t workspace_limit_bytes() {
    const char* s = getenv("LSMB_WORKSPACE_MB");
    uint64_t mb = s ? strtoull(s, nullptr, 10) : 8192;
    if (mb < 16) mb = 16;
    return mb << 20;
}
}  // namespace

void set_host_max_keys(uint64_t n) { g_host_max_keys.store(n == ~0ull ? n - 1 : n, std::memory_order_relaxed); }

uint64_t host_max_keys() {
    uint64_t v = g_host_max_keys.load(std::memory_order_relaxed);
    if (v == ~0ull) {
        const char* s = getenv("LSMB_HOST_MAX_KEYS");
        v = s ? strtoull(s, nullptr, 10) : kDefaultHostMaxKeys;
        g_host_max_keys.store(v, std::memory_order_relaxed);
    }
    return v;
}

hipStream_t pick_stream(lsmb_ctx* c, void* stream) {
    return stream ? reinterpret_cast<hipStream_t>(stream) : c->st;
}

// LSMB_STATS builds only (diagnostics, never the product): pass A counts the
// positions that went past a ring or a full region to exact global atomics.
void report_stats(lsmb_ctx* c) {
#ifdef LSMB_STATS
    uint32_t st[16];
    if (hipMemcpyAsync(st, c->err.p, 64, hipMemcpyDeviceToHost, c->st) != hipSuccess ||
        hipStreamSynchronize(c->st) != hipSuccess)
        return;
    fprintf(stderr, "[lsmb stats] ring_overflow=%u region_full=%u\n", st[9], st[7]);
    (void)hipMemsetAsync(c->err.p, 0, 64, c->st);
#else
    (void)c;
#endif
}

namespace {
int build_dev_ws(lsmb_ctx* c, const KeyBatch& kb_all, uint32_t num_bits, uint32_t k, uint32_t* dw, hipStream_t st,
                 BuildStrategy s, int sweep, bool fresh, hipEvent_t done = nullptr);
}  // namespace

// Device build of one batch, chunked so the partition workspace stays bounded.
int build_dev(lsmb_ctx* c, const KeyBatch& kb_all, uint32_t num_bits, uint32_t k, uint32_t* dw,
              hipStream_t st, int sweep, bool fresh) {
    BuildStrategy s = pick_build_strategy(num_bits, k, kb_all.n);
    // LSMB_FORCE_STRATEGY=atomic: measurement override;
    // the filter is the same either way.
    if (const char* f = getenv("LSMB_FORCE_STRATEGY"))
        if ((s == BuildStrategy::Partition || s == BuildStrategy::Tiled) && !strcmp(f, "atomic")) s = BuildStrategy::Atomic;
    c->tm.valid = false;
    if (s == BuildStrategy::None) {  // fresh: new() with no inserts, all-zero words
        if (fresh && num_bits) HIP_TRY(hipMemsetAsync(dw, 0, nwords64(num_bits) * 8, st));
        return LSMB_OK;
    }
    if (s != BuildStrategy::Tiled && s != BuildStrategy::Partition)
        return build_dev_ws(c, kb_all, num_bits, k, dw, st, s, sweep, fresh);
    // Tiled and partition builds use the context's shared workspace: a build
    // issued on a different stream than the last one waits for it (two
    // streams' builds would otherwise overwrite each other's regions).  On the
    // same stream, stream order already serialises them: no wait packet (a
    // barrier packet between consecutive builds costs the stream ~10 us).
    // ws_done is completed by the build's last kernel itself (launch_done): a
    // separate event record would put a marker packet, ~6 us, between
    // back-to-back builds.
    if (c->ws_stream && c->ws_stream != st) HIP_TRY(hipStreamWaitEvent(st, c->ws_done, 0));
    const int rc = build_dev_ws(c, kb_all, num_bits, k, dw, st, s, sweep, fresh, c->ws_done);
    if (rc != LSMB_OK) HIP_TRY(hipEventRecord(c->ws_done, st));  // (a failed build may have launched nothing)
    c->ws_stream = st;
    return rc;
}

namespace {
int build_dev_ws(lsmb_ctx* c, const KeyBatch& kb_all, uint32_t num_bits, uint32_t k, uint32_t* dw, hipStream_t st,
                 BuildStrategy s, int sweep, bool fresh, hipEvent_t done) {
    if (s == BuildStrategy::Tiled) {
        const TiledPlan tp = plan_tiled(num_bits, kb_all.n, c->num_cus);
        HIP_TRY(c->ws_regions.ensure(tp.scratch_bytes));
        PartitionWorkspace ws;
        ws.regions = (uint64_t*)c->ws_regions.p;
        ws.region_bytes = c->ws_regions.bytes;
        if (!getenv("LSMB_TILED_NO_PREHASH")) {  // measurement switch
            HIP_TRY(c->ws_hashes.ensure(kb_all.n * 16));
            ws.hashes = (uint4*)c->ws_hashes.p;
            ws.hash_bytes = c->ws_hashes.bytes;
        }
        HIP_TRY(launch_build(kb_all, num_bits, k, dw, s, ws, c->num_cus, st, c->timing ? &c->tm : nullptr, sweep,
                             fresh, done));
        return LSMB_OK;
    }
    if (s != BuildStrategy::Partition) {
        HIP_TRY(launch_build(kb_all, num_bits, k, dw, s, PartitionWorkspace{}, c->num_cus, st,
                             c->timing ? &c->tm : nullptr, sweep, fresh, done));
        return LSMB_OK;
    }
    uint64_t chunk = partition_chunk_keys(num_bits, k, workspace_limit_bytes(), c->num_cus);
    if (chunk == 0) return fail(LSMB_ENOMEM, "partition workspace limit too small");
    chunk = std::min(chunk, kb_all.n);
    const PartitionPlan pl = plan_partition(num_bits, k, chunk, c->num_cus);
    HIP_TRY(c->ws_regions.ensure(pl.region_bytes));
    HIP_TRY(c->ws_counts.ensure(pl.counts_bytes));
    PartitionWorkspace ws;
    ws.regions = (uint64_t*)c->ws_regions.p;
    ws.counts = (uint32_t*)c->ws_counts.p;
    ws.err = (uint32_t*)c->err.p;
    ws.region_bytes = c->ws_regions.bytes;
    ws.counts_bytes = c->ws_counts.bytes;
    if (fresh && k == 7) {
        // a fresh k = 7 build (the LIST pass A, bloom_build.hip): the overflow
        // lists (per workgroup per sweep), and the overflow words + unit marks
        // of the whole filter for lists that fill up, zeroed once when
        // (re)allocated
        const uint64_t units = ((nwords64(num_bits) * 2) + kSliceWords32 - 1) / kSliceWords32;
        // each buffer is zeroed right after it is (re)allocated, before the
        // next allocation can fail: a grown buffer never stays unzeroed
        const size_t ob = c->ws_ovf.bytes, db = c->ws_dirty.bytes;
        HIP_TRY(c->ws_ovf.ensure(units * kSliceWords32 * 4));
        if (c->ws_ovf.bytes != ob) HIP_TRY(hipMemsetAsync(c->ws_ovf.p, 0, c->ws_ovf.bytes, st));
        HIP_TRY(c->ws_dirty.ensure(units * 4));
        if (c->ws_dirty.bytes != db) HIP_TRY(hipMemsetAsync(c->ws_dirty.p, 0, c->ws_dirty.bytes, st));
        ws.ovf = (uint32_t*)c->ws_ovf.p;
        ws.dirty = (uint32_t*)c->ws_dirty.p;
        ws.ovf_units = std::min<uint64_t>(c->ws_ovf.bytes / (kSliceWords32 * 4), c->ws_dirty.bytes / 4);
        HIP_TRY(c->ws_ovl.ensure((uint64_t)pl.grid * pl.sweeps * kOvfListCap * 4));
        HIP_TRY(c->ws_ovn.ensure((uint64_t)pl.grid * pl.sweeps * 4));
        ws.ovl = (uint32_t*)c->ws_ovl.p;
        ws.ovn = (uint32_t*)c->ws_ovn.p;
        ws.ovl_groups = (uint32_t)std::min<uint64_t>(c->ws_ovn.bytes / 4, c->ws_ovl.bytes / (kOvfListCap * 4ull));
    }
    const bool fixed16 = !kb_all.offsets && kb_all.key_len == 16 && (reinterpret_cast<uintptr_t>(kb_all.data) & 15) == 0;
    if (!fixed16) {  // pre-hashed pass A (ks::Hashed): 16 B per key of the chunk
        HIP_TRY(c->ws_hashes.ensure(chunk * 16));
        ws.hashes = (uint4*)c->ws_hashes.p;
        ws.hash_bytes = c->ws_hashes.bytes;
    }
    for (uint64_t first = 0; first < kb_all.n; first += chunk) {
        KeyBatch kb = kb_all;
        kb.n = std::min(chunk, kb_all.n - first);
        if (kb.offsets)
            kb.offsets += first;  // VarLen offsets are absolute into data
        else
            kb.data += first * kb.key_len;
        // fresh: the first chunk writes every word of the range, the rest accumulate
        HIP_TRY(launch_build(kb, num_bits, k, dw, s, ws, c->num_cus, st, c->timing ? &c->tm : nullptr, sweep,
                             fresh && first == 0, done));  // (each chunk's last kernel re-arms `done`)
    }
    return LSMB_OK;
}
}  // namespace

// Host single-key walks (the same arithmetic the kernels run).
template <class W, class F>
void walk_key(const uint8_t* key, uint64_t len, uint32_t num_bits, uint32_t k, F&& f) {
    const typename W::Mod md = W::Mod::make(num_bits);
    const H128 h = xxh3_128(key, len);
    W w(md, h.lo, h.hi);
    for (uint32_t i = 0; i < k; i++) {
        if (!f(w.pos())) return;
        w.next(md);
    }
}

template <class F>
void for_positions(const uint8_t* key, uint64_t len, uint32_t num_bits, uint32_t k, F&& f) {
    if (Mod14::fits(num_bits))
        walk_key<Walk14>(key, len, num_bits, k, f);
    else if (fits_walk32(num_bits))
        walk_key<Walk32>(key, len, num_bits, k, f);
    else
        walk_key<Walk64>(key, len, num_bits, k, f);
}

// offsets[0..n] must be non-decreasing (key i = data[offsets[i] .. offsets[i+1]).
int check_offsets(const uint64_t* offsets, uint64_t n) {
    for (uint64_t i = 0; i < n; i++)
        if (offsets[i + 1] < offsets[i])
            return fail(LSMB_EINVAL, "offsets not non-decreasing at %llu", (unsigned long long)i);
    return LSMB_OK;
}

uint64_t h2d_chunk_bytes() {
    const char* s = getenv("LSMB_H2D_CHUNK_MB");
    uint64_t mb = s ? strtoull(s, nullptr, 10) : 128;
    if (mb < 1) mb = 1;
    return mb << 20;
}

// Build from keys in host memory (the flush / compaction path: keys come from a
// memtable or merge iterator, src/db/mod.rs:379-383).  The keys go up in chunks
// of <= h2d_chunk_bytes() through two device staging slots: chunk i+1's H2D on
// the copy stream overlaps chunk i's kernels on the build stream, so the build
// hides under the PCIe transfer.  words_in == NULL starts from a zeroed filter
// (BloomFilter::new), else from those words (OR-accumulate); the finished words
// are copied to words_out (host, any alignment: lsmb_build_block points it at
// the serialized block body).  Synchronous.
// Small host builds (an SST flush of a few thousand keys): one pinned staging
// buffer, plain memcpys into and out of it and true async DMA on the build
// stream — pageable copies would each stage synchronously — and no copy
// stream.  Latency, not bandwidth, is what these calls pay.
constexpr uint64_t kSmallHostBuild = 1ull << 20;  // bytes of keys + offsets + words

int host_build_small(lsmb_ctx* c, const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                     uint32_t num_bits, uint32_t k, const uint64_t* words_in, uint8_t* words_out) {
    const uint64_t nw = nwords64(num_bits);
    const uint64_t base = offsets ? offsets[0] : 0;
    const uint64_t kbytes = offsets ? offsets[n] - base : n * (uint64_t)key_len;
    const uint64_t obytes = offsets ? (n + 1) * 8 : 0;
    const uint64_t kpad = (kbytes + 15) & ~15ull, opad = (obytes + 15) & ~15ull;
    const uint64_t need = kpad + opad + nw * 8 + 64;
    if (c->pin_small_cap < need) {
        c->pinned_retired.retire(c->pin_small);  // a D2H of an earlier call may not have left it
        c->pin_small = nullptr;
        c->pin_small_cap = 0;
        const uint64_t cap = std::max<uint64_t>(need, kSmallHostBuild + 64);
        if (hipHostMalloc((void**)&c->pin_small, cap, 0) != hipSuccess)
            return fail(LSMB_ENOMEM, "pinned staging (%llu B)", (unsigned long long)cap);
        c->pin_small_cap = cap;
    }
    uint8_t* pk = c->pin_small;
    uint64_t* po = (uint64_t*)(c->pin_small + kpad);
    uint64_t* pw = (uint64_t*)(c->pin_small + kpad + opad);
    HIP_TRY(c->words.ensure(nw * 8));
    HIP_TRY(c->kslot[0].ensure(kpad + 16));
    uint32_t* dw = (uint32_t*)c->words.p;
    // the previous small build's D2H out of this buffer has completed (synchronous calls)
    if (kbytes) memcpy(pk, data + base, kbytes);
    if (kbytes) HIP_TRY(hipMemcpyAsync(c->kslot[0].p, pk, kbytes, hipMemcpyHostToDevice, c->st));
    if (offsets) {
        for (uint64_t j = 0; j <= n; j++) po[j] = offsets[j] - base;
        HIP_TRY(c->oslot[0].ensure(obytes));
        HIP_TRY(hipMemcpyAsync(c->oslot[0].p, po, obytes, hipMemcpyHostToDevice, c->st));
    }
    if (words_in) {
        memcpy(pw, words_in, nw * 8);
        HIP_TRY(hipMemcpyAsync(dw, pw, nw * 8, hipMemcpyHostToDevice, c->st));
    } else {
        HIP_TRY(hipMemsetAsync(dw, 0, nw * 8, c->st));
    }
    KeyBatch kb{(const uint8_t*)c->kslot[0].p, offsets ? (const uint64_t*)c->oslot[0].p : nullptr, key_len,
                (!offsets && key_len == 0) ? 1 : n};
    if (int rc = build_dev(c, kb, num_bits, k, dw, c->st)) return rc;
    HIP_TRY(hipMemcpyAsync(pw, dw, nw * 8, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    memcpy(words_out, pw, nw * 8);
    return LSMB_OK;
}

int host_build_dev(lsmb_ctx* c, const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                   uint32_t num_bits, uint32_t k, uint32_t* dw) {
    if (!offsets && key_len == 0) {
        // every key is the empty key: one insert covers them all
        HIP_TRY(c->kslot[0].ensure(16));
        KeyBatch kb{(const uint8_t*)c->kslot[0].p, nullptr, 0, 1};
        if (int rc = build_dev(c, kb, num_bits, k, dw, c->st)) return rc;
        n = 0;
    }
    const uint64_t budget = h2d_chunk_bytes();
    const uint64_t max_keys = 32ull << 20;  // per chunk (bounds the offsets slot)
    uint64_t f = 0;
    for (int i = 0; f < n; i++) {
        const int s = i & 1;
        uint64_t e;
        if (offsets) {  // largest e with offsets[e] - offsets[f] <= budget, at least one key
            const uint64_t* hi = std::upper_bound(offsets + f + 1, offsets + n + 1, offsets[f] + budget);
            e = std::max<uint64_t>(f + 1, (uint64_t)(hi - offsets) - 1);
            e = std::min(e, f + max_keys);
        } else {
            e = std::min(n, f + std::max<uint64_t>(1, budget / key_len));
        }
        const uint64_t m = e - f;
        const uint64_t base = offsets ? offsets[f] : f * key_len;
        const uint64_t bytes = offsets ? offsets[e] - offsets[f] : m * key_len;
        // slot s was last read by chunk i-2's kernels
        if (i >= 2) HIP_TRY(hipEventSynchronize(c->ev_built[s]));
        HIP_TRY(c->kslot[s].ensure(std::max<uint64_t>(bytes, std::min(budget, n * (uint64_t)(key_len ? key_len : 1))) + 16));
        if (bytes) HIP_TRY(hipMemcpyAsync(c->kslot[s].p, data + base, bytes, hipMemcpyHostToDevice, c->cst));
        if (offsets) {
            if (c->offs_pin_cap[s] < m + 1) {
                c->pinned_retired.retire(c->offs_pin[s]);
                c->offs_pin[s] = nullptr;
                c->offs_pin_cap[s] = 0;
                const uint64_t cap = std::max<uint64_t>(m + 1, std::min<uint64_t>(n, max_keys) + 1);
                if (hipHostMalloc((void**)&c->offs_pin[s], cap * 8, 0) != hipSuccess)
                    return fail(LSMB_ENOMEM, "pinned offsets staging (%llu B)", (unsigned long long)(cap * 8));
                c->offs_pin_cap[s] = cap;
            }
            uint64_t* o = c->offs_pin[s];
            for (uint64_t j = 0; j <= m; j++) o[j] = offsets[f + j] - base;
            HIP_TRY(c->oslot[s].ensure(c->offs_pin_cap[s] * 8));
            HIP_TRY(hipMemcpyAsync(c->oslot[s].p, o, (m + 1) * 8, hipMemcpyHostToDevice, c->cst));
        }
        HIP_TRY(hipEventRecord(c->ev_copy[s], c->cst));
        HIP_TRY(hipStreamWaitEvent(c->st, c->ev_copy[s], 0));
        KeyBatch kb{(const uint8_t*)c->kslot[s].p, offsets ? (const uint64_t*)c->oslot[s].p : nullptr, key_len, m};
        if (int rc = build_dev(c, kb, num_bits, k, dw, c->st)) return rc;
        HIP_TRY(hipEventRecord(c->ev_built[s], c->st));
        f = e;
    }
    return LSMB_OK;
}

// crc (optional): CRC-32 of the words appended to *crc (the CRC of the bytes
// before them), computed on the device copy for device builds.
int host_build(lsmb_ctx* c, const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
               uint32_t num_bits, uint32_t k, const uint64_t* words_in, uint8_t* words_out, uint32_t* crc = nullptr) {
    const uint64_t nw = nwords64(num_bits);
    {
        const uint64_t kb = offsets ? offsets[n] - offsets[0] : n * (uint64_t)key_len;
        if (kb + (offsets ? (n + 1) * 8 : 0) + nw * 8 <= kSmallHostBuild) {
            const int rc = host_build_small(c, data, offsets, key_len, n, num_bits, k, words_in, words_out);
            if (!rc && crc) *crc = crc32_host(words_out, nw * 8, *crc);
            return rc;
        }
    }
    HIP_TRY(c->words.ensure(nw * 8));
    uint32_t* dw = (uint32_t*)c->words.p;
    if (words_in)
        HIP_TRY(hipMemcpyAsync(dw, words_in, nw * 8, hipMemcpyHostToDevice, c->st));
    else
        HIP_TRY(hipMemsetAsync(dw, 0, nw * 8, c->st));
    if (int rc = host_build_dev(c, data, offsets, key_len, n, num_bits, k, dw)) return rc;
    HIP_TRY(hipMemcpyAsync(words_out, dw, nw * 8, hipMemcpyDeviceToHost, c->st));
    if (crc) {
        if (int rc = crc32_dev(c, (const uint8_t*)dw, nw * 8, *crc, c->st, crc)) return rc;
    }
    HIP_TRY(hipStreamSynchronize(c->st));
    return LSMB_OK;
}

// The library's own host build: BloomFilter::insert per key
// (src/bloom/mod.rs:70-78) with the same xxh3 / exact-modulo code the kernels
// run, compiled for the host.  Used below host_max_keys(), where a device round
// trip (H2D, launch, D2H, sync: ~40 us) costs more than the whole loop.
template <class W>
static void host_insert_batch_w(const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                                uint32_t num_bits, uint32_t k, uint64_t* words) {
    const Mod32 md = Mod32::make(num_bits);
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t* key = offsets ? data + offsets[i] : data + i * (uint64_t)key_len;
        const uint64_t len = offsets ? offsets[i + 1] - offsets[i] : key_len;
        const H128 h = xxh3_128(key, len);
        W w(md, h.lo, h.hi);
        for (uint32_t j = 0; j < k; j++) {
            const uint32_t p = w.pos();
            words[p >> 6] |= 1ull << (p & 63);
            w.next(md);
        }
    }
}

void host_insert_batch(const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                       uint32_t num_bits, uint32_t k, uint64_t* words) {
    if (k == 0 || n == 0) return;
    if (fits_walk32(num_bits))
        host_insert_batch_w<Walk32>(data, offsets, key_len, n, num_bits, k, words);
    else
        host_insert_batch_w<Walk64>(data, offsets, key_len, n, num_bits, k, words);
}

bool bloom_params(uint64_t n, double fpr, uint32_t* num_bits, uint32_t* num_hashes) {
    if (n == 0 || !(fpr > 0.0 && fpr < 1.0)) return false;
    auto sat = [](double x) -> uint32_t {  // Rust `f64 as u32` saturates
        if (!(x == x) || x <= 0.0) return 0;
        if (x >= 4294967295.0) return 4294967295u;
        return (uint32_t)x;
    };
    const double bpk = -1.44 * log2(fpr);                      // mod.rs:46
    uint32_t nb = sat(ceil((double)n * bpk));                   // mod.rs:49
    if (nb < 64) nb = 64;                                       // mod.rs:52
    uint32_t k = sat(ceil(bpk * log(2.0)));                     // mod.rs:55
    if (k < 1) k = 1;                                           // mod.rs:56
    *num_bits = nb;
    *num_hashes = k;
    return true;
}

}  // namespace lsmb

extern "C" {

int lsmb_abi_version(void) { return LSMB_ABI_VERSION; }
const char* lsmb_last_error(void) { return last_error().c_str(); }

int lsmb_params(uint64_t n, double fpr, uint32_t* num_bits, uint32_t* num_hashes) {
    if (!num_bits || !num_hashes) return fail(LSMB_EINVAL, "null output pointer");
    if (n == 0) return fail(LSMB_EINVAL, "expected_items must be > 0");
    if (!bloom_params(n, fpr, num_bits, num_hashes)) return fail(LSMB_EINVAL, "FPR must be in (0, 1)");
    return LSMB_OK;
}

uint64_t lsmb_num_words(uint32_t num_bits) { return nwords64(num_bits); }
uint64_t lsmb_serialized_size(uint32_t num_bits) { return 12 + 8 * nwords64(num_bits); }

int lsmb_serialize(const uint64_t* words, uint32_t num_bits, uint32_t k, uint8_t* out, uint64_t out_len) {
    const uint64_t nw = nwords64(num_bits);
    if (out_len < 12 + 8 * nw) return fail(LSMB_EINVAL, "serialize: output buffer too small");
    if (nw && !words) return fail(LSMB_EINVAL, "serialize: null words");
    const uint32_t hdr[3] = {k, num_bits, (uint32_t)nw};
    for (int j = 0; j < 3; j++)
        for (int b = 0; b < 4; b++) out[4 * j + b] = (uint8_t)(hdr[j] >> (8 * b));
    // words are little-endian u64 on this (x86-64) host: a straight copy.
    if (nw) memcpy(out + 12, words, 8 * nw);
    return LSMB_OK;
}

int lsmb_deserialize_header(const uint8_t* data, uint64_t len, uint32_t* k, uint32_t* num_bits,
                            uint32_t* num_u64s) {
    if (len < 12 || !data) return fail(LSMB_ECORRUPT, "bloom filter too short for header");
    const uint32_t nh = rd32le(data), nb = rd32le(data + 4), nw = rd32le(data + 8);
    const uint64_t expect = nwords64(nb);
    if ((uint64_t)nw != expect)
        return fail(LSMB_ECORRUPT, "bloom filter num_u64s mismatch: got %u, expected %llu", nw,
                    (unsigned long long)expect);
    const uint64_t want = 12 + 8 * (uint64_t)nw;
    if (len != want)
        return fail(LSMB_ECORRUPT, "bloom filter data length mismatch: got %llu, expected %llu",
                    (unsigned long long)len, (unsigned long long)want);
    if (k) *k = nh;
    if (num_bits) *num_bits = nb;
    if (num_u64s) *num_u64s = nw;
    return LSMB_OK;
}

int lsmb_deserialize(const uint8_t* data, uint64_t len, uint64_t* words, uint64_t cap) {
    uint32_t k, nb, nw;
    int rc = lsmb_deserialize_header(data, len, &k, &nb, &nw);
    if (rc) return rc;
    if (cap < nw) return fail(LSMB_EINVAL, "deserialize: words buffer too small");
    if (nw) memcpy(words, data + 12, 8 * (uint64_t)nw);
    return LSMB_OK;
}

int lsmb_positions(const uint8_t* key, uint64_t len, uint32_t num_bits, uint32_t k, uint32_t* out) {
    if (int rc = check_filter(num_bits, k)) return rc;
    uint32_t i = 0;
    if (k) for_positions(key, len, num_bits, k, [&](uint32_t p) { out[i++] = p; return true; });
    return LSMB_OK;
}

int lsmb_insert(uint64_t* words, uint32_t num_bits, uint32_t k, const uint8_t* key, uint64_t len) {
    if (int rc = check_filter(num_bits, k)) return rc;
    if (k)
        for_positions(key, len, num_bits, k, [&](uint32_t p) {
            words[p >> 6] |= 1ull << (p & 63);
            return true;
        });
    return LSMB_OK;
}

int lsmb_may_contain(const uint64_t* words, uint32_t num_bits, uint32_t k, const uint8_t* key,
                     uint64_t len) {
    if (int rc = check_filter(num_bits, k)) return rc;
    bool all = true;  // k == 0: the reference's k-loop is empty -> true
    if (k)
        for_positions(key, len, num_bits, k, [&](uint32_t p) {
            all = (words[p >> 6] >> (p & 63)) & 1;
            return all;  // early exit on the first clear bit (mod.rs:88-90)
        });
    return all ? 1 : 0;
}

int lsmb_open(lsmb_ctx** out, int device) {
    if (!out) return fail(LSMB_EINVAL, "null ctx pointer");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(LSMB_ENODEV, "no HIP device visible (this engine runs its batched path on MI355X only)");
    if (device < 0 && hipGetDevice(&device) != hipSuccess) device = 0;
    if (device >= n) return fail(LSMB_ENODEV, "device %d out of range (%d visible)", device, n);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess)
        return fail(LSMB_ENODEV, "hipGetDeviceProperties(%d) failed", device);
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(LSMB_ENODEV, "device %d is %s; kernels are built for gfx950 only", device, prop.gcnArchName);
    lsmb_ctx* c = new lsmb_ctx;
    c->dev = device;
    c->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    DevGuard g(device);
    // The context's stream is a BLOCKING stream: it is ordered with the legacy
    // null stream, which is what torch's default stream is.  The device entry
    // points map stream == NULL to this stream, so a caller that allocates or
    // zeroes buffers on the null stream and then builds with stream == NULL
    // gets the two in order (tests/test_gpu_parity.py relies on it).  Two
    // contexts' blocking streams do not wait for each other; the library
    // itself issues nothing on the null stream after lsmb_open (the filter
    // set uploads on a non-blocking stream of its own).
    if (hipStreamCreateWithFlags(&c->st, hipStreamDefault) != hipSuccess ||
        hipEventCreateWithFlags(&c->desc_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ws_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreate(&c->tm.t0) != hipSuccess || hipEventCreate(&c->tm.t1) != hipSuccess ||
        hipEventCreate(&c->tm.t2) != hipSuccess ||
        hipStreamCreateWithFlags(&c->cst, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_copy[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_copy[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_built[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_built[1], hipEventDisableTiming) != hipSuccess) {
        delete c;
        return fail(LSMB_ENODEV, "stream/event creation failed on device %d", device);
    }
    if (c->err.ensure(64) != hipSuccess || hipMemsetAsync(c->err.p, 0, 64, c->st) != hipSuccess ||
        hipStreamSynchronize(c->st) != hipSuccess) {
        lsmb_close(c);
        return fail(LSMB_ENOMEM, "counter allocation failed on device %d", device);
    }
    *out = c;
    return LSMB_OK;
}

void lsmb_close(lsmb_ctx* c) {
    if (!c) return;
    {
        DevGuard g(c->dev);
        hipStreamSynchronize(c->st);
        if (c->cst) hipStreamSynchronize(c->cst);
        for (DevBuf* b : {&c->ws_regions, &c->ws_counts, &c->ws_hashes, &c->ws_ovf, &c->ws_dirty, &c->ws_ovl, &c->ws_ovn, &c->crc_parts, &c->err, &c->keys, &c->offs, &c->words, &c->out,
                          &c->filt_words, &c->filt_desc, &c->kslot[0], &c->kslot[1], &c->oslot[0], &c->oslot[1]})
            b->release();
        for (int s = 0; s < 2; s++) {
            if (c->offs_pin[s]) hipHostFree(c->offs_pin[s]);  // teardown
            if (c->ev_copy[s]) hipEventDestroy(c->ev_copy[s]);
            if (c->ev_built[s]) hipEventDestroy(c->ev_built[s]);
        }
        if (c->cst) hipStreamDestroy(c->cst);
        if (c->pin_small) hipHostFree(c->pin_small);  // teardown
        c->pinned_retired.release();
        hipEventDestroy(c->tm.t0);
        hipEventDestroy(c->tm.t1);
        hipEventDestroy(c->tm.t2);
        hipEventDestroy(c->desc_done);
        if (c->ws_done) hipEventDestroy(c->ws_done);
        if (c->desc_pinned) hipHostFree(c->desc_pinned);  // teardown
        hipStreamDestroy(c->st);
    }
    delete c;
}

int lsmb_sync(lsmb_ctx* c) {
    if (!c) return fail(LSMB_EINVAL, "null ctx");
    DevGuard g(c->dev);
    HIP_TRY(hipStreamSynchronize(c->st));
    report_stats(c);
    return LSMB_OK;
}

int lsmb_build_fixed_dev(lsmb_ctx* c, const void* d_keys, uint32_t key_len, uint64_t n,
                         uint32_t num_bits, uint32_t k, void* d_words, void* stream) {
    if (!c) return fail(LSMB_EINVAL, "null ctx");
    if (int rc = check_filter(num_bits, k)) return rc;
    if (n && (!d_keys || !d_words)) return fail(LSMB_EINVAL, "null device pointer");
    if (n && key_len == 0) {
        // every key is the empty key: one insert covers them all
        KeyBatch kb{(const uint8_t*)d_keys, nullptr, 0, 1};
        DevGuard g(c->dev);
        return build_dev(c, kb, num_bits, k, (uint32_t*)d_words, pick_stream(c, stream));
    }
    DevGuard g(c->dev);
    KeyBatch kb{(const uint8_t*)d_keys, nullptr, key_len, n};
    return build_dev(c, kb, num_bits, k, (uint32_t*)d_words, pick_stream(c, stream));
}

int lsmb_build_var_dev(lsmb_ctx* c, const void* d_data, const void* d_offsets, uint64_t n,
                       uint32_t num_bits, uint32_t k, void* d_words, void* stream) {
    if (!c) return fail(LSMB_EINVAL, "null ctx");
    if (int rc = check_filter(num_bits, k)) return rc;
    if (n && (!d_offsets || !d_words)) return fail(LSMB_EINVAL, "null device pointer");
    DevGuard g(c->dev);
    KeyBatch kb{(const uint8_t*)d_data, (const uint64_t*)d_offsets, 0, n};
    return build_dev(c, kb, num_bits, k, (uint32_t*)d_words, pick_stream(c, stream));
}

// BloomFilterBuilder::{new, add_key, build} (src/bloom/builder.rs:14-28): BloomFilter::new
// (src/bloom/mod.rs:38-67, all-zero words) + insert of every key.  The words
// are output-only: the partition build writes each of them once in pass B
// without reading it, so no zeroing pass and no read of the old words.
int lsmb_build_fixed_dev_new(lsmb_ctx* c, const void* d_keys, uint32_t key_len, uint64_t n, uint32_t num_bits,
                             uint32_t k, void* d_words, void* stream) {
    if (!c) return fail(LSMB_EINVAL, "null ctx");
    if (int rc = check_filter(num_bits, k)) return rc;
    if (!d_words || (n && !d_keys)) return fail(LSMB_EINVAL, "null device pointer");
    DevGuard g(c->dev);
    KeyBatch kb{(const uint8_t*)d_keys, nullptr, key_len, key_len ? n : (n ? 1 : 0)};
    return build_dev(c, kb, num_bits, k, (uint32_t*)d_words, pick_stream(c, stream), -1, /*fresh=*/true);
}

int lsmb_build_var_dev_new(lsmb_ctx* c, const void* d_data, const void* d_offsets, uint64_t n, uint32_t num_bits,
                           uint32_t k, void* d_words, void* stream) {
    if (!c) return fail(LSMB_EINVAL, "null ctx");
    if (int rc = check_filter(num_bits, k)) return rc;
    if (!d_words || (n && !d_offsets)) return fail(LSMB_EINVAL, "null device pointer");
    DevGuard g(c->dev);
    KeyBatch kb{(const uint8_t*)d_data, (const uint64_t*)d_offsets, 0, n};
    return build_dev(c, kb, num_bits, k, (uint32_t*)d_words, pick_stream(c, stream), -1, /*fresh=*/true);
}

// Builds of n <= host_max_keys() keys run the library's host loop (no device
// round trip, ctx may be NULL); bigger ones need a device context.
static int need_ctx(lsmb_ctx* c, uint64_t n) {
    if (!c)
        return fail(LSMB_EINVAL, "null ctx: builds of more than %llu keys run on the GPU (lsmb_host_max_keys)",
                    (unsigned long long)host_max_keys());
    (void)n;
    return LSMB_OK;
}

int lsmb_build_sweeps(uint32_t num_bits, uint32_t k, uint64_t n) {
    if (pick_build_strategy(num_bits, k, n) != BuildStrategy::Partition) return 1;
    return (int)plan_partition(num_bits, k, n, 256).sweeps;
}

int lsmb_sweep_words(uint32_t num_bits, uint32_t k, uint64_t n, int sweep, uint64_t* word_lo, uint64_t* word_hi) {
    if (!word_lo || !word_hi) return fail(LSMB_EINVAL, "null output pointer");
    const int ns = lsmb_build_sweeps(num_bits, k, n);
    if (sweep < 0 || sweep >= ns) return fail(LSMB_EINVAL, "sweep %d out of range [0, %d)", sweep, ns);
    const uint64_t nw = nwords64(num_bits);
    if (ns == 1) {
        *word_lo = 0;
        *word_hi = nw;
        return LSMB_OK;
    }
    const PartitionPlan pl = plan_partition(num_bits, k, n, 256);
    const uint64_t w_per_slice = (1ull << pl.slice_log2) / 64;
    *word_lo = std::min<uint64_t>(nw, (uint64_t)sweep * pl.bins_per_sweep * w_per_slice);
    *word_hi = std::min<uint64_t>(nw, ((uint64_t)sweep + 1) * pl.bins_per_sweep * w_per_slice);
    return LSMB_OK;
}

int lsmb_build_fixed_dev_sweep(lsmb_ctx* c, const void* d_keys, uint32_t key_len, uint64_t n, uint32_t num_bits,
                               uint32_t k, void* d_words, int sweep, void* stream) {
    if (!c) return fail(LSMB_EINVAL, "null ctx");
    if (int rc = check_filter(num_bits, k)) return rc;
    if (n && (!d_keys || !d_words)) return fail(LSMB_EINVAL, "null device pointer");
    const int ns = lsmb_build_sweeps(num_bits, k, n);
    if (sweep < 0 || sweep >= ns) return fail(LSMB_EINVAL, "sweep %d out of range [0, %d)", sweep, ns);
    DevGuard g(c->dev);
    KeyBatch kb{(const uint8_t*)d_keys, nullptr, key_len, key_len ? n : (n ? 1 : 0)};
    return build_dev(c, kb, num_bits, k, (uint32_t*)d_words, pick_stream(c, stream), sweep);
}

int lsmb_build_fixed_dev_sweep_new(lsmb_ctx* c, const void* d_keys, uint32_t key_len, uint64_t n, uint32_t num_bits,
                                   uint32_t k, void* d_words, int sweep, void* stream) {
    if (!c) return fail(LSMB_EINVAL, "null ctx");
    if (int rc = check_filter(num_bits, k)) return rc;
    if (!d_words || (n && !d_keys)) return fail(LSMB_EINVAL, "null device pointer");
    const int ns = lsmb_build_sweeps(num_bits, k, n);
    if (sweep < 0 || sweep >= ns) return fail(LSMB_EINVAL, "sweep %d out of range [0, %d)", sweep, ns);
    DevGuard g(c->dev);
    KeyBatch kb{(const uint8_t*)d_keys, nullptr, key_len, key_len ? n : (n ? 1 : 0)};
    return build_dev(c, kb, num_bits, k, (uint32_t*)d_words, pick_stream(c, stream), sweep, /*fresh=*/true);
}

int lsmb_build_fixed(lsmb_ctx* c, const uint8_t* keys, uint32_t key_len, uint64_t n, uint32_t num_bits,
                     uint32_t k, uint64_t* words) {
    if (int rc = check_filter(num_bits, k)) return rc;
    if (n == 0 || k == 0) return LSMB_OK;
    if (!keys && key_len) return fail(LSMB_EINVAL, "null keys");
    if (!words) return fail(LSMB_EINVAL, "null words");
    if (n <= host_max_keys()) {
        host_insert_batch(keys, nullptr, key_len, key_len ? n : 1, num_bits, k, words);
        return LSMB_OK;
    }
    if (int rc = need_ctx(c, n)) return rc;
    DevGuard g(c->dev);
    return host_build(c, keys, nullptr, key_len, n, num_bits, k, words, (uint8_t*)words);
}

int lsmb_build_var(lsmb_ctx* c, const uint8_t* data, const uint64_t* offsets, uint64_t n,
                   uint32_t num_bits, uint32_t k, uint64_t* words) {
    if (int rc = check_filter(num_bits, k)) return rc;
    if (n == 0 || k == 0) return LSMB_OK;
    if (!offsets || !words) return fail(LSMB_EINVAL, "null pointer");
    if (int rc = check_offsets(offsets, n)) return rc;
    if (n <= host_max_keys()) {
        host_insert_batch(data, offsets, 0, n, num_bits, k, words);
        return LSMB_OK;
    }
    if (int rc = need_ctx(c, n)) return rc;
    DevGuard g(c->dev);
    return host_build(c, data, offsets, 0, n, num_bits, k, words, (uint8_t*)words);
}

static int build_block(lsmb_ctx* c, const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                       uint32_t num_bits, uint32_t k, uint8_t* block, uint64_t block_len, uint32_t* crc) {
    if (int rc = check_filter(num_bits, k)) return rc;
    const uint64_t nw = nwords64(num_bits);
    const uint64_t size = 12 + 8 * nw;
    if (!block) return fail(LSMB_EINVAL, "null block");
    if (block_len < size)
        return fail(LSMB_EINVAL, "block buffer %llu B < serialized size %llu B", (unsigned long long)block_len,
                    (unsigned long long)size);
    if (n && !offsets && !data && key_len) return fail(LSMB_EINVAL, "null keys");
    if (n && offsets) {
        if (int rc = check_offsets(offsets, n)) return rc;
    }
    // header of BloomFilter::serialize (src/bloom/mod.rs:102-115)
    const uint32_t hdr[3] = {k, num_bits, (uint32_t)nw};
    for (int i = 0; i < 3; i++)
        for (int b = 0; b < 4; b++) block[4 * i + b] = (uint8_t)(hdr[i] >> (8 * b));
    if (n == 0 || k == 0) {  // new() + no inserts: all-zero words
        memset(block + 12, 0, nw * 8);
        if (crc) *crc = crc32_host(block, size, 0);
        return LSMB_OK;
    }
    if (n <= host_max_keys()) {
        // the block body is not 8-byte aligned (12-B header): build into an
        // aligned word array, then copy
        std::vector<uint64_t> w(nw, 0);
        host_insert_batch(data, offsets, key_len, (!offsets && key_len == 0) ? 1 : n, num_bits, k, w.data());
        memcpy(block + 12, w.data(), nw * 8);
        if (crc) *crc = crc32_host(block, size, 0);
        return LSMB_OK;
    }
    if (int rc = need_ctx(c, n)) return rc;
    DevGuard g(c->dev);
    if (crc) *crc = crc32_host(block, 12, 0);  // the header; the words' CRC is appended on the device
    return host_build(c, data, offsets, key_len, n, num_bits, k, nullptr, block + 12, crc);
}

int lsmb_build_block(lsmb_ctx* c, const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                     uint32_t num_bits, uint32_t k, uint8_t* block, uint64_t block_len) {
    return build_block(c, data, offsets, key_len, n, num_bits, k, block, block_len, nullptr);
}

int lsmb_build_block_crc(lsmb_ctx* c, const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                         uint32_t num_bits, uint32_t k, uint8_t* block, uint64_t block_len, uint32_t* crc) {
    if (!crc) return fail(LSMB_EINVAL, "null crc");
    return build_block(c, data, offsets, key_len, n, num_bits, k, block, block_len, crc);
}



uint64_t lsmb_host_max_keys(void) { return host_max_keys(); }

void lsmb_set_host_max_keys(uint64_t n) { set_host_max_keys(n); }

// Copies a host key batch into the context's staging buffers (ctx stream).
static int stage_host_keys(lsmb_ctx* c, const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                           KeyBatch* kb) {
    uint64_t kbytes;
    if (offsets) {
        for (uint64_t i = 0; i < n; i++)
            if (offsets[i + 1] < offsets[i]) return fail(LSMB_EINVAL, "offsets not non-decreasing");
        kbytes = offsets[n] - offsets[0];
        c->offs_tmp.resize(n + 1);
        for (uint64_t i = 0; i <= n; i++) c->offs_tmp[i] = offsets[i] - offsets[0];
        HIP_TRY(c->offs.ensure((n + 1) * 8));
        HIP_TRY(hipMemcpyAsync(c->offs.p, c->offs_tmp.data(), (n + 1) * 8, hipMemcpyHostToDevice, c->st));
        HIP_TRY(c->keys.ensure(kbytes + 16));
        if (kbytes) HIP_TRY(hipMemcpyAsync(c->keys.p, data + offsets[0], kbytes, hipMemcpyHostToDevice, c->st));
    } else {
        kbytes = (uint64_t)key_len * n;
        HIP_TRY(c->keys.ensure(kbytes + 16));
        if (kbytes) HIP_TRY(hipMemcpyAsync(c->keys.p, data, kbytes, hipMemcpyHostToDevice, c->st));
    }
    *kb = KeyBatch{(const uint8_t*)c->keys.p, offsets ? (const uint64_t*)c->offs.p : nullptr, key_len, n};
    return LSMB_OK;
}

static int probe_common(lsmb_ctx* c, const uint32_t* const* wptrs, const uint32_t* filt_bits,
                        const uint32_t* filt_k, uint32_t nfilt, const KeyBatch& kb, uint8_t* d_out,
                        hipStream_t st) {
    if (nfilt == 0 || nfilt > 64) return fail(LSMB_EINVAL, "nfilt must be in [1, 64]");
    c->hfilt.resize(nfilt);
    for (uint32_t f = 0; f < nfilt; f++) {
        if (int rc = check_filter(filt_bits[f], filt_k[f])) return rc;
        ProbeFilter& p = c->hfilt[f];
        memset(&p, 0, sizeof p);
        p.words32 = wptrs[f];
        p.md = Mod32::make(filt_bits[f] ? filt_bits[f] : 1);
        p.num_bits = filt_bits[f];
        p.k = filt_k[f];
        p.out_bit = f;
        p.group = f;
    }
    if (kb.n == 0) return LSMB_OK;  // (no launch: nothing would complete the guard event below)
    // The bit-sliced kernels (filters sharing one size, the store's SST
    // filters) take the filters in their kernel arguments: nothing to upload
    // and no event to record, so back-to-back probes are back-to-back kernels.
    if (!probe_reads_descriptors(c->hfilt.data(), nfilt)) {
        HIP_TRY(launch_probe(kb, c->hfilt.data(), nfilt, nullptr, d_out, c->num_cus, st));
        return LSMB_OK;
    }
    // Descriptors go to the device only when they change (a probe loop over the
    // same level filters re-uses them); the upload waits for the last kernel
    // that read the previous set, so no host sync sits between repeat probes.
    HIP_TRY(c->filt_desc.ensure(sizeof(ProbeFilter) * 64));
    const bool same = c->desc_uploaded.size() == nfilt &&
                      memcmp(c->desc_uploaded.data(), c->hfilt.data(), sizeof(ProbeFilter) * nfilt) == 0;
    if (!same) {
        if (!c->desc_pinned) HIP_TRY(hipHostMalloc((void**)&c->desc_pinned, sizeof(ProbeFilter) * 64, 0));
        HIP_TRY(hipEventSynchronize(c->desc_done));
        memcpy(c->desc_pinned, c->hfilt.data(), sizeof(ProbeFilter) * nfilt);
        HIP_TRY(hipMemcpyAsync(c->filt_desc.p, c->desc_pinned, sizeof(ProbeFilter) * nfilt,
                               hipMemcpyHostToDevice, st));
        c->desc_uploaded = c->hfilt;
    }
    HIP_TRY(launch_probe(kb, c->hfilt.data(), nfilt, (ProbeFilter*)c->filt_desc.p, d_out, c->num_cus, st,
                         c->desc_done));  // (the dispatch completes the guard event)
    return LSMB_OK;
}

int lsmb_probe_dev(lsmb_ctx* c, const void* const* d_filt_words, const uint32_t* filt_bits,
                   const uint32_t* filt_k, uint32_t nfilt, const void* d_data, const void* d_offsets,
                   uint32_t key_len, uint64_t n, void* d_out, void* stream) {
    if (!c) return fail(LSMB_EINVAL, "null ctx");
    if (!d_filt_words || !filt_bits || !filt_k) return fail(LSMB_EINVAL, "null filter arrays");
    if (n && !d_out) return fail(LSMB_EINVAL, "null output");
    DevGuard g(c->dev);
    KeyBatch kb{(const uint8_t*)d_data, (const uint64_t*)d_offsets, key_len, n};
    return probe_common(c, (const uint32_t* const*)d_filt_words, filt_bits, filt_k, nfilt, kb,
                        (uint8_t*)d_out, pick_stream(c, stream));
}

int lsmb_probe(lsmb_ctx* c, const uint64_t* const* filt_words, const uint32_t* filt_bits,
               const uint32_t* filt_k, uint32_t nfilt, const uint8_t* data, const uint64_t* offsets,
               uint32_t key_len, uint64_t n, uint8_t* out) {
    if (!c) return fail(LSMB_EINVAL, "null ctx");
    if (!filt_words || !filt_bits || !filt_k) return fail(LSMB_EINVAL, "null filter arrays");
    if (nfilt == 0 || nfilt > 64) return fail(LSMB_EINVAL, "nfilt must be in [1, 64]");
    if (n == 0) return LSMB_OK;
    if (!out) return fail(LSMB_EINVAL, "null output");
    DevGuard g(c->dev);
    // filters -> one device arena
    uint64_t tot = 0;
    std::vector<uint64_t> at(nfilt);
    for (uint32_t f = 0; f < nfilt; f++) {
        at[f] = tot;
        tot += (nwords64(filt_bits[f]) + 1) & ~1ull;  // keep 16-B alignment
    }
    HIP_TRY(c->filt_words.ensure(std::max<uint64_t>(tot, 2) * 8));
    std::vector<const uint32_t*> dptr(nfilt);
    for (uint32_t f = 0; f < nfilt; f++) {
        uint64_t* d = (uint64_t*)c->filt_words.p + at[f];
        if (nwords64(filt_bits[f]))
            HIP_TRY(hipMemcpyAsync(d, filt_words[f], nwords64(filt_bits[f]) * 8, hipMemcpyHostToDevice, c->st));
        dptr[f] = (const uint32_t*)d;
    }
    const uint32_t stride = (nfilt + 7) / 8;
    HIP_TRY(c->out.ensure(n * stride));
    KeyBatch kb;
    if (int rc = stage_host_keys(c, data, offsets, key_len, n, &kb)) return rc;
    if (int rc = probe_common(c, dptr.data(), filt_bits, filt_k, nfilt, kb, (uint8_t*)c->out.p, c->st)) return rc;
    HIP_TRY(hipMemcpyAsync(out, c->out.p, n * stride, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return LSMB_OK;
}

int lsmb_or_reduce_dev(lsmb_ctx* c, void* dst, const void* src, uint64_t nwords, uint32_t nsrc,
                       uint64_t stride_words, void* stream) {
    if (!c) return fail(LSMB_EINVAL, "null ctx");
    if (nwords == 0 || nsrc == 0) return LSMB_OK;
    DevGuard g(c->dev);
    HIP_TRY(launch_or_reduce((uint32_t*)dst, (const uint32_t*)src, 2 * nwords, nsrc, 2 * stride_words,
                             pick_stream(c, stream)));
    return LSMB_OK;
}

int lsmb_gen_splitmix_dev(lsmb_ctx* c, uint64_t seed, uint64_t first, uint64_t n, uint32_t mod, uint32_t add,
                          void* d_out, void* stream) {
    if (!c) return fail(LSMB_EINVAL, "null ctx");
    if (n && !d_out) return fail(LSMB_EINVAL, "null device pointer");
    if (((uintptr_t)d_out) & 7) return fail(LSMB_EINVAL, "d_out must be 8-byte aligned");
    DevGuard g(c->dev);
    HIP_TRY(launch_gen_splitmix(seed, first, n, mod, add, (uint64_t*)d_out, pick_stream(c, stream)));
    return LSMB_OK;
}

int lsmb_gen_key16_dev(lsmb_ctx* c, uint64_t seed, uint64_t first, uint64_t n, void* d_keys, void* stream) {
    if (!c) return fail(LSMB_EINVAL, "null ctx");
    if (n == 0) return LSMB_OK;
    if (reinterpret_cast<uintptr_t>(d_keys) & 15) return fail(LSMB_EINVAL, "d_keys must be 16-byte aligned");
    DevGuard g(c->dev);
    HIP_TRY(launch_gen_key16(seed, first, n, (uint8_t*)d_keys, pick_stream(c, stream)));
    return LSMB_OK;
}

const char* lsmb_build_strategy(uint32_t num_bits, uint32_t k, uint64_t n) {
    return strategy_name(pick_build_strategy(num_bits, k, n));
}

int lsmb_set_timing(lsmb_ctx* c, int enable) {
    if (!c) return fail(LSMB_EINVAL, "null ctx");
    c->timing = enable != 0;
    return LSMB_OK;
}

int lsmb_last_build_ms(lsmb_ctx* c, float* out3) {
    if (!c || !out3) return fail(LSMB_EINVAL, "null argument");
    if (!c->tm.valid) return fail(LSMB_EINVAL, "no timed build on this context");
    DevGuard g(c->dev);
    // the build may run on a caller's stream: wait for its end marker, not c->st
    HIP_TRY(hipEventSynchronize(c->tm.t2));
    HIP_TRY(hipEventElapsedTime(&out3[0], c->tm.t0, c->tm.t2));
    HIP_TRY(hipEventElapsedTime(&out3[1], c->tm.t0, c->tm.t1));
    HIP_TRY(hipEventElapsedTime(&out3[2], c->tm.t1, c->tm.t2));
    return LSMB_OK;
}

// ---------------------------------------------------------------- filter sets
// A device-resident set of up to 64 SSTable filters with their key ranges:
// the multi-get pre-check of DB::get (src/db/mod.rs:243-267 -> SSTable::get,
// src/sstable/reader.rs:192-199), without re-opening and re-deserializing
// every table per lookup (mod.rs:245,259).
struct lsmb_fset {
    lsmb_ctx* c = nullptr;
    struct Slot {
        bool live = false;
        DevBuf words;
        uint32_t num_bits = 0, k = 0;
        std::vector<uint8_t> lo, hi;
    };
    Slot slot[64];
    DevBuf ranges;  // the distinct boundary keys' bytes
    DevBuf points;  // FsetPoint[npts] then regmask[2 * npts + 1]
    DevBuf desc;    // RangedFilter[ndesc]
    FsetRanges rg{};
    FsetClasses cl{};
    uint32_t ndesc = 0;
    uint32_t shared_nb = 0, shared_k = 0;  // (num_bits, k) of every live slot, or 0 when they differ
    bool dirty = true;
    // Uploads go through the set's own non-blocking stream; before a buffer a
    // probe may still read is rewritten, the host waits for the events
    // recorded after this set's probes (one per stream used) — never for the
    // whole device, so another context's builds keep running.
    hipStream_t ust = nullptr;
    std::vector<std::pair<hipStream_t, hipEvent_t>> probe_ev;
};

namespace {

int fset_wait_probes(lsmb_fset* fs) {
    for (auto& pe : fs->probe_ev) HIP_TRY(hipEventSynchronize(pe.second));
    return LSMB_OK;
}

// After a probe on stream st: remember it so later rewrites wait for it.  At
// most kFsetProbeStreams streams are tracked (a caller probing on pooled or
// per-request streams would otherwise grow the list, and every add would wait
// on all of it): a new stream past that takes the least recently used entry,
// whose probe the host waits for first.
constexpr size_t kFsetProbeStreams = 4;

// The event that will mark the completion of the next probe on stream st
// (the set's buffers are rewritten only after every probe that reads them
// is done): one per stream, at most kFsetProbeStreams of them, the least
// recently used evicted after a wait.  The probe's own dispatch completes it
// (launch_done), so repeated probes put no marker packets in the stream.
int fset_probe_event(lsmb_fset* fs, hipStream_t st, hipEvent_t* out) {
    for (size_t i = 0; i < fs->probe_ev.size(); i++)
        if (fs->probe_ev[i].first == st) {
            *out = fs->probe_ev[i].second;
            std::rotate(fs->probe_ev.begin() + i, fs->probe_ev.begin() + i + 1, fs->probe_ev.end());  // most recent last
            return LSMB_OK;
        }
    hipEvent_t ev;
    if (fs->probe_ev.size() < kFsetProbeStreams) {
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    } else {
        ev = fs->probe_ev.front().second;
        HIP_TRY(hipEventSynchronize(ev));
        fs->probe_ev.erase(fs->probe_ev.begin());
    }
    fs->probe_ev.push_back({st, ev});
    *out = ev;
    return LSMB_OK;
}

// Rebuilds the device descriptors after an add/remove (rare; probes re-use
// them): the descriptors, and the sorted boundary points of the live tables'
// key ranges with one in-range mask per region (FsetRanges, kernels.hpp).
int fset_refresh(lsmb_fset* fs) {
    if (!fs->dirty) return LSMB_OK;
    std::vector<const lsmb_fset::Slot*> live;
    std::vector<uint32_t> slot_of;
    for (uint32_t s = 0; s < 64; s++)
        if (fs->slot[s].live) {
            live.push_back(&fs->slot[s]);
            slot_of.push_back(s);
        }
    // distinct bounds, sorted as Rust's [u8] Ord (std::vector<uint8_t> < is
    // the same unsigned lexicographic order, a proper prefix first)
    std::vector<std::vector<uint8_t>> pts;
    for (const auto* S : live) {
        pts.push_back(S->lo);
        pts.push_back(S->hi);
    }
    std::sort(pts.begin(), pts.end());
    pts.erase(std::unique(pts.begin(), pts.end()), pts.end());
    const uint32_t m = (uint32_t)pts.size();
    // region masks over descriptor indices: region 2r = (P[r-1], P[r]),
    // region 2r+1 = {P[r]}
    std::vector<uint64_t> regmask(2 * m + 1, 0);
    for (uint32_t d = 0; d < live.size(); d++) {
        const auto* S = live[d];
        if (S->hi < S->lo) continue;  // an empty range holds no key
        const uint32_t a = (uint32_t)(std::lower_bound(pts.begin(), pts.end(), S->lo) - pts.begin());
        const uint32_t b = (uint32_t)(std::lower_bound(pts.begin(), pts.end(), S->hi) - pts.begin());
        for (uint32_t reg = 2 * a + 1; reg <= 2 * b + 1; reg++) regmask[reg] |= 1ull << d;
    }
    std::vector<uint8_t> blob;
    std::vector<uint64_t> at;
    for (const auto& p : pts) {
        at.push_back(blob.size());
        blob.insert(blob.end(), p.begin(), p.end());
    }
    if (int rc = fset_wait_probes(fs)) return rc;  // no probe may still read the old descriptors
    // grow geometrically from 4 KiB (an outgrown buffer is retired, not freed:
    // DevBuf)
    size_t want = 4096;
    while (want < blob.size()) want *= 2;
    HIP_TRY(fs->ranges.ensure(want));
    if (!blob.empty()) HIP_TRY(hipMemcpyAsync(fs->ranges.p, blob.data(), blob.size(), hipMemcpyHostToDevice, fs->ust));
    const uint8_t* rb = (const uint8_t*)fs->ranges.p;
    std::vector<uint8_t> pbuf(sizeof(FsetPoint) * kFsetMaxPoints + 8 * (2 * kFsetMaxPoints + 1));
    FsetPoint* fp = (FsetPoint*)pbuf.data();
    for (uint32_t j = 0; j < m; j++) {
        const auto& p = pts[j];
        uint8_t pad[16] = {0};
        memcpy(pad, p.data(), std::min<size_t>(16, p.size()));
        uint64_t w0 = 0, w1 = 0;
        for (int b = 0; b < 8; b++) {
            w0 = (w0 << 8) | pad[b];
            w1 = (w1 << 8) | pad[8 + b];
        }
        fp[j].w0 = w0;
        fp[j].w1 = w1;
        fp[j].p = rb + at[j];
        fp[j].len = (uint32_t)p.size();
        fp[j].pad = 0;
    }
    memcpy(pbuf.data() + sizeof(FsetPoint) * m, regmask.data(), 8 * regmask.size());
    HIP_TRY(fs->points.ensure(pbuf.size()));
    HIP_TRY(hipMemcpyAsync(fs->points.p, pbuf.data(), sizeof(FsetPoint) * m + 8 * regmask.size(), hipMemcpyHostToDevice,
                           fs->ust));
    fs->rg.pts = (const FsetPoint*)fs->points.p;
    fs->rg.regmask = (const uint64_t*)((const uint8_t*)fs->points.p + sizeof(FsetPoint) * m);
    fs->rg.npts = m;
    std::vector<RangedFilter> d;
    for (uint32_t j = 0; j < live.size(); j++) {
        const auto* S = live[j];
        RangedFilter r;
        memset(&r, 0, sizeof r);
        r.f.words32 = (const uint32_t*)S->words.p;
        r.f.md = Mod32::make(S->num_bits ? S->num_bits : 1);
        r.f.num_bits = S->num_bits;
        r.f.k = S->k;
        r.f.out_bit = slot_of[j];
        r.f.group = slot_of[j];
        d.push_back(r);
    }
    HIP_TRY(fs->desc.ensure(sizeof(RangedFilter) * 64));
    if (!d.empty())
        HIP_TRY(hipMemcpyAsync(fs->desc.p, d.data(), sizeof(RangedFilter) * d.size(), hipMemcpyHostToDevice, fs->ust));
    // size classes: descriptors grouped by (num_bits, k); the classes with the
    // smallest tables go to LDS first (most filters per byte), the rest and
    // k = 0 filters are walked from L2
    std::vector<FsetClass> cls;
    {
        std::vector<std::pair<uint64_t, uint32_t>> keyd;  // (num_bits << 32 | k, descriptor)
        for (uint32_t j = 0; j < d.size(); j++)
            if (d[j].f.k) keyd.push_back({((uint64_t)d[j].f.num_bits << 32) | d[j].f.k, j});
        std::sort(keyd.begin(), keyd.end());
        std::vector<FsetClass> all;
        for (size_t a = 0; a < keyd.size();) {
            size_t b = a;
            while (b < keyd.size() && keyd[b].first == keyd[a].first) b++;
            FsetClass c;
            memset(&c, 0, sizeof c);
            c.num_bits = (uint32_t)(keyd[a].first >> 32);
            c.k = (uint32_t)keyd[a].first;
            c.md = Mod32::make(c.num_bits);
            c.md14 = Mod14::make(Mod14::fits(c.num_bits) ? c.num_bits : 1);
            c.nmem = (uint32_t)(b - a);
            c.width = c.nmem <= 8 ? 1 : c.nmem <= 16 ? 2 : c.nmem <= 32 ? 4 : 8;
            for (size_t j = a; j < b; j++) {
                c.mem[j - a] = (uint8_t)keyd[j].second;
                c.mask |= 1ull << keyd[j].second;
            }
            all.push_back(c);
            a = b;
        }
        auto tbytes = [](const FsetClass& c) { return (((uint64_t)c.num_bits + 31) / 32) * 32 * c.width; };
        std::stable_sort(all.begin(), all.end(),
                         [&](const FsetClass& x, const FsetClass& y) { return tbytes(x) < tbytes(y); });
        uint64_t off = 0, in_lds = 0;
        for (auto& c : all) {
            const uint64_t tb = (tbytes(c) + 15) & ~15ull;
            if (cls.size() < kFsetMaxClasses && off + tb <= kFsetTableBytes) {
                c.off = (uint32_t)off;
                off += tb;
                in_lds |= c.mask;
                cls.push_back(c);
            }
        }
        uint64_t all_desc = d.size() == 64 ? ~0ull : (1ull << d.size()) - 1;
        fs->cl.ncls = (uint32_t)cls.size();
        fs->cl.table_bytes = (uint32_t)off;
        fs->cl.walk_mask = all_desc & ~in_lds;
    }
    for (size_t i = 0; i < cls.size(); i++) fs->cl.cls[i] = cls[i];
    HIP_TRY(hipStreamSynchronize(fs->ust));  // blob, pbuf and d are host temporaries
    fs->ndesc = (uint32_t)d.size();
    fs->shared_nb = d.empty() ? 0 : d[0].f.num_bits;
    fs->shared_k = d.empty() ? 0 : d[0].f.k;
    for (const auto& r : d)
        if (r.f.num_bits != fs->shared_nb || r.f.k != fs->shared_k) fs->shared_nb = fs->shared_k = 0;
    fs->dirty = false;
    return LSMB_OK;
}

// expect_crc (optional): CRC-32 of the whole serialized block (`hdr` = its
// 12-B header), checked against the device copy before the slot goes live.
int fset_add_common(lsmb_fset* fs, const uint8_t* words_le, uint32_t num_bits, uint32_t k, const uint8_t* min_key,
                    uint64_t min_len, const uint8_t* max_key, uint64_t max_len, const uint8_t* hdr = nullptr,
                    const uint32_t* expect_crc = nullptr) {
    if (int rc = check_filter(num_bits, k)) return rc;
    if ((min_len && !min_key) || (max_len && !max_key)) return fail(LSMB_EINVAL, "null key range");
    if (min_len > UINT32_MAX || max_len > UINT32_MAX) return fail(LSMB_EINVAL, "range key too long");
    int s = 0;
    while (s < 64 && fs->slot[s].live) s++;
    if (s == 64) return fail(LSMB_EINVAL, "filter set full (64 filters)");
    DevGuard g(fs->c->dev);
    auto& S = fs->slot[s];
    const uint64_t nw = nwords64(num_bits);
    if (int rc = fset_wait_probes(fs)) return rc;  // the slot's old buffer may still be read by a probe
    HIP_TRY(S.words.ensure(std::max<uint64_t>(nw, 2) * 8));
    if (nw) {
        HIP_TRY(hipMemcpyAsync(S.words.p, words_le, nw * 8, hipMemcpyHostToDevice, fs->ust));
        HIP_TRY(hipStreamSynchronize(fs->ust));
    }
    if (expect_crc) {  // the copy now in HBM, not the host bytes, is what probes will read
        uint32_t got = 0;
        if (int rc = crc32_dev(fs->c, (const uint8_t*)S.words.p, nw * 8, crc32_host(hdr, 12, 0), fs->ust, &got))
            return rc;
        if (got != *expect_crc)
            return fail(LSMB_ECORRUPT, "bloom block CRC-32 mismatch: expected %08x, device copy %08x", *expect_crc, got);
    }
    S.num_bits = num_bits;
    S.k = k;
    S.lo.assign(min_key, min_key + min_len);
    S.hi.assign(max_key, max_key + max_len);
    S.live = true;
    fs->dirty = true;
    return s;
}

}  // namespace

int lsmb_fset_open(lsmb_ctx* c, lsmb_fset** out) {
    if (!c || !out) return fail(LSMB_EINVAL, "null argument");
    *out = nullptr;
    DevGuard g(c->dev);
    lsmb_fset* fs = new lsmb_fset;
    fs->c = c;
    if (hipStreamCreateWithFlags(&fs->ust, hipStreamNonBlocking) != hipSuccess) {
        delete fs;
        return fail(LSMB_EHIP, "filter set: stream creation failed");
    }
    *out = fs;
    return LSMB_OK;
}

void lsmb_fset_close(lsmb_fset* fs) {
    if (!fs) return;
    {
        DevGuard g(fs->c->dev);
        fset_wait_probes(fs);
        for (auto& pe : fs->probe_ev) hipEventDestroy(pe.second);
        if (fs->ust) hipStreamSynchronize(fs->ust), hipStreamDestroy(fs->ust);
        for (auto& S : fs->slot) S.words.release();
        fs->ranges.release();
        fs->points.release();
        fs->desc.release();
    }
    delete fs;
}

int lsmb_fset_add(lsmb_fset* fs, const uint8_t* block, uint64_t len, const uint8_t* min_key, uint64_t min_len,
                  const uint8_t* max_key, uint64_t max_len) {
    if (!fs) return fail(LSMB_EINVAL, "null filter set");
    uint32_t k, nb, nw;
    if (int rc = lsmb_deserialize_header(block, len, &k, &nb, &nw)) return rc;
    return fset_add_common(fs, block + 12, nb, k, min_key, min_len, max_key, max_len);
}

int lsmb_fset_add_crc(lsmb_fset* fs, const uint8_t* block, uint64_t len, uint32_t crc, const uint8_t* min_key,
                      uint64_t min_len, const uint8_t* max_key, uint64_t max_len) {
    if (!fs) return fail(LSMB_EINVAL, "null filter set");
    uint32_t k, nb, nw;
    if (int rc = lsmb_deserialize_header(block, len, &k, &nb, &nw)) return rc;
    return fset_add_common(fs, block + 12, nb, k, min_key, min_len, max_key, max_len, block, &crc);
}

int lsmb_fset_add_words(lsmb_fset* fs, const uint64_t* words, uint32_t num_bits, uint32_t num_hashes,
                        const uint8_t* min_key, uint64_t min_len, const uint8_t* max_key, uint64_t max_len) {
    if (!fs) return fail(LSMB_EINVAL, "null filter set");
    if (!words && nwords64(num_bits)) return fail(LSMB_EINVAL, "null words");
    return fset_add_common(fs, (const uint8_t*)words, num_bits, num_hashes, min_key, min_len, max_key, max_len);
}

int lsmb_fset_remove(lsmb_fset* fs, int slot) {
    if (!fs) return fail(LSMB_EINVAL, "null filter set");
    if (slot < 0 || slot >= 64 || !fs->slot[slot].live) return fail(LSMB_EINVAL, "no filter in slot %d", slot);
    fs->slot[slot].live = false;  // the buffer is re-used by a later add
    fs->dirty = true;
    return LSMB_OK;
}

uint64_t lsmb_fset_live_mask(const lsmb_fset* fs) {
    uint64_t m = 0;
    if (fs)
        for (int s = 0; s < 64; s++)
            if (fs->slot[s].live) m |= 1ull << s;
    return m;
}

int lsmb_fset_probe_dev_rows(lsmb_fset* fs, const void* d_data, const void* d_offsets, uint32_t key_len, uint64_t n,
                             void* d_out, uint32_t row_bytes, void* stream) {
    if (!fs) return fail(LSMB_EINVAL, "null filter set");
    if (row_bytes != 1 && row_bytes != 2 && row_bytes != 4 && row_bytes != 8)
        return fail(LSMB_EINVAL, "row_bytes must be 1, 2, 4 or 8");
    const uint64_t live = lsmb_fset_live_mask(fs);
    if (row_bytes < 8 && (live >> (8 * row_bytes)) != 0)
        return fail(LSMB_EINVAL, "a live slot does not fit %u-byte rows", row_bytes);
    if (n == 0) return LSMB_OK;
    if (!d_out || !d_data) return fail(LSMB_EINVAL, "null keys or output");
    DevGuard g(fs->c->dev);
    if (int rc = fset_refresh(fs)) return rc;
    const hipStream_t st = pick_stream(fs->c, stream);
    if (fs->ndesc == 0) {
        HIP_TRY(hipMemsetAsync(d_out, 0, n * row_bytes, st));
        return LSMB_OK;
    }
    KeyBatch kb{(const uint8_t*)d_data, (const uint64_t*)d_offsets, key_len, n};
    hipEvent_t ev;
    if (int rc = fset_probe_event(fs, st, &ev)) return rc;
    HIP_TRY(launch_fset_probe(kb, (const RangedFilter*)fs->desc.p, fs->ndesc, fs->rg, fs->cl, fs->shared_nb, fs->shared_k,
                              (uint8_t*)d_out, row_bytes, fs->c->num_cus, st, ev));
    return LSMB_OK;
}

int lsmb_fset_probe_dev(lsmb_fset* fs, const void* d_data, const void* d_offsets, uint32_t key_len, uint64_t n,
                        void* d_out, void* stream) {
    return lsmb_fset_probe_dev_rows(fs, d_data, d_offsets, key_len, n, d_out, 8, stream);
}

int lsmb_fset_probe(lsmb_fset* fs, const uint8_t* data, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                    uint64_t* out_mask) {
    if (!fs) return fail(LSMB_EINVAL, "null filter set");
    if (n == 0) return LSMB_OK;
    if (!out_mask || (!data && (offsets ? offsets[n] > offsets[0] : key_len > 0)))
        return fail(LSMB_EINVAL, "null keys or output");
    lsmb_ctx* c = fs->c;
    DevGuard g(c->dev);
    if (int rc = fset_refresh(fs)) return rc;
    HIP_TRY(c->out.ensure(n * 8));
    KeyBatch kb;
    if (int rc = stage_host_keys(c, data, offsets, key_len, n, &kb)) return rc;
    if (fs->ndesc == 0) {
        memset(out_mask, 0, n * 8);
        return LSMB_OK;
    }
    hipEvent_t ev;
    if (int rc = fset_probe_event(fs, c->st, &ev)) return rc;
    HIP_TRY(launch_fset_probe(kb, (const RangedFilter*)fs->desc.p, fs->ndesc, fs->rg, fs->cl, fs->shared_nb, fs->shared_k,
                              (uint8_t*)c->out.p, 8, c->num_cus, c->st, ev));
    HIP_TRY(hipMemcpyAsync(out_mask, c->out.p, n * 8, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return LSMB_OK;
}

}  // extern "C"
