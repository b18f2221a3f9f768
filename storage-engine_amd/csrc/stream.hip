// stream.hip — key ingestion from host structures while they are walked.
//
// The store's flush walks the frozen memtable and adds every key to the
// SSTable builder (src/db/mod.rs:379-383 -> SSTableBuilder::add ->
// BloomFilterBuilder::add_key, src/sstable/builder.rs:93,
// src/bloom/builder.rs:21-23); compaction does the same over its merged
// entries (src/compaction/scheduler.rs:113-125,152-158).  An lsmb_stream is
// that add_key loop on the GPU path: each key is appended to pinned host
// staging (a memcpy, no hashing), and every time a staging chunk fills it is
// uploaded on the context's copy stream and built on its build stream while
// the caller keeps walking and appending into the other chunk.  At finish the
// last partial chunk goes up, and the words come straight back into the
// serialized bloom block.  A run that stays at or below lsmb_host_max_keys()
// keys never touches the device: finish builds it with the host loop.
#include <string.h>

#include <algorithm>

#include "ctx.hpp"

using namespace lsmb;

namespace {

uint64_t stream_chunk_bytes() {
    const char* s = getenv("LSMB_STREAM_CHUNK_MB");
    uint64_t mb = s ? strtoull(s, nullptr, 10) : 128;
    if (mb < 1) mb = 1;
    return mb << 20;
}

constexpr uint64_t kStreamMinBytes = 64 << 10;  // first pinned allocation (grows x2 up to the chunk)

}  // namespace

struct lsmb_stream {
    lsmb_ctx* c = nullptr;
    uint32_t num_bits = 0, k = 0;
    uint64_t nw = 0;
    DevBuf words;  // the filter being built (device)
    struct Slot {
        uint8_t* data = nullptr;  // pinned key bytes
        uint64_t* offs = nullptr; // pinned offsets, offs[0] = 0
        uint64_t data_cap = 0, keys_cap = 0;
        uint64_t bytes = 0, nkeys = 0;
        DevBuf ddata, doffs;
        hipEvent_t copied = nullptr, built = nullptr;
        bool inflight = false;    // an upload / build of this slot was issued
    } slot[2];
    int cur = 0;
    uint64_t chunk = 0;           // key bytes per submitted chunk
    uint64_t total = 0;           // keys added since open / reset
    bool on_device = false;       // a chunk was submitted (the words live on the device)
    int failed = 0;               // sticky error code of an add
    PinnedPool retired;           // outgrown pinned staging (hipHostFree waits for the device)
};

namespace {

// Staging memory: pinned (DMA-able) for a device stream, plain heap for a
// host-only one (ctx == NULL).
void* host_alloc(bool pinned, uint64_t bytes) {
    void* p = nullptr;
    if (pinned) return hipHostMalloc(&p, bytes, 0) == hipSuccess ? p : nullptr;
    return malloc(bytes);
}
// Outgrown staging: pinned blocks are retired until close (a free would wait
// for every stream of the device), heap blocks freed.
void host_retire(lsmb_stream* st, bool pinned, void* p) {
    if (!p) return;
    if (pinned)
        st->retired.retire(p);
    else
        free(p);
}

int slot_reserve(lsmb_stream* st, lsmb_stream::Slot& s, bool pinned, uint64_t want_bytes, uint64_t want_keys) {
    if (want_bytes > s.data_cap) {
        uint64_t cap = std::max<uint64_t>(kStreamMinBytes, s.data_cap * 2);
        while (cap < want_bytes) cap *= 2;
        uint8_t* p = (uint8_t*)host_alloc(pinned, cap);
        if (!p) return fail(LSMB_ENOMEM, "stream: key staging (%llu B)", (unsigned long long)cap);
        if (s.bytes) memcpy(p, s.data, s.bytes);
        host_retire(st, pinned, s.data);
        s.data = p;
        s.data_cap = cap;
    }
    if (want_keys + 1 > s.keys_cap) {
        uint64_t cap = std::max<uint64_t>(kStreamMinBytes / 8, s.keys_cap * 2);
        while (cap < want_keys + 1) cap *= 2;
        uint64_t* p = (uint64_t*)host_alloc(pinned, cap * 8);
        if (!p) return fail(LSMB_ENOMEM, "stream: offsets staging (%llu B)", (unsigned long long)(cap * 8));
        if (s.offs)
            memcpy(p, s.offs, (s.nkeys + 1) * 8);
        else
            p[0] = 0;
        host_retire(st, pinned, s.offs);
        s.offs = p;
        s.keys_cap = cap;
    }
    return LSMB_OK;
}

// Uploads and builds the current slot (asynchronously), then switches slots.
int submit(lsmb_stream* st) {
    lsmb_stream::Slot& s = st->slot[st->cur];
    if (s.nkeys == 0) return LSMB_OK;
    lsmb_ctx* c = st->c;
    DevGuard g(c->dev);
    if (!st->on_device) {  // BloomFilter::new: zeroed words, then the first chunk
        HIP_TRY(st->words.ensure(std::max<uint64_t>(st->nw, 2) * 8));
        HIP_TRY(hipMemsetAsync(st->words.p, 0, st->nw * 8, c->st));
        st->on_device = true;
    }
    // The slot's device buffers were last read by its previous build.
    if (s.inflight) HIP_TRY(hipStreamWaitEvent(c->cst, s.built, 0));
    HIP_TRY(s.ddata.ensure(std::max<uint64_t>(s.bytes, 1) + 16));
    HIP_TRY(s.doffs.ensure((s.nkeys + 1) * 8));
    if (s.bytes) HIP_TRY(hipMemcpyAsync(s.ddata.p, s.data, s.bytes, hipMemcpyHostToDevice, c->cst));
    HIP_TRY(hipMemcpyAsync(s.doffs.p, s.offs, (s.nkeys + 1) * 8, hipMemcpyHostToDevice, c->cst));
    HIP_TRY(hipEventRecord(s.copied, c->cst));
    HIP_TRY(hipStreamWaitEvent(c->st, s.copied, 0));
    KeyBatch kb{(const uint8_t*)s.ddata.p, (const uint64_t*)s.doffs.p, 0, s.nkeys};
    if (int rc = build_dev(c, kb, st->num_bits, st->k, (uint32_t*)st->words.p, c->st)) return rc;
    HIP_TRY(hipEventRecord(s.built, c->st));
    s.inflight = true;
    // switch: the other slot's pinned buffers may be refilled once its upload
    // has left them
    st->cur ^= 1;
    lsmb_stream::Slot& o = st->slot[st->cur];
    if (o.inflight) HIP_TRY(hipEventSynchronize(o.copied));
    o.bytes = 0;
    o.nkeys = 0;
    if (o.offs) o.offs[0] = 0;
    return LSMB_OK;
}

int stream_add(lsmb_stream* st, const uint8_t* key, uint64_t len) {
    lsmb_stream::Slot* s = &st->slot[st->cur];
    if (st->c && s->nkeys && (s->bytes + len > st->chunk || s->nkeys + 1 > (st->chunk >> 3))) {
        if (int rc = submit(st)) return rc;
        s = &st->slot[st->cur];
    }
    if (s->bytes + len > s->data_cap || s->nkeys + 2 > s->keys_cap)
        if (int rc = slot_reserve(st, *s, st->c != nullptr, s->bytes + len, s->nkeys + 1)) return rc;
    if (len) memcpy(s->data + s->bytes, key, len);
    s->bytes += len;
    s->offs[++s->nkeys] = s->bytes;
    st->total++;
    return LSMB_OK;
}

void stream_rewind(lsmb_stream* st) {
    for (auto& s : st->slot) {
        s.bytes = 0;
        s.nkeys = 0;
        if (s.offs) s.offs[0] = 0;
    }
    st->cur = 0;
    st->total = 0;
    st->on_device = false;
    st->failed = 0;
}

// Finishes the filter into `out` (host, any alignment): the device words, or
// the host loop when the run never left the host.
int stream_finish(lsmb_stream* st, uint8_t* out) {
    if (st->failed) return fail(st->failed, "stream: an earlier add failed");
    lsmb_stream::Slot& s = st->slot[st->cur];
    if (!st->on_device && st->total <= host_max_keys()) {
        std::vector<uint64_t> w(st->nw, 0);
        host_insert_batch(s.data ? s.data : (const uint8_t*)"", s.offs, 0, s.nkeys, st->num_bits, st->k, w.data());
        if (st->nw) memcpy(out, w.data(), st->nw * 8);
        stream_rewind(st);
        return LSMB_OK;
    }
    if (!st->c) {
        stream_rewind(st);
        return fail(LSMB_EINVAL, "stream without a ctx: more than %llu keys need the GPU (lsmb_host_max_keys)",
                    (unsigned long long)host_max_keys());
    }
    if (int rc = submit(st)) return rc;
    lsmb_ctx* c = st->c;
    DevGuard g(c->dev);
    if (!st->on_device) {  // (no keys at all but a device-sized threshold of 0)
        memset(out, 0, st->nw * 8);
        stream_rewind(st);
        return LSMB_OK;
    }
    HIP_TRY(hipMemcpyAsync(out, st->words.p, st->nw * 8, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    stream_rewind(st);
    return LSMB_OK;
}

}  // namespace

extern "C" {

int lsmb_stream_open(lsmb_ctx* c, uint32_t num_bits, uint32_t num_hashes, lsmb_stream** out) {
    if (!out) return fail(LSMB_EINVAL, "null stream pointer");
    *out = nullptr;
    if (int rc = check_filter(num_bits, num_hashes)) return rc;
    lsmb_stream* st = new lsmb_stream;
    st->c = c;
    st->num_bits = num_bits;
    st->k = num_hashes;
    st->nw = nwords64(num_bits);
    st->chunk = stream_chunk_bytes();
    if (c) {
        DevGuard g(c->dev);
        for (auto& s : st->slot)
            if (hipEventCreateWithFlags(&s.copied, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&s.built, hipEventDisableTiming) != hipSuccess) {
                lsmb_stream_close(st);
                return fail(LSMB_EHIP, "stream: event creation failed");
            }
    }
    for (auto& s : st->slot)
        if (int rc = slot_reserve(st, s, c != nullptr, kStreamMinBytes, kStreamMinBytes / 16)) {
            lsmb_stream_close(st);
            return rc;
        }
    *out = st;
    return LSMB_OK;
}

int lsmb_stream_reset(lsmb_stream* st, uint32_t num_bits, uint32_t num_hashes) {
    if (!st) return fail(LSMB_EINVAL, "null stream");
    if (int rc = check_filter(num_bits, num_hashes)) return rc;
    if (st->c) {
        DevGuard g(st->c->dev);
        HIP_TRY(hipStreamSynchronize(st->c->st));  // the previous filter's kernels are done with the buffers
    }
    stream_rewind(st);
    st->num_bits = num_bits;
    st->k = num_hashes;
    st->nw = nwords64(num_bits);
    return LSMB_OK;
}

int lsmb_stream_add(lsmb_stream* st, const uint8_t* key, uint64_t len) {
    if (!st) return fail(LSMB_EINVAL, "null stream");
    if (len && !key) return fail(LSMB_EINVAL, "null key");
    if (st->failed) return fail(st->failed, "stream: an earlier add failed");
    const int rc = stream_add(st, key, len);
    if (rc) st->failed = rc;
    return rc;
}

int lsmb_stream_add_batch(lsmb_stream* st, const uint8_t* data, const uint64_t* offsets, uint64_t n) {
    if (!st) return fail(LSMB_EINVAL, "null stream");
    if (n && !offsets) return fail(LSMB_EINVAL, "null offsets");
    for (uint64_t i = 0; i < n; i++)
        if (offsets[i + 1] < offsets[i]) return fail(LSMB_EINVAL, "offsets not non-decreasing at %llu", (unsigned long long)i);
    for (uint64_t i = 0; i < n; i++) {
        if (int rc = lsmb_stream_add(st, data + offsets[i], offsets[i + 1] - offsets[i])) return rc;
    }
    return LSMB_OK;
}

uint64_t lsmb_stream_count(const lsmb_stream* st) { return st ? st->total : 0; }

int lsmb_stream_finish_block(lsmb_stream* st, uint8_t* block, uint64_t block_len) {
    if (!st || !block) return fail(LSMB_EINVAL, "null argument");
    const uint64_t size = 12 + 8 * st->nw;
    if (block_len < size) return fail(LSMB_EINVAL, "block buffer %llu B < serialized size %llu B",
                                      (unsigned long long)block_len, (unsigned long long)size);
    // header of BloomFilter::serialize (src/bloom/mod.rs:102-115)
    const uint32_t hdr[3] = {st->k, st->num_bits, (uint32_t)st->nw};
    for (int i = 0; i < 3; i++)
        for (int b = 0; b < 4; b++) block[4 * i + b] = (uint8_t)(hdr[i] >> (8 * b));
    return stream_finish(st, block + 12);
}

int lsmb_stream_finish_words(lsmb_stream* st, uint64_t* words) {
    if (!st || (!words && st->nw)) return fail(LSMB_EINVAL, "null argument");
    return stream_finish(st, (uint8_t*)words);
}

void lsmb_stream_close(lsmb_stream* st) {
    if (!st) return;
    const bool pinned = st->c != nullptr;
    if (pinned) {
        DevGuard g(st->c->dev);
        hipStreamSynchronize(st->c->st);
        hipStreamSynchronize(st->c->cst);
        for (auto& s : st->slot) {
            s.ddata.release();
            s.doffs.release();
            if (s.copied) hipEventDestroy(s.copied);
            if (s.built) hipEventDestroy(s.built);
        }
        st->words.release();
    }
    for (auto& s : st->slot) {
        host_retire(st, pinned, s.data);
        host_retire(st, pinned, s.offs);
    }
    st->retired.release();
    delete st;
}

}  // extern "C"
