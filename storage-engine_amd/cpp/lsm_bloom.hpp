// lsm_bloom.hpp — C++ host mirror of the reference's `crate::bloom` surface
// (G1DO/Storage-Engine src/bloom/mod.rs, src/bloom/builder.rs) over the C ABI
// in include/lsmbloom.h.  Header-only; link against liblsmbloom.
//
// Rust (reference)                                C++ (this header)
//   BloomFilter::new(n, fpr)        mod.rs:38-67    BloomFilter(n, fpr)
//   bf.insert(key)                  mod.rs:70-78    bf.insert(key)
//   bf.may_contain(key)             mod.rs:82-94    bf.may_contain(key)
//   bf.serialize()                  mod.rs:102-115  bf.serialize()
//   BloomFilter::deserialize(data)  mod.rs:123-168  BloomFilter::deserialize(data)   (throws Corruption)
//   bf.num_hashes() / num_bits()    mod.rs:171-178  same
//   BloomFilterBuilder::new(n, fpr) builder.rs:14   BloomFilterBuilder(n, fpr)
//   b.add_key(key)                  builder.rs:21   b.add_key(key)    (buffers the key)
//   b.build()                       builder.rs:26   b.build()         (one GPU batch)
// Reference panics (assert!, % by zero) become std::invalid_argument;
// Err(Error::Corruption(msg)) (src/error.rs:12) becomes lsm::bloom::Corruption.
// The batched build/probe run on the GPU: without a gfx950 device they throw
// (no CPU fallback), except builds of at most lsmb_host_max_keys() keys, which
// run the library's own host loop (same bits, no device round trip).
#pragma once

#include <stdint.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

#include "../../include/lsmbloom.h"

namespace lsm::bloom {

struct Corruption : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct GpuError : std::runtime_error {
    int code;
    GpuError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline int check(int rc) {
    if (rc >= 0) return rc;
    const std::string msg = lsmb_last_error();
    if (rc == LSMB_ECORRUPT) throw Corruption(msg);
    if (rc == LSMB_EINVAL) throw std::invalid_argument(msg);
    throw GpuError(rc, msg);
}

// One GPU (lsmb_ctx).  Movable, not copyable.
class Context {
   public:
    explicit Context(int device = -1) { check(lsmb_open(&c_, device)); }
    ~Context() { lsmb_close(c_); }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    Context(Context&& o) noexcept : c_(o.c_) { o.c_ = nullptr; }
    lsmb_ctx* get() const { return c_; }

    // Default context of the calling thread, opened on first use.  A context
    // is used by one thread at a time (lsmbloom.h), and the store builds from
    // more than one thread at once (flush + the background compaction thread,
    // src/compaction/scheduler.rs:37), so each thread gets its own — the same
    // choice as the Rust shim's thread_local CTX.
    static Context& shared() {
        thread_local Context ctx(-1);
        return ctx;
    }

   private:
    lsmb_ctx* c_ = nullptr;
};

class BloomFilter {
   public:
    BloomFilter(size_t expected_items, double false_positive_rate) {
        check(lsmb_params(expected_items, false_positive_rate, &num_bits_, &num_hashes_));
        bits_.assign(lsmb_num_words(num_bits_), 0);
    }

    void insert(std::string_view key) { insert(key.data(), key.size()); }
    void insert(const void* key, size_t len) {
        check(lsmb_insert(bits_.data(), num_bits_, num_hashes_, static_cast<const uint8_t*>(key), len));
    }
    bool may_contain(std::string_view key) const { return may_contain(key.data(), key.size()); }
    bool may_contain(const void* key, size_t len) const {
        return check(lsmb_may_contain(bits_.data(), num_bits_, num_hashes_, static_cast<const uint8_t*>(key),
                                      len)) == 1;
    }

    std::vector<uint8_t> serialize() const {
        std::vector<uint8_t> out(lsmb_serialized_size(num_bits_));
        check(lsmb_serialize(bits_.data(), num_bits_, num_hashes_, out.data(), out.size()));
        return out;
    }
    static BloomFilter deserialize(const std::vector<uint8_t>& data) { return deserialize(data.data(), data.size()); }
    static BloomFilter deserialize(const uint8_t* data, size_t len) {
        uint32_t k = 0, nb = 0, nw = 0;
        check(lsmb_deserialize_header(data, len, &k, &nb, &nw));
        BloomFilter f;
        f.num_hashes_ = k;
        f.num_bits_ = nb;
        f.bits_.assign(nw, 0);
        check(lsmb_deserialize(data, len, f.bits_.data(), nw));
        return f;
    }

    uint32_t num_hashes() const { return num_hashes_; }
    uint32_t num_bits() const { return num_bits_; }
    const std::vector<uint64_t>& words() const { return bits_; }
    std::vector<uint64_t>& words() { return bits_; }

    // Additive batched probe (the reference has no multi-get): for each key,
    // a bitmask row over `filters` (bit f = may_contain(filters[f], key)).
    static std::vector<uint8_t> may_contain_batch(const std::vector<const BloomFilter*>& filters,
                                                  const std::vector<std::string>& keys,
                                                  Context& ctx = Context::shared()) {
        const uint32_t nf = static_cast<uint32_t>(filters.size());
        std::vector<const uint64_t*> w(nf);
        std::vector<uint32_t> nb(nf), kk(nf);
        for (uint32_t f = 0; f < nf; f++) {
            w[f] = filters[f]->bits_.data();
            nb[f] = filters[f]->num_bits_;
            kk[f] = filters[f]->num_hashes_;
        }
        std::vector<uint64_t> offs(keys.size() + 1, 0);
        std::string data;
        for (size_t i = 0; i < keys.size(); i++) {
            data += keys[i];
            offs[i + 1] = data.size();
        }
        std::vector<uint8_t> out(keys.size() * ((nf + 7) / 8));
        check(lsmb_probe(ctx.get(), w.data(), nb.data(), kk.data(), nf,
                         reinterpret_cast<const uint8_t*>(data.data()), offs.data(), 0, keys.size(), out.data()));
        return out;
    }

   private:
    BloomFilter() = default;
    friend class BloomFilterBuilder;
    std::vector<uint64_t> bits_;
    uint32_t num_hashes_ = 0;
    uint32_t num_bits_ = 0;
};

// Buffers the run's keys in a packed arena and builds the whole filter in one
// GPU batch at build() (the reference inserts on the fly, builder.rs:5-7, 21-23);
// the bits are identical.
class BloomFilterBuilder {
   public:
    BloomFilterBuilder(size_t estimated_keys, double false_positive_rate, Context* ctx = nullptr)
        : filter_(estimated_keys, false_positive_rate), ctx_(ctx) {
        offsets_.push_back(0);
    }
    void add_key(std::string_view key) { add_key(key.data(), key.size()); }
    void add_key(const void* key, size_t len) {
        const uint8_t* p = static_cast<const uint8_t*>(key);
        data_.insert(data_.end(), p, p + len);
        offsets_.push_back(data_.size());
    }
    BloomFilter build() {
        if (offsets_.size() > 1) {
            check(lsmb_build_var(ctx_for(offsets_.size() - 1), data_.data(), offsets_.data(), offsets_.size() - 1,
                                 filter_.num_bits_, filter_.num_hashes_, filter_.bits_.data()));
        }
        return std::move(filter_);
    }
    // build().serialize() in one call (lsmb_build_block): the bloom block
    // SSTableBuilder::finish writes (src/sstable/builder.rs:177-179), with the
    // words copied device -> block directly.
    std::vector<uint8_t> build_serialized() {
        std::vector<uint8_t> block(lsmb_serialized_size(filter_.num_bits_));
        check(lsmb_build_block(ctx_for(offsets_.size() - 1), data_.empty() ? nullptr : data_.data(), offsets_.data(),
                               0, offsets_.size() - 1, filter_.num_bits_, filter_.num_hashes_, block.data(),
                               block.size()));
        return block;
    }

   private:
    // Builds of at most lsmb_host_max_keys() keys (an SST flush at the
    // reference's default 1 000-key sizing) run the library's host loop and
    // need no GPU; bigger ones take the GPU context (throws without one).
    lsmb_ctx* ctx_for(size_t n) {
        if (n <= lsmb_host_max_keys()) return nullptr;
        return (ctx_ ? *ctx_ : Context::shared()).get();
    }
    BloomFilter filter_;
    Context* ctx_;
    std::vector<uint8_t> data_;
    std::vector<uint64_t> offsets_;
};

// Device-resident SSTable filters with key ranges (lsmb_fset): probe(keys)[i]
// bit s = (min_s <= key i <= max_s) && may_contain(filter s, key i), the
// checks SSTable::get makes before reading the index (reader.rs:192-199).
class FilterSet {
   public:
    explicit FilterSet(Context& ctx = Context::shared()) { check(lsmb_fset_open(ctx.get(), &fs_)); }
    ~FilterSet() { lsmb_fset_close(fs_); }
    FilterSet(const FilterSet&) = delete;
    FilterSet& operator=(const FilterSet&) = delete;

    // From a serialized bloom block (throws Corruption like deserialize); returns the slot.
    int add(const std::vector<uint8_t>& block, std::string_view min_key, std::string_view max_key) {
        return check(lsmb_fset_add(fs_, block.data(), block.size(), u8(min_key), min_key.size(), u8(max_key),
                                   max_key.size()));
    }
    int add(const BloomFilter& f, std::string_view min_key, std::string_view max_key) {
        return check(lsmb_fset_add_words(fs_, f.words().data(), f.num_bits(), f.num_hashes(), u8(min_key),
                                         min_key.size(), u8(max_key), max_key.size()));
    }
    void remove(int slot) { check(lsmb_fset_remove(fs_, slot)); }
    uint64_t live_mask() const { return lsmb_fset_live_mask(fs_); }

    std::vector<uint64_t> probe(const std::vector<std::string>& keys) {
        std::vector<uint64_t> offs(keys.size() + 1, 0);
        std::string data;
        for (size_t i = 0; i < keys.size(); i++) {
            data += keys[i];
            offs[i + 1] = data.size();
        }
        std::vector<uint64_t> out(keys.size());
        check(lsmb_fset_probe(fs_, u8(data), offs.data(), 0, keys.size(), out.data()));
        return out;
    }

   private:
    static const uint8_t* u8(std::string_view s) { return reinterpret_cast<const uint8_t*>(s.data()); }
    lsmb_fset* fs_ = nullptr;
};

}  // namespace lsm::bloom
