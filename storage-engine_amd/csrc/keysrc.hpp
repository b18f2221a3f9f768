// keysrc.hpp — how the kernels read one key and hash it (device side, internal).
#pragma once

#include "bloom_math.hpp"

namespace lsmb {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// 16-byte streaming load that bypasses cache allocation (read-once data).
__device__ __forceinline__ uint4 ld_stream16(const uint4* p) {
    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

namespace ks {

// 16-byte keys on a 16-byte-aligned base: one dwordx4 load per key, streamed
// past the caches (each key is read exactly once).
struct Fixed16 {
    static constexpr bool kPrehash = false;  // hashed inline by pass A
    using Seed = H128;  // what hash_pre returns: the walk's start
    const uint4* k;
    __device__ __forceinline__ H128 hash(uint64_t i) const {
        uint4 v = ld_stream16(k + i);
        return xxh3_16(((uint64_t)v.y << 32) | v.x, ((uint64_t)v.w << 32) | v.z);
    }
    __device__ __forceinline__ const uint8_t* bytes(uint64_t i) const { return reinterpret_cast<const uint8_t*>(k + i); }
    __device__ __forceinline__ uint64_t key_len(uint64_t) const { return 16; }
    // Split load / hash, so a kernel can issue key i's load iterations ahead.
    using Pre = uint4;
    __device__ __forceinline__ Pre fetch(uint64_t i, bool ok) const {
        return ok ? ld_stream16(k + i) : make_uint4(0, 0, 0, 0);
    }
    __device__ __forceinline__ H128 hash_pre(const Pre& v, uint64_t) const {
        return xxh3_16(((uint64_t)v.y << 32) | v.x, ((uint64_t)v.w << 32) | v.z);
    }
};

// Any fixed key length, any alignment.
struct FixedN {
    static constexpr bool kPrehash = true;  // partitioned builds hash in k_hash first
    using Seed = H128;
    const uint8_t* d;
    uint32_t len;
    __device__ __forceinline__ H128 hash(uint64_t i) const { return xxh3_128(d + i * len, len); }
    __device__ __forceinline__ const uint8_t* bytes(uint64_t i) const { return d + i * len; }
    __device__ __forceinline__ uint64_t key_len(uint64_t) const { return len; }
    struct Pre {};
    __device__ __forceinline__ Pre fetch(uint64_t, bool) const { return Pre{}; }
    __device__ __forceinline__ H128 hash_pre(const Pre&, uint64_t i) const { return hash(i); }
};

// Packed variable-length keys: key i = d[o[i] .. o[i+1]).
struct VarLen {
    static constexpr bool kPrehash = true;  // partitioned builds hash in k_hash first
    using Seed = H128;
    const uint8_t* d;
    const uint64_t* o;
    __device__ __forceinline__ H128 hash(uint64_t i) const {
        uint64_t a = o[i], b = o[i + 1];
        return xxh3_128(d + a, b - a);
    }
    __device__ __forceinline__ const uint8_t* bytes(uint64_t i) const { return d + o[i]; }
    __device__ __forceinline__ uint64_t key_len(uint64_t i) const { return o[i + 1] - o[i]; }
    // The offset pair is fetched ahead; the key bytes are read by the hash.
    struct Pre {
        uint64_t a, b;
    };
    __device__ __forceinline__ Pre fetch(uint64_t i, bool ok) const { return ok ? Pre{o[i], o[i + 1]} : Pre{0, 0}; }
    __device__ __forceinline__ H128 hash_pre(const Pre& p, uint64_t) const { return xxh3_128(d + p.a, p.b - p.a); }
};

// Keys already hashed by k_hash: (h1, h2) of key i as one 16-B record, read
// with one coalesced dwordx4 like Fixed16.  Pass A over variable-length keys
// runs on these: its phase-synchronous loop (one key per lane per phase,
// barriers between phases, one workgroup per CU) would otherwise expose the
// latency of every key-byte load and the length-class divergence of XXH3.
struct Hashed {
    static constexpr bool kPrehash = false;
    using Seed = H128;
    const uint4* h;
    __device__ __forceinline__ H128 hash(uint64_t i) const { return hash_pre(ld_stream16(h + i), i); }
    using Pre = uint4;
    __device__ __forceinline__ Pre fetch(uint64_t i, bool ok) const {
        return ok ? ld_stream16(h + i) : make_uint4(0, 0, 0, 0);
    }
    __device__ __forceinline__ H128 hash_pre(const Pre& v, uint64_t) const {
        return H128{((uint64_t)v.y << 32) | v.x, ((uint64_t)v.w << 32) | v.z};
    }
};

// 12-B walk records (WalkRec) written by k_hash / k_hash_var for a
// partitioned build: pass A reads three coalesced dwords per key and walks
// without reductions (RecWalk32 / RecWalk64).
struct Recs {
    static constexpr bool kPrehash = false;
    using Seed = WalkRec;
    const uint32_t* q;  // 3 u32 per key
    using Pre = WalkRec;
    __device__ __forceinline__ Pre fetch(uint64_t i, bool ok) const {
        if (!ok) return WalkRec{0, 0, 0};
        const uint32_t* p = q + 3 * i;
        return WalkRec{__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1),
                       __builtin_nontemporal_load(p + 2)};
    }
    __device__ __forceinline__ WalkRec hash_pre(const Pre& v, uint64_t) const { return v; }
};

}  // namespace ks

// Register pins (an empty asm consuming the value) for a walk seed.
__device__ __forceinline__ void pin_seed(const H128& h) {
    asm volatile("" ::"v"((uint32_t)h.lo), "v"((uint32_t)(h.lo >> 32)), "v"((uint32_t)h.hi), "v"((uint32_t)(h.hi >> 32)));
}
__device__ __forceinline__ void pin_seed(const WalkRec& q) { asm volatile("" ::"v"(q.r), "v"(q.s), "v"(q.c)); }
}  // namespace lsmb
