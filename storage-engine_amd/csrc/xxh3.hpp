// xxh3.hpp — XXH3-128 (seed 0, default secret) for CDNA4 lanes and the host.
//
// The reference hashes every key with `xxhash_rust::xxh3::xxh3_128(key)`
// (src/bloom/mod.rs:182; crate xxhash-rust 0.8.15, Cargo.lock:694-697) and
// splits the u128 into h1 = low64, h2 = high64 (src/bloom/mod.rs:184-186).
// This header is the product's own implementation of the published XXH3
// algorithm, shaped for one-key-per-lane GPU execution:
//   * the 192-byte default secret is held as 24 little-endian u64 words, so a
//     secret read at a compile-time offset folds to an immediate;
//   * 64x64->128 products are four v_mad_u64_u32 on the device;
//   * key bytes are read with 8-byte unaligned loads (gfx950 global memory
//     accepts unaligned dword access), never byte-by-byte except for <4 B keys;
//   * `xxh3_16` is the fixed-16-byte fast path fed straight from a 16-byte
//     coalesced load (BASELINE configs C1/C2/C3/C5).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define LSMB_HD __host__ __device__ __forceinline__

namespace lsmb {

struct H128 {
    uint64_t lo, hi;
};

namespace xx {

constexpr uint32_t P32_1 = 0x9E3779B1U, P32_2 = 0x85EBCA77U, P32_3 = 0xC2B2AE3DU;
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ULL, P64_2 = 0xC2B2AE3D27D4EB4FULL,
                   P64_3 = 0x165667B19E3779F9ULL, P64_4 = 0x85EBCA77C2B2AE63ULL,
                   P64_5 = 0x27D4EB2F165667C5ULL;
constexpr uint64_t MX1 = 0x165667919E3779F9ULL, MX2 = 0x9FB21C651E98DF25ULL;

// Default secret as 24 LE u64 words (plus one zero word so an unaligned read
// of the last word can always touch w[i+1]).
LSMB_HD constexpr uint64_t secret_word(int i) {
    constexpr uint64_t W[25] = {
        0xbe4ba423396cfeb8ULL, 0x1cad21f72c81017cULL, 0xdb979083e96dd4deULL, 0x1f67b3b7a4a44072ULL,
        0x78e5c0cc4ee679cbULL, 0x2172ffcc7dd05a82ULL, 0x8e2443f7744608b8ULL, 0x4c263a81e69035e0ULL,
        0xcb00c391bb52283cULL, 0xa32e531b8b65d088ULL, 0x4ef90da297486471ULL, 0xd8acdea946ef1938ULL,
        0x3f349ce33f76faa8ULL, 0x1d4f0bc7c7bbdcf9ULL, 0x3159b4cd4be0518aULL, 0x647378d9c97e9fc8ULL,
        0xc3ebd33483acc5eaULL, 0xeb6313faffa081c5ULL, 0x49daf0b751dd0d17ULL, 0x9e68d429265516d3ULL,
        0xfca1477d58be162bULL, 0xce31d07ad1b8f88fULL, 0x280416958f3acb45ULL, 0x7e404bbbcafbd7afULL,
        0ULL};
    return W[i];
}

// LE u64 of the secret at byte offset `off` (folds when `off` is a constant).
LSMB_HD constexpr uint64_t sec64(int off) {
    return (off & 7) == 0 ? secret_word(off >> 3)
                          : (secret_word(off >> 3) >> (8 * (off & 7))) |
                                (secret_word((off >> 3) + 1) << (64 - 8 * (off & 7)));
}
LSMB_HD constexpr uint32_t sec32(int off) { return (uint32_t)sec64(off); }

LSMB_HD uint64_t ld64(const uint8_t* p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}
LSMB_HD uint32_t ld32(const uint8_t* p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}

// 64x64 -> 128.  On the device: four v_mad_u64_u32 (32x32+64 -> 64), the
// minimum; `a*b` plus `__umul64hi` would issue about twice as many multiplies.
LSMB_HD H128 mul128(uint64_t a, uint64_t b) {
#ifdef __HIP_DEVICE_COMPILE__
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
    const uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t p00 = (uint64_t)a0 * b0;
    const uint64_t t = (uint64_t)a0 * b1 + (p00 >> 32);
    const uint64_t u = (uint64_t)a1 * b0 + (uint32_t)t;
    return H128{(u << 32) | (uint32_t)p00, (uint64_t)a1 * b1 + (t >> 32) + (u >> 32)};
#else
    unsigned __int128 r = (unsigned __int128)a * b;
    return H128{(uint64_t)r, (uint64_t)(r >> 64)};
#endif
}
// High 64 bits of a 64x64 product.
LSMB_HD uint64_t mulhi64(uint64_t a, uint64_t b) { return mul128(a, b).hi; }
LSMB_HD uint64_t fold(uint64_t a, uint64_t b) {
    H128 r = mul128(a, b);
    return r.lo ^ r.hi;
}
LSMB_HD uint64_t aval3(uint64_t h) {
    h ^= h >> 37;
    h *= MX1;
    return h ^ (h >> 32);
}
LSMB_HD uint64_t aval64(uint64_t h) {
    h ^= h >> 33;
    h *= P64_2;
    h ^= h >> 29;
    h *= P64_3;
    return h ^ (h >> 32);
}
LSMB_HD uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
LSMB_HD uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }
LSMB_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// len in [9, 16]: lo = first 8 bytes, hi = last 8 bytes (overlapping when len < 16).
LSMB_HD H128 len9to16(uint64_t lo, uint64_t hi, uint64_t len) {
    constexpr uint64_t flipl = sec64(32) ^ sec64(40);
    constexpr uint64_t fliph = sec64(48) ^ sec64(56);
    H128 m = mul128(lo ^ hi ^ flipl, P64_1);
    m.lo += (len - 1) << 54;
    hi ^= fliph;
    m.hi += hi + (uint64_t)(uint32_t)hi * (uint64_t)(P32_2 - 1);
    m.lo ^= bswap64(m.hi);
    H128 h = mul128(m.lo, P64_2);
    h.hi += m.hi * P64_2;
    return H128{aval3(h.lo), aval3(h.hi)};
}

LSMB_HD H128 len0() {
    constexpr uint64_t a = sec64(64) ^ sec64(72), b = sec64(80) ^ sec64(88);
    return H128{aval64(a), aval64(b)};
}

// Key bytes are read through a Reader (r.ld64(o) / r.ld32(o) / r.u8(o): LE
// loads at byte offset o of the key): PtrReader for memory the lane addresses
// directly, or a kernel's LDS window (k_hash_var) — one implementation of
// every length class for both.
struct PtrReader {
    const uint8_t* p;
    LSMB_HD uint64_t ld64(uint64_t o) const { return xx::ld64(p + o); }
    LSMB_HD uint32_t ld32(uint64_t o) const { return xx::ld32(p + o); }
    LSMB_HD uint32_t u8(uint64_t o) const { return p[o]; }
};

template <class R>
LSMB_HD H128 len1to3(const R& r, uint32_t len) {
    uint32_t c1 = r.u8(0), c2 = r.u8(len >> 1), c3 = r.u8(len - 1);
    uint32_t cl = (c1 << 16) | (c2 << 24) | c3 | (len << 8);
    uint32_t ch = rotl32(bswap32(cl), 13);
    constexpr uint64_t fl = (uint64_t)(sec32(0) ^ sec32(4));
    constexpr uint64_t fh = (uint64_t)(sec32(8) ^ sec32(12));
    return H128{aval64((uint64_t)cl ^ fl), aval64((uint64_t)ch ^ fh)};
}

template <class R>
LSMB_HD H128 len4to8(const R& r, uint32_t len) {
    uint64_t v = (uint64_t)r.ld32(0) | ((uint64_t)r.ld32(len - 4) << 32);
    constexpr uint64_t flip = sec64(16) ^ sec64(24);
    H128 m = mul128(v ^ flip, P64_1 + ((uint64_t)len << 2));
    m.hi += m.lo << 1;
    m.lo ^= m.hi >> 3;
    m.lo ^= m.lo >> 35;
    m.lo *= MX2;
    m.lo ^= m.lo >> 28;
    m.hi = aval3(m.hi);
    return m;
}

template <class R>
LSMB_HD void mix32(H128& acc, const R& r, uint64_t a, uint64_t b, int so) {
    uint64_t a0 = r.ld64(a), a1 = r.ld64(a + 8), b0 = r.ld64(b), b1 = r.ld64(b + 8);
    acc.lo += fold(a0 ^ sec64(so), a1 ^ sec64(so + 8));
    acc.lo ^= b0 + b1;
    acc.hi += fold(b0 ^ sec64(so + 16), b1 ^ sec64(so + 24));
    acc.hi ^= a0 + a1;
}

LSMB_HD H128 mid_finish(H128 acc, uint64_t len) {
    uint64_t lo = acc.lo + acc.hi;
    uint64_t hi = acc.lo * P64_1 + acc.hi * P64_4 + len * P64_2;
    return H128{aval3(lo), 0 - aval3(hi)};
}

template <class R>
LSMB_HD H128 len17to128(const R& r, uint32_t len) {
    H128 acc{(uint64_t)len * P64_1, 0};
    if (len > 32) {
        if (len > 64) {
            if (len > 96) mix32(acc, r, 48, len - 64, 96);
            mix32(acc, r, 32, len - 48, 64);
        }
        mix32(acc, r, 16, len - 32, 32);
    }
    mix32(acc, r, 0, len - 16, 0);
    return mid_finish(acc, len);
}

template <class R>
LSMB_HD H128 len129to240(const R& r, uint32_t len) {
    H128 acc{(uint64_t)len * P64_1, 0};
#pragma unroll
    for (int i = 0; i < 4; i++) mix32(acc, r, 32 * i, 32 * i + 16, 32 * i);
    acc.lo = aval3(acc.lo);
    acc.hi = aval3(acc.hi);
    const uint32_t rounds = len >> 5;  // 4..7
    // unrolled over the three possible extra rounds: the secret offsets are
    // compile-time constants (immediates), not per-round loads
#pragma unroll
    for (uint32_t i = 4; i < 7; i++)
        if (i < rounds) mix32(acc, r, 32 * i, 32 * i + 16, 3 + 32 * (int)(i - 4));
    mix32(acc, r, len - 16, len - 32, 136 - 17 - 16);
    return mid_finish(acc, len);
}

template <class R>
LSMB_HD void stripe(uint64_t acc[8], const R& r, uint64_t o, int so) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t v = r.ld64(o + 8 * i);
        uint64_t k = v ^ sec64(so + 8 * i);
        acc[i ^ 1] += v;
        acc[i] += (uint64_t)(uint32_t)k * (k >> 32);
    }
}

LSMB_HD uint64_t merge(const uint64_t acc[8], int so, uint64_t start) {
    uint64_t r = start;
#pragma unroll
    for (int i = 0; i < 4; i++)
        r += fold(acc[2 * i] ^ sec64(so + 16 * i), acc[2 * i + 1] ^ sec64(so + 16 * i + 8));
    return aval3(r);
}

// len > 240: 1 KiB blocks of 16 stripes + scramble, then the tail stripes.
template <class R>
LSMB_HD H128 hash_long(const R& r, uint64_t len) {
    uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    const uint64_t nblocks = (len - 1) >> 10;
    for (uint64_t b = 0; b < nblocks; b++) {
        for (int s = 0; s < 16; s++) stripe(acc, r, (b << 10) + 64 * s, 8 * s);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            uint64_t a = acc[i];
            a ^= a >> 47;
            a ^= sec64(128 + 8 * i);
            acc[i] = a * P32_1;
        }
    }
    const uint64_t last = nblocks << 10;
    const int nstripes = (int)(((len - 1) - (nblocks << 10)) >> 6);
    for (int s = 0; s < nstripes; s++) stripe(acc, r, last + 64 * s, 8 * s);
    stripe(acc, r, len - 64, 192 - 64 - 7);
    return H128{merge(acc, 11, len * P64_1), merge(acc, 192 - 64 - 11, ~(len * P64_2))};
}

}  // namespace xx

// XXH3-128 of an arbitrary key read through `r` (see xx::PtrReader).
template <class R>
LSMB_HD H128 xxh3_128_r(const R& r, uint64_t len) {
    if (len <= 16) {
        if (len > 8) return xx::len9to16(r.ld64(0), r.ld64(len - 8), len);
        if (len >= 4) return xx::len4to8(r, (uint32_t)len);
        if (len) return xx::len1to3(r, (uint32_t)len);
        return xx::len0();
    }
    if (len <= 128) return xx::len17to128(r, (uint32_t)len);
    if (len <= 240) return xx::len129to240(r, (uint32_t)len);
    return xx::hash_long(r, len);
}

// XXH3-128 of an arbitrary key.
LSMB_HD H128 xxh3_128(const uint8_t* p, uint64_t len) { return xxh3_128_r(xx::PtrReader{p}, len); }

// Fixed 16-byte key given as its two LE u64 halves.
LSMB_HD H128 xxh3_16(uint64_t lo, uint64_t hi) { return xx::len9to16(lo, hi, 16); }

}  // namespace lsmb
