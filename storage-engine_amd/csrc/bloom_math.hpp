// bloom_math.hpp — exact Bloom position arithmetic for CDNA4 lanes and the host.
//
// The reference computes, for i in 0..k (src/bloom/mod.rs:192-197):
//     pos_i = (h1 +wrap i *wrap h2) % (num_bits as u64)
// i.e. 64-bit wrapping arithmetic FIRST, then a 64-bit modulo by a u32.  CDNA4
// has no integer divider, so a literal `%` is a long software sequence per
// position.  We evaluate the same integers with:
//
//   * one exact reduction per key for h1 and for h2 (`Mod32::reduce`): a
//     64-bit reciprocal m = floor((2^64-1)/d) gives q' = mulhi(x, m) in
//     {q-1, q}, so r = x - q'd needs at most one conditional subtract;
//   * a strength-reduced walk over i: x_i = x_{i-1} + h2 (mod 2^64) with carry
//     c_i, hence x_i mod d = (r_{i-1} + (h2 mod d) - c_i * (2^64 mod d)) mod d,
//     which costs a 64-bit add, a carry test and two conditional fix-ups.
//
// Both are exact for every d in [1, 2^32); tests/test_host_logic.py checks
// them against the oracle's literal `%` on random and edge-case inputs.
#pragma once

#include "xxh3.hpp"

namespace lsmb {

struct Mod32 {
    uint64_t d;     // divisor (num_bits), 1 <= d < 2^32
    uint64_t m;     // floor((2^64 - 1) / d)
    uint64_t t;     // 2^64 mod d

    static Mod32 make(uint32_t d32) {
        Mod32 r;
        r.d = d32;
        r.m = ~0ULL / r.d;
        r.t = (~0ULL % r.d + 1) % r.d;
        return r;
    }

    LSMB_HD uint64_t reduce(uint64_t x) const {
#ifdef __HIP_DEVICE_COMPILE__
        uint64_t q = __umul64hi(x, m);
#else
        uint64_t q = (uint64_t)(((unsigned __int128)x * m) >> 64);
#endif
        uint64_t r = x - q * d;
        return r >= d ? r - d : r;
    }
};

// Walks the k positions of one key in order i = 0, 1, ..., k-1.
struct PosWalk {
    uint64_t x;     // h1 + i*h2 (mod 2^64)
    uint64_t h2;
    uint64_t r;     // x mod d
    uint64_t s;     // h2 mod d

    LSMB_HD PosWalk(const Mod32& md, uint64_t h1, uint64_t h2_) : x(h1), h2(h2_) {
        r = md.reduce(h1);
        s = md.reduce(h2_);
    }
    LSMB_HD uint32_t pos() const { return (uint32_t)r; }
    LSMB_HD void next(const Mod32& md) {
        uint64_t nx = x + h2;
        bool carry = nx < x;
        x = nx;
        uint64_t u = r + s;
        if (u >= md.d) u -= md.d;
        if (carry) u = (u >= md.t) ? u - md.t : u + md.d - md.t;
        r = u;
    }
};

// BloomFilter::new sizing (src/bloom/mod.rs:38-67), host only.  Returns false
// where the reference panics (expected_items == 0, fpr outside (0, 1)).
bool bloom_params(uint64_t expected_items, double fpr, uint32_t* num_bits, uint32_t* num_hashes);

}  // namespace lsmb
