// bloom_math.hpp — exact Bloom position arithmetic for CDNA4 lanes and the host.
//
// The reference computes, for i in 0..k (src/bloom/mod.rs:192-197):
//     pos_i = (h1 +wrap i *wrap h2) % (num_bits as u64)
// i.e. 64-bit wrapping arithmetic FIRST, then a 64-bit modulo by a u32.  CDNA4
// has no integer divider, so a literal `%` is a long software sequence per
// position.  We evaluate the same integers with:
//
//   * one exact reduction per key for h1 and for h2 (`Mod32::reduce`):
//       y = hi32(x) * (2^32 mod d) + lo32(x)        (one v_mad_u64_u32; y < d*2^32)
//       q = (u32)(f64(y) * f64(1/d))                (|q - floor(y/d)| <= 1, see below)
//       r = y - q*d, then one fix-up each way.
//     f64(y) is exact when y < 2^53 and otherwise off by at most
//     y*2^-53 < d*2^-21, so y/d is known to within 2^-21 + 2^-20 and the
//     truncated quotient is off by at most one;
//   * a strength-reduced walk over i: x_i = x_{i-1} + h2 (mod 2^64) with carry
//     c_i, hence x_i mod d = (r_{i-1} + (h2 mod d) - c_i * (2^64 mod d)) mod d.
//     For d <= 2^31 every intermediate fits 32 bits (`Walk32`), and each
//     "mod d" fix-up is a subtract and an unsigned min.
//
// The host compiles the very same code (fma() matches v_fma_f64), and
// tests/test_capi_host.py checks it against the oracle's literal `%` over
// random and edge-case moduli in [1, 2^32).
#pragma once

#include <math.h>

#include "xxh3.hpp"

namespace lsmb {

// f64 of y < 2^64 as hi32(y)·2^32 + lo32(y), one rounding (the fma).  On the
// device the high word is converted with an explicit v_cvt_f64_u32: left to
// the compiler, (double)(uint32_t)(y >> 32) is widened to a 64-bit uitofp
// whose lowering adds a +0.0 (one more f64 add per reduction).
LSMB_HD double f64_of_u64(uint64_t y) {
#ifdef __HIP_DEVICE_COMPILE__
    double hd;
    asm("v_cvt_f64_u32 %0, %1" : "=v"(hd) : "v"((uint32_t)(y >> 32)));
#else
    const double hd = (double)(uint32_t)(y >> 32);
#endif
    return fma(hd, 4294967296.0, (double)(uint32_t)y);
}

struct Mod32 {
    uint32_t d;     // divisor (num_bits), 1 <= d < 2^32
    uint32_t t32;   // 2^32 mod d
    uint32_t t64;   // 2^64 mod d
    uint32_t dt;    // d - t64 (in (0, d])
    double inv;     // 1/d rounded, then 4 ulps toward 0: strictly below 1/d

    static Mod32 make(uint32_t d32) {
        Mod32 r;
        r.d = d32;
        r.t32 = (uint32_t)((1ull << 32) % d32);
        r.t64 = (uint32_t)((uint64_t)(((unsigned __int128)1 << 64) % d32));
        r.dt = d32 - r.t64;
        r.inv = 1.0 / (double)d32;
        for (int i = 0; i < 4; i++) r.inv = nextafter(r.inv, 0.0);
        return r;
    }

    // With inv biased low, q = trunc(f64(y) * inv) never exceeds floor(y/d)
    // and is at most one below it: f64(y) and the product each round by at
    // most 2^-53 relative, and inv sits between 2^-51 and 2^-49 below 1/d,
    // so qd < y/d and y/d - qd < 2^32 * 2^-48.  So y - q*d lies in [0, 2d).
    LSMB_HD uint32_t reduce(uint64_t x) const {
        const uint64_t y = (uint64_t)(uint32_t)(x >> 32) * t32 + (uint32_t)x;
        const uint32_t q = (uint32_t)(f64_of_u64(y) * inv);  // < y/d < 2^32
        uint64_t r = y - (uint64_t)q * d;
        if (r >= d) r -= d;
        return (uint32_t)r;
    }
    // The same for d <= 2^31 (Walk32's domain): r < 2d <= 2^32 fits a u32, so
    // the remainder is one 32-bit multiply-subtract and one conditional
    // subtract (an unsigned min): 10 VALU instructions against 19.
    LSMB_HD uint32_t reduce31(uint64_t x) const {
        const uint64_t y = (uint64_t)(uint32_t)(x >> 32) * t32 + (uint32_t)x;
        const uint32_t q = (uint32_t)(f64_of_u64(y) * inv);
        const uint32_t r = (uint32_t)y - q * d;  // y - q d mod 2^32, exact: in [0, 2d)
        const uint32_t s = r - d;
        return s < r ? s : r;
    }
};

// The same reduction for small moduli, d < 2^14 (SST-sized filters: the
// store's new(1000, 0.01) is 9 568 bits).  x's four 16-bit limbs times
// t_j = 2^(16 j) mod d sum to y < 2^16 + 3·2^16·d < 2^32, so y/d < 2^18.
// inv is 1/d rounded to f32 and stepped 4 ulps toward 0 (3 to 9 · 2^-24
// below 1/d), so q = trunc(f32(y)·inv) is below y/d (the two roundings add at
// most 2·2^-24) and above y/d - 2^18·11·2^-24: q is floor(y/d) or one less,
// and one conditional subtract finishes it.  24-bit multiplies and f32 only:
// no 64-bit products, no f64.
struct Mod14 {
    uint32_t d, t16, t32, t48;  // 2^(16 j) mod d
    uint32_t t64, dt;           // 2^64 mod d, d - t64 (the walk's carry step)
    float inv;                  // 1.0f / d

    static Mod14 make(uint32_t d32) {
        Mod14 r;
        r.d = d32;
        r.t16 = (uint32_t)((1ull << 16) % d32);
        r.t32 = (uint32_t)((1ull << 32) % d32);
        r.t48 = (uint32_t)((1ull << 48) % d32);
        r.t64 = (uint32_t)((uint64_t)(((unsigned __int128)1 << 64) % d32));
        r.dt = d32 - r.t64;
        r.inv = 1.0f / (float)d32;
        for (int i = 0; i < 4; i++) r.inv = nextafterf(r.inv, 0.0f);
        return r;
    }
    static LSMB_HD bool fits(uint32_t d) { return d >= 1 && d < (1u << 14); }

    // a·b for a, b < 2^24 (exact when the product fits 32 bits): one
    // full-rate v_mul_u32_u24 on the device instead of a quarter-rate mul_lo
    static LSMB_HD uint32_t mul24(uint32_t a, uint32_t b) {
#ifdef __HIP_DEVICE_COMPILE__
        return __umul24(a, b);
#else
        return a * b;
#endif
    }
    LSMB_HD uint32_t reduce(uint64_t x) const {
        const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
        const uint32_t y = (lo & 0xFFFFu) + mul24(lo >> 16, t16) + mul24(hi & 0xFFFFu, t32) + mul24(hi >> 16, t48);
        const uint32_t q = (uint32_t)((float)y * inv);
        const uint32_t r = y - mul24(q, d);  // in [0, 2d) (q < 2^18, d < 2^14)
        const uint32_t b = r - d;
        return b < r ? b : r;
    }
    LSMB_HD uint32_t reduce31(uint64_t x) const { return reduce(x); }
};

// k positions of one key, i = 0, 1, ..., for d <= 2^31 (all sums fit 32 bits).
// Position i+1 = (pos_i + h2 - c*2^64) mod d, where c = 1 when the wrapping
// u64 sum h1 + i*h2 (src/bloom/mod.rs:194) carries out; so the two possible
// increments, h2 mod d and (h2 - 2^64) mod d, are reduced once per key and
// each step is a 64-bit add with carry, a select, an add and one conditional
// subtract.
template <class M>
struct Walk32T {
    using Mod = M;
    uint64_t x, h2;
    uint32_t r, s0, s1, d;

    LSMB_HD Walk32T(const M& md, uint64_t h1, uint64_t h2_) : x(h1), h2(h2_), d(md.d) {
        r = md.reduce31(h1);
        s0 = md.reduce31(h2_);
        const uint32_t t = s0 + md.dt;  // < 2d <= 2^32
        s1 = t - md.d < t ? t - md.d : t;
    }
    LSMB_HD Walk32T(const M& md, const H128& h) : Walk32T(md, h.lo, h.hi) {}
    LSMB_HD uint32_t pos() const { return r; }
    LSMB_HD void next(const M&) {
        uint64_t nx;
        const bool carry = __builtin_add_overflow(x, h2, &nx);
        x = nx;
        const uint32_t u = r + (carry ? s1 : s0);  // < 2d
        r = u - d < u ? u - d : u;
    }
};

using Walk32 = Walk32T<Mod32>;
using Walk14 = Walk32T<Mod14>;  // d < 2^14 (Mod14's reduction)

// The same walk for any d < 2^32.  r + s < 2d can exceed 2^32 when d > 2^31:
// the 32-bit add's carry-out stands for the 33rd bit, so one conditional
// subtraction still finishes the step (no 64-bit sums: C5's 2^32-1-bit
// filter walks as cheaply as Walk32).
LSMB_HD uint32_t add_mod_wide(uint32_t a, uint32_t b, uint32_t d) {  // (a + b) mod d, a, b < d
    uint32_t u;
    const bool c = __builtin_add_overflow(a, b, &u);
    return (c || u >= d) ? u - d : u;
}

struct Walk64 {
    using Mod = Mod32;
    uint64_t x, h2;
    uint32_t r, s0, s1, d;

    LSMB_HD Walk64(const Mod32& md, uint64_t h1, uint64_t h2_) : x(h1), h2(h2_), d(md.d) {
        r = md.reduce(h1);
        s0 = md.reduce(h2_);
        s1 = md.dt == md.d ? s0 : add_mod_wide(s0, md.dt, md.d);  // (s0 + 2^64 - t64) mod d
    }
    LSMB_HD Walk64(const Mod32& md, const H128& h) : Walk64(md, h.lo, h.hi) {}
    LSMB_HD uint32_t pos() const { return r; }
    LSMB_HD void next(const Mod32&) {
        uint64_t nx;
        const bool carry = __builtin_add_overflow(x, h2, &nx);
        x = nx;
        r = add_mod_wide(r, carry ? s1 : s0, d);
    }
};

// The 64-bit-safe walk, used where d may exceed 2^31.
using PosWalk = Walk64;

// num_bits = 2^32 - 1: BloomFilter::new saturates `as u32` there
// (src/bloom/mod.rs:49), so every filter sized for more than ~4.5e8 keys at
// fpr 0.01 has it (C5's new(1e9, 0.01)).  2^32 = 1 (mod d): x mod d folds
// the two halves (an add with end-around carry), and 2^64 mod d = 1, so no
// reduction needs a quotient estimate.
LSMB_HD uint32_t fold_m32(uint64_t x) {  // x mod (2^32 - 1)
    uint32_t u;
    const bool c = __builtin_add_overflow((uint32_t)x, (uint32_t)(x >> 32), &u);
    u += c ? 1u : 0u;  // (<= 2^32 - 1 after a carry)
    return u == 0xFFFFFFFFu ? 0u : u;
}

struct WalkM {  // d = 2^32 - 1 exactly; positions identical to Walk64's
    using Mod = Mod32;
    uint64_t x, h2;
    uint32_t r, s0, s1;

    LSMB_HD WalkM(const Mod32&, uint64_t h1, uint64_t h2_) : x(h1), h2(h2_) {
        r = fold_m32(h1);
        s0 = fold_m32(h2_);
        s1 = s0 ? s0 - 1 : 0xFFFFFFFEu;  // (h2 - 2^64) mod d = s0 - 1
    }
    LSMB_HD WalkM(const Mod32& md, const H128& h) : WalkM(md, h.lo, h.hi) {}
    LSMB_HD uint32_t pos() const { return r; }
    LSMB_HD void next(const Mod32&) {
        uint64_t nx;
        const bool carry = __builtin_add_overflow(x, h2, &nx);
        x = nx;
        r = add_mod_wide(r, carry ? s1 : s0, 0xFFFFFFFFu);
    }
};
constexpr uint32_t kMersenneBits = 0xFFFFFFFFu;  // the num_bits WalkM serves

// A key's walk reduced to 12 bytes, for builds that hash in a separate kernel
// (variable-length and odd-length keys): r = h1 mod d, s = h2 mod d and the
// carries c_i of the wrapping sums h1 + i*h2 (bit i-1 = carry out of
// x_{i-1} + h2, i = 1 .. 31).  The walks below replay Walk32 / Walk64 from it
// exactly (tests: every C4 build against the oracle), without the two
// reductions and the 64-bit sums in the pass that consumes it.
struct WalkRec {
    uint32_t r, s, c;

    static LSMB_HD WalkRec make(const Mod32& md, const H128& h, uint32_t k) {
        WalkRec q;
        if (md.d <= 0x80000000u) {  // (uniform) the 32-bit remainder path, as Walk32 takes
            q.r = md.reduce31(h.lo);
            q.s = md.reduce31(h.hi);
        } else if (md.d == 0xFFFFFFFFu) {  // the saturated filter: folds (WalkM)
            q.r = fold_m32(h.lo);
            q.s = fold_m32(h.hi);
        } else {
            q.r = md.reduce(h.lo);
            q.s = md.reduce(h.hi);
        }
        const uint32_t steps = k < 2 ? 0u : (k - 1 < 31 ? k - 1 : 31u);
#ifdef __HIP_DEVICE_COMPILE__
        // The carries through one add-with-carry chain: x += h2 leaves the
        // carry in vcc, and acc = acc + acc + vcc shifts it in (3 VALU a step
        // against ~5 for a 64-bit add, a compare and a select-or); the first
        // carry lands in the top bit, so the bits are reversed at the end.
        uint32_t lo = (uint32_t)h.lo, hi = (uint32_t)(h.lo >> 32), acc = 0;
        const uint32_t dlo = (uint32_t)h.hi, dhi = (uint32_t)(h.hi >> 32);
        for (uint32_t i = 0; i < steps; i++)
            asm volatile("v_add_co_u32 %0, vcc, %0, %3\n\tv_addc_co_u32 %1, vcc, %1, %4, vcc\n\t"
                         "v_addc_co_u32 %2, vcc, %2, %2, vcc"
                         : "+v"(lo), "+v"(hi), "+v"(acc)
                         : "v"(dlo), "v"(dhi)
                         : "vcc");
        q.c = steps ? __builtin_bitreverse32(acc) >> (32 - steps) : 0u;
#else
        q.c = 0;
        uint64_t x = h.lo;
        for (uint32_t i = 0; i < steps; i++) {
            uint64_t nx;
            if (__builtin_add_overflow(x, h.hi, &nx)) q.c |= 1u << i;
            x = nx;
        }
#endif
        return q;
    }
};

struct RecWalk32 {  // d <= 2^31, as Walk32
    using Mod = Mod32;
    uint32_t r, s0, s1, c, d;
    LSMB_HD RecWalk32(const Mod32& md, const WalkRec& q) : r(q.r), s0(q.s), c(q.c), d(md.d) {
        const uint32_t t = s0 + md.dt;
        s1 = t - md.d < t ? t - md.d : t;
    }
    LSMB_HD uint32_t pos() const { return r; }
    LSMB_HD void next(const Mod32&) {
        const uint32_t u = r + ((c & 1u) ? s1 : s0);
        c >>= 1;
        r = u - d < u ? u - d : u;
    }
};

struct RecWalk64 {  // any d < 2^32, as Walk64
    using Mod = Mod32;
    uint32_t r, s0, s1, c, d;
    LSMB_HD RecWalk64(const Mod32& md, const WalkRec& q) : r(q.r), s0(q.s), c(q.c), d(md.d) {
        s1 = md.dt == md.d ? s0 : add_mod_wide(s0, md.dt, md.d);
    }
    LSMB_HD uint32_t pos() const { return r; }
    LSMB_HD void next(const Mod32&) {
        r = add_mod_wide(r, (c & 1u) ? s1 : s0, d);
        c >>= 1;
    }
};

LSMB_HD bool fits_walk32(uint32_t d) { return d <= 0x80000000u; }

// BloomFilter::new sizing (src/bloom/mod.rs:38-67), host only.  Returns false
// where the reference panics (expected_items == 0, fpr outside (0, 1)).
bool bloom_params(uint64_t expected_items, double fpr, uint32_t* num_bits, uint32_t* num_hashes);

}  // namespace lsmb
