// reduce_test.cpp — the exact reductions of bloom_math.hpp against a literal
// 64-bit %, at the inputs that stress their quotient estimates: x = q*d + r
// with r in {0, 1, d-1} (y/d an integer or just below one, where a quotient
// estimate one too high would go negative), x near 0 and near 2^64, and random
// x.  Mod32::reduce (any d < 2^32), Mod32::reduce31 (d <= 2^31, the 32-bit
// remainder path Walk32 takes) and Mod14::reduce (d < 2^14).  Their biased-low
// reciprocals (make) must keep every quotient estimate at floor(y/d) or one
// below; and WalkM's positions for d = 2^32 - 1.  Host build of the device
// header (tests/test_capi_host.py).
#include <stdio.h>

#include <random>

#include "../../storage-engine_amd/csrc/bloom_math.hpp"

using namespace lsmb;

static long bad = 0, checked = 0;

template <class F>
static void check(uint32_t d, uint64_t x, F&& f, const char* what) {
    const uint32_t want = (uint32_t)(x % d), got = f(x);
    checked++;
    if (got != want && bad++ < 20) printf("FAIL %s d=%u x=%llu got=%u want=%u\n", what, d, (unsigned long long)x, got, want);
}

static void moduli(uint32_t d, std::mt19937_64& rng, int nrand) {
    const Mod32 m = Mod32::make(d);
    const bool w31 = d <= 0x80000000u;
    const bool small = Mod14::fits(d);
    Mod14 m14{};
    if (small) m14 = Mod14::make(d);
    auto all = [&](uint64_t x) {
        check(d, x, [&](uint64_t v) { return m.reduce(v); }, "reduce");
        if (w31) check(d, x, [&](uint64_t v) { return m.reduce31(v); }, "reduce31");
        if (small) check(d, x, [&](uint64_t v) { return m14.reduce(v); }, "mod14");
    };
    const uint64_t qmax = ~0ull / d;
    const uint64_t qs[] = {0, 1, 2, qmax, qmax - 1, qmax / 2, qmax >> 32, (qmax >> 32) + 1, 1ull << 32};
    for (uint64_t q : qs) {
        if (q > qmax) continue;
        for (uint64_t r : {(uint64_t)0, (uint64_t)1, (uint64_t)d - 1}) {
            if (r >= d) continue;
            const unsigned __int128 x = (unsigned __int128)q * d + r;
            if (x <= ~0ull) all((uint64_t)x);
        }
    }
    for (unsigned long long x : {0ull, 1ull, ~0ull, ~0ull - 1, 1ull << 32, (1ull << 32) - 1, 1ull << 63, (1ull << 63) - 1})
        all(x);
    for (int t = 0; t < nrand; t++) {
        uint64_t x = rng();
        if (t & 1) x -= x % d;          // a multiple of d
        else if (t % 3 == 0) x = x - x % d + d - 1;  // just below one (may wrap: still a valid input)
        all(x);
    }
}

int main() {
    std::mt19937_64 rng(11);
    const uint32_t fixed_d[] = {1, 2, 3, 5, 7, 64, 957, 9568, 9569, 16383, 65535, 65536, 65537, 956716,
                                956715292, 1000000000, 0x3FFFFFFFu, 0x40000000u, 0x40000001u, 0x7FFFFFFFu,
                                0x80000000u, 0x80000001u, 3000000000u, 0xFFFFFFFEu, 0xFFFFFFFFu};
    for (uint32_t d : fixed_d) moduli(d, rng, 20000);
    for (int t = 0; t < 3000; t++) {
        uint32_t d = (uint32_t)(rng() >> (32 + rng() % 32));
        if (d == 0) d = 1;
        moduli(d, rng, 200);
    }
    for (uint32_t d = 1; d < (1u << 14); d++) moduli(d, rng, 40);  // every Mod14 modulus
    // WalkM (d = 2^32 - 1): seven positions per (h1, h2) against a literal
    // (h1 + i h2 mod 2^64) % d, random and edge hashes (0, d, 2^64 - 1, ...)
    {
        const uint32_t d = 0xFFFFFFFFu;
        const Mod32 md = Mod32::make(d);
        const uint64_t edge[] = {0, 1, d, (uint64_t)d + 1, 2ull * d, ~0ull, ~0ull - 1, 1ull << 63, (uint64_t)d << 32,
                                 ((uint64_t)d << 32) + d};
        auto walk = [&](uint64_t h1, uint64_t h2) {
            WalkM w(md, h1, h2);
            for (uint64_t i = 0; i < 7; i++) {
                const uint64_t want = (h1 + i * h2) % d;
                checked++;
                if (w.pos() != want && bad++ < 20)
                    printf("FAIL walkM h1=%llu h2=%llu i=%llu got=%u want=%llu\n", (unsigned long long)h1,
                           (unsigned long long)h2, (unsigned long long)i, w.pos(), (unsigned long long)want);
                w.next(md);
            }
        };
        for (uint64_t a : edge)
            for (uint64_t b : edge) walk(a, b);
        for (int t = 0; t < 2000000; t++) walk(rng(), rng());
    }
    printf("reduce: %ld checked, %ld bad\n", checked, bad);
    return bad ? 1 : 0;
}
