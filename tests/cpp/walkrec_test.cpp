// walkrec_test.cpp — the 12-B walk records of partitioned var-len / odd-length
// builds (WalkRec, RecWalk32, RecWalk64 in bloom_math.hpp) replay the walks
// from (h1, h2) (Walk32, Walk64) position for position, and both equal the
// reference's literal (h1 +wrap i*h2) % num_bits (src/bloom/mod.rs:192-197).
// Host build of the device header (tests/test_capi_host.py compiles and runs it).
#include <stdio.h>

#include <random>

#include "../../storage-engine_amd/csrc/bloom_math.hpp"

using namespace lsmb;

int main() {
    std::mt19937_64 rng(7);
    long checked = 0, bad = 0;
    const uint32_t fixed_d[] = {1, 2, 3, 64, 957, 9568, 956716, 956715292, 1000000000, 0x7FFFFFFFu, 0x80000000u,
                                0x80000001u, 3000000000u, 0xFFFFFFFEu, 0xFFFFFFFFu};
    for (int t = 0; t < 200000; t++) {
        const uint32_t d = t < 15 * 64 ? fixed_d[t % 15] : (uint32_t)(rng() | 1) >> (rng() % 32);
        if (d == 0) continue;
        const Mod32 md = Mod32::make(d);
        uint64_t h1 = rng(), h2 = rng();
        if (t % 7 == 0) h2 = ~0ull - (rng() % 1000);  // carries at every step
        if (t % 11 == 0) h1 = ~0ull - (rng() % 1000);
        const uint32_t k = 1 + (uint32_t)(rng() % 32);
        const WalkRec q = WalkRec::make(md, H128{h1, h2}, k);
        Walk64 w64(md, h1, h2);
        RecWalk64 r64(md, q);
        const bool small = fits_walk32(d);
        Walk32 w32(md, h1, h2);
        RecWalk32 r32(md, q);
        for (uint32_t i = 0; i < k; i++) {
            const uint32_t ref = (uint32_t)((h1 + (uint64_t)i * h2) % d);
            if (w64.pos() != ref || r64.pos() != ref) bad++;
            if (small && (w32.pos() != ref || r32.pos() != ref)) bad++;
            checked++;
            w64.next(md), r64.next(md);
            if (small) w32.next(md), r32.next(md);
        }
    }
    printf("walkrec: %ld positions, %ld mismatches\n", checked, bad);
    return bad ? 1 : 0;
}
