/* oracle_mt_tsan.c — the oracle's multithreaded builds (bench.py's CPU
 * baseline "all host cores" leg and the full-size fixture generator) under
 * ThreadSanitizer: 8 threads set bits of one shared filter with atomic
 * fetch_or; the result must equal the 1-thread build, and TSan must report no
 * race.  Built and run by tools/sanitize.sh (test infrastructure). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void oracle_gen_key16(uint64_t seed, uint64_t first, uint64_t n, uint8_t* out);
void oracle_bloom_build_fixed(const uint8_t* keys, uint32_t key_len, uint64_t n, uint32_t num_bits, uint32_t k,
                              uint64_t* words);
int oracle_bloom_build_fixed_mt(const uint8_t* keys, uint32_t key_len, uint64_t n, uint32_t num_bits, uint32_t k,
                                uint64_t* words, int threads);
void oracle_bloom_build_var(const uint8_t* data, const uint64_t* offsets, uint64_t n, uint32_t num_bits, uint32_t k,
                            uint64_t* words);
int oracle_bloom_build_var_mt(const uint8_t* data, const uint64_t* offsets, uint64_t n, uint32_t num_bits,
                              uint32_t k, uint64_t* words, int threads);

int main(void) {
    const uint64_t n = 200000;
    const uint32_t nb = 1917011, nw = (nb + 63) / 64;
    uint8_t* keys = malloc(16 * n);
    uint64_t* a = calloc(nw, 8);
    uint64_t* b = calloc(nw, 8);
    oracle_gen_key16(0x5EED0001, 0, n, keys);
    oracle_bloom_build_fixed(keys, 16, n, nb, 7, a);
    int rc = oracle_bloom_build_fixed_mt(keys, 16, n, nb, 7, b, 8);
    int fail = rc != 0 || memcmp(a, b, 8ull * nw) != 0;
    /* var-len: keys of 0..60 bytes cut from the key stream */
    uint64_t* off = malloc(8 * (n + 1));
    off[0] = 0;
    for (uint64_t i = 0; i < n; i++) off[i + 1] = off[i] + (i * 7919 % 61) % (16 * n / n);
    memset(a, 0, 8ull * nw);
    memset(b, 0, 8ull * nw);
    oracle_bloom_build_var(keys, off, n, nb, 7, a);
    rc = oracle_bloom_build_var_mt(keys, off, n, nb, 7, b, 8);
    fail |= rc != 0 || memcmp(a, b, 8ull * nw) != 0;
    printf("oracle_mt_tsan: %s\n", fail ? "FAILED" : "ok");
    free(keys);
    free(a);
    free(b);
    free(off);
    return fail;
}
