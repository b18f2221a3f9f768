/*
 * bloom_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's Bloom-filter hot path
 * (G1DO/Storage-Engine `src/bloom/mod.rs`) and of the third-party hash it calls
 * (`xxhash-rust` 0.8.15, feature `xxh3`, `Cargo.toml:15-16`, `Cargo.lock:694-697`;
 * called at `src/bloom/mod.rs:182`).  XXH3 output is frozen since xxHash 0.8.0,
 * so the published XXH3-128 algorithm (seed 0, default 192-byte secret) is
 * restated here from the specification.
 *
 * This file is the CHECKER.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product (storage-engine_amd/) never links,
 * loads or calls anything under oracle/.
 *
 * Pinning: tests/test_oracle_golden.py checks every function here against
 * the JSON fixtures in tests/golden, which tests/golden/gen_golden.py produced from the
 * Python `xxhash` module (bundling libxxhash 0.8.2), cross-checked against the
 * system libxxhash 0.8.1, plus the reference tests' deterministic assertions
 * (tests/bloom_tests.rs, tests/bloom_serialize_tests.rs).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

/* ------------------------------------------------------------------------- */
/* XXH3-128 (published algorithm; restated)                                  */
/* ------------------------------------------------------------------------- */

#define P32_1 0x9E3779B1U
#define P32_2 0x85EBCA77U
#define P32_3 0xC2B2AE3DU
#define P64_1 0x9E3779B185EBCA87ULL
#define P64_2 0xC2B2AE3D27D4EB4FULL
#define P64_3 0x165667B19E3779F9ULL
#define P64_4 0x85EBCA77C2B2AE63ULL
#define P64_5 0x27D4EB2F165667C5ULL
#define PMX1 0x165667919E3779F9ULL
#define PMX2 0x9FB21C651E98DF25ULL

/* XXH3 default secret (192 bytes), a published constant of the algorithm. */
static const uint8_t K_SECRET[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};

static uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }
static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static uint32_t bswap32(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xff00U) | ((x << 8) & 0xff0000U) | (x << 24);
}
static uint64_t bswap64(uint64_t x) {
    return ((uint64_t)bswap32((uint32_t)x) << 32) | bswap32((uint32_t)(x >> 32));
}

typedef struct { uint64_t lo, hi; } u128;

static u128 mul64x64(uint64_t a, uint64_t b) {
    unsigned __int128 r = (unsigned __int128)a * b;
    u128 o = {(uint64_t)r, (uint64_t)(r >> 64)};
    return o;
}
static uint64_t fold64(uint64_t a, uint64_t b) {
    u128 r = mul64x64(a, b);
    return r.lo ^ r.hi;
}
static uint64_t avalanche3(uint64_t h) {
    h ^= h >> 37;
    h *= PMX1;
    return h ^ (h >> 32);
}
static uint64_t avalanche64(uint64_t h) {
    h ^= h >> 33;
    h *= P64_2;
    h ^= h >> 29;
    h *= P64_3;
    return h ^ (h >> 32);
}

static u128 h_0(void) {
    u128 o;
    o.lo = avalanche64(rd64(K_SECRET + 64) ^ rd64(K_SECRET + 72));
    o.hi = avalanche64(rd64(K_SECRET + 80) ^ rd64(K_SECRET + 88));
    return o;
}

static u128 h_1to3(const uint8_t* in, size_t len) {
    uint8_t c1 = in[0], c2 = in[len >> 1], c3 = in[len - 1];
    uint32_t cl = ((uint32_t)c1 << 16) | ((uint32_t)c2 << 24) | (uint32_t)c3 | ((uint32_t)len << 8);
    uint32_t ch = rotl32(bswap32(cl), 13);
    uint64_t fl = (uint64_t)(rd32(K_SECRET) ^ rd32(K_SECRET + 4));
    uint64_t fh = (uint64_t)(rd32(K_SECRET + 8) ^ rd32(K_SECRET + 12));
    u128 o = {avalanche64((uint64_t)cl ^ fl), avalanche64((uint64_t)ch ^ fh)};
    return o;
}

static u128 h_4to8(const uint8_t* in, size_t len) {
    uint32_t lo = rd32(in), hi = rd32(in + len - 4);
    uint64_t v = (uint64_t)lo + ((uint64_t)hi << 32);
    uint64_t flip = rd64(K_SECRET + 16) ^ rd64(K_SECRET + 24);
    u128 m = mul64x64(v ^ flip, P64_1 + ((uint64_t)len << 2));
    m.hi += m.lo << 1;
    m.lo ^= m.hi >> 3;
    m.lo ^= m.lo >> 35;
    m.lo *= PMX2;
    m.lo ^= m.lo >> 28;
    m.hi = avalanche3(m.hi);
    return m;
}

static u128 h_9to16(const uint8_t* in, size_t len) {
    uint64_t fl = rd64(K_SECRET + 32) ^ rd64(K_SECRET + 40);
    uint64_t fh = rd64(K_SECRET + 48) ^ rd64(K_SECRET + 56);
    uint64_t lo = rd64(in), hi = rd64(in + len - 8);
    u128 m = mul64x64(lo ^ hi ^ fl, P64_1);
    m.lo += (uint64_t)(len - 1) << 54;
    hi ^= fh;
    m.hi += hi + (uint64_t)(uint32_t)hi * (uint64_t)(P32_2 - 1);
    m.lo ^= bswap64(m.hi);
    u128 h = mul64x64(m.lo, P64_2);
    h.hi += m.hi * P64_2;
    h.lo = avalanche3(h.lo);
    h.hi = avalanche3(h.hi);
    return h;
}

static uint64_t mix16(const uint8_t* in, const uint8_t* sec) {
    return fold64(rd64(in) ^ rd64(sec), rd64(in + 8) ^ rd64(sec + 8));
}

static void mix32(u128* acc, const uint8_t* a, const uint8_t* b, const uint8_t* sec) {
    acc->lo += mix16(a, sec);
    acc->lo ^= rd64(b) + rd64(b + 8);
    acc->hi += mix16(b, sec + 16);
    acc->hi ^= rd64(a) + rd64(a + 8);
}

static u128 finish_mid(u128 acc, size_t len) {
    u128 o;
    o.lo = acc.lo + acc.hi;
    o.hi = acc.lo * P64_1 + acc.hi * P64_4 + (uint64_t)len * P64_2;
    o.lo = avalanche3(o.lo);
    o.hi = (uint64_t)0 - avalanche3(o.hi);
    return o;
}

static u128 h_17to128(const uint8_t* in, size_t len) {
    u128 acc = {(uint64_t)len * P64_1, 0};
    if (len > 32) {
        if (len > 64) {
            if (len > 96) mix32(&acc, in + 48, in + len - 64, K_SECRET + 96);
            mix32(&acc, in + 32, in + len - 48, K_SECRET + 64);
        }
        mix32(&acc, in + 16, in + len - 32, K_SECRET + 32);
    }
    mix32(&acc, in, in + len - 16, K_SECRET);
    return finish_mid(acc, len);
}

static u128 h_129to240(const uint8_t* in, size_t len) {
    u128 acc = {(uint64_t)len * P64_1, 0};
    size_t rounds = len / 32, i;
    for (i = 0; i < 4; i++) mix32(&acc, in + 32 * i, in + 32 * i + 16, K_SECRET + 32 * i);
    acc.lo = avalanche3(acc.lo);
    acc.hi = avalanche3(acc.hi);
    for (i = 4; i < rounds; i++)
        mix32(&acc, in + 32 * i, in + 32 * i + 16, K_SECRET + 3 + 32 * (i - 4));
    /* last 32 bytes: secret at 136 - 17 - 16, seed negated (seed = 0). */
    mix32(&acc, in + len - 16, in + len - 32, K_SECRET + 136 - 17 - 16);
    return finish_mid(acc, len);
}

static void accumulate512(uint64_t acc[8], const uint8_t* in, const uint8_t* sec) {
    for (int i = 0; i < 8; i++) {
        uint64_t v = rd64(in + 8 * i);
        uint64_t k = v ^ rd64(sec + 8 * i);
        acc[i ^ 1] += v;
        acc[i] += (uint64_t)(uint32_t)k * (k >> 32);
    }
}

static void scramble(uint64_t acc[8], const uint8_t* sec) {
    for (int i = 0; i < 8; i++) {
        uint64_t a = acc[i];
        a ^= a >> 47;
        a ^= rd64(sec + 8 * i);
        acc[i] = a * P32_1;
    }
}

static uint64_t merge_accs(const uint64_t acc[8], const uint8_t* sec, uint64_t start) {
    uint64_t r = start;
    for (int i = 0; i < 4; i++)
        r += fold64(acc[2 * i] ^ rd64(sec + 16 * i), acc[2 * i + 1] ^ rd64(sec + 16 * i + 8));
    return avalanche3(r);
}

static u128 h_long(const uint8_t* in, size_t len) {
    uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    const size_t stripes_per_block = (192 - 64) / 8; /* 16 */
    const size_t block_len = 64 * stripes_per_block; /* 1024 */
    size_t nb_blocks = (len - 1) / block_len, n, s;
    for (n = 0; n < nb_blocks; n++) {
        for (s = 0; s < stripes_per_block; s++)
            accumulate512(acc, in + n * block_len + s * 64, K_SECRET + s * 8);
        scramble(acc, K_SECRET + 192 - 64);
    }
    size_t nb_stripes = ((len - 1) - block_len * nb_blocks) / 64;
    for (s = 0; s < nb_stripes; s++)
        accumulate512(acc, in + nb_blocks * block_len + s * 64, K_SECRET + s * 8);
    accumulate512(acc, in + len - 64, K_SECRET + 192 - 64 - 7);
    u128 o;
    o.lo = merge_accs(acc, K_SECRET + 11, (uint64_t)len * P64_1);
    o.hi = merge_accs(acc, K_SECRET + 192 - 64 - 11, ~((uint64_t)len * P64_2));
    return o;
}

/* xxh3_128(key) with seed 0: returns low64 in *lo, high64 in *hi. */
void oracle_xxh3_128(const uint8_t* in, size_t len, uint64_t* lo, uint64_t* hi) {
    u128 r;
    if (len == 0) r = h_0();
    else if (len <= 3) r = h_1to3(in, len);
    else if (len <= 8) r = h_4to8(in, len);
    else if (len <= 16) r = h_9to16(in, len);
    else if (len <= 128) r = h_17to128(in, len);
    else if (len <= 240) r = h_129to240(in, len);
    else r = h_long(in, len);
    *lo = r.lo;
    *hi = r.hi;
}

/* ------------------------------------------------------------------------- */
/* src/bloom/mod.rs restatement                                              */
/* ------------------------------------------------------------------------- */

/* Rust `f64 as u32` saturates: NaN -> 0, <0 -> 0, >u32::MAX -> u32::MAX. */
static uint32_t sat_u32(double x) {
    if (!(x == x) || x <= 0.0) return 0;
    if (x >= 4294967295.0) return 4294967295U;
    return (uint32_t)x;
}

/* BloomFilter::new sizing, src/bloom/mod.rs:38-67.  Returns 0, or -1 where the
 * reference panics (expected_items == 0 or fpr outside (0, 1), :39-43). */
int oracle_bloom_params(uint64_t expected_items, double fpr, uint32_t* num_bits, uint32_t* k) {
    if (expected_items == 0) return -1;
    if (!(fpr > 0.0 && fpr < 1.0)) return -1;
    double bpk = -1.44 * log2(fpr);                                   /* :46 */
    uint32_t nb = sat_u32(ceil((double)expected_items * bpk));        /* :49 */
    if (nb < 64) nb = 64;                                             /* :52 */
    uint32_t nh = sat_u32(ceil(bpk * log(2.0)));                      /* :55 */
    if (nh < 1) nh = 1;                                               /* :56 */
    *num_bits = nb;
    *k = nh;
    return 0;
}

/* get_position, src/bloom/mod.rs:192-197: (h1 +wrap i*h2) % num_bits. */
static uint32_t get_position(uint64_t h1, uint64_t h2, uint32_t i, uint32_t num_bits) {
    return (uint32_t)((h1 + (uint64_t)i * h2) % (uint64_t)num_bits);
}

/* positions of one key (hash_key :181-189 then get_position), for tests. */
void oracle_bloom_positions(const uint8_t* key, size_t len, uint32_t num_bits, uint32_t k,
                            uint32_t* out) {
    uint64_t h1, h2;
    oracle_xxh3_128(key, len, &h1, &h2);
    for (uint32_t i = 0; i < k; i++) out[i] = get_position(h1, h2, i, num_bits);
}

/* insert, src/bloom/mod.rs:70-78 with set_bit :200-204. */
void oracle_bloom_insert(uint64_t* words, uint32_t num_bits, uint32_t k, const uint8_t* key,
                         size_t len) {
    uint64_t h1, h2;
    oracle_xxh3_128(key, len, &h1, &h2);
    for (uint32_t i = 0; i < k; i++) {
        uint32_t p = get_position(h1, h2, i, num_bits);
        words[p / 64] |= (uint64_t)1 << (p % 64);
    }
}

/* may_contain, src/bloom/mod.rs:82-94 with check_bit :207-211. */
int oracle_bloom_may_contain(const uint64_t* words, uint32_t num_bits, uint32_t k,
                             const uint8_t* key, size_t len) {
    uint64_t h1, h2;
    oracle_xxh3_128(key, len, &h1, &h2);
    for (uint32_t i = 0; i < k; i++) {
        uint32_t p = get_position(h1, h2, i, num_bits);
        if (!((words[p / 64] >> (p % 64)) & 1)) return 0;
    }
    return 1;
}

/* Batch drivers: the per-key loop of SSTableBuilder::add (src/sstable/builder.rs:93). */
void oracle_bloom_build_fixed(const uint8_t* keys, uint32_t key_len, uint64_t n,
                              uint32_t num_bits, uint32_t k, uint64_t* words) {
    for (uint64_t i = 0; i < n; i++)
        oracle_bloom_insert(words, num_bits, k, keys + i * (uint64_t)key_len, key_len);
}

void oracle_bloom_build_var(const uint8_t* data, const uint64_t* offsets, uint64_t n,
                            uint32_t num_bits, uint32_t k, uint64_t* words) {
    for (uint64_t i = 0; i < n; i++)
        oracle_bloom_insert(words, num_bits, k, data + offsets[i], offsets[i + 1] - offsets[i]);
}

/* Multi-filter probe: bit f of out[i*stride + f/8] = may_contain(filter f, key i),
 * i.e. what SSTable::get's bloom check (src/sstable/reader.rs:197) answers per SST.
 * offsets == NULL -> fixed key_len keys. */
void oracle_bloom_probe(const uint64_t* const* filt_words, const uint32_t* filt_bits,
                        const uint32_t* filt_k, uint32_t nfilt, const uint8_t* data,
                        const uint64_t* offsets, uint32_t key_len, uint64_t n, uint8_t* out) {
    uint32_t stride = (nfilt + 7) / 8;
    memset(out, 0, n * stride);
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t* key = offsets ? data + offsets[i] : data + i * (uint64_t)key_len;
        size_t len = offsets ? (size_t)(offsets[i + 1] - offsets[i]) : key_len;
        for (uint32_t f = 0; f < nfilt; f++)
            if (oracle_bloom_may_contain(filt_words[f], filt_bits[f], filt_k[f], key, len))
                out[i * stride + f / 8] |= (uint8_t)(1u << (f % 8));
    }
}

/* serialize, src/bloom/mod.rs:102-115.  out must hold 12 + 8*num_u64s bytes. */
uint64_t oracle_bloom_serialize(const uint64_t* words, uint32_t num_bits, uint32_t k, uint8_t* out) {
    uint32_t nw = (uint32_t)(((uint64_t)num_bits + 63) / 64);
    uint32_t hdr[3] = {k, num_bits, nw};
    for (int j = 0; j < 3; j++)
        for (int b = 0; b < 4; b++) out[4 * j + b] = (uint8_t)(hdr[j] >> (8 * b));
    for (uint32_t w = 0; w < nw; w++)
        for (int b = 0; b < 8; b++) out[12 + 8 * (uint64_t)w + b] = (uint8_t)(words[w] >> (8 * b));
    return 12 + 8 * (uint64_t)nw;
}

/* deserialize validation, src/bloom/mod.rs:123-168.
 * Returns 0 ok, -1 too short (:126-130), -2 num_u64s mismatch (:136-143),
 * -3 length mismatch (:146-153).  On success fills header and (if words) the words. */
int oracle_bloom_deserialize(const uint8_t* data, uint64_t len, uint32_t* k, uint32_t* num_bits,
                             uint32_t* num_u64s, uint64_t* words) {
    if (len < 12) return -1;
    uint32_t nh = rd32(data), nb = rd32(data + 4), nw = rd32(data + 8);
    uint64_t expect = ((uint64_t)nb + 63) / 64;
    if ((uint64_t)nw != expect) return -2;
    if (len != 12 + 8 * (uint64_t)nw) return -3;
    *k = nh;
    *num_bits = nb;
    *num_u64s = nw;
    if (words)
        for (uint32_t w = 0; w < nw; w++) words[w] = rd64(data + 12 + 8 * (uint64_t)w);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Deterministic synthetic keys (the workload generator of BASELINE.md)      */
/* ------------------------------------------------------------------------- */

static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

/* key16(seed, i) = LE64(sm(seed+2i)) || LE64(sm(seed+2i+1)) for i in [first, first+n). */
void oracle_gen_key16(uint64_t seed, uint64_t first, uint64_t n, uint8_t* out) {
    for (uint64_t j = 0; j < n; j++) {
        uint64_t i = first + j;
        uint64_t a = splitmix64(seed + 2 * i), b = splitmix64(seed + 2 * i + 1);
        for (int t = 0; t < 8; t++) {
            out[16 * j + t] = (uint8_t)(a >> (8 * t));
            out[16 * j + 8 + t] = (uint8_t)(b >> (8 * t));
        }
    }
}

/* ------------------------------------------------------------------------- */
/* Multi-threaded CPU baseline (same bits: OR is order-independent)         */
/* ------------------------------------------------------------------------- */

typedef struct {
    const uint8_t* keys;
    const uint64_t* offsets; /* var-len keys when non-NULL */
    uint32_t key_len;
    uint64_t begin, end;
    uint32_t num_bits, k;
    uint64_t* words;
} mt_job;

static void* mt_worker(void* arg) {
    mt_job* j = (mt_job*)arg;
    for (uint64_t i = j->begin; i < j->end; i++) {
        uint64_t h1, h2;
        if (j->offsets)
            oracle_xxh3_128(j->keys + j->offsets[i], j->offsets[i + 1] - j->offsets[i], &h1, &h2);
        else
            oracle_xxh3_128(j->keys + i * (uint64_t)j->key_len, j->key_len, &h1, &h2);
        for (uint32_t t = 0; t < j->k; t++) {
            uint32_t p = get_position(h1, h2, t, j->num_bits);
            __atomic_fetch_or(&j->words[p / 64], (uint64_t)1 << (p % 64), __ATOMIC_RELAXED);
        }
    }
    return NULL;
}

static int run_mt(const uint8_t* keys, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                  uint32_t num_bits, uint32_t k, uint64_t* words, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 1024) threads = 1024;
    pthread_t tid[1024];
    mt_job jobs[1024];
    for (int t = 0; t < threads; t++) {
        jobs[t].keys = keys;
        jobs[t].offsets = offsets;
        jobs[t].key_len = key_len;
        jobs[t].begin = n * (uint64_t)t / (uint64_t)threads;
        jobs[t].end = n * (uint64_t)(t + 1) / (uint64_t)threads;
        jobs[t].num_bits = num_bits;
        jobs[t].k = k;
        jobs[t].words = words;
        if (pthread_create(&tid[t], NULL, mt_worker, &jobs[t]) != 0) return -1;
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    return 0;
}

int oracle_bloom_build_fixed_mt(const uint8_t* keys, uint32_t key_len, uint64_t n,
                                uint32_t num_bits, uint32_t k, uint64_t* words, int threads) {
    return run_mt(keys, NULL, key_len, n, num_bits, k, words, threads);
}

/* oracle_bloom_build_var on `threads` threads (same bits: OR is order-independent). */
int oracle_bloom_build_var_mt(const uint8_t* data, const uint64_t* offsets, uint64_t n,
                              uint32_t num_bits, uint32_t k, uint64_t* words, int threads) {
    return run_mt(data, offsets, 0, n, num_bits, k, words, threads);
}
