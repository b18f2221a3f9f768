// flush_e2e.cpp — flush-shaped end-to-end driver for the streaming ingestion
// API (lsmb_stream), in C++ the way a C/Rust store links the library.
//
// The reference's flush (src/db/mod.rs:377-383) walks the frozen memtable and
// adds every key to the SSTable builder, whose bloom builder inserts it at once
// (src/sstable/builder.rs:93 -> src/bloom/builder.rs:21-23 -> insert,
// src/bloom/mod.rs:70-78); finish() then serializes the filter
// (builder.rs:177-182).  Here the memtable is an ordered std::map (a
// pointer-chasing ordered structure like the reference's arena skiplist) of N
// random 16-byte keys, and three timings are taken over the same walk:
//   walk       the walk alone (touch every key);
//   host       walk + lsmb_insert per key + lsmb_serialize: the reference's
//              algorithm on one host thread (the library's host loop);
//   stream     walk + lsmb_stream_add per key + lsmb_stream_finish_block:
//              chunks upload and build on the GPU while the walk goes on.
// Prints one JSON line; "bit_exact" compares the two blocks.
// Usage: flush_e2e [N = 4000000]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <map>
#include <string>
#include <vector>

#include "../include/lsmbloom.h"

static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CHECK(x)                                                                   \
    do {                                                                           \
        int rc_ = (x);                                                             \
        if (rc_ < 0) {                                                             \
            fprintf(stderr, "%s failed: %d %s\n", #x, rc_, lsmb_last_error());     \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 4000000;
    // the frozen memtable: key16(0x5EED0001, i) -> empty value (a tombstone is
    // an ordinary key for the filter, src/memtable/mod.rs:46-48)
    std::map<std::string, std::string> mem;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t w[2] = {splitmix64(0x5EED0001ull + 2 * i), splitmix64(0x5EED0001ull + 2 * i + 1)};
        mem.emplace(std::string((const char*)w, 16), std::string());
    }
    uint32_t nb = 0, k = 0;
    CHECK(lsmb_params(n, 0.01, &nb, &k));
    const uint64_t size = lsmb_serialized_size(nb);

    // walk alone
    double t0 = now();
    uint64_t sink = 0;
    for (const auto& kv : mem) sink += (uint8_t)kv.first[0];
    const double t_walk = now() - t0;

    // reference algorithm on the host: insert per key, then serialize
    std::vector<uint64_t> words(lsmb_num_words(nb), 0);
    std::vector<uint8_t> blk_host(size);
    t0 = now();
    for (const auto& kv : mem)
        CHECK(lsmb_insert(words.data(), nb, k, (const uint8_t*)kv.first.data(), kv.first.size()));
    CHECK(lsmb_serialize(words.data(), nb, k, blk_host.data(), size));
    const double t_host = now() - t0;

    // streaming ingestion on the GPU
    lsmb_ctx* ctx = nullptr;
    CHECK(lsmb_open(&ctx, 0));
    lsmb_stream* st = nullptr;
    CHECK(lsmb_stream_open(ctx, nb, k, &st));
    std::vector<uint8_t> blk(size);
    double t_stream = 1e30;
    for (int rep = 0; rep < 3; rep++) {  // first rep grows the pinned staging
        t0 = now();
        for (const auto& kv : mem) CHECK(lsmb_stream_add(st, (const uint8_t*)kv.first.data(), kv.first.size()));
        CHECK(lsmb_stream_finish_block(st, blk.data(), size));
        const double t = now() - t0;
        if (rep && t < t_stream) t_stream = t;
    }
    const bool exact = memcmp(blk.data(), blk_host.data(), size) == 0;
    lsmb_stream_close(st);
    lsmb_close(ctx);
    printf("{\"keys\": %llu, \"num_bits\": %u, \"k\": %u, \"walk_ms\": %.3f, \"host_insert_1t_ms\": %.3f, "
           "\"stream_ms\": %.3f, \"stream_Mkeys_s\": %.1f, \"host_Mkeys_s\": %.1f, \"bit_exact\": %s, \"sink\": %llu}\n",
           (unsigned long long)n, nb, k, t_walk * 1e3, t_host * 1e3, t_stream * 1e3, n / t_stream / 1e6,
           n / t_host / 1e6, exact ? "true" : "false", (unsigned long long)(sink & 1));
    return exact ? 0 : 2;
}
