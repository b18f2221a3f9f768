// host_sanitize.cpp — the library's host-side code under AddressSanitizer /
// UndefinedBehaviorSanitizer and ThreadSanitizer (tools/sanitize.sh builds
// it; SURVEY.md section 5, "Race detection / sanitizers").  No GPU is needed:
// every call here takes the library's host paths.
//   * deserialize validation (src/bloom/mod.rs:123-168) on corrupt, truncated,
//     padded and random blobs, and serialize round trips;
//   * host builds (fixed / var-len, every XXH3 length class, empty keys) vs
//     single-key insert and may_contain;
//   * a host-only key stream (ctx = NULL) that grows its staging many times;
//   * CRC-32 host functions vs a bitwise reference;
//   * the same host entry points from 8 threads at once (thread-local error
//     strings, the host_max_keys threshold read / written concurrently).
// Exit status 0 = every check passed (the sanitizers abort on a finding).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lsmbloom.h"

static int g_fail = 0;
#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);     \
            g_fail++;                                                          \
        }                                                                      \
    } while (0)

static uint32_t crc_bitwise(const uint8_t* p, size_t n) {
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; i++) {
        c ^= p[i];
        for (int b = 0; b < 8; b++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1)));
    }
    return ~c;
}

static void deserialize_cases(std::mt19937_64& rng) {
    // round trips over many sizes
    for (uint32_t nb : {1u, 63u, 64u, 65u, 957u, 9568u, 100000u, 956716u}) {
        std::vector<uint64_t> w(lsmb_num_words(nb));
        for (auto& x : w) x = rng();
        std::vector<uint8_t> blk(lsmb_serialized_size(nb));
        CHECK(lsmb_serialize(w.data(), nb, 7, blk.data(), blk.size()) == LSMB_OK);
        uint32_t k = 0, b = 0, n = 0;
        CHECK(lsmb_deserialize_header(blk.data(), blk.size(), &k, &b, &n) == LSMB_OK && k == 7 && b == nb);
        std::vector<uint64_t> back(w.size() + 1);
        CHECK(lsmb_deserialize(blk.data(), blk.size(), back.data(), back.size()) == LSMB_OK);
        CHECK(memcmp(back.data(), w.data(), w.size() * 8) == 0);
        // truncated / trailing / too small a words buffer
        CHECK(lsmb_deserialize(blk.data(), blk.size() - 1, back.data(), back.size()) == LSMB_ECORRUPT);
        std::vector<uint8_t> pad(blk);
        pad.push_back(0);
        CHECK(lsmb_deserialize(pad.data(), pad.size(), back.data(), back.size()) == LSMB_ECORRUPT);
        if (w.size()) CHECK(lsmb_deserialize(blk.data(), blk.size(), back.data(), w.size() - 1) == LSMB_EINVAL);
        CHECK(lsmb_serialize(w.data(), nb, 7, blk.data(), blk.size() - 1) == LSMB_EINVAL);
    }
    // garbage: random lengths and headers, every length below the header too
    for (int t = 0; t < 20000; t++) {
        const size_t len = t < 16 ? (size_t)t : (size_t)(rng() % 4096);
        std::vector<uint8_t> g(len + 1);
        for (auto& x : g) x = (uint8_t)rng();
        if (len >= 12 && (t & 1)) {  // plausible headers, inconsistent sizes
            const uint32_t nb = (uint32_t)(rng() % 40000), nw = (uint32_t)((nb + 63) / 64 + (rng() % 3) - 1);
            memcpy(g.data() + 4, &nb, 4);
            memcpy(g.data() + 8, &nw, 4);
        }
        uint32_t k, nb, nw;
        const int rc = lsmb_deserialize_header(len ? g.data() : nullptr, len, &k, &nb, &nw);
        if (rc == LSMB_OK) {
            CHECK(len == 12 + 8 * (uint64_t)nw && nw == lsmb_num_words(nb));
            std::vector<uint64_t> w(nw + 1);
            CHECK(lsmb_deserialize(g.data(), len, w.data(), w.size()) == LSMB_OK);
        } else {
            CHECK(rc == LSMB_ECORRUPT && strlen(lsmb_last_error()) > 0);
        }
    }
}

static std::vector<std::string> keys_of(std::mt19937_64& rng, int n) {
    std::vector<std::string> ks;
    for (int i = 0; i < n; i++) {
        // every XXH3 length class: 0, 1-3, 4-8, 9-16, 17-128, 129-240, > 240
        static const int lens[] = {0, 1, 3, 4, 8, 9, 16, 17, 100, 128, 129, 240, 241, 600, 5000};
        const int len = (i % 3 == 0) ? lens[rng() % 15] : (int)(rng() % 300);
        std::string s(len, '\0');
        for (auto& c : s) c = (char)rng();
        ks.push_back(s);
    }
    return ks;
}

static void host_build_cases(std::mt19937_64& rng) {
    for (uint32_t nb : {64u, 957u, 9568u, 2000003u}) {
        const auto ks = keys_of(rng, 1500);
        std::vector<uint8_t> data;
        std::vector<uint64_t> offs{0};
        for (auto& s : ks) {
            data.insert(data.end(), s.begin(), s.end());
            offs.push_back(data.size());
        }
        data.push_back(0);
        std::vector<uint64_t> wb(lsmb_num_words(nb)), wi(lsmb_num_words(nb));
        CHECK(lsmb_build_var(nullptr, data.data(), offs.data(), ks.size(), nb, 7, wb.data()) == LSMB_OK);
        for (auto& s : ks) CHECK(lsmb_insert(wi.data(), nb, 7, (const uint8_t*)s.data(), s.size()) == LSMB_OK);
        CHECK(wb == wi);
        for (auto& s : ks) CHECK(lsmb_may_contain(wb.data(), nb, 7, (const uint8_t*)s.data(), s.size()) == 1);
        // serialized block straight from the host path
        std::vector<uint8_t> blk(lsmb_serialized_size(nb));
        CHECK(lsmb_build_block(nullptr, data.data(), offs.data(), 0, ks.size(), nb, 7, blk.data(), blk.size()) == LSMB_OK);
        CHECK(memcmp(blk.data() + 12, wb.data(), wb.size() * 8) == 0);
        uint32_t crc = 0;
        CHECK(lsmb_build_block_crc(nullptr, data.data(), offs.data(), 0, ks.size(), nb, 7, blk.data(), blk.size(),
                                   &crc) == LSMB_OK);
        CHECK(crc == crc_bitwise(blk.data(), blk.size()));
        // fixed-length keys, key_len 0 (every key empty), unordered offsets
        std::vector<uint64_t> wf(lsmb_num_words(nb)), wf1(lsmb_num_words(nb));
        CHECK(lsmb_build_fixed(nullptr, data.data(), 7, 200, nb, 7, wf.data()) == LSMB_OK);
        for (int i = 0; i < 200; i++) lsmb_insert(wf1.data(), nb, 7, data.data() + 7 * i, 7);
        CHECK(wf == wf1);
        CHECK(lsmb_build_fixed(nullptr, nullptr, 0, 10, nb, 7, wf.data()) == LSMB_OK);
        std::vector<uint64_t> bad{5, 3};
        CHECK(lsmb_build_var(nullptr, data.data(), bad.data(), 1, nb, 7, wf.data()) == LSMB_EINVAL);
    }
    // reference panics -> EINVAL
    uint64_t w = 0;
    CHECK(lsmb_insert(&w, 0, 7, (const uint8_t*)"x", 1) == LSMB_EINVAL);
    uint32_t nb, k;
    CHECK(lsmb_params(0, 0.01, &nb, &k) == LSMB_EINVAL && lsmb_params(10, 1.0, &nb, &k) == LSMB_EINVAL);
    CHECK(lsmb_params(1000000000, 0.01, &nb, &k) == LSMB_OK && nb == 4294967295u && k == 7);
    // a GPU-sized build without a context is refused, not run on the host
    std::vector<uint8_t> big(16 * 5000);
    std::vector<uint64_t> wb(lsmb_num_words(100000));
    CHECK(lsmb_build_fixed(nullptr, big.data(), 16, 5000, 100000, 7, wb.data()) == LSMB_EINVAL);
}

static void stream_cases(std::mt19937_64& rng) {
    // a host-only stream (ctx = NULL) whose pinned-or-heap staging grows many
    // times (64 KiB first allocation): the threshold is raised so it finishes
    // with the host loop
    const uint64_t old = lsmb_host_max_keys();
    lsmb_set_host_max_keys(1u << 20);
    const uint32_t nb = 3000017;
    lsmb_stream* st = nullptr;
    CHECK(lsmb_stream_open(nullptr, nb, 7, &st) == LSMB_OK);
    for (int round = 0; round < 2; round++) {
        const auto ks = keys_of(rng, 20000);
        std::vector<uint64_t> wi(lsmb_num_words(nb));
        for (auto& s : ks) {
            CHECK(lsmb_stream_add(st, (const uint8_t*)s.data(), s.size()) == LSMB_OK);
            lsmb_insert(wi.data(), nb, 7, (const uint8_t*)s.data(), s.size());
        }
        CHECK(lsmb_stream_count(st) == ks.size());
        std::vector<uint8_t> blk(lsmb_serialized_size(nb));
        CHECK(lsmb_stream_finish_block(st, blk.data(), blk.size()) == LSMB_OK);
        CHECK(memcmp(blk.data() + 12, wi.data(), wi.size() * 8) == 0);
        CHECK(lsmb_stream_reset(st, nb, 7) == LSMB_OK);
    }
    CHECK(lsmb_stream_add(st, nullptr, 3) == LSMB_EINVAL);
    lsmb_stream_close(st);
    lsmb_set_host_max_keys(old);
}

static void crc_cases(std::mt19937_64& rng) {
    for (size_t n : {0ul, 1ul, 3ul, 4ul, 5ul, 15ul, 16ul, 17ul, 511ul, 4096ul, 100003ul}) {
        std::vector<uint8_t> b(n + 1);
        for (auto& x : b) x = (uint8_t)rng();
        CHECK(lsmb_crc32(0, b.data(), n) == crc_bitwise(b.data(), n));
        const size_t h = n / 3;
        CHECK(lsmb_crc32_combine(lsmb_crc32(0, b.data(), h), lsmb_crc32(0, b.data() + h, n - h), n - h) ==
              crc_bitwise(b.data(), n));
    }
}

static void threaded_cases() {
    // host entry points from 8 threads at once: builds, probes, errors, the
    // threshold (an atomic) read while another thread sets it
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 8; t++)
        th.emplace_back([t, &bad] {
            std::mt19937_64 rng(100 + t);
            const uint32_t nb = 9568;
            for (int it = 0; it < 200; it++) {
                std::vector<uint8_t> keys(16 * 1000);
                for (auto& x : keys) x = (uint8_t)rng();
                std::vector<uint64_t> w(lsmb_num_words(nb));
                if (lsmb_build_fixed(nullptr, keys.data(), 16, 1000, nb, 7, w.data()) != LSMB_OK) bad++;
                for (int i = 0; i < 1000; i += 97)
                    if (lsmb_may_contain(w.data(), nb, 7, keys.data() + 16 * i, 16) != 1) bad++;
                uint64_t one = 0;
                if (lsmb_insert(&one, 0, 3, keys.data(), 1) != LSMB_EINVAL || !strstr(lsmb_last_error(), "num_bits")) bad++;
                if (t == 0) lsmb_set_host_max_keys(it & 1 ? 2048 : 4096);
                (void)lsmb_host_max_keys();
            }
        });
    for (auto& x : th) x.join();
    lsmb_set_host_max_keys(2048);
    CHECK(bad.load() == 0);
}

int main() {
    std::mt19937_64 rng(42);
    deserialize_cases(rng);
    host_build_cases(rng);
    stream_cases(rng);
    crc_cases(rng);
    threaded_cases();
    // no device here: the batched path fails loudly
    lsmb_ctx* c = nullptr;
    const int rc = lsmb_open(&c, 0);
    CHECK(rc == LSMB_ENODEV || rc == LSMB_OK);
    if (c) lsmb_close(c);
    printf("host_sanitize: %s (%d failures)\n", g_fail ? "FAILED" : "ok", g_fail);
    return g_fail ? 1 : 0;
}
