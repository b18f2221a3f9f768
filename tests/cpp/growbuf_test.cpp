// Host test of the grow-only buffer policy (storage-engine_amd/csrc/growbuf.hpp)
// with an allocator that has a fixed budget: growth under memory pressure must
// free the retired and then the live buffer before it gives up.
// Built and run by tests/test_growbuf.py (g++, no GPU).
#include <stdio.h>
#include <stdlib.h>

#include <map>

#include "../../storage-engine_amd/csrc/growbuf.hpp"

struct Budget {
    size_t limit = 0, used = 0, frees = 0;
    std::map<void*, size_t> live;
};
static Budget g;

struct MockAlloc {
    void* alloc(size_t n) {
        if (g.used + n > g.limit) return nullptr;
        void* q = malloc(n ? n : 1);
        g.used += n;
        g.live[q] = n;
        return q;
    }
    void free(void* q) {
        g.used -= g.live.at(q);
        g.live.erase(q);
        g.frees++;
        ::free(q);
    }
};

static int fails = 0;
#define CHECK(c)                                                   \
    do {                                                           \
        if (!(c)) {                                                \
            printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);    \
            fails++;                                               \
        }                                                          \
    } while (0)

int main() {
    // 1. plenty of memory: growth retires, never frees, capacity >= 1.5x
    g = Budget{};
    g.limit = 1 << 20;
    {
        lsmb::GrowBuf<MockAlloc> b;
        CHECK(b.ensure(100) && b.bytes == 100);
        CHECK(b.ensure(120) && b.bytes == 150);
        CHECK(b.retired.size() == 1 && g.frees == 0);
        CHECK(b.ensure(150) && b.bytes == 150 && b.retired.size() == 1);  // no growth
        b.release();
        CHECK(g.used == 0 && g.live.empty());
    }
    // 2. the 1.5x capacity does not fit, `want` does
    g = Budget{};
    g.limit = 1000;
    {
        lsmb::GrowBuf<MockAlloc> b;
        CHECK(b.ensure(400));
        CHECK(b.ensure(500) && b.bytes == 600);  // 400 + 600 = 1000 fits
        b.release();
    }
    g = Budget{};
    g.limit = 1000;
    {
        lsmb::GrowBuf<MockAlloc> b;
        CHECK(b.ensure(450));
        CHECK(b.ensure(500) && b.bytes == 500);  // 675 does not fit next to 450, 500 does
        CHECK(g.frees == 0);
        b.release();
    }
    // 3. old + new do not fit together: the retired buffers go first, then the live one
    g = Budget{};
    g.limit = 900;
    {
        lsmb::GrowBuf<MockAlloc> b;
        CHECK(b.ensure(200));
        CHECK(b.ensure(300) && b.retired.size() == 1);  // 200 retired + 300 live
        CHECK(b.ensure(500) && b.bytes == 500);         // frees the retired 200 first
        CHECK(g.frees == 1 && b.retired.size() == 1);   // 300 retired now
        CHECK(b.ensure(900) && b.bytes == 900);         // 300 + 500 + 900 > 900: frees both
        CHECK(b.retired.empty() && g.used == 900);
        b.release();
        CHECK(g.used == 0);
    }
    // 4. the live buffer alone is what stands in the way (no retired buffers)
    g = Budget{};
    g.limit = 1000;
    {
        lsmb::GrowBuf<MockAlloc> b;
        CHECK(b.ensure(600));
        CHECK(b.ensure(700) && b.bytes == 700 && g.used == 700 && b.retired.empty());
        b.release();
    }
    // 5. does not fit at all: failure, and the buffer is left empty (never dangling)
    g = Budget{};
    g.limit = 1000;
    {
        lsmb::GrowBuf<MockAlloc> b;
        CHECK(b.ensure(600));
        CHECK(!b.ensure(1001));
        CHECK(b.bytes == 0 && b.p == nullptr && g.used == 0);
        CHECK(b.ensure(10) && b.bytes == 10);  // usable again
        b.release();
        CHECK(g.used == 0 && g.live.empty());
    }
    printf(fails ? "growbuf: %d FAILED\n" : "growbuf: all passed\n", fails);
    return fails ? 1 : 0;
}
