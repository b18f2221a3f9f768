// crc32.hip — CRC-32 (IEEE 802.3, reflected, poly 0xEDB88320, init and
// xorout 0xFFFFFFFF) of bloom blocks: the checksum the store already uses for
// its WAL records and manifest (`crc32fast::hash`, src/wal/record.rs:96,122,
// src/manifest/mod.rs:5), here as the optional integrity check of the
// serialized filter that SURVEY.md §8 f4 lists (the reference's bloom block
// carries none).
//
// Device: each lane CRCs a 512-B piece with slicing-by-4 tables in LDS; the
// workgroup combines its 256 pieces in a tree (CRC(A‖B) = CRC(A)·x^(8|B|) ⊕
// CRC(B) in GF(2)[x] mod P, the combine of zlib's crc32_combine); the host
// combines the workgroups' CRCs in order.  A 120 MB C2 block is 915 workgroups.
#include <string.h>

#include <vector>

#include "ctx.hpp"

namespace lsmb {
namespace {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr uint32_t kCrcLanes = 256, kCrcPiece = 512;         // bytes per lane
constexpr uint64_t kCrcBlock = (uint64_t)kCrcLanes * kCrcPiece;  // bytes per workgroup

// a·b mod P, reflected bit order (bit 31 = x^0).
LSMB_HD uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (uint32_t m = 1u << 31; m && a; m >>= 1) {
        if (a & m) {
            p ^= b;
            a ^= m;
        }
        b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
    }
    return p;
}

// x^(8 n) mod P: square-and-multiply over x^(2^k) (x^1 = 0x40000000).
LSMB_HD uint32_t x8nmodp(uint64_t n) {
    uint32_t x2k = 0x40000000u;  // x^(2^0)
    // x^8 = x^(2^3): square three times
    for (int i = 0; i < 3; i++) x2k = multmodp(x2k, x2k);
    uint32_t p = 1u << 31;  // x^0
    while (n) {
        if (n & 1) p = multmodp(x2k, p);
        n >>= 1;
        x2k = multmodp(x2k, x2k);
    }
    return p;
}

// CRC(A‖B) from CRC(A), CRC(B) and |B| (standard, pre/post-inverted CRCs).
LSMB_HD uint32_t crc_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
    return multmodp(x8nmodp(len_b), crc_a) ^ crc_b;
}

struct CrcTables {
    uint32_t t[4][256];
};

void make_tables(CrcTables& T) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int j = 0; j < 8; j++) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
        T.t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; i++)
        for (int s = 1; s < 4; s++) T.t[s][i] = (T.t[s - 1][i] >> 8) ^ T.t[0][T.t[s - 1][i] & 0xFF];
}

const CrcTables& tables() {
    static const CrcTables T = [] {
        CrcTables t;
        make_tables(t);
        return t;
    }();
    return T;
}

// The x^(8·512·2^l) factors of the workgroup tree (l = 0..7), for full pieces.
struct TreePowers {
    uint32_t p[8];
};

TreePowers tree_powers() {
    TreePowers tp;
    for (int l = 0; l < 8; l++) tp.p[l] = x8nmodp((uint64_t)kCrcPiece << l);
    return tp;
}

// Workgroup w: CRC of bytes [w·128 KiB, min((w+1)·128 KiB, len)).
__global__ __launch_bounds__(kCrcLanes) void k_crc32(const uint8_t* __restrict__ d, uint64_t len, TreePowers tp,
                                                     uint32_t* __restrict__ out) {
    __shared__ uint32_t t[4][256];
    __shared__ uint32_t part[kCrcLanes];
    const uint32_t lane = threadIdx.x;
    {  // slicing-by-4 tables, one entry per lane
        uint32_t c0 = lane;
        for (int j = 0; j < 8; j++) c0 = (c0 & 1) ? (c0 >> 1) ^ kPoly : c0 >> 1;
        t[0][lane] = c0;
        __syncthreads();
        for (int s = 1; s < 4; s++) {
            t[s][lane] = (t[s - 1][lane] >> 8) ^ t[0][t[s - 1][lane] & 0xFF];
            __syncthreads();
        }
    }
    const uint64_t base = (uint64_t)blockIdx.x * kCrcBlock;
    const uint64_t a = base + (uint64_t)lane * kCrcPiece;
    const uint64_t e = a + kCrcPiece < len ? a + kCrcPiece : len;
    uint32_t c = 0xFFFFFFFFu;
    uint64_t i = a;
    if (a < e) {
        // 4 bytes per step (slicing-by-4); the piece start is 512-B aligned
        // from d: 16-B loads where d is 16-B aligned, dword loads where it is
        // only 4-B aligned (a uint4 access must be 16-B aligned), else the
        // byte loop
        auto step4 = [&](uint32_t w) {
            const uint32_t x = c ^ w;
            c = t[3][x & 0xFF] ^ t[2][(x >> 8) & 0xFF] ^ t[1][(x >> 16) & 0xFF] ^ t[0][x >> 24];
        };
        const uintptr_t al = reinterpret_cast<uintptr_t>(d);
        if ((al & 15) == 0) {
            for (; i + 16 <= e; i += 16) {
                const uint4 v = *reinterpret_cast<const uint4*>(d + i);
                step4(v.x), step4(v.y), step4(v.z), step4(v.w);
            }
        } else if ((al & 3) == 0) {
            for (; i + 16 <= e; i += 16) {
                const uint32_t* q = reinterpret_cast<const uint32_t*>(d + i);
                const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
                step4(w0), step4(w1), step4(w2), step4(w3);
            }
        }
        for (; i < e; i++) c = t[0][(c ^ d[i]) & 0xFF] ^ (c >> 8);
    }
    part[lane] = c ^ 0xFFFFFFFFu;
    __syncthreads();
    // tree: at level l, lane j (j % 2^(l+1) == 0) combines its run with the
    // run starting 2^l pieces later (length: full, or the tail's actual bytes)
    for (uint32_t l = 0; (1u << l) < kCrcLanes; l++) {
        const uint32_t step = 1u << l;
        if ((lane & (2 * step - 1)) == 0 && lane + step < kCrcLanes) {
            const uint64_t rb = a + (uint64_t)step * kCrcPiece;  // right run's first byte
            if (rb < len) {
                const uint64_t re = rb + (uint64_t)step * kCrcPiece;
                const uint64_t rlen = (re < len ? re : len) - rb;
                const uint32_t f = rlen == ((uint64_t)kCrcPiece << l) ? tp.p[l] : x8nmodp(rlen);
                part[lane] = multmodp(f, part[lane]) ^ part[lane + step];
            }
        }
        __syncthreads();
    }
    if (lane == 0) out[blockIdx.x] = part[0];
}

}  // namespace

uint32_t crc32_host(const uint8_t* p, uint64_t len, uint32_t crc) {
    const CrcTables& T = tables();
    uint32_t c = ~crc;
    uint64_t i = 0;
    for (; i + 4 <= len; i += 4) {
        uint32_t w;
        memcpy(&w, p + i, 4);
        const uint32_t x = c ^ w;
        c = T.t[3][x & 0xFF] ^ T.t[2][(x >> 8) & 0xFF] ^ T.t[1][(x >> 16) & 0xFF] ^ T.t[0][x >> 24];
    }
    for (; i < len; i++) c = T.t[0][(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return ~c;
}

uint32_t crc32_combine_host(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) { return crc_combine(crc_a, crc_b, len_b); }

// CRC-32 of device bytes, appended to `crc` (the CRC of the bytes before them;
// 0 for none).  Enqueued on st, then synchronised (the partials come back).
int crc32_dev(lsmb_ctx* c, const uint8_t* d, uint64_t len, uint32_t crc, hipStream_t st, uint32_t* out) {
    if (len == 0) {
        *out = crc;
        return LSMB_OK;
    }
    const uint64_t nwg = (len + kCrcBlock - 1) / kCrcBlock;
    if (nwg > 0x7FFFFFFFull) return fail(LSMB_EINVAL, "crc32: %llu bytes is too long", (unsigned long long)len);
    HIP_TRY(c->crc_parts.ensure(nwg * 4));
    static const TreePowers tp = tree_powers();
    k_crc32<<<dim3((uint32_t)nwg), dim3(kCrcLanes), 0, st>>>(d, len, tp, (uint32_t*)c->crc_parts.p);
    HIP_TRY(hipGetLastError());
    std::vector<uint32_t> parts(nwg);
    HIP_TRY(hipMemcpyAsync(parts.data(), c->crc_parts.p, nwg * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    static const uint32_t full = x8nmodp(kCrcBlock);
    uint32_t r = crc;
    for (uint64_t w = 0; w < nwg; w++) {
        const uint64_t blen = w + 1 < nwg ? kCrcBlock : len - w * kCrcBlock;
        r = multmodp(blen == kCrcBlock ? full : x8nmodp(blen), r) ^ parts[w];
    }
    *out = r;
    return LSMB_OK;
}

}  // namespace lsmb

using namespace lsmb;

extern "C" {

uint32_t lsmb_crc32(uint32_t crc, const uint8_t* data, uint64_t len) {
    if (!data || !len) return crc;
    return crc32_host(data, len, crc);
}

uint32_t lsmb_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) { return crc32_combine_host(crc_a, crc_b, len_b); }

int lsmb_crc32_dev(lsmb_ctx* c, uint32_t crc, const void* d_data, uint64_t len, uint32_t* out, void* stream) {
    if (!c || !out) return fail(LSMB_EINVAL, "null argument");
    if (len && !d_data) return fail(LSMB_EINVAL, "null device pointer");
    DevGuard g(c->dev);
    return crc32_dev(c, (const uint8_t*)d_data, len, crc, stream ? (hipStream_t)stream : c->st, out);
}

}  // extern "C"
