// hash_var.hpp — k_hash_var: XXH3-128 of packed variable-length keys through
// an LDS window (device side, internal; included by bloom_build.hip and
// tools/mb_varhash.hip).
#pragma once

#include "keysrc.hpp"

namespace lsmb {

// Key bytes from a workgroup's LDS window (k_hash_var): LE loads at any byte
// offset (the window has >= 12 B of slack past its last byte).
struct LdsReader {
    const uint32_t* w;
    uint32_t base;  // the key's first byte in the window
    // Byte-aligned LDS loads: gfx950 kernels run in unaligned access mode, so
    // the compiler emits one ds_read at any byte address, folds constant
    // offsets into it and merges a 16-B run (mix32's a, a + 8) into one
    // ds_read_b128.  Building each 8 B from aligned dwords with v_alignbit
    // took ~5 VALU and 3 ds_read_b32 (k_hash_var: 2692 -> 2203 static VALU).
    __device__ __forceinline__ uint64_t ld64(uint64_t o) const {
        uint64_t v;
        __builtin_memcpy(&v, reinterpret_cast<const uint8_t*>(w) + base + (uint32_t)o, 8);
        return v;
    }
    __device__ __forceinline__ uint32_t ld32(uint64_t o) const {
        uint32_t v;
        __builtin_memcpy(&v, reinterpret_cast<const uint8_t*>(w) + base + (uint32_t)o, 4);
        return v;
    }
    __device__ __forceinline__ uint32_t u8(uint64_t o) const {
        return reinterpret_cast<const uint8_t*>(w)[base + (uint32_t)o];
    }
};

// k_hash for packed variable-length keys.  A workgroup's 256 keys are one
// contiguous byte range (C4: ~34 KB).  It is staged into LDS with coalesced,
// aligned 16-B loads — all of a thread's loads issued before its first LDS
// write, so ~10 KB per wave are in flight — and every lane hashes a key from
// LDS.  Per-lane reads straight from HBM touch a different cache line per
// lane per load.  Lanes are assigned to keys by length class (a counting sort
// of the 256 keys by ceil(len/32)), so a wave runs one XXH3 length path
// instead of all of them: mixed 8-256 B keys cost the divergent sum of the
// 0-16 / 17-128 / 129-240 / long paths otherwise (tools/mb_varhash.hip).
// Keys that do not fit the window start another round at the first unhashed
// key; a key longer than the whole window is hashed from global memory.
// Occupancy is the lever (tools/mb_varhash.hip, C4 lengths): a 36 KiB window
// and no per-key LDS arrays fit four workgroups per CU, and the kernel's 127
// VGPRs four waves per SIMD — 3.24 ms per 1e8 keys against 3.99 ms for a 40
// KiB window with LDS offset arrays (three workgroups, 133 VGPRs).  C4's
// 256-key blocks average 33.8 KB (sd ~1.2 KB), so ~3 % take a second round.
constexpr uint32_t kHashKeys = 256;       // keys (= threads) per workgroup
constexpr uint32_t kHashWin = 36 * 1024;  // LDS window bytes

__device__ __forceinline__ uint32_t len_class(uint64_t len) {
    if (len <= 16) return 0;
    if (len <= 240) return 1 + (uint32_t)((len - 1) >> 5);  // 1..8: the 17-128 / 129-240 round counts
    return 9;
}

// Where a hash kernel puts key i's hash: the 16-B (h1, h2) record (filter
// tiles, tools), or the 12-B walk record of a partitioned build (WalkRec:
// h1 and h2 reduced mod num_bits plus the walk's carries).
// kWords: the record's u32 words; words(): its contents; base(): record 0.
struct OutH128 {
    uint4* p;
    static constexpr uint32_t kWords = 4;
    __host__ __device__ OutH128(uint4* q) : p(q) {}
    __device__ __forceinline__ void put(uint64_t i, const H128& h) const {
        p[i] = make_uint4((uint32_t)h.lo, (uint32_t)(h.lo >> 32), (uint32_t)h.hi, (uint32_t)(h.hi >> 32));
    }
    __device__ __forceinline__ void words(const H128& h, uint32_t* w) const {
        w[0] = (uint32_t)h.lo, w[1] = (uint32_t)(h.lo >> 32), w[2] = (uint32_t)h.hi, w[3] = (uint32_t)(h.hi >> 32);
    }
    __device__ __forceinline__ uint32_t* base() const { return reinterpret_cast<uint32_t*>(p); }
};
struct OutRec {
    uint32_t* p;
    Mod32 md;
    uint32_t k;
    static constexpr uint32_t kWords = 3;
    __device__ __forceinline__ void put(uint64_t i, const H128& h) const {
        const WalkRec q = WalkRec::make(md, h, k);
        uint32_t* o = p + 3 * i;
        o[0] = q.r, o[1] = q.s, o[2] = q.c;
    }
    __device__ __forceinline__ void words(const H128& h, uint32_t* w) const {
        const WalkRec q = WalkRec::make(md, h, k);
        w[0] = q.r, w[1] = q.s, w[2] = q.c;
    }
    __device__ __forceinline__ uint32_t* base() const { return p; }
};

#ifndef LSMB_HV_REL
#define LSMB_HV_REL 1  // key offsets handed to the sorted lanes through LDS (A/B knob)
#endif
#ifndef LSMB_HV_COAL
#define LSMB_HV_COAL 1  // records staged in LDS and written as one coalesced block (A/B knob)
#endif

// WPE: waves per SIMD the register allocation must allow (0: compiler's
// choice).  The hash paths want ~130 VGPRs; at <= 128 four waves fit a SIMD.
template <int MODE = 0, uint32_t KEYS = kHashKeys, uint32_t WIN = kHashWin, int WPE = 0, class Out = OutH128>
__global__ __launch_bounds__(KEYS) __attribute__((amdgpu_waves_per_eu(WPE ? WPE : 1)))
void k_hash_var(const uint8_t* __restrict__ d, const uint64_t* __restrict__ o, uint64_t n, Out out) {
    constexpr uint32_t kPieces = WIN / (KEYS * 16);  // 16-B loads per thread per round
    static_assert(kPieces * KEYS * 16 == WIN, "window must be a whole number of rounds of loads");
    __shared__ uint32_t win[WIN / 4 + 8];
    __shared__ uint32_t cls_cnt[16];
    __shared__ uint16_t perm[KEYS];
    // the block's key offsets relative to its first (a block's keys span < 4 GiB)
    __shared__ uint32_t rel[LSMB_HV_REL ? KEYS + 1 : 1];
    static_assert(!LSMB_HV_COAL || KEYS * Out::kWords * 4 <= WIN, "records are staged in the window");
    const uint32_t t = threadIdx.x;
    const uint64_t i0 = (uint64_t)blockIdx.x * KEYS;
    const uint32_t m = (uint32_t)min<uint64_t>(KEYS, n - i0);
    // The first window's loads go out before anything else, as LDS-DMA (no
    // VGPRs held across the lane sort): the window and the offsets then share
    // one memory round trip instead of two back to back (C4: k_hash_var +
    // pass A 4.27 -> 4.13 ms).  A persistent form that keeps the next block's
    // window in flight in a second window while hashing (two workgroups per
    // CU) took 5.76 ms: the hash needs the four workgroups' waves.
    {
        const uintptr_t A0 = (uintptr_t)(d + o[i0]) & ~(uintptr_t)15;
        const uint32_t nb0 = (uint32_t)(min(A0 + (uintptr_t)WIN, (uintptr_t)(d + o[i0 + m])) - A0);
        const uint32_t wv = t >> 6;
#pragma unroll
        for (uint32_t r = 0; r < kPieces; r++) {
            const uint32_t q = (r * KEYS + t) * 16;
            if (q < nb0)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(A0 + q),
                                                 (__attribute__((address_space(3))) void*)(win + (r * KEYS + wv * 64) * 4),
                                                 16, 0, 0);
        }
    }
    // lane assignment by length class (a counting sort of the block's keys)
    uint32_t cls = 15;
    const uint64_t kbase = o[i0];
    // (a block spanning 4 GiB or more — keys of 16 MiB on average — reads its
    // offsets from global memory again instead)
    const bool use_rel = LSMB_HV_REL && o[i0 + m] - kbase <= 0xFFFFFFFFull;  // block-uniform
    if (t < m) {
        const uint64_t a = o[i0 + t], b = o[i0 + t + 1];
        cls = MODE == 2 ? 0 : len_class(b - a);  // MODE 2 (microbenchmark): no sort
        if (use_rel) {
            rel[t] = (uint32_t)(a - kbase);
            if (t == m - 1) rel[m] = (uint32_t)(b - kbase);
        }
    }
    if (t < 16) cls_cnt[t] = 0;
    // Every wave's window DMA has landed before any wave reads the window.  A
    // wave of a partial last block with no key (t >= m for all its lanes) may
    // still issue pieces and then has no later global load it waits on; the
    // workgroup barrier alone does not order its DMA (non-tgsplit mode).
    // Waves with keys waited on their offset loads anyway.
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint32_t rank = atomicAdd(&cls_cnt[cls], 1u);
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t c = 0; c < cls; c++) base += cls_cnt[c];
    perm[base + rank] = (uint16_t)t;
    __syncthreads();
    const uint32_t j = perm[t];  // the key this lane hashes
    uint64_t ka = 0, kb = 0;
    if (j < m) {
        if (use_rel) {  // (written before the perm barrier)
            ka = kbase + rel[j];
            kb = kbase + rel[j + 1];
        } else {
            ka = o[i0 + j];
            kb = o[i0 + j + 1];
        }
    }
    const uintptr_t end = (uintptr_t)(d + o[i0 + m]);  // one past the last key byte
    const uintptr_t pa = (uintptr_t)(d + ka), pb = (uintptr_t)(d + kb);
    H128 h{0, 0};
    uint32_t f = 0;  // first key not hashed yet (uniform)
    while (f < m) {
        // Window [A, wend): A = the 16-B block holding key f's first byte.
        // Every 16-B piece loaded holds at least one key byte, so no load
        // leaves the data's pages.
        const uintptr_t A = (uintptr_t)(d + o[i0 + f]) & ~(uintptr_t)15;
        const uintptr_t wend = min(A + (uintptr_t)WIN, end);
        const uint32_t nb = (uint32_t)(wend - A);
        if (f > 0) {  // (round 0's window is already in LDS)
            uint4 v[kPieces];
#pragma unroll
            for (uint32_t r = 0; r < kPieces; r++) {
                const uint32_t q = (r * KEYS + t) * 16;
                v[r] = q < nb ? ld_stream16((const uint4*)(A + q)) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (uint32_t r = 0; r < kPieces; r++) {
                const uint32_t q = (r * KEYS + t) * 16;
                if (q < nb) *(uint4*)((char*)win + q) = v[r];
            }
        }
        __syncthreads();
        // keys f.. that end inside the window: a prefix (offsets ascend)
        const bool fits = j >= f && j < m && pb <= wend;
        if (MODE == 1) {  // microbenchmark: staging only
            if (fits) h.lo ^= win[(pa - A) >> 2];
        } else if (fits) {
            h = xxh3_128_r(LdsReader{win, (uint32_t)(pa - A)}, kb - ka);
        }
        const uint32_t c = (uint32_t)__syncthreads_count(fits);
        if (c == 0) {  // key f alone is longer than the window
            if (j == f) h = xxh3_128(d + ka, kb - ka);
            f++;
        } else {
            f += c;
        }
    }
    if (!LSMB_HV_COAL) {
        if (j < m) out.put(i0 + j, h);
        return;
    }
    // The lanes hash keys in length-class order, so their records are
    // scattered over the block's range: stage them in the window (every lane
    // is past its last window read: the loop ends on a barrier) and write the
    // block's records as one contiguous run of 16-B stores.
    constexpr uint32_t W = Out::kWords;
    if (j < m) {
        uint32_t r[W];
        out.words(h, r);
#pragma unroll
        for (uint32_t q = 0; q < W; q++) win[j * W + q] = r[q];
    }
    __syncthreads();
    uint32_t* dst = out.base() + i0 * W;
    const uint32_t nw = m * W;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        for (uint32_t x = t; x < nw / 4; x += KEYS) reinterpret_cast<uint4*>(dst)[x] = reinterpret_cast<const uint4*>(win)[x];
        for (uint32_t x = (nw & ~3u) + t; x < nw; x += KEYS) dst[x] = win[x];
    } else {
        for (uint32_t x = t; x < nw; x += KEYS) dst[x] = win[x];
    }
}

}  // namespace lsmb
