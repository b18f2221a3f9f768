// bloom_probe.hip — batched multi-filter probe kernels for gfx950 (MI355X).
//
// Answers, for a batch of Q keys and F filters, exactly what the reference's
// per-SSTable check `bloom.may_contain(key)` (src/sstable/reader.rs:197 ->
// src/bloom/mod.rs:82-94) answers for each (key, filter) pair; DB::get walks
// L0 newest-first then L1+ and calls it once per SSTable (src/db/mod.rs:243-267).
// Each key is hashed ONCE (XXH3-128) whatever F is.
//
//   k_probe_sliced   all F filters share (num_bits, k) — the store's SSTable
//                    filters do: SSTableBuilder::new always sizes new(1000, 0.01)
//                    (src/sstable/builder.rs:51,74), 9 568 bits, k = 7.  Each
//                    workgroup bit-slices the F filters into one LDS table
//                    (entry p = the F filters' bit p), so a key costs k LDS
//                    reads and one AND chain for all F filters at once.
//   k_probe_generic  any mix of filters: per filter an exact position walk,
//                    bits read from HBM/L2 with early exit (mod.rs:88-90; the
//                    answer does not depend on early exit).
//
// Output row i (ceil(F/8) bytes): bit f%8 of byte f/8 = may_contain(f, key i).
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "kernels.hpp"
#include "keysrc.hpp"


namespace lsmb {
namespace {

constexpr uint32_t kProbeTableBytes = 64 * 1024;  // bit-sliced tables: the launchers' LDS cap
#ifndef LSMB_PROBE_DEPTH
#define LSMB_PROBE_DEPTH 5
#endif
constexpr int kProbeDepth = LSMB_PROBE_DEPTH;  // C3 probe: rounds of keys in flight

using ks::Fixed16;
using ks::FixedN;
using ks::VarLen;

template <typename T>
__device__ __forceinline__ void store_row(uint8_t* out, uint64_t i, uint32_t stride, T m) {
    if (sizeof(T) == 1) {
        out[i] = (uint8_t)m;
    } else if (stride == sizeof(T)) {
        reinterpret_cast<T*>(out)[i] = m;
    } else {
        for (uint32_t s = 0; s < stride; s++) out[i * stride + s] = (uint8_t)(m >> (8 * s));
    }
}

// A filter set's answer rows: row i = the u64 mask's low rb bytes (rb = 1, 2,
// 4 or 8: the caller's row width, covering the highest live slot), stored
// non-temporal (nothing in the call reads them; tools/archive/r04_out_nt.sh).
// rb is uniform, so the width select is scalar.
struct MaskOut {
    uint8_t* p;
    uint32_t rb;
    __device__ __forceinline__ void put(uint64_t i, uint64_t o) const {
        if (rb == 8) __builtin_nontemporal_store(o, reinterpret_cast<uint64_t*>(p) + i);
        else if (rb == 4) __builtin_nontemporal_store((uint32_t)o, reinterpret_cast<uint32_t*>(p) + i);
        else if (rb == 2) __builtin_nontemporal_store((uint16_t)o, reinterpret_cast<uint16_t*>(p) + i);
        else __builtin_nontemporal_store((uint8_t)o, p + i);
    }
};

// The bit-sliced probe's filters, passed by value in the kernel arguments:
// the kernel reads them with scalar loads at launch instead of chasing a
// device descriptor array, and lsmb_probe then needs no descriptor upload
// (nor the event that guards its reuse) for this path.
struct SlicedFilters {
    const uint32_t* w[32];  // filter f's words (LE u32 view of the u64 words)
    uint32_t ob[32];        // filter f's output bit
};

// Answer rows are stored with the non-temporal policy: nothing in the call
// reads them, and they then leave L2 / MALL to the keys (C3 probe 0.0432 ->
// 0.0425 ms, filter sets -1 %; profiles/r04/r04outnt_probe_rows_ab.log).

// Grid-wide rounds over n items for the 1024-thread C3 probe: round j is
// items [j*gs, (j+1)*gs), lane L of the grid takes item j*gs + L.  Each
// round's keys and rows are addressed through a buffer resource whose base
// the scalar unit advances: no 64-bit lane addresses, indices or bounds
// compares, and the last round's out-of-range lanes load zeros and their
// stores are dropped by the resource's num_records (windows past the last
// round are empty).  The counts are made scalar with readfirstlane, so every
// window bound is SALU work; launchers keep n below 2^40 (rounds < 2^31).
struct Rounds {
    uint32_t gs, lane, rounds, last;
    __device__ __forceinline__ Rounds(uint64_t n, uint32_t bs) {
        gs = gridDim.x * bs;
        lane = blockIdx.x * bs + threadIdx.x;
        rounds = (uint32_t)__builtin_amdgcn_readfirstlane((int)((n + gs - 1) / gs));
        last = (uint32_t)__builtin_amdgcn_readfirstlane((int)(n - (uint64_t)(rounds - 1) * gs));
    }
    // round j's window of `unit`-byte items at base
    __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t j, uint32_t unit) const {
        const uint32_t full = j + 1 < rounds ? gs : last;  // two scalar selects, no branches
        const uint32_t cnt = j < rounds ? full : 0u;
        return __builtin_amdgcn_make_buffer_rsrc((void*)((const uint8_t*)base + (uint64_t)j * (gs * unit)), 0,
                                                 (int)(cnt * unit), 0x00020000);
    }
    __device__ __forceinline__ u32x4 keys16(const uint4* k, uint32_t j) const {
        return __builtin_amdgcn_raw_buffer_load_b128(rsrc(k, j, 16), lane * 16, 0, 2 /* nt */);
    }
};

// T holds up to 8*sizeof(T) filters' bits per position.
// W: Walk32 when num_bits <= 2^31 (every intermediate fits 32 bits), else
// Walk64.  K > 0: k fixed at compile time (7 = BloomFilter::new at fpr 0.01).
// BS: workgroup size.  The table is built once per workgroup; the hot
// (16-B keys, 8-bit entries, k = 7) instantiations run 1024-thread
// workgroups, two per CU, so a CU builds it twice instead of eight times.
template <class Src, typename T, class W, int K, int BS = 256>
__global__ __launch_bounds__(BS) void k_probe_sliced(Src src, uint64_t n, typename W::Mod md, uint32_t k_,
                                                      uint32_t num_bits, const SlicedFilters sf,
                                                      uint32_t nfilt, uint32_t stride,
                                                      uint8_t* __restrict__ out) {
    // 1024-thread instantiations (the hot 16-B-key / k = 7 ones) hold the
    // table in static LDS of the 64 KiB maximum: a static array's base is a
    // compile-time 0, so a table read is one ds_read at the position itself
    // (a dynamic extern array's base is a link-time symbol: one more VALU add
    // per read, 7 per key).  Two such workgroups still fit a CU.
    extern __shared__ __align__(16) uint8_t smem_dyn[];
    __shared__ __align__(16) uint8_t smem_stat[BS == 1024 ? kProbeTableBytes : 16];
    uint8_t* const smem_raw = BS == 1024 ? smem_stat : smem_dyn;
    T* table = reinterpret_cast<T*>(smem_raw);
    // The C3 instantiation (16-B keys, one-byte rows, k = 7, 1024 threads)
    // walks the keys in Rounds; its first keys are requested before the
    // table is built, so that load's latency overlaps the filter-word loads
    // instead of following them.
    constexpr bool kRounds = std::is_same<Src, Fixed16>::value && BS == 1024 && K > 0 && sizeof(T) == 1;
    const Rounds R(kRounds ? n : 1, BS);
    auto round_keys = [&](uint32_t j) -> u32x4 {
        if constexpr (kRounds)
            return R.keys16(src.k, j);
        else
            return u32x4{0, 0, 0, 0};
    };
    // kProbeDepth (5) rounds in flight: round j + 5 is requested once round j
    // is done, so each load has four rounds of hashing to arrive (3 rounds:
    // 0.0423-0.0428 ms per C3 batch, 4: 0.0428-0.043, 5: 0.0411-0.0413,
    // 6: 0.0433; profiles/r05/r05g_probe_depth_pipe_ab.log, r05f).  The
    // scheduling barriers keep the rounds in program order: left alone, the
    // scheduler interleaves the independent rounds and the loop head then
    // waits for every load.
    u32x4 kr[kProbeDepth];
#pragma unroll
    for (int d = 0; d < kProbeDepth; d++) {
        kr[d] = round_keys(d);
        __builtin_amdgcn_sched_barrier(0);
    }
    const uint32_t nw32 = (uint32_t)(((uint64_t)num_bits + 31) / 32);  // 64-bit: num_bits may be 2^32-1
    // The filters' word pointers and output bits, loaded once and all at
    // once (a per-filter descriptor -> word load chain would serialise 2F
    // global round trips before the first key).
    // Branch-free: an absent filter slot re-reads filter 0's words under a
    // zero mask.  (Per-slot branches here also cost the round loop below its
    // load overlap: the compiler's wait analysis then made its head wait for
    // every key load in flight.)
    constexpr uint32_t FMAX = 8 * sizeof(T);
    const uint32_t* wp[FMAX];
    uint32_t ob[FMAX], vm[FMAX];
#pragma unroll
    for (uint32_t f = 0; f < FMAX; f++) {
        const uint32_t g = f < nfilt ? f : 0u;
        wp[f] = sf.w[g];
        ob[f] = sf.ob[g];
        vm[f] = f < nfilt ? 1u : 0u;
    }
    // One-byte entries with filter f on bit f (the probe's own layout): each
    // (word, byte) item is an 8x8 bit transpose of the filters' bytes, three
    // masked delta swaps on a u64, spread over all 1024 threads (a per-word
    // loop of 32 x 8 bit extracts ran on 299 threads: ~900 VALU each).
    bool ident = sizeof(T) == 1;
#pragma unroll
    for (uint32_t f = 0; f < FMAX; f++) ident = ident && (f >= nfilt || ob[f] == f);  // absent slots: vm[f] = 0
    if (ident) {
        for (uint32_t it = threadIdx.x; it < 4 * nw32; it += blockDim.x) {
            const uint32_t w = it >> 2, sh = 8 * (it & 3);
            uint64_t x = 0;
#pragma unroll
            for (uint32_t f = 0; f < FMAX; f++) x |= (uint64_t)((wp[f][w] >> sh) & (0xFFu * vm[f])) << (8 * f);
            // row f, column i (filter f's bit 8 (it&3) + i) -> row i, column f
            uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
            x ^= t ^ (t << 7);
            t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
            x ^= t ^ (t << 14);
            t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
            x ^= t ^ (t << 28);
            *reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(table) + 8 * it) = x;
        }
    }
    for (uint32_t w = threadIdx.x; !ident && w < nw32; w += blockDim.x) {
        uint32_t xs[FMAX];
#pragma unroll
        for (uint32_t f = 0; f < FMAX; f++) xs[f] = wp[f][w];
        T acc[32];
#pragma unroll
        for (int b = 0; b < 32; b++) acc[b] = 0;
#pragma unroll
        for (uint32_t f = 0; f < FMAX; f++) {
#pragma unroll
            for (int b = 0; b < 32; b++) acc[b] |= (T)((T)((xs[f] >> b) & vm[f]) << ob[f]);
        }
#pragma unroll
        for (int b = 0; b < 32; b++) table[w * 32 + b] = acc[b];
    }
    __syncthreads();
    T all = 0;
    for (uint32_t f = 0; f < nfilt; f++) all |= (T)((T)1 << sf.ob[f]);
    if constexpr (kRounds) {
        auto row = [&](const u32x4 v, uint32_t j) {
            const H128 h = xxh3_16(((uint64_t)v.y << 32) | v.x, ((uint64_t)v.w << 32) | v.z);
            W pw(md, h.lo, h.hi);
            T m = all;
#pragma unroll
            for (int jj = 0; jj < K; jj++) {
                m &= table[pw.pos()];
                if (jj + 1 < K) pw.next(md);
            }
            __builtin_amdgcn_raw_buffer_store_b8(m, R.rsrc(out, j, 1), R.lane, 0, 2 /* nt */);
        };
        for (uint32_t j = 0; j < R.rounds; j += kProbeDepth) {  // past the last round: empty windows (zeros, dropped rows)
#pragma unroll
            for (int d = 0; d < kProbeDepth; d++) {
                row(kr[d], j + d);
                __builtin_amdgcn_sched_barrier(0);
                kr[d] = round_keys(j + d + kProbeDepth);
                if (j + d + 1 == R.rounds) return;
            }
        }
        return;
    }
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    typename Src::Pre pre = src.fetch(i, i < n);  // next key's load is in flight while this one hashes
    for (; i < n; i += gs) {
        const typename Src::Pre cur = pre;
        pre = src.fetch(i + gs, i + gs < n);
        const H128 h = src.hash_pre(cur, i);
        W pw(md, h.lo, h.hi);
        T m = all;
        if (K > 0) {
#pragma unroll
            for (int j = 0; j < K; j++) {
                m &= table[pw.pos()];
                if (j + 1 < K) pw.next(md);
            }
        } else {
            for (uint32_t j = 0; j < k_; j++) {
                m &= table[pw.pos()];
                pw.next(md);
            }
        }
        store_row<T>(out, i, stride, m);
    }
}

template <class Src>
__global__ __launch_bounds__(256) void k_probe_generic(Src src, uint64_t n,
                                                       const ProbeFilter* __restrict__ filters,
                                                       uint32_t nfilt, uint32_t stride,
                                                       uint8_t* __restrict__ out) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        H128 h = src.hash(i);
        uint64_t m = 0;
        for (uint32_t f = 0; f < nfilt; f++) {
            const ProbeFilter& F = filters[f];
            bool hit = true;
            if (F.k) {
                PosWalk pw(F.md, h.lo, h.hi);
                for (uint32_t j = 0; j < F.k; j++) {
                    const uint32_t p = pw.pos();
                    if (!((F.words32[p >> 5] >> (p & 31)) & 1u)) {
                        hit = false;
                        break;
                    }
                    pw.next(F.md);
                }
            }
            if (hit) m |= 1ull << F.out_bit;
        }
        for (uint32_t s = 0; s < stride; s++) out[i * stride + s] = (uint8_t)(m >> (8 * s));
    }
}

// Lexicographic byte-string order, as Rust's `[u8]` Ord (a proper prefix
// sorts first): <0, 0, >0.  Eight bytes per step as big-endian u64 (unaligned
// dwordx2 loads), the tail byte by byte.
__device__ __forceinline__ int key_cmp(const uint8_t* a, uint64_t la, const uint8_t* b, uint32_t lb) {
    const uint64_t m = la < lb ? la : lb;
    uint64_t i = 0;
    for (; i + 8 <= m; i += 8) {
        const uint64_t x = __builtin_bswap64(xx::ld64(a + i)), y = __builtin_bswap64(xx::ld64(b + i));
        if (x != y) return x < y ? -1 : 1;
    }
    for (; i < m; i++)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

// A byte string's first 16 bytes, zero-padded, as two big-endian words.  Two
// strings whose padded prefixes differ order as the prefixes do (a difference
// inside the padding means the shorter one is a proper prefix of the other);
// equal prefixes order by length when both fit 16 bytes, else by key_cmp.
struct Pfx16 {
    uint64_t w0, w1;
    uint32_t len;
};

__device__ __forceinline__ Pfx16 prefix16(const uint8_t* p, uint64_t len) {
    Pfx16 r;
    r.len = len > 0xffffffffull ? 0xffffffffu : (uint32_t)len;
    if (len >= 16) {
        r.w0 = __builtin_bswap64(xx::ld64(p));
        r.w1 = __builtin_bswap64(xx::ld64(p + 8));
    } else {
        r.w0 = r.w1 = 0;
        for (uint32_t i = 0; i < (uint32_t)len; i++) {
            const uint64_t b = p[i];
            if (i < 8) r.w0 |= b << (56 - 8 * i);
            else r.w1 |= b << (56 - 8 * (i - 8));
        }
    }
    return r;
}

// Per workgroup: the set's boundary points and region masks into LDS.
struct FsetLds {
    uint64_t w0[kFsetMaxPoints], w1[kFsetMaxPoints];
    const uint8_t* p[kFsetMaxPoints];
    uint32_t len[kFsetMaxPoints];
    uint64_t regmask[2 * kFsetMaxPoints + 1];
};

__device__ __forceinline__ void stage_ranges(const FsetRanges& rg, FsetLds& L) {
    for (uint32_t j = threadIdx.x; j < rg.npts; j += blockDim.x) {
        const FsetPoint q = rg.pts[j];
        L.w0[j] = q.w0;
        L.w1[j] = q.w1;
        L.p[j] = q.p;
        L.len[j] = q.len;
    }
    for (uint32_t j = threadIdx.x; j < 2 * rg.npts + 1; j += blockDim.x) L.regmask[j] = rg.regmask[j];
}

// The key's region among the sorted points: a branch-free binary search on
// the 16-byte prefixes (a uniform loop of ceil(log2(npts + 1)) steps), then
// exact compares over the run of points whose prefix equals the key's (rare:
// keys or bounds longer than 16 bytes sharing their first 16).
__device__ __forceinline__ uint32_t key_region(const Pfx16& kx, const uint8_t* kp, uint64_t kl, const FsetLds& L,
                                               uint32_t m) {
    uint32_t lo = 0;
    for (uint32_t step = m ? 1u << (31 - __builtin_clz(m)) : 0u; step; step >>= 1) {
        const uint32_t j = lo + step - 1;
        if (j < m) {
            const uint64_t a = L.w0[j], b = L.w1[j];
            if (a < kx.w0 || (a == kx.w0 && b < kx.w1)) lo += step;
        }
    }
    uint32_t e = 0;
    while (lo < m && L.w0[lo] == kx.w0 && L.w1[lo] == kx.w1) {
        const uint32_t pl = L.len[lo];
        const int c = (kl <= 16 && pl <= 16) ? (kl < pl ? -1 : (kl > pl ? 1 : 0)) : key_cmp(kp, kl, L.p[lo], pl);
        if (c > 0) {
            lo++;
            continue;
        }
        e = c == 0;
        break;
    }
    return 2 * lo + e;
}

// Filter-set probe (multi-get pre-check): per key, for every SSTable of the
// set, the two checks SSTable::get makes before touching the index
// (src/sstable/reader.rs:192-199): key inside [min_key, max_key], then
// bloom.may_contain(key).  One hash per key; the range check of all tables
// is one region lookup (key_region); descriptors staged in LDS.
template <class Src>
__global__ __launch_bounds__(256) void k_fset_probe(Src src, uint64_t n, const RangedFilter* __restrict__ filters,
                                                    uint32_t nfilt, FsetRanges rg, MaskOut out) {
    __shared__ RangedFilter fl[64];
    __shared__ FsetLds L;
    for (uint32_t f = threadIdx.x; f < nfilt; f += blockDim.x) fl[f] = filters[f];
    stage_ranges(rg, L);
    __syncthreads();
    const uint32_t npts = rg.npts;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const H128 h = src.hash(i);
        const uint8_t* kp = src.bytes(i);
        const uint64_t kl = src.key_len(i);
        uint64_t rmask = L.regmask[key_region(prefix16(kp, kl), kp, kl, L, npts)];
        uint64_t m = 0;
        // Positions of the last (num_bits, k <= 8) walked: the store's SST
        // filters all share one sizing (builder.rs:51,74), so one walk serves
        // every table in range.
        uint32_t cpos[8];
        uint32_t cnb = 0, ck = 0;
        while (rmask) {
            const uint32_t f = (uint32_t)__builtin_ctzll(rmask);
            rmask &= rmask - 1;
            const RangedFilter& R = fl[f];
            bool hit = true;
            if (R.f.k && R.f.k <= 8) {
                if (R.f.num_bits != cnb || R.f.k != ck) {
                    PosWalk pw(R.f.md, h.lo, h.hi);
#pragma unroll
                    for (uint32_t j = 0; j < 8; j++) {
                        if (j < R.f.k) {
                            cpos[j] = pw.pos();
                            pw.next(R.f.md);
                        }
                    }
                    cnb = R.f.num_bits;
                    ck = R.f.k;
                }
#pragma unroll
                for (uint32_t j = 0; j < 8; j++)
                    if (j < ck) hit = hit && ((R.f.words32[cpos[j] >> 5] >> (cpos[j] & 31)) & 1u);
            } else if (R.f.k) {
                PosWalk pw(R.f.md, h.lo, h.hi);
                for (uint32_t j = 0; j < R.f.k; j++) {
                    const uint32_t p = pw.pos();
                    if (!((R.f.words32[p >> 5] >> (p & 31)) & 1u)) {
                        hit = false;
                        break;
                    }
                    pw.next(R.f.md);
                }
            }
            if (hit) m |= 1ull << R.f.out_bit;
        }
        out.put(i, m);
    }
}

// Filter-set probe when every filter of the set shares (num_bits, k) and the
// bit-sliced table fits LDS (the store's SST filters: new(1000, 0.01), 9 568
// bits, k = 7): entry p of the table holds the set's bit p, one bit per
// descriptor.  A key pays one region lookup for the range checks, then k LDS
// reads ANDed over all in-range filters at once (bits read from L2 per
// filter in k_fset_probe).
// W: Walk14 (the set's num_bits < 2^14, e.g. SST filters) or Walk32.
template <class Src, typename T, int K, int BS = 256, class W = Walk32>
__global__ __launch_bounds__(BS) void k_fset_sliced(Src src, uint64_t n, const RangedFilter* __restrict__ filters,
                                                     uint32_t nfilt, FsetRanges rg, uint32_t k_,
                                                     typename W::Mod md, MaskOut out) {
    // static table for the 1024-thread instantiations, as in k_probe_sliced
    extern __shared__ __align__(16) uint8_t smem_dyn[];
    __shared__ __align__(16) uint8_t smem_stat[BS == 1024 ? kProbeTableBytes : 16];
    uint8_t* const smem_raw = BS == 1024 ? smem_stat : smem_dyn;
    __shared__ RangedFilter fl[64];
    __shared__ FsetLds L;
    T* table = reinterpret_cast<T*>(smem_raw);
    for (uint32_t f = threadIdx.x; f < nfilt; f += blockDim.x) fl[f] = filters[f];
    stage_ranges(rg, L);
    __syncthreads();
    const uint32_t num_bits = fl[0].f.num_bits;
    bool ident = true;  // slots 0..nfilt-1 all live: table bit f is output bit f
    for (uint32_t f = 0; f < nfilt; f++) ident = ident && fl[f].f.out_bit == f;
    const uint32_t nw32 = (num_bits + 31) / 32;  // num_bits <= 2^19 here: no wrap
    if constexpr (sizeof(T) == 1) {
        // one-byte entries (<= 8 tables): 8x8 bit transposes over all threads,
        // as k_probe_sliced builds its table (absent slots: filter 0, masked)
        const uint32_t* wp[8];
        uint32_t vm[8];
#pragma unroll
        for (uint32_t f = 0; f < 8; f++) {
            wp[f] = fl[f < nfilt ? f : 0].f.words32;
            vm[f] = f < nfilt ? 0xFFu : 0u;
        }
        for (uint32_t it = threadIdx.x; it < 4 * nw32; it += blockDim.x) {
            const uint32_t w = it >> 2, sh = 8 * (it & 3);
            uint64_t x = 0;
#pragma unroll
            for (uint32_t f = 0; f < 8; f++) x |= (uint64_t)((wp[f][w] >> sh) & vm[f]) << (8 * f);
            uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
            x ^= t ^ (t << 7);
            t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
            x ^= t ^ (t << 14);
            t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
            x ^= t ^ (t << 28);
            *reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(table) + 8 * it) = x;
        }
    }
    for (uint32_t w = threadIdx.x; sizeof(T) > 1 && w < nw32; w += blockDim.x) {
        T acc[32];
#pragma unroll
        for (int b = 0; b < 32; b++) acc[b] = 0;
        for (uint32_t f = 0; f < nfilt; f++) {
            const uint32_t x = fl[f].f.words32[w];
#pragma unroll
            for (int b = 0; b < 32; b++) acc[b] |= (T)((T)((x >> b) & 1u) << f);
        }
#pragma unroll
        for (int b = 0; b < 32; b++) table[w * 32 + b] = acc[b];
    }
    __syncthreads();
    const uint32_t npts = rg.npts;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const H128 h = src.hash(i);
        const uint8_t* kp = src.bytes(i);
        const uint64_t kl = src.key_len(i);
        T m = (T)L.regmask[key_region(prefix16(kp, kl), kp, kl, L, npts)];
        if (m) {
            W pw(md, h.lo, h.hi);
            if (K > 0) {
#pragma unroll
                for (int j = 0; j < K; j++) {
                    m &= table[pw.pos()];
                    if (j + 1 < K) pw.next(md);
                }
            } else {
                for (uint32_t j = 0; j < k_; j++) {
                    m &= table[pw.pos()];
                    pw.next(md);
                }
            }
        }
        uint64_t o = (uint64_t)m;
        if (!ident) {
            o = 0;
            for (uint32_t f = 0; f < nfilt; f++)
                if ((m >> f) & 1) o |= 1ull << fl[f].f.out_bit;
        }
        out.put(i, o);
    }
}

// Filter-set probe over size classes (FsetClasses): a mixed set — e.g. L0
// flush outputs new(1000, .01) next to bigger compaction outputs — keeps one
// bit-sliced LDS table per (num_bits, k) class instead of walking every
// filter in L2.  Per key and class with an in-range member: one walk, k
// table reads ANDed over the class's members; the class's hits map back to
// descriptor bits; the range mask then keeps the in-range ones.
// Workgroups per CU: two for 16-B keys (registers capped at 64 for 8 waves
// per SIMD: 62, no spills; mixed set 0.151 -> 0.132 ms), one for the
// var-len / odd-length sources, which would spill at that cap.
constexpr uint32_t kClassBlock = 1024;
template <class Src>
constexpr uint32_t class_wgs_per_cu() { return std::is_same<Src, ks::Fixed16>::value ? 2u : 1u; }

template <class Src>
__global__ __launch_bounds__(kClassBlock, 4 * class_wgs_per_cu<Src>()) void k_fset_classes(Src src, uint64_t n, const RangedFilter* __restrict__ filters,
                                                      uint32_t nfilt, FsetRanges rg, FsetClasses cl,
                                                      MaskOut out) {
    extern __shared__ __align__(16) uint8_t smem_raw[];
    __shared__ RangedFilter fl[64];
    __shared__ FsetLds L;
    __shared__ uint8_t mem[kFsetMaxClasses][64];  // member j -> descriptor (per-lane indexed)
    const FsetClass* C = cl.cls;                  // uniform: scalar loads of the kernel arguments
    for (uint32_t f = threadIdx.x; f < nfilt; f += blockDim.x) fl[f] = filters[f];
    for (uint32_t i = threadIdx.x; i < cl.ncls * 64; i += blockDim.x) mem[i / 64][i % 64] = cl.cls[i / 64].mem[i % 64];
    stage_ranges(rg, L);
    __syncthreads();
    // class tables: thread w builds the 32 entries of word w, 32 members a pass
    for (uint32_t c = 0; c < cl.ncls; c++) {
        const uint32_t nw32 = (C[c].num_bits + 31) / 32, nm = C[c].nmem, width = C[c].width;
        uint8_t* t = smem_raw + C[c].off;
        if (width == 1) {  // (uniform) <= 8 members: 8x8 bit transposes over all threads, as k_fset_sliced
            const uint32_t* wp[8];
            uint32_t vm[8];
#pragma unroll
            for (uint32_t j = 0; j < 8; j++) {
                wp[j] = fl[mem[c][j < nm ? j : 0]].f.words32;
                vm[j] = j < nm ? 0xFFu : 0u;
            }
            for (uint32_t it = threadIdx.x; it < 4 * nw32; it += blockDim.x) {
                const uint32_t w = it >> 2, sh = 8 * (it & 3);
                uint64_t x = 0;
#pragma unroll
                for (uint32_t j = 0; j < 8; j++) x |= (uint64_t)((wp[j][w] >> sh) & vm[j]) << (8 * j);
                uint64_t q = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
                x ^= q ^ (q << 7);
                q = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
                x ^= q ^ (q << 14);
                q = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
                x ^= q ^ (q << 28);
                *reinterpret_cast<uint64_t*>(t + 8 * it) = x;
            }
            continue;
        }
        for (uint32_t w = threadIdx.x; w < nw32; w += blockDim.x) {
            for (uint32_t j0 = 0; j0 < nm; j0 += 32) {
                uint32_t acc[32];
#pragma unroll
                for (int b = 0; b < 32; b++) acc[b] = 0;
                for (uint32_t j = j0; j < nm && j < j0 + 32; j++) {
                    const uint32_t x = fl[mem[c][j]].f.words32[w];
#pragma unroll
                    for (int b = 0; b < 32; b++) acc[b] |= ((x >> b) & 1u) << (j - j0);
                }
#pragma unroll
                for (int b = 0; b < 32; b++) {
                    const uint32_t e = w * 32 + b;
                    if (width == 1) t[e] = (uint8_t)acc[b];
                    else if (width == 2) reinterpret_cast<uint16_t*>(t)[e] = (uint16_t)acc[b];
                    else if (width == 4) reinterpret_cast<uint32_t*>(t)[e] = acc[b];
                    else reinterpret_cast<uint32_t*>(t)[2 * e + (j0 >> 5)] = acc[b];
                }
            }
        }
    }
    __syncthreads();
    bool ident = true;  // descriptor d is output slot d
    for (uint32_t f = 0; f < nfilt; f++) ident = ident && fl[f].f.out_bit == f;
    const uint32_t npts = rg.npts, ncls = cl.ncls;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const H128 h = src.hash(i);
        const uint8_t* kp = src.bytes(i);
        const uint64_t kl = src.key_len(i);
        const uint64_t rm = L.regmask[key_region(prefix16(kp, kl), kp, kl, L, npts)];
        uint64_t o = 0;  // descriptor bits
        for (uint32_t c = 0; c < ncls; c++) {
            if (!(rm & C[c].mask)) continue;
            const uint8_t* t = smem_raw + C[c].off;
            const uint32_t width = C[c].width, kc = C[c].k;
            uint64_t acc = ~0ull;
            // entry type and walk (Walk14 below 2^14 bits): uniform per class
            auto walk = [&](auto tag, auto pw, const auto& md) {
                using E = decltype(tag);
                const E* te = reinterpret_cast<const E*>(t);
                if (kc == 7) {
#pragma unroll
                    for (int j = 0; j < 7; j++) {
                        acc &= te[pw.pos()];
                        if (j < 6) pw.next(md);
                    }
                } else {
                    for (uint32_t j = 0; j < kc; j++) {
                        acc &= te[pw.pos()];
                        pw.next(md);
                    }
                }
            };
            auto walk_w = [&](auto pw, const auto& md) {
                if (width == 1) walk(uint8_t{}, pw, md);
                else if (width == 2) walk(uint16_t{}, pw, md);
                else if (width == 4) walk(uint32_t{}, pw, md);
                else walk(uint64_t{}, pw, md);
            };
            if (Mod14::fits(C[c].num_bits)) {
                const Mod14 md = C[c].md14;
                walk_w(Walk14(md, h.lo, h.hi), md);
            } else {
                const Mod32 md = C[c].md;
                walk_w(Walk32(md, h.lo, h.hi), md);
            }
            if (C[c].nmem < 64) acc &= (1ull << C[c].nmem) - 1;
            while (acc) {
                const uint32_t j = (uint32_t)__builtin_ctzll(acc);
                acc &= acc - 1;
                o |= 1ull << mem[c][j];
            }
        }
        uint64_t wm = rm & cl.walk_mask;
        while (wm) {
            const uint32_t f = (uint32_t)__builtin_ctzll(wm);
            wm &= wm - 1;
            const RangedFilter& R = fl[f];
            bool hit = true;
            if (R.f.k) {
                PosWalk pw(R.f.md, h.lo, h.hi);
                for (uint32_t j = 0; j < R.f.k; j++) {
                    const uint32_t p = pw.pos();
                    if (!((R.f.words32[p >> 5] >> (p & 31)) & 1u)) {
                        hit = false;
                        break;
                    }
                    pw.next(R.f.md);
                }
            }
            if (hit) o |= 1ull << f;
        }
        o &= rm;
        if (!ident) {
            uint64_t s = 0;
            while (o) {
                const uint32_t d = (uint32_t)__builtin_ctzll(o);
                o &= o - 1;
                s |= 1ull << fl[d].f.out_bit;
            }
            o = s;
        }
        out.put(i, o);
    }
}

// 1024-thread sliced-probe workgroups per CU: measured best 1 for the probe
// (0.0625 vs 0.0648 ms at 2) and 2 for the filter set (0.082 vs 0.093 at 1);
// LSMB_PROBE_WGS_PER_CU overrides both (measurement knob, tools/probe_wgs.sh).
uint64_t probe_wgs_per_cu(uint64_t dflt) {
    static const long v = [] {
        const char* e = getenv("LSMB_PROBE_WGS_PER_CU");
        return e ? atol(e) : 0L;
    }();
    return v >= 1 && v <= 8 ? (uint64_t)v : dflt;
}

template <class Src>
hipError_t fset_probe_with(const Src& src, uint64_t n, const RangedFilter* df, uint32_t nfilt, const FsetRanges& rg,
                           const FsetClasses& cl, uint32_t shared_nb, uint32_t shared_k, MaskOut out, int num_cus,
                           hipStream_t st, hipEvent_t done) {
    uint64_t g = (n + 255) / 256;
    const uint64_t gmax = (uint64_t)num_cus * 8;
    if (g > gmax) g = gmax;
    if (g < 1) g = 1;
    if (!(shared_nb > 0 && shared_k > 0) && cl.ncls > 0 && cl.table_bytes <= kFsetTableBytes) {
        const size_t smem = cl.table_bytes;
        uint64_t gc = (n + kClassBlock - 1) / kClassBlock;
        if (gc > (uint64_t)num_cus * class_wgs_per_cu<Src>()) gc = (uint64_t)num_cus * class_wgs_per_cu<Src>();
        if (gc < 1) gc = 1;
        hipFuncSetAttribute((const void*)k_fset_classes<Src>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        return launch_done(k_fset_classes<Src>, dim3((uint32_t)gc), dim3(kClassBlock), (uint32_t)smem, st, done, src, n, df,
                           nfilt, rg, cl, out);
    }
    if (shared_nb > 0 && shared_k > 0) {
        const size_t tsz = nfilt <= 8 ? 1 : nfilt <= 16 ? 2 : nfilt <= 32 ? 4 : 8;
        const size_t smem = (size_t)(((uint64_t)shared_nb + 31) / 32) * 32 * tsz;
        if (smem <= kProbeTableBytes) {
            const Mod32 m32 = Mod32::make(shared_nb);
            auto go = [&](auto kern, auto md, uint32_t bs = 256) {
                if (bs != 1024)  // (the 1024-thread kernels' table is static LDS)
                    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
                const uint64_t gb = bs == 256 ? g : std::min<uint64_t>((n + bs - 1) / bs, probe_wgs_per_cu(2) * num_cus);
                return launch_done(kern, dim3((uint32_t)std::max<uint64_t>(gb, 1)), dim3(bs),
                                   bs == 1024 ? 0u : (uint32_t)smem, st, done, src, n, df, nfilt, rg, shared_k, md, out);
            };
            // (launch_done has consumed any launch error: return its result)
            if (tsz == 1) {
                if (shared_k == 7 && std::is_same<Src, Fixed16>::value && Mod14::fits(shared_nb))
                    return go(k_fset_sliced<Src, uint8_t, 7, 1024, Walk14>, Mod14::make(shared_nb), 1024);
                if (shared_k == 7 && std::is_same<Src, Fixed16>::value)
                    return go(k_fset_sliced<Src, uint8_t, 7, 1024>, m32, 1024);
                if (shared_k == 7) return go(k_fset_sliced<Src, uint8_t, 7>, m32);
                return go(k_fset_sliced<Src, uint8_t, 0>, m32);
            }
            if (tsz == 2) return go(k_fset_sliced<Src, uint16_t, 0>, m32);
            if (tsz == 4) return go(k_fset_sliced<Src, uint32_t, 0>, m32);
            return go(k_fset_sliced<Src, uint64_t, 0>, m32);
        }
    }
    return launch_done(k_fset_probe<Src>, dim3((uint32_t)g), dim3(256), 0u, st, done, src, n, df, nfilt, rg, out);
}

// Bytes of the bit-sliced LDS table the probe of these filters builds (all
// share (num_bits, k), at most 32, the table within kProbeTableBytes), or 0
// when they are walked from L2 by k_probe_generic instead.
size_t sliced_bytes(const ProbeFilter* hf, uint32_t nfilt) {
    bool same = nfilt > 0 && nfilt <= 32 && hf[0].k > 0;
    for (uint32_t f = 1; f < nfilt && same; f++) same = hf[f].num_bits == hf[0].num_bits && hf[f].k == hf[0].k;
    if (!same) return 0;
    const size_t ent = (size_t)(((uint64_t)hf[0].num_bits + 31) / 32) * 32;  // 64-bit: nb + 31 wraps at 2^32-1
    const size_t smem = ent * (nfilt <= 8 ? 1 : nfilt <= 16 ? 2 : 4);
    return smem <= kProbeTableBytes ? smem : 0;
}

template <class Src>
hipError_t probe_with(const Src& src, uint64_t n, const ProbeFilter* hf, uint32_t nfilt,
                      const ProbeFilter* df, uint8_t* out, int num_cus, hipStream_t st, hipEvent_t done) {
    const uint32_t stride = (nfilt + 7) / 8;
    uint64_t g = (n + 255) / 256;
    const uint64_t gmax = (uint64_t)num_cus * 8;
    if (g > gmax) g = gmax;
    if (g < 1) g = 1;
    {
        const size_t smem = sliced_bytes(hf, nfilt);
        const uint32_t nb = hf[0].num_bits;
        const size_t tsz = nfilt <= 8 ? 1 : nfilt <= 16 ? 2 : 4;
        if (smem) {
            SlicedFilters sf{};
            for (uint32_t f = 0; f < nfilt; f++) {
                sf.w[f] = hf[f].words32;
                sf.ob[f] = hf[f].out_bit;
            }
            auto go = [&](auto kern, auto md, uint32_t bs = 256) {
                if (bs != 1024)  // (the 1024-thread kernels' table is static LDS)
                    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
                const uint64_t gb = bs == 256 ? g : std::min<uint64_t>((n + bs - 1) / bs, probe_wgs_per_cu(1) * num_cus);
                kern<<<dim3((uint32_t)std::max<uint64_t>(gb, 1)), dim3(bs), bs == 1024 ? 0 : smem, st>>>(
                    src, n, md, hf[0].k, nb, sf, nfilt, stride, out);
            };
            const Mod32 m32 = hf[0].md;
            // (the 1024-thread kernel counts its grid-wide rounds in 31 bits)
            const bool w32 = fits_walk32(nb), k7 = hf[0].k == 7 && n < (1ull << 40);
            if (tsz == 1) {
                if (k7 && std::is_same<Src, Fixed16>::value && Mod14::fits(nb))
                    go(k_probe_sliced<Src, uint8_t, Walk14, 7, 1024>, Mod14::make(nb), 1024);
                else if (w32 && k7 && std::is_same<Src, Fixed16>::value)
                    go(k_probe_sliced<Src, uint8_t, Walk32, 7, 1024>, m32, 1024);
                else if (w32 && k7) go(k_probe_sliced<Src, uint8_t, Walk32, 7>, m32);
                else if (w32) go(k_probe_sliced<Src, uint8_t, Walk32, 0>, m32);
                else go(k_probe_sliced<Src, uint8_t, Walk64, 0>, m32);
            } else if (tsz == 2) {
                if (w32) go(k_probe_sliced<Src, uint16_t, Walk32, 0>, m32);
                else go(k_probe_sliced<Src, uint16_t, Walk64, 0>, m32);
            } else {
                if (w32) go(k_probe_sliced<Src, uint32_t, Walk32, 0>, m32);
                else go(k_probe_sliced<Src, uint32_t, Walk64, 0>, m32);
            }
            return hipGetLastError();
        }
    }
    return launch_done(k_probe_generic<Src>, dim3((uint32_t)g), dim3(256), 0u, st, done, src, n, df, nfilt, stride, out);
}

}  // namespace

hipError_t launch_fset_probe(const KeyBatch& kb, const RangedFilter* df, uint32_t nfilt, const FsetRanges& rg,
                             const FsetClasses& cl, uint32_t shared_nb, uint32_t shared_k, uint8_t* out_rows,
                             uint32_t row_bytes, int num_cus, hipStream_t st, hipEvent_t done) {
    if (kb.n == 0) return hipSuccess;
    if (nfilt > 64 || rg.npts > kFsetMaxPoints || cl.ncls > kFsetMaxClasses) return hipErrorInvalidValue;
    if (row_bytes != 1 && row_bytes != 2 && row_bytes != 4 && row_bytes != 8) return hipErrorInvalidValue;
    const MaskOut out{out_rows, row_bytes};
    if (kb.offsets)
        return fset_probe_with(VarLen{kb.data, kb.offsets}, kb.n, df, nfilt, rg, cl, shared_nb, shared_k, out, num_cus,
                               st, done);
    if (kb.key_len == 16 && (reinterpret_cast<uintptr_t>(kb.data) & 15) == 0)
        return fset_probe_with(Fixed16{reinterpret_cast<const uint4*>(kb.data)}, kb.n, df, nfilt, rg, cl, shared_nb,
                               shared_k, out, num_cus, st, done);
    return fset_probe_with(FixedN{kb.data, kb.key_len}, kb.n, df, nfilt, rg, cl, shared_nb, shared_k, out, num_cus,
                           st, done);
}

bool probe_reads_descriptors(const ProbeFilter* hf, uint32_t nfilt) { return sliced_bytes(hf, nfilt) == 0; }

hipError_t launch_probe(const KeyBatch& kb, const ProbeFilter* hf, uint32_t nfilt,
                        ProbeFilter* df, uint8_t* out, int num_cus, hipStream_t st, hipEvent_t done) {
    if (kb.n == 0) return hipSuccess;
    if (kb.offsets) return probe_with(VarLen{kb.data, kb.offsets}, kb.n, hf, nfilt, df, out, num_cus, st, done);
    if (kb.key_len == 16 && (reinterpret_cast<uintptr_t>(kb.data) & 15) == 0)
        return probe_with(Fixed16{reinterpret_cast<const uint4*>(kb.data)}, kb.n, hf, nfilt, df, out,
                          num_cus, st, done);
    return probe_with(FixedN{kb.data, kb.key_len}, kb.n, hf, nfilt, df, out, num_cus, st, done);
}

}  // namespace lsmb
