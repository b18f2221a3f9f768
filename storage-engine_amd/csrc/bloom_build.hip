// bloom_build.hip — Bloom filter build kernels for gfx950 (MI355X).
//
// Replaces the per-key insert loop of the reference
// (SSTableBuilder::add -> BloomFilterBuilder::add_key -> BloomFilter::insert,
//  src/sstable/builder.rs:93, src/bloom/builder.rs:21-23, src/bloom/mod.rs:70-78)
// with a batched build over a whole flushing/compacting run.  The bits produced
// are exactly the reference's: the same XXH3-128 split (mod.rs:181-189), the
// same wrapping double-hash positions (mod.rs:192-197) and the same LSB-first
// word layout (mod.rs:200-204), seen here as little-endian u32 words
// (bit p of u64 word p/64 == bit p%32 of u32 word p/32).  OR is associative,
// commutative and idempotent, so any key order / partition gives identical bits.
//
// Strategies (pick_build_strategy):
//   Lds        whole filter fits one CU's LDS (<= 160 KiB): every workgroup
//              builds a private copy with ds_or, then ORs non-zero words into
//              HBM with one global atomic per word.
//   Partition  big filters (BASELINE C2/C5: 120 MB / 512 MiB): two passes.
//              Pass A hashes keys and appends each position's 20-bit offset
//              within its 2^20-bit slice to a per-slice 64-B segment buffer
//              in LDS (3 offsets per u64, ds_or_b64); every full segment is
//              flushed with whole-segment stores into the workgroup's private
//              region for that slice (no global atomics, no partial-line
//              writes, 2.67 B per position instead of 4).  Pass B gives each
//              slice to one workgroup, which pulls the slice's words into
//              128 KiB of LDS, applies every offset from every region with
//              ds_or, and writes the slice back once.  No random global
//              atomics on the filter (the memory-side atomic unit serves ~20 G
//              scattered requests/s chip-wide; 7e8 of them would take ~35 ms).
//   Atomic     few keys into a huge filter: direct global atomicOr.
#include <mutex>
#include <vector>

#include <type_traits>

#include "kernels.hpp"
#include "keysrc.hpp"
#include "hash_var.hpp"

// LSMB_ABL (timing ablations for tools/, never in the product build):
//   1 = no segment flush, 2 = no claims/stores, 8 = no region stores,
//   16 = region stores issued but all dropped (out-of-range offset).
#ifndef LSMB_ABL
#define LSMB_ABL 0
#endif
#ifndef LSMB_APPLY_U
#define LSMB_APPLY_U 8  // pass B: 16-B region loads in flight per lane
#endif
// LSMB_STAMP=1 (diagnostic build for tools/, never the product): pass A's
// phase sections timed with s_memtime, summed per wave in scalar registers
// and added into g_stamp once per wave (MI355X stamp idiom): claims + hash +
// slot writes | barrier 1 wait | flush | barrier 2 wait.  Read its shares,
// not its length.
#ifndef LSMB_STAMP
#define LSMB_STAMP 0
#endif

namespace lsmb {
namespace {

#if LSMB_STAMP
__device__ unsigned long long g_stamp[8];
__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#endif

using ks::Fixed16;
using ks::FixedN;
using ks::VarLen;
using ks::Hashed;

__device__ __forceinline__ void or_bit_global(uint32_t* w, uint32_t p) {
    atomicOr(w + (p >> 5), 1u << (p & 31));
}

// ---------------------------------------------------------------- Lds strategy
template <class Src>
__global__ __launch_bounds__(1024) void k_build_lds(Src src, uint64_t n, Mod32 md, uint32_t k,
                                                    uint32_t nw32, uint32_t* __restrict__ gw) {
    extern __shared__ uint32_t filt[];
    for (uint32_t w = threadIdx.x; w < nw32; w += blockDim.x) filt[w] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        H128 h = src.hash(i);
        PosWalk pw(md, h.lo, h.hi);
        for (uint32_t j = 0; j < k; j++) {
            uint32_t p = pw.pos();
            atomicOr(&filt[p >> 5], 1u << (p & 31));
            pw.next(md);
        }
    }
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < nw32; w += blockDim.x) {
        uint32_t v = filt[w];
        if (v) atomicOr(gw + w, v);
    }
}

// ---------------------------------------------------------------- Tiled strategy
// Mid-size filters (160 KiB .. 4 MiB: compaction-sized SSTables).  Global
// atomics on such a filter run at the memory side (device-scope atomics are
// not L2-local across the 8 XCDs): ~26 G/s, 0.27 ms for 1 M keys.  Instead,
// workgroup (c, s) zeroes one 2^20-bit slice in LDS, hashes key chunk c and
// sets the positions that fall in slice s with ds_or, then stores the slice
// to its scratch tile with plain coalesced stores.  Every key is hashed once
// per slice (<= kTiledMaxSlices), which is cheaper than the atomics there.
template <class Src>
__global__ __launch_bounds__(1024) void k_build_tiled(Src src, uint64_t n, Mod32 md, uint32_t k, uint32_t nslices,
                                                      uint32_t nw32, uint64_t stride32,
                                                      uint32_t* __restrict__ tiles) {
    extern __shared__ uint32_t sl[];
    const uint32_t s = blockIdx.x % nslices, c = blockIdx.x / nslices, chunks = gridDim.x / nslices;
    for (uint32_t w = threadIdx.x; w < kSliceWords32; w += 1024) sl[w] = 0;
    __syncthreads();
    const uint64_t per = (n + chunks - 1) / chunks;
    const uint64_t i0 = (uint64_t)c * per, i1 = min(n, i0 + per);
    for (uint64_t i = i0 + threadIdx.x; i < i1; i += 1024) {
        const H128 h = src.hash(i);
        Walk32 pw(md, h.lo, h.hi);
        for (uint32_t j = 0; j < k; j++) {
            const uint32_t p = pw.pos();
            if ((p >> kSliceLog2) == s) atomicOr(&sl[(p & kSliceMask) >> 5], 1u << (p & 31));
            pw.next(md);
        }
    }
    __syncthreads();
    const uint32_t w0 = s * kSliceWords32;
    const uint32_t nw = min(kSliceWords32, nw32 - w0);
    uint4* dst = reinterpret_cast<uint4*>(tiles + (uint64_t)c * stride32 + w0);
    const uint4* srcw = reinterpret_cast<const uint4*>(sl);
    for (uint32_t q = threadIdx.x; q < (nw + 3) / 4; q += 1024) dst[q] = srcw[q];
}

// ---------------------------------------------------------------- Atomic strategy
template <class Src>
__global__ __launch_bounds__(256) void k_build_atomic(Src src, uint64_t n, Mod32 md, uint32_t k,
                                                      uint32_t* __restrict__ gw) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        H128 h = src.hash(i);
        PosWalk pw(md, h.lo, h.hi);
        for (uint32_t j = 0; j < k; j++) {
            or_bit_global(gw, pw.pos());
            pw.next(md);
        }
    }
}

// ---------------------------------------------------------------- Partition strategy
struct PassA {
    uint32_t b0, nb;        // this sweep's slices [b0, b0 + nb)
    uint32_t nbins;         // slices of the whole filter
    uint32_t grid, cap;     // regions per slice, region capacity (segments)
    uint32_t ring;          // ring entries per slice (multiple of 8, >= kSegEntries)
    uint64_t* regions;      // [grid][nbins][cap][8] u64: workgroup w's regions are contiguous
    uint32_t* counts;       // [nbins][grid] segments written
    uint32_t* gw;           // filter words (ring / region overflow only)
    // Fresh builds (k_bin<..., LIST = true>, see or_pos_list): a position
    // past its ring or region goes to the workgroup's list ovl[w][0, ovl_cap)
    // (length in ovn[w]), which k_ovf_apply ORs into the filter after pass B;
    // past a full list, its bit goes to the all-zero overflow words `ovf` and
    // its 2^20-bit unit is marked in `dirty`, which pass B folds in and clears.
    uint32_t* ovf;
    uint32_t* dirty;
    uint32_t* ovl;
    uint32_t* ovn;
    uint32_t ovl_cap;
    uint32_t* err;          // device counters (LSMB_STATS builds)
};

__device__ __forceinline__ uint64_t* region_ptr(const PassA& a, uint32_t b, uint32_t w) {
    return a.regions + ((uint64_t)w * a.nbins + b) * a.cap * kSegSlotWords;
}

// Workgroup barrier that waits for this wave's LDS operations only.
// __syncthreads() also drains vmcnt, i.e. waits for every outstanding global
// store and prefetch load; pass A's region stores and next-key loads are
// consumed by no other wave of this launch, so they stay in flight across
// phases.  The store data leaves the VGPRs at issue.
__device__ __forceinline__ void lds_barrier() {
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int SL = kSliceLog2>
__device__ __forceinline__ void or_pos_global(uint32_t* gw, uint32_t b, uint32_t off) {
    const uint32_t p = (b << SL) | off;
    atomicOr(gw + (p >> 5), 1u << (p & 31));
}

// The overflow path of a fresh build: a fresh build's pass B writes every
// filter word without reading it, so pass A must not touch the words.
template <int SL = kSliceLog2>
__device__ __forceinline__ void or_pos_list(const PassA& a, uint32_t* ovn_lds, uint32_t w, uint32_t b, uint32_t off) {
    const uint32_t p = (b << SL) | off;
    const uint32_t i = atomicAdd(ovn_lds, 1u);
    if (i < a.ovl_cap) {
        a.ovl[(uint64_t)w * a.ovl_cap + i] = p;
    } else {
        atomicOr(a.ovf + (p >> 5), 1u << (p & 31));
        a.dirty[p >> kSliceLog2] = 1u;
    }
}

// Three SL-bit offsets (SL = 20 or 21) in one u64: x | y << SL | z << 2 SL,
// built from 32-bit shift-or instructions (no 64-bit shifts).
template <int SL = kSliceLog2>
__device__ __forceinline__ uint2 pack3w(uint32_t x, uint32_t y, uint32_t z) {
    static_assert(SL == 20 || SL == 21, "3 offsets per u64");
    return make_uint2(x | (y << SL), (y >> (32 - SL)) | (z << (2 * SL - 32)));
}
template <int SL = kSliceLog2>
__device__ __forceinline__ uint64_t pack3(uint32_t x, uint32_t y, uint32_t z) {
    const uint2 w = pack3w<SL>(x, y, z);
    return ((uint64_t)w.y << 32) | w.x;
}

// Pass A (k_bin): hash keys, bin every position's 20-bit in-slice offset by
// slice, write the bins to HBM as 64-B segments of packed offsets.
//
// One 1024-thread workgroup per CU owns a contiguous key range and walks it in
// phases of one key per lane.  LDS holds, per slice of the sweep, a ring of R
// u32 offsets (R a multiple of 8) and a fill word
//     lo16 = ring start + 4 * claims (bytes, unwrapped), hi16 = claims,
// plus one sink slice (index nb) that absorbs the claims of lanes with no
// position (tail keys, positions outside the sweep) with an increment of 0.
//   claim   one ds_add_rtn of (4 | 1 << 16) returns the entry's slot; the
//           offset is stored with one ds_write_b32 (branch-free).  A claim
//           past the ring (adversarial duplicates only; rare at the planned R)
//           stores into the sink and sets its bit with a global atomicOr:
//           pass B reads the filter words after pass A, so the result is exact;
//   barrier
//   flush   wave v owns slices [v*SPW, (v+1)*SPW), one lane each, which keeps
//           its ring's start and its region's segment count in registers.
//           Every full 24-entry segment becomes a job; two lanes per job read
//           its three 8-entry groups (ds_read_b128; 8 | R, so a group never
//           wraps), pack 3 offsets per u64 (entry e at bits 20*(e>>3) of word
//           e&7) and store 32 B each to the region.  The owner advances the
//           start and rewrites the fill word;
//   barrier
// The next key's load is issued two phases ahead and its hash is computed
// while this phase's claims are in flight.  No waiting loops, no global
// atomics on the hot path.  EXACT: k == KMAX at compile time (k = 7 is what
// BloomFilter::new yields for fpr = 0.01).
constexpr uint32_t kAhead = 4;  // pass A key prefetch distance, in phases

// PER: keys per lane per phase.  Sweeps (!FULL) keep ~1/sweeps of the
// positions, so their phases take two keys per lane: half the barriers and
// flush rounds per key (PartitionPlan::keys_per_lane; the ring is sized for it).
// SL: bin width log2 (20; 21 for sweeps of filters above 2^30 bits, whose
// pass B applies each bin as two 2^20-bit halves).
// LIST: a fresh build's pass A (overflow to the lists, or_pos_list); the
// OR-accumulate kernels set overflow bits in the filter words directly.
template <class Src, class W, int KMAX, bool EXACT, bool FULL, int PER = 1, int SL = kSliceLog2, bool LIST = false>
__global__ __launch_bounds__(kBinBlock) void k_bin(Src src, uint64_t n, Mod32 md, uint32_t k_, PassA a) {
    static_assert(PER == 1 || EXACT, "two keys per lane: exact k only");
    constexpr uint32_t kMask = (1u << SL) - 1;
    constexpr int NP = PER * KMAX;  // positions per lane per phase
    // The whole LDS, statically: its base is then a compile-time 0, so ring,
    // fill and job addresses need no base add (a dynamic extern array's base
    // is a link-time symbol: one more VALU add per LDS address).  Pass A
    // always runs one workgroup per CU with all of the LDS.
    __shared__ uint32_t sm[kLdsBytes / 4];
    const uint32_t k = EXACT ? (uint32_t)KMAX : k_;
    const uint32_t R = a.ring, R4 = 4 * a.ring, nb = a.nb;
    uint32_t* fill = sm + (size_t)(nb + 1) * R;  // nb + 1 fill words (the last: sink)
    // per-wave flush job tables, 16-B aligned after the fill words
    uint4* jobtab = reinterpret_cast<uint4*>(sm + ((((size_t)(nb + 1) * (R + 1)) + 3) & ~(size_t)3));
    const uint32_t tid = threadIdx.x, w = blockIdx.x, lane = tid & 63, wave = tid >> 6;
    // overflow list length (LIST): the word after the job tables
    uint32_t* ovn = reinterpret_cast<uint32_t*>(jobtab + (kBinBlock / 64) * kBinJobsPerWave);
    for (uint32_t i = tid; i <= nb; i += kBinBlock) fill[i] = 0;
    if (LIST && tid == 0) *ovn = 0;
    // a position past its ring or region
    auto overflow = [&](uint32_t b, uint32_t off) {
        if constexpr (LIST)
            or_pos_list<SL>(a, ovn, w, b, off);
        else
            or_pos_global<SL>(a.gw, b, off);
    };
    // Workgroup w's regions as a raw buffer: a store at an offset past
    // num_records is dropped by the hardware, which lets every lane issue the
    // flush stores unconditionally (see the flush).
    const __amdgpu_buffer_rsrc_t rgn = __builtin_amdgcn_make_buffer_rsrc(
        region_ptr(a, 0, w), 0, (int)(a.nbins * a.cap * kSegSlotBytes), 0x00020000);
    constexpr uint32_t kDrop = 0x80000000u;  // >= num_records (plan keeps it < 2^31)
    constexpr uint32_t kInc = 4u | (1u << 16);
    const uint32_t sink = nb << SL;  // local position of the sink slice
    const uint32_t lim = R << 16;            // fill < lim <=> claims < R

    // Workgroup w owns keys [w*per, (w+1)*per): a contiguous, coalesced run.
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t i0 = (uint64_t)w * per, i1 = min(n, i0 + per);
    const uint64_t iters = i1 > i0 ? (i1 - i0 + PER * kBinBlock - 1) / (PER * kBinBlock) : 0;  // uniform
    const uint32_t spw = (nb + 15) / 16;  // slices per wave (<= 64)
    const uint32_t own = wave * spw + lane;
    const bool owner = lane < spw && own < nb;
    uint32_t start = 0, segs = 0;  // owner: ring start (bytes), region segments written

    // Local positions (p - b0 * 2^20) of the key this lane claims in the
    // current phase; `sink` where there is none.  kinc: this key's increment.
    uint32_t pos[NP], kinc[PER];
    auto walk_positions = [&](const typename Src::Seed& h, bool ok, uint32_t* out) {
        W walk(md, h);
#pragma unroll
        for (int q = 0; q < KMAX; q++) {
            if (EXACT || (uint32_t)q < k) {
                const uint32_t lp = walk.pos() - (FULL ? 0u : (a.b0 << SL));
                out[q] = (FULL || lp < sink) ? lp : sink;
                if (q + 1 < KMAX) walk.next(md);
            }
        }
        // lanes past the key range (the last phases only): sink positions
        if (__builtin_expect(__ballot(!ok) != 0, 0)) {
#pragma unroll
            for (int q = 0; q < KMAX; q++)
                if (!ok && (EXACT || (uint32_t)q < k)) out[q] = sink;
        }
    };
    // a lane's keys of phase `it`: key_index(it) + j, j < PER
    auto key_index = [&](uint64_t it) { return i0 + (it * kBinBlock + tid) * PER; };
    auto key_ok = [&](uint64_t it, int j = 0) { return it < iters && key_index(it) + j < i1; };
    using Pre = typename Src::Pre;
    auto fetch_keys = [&](uint64_t it, Pre (&out)[PER]) {
#pragma unroll
        for (int j = 0; j < PER; j++) out[j] = src.fetch(key_index(it) + j, key_ok(it, j));
    };
    // Keys are loaded kAhead phases before they are hashed, into kAhead
    // buffers with static roles (the loop is unrolled kAhead times, so no
    // register copy forces a vmcnt drain).  gfx9 retires loads and stores in
    // one in-order vmcnt queue: a key load completes only after every older
    // region store, so the distance must cover the store round trip too.
    Pre pb0[PER], pb1[PER], pb2[PER], pb3[PER];  // phase m's keys live in pb[m % 4]
#pragma unroll
    for (int j = 0; j < PER; j++) {
        const bool ok = key_ok(0, j);
        const Pre p = src.fetch(key_index(0) + j, ok);
        const typename Src::Seed h = ok ? src.hash_pre(p, key_index(0) + j) : typename Src::Seed{};
        walk_positions(h, ok, pos + j * KMAX);
        kinc[j] = ok ? kInc : 0u;
    }
    fetch_keys(1, pb1);
    fetch_keys(2, pb2);
    fetch_keys(3, pb3);
    fetch_keys(4, pb0);
    __syncthreads();

#if LSMB_STAMP
    uint64_t st_sum[4] = {0, 0, 0, 0}, st_prev = stamp(), st_t;
#endif
    // One phase: claim key it's positions, hash and walk key it+1 (from
    // `pre`) and reload `pre` with key it+1+kAhead, store the entries,
    // barrier, flush, barrier.  (Moving the walk past the first barrier, next
    // to the flush's LDS round trips, measured neutral at C2 and 0.15 ms
    // slower on C5's sweeps: DESIGN.md section 4.2.)
    auto phase = [&](uint64_t it, Pre (&pre)[PER]) __attribute__((always_inline)) {
        // Claims for this phase's keys, back to back.
        uint32_t got[NP];
#pragma unroll
        for (int q = 0; q < NP; q++) {
            if (EXACT || (uint32_t)q < k) {
                if (FULL) {
                    got[q] = (LSMB_ABL & 2) ? pos[q] : atomicAdd(fill + (pos[q] >> SL), kinc[q / KMAX]);
                } else {
                    // A sweep keeps ~nb/nbins of the positions: the others are
                    // masked off rather than sent to the sink, whose single
                    // fill word and slot would serialise them (same-address
                    // LDS atomics and writes).
                    got[q] = pos[q] < sink ? atomicAdd(fill + (pos[q] >> SL), kInc) : 0u;
                }
            }
        }
        // While the claims are in flight: hash and walk key it+1, pinned here
        // (an empty asm that consumes the positions): otherwise the compiler
        // sinks the whole hash + walk below the barrier, where every wave
        // computes while none has LDS work, and the claims' round trip is
        // exposed instead.
        uint32_t npos[NP], nkinc[PER];
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const bool ok = key_ok(it + 1, j);
            walk_positions(src.hash_pre(pre[j], key_index(it + 1) + j), ok, npos + j * KMAX);
            nkinc[j] = ok ? kInc : 0u;
        }
        fetch_keys(it + 1 + kAhead, pre);
#pragma unroll
        for (int q = 0; q < NP; q++)
            if (EXACT || (uint32_t)q < k) asm volatile("" ::"v"(npos[q]));
        // Store the claimed entries.  Fast path (every claim of the wave fits
        // its ring): slot address = b * R4 + wrapped ring offset, one full-rate
        // 24-bit multiply-add, no per-position select.  A wave with an
        // overflowing claim (adversarial duplicates only) takes the checked
        // path: overflowing claims skip the ring and set their bit with a
        // global atomic (pass B reads the filter words after pass A, so the
        // result is exact).
        uint32_t gmax = 0;
#pragma unroll
        for (int q = 0; q < NP; q++)
            if (EXACT || (uint32_t)q < k) gmax = max(gmax, got[q]);
        auto slot = [&](int q) {
            uint32_t x = got[q] & 0xFFFFu;
            x = min(x, x - R4);
            return __umul24(pos[q] >> SL, R4) + x;
        };
        if (__builtin_expect(__ballot(gmax >= lim) == 0, 1)) {
#pragma unroll
            for (int q = 0; q < NP; q++) {
                if (EXACT || (uint32_t)q < k) {
                    if (LSMB_ABL & 2) continue;
                    if (FULL || pos[q] < sink) *(uint32_t*)((char*)sm + slot(q)) = pos[q] & kMask;
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < NP; q++) {
                if ((EXACT || (uint32_t)q < k) && (FULL || pos[q] < sink)) {
                    if (got[q] < lim) {
                        *(uint32_t*)((char*)sm + slot(q)) = pos[q] & kMask;
                    } else if (pos[q] < sink) {  // (the sink's claims add 0: never past its ring)
                        overflow(a.b0 + (pos[q] >> SL), pos[q] & kMask);
#ifdef LSMB_STATS
                        atomicAdd(a.err + 9, 1u);
#endif
                    }
                }
            }
        }
#pragma unroll
        for (int q = 0; q < NP; q++) pos[q] = npos[q];
#pragma unroll
        for (int j = 0; j < PER; j++) kinc[j] = nkinc[j];
#if LSMB_STAMP
        st_t = stamp(), st_sum[0] += st_t - st_prev, st_prev = st_t;
#endif
        lds_barrier();
#if LSMB_STAMP
        st_t = stamp(), st_sum[1] += st_t - st_prev, st_prev = st_t;
#endif

        // Flush, wave-cooperative: every owner lane whose slice holds a full
        // 24-entry segment posts it as a job {group addresses, region offset}
        // in its wave's LDS job table; then four lanes write each job's 64-B
        // segment, 16 B each, so one store instruction writes 16 segments.
        // Region stores cost per instruction issued, not per byte (scattered
        // 16-B stores with most lanes idle: 0.34 of pass A's 1.05 ms at C2),
        // so the flush issues exactly kCoopRounds stores per wave per phase,
        // at a dropped offset where a lane has nothing to write — a static
        // store count also keeps the compiler's vmcnt waits for the
        // prefetched keys exact.  A second segment of the same slice, or a
        // region already full, takes the per-lane path below (rare).
        uint32_t cnt = 0;
        if (owner) {
            cnt = min(fill[own] >> 16, R);
            if (LSMB_ABL & 1) {
                fill[own] = start;
                cnt = 0;
            }
        }
        const bool has = cnt >= (uint32_t)kSegEntries;
        const char* ring = (const char*)sm + own * R4;
        uint4 x0, x1, y0, y1, z0, z1;
        auto read_segment = [&]() {
            // the segment's three 8-entry groups (8 | R: a group never wraps)
            uint32_t g0 = start, g1 = start + 32, g2 = start + 64;
            g1 = min(g1, g1 - R4);
            g2 = min(g2, g2 - R4);
            x0 = *(const uint4*)(ring + g0), x1 = *(const uint4*)(ring + g0 + 16);
            y0 = *(const uint4*)(ring + g1), y1 = *(const uint4*)(ring + g1 + 16);
            z0 = *(const uint4*)(ring + g2), z1 = *(const uint4*)(ring + g2 + 16);
        };
        auto store_segment = [&](uint32_t off) {
            const uint2 q0 = pack3w<SL>(x0.x, y0.x, z0.x), q1 = pack3w<SL>(x0.y, y0.y, z0.y);
            const uint2 q2 = pack3w<SL>(x0.z, y0.z, z0.z), q3 = pack3w<SL>(x0.w, y0.w, z0.w);
            const uint2 q4 = pack3w<SL>(x1.x, y1.x, z1.x), q5 = pack3w<SL>(x1.y, y1.y, z1.y);
            const uint2 q6 = pack3w<SL>(x1.z, y1.z, z1.z), q7 = pack3w<SL>(x1.w, y1.w, z1.w);
            if (!(LSMB_ABL & 8)) {
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{q0.x, q0.y, q1.x, q1.y}, rgn, off, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{q2.x, q2.y, q3.x, q3.y}, rgn, off + 16, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{q4.x, q4.y, q5.x, q5.y}, rgn, off + 32, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{q6.x, q6.y, q7.x, q7.y}, rgn, off + 48, 0, 0);
            }
        };
        auto spill_segment = [&]() {  // region full (adversarial inputs): exact global atomics
            if constexpr (LIST) {
                // (rolled over the ring: one inlined list append per site, not 24)
#pragma unroll 1
                for (uint32_t t = 0; t < (uint32_t)kSegEntries; t++) {
                    uint32_t e = start + 4 * t;
                    e = min(e, e - R4);
                    overflow(a.b0 + own, *(const uint32_t*)(ring + e));
                }
            } else {
                const uint32_t vals[24] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w,
                                           y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w,
                                           z0.x, z0.y, z0.z, z0.w, z1.x, z1.y, z1.z, z1.w};
                for (int t = 0; t < 24; t++) or_pos_global<SL>(a.gw, a.b0 + own, vals[t]);
            }
#ifdef LSMB_STATS
            atomicAdd(a.err + 7, 24u);
#endif
        };
        // 1. post jobs (owner lanes with a full segment and room in the region)
        const bool coop = has && segs < a.cap;
        const uint64_t cm = __ballot(coop);
        const uint32_t jobs = min((uint32_t)__popcll(cm), kBinJobsPerWave);  // wave-uniform
        bool posted = false;
        if (coop) {
            const uint32_t j = __builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
            if (j < kBinJobsPerWave) {
                const uint32_t rb = own * R4;
                uint32_t g1 = start + 32, g2 = start + 64;
                g1 = min(g1, g1 - R4);
                g2 = min(g2, g2 - R4);
                jobtab[wave * kBinJobsPerWave + j] =
                    make_uint4(rb + start, rb + g1, rb + g2, ((a.b0 + own) * a.cap + segs) * kSegSlotBytes);
                posted = true;
            }
        }
        // (the job table is this wave's own: its LDS writes and reads stay in order)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        // 2. kCoopRounds store instructions: lane L writes 16 B of job r*16 + L/4
        constexpr uint32_t kCoopRounds = (kBinJobsPerWave + 15) / 16;
#pragma unroll
        for (uint32_t r = 0; r < kCoopRounds; r++) {
            const uint32_t j = r * 16 + (lane >> 2), l = lane & 3;
            uint32_t off = kDrop;
            // a lane with no job stores at a dropped offset: its data is never
            // written, so it need not be defined (no register clears)
            uint2 w0, w1;
            asm("" : "=v"(w0.x), "=v"(w0.y), "=v"(w1.x), "=v"(w1.y));
            if (j < jobs) {
                const uint4 jb = jobtab[wave * kBinJobsPerWave + j];
                // segment word 2l+e = pack3<SL>(group0[2l+e], group1[2l+e], group2[2l+e])
                const uint2 a0 = *(const uint2*)((const char*)sm + jb.x + 8 * l);
                const uint2 a1 = *(const uint2*)((const char*)sm + jb.y + 8 * l);
                const uint2 a2 = *(const uint2*)((const char*)sm + jb.z + 8 * l);
                w0 = pack3w<SL>(a0.x, a1.x, a2.x);
                w1 = pack3w<SL>(a0.y, a1.y, a2.y);
                off = (LSMB_ABL & 16) ? kDrop : jb.w + 16 * l;
            }
            if (!(LSMB_ABL & 8)) __builtin_amdgcn_raw_buffer_store_b128(u32x4{w0.x, w0.y, w1.x, w1.y}, rgn, off, 0, 0);
        }
        // 3. owners advance past the posted segment; the rest per lane
        if (has) {
            if (!posted) {
                read_segment();
                if (segs < a.cap)
                    store_segment(((a.b0 + own) * a.cap + segs) * kSegSlotBytes);
                else
                    spill_segment();
            }
            const uint32_t nf = cnt / (uint32_t)kSegEntries;
            uint32_t s = start + 96;
            start = min(s, s - R4);
            segs = min(segs + 1, a.cap);
            // more full segments (filters with few, busy slices)
            for (uint32_t j = 1; j < nf; j++) {
                read_segment();
                if (segs < a.cap)
                    store_segment(((a.b0 + own) * a.cap + segs) * kSegSlotBytes);
                else
                    spill_segment();
                s = start + 96;
                start = min(s, s - R4);
                segs = min(segs + 1, a.cap);
            }
            const uint32_t rem = cnt - nf * (uint32_t)kSegEntries;
            fill[own] = (start + 4 * rem) | (rem << 16);
        }
#if LSMB_STAMP
        st_t = stamp(), st_sum[2] += st_t - st_prev, st_prev = st_t;
#endif
        lds_barrier();
#if LSMB_STAMP
        st_t = stamp(), st_sum[3] += st_t - st_prev, st_prev = st_t;
#endif
    };
    // Whole groups of kAhead phases (the last group's extra phases carry no
    // keys): no early exit, so the buffers keep their registers.
    const uint64_t groups = (iters + kAhead - 1) / kAhead;
    for (uint64_t g = 0; g < groups; g++) {
        const uint64_t it = g * kAhead;
        phase(it, pb1);
        phase(it + 1, pb2);
        phase(it + 2, pb3);
        phase(it + 3, pb0);
    }

#if LSMB_STAMP
    if (lane == 0) {
        for (int q = 0; q < 4; q++) atomicAdd(&g_stamp[q], (unsigned long long)st_sum[q]);
        atomicAdd(&g_stamp[4], (unsigned long long)groups * kAhead);
        atomicAdd(&g_stamp[5], 1ull);
    }
#endif
    // Segments still queued, then the last open segment (< 24 entries, padded
    // with copies of its first offset: setting a bit twice is a no-op), then
    // the region's segment count.  Rare tail work, one lane per slice.
    if (owner) {
        uint32_t cnt = min(fill[own] >> 16, R);
        while (cnt) {
            const uint32_t m = min(cnt, (uint32_t)kSegEntries);
            uint32_t v[kSegEntries];
#pragma unroll
            for (int t = 0; t < kSegEntries; t++) {
                uint32_t s = start + 4 * ((uint32_t)t < m ? t : 0);
                s = min(s, s - R4);
                v[t] = *(const uint32_t*)((const char*)sm + own * R4 + s);
            }
            if (segs < a.cap) {
                uint64_t* dst = region_ptr(a, a.b0 + own, w) + (uint64_t)segs * kSegSlotWords;
#pragma unroll
                for (int t = 0; t < kSegWords; t++) dst[t] = pack3<SL>(v[t], v[t + 8], v[t + 16]);
                segs++;
            } else {
                for (uint32_t t = 0; t < m; t++) overflow(a.b0 + own, v[t]);
            }
            const uint32_t s = start + 4 * m;
            start = min(s, s - R4);
            cnt -= m;
        }
        a.counts[(uint64_t)(a.b0 + own) * a.grid + w] = segs;
    }
    if constexpr (LIST) {  // the overflow list's length, for k_ovf_apply
        __syncthreads();
        if (tid == 0) a.ovn[w] = min(*ovn, a.ovl_cap);
    }
}

// Fresh partition builds, after pass B: OR the positions pass A listed as
// overflow (PassA::ovl) into the filter with global atomics.  Block w takes
// list w (pass A workgroup w of a sweep).
__global__ __launch_bounds__(256) void k_ovf_apply(const uint32_t* __restrict__ ovl, const uint32_t* __restrict__ ovn,
                                                   uint32_t cap, uint32_t* __restrict__ gw) {
    const uint32_t w = blockIdx.x, n = ovn[w];
    const uint32_t* l = ovl + (uint64_t)w * cap;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t p = l[i];
        atomicOr(gw + (p >> 5), 1u << (p & 31));
    }
}

// Pass B: one 2^20-bit slice per workgroup, applied in LDS.
//   1. the slice's words go to LDS with every load issued before the first
//      LDS write (a load / wait / write loop pays one HBM round trip per 8 B
//      of each thread: 16 per slice);
//   2. wave v applies regions v, v+16, ...; their segment counts arrive in
//      one lane-parallel load up front (lane j: region v + 16 j), then each
//      region's 16-B pieces are loaded U per lane at a time and every 20-bit
//      offset is ORed into LDS;
//   3. the slice is written back once, with non-temporal stores.
// fresh (BloomFilter::new + inserts, LIST pass A): the slice starts from zero
// instead of its words in HBM, which are then write-only; a unit marked in
// `dirty` ORs in (and clears) its overflow words.
// SL = 21 (2^21-bit bins): a bin is applied as two 2^20-bit halves by two
// workgroups, each reading all of the bin's offsets and keeping its own.
// Units u -> (bin, half) so that the two halves of a bin are blocks u and
// u + 8 (or u + w in a last group of w < 8 bins): the same XCD under
// round-robin dispatch, close in time, so the second read of the bin's
// regions mostly hits in L2 / MALL.
template <int SL = kSliceLog2>
__global__ __launch_bounds__(kApplyBlock) void k_apply(const uint64_t* __restrict__ regions,
                                                       const uint32_t* __restrict__ counts,
                                                       uint32_t grid, uint32_t cap, uint32_t nbins,
                                                       uint32_t* __restrict__ gw, uint64_t nw32,
                                                       uint32_t bfirst, uint32_t bend,
                                                       uint32_t* __restrict__ ovf, uint32_t* __restrict__ dirty,
                                                       uint32_t fresh) {
    constexpr uint32_t H = 1u << (SL - kSliceLog2);  // 2^20-bit halves per bin
    constexpr uint32_t kMask = (1u << SL) - 1;
    __shared__ uint32_t filt[kSliceWords32];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr uint32_t NWAVE = kApplyBlock / 64;
    constexpr uint32_t PER = kSliceWords32 / 2 / kApplyBlock;  // u64 words per thread
    const uint32_t nunits = (bend - bfirst) * H;
    for (uint32_t u = blockIdx.x; u < nunits; u += gridDim.x) {
        uint32_t b = bfirst + u, half = 0;
        if constexpr (H > 1) {
            const uint32_t g = u / (8 * H), r = u % (8 * H);
            const uint32_t wdt = min(8u, bend - bfirst - g * 8);
            b = bfirst + g * 8 + r % wdt;
            half = r / wdt;
        }
        const uint64_t w0 = ((uint64_t)b * H + half) * kSliceWords32;
        if (w0 >= nw32) continue;  // (block-uniform) the last bin's missing half
        const uint32_t nw2 = (uint32_t)min((uint64_t)kSliceWords32, nw32 - w0) / 2;  // u64 words
        uint2* g2 = reinterpret_cast<uint2*>(gw + w0);
        uint2* f2 = reinterpret_cast<uint2*>(filt);
        const uint32_t unit = (uint32_t)(w0 / kSliceWords32);
        const bool dty = dirty && dirty[unit] != 0u;  // block-uniform (fresh builds only)
        {
            uint2 v[PER];
#pragma unroll
            for (uint32_t u = 0; u < PER; u++) {
                const uint32_t i = tid + u * kApplyBlock;
                v[u] = (i < nw2 && !fresh) ? g2[i] : make_uint2(0, 0);
            }
#pragma unroll
            for (uint32_t u = 0; u < PER; u++) {
                const uint32_t i = tid + u * kApplyBlock;
                if (i < nw2) f2[i] = v[u];
            }
        }
        if (__builtin_expect(dty, 0)) {  // (rolled, after the slice load: no registers held across)
            uint2* o2 = reinterpret_cast<uint2*>(ovf + w0);
#pragma unroll 1
            for (uint32_t i = tid; i < nw2; i += kApplyBlock) {
                const uint2 o = o2[i];
                f2[i].x |= o.x;
                f2[i].y |= o.y;
                o2[i] = make_uint2(0, 0);
            }
        }
        const uint32_t nreg = wave < grid ? (grid - 1 - wave) / NWAVE + 1 : 0;  // <= 64 (grid <= 1024)
        const uint32_t cnt = lane < nreg ? counts[(uint64_t)b * grid + wave + lane * NWAVE] : 0u;
        __syncthreads();
        for (uint32_t j = 0; j < nreg; j++) {
            const uint32_t r = wave + j * NWAVE;
            const uint32_t nseg = __shfl(cnt, (int)j);
            const uint4* src = reinterpret_cast<const uint4*>(regions + ((uint64_t)r * nbins + b) * cap * kSegSlotWords);
            const uint32_t n16 = nseg * (kSegWords / 2);  // 16-B pieces (2 words, 6 offsets)
            constexpr uint32_t U = LSMB_APPLY_U;           // loads in flight per lane
            for (uint32_t i0 = 0; i0 < n16; i0 += 64 * U) {
                uint4 v[U];
#pragma unroll
                for (uint32_t u = 0; u < U; u++) {
                    const uint32_t i = i0 + u * 64 + lane;
                    const uint32_t ia = kSegSlotWords == kSegWords ? i : (i / 4) * (kSegSlotWords / 2) + (i % 4);
                    v[u] = i < n16 ? ld_stream16(src + ia) : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (uint32_t u = 0; u < U; u++) {
                    if (i0 + u * 64 + lane < n16) {
                        const uint64_t lo = ((uint64_t)v[u].y << 32) | v[u].x;
                        const uint64_t hi = ((uint64_t)v[u].w << 32) | v[u].z;
#pragma unroll
                        for (int e = 0; e < 3; e++) {
                            const uint32_t o0 = (uint32_t)(lo >> (SL * e)) & kMask;
                            const uint32_t o1 = (uint32_t)(hi >> (SL * e)) & kMask;
                            if (H == 1 || (o0 >> kSliceLog2) == half)
                                atomicOr(&filt[(o0 & kSliceMask) >> 5], 1u << (o0 & 31));
                            if (H == 1 || (o1 >> kSliceLog2) == half)
                                atomicOr(&filt[(o1 & kSliceMask) >> 5], 1u << (o1 & 31));
                        }
                    }
                }
            }
        }
        __syncthreads();
        // Non-temporal write-back (one global_store_dwordx2 ... nt per word
        // pair): this build reads the words no more, and dirty lines left in
        // L2 / MALL were written back during the next build's pass A instead
        // (C2 pass A 1.003 -> 0.979 ms, step 1.389 -> 1.371 ms;
        // profiles/r04/r04ntw_writeback_ab.log).
        for (uint32_t i = tid; i < nw2; i += kApplyBlock) {
            const uint2 v = f2[i];
            __builtin_nontemporal_store(v.x, &g2[i].x);
            __builtin_nontemporal_store(v.y, &g2[i].y);
        }
        if (dty && tid == 0) dirty[unit] = 0u;  // every thread read it before the first barrier
        __syncthreads();
    }
}

// ---------------------------------------------------------------- helpers
__global__ __launch_bounds__(256) void k_or_reduce(uint32_t* __restrict__ dst,
                                                   const uint32_t* __restrict__ src, uint64_t nw32,
                                                   uint32_t nsrc, uint64_t stride32) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw32; i += stride) {
        uint32_t v = dst[i];
        for (uint32_t j = 0; j < nsrc; j++) v |= src[j * stride32 + i];
        dst[i] = v;
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void k_gen_key16(uint64_t seed, uint64_t first, uint64_t n,
                                                   uint4* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
        const uint64_t i = first + j;
        const uint64_t a = splitmix64(seed + 2 * i), b = splitmix64(seed + 2 * i + 1);
        out[j] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    }
}

// out[j] = mod ? add + sm(seed + first + j) % mod : sm(seed + first + j)
// (tests/keygen.py varlen: key lengths with mod 249 / add 8, key bytes with mod 0).
__global__ __launch_bounds__(256) void k_gen_splitmix(uint64_t seed, uint64_t first, uint64_t n, uint32_t mod,
                                                      uint32_t add, uint64_t* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
        const uint64_t x = splitmix64(seed + first + j);
        out[j] = mod ? add + x % mod : x;
    }
}

// (h1, h2) = xxh3_128(key i) for every key, as 16-B records (ks::Hashed) or
// 12-B walk records (ks::Recs).  Full occupancy and no barriers, so the
// per-lane key-byte loads of many waves overlap; pass A then reads
// coalesced records.
template <class Src, class Out>
__global__ __launch_bounds__(256) void k_hash(Src src, uint64_t n, Out out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out.put(i, src.hash(i));
}

// The max-dynamic-LDS attribute is a property of the kernel, not of a launch:
// set it once per kernel (to the whole 160 KiB), not before every launch.
void set_max_lds(const void* fn) {
    static std::mutex mu;
    static std::vector<const void*> done;
    std::lock_guard<std::mutex> g(mu);
    for (const void* d : done)
        if (d == fn) return;
    hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes);
    done.push_back(fn);
}

// k_hash_var geometry: keys per workgroup and LDS window (measurement knobs
// LSMB_HV_KEYS / LSMB_HV_WIN; the window is a whole number of 16-B load rounds).
#ifndef LSMB_HV_KEYS
#define LSMB_HV_KEYS 256
#endif
#ifndef LSMB_HV_WIN
#define LSMB_HV_WIN (36 * 1024)
#endif
#ifndef LSMB_HV_WPE
#define LSMB_HV_WPE 0
#endif
template <class Out>
void launch_hash_var(const VarLen& src, uint64_t n, Out out, hipStream_t st) {
    const uint64_t g = (n + LSMB_HV_KEYS - 1) / LSMB_HV_KEYS;
    k_hash_var<0, LSMB_HV_KEYS, LSMB_HV_WIN, LSMB_HV_WPE, Out><<<dim3((uint32_t)g), dim3(LSMB_HV_KEYS), 0, st>>>(src.d, src.o, n, out);
}

template <class W>
struct WalkTag {  // a walk type as a value (dispatch lambdas)
    using type = W;
};

template <class Src>
hipError_t build_with(const Src& src, uint64_t n, uint32_t num_bits, uint32_t k, uint32_t* gw,
                      BuildStrategy s, const PartitionWorkspace& ws, int num_cus, hipStream_t st,
                      BuildTimers* tm, int sweep, bool fresh, bool t0_done = false, hipEvent_t done = nullptr) {
    // `done` is completed by the last kernel's own dispatch where the path ends
    // in one (launch_done); otherwise recorded after it.
    bool done_set = false;
    const Mod32 md = Mod32::make(num_bits);
    // sweep >= 0 (partition builds): only that sweep's slices — pass A keeps
    // their positions, pass B applies them; every other strategy has one sweep
    if (sweep > 0 && s != BuildStrategy::Partition) return done ? hipEventRecord(done, st) : hipSuccess;
    const uint32_t nw32 = (uint32_t)(2 * (((uint64_t)num_bits + 63) / 64));
    if (tm && !t0_done) hipEventRecord(tm->t0, st);
    constexpr bool kRecSrc = std::is_same<Src, ks::Recs>::value;  // walk records: partition builds only
    // fresh: the words are output-only.  Single-sweep k = 7 partition builds
    // write every word in pass B without reading it; the rest start from zeros.
    if (fresh && s != BuildStrategy::Partition) {
        const hipError_t e = hipMemsetAsync(gw, 0, (size_t)nw32 * 4, st);
        if (e != hipSuccess) return e;
    }
    if (s != BuildStrategy::Partition) {
      if constexpr (kRecSrc) {
        return hipErrorInvalidValue;
      } else if (s == BuildStrategy::Lds) {
        const size_t smem = (size_t)nw32 * 4;
        // ~8 Ki keys per workgroup keeps the final per-word OR cheap.
        uint64_t g = (n + 8191) / 8192;
        const uint64_t gmax = (uint64_t)num_cus * (smem <= 40 * 1024 ? 4 : 1);
        if (g > gmax) g = gmax;
        if (g < 1) g = 1;
        set_max_lds((const void*)k_build_lds<Src>);
        k_build_lds<Src><<<dim3((uint32_t)g), dim3(1024), smem, st>>>(src, n, md, k, nw32, gw);
        if (tm) hipEventRecord(tm->t1, st);
    } else if (s == BuildStrategy::Tiled) {
        const TiledPlan tp = plan_tiled(num_bits, n, num_cus);
        if (!ws.regions || tp.scratch_bytes > ws.region_bytes) return hipErrorInvalidValue;
        uint32_t* tiles = reinterpret_cast<uint32_t*>(ws.regions);
        if (ws.hashes && ws.hash_bytes >= n * 16 && !std::is_same<Src, Hashed>::value) {
            // every slice's workgroups re-read the keys: hash them once into
            // 16-B records (L2/MALL-resident at these sizes) and tile over those
            const uint64_t g = (n + 255) / 256;
            if (g > 0x7FFFFFFFull) return hipErrorInvalidValue;
            if constexpr (std::is_same<Src, VarLen>::value)
                launch_hash_var(src, n, OutH128(ws.hashes), st);
            else
                k_hash<Src, OutH128><<<dim3((uint32_t)g), dim3(256), 0, st>>>(src, n, OutH128(ws.hashes));
            const Hashed hs{ws.hashes};
            set_max_lds((const void*)k_build_tiled<Hashed>);
            k_build_tiled<Hashed><<<dim3(tp.chunks * tp.nslices), dim3(1024), kSliceWords32 * 4, st>>>(
                hs, n, md, k, tp.nslices, nw32, tp.stride32, tiles);
        } else {
            set_max_lds((const void*)k_build_tiled<Src>);
            k_build_tiled<Src><<<dim3(tp.chunks * tp.nslices), dim3(1024), kSliceWords32 * 4, st>>>(
                src, n, md, k, tp.nslices, nw32, tp.stride32, tiles);
        }
        if (tm) hipEventRecord(tm->t1, st);
        hipError_t e = launch_or_reduce(gw, tiles, nw32, tp.chunks, tp.stride32, st, done);
        if (e != hipSuccess) return e;
        done_set = done != nullptr;
    } else if (s == BuildStrategy::Atomic) {
        uint64_t g = (n + 255) / 256;
        if (g > (uint64_t)num_cus * 8) g = (uint64_t)num_cus * 8;
        k_build_atomic<Src><<<dim3((uint32_t)g), dim3(256), 0, st>>>(src, n, md, k, gw);
        if (tm) hipEventRecord(tm->t1, st);
      }
    } else if constexpr (Src::kPrehash) {
        // hashed first, into 12-B walk records (pass A then walks without
        // the reductions; partition builds have k <= 32)
        if (ws.hash_bytes < n * 12) return hipErrorInvalidValue;
        const uint64_t g = (n + 255) / 256;
        if (g > 0x7FFFFFFFull) return hipErrorInvalidValue;
        const OutRec rec{reinterpret_cast<uint32_t*>(ws.hashes), md, k};
        if constexpr (std::is_same<Src, VarLen>::value)
            launch_hash_var(src, n, rec, st);
        else
            k_hash<Src, OutRec><<<dim3((uint32_t)g), dim3(256), 0, st>>>(src, n, rec);
        // pass A's timer (t1) covers k_hash + k_bin
        return build_with(ks::Recs{reinterpret_cast<const uint32_t*>(ws.hashes)}, n, num_bits, k, gw, s, ws, num_cus,
                          st, tm, sweep, fresh, /*t0_done=*/true, done);
    } else {
        const PartitionPlan pl = plan_partition(num_bits, k, n, num_cus);
        if (pl.region_bytes > ws.region_bytes || pl.counts_bytes > ws.counts_bytes) return hipErrorInvalidValue;
        const uint32_t bfirst = sweep >= 0 ? (uint32_t)sweep * pl.bins_per_sweep : 0u;
        const uint32_t bend = sweep >= 0 ? min(pl.nbins, bfirst + pl.bins_per_sweep) : pl.nbins;
        // Fresh k = 7 builds run the LIST pass A (one key per lane per phase:
        // the two-key phases of multi-sweep plans overflow ~0.45 % of C5's
        // positions, which the lists would then OR in serially) and a pass B
        // that never reads the words; other k zero their word range first and
        // accumulate.
        const bool list = fresh && k == 7;
        if (list && (!ws.ovf || !ws.dirty || ws.ovf_units * kSliceWords32 < nw32 || !ws.ovl ||
                     ws.ovl_groups < pl.grid * pl.sweeps))
            return hipErrorInvalidValue;
        if (fresh && !list) {
            const uint64_t wlo = (uint64_t)bfirst << (pl.slice_log2 - 5);
            const uint64_t whi = min((uint64_t)nw32, (uint64_t)bend << (pl.slice_log2 - 5));
            if (whi > wlo) {
                const hipError_t e = hipMemsetAsync(gw + wlo, 0, (size_t)(whi - wlo) * 4, st);
                if (e != hipSuccess) return e;
            }
        }
        const bool w32 = fits_walk32(num_bits);
        // walks: from (h1, h2), or replayed from 12-B records
        constexpr bool kRec = std::is_same<Src, ks::Recs>::value;
        using Walk32 = std::conditional_t<kRec, RecWalk32, lsmb::Walk32>;
        using Walk64 = std::conditional_t<kRec, RecWalk64, lsmb::Walk64>;
        for (uint32_t sw = 0; sw < pl.sweeps; sw++) {
            if (sweep >= 0 && sw != (uint32_t)sweep) continue;
            PassA a;
            a.b0 = sw * pl.bins_per_sweep;
            a.nb = min(pl.bins_per_sweep, pl.nbins - a.b0);
            a.grid = pl.grid;
            a.cap = pl.cap_segs;
            a.ring = pl.ring;
            a.regions = ws.regions;
            a.counts = ws.counts;
            a.gw = gw;
            a.ovf = ws.ovf;
            a.dirty = ws.dirty;
            a.ovl = ws.ovl + (uint64_t)sw * pl.grid * kOvfListCap;  // one list per workgroup per sweep
            a.ovn = ws.ovn + (uint64_t)sw * pl.grid;
            a.ovl_cap = kOvfListCap;
            a.err = ws.err;
            a.nbins = pl.nbins;
            // (k_bin's LDS is static, kLdsBytes; the plan's layout fits it)
            if ((size_t)(a.nb + 1) * (4 * a.ring + kBinExtraBytes) + kBinJobBytes > kLdsBytes) return hipErrorInvalidValue;
            auto go = [&](auto kern) { kern<<<dim3(pl.grid), dim3(kBinBlock), 0, st>>>(src, n, md, k, a); };
            const bool full = pl.sweeps == 1;
            auto go7 = [&](auto slc) {  // k = 7 (BloomFilter::new at fpr 0.01), bin width 2^SL
                constexpr int SL = decltype(slc)::value;
                const bool two = pl.keys_per_lane == 2;
                auto pick = [&](auto wtag) {
                    using W = typename decltype(wtag)::type;
                    if (list) {
                        if (full) go(k_bin<Src, W, 7, true, true, 1, SL, true>);
                        else go(k_bin<Src, W, 7, true, false, 1, SL, true>);
                    } else {
                        if (full && two) go(k_bin<Src, W, 7, true, true, 2, SL>);
                        else if (full) go(k_bin<Src, W, 7, true, true, 1, SL>);
                        else if (two) go(k_bin<Src, W, 7, true, false, 2, SL>);
                        else go(k_bin<Src, W, 7, true, false, 1, SL>);
                    }
                };
                if (w32) {
                    pick(WalkTag<Walk32>{});
                } else if constexpr (!kRec) {
                    // the saturated u32 filter (C5): folds instead of reductions
                    if (num_bits == kMersenneBits) pick(WalkTag<WalkM>{});
                    else pick(WalkTag<Walk64>{});
                } else {
                    pick(WalkTag<Walk64>{});
                }
            };
            if (k == 7) {
                if (pl.slice_log2 == 21) go7(std::integral_constant<int, 21>{});
                else go7(std::integral_constant<int, kSliceLog2>{});
            } else if (k <= 8) {
                if (w32) go(k_bin<Src, Walk32, 8, false, false>); else go(k_bin<Src, Walk64, 8, false, false>);
            } else if (k <= 16) {
                if (w32) go(k_bin<Src, Walk32, 16, false, false>); else go(k_bin<Src, Walk64, 16, false, false>);
            } else {
                if (w32) go(k_bin<Src, Walk32, 32, false, false>); else go(k_bin<Src, Walk64, 32, false, false>);
            }
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
#if LSMB_STAMP
        {
            unsigned long long h[8];
            hipStreamSynchronize(st);
            hipMemcpyFromSymbol(h, HIP_SYMBOL(g_stamp), sizeof h);
            const double ph = (double)h[4] ? (double)h[4] : 1.0;  // wave-phases
            const double tot = (double)(h[0] + h[1] + h[2] + h[3]);
            fprintf(stderr, "[stamp] waves %llu phases/wave %.1f cycles/phase %.0f: work %.0f (%.1f%%) b1 %.0f (%.1f%%) "
                            "flush %.0f (%.1f%%) b2 %.0f (%.1f%%)\n",
                    h[5], ph / (double)h[5], tot / ph, h[0] / ph, 100 * h[0] / tot, h[1] / ph, 100 * h[1] / tot,
                    h[2] / ph, 100 * h[2] / tot, h[3] / ph, 100 * h[3] / tot);
            const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), z, sizeof z);
        }
#endif
        if (tm) hipEventRecord(tm->t1, st);
        if (bend > bfirst) {
            uint32_t* dmark = list ? ws.dirty : nullptr;
            hipEvent_t apply_done = list ? nullptr : done;  // (the last kernel completes `done`)
            hipError_t e;
            if (pl.slice_log2 == 21)
                e = launch_done(k_apply<21>, dim3(2 * (bend - bfirst)), dim3(kApplyBlock), 0u, st, apply_done, ws.regions,
                                ws.counts, pl.grid, pl.cap_segs, pl.nbins, gw, nw32, bfirst, bend, ws.ovf, dmark, list);
            else
                e = launch_done(k_apply<kSliceLog2>, dim3(bend - bfirst), dim3(kApplyBlock), 0u, st, apply_done, ws.regions,
                                ws.counts, pl.grid, pl.cap_segs, pl.nbins, gw, nw32, bfirst, bend, ws.ovf, dmark, list);
            if (e != hipSuccess) return e;
            if (list) {  // the lists of the sweeps this call ran
                const uint32_t s0 = sweep >= 0 ? (uint32_t)sweep : 0u, ns = sweep >= 0 ? 1u : pl.sweeps;
                e = launch_done(k_ovf_apply, dim3(ns * pl.grid), dim3(256), 0u, st, done,
                                (const uint32_t*)(ws.ovl + (uint64_t)s0 * pl.grid * kOvfListCap),
                                (const uint32_t*)(ws.ovn + (uint64_t)s0 * pl.grid), (uint32_t)kOvfListCap, gw);
                if (e != hipSuccess) return e;
            }
            done_set = done != nullptr;
        }
    }
    if (done && !done_set) hipEventRecord(done, st);
    if (tm) {
        hipEventRecord(tm->t2, st);
        tm->valid = true;
    }
    return hipGetLastError();
}

}  // namespace

const char* strategy_name(BuildStrategy s) {
    switch (s) {
        case BuildStrategy::None: return "none";
        case BuildStrategy::Lds: return "lds";
        case BuildStrategy::Partition: return "partition";
        case BuildStrategy::Atomic: return "atomic";
        case BuildStrategy::Tiled: return "tiled";
    }
    return "?";
}

BuildStrategy pick_build_strategy(uint32_t num_bits, uint32_t k, uint64_t n) {
    if (n == 0 || k == 0 || num_bits == 0) return BuildStrategy::None;
    const uint64_t nw32 = 2 * (((uint64_t)num_bits + 63) / 64);
    if (nw32 <= kLdsFilterMaxWords32) return BuildStrategy::Lds;
    if (k > 32) return BuildStrategy::Atomic;
    // Few keys into a big filter: scattered atomics beat a full-slice RMW.
    if (n * (uint64_t)k < nw32 / 16) return BuildStrategy::Atomic;
    // Fewer than 64 slices (< 8 MiB filters): too few LDS buffers to spread
    // a workgroup's claims; memory-side atomics on the small filter instead.
    if (nw32 <= (uint64_t)kTiledMaxSlices * kSliceWords32 && k <= 32) return BuildStrategy::Tiled;
    if (nw32 < 64ull * kSliceWords32) return BuildStrategy::Atomic;
    return BuildStrategy::Partition;
}

namespace {
PartitionPlan plan_partition_sl(uint32_t num_bits, uint32_t k, uint64_t n, int num_cus, uint32_t sl) {
    PartitionPlan pl;
    pl.slice_log2 = sl;
    pl.nbins = (uint32_t)(((uint64_t)num_bits + (1ull << sl) - 1) >> sl);
    // Entries a slice's ring receives per pass A phase (1024 keys), and the
    // ring that holds a segment's worth of leftovers plus a phase's arrivals
    // with margin.  Claims past the ring fall back to exact global atomics.
    const double lambda = (double)kBinBlock * k * fmin(1.0, (double)(1u << sl) / (double)num_bits);
    uint32_t need = kSegEntries + (uint32_t)ceil(lambda + 2.0 * sqrt(lambda));
    need = (need + 7) & ~7u;
    if (need > kMaxRing) need = kMaxRing;
    // Fewest sweeps whose slices fit LDS with that ring; each sweep re-reads
    // and re-hashes the keys and keeps only its own slices' positions.
    pl.sweeps = (pl.nbins + kMaxBinsPerSweep - 1) / kMaxBinsPerSweep;
    for (;; pl.sweeps++) {
        pl.bins_per_sweep = (pl.nbins + pl.sweeps - 1) / pl.sweeps;
        uint32_t r = (kBinLdsBudget / (pl.bins_per_sweep + 1) - kBinExtraBytes) / 4;  // + the sink slice
        r &= ~7u;
        if (r > kMaxRing) r = kMaxRing;
        if (r >= need || pl.bins_per_sweep == 1) {
            pl.ring = r;
            break;
        }
    }
    // k = 7 sweeps take two keys per lane per phase when the ring holds a
    // phase's doubled arrivals to within one 8-entry group: C5's 32-entry
    // rings (2^21-bit bins, 1024 per sweep; need2 = 40) then send ~0.45 % of
    // the positions to the exact global-atomic path, and pass A still gains
    // (C5 shard: 2.38 -> 2.33 ms).  Single-sweep filters keep one even where
    // the rings would hold two: it is slower there (4.97e8 bits, 100 M keys:
    // 0.995 -> 1.026 ms).  LSMB_SWEEP_PER=1 / =2 forces one / two
    // (measurement knob).
    if (k == 7) {
        const char* e = getenv("LSMB_SWEEP_PER");
        const uint32_t need2 = (kSegEntries + (uint32_t)ceil(2 * lambda + 2.0 * sqrt(2 * lambda)) + 7) & ~7u;
        // Not for the saturated 2^32-1-bit filter: with its fold walk (WalkM)
        // the doubled phase is slower (C5 shard, accumulate: pass A 2.074 ->
        // 2.136 ms; tools/r04_c5per.sh).
        const bool auto2 = pl.sweeps > 1 && pl.ring + 8 >= need2 && num_bits != kMersenneBits;
        if ((auto2 && !(e && atoi(e) == 1)) || (e && atoi(e) == 2)) pl.keys_per_lane = 2;
    }
    // 1024-thread workgroups (one resident per CU), at least ~kBinBlock keys
    // each: two per CU for 2^20-bit bins — pass B then streams twice as many,
    // half-size regions per slice (C2: pass B 0.448 -> 0.411 ms, pass A
    // unchanged) — one for 2^21-bit bins, whose two half-bin workgroups each
    // read every region (C5 shard: pass B 0.843 -> 0.986 ms at two).
    // LSMB_BIN_WGS_PER_CU overrides (measurement knob, tools/bin_wgs.sh).
    const uint64_t gmax = (n + kBinBlock - 1) / kBinBlock;
    static const long wenv = [] {
        const char* e = getenv("LSMB_BIN_WGS_PER_CU");
        return e ? atol(e) : 0L;
    }();
    const uint64_t wpc = wenv >= 1 && wenv <= 4 ? (uint64_t)wenv : (sl == kSliceLog2 ? 2 : 1);
    uint64_t g = (uint64_t)num_cus * wpc;
    if (g > gmax) g = gmax;
    if (g < 1) g = 1;
    pl.grid = (uint32_t)g;
    const uint64_t keys_w = (n + g - 1) / g;  // workgroup w hashes keys [w*keys_w, (w+1)*keys_w)
    double p = (double)(1u << sl) / (double)num_bits;
    if (p > 1.0) p = 1.0;
    const double mu = (double)keys_w * k * p;
    const double cap_e = mu + 8.0 * sqrt(mu) + 2.0 * kSegEntries;
    pl.cap_segs = (uint32_t)ceil(cap_e / kSegEntries);
    // A region holds at most kMaxRegionSegs segments
    // a bigger plan is reported as unbounded so callers chunk the keys.
    // (and a workgroup's regions within pass A's 2^31-byte buffer range)
    const bool fits = pl.cap_segs <= kMaxRegionSegs && (uint64_t)pl.nbins * pl.cap_segs * kSegSlotBytes < (1ull << 31);
    pl.region_bytes = fits ? (uint64_t)pl.nbins * pl.grid * pl.cap_segs * kSegSlotBytes : ~0ull >> 2;
    pl.counts_bytes = (uint64_t)pl.nbins * pl.grid * 4;
    return pl;
}
}  // namespace

// Bins of 2^20 bits (one pass B workgroup's LDS) unless the filter needs
// several sweeps: then 2^21-bit bins halve the sweeps (each re-reads and
// re-hashes every key) for a second read of each bin's regions in pass B.
// k = 7 only (the kernels instantiated for it); LSMB_SLICE_LOG2=20 pins 2^20,
// =21 forces 2^21 (measurement knobs).
PartitionPlan plan_partition(uint32_t num_bits, uint32_t k, uint64_t n, int num_cus) {
    const PartitionPlan p20 = plan_partition_sl(num_bits, k, n, num_cus, kSliceLog2);
    const char* e = getenv("LSMB_SLICE_LOG2");
    if (k == 7 && e && atoi(e) == 21 && num_bits > (1u << 21))  // measurement: force 2^21-bit bins
        return plan_partition_sl(num_bits, k, n, num_cus, 21);
    if (p20.sweeps < 2 || k != 7) return p20;
    if (e && atoi(e) == 20) return p20;
    const PartitionPlan p21 = plan_partition_sl(num_bits, k, n, num_cus, 21);
    return p21.sweeps < p20.sweeps ? p21 : p20;
}

TiledPlan plan_tiled(uint32_t num_bits, uint64_t n, int num_cus) {
    TiledPlan tp;
    const uint64_t nw32 = 2 * (((uint64_t)num_bits + 63) / 64);
    tp.nslices = (uint32_t)((nw32 + kSliceWords32 - 1) / kSliceWords32);
    // ~2 workgroups per CU in all, at least 4 Ki keys per chunk
    uint64_t ch = (2ull * (uint64_t)num_cus + tp.nslices - 1) / tp.nslices;
    const uint64_t by_keys = (n + 4095) / 4096;
    if (ch > by_keys) ch = by_keys;
    if (ch < 1) ch = 1;
    tp.chunks = (uint32_t)ch;
    tp.stride32 = (uint64_t)tp.nslices * kSliceWords32;
    tp.scratch_bytes = (uint64_t)tp.chunks * tp.stride32 * 4;
    return tp;
}

uint64_t partition_chunk_keys(uint32_t num_bits, uint32_t k, uint64_t max_bytes, int num_cus) {
    uint64_t lo = 0, hi = (1ull << 40);
    while (lo + 1 < hi) {  // largest n whose plan fits
        const uint64_t mid = lo + (hi - lo) / 2;
        const PartitionPlan pl = plan_partition(num_bits, k, mid, num_cus);
        if (pl.region_bytes + pl.counts_bytes <= max_bytes) lo = mid; else hi = mid;
    }
    return lo;
}

hipError_t launch_build(const KeyBatch& kb, uint32_t num_bits, uint32_t k, uint32_t* gw,
                        BuildStrategy s, const PartitionWorkspace& ws, int num_cus, hipStream_t st,
                        BuildTimers* tm, int sweep, bool fresh, hipEvent_t done) {
    if (s == BuildStrategy::None) {
        if (fresh && num_bits) {
            const hipError_t e = hipMemsetAsync(gw, 0, (size_t)(((uint64_t)num_bits + 63) / 64) * 8, st);  // new(), no inserts
            if (e != hipSuccess) return e;
        }
        return done ? hipEventRecord(done, st) : hipSuccess;
    }
    if (kb.offsets)
        return build_with(VarLen{kb.data, kb.offsets}, kb.n, num_bits, k, gw, s, ws, num_cus, st, tm, sweep, fresh, false, done);
    if (kb.key_len == 16 && (reinterpret_cast<uintptr_t>(kb.data) & 15) == 0)
        return build_with(Fixed16{reinterpret_cast<const uint4*>(kb.data)}, kb.n, num_bits, k, gw, s, ws,
                          num_cus, st, tm, sweep, fresh, false, done);
    return build_with(FixedN{kb.data, kb.key_len}, kb.n, num_bits, k, gw, s, ws, num_cus, st, tm, sweep, fresh, false, done);
}

hipError_t launch_or_reduce(uint32_t* dst, const uint32_t* src, uint64_t nw32, uint32_t nsrc,
                            uint64_t stride32, hipStream_t st, hipEvent_t done) {
    uint64_t g = (nw32 + 255) / 256;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    return launch_done(k_or_reduce, dim3((uint32_t)g), dim3(256), 0u, st, done, dst, src, nw32, nsrc, stride32);
}

hipError_t launch_gen_key16(uint64_t seed, uint64_t first, uint64_t n, uint8_t* d_keys, hipStream_t st) {
    uint64_t g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    k_gen_key16<<<dim3((uint32_t)g), dim3(256), 0, st>>>(seed, first, n, reinterpret_cast<uint4*>(d_keys));
    return hipGetLastError();
}

hipError_t launch_gen_splitmix(uint64_t seed, uint64_t first, uint64_t n, uint32_t mod, uint32_t add,
                               uint64_t* d_out, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t g = std::min<uint64_t>((n + 255) / 256, 8192);
    k_gen_splitmix<<<dim3((uint32_t)g), dim3(256), 0, st>>>(seed, first, n, mod, add, d_out);
    return hipGetLastError();
}

}  // namespace lsmb
