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
#include "kernels.hpp"
#include "keysrc.hpp"

namespace lsmb {
namespace {

using ks::Fixed16;
using ks::FixedN;
using ks::VarLen;

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
    uint32_t grid, cap;     // regions per slice, region capacity (segments)
    uint64_t* regions;      // [nbins][grid][cap][8] u64
    uint32_t* counts;       // [nbins][grid] segments written
    uint32_t* gw;           // filter words (overflow fallback only)
    uint32_t* err;          // set to 1 if a bounded wait ever times out (a bug; never expected)
};

// Every wait in pass A is bounded: a protocol bug must surface as an error
// (LSMB_EHIP at the next sync), never as a hung GPU.
#ifndef LSMB_SPIN_LIMIT
#define LSMB_SPIN_LIMIT (1u << 22)
#endif
constexpr uint32_t kSpinLimit = LSMB_SPIN_LIMIT;

// Exponential backoff for every wait in pass A: pollers must not crowd the
// LDS that the lanes they wait for need (64 * 2^j clocks, j <= 5).
__device__ __forceinline__ void backoff(uint32_t spin) {
    switch (spin < 5 ? spin : 5) {
        case 0: __builtin_amdgcn_s_sleep(1); break;
        case 1: __builtin_amdgcn_s_sleep(2); break;
        case 2: __builtin_amdgcn_s_sleep(4); break;
        case 3: __builtin_amdgcn_s_sleep(8); break;
        case 4: __builtin_amdgcn_s_sleep(16); break;
        default: __builtin_amdgcn_s_sleep(32); break;
    }
}

__device__ __forceinline__ uint64_t* region_ptr(const PassA& a, uint32_t b, uint32_t w) {
    return a.regions + ((uint64_t)b * a.grid + w) * a.cap * kSegWords;
}

// LDS accessors through address_space(3) pointers, so every access in the
// protocol is a DS instruction (a wave's DS operations execute in issue
// order); a plain generic pointer would compile to FLAT accesses, which are
// slower and complete out of order.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_v4;

__device__ __forceinline__ lds_u32* to_lds(uint32_t* p) { return (lds_u32*)p; }
__device__ __forceinline__ uint32_t lds_load_volatile(const uint32_t* p) { return *(volatile lds_u32*)(lds_u32*)(p); }
__device__ __forceinline__ void lds_store_volatile(uint32_t* p, uint32_t v) { *(volatile lds_u32*)to_lds(p) = v; }

// Packs 24 offsets into 8 words (3 x 20 bits each) and writes them as
// segment `seg` of region (b, w); past the region's capacity (adversarial
// inputs, e.g. one key repeated millions of times) the offsets go straight
// into the filter with global atomics instead: exact.  `slot(e)` returns
// offset e.
template <class SlotFn>
__device__ __forceinline__ void write_segment(const PassA& a, SlotFn slot, uint32_t b, uint32_t w, uint32_t seg) {
    if (seg < a.cap) {
        uint4* dst = reinterpret_cast<uint4*>(region_ptr(a, b, w) + (uint64_t)seg * kSegWords);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint64_t w0 = (uint64_t)(slot(6 * j) & kSliceMask) | ((uint64_t)(slot(6 * j + 1) & kSliceMask) << 20) |
                                ((uint64_t)(slot(6 * j + 2) & kSliceMask) << 40);
            const uint64_t w1 = (uint64_t)(slot(6 * j + 3) & kSliceMask) |
                                ((uint64_t)(slot(6 * j + 4) & kSliceMask) << 20) |
                                ((uint64_t)(slot(6 * j + 5) & kSliceMask) << 40);
            dst[j] = make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
        }
    } else {
        for (int e = 0; e < kSegEntries; e++) {
            const uint32_t p = (b << kSliceLog2) | (slot(e) & kSliceMask);
            atomicOr(a.gw + (p >> 5), 1u << (p & 31));
        }
    }
}

// LDS state of pass A, per slice of the sweep:
//   slots[lb][24]  u32 20-bit offsets of the open segment
//   claims[lb]     slots handed out (>= 24: segment full, claim void)
//   done[lb]       slots written
//   cur[lb]        segments this workgroup has written for the slice
// A lane claims a slot (ds_add_rtn on claims), writes its offset (ds_write),
// then counts itself in done (ds_add_rtn).  A wave's DS operations execute in
// issue order, so the lane whose done-increment returns 23 knows all 24
// offsets are in place: it flushes the segment and re-opens the buffer
// (done = 0, then claims = 0).  The claim -> write -> done sequence of every
// valid claim never waits on anything, so re-opens always happen; the only
// waiting lanes are void claims (buffer full) polling for the re-open.  That
// matters under SIMT lockstep: a wave's lanes cannot pass a divergent spin
// loop until all of them can, so no lane may spin on work another lane could
// be holding back.  Every wait is bounded (err flag) and backs off.
__device__ __forceinline__ void flush_segment(const PassA& a, uint32_t* slots, uint32_t* claims, uint32_t* done,
                                              uint32_t* cur, uint32_t lb, uint32_t w) {
    const volatile lds_v4* sl4 = (const volatile lds_v4*)to_lds(slots + lb * kSegEntries);  // 16-B aligned
    uint32_t v[kSegEntries];
#pragma unroll
    for (int j = 0; j < kSegEntries / 4; j++) {
        const u32x4 x = sl4[j];
        v[4 * j] = x.x;
        v[4 * j + 1] = x.y;
        v[4 * j + 2] = x.z;
        v[4 * j + 3] = x.w;
    }
    const uint32_t c = lds_load_volatile(cur + lb);
    write_segment(a, [&](int e) { return v[e]; }, a.b0 + lb, w, c);
    lds_store_volatile(cur + lb, c + 1);
    lds_store_volatile(done + lb, 0);
    lds_store_volatile(claims + lb, 0);
}

// Pass A.  One key per lane per iteration; W = Walk32 when num_bits <= 2^31,
// else Walk64.  KMAX bounds k: a key's k claims, writes and done-counts are
// each issued back to back.
template <class Src, class W, int KMAX>
__global__ __launch_bounds__(kBinBlock) void k_bin(Src src, uint64_t n, Mod32 md, uint32_t k, PassA a) {
    extern __shared__ uint32_t smem32[];
    uint32_t* slots = smem32;                               // nb * 24
    uint32_t* claims = slots + (size_t)a.nb * kSegEntries;  // nb
    uint32_t* done = claims + a.nb;                         // nb
    uint32_t* cur = done + a.nb;                            // nb
    uint32_t* jobs = cur + a.nb;                            // 16 per wave: cooperative flush queue
    const uint32_t tid = threadIdx.x, w = blockIdx.x, lane = tid & 63;
    uint32_t* myjobs = jobs + (tid >> 6) * 16;
    for (uint32_t i = tid; i < a.nb * (kSegEntries + 3); i += kBinBlock) smem32[i] = 0;
    __syncthreads();

    // Workgroup w owns keys [w*per, (w+1)*per): a contiguous, coalesced run.
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t i0 = (uint64_t)w * per, i1 = min(n, i0 + per);
    // The loop is uniform across the workgroup (lanes past i1 just carry no
    // positions): the cooperative flush below needs every lane of the wave.
    const uint64_t iters = i1 > i0 ? (i1 - i0 + kBinBlock - 1) / kBinBlock : 0;
    for (uint64_t it = 0; it < iters; it++) {
        const uint64_t i = i0 + it * kBinBlock + tid;
        uint32_t lb[KMAX], off[KMAX], slot[KMAX], dn[KMAX];
#pragma unroll
        for (int q = 0; q < KMAX; q++) lb[q] = 0xFFFFFFFFu;
        if (i < i1) {
            const H128 h = src.hash(i);
            W walk(md, h.lo, h.hi);
#pragma unroll
            for (int q = 0; q < KMAX; q++) {
                if ((uint32_t)q < k) {
                    const uint32_t p = walk.pos();
                    const uint32_t b = (p >> kSliceLog2) - a.b0;
                    if (b < a.nb) {
                        lb[q] = b;
                        off[q] = p & kSliceMask;
                    }
                    walk.next(md);
                }
            }
        }
#pragma unroll
        for (int q = 0; q < KMAX; q++)
            if (lb[q] != 0xFFFFFFFFu) slot[q] = atomicAdd(&claims[lb[q]], 1u);
#pragma unroll
        for (int q = 0; q < KMAX; q++)
            if (lb[q] != 0xFFFFFFFFu && slot[q] < (uint32_t)kSegEntries)
                lds_store_volatile(slots + lb[q] * kSegEntries + slot[q], off[q]);
#pragma unroll
        for (int q = 0; q < KMAX; q++)
            if (lb[q] != 0xFFFFFFFFu && slot[q] < (uint32_t)kSegEntries) dn[q] = atomicAdd(&done[lb[q]], 1u);
        // flushes (wait-free), then retries of void claims: one code path
        // each, the operands picked out of the unrolled arrays with selects
        uint32_t fmask = 0, rmask = 0;
#pragma unroll
        for (int q = 0; q < KMAX; q++) {
            if (lb[q] != 0xFFFFFFFFu) {
                if (slot[q] < (uint32_t)kSegEntries)
                    fmask |= (uint32_t)(dn[q] == (uint32_t)kSegEntries - 1) << q;
                else
                    rmask |= 1u << q;
            }
        }
        // Wave-cooperative flushes: a store instruction costs the same
        // whatever its active lanes, so completed segments are written 16 at
        // a time, 4 lanes x 16 B each, instead of 4 stores by each owner.
        // Each round the wave's owners (lanes with a completed segment) post
        // their slice in this wave's LDS job list; lane 4j+p packs piece p of
        // job j (offsets 6p..6p+5) and stores it; then the owners re-open
        // their buffers.  All in program order within one wave: no waiting.
        while (true) {
            const bool have = fmask != 0;
            uint32_t L = 0;
            if (have) {
                const int qs = __ffs(fmask) - 1;
#pragma unroll
                for (int q = 0; q < KMAX; q++)
                    if (q == qs) L = lb[q];
            }
            const uint64_t bal = __ballot(have);
            if (bal == 0) break;
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            const bool served = have && rank < 16;
            if (served) lds_store_volatile(myjobs + rank, L);
            const uint32_t njobs = min(16u, (uint32_t)__popcll(bal));
            const uint32_t j = lane >> 2, piece = lane & 3;
            if (j < njobs) {
                const uint32_t JL = lds_load_volatile(myjobs + j);
                const uint32_t c = lds_load_volatile(cur + JL);
                const uint32_t* sl = slots + JL * kSegEntries + 6 * piece;
                uint32_t e[6];
#pragma unroll
                for (int t = 0; t < 6; t++) e[t] = lds_load_volatile(sl + t);
                const uint32_t b = a.b0 + JL;
                if (c < a.cap) {
                    uint4* dst = reinterpret_cast<uint4*>(region_ptr(a, b, w) + (uint64_t)c * kSegWords) + piece;
                    *dst = make_uint4(e[0] | (e[1] << 20), (e[1] >> 12) | (e[2] << 8), e[3] | (e[4] << 20),
                                      (e[4] >> 12) | (e[5] << 8));
                } else {
#pragma unroll
                    for (int t = 0; t < 6; t++) {
                        const uint32_t p = (b << kSliceLog2) | e[t];
                        atomicOr(a.gw + (p >> 5), 1u << (p & 31));
                    }
                }
            }
            if (served) {
                const uint32_t c = lds_load_volatile(cur + L);
                lds_store_volatile(cur + L, c + 1);
                lds_store_volatile(done + L, 0);
                lds_store_volatile(claims + L, 0);
                fmask &= fmask - 1;
            }
        }
        // Retry loop with a WAVE-UNIFORM exit (ballot): every lane's claim,
        // write, done-count and flush happen inside the iteration that makes
        // them.  (With a per-lane `break`, the compiler moves the success
        // path to the loop exit, which a lane only reaches once all its
        // wave-mates are done: a wave-mate waiting on that very segment then
        // never sees it complete.)
        uint32_t idle = 0;
#ifdef LSMB_STATS
        if (rmask) atomicAdd(a.err + 9, (uint32_t)__popc(rmask));          // void claims
        if (__ballot(rmask != 0) && lane == 0) atomicAdd(a.err + 10, 1u);  // wave-iterations that retry
        if (lane == 0) atomicAdd(a.err + 11, 1u);                          // wave-iterations
#endif
        for (uint32_t spin = 0; __ballot(rmask != 0); spin++) {
#ifdef LSMB_STATS
            if (lane == 0) atomicAdd(a.err + 12, 1u);  // retry-loop iterations
#endif
            if (rmask) {
                const int qs = __ffs(rmask) - 1;
                uint32_t L = 0, O = 0;
#pragma unroll
                for (int q = 0; q < KMAX; q++)
                    if (q == qs) {
                        L = lb[q];
                        O = off[q];
                    }
                if (lds_load_volatile(claims + L) < (uint32_t)kSegEntries) {  // poll before claiming
                    const uint32_t s1 = atomicAdd(&claims[L], 1u);
                    if (s1 < (uint32_t)kSegEntries) {
                        lds_store_volatile(slots + L * kSegEntries + s1, O);
                        if (atomicAdd(&done[L], 1u) == (uint32_t)kSegEntries - 1)
                            flush_segment(a, slots, claims, done, cur, L, w);
                        rmask &= rmask - 1;
                    }
                }
            }
            if (spin == kSpinLimit) {
                if (rmask && atomicOr(a.err, 2u) == 0u) {  // first timeout: dump the stuck slice
                    const int qs = __ffs(rmask) - 1;
                    uint32_t L = 0;
#pragma unroll
                    for (int q = 0; q < KMAX; q++)
                        if (q == qs) L = lb[q];
                    a.err[1] = lds_load_volatile(claims + L);
                    a.err[2] = lds_load_volatile(done + L);
                    a.err[3] = lds_load_volatile(cur + L);
                    a.err[4] = L;
                }
                break;
            }
            backoff(idle++);
        }
    }
    __syncthreads();
    // Final partial segments, padded with copies of their first offset
    // (setting a bit twice is a no-op), then the per-region segment counts.
    for (uint32_t lb = tid; lb < a.nb; lb += kBinBlock) {
        const uint32_t f = claims[lb];
        uint32_t c = cur[lb];
        if (f) {
            const uint32_t* sl = slots + lb * kSegEntries;
            write_segment(a, [&](int e) { return (uint32_t)e < f ? sl[e] : sl[0]; }, a.b0 + lb, w, c);
            c++;
        }
        a.counts[(uint64_t)(a.b0 + lb) * a.grid + w] = min(c, a.cap);
    }
}

// Pass B: one 2^20-bit slice per workgroup, applied in LDS.
__global__ __launch_bounds__(kApplyBlock) void k_apply(const uint64_t* __restrict__ regions,
                                                       const uint32_t* __restrict__ counts,
                                                       uint32_t grid, uint32_t cap, uint32_t nbins,
                                                       uint32_t* __restrict__ gw, uint64_t nw32) {
    __shared__ uint32_t filt[kSliceWords32];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr uint32_t NWAVE = kApplyBlock / 64;
    for (uint32_t b = blockIdx.x; b < nbins; b += gridDim.x) {
        const uint64_t w0 = (uint64_t)b * kSliceWords32;
        const uint32_t nw = (uint32_t)min((uint64_t)kSliceWords32, nw32 - w0);  // even
        uint2* g2 = reinterpret_cast<uint2*>(gw + w0);
        uint2* f2 = reinterpret_cast<uint2*>(filt);
        for (uint32_t i = tid; i < nw / 2; i += kApplyBlock) f2[i] = g2[i];
        __syncthreads();
        for (uint32_t r = wave; r < grid; r += NWAVE) {
            const uint32_t nseg = counts[(uint64_t)b * grid + r];
            const uint4* src = reinterpret_cast<const uint4*>(regions + ((uint64_t)b * grid + r) * cap * kSegWords);
            const uint32_t n16 = nseg * (kSegWords / 2);  // 16-B pieces (2 words, 6 offsets)
            constexpr uint32_t U = 4;                      // loads in flight per lane
            for (uint32_t i0 = 0; i0 < n16; i0 += 64 * U) {
                uint4 v[U];
#pragma unroll
                for (uint32_t u = 0; u < U; u++) {
                    const uint32_t i = i0 + u * 64 + lane;
                    v[u] = i < n16 ? ld_stream16(src + i) : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (uint32_t u = 0; u < U; u++) {
                    if (i0 + u * 64 + lane < n16) {
                        const uint64_t lo = ((uint64_t)v[u].y << 32) | v[u].x;
                        const uint64_t hi = ((uint64_t)v[u].w << 32) | v[u].z;
#pragma unroll
                        for (int e = 0; e < 3; e++) {
                            const uint32_t o0 = (uint32_t)(lo >> (20 * e)) & kSliceMask;
                            const uint32_t o1 = (uint32_t)(hi >> (20 * e)) & kSliceMask;
                            atomicOr(&filt[o0 >> 5], 1u << (o0 & 31));
                            atomicOr(&filt[o1 >> 5], 1u << (o1 & 31));
                        }
                    }
                }
            }
        }
        __syncthreads();
        for (uint32_t i = tid; i < nw / 2; i += kApplyBlock) g2[i] = f2[i];
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

template <class Src>
hipError_t build_with(const Src& src, uint64_t n, uint32_t num_bits, uint32_t k, uint32_t* gw,
                      BuildStrategy s, const PartitionWorkspace& ws, int num_cus, hipStream_t st,
                      BuildTimers* tm) {
    const Mod32 md = Mod32::make(num_bits);
    const uint32_t nw32 = (uint32_t)(2 * (((uint64_t)num_bits + 63) / 64));
    if (tm) hipEventRecord(tm->t0, st);
    if (s == BuildStrategy::Lds) {
        const size_t smem = (size_t)nw32 * 4;
        // ~8 Ki keys per workgroup keeps the final per-word OR cheap.
        uint64_t g = (n + 8191) / 8192;
        const uint64_t gmax = (uint64_t)num_cus * (smem <= 40 * 1024 ? 4 : 1);
        if (g > gmax) g = gmax;
        if (g < 1) g = 1;
        hipFuncSetAttribute((const void*)k_build_lds<Src>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)smem);
        k_build_lds<Src><<<dim3((uint32_t)g), dim3(1024), smem, st>>>(src, n, md, k, nw32, gw);
        if (tm) hipEventRecord(tm->t1, st);
    } else if (s == BuildStrategy::Atomic) {
        uint64_t g = (n + 255) / 256;
        if (g > (uint64_t)num_cus * 8) g = (uint64_t)num_cus * 8;
        k_build_atomic<Src><<<dim3((uint32_t)g), dim3(256), 0, st>>>(src, n, md, k, gw);
        if (tm) hipEventRecord(tm->t1, st);
    } else {
        const PartitionPlan pl = plan_partition(num_bits, k, n, num_cus);
        if (pl.region_bytes > ws.region_bytes || pl.counts_bytes > ws.counts_bytes) return hipErrorInvalidValue;
        const bool w32 = fits_walk32(num_bits);
        for (uint32_t sw = 0; sw < pl.sweeps; sw++) {
            PassA a;
            a.b0 = sw * pl.bins_per_sweep;
            a.nb = min(pl.bins_per_sweep, pl.nbins - a.b0);
            a.grid = pl.grid;
            a.cap = pl.cap_segs;
            a.regions = ws.regions;
            a.counts = ws.counts;
            a.gw = gw;
            a.err = ws.err;
            const size_t smem = (size_t)a.nb * kLdsBytesPerBin + (kBinBlock / 64) * 16 * 4;
            auto go = [&](auto kern) {
                hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
                kern<<<dim3(pl.grid), dim3(kBinBlock), smem, st>>>(src, n, md, k, a);
            };
            if (k <= 8) {
                if (w32) go(k_bin<Src, Walk32, 8>); else go(k_bin<Src, Walk64, 8>);
            } else if (k <= 16) {
                if (w32) go(k_bin<Src, Walk32, 16>); else go(k_bin<Src, Walk64, 16>);
            } else {
                if (w32) go(k_bin<Src, Walk32, 32>); else go(k_bin<Src, Walk64, 32>);
            }
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        if (tm) hipEventRecord(tm->t1, st);
        k_apply<<<dim3(pl.nbins), dim3(kApplyBlock), 0, st>>>(ws.regions, ws.counts, pl.grid, pl.cap_segs,
                                                              pl.nbins, gw, nw32);
    }
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
    if (nw32 < 64ull * kSliceWords32) return BuildStrategy::Atomic;
    return BuildStrategy::Partition;
}

PartitionPlan plan_partition(uint32_t num_bits, uint32_t k, uint64_t n, int num_cus) {
    PartitionPlan pl;
    pl.nbins = (uint32_t)(((uint64_t)num_bits + kSliceMask) >> kSliceLog2);
    // <= 1536 slices per sweep keeps a pass A workgroup within 150 KiB of
    // LDS (one 1024-thread workgroup per CU); bigger filters take more sweeps
    // (each re-reads and re-hashes the keys, and keeps only its slices).
    pl.sweeps = (pl.nbins + kMaxBinsPerSweep - 1) / kMaxBinsPerSweep;
    pl.bins_per_sweep = (pl.nbins + pl.sweeps - 1) / pl.sweeps;
    const uint32_t per_cu = pl.bins_per_sweep * kLdsBytesPerBin <= 80 * 1024 ? 2 : 1;
    // at least ~kBinBlock keys per workgroup
    const uint64_t gmax = (n + kBinBlock - 1) / kBinBlock;
    uint64_t g = (uint64_t)num_cus * per_cu;
    if (g > gmax) g = gmax;
    if (g < 1) g = 1;
    pl.grid = (uint32_t)g;
    const uint64_t keys_w = (n + g - 1) / g;  // workgroup w hashes keys [w*keys_w, (w+1)*keys_w)
    double p = (double)(1u << kSliceLog2) / (double)num_bits;
    if (p > 1.0) p = 1.0;
    const double mu = (double)keys_w * k * p;
    const double cap_e = mu + 8.0 * sqrt(mu) + 2.0 * kSegEntries;
    pl.cap_segs = (uint32_t)ceil(cap_e / kSegEntries);
    pl.region_bytes = (uint64_t)pl.nbins * pl.grid * pl.cap_segs * 64;
    pl.counts_bytes = (uint64_t)pl.nbins * pl.grid * 4;
    return pl;
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
                        BuildTimers* tm) {
    if (s == BuildStrategy::None) return hipSuccess;
    if (kb.offsets) return build_with(VarLen{kb.data, kb.offsets}, kb.n, num_bits, k, gw, s, ws, num_cus, st, tm);
    if (kb.key_len == 16 && (reinterpret_cast<uintptr_t>(kb.data) & 15) == 0)
        return build_with(Fixed16{reinterpret_cast<const uint4*>(kb.data)}, kb.n, num_bits, k, gw, s, ws,
                          num_cus, st, tm);
    return build_with(FixedN{kb.data, kb.key_len}, kb.n, num_bits, k, gw, s, ws, num_cus, st, tm);
}

hipError_t launch_or_reduce(uint32_t* dst, const uint32_t* src, uint64_t nw32, uint32_t nsrc,
                            uint64_t stride32, hipStream_t st) {
    uint64_t g = (nw32 + 255) / 256;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    k_or_reduce<<<dim3((uint32_t)g), dim3(256), 0, st>>>(dst, src, nw32, nsrc, stride32);
    return hipGetLastError();
}

hipError_t launch_gen_key16(uint64_t seed, uint64_t first, uint64_t n, uint8_t* d_keys, hipStream_t st) {
    uint64_t g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    k_gen_key16<<<dim3((uint32_t)g), dim3(256), 0, st>>>(seed, first, n, reinterpret_cast<uint4*>(d_keys));
    return hipGetLastError();
}

}  // namespace lsmb
