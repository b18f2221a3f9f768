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
    uint32_t* err;          // device error word: nonzero = a waiting loop hit LSMB_SPIN_LIMIT (a bug)
};

__device__ __forceinline__ uint64_t* region_ptr(const PassA& a, uint32_t b, uint32_t w) {
    return a.regions + ((uint64_t)b * a.grid + w) * a.cap * kSegWords;
}

// LDS accessors through address_space(3) pointers, so every access in the
// protocol is a DS instruction (a wave's DS operations execute in issue
// order); a plain generic pointer would compile to FLAT accesses.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint64_t lds_u64;
typedef __attribute__((address_space(3))) u32x4 lds_v4;

// Orders this wave's earlier LDS writes before its later LDS atomics as seen
// by other waves (s_waitcnt lgkmcnt(0)); also a compiler barrier.
__device__ __forceinline__ void lds_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); }
__device__ __forceinline__ void lds_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); }

__device__ __forceinline__ void or_pos_global(uint32_t* gw, uint32_t b, uint32_t off) {
    const uint32_t p = (b << kSliceLog2) | off;
    atomicOr(gw + (p >> 5), 1u << (p & 31));
}

// Writes one packed segment (8 words, 24 offsets) as segment `seg` of region (b, w).
__device__ __forceinline__ void write_segment(const PassA& a, const uint64_t* words, uint32_t b, uint32_t w,
                                              uint32_t seg) {
    uint64_t* dst = region_ptr(a, b, w) + (uint64_t)seg * kSegWords;
    for (int j = 0; j < kSegWords; j++) dst[j] = words[j];
}

// Pass A LDS state, per slice of the sweep (136 B):
//   half[lb][2][8]  u64  a ring of two 24-offset segments; entry e of a
//                        segment is bits [20*(e>>3), +20) of word e&7
//   state[lb]       u32  [gen1:8 | gen0:8 | claims:16]
//   done[lb]        u32  [done1:16 | done0:16]
// plus a 64-entry flush queue per wave.
// Claim c (0, 1, 2, ...) is entry c%24 of segment s = c/24, which lives in
// half s&1 and is written as segment s of the workgroup's region; gen_h counts
// the segments half h has flushed, so the half is free for s exactly when
// gen_{s&1} == s/2.  A lane claims with ONE ds_add_rtn on state, whose return
// value is an atomic snapshot of (claims, gen0, gen1):
//   - half free: OR the offset into it, then count it in done_h (the lane that
//     brings done_h to 24 queues the segment's flush);
//   - half still holding segment s-2 (rare): the lane keeps the claim in a
//     small per-lane deferred list and completes it (OR + done) in a later
//     iteration, once gen_h shows the half flushed;
//   - region full (c >= cap*24; adversarial inputs): the claim is undone (the
//     counter stays bounded) and the bit is set with a global atomic (exact:
//     pass B reads the filter words after pass A).
// Queued flushes run at the end of each key iteration, wave-cooperatively;
// meanwhile the other half takes the slice's new claims.
// Progress: an immediate claim's OR and done-count follow its claim within
// the same iteration with no waiting; a deferred claim for segment s waits
// only for segment s-2's flush, whose claims are immediate or deferred on
// s-4, and so on down to a segment with only immediate claims.  Every loop
// that waits (deferred list full, final drain) retries the wave's deferred
// claims AND flushes its queue on each pass, and exits wave-uniformly
// (ballot), so no lane ever holds back the work another lane waits for.
// cap <= kMaxRegionSegs keeps claims < 2^16 and gens < 2^8.
constexpr int kDefer = 2;       // deferred claims a lane can hold across iterations
constexpr uint32_t kQueue = 64;  // per-wave flush queue entries

struct BinLds {
    uint64_t* half;
    uint32_t* state;
    uint32_t* done;
    uint32_t* jq;  // this wave's flush queue: slice*2 + half
};

// Entry c of its slice: (word index within the slice's 16-word ring, bit shift).
__device__ __forceinline__ void entry_slot(uint32_t c, uint32_t& word, uint32_t& sh) {
    const uint32_t sg = c / (uint32_t)kSegEntries, e = c - sg * (uint32_t)kSegEntries;
    word = ((sg & 1) << 3) | (e & 7);
    sh = (e >> 3) * 20;
}

// Flushes the wave's queued segments, 16 per round: lane 4j+p copies piece p
// (16 B) of job j to the region and zeroes it; then lane j releases job j's
// half (done_h -= 24, gen_h += 1).  A store instruction costs the same
// whatever its active lanes, hence the cooperation.
__device__ __forceinline__ void flush_queue(const PassA& a, const BinLds& L, uint32_t w, uint32_t lane, uint32_t& qn) {
    for (uint32_t r = 0; r < qn; r += 16) {
        const uint32_t nj = min(16u, qn - r);
        const uint32_t j = lane >> 2, piece = lane & 3;
        if (j < nj) {
            const uint32_t JJ = *(volatile lds_u32*)(lds_u32*)(L.jq + r + j);
            const uint32_t JL = JJ >> 1, JH = JJ & 1;
            const uint32_t g = (*(volatile lds_u32*)(lds_u32*)(L.state + JL) >> (16 + 8 * JH)) & 0xFFu;
            const uint32_t sg = 2 * g + JH;  // < cap: claims past the region's capacity are undone
            volatile lds_v4* hp = (volatile lds_v4*)(lds_u64*)(L.half + JL * 16 + JH * 8 + 2 * piece);
            const u32x4 v = *hp;
            *hp = u32x4{0, 0, 0, 0};
            uint4* dst = reinterpret_cast<uint4*>(region_ptr(a, a.b0 + JL, w) + (uint64_t)sg * kSegWords) + piece;
            *dst = make_uint4(v.x, v.y, v.z, v.w);
        }
        lds_release();
        if (lane < nj) {
            const uint32_t JJ = *(volatile lds_u32*)(lds_u32*)(L.jq + r + lane);
            const uint32_t S = JJ >> 1, H = JJ & 1;
            atomicSub(L.done + S, (uint32_t)kSegEntries << (16 * H));
            lds_release();
            atomicAdd(L.state + S, 1u << (16 + 8 * H));
        }
#ifdef LSMB_STATS
        if (lane == 0) atomicAdd(a.err + 12, 1u);
#endif
    }
    qn = 0;
}

// Appends the lanes' jobs (has) to the wave's queue (flushing first if full).
__device__ __forceinline__ void queue_job(const PassA& a, const BinLds& L, uint32_t w, uint32_t lane, uint32_t& qn,
                                          bool has, uint32_t J) {
    const uint64_t bal = __ballot(has);
    if (bal == 0) return;
    const uint32_t cnt = (uint32_t)__popcll(bal);
    if (qn + cnt > kQueue) flush_queue(a, L, w, lane, qn);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    if (has) *(volatile lds_u32*)(lds_u32*)(L.jq + qn + rank) = J;
    qn += cnt;
}

// Completes the lane's deferred claims whose half has been flushed since and
// queues the flushes they trigger.
__device__ __forceinline__ void retry_deferred(const PassA& a, const BinLds& L, uint32_t w, uint32_t lane, uint32_t& qn,
                                               const uint32_t (&dkey)[kDefer], const uint32_t (&doff)[kDefer],
                                               uint32_t& dmask) {
    uint32_t ready = 0;
    if (dmask) {
#pragma unroll
        for (int d = 0; d < kDefer; d++) {
            if (dmask >> d & 1) {
                const uint32_t lb = dkey[d] >> 16, c = dkey[d] & 0xFFFFu;
                const uint32_t sg = c / (uint32_t)kSegEntries, hh = sg & 1;
                const uint32_t g = (*(volatile lds_u32*)(lds_u32*)(L.state + lb) >> (16 + 8 * hh)) & 0xFFu;
                if (g == ((sg >> 1) & 0xFFu)) {
                    uint32_t word, sh;
                    entry_slot(c, word, sh);
                    atomicOr(L.half + lb * 16 + word, (uint64_t)doff[d] << sh);
                    ready |= 1u << d;
                }
            }
        }
    }
    if (!__ballot(ready != 0)) return;
    lds_release();
    uint32_t dn[kDefer];
#pragma unroll
    for (int d = 0; d < kDefer; d++)
        if (ready >> d & 1)
            dn[d] = atomicAdd(L.done + (dkey[d] >> 16), 1u << (16 * (((dkey[d] & 0xFFFFu) / (uint32_t)kSegEntries) & 1)));
    lds_acquire();
#pragma unroll
    for (int d = 0; d < kDefer; d++) {
        const uint32_t hh = ((dkey[d] & 0xFFFFu) / (uint32_t)kSegEntries) & 1;
        const bool job = (ready >> d & 1) && ((dn[d] >> (16 * hh)) & 0xFFFFu) == (uint32_t)kSegEntries - 1;
        queue_job(a, L, w, lane, qn, job, (dkey[d] >> 16) * 2 + hh);
    }
    dmask &= ~ready;
}

// Passes a waiting loop may make before pass A reports an internal error
// (LSMB_EHIP) instead of hanging: never reached unless the protocol is broken.
#ifndef LSMB_SPIN_LIMIT
#define LSMB_SPIN_LIMIT (1u << 24)
#endif

// Pass A.  One key per lane per iteration; W = Walk32 when num_bits <= 2^31,
// else Walk64.  KMAX bounds k.  FULL: this sweep covers every slice (no
// per-position sweep check).
template <class Src, class W, int KMAX, bool FULL>
__global__ __launch_bounds__(kBinBlock) void k_bin(Src src, uint64_t n, Mod32 md, uint32_t k, PassA a) {
    extern __shared__ uint64_t smem64[];
    BinLds L;
    L.half = smem64;                                    // nb * 16
    L.state = (uint32_t*)(L.half + (size_t)a.nb * 16);  // nb
    L.done = L.state + a.nb;                            // nb
    const uint32_t tid = threadIdx.x, w = blockIdx.x, lane = tid & 63;
    L.jq = L.done + a.nb + (tid >> 6) * kQueue;
    const uint32_t climit = a.cap * (uint32_t)kSegEntries;
    {
        uint32_t* z = reinterpret_cast<uint32_t*>(smem64);
        for (uint32_t i = tid; i < a.nb * (kLdsBytesPerBin / 4); i += kBinBlock) z[i] = 0;
    }
    __syncthreads();

    uint32_t qn = 0;                                 // wave-uniform: queued flushes
    uint32_t dkey[kDefer], doff[kDefer], dmask = 0;  // deferred claims: (slice << 16 | claim), offset
    // Workgroup w owns keys [w*per, (w+1)*per): a contiguous, coalesced run.
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t i0 = (uint64_t)w * per, i1 = min(n, i0 + per);
    // The loop is uniform across the workgroup (lanes past i1 just carry no
    // positions): the cooperative flush needs every lane of the wave.
    const uint64_t iters = i1 > i0 ? (i1 - i0 + kBinBlock - 1) / kBinBlock : 0;
    for (uint64_t it = 0; it < iters; it++) {
        const uint64_t i = i0 + it * kBinBlock + tid;
        uint32_t lb[KMAX], off[KMAX], st[KMAX];
        uint32_t pend = 0;
        if (i < i1) {
            const H128 h = src.hash(i);
            W walk(md, h.lo, h.hi);
#pragma unroll
            for (int q = 0; q < KMAX; q++) {
                if ((uint32_t)q < k) {
                    const uint32_t p = walk.pos();
                    const uint32_t b = (p >> kSliceLog2) - (FULL ? 0u : a.b0);
                    lb[q] = b;
                    off[q] = p & kSliceMask;
                    if (FULL || b < a.nb) pend |= 1u << q;
                    walk.next(md);
                }
            }
        }
        // Claims, issued back to back (a result used inside its own `if`
        // makes the compiler wait for each in turn).
#pragma unroll
        for (int q = 0; q < KMAX; q++)
            if (pend >> q & 1) st[q] = atomicAdd(L.state + lb[q], 1u);
        // Immediate claims: OR the offset in.  Others: region full -> undo +
        // global atomic; half busy -> deferred.
        uint32_t cmask = 0, dnew = 0;
#pragma unroll
        for (int q = 0; q < KMAX; q++) {
            if (pend >> q & 1) {
                const uint32_t c = st[q] & 0xFFFFu, sg = c / (uint32_t)kSegEntries, hh = sg & 1;
                const uint32_t e = c - sg * (uint32_t)kSegEntries;
                const bool free_half = ((st[q] >> (16 + 8 * hh)) & 0xFFu) == ((sg >> 1) & 0xFFu);
                if (c >= climit) {
                    atomicSub(L.state + lb[q], 1u);
                    or_pos_global(a.gw, a.b0 + lb[q], off[q]);
                } else if (free_half) {
                    atomicOr(L.half + lb[q] * 16 + (hh << 3) + (e & 7), (uint64_t)off[q] << ((e >> 3) * 20));
                    cmask |= 1u << q;
                    st[q] = hh;  // from here on: the half
                } else {
                    dnew |= 1u << q;
                }
            }
        }
        lds_release();
        uint32_t dn[KMAX];
#pragma unroll
        for (int q = 0; q < KMAX; q++)
            if (cmask >> q & 1) dn[q] = atomicAdd(L.done + lb[q], 1u << (16 * st[q]));
        lds_acquire();
#ifdef LSMB_STATS
        if (dnew) atomicAdd(a.err + 9, (uint32_t)__popc(dnew));
        if (lane == 0) atomicAdd(a.err + 11, 1u);
#endif
#pragma unroll
        for (int q = 0; q < KMAX; q++) {
            if ((uint32_t)q < k) {
                const bool job = (cmask >> q & 1) && ((dn[q] >> (16 * st[q])) & 0xFFFFu) == (uint32_t)kSegEntries - 1;
                queue_job(a, L, w, lane, qn, job, lb[q] * 2 + st[q]);
            }
        }
        // Older deferred claims (their halves may have been flushed since),
        // then every queued flush.
        retry_deferred(a, L, w, lane, qn, dkey, doff, dmask);
        flush_queue(a, L, w, lane, qn);
        // New deferred claims go to free list entries; while a lane has more
        // than fit, the wave keeps completing deferred claims and flushing.
        if (__ballot(dnew != 0)) {
            for (uint32_t spin = 0;; spin++) {
#pragma unroll
                for (int q = 0; q < KMAX; q++) {
                    if (dnew >> q & 1) {
                        const int fr = __ffs(~dmask & ((1u << kDefer) - 1)) - 1;
                        if (fr >= 0) {
                            const uint32_t c = st[q] & 0xFFFFu;
#pragma unroll
                            for (int d = 0; d < kDefer; d++)
                                if (d == fr) {
                                    dkey[d] = (lb[q] << 16) | c;
                                    doff[d] = off[q];
                                }
                            dmask |= 1u << fr;
                            dnew &= ~(1u << q);
                        }
                    }
                }
                if (!__ballot(dnew != 0)) break;
                if (spin == LSMB_SPIN_LIMIT) {
                    if (lane == 0) atomicOr(a.err, 2u);
                    break;
                }
#ifdef LSMB_STATS
                if (lane == 0) atomicAdd(a.err + 10, 1u);
#endif
                retry_deferred(a, L, w, lane, qn, dkey, doff, dmask);
                flush_queue(a, L, w, lane, qn);
                if (spin) __builtin_amdgcn_s_sleep(2);
            }
        }
    }
    // Drain: complete every deferred claim.
    for (uint32_t spin = 0; __ballot(dmask != 0); spin++) {
        if (spin == LSMB_SPIN_LIMIT) {
            if (lane == 0) atomicOr(a.err, 4u);
            break;
        }
        retry_deferred(a, L, w, lane, qn, dkey, doff, dmask);
        flush_queue(a, L, w, lane, qn);
        if (spin) __builtin_amdgcn_s_sleep(2);
    }
    __syncthreads();
    // The open segment of each slice (claims % 24 entries), padded with
    // copies of its first offset (setting a bit twice is a no-op), then the
    // per-region segment counts.
    for (uint32_t lb = tid; lb < a.nb; lb += kBinBlock) {
        const uint32_t c = min(L.state[lb] & 0xFFFFu, climit);
        const uint32_t sg = c / (uint32_t)kSegEntries, r = c % (uint32_t)kSegEntries;
        if (r) {
            uint64_t words[kSegWords];
            const uint64_t* hp = L.half + lb * 16 + (sg & 1) * 8;
            for (int j = 0; j < kSegWords; j++) words[j] = hp[j];
            const uint64_t first = words[0] & kSliceMask;
            for (uint32_t e = r; e < (uint32_t)kSegEntries; e++) words[e & 7] |= first << (20 * (e >> 3));
            write_segment(a, words, a.b0 + lb, w, sg);
        }
        a.counts[(uint64_t)(a.b0 + lb) * a.grid + w] = sg + (r ? 1u : 0u);
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
            const size_t smem = (size_t)a.nb * kLdsBytesPerBin + (kBinBlock / 64) * kQueue * 4;  // + flush queues
            auto go = [&](auto kern) {
                hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
                kern<<<dim3(pl.grid), dim3(kBinBlock), smem, st>>>(src, n, md, k, a);
            };
            const bool full = pl.sweeps == 1;
            if (k <= 8) {
                if (w32) {
                    if (full) go(k_bin<Src, Walk32, 8, true>); else go(k_bin<Src, Walk32, 8, false>);
                } else {
                    if (full) go(k_bin<Src, Walk64, 8, true>); else go(k_bin<Src, Walk64, 8, false>);
                }
            } else if (k <= 16) {
                if (w32) go(k_bin<Src, Walk32, 16, false>); else go(k_bin<Src, Walk64, 16, false>);
            } else {
                if (w32) go(k_bin<Src, Walk32, 32, false>); else go(k_bin<Src, Walk64, 32, false>);
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
    // <= kMaxBinsPerSweep slices per sweep keep a pass A workgroup within its
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
    // A region holds at most kMaxRegionSegs segments (pass A's state word);
    // a bigger plan is reported as unbounded so callers chunk the keys.
    pl.region_bytes = pl.cap_segs > kMaxRegionSegs ? ~0ull >> 2 : (uint64_t)pl.nbins * pl.grid * pl.cap_segs * 64;
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
