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
    uint32_t ring;          // ring entries per slice (multiple of 4, >= kSegEntries)
    uint64_t* regions;      // [nbins][grid][cap][8] u64
    uint32_t* counts;       // [nbins][grid] segments written
    uint32_t* gw;           // filter words (ring / region overflow only)
    uint32_t* err;          // device counters (LSMB_STATS builds)
};

__device__ __forceinline__ uint64_t* region_ptr(const PassA& a, uint32_t b, uint32_t w) {
    return a.regions + ((uint64_t)b * a.grid + w) * a.cap * kSegWords;
}

__device__ __forceinline__ void or_pos_global(uint32_t* gw, uint32_t b, uint32_t off) {
    const uint32_t p = (b << kSliceLog2) | off;
    atomicOr(gw + (p >> 5), 1u << (p & 31));
}

// Pass A (k_bin): hash keys, bin every position's 20-bit in-slice offset by
// slice, write the bins to HBM as 64-B segments of packed offsets.
//
// One 1024-thread workgroup per CU owns a contiguous key range and walks it in
// phases of one key per lane.  LDS holds, per slice of the sweep, a ring of
// R u32 offsets plus its fill (bytes used) and the number of segments already
// written to the workgroup's region for that slice:
//   claim   one ds_add_rtn of 4 on the fill returns the entry's byte offset;
//           the offset is stored with one ds_write_b32.  A claim past the ring
//           (adversarial duplicates only; rare at the planned R) sets its bit
//           with a global atomicOr instead: pass B reads the filter words
//           after pass A, so the result is the same;
//   barrier
//   flush   wave v owns slices [v*SPW, (v+1)*SPW), one lane each.  Every full
//           24-entry segment of an owned ring becomes a job; jobs are packed
//           wave-cooperatively (4 lanes x 16 B per segment, 3 offsets per u64:
//           entry e at bits 20*(e>>3) of word e&7) and stored to the region.
//           The owner then moves the ring's remainder (< 24 entries) to the
//           front and resets the fill;
//   barrier
// The next key's load is issued two phases ahead and its hash is computed
// while this phase's claims are in flight, so VALU and LDS work overlap.
// The protocol has no waiting loops and no global atomics on the hot path.
template <class Src, class W, int KMAX, bool FULL>
__global__ __launch_bounds__(kBinBlock) void k_bin(Src src, uint64_t n, Mod32 md, uint32_t k, PassA a) {
    extern __shared__ uint32_t sm[];
    const uint32_t R = a.ring, R4 = 4 * a.ring, nb = a.nb;
    uint32_t* fill = sm + (size_t)nb * R;  // bytes used in each ring
    uint32_t* segs = fill + nb;            // segments written to each region
    const uint32_t tid = threadIdx.x, w = blockIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t* jobs = segs + nb + wave * kJobSlots;
    for (uint32_t i = tid; i < 2 * nb; i += kBinBlock) fill[i] = 0;

    // Workgroup w owns keys [w*per, (w+1)*per): a contiguous, coalesced run.
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t i0 = (uint64_t)w * per, i1 = min(n, i0 + per);
    const uint64_t iters = i1 > i0 ? (i1 - i0 + kBinBlock - 1) / kBinBlock : 0;  // uniform over the workgroup
    const uint32_t spw = (nb + 15) / 16;  // slices per wave (<= 64)
    const uint32_t own = wave * spw + lane;
    const bool owner = lane < spw && own < nb;

    // Positions of the key this lane claims in the current phase; ~0u = none.
    uint32_t pos[KMAX];
    auto positions = [&](const typename Src::Pre& pre, uint64_t i, bool ok, uint32_t (&out)[KMAX]) {
#pragma unroll
        for (int q = 0; q < KMAX; q++) out[q] = ~0u;
        if (ok) {
            const H128 h = src.hash_pre(pre, i);
            W walk(md, h.lo, h.hi);
#pragma unroll
            for (int q = 0; q < KMAX; q++) {
                if ((uint32_t)q < k) {
                    const uint32_t p = walk.pos();
                    if (FULL || (p >> kSliceLog2) - a.b0 < nb) out[q] = p;
                    walk.next(md);
                }
            }
        }
    };
    auto key_index = [&](uint64_t it) { return i0 + it * kBinBlock + tid; };
    typename Src::Pre pre0 = src.fetch(key_index(0), key_index(0) < i1);
    typename Src::Pre pre1 = src.fetch(key_index(1), iters > 1 && key_index(1) < i1);
    typename Src::Pre pre2 = src.fetch(key_index(2), iters > 2 && key_index(2) < i1);
    positions(pre0, key_index(0), iters > 0 && key_index(0) < i1, pos);
    __syncthreads();

    for (uint64_t it = 0; it < iters; it++) {
        // Claims for this phase's key, back to back.
        uint32_t got[KMAX];
#pragma unroll
        for (int q = 0; q < KMAX; q++) {
            got[q] = ~0u;
            if ((uint32_t)q < k && pos[q] != ~0u) {
                const uint32_t b = (pos[q] >> kSliceLog2) - (FULL ? 0u : a.b0);
                got[q] = atomicAdd(fill + b, 4u);
            }
        }
        // Next phase's key: hash while the claims are in flight.
        uint32_t npos[KMAX];
        {
            const uint64_t inext = key_index(it + 1);
            positions(pre1, inext, it + 1 < iters && inext < i1, npos);
            pre1 = pre2;
            pre2 = src.fetch(key_index(it + 3), it + 3 < iters && key_index(it + 3) < i1);
        }
        // Store the claimed entries.
#pragma unroll
        for (int q = 0; q < KMAX; q++) {
            if ((uint32_t)q < k && pos[q] != ~0u) {
                const uint32_t b = (pos[q] >> kSliceLog2) - (FULL ? 0u : a.b0);
                const uint32_t off = pos[q] & kSliceMask;
                if (got[q] < R4) {
                    *(uint32_t*)((char*)sm + (b * R4 + got[q])) = off;
                } else {
                    or_pos_global(a.gw, a.b0 + b, off);
#ifdef LSMB_STATS
                    atomicAdd(a.err + 9, 1u);
#endif
                }
            }
        }
#pragma unroll
        for (int q = 0; q < KMAX; q++) pos[q] = npos[q];
        __syncthreads();

        // Flush the owned slices' full segments.
        uint32_t cnt = 0, nf = 0, sg0 = 0;
        if (owner) {
            cnt = min(fill[own], R4) >> 2;
            nf = cnt / (uint32_t)kSegEntries;
            sg0 = segs[own];
        }
        for (uint32_t j = 0; __ballot(j < nf); j++) {
            const bool has = j < nf;
            const uint64_t bal = __ballot(has);
            const uint32_t total = (uint32_t)__popcll(bal);
            if (has) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                jobs[rank] = own | (j << 11) | ((sg0 + j) << 16);
            }
            for (uint32_t r = 0; r < total; r += 16) {
                const uint32_t jj = r + (lane >> 2), piece = lane & 3;
                if (jj < total) {
                    const uint32_t J = jobs[jj];
                    const uint32_t b = J & 2047u, rj = (J >> 11) & 31u, sg = J >> 16;
                    const uint32_t* e = sm + b * R + rj * kSegEntries + 2 * piece;
                    const uint2 x = *(const uint2*)e, y = *(const uint2*)(e + 8), z = *(const uint2*)(e + 16);
                    const uint64_t w0 = (uint64_t)x.x | ((uint64_t)y.x << 20) | ((uint64_t)z.x << 40);
                    const uint64_t w1 = (uint64_t)x.y | ((uint64_t)y.y << 20) | ((uint64_t)z.y << 40);
                    if (sg < a.cap) {
                        uint4* dst = reinterpret_cast<uint4*>(region_ptr(a, a.b0 + b, w) + (uint64_t)sg * kSegWords) + piece;
                        *dst = make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
                    } else {  // region full (adversarial inputs): exact global atomics
                        const uint32_t vals[6] = {x.x, y.x, z.x, x.y, y.y, z.y};
#pragma unroll
                        for (int t = 0; t < 6; t++) or_pos_global(a.gw, a.b0 + b, vals[t]);
#ifdef LSMB_STATS
                        atomicAdd(a.err + 7, 6u);
#endif
                    }
                }
            }
        }
        if (owner && nf) {
            // Remainder to the front of the ring (source starts at entry >= 24,
            // so it never overlaps the destination; reading up to 3 entries
            // past the fill is harmless).
            const uint32_t rem = cnt - nf * (uint32_t)kSegEntries;
            const uint4* s4 = reinterpret_cast<const uint4*>(sm + own * R + nf * kSegEntries);
            uint4* d4 = reinterpret_cast<uint4*>(sm + own * R);
            for (uint32_t c = 0; c < rem; c += 4) d4[c >> 2] = s4[c >> 2];
            fill[own] = rem * 4;
            segs[own] = min(sg0 + nf, a.cap);  // keeps job words' 16-bit segment field exact
        }
        __syncthreads();
    }

    // The last open segment of each owned slice (fill < 24 entries), padded
    // with copies of its first offset (setting a bit twice is a no-op), and
    // the region's segment count.
    if (owner) {
        const uint32_t cnt = fill[own] >> 2;
        uint32_t sg = segs[own];
        if (cnt) {
            const uint32_t* e = sm + own * R;
            uint32_t v[kSegEntries];
#pragma unroll
            for (int t = 0; t < kSegEntries; t++) v[t] = (uint32_t)t < cnt ? e[t] : e[0];
            if (sg < a.cap) {
                uint64_t* dst = region_ptr(a, a.b0 + own, w) + (uint64_t)sg * kSegWords;
#pragma unroll
                for (int t = 0; t < kSegWords; t++)
                    dst[t] = (uint64_t)v[t] | ((uint64_t)v[t + 8] << 20) | ((uint64_t)v[t + 16] << 40);
            } else {
                for (uint32_t t = 0; t < cnt; t++) or_pos_global(a.gw, a.b0 + own, v[t]);
            }
            sg++;
        }
        a.counts[(uint64_t)(a.b0 + own) * a.grid + w] = min(sg, a.cap);
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
            a.ring = pl.ring;
            a.regions = ws.regions;
            a.counts = ws.counts;
            a.gw = gw;
            a.err = ws.err;
            const size_t smem = (size_t)a.nb * (4 * a.ring + kBinExtraBytes) + (kBinBlock / 64) * kJobSlots * 4;
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
    // Entries a slice's ring receives per pass A phase (1024 keys), and the
    // ring that holds a segment's worth of leftovers plus a phase's arrivals
    // with margin.  Claims past the ring fall back to exact global atomics.
    const double lambda = (double)kBinBlock * k * fmin(1.0, (double)(1u << kSliceLog2) / (double)num_bits);
    uint32_t need = kSegEntries + (uint32_t)ceil(lambda + 2.0 * sqrt(lambda));
    need = (need + 3) & ~3u;
    if (need > kMaxRing) need = kMaxRing & ~3u;
    // Fewest sweeps whose slices fit LDS with that ring; each sweep re-reads
    // and re-hashes the keys and keeps only its own slices' positions.
    pl.sweeps = (pl.nbins + kMaxBinsPerSweep - 1) / kMaxBinsPerSweep;
    for (;; pl.sweeps++) {
        pl.bins_per_sweep = (pl.nbins + pl.sweeps - 1) / pl.sweeps;
        uint32_t r = (kBinLdsBudget / pl.bins_per_sweep - kBinExtraBytes) / 4;
        r &= ~3u;
        if (r > kMaxRing) r = kMaxRing & ~3u;
        if (r >= need || pl.bins_per_sweep == 1) {
            pl.ring = r;
            break;
        }
    }
    // one 1024-thread workgroup per CU, at least ~kBinBlock keys each
    const uint64_t gmax = (n + kBinBlock - 1) / kBinBlock;
    uint64_t g = (uint64_t)num_cus;
    if (g > gmax) g = gmax;
    if (g < 1) g = 1;
    pl.grid = (uint32_t)g;
    const uint64_t keys_w = (n + g - 1) / g;  // workgroup w hashes keys [w*keys_w, (w+1)*keys_w)
    double p = (double)(1u << kSliceLog2) / (double)num_bits;
    if (p > 1.0) p = 1.0;
    const double mu = (double)keys_w * k * p;
    const double cap_e = mu + 8.0 * sqrt(mu) + 2.0 * kSegEntries;
    pl.cap_segs = (uint32_t)ceil(cap_e / kSegEntries);
    // A region holds at most kMaxRegionSegs segments (pass A's job word);
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
