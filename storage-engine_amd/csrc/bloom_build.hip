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
//              Pass A hashes a tile of keys, counting-sorts its k*tile
//              positions by 2^20-bit slice in LDS, reserves one run per
//              (tile, slice) with a single global atomic and writes the run
//              contiguously.  Pass B gives each slice to one workgroup, which
//              pulls the slice's words into 128 KiB of LDS, applies every
//              position with ds_or, and writes the slice back once.  No
//              random global atomics on the filter (the memory-side atomic
//              unit serves ~20 G scattered requests/s chip-wide; 7e8 of them
//              would take ~35 ms at C2).
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
// Exclusive scan of a[0..nb) in place (LDS); returns the total.  tmp holds
// one word per wave plus the total.
template <int BLOCK>
__device__ uint32_t block_scan_inplace(uint32_t* a, uint32_t nb, uint32_t* tmp) {
    constexpr int NW = BLOCK / 64;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t per = (nb + BLOCK - 1) / BLOCK;
    const uint32_t s = min(tid * per, nb), e = min(s + per, nb);
    uint32_t sum = 0;
    for (uint32_t b = s; b < e; b++) sum += a[b];
    uint32_t x = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(x, off, 64);
        if (lane >= (uint32_t)off) x += y;
    }
    if (lane == 63) tmp[wave] = x;
    __syncthreads();
    if (tid == 0) {
        uint32_t run = 0;
        for (int w = 0; w < NW; w++) {
            uint32_t t = tmp[w];
            tmp[w] = run;
            run += t;
        }
        tmp[NW] = run;
    }
    __syncthreads();
    uint32_t excl = tmp[wave] + x - sum;
    for (uint32_t b = s; b < e; b++) {
        uint32_t v = a[b];
        a[b] = excl;
        excl += v;
    }
    __syncthreads();
    return tmp[NW];
}

// Pass A: hash + bin.  KPT keys per thread per tile, at most KMAX hashes each.
template <class Src, int KMAX, int KPT>
__global__ __launch_bounds__(kBinBlock) void k_bin(Src src, uint64_t n, Mod32 md, uint32_t k,
                                                   uint32_t nbins, uint32_t cap,
                                                   uint32_t* __restrict__ bins,
                                                   uint32_t* __restrict__ cursor,
                                                   uint32_t* __restrict__ gw) {
    extern __shared__ uint32_t smem[];
    uint32_t* hist = smem;            // counts, then exclusive offsets (lbase)
    uint32_t* gbase = hist + nbins;   // global run start per slice
    uint32_t* tmp = gbase + nbins;    // scan scratch (32 words)
    uint32_t* stage = tmp + 32;       // kBinBlock*KPT*k positions, slice-sorted
    const uint32_t tid = threadIdx.x;
    constexpr uint64_t TILE = (uint64_t)kBinBlock * KPT;
    const uint64_t ntiles = (n + TILE - 1) / TILE;

    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        for (uint32_t b = tid; b < nbins; b += kBinBlock) hist[b] = 0;
        __syncthreads();
        uint32_t pos[KPT][KMAX], slot[KPT][KMAX];
        const uint64_t base = t * TILE;
#pragma unroll
        for (int j = 0; j < KPT; j++) {
            const uint64_t i = base + (uint64_t)j * kBinBlock + tid;
            if (i < n) {
                H128 h = src.hash(i);
                PosWalk pw(md, h.lo, h.hi);
#pragma unroll
                for (int q = 0; q < KMAX; q++) {
                    if ((uint32_t)q < k) {
                        pos[j][q] = pw.pos();
                        slot[j][q] = atomicAdd(&hist[pos[j][q] >> kSliceLog2], 1u);
                        pw.next(md);
                    }
                }
            }
        }
        __syncthreads();
        const uint32_t total = block_scan_inplace<kBinBlock>(hist, nbins, tmp);
        for (uint32_t b = tid; b < nbins; b += kBinBlock) {
            const uint32_t c = (b + 1 < nbins ? hist[b + 1] : total) - hist[b];
            gbase[b] = c ? atomicAdd(&cursor[b], c) : 0u;
        }
#pragma unroll
        for (int j = 0; j < KPT; j++) {
            const uint64_t i = base + (uint64_t)j * kBinBlock + tid;
            if (i < n) {
#pragma unroll
                for (int q = 0; q < KMAX; q++)
                    if ((uint32_t)q < k) stage[hist[pos[j][q] >> kSliceLog2] + slot[j][q]] = pos[j][q];
            }
        }
        __syncthreads();
        for (uint32_t e = tid; e < total; e += kBinBlock) {
            const uint32_t p = stage[e], b = p >> kSliceLog2;
            const uint32_t g = gbase[b] + (e - hist[b]);
            if (g < cap)
                bins[(uint64_t)b * cap + g] = p;
            else
                or_bit_global(gw, p);  // run overflow (e.g. duplicate-heavy input): exact, slower
        }
        __syncthreads();
    }
}

// Pass B: one 2^20-bit slice per workgroup, applied in LDS.
__global__ __launch_bounds__(kApplyBlock) void k_apply(const uint32_t* __restrict__ bins,
                                                       const uint32_t* __restrict__ cursor,
                                                       uint32_t cap, uint32_t nbins,
                                                       uint32_t* __restrict__ gw, uint64_t nw32) {
    __shared__ uint32_t filt[kSliceWords32];
    const uint32_t tid = threadIdx.x;
    for (uint32_t b = blockIdx.x; b < nbins; b += gridDim.x) {
        const uint64_t w0 = (uint64_t)b * kSliceWords32;
        const uint32_t nw = (uint32_t)min((uint64_t)kSliceWords32, nw32 - w0);  // even
        uint2* g2 = reinterpret_cast<uint2*>(gw + w0);
        uint2* f2 = reinterpret_cast<uint2*>(filt);
        for (uint32_t w = tid; w < nw / 2; w += kApplyBlock) f2[w] = g2[w];
        __syncthreads();
        const uint32_t cnt = min(cursor[b], cap);
        const uint32_t* src = bins + (uint64_t)b * cap;
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        const uint32_t n4 = cnt >> 2;
        for (uint32_t e = tid; e < n4; e += kApplyBlock) {
            const uint4 v = ld_stream16(s4 + e);
            atomicOr(&filt[(v.x >> 5) & (kSliceWords32 - 1)], 1u << (v.x & 31));
            atomicOr(&filt[(v.y >> 5) & (kSliceWords32 - 1)], 1u << (v.y & 31));
            atomicOr(&filt[(v.z >> 5) & (kSliceWords32 - 1)], 1u << (v.z & 31));
            atomicOr(&filt[(v.w >> 5) & (kSliceWords32 - 1)], 1u << (v.w & 31));
        }
        for (uint32_t e = (n4 << 2) + tid; e < cnt; e += kApplyBlock) {
            const uint32_t p = src[e];
            atomicOr(&filt[(p >> 5) & (kSliceWords32 - 1)], 1u << (p & 31));
        }
        __syncthreads();
        for (uint32_t w = tid; w < nw / 2; w += kApplyBlock) g2[w] = f2[w];
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
        uint32_t nbins, cap;
        partition_sizing(num_bits, k, n, &nbins, &cap);
        if ((uint64_t)nbins * cap > ws.entries || nbins > ws.nbins_cap) return hipErrorInvalidValue;
        hipError_t e = hipMemsetAsync(ws.cursor, 0, (size_t)nbins * 4, st);
        if (e != hipSuccess) return e;
        const void* fn;
        size_t smem;
        auto launch = [&](auto kern, int kmax, int kp) {
            smem = ((size_t)2 * nbins + 32 + (size_t)kBinBlock * kp * k) * 4;
            fn = (const void*)kern;
            (void)kmax;
            hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
            int per_cu = 0;
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBinBlock, smem);
            if (per_cu < 1) per_cu = 1;
            const uint64_t tile = (uint64_t)kBinBlock * kp;
            uint64_t g = (n + tile - 1) / tile, gmax = (uint64_t)num_cus * per_cu;
            if (g > gmax) g = gmax;
            kern<<<dim3((uint32_t)g), dim3(kBinBlock), smem, st>>>(src, n, md, k, nbins, cap, ws.bins,
                                                                ws.cursor, gw);
        };
        if (k <= 8)
            launch(k_bin<Src, 8, 4>, 8, 4);
        else if (k <= 16)
            launch(k_bin<Src, 16, 2>, 16, 2);
        else
            launch(k_bin<Src, 32, 1>, 32, 1);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        if (tm) hipEventRecord(tm->t1, st);
        k_apply<<<dim3(nbins), dim3(kApplyBlock), 0, st>>>(ws.bins, ws.cursor, cap, nbins, gw, nw32);
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
    return BuildStrategy::Partition;
}

void partition_sizing(uint32_t num_bits, uint32_t k, uint64_t n, uint32_t* nbins, uint32_t* cap) {
    const uint64_t nb = ((uint64_t)num_bits + (1ull << kSliceLog2) - 1) >> kSliceLog2;
    const double p = (double)(1ull << kSliceLog2) / (double)num_bits;
    const double mu = (double)n * k * (p > 1.0 ? 1.0 : p);
    double c = mu + 8.0 * sqrt(mu) + 64.0;
    uint64_t ci = (uint64_t)c;
    ci = (ci + 3) & ~3ull;
    if (ci > 0xFFFFFFF0ull) ci = 0xFFFFFFF0ull;
    *nbins = (uint32_t)nb;
    *cap = (uint32_t)ci;
}

uint64_t partition_chunk_keys(uint32_t num_bits, uint32_t k, uint64_t max_entries) {
    if (k == 0) return ~0ull;
    uint64_t hi = max_entries / k + 1, lo = 0;
    while (lo + 1 < hi) {  // largest n with nbins*cap <= max_entries
        uint64_t mid = lo + (hi - lo) / 2;
        uint32_t nb, cap;
        partition_sizing(num_bits, k, mid, &nb, &cap);
        if ((uint64_t)nb * cap <= max_entries) lo = mid; else hi = mid;
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
