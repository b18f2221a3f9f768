// kernels.hpp — launchers for the Bloom build / probe kernels (internal).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bloom_math.hpp"

namespace lsmb {

// Geometry of the partitioned build (see DESIGN.md "Build kernels").
constexpr int kSliceLog2 = 20;                        // 2^20 bits = 128 KiB LDS slice
constexpr uint32_t kSliceWords32 = 1u << (kSliceLog2 - 5);
constexpr uint32_t kSliceMask = (1u << kSliceLog2) - 1;
constexpr int kSegEntries = 24;                       // 20-bit offsets per 64-B segment
constexpr int kSegWords = 8;                          // 3 offsets per u64 word
#ifndef LSMB_SEG_STRIDE
#define LSMB_SEG_STRIDE 64  // bytes between a region's segments (measurement knob: 128 = one segment per line)
#endif
constexpr uint32_t kSegSlotBytes = LSMB_SEG_STRIDE;
constexpr uint32_t kSegSlotWords = kSegSlotBytes / 8;
constexpr int kBinBlock = 1024;                       // pass A workgroup
constexpr int kApplyBlock = 1024;                     // pass B workgroup
constexpr uint32_t kLdsFilterMaxWords32 = 40 * 1024;  // 160 KiB: whole filter in LDS
constexpr uint32_t kLdsBytes = 160 * 1024;            // LDS per CU (gfx950)
// pass A flush: segments per wave per phase posted to the cooperative stores
// (2 rounds of up to 16; C2 averages ~19).  28, not 32: the 1 KiB saved lets
// a 1e9-bit filter (954 slices, C2's exact 10 bits/key) keep 40-entry rings
// in one sweep.
constexpr uint32_t kBinJobsPerWave = 28;
constexpr uint32_t kBinJobBytes = (kBinBlock / 64) * kBinJobsPerWave * 16 + 16;  // job tables (+ alignment)
constexpr uint32_t kBinLdsBudget = kLdsBytes - kBinJobBytes;  // pass A: rings + fill words
constexpr uint32_t kBinExtraBytes = 4;                // per slice besides its ring: fill word
constexpr uint32_t kMaxBinsPerSweep = 1024;           // one owner lane per slice: <= 64 slices per wave
constexpr uint32_t kMaxRing = 1024;                   // ring entries per slice
constexpr uint32_t kMaxRegionSegs = 1u << 24;         // region capacity bound (segments)
constexpr uint32_t kOvfListCap = 16384;               // fresh builds: overflow positions listed per pass A workgroup

// How a key batch is presented to the kernels.
struct KeyBatch {
    const uint8_t* data;      // fixed: key i at data + i*key_len; var: data + offsets[i]
    const uint64_t* offsets;  // NULL for fixed-length keys
    uint32_t key_len;
    uint64_t n;
};

enum class BuildStrategy { None, Lds, Partition, Atomic, Tiled };

BuildStrategy pick_build_strategy(uint32_t num_bits, uint32_t k, uint64_t n);
const char* strategy_name(BuildStrategy s);

// Partitioned build layout for one chunk of keys.  Pass A workgroup w writes
// the 20-bit slice offsets of its keys' positions that fall in slice b into
// its private region (b, w) as 64-B segments; pass B reads every region of
// slice b.  No global atomics: each region has one writer.
struct PartitionPlan {
    uint32_t slice_log2 = kSliceLog2;  // bin width: 2^20 bits, or 2^21 where that saves sweeps
    uint32_t nbins = 0;           // ceil(num_bits / 2^slice_log2)
    uint32_t grid = 0;            // pass A workgroups = regions per slice
    uint32_t cap_segs = 0;        // region capacity, segments
    uint32_t bins_per_sweep = 0;  // slices buffered in LDS per pass A launch
    uint32_t ring = 0;            // pass A ring entries per slice (multiple of 4, >= kSegEntries)
    uint32_t sweeps = 0;
    uint32_t keys_per_lane = 1;   // pass A keys per lane per phase (2: k = 7 sweeps)
    uint64_t region_bytes = 0;    // nbins * grid * cap_segs * 64
    uint64_t counts_bytes = 0;    // nbins * grid * 4
};

PartitionPlan plan_partition(uint32_t num_bits, uint32_t k, uint64_t n, int num_cus);

// Tiled strategy (filters of 2..kTiledMaxSlices slices): workgroup (c, s)
// builds slice s from key chunk c in LDS and stores it to scratch tile
// [c][s]; k_or_reduce then ORs the chunk tiles into the filter.
constexpr uint32_t kTiledMaxSlices = 32;
struct TiledPlan {
    uint32_t nslices = 0, chunks = 0;
    uint64_t stride32 = 0;       // u32 words per chunk tile row (nslices * 2^15)
    uint64_t scratch_bytes = 0;  // chunks * stride32 * 4
};
TiledPlan plan_tiled(uint32_t num_bits, uint64_t n, int num_cus);

// Largest key count whose plan fits `max_bytes` of workspace.
uint64_t partition_chunk_keys(uint32_t num_bits, uint32_t k, uint64_t max_bytes, int num_cus);

struct PartitionWorkspace {
    uint4* hashes = nullptr;  // 16 B per key: k_hash output for var-len / odd-length keys
    uint64_t hash_bytes = 0;
    uint64_t* regions = nullptr;
    uint32_t* counts = nullptr;
    uint32_t* err = nullptr;  // device flag, see PassA::err
    // Pass A's overflow bits (ring / region overflow, adversarial inputs) and
    // per-2^20-bit-unit marks, both all-zero between builds (pass B clears
    // what it consumes): ovf_units * 2^15 u32 words, ovf_units marks.
    uint32_t* ovf = nullptr;
    uint32_t* dirty = nullptr;
    uint64_t ovf_units = 0;
    // fresh builds: per pass A workgroup, a list of kOvfListCap overflow
    // positions and its length (ovl_groups workgroups' worth)
    uint32_t* ovl = nullptr;
    uint32_t* ovn = nullptr;
    uint32_t ovl_groups = 0;
    uint64_t region_bytes = 0;
    uint64_t counts_bytes = 0;
};

struct BuildTimers {
    hipEvent_t t0, t1, t2;
    bool valid = false;
};

// Builds into d_words32 (OR-accumulate; fresh: BloomFilter::new + inserts,
// the words are output-only and every word of the build's range is written).
// For the Partition strategy the workspace must hold plan_partition(num_bits,
// k, kb.n, num_cus) and the overflow words of the whole filter.  Records
// t0/t1/t2 (start / pass A done / end) when timers != NULL.  sweep >= 0
// builds only the bits of that partition sweep's slices (sweep 0 = the whole
// build for the other strategies; see build_sweeps / sweep_words).
hipError_t launch_build(const KeyBatch& kb, uint32_t num_bits, uint32_t k, uint32_t* d_words32,
                        BuildStrategy s, const PartitionWorkspace& ws, int num_cus,
                        hipStream_t st, BuildTimers* timers, int sweep = -1, bool fresh = false,
                        hipEvent_t done = nullptr);  // done: completed by the build's last kernel (launch_done)

// Filter descriptor for the probe kernels (device-side array).
struct ProbeFilter {
    const uint32_t* words32;
    Mod32 md;
    uint32_t num_bits;
    uint32_t k;
    uint32_t out_bit;  // bit index in the output mask row
    uint32_t group;    // filters with equal (num_bits, k) share one position walk
};

// A filter of a filter set (lsmb_fset): the SSTable's filter plus its key
// range [lo, hi] (SSTable meta min_key/max_key, src/sstable/reader.rs:192).
struct RangedFilter {
    ProbeFilter f;  // f.out_bit = the slot
    const uint8_t* lo;
    const uint8_t* hi;
    uint32_t lo_len, hi_len;
};

// The key ranges of a filter set as sorted boundary points (built on the host
// per set): the distinct min/max keys of the live tables in Rust [u8] order.
// For a key, region 2r = strictly between points r-1 and r, region 2r+1 =
// equal to point r; regmask[region] = the descriptors (bit d = descriptor d)
// whose [min_key, max_key] holds every key of that region.  So the range
// pre-check of all F tables is one rank search over <= 2F points.
constexpr uint32_t kFsetMaxPoints = 128;
struct FsetPoint {
    uint64_t w0, w1;   // zero-padded 16-byte prefix as two big-endian words
    const uint8_t* p;  // the full key (device memory)
    uint32_t len, pad;
};
struct FsetRanges {
    const FsetPoint* pts;     // npts, sorted
    const uint64_t* regmask;  // 2 * npts + 1
    uint32_t npts;
};

// Size classes of a filter set: the live filters grouped by (num_bits, k),
// each class a bit-sliced LDS table (entry p = its members' bit p, `width`
// bytes), the classes together within kFsetTableBytes of LDS.  Filters of
// classes that do not fit (and k = 0 filters) are walked from L2.
constexpr uint32_t kFsetMaxClasses = 8;
constexpr uint32_t kFsetTableBytes = 64 * 1024;
struct FsetClass {
    Mod32 md;
    Mod14 md14;        // valid when num_bits < 2^14 (small): the walk's cheaper reduction
    uint32_t num_bits, k;
    uint32_t off;      // byte offset of the class table in the LDS tables
    uint32_t width;    // entry bytes: 1, 2, 4 or 8 (members <= 8, 16, 32, 64)
    uint32_t nmem, pad;
    uint64_t mask;     // the members' descriptor bits
    uint8_t mem[64];   // member j -> descriptor index
};
struct FsetClasses {
    FsetClass cls[kFsetMaxClasses];  // by value: the kernel reads them as uniform kernel arguments
    uint32_t ncls;
    uint32_t table_bytes;  // LDS bytes of all class tables
    uint64_t walk_mask;    // descriptors walked from L2
};

// out[i] bit s = (lo_s <= key i <= hi_s) && may_contain(filter s, key i), for
// the nfilt (<= 64) descriptors at d_filters (device memory).  One class
// holding every descriptor takes the bit-sliced kernel with a compile-time
// entry width; several classes the per-class tables; none the L2 walk.
// done (optional): an event the dispatch itself completes (see launch_done).
hipError_t launch_fset_probe(const KeyBatch& kb, const RangedFilter* d_filters, uint32_t nfilt, const FsetRanges& rg,
                             const FsetClasses& cl, uint32_t shared_nb, uint32_t shared_k, uint8_t* d_out_rows,
                             uint32_t row_bytes, int num_cus, hipStream_t st, hipEvent_t done = nullptr);

// A kernel launch whose completion also completes `done` (when non-null):
// hipExtLaunchKernelGGL tracks the event with the dispatch's own completion
// signal, where hipEventRecord after the launch would put a marker packet in
// the stream — ~6 us between back-to-back kernels (rocprofv3, the C3 probe).
template <typename K, typename... Args>
hipError_t launch_done(K kern, dim3 grid, dim3 block, uint32_t smem, hipStream_t st, hipEvent_t done, Args... args) {
    if (done)
        hipExtLaunchKernelGGL(kern, grid, block, smem, st, nullptr, done, 0, args...);
    else
        kern<<<grid, block, smem, st>>>(args...);
    return hipGetLastError();
}

// True when launch_probe walks these filters with k_probe_generic, the one
// probe kernel that reads the device descriptor copy (the bit-sliced kernels
// take the filters in their arguments).
bool probe_reads_descriptors(const ProbeFilter* h_filters, uint32_t nfilt);

hipError_t launch_probe(const KeyBatch& kb, const ProbeFilter* h_filters, uint32_t nfilt,
                        ProbeFilter* d_filters_scratch, uint8_t* d_out, int num_cus,
                        hipStream_t st, hipEvent_t done = nullptr);

hipError_t launch_or_reduce(uint32_t* dst, const uint32_t* src, uint64_t nwords32, uint32_t nsrc,
                            uint64_t stride32, hipStream_t st, hipEvent_t done = nullptr);

hipError_t launch_gen_splitmix(uint64_t seed, uint64_t first, uint64_t n, uint32_t mod, uint32_t add,
                               uint64_t* d_out, hipStream_t st);
hipError_t launch_gen_key16(uint64_t seed, uint64_t first, uint64_t n, uint8_t* d_keys,
                            hipStream_t st);

}  // namespace lsmb
