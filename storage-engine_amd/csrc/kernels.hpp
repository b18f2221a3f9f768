// kernels.hpp — launchers for the Bloom build / probe kernels (internal).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bloom_math.hpp"

namespace lsmb {

// Geometry of the partitioned build (see DESIGN.md "Build kernels").
constexpr int kSliceLog2 = 20;                        // 2^20 bits = 128 KiB LDS slice
constexpr uint32_t kSliceWords32 = 1u << (kSliceLog2 - 5);
constexpr int kBinBlock = 512;                        // pass A workgroup
constexpr int kApplyBlock = 1024;                     // pass B workgroup
constexpr uint32_t kLdsFilterMaxWords32 = 40 * 1024;  // 160 KiB: whole filter in LDS

// How a key batch is presented to the kernels.
struct KeyBatch {
    const uint8_t* data;      // fixed: key i at data + i*key_len; var: data + offsets[i]
    const uint64_t* offsets;  // NULL for fixed-length keys
    uint32_t key_len;
    uint64_t n;
};

enum class BuildStrategy { None, Lds, Partition, Atomic };

BuildStrategy pick_build_strategy(uint32_t num_bits, uint32_t k, uint64_t n);
const char* strategy_name(BuildStrategy s);

struct PartitionWorkspace {
    uint32_t* bins = nullptr;    // nbins * cap entries
    uint32_t* cursor = nullptr;  // nbins counters
    uint64_t entries = 0;        // capacity of `bins` in entries
    uint32_t nbins_cap = 0;      // capacity of `cursor`
};

// Workspace the partitioned build needs for `n` keys (entries, counters).
void partition_sizing(uint32_t num_bits, uint32_t k, uint64_t n, uint32_t* nbins, uint32_t* cap);

// Largest key count a workspace of `entries` entries can take in one chunk.
uint64_t partition_chunk_keys(uint32_t num_bits, uint32_t k, uint64_t max_entries);

struct BuildTimers {
    hipEvent_t t0, t1, t2;
    bool valid = false;
};

// Builds into d_words32 (OR-accumulate).  `ws` must be sized by the caller for
// the Partition strategy (partition_sizing).  Records t0/t1/t2 when timers != NULL.
hipError_t launch_build(const KeyBatch& kb, uint32_t num_bits, uint32_t k, uint32_t* d_words32,
                        BuildStrategy s, const PartitionWorkspace& ws, int num_cus,
                        hipStream_t st, BuildTimers* timers);

// Filter descriptor for the probe kernels (device-side array).
struct ProbeFilter {
    const uint32_t* words32;
    Mod32 md;
    uint32_t num_bits;
    uint32_t k;
    uint32_t out_bit;  // bit index in the output mask row
    uint32_t group;    // filters with equal (num_bits, k) share one position walk
};

hipError_t launch_probe(const KeyBatch& kb, const ProbeFilter* h_filters, uint32_t nfilt,
                        ProbeFilter* d_filters_scratch, uint8_t* d_out, int num_cus,
                        hipStream_t st);

hipError_t launch_or_reduce(uint32_t* dst, const uint32_t* src, uint64_t nwords32, uint32_t nsrc,
                            uint64_t stride32, hipStream_t st);

hipError_t launch_gen_key16(uint64_t seed, uint64_t first, uint64_t n, uint8_t* d_keys,
                            hipStream_t st);

}  // namespace lsmb
