// mb_tile.hip — model of a tile-sorted pass A (a candidate, not the product):
// two 512-thread workgroups per CU (half the LDS each) instead of one
// 1024-thread workgroup with per-bin rings.  Per tile of 2048 keys:
//   1. hash + walk 4 keys per lane; one ds_add_rtn per position on its bin's
//      count returns its rank in the bin (positions and ranks stay in VGPRs);
//   2. one wave turns the 913 counts into bin bases (exclusive scan) and
//      zeroes the counts;
//   3. every position reads its bin's base and writes its 20-bit offset to
//      sorted[base + rank] (the tile, bin-sorted, in LDS);
//   4. write-out: the sorted tile leaves as coalesced 16-B stores to a per-
//      workgroup staging area (a LOWER BOUND on the real write-out, which
//      packs 3 offsets per u64 and appends each bin's run to its own region).
// Three barriers per 2048 keys (pass A: two per 1024), and two independent
// workgroups per CU whose VALU-heavy and LDS-heavy steps can overlap.  Also
// times pass A's geometry without binning (the hash + walk floor) for scale.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../storage-engine_amd/csrc mb_tile.hip -o mb_tile
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "bloom_math.hpp"
#include "keysrc.hpp"

using namespace lsmb;

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

__device__ __forceinline__ uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

__global__ void k_gen(uint4* out, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t a = sm64(0x5EED0001 + 2 * i), b = sm64(0x5EED0001 + 2 * i + 1);
        out[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    }
}

constexpr uint32_t kT = 512;         // threads per workgroup
constexpr uint32_t kKPL = 4;         // keys per lane per tile
constexpr uint32_t kTileKeys = kT * kKPL;
constexpr uint32_t kTilePos = kTileKeys * 7;
constexpr uint32_t kNB = 913;        // bins (C2: 956715292 bits / 2^20, + 1)

// STEP: 1 = hash + claims only; 2 = + scan; 3 = + scatter; 4 = + write-out
template <int STEP>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(4))) void k_tile(const uint4* keys, uint64_t n, Mod32 md, uint4* stage, uint32_t* out) {
    __shared__ uint32_t sorted[kTilePos];
    __shared__ uint32_t cnt[1024];
    __shared__ uint32_t base[1024];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (uint32_t i = tid; i < 1024; i += kT) cnt[i] = 0;
    __syncthreads();
    ks::Fixed16 src{keys};
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t i0 = blockIdx.x * per, i1 = min(n, i0 + per);
    const uint32_t tiles = (uint32_t)((i1 - i0 + kTileKeys - 1) / kTileKeys);
    uint4* st = stage + (uint64_t)blockIdx.x * (kTilePos / 4);
    uint32_t acc = 0;
    for (uint32_t t = 0; t < tiles; t++) {
        uint32_t pos[kKPL * 7], rk[kKPL * 7];
#pragma unroll
        for (uint32_t j = 0; j < kKPL; j++) {
            const uint64_t i = i0 + (uint64_t)t * kTileKeys + j * kT + tid;
            const bool ok = i < i1;
            const H128 h = src.hash(ok ? i : i0);
            Walk32 pw(md, h.lo, h.hi);
#pragma unroll
            for (uint32_t q = 0; q < 7; q++) {
                const uint32_t p = ok ? pw.pos() : (912u << 20);
                pos[j * 7 + q] = p;
                rk[j * 7 + q] = atomicAdd(&cnt[p >> 20], 1u);
                if (q < 6) pw.next(md);
            }
        }
        __syncthreads();
        if (STEP >= 2 && wave == 0) {
            // exclusive scan of 1024 counts: 16 per lane
            uint32_t c[16], s = 0;
#pragma unroll
            for (int e = 0; e < 16; e++) c[e] = cnt[lane * 16 + e], s += c[e];
            uint32_t x = s;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d);
                if (lane >= (uint32_t)d) x += y;
            }
            uint32_t b = x - s;
#pragma unroll
            for (int e = 0; e < 16; e++) base[lane * 16 + e] = b, b += c[e], cnt[lane * 16 + e] = 0;
        } else if (STEP < 2 && wave == 0) {
#pragma unroll
            for (int e = 0; e < 16; e++) cnt[lane * 16 + e] = 0;
        }
        __syncthreads();
        if (STEP >= 3) {
#pragma unroll
            for (uint32_t q = 0; q < kKPL * 7; q++) sorted[base[pos[q] >> 20] + rk[q]] = pos[q] & 0xFFFFFu;
            __syncthreads();
        } else {
#pragma unroll
            for (uint32_t q = 0; q < kKPL * 7; q++) acc += pos[q] ^ rk[q];
        }
        if (STEP >= 4) {
            const uint4* s4 = reinterpret_cast<const uint4*>(sorted);
#pragma unroll
            for (uint32_t e = tid; e < kTilePos / 4; e += kT) st[e] = s4[e];  // (one area per workgroup, rewritten)
        }
    }
    out[blockIdx.x * blockDim.x + tid] = acc;
}

// pass A's geometry, hash + walk only (1024 threads, one workgroup per CU)
__global__ __launch_bounds__(1024) void k_geom(const uint4* keys, uint64_t n, Mod32 md, uint4*, uint32_t* out) {
    __shared__ uint32_t sm[160 * 1024 / 4 - 64];
    ks::Fixed16 src{keys};
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t i0 = blockIdx.x * per, i1 = min(n, i0 + per);
    uint32_t acc = 0;
    for (uint64_t i = i0 + threadIdx.x; i < i1; i += 1024) {
        H128 h = src.hash(i);
        Walk32 pw(md, h.lo, h.hi);
#pragma unroll
        for (uint32_t j = 0; j < 7; j++) {
            acc += pw.pos();
            if (j < 6) pw.next(md);
        }
    }
    sm[threadIdx.x] = acc;
    __syncthreads();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc + sm[1023 - threadIdx.x];
}

int main(int argc, char** argv) {
    uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 100000000ull;
    uint4 *keys, *stage;
    uint32_t* out;
    CK(hipMalloc(&keys, n * 16));
    CK(hipMalloc(&out, 1024 * 1024 * 4));
    CK(hipMalloc(&stage, (size_t)1024 * kTilePos * 4));
    k_gen<<<8192, 256>>>(keys, n);
    CK(hipDeviceSynchronize());
    Mod32 md = Mod32::make(956715292u);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](auto kern, int grid, int block, const char* name) {
        for (int w = 0; w < 3; w++) kern<<<grid, block>>>(keys, n, md, stage, out);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        const int it = 20;
        for (int w = 0; w < it; w++) kern<<<grid, block>>>(keys, n, md, stage, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipGetLastError());
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= it;
        printf("%-44s %8.4f ms  %9.1f Mkeys/s\n", name, ms, n / ms / 1e3);
        fflush(stdout);
    };
    run(k_geom, 256, 1024, "pass A geometry: hash + walk (1 WG/CU)");
    run(k_geom, 512, 1024, "pass A geometry: hash + walk (512 WGs)");
    run(k_tile<1>, 512, kT, "tile: hash + claims (2 WG/CU)");
    run(k_tile<2>, 512, kT, "tile: + scan");
    run(k_tile<3>, 512, kT, "tile: + scatter");
    run(k_tile<4>, 512, kT, "tile: + write-out (lower bound)");
    run(k_tile<4>, 1024, kT, "tile: + write-out, 1024 WGs");
    return 0;
}
