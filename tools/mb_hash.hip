// mb_hash.hip — micro-benchmarks of the per-key compute of the build path
// (XXH3-128 of a 16-B key + the k exact positions), no filter traffic.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../storage-engine_amd/csrc mb_hash.hip -o mb_hash
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "bloom_math.hpp"
#include "keysrc.hpp"

using namespace lsmb;

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
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

// 0: load only; 1: hash; 2: hash + 7 positions (Walk64); 3: hash + 7 positions (Walk32);
// 4: hash + 7 positions, k = 7 unrolled (Walk32, as pass A's C2 kernel walks)
template <int MODE>
__global__ __launch_bounds__(256) void k_mb(const uint4* keys, uint64_t n, Mod32 md, uint32_t k, uint32_t* out) {
    uint32_t acc = 0;
    ks::Fixed16 src{keys};
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (MODE == 0) {
            uint4 v = ld_stream16(keys + i);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        } else {
            H128 h = src.hash(i);
            if (MODE == 1) {
                acc ^= (uint32_t)(h.lo ^ h.hi ^ (h.hi >> 32));
            } else if (MODE == 4) {
                Walk32 pw(md, h.lo, h.hi);
#pragma unroll
                for (uint32_t j = 0; j < 7; j++) {
                    acc += pw.pos();
                    if (j < 6) pw.next(md);
                }
            } else if (MODE == 3) {
                Walk32 pw(md, h.lo, h.hi);
                for (uint32_t j = 0; j < k; j++) {
                    acc += pw.pos();
                    pw.next(md);
                }
            } else {
                Walk64 pw(md, h.lo, h.hi);
                for (uint32_t j = 0; j < k; j++) {
                    acc += pw.pos();
                    pw.next(md);
                }
            }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// Pass A's geometry without its binning: 1024-thread workgroups holding all
// of a CU's LDS (one resident per CU), each over a contiguous key range, k = 7
// positions per key.  CLAIM = 1 adds pass A's claims (one ds_add_rtn per
// position on one of 913 fill words) and slot writes (one ds_write_b32 into a
// 40-entry ring per bin): binning with no flush and no barriers.
template <int CLAIM>
__global__ __launch_bounds__(1024) void k_geom(const uint4* keys, uint64_t n, Mod32 md, uint32_t* out) {
    __shared__ uint32_t sm[160 * 1024 / 4 - 64];
    constexpr uint32_t NB = 913, R4 = 160;
    uint32_t* fill = sm + NB * 40;
    for (uint32_t i = threadIdx.x; i < NB; i += 1024) fill[i] = 0;
    __syncthreads();
    ks::Fixed16 src{keys};
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t i0 = blockIdx.x * per, i1 = min(n, i0 + per);
    uint32_t acc = 0;
    for (uint64_t i = i0 + threadIdx.x; i < i1; i += 1024) {
        H128 h = src.hash(i);
        Walk32 pw(md, h.lo, h.hi);
#pragma unroll
        for (uint32_t j = 0; j < 7; j++) {
            const uint32_t p = pw.pos();
            if (CLAIM) {
                const uint32_t b = p >> 20;
                const uint32_t g = atomicAdd(fill + b, 4u) & 0xFFFFu;
                const uint32_t x = g % R4;
                *(uint32_t*)((char*)sm + __umul24(b, R4) + x) = p & 0xFFFFF;
            } else {
                acc += p;
            }
            if (j < 6) pw.next(md);
        }
    }
    __syncthreads();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc + sm[threadIdx.x];
}

int main(int argc, char** argv) {
    uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 100000000ull;
    uint4* keys;
    uint32_t* out;
    CK(hipMalloc(&keys, n * 16));
    const int grid = 256 * 16, block = 256;
    CK(hipMalloc(&out, grid * block * 4));
    k_gen<<<8192, 256>>>(keys, n);
    CK(hipDeviceSynchronize());
    Mod32 md = Mod32::make(956715292u);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](auto kern, const char* name) {
        for (int w = 0; w < 3; w++) kern<<<grid, block>>>(keys, n, md, 7, out);
        hipEventRecord(a);
        const int it = 20;
        for (int w = 0; w < it; w++) kern<<<grid, block>>>(keys, n, md, 7, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= it;
        printf("%-28s %8.4f ms  %9.1f Mkeys/s  %7.1f GB/s of keys\n", name, ms, n / ms / 1e3, n * 16 / ms / 1e6);
    };
    run(k_mb<0>, "load keys only");
    run(k_mb<1>, "xxh3_128 (16 B)");
    run(k_mb<2>, "xxh3 + 7 positions (W64)");
    run(k_mb<3>, "xxh3 + 7 positions (W32)");
    run(k_mb<4>, "xxh3 + 7 pos (W32, k=7 unr.)");
    auto geom = [&](auto kern, const char* name) {
        for (int w = 0; w < 3; w++) kern<<<512, 1024>>>(keys, n, md, out);
        hipEventRecord(a);
        const int it = 20;
        for (int w = 0; w < it; w++) kern<<<512, 1024>>>(keys, n, md, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= it;
        printf("%-28s %8.4f ms  %9.1f Mkeys/s  %7.1f GB/s of keys\n", name, ms, n / ms / 1e3, n * 16 / ms / 1e6);
    };
    geom(k_geom<0>, "pass A geometry: hash+walk");
    geom(k_geom<1>, "  + claims + slot writes");
    return 0;
}
