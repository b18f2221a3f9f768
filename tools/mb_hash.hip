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

// 0: load only; 1: hash; 2: hash + 7 positions (Walk64); 3: hash + 7 positions (Walk32)
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
    return 0;
}
