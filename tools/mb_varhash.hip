// mb_varhash.hip — where the C4 var-len hash time goes (k_hash_var, hash_var.hpp).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../storage-engine_amd/csrc mb_varhash.hip -o mb_varhash
// Run:   ./mb_varhash [n]   (default 100 M keys; lengths 8 + sm(i) % 249, or fixed)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "hash_var.hpp"

using namespace lsmb;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

static uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

__global__ void k_fill(uint64_t* w, uint64_t nw) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * blockDim.x)
        w[i] = i * 0x9E3779B97F4A7C15ULL;
}

// per-lane global reads (k_hash<VarLen> of bloom_build.hip)
__global__ __launch_bounds__(256) void k_hash_direct(const uint8_t* d, const uint64_t* o, uint64_t n, uint4* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const H128 h = xxh3_128(d + o[i], o[i + 1] - o[i]);
    out[i] = make_uint4((uint32_t)h.lo, (uint32_t)(h.lo >> 32), (uint32_t)h.hi, (uint32_t)(h.hi >> 32));
}

template <class F>
static float timeit(F&& f, int reps = 5) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; r++) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 100000000ull;
    for (int mode = 0; mode < 4; mode++) {
        // 0: C4 lengths (8..256 uniform); 1: all 132; 2: all 64; 3: all 200
        std::vector<uint64_t> off(n + 1, 0);
        for (uint64_t i = 0; i < n; i++) {
            uint64_t len = mode == 0 ? 8 + sm64(0x5EED0003ull + i) % 249 : mode == 1 ? 132 : mode == 2 ? 64 : 200;
            off[i + 1] = off[i] + len;
        }
        const uint64_t bytes = off[n];
        uint8_t* d;
        uint64_t* o;
        uint4* out;
        CK(hipMalloc(&d, bytes + 64));
        CK(hipMalloc(&o, (n + 1) * 8));
        CK(hipMalloc(&out, n * 16));
        k_fill<<<4096, 256>>>((uint64_t*)d, bytes / 8);
        CK(hipMemcpy(o, off.data(), (n + 1) * 8, hipMemcpyHostToDevice));
        const uint32_t g = (uint32_t)((n + 255) / 256);
        const float t_stage = timeit([&] { k_hash_var<1><<<g, 256>>>(d, o, n, OutH128(out)); });
        const float t_lds = timeit([&] { k_hash_var<0><<<g, 256>>>(d, o, n, OutH128(out)); });
        const float t_dir = timeit([&] { k_hash_direct<<<g, 256>>>(d, o, n, out); });
        const uint32_t g2 = (uint32_t)((n + 127) / 128);
        const float t_128_20 = timeit([&] { k_hash_var<0, 128, 20480><<<g2, 128>>>(d, o, n, OutH128(out)); });
        const float t_128_24 = timeit([&] { k_hash_var<0, 128, 24576><<<g2, 128>>>(d, o, n, OutH128(out)); });
        const float t_256_32 = timeit([&] { k_hash_var<0, 256, 32768><<<g, 256>>>(d, o, n, OutH128(out)); });
        const uint32_t g3 = (uint32_t)((n + 63) / 64);
        const float t_64_12 = timeit([&] { k_hash_var<0, 64, 12288><<<g3, 64>>>(d, o, n, OutH128(out)); });
        const float t_nosort = timeit([&] { k_hash_var<2><<<g, 256>>>(d, o, n, OutH128(out)); });
        const float tB = timeit([&] { k_hash_var<0, 256, 36864, 4><<<g, 256>>>(d, o, n, OutH128(out)); });
        const float tC = timeit([&] { k_hash_var<0, 256, 40960, 3><<<g, 256>>>(d, o, n, OutH128(out)); });
        const uint32_t g192 = (uint32_t)((n + 191) / 192);
        const float tD = timeit([&] { k_hash_var<0, 192, 36864, 4><<<g192, 192>>>(d, o, n, OutH128(out)); });
        const float tE = timeit([&] { k_hash_var<0, 128, 18432, 4><<<g2, 128>>>(d, o, n, OutH128(out)); });
        const float tF = timeit([&] { k_hash_var<0, 256, 36864, 0><<<g, 256>>>(d, o, n, OutH128(out)); });
        printf("   no class sort %.3f | 256/36K/w4 %.3f  256/40K/w3 %.3f  192/36K/w4 %.3f  128/18K/w4 %.3f  256/36K %.3f ms\n",
               t_nosort, tB, tC, tD, tE, tF);
        // k_hash_var (LDS window) vs per-lane global reads: identical records
        std::vector<uint4> ha(n), hb(n);
        k_hash_var<0><<<g, 256>>>(d, o, n, OutH128(out));
        CK(hipMemcpy(ha.data(), out, n * 16, hipMemcpyDeviceToHost));
        k_hash_direct<<<g, 256>>>(d, o, n, out);
        CK(hipMemcpy(hb.data(), out, n * 16, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint64_t i = 0; i < n; i++)
            bad += ha[i].x != hb[i].x || ha[i].y != hb[i].y || ha[i].z != hb[i].z || ha[i].w != hb[i].w;
        printf("   window vs direct mismatches %llu\n", (unsigned long long)bad);
        CK(hipDeviceSynchronize());
        printf("mode %d (%s): %.1f B/key  stage-only %.3f ms (%.0f GB/s)  lds-hash %.3f ms  direct-hash %.3f ms"
               "  | 128/20K %.3f  128/24K %.3f  256/32K %.3f  64/12K %.3f\n", mode,
               mode == 0 ? "8-256" : mode == 1 ? "132" : mode == 2 ? "64" : "200", (double)bytes / n, t_stage,
               (bytes + 24.0 * n) / t_stage / 1e6, t_lds, t_dir, t_128_20, t_128_24, t_256_32, t_64_12);
        fflush(stdout);
        CK(hipFree(d));
        CK(hipFree(o));
        CK(hipFree(out));
    }
    return 0;
}
