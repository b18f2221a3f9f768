// mb_bin.hip — staged cost of the pass-A loop (C2 geometry: 100M keys, 913 slices, k=7).
// STAGE 0: hash+walk; 1: +claims (ds_add_rtn); 2: +slot writes +done adds;
//       3: +flush reads/pack (no global stores); 4: +global segment stores.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../storage-engine_amd/csrc mb_bin.hip -o mb_bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "bloom_math.hpp"
#include "keysrc.hpp"

using namespace lsmb;

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

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_v4;
__device__ __forceinline__ void st(uint32_t* p, uint32_t v) { *(volatile lds_u32*)(lds_u32*)p = v; }

template <int STAGE, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k(const uint4* keys, uint64_t n, Mod32 md, uint32_t nb, uint4* out,
                                           uint32_t* sink) {
    extern __shared__ uint32_t sm[];
    uint32_t* slots = sm;
    uint32_t* claims = slots + nb * 24;
    uint32_t* done = claims + nb;
    for (uint32_t i = threadIdx.x; i < nb * 26; i += BLOCK) sm[i] = 0;
    __syncthreads();
    ks::Fixed16 src{keys};
    uint32_t acc = 0;
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t i0 = (uint64_t)blockIdx.x * per, i1 = min(n, i0 + per);
    for (uint64_t i = i0 + threadIdx.x; i < i1; i += BLOCK) {
        const H128 h = src.hash(i);
        Walk32 w(md, h.lo, h.hi);
        uint32_t lb[7], off[7], slot[7], dn[7];
#pragma unroll
        for (int q = 0; q < 7; q++) {
            const uint32_t p = w.pos();
            lb[q] = p >> 20;
            off[q] = p & 0xFFFFF;
            w.next(md);
        }
        if (STAGE == 0) {
#pragma unroll
            for (int q = 0; q < 7; q++) acc += lb[q] ^ off[q];
            continue;
        }
#pragma unroll
        for (int q = 0; q < 7; q++) slot[q] = atomicAdd(&claims[lb[q]], 1u) % 24;
        if (STAGE == 1) {
#pragma unroll
            for (int q = 0; q < 7; q++) acc += slot[q];
            continue;
        }
#pragma unroll
        for (int q = 0; q < 7; q++) st(slots + lb[q] * 24 + slot[q], off[q]);
#pragma unroll
        for (int q = 0; q < 7; q++) dn[q] = atomicAdd(&done[lb[q]], 1u) % 24;
        if (STAGE == 2) {
#pragma unroll
            for (int q = 0; q < 7; q++) acc += dn[q];
            continue;
        }
        uint32_t fmask = 0;
#pragma unroll
        for (int q = 0; q < 7; q++) fmask |= (uint32_t)(dn[q] == 23) << q;
        while (fmask) {
            const int qs = __ffs(fmask) - 1;
            fmask &= fmask - 1;
            uint32_t L = 0;
#pragma unroll
            for (int q = 0; q < 7; q++)
                if (q == qs) L = lb[q];
            const volatile lds_v4* s4 = (const volatile lds_v4*)(lds_u32*)(slots + L * 24);
            uint32_t v[24];
#pragma unroll
            for (int j = 0; j < 6; j++) {
                const u32x4 x = s4[j];
                v[4 * j] = x.x;
                v[4 * j + 1] = x.y;
                v[4 * j + 2] = x.z;
                v[4 * j + 3] = x.w;
            }
            uint4 o[4];
#pragma unroll
            for (int j = 0; j < 4; j++)
                o[j] = make_uint4(v[6 * j] | (v[6 * j + 1] << 20), (v[6 * j + 1] >> 12) | (v[6 * j + 2] << 8),
                                  v[6 * j + 3] | (v[6 * j + 4] << 20), (v[6 * j + 4] >> 12) | (v[6 * j + 5] << 8));
            if (STAGE == 3) {
                acc += o[0].x ^ o[1].y ^ o[2].z ^ o[3].w;
            } else if (STAGE == 5) {  // same stores, regular per-lane addresses
                uint4* dst = out + ((uint64_t)(blockIdx.x * BLOCK + threadIdx.x) * 64 + (i & 63)) * 4;
#pragma unroll
                for (int j = 0; j < 4; j++) dst[j] = o[j];
            } else if (STAGE == 6) {  // scattered, nontemporal
                uint4* dst = out + ((uint64_t)(L * gridDim.x + blockIdx.x) * 64 + (i & 63)) * 4;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
                    v4 x = {o[j].x, o[j].y, o[j].z, o[j].w};
                    __builtin_nontemporal_store(x, reinterpret_cast<v4*>(dst + j));
                }
            } else {
                uint4* dst = out + ((uint64_t)(L * gridDim.x + blockIdx.x) * 64 + (i & 63)) * 4;
#pragma unroll
                for (int j = 0; j < 4; j++) dst[j] = o[j];
            }
        }
    }
    sink[blockIdx.x * BLOCK + threadIdx.x] = acc;
}

int main() {
    const uint64_t n = 100000000ull;
    const uint32_t nbits = 956715292u, nb = (nbits + (1u << 20) - 1) >> 20;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint4 *keys, *out;
    uint32_t* sink;
    hipMalloc(&keys, n * 16);
    hipMalloc(&out, (size_t)nb * cus * 64 * 64);
    hipMalloc(&sink, (size_t)cus * 1024 * 4 * 4);
    k_gen<<<8192, 256>>>(keys, n);
    hipDeviceSynchronize();
    const Mod32 md = Mod32::make(nbits);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](auto kern, int block, int per_cu, const char* name) {
        const size_t smem = (size_t)nb * 26 * 4;
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        kern<<<cus * per_cu, block, smem>>>(keys, n, md, nb, out, sink);
        hipEventRecord(a);
        for (int r = 0; r < 5; r++) kern<<<cus * per_cu, block, smem>>>(keys, n, md, nb, out, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("%-44s %8.4f ms\n", name, ms / 5);
    };
    run(k<0, 1024>, 1024, 1, "stage 0 hash+walk (1024 thr, 1 WG/CU)");
    run(k<1, 1024>, 1024, 1, "stage 1 + claims");
    run(k<2, 1024>, 1024, 1, "stage 2 + slot writes + done adds");
    run(k<3, 1024>, 1024, 1, "stage 3 + flush reads/pack");
    run(k<4, 1024>, 1024, 1, "stage 4 + global segment stores");
    run(k<5, 1024>, 1024, 1, "stage 5 = 4 with per-lane regular addresses");
    run(k<6, 1024>, 1024, 1, "stage 6 = 4 with nontemporal stores");
    return 0;
}
