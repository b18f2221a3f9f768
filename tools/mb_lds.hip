// mb_lds.hip — LDS random-access throughput on gfx950 (calibrates pass A/B design).
// Each lane performs ITERS operations at pseudo-random LDS addresses.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

constexpr int ITERS = 4096;

__device__ __forceinline__ uint32_t rnd(uint32_t& s) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
}

// MODE 0: ds_add_rtn_u32 over NB counters; 1: ds_add_u32 (no return);
// 2: ds_or_b64 over NB*8 words; 3: ds_write_b32 over NB*16 words;
// 4: ds_or_b32 over 32768 words (pass B); 5: ds_read_b32 random over NB counters;
// 7 / 8: mode 4 with ~1/2 / ~1/4 of the lanes active (exec-masked)
template <int MODE>
__global__ __launch_bounds__(1024) void k(uint32_t nb, uint32_t* out) {
    extern __shared__ uint32_t lds[];
    uint64_t* l64 = reinterpret_cast<uint64_t*>(lds);
    const uint32_t words = MODE == 4 ? 32768 : MODE == 2 ? nb * 16 : MODE == 3 ? nb * 16 : nb;
    const uint32_t m = nb - 1;  // nb is a power of two here
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) lds[i] = 0;
    __syncthreads();
    uint32_t s = (blockIdx.x * 1024 + threadIdx.x) * 2654435761u + 1, acc = 0;
    for (int it = 0; it < ITERS; it++) {
        const uint32_t r = rnd(s);
        if (MODE == 0) acc += atomicAdd(&lds[r & m], 1u);
        if (MODE == 1) atomicAdd(&lds[r & m], 1u);
        if (MODE == 2) atomicOr(reinterpret_cast<unsigned long long*>(&l64[r & (8 * nb - 1)]), (unsigned long long)r << 7);
        if (MODE == 3) lds[r & (16 * nb - 1)] = r;
        if (MODE == 4) atomicOr(&lds[r & 32767], 1u << (r >> 27));
        if (MODE == 5) acc += lds[r & m];
        // round 6: does a half-masked ds_or cost half?  (k_apply<21>'s halves
        // each issue every offset's ds_or with ~half of the lanes active)
        if (MODE == 7 && ((r >> 26) & 1)) atomicOr(&lds[r & 32767], 1u << (r >> 27));
        if (MODE == 8 && ((r >> 25) & 3) == 0) atomicOr(&lds[r & 32767], 1u << (r >> 27));
    }
    __syncthreads();
    out[blockIdx.x * 1024 + threadIdx.x] = acc + lds[threadIdx.x % words];
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int grid = cus * 2;
    uint32_t* out;
    CK(hipMalloc(&out, grid * 1024 * 4));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const uint32_t nb = 1024;
    auto run = [&](auto kern, const char* name, size_t smem) {
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        kern<<<grid, 1024, smem>>>(nb, out);
        hipEventRecord(a);
        kern<<<grid, 1024, smem>>>(nb, out);
        hipEventRecord(b);
        CK(hipEventSynchronize(b));
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double ops = (double)grid * 1024 * ITERS;
        const double per_cu_cycle = ops / cus / (ms * 1e-3 * 2.4e9);
        printf("%-40s %8.3f ms  %7.1f G lane-ops/s  %5.2f lane-ops/clk/CU  (%.1f clk per wave-instr)\n", name, ms,
               ops / ms / 1e6, per_cu_cycle, 64.0 / per_cu_cycle);
    };
    run(k<0>, "ds_add_rtn_u32 random / 1024 ctr", 1024 * 4);
    run(k<1>, "ds_add_u32 (no rtn) random / 1024 ctr", 1024 * 4);
    run(k<2>, "ds_or_b64 random / 1024*8 words", 1024 * 64);
    run(k<3>, "ds_write_b32 random / 1024*16 words", 1024 * 64);
    run(k<4>, "ds_or_b32 random / 32768 words", 32768 * 4);
    run(k<5>, "ds_read_b32 random / 1024 ctr", 1024 * 4);
    run(k<6>, "VALU only (xorshift)", 1024 * 4);
    run(k<7>, "ds_or_b32 / 32768 words, 1/2 lanes active", 32768 * 4);
    run(k<8>, "ds_or_b32 / 32768 words, 1/4 lanes active", 32768 * 4);
    return 0;
}
