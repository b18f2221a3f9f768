// mb_mall.hip — does a buffer that one kernel writes and the next reads stay
// in the Infinity Cache (MALL, 256 MB on MI355X)?  The question behind
// chunking the var-len build: k_hash_var writes 12-B walk
// records that k_bin reads right after; in chunks small enough to stay
// cache-resident, the round trip would not cost HBM time.
// For each size S: write S (plain or nontemporal stores), then read it back
// (plain / nontemporal loads), each timed alone with HIP events; and the same
// with a 2 GB streaming read between them (k_hash_var streams the key bytes
// while it writes the records).  GB/s per kernel.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 mb_mall.hip -o mb_mall
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));       \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

template <bool NT>
__global__ __launch_bounds__(256) void k_write(uint4* p, uint64_t n, uint32_t v) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 x = make_uint4(v ^ (uint32_t)i, v, (uint32_t)i, v + 1);
        if (NT) {
            __builtin_nontemporal_store(x.x, &p[i].x);
            __builtin_nontemporal_store(x.y, &p[i].y);
            __builtin_nontemporal_store(x.z, &p[i].z);
            __builtin_nontemporal_store(x.w, &p[i].w);
        } else {
            p[i] = x;
        }
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void k_read(const uint4* p, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 x;
        if (NT) {
            x.x = __builtin_nontemporal_load(&p[i].x);
            x.y = __builtin_nontemporal_load(&p[i].y);
            x.z = __builtin_nontemporal_load(&p[i].z);
            x.w = __builtin_nontemporal_load(&p[i].w);
        } else {
            x = p[i];
        }
        acc ^= x.x ^ x.y ^ x.z ^ x.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const uint64_t big = 2ull << 30, maxs = 1280ull << 20;
    uint4 *buf, *other;
    uint32_t* out;
    CK(hipMalloc(&buf, maxs));
    CK(hipMalloc(&other, big));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(other, 1, big));
    const int grid = 256 * 16, block = 256;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timed = [&](auto launch) {
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms;
    };
    for (uint64_t mb : {32, 64, 96, 128, 192, 256, 512, 1280}) {
        const uint64_t S = mb << 20, n = S / 16;
        for (int ntw = 0; ntw < 2; ntw++)
            for (int ntr = 0; ntr < 2; ntr++)
                for (int mid = 0; mid < 2; mid++) {
                    double tw = 0, tr = 0;
                    const int reps = 6;
                    for (int r = 0; r < reps + 1; r++) {
                        const float w = timed([&] {
                            if (ntw) k_write<true><<<grid, block>>>(buf, n, r);
                            else k_write<false><<<grid, block>>>(buf, n, r);
                        });
                        if (mid) k_read<true><<<grid, block>>>(other, big / 16, out);
                        const float rd = timed([&] {
                            if (ntr) k_read<true><<<grid, block>>>(buf, n, out);
                            else k_read<false><<<grid, block>>>(buf, n, out);
                        });
                        if (r) tw += w, tr += rd;
                    }
                    tw /= reps, tr /= reps;
                    printf("{\"MB\": %llu, \"nt_store\": %d, \"nt_load\": %d, \"2GB_stream_between\": %d, "
                           "\"write_ms\": %.4f, \"write_GBs\": %.0f, \"read_ms\": %.4f, \"read_GBs\": %.0f}\n",
                           (unsigned long long)mb, ntw, ntr, mid, tw, S / tw / 1e6, tr, S / tr / 1e6);
                }
    }
    return 0;
}
