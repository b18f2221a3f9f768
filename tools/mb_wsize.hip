// mb_wsize.hip — what WRITE_SIZE reports for pass A's region writes.
//
// k_bin writes 1.88 GB of 64-B segments per C2 build and rocprofv3 reports a
// WRITE_SIZE of 2.42 GB.  Each workgroup's region of a slice
// grows one 64-B segment at a time, and the two halves of a 128-B line are
// written far apart in time (hundreds of thousands of other segments in
// between).  These kernels write the same 2 GiB four ways:
//   stream   16 B per lane, consecutive (the guide's calibrated pattern)
//   seg_rand every 64-B segment once, in a pseudo-random order
//   seg_far  round t writes segment t of every region (2^18 regions of 128
//            segments): a line's two halves are 16 MB of writes apart — k_bin's shape
//   seg_pair as seg_far, but segments 2t and 2t+1 in the same round (whole lines)
// Run: rocprofv3 --pmc WRITE_SIZE --output-format csv -d DIR -o run -- ./mb_wsize
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e = (x);                                                                    \
        if (e != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

constexpr uint64_t kBytes = 2ull << 30;
constexpr uint32_t kSegs = (uint32_t)(kBytes / 64);  // 2^25
constexpr uint32_t kRegions = 1u << 18, kPerRegion = kSegs / kRegions;  // 128 segments each

// seg_dist<LR>: 2^LR regions of 2^(25-LR) segments; round t writes segment t
// of every region (regions permuted), so a line's two halves are 2^LR
// segments (2^(LR+6) bytes of other writes) apart in time.
template <int LR>
__global__ void k_seg_dist(uint4* out) {
    constexpr uint32_t R = 1u << LR, P = kSegs >> LR;
    const uint64_t nthreads = (uint64_t)kSegs * 4;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nthreads;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)(i >> 2), l = (uint32_t)(i & 3);
        const uint32_t t = s >> LR, r = ((s & (R - 1)) * 40503u) & (R - 1);
        out[((uint64_t)r * P + t) * 4 + l] = make_uint4(s, l, 7, 9);
    }
}

__global__ void k_stream(uint4* out) {
    const uint64_t n = kBytes / 16;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

// 4 lanes per segment, 16 B each; segment s -> slot f(s)
template <int MODE>
__global__ void k_seg(uint4* out) {
    const uint64_t nthreads = (uint64_t)kSegs * 4;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nthreads;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)(i >> 2), l = (uint32_t)(i & 3);
        uint32_t slot;
        if (MODE == 0) {  // random order: an odd multiplier permutes [0, 2^25)
            slot = (s * 2654435761u) & (kSegs - 1);
        } else if (MODE == 1) {  // round t = s / kRegions writes segment t of region (permuted) r
            const uint32_t t = s / kRegions, r = ((s % kRegions) * 40503u) & (kRegions - 1);
            slot = r * kPerRegion + t;
        } else {  // pairs: round t writes segments 2t' and 2t'+1 of each region back to back
            const uint32_t p = s >> 1, h = s & 1;
            const uint32_t t = p / kRegions, r = ((p % kRegions) * 40503u) & (kRegions - 1);
            slot = r * kPerRegion + 2 * t + h;
        }
        out[(uint64_t)slot * 4 + l] = make_uint4(s, l, 7, 9);
    }
}

// k_bin's cooperative flush: one buffer_store_b128 per lane, lanes with
// nothing to write at an offset past num_records (dropped by the hardware).
// MODE 0: every lane dropped; MODE 1: every other group of 4 lanes dropped.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int MODE>
__global__ void k_drop(uint4* out) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7FFFFFF0, 0x00020000);
    const uint64_t nthreads = (uint64_t)kSegs * 4;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nthreads;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const bool drop = MODE == 0 || ((i >> 2) & 1);
        const uint32_t off = drop ? 0x80000000u : (uint32_t)(((i >> 3) * 4 + (i & 3)) * 16);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{(uint32_t)i, 1, 2, 3}, rs, off, 0, 0);
    }
}

int main() {
    uint4* out;
    CK(hipMalloc(&out, kBytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char* name, auto launch) {
        launch();
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%-9s %.3f ms  %.0f GB/s (2 GiB written per launch)\n", name, ms, kBytes / (ms * 1e-3) / 1e9);
    };
    run("stream", [&] { k_stream<<<4096, 256>>>(out); });
    run("seg_rand", [&] { k_seg<0><<<4096, 256>>>(out); });
    run("seg_far", [&] { k_seg<1><<<4096, 256>>>(out); });
    run("seg_pair", [&] { k_seg<2><<<4096, 256>>>(out); });
    run("dist_2^12", [&] { k_seg_dist<12><<<4096, 256>>>(out); });
    run("dist_2^16", [&] { k_seg_dist<16><<<4096, 256>>>(out); });
    run("dist_2^20", [&] { k_seg_dist<20><<<4096, 256>>>(out); });
    run("dist_2^23", [&] { k_seg_dist<23><<<4096, 256>>>(out); });
    run("drop_all", [&] { k_drop<0><<<4096, 256>>>(out); });
    run("drop_half", [&] { k_drop<1><<<4096, 256>>>(out); });  // 1 GiB really written
    CK(hipDeviceSynchronize());
    CK(hipFree(out));
    return 0;
}
