// mb_mall.hip (round 6) — is a re-read of a resident 32-384 MB buffer served
// faster than HBM streaming?  The Infinity Cache (MALL) is 256 MB on MI355X.
// the round-5 version timed single launches
// of one 16-B load per lane per grid-stride step, launch/ramp-dominated below
// ~256 MB, and never a steady-state re-read.  This one:
//   * k_pass<U>: every lane keeps U = 8 independent 16-B loads in flight, the
//     grid fills the chip (8 workgroups of 256 lanes per CU), and one launch
//     makes R passes over the buffer (a persistent re-read), so a timed launch
//     moves R x S bytes (>= 0.6 GB: launch cost < 1 %);
//   * HBM baseline: the same kernel shape streaming a 4 GiB buffer once
//     (R = 1) and 2 GiB twice (R = 2: too big to be resident);
//   * per size S: re-read R = 20 times after the buffer was made resident by a
//     plain read (clean lines), and separately right after a write (dirty
//     lines), as one launch; and as 20 back-to-back single-pass launches;
//   * the C4 chunking question itself: a kernel that streams 1 GB of "key
//     bytes" (plain or non-temporal loads) while it writes S of "records", then
//     one pass reading the records back, against the same read from a cold
//     buffer (flushed by a 4 GiB stream).
// One JSON object per line on stdout (GB/s = bytes moved / event time).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/mb_mall.hip -o tools/mb_mall
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

constexpr int U = 8;

__device__ __forceinline__ uint32_t fold(uint4 x) { return x.x ^ x.y ^ x.z ^ x.w; }

// R passes over p[0, n) (16-B elements), U loads in flight per lane.
template <bool NT>
__global__ __launch_bounds__(256) void k_pass(const uint4* __restrict__ p, uint64_t n, int R, uint32_t* out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (int r = 0; r < R; r++) {
        uint64_t i = t;
        for (; i + (U - 1) * stride < n; i += U * stride) {
            uint4 x[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (NT) {
                    const uint32_t* q = (const uint32_t*)&p[i + u * stride];
                    x[u].x = __builtin_nontemporal_load(q), x[u].y = __builtin_nontemporal_load(q + 1);
                    x[u].z = __builtin_nontemporal_load(q + 2), x[u].w = __builtin_nontemporal_load(q + 3);
                } else {
                    x[u] = p[i + u * stride];
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++) acc ^= fold(x[u]);
        }
        for (; i < n; i += stride) acc ^= fold(p[i]);
        acc = acc * 3 + r;  // each pass's loads are live
    }
    if (acc == 0x9e3779b9u) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_write(uint4* p, uint64_t n, uint32_t v) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        p[i] = make_uint4(v ^ (uint32_t)i, v, (uint32_t)i, v + 1);
}

// k_hash_var's traffic shape: stream `nk` 16-B elements of key bytes (plain
// or non-temporal loads, coalesced grid-stride) and write the `nr` 16-B
// records interleaved with them (element i with i % per == 0 writes record
// i / per).
template <bool NT>
__global__ __launch_bounds__(256) void k_stream_write(const uint4* __restrict__ keys, uint64_t nk, uint4* rec,
                                                      uint64_t nr, uint32_t* out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t per = nk / nr;  // key elements per record (>= 1)
    uint32_t acc = 0;
#pragma unroll 4
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nk; i += stride) {
        uint4 y;
        if (NT) {
            const uint32_t* q = (const uint32_t*)&keys[i];
            y.x = __builtin_nontemporal_load(q), y.y = __builtin_nontemporal_load(q + 1);
            y.z = __builtin_nontemporal_load(q + 2), y.w = __builtin_nontemporal_load(q + 3);
        } else {
            y = keys[i];
        }
        acc = acc * 5 + fold(y);
        if (i % per == 0 && i / per < nr) rec[i / per] = make_uint4(y.x, acc, (uint32_t)i, y.w);
    }
    if (acc == 0x9e3779b9u) out[0] = acc;
}

int main(int argc, char** argv) {
    const uint64_t big = 4ull << 30, maxs = 384ull << 20;
    uint4 *buf, *other;
    uint32_t* out;
    CK(hipMalloc(&buf, maxs));
    CK(hipMalloc(&other, big));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(other, 1, big));
    CK(hipMemset(buf, 2, maxs));
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int grid = cus * 8, block = 256;
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
        return (double)ms;
    };
    auto flush = [&] { k_pass<false><<<grid, block>>>(other, big / 16, 1, out); };
    auto emit = [](const char* what, uint64_t mb, int R, double ms, double bytes) {
        printf("{\"what\": \"%s\", \"MB\": %llu, \"R\": %d, \"ms\": %.4f, \"GBs\": %.0f}\n", what,
               (unsigned long long)mb, R, ms, bytes / ms / 1e6);
        fflush(stdout);
    };
    // warm the clocks
    for (int i = 0; i < 20; i++) flush();
    CK(hipDeviceSynchronize());
    // HBM baseline: the same kernel shape over buffers far above 256 MB
    for (int rep = 0; rep < 3; rep++) {
        double ms = timed([&] { k_pass<false><<<grid, block>>>(other, big / 16, 1, out); });
        emit("hbm_stream_4GiB", big >> 20, 1, ms, (double)big);
        ms = timed([&] { k_pass<false><<<grid, block>>>(other, (big / 2) / 16, 2, out); });
        emit("hbm_stream_2GiB_x2", (big / 2) >> 20, 2, ms, (double)big);
        ms = timed([&] { k_pass<true><<<grid, block>>>(other, big / 16, 1, out); });
        emit("hbm_stream_4GiB_nt", big >> 20, 1, ms, (double)big);
    }
    const int R = 20;
    for (uint64_t mb : {32, 64, 100, 128, 160, 200, 256, 384}) {
        const uint64_t S = mb << 20, n = S / 16;
        for (int rep = 0; rep < 2; rep++) {
            flush();
            k_pass<false><<<grid, block>>>(buf, n, 1, out);  // resident by a plain read (clean)
            double ms = timed([&] { k_pass<false><<<grid, block>>>(buf, n, R, out); });
            emit("reread_after_read", mb, R, ms, (double)S * R);
            flush();
            k_write<<<grid, block>>>(buf, n, rep);  // resident by a write (dirty)
            ms = timed([&] { k_pass<false><<<grid, block>>>(buf, n, R, out); });
            emit("reread_after_write", mb, R, ms, (double)S * R);
            flush();
            k_pass<false><<<grid, block>>>(buf, n, 1, out);
            ms = timed([&] {
                for (int r = 0; r < R; r++) k_pass<false><<<grid, block>>>(buf, n, 1, out);
            });
            emit("reread_launches", mb, R, ms, (double)S * R);
            // the C4 question: records written while 1 GiB of key bytes streams,
            // then read back once; against the same read from a cold buffer
            for (int nt = 0; nt < 2; nt++) {
                flush();
                const uint64_t nk = (1ull << 30) / 16;
                const double tw = timed([&] {
                    if (nt) k_stream_write<true><<<grid, block>>>(other, nk, buf, n, out);
                    else k_stream_write<false><<<grid, block>>>(other, nk, buf, n, out);
                });
                emit(nt ? "stream_nt_and_write" : "stream_and_write", mb, 1, tw, (double)(nk * 16 + S));
                ms = timed([&] { k_pass<false><<<grid, block>>>(buf, n, 1, out); });
                emit(nt ? "readback_after_stream_nt_write" : "readback_after_stream_write", mb, 1, ms, (double)S);
            }
            flush();
            ms = timed([&] { k_pass<false><<<grid, block>>>(buf, n, 1, out); });
            emit("read_cold", mb, 1, ms, (double)S);
        }
    }
    return 0;
}
