// mb_valu.hip — issue cost of the VALU instructions the build and probe paths
// are made of (XXH3-128 + exact positions + ring bookkeeping), on gfx950.
// Each thread runs 8 independent chains of one instruction (inline asm, so the
// compiler cannot change it); 4 or 8 waves per SIMD; cycles per wave-
// instruction per SIMD = kernel time x clock x 1024 SIMDs / wave-instructions,
// with the clock read from s_memtime inside the kernel (shader cycles).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 mb_valu.hip -o mb_valu
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

constexpr int kIters = 4096;

// one instruction (or pair) applied to chain register a (32-bit) / A (64-bit)
#define OP_V32(insn) asm volatile(insn " %0, %0, %1" : "+v"(a[c]) : "v"(b))
#define OP_V64(insn) asm volatile(insn " %0, %0, %1" : "+v"(A[c]) : "v"(B))

template <int OP>
__global__ __launch_bounds__(256) void k_op(uint32_t seed, uint32_t* out, unsigned long long* cyc) {
    uint32_t a[8];
    uint64_t A[8];
    double D[8];
    const uint32_t b = seed ^ threadIdx.x;
    uint64_t B = ((uint64_t)b << 32) | (b * 3u + 1u);
    const double Db = 1.0 + b * 1e-9;
#pragma unroll
    for (int c = 0; c < 8; c++) {
        a[c] = b + c;
        A[c] = B + c;
        D[c] = Db + c;
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int c = 0; c < 8; c++) {
            if constexpr (OP == 0) OP_V32("v_xor_b32");
            if constexpr (OP == 1) OP_V32("v_add_u32");
            if constexpr (OP == 2) OP_V32("v_mul_u32_u24");
            if constexpr (OP == 3) OP_V32("v_mul_lo_u32");
            if constexpr (OP == 4) OP_V32("v_mul_hi_u32");
            if constexpr (OP == 5) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(A[c]) : "v"(b) : "vcc");
            if constexpr (OP == 6) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(A[c]) : "v"(B));
            if constexpr (OP == 7) asm volatile("v_cmp_lt_u64 vcc, %0, %1\n\tv_cndmask_b32 %2, %3, %2, vcc"
                                                : "+v"(A[c]), "+v"(B), "+v"(a[c]) : "v"(b) : "vcc");
            if constexpr (OP == 8) asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc"
                                                : "+v"(a[c]), "+v"(a[(c + 1) & 7]) : "v"(b), "v"(b) : "vcc");
            if constexpr (OP == 9) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(D[c]) : "v"(a[c]));
            if constexpr (OP == 10) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(D[c]) : "v"(Db));
            if constexpr (OP == 11) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(D[c]) : "v"(Db));
            if constexpr (OP == 12) asm volatile("v_cvt_u32_f64 %0, %1" : "=v"(a[c]) : "v"(D[c]));
            if constexpr (OP == 13) asm volatile("v_alignbit_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 14) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 15) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 16) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a[c]));
            if constexpr (OP == 17) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 18) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(A[c]));
            if constexpr (OP == 19) asm volatile("v_bfe_u32 %0, %0, 3, 20" : "+v"(a[c]));
            // round 5: the rest of the per-key instruction mix, and encodings
            if constexpr (OP == 20) OP_V32("v_and_b32");
            if constexpr (OP == 21) OP_V32("v_or_b32");
            if constexpr (OP == 22) OP_V32("v_sub_u32");
            if constexpr (OP == 23) OP_V32("v_lshlrev_b32");
            if constexpr (OP == 24) OP_V32("v_lshrrev_b32");
            if constexpr (OP == 25) asm volatile("v_mov_b32 %0, %1" : "=v"(a[c]) : "v"(a[(c + 3) & 7]));
            if constexpr (OP == 26) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[c]) : "v"(b) : "vcc");
            if constexpr (OP == 27) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 28) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 29) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 30) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 31) OP_V32("v_max_u32");
            if constexpr (OP == 32) asm volatile("v_bfi_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 33) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[c]) : "v"(b) : "vcc");
            if constexpr (OP == 34) asm volatile("v_sub_co_u32 %0, vcc, %0, %1" : "+v"(a[c]) : "v"(b) : "vcc");
            if constexpr (OP == 35) asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(a[c]), "v"(b) : "vcc");
            if constexpr (OP == 36) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 37) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(A[c]) : "v"(B));
            if constexpr (OP == 38) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(A[c]) : "v"(B));
            if constexpr (OP == 39) asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(a[c]));
            if constexpr (OP == 40) asm volatile("v_max3_u32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 41) OP_V32("v_ashrrev_i32");
            if constexpr (OP == 42) asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a[c]));
            if constexpr (OP == 43) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 44) asm volatile("v_min_u32_e64 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 45) asm volatile("v_subrev_u32 %0, %1, %0" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 46) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 47) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x80" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 48) asm volatile("v_xad_u32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 49) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a[c]) : "v"(b) : "vcc");
            if constexpr (OP == 50) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 51) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(A[c]) : "v"(B));
            if constexpr (OP == 52) asm volatile("v_med3_u32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(b));
            if constexpr (OP == 53) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(b));
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) r ^= a[c] ^ (uint32_t)A[c] ^ (uint32_t)(A[c] >> 32) ^ (uint32_t)(uint64_t)D[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) atomicMax(cyc, (unsigned long long)(t1 - t0));
}

static const char* kNames[] = {"v_xor_b32",      "v_add_u32",        "v_mul_u32_u24",       "v_mul_lo_u32",
                               "v_mul_hi_u32",   "v_mad_u64_u32",    "v_lshl_add_u64",      "v_cmp_lt_u64+cndmask",
                               "v_add_co+addc",  "v_cvt_f64_u32",    "v_mul_f64",           "v_fma_f64",
                               "v_cvt_u32_f64",  "v_alignbit_b32",   "v_add3_u32",          "v_min_u32",
                               "v_cvt_f32_u32",  "v_mul_f32",        "v_lshrrev_b64",       "v_bfe_u32",
                               "v_and_b32",      "v_or_b32",         "v_sub_u32",           "v_lshlrev_b32",
                               "v_lshrrev_b32",  "v_mov_b32",        "v_cndmask_b32(vcc)",  "v_lshl_or_b32",
                               "v_lshl_add_u32", "v_perm_b32",       "v_mad_u32_u24",       "v_max_u32",
                               "v_bfi_b32",      "v_add_co_u32",     "v_sub_co_u32",        "v_cmp_gt_u32(e32)",
                               "v_fma_f32",      "v_pk_add_f32",     "v_pk_fma_f32",        "v_cvt_u32_f32",
                               "v_max3_u32",     "v_ashrrev_i32",    "v_add_u32(literal)",  "v_xor_b32_e64",
                               "v_min_u32_e64",  "v_subrev_u32",     "v_and_or_b32",        "v_bitop3_b32",
                               "v_xad_u32",      "v_addc_co_u32",    "v_add_f32",           "v_pk_mul_f32",
                               "v_med3_u32",     "v_mul_hi_u32_u24"};
static const int kInsnPerOp[] = {1, 1, 1, 1, 1, 1, 1, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};

template <int OP>
void run(int wps, uint32_t* out, unsigned long long* cyc, int ncu) {
    const int blocks = ncu * 4 * wps / 4;  // 4 waves per 256-thread block
    CK(hipMemset(cyc, 0, 8));
    k_op<OP><<<blocks, 256>>>(1, out, cyc);  // warm-up
    CK(hipDeviceSynchronize());
    CK(hipMemset(cyc, 0, 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    k_op<OP><<<blocks, 256>>>(2, out, cyc);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long c = 0;
    CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    const double winsn = (double)blocks * 4 * kIters * 8 * kInsnPerOp[OP];  // wave-instructions
    const double simds = ncu * 4.0;
    // per SIMD: wave-instructions it issued = winsn / simds; its cycles ~ the
    // longest wave's s_memtime span (waves of a SIMD run concurrently)
    const double cyc_per = (double)c / (winsn / simds);
    const double clk = (double)c / (ms * 1e-3) * 1e-9;
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cycles_per_wave_insn_per_simd\": %.3f, "
           "\"clock_GHz_est\": %.3f, \"wave_insn_per_s\": %.4g}\n",
           kNames[OP], wps, ms, cyc_per, clk, winsn / (ms * 1e-3));
}

template <int... OPS>
void run_all(int wps, uint32_t* out, unsigned long long* cyc, int ncu, int first, std::integer_sequence<int, OPS...>) {
    ((OPS >= first ? run<OPS>(wps, out, cyc, ncu) : void()), ...);
}

int main(int argc, char** argv) {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t* out;
    unsigned long long* cyc;
    CK(hipMalloc(&out, (size_t)ncu * 4 * 8 * 64 * 4));
    CK(hipMalloc(&cyc, 8));
    const int nops = argc > 1 ? atoi(argv[1]) : 54;  // ops [first, 54): argv[2]
    const int first = argc > 2 ? atoi(argv[2]) : 0;
    (void)nops;
    for (int wps : {4, 8}) run_all(wps, out, cyc, ncu, first, std::make_integer_sequence<int, 54>{});
    CK(hipFree(out));
    CK(hipFree(cyc));
    return 0;
}
