// mfma_q4k_ceiling.hip — what the matrix cores can deliver for EXACT Q4_K x Q8_K dot products on gfx950 (diagnostic).
//
// Q4_K (ggml-common.h:282-297) stores per 32-weight sub-block j a 6-bit scale sc_j and 4-bit codes q; ggml's integer
// dot (ggml-quants.c:7713-8279) is isum = sum_j sc_j * sum_{k in j} q8_k * q_k, exact in int32. Three ways to put it on
// the matrix cores, each timed here as a register-resident loop (no memory traffic: the ceiling, not a GEMM):
//
//   fp16   the engine's design: the weight operand is the product sc_j * q (<= 945, exact in fp16), the Q8_K code
//          exact in fp16, v_mfma_f32_16x16x32_f16 with fp32 accumulation — sub-block scales cost nothing.
//   i8sc   int8 MFMA on the raw codes, one 32-deep K step = one sub-block (v_mfma_i32_32x32x32_i8, fresh
//          accumulator via C = 0), then the sub-block scale per output column in VALU: 16 v_mad_u32_u24 per MFMA.
//   i8hl   int8 MFMA with sc * q split as 64 * hi + lo (hi <= 14, lo <= 63: both int8) — the scale folded in, two MFMAs
//          (hi, lo) per K step, exact int32 over the whole block (v_mfma_i32_16x16x64_i8).
//
// Each loop reports "Q4_K-equivalent TOPS" = 2 * M * N * K of Q4_K work per second, to compare with the fp16 dense peak
// (2.5 PF spec) and the int8 peak (5 PF spec). One 512-thread workgroup per CU (2 waves per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef int i4 __attribute__((ext_vector_type(4)));
typedef int i16v __attribute__((ext_vector_type(16)));

constexpr int ITERS = 4096;

// fp16: per iteration 4 independent 16x16x32 MFMAs = 4 * 16*16*32*2 flop
__global__ __launch_bounds__(512) void k_fp16(float * out, int seed) {
    half8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (_Float16) ((threadIdx.x + i + seed) & 7); b[i] = (_Float16) ((threadIdx.x * 3 + i) & 15); }
    f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int it = 0; it < ITERS; ++it) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

// i8sc: per iteration 2 sub-blocks x one 32x32x32 i8 MFMA (fresh accumulator) + 16 integer MADs each
__global__ __launch_bounds__(512) void k_i8sc(float * out, int seed) {
    long a = 0x0102030405060708l * ((threadIdx.x + seed) & 3), b = 0x0f0e0d0c0b0a0908l;
    i4 av = {(int) a, (int) (a >> 32), (int) b, (int) (b >> 32)};
    i4 bv = {(int) b, (int) (b >> 32), (int) a, (int) (a >> 32)};
    i16v isum = {};
    const i16v zero = {};
    unsigned sc0 = (threadIdx.x & 63) + 1, sc1 = (threadIdx.x * 7) & 63;
    for (int it = 0; it < ITERS; ++it) {
        i16v p0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, zero, 0, 0, 0);
        i16v p1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(bv, av, zero, 0, 0, 0);
        // |P| <= 32 * 15 * 127 fits 24 bits, sc <= 63: one v_mad_i32_i24 per output per sub-block
        for (int r = 0; r < 16; ++r) isum[r] = __mul24((int) sc0, p0[r]) + isum[r];
        for (int r = 0; r < 16; ++r) isum[r] = __mul24((int) sc1, p1[r]) + isum[r];
        sc0 ^= it; sc1 += 1;
    }
    int t = 0;
    for (int r = 0; r < 16; ++r) t += isum[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float) t;
}

// i8hl: per iteration 4 independent 16x16x64 i8 MFMAs (2 K-steps x {hi, lo})
__global__ __launch_bounds__(512) void k_i8hl(float * out, int seed) {
    i4 a = {(int) (threadIdx.x + seed), 0x01020304, 0x0a0b0c0d, 0x11121314};
    i4 b = {0x05060708, (int) threadIdx.x, 0x1a1b1c1d, 0x21222324};
    i4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int it = 0; it < ITERS; ++it) {
        c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float) (c0[0] + c1[1] + c2[2] + c3[3]);
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = ncu, threads = 512;   // one 8-wave workgroup per CU: 2 waves per SIMD, as the GEMMs run
    float * out;
    hipMalloc(&out, (size_t) blocks * threads * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double waves = (double) blocks * threads / 64;
    struct { const char * name; void (*k)(float *, int); double qflop_per_wave_iter; } runs[] = {
        // fp16: 4 MFMAs x 16x16x32 -> 4 * 16*16*32*2 Q4_K flop (each is real Q4_K work)
        {"fp16 (sc*q folded, 16x16x32 f16)", k_fp16, 4.0 * 16 * 16 * 32 * 2},
        // i8sc: 2 sub-blocks x 32x32x32 of Q4_K work
        {"i8sc (raw codes, 32x32x32 i8 + VALU scale)", k_i8sc, 2.0 * 32 * 32 * 32 * 2},
        // i8hl: 4 MFMAs, but hi + lo together are one K step of Q4_K work: 2 x 16x16x64
        {"i8hl (sc*q = 64hi+lo, 16x16x64 i8 x2)", k_i8hl, 2.0 * 16 * 16 * 64 * 2},
    };
    printf("{\"cus\": %d, \"results\": [", ncu);
    for (int r = 0; r < 3; ++r) {
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(runs[r].k, dim3(blocks), dim3(threads), 0, 0, out, w);
        hipEventRecord(e0);
        const int reps = 10;
        for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(runs[r].k, dim3(blocks), dim3(threads), 0, 0, out, w);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double tops = runs[r].qflop_per_wave_iter * ITERS * waves * reps / (ms * 1e-3) / 1e12;
        printf("%s{\"loop\": \"%s\", \"ms\": %.3f, \"q4k_equiv_tops\": %.1f}", r ? ", " : "", runs[r].name, ms / reps, tops);
    }
    printf("]}\n");
    hipFree(out);
    return 0;
}
