// bwbench.hip — bandwidth reference points for the activation quantizers (diagnostic, not shipped): plain streaming
// kernels over the fc1 activation size (96 000 x 5 120 fp16 = 983 MB) beside the engine's GELU+Q8_K and
// LayerNorm+Q8_K launchers (linked from build/q2a_exact.o), timed with HIP events.
#include "q2a_internal.h"
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_copy16(const uint4 * __restrict__ x, uint4 * __restrict__ y, int64_t n) {
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) y[i] = x[i];
}
__global__ void k_read16(const uint4 * __restrict__ x, int64_t n, unsigned * out) {
    unsigned a = 0;
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        const uint4 v = x[i];
        a ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (a == 0x12345678u) out[0] = a;
}
__global__ void k_write16(uint4 * __restrict__ y, int64_t n) {
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x)
        y[i] = make_uint4((unsigned) i, 1, 2, 3);
}
__global__ void k_fill_h(q2a_half * x, int64_t n) {
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        const unsigned h = (unsigned) (i * 2654435761u);
        x[i] = (q2a_half) (((float) (h % 2000) - 1000.f) / 250.f);   // [-4, 4)
    }
}

int main() {
    const int M = 96000, K = 5120, D = 1280;
    const int64_t n = (int64_t) M * K;
    q2a_half *x, *codes;
    float *dy, *xf;
    q2a_half * aext;
    uint16_t * lut;
    unsigned * dummy;
    float *g, *bb;
    hipMalloc(&x, n * 2);
    hipMalloc(&codes, n * 2);
    hipMalloc(&dy, (int64_t) M * (K / 256) * 4 + 4096);
    hipMalloc(&aext, (int64_t) M * (K / 256) * 32 + 4096);
    hipMalloc(&lut, 131072);
    hipMalloc(&dummy, 64);
    hipMalloc(&xf, (int64_t) M * D * 4);
    hipMalloc(&g, D * 4);
    hipMalloc(&bb, D * 4);
    hipMemset(lut, 0, 131072);
    hipMemset(g, 0, D * 4);
    hipMemset(bb, 0, D * 4);
    hipLaunchKernelGGL(k_fill_h, dim3(4096), dim3(256), 0, 0, x, n);
    hipLaunchKernelGGL(k_fill_h, dim3(4096), dim3(256), 0, 0, (q2a_half *) xf, (int64_t) M * D * 2);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char * name, double bytes, auto fn) {
        for (int w = 0; w < 2; ++w) fn();
        hipEventRecord(e0);
        const int reps = 10;
        for (int r = 0; r < reps; ++r) fn();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1000 / reps;
        printf("{\"kernel\": \"%s\", \"us\": %.1f, \"bytes\": %.0f, \"TB_per_s\": %.2f}\n", name, us, bytes, bytes / (us * 1e-6) / 1e12);
    };
    const int64_t n16 = n * 2 / 16;
    for (int grid : {1024, 2048, 8192}) {
        char nm[64];
        snprintf(nm, sizeof nm, "copy 983MB->983MB grid %d", grid);
        timeit(nm, 2.0 * n * 2, [&] { hipLaunchKernelGGL(k_copy16, dim3(grid), dim3(256), 0, 0, (const uint4 *) x, (uint4 *) codes, n16); });
    }
    timeit("read 983MB", 1.0 * n * 2, [&] { hipLaunchKernelGGL(k_read16, dim3(2048), dim3(256), 0, 0, (const uint4 *) x, n16, dummy); });
    timeit("write 983MB", 1.0 * n * 2, [&] { hipLaunchKernelGGL(k_write16, dim3(2048), dim3(256), 0, 0, (uint4 *) codes, n16); });
    const double gq_bytes = n * 2.0 + n * 2.0 + (double) M * (K / 256) * (4 + 32);
    timeit("gelu+q8k (engine)", gq_bytes, [&] { q2a_launch_gelu_quant_q8k(x, M, K, lut, codes, dy, aext, M, 0); });
    q2a_quant_args qa{};
    qa.XH = x; qa.M = M; qa.K = K; qa.mode = 1; qa.outH = codes; qa.dy = dy; qa.aext = aext; qa.dy_ld = M;
    timeit("q8k of fp16 rows (engine)", gq_bytes, [&] { q2a_launch_quant_act(qa, 0); });
    q2a_ln_args la{};
    la.X = xf; la.M = M; la.D = D; la.g = g; la.b = bb; la.mode = 1; la.outH = codes; la.dy = dy; la.aext = aext; la.dy_ld = M;
    const double ln_bytes = (double) M * D * 4 + (double) M * D * 2 + (double) M * (D / 256) * 36;
    timeit("layernorm+q8k (engine)", ln_bytes, [&] { q2a_launch_layernorm(la, 0); });
    q2a_quant_args qf{};
    qf.X = xf; qf.M = M; qf.K = D; qf.mode = 1; qf.outH = codes; qf.dy = dy; qf.aext = aext; qf.dy_ld = M;
    timeit("q8k of f32 rows (attention out, engine)", ln_bytes, [&] { q2a_launch_quant_act(qf, 0); });
    return 0;
}
