// op_sel of the scale operands of v_mfma_scale_f32_16x16x128_f8f6f4: A = B = 1.0 (e4m3), A scale 2^0, B scale
// register packed with e8m0 codes (byte 0: 2^0, byte 1: 2^1, byte 2: 2^2, byte 3: 2^3); D = 128 * the selected scale.
//   hipcc --offload-arch=gfx950 -O2 diag/mfma_f8_opsel.hip -o diag/f8opsel && diag/f8opsel
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
template <int SEL>
__global__ void k_sel(float * d) {
    v8i ones;
    for (int i = 0; i < 8; ++i) ones[i] = 0x38383838;
    const int sb = 127 | (128 << 8) | (129 << 16) | (130 << 24);
    v4f acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(ones, ones, acc, 0, 0, 0, 127, SEL, sb);
    if (threadIdx.x == 0) d[SEL] = acc[0];
}
int main() {
    float * dd;
    if (hipMalloc(&dd, 16) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_sel<0>, dim3(1), dim3(64), 0, 0, dd);
    hipLaunchKernelGGL(k_sel<1>, dim3(1), dim3(64), 0, 0, dd);
    hipLaunchKernelGGL(k_sel<2>, dim3(1), dim3(64), 0, 0, dd);
    hipLaunchKernelGGL(k_sel<3>, dim3(1), dim3(64), 0, 0, dd);
    float h[4];
    if (hipMemcpy(h, dd, 16, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    printf("{\"opsel0\": %g, \"opsel1\": %g, \"opsel2\": %g, \"opsel3\": %g, \"expect\": \"128 256 512 1024\"}\n", h[0], h[1], h[2], h[3]);
    return 0;
}
