// Which bytes of the A operand does lane L's scale byte apply to, for v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3)?
// A = one nonzero byte position (lane group g, byte j) of 1.0 in every row, B = all 1.0, every scale 2^0 except the
// A scales of lane group s (lanes 16s .. 16s+15): 2^1. D[0][0] is then 2 when group s's scale covers (g, j), else 1.
//   hipcc --offload-arch=gfx950 -O2 diag/mfma_f8_scale_map.hip -o diag/f8scale && diag/f8scale
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
__global__ void k_map(float * d, int g0, int j0, int sgrp) {
    const int l = threadIdx.x;
    v8i a, ones;
    for (int i = 0; i < 8; ++i) { ones[i] = 0x38383838; a[i] = 0; }
    if ((l >> 4) == g0) a[j0 >> 2] = 0x38 << (8 * (j0 & 3));
    const int s = (l >> 4) == sgrp ? 128 : 127;
    v4f acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, ones, acc, 0, 0, 0, s, 0, 127);
    if (l == 0) d[0] = acc[0];
}
int main() {
    float * dd;
    if (hipMalloc(&dd, 64) != hipSuccess) return 1;
    for (int sgrp = 0; sgrp < 4; ++sgrp) {
        printf("scale of lane group %d covers (g,j):", sgrp);
        for (int g = 0; g < 4; ++g)
            for (int j = 0; j < 32; ++j) {
                hipLaunchKernelGGL(k_map, dim3(1), dim3(64), 0, 0, dd, g, j, sgrp);
                float h;
                if (hipMemcpy(&h, dd, 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
                if (h == 2.0f) printf(" %d,%d", g, j);
                else if (h != 1.0f) printf(" ?%d,%d=%g", g, j, h);
            }
        printf("\n");
    }
    return 0;
}
