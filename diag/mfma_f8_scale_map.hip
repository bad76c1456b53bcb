// Which bytes of the A operand does the A scale of lane group s cover, for v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3)?
// A = 1.0 (e4m3) in one byte position (lane group g, byte j) of every row and 0 elsewhere, B = all 1.0 (operands
// from memory), A scales 2^0 except lane group s (lanes 16s .. 16s+15): 2^1, runtime registers. D[0][0] = 2 when
// group s's scale covers byte (g, j), else 1.
//   hipcc --offload-arch=gfx950 -O2 diag/mfma_f8_scale_map.hip -o diag/f8scale && diag/f8scale
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
__global__ void k_map(const uint8_t * a, const uint8_t * b, const int * sc, float * d) {
    const int l = threadIdx.x;
    v8i av, bv;
    __builtin_memcpy(&av, a + l * 32, 32);
    __builtin_memcpy(&bv, b + l * 32, 32);
    v4f acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 0, 0, 0, sc[l], 0, sc[64 + l]);
    d[l * 4 + 0] = acc[0];
}
int main() {
    uint8_t *da, *db;
    int * ds;
    float * dd;
    if (hipMalloc(&da, 2048) || hipMalloc(&db, 2048) || hipMalloc(&ds, 512) || hipMalloc(&dd, 1024)) return 1;
    uint8_t hb[2048];
    memset(hb, 0x38, sizeof(hb));
    hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
    for (int s = 0; s < 4; ++s) {
        int hs[128];
        for (int l = 0; l < 64; ++l) { hs[l] = (l >> 4) == s ? 128 : 127; hs[64 + l] = 127; }
        hipMemcpy(ds, hs, sizeof(hs), hipMemcpyHostToDevice);
        printf("A scale of lane group %d covers bytes (g,j):", s);
        for (int g = 0; g < 4; ++g)
            for (int j = 0; j < 32; ++j) {
                uint8_t ha[2048];
                memset(ha, 0, sizeof(ha));
                for (int l = 0; l < 64; ++l)
                    if ((l >> 4) == g) ha[l * 32 + j] = 0x38;
                hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
                hipLaunchKernelGGL(k_map, dim3(1), dim3(64), 0, 0, da, db, ds, dd);
                float h;
                hipMemcpy(&h, dd, 4, hipMemcpyDeviceToHost);
                if (h == 2.0f) printf(" %d,%d", g, j);
                else if (h != 1.0f) printf(" ?%d,%d=%g", g, j, h);
            }
        printf("\n");
    }
    return 0;
}
