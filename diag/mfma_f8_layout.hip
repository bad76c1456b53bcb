// Lane layout probe for v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 operands, e8m0 scales) with exact small-integer data
// (cdna_hip_programming.md: "check the map with exact integer data before relying on it"). For each hypothesis of
// the A / B K mapping the kernel's D is compared with the CPU product; also checks v_cvt_pk_fp8_f32's encoding.
//   hipcc --offload-arch=gfx950 -O2 diag/mfma_f8_layout.hip -o /tmp/f8probe && /tmp/f8probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void k_probe(const uint8_t * a, const uint8_t * b, float * d, int sa, int sb, int * cvt) {
    const int l = threadIdx.x;
    if (sa < 0) sa = 127 + (l >> 4);   // per-lane scales: lane group g scales its 32 A values by 2^g
    v8i av, bv;
    __builtin_memcpy(&av, a + l * 32, 32);
    __builtin_memcpy(&bv, b + l * 32, 32);
    v4f acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 0, 0, 0, sa, 0, sb);
    for (int i = 0; i < 4; ++i) d[l * 4 + i] = acc[i];
    if (l == 0) {
        cvt[0] = __builtin_amdgcn_cvt_pk_fp8_f32(1.0f, 2.0f, 0, false);
        cvt[1] = __builtin_amdgcn_cvt_pk_fp8_f32(-0.75f, 448.0f, 0, false);
        cvt[2] = __builtin_amdgcn_cvt_pk_fp8_f32(0.0625f, 1.0f / 512.0f, 0, false);
    }
}

static uint8_t e4m3(int v) {   // small integers -4..4 -> OCP e4m3fn bits
    if (v == 0) return 0;
    const uint8_t s = v < 0 ? 0x80 : 0;
    int m = v < 0 ? -v : v;
    int e = 0;
    while ((1 << (e + 1)) <= m) ++e;
    const int frac = ((m << 3) >> e) & 7;   // 3 mantissa bits
    return s | (uint8_t) (((e + 7) << 3) | frac);
}

int main() {
    int A[16][128], B[128][16];
    uint32_t st = 12345;
    auto rnd = [&]() { st = st * 1664525u + 1013904223u; return (int) ((st >> 20) % 9) - 4; };
    for (int r = 0; r < 16; ++r)
        for (int k = 0; k < 128; ++k) A[r][k] = rnd();
    for (int k = 0; k < 128; ++k)
        for (int c = 0; c < 16; ++c) B[k][c] = rnd();
    double ref[16][16];
    for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
            double s = 0;
            for (int k = 0; k < 128; ++k) s += (double) A[r][k] * B[k][c];
            ref[r][c] = s;
        }
    uint8_t *da, *db;
    float * dd;
    int * dc;
    hipMalloc(&da, 64 * 32); hipMalloc(&db, 64 * 32); hipMalloc(&dd, 64 * 4 * 4); hipMalloc(&dc, 16);
    // hypotheses: lane l = row (l & 15), group g = l >> 4, byte j of the lane's 32 -> k
    auto kmap = [](int hyp, int g, int j) {
        if (hyp == 0) return 32 * g + j;                                   // contiguous 32 per group
        if (hyp == 1) return j < 16 ? 16 * g + j : 64 + 16 * g + (j - 16);  // two 16-byte halves
        if (hyp == 2) return 8 * g + (j & 7) + 32 * (j >> 3);               // 8-byte interleave
        return 4 * g + (j & 3) + 16 * (j >> 2);                             // 4-byte interleave
    };
    for (int hyp = 0; hyp < 4; ++hyp) {
        uint8_t ha[64 * 32], hb[64 * 32];
        for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 32; ++j) {
                const int k = kmap(hyp, l >> 4, j);
                ha[l * 32 + j] = e4m3(A[l & 15][k]);
                hb[l * 32 + j] = e4m3(B[k][l & 15]);
            }
        hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
        hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
        for (int sc = 0; sc < 3; ++sc) {
            const int sa = sc == 2 ? -1 : sc ? 128 : 127, sb = 127;   // e8m0: 127 = 2^0, 128 = 2^1; -1: per lane group
            hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, da, db, dd, sa, sb, dc);
            float hd[256];
            hipMemcpy(hd, dd, sizeof(hd), hipMemcpyDeviceToHost);
            double err = 0;
            for (int l = 0; l < 64; ++l)
                for (int i = 0; i < 4; ++i) {
                    const int col = l & 15, row = 4 * (l >> 4) + i;
                    double want = (sc ? 2.0 : 1.0) * ref[row][col];
                    if (sc == 2) {   // per-group scale 2^g on the A values the hypothesis puts in group g
                        want = 0;
                        for (int k = 0; k < 128; ++k) {
                            int g = -1;
                            for (int gg = 0; gg < 4 && g < 0; ++gg)
                                for (int j = 0; j < 32; ++j)
                                    if (kmap(hyp, gg, j) == k) { g = gg; break; }
                            want += ldexp((double) A[row][k] * B[k][col], g);
                        }
                    }
                    err = fmax(err, fabs(hd[l * 4 + i] - want));
                }
            printf("{\"hypothesis\": %d, \"scale_a\": %d, \"max_abs_err\": %g}\n", hyp, sa, err);
        }
    }
    int cv[3];
    hipMemcpy(cv, dc, 12, hipMemcpyDeviceToHost);
    printf("{\"cvt_pk_fp8(1,2)\": \"0x%04x\", \"cvt(-0.75,448)\": \"0x%04x\", \"cvt(1/16,1/512)\": \"0x%04x\", \"expect\": \"0x4038, 0x7eb4, 0x0118\"}\n",
           cv[0] & 0xffff, cv[1] & 0xffff, cv[2] & 0xffff);
    return 0;
}
