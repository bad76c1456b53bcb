// q2a_quant.h — device-side activation quantizers shared by the LayerNorm/quantizer kernels and the fused
// GEMM epilogue. Each mirrors the conversion ggml applies to a MUL_MAT src1 on x86:
//   Q8_K: quantize_row_q8_K_ref (ggml-quants.c:3785-3822), used for Q4_K weights
//   Q8_0: the AVX2 branch of quantize_row_q8_0 (ggml-quants.c:943-1000), used for Q8_0 / Q4_0 weights
// Codes are emitted as fp16 (exact small integers) because they feed fp16 MFMA.
#pragma once
#include "q2a_internal.h"

namespace {

// Cross-lane steps of the Q8_K quantizers on the VALU (v_permlane32_swap / v_permlane16_swap, DPP row_ror / quad_perm)
// instead of the LDS pipe (ds_bpermute / ds_swizzle): max and integer sums, exact in any order. A swap of x with
// itself leaves {x, partner} or {partner, x} in the two results, so their max is lane ^ 32 (^ 16) combined with the
// lane. LayerNorm + Q8_K 9.7 -> 9.3 ms per step at 64 clips, bit-identical (diag/gpurun_r06y.sh).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
    return (uint32_t) __builtin_amdgcn_mov_dpp((int) v, CTRL, 0xF, 0xF, false);
}
// row_ror:n — lane i receives lane (i - n) mod 16 of its 16-lane row; quad_perm xor 2 / xor 1
constexpr int DPP_ROR8 = 0x128, DPP_ROR4 = 0x124, DPP_ROR12 = 0x12C, DPP_XOR2 = 0x4E, DPP_XOR1 = 0xB1;

// max over the 64 lanes (exact in any order)
__device__ __forceinline__ float wave_max_f(float x) {
    x = fmaxf(x, __uint_as_float(dpp_u<DPP_ROR8>(__float_as_uint(x))));
    x = fmaxf(x, __uint_as_float(dpp_u<DPP_ROR4>(__float_as_uint(x))));
    x = fmaxf(x, __uint_as_float(dpp_u<DPP_XOR2>(__float_as_uint(x))));
    x = fmaxf(x, __uint_as_float(dpp_u<DPP_XOR1>(__float_as_uint(x))));
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(t[0]), __uint_as_float(t[1]));
}

// The Q8_K scale comes from the signed value of the FIRST element (in row order) whose |x| is the block maximum
// (quantize_row_q8_K_ref's strict '>' scan, :3793-3798). Found in two cheap steps instead of carrying
// (|x|, x, index) through every reduction step: (1) a plain max of |x| over the block's lanes, (2) a ballot of
// the lanes holding an element equal to it — the lowest such lane holds the first occurrence (elements are laid out
// in lane order), and its own first matching element gives the sign. `first_e` = that lane's first index with
// |x| == amax (or 4/16 if none); lane order = element order within the block.
__device__ __forceinline__ float first_max_value(float amax, float local_first, bool has, int lane, int group_lanes) {
    const unsigned long long m = __ballot(has);
    const int g0 = lane & ~(group_lanes - 1);
    const unsigned long long gm = group_lanes == 64 ? m : (m >> g0) & ((1ull << group_lanes) - 1);
    const int src = g0 + (gm ? __builtin_ctzll(gm) : 0);
    const float v = group_lanes == 64 ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(local_first), src))
                                      : __shfl(local_first, src);
    return gm ? v : amax;
}

// quantize one 256-block (one float4 per lane) to Q8_K codes; writes codes, d and the bsum hi/lo operand
__device__ __forceinline__ void quant_q8k_block(float4 y, int lane, q2a_half * codes, float * dy_out, q2a_half * aext) {
    // max |x| and the signed value of its FIRST occurrence (strict '>' scan, :3793-3798)
    float vv[4] = {y.x, y.y, y.z, y.w};
    const float amax = wave_max_f(fmaxf(fmaxf(fabsf(y.x), fabsf(y.y)), fmaxf(fabsf(y.z), fabsf(y.w))));
    float lf = 0.f;
    bool has = false;
    for (int e = 3; e >= 0; --e)
        if (fabsf(vv[e]) == amax) { lf = vv[e]; has = true; }
    const float mx = first_max_value(amax, lf, has, lane, 64);
    int q[4] = {0, 0, 0, 0};
    float d = 1.f;   // all-zero block (ggml stores 0): the codes are 0 so d never contributes; a nonzero d keeps
                     // the block-ratio rescaling of the wide Q4_K GEMM finite
    if (amax != 0.f) {
        const float iscale = -127.f / mx;
        for (int e = 0; e < 4; ++e) q[e] = min(127, (int) rintf(iscale * vv[e]));
        d = 1 / iscale;
    }
    typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
    *(h4_t *) codes = h4_t{(_Float16) (float) q[0], (_Float16) (float) q[1], (_Float16) (float) q[2], (_Float16) (float) q[3]};
    if (lane == 0) *dy_out = d;
    // bsums over 16 = 4 lanes, then bsum32_j = lanes 8j..8j+7
    int s = q[0] + q[1] + q[2] + q[3];
    s += (int) dpp_u<DPP_XOR1>((uint32_t) s);
    s += (int) dpp_u<DPP_XOR2>((uint32_t) s);
    s += (int) dpp_u<DPP_ROR12>((uint32_t) s);   // + lane + 4: lanes 8j now hold lanes 8j .. 8j + 7 (others unused)
    if ((lane & 7) == 0) {
        const int j = lane >> 3;
        const int hi = (s >= 0) ? (s >> 6) : -((-s + 63) >> 6);   // floor(s / 64)
        const int lo = s - 64 * hi;
        aext[2 * j + 0] = (_Float16) (float) hi;
        aext[2 * j + 1] = (_Float16) (float) lo;
    }
}

// quantize one 256-block held by 16 lanes (16 consecutive values per lane; lane group = lane >> 4 = one row):
// same arithmetic as quant_q8k_block, four rows per wave at once. Cross-lane steps stay inside the 16-lane group
// (DPP within the row). codes: this lane's 16 codes; aext: the row's 16-half bsum operand.

// the arithmetic of quant_q8k_row16 with this lane's 16 codes stored (when st) and the block's d and this lane
// PAIR's bsum32 (sub-block sub / 2) returned instead of stored
__device__ __forceinline__ void quant_q8k_row16c(const float (&v)[16], int sub, q2a_half * codes, bool st, float & d_out,
                                                 int & s_out) {
    // this lane's first element of largest |x| (a backward scan keeps the earliest on ties), then the block max
    float lm = v[15];
#pragma unroll
    for (int e = 14; e >= 0; --e) lm = fabsf(v[e]) >= fabsf(lm) ? v[e] : lm;
    float amax = fabsf(lm);
    amax = fmaxf(amax, __uint_as_float(dpp_u<DPP_ROR8>(__float_as_uint(amax))));   // max over the 16-lane row (DPP)
    amax = fmaxf(amax, __uint_as_float(dpp_u<DPP_ROR4>(__float_as_uint(amax))));
    amax = fmaxf(amax, __uint_as_float(dpp_u<DPP_XOR2>(__float_as_uint(amax))));
    amax = fmaxf(amax, __uint_as_float(dpp_u<DPP_XOR1>(__float_as_uint(amax))));
    const int lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const float mx = first_max_value(amax, lm, fabsf(lm) == amax, lane, 16);
    // codes as floats: rint(iscale x) is the reference's MIN(127, nearest_int(.)) value — the MIN never binds:
    // |x| <= |mx| and |iscale| <= (127/|mx|)(1 + 2^-24), so |iscale x| < 127.5. The bsum of 16 codes (|s| <= 2032) is
    // exact in f32. Products two per v_pk_mul_f32.
    typedef float f2_t __attribute__((ext_vector_type(2)));
    float q[16];
    float d = 1.f;   // all-zero block: see quant_q8k_block
    if (amax != 0.f) {
        const float iscale = -127.f / mx;
        const f2_t is2 = {iscale, iscale};
#pragma unroll
        for (int e = 0; e < 16; e += 2) {
            const f2_t y = is2 * f2_t{v[e], v[e + 1]};
            q[e] = rintf(y[0]);
            q[e + 1] = rintf(y[1]);
        }
        d = 1 / iscale;
    } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) q[e] = 0.f;
    }
    typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
    h8_t c0, c1;
#pragma unroll
    for (int e = 0; e < 8; ++e) { c0[e] = (_Float16) q[e]; c1[e] = (_Float16) q[8 + e]; }
    if (st) {
        *(h8_t *) codes = c0;
        *(h8_t *) (codes + 8) = c1;
    }
    f2_t s2 = {0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 16; e += 2) s2 = s2 + f2_t{q[e], q[e + 1]};
    int s = (int) (s2[0] + s2[1]);
    s += (int) dpp_u<DPP_XOR1>((uint32_t) s);                  // bsum32 of sub-block j = sub / 2
    d_out = d;
    s_out = s;
}

__device__ __forceinline__ void quant_q8k_row16(const float (&v)[16], int sub, q2a_half * codes, float * dy_out,
                                                q2a_half * aext) {
    float d;
    int s;
    quant_q8k_row16c(v, sub, codes, true, d, s);
    if (sub == 0) *dy_out = d;
    if ((sub & 1) == 0) {
        const int hi = (s >= 0) ? (s >> 6) : -((-s + 63) >> 6);   // floor(s / 64)
        const int lo = s - 64 * hi;
        typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
        *(h2_t *) (aext + sub) = h2_t{(_Float16) (float) hi, (_Float16) (float) lo};
    }
}

// NB independent 256-blocks, one float4 per lane each (block u = lanes 0..63 x 4 of y[u]): quant_q8k_block's
// arithmetic with the NB reduction chains interleaved (the LayerNorm kernel's row is NB = D/256 blocks)
template <int NB>
__device__ __forceinline__ void quant_q8k_blocks(const float4 (&y)[NB], int lane, q2a_half * codes, int64_t code_stride,
                                                 float * dy_out, int64_t dy_stride, q2a_half * aext, int64_t aext_stride) {
    float amax[NB], mx[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) amax[u] = fmaxf(fmaxf(fabsf(y[u].x), fabsf(y[u].y)), fmaxf(fabsf(y[u].z), fabsf(y[u].w)));
#pragma unroll
    for (int u = 0; u < NB; ++u) amax[u] = wave_max_f(amax[u]);
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const float vv[4] = {y[u].x, y[u].y, y[u].z, y[u].w};
        float lf = 0.f;
        bool has = false;
#pragma unroll
        for (int e = 3; e >= 0; --e)
            if (fabsf(vv[e]) == amax[u]) { lf = vv[e]; has = true; }
        mx[u] = first_max_value(amax[u], lf, has, lane, 64);
    }
    int s[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const float vv[4] = {y[u].x, y[u].y, y[u].z, y[u].w};
        int q[4] = {0, 0, 0, 0};
        float d = 1.f;   // all-zero block: see quant_q8k_block
        if (amax[u] != 0.f) {
            const float iscale = -127.f / mx[u];
#pragma unroll
            for (int e = 0; e < 4; ++e) q[e] = min(127, (int) rintf(iscale * vv[e]));
            d = 1 / iscale;
        }
        typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
        *(h4_t *) (codes + u * code_stride) = h4_t{(_Float16) (float) q[0], (_Float16) (float) q[1], (_Float16) (float) q[2], (_Float16) (float) q[3]};
        if (lane == 0) dy_out[u * dy_stride] = d;
        s[u] = q[0] + q[1] + q[2] + q[3];
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) s[u] += (int) dpp_u<DPP_XOR1>((uint32_t) s[u]);
#pragma unroll
    for (int u = 0; u < NB; ++u) s[u] += (int) dpp_u<DPP_XOR2>((uint32_t) s[u]);
#pragma unroll
    for (int u = 0; u < NB; ++u) s[u] += (int) dpp_u<DPP_ROR12>((uint32_t) s[u]);   // + lane + 4: lanes 8j: their 8 lanes
    if ((lane & 7) == 0) {
        const int j = lane >> 3;
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int hi = (s[u] >= 0) ? (s[u] >> 6) : -((-s[u] + 63) >> 6);   // floor(s / 64)
            const int lo = s[u] - 64 * hi;
            typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
            *(h2_t *) (aext + u * aext_stride + 2 * j) = h2_t{(_Float16) (float) hi, (_Float16) (float) lo};
        }
    }
}

// quantize one 32-block (8 lanes x float4) to Q8_0 codes with the x86 AVX2 semantics
__device__ __forceinline__ void quant_q80_block(float4 y, int lane, q2a_half * codes, float * dy_out) {
    float amax = fmaxf(fmaxf(fabsf(y.x), fabsf(y.y)), fmaxf(fabsf(y.z), fabsf(y.w)));
    amax = fmaxf(amax, __shfl_xor(amax, 1));
    amax = fmaxf(amax, __shfl_xor(amax, 2));
    amax = fmaxf(amax, __shfl_xor(amax, 4));
    const float d = amax / 127.f;
    const float id = (amax != 0.0f) ? 127.f / amax : 0.0f;
    codes[0] = (_Float16) rintf(y.x * id);
    codes[1] = (_Float16) rintf(y.y * id);
    codes[2] = (_Float16) rintf(y.z * id);
    codes[3] = (_Float16) rintf(y.w * id);
    if ((lane & 7) == 0) *dy_out = (float) (_Float16) d;    // block d is stored as fp16 (GGML_FP32_TO_FP16)
}

// Rows are [M*nseg][D] (a quantizer run splits a long row into nseg segments of D); the block scales are
// written block-major: block bf of logical row m (= row / nseg) goes to dy[bf * ld + m] (aext likewise x16).

}  // namespace
