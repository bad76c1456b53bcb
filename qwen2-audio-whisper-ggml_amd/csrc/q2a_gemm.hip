// q2a_gemm.hip — fused weight GEMM for gfx950: C[M][N] = A[M][K] . W[N][K]^T on fp16 MFMA
// (v_mfma_f32_16x16x32_f16, fp32 accumulation) with the reference's per-op epilogues fused in.
//
// Reference ops replaced: MUL_MAT (ggml_compute_forward_mul_mat ggml.c:12439-12652) plus the
// ADD (bias / residual), SCALE (Q*1/8), GELU, CONT/permute nodes around it (qwen2-whisper.cpp:2029-2154) and the
// IM2COL+MUL_MAT conv pair (ggml_conv_1d ggml.c:6635-6652, as an implicit GEMM with overlapping A rows).
//
// Exactness: every A/W operand fed here is exactly representable in fp16 (ggml rounds activations to fp16 for
// F16 weights; Q8_K/Q8_0 codes and sc*q weight products are small integers), products are exact in fp32 and
// only the fp32 summation order differs from ggml. For the k-quant formats the integer per-block sums are kept
// in a fresh accumulator per K-block and combined with ggml's scale formula (ggml-quants.c:7795-7858).
//
// Tiling (template): BM x BN x 64 per workgroup of WM x WN waves; each wave owns a (BM/WM) x (BN/WN) block of
// 16x16 MFMA tiles. Large batches use 256x256 tiles with 8 waves (128x64 per wave: each A fragment feeds 4 MFMAs,
// each W fragment 8), small ones 128x128 with 4 waves. LDS operand images are filled by global_load_lds_dwordx4
// (16 B/lane, lane-linear destination) with the XOR swizzle applied on the global SOURCE address and undone on the
// ds_read (cdna_hip_programming.md §5.4 rule 21); two LDS stages, the next stage's loads issued before the MFMAs
// of the current one. Workgroups are remapped XCD-contiguously (bijective) and rasterised in groups of 8 M-tiles
// per N column so the tiles resident on one XCD share A and W panels through its L2.
#include "q2a_internal.h"
#include "q2a_quant.h"

#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void * lds_ptr_t;

// timing diagnostic Q2A_DIAG_NO_STORE (wrong results): the epilogue computes every value but its global stores
// are predicated off by a condition the compiler cannot fold
#ifdef Q2A_DIAG_NO_STORE
#define Q2A_ST (p.K < 0)
#else
#define Q2A_ST true
#endif

// epilogue global store (round 1 measured non-temporal stores +22 ms/step: plain stores)
template <class V>
__device__ __forceinline__ void q2a_st(const V & v, V * ptr) {
    *ptr = v;
}

// Schedule decisions of the 8-phase kernel, measured (the rejected alternatives' code is in
// diag/experiment_knobs_r05.patch; DESIGN.md §4-§5 has the numbers):
//   * fp16 outputs (fc1 pre-activation, Q / K hi|lo) staged through LDS and stored as whole 512-B rows;
//   * fc1 (Q4_K pre-activation) on persistent tiles whose epilogue stores retire under the next tile (round 4,
//     diag/gpurun_r04d.sh: 1.268 against 1.341 ms per launch, outputs bit-identical);
//   * waves 4-7 one barrier behind waves 0-3 (round 4, diag/gpurun_r04b.sh: fc1 tile 98.0k -> 82.4k cycles, every
//     weight GEMM 4-7 % faster);
//   * not adopted: glds issued inside the MFMA segments, two phases of 32 MFMAs per K-step (round 5, 1-3 ms per step
//     slower), the alternating quadrant order (r05h: Q4_K +2-4 %, spills), fragment reads before the Q4_K block start
//     (r05r: neutral); the conv GEMMs' 128x128 / more-stage exact tiles (r04m).

// Timing diagnostic Q2A_DIAG_STAMPS=<epi>: the 8-phase kernels of epilogue <epi> record s_memtime at fixed points of
// every workgroup's tile (waves 0 and 4, lane 0) into g_q2a_stamps, read back by q2a_diag_stamps (diag/tile_stamps.py):
// 0 entry | 1 prologue landed | 2 main loop end | 3 final multiply done | 4 epilogue staged | 5 stores issued |
// 6 stores drained | 7 sum of the Q4_K block starts | 8 / 9 s_memrealtime at entry / end (100 MHz). Never in libq2a.so.
#ifdef Q2A_DIAG_STAMPS
constexpr int Q2A_STAMP_SLOTS = 16;
__device__ uint64_t g_q2a_stamps[16384 * 2 * Q2A_STAMP_SLOTS];
__device__ __forceinline__ void q2a_stamp_put(int k, uint64_t v) {
    if ((threadIdx.x & 255) == 0) g_q2a_stamps[((int64_t) blockIdx.x * 2 + (threadIdx.x >> 8)) * Q2A_STAMP_SLOTS + k] = v;
}
#define Q2A_STAMP(ON, k) do { if (ON) q2a_stamp_put((k), __builtin_amdgcn_s_memtime()); } while (0)
#define Q2A_STAMP_RT(ON, k) do { if (ON) q2a_stamp_put((k), __builtin_amdgcn_s_memrealtime()); } while (0)
#else
#define Q2A_STAMP(ON, k) do { } while (0)
#define Q2A_STAMP_RT(ON, k) do { } while (0)
#endif

constexpr int BK = 64;
constexpr int ROWB = BK * 2;   // bytes per LDS row (64 halves)
constexpr int GROUP_M = 4;   // swept 2..32 at the batched shapes (round 1): 4 best by ~1 %

__device__ __forceinline__ float gelu_lut(float x, const uint16_t * tab) {
    // ggml_vec_gelu_f32 with GGML_GELU_FP16 (ggml.c:2556-2570). The table read is unconditional (every fp16 bit
    // pattern indexes the 64 Ki-entry table) and the two range branches are selects: a lookup inside the branches
    // compiled to a load + vmcnt(0) per element, the epilogue's lookups one serial round trip each
    const _Float16 h = (_Float16) x;
    uint16_t u;
    __builtin_memcpy(&u, &h, 2);
    const uint16_t g = __ldg(tab + u);
    _Float16 gh;
    __builtin_memcpy(&gh, &g, 2);
    return x <= -10.0f ? 0.0f : x >= 10.0f ? x : (float) gh;
}

// same lookup against the compact |x| <= 10 table staged in LDS, result as fp16 (it is fp16 by construction)
__device__ __forceinline__ _Float16 gelu_lut_c16(float x, const uint16_t * lut) {
    const _Float16 h = (_Float16) x;
    uint16_t u;
    __builtin_memcpy(&u, &h, 2);
    const uint16_t g = lut[(u & 0x7FFF) + ((u & 0x8000) ? Q2A_GELU_C_HALF : 0)];
    _Float16 gh;
    __builtin_memcpy(&gh, &g, 2);
    return x <= -10.0f ? (_Float16) 0.0f : x >= 10.0f ? h : gh;
}

// 8 lookups of gelu_lut_c16 issued back to back behind ONE wait. A compiler-visible lookup is sunk into the branch of
// the |x| >= 10 select, each followed by its own lgkmcnt(0): 8 dependent LDS round trips instead of one. The index is
// clamped into the table so the read is unconditional (the select discards it outside |x| < 10).
__device__ __forceinline__ void gelu_c16_x8(const float (&x)[8], _Float16 (&y)[8], const uint16_t * lut) {
    const uint32_t lut0 = (uint32_t) (uintptr_t) (const __attribute__((address_space(3))) uint16_t *) lut;
    uint32_t g[8];
    _Float16 h[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        h[e] = (_Float16) x[e];
        uint16_t u;
        __builtin_memcpy(&u, &h[e], 2);
        const uint32_t idx = min((uint32_t) (u & 0x7FFF), (uint32_t) (Q2A_GELU_C_HALF - 1)) + ((u & 0x8000) ? Q2A_GELU_C_HALF : 0);
        asm volatile("ds_read_u16 %0, %1" : "=v"(g[e]) : "v"(lut0 + idx * 2) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(g[0]), "+v"(g[1]), "+v"(g[2]), "+v"(g[3]), "+v"(g[4]), "+v"(g[5]), "+v"(g[6]),
                 "+v"(g[7]) :: "memory");
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const uint16_t gg = (uint16_t) g[e];
        _Float16 gh;
        __builtin_memcpy(&gh, &gg, 2);
        y[e] = x[e] <= -10.0f ? (_Float16) 0.0f : x[e] >= 10.0f ? h[e] : gh;
    }
}

// (unconditional read at a clamped index + selects, like gelu_lut: inside the range branches each read waited alone)
__device__ __forceinline__ float gelu_lut_c(float x, const uint16_t * lut) {
    const _Float16 h = (_Float16) x;
    uint16_t u;
    __builtin_memcpy(&u, &h, 2);
    const uint16_t g = lut[min((uint32_t) (u & 0x7FFF), (uint32_t) (Q2A_GELU_C_HALF - 1)) + ((u & 0x8000) ? Q2A_GELU_C_HALF : 0)];
    _Float16 gh;
    __builtin_memcpy(&gh, &g, 2);
    return x <= -10.0f ? 0.0f : x >= 10.0f ? x : (float) gh;
}

// Q4_K block-ratio accumulation (every Q4_K kernel, 8-phase and small-tile, runs exactly these float operations in
// the same order, so a clip's outputs do not depend on the tile regime its batch size selects):
//   block start  acc <- fma(acc, alpha[m] * beta[n], ngamma[n] * S2[m][n])   (ngamma = -dmin/dx, stored negated:
//                the product's sign flip is exact, and no per-element negation is issued)
//   block body   acc += the block's MFMAs (exact integer products, K order fixed by the 64-deep K-steps)
//   after last   acc * (dy_last[m] * dx_last[n])
__device__ __forceinline__ float kq_rescale(float a, float al, float be, float nga, float s2) {
#pragma clang fp contract(off)
    const float t = al * be;
    const float u = nga * s2;
    return __builtin_fmaf(a, t, u);
}
// kq_rescale on elements 2h, 2h + 1 of an accumulator float4 (same IEEE operations, two lanes per packed op)
__device__ __forceinline__ void kq_rescale2(f4 & a, int h, float al, const f4 & be, const f4 & nga, const f4 & s2) {
#pragma clang fp contract(off)
    const f2 a2 = {a[2 * h], a[2 * h + 1]};
    const f2 t = f2{al, al} * f2{be[2 * h], be[2 * h + 1]};
    const f2 u = f2{nga[2 * h], nga[2 * h + 1]} * f2{s2[2 * h], s2[2 * h + 1]};
    const f2 r = __builtin_elementwise_fma(a2, t, u);
    a[2 * h] = r[0];
    a[2 * h + 1] = r[1];
}
// block 0 of the recurrence: acc is 0, so kq_rescale2 reduces to its second product (fma(0, t, u) = u exactly)
__device__ __forceinline__ void kq_first2(f4 & a, int h, const f4 & nga, const f4 & s2) {
    const f2 u = f2{nga[2 * h], nga[2 * h + 1]} * f2{s2[2 * h], s2[2 * h + 1]};
    a[2 * h] = u[0];
    a[2 * h + 1] = u[1];
}
__device__ __forceinline__ float kq_final(float a, float yc, float dx) {
#pragma clang fp contract(off)
    const float t = yc * dx;
    return a * t;
}
__device__ __forceinline__ float kq_alpha(float yp, float yc) { return yp * __builtin_amdgcn_rcpf(yc); }

__device__ __forceinline__ int64_t a_row_off(const q2a_gemm_args & p, int m) {
    return ((int64_t) (m / p.a_rpg) * p.a_gstride + (int64_t) (m % p.a_rpg) * p.a_step) * p.lda;
}

// one 16x16x32 MFMA on fp16 operands, or on the same bits read as bf16 (bf16-activation mode)
template <bool BF>
__device__ __forceinline__ f4 mma16(half8 a, half8 b, f4 c) {
    if constexpr (BF) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, a), __builtin_bit_cast(bf8, b), c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// 16-bit activation store: fp16 RNE, or bf16 RNE in the bf16-activation mode (bits in a _Float16 slot)
template <bool BF>
__device__ __forceinline__ _Float16 to16(float v) {
    if constexpr (BF) return __builtin_bit_cast(_Float16, (__bf16) v);
    else return (_Float16) v;
}

__device__ __forceinline__ half8 frag(const char * img, int row, int chunk) {
    return *(const half8 *) (img + row * ROWB + ((chunk ^ (row & 7)) << 4));
}

// ---- 8-phase pipelined main loop (256x256 tile, 8 waves as 2(M) x 4(N), 128x64 per wave).
// LDS holds 8 half-tile images of 128 rows x 64 K (16 KiB each): two K-step buffers E/O x {A_q0, A_q1, B_q0, B_q1}
// where A_qX = the X-th 64-row half of each M-wave's 128 rows and B_qX = the X-th 32-column half of each N-wave's
// 64 columns, so a wave's output quadrant (qm, qn) reads exactly A_q{qm} and B_q{qn}. One K-step = 4 phases, one
// quadrant each (16 MFMAs); every phase issues one half-tile of glds (2 instructions per thread) and waits with a
// counted vmcnt, so five phases of loads stay in flight across the raw barriers: a staged image is first read six
// phases after its issue, and each slot is restaged the phase after its last read ("GEMM pipeline").
//
// BLK = 256 (Q4_K weights x Q8_K activations) keeps ONE accumulator per output in units of the current block's
// scale u_b = dy_b[m] * dx_b[n]: at the start of block b, acc <- acc * (dy_{b-1}/dy_b)[m] * (dx_{b-1}/dx_b)[n]
// - (dmin_b/dx_b)[n] * S2_b (the min term, one 16x16x16 MFMA on the (hi,lo)-split bsums), then the block's MFMAs
// add its exact integer sum; after the last block acc * u_last. Algebraically ggml's sum_b (d*isum - dmin*summs)
// (ggml-quants.c:7795-7858); the per-block separation of the integer sums is kept, only the fp32 combination
// order differs. The 21 KiB of block scales are staged by glds once per block (phase 2), with the vmcnt counts of
// the following five phases raised by those 3 instructions. Zero scales never occur (quantizers store d = 1 for
// an all-zero activation block, the pack stores dx = 1 and zero weights for a d = 0 weight block).
constexpr int SBUF_OFF = 8 * 128 * ROWB;     // 128 KiB: scale staging after the 8 operand images
constexpr int SBUF_BYTES = 25 * 1024;       // 21 pieces of 1 KiB (+3 pad slots for the uniform 3 glds per thread)
constexpr int ALPHA_OFF = 24 * 1024;        //   + alpha = dy_{b-1}/dy_b per tile row (1 KiB), computed a block ahead

// PERS = 1: the persistent form (k_gemm<..., PIPE = 2>): the workgroup walks a sequence of tiles (next(m0, n0) gives the
// next one, false at the end) and runs the K-step pipeline ACROSS tile boundaries — the last block's tail stages load
// the next tile's first two K-steps and its phase-2 scale pieces the next tile's block-0 scales, while the finishing
// tile's final-multiply and bias operands go to a separate 3 KiB area (FIN_OFF) — then calls epi(m0, n0) for the
// finished tile, whose global stores (S_EPI per wave) retire under the next tile's first five phases: their counted
// vmcnt waits are raised by S_EPI, so nothing drains between tiles.
constexpr int FIN_OFF = SBUF_OFF + 21 * 1024;   // dy_last | dx_last | bias of the finishing tile (persistent form): the
                                                //   three pad pieces' slots, which every other block fills with dummies
// (S_EPI = 16 * PERS global stores per wave of the persistent epilogue: 16 for fc1's fp16 pre-activation, 32 for the
// Q|K|V hi and lo images)
struct no_tiles {
    __device__ bool operator()(int &, int &) const { return false; }
};
struct no_epi {
    __device__ void operator()(f4 (&)[8][4], int, int) const {}
};
template <int BLK, bool LUT, bool BF, bool ST = false, int PERS = 0, class NEXT = no_tiles, class EPIF = no_epi>
__device__ __forceinline__ void mainloop_8phase(const q2a_gemm_args & p, f4 (&acc)[8][4], char * lds_raw, int m0, int n0,
                                                int lane, int wave, int wm, int wn, NEXT next = NEXT{}, EPIF epi = EPIF{}) {
    constexpr int HT = 128 * ROWB;                        // one half-tile image (16 KiB)
    // per-lane element offsets of this thread's two glds rows in each image (image row ir = i*64 + wave*8 + lane/8)
    uint32_t aoff[2][2], woff[2][2];
    auto set_offsets = [&](int tm0, int tn0) {
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int ir = i * 64 + wave * 8 + (lane >> 3);
                const int sw = ((lane & 7) ^ (ir & 7)) << 3;
                const int am = tm0 + (ir >> 6) * 128 + x * 64 + (ir & 63);
                aoff[x][i] = (uint32_t) (a_row_off(p, min(am, p.M - 1)) + sw);
                const int wr = tn0 + (ir >> 5) * 64 + x * 32 + (ir & 31);
                woff[x][i] = (uint32_t) ((int64_t) wr * p.ldw + sw);
            }
    };
    set_offsets(m0, n0);
    const int nk = p.K / BK;
    // image h of buffer b: h = 0 A_q0, 1 A_q1, 2 B_q0, 3 B_q1
    auto stage = [&](int b, int h, int kt) {
        const int k0 = kt * BK;
        char * dst = lds_raw + (b * 4 + h) * HT + wave * 8 * ROWB;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            uint32_t o = h < 2 ? aoff[h][i] : woff[h - 2][i];
            asm volatile("" : "+v"(o));                    // 32-bit offset kept; the 64-bit address is formed here
            const q2a_half * src = (h < 2 ? p.A : p.W) + o + k0;
            __builtin_amdgcn_global_load_lds((const void *) src, (lds_ptr_t) (dst + i * 64 * ROWB), 16, 0, 0);
        }
    };
    // the last iteration's stages past the end of K: slots 0..4 receive the compact GELU table for the epilogue
    // lookups when it needs one, everything else a harmless re-load of the last K-step (keeps the vmcnt counts)
    auto stage_tail = [&](int b, int h) {
        if (LUT && b * 4 + h < 5) {
            char * dst = lds_raw + (b * 4 + h) * HT + wave * 8 * ROWB;
            uint32_t l16 = lane * 16;
            asm volatile("" : "+v"(l16));
            const char * src = (const char *) p.gelu_c + (b * 4 + h) * HT + wave * 8 * ROWB + l16;
#pragma unroll
            for (int i = 0; i < 2; ++i)
                __builtin_amdgcn_global_load_lds((const void *) (src + i * 64 * ROWB), (lds_ptr_t) (dst + i * 64 * ROWB), 16, 0, 0);
        } else {
            stage(b, h, nk - 1);
        }
    };
    // block scales of Q4_K block kb -> LDS pieces: 0 dy_{kb-1} | 1 dy_kb | 2 beta | 3 gamma | 4 dx | 5-12 aext | 13-20 wext
    char * sbuf = lds_raw + SBUF_OFF;
    // this wave's three pieces: wave-uniform base/stride per piece (SGPRs), picked once
    const char * sb_base[3];
    int sb_stride[3];
    bool sb_prev[3];
    auto set_scale_bases = [&](int tm0, int tn0) {
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int pc = wave * 3 + u;
            sb_prev[u] = pc == 0;
            if (pc <= 1 || pc >= 21) { sb_base[u] = (const char *) (p.dy + tm0); sb_stride[u] = p.dy_ld * 4; }
            else if (pc == 2) { sb_base[u] = (const char *) (p.beta + tn0); sb_stride[u] = p.N * 4; }
            else if (pc == 3) { sb_base[u] = (const char *) (p.gamma + tn0); sb_stride[u] = p.N * 4; }
            else if (pc == 4) { sb_base[u] = (const char *) (p.dx + tn0); sb_stride[u] = p.N * 4; }
            else if (pc < 13) { sb_base[u] = (const char *) (p.aext + (int64_t) tm0 * 16) + (pc - 5) * 1024; sb_stride[u] = p.dy_ld * 32; }
            else { sb_base[u] = (const char *) (p.wext + (int64_t) tn0 * 16) + (pc - 13) * 1024; sb_stride[u] = p.N * 32; }
        }
    };
    set_scale_bases(m0, n0);
    auto stage_scales = [&](int kb) {
        kb = min(kb, p.K / 256 - 1);
        uint32_t l16 = lane * 16;
        asm volatile("" : "+v"(l16));                      // per-lane part added at the use: no hoisted 64-bit VGPR pointers
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int k = sb_prev[u] ? max(kb - 1, 0) : kb;
            const char * src = sb_base[u] + (int64_t) k * sb_stride[u] + l16;   // (64-bit product: aext strides reach 2^31)
            __builtin_amdgcn_global_load_lds((const void *) src, (lds_ptr_t) (sbuf + (wave * 3 + u) * 1024), 16, 0, 0);
        }
    };
    // persistent form, phase 2 of a tile's last block: the three pad pieces (wave 7) carry the finishing tile's
    // dy_last, dx_last and bias into FIN_OFF; the 21 real pieces carry the next tile's block-0 scales (or, for the
    // workgroup's last tile, the current block again) — same 3 glds per wave as every block
    // sources of those three glds, worked out in scalar registers before the last block starts (an address formed
    // inside the K-step would hold VGPRs at the loop's register peak)
    const char * sl_src[3];
    auto prep_scales_last = [&](bool has_next, int tm0, int tn0) {
        const int nkb = p.K / 256;
        const int kb = has_next ? 0 : nkb - 1;
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int pc = wave * 3 + u;
            if (pc >= 21) {   // the finishing tile's final-multiply / bias operands
                sl_src[u] = pc == 21 ? (const char *) (p.dy + (int64_t) (nkb - 1) * p.dy_ld + m0)
                          : pc == 22 ? (const char *) (p.dx + (int64_t) (nkb - 1) * p.N + n0)
                                     : (const char *) (p.bias + n0);
            } else {
                // this piece's bytes per tile row / column: the base moves to the next tile in scalar arithmetic
                // (the current tile's last-block scales were staged one block ago)
                if (has_next) {
                    const int mc = pc <= 1 ? 4 : (pc >= 5 && pc < 13) ? 32 : 0;
                    const int nc = (pc >= 2 && pc <= 4) ? 4 : pc >= 13 ? 32 : 0;
                    sb_base[u] += (int64_t) (tm0 - m0) * mc + (int64_t) (tn0 - n0) * nc;
                }
                sl_src[u] = sb_base[u] + (int64_t) (sb_prev[u] ? max(kb - 1, 0) : kb) * sb_stride[u];
            }
            asm volatile("" : "+s"(sl_src[u]));
        }
    };
    auto stage_scales_last = [&]() {
        uint32_t l16 = lane * 16;
        asm volatile("" : "+v"(l16));
#pragma unroll
        for (int u = 0; u < 3; ++u)
            __builtin_amdgcn_global_load_lds((const void *) (sl_src[u] + l16), (lds_ptr_t) (sbuf + (wave * 3 + u) * 1024), 16, 0, 0);
    };
    // start of block kb: acc <- acc * alpha[m] * beta[n] + ngamma[n] * S2[m][n]
    // LDS reads below go through integer AS3 addresses (no IR link to the glds destination array): hipcc would
    // otherwise guard each read of the scale buffer with a vmcnt(0) that drains the whole pipeline
    typedef const __attribute__((address_space(3))) float * lds_fp;
    typedef const __attribute__((address_space(3))) f4 * lds_f4p;
    const uint32_t lds0 = (uint32_t) (uintptr_t) (const __attribute__((address_space(3))) char *) lds_raw;
    const uint32_t sb0 = lds0 + SBUF_OFF;
    // start of block kb: acc <- acc * alpha[m] * beta[n] + ngamma[n] * S2[m][n]. The scale-buffer reads are inline
    // asm with an explicit lgkmcnt wait tied to their results: a compiler-visible LDS read of this array gets a
    // vmcnt(0) guard against the in-flight glds that would drain the whole pipeline once per block.
    // alpha for this wave's 32 rows of the tile into the alpha array (the block's scales must be resident)
    auto alpha_compute = [&]() {
        const uint32_t row = (uint32_t) (wave * 32 + (lane & 31));
        float yp, yc;
        asm volatile("ds_read_b32 %0, %1" : "=v"(yp) : "v"(sb0 + row * 4));
        asm volatile("ds_read_b32 %0, %1 offset:1024" : "=v"(yc) : "v"(sb0 + row * 4));
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(yp), "+v"(yc));
        const float al = kq_alpha(yp, yc);
        asm volatile("ds_write_b32 %0, %1" :: "v"(sb0 + ALPHA_OFF + row * 4), "v"(al) : "memory");
    };
#ifdef Q2A_DIAG_STAMPS
    uint64_t bs_cycles = 0, bs_t0 = 0;
#define BS_T0() do { if (ST) bs_t0 = __builtin_amdgcn_s_memtime(); } while (0)
#define BS_T1() do { if (ST) bs_cycles += __builtin_amdgcn_s_memtime() - bs_t0; } while (0)
#else
#define BS_T0() do { } while (0)
#define BS_T1() do { } while (0)
#endif
    auto block_start = [&](auto first) {   // first: std::true_type for block 0 (acc = 0: only the min term)
        // C^T accumulators: lane holds columns n = 16j + 4(lane>>4) + r of row m = 16i + (lane&15), so alpha (per
        // row) is one scalar per row block and beta / gamma (per column) one float4 per column block
        const uint32_t s_al = sb0 + ALPHA_OFF + (wm * 128 + (lane & 15)) * 4;
        const uint32_t s_ae = sb0 + 5 * 1024 + (wm * 128 + (lane & 15)) * 32 + (lane >> 4) * 8;
        const uint32_t s_cn = sb0 + 2048 + (wn * 64 + (lane >> 4) * 4) * 4;                  // beta | gamma at +1024
        const uint32_t s_we = sb0 + 13 * 1024 + (wn * 64 + (lane & 15)) * 32 + (lane >> 4) * 8;
        f4 bet[4], gam[4];
        half4 we[4];
        float al[3];
        half4 ae[3];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bet[j]) : "v"(s_cn), "i"(j * 64));
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(gam[j]) : "v"(s_cn), "i"(1024 + j * 64));
            asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(we[j]) : "v"(s_we), "i"(j * 512));
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(al[i]) : "v"(s_al), "i"(i * 64));
            asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(ae[i]) : "v"(s_ae), "i"(i * 512));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(bet[0]), "+v"(bet[1]), "+v"(bet[2]), "+v"(bet[3]), "+v"(gam[0]),
                     "+v"(gam[1]), "+v"(gam[2]), "+v"(gam[3]), "+v"(we[0]), "+v"(we[1]), "+v"(we[2]), "+v"(we[3]),
                     "+v"(al[0]), "+v"(ae[0]), "+v"(al[1]), "+v"(ae[1]));
        // min-term MFMAs one row block ahead of their rescale (their latency under the previous block's VALU), row
        // data two ahead
        auto minterm = [&](f4 (&s2)[4], half4 a) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                s2[j] = __builtin_amdgcn_mfma_f32_16x16x16f16(we[j], a, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            }
        };
        if constexpr (PERS) {
            // register-lean form (the persistent kernel carries more state): min-term MFMAs one 16x16 block ahead
            // instead of one row block ahead (8 instead of 32 VGPRs of results); the same operations on every value
            f4 s2r[2];
            s2r[0] = __builtin_amdgcn_mfma_f32_16x16x16f16(we[0], ae[0], f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (i + 2 < 8) {
                    asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(al[(i + 2) % 3]) : "v"(s_al), "i"((i + 2) * 64));
                    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(ae[(i + 2) % 3]) : "v"(s_ae), "i"((i + 2) * 512));
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int c = (i * 4 + j) & 1;
                    if (j + 1 < 4) s2r[c ^ 1] = __builtin_amdgcn_mfma_f32_16x16x16f16(we[j + 1], ae[i % 3], f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                    else if (i + 1 < 8) s2r[c ^ 1] = __builtin_amdgcn_mfma_f32_16x16x16f16(we[0], ae[(i + 1) % 3], f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        if constexpr (decltype(first)::value) kq_first2(acc[i][j], h, gam[j], s2r[c]);
                        else kq_rescale2(acc[i][j], h, al[i % 3], bet[j], gam[j], s2r[c]);
                    }
                }
                if (i + 2 < 8) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(al[(i + 2) % 3]), "+v"(ae[(i + 2) % 3]));
                __builtin_amdgcn_sched_barrier(0);
            }
            return;
        }
        f4 s2v[2][4];
        minterm(s2v[0], ae[0]);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (i + 2 < 8) {
                asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(al[(i + 2) % 3]) : "v"(s_al), "i"((i + 2) * 64));
                asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(ae[(i + 2) % 3]) : "v"(s_ae), "i"((i + 2) * 512));
            }
            if (i + 1 < 8) minterm(s2v[(i + 1) & 1], ae[(i + 1) % 3]);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int h = 0; h < 2; ++h) {   // kq_rescale two columns per instruction (v_pk_mul / v_pk_fma)
                    if constexpr (decltype(first)::value) kq_first2(acc[i][j], h, gam[j], s2v[i & 1][j]);
                    else kq_rescale2(acc[i][j], h, al[i % 3], bet[j], gam[j], s2v[i & 1][j]);
                }
            if (i + 2 < 8) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(al[(i + 2) % 3]), "+v"(ae[(i + 2) % 3]));
            __builtin_amdgcn_sched_barrier(0);   // one row block at a time: bounds the live min-term results
        }
    };
    // fragment reads: 8 per-lane LDS byte addresses ([buffer][k-half]) + compile-time offsets, re-laundered every
    // phase so the compiler cannot hoist one address register per (image, tile) out of the loop
    uint32_t abase[2][2], bbase[2][2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
        const uint32_t lb = (lane & 15) * ROWB + ((((lane >> 4) | (s2 << 2)) ^ (lane & 7)) << 4);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            abase[b][s2] = lds0 + b * 4 * HT + wm * 64 * ROWB + lb;
            bbase[b][s2] = lds0 + (b * 4 + 2) * HT + wn * 32 * ROWB + lb;
        }
    }
    auto launder = [&]() {
        asm volatile("" : "+v"(abase[0][0]), "+v"(abase[0][1]), "+v"(abase[1][0]), "+v"(abase[1][1]),
                          "+v"(bbase[0][0]), "+v"(bbase[0][1]), "+v"(bbase[1][0]), "+v"(bbase[1][1]));
    };
    typedef const __attribute__((address_space(3))) half8 * lds_h8p;
    half8 af[4][2], bf[2][2][2];
    auto read_a = [&](int b, int qm) {
        launder();
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) af[i][s2] = *(lds_h8p) (uintptr_t) (abase[b][s2] + qm * HT + i * 16 * ROWB);
    };
    auto read_b = [&](int b, int qn) {
        launder();
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) bf[qn][j][s2] = *(lds_h8p) (uintptr_t) (bbase[b][s2] + qn * HT + j * 16 * ROWB);
    };
    auto mma_h = [&](int qm, int qn, int s2) {   // one 32-deep half of a quadrant's K-step: 8 MFMAs
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                acc[qm * 4 + i][qn * 2 + j] = mma16<BF>(bf[qn][j][s2], af[i][s2], acc[qm * 4 + i][qn * 2 + j]);
    };
    auto mma = [&](int qm, int qn) { mma_h(qm, qn, 0); mma_h(qm, qn, 1); };
    // staggered halves: the fragment reads retire BEFORE the barrier, so an image restaged the phase after its last
    // read (A_q0) cannot overtake the other half's reads, which now run one barrier later (cdna_hip_programming.md
    // §5 WAR rule)
#define Q2A_PB(N)                                               \
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");   \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");          \
    __builtin_amdgcn_s_barrier();                               \
    asm volatile("" ::: "memory");                              \
    __builtin_amdgcn_s_setprio(1)
#define Q2A_PE()                                                \
    __builtin_amdgcn_s_setprio(0);                              \
    asm volatile("" ::: "memory");                              \
    __builtin_amdgcn_s_barrier();                               \
    asm volatile("" ::: "memory")
// the four phases of one K-step in buffer B; S1..S4 = the stage statements issued in each phase
// (phase 2 of a Q4_K block's first K-step also issues the block's 3 scale pieces)
#define Q2A_KSTEP(B, S1, S2, S3, S4, V1, V2, V3, V4)                     \
    read_b(B, 0); read_a(B, 0); S1; Q2A_PB(V1); mma(0, 0); Q2A_PE();     \
    read_b(B, 1);               S2; Q2A_PB(V2); mma(0, 1); Q2A_PE();     \
    read_a(B, 1);               S3; Q2A_PB(V3); mma(1, 1); Q2A_PE();     \
                                S4; Q2A_PB(V4); mma(1, 0); Q2A_PE()

    // prologue: the images "phases 2..8 of iteration -1" would have staged (block 0's scales before them)
    if constexpr (BLK == 256) stage_scales(0);
    stage(0, 0, 0); stage(0, 2, 0); stage(0, 3, 0); stage(0, 1, 0);
    stage(1, 0, 1); stage(1, 2, 1); stage(1, 3, 1);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // wave stagger: the M-half wm = 1 (waves 4-7, the SIMD partners of waves 0-3) runs one barrier behind, so each
    // SIMD alternates one wave's MFMA segment with its partner's fragment reads / glds issue (MI355X_MICROARCH.md,
    // "Two waves per SIMD" item 9); the other half pays the extra barrier after the loop
    Q2A_STAMP(ST, 1);
    auto stagger_in = [&]() { if (wm == 1) { __builtin_amdgcn_s_barrier(); asm volatile("" ::: "memory"); } };
    auto stagger_out = [&]() { if (wm == 0) { __builtin_amdgcn_s_barrier(); asm volatile("" ::: "memory"); } };

    if constexpr (BLK == 0) {
        stagger_in();
        int kt = 0;
        for (; kt < nk - 2; kt += 2) {
            Q2A_KSTEP(0, stage(1, 1, kt + 1), stage(0, 0, kt + 2), stage(0, 2, kt + 2), stage(0, 3, kt + 2), 10, 10, 10, 10);
            Q2A_KSTEP(1, stage(0, 1, kt + 2), stage(1, 0, kt + 3), stage(1, 2, kt + 3), stage(1, 3, kt + 3), 10, 10, 10, 10);
        }
        Q2A_KSTEP(0, stage(1, 1, kt + 1), stage_tail(0, 0), stage_tail(0, 2), stage_tail(0, 3), 10, 10, 10, 10);
        Q2A_KSTEP(1, stage_tail(0, 1), stage_tail(1, 0), stage_tail(1, 2), stage_tail(1, 3), 10, 10, 10, 10);
    } else if constexpr (PERS) {
        static_assert(BLK == 256, "persistent 8-phase loop: Q4_K only");
        constexpr int S_EPI = 16 * PERS;
        static_assert(13 + S_EPI < 64, "vmcnt immediate range");
        // every tile's block 0 runs with its first five waits raised by S_EPI (the previous tile's epilogue stores sit
        // between its phase 0 and phase 1); for the first tile nothing is there, so the prologue drains its loads
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        alpha_compute();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        stagger_in();
        for (;;) {
            int m0n = 0, n0n = 0;
            const bool has_next = next(m0n, n0n);
            // the next tile's first K-steps (tail stages), or a harmless re-load of this tile's last one
            auto stage_next = [&](int b, int h) { stage(b, h, has_next ? b : nk - 1); };
            int kt = 0;
            BS_T0();
            block_start(std::true_type{});
            BS_T1();
            asm volatile("" ::: "memory");
            Q2A_KSTEP(0, stage(1, 1, kt + 1), (stage(0, 0, kt + 2), stage_scales(kt / 4 + 1)), stage(0, 2, kt + 2),
                      stage(0, 3, kt + 2), 10 + S_EPI, 13 + S_EPI, 13 + S_EPI, 13 + S_EPI);
            Q2A_KSTEP(1, stage(0, 1, kt + 2), stage(1, 0, kt + 3), stage(1, 2, kt + 3), stage(1, 3, kt + 3), 13 + S_EPI, 13, 10, 10);
            Q2A_KSTEP(0, (alpha_compute(), stage(1, 1, kt + 3)), stage(0, 0, kt + 4), stage(0, 2, kt + 4), stage(0, 3, kt + 4),
                      10, 10, 10, 10);
            Q2A_KSTEP(1, stage(0, 1, kt + 4), stage(1, 0, kt + 5), stage(1, 2, kt + 5), stage(1, 3, kt + 5), 10, 10, 10, 10);
            for (kt = 4; kt < nk - 4; kt += 4) {
            BS_T0();
                block_start(std::false_type{});
                BS_T1();
                asm volatile("" ::: "memory");
                Q2A_KSTEP(0, stage(1, 1, kt + 1), (stage(0, 0, kt + 2), stage_scales(kt / 4 + 1)), stage(0, 2, kt + 2),
                          stage(0, 3, kt + 2), 10, 13, 13, 13);
                Q2A_KSTEP(1, stage(0, 1, kt + 2), stage(1, 0, kt + 3), stage(1, 2, kt + 3), stage(1, 3, kt + 3), 13, 13, 10, 10);
                Q2A_KSTEP(0, (alpha_compute(), stage(1, 1, kt + 3)), stage(0, 0, kt + 4), stage(0, 2, kt + 4), stage(0, 3, kt + 4),
                          10, 10, 10, 10);
                Q2A_KSTEP(1, stage(0, 1, kt + 4), stage(1, 0, kt + 5), stage(1, 2, kt + 5), stage(1, 3, kt + 5), 10, 10, 10, 10);
            }
            prep_scales_last(has_next, m0n, n0n);
            BS_T0();
            block_start(std::false_type{});   // (nk >= 8: the last block is never block 0)
            BS_T1();
            asm volatile("" ::: "memory");
            Q2A_KSTEP(0, stage(1, 1, kt + 1), (stage(0, 0, kt + 2), stage_scales_last()), stage(0, 2, kt + 2),
                      stage(0, 3, kt + 2), 10, 13, 13, 13);
            Q2A_KSTEP(1, stage(0, 1, kt + 2), stage(1, 0, kt + 3), stage(1, 2, kt + 3), stage(1, 3, kt + 3), 13, 13, 10, 10);
            Q2A_KSTEP(0, stage(1, 1, kt + 3), ((has_next ? set_offsets(m0n, n0n) : (void) 0), stage_next(0, 0)), stage_next(0, 2),
                      stage_next(0, 3), 10, 10, 10, 10);
            Q2A_KSTEP(1, stage_next(0, 1), stage_next(1, 0), stage_next(1, 2), stage_next(1, 3), 10, 10, 10, 10);
            __builtin_amdgcn_sched_barrier(0);
            epi(acc, m0, n0);
            __builtin_amdgcn_sched_barrier(0);   // the finished tile's values die before the next tile's block 0 starts
            if (!has_next) break;
            m0 = m0n;
            n0 = n0n;
        }
    } else {
        static_assert(BLK == 256, "8-phase k-quant loop is Q4_K only");
        alpha_compute();                                     // block 0 (alpha = 1: acc is 0 anyway)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // raw barrier: __syncthreads would drain the prologue glds
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        stagger_in();
        int kt = 0;
        for (; kt < nk - 4; kt += 4) {
            BS_T0();
            if (kt == 0) block_start(std::true_type{});
            else block_start(std::false_type{});
            BS_T1();
            asm volatile("" ::: "memory");
            Q2A_KSTEP(0, stage(1, 1, kt + 1), (stage(0, 0, kt + 2), stage_scales(kt / 4 + 1)), stage(0, 2, kt + 2),
                      stage(0, 3, kt + 2), 10, 13, 13, 13);
            Q2A_KSTEP(1, stage(0, 1, kt + 2), stage(1, 0, kt + 3), stage(1, 2, kt + 3), stage(1, 3, kt + 3), 13, 13, 10, 10);
            // phase 9: the next block's alpha (its scales, staged in phase 2, landed by phase 7)
            Q2A_KSTEP(0, (alpha_compute(), stage(1, 1, kt + 3)), stage(0, 0, kt + 4), stage(0, 2, kt + 4), stage(0, 3, kt + 4),
                      10, 10, 10, 10);
            Q2A_KSTEP(1, stage(0, 1, kt + 4), stage(1, 0, kt + 5), stage(1, 2, kt + 5), stage(1, 3, kt + 5), 10, 10, 10, 10);
        }
        // last block: its scales stay in place for the final multiply (the scale re-stage keeps the vmcnt counts)
        BS_T0();
        if (kt == 0) block_start(std::true_type{});
        else block_start(std::false_type{});
        BS_T1();
        asm volatile("" ::: "memory");
        Q2A_KSTEP(0, stage(1, 1, kt + 1), (stage(0, 0, kt + 2), stage_scales(kt / 4)), stage(0, 2, kt + 2),
                  stage(0, 3, kt + 2), 10, 13, 13, 13);
        Q2A_KSTEP(1, stage(0, 1, kt + 2), stage(1, 0, kt + 3), stage(1, 2, kt + 3), stage(1, 3, kt + 3), 13, 13, 10, 10);
        Q2A_KSTEP(0, stage(1, 1, kt + 3), stage_tail(0, 0), stage_tail(0, 2), stage_tail(0, 3), 10, 10, 10, 10);
        Q2A_KSTEP(1, stage_tail(0, 1), stage_tail(1, 0), stage_tail(1, 2), stage_tail(1, 3), 10, 10, 10, 10);
    }
#undef Q2A_KSTEP
#undef Q2A_PB
#undef Q2A_PE
#undef BS_T0
#undef BS_T1
    stagger_out();
    Q2A_STAMP(ST, 2);
#ifdef Q2A_DIAG_STAMPS
    if (ST) q2a_stamp_put(7, bs_cycles);
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tail re-loads still land in LDS: drain before the epilogue
    __syncthreads();
    if constexpr (PERS) return;                          // (every tile's epilogue already ran inside the loop)
    if constexpr (BLK == 256) {
        // acc is in units of the last block's scale: multiply by dy_last[m] * dx_last[n]
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const f4 dx4 = *(lds_f4p) (uintptr_t) (sb0 + 4096 + (wn * 64 + j * 16 + (lane >> 4) * 4) * 4);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float yc = *(lds_fp) (uintptr_t) (sb0 + 1024 + (wm * 128 + i * 16 + (lane & 15)) * 4);
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[i][j][r] = kq_final(acc[i][j][r], yc, dx4[r]);
            }
        }
    }
}

template <int BM, int BN, int WM, int WN, int EPI, int BLK_, int PIPE>
__global__ __launch_bounds__(WM * WN * 64, 1) void k_gemm(const q2a_gemm_args p_arg) {
    q2a_gemm_args p = p_arg;   // (the grouped STORE_F launch swaps in its second GEMM's operands below)
    constexpr bool BF = BLK_ == Q2A_BLK_BF16;              // bf16 operands, no block scales
#ifdef Q2A_DIAG_STAMPS
    constexpr bool ST = PIPE == 1 && EPI == Q2A_DIAG_STAMPS;   // timing stamps (diagnostic builds only)
#else
    constexpr bool ST = false;
#endif
    constexpr bool EX = BLK_ == Q2A_BLK_EXACT;             // fp16 operands, f64 sum of per-K-step partials
    constexpr int BLK = (BF || EX) ? 0 : BLK_;
    static_assert(!EX || PIPE == 0, "exact accumulation: small-tile kernels only");
    if constexpr (EX) {
        if (p.gate && ((*p.gate != 0) != (p.gate_on != 0))) return;   // the other launch of this node computes it
    }
    constexpr int NW = WM * WN;
    constexpr int MI = BM / WM / 16, NJ = BN / WN / 16;   // 16x16 tiles per wave
    constexpr int LA = BM / 8 / NW, LB = BN / 8 / NW;     // glds instructions per wave per stage
    static_assert(LA >= 1 && LB >= 1, "tile too small for the wave count");
    // k-quant block scales of the tile, staged through LDS (block-major global layout => contiguous per block):
    //   BLK=256: dy_{b-1}[BM] | dy_b[BM] f32 | aext[BM][16] f16 | beta[BN] | gamma[BN] | dx[BN] f32 | wext[BN][16] f16
    //            (two buffers by block parity: block b+1's scales land while block b computes)
    //   BLK=32 : dy[2][BM] f32 | dx[2][BN] f32 for the two 32-blocks of a K-step            (two buffers)
    constexpr int SB = BLK == 256 ? (BM * 8 + BM * 32 + BN * 12 + BN * 32) : BLK == 32 ? 2 * (BM * 4 + BN * 4) : 0;
    constexpr int NSB = BLK ? 2 : 1;
    constexpr int NT = NW * 64;
    constexpr int SCH = (SB / 16 + NT - 1) / NT;          // 16-B scale chunks per thread
    constexpr int OPB = (BM + BN) * ROWB;                 // one operand stage (A image | W image)
    // GELU epilogues of the 8-phase kernel look the table up in LDS (staged into operand slots 0..4 = [0, 80 KiB)),
    // so their transpose staging moves behind it
    constexpr bool LUT_EPI = PIPE && (EPI == Q2A_EPI_GELU_H || EPI == Q2A_EPI_GELU_F || EPI == Q2A_EPI_CONV2 ||
                                      EPI == Q2A_EPI_GELU_Q8K);
    constexpr int EPI_OFF = LUT_EPI ? Q2A_GELU_C_BYTES : 0;
    // per-wave epilogue staging: V^T [64 d][WR + 4 t] fp16 (QKV), or with the lo image the hi | lo pair of [64 d][WR/2
    // + 4 t] (half the wave's rows at a time); the other epilogues keep their 32-row budget
    constexpr int EPI_WREG = EPI == Q2A_EPI_QKV ? (MI == 1 ? 2 * 64 * (BM / WM + 4) * 2   // (16-row waves: one pass, hi | lo)
                                                           : std::max(64 * (BM / WM + 4) * 2, 2 * 64 * (BM / WM / 2 + 4) * 2))
                                                : 2 * 32 * (BN / WN + 8) * 2;
    // small-tile kernels: NS operand stages (NS - 1 K-steps of loads in flight, counted vmcnt, raw barriers) within
    // ~150 KiB of LDS. Q4_K: block b+1's scales arrive by glds in 1 KiB pieces (SBP per block, one per wave on the
    // first SP K-steps of block b) into the other of two buffers, plus one pad piece per wave for the dummy pieces
    // that keep every step's glds count uniform (so the vmcnt counts are compile-time); a piece issued at step s has
    // landed by the end of step s + NS - 2, so SP + NS <= 6 puts it in place before block b+1 starts at step 4b + 4.
    // The Q8_0 path drains its per-step register-staged scale loads every step and keeps 2 stages.
    constexpr int SBP = BLK == 256 ? (SB + 1023) / 1024 : 0;          // 1 KiB pieces per Q4_K block
    constexpr int SP = BLK == 256 ? (SBP + NW - 1) / NW : 0;          // K-steps per block that issue a piece
    static_assert(BLK != 256 || SP <= 4, "Q4_K scale pieces must fit the block's 4 K-steps");
    // the two-stage 128-row Q4_K tiles keep ONE scale buffer: block b+1's pieces are issued on steps 4b+1 .. 4b+SP,
    // after the barrier that ends block b's start (the only reader of block b's scales besides the final multiply of
    // the last block), and land within their step (NS = 2 drains every step). 90 -> 79 KiB of LDS for 128x128, so two
    // workgroups share a CU as in the F16 tiles (a single clip's QKV / fc1 GEMMs are latency-bound at one per CU)
    constexpr int NBUF = (BLK == 256 && !PIPE && BM > 64) ? 1 : 2;
    constexpr int SCALE_LDS = BLK == 256 ? (NBUF * SBP + NW) * 1024 : BLK ? NSB * SB : 0;
    constexpr int NS_FIT = (150 * 1024 - SCALE_LDS) / OPB;
    constexpr int NS_MAX = BLK == 256 ? 6 - SP : 5;
    // deep pipelines only on the narrow 64-row tiles (grids under one workgroup per CU); the 128-row tiles keep two
    // stages so two workgroups share a CU (their grids have several tiles per CU)
    constexpr int NS = EX ? 2 : PIPE || BLK == 32 || BM > 64 ? 2 : (NS_FIT >= NS_MAX ? NS_MAX : NS_FIT >= 2 ? NS_FIT : 2);
    static_assert(PIPE || BLK != 256 || SP + NS <= 6, "Q4_K scale prefetch distance");
    static_assert(NBUF == 2 || (NS == 2 && SP <= 3), "single Q4_K scale buffer: pieces on steps 4b+1 .. 4b+3");
    constexpr int LDS_MAIN = PIPE == 2 ? SBUF_OFF + SBUF_BYTES + 512 : PIPE ? (BLK ? SBUF_OFF + SBUF_BYTES : 2 * OPB) : NS * OPB + SCALE_LDS;
    constexpr int LDS_BYTES = LDS_MAIN > EPI_OFF + NW * EPI_WREG ? LDS_MAIN : EPI_OFF + NW * EPI_WREG;
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
    __shared__ __attribute__((aligned(16))) char lds_raw[LDS_BYTES];
#define LDS_STAGE(b_) (lds_raw + (b_) * OPB)
    char * sbuf = lds_raw + NS * OPB;                     // scale staging (only when BLK)
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;

    // XCD-contiguous bijective remap, then grouped rasterisation (GROUP_M M-tiles per N column)
    constexpr bool GROUPABLE = !PIPE && !BF && !EX && (BLK == 0 || BLK == 256) && EPI == Q2A_EPI_STORE_F;
    const int ngrp = (GROUPABLE && p.ngroup == 2) ? 2 : 1;
    const int ksplit = (!PIPE && !EX && (BLK == 0 || BLK == 32) && (EPI == Q2A_EPI_RESID || EPI == Q2A_EPI_STORE_F) &&
                        p.ksplit > 1 && ngrp == 1) ? p.ksplit : 1;
    const int nbn = p.N / BN, nbm = (p.M - p.m_base + BM - 1) / BM, ntl = nbn * nbm, nwg = ntl * ksplit * ngrp;
    const int bid = blockIdx.x, xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
    int wgid_all = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    if constexpr (GROUPABLE) {
        if (ngrp == 2 && wgid_all >= ntl) {
            wgid_all -= ntl;
            p.W = p.W2; p.bias = p.bias2; p.outF = p.outF2; p.out_scale = p.out_scale2; p.store_bias = p.store_bias2;
            if constexpr (BLK == 256) { p.dx = p.dx2; p.dmin = p.dmin2; p.beta = p.beta2; p.gamma = p.gamma2; p.wext = p.wext2; }
        }
    }
    const int ks = wgid_all / ntl, wgid = wgid_all - ks * ntl;   // K-split index, tile index
    constexpr int GM = GROUP_M;
    const int gsize = GM * nbn, g = wgid / gsize, gr = wgid % gsize;
    const int gm = min(GM, nbm - g * GM);
    const int tm = g * GM + gr % gm, tn = gr / gm;
    const int m0 = p.m_base + tm * BM, n0 = tn * BN;

    f4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    if constexpr (PIPE == 2) {
        // persistent 8-phase tiles (launch_pipe8: fc1's pre-activation, M a multiple of 256, K >= 512): virtual
        // workgroup ids v = blockIdx.x + r * gridDim.x mapped exactly like the one-tile-per-workgroup grid (gridDim is
        // a multiple of 8, so v and blockIdx.x share an XCD), the pipeline runs across the tiles (mainloop_8phase PERS)
        static_assert((EPI == Q2A_EPI_PRE_H || EPI == Q2A_EPI_QKV) && BLK == 256 && BM == 256 && BN == 256 && NW == 8,
                      "persistent form: Q4_K fc1 pre-activation / Q|K|V with row-major V");
        constexpr bool QKV = EPI == Q2A_EPI_QKV;
        auto tile_at = [&](int v, int & tm0, int & tn0) {
            const int x8 = v & 7;
            const int w = (x8 < rr ? x8 * (qq + 1) : rr * (qq + 1) + (x8 - rr) * qq) + (v >> 3);
            const int g2 = w / gsize, gr2 = w % gsize, gm2 = min(GM, nbm - g2 * GM);
            tm0 = p.m_base + (g2 * GM + gr2 % gm2) * BM;
            tn0 = (gr2 / gm2) * BN;
        };
        // the workgroup's tile list (m0 | n0 per entry) in LDS behind the final-multiply area: the loop then carries
        // one counter instead of the raster's constants (SGPR pressure: past 106 the compiler spills)
        int * tlist = (int *) (lds_raw + SBUF_OFF + SBUF_BYTES);
        const int ntw = (ntl - bid + (int) gridDim.x - 1) / (int) gridDim.x;   // tiles of this workgroup (>= 1)
        for (int r = tid; r < ntw; r += NT) {
            int a0, b0;
            tile_at(bid + r * (int) gridDim.x, a0, b0);
            tlist[2 * r] = a0;
            tlist[2 * r + 1] = b0;
        }
        __syncthreads();
        const uint32_t tl0 = (uint32_t) (uintptr_t) (const __attribute__((address_space(3))) char *) lds_raw + SBUF_OFF + SBUF_BYTES;
        int rcur = 0;
        auto next = [&](int & tm0, int & tn0) -> bool {
            if (rcur + 1 >= ntw) return false;
            ++rcur;
            int2 v;
            asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(tl0 + rcur * 8) : "memory");
            tm0 = __builtin_amdgcn_readfirstlane(v.x);
            tn0 = __builtin_amdgcn_readfirstlane(v.y);
            return true;
        };
        const uint32_t fin = (uint32_t) (uintptr_t) (const __attribute__((address_space(3))) char *) lds_raw + FIN_OFF;
        // the finished tile: acc * (dy_last[m] * dx_last[n]) + bias[n] (Q: * qscale) -> fp16 (the PIPE = 1 epilogues'
        // operations, bit for bit), straight from registers: fc1 one image, Q|K|V the hi and the lo image
        // (fp16(v - hi)) of the tile's part (256 | D: a tile lies in one of Q, K, V; V row-major, q2a_gemm_args.v_rows).
        // Whole 128-B output lines per store: a 16-row block's wave columns (64 fp16 = one line per row) leave as two
        // stores of 8 rows x 8 lanes x 16 B instead of two of 16 rows x 64 B. Register moves only (VALU, no LDS):
        //   1. v_permlane16_swap pairs lanes q, q^1 (rows of 16 lanes): lane (q, l) then holds 16 B of row l for each
        //      column-tile pair jp, chunk c = 2 (q & 1) + (q >> 1) (+ 4 jp) of the row's eight 16-B chunks;
        //   2. DPP row_ror:8 pairs lanes l, l ^ 8: the lower half keeps chunk c of its row and takes chunk c + 4 of
        //      row l + 8 (store B), the upper half the other way round (store A) — every row's 8 chunks in one store.
        // Exactly S_EPI = 16 (fc1) / 32 (Q|K|V) stores per wave on every tile (M % 256 == 0: no row is skipped).
        auto epi = [&](f4 (&ac)[8][4], int tm0, int tn0) {
            const int ln = (int) __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));   // lane, rematerialised
            const int q = ln >> 4, l16 = ln & 15;
            const int pcol = 16 * (q & 1) + 8 * (q >> 1);
            f4 dx4[4], b4[4];
            float yc[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t c = fin + (wn * 64 + j * 16 + q * 4) * 4;
                asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(dx4[j]) : "v"(c));
                asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(b4[j]) : "v"(c));
            }
#pragma unroll
            for (int i = 0; i < 8; ++i)
                asm volatile("ds_read_b32 %0, %1" : "=v"(yc[i]) : "v"(fin + (wm * 128 + i * 16 + l16) * 4));
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(dx4[0]), "+v"(dx4[1]), "+v"(dx4[2]), "+v"(dx4[3]), "+v"(b4[0]),
                         "+v"(b4[1]), "+v"(b4[2]), "+v"(b4[3]), "+v"(yc[0]), "+v"(yc[1]), "+v"(yc[2]), "+v"(yc[3]),
                         "+v"(yc[4]), "+v"(yc[5]), "+v"(yc[6]), "+v"(yc[7]));
            typedef _Float16 h4p __attribute__((ext_vector_type(4)));
            const int hi8 = l16 >> 3;
            // destination images and column of this lane's 16-B piece (QKV: within the part's [M][D] rows)
            const int part = QKV ? tn0 / p.D : 0;
            q2a_half * dhi = QKV ? (part == 0 ? p.qh : part == 1 ? p.kh : p.vt) : p.outH;
            q2a_half * dlo = QKV ? (part == 0 ? p.ql : part == 1 ? p.kl : p.vtl) : nullptr;
            const int64_t ld = QKV ? p.D : p.ldo;
            const int colw = tn0 - part * p.D + wn * 64 + pcol + 32 * hi8;
            const float vsc = QKV && part == 0 ? p.qscale : 1.0f;
            // one image's two 16-B pieces per lane (jp = 0, 1) -> stores A (rows 16i + (l & 7)) and B (+ 8)
            auto store_lines = [&](uint32_t (&hv)[2][4], q2a_half * dst, int i) {
                uint32_t sa4[4], sb4[4];   // (scalars, not uint4: a lane-varying select of a uint4 array went to scratch)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    // lanes l < 8 send their jp = 1 piece to lane l + 8, lanes l >= 8 their jp = 0 piece to lane l - 8
                    const uint32_t snd = hi8 ? hv[0][k] : hv[1][k];
                    const uint32_t rcv = (uint32_t) __builtin_amdgcn_mov_dpp((int) snd, 0x128, 0xF, 0xF, false);   // row_ror:8
                    sa4[k] = hi8 ? rcv : hv[0][k];   // rows 16 i + (l & 7): chunk c (l < 8) / c + 4 (l >= 8)
                    sb4[k] = hi8 ? hv[1][k] : rcv;   // rows 16 i + 8 + (l & 7)
                }
                q2a_half * o0 = dst + (int64_t) (tm0 + wm * 128 + i * 16 + (l16 & 7)) * ld + colw;
                if (Q2A_ST) q2a_st(make_uint4(sa4[0], sa4[1], sa4[2], sa4[3]), (uint4 *) o0);
                if (Q2A_ST) q2a_st(make_uint4(sb4[0], sb4[1], sb4[2], sb4[3]), (uint4 *) (o0 + 8 * ld));
            };
            auto pair_swap = [&](h4p ha, h4p hb, uint32_t (&out)[4]) {
                uint2 ua, ub;
                __builtin_memcpy(&ua, &ha, 8);
                __builtin_memcpy(&ub, &hb, 8);
                // odd rows of ua <-> even rows of ub: (ua, ub) is then this lane's 8 consecutive columns
                const auto rx = __builtin_amdgcn_permlane16_swap(ua.x, ub.x, false, false);
                const auto ry = __builtin_amdgcn_permlane16_swap(ua.y, ub.y, false, false);
                out[0] = rx[0]; out[1] = ry[0]; out[2] = rx[1]; out[3] = ry[1];
            };
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                uint32_t hv[2][4], lv[2][4];
#pragma unroll
                for (int jp = 0; jp < 2; ++jp) {
                    h4p ha, hb, la, lb;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
#pragma clang fp contract(off)
                        float va = kq_final(ac[i][2 * jp][r], yc[i], dx4[2 * jp][r]) + b4[2 * jp][r];
                        float vb = kq_final(ac[i][2 * jp + 1][r], yc[i], dx4[2 * jp + 1][r]) + b4[2 * jp + 1][r];
                        if (QKV) {   // ggml_scale after the bias add (exact 2^-3 times fl(log2 e): one rounding)
                            va = va * vsc;
                            vb = vb * vsc;
                        }
                        ha[r] = (_Float16) va;
                        hb[r] = (_Float16) vb;
                        if (QKV) {
                            la[r] = (_Float16) (va - (float) ha[r]);
                            lb[r] = (_Float16) (vb - (float) hb[r]);
                        }
                    }
                    pair_swap(ha, hb, hv[jp]);
                    if (QKV) pair_swap(la, lb, lv[jp]);
                }
                store_lines(hv, dhi, i);
                if (QKV) store_lines(lv, dlo, i);
            }
            // (no reset: the next tile's block-0 start writes every accumulator, kq_first2)
        };
        Q2A_STAMP(ST, 0);
        Q2A_STAMP_RT(ST, 8);
        mainloop_8phase<BLK, false, false, ST, QKV ? 2 : 1>(p, acc, lds_raw, m0, n0, lane, wave, wm, wn, next, epi);
        Q2A_STAMP(ST, 6);
        Q2A_STAMP_RT(ST, 9);
        return;
    } else if constexpr (PIPE == 1) {
        Q2A_STAMP(ST, 0);
        Q2A_STAMP_RT(ST, 8);
        mainloop_8phase<BLK, LUT_EPI, BF, ST>(p, acc, lds_raw, m0, n0, lane, wave, wm, wn);
        Q2A_STAMP(ST, 3);
    } else {
        // per-lane source rows of this wave's glds instructions (rows past M clamp to M-1: loaded, never stored)
        int64_t arow[LA], wrow[LB];
    #pragma unroll
        for (int i = 0; i < LA; ++i) {
            const int r = (wave * LA + i) * 8 + (lane >> 3);
            arow[i] = a_row_off(p, min(m0 + r, p.M - 1)) + (((lane & 7) ^ (r & 7)) << 3);
        }
    #pragma unroll
        for (int i = 0; i < LB; ++i) {
            const int r = (wave * LB + i) * 8 + (lane >> 3);
            wrow[i] = (int64_t) (n0 + r) * p.ldw + (((lane & 7) ^ (r & 7)) << 3);
        }
        auto stage = [&](char * buf, int k0) {
    #pragma unroll
            for (int i = 0; i < LA; ++i)
                __builtin_amdgcn_global_load_lds((const void *) (p.A + arow[i] + k0),
                                                 (lds_ptr_t) (buf + (wave * LA + i) * 8 * ROWB), 16, 0, 0);
    #pragma unroll
            for (int i = 0; i < LB; ++i)
                __builtin_amdgcn_global_load_lds((const void *) (p.W + wrow[i] + k0),
                                                 (lds_ptr_t) (buf + (BM + (wave * LB + i) * 8) * ROWB), 16, 0, 0);
        };

        // scale chunk c of K-block group g (BLK=256: block g; BLK=32: blocks 2g, 2g+1) -> global source
        auto scale_src = [&](int c, int g) -> const uint4 * {
            if (BLK == 256) {
                if (c < BM / 4) return (const uint4 *) (p.dy + (int64_t) max(g - 1, 0) * p.dy_ld + m0) + c;
                c -= BM / 4;
                if (c < BM / 4) return (const uint4 *) (p.dy + (int64_t) g * p.dy_ld + m0) + c;
                c -= BM / 4;
                if (c < BM * 2) return (const uint4 *) (p.aext + ((int64_t) g * p.dy_ld + m0) * 16) + c;
                c -= BM * 2;
                if (c < BN / 4) return (const uint4 *) (p.beta + (int64_t) g * p.N + n0) + c;
                c -= BN / 4;
                if (c < BN / 4) return (const uint4 *) (p.gamma + (int64_t) g * p.N + n0) + c;
                c -= BN / 4;
                if (c < BN / 4) return (const uint4 *) (p.dx + (int64_t) g * p.N + n0) + c;
                c -= BN / 4;
                return (const uint4 *) (p.wext + ((int64_t) g * p.N + n0) * 16) + c;
            } else {
                if (c < BM / 2) return (const uint4 *) (p.dy + (int64_t) (2 * g + c / (BM / 4)) * p.dy_ld + m0) + c % (BM / 4);
                c -= BM / 2;
                return (const uint4 *) (p.dx + (int64_t) (2 * g + c / (BN / 4)) * p.N + n0) + c % (BN / 4);
            }
        };
        // Q4_K: piece q (0 <= q < SP * NW) of block g: chunk q * 64 + lane of the SB layout (16 B per lane), or a
        // dummy re-load into this wave's pad piece when q >= SBP or the block does not exist
        uint32_t l16s = lane * 16;
        auto scale_piece = [&](int q, int g) {
            asm volatile("" : "+v"(l16s));
            const int c = q * 64 + lane;
            const bool real = q < SBP && g < p.K / 256 && c < SB / 16;
            const uint4 * src = real ? scale_src(c, g) : (const uint4 *) p.dy + lane;
            char * dst = real ? sbuf + (g & (NBUF - 1)) * SBP * 1024 + q * 1024 : sbuf + NBUF * SBP * 1024 + wave * 1024;
            if (q >= SBP || g >= p.K / 256) dst = sbuf + NBUF * SBP * 1024 + wave * 1024;
            __builtin_amdgcn_global_load_lds((const void *) src, (lds_ptr_t) dst, 16, 0, 0);
        };
        uint4 sreg[BLK == 32 ? SCH : 1];
        auto scale_load = [&](int g) {
    #pragma unroll
            for (int u = 0; u < SCH; ++u) {
                const int c = tid + u * NT;
                if (c < SB / 16) sreg[u] = *scale_src(c, g);
            }
        };
        auto scale_store = [&](int buf) {
    #pragma unroll
            for (int u = 0; u < SCH; ++u) {
                const int c = tid + u * NT;
                if (c < SB / 16) *(uint4 *) (sbuf + buf * SB + c * 16) = sreg[u];
            }
        };

        // Q8_0 / Q4_0 (BLK = 32): a fresh accumulator per 32-block, combined acc += (dx*dy)*blk after each
        // exact mode (EX): the same fresh accumulator per 64-deep K-step, added into acc64 after it
        constexpr bool FRESH = BLK == 32 || EX;
        f4 blk[FRESH ? MI : 1][FRESH ? NJ : 1];
        double acc64[EX ? MI : 1][EX ? NJ : 1][4];
        if (FRESH) {
    #pragma unroll
            for (int i = 0; i < (FRESH ? MI : 1); ++i)
    #pragma unroll
                for (int j = 0; j < (FRESH ? NJ : 1); ++j) {
                    blk[i][j] = f4{0.f, 0.f, 0.f, 0.f};
                    if (EX)
    #pragma unroll
                        for (int r = 0; r < 4; ++r) acc64[i][j][r] = 0.0;
                }
        }
        // Q4_K (BLK = 256): the block-ratio recurrence of the 8-phase kernel (kq_rescale), op for op
        auto kq_block_start = [&](const char * sb, auto first) {   // first: std::true_type for block 0 (acc = 0)
            const float * s_dyp = (const float *) sb;
            const float * s_dy = s_dyp + BM;
            const q2a_half * s_ae = (const q2a_half *) (sb + BM * 8);
            const float * s_be = (const float *) (sb + BM * 40);
            const float * s_ga = s_be + BN;
            const q2a_half * s_we = (const q2a_half *) (sb + BM * 40 + BN * 12);
            f4 be[NJ], ga[NJ];
            half4 we[NJ];
    #pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int n4 = wn * (BN / WN) + j * 16 + (lane >> 4) * 4;
                be[j] = *(const f4 *) (s_be + n4);
                ga[j] = *(const f4 *) (s_ga + n4);
                we[j] = *(const half4 *) (s_we + (wn * (BN / WN) + j * 16 + (lane & 15)) * 16 + (lane >> 4) * 4);
            }
    #pragma unroll
            for (int i = 0; i < MI; ++i) {
                const int row = wm * (BM / WM) + i * 16 + (lane & 15);
                const float al = kq_alpha(s_dyp[row], s_dy[row]);
                const half4 ae = *(const half4 *) (s_ae + row * 16 + (lane >> 4) * 4);
    #pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const f4 s2 = __builtin_amdgcn_mfma_f32_16x16x16f16(we[j], ae, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    #pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        if constexpr (decltype(first)::value) acc[i][j][r] = ga[j][r] * s2[r];   // = kq_rescale(0, ...)
                        else acc[i][j][r] = kq_rescale(acc[i][j][r], al, be[j][r], ga[j][r], s2[r]);
                    }
                }
            }
        };

        const int nk = p.K / BK / ksplit;                 // K-steps of this split
        const int kb0 = ks * nk * BK;                     // its first K element
        const int gb0 = BLK == 256 ? kb0 / 256 : kb0 / BK;   // its first scale group (whole groups per split)
        const int nkb = p.K / 256;                        // Q4_K blocks
        // prologue: block 0's scales, then stages 0 .. NS-2; K-step kt reads stage kt % NS and, before its MFMAs,
        // issues stage kt + NS - 1 into the slot K-step kt - 1 read (behind the barrier that ended kt - 1)
        constexpr int GL = LA + LB;                       // glds instructions per stage per thread
        if (BLK == 32) scale_load(gb0);
        if (BLK == 256) {                                 // block 0's scales, every piece
    #pragma unroll
            for (int u = 0; u < SP; ++u) scale_piece(u * NW + wave, 0);
        }
    #pragma unroll
        for (int q = 0; q < NS - 1; ++q)
            if (q < nk) stage(LDS_STAGE(q), kb0 + q * BK);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (BLK == 32) scale_store(0);
        __syncthreads();

        for (int kt = 0; kt < nk; ++kt) {
            const int cur = kt % NS;
            const bool issue = kt + NS - 1 < nk;
            if (issue) stage(LDS_STAGE((kt + NS - 1) % NS), kb0 + (kt + NS - 1) * BK);
            // Q4_K: block b starts at K-step 4b with its scales resident (buffer b&1), and block b+1's scales are
            // fetched then and land in the other buffer at the end of that K-step;
            // Q8_0: the next K-step's two blocks are fetched one step ahead into the other buffer.
            bool sload = false;
            if (BLK == 256) {
                // (block 0 through the general form as well: fma(0, t, u) = u is what the 8-phase kernel's block-0
                // start computes; a second inlined copy here costs 248 -> 272 registers, one workgroup per CU)
                if (kt % 4 == 0) kq_block_start(sbuf + ((kt / 4) & (NBUF - 1)) * SBP * 1024, std::false_type{});
                if (NBUF == 2 && kt % 4 < SP) scale_piece((kt % 4) * NW + wave, kt / 4 + 1);   // uniform: one per wave
                if (NBUF == 1 && kt % 4 >= 1 && kt % 4 <= SP) scale_piece((kt % 4 - 1) * NW + wave, kt / 4 + 1);
            } else if (BLK == 32 && kt + 1 < nk) {
                sload = true;
                scale_load(gb0 + kt + 1);
            }
            const char * ia = LDS_STAGE(cur);
            const char * iw = LDS_STAGE(cur) + BM * ROWB;
    #pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int chunk = s * 4 + (lane >> 4);
                half8 b[NJ];
    #pragma unroll
                for (int j = 0; j < NJ; ++j) b[j] = frag(iw, wn * (BN / WN) + j * 16 + (lane & 15), chunk);
    #pragma unroll
                for (int i = 0; i < MI; ++i) {
                    const half8 a = frag(ia, wm * (BM / WM) + i * 16 + (lane & 15), chunk);
    #pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        // W as the A operand: C^T tiles (lane = 4 consecutive columns of one row, see the epilogue)
                        if (!FRESH) acc[i][j] = mma16<BF>(b[j], a, acc[i][j]);
                        else blk[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[j], a, blk[i][j], 0, 0, 0);
                    }
                }
                if (BLK == 32) {
                    const char * sb = sbuf + (kt & 1) * SB;
                    const float * s_dy = (const float *) sb + s * BM;
                    const float * s_dx = (const float *) (sb + 2 * BM * 4) + s * BN;
                    // C^T tiles: per-column scales as float4 (columns 16j + 4(lane>>4) + r), per-row as a scalar
                    f4 dx[NJ];
    #pragma unroll
                    for (int j = 0; j < NJ; ++j) dx[j] = *(const f4 *) (s_dx + wn * (BN / WN) + j * 16 + (lane >> 4) * 4);
    #pragma unroll
                    for (int i = 0; i < MI; ++i) {
                        const float dyi = s_dy[wm * (BM / WM) + i * 16 + (lane & 15)];
    #pragma unroll
                        for (int j = 0; j < NJ; ++j) {
    #pragma unroll
                            for (int r = 0; r < 4; ++r) acc[i][j][r] += (dx[j][r] * dyi) * blk[i][j][r];
                            blk[i][j] = f4{0.f, 0.f, 0.f, 0.f};
                        }
                    }
                }
            }
            if constexpr (EX) {   // this K-step's 64-deep partial into the f64 sums
    #pragma unroll
                for (int i = 0; i < MI; ++i)
    #pragma unroll
                    for (int j = 0; j < NJ; ++j) {
    #pragma unroll
                        for (int r = 0; r < 4; ++r) acc64[i][j][r] += (double) blk[i][j][r];
                        blk[i][j] = f4{0.f, 0.f, 0.f, 0.f};
                    }
            }
            // stage kt + 1 must have landed before the barrier; the NS - 2 younger stages stay in flight (raw
            // s_barrier: __syncthreads would drain them). Steps that fetched scales into registers drain fully.
            if (sload) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                scale_store((kt & 1) ^ 1);
            } else if (issue && NS > 2) {
                if constexpr (BLK == 256) {
                    // younger than stage kt+1: the NS-2 stages of steps kt+3-NS .. kt and the scale pieces of those
                    // steps (steps with s % 4 < SP)
                    constexpr int W0 = GL * (NS - 2);
                    auto npc = [](int r) {   // pieces issued in the NS-2 steps ending at a step with kt % 4 == r
                        int n = 0;
                        for (int d = 0; d < NS - 2; ++d) n += (((r - d) % 4 + 4) % 4) < SP;
                        return n;
                    };
                    switch (kt & 3) {
                        case 0: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(W0 + npc(0)) : "memory"); break;
                        case 1: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(W0 + npc(1)) : "memory"); break;
                        case 2: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(W0 + npc(2)) : "memory"); break;
                        default: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(W0 + npc(3)) : "memory"); break;
                    }
                } else {
                    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(GL * (NS - 2)) : "memory");
                }
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if constexpr (BLK == 256) {
            // acc is in units of the last block's scale: multiply by dy_last[m] * dx_last[n]
            const char * sb = sbuf + ((nkb - 1) & (NBUF - 1)) * SBP * 1024;
            const float * s_dy = (const float *) sb + BM;
            const float * s_dx = (const float *) (sb + BM * 40 + BN * 8);
    #pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const f4 dx4 = *(const f4 *) (s_dx + wn * (BN / WN) + j * 16 + (lane >> 4) * 4);
    #pragma unroll
                for (int i = 0; i < MI; ++i) {
                    const float yc = s_dy[wm * (BM / WM) + i * 16 + (lane & 15)];
    #pragma unroll
                    for (int r = 0; r < 4; ++r) acc[i][j][r] = kq_final(acc[i][j][r], yc, dx4[r]);
                }
            }
        }
        if constexpr (EX) {   // the f64 sums rounded to f32 once: the epilogue then runs unchanged
    #pragma unroll
            for (int i = 0; i < MI; ++i)
    #pragma unroll
                for (int j = 0; j < NJ; ++j)
    #pragma unroll
                    for (int r = 0; r < 4; ++r) acc[i][j][r] = (float) acc64[i][j][r];
        }
    }

    if constexpr (EPI == Q2A_EPI_GELU_Q8K && PIPE == 1) {
        // fc1 + GELU + Q8_K quantization of the produced activation (quantize_row_q8_K_ref, the conversion ggml
        // applies to the fc2 input): the 256-column tile is exactly one Q8_K block per row. Per pass, the four
        // waves of one M-half write gelu values (exact fp16) of their 128 rows into LDS behind the GELU table;
        // then every wave quantizes 16 whole rows (a half4 per lane) and writes codes, d and the bsum operand.
        constexpr int RSH = 256 + 8;                                  // padded row stride (halves)
        static_assert(BN == 256 && WN == 4 && WM == 2 && BM == 256, "Q8_K epilogue layout");
        static_assert(Q2A_GELU_C_BYTES + 128 * RSH * 2 <= LDS_BYTES, "Q8_K staging exceeds LDS");
        _Float16 * tl = (_Float16 *) (lds_raw + Q2A_GELU_C_BYTES);
        float * sd = (float *) (lds_raw + Q2A_GELU_C_BYTES + 128 * RSH * 2);   // d of the pass's 128 rows
        _Float16 * sa = (_Float16 *) (sd + 128);                                // their bsum operands [128][16]
        static_assert(Q2A_GELU_C_BYTES + 128 * RSH * 2 + 128 * 4 + 128 * 32 <= LDS_BYTES, "Q8_K side staging exceeds LDS");
        const uint16_t * lut = (const uint16_t *) lds_raw;
        const int kb = n0 / 256;
        f4 bias4[NJ];   // C^T tiles: columns 16j + 4(lane>>4) + r of row 16i + (lane&15)
#pragma unroll
        for (int j = 0; j < NJ; ++j) bias4[j] = *(const f4 *) (p.bias + n0 + wn * 64 + j * 16 + (lane >> 4) * 4);
        __syncthreads();   // the staging overlaps the scale buffer the final multiply just read
#pragma unroll
        for (int ps = 0; ps < 2; ++ps) {
            if (wm == ps) {
                typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; j += 2) {
                        float xs[8];
                        _Float16 ys[8];
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            xs[r] = acc[i][j][r] + bias4[j][r];
                            xs[4 + r] = acc[i][j + 1][r] + bias4[j + 1][r];
                        }
                        gelu_c16_x8(xs, ys, lut);
#pragma unroll
                        for (int jj = 0; jj < 2; ++jj) {
                            const h4_t hv = {ys[4 * jj], ys[4 * jj + 1], ys[4 * jj + 2], ys[4 * jj + 3]};
                            *(h4_t *) (tl + (i * 16 + (lane & 15)) * RSH + wn * 64 + (j + jj) * 16 + (lane >> 4) * 4) = hv;
                        }
                    }
            }
            __syncthreads();
            // 16 lanes per row, four rows per wave-iteration, 16 rows per wave per pass
            const int sub = lane & 15;
#pragma unroll
            for (int it = 0; it < 4; ++it) {
                const int rl = wave * 16 + it * 4 + (lane >> 4);
                const int m = m0 + ps * 128 + rl;
                typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
                const h8_t h0 = *(const h8_t *) (tl + rl * RSH + sub * 16);
                const h8_t h1 = *(const h8_t *) (tl + rl * RSH + sub * 16 + 8);
                float v[16];
#pragma unroll
                for (int e = 0; e < 8; ++e) { v[e] = (float) h0[e]; v[8 + e] = (float) h1[e]; }
                float d;
                int sm;
                quant_q8k_row16c(v, sub, p.outH + (int64_t) min(m, p.M - 1) * p.ldo + n0 + sub * 16, m < p.M, d, sm);
                if (sub == 0) sd[rl] = d;
                if ((sub & 1) == 0) {   // the bsum operand pair (64·hi + lo = bsum32, both exact in fp16)
                    const int hi = (sm >= 0) ? (sm >> 6) : -((-sm + 63) >> 6);
                    typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
                    *(h2_t *) (sa + rl * 16 + sub) = h2_t{(_Float16) (float) hi, (_Float16) (float) (sm - 64 * hi)};
                }
            }
            __syncthreads();
            // the pass's side outputs are contiguous in their block-major arrays (rows m0 + 128ps ..): d 512 B, bsum
            // operands 4 KiB — whole 16-B pieces per lane instead of one 4-B write per row (partial sectors)
            const int mb = m0 + ps * 128;
            if (tid < 32) {
                const int r0 = 4 * tid;
                float * dst = p.qdy + (int64_t) kb * p.dy_ld + mb + r0;
                if (mb + r0 + 3 < p.M) *(float4 *) dst = *(const float4 *) (sd + r0);
                else for (int r = 0; r < 4; ++r) if (mb + r0 + r < p.M) dst[r] = sd[r0 + r];
            }
            if (tid < 256) {
                const int r = tid >> 1;
                if (mb + r < p.M)
                    *(uint4 *) (p.qaext + ((int64_t) kb * p.dy_ld + mb + r) * 16 + (tid & 1) * 8) =
                        *(const uint4 *) (sa + r * 16 + (tid & 1) * 8);
            }
            __syncthreads();
        }
        return;
    } else if constexpr (EPI == Q2A_EPI_GELU_Q8K) {
        // fc1 + GELU + Q8_K quantization of the produced activation (the conversion ggml applies before fc2,
        // quantize_row_q8_K_ref): the 256-column tile is exactly one Q8_K block per row. Stage 64 rows x 256 f32
        // through LDS per pass, then one wave quantizes one row (a float4 per lane) exactly like k_rownorm.
        static_assert(BN == 256 && WN == 4, "Q8_K epilogue needs a 256-column tile");
        constexpr int RS = 260;                               // padded row stride (floats)
        constexpr int PRQ = 64;
        static_assert(PRQ * RS * 4 <= 2 * OPB, "Q8_K staging exceeds LDS");
        float * tl = (float *) lds_raw;
        const int kb = n0 / 256;
        f4 bias4[NJ];   // C^T tiles: columns 16j + 4(lane>>4) + r of row 16i + (lane&15)
#pragma unroll
        for (int j = 0; j < NJ; ++j) bias4[j] = *(const f4 *) (p.bias + n0 + wn * 64 + j * 16 + (lane >> 4) * 4);
        __syncthreads();
#pragma unroll
        for (int ps = 0; ps < BM / PRQ; ++ps) {
            if (wm * (BM / WM) / PRQ == ps || (BM / WM) > PRQ) {
#pragma unroll
                for (int i = 0; i < MI; ++i) {
                    const int rw = wm * (BM / WM) + i * 16;          // tile row of this 16-row block
                    if (rw < ps * PRQ || rw >= (ps + 1) * PRQ) continue;
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        f4 gv;
#pragma unroll
                        for (int r = 0; r < 4; ++r) gv[r] = gelu_lut(acc[i][j][r] + bias4[j][r], p.gelu_tab);
                        *(f4 *) (tl + (rw - ps * PRQ + (lane & 15)) * RS + wn * 64 + j * 16 + (lane >> 4) * 4) = gv;
                    }
                }
            }
            __syncthreads();
#pragma unroll
            for (int rr = 0; rr < PRQ / NW; ++rr) {
                const int rl = wave * (PRQ / NW) + rr;
                const int m = m0 + ps * PRQ + rl;
                if (m < p.M) {
                    const float4 y = *(const float4 *) (tl + rl * RS + 4 * lane);
                    quant_q8k_block(y, lane, p.outH + (int64_t) m * p.ldo + n0 + 4 * lane, p.qdy + (int64_t) kb * p.dy_ld + m,
                                    p.qaext + ((int64_t) kb * p.dy_ld + m) * 16);
                }
            }
            __syncthreads();
        }
        return;
    }

    // ---- epilogue. The accumulators are C^T tiles (the MFMAs take W as A and the activations as B): lane holds the
    // 4 CONSECUTIVE output columns n = 16j + 4q + r (q = lane>>4) of ONE row m = 16i + (lane&15), so results go to
    // memory straight from registers: f32 outputs as one float4 per (i, j); fp16 outputs as 16 B after one lane
    // exchange (xor 16) that pairs column chunks of tiles j and j+1. Only V^T (t-major) is transposed through LDS.
    constexpr int WR = BM / WM, WC = BN / WN;        // rows x cols owned by a wave (WC == 64)
    static_assert(WC == 64 && NJ == 4, "epilogue assumes 64 columns per wave");
    const int rbase = m0 + wm * WR, cbase = n0 + wn * WC;
    const int q = lane >> 4, l16 = lane & 15;
    int part = 0;
    if (EPI == Q2A_EPI_QKV) part = cbase / p.D;     // q | k | v: uniform per wave (D % 64 == 0)
    f4 bias4[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
        bias4[j] = (EPI == Q2A_EPI_STORE_F && !p.store_bias) ? f4{0.f, 0.f, 0.f, 0.f}
                                                               : *(const f4 *) (p.bias + cbase + j * 16 + 4 * q);
    const float vscale = (EPI == Q2A_EPI_QKV && part == 0) ? p.qscale : 1.0f;
    const uint16_t * lut = (const uint16_t *) lds_raw;
    // per-element value before the store: bias, GELU (LDS table when staged), Q scale
    // (no FMA contraction across the value: a later hi/lo split v - fp16(v) must see the ROUNDED v in every tile
    // regime — contracted into fma(acc + bias, qscale, -hi) it would not, and the regimes would differ in Q lo)
    auto val = [&](int i, int j, int r) -> float {
#pragma clang fp contract(off)
        float v = acc[i][j][r];
        if (EPI != Q2A_EPI_STORE_F || p.store_bias) v = v + bias4[j][r];
        if (LUT_EPI && EPI != Q2A_EPI_GELU_H) v = gelu_lut_c(v, lut);
        else if (!LUT_EPI && (EPI == Q2A_EPI_GELU_H || EPI == Q2A_EPI_GELU_F || EPI == Q2A_EPI_CONV2)) v = gelu_lut(v, p.gelu_tab);
        if (EPI == Q2A_EPI_QKV) v = v * vscale;   // ggml_scale after the bias add (:2054), exact 2^-3
        if (EPI == Q2A_EPI_STORE_F && p.out_scale != 0.0f) v = v * p.out_scale;
        return v;
    };
    typedef _Float16 h4v __attribute__((ext_vector_type(4)));
    // 8 fp16 = this lane's 16-B piece of columns [32 jp + 16 (q&1) + 8 (q>>1), +8) from chunks (a: tile 2jp, b: 2jp+1)
    // (v_permlane16_swap: the odd 16-lane rows of a's words trade places with the even rows of b's, VALU only)
    auto pair16 = [&](h4v a, h4v b) -> uint4 {
        uint2 ua, ub;
        __builtin_memcpy(&ua, &a, 8);
        __builtin_memcpy(&ub, &b, 8);
        const auto rx = __builtin_amdgcn_permlane16_swap(ua.x, ub.x, false, false);
        const auto ry = __builtin_amdgcn_permlane16_swap(ua.y, ub.y, false, false);
        return make_uint4(rx[0], ry[0], rx[1], ry[1]);
    };
    // whole 128-B lines per store: x0 / x1 are this lane's 16-B pieces of row 16i + l16 for the two halves of a line;
    // lanes l, l ^ 8 trade one piece (DPP row_ror:8) so that store A covers rows 16i + (l & 7) and store B rows
    // 16i + 8 + (l & 7), 8 rows x 128 B each (instead of 16 rows x 64 B), the upper eight lanes writing the line's
    // second half: column offset + 64 B for l >= 8
    const int hi8 = l16 >> 3;
    auto line_pair = [&](const uint4 & x0, const uint4 & x1, uint4 & a, uint4 & b) {
        const uint32_t p0[4] = {x0.x, x0.y, x0.z, x0.w}, p1[4] = {x1.x, x1.y, x1.z, x1.w};
        uint32_t ra[4], rb[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {   // (scalar selects: a lane-varying select of a vector array went to scratch)
            const uint32_t snd = hi8 ? p0[k] : p1[k];
            const uint32_t rcv = (uint32_t) __builtin_amdgcn_mov_dpp((int) snd, 0x128, 0xF, 0xF, false);   // row_ror:8
            ra[k] = hi8 ? rcv : p0[k];
            rb[k] = hi8 ? p1[k] : rcv;
        }
        a = make_uint4(ra[0], ra[1], ra[2], ra[3]);
        b = make_uint4(rb[0], rb[1], rb[2], rb[3]);
    };
    const int pcol = 16 * (q & 1) + 8 * (q >> 1);    // column of this lane's 16-B piece within a 32-column pair
    if (PIPE == 1 && (EPI == Q2A_EPI_PRE_H || (EPI == Q2A_EPI_QKV && (part < 2 || p.v_rows)))) {
      if constexpr (PIPE == 1 && (EPI == Q2A_EPI_PRE_H || EPI == Q2A_EPI_QKV)) {
        // fp16 outputs of the 8-phase tile (fc1's pre-activation; Q / K hi and lo), staged through LDS so every store
        // instruction writes two WHOLE 512-B output rows: all 8 waves write the tile [256 rows][256 cols] into the idle
        // operand images (16-B granules XOR-swizzled by row: conflict-free 8-B writes of 16 rows and 16-B reads of
        // one row), then each wave stores 32 rows. The register layout's natural store was 16 rows x 64 B per
        // instruction (and a lane exchange per pair of column tiles): the fc1 epilogue cost ~0.3 ms per launch.
        static_assert(BM == 256 && BN == 256 && NW == 8, "staged fp16 epilogue layout");
        constexpr int NPASS = (EPI == Q2A_EPI_QKV && !BF) ? 2 : 1;   // Q / K: the hi image, then the lo image
        constexpr int RB = 256 * 2;                                 // staged row bytes
        char * stg = lds_raw;                                       // 256 x 512 B = 128 KiB (operand images)
        const int orq = EPI == Q2A_EPI_PRE_H && p.o_rpg < p.M;      // a real output-row remap (conv paths only)
        h4v lo[NPASS == 2 ? MI : 1][NPASS == 2 ? NJ : 1];          // the lo image, packed (the accumulators die)
#pragma unroll
        for (int pass = 0; pass < NPASS; ++pass) {
            __syncthreads();   // every wave done with the operand images / the previous pass's staged rows
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                const int row = wm * WR + i * 16 + l16;
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int col = wn * WC + j * 16 + 4 * q;       // 4 consecutive fp16 columns
                    h4v hv;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        if constexpr (EPI == Q2A_EPI_PRE_H) {       // pre-activation (no x <= -10 marker: see
                            hv[r] = (_Float16) val(i, j, r);       // q2a_internal.h, Q2A_EPI_PRE_H)
                        } else if (pass == 0) {                     // hi, and the exact remainder's fp16 (lo)
                            const float v = val(i, j, r);
                            const _Float16 h = to16<BF>(v);
                            hv[r] = h;
                            if constexpr (NPASS == 2) lo[i][j][r] = (_Float16) (v - (float) h);
                        } else {
                            if constexpr (NPASS == 2) hv[r] = lo[i][j][r];
                        }
                    }
                    *(h4v *) (stg + row * RB + (((col >> 3) ^ (row & 31)) << 4) + ((col & 4) << 1)) = hv;
                }
            }
            __syncthreads();
            Q2A_STAMP(ST && pass == NPASS - 1, 4);
            const int g = lane & 31;
#pragma unroll 4
            for (int k = 0; k < 16; ++k) {
                const int row = wave * 32 + 2 * k + (lane >> 5), m = m0 + row;
                const uint4 v = *(const uint4 *) (stg + row * RB + ((g ^ (row & 31)) << 4));
                if (m >= p.M || !Q2A_ST) continue;
                if constexpr (EPI == Q2A_EPI_PRE_H) {
                    const int64_t orow = orq ? (int64_t) (m / p.o_rpg) * p.o_gstride + m % p.o_rpg + p.o_off : (int64_t) m + p.o_off;
                    q2a_st(v, (uint4 *) (p.outH + orow * p.ldo + n0 + g * 8));
                    if (p.o_dup) *(uint4 *) (p.outH + orow * p.ldo + n0 + g * 8 + p.o_dup) = v;
                } else {
                    q2a_half * dst = pass == 0 ? (part == 0 ? p.qh : part == 1 ? p.kh : p.vt)
                                               : (part == 0 ? p.ql : part == 1 ? p.kl : p.vtl);
                    q2a_st(v, (uint4 *) (dst + (int64_t) m * p.D + n0 - part * p.D + g * 8));
                }
            }
        }
        Q2A_STAMP(ST, 5);
#ifdef Q2A_DIAG_STAMPS
        if (ST) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        Q2A_STAMP(ST, 6);
        Q2A_STAMP_RT(ST, 9);
      }
    } else if (EPI == Q2A_EPI_QKV && part == 2 && !p.v_rows) {
      if constexpr (EPI == Q2A_EPI_QKV) {
            // V^T [clip][head][d][TP]: the wave's WR rows (t) of its 64 columns (d, one head) staged [d][t] in its own LDS
            // region, then stored two d-rows per instruction, 32 lanes x 8 B (4 t) = 256 contiguous bytes per row. (Per
            // 32-row pass with one lane per d-row, every store instruction touched 64 rows of 8 B: 3.5 ms/step more than
            // the bytes cost.) T % 4 == 0, so a 4-t group never straddles a clip boundary.
            const int h = (cbase - 2 * p.D) >> 6;
            const int clip0 = rbase / p.T, t0 = rbase - clip0 * p.T;   // WR <= T: at most one wrap
            // F32-class P.V (vtl set): the lo image fp16(v - fp16(v)) too. Every wave stages its hi | lo pair for
            // half of its rows at a time in its own region (8 x 17 KiB for the 256-row tile), stores both, then the
            // other half: no wave waits for another (one image at a time for the whole WR rows would keep the lo
            // values in registers across the store loop; the whole pair at once does not fit 8 regions)
            const bool two = !BF && p.vtl;
            // stage row blocks [i0, i0 + NI) of the wave's WR rows (t) as [d][t] images with VS halves per d-row, then
            // store them: two d-rows per instruction, 32 lanes x 8 B (4 t) each
            auto vt_epi = [&](char * region, auto i0c, auto nic, auto vsc, bool lo) {
                constexpr int I0 = decltype(i0c)::value, NI = decltype(nic)::value, VS = decltype(vsc)::value;
                static_assert(64 * VS * 2 * 2 <= EPI_WREG || NI == MI, "epilogue staging layout");
                _Float16 * wl = (_Float16 *) region;
                _Float16 * wlo = wl + 64 * VS;
    #pragma unroll
                for (int i = I0; i < I0 + NI; ++i)
    #pragma unroll
                    for (int j = 0; j < NJ; ++j)
    #pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float v = val(i, j, r);
                            const _Float16 vh = to16<BF>(v);
                            const int o = (j * 16 + 4 * q + r) * VS + (i - I0) * 16 + l16;
                            wl[o] = vh;
                            if (lo) wlo[o] = (_Float16) (v - (float) vh);
                        }
                // wave-private region: the wave's LDS writes are ordered before its reads (and its reads before the
                // next call's writes)
                for (int img = 0; img < (lo ? 2 : 1); ++img) {
                    const _Float16 * src = img ? wlo : wl;
                    q2a_half * vdst = img ? p.vtl : p.vt;
                    // LPR lanes per d-row (4 t = 8 B each), 64 / LPR d-rows per store instruction
                    constexpr int LPR = NI * 4 >= 32 ? 32 : NI * 4, RPI = 64 / LPR;
    #pragma unroll
                    for (int dd = 0; dd < 64; dd += RPI) {
                        const int d = dd + lane / LPR;
    #pragma unroll
                        for (int a = lane % LPR; a < NI * 4; a += LPR) {
                            const int ml = I0 * 16 + 4 * a, m = rbase + ml;
                            // one clip (M == T): the tile rows T <= t < TP write V^T's pad columns as zeros (the
                            // attention reads them as zero weights), so no caller has to clear them
                            const bool pad = m >= p.M;
                            if (pad && (p.M != p.T || m >= p.TP)) continue;
                            const bool wrap = !pad && t0 + ml >= p.T;
                            // (a pad row of a wave starting at or past T has clip0 = 1: it is clip 0's t = m)
                            const int clip = pad ? 0 : clip0 + (wrap ? 1 : 0), t = pad ? m : t0 + ml - (wrap ? p.T : 0);
                            const uint2 v = pad ? make_uint2(0u, 0u) : *(const uint2 *) (src + d * VS + 4 * a);
                            if (Q2A_ST) q2a_st(v, (uint2 *) (vdst + (((int64_t) clip * p.H + h) * 64 + d) * p.TP + t));
                        }
                    }
                }
            };
            typedef std::integral_constant<int, 0> c0;
            typedef std::integral_constant<int, MI> cmi;
            typedef std::integral_constant<int, MI / 2> cmh;
            __syncthreads();
            char * region = lds_raw + EPI_OFF + wave * EPI_WREG;
            if (!two) {
                vt_epi(region, c0{}, cmi{}, std::integral_constant<int, WR + 4>{}, false);
            } else if constexpr (MI == 1) {   // 16-row waves: the hi | lo pair of all rows in one pass
                vt_epi(region, c0{}, cmi{}, std::integral_constant<int, WR + 4>{}, true);
            } else {
                vt_epi(region, c0{}, cmh{}, std::integral_constant<int, WR / 2 + 4>{}, true);
                vt_epi(region, cmh{}, cmh{}, std::integral_constant<int, WR / 2 + 4>{}, true);
            }
      }
    } else if (EPI == Q2A_EPI_QKV || EPI == Q2A_EPI_GELU_H || EPI == Q2A_EPI_PRE_H) {
        // output row remap (conv1's padded per-clip rows): one division per wave, its rows span < o_rpg
        constexpr bool REMAP = EPI == Q2A_EPI_GELU_H || EPI == Q2A_EPI_PRE_H;
        const int oq = (REMAP && p.o_rpg < p.M) ? rbase / p.o_rpg : 0;
        const int orr = REMAP ? rbase - oq * p.o_rpg : 0;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            uint4 hvj[2], lvj[2];
#pragma unroll
            for (int jp = 0; jp < NJ / 2; ++jp) {
                h4v ha, hb, la, lb;
                if constexpr (EPI == Q2A_EPI_GELU_H && LUT_EPI) {
                    float xs[8];
                    _Float16 ys[8];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        xs[r] = acc[i][2 * jp][r] + bias4[2 * jp][r];
                        xs[4 + r] = acc[i][2 * jp + 1][r] + bias4[2 * jp + 1][r];
                    }
                    gelu_c16_x8(xs, ys, lut);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        ha[r] = ys[r];
                        hb[r] = ys[4 + r];
                        if (BF) {   // the fp16 GELU value handed on as bf16
                            ha[r] = to16<true>((float) ha[r]);
                            hb[r] = to16<true>((float) hb[r]);
                        }
                    }
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (EPI == Q2A_EPI_GELU_H && LUT_EPI) {
                    } else if (EPI == Q2A_EPI_PRE_H) {   // pre-activation (q2a_internal.h, Q2A_EPI_PRE_H)
                        ha[r] = (_Float16) val(i, 2 * jp, r);
                        hb[r] = (_Float16) val(i, 2 * jp + 1, r);
                    } else {
                        const float va = val(i, 2 * jp, r), vb = val(i, 2 * jp + 1, r);
                        ha[r] = to16<BF>(va);
                        hb[r] = to16<BF>(vb);
                        if (EPI == Q2A_EPI_QKV && !BF) {
                            la[r] = (_Float16) (va - (float) ha[r]);
                            lb[r] = (_Float16) (vb - (float) hb[r]);
                        }
                    }
                }
                hvj[jp] = pair16(ha, hb);
                if (EPI == Q2A_EPI_QKV && !BF) lvj[jp] = pair16(la, lb);
            }
            uint4 hA, hB, lA, lB;
            line_pair(hvj[0], hvj[1], hA, hB);
            if (EPI == Q2A_EPI_QKV && !BF) line_pair(lvj[0], lvj[1], lA, lB);
            const int col = pcol + 32 * hi8;
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const int ml = i * 16 + 8 * hf + (l16 & 7), m = rbase + ml;
                const uint4 hv = hf ? hB : hA;
                if (m < p.M) {
                    if (REMAP) {
                        const bool wrap = orr + ml >= p.o_rpg;
                        const int64_t row = (int64_t) (oq + (wrap ? 1 : 0)) * p.o_gstride + (orr + ml - (wrap ? p.o_rpg : 0)) + p.o_off;
                        if (Q2A_ST) q2a_st(hv, (uint4 *) (p.outH + row * p.ldo + cbase + col));
                        if (p.o_dup) *(uint4 *) (p.outH + row * p.ldo + cbase + col + p.o_dup) = hv;
                    } else {
                        const int64_t o = (int64_t) m * p.D + cbase - part * p.D + col;
                        if (Q2A_ST) q2a_st(hv, (uint4 *) ((part == 0 ? p.qh : part == 1 ? p.kh : p.vt) + o));
                        if (EPI == Q2A_EPI_QKV && !BF && Q2A_ST)
                            q2a_st(hf ? lB : lA, (uint4 *) ((part == 0 ? p.ql : part == 1 ? p.kl : p.vtl) + o));
                    }
                }
            }
        }
    } else if ((EPI == Q2A_EPI_RESID || EPI == Q2A_EPI_STORE_F) && ksplit > 1) {
        // split-K partial: raw accumulators to part[ks] ([M][N] f32); bias and residual in the reduce pass
        float * pb = p.part + (int64_t) ks * p.split_stride;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int m = rbase + i * 16 + l16;
            if (m >= p.M) continue;
#pragma unroll
            for (int j = 0; j < NJ; ++j) *(f4 *) (pb + (int64_t) m * p.N + cbase + j * 16 + 4 * q) = acc[i][j];
        }
    } else if constexpr (EPI == Q2A_EPI_RESID && PIPE) {
        static_assert(MI == 8 && NJ == 4 && NW == 8, "8-phase residual epilogue layout");
        // residual add, 8-phase tile: every load is consumed before the first store. vmcnt retires in order and
        // counts stores, and with loads and stores both pending the compiler waits vmcnt(0): a residual load between
        // the stores of two row blocks waits for the earlier stores to land, eight store round trips per wave.
        //   1. rows 0..63 of the wave's 128 by glds into the idle operand images (16 KiB per wave, 16-B granules
        //      XOR-swizzled by row: the column-chunk reads are conflict-free); one wait
        //   2. their results (acc + bias) + x back into the same LDS slots: acc rows 0..63 are dead
        //   3. rows 64..127 by register loads into the freed registers; one wait
        //   4. stores of rows 0..63 out of LDS, row-contiguous (4 rows x 256 B per instruction instead of 16 rows x
        //      64 B); then rows 64..127's results into the same slots and stored the same way. Integer-address LDS
        //      reads/writes, opaque to the compiler: no vmcnt guard for the glds target behind the stores.
        const float * rsrc = p.resid ? p.resid : p.outF;
        char * rl = lds_raw + wave * (64 * 256);
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int lr = 4 * t + (lane >> 4), ch = (lane & 15) ^ (lr & 15);
            const int m = min(rbase + lr, p.M - 1);
            __builtin_amdgcn_global_load_lds((const void *) (rsrc + (int64_t) m * p.ldo + cbase + ch * 4),
                                             (lds_ptr_t) (rl + t * 1024), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("" : "+v"(bias4[0]), "+v"(bias4[1]), "+v"(bias4[2]), "+v"(bias4[3]));
        const uint32_t rl0 = (uint32_t) (uintptr_t) (const __attribute__((address_space(3))) char *) rl;
        auto slot = [&](int i, int j) -> uint32_t {
            return rl0 + (uint32_t) (i * 16 + l16) * 256 + ((uint32_t) ((4 * j + q) ^ l16) << 4);
        };
#pragma unroll
        for (int i = 0; i < MI / 2; ++i) {
            f4 add[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) asm volatile("ds_read_b128 %0, %1" : "=v"(add[j]) : "v"(slot(i, j)));
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(add[0]), "+v"(add[1]), "+v"(add[2]), "+v"(add[3]));
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                f4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = val(i, j, r) + add[j][r];   // (acc + bias) + x
                asm volatile("ds_write_b128 %0, %1" :: "v"(slot(i, j)), "v"(v) : "memory");
            }
        }
        f4 add_hi[MI / 2][NJ];
#pragma unroll
        for (int i = MI / 2; i < MI; ++i) {
            const int m = min(rbase + i * 16 + l16, p.M - 1);
#pragma unroll
            for (int j = 0; j < NJ; ++j) add_hi[i - MI / 2][j] = *(const f4 *) (rsrc + (int64_t) m * p.ldo + cbase + 16 * j + 4 * q);
        }
#pragma unroll
        for (int i = 0; i < MI / 2; ++i)
            asm volatile("" : "+v"(add_hi[i][0]), "+v"(add_hi[i][1]), "+v"(add_hi[i][2]), "+v"(add_hi[i][3]));
        // stores out of LDS, row-contiguous: instruction k writes rows 4k .. 4k + 3 of the 64-row half, 256 B each
        // (lane l: row 4k + l/16, 16-B chunk l % 16)
        auto store_half = [&](int r0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const int ch = lane & 15;
#pragma unroll
            for (int k0 = 0; k0 < 16; k0 += 8) {   // 8 reads behind one wait, then their 8 stores
                f4 v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int lr = 4 * (k0 + k) + (lane >> 4);
                    asm volatile("ds_read_b128 %0, %1" : "=v"(v[k]) : "v"(rl0 + (uint32_t) lr * 256 + ((uint32_t) (ch ^ (lr & 15)) << 4)));
                }
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                             "+v"(v[7]));
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int m = rbase + r0 + 4 * (k0 + k) + (lane >> 4);
                    if (m < p.M && Q2A_ST) q2a_st(v[k], (f4 *) (p.outF + (int64_t) m * p.ldo + cbase + ch * 4));
                }
            }
        };
        store_half(0);
        // rows 64..127: (acc + bias) + x into the same LDS slots (each wave reads only its own region, in order), then
        // stored the same way
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = MI / 2; i < MI; ++i) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                f4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = val(i, j, r) + add_hi[i - MI / 2][j][r];
                asm volatile("ds_write_b128 %0, %1" :: "v"(slot(i - MI / 2, j)), "v"(v) : "memory");
            }
        }
        store_half(64);
    } else {
        // f32 outputs: residual add (O-proj, fc2), GELU (+ positional rows for conv2), plain store; whole 128-B lines per
        // store (line_pair on the column tiles 2jp, 2jp + 1: 8 rows x 128 B instead of 16 rows x 64 B). Every lane
        // computes its row (loads clamped to row M-1) so the lane exchange sees defined values; stores check the row.
        const int pq = EPI == Q2A_EPI_CONV2 ? rbase / p.T : 0;
        const int pt0 = EPI == Q2A_EPI_CONV2 ? rbase - pq * p.T : 0;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int ml = i * 16 + l16, m = rbase + ml, mc = min(m, p.M - 1);
            f4 add[NJ];
            if (EPI == Q2A_EPI_RESID) {
                const float * rrow = (p.resid ? p.resid : p.outF) + (int64_t) mc * p.ldo + cbase + 4 * q;
#pragma unroll
                for (int j = 0; j < NJ; ++j) add[j] = *(const f4 *) (rrow + 16 * j);
            } else if (EPI == Q2A_EPI_CONV2) {
                const int tpos = pt0 + ml >= p.T ? pt0 + ml - p.T : pt0 + ml;
                const float * perow = p.pe + (int64_t) tpos * p.ldo + cbase + 4 * q;
#pragma unroll
                for (int j = 0; j < NJ; ++j) add[j] = *(const f4 *) (perow + 16 * j);
            }
            f4 v[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[j][r] = val(i, j, r);
                    if (EPI == Q2A_EPI_RESID) v[j][r] = v[j][r] + add[j][r];        // (acc + bias) + x
                    else if (EPI == Q2A_EPI_CONV2) v[j][r] = add[j][r] + v[j][r];   // pe + gelu(...)
                }
                if (EPI == Q2A_EPI_GELU_F && p.outH && m < p.M) {   // fp16 copy (exact: GELU table values are fp16) for the next GEMM
                    typedef _Float16 h4s __attribute__((ext_vector_type(4)));
                    const h4s hv = {(_Float16) v[j][0], (_Float16) v[j][1], (_Float16) v[j][2], (_Float16) v[j][3]};
                    *(h4s *) (p.outH + (int64_t) m * p.ldo + cbase + 4 * q + 16 * j) = hv;
                }
            }
#pragma unroll
            for (int jp = 0; jp < NJ / 2; ++jp) {
                uint4 a, b;
                line_pair(__builtin_bit_cast(uint4, v[2 * jp]), __builtin_bit_cast(uint4, v[2 * jp + 1]), a, b);
                const int col = cbase + 4 * q + 16 * (2 * jp + hi8);
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {
                    const int mr = rbase + i * 16 + 8 * hf + (l16 & 7);
                    if (mr < p.M && Q2A_ST) q2a_st(hf ? b : a, (uint4 *) (p.outF + (int64_t) mr * p.ldo + col));
                }
            }
        }
        Q2A_STAMP(ST, 5);
#ifdef Q2A_DIAG_STAMPS
        if (ST) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        Q2A_STAMP(ST, 6);
        Q2A_STAMP_RT(ST, 9);
    }
#undef LDS_STAGE
}

// split-K reduce: out[m][n] = ((p_0 + p_1 + ...) + bias[n]) + x[m][n], partials summed in split order; x = resid rows
// or out itself. RES = 0 (Q2A_EPI_STORE_F): ((p_0 + p_1 + ...) [+ bias[n]]) [* oscale]
template <int RES>
__global__ void k_split_reduce(const float * __restrict__ part, int S, int64_t stride, int M, int N, const float * bias,
                               float * out, int64_t ldo, const float * resid, float oscale) {
    const int64_t i4 = ((int64_t) blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i4 >= (int64_t) M * N) return;
    const int m = (int) (i4 / N), n = (int) (i4 - (int64_t) m * N);
    f4 acc = *(const f4 *) (part + i4);
    for (int s = 1; s < S; ++s) {
        const f4 v = *(const f4 *) (part + s * stride + i4);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = acc[r] + v[r];
    }
    f4 * o = (f4 *) (out + (int64_t) m * ldo + n);
    if (RES) {
        const f4 b = *(const f4 *) (bias + n);
        f4 x = resid ? *(const f4 *) (resid + (int64_t) m * ldo + n) : *o;
#pragma unroll
        for (int r = 0; r < 4; ++r) x[r] = (acc[r] + b[r]) + x[r];
        *o = x;
    } else {
        if (bias) {
            const f4 b = *(const f4 *) (bias + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = acc[r] + b[r];
        }
        if (oscale != 0.0f) {
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = acc[r] * oscale;
        }
        *o = acc;
    }
}

template <int BM, int BN, int WM, int WN, int EPI, int BLK, int PIPE = 0>
hipError_t launch_cfg(const q2a_gemm_args & a, hipStream_t s) {
    const bool grouped = !PIPE && (BLK == 0 || BLK == 256) && EPI == Q2A_EPI_STORE_F && a.ngroup == 2;
    const bool split = !PIPE && (BLK == 0 || BLK == Q2A_BLK_BF16 || BLK == 32) &&
                       (EPI == Q2A_EPI_RESID || EPI == Q2A_EPI_STORE_F) && a.ksplit > 1 && !grouped;
    const int nwg = (a.N / BN) * ((a.M - a.m_base + BM - 1) / BM) * (split ? a.ksplit : 1) * (grouped ? 2 : 1);
    hipLaunchKernelGGL((k_gemm<BM, BN, WM, WN, EPI, BLK, PIPE>), dim3(nwg), dim3(WM * WN * 64), 0, s, a);
    if (split) {
        const int64_t n4 = (int64_t) a.M * a.N / 4;
        if constexpr (EPI == Q2A_EPI_RESID)
            hipLaunchKernelGGL(k_split_reduce<1>, dim3((unsigned) ((n4 + 255) / 256)), dim3(256), 0, s, a.part, a.ksplit,
                               a.split_stride, a.M, a.N, a.bias, a.outF, a.ldo, a.resid, 0.0f);
        else
            hipLaunchKernelGGL(k_split_reduce<0>, dim3((unsigned) ((n4 + 255) / 256)), dim3(256), 0, s, a.part, a.ksplit,
                               a.split_stride, a.M, a.N, a.store_bias ? a.bias : nullptr, a.outF, a.ldo, a.resid, a.out_scale);
    }
    return hipGetLastError();
}

// Tile regimes (every regime sums K in the same order, so they change speed, not results). The rejected tile / raster /
// stagger / tail alternatives measured in rounds 1-5 are recorded in DESIGN.md and diag/experiment_knobs_r05.patch.

// M-waves of the small-batch tiles (a single clip's GEMMs): 2 = 4-wave workgroups, 4 = 8 waves (16 / 32 rows per wave;
// every wave keeps 64 columns, so the K order per output and the epilogues are those of the 4-wave form). The narrow
// 64x128 tiles run 8 waves: a single clip's O / fc2 tiles are glds-issue-bound at one wave per SIMD; two per SIMD
// overlap one wave's issue with the other's MFMAs — Q4_K one clip 8.35 -> 7.73 ms per encode (fc2 2.26 -> 1.78, O
// 0.79 -> 0.68), F16 unchanged; the 128x128 tiles with 8 waves: F16 fc1 -5 %, Q4_K QKV / fc1 +18 %: kept at 4
// (round 5, diag/gpurun_r05e.sh, profiles/r05e_small_tiles_8waves.json)

// small M (one or a few clips): 64-row tiles when 128x128 tiles would leave CUs idle
bool narrow_tiles(int M, int N) {
    return (int64_t) ((M + 127) / 128) * (N / 128) < 256;
}

bool wide_tiles(int M, int N) {
    // big M: 256-wide tiles on 8 waves (k-quant variants keep 128 rows: the per-block accumulators double the
    // register footprint); small M (a single clip): 128x128 on 4 waves so the grid still covers the 256 CUs
    return (int64_t) ((M + 255) / 256) * (N / 256) >= 512 && N % 256 == 0;
}

// compute units of the current device, cached per device ordinal
int cu_count() {
    static int cus[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (!cus[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
        cus[dev] = n;
    }
    return cus[dev];
}

// The 8-phase kernel holds a whole CU per 256x256 tile, so a grid whose last round is partly filled leaves the rest of
// the chip idle for one whole tile time: the O / fc2 GEMMs at 64 clips are 375 x 5 = 1 875 tiles = 7.32 rounds on 256
// CUs, fc1 7 500 = 29.3. When the last round would fill at most 5/8 of the CUs, the whole rounds run on the 8-phase
// kernel (rows [0, m_main)) and the remaining rows on 128x128 tiles (two workgroups per CU, a quarter of the work per
// tile), which sum K in the same order with the same block recurrence: outputs are bit-identical to the one-launch grid
// (batch invariance). Only for epilogues whose row addressing is absolute (no per-tile row remap), and
// only for deep K: measured at 64 clips Q4_K (diag/gpurun_r03ta.sh, same box, alternating) fc2 (K = 5120) 45.2 -> 44.4
// ms/step, but O (K = 1280) 17.05 -> 17.3 and fc1 (K = 1280) 48.6 -> 48.75 — a shallow tile's partial round costs less
// than the second launch and the 128x128 tiles' lower rate.
template <int EPI, int BLK>
hipError_t launch_pipe8(const q2a_gemm_args & a, hipStream_t s) {
    if constexpr ((EPI == Q2A_EPI_PRE_H || EPI == Q2A_EPI_QKV) && BLK == 256) {
        // persistent tiles (k_gemm PIPE = 2): whole 256-row tiles only, at least two Q4_K blocks; Q|K|V only with V
        // row-major (the V^T image needs the LDS-staged transposing epilogue)
        const int cus = cu_count();
        const int ntl = (a.N / 256) * ((a.M - a.m_base) / 256);
        const int grid = std::min(ntl, cus / 8 * 8);
        // (the workgroup's tile list holds 64 entries)
        if ((a.M - a.m_base) % 256 == 0 && a.K >= 512 && ntl > 0 && cus >= 8 && ntl <= 64 * grid &&
            (EPI != Q2A_EPI_QKV || (a.v_rows && a.vtl && a.D % 256 == 0))) {
            hipLaunchKernelGGL((k_gemm<256, 256, 2, 4, EPI, BLK, 2>), dim3(grid), dim3(512), 0, s, a);
            return hipGetLastError();
        }
    }
    constexpr bool TAILABLE = (EPI == Q2A_EPI_RESID || EPI == Q2A_EPI_PRE_H || EPI == Q2A_EPI_GELU_H);
    if constexpr (TAILABLE) {
        const int cus = cu_count();
        const int nbn = a.N / 256, nbm = (a.M - a.m_base + 255) / 256;
        const int64_t ntl = (int64_t) nbn * nbm, rem = cus > 0 ? ntl % cus : 0;
        const int m_main = (int) ((ntl - rem) / nbn);   // whole M-tiles inside the full rounds
        if (a.K >= 4096 && a.m_base == 0 && rem > 0 && rem * 8 <= (int64_t) cus * 5 && m_main > 0 && m_main < nbm) {
            q2a_gemm_args h = a;
            h.M = m_main * 256;
            const hipError_t err = launch_cfg<256, 256, 2, 4, EPI, BLK, 1>(h, s);
            if (err != hipSuccess) return err;
            q2a_gemm_args t = a;
            t.m_base = m_main * 256;
            return launch_cfg<128, 128, 2, 2, EPI, BLK>(t, s);
        }
    }
    return launch_cfg<256, 256, 2, 4, EPI, BLK, 1>(a, s);
}

// the 8-phase kernels: 256x256 tiles, 32-bit operand offsets, K-steps in pairs (fp16) or whole Q4_K blocks
bool pipe8_ok(const q2a_gemm_args & a, int blk) {
    if (!wide_tiles(a.M, a.N)) return false;
    const int64_t last = (int64_t) ((a.M - 1) / a.a_rpg) * a.a_gstride + (int64_t) ((a.M - 1) % a.a_rpg) * a.a_step;
    if ((last + 1) * a.lda >= (1ll << 32) || (int64_t) a.N * a.ldw >= (1ll << 32)) return false;
    if (blk == 0 || blk == Q2A_BLK_BF16) return (a.K / BK) % 2 == 0;
    if (blk == 256) return (a.K / BK) % 4 == 0;
    return false;
}

template <int EPI>
hipError_t launch_epi(const q2a_gemm_args & a, int blk, hipStream_t s) {
    const bool big = wide_tiles(a.M, a.N);
    const bool p8 = pipe8_ok(a, blk) && (blk != 256 || a.beta);
    if constexpr (EPI == Q2A_EPI_GELU_Q8K) {
        if (!big || blk != 256) return hipErrorInvalidValue;
        if (p8) return launch_cfg<256, 256, 2, 4, EPI, 256, 1>(a, s);
        return launch_cfg<128, 256, 2, 4, EPI, 256>(a, s);
    } else {
        // every configuration sums K in the same order (64-deep K-steps, two 32-deep MFMAs each; Q4_K with the
        // same block recurrence): a clip's outputs are bit-identical whichever tile regime its batch size selects
        const bool narrow = !big && narrow_tiles(a.M, a.N) && a.ksplit <= 1 && a.ngroup != 2;
        if (blk == 0) {
            if (p8) return launch_pipe8<EPI, 0>(a, s);
            if (narrow) return launch_cfg<64, 128, 4, 2, EPI, 0>(a, s);
            return big ? launch_cfg<256, 256, 2, 4, EPI, 0>(a, s) : launch_cfg<128, 128, 2, 2, EPI, 0>(a, s);
        }
        if constexpr (EPI == Q2A_EPI_GELU_H || EPI == Q2A_EPI_CONV2 || EPI == Q2A_EPI_STORE_F) {
            // the conv GEMMs' exact accumulation: 64x128 tiles in every regime (one K order, batch invariant)
            if (blk == Q2A_BLK_EXACT) return launch_cfg<64, 128, 2, 2, EPI, Q2A_BLK_EXACT>(a, s);
        }
        if (blk == 256) {
            if (!a.beta || !a.gamma) return hipErrorInvalidValue;   // the block recurrence needs beta / gamma
            if (p8) return launch_pipe8<EPI, 256>(a, s);
            if (narrow) return launch_cfg<64, 128, 4, 2, EPI, 256>(a, s);
            return big ? launch_cfg<128, 256, 2, 4, EPI, 256>(a, s) : launch_cfg<128, 128, 2, 2, EPI, 256>(a, s);
        }
        if (blk == 32) {
            if (narrow) return launch_cfg<64, 128, 4, 2, EPI, 32>(a, s);
            return big ? launch_cfg<128, 256, 2, 4, EPI, 32>(a, s) : launch_cfg<128, 128, 2, 2, EPI, 32>(a, s);
        }
        if constexpr (EPI == Q2A_EPI_QKV || EPI == Q2A_EPI_RESID || EPI == Q2A_EPI_GELU_H || EPI == Q2A_EPI_STORE_F) {
            if (blk == Q2A_BLK_BF16) {
                constexpr int B16 = Q2A_BLK_BF16;
                if (p8) return launch_pipe8<EPI, B16>(a, s);
                if (narrow) return launch_cfg<64, 128, 4, 2, EPI, B16>(a, s);
                return big ? launch_cfg<256, 256, 2, 4, EPI, B16>(a, s) : launch_cfg<128, 128, 2, 2, EPI, B16>(a, s);
            }
        }
        return hipErrorInvalidValue;
    }
}

}  // namespace

// Split-K of the small-tile residual GEMMs: off in the product library (round 1's single-clip form, kept for the
// q2a_test_* entry points' ksplit argument). Partial sums combined across splits change the fp32 summation order, so a clip's output would
// depend on whether its batch took the small-tile or the 8-phase regime; without it every regime sums K identically
// (batch invariance).
static bool splitk_on() { return false; }

int q2a_gemm_resid_ksplit(int M, int N, int K, int blk) {
    if (!splitk_on() || !(blk == 0 || blk == Q2A_BLK_BF16) || wide_tiles(M, N) || N % 128) return 0;
    const int nk = K / BK;
    const int S = K >= 4096 ? 4 : K >= 1024 ? 2 : 0;
    return S && nk % S == 0 ? S : 0;
}

int q2a_gemm_kq_ksplit(int M, int N, int K, int blk) {
    // Q8_0 / Q4_0 only (opt-in); Q4_K never splits (its block recurrence runs through every K-block in order)
    if (!splitk_on() || blk != 32 || wide_tiles(M, N) || N % 128) return 0;
    // whole scale groups per split: 4 K-steps per Q4_K block, 1 per Q8_0/Q4_0 pair of blocks
    const int nk = K / BK, unit = blk == 256 ? 4 : 1;
    for (int S : {4, 5, 2, 3})
        if (nk % (S * unit) == 0 && nk / S >= 2 * unit) return S;
    return 0;
}

hipError_t q2a_launch_gemm(const q2a_gemm_args & a_in, int epi, int blk, hipStream_t s) {
    q2a_gemm_args a = a_in;
    a.m_base = 0;
    if (a.ngroup == 2 && (epi != Q2A_EPI_STORE_F || (blk != 0 && blk != 256) || wide_tiles(a.M, a.N))) return hipErrorInvalidValue;
    if (a.ngroup == 2 && blk == 256 && (!a.dx2 || !a.beta2 || !a.gamma2 || !a.wext2)) return hipErrorInvalidValue;
    if (!(epi == Q2A_EPI_RESID || (epi == Q2A_EPI_STORE_F && a.split_store)) || !a.part || a.ldo != a.N || a.ngroup == 2)
        a.ksplit = 0;
    else if (blk == 256 || blk == 32) a.ksplit = a.split_kq ? q2a_gemm_kq_ksplit(a.M, a.N, a.K, blk) : 0;
    else a.ksplit = q2a_gemm_resid_ksplit(a.M, a.N, a.K, blk);
    if (a.N % 128 != 0 || a.K % BK != 0 || a.M <= 0) return hipErrorInvalidValue;
    if (blk > 1 && (a.K % blk != 0)) return hipErrorInvalidValue;
    switch (epi) {
        case Q2A_EPI_QKV: return launch_epi<Q2A_EPI_QKV>(a, blk, s);
        case Q2A_EPI_RESID: return launch_epi<Q2A_EPI_RESID>(a, blk, s);
        case Q2A_EPI_GELU_H: return launch_epi<Q2A_EPI_GELU_H>(a, blk, s);
        case Q2A_EPI_CONV2: return launch_epi<Q2A_EPI_CONV2>(a, blk, s);
        case Q2A_EPI_GELU_F: return launch_epi<Q2A_EPI_GELU_F>(a, blk, s);
        case Q2A_EPI_STORE_F: return launch_epi<Q2A_EPI_STORE_F>(a, blk, s);
        case Q2A_EPI_GELU_Q8K: return launch_epi<Q2A_EPI_GELU_Q8K>(a, blk, s);
        case Q2A_EPI_PRE_H: return launch_epi<Q2A_EPI_PRE_H>(a, blk, s);
        default: return hipErrorInvalidValue;
    }
}

bool q2a_gemm_wide_tiles(int M, int N, int blk) { (void) blk; return wide_tiles(M, N); }
int q2a_cu_count() { return cu_count(); }

bool q2a_gemm_pipe8(const q2a_gemm_args & a, int blk) { return pipe8_ok(a, blk) && (blk != 256 || a.beta); }

#ifdef Q2A_DIAG_STAMPS
// diagnostic builds only: copy the stamp array (Q2A_DIAG_STAMPS comment above) to the host
extern "C" int q2a_diag_stamps(uint64_t * host, int64_t n) {
    n = n < (int64_t) (sizeof(g_q2a_stamps) / 8) ? n : (int64_t) (sizeof(g_q2a_stamps) / 8);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_q2a_stamps), (size_t) n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}
extern "C" int q2a_diag_stamps_clear(void) {
    static uint64_t z[16384 * 2 * Q2A_STAMP_SLOTS];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_q2a_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -3;
}
#endif
