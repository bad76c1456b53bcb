// q2a_internal.h — device-side argument structs and launch wrappers shared by the kernel files and the
// engine. Not part of the public C ABI (include/q2a_encoder.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 q2a_half;

// sets the calling thread's q2a_last_error() text (defined with the engine; used by q2a_group.cpp)
extern "C" void q2a_internal_set_error(const char * msg);
// an engine's device-layout weight blob (device pointer, bytes) and device ordinal (used by q2a_group.cpp to broadcast
// an open engine's weights instead of packing the model file again)
struct q2a_engine;
extern "C" int q2a_internal_engine_blob(const q2a_engine * e, const void ** blob, int64_t * bytes, int * device);

// Epilogue kinds of the fused weight GEMM (one template instantiation each)
enum q2a_epi {
    Q2A_EPI_QKV = 0,        // +bias, Q*(1/sqrt(dh)) -> Qh/Ql, K -> Kh/Kl (fp16 hi/lo), V -> Vt (fp16, [clip][head][d][TP])
    Q2A_EPI_RESID = 1,      // outF[m][n] = (acc + bias[n]) + outF[m][n]           (O-proj, fc2)
    Q2A_EPI_GELU_H = 2,     // outH[orow(m)][n] = fp16(gelu_lut(acc + bias[n]))   (fc1, conv1)
    Q2A_EPI_CONV2 = 3,      // outF[m][n] = gelu_lut(acc + bias[n]) + pe[m % T][n] (conv2 + positional add)
    Q2A_EPI_GELU_F = 4,     // outF[m][n] = gelu_lut(acc + bias[n])               (fc1 on the quantized paths)
    Q2A_EPI_STORE_F = 5,    // outF[m][n] = acc                                   (unit tests)
    Q2A_EPI_GELU_Q8K = 6,   // gelu_lut(acc + bias) quantized to Q8_K in-tile: codes -> outH, d -> dy, bsums -> aext
                            // (fc1 on the Q4_K path; needs the 256-column tile = one Q8_K block per row)
    Q2A_EPI_PRE_H = 7,      // outH[m][n] = fp16(acc + bias[n]): the fc1 pre-activation, whose GELU (the fp16 LUT)
                            // the Q8_K quantizer applies (q2a_launch_gelu_quant_q8k). ggml's x <= -10 branch (+0) needs
                            // no marker: for every fp16 h <= -10 the table holds -0 (tanhf saturates: 0.5 h (1 - 1)),
                            // or +0 (the patched -inf entry), and Q8_K turns +0 and -0 into the same code 0 (|x| for
                            // the block max, nearest_int(-0) = 0), so the fc2 operand is bit-identical
};

// compact GELU table: entries for fp16 bits 0x0000..0x4900 (+0..+10) then 0x8000..0xC900 (-0..-10), padded to
// five 16 KiB glds images
constexpr int Q2A_GELU_C_HALF = 0x4901;
constexpr int Q2A_GELU_C_BYTES = 5 * 16384;
static_assert(2 * Q2A_GELU_C_HALF * 2 <= Q2A_GELU_C_BYTES, "compact GELU table size");

struct q2a_gemm_args {
    // A: fp16 [rows][lda]; logical row m lives at row  (m / a_rpg) * a_gstride + (m % a_rpg) * a_step
    const q2a_half * A;
    int64_t lda;
    int a_rpg, a_gstride, a_step;
    // W: fp16 [N][ldw] (row n = output feature, K contiguous)
    const q2a_half * W;
    int64_t ldw;
    int M, N, K;
    // epilogue
    const float * bias;
    float * outF;
    int64_t ldo;
    q2a_half * outH;                  // (Q2A_EPI_GELU_F: optional fp16 copy of outF, same row stride)
    int o_rpg, o_gstride, o_off;      // output row remap for outH: (m / o_rpg) * o_gstride + (m % o_rpg) + o_off
    int o_dup;                        // Q2A_EPI_GELU_H: also store the row at column offset o_dup (0 = no copy)
    const float * pe;
    int T;                            // positions per clip
    q2a_half *qh, *ql, *kh, *kl, *vt;
    int D, H, TP;
    float qscale;
    const uint16_t * gelu_tab;        // 65536-entry fp16 table: fp16(gelu_f32(fp16 x)) (ggml.c:3797-3806)
    const uint16_t * gelu_c;          // compact |x| <= 10 image of it (Q2A_GELU_C_BYTES, staged into LDS by the 8-phase GEMM)
    // blocked (k-quant) accumulation: acc += dy[b][m]*dx[b][n]*S1 - dy[b][m]*dmin[b][n]*S2 per K-block b.
    // All block arrays are block-major so one block's scales for a tile are contiguous (staged through LDS).
    const float * dy;                 // [nblk][dy_ld]
    const float * dx;                 // [nblk][N]
    const float * dmin;               // [nblk][N] (Q4_K only)
    const q2a_half * aext;            // [nblk][dy_ld][16] bsum hi/lo pairs (Q4_K only)
    const q2a_half * wext;            // [nblk][N][16] (64*m_j, m_j) pairs (Q4_K only)
    const float * beta;               // [nblk][N] dx_{b-1}/dx_b  (Q4_K 8-phase path: block-ratio rescaling)
    const float * gamma;              // [nblk][N] -(dmin_b/dx_b), negated so the recurrence's addend is gamma * S2
    float * qdy;                      // Q2A_EPI_GELU_Q8K outputs: block-major d [N/256][dy_ld] and
    q2a_half * qaext;                 //   bsum operand [N/256][dy_ld][16] of the produced activation
    int nblk;
    // deterministic split-K of the small-tile residual GEMMs (set by the launcher): split s of ksplit writes its
    // partial sum to part + s * split_stride ([M][N] f32) and a reduce pass applies ((p0 + p1 ...) + bias) + x
    int ksplit;
    float * part;
    int64_t split_stride;
    int dy_ld;                        // row stride of dy/aext (M rounded up to 256)
    // ggml-backend fusions (ggml-q2a.hip): MUL_MAT -> ADD(bias) [-> ADD(residual)] on the f32 epilogues
    const float * resid;              // Q2A_EPI_RESID: residual rows [M][ldo] (null = outF itself, in place)
    int store_bias;                   // Q2A_EPI_STORE_F: 1 = outF = acc + bias[n], 0 = raw accumulators
    float out_scale;                  // Q2A_EPI_STORE_F: != 0 -> outF = (acc [+ bias]) * out_scale (ggml_scale after the add)
    int split_store;                  // Q2A_EPI_STORE_F: 1 = allow the small-tile split-K (part/split_stride) like RESID
    // Q2A_EPI_STORE_F, small tiles, fp16 or Q4_K weights: ngroup = 2 runs a second GEMM with the same A (and, for
    // Q4_K, the same Q8_K activation scales), M, N, K in the same launch (its own W / bias / output / scale and
    // weight block scales), e.g. the K and Q projections of one layer; no split-K then
    int ngroup;
    const q2a_half * W2;
    const float * bias2;
    float * outF2;
    float out_scale2;
    int store_bias2;
    const float * dx2;                // Q4_K second weight: dx / dmin / beta / gamma / wext like the first
    const float * dmin2;
    const float * beta2;
    const float * gamma2;
    const q2a_half * wext2;
    int split_kq;                     // allow the small-tile split-K for k-quant / Q8_0 / Q4_0 weights (q2a_gemm_kq_ksplit)
    // Q2A_BLK_EXACT kernels: when gate is set, the launch computes only if (*gate != 0) == (gate_on != 0) — a
    // device-side choice between two launches of one node (every workgroup reads the flag and leaves otherwise)
    const int * gate;
    int gate_on;
    q2a_half * vtl;                   // Q2A_EPI_QKV: V^T lo image fp16(v - fp16(v)), same layout as vt (null = not written)
    int v_rows;                       // Q2A_EPI_QKV: 1 = V hi / lo row-major [M][D] into vt / vtl (like Q and K; the engine's
                                      //   reference contract), 0 = V^T [clip][head][64][TP] (bf16 contract, ggml backend)
    int m_base;                       // first output row of the launch (tiles cover rows [m_base, M)); set by the launcher
};

// the launcher's split factor for a small-tile Q2A_EPI_RESID GEMM (0 = none): a function of K only, so every batch
// size on the small-tile path sums in the same order (batch and single-clip results stay bit-identical)
int q2a_gemm_resid_ksplit(int M, int N, int K, int blk);
// the same for the block-quantized weights (whole scale groups per split), used when a.split_kq is set
int q2a_gemm_kq_ksplit(int M, int N, int K, int blk);
// blk: 0 (plain fp16 GEMM), 256 (Q4_K x Q8_K), 32 (Q8_0/Q4_0 x Q8_0), Q2A_BLK_BF16 (bf16 x bf16 MFMA, no block
// scales: the bf16-activation mode, whose fp16-typed operand and output pointers then hold bf16 bits)
constexpr int Q2A_BLK_BF16 = 1;
// Q2A_BLK_EXACT: fp16 x fp16 (like blk 0) with each 64-deep K-step's MFMA sum (two chained 16x16x32) added into f64
// accumulators, rounded to f32 once before the epilogue — the conv GEMMs (q2a_engine conv1 / conv2, the ggml
// backend's conv MUL_MAT): summed this way the conv output is within rounding of the exact dot product instead of
// carrying a 120-deep f32 accumulation chain ("the conv's own summation")
constexpr int Q2A_BLK_EXACT = 2;
hipError_t q2a_launch_gemm(const q2a_gemm_args & a, int epi, int blk, hipStream_t s);
// true when the launcher will use the 256-column tile configuration for this shape (Q2A_EPI_GELU_Q8K needs it)
bool q2a_gemm_wide_tiles(int M, int N, int blk);
// compute units of the current device (cached per device ordinal; 0 when it cannot be queried)
int q2a_cu_count();
// true when the launcher will use the 8-phase 256x256 kernel for these arguments (its Q4_K flavour fuses
// Q2A_EPI_GELU_Q8K efficiently)
bool q2a_gemm_pipe8(const q2a_gemm_args & a, int blk);

struct q2a_attn_args {
    const q2a_half *qh, *ql, *kh, *kl, *vt;
    int n_clips, T, D, H, TP;
    q2a_half * outH;     // [clips*T][D] fp16 (F16 path) or
    float * outF;        // [clips*T][D] f32  (quantized paths)
    int bf16;            // bf16-activation mode: qh/kh/vt and outH hold bf16, ql/kl unused, one MFMA per QK^T step
    const q2a_half * vtl;   // V^T lo image (v - fp16(v)) when q2a_attention_wants_vlo(), else unused
    int v_rows;             // reference contract: 1 = vt / vtl hold V hi / lo row-major [clips*T][D] (the K layout; the
                            //   kernel reads its P.V operand by transposing LDS reads), 0 = V^T [clip][head][64][TP]
};
// Reference contract (bf16 == 0): qh/ql hold Q * Q2A_LOG2E (after the 1/sqrt(dh) scale), split hi/lo — the kernel
// works in log2 units (P = exp2(S' - m')); every producer (QKV epilogue qscale, ggml backend prep, test entry) folds it.
// bf16 contract: qh holds Q scaled by 1/sqrt(dh) only.
constexpr float Q2A_LOG2E = 1.4426950408889634f;
hipError_t q2a_launch_attention(const q2a_attn_args & a, hipStream_t s);
// true when this build's reference-contract attention reads a V^T lo image (the QKV epilogue must then write it)
bool q2a_attention_wants_vlo();

// ---- exact-order kernels (q2a_exact.hip, compiled with -ffp-contract=off)
struct q2a_mel_args {
    const float * pcm;          // [clips][pcm_stride]
    int64_t pcm_stride;
    const int32_t * n_samples;  // [clips] (device)
    const int32_t * seek;       // [clips] first frame of the window (device)
    int n_clips;
    int n_mel, n_bins;          // 128, 201
    int n_frames_win;           // 2*n_ctx = 3000
    int max_frames;             // max n_len over the batch (grid extent)
    const float * filters;      // [n_mel][n_bins]
    const float * tab;          // hann[400] | cos[400] | sin[400]
    const int2 * frange;        // [n_mel] non-zero 4-aligned bin-group range per filter (q2a_launch_filter_ranges), or NULL
    float * mel;                // [clips][n_mel][n_frames_win] raw log10 values
    int32_t * clip_max;         // [clips] ordered-int encoding of the max over ALL frames
    q2a_half * xc1;             // [clips][n_frames_win+2][3*n_mel] conv1 operand, rows 0/last = 0: F16 conv kernel
                                //   hi|mid|lo (the f32 mel value exactly), F32 kernel hi|lo|hi
    int xc_f32;                 // 1: all-F32 model files (F32 conv kernel, hi|lo|hi against wh|wh|wl)
};
hipError_t q2a_launch_mel(const q2a_mel_args & a, hipStream_t s);
hipError_t q2a_launch_filter_ranges(const float * filters, int n_mel, int n_bins, int2 * out, hipStream_t s);

// LayerNorm over rows of X [M][D] (ggml_norm + mul + add, eps 1e-5), output by mode:
//   0: fp16 [M][D]                     (F16 weights)
//   1: Q8_K as fp16 codes + dy[M][D/256] + aext (Q4_K weights)
//   2: Q8_0 as fp16 codes + dy[M][D/32]  (Q8_0 / Q4_0 weights)
//   3: fp16 split [hi | lo | hi] rows of 3D (F32 weights: exact-f32-class products against [Wh | Wh | Wl])
//   4: bf16 RNE [M][D]                 (bf16-activation mode)
struct q2a_ln_args {
    const float * X;
    int M, D;
    const float * g;
    const float * b;
    int mode;
    q2a_half * outH;
    float * dy;          // block-major [D/blk][dy_ld]
    q2a_half * aext;     // block-major [D/256][dy_ld][16]
    int dy_ld;
};
hipError_t q2a_launch_layernorm(const q2a_ln_args & a, hipStream_t s);

// activation quantizer for F32 rows (attention output / gelu output on the quantized paths): modes 1, 2
struct q2a_quant_args {
    const float * X;
    const q2a_half * XH;   // fp16 input instead of X when non-NULL
    int M, K;
    int mode;
    q2a_half * outH;
    float * dy;
    q2a_half * aext;
    int dy_ld;
};
hipError_t q2a_launch_quant_act(const q2a_quant_args & a, hipStream_t s);
// GELU (ggml's fp16 table gelu_tab, 64 Ki entries, staged in LDS) of an fp16 pre-activation written by Q2A_EPI_PRE_H,
// then Q8_K quantization — the same codes as Q2A_EPI_GELU_H + q2a_launch_quant_act(mode 1, XH). XH [M][K], K % 256 == 0.
hipError_t q2a_launch_gelu_quant_q8k(const q2a_half * XH, int M, int K, const uint16_t * gelu_tab, q2a_half * outH,
                                     float * dy, q2a_half * aext, int dy_ld, hipStream_t s);

// One ggml weight matrix [N][K] (raw ggml rows, host memory; F16 / Q4_K / Q8_0 / Q4_0) packed into the GEMM's
// operand layout: fp16 W' [N][K] plus the block-major scale arrays, at byte offsets off[0..5] = W, DX, DMIN, WEXT,
// BETA, GAMMA of `out` (0 = absent). Used by the ggml-backend plugin for weights living in its buffers.
#ifdef __cplusplus
#include <vector>
int q2a_pack_linear(const uint8_t * raw, int wtype, int N, int K, std::vector<uint8_t> & out, uint64_t off[6]);
// the section offsets of q2a_pack_linear's layout (W [N][K] fp16 | dx | dmin | wext | beta | gamma, the per-block
// sections block-major [K/blk][N](x16 for wext)) and its total bytes (0 = unsupported type or shape)
uint64_t q2a_pack_layout(int wtype, int N, int K, uint64_t off[6]);
#endif

// AvgPool1d(2,2) over time + final LayerNorm -> out [clips][T/2][D] f32
struct q2a_pool_args {
    const float * X;     // [clips*T][D]
    int n_clips, T, D;
    const float * g;
    const float * b;
    float * out;
    const int32_t * clip_ok;   // [clips] 1 = write output, 0 = leave untouched (reference early return)
};
hipError_t q2a_launch_pool_ln(const q2a_pool_args & a, hipStream_t s);
