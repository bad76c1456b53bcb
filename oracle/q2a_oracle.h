// q2a_oracle.h — TEST INFRASTRUCTURE ONLY: CPU restatement of the reference hot path (the checker).
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load libq2a_oracle.so.
// Pinned against golden vectors produced by the real reference (oracle/_ref/ref_harness, see
// tests/golden/make_golden.py). Every function cites the reference file:line it restates.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int n_layer, d, n_head, n_mels, n_ctx;   // n_ctx = 1500 positions (2*n_ctx mel frames)
    int wtype;                               // ggml type of the 6 linear matrices: 0 F32, 1 F16, 2 Q4_0, 8 Q8_0, 12 Q4_K
    int conv_type;                           // 0 F32 or 1 F16 (qwen2-whisper.cpp:1543)
    const void * conv1_w; const float * conv1_b;   // [D][M][3], [D]
    const void * conv2_w; const float * conv2_b;   // [D][D][3], [D]
    const float * pe;                              // [n_ctx][D]
    const float * ln_post_w; const float * ln_post_b;
    // per-layer arrays of n_layer pointers (raw ggml row data for the matrices, ne0 = in-features)
    const void * const * q_w; const float * const * q_b;
    const void * const * k_w;
    const void * const * v_w; const float * const * v_b;
    const void * const * o_w; const float * const * o_b;
    const float * const * ln1_w; const float * const * ln1_b;
    const void * const * fc1_w; const float * const * fc1_b;
    const void * const * fc2_w; const float * const * fc2_b;
    const float * const * ln2_w; const float * const * ln2_b;
} oracle_model;

// Optional layer-0 intermediates (each may be NULL); [T][D] row-major unless noted.
typedef struct {
    float * conv_out;   // residual stream input after conv2+gelu+pe add  [T][D]
    float * ln1;        // LN1 output (after affine)                     [T][D]
    float * q;          // (Wq x + bq) * 1/sqrt(dh)                      [T][D]
    float * k;          // Wk x                                          [T][D]
    float * v;          // Wv x + bv                                     [T][D]
    float * attn;       // merged heads before O-proj                    [T][D]
    float * x1;         // after O-proj + bias + residual                [T][D]
    float * gelu;       // gelu(fc1)                                     [T][4D]
    float * x2;         // layer-0 output                                [T][D]
} oracle_dump;

// log_mel_spectrogram (qwen2-whisper.cpp:2575-2665). out: [n_mel][n_len], returns n_len.
int oracle_log_mel(const float * pcm, int n_samples, const float * filters, int n_mel, int n_fft_bins,
                   int n_threads, float * out, int out_cap_frames);

// whisper_encode_qwen2_internal conv+encoder graphs (qwen2-whisper.cpp:1892-2203) on a prepared
// [n_mels][2*n_ctx] mel window. out: [n_ctx/2][D].
int oracle_encode(const oracle_model * m, const float * mel_window, float * out, oracle_dump * dump, int n_threads);

// GELU with the fp16 LUT semantics (ggml.c:2556-2570, table ggml.c:3797-3806)
float oracle_gelu(float x);

// One weight GEMM with ggml's activation conversion: Y[M][N] = X[M][K] . W[N][K]^T
void oracle_gemm(int wtype, const void * W, const float * X, int M, int N, int K, float * Y, int n_threads);

// activation quantizers as ggml's from_float on x86 (quantize_row_q8_K -> _ref ggml-quants.c:3785-3822;
// quantize_row_q8_0 AVX2 branch ggml-quants.c:943-1000)
void oracle_quantize_act_q8_K(const float * x, void * y, int64_t k);
void oracle_quantize_act_q8_0(const float * x, void * y, int64_t k);

uint16_t oracle_fp32_to_fp16(float f);
float oracle_fp16_to_fp32(uint16_t h);

#ifdef __cplusplus
}
#endif
