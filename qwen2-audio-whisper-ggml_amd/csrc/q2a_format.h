// q2a_format.h — host-side model-file format tooling for the Qwen2-Audio encoder path.
//
// The on-disk layout is the reference's unchanged ggml file (models/convert-pt-to-ggml.py:268-337, read by
// whisper_model_load src/qwen2-whisper.cpp:1350-1872):
//   u32 magic 0x67676d6c | i32 hparams[11] | i32 n_mel, n_fft, f32 filters[n_mel*n_fft] |
//   i32 n_vocab, {u32 len, bytes}* | tensors: {i32 n_dims, i32 name_len, i32 ttype, i32 ne[n_dims], name, data}*
// Quantized files carry ftype + GGML_QNT_VERSION(2)*1000 in hparams[10] (qwen2-whisper.cpp:1414-1416).
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// ggml_type ids (ggml/include/ggml.h:357-392) used on this path
enum q2a_ggml_type {
    Q2A_TYPE_F32 = 0,
    Q2A_TYPE_F16 = 1,
    Q2A_TYPE_Q4_0 = 2,
    Q2A_TYPE_Q8_0 = 8,
    Q2A_TYPE_Q4_K = 12,
    Q2A_TYPE_Q8_K = 15,
};

// ggml_ftype ids (ggml/include/ggml.h:411-423)
enum q2a_ggml_ftype {
    Q2A_FTYPE_ALL_F32 = 0,
    Q2A_FTYPE_MOSTLY_F16 = 1,
    Q2A_FTYPE_MOSTLY_Q4_0 = 2,
    Q2A_FTYPE_MOSTLY_Q8_0 = 7,
    Q2A_FTYPE_MOSTLY_Q4_K = 12,
};

#define Q2A_FILE_MAGIC 0x67676d6cu
#define Q2A_QNT_VERSION_FACTOR 1000
#define Q2A_QK_K 256
#define Q2A_QK8_0 32
#define Q2A_QK4_0 32

// block layouts (ggml/src/ggml-common.h:143-149, 186-191, 282-297, 329-335)
typedef struct { uint16_t d; uint8_t qs[16]; } q2a_block_q4_0;           // 18 B / 32 weights
typedef struct { uint16_t d; int8_t qs[32]; } q2a_block_q8_0;            // 34 B / 32 weights
typedef struct { uint16_t d, dmin; uint8_t scales[12]; uint8_t qs[128]; } q2a_block_q4_K;  // 144 B / 256
typedef struct { float d; int8_t qs[256]; int16_t bsums[16]; } q2a_block_q8_K;             // 292 B / 256

// whisper_hparams order as stored (qwen2-whisper.cpp:1374-1384)
typedef struct {
    int32_t n_vocab, n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer;
    int32_t n_text_ctx, n_text_state, n_text_head, n_text_layer, n_mels, ftype;
} q2a_hparams;

// ---- numerics helpers shared with the engine host code -------------------------------------------
uint16_t q2a_fp32_to_fp16(float f);   // IEEE binary16, round-to-nearest-even (== F16C _cvtss_sh(x, 0))
float    q2a_fp16_to_fp32(uint16_t h);
size_t   q2a_row_size(int ggml_type, int64_t ncols);   // bytes of one row (ggml_row_size)

// ---- deterministic synthetic inputs (SURVEY.md §8d "Synthetic inputs") ----------------------------
uint64_t q2a_splitmix64(uint64_t x);
double   q2a_gauss(uint64_t seed, uint32_t stream, uint64_t index);
// clip c: 0.3 sin(2π(220+37c)t) + 0.1 sin(2π(1000+53c)t) + 0.05 N(0,1), 16 kHz
void q2a_synth_clip(float * out, int64_t n_samples, int clip_index);
// Slaney-normalised mel filterbank [n_mel][n_fft/2+1] (librosa.filters.mel(sr, n_fft, n_mel) semantics)
void q2a_mel_filters_slaney(float * out, int n_mel, int n_fft, int sample_rate);

// Write a synthetic model in the reference layout. ftype 0 = all F32, 1 = F16 (the converter's rules,
// convert-pt-to-ggml.py:309-321). Returns 0 on success.
int q2a_write_synthetic_model(const char * path, const q2a_hparams * hp, uint64_t seed, int n_threads);

// Write a synthetic Qwen2-Audio multi-modal projector file (one Linear d_in -> d_out with bias) in the same ggml
// container (see q2a_format.cpp). ftype 0 = F32 weight, 1 = F16. Returns 0 on success.
int q2a_write_synthetic_projector(const char * path, int d_in, int d_out, int ftype, uint64_t seed);

// Re-quantize a F16/F32 model file the way whisper.cpp's quantize flow does (examples/common-ggml.cpp:41-244
// with to_quant {".*"} and skip {"embed_positions.weight","conv1.bias","conv2.bias"}; only 2-D tensors).
// qtype: Q2A_TYPE_Q4_K / Q2A_TYPE_Q8_0 / Q2A_TYPE_Q4_0. Byte-identical to ggml_quantize_chunk. 0 on success.
int q2a_quantize_model(const char * in_path, const char * out_path, int qtype, int n_threads);

// Row quantizers (ggml "_ref" weight quantizers, byte-exact): k must be a multiple of the block size.
void q2a_quantize_row_q4_K(const float * x, void * y, int64_t k);   // quantize_row_q4_K_ref ggml-quants.c:2483
void q2a_quantize_row_q8_0(const float * x, void * y, int64_t k);   // quantize_row_q8_0_ref ggml-quants.c:848
void q2a_quantize_row_q4_0(const float * x, void * y, int64_t k);   // quantize_row_q4_0_ref ggml-quants.c:761

// Reference numerics tables (built on the host, compiled without FMA contraction, like the reference):
//   GELU fp16 table (ggml.c:3797-3806): tab[h] = fp16(gelu_f32(fp32(h)))
//   mel tables (whisper_global_cache, qwen2-whisper.cpp:2404-2437): hann[400] | cos[400] | sin[400]
void q2a_make_gelu_table(uint16_t * tab65536);
void q2a_make_mel_tables(float * hann_cos_sin1200);

// ---- model-file reader -----------------------------------------------------------------------------
typedef struct {
    char name[96];
    int32_t type;
    int32_t n_dims;
    int64_t ne[4];
    size_t nbytes;
    size_t offset;      // into q2a_model_file.data
} q2a_tensor_desc;

typedef struct {
    q2a_hparams hp;
    int32_t qntvr;          // quantization version (hparams.ftype / 1000)
    int32_t wtype;          // ggml type of the big matrices (from ftype)
    int32_t n_mel_filt, n_fft_filt;
    float * filters;        // [n_mel_filt][n_fft_filt]
    int32_t n_tensors;
    q2a_tensor_desc * tensors;
    uint8_t * data;         // all tensor payloads back to back
    size_t data_size;
} q2a_model_file;

// Parse a model file. Returns NULL on error and writes a message into err (if non-NULL).
q2a_model_file * q2a_model_file_read(const char * path, char * err, size_t err_len);
void q2a_model_file_free(q2a_model_file * mf);
const q2a_tensor_desc * q2a_model_file_find(const q2a_model_file * mf, const char * name);

#ifdef __cplusplus
}
#endif
