/*
 * q2a_encoder.h — C ABI of the MI355X-native Qwen2-Audio encoder hot path (libq2a.so, gfx950).
 *
 * This is the drop-in boundary for the reference's hot path: PCM -> log-mel -> Conv1d x2 + GELU -> 32 pre-LN
 * encoder blocks -> AvgPool1d(2) -> LayerNorm, i.e. what `whisper_full()` computes in the reference
 * (src/qwen2-whisper.cpp:2341-2383: whisper_encoder_output_with_state -> whisper_pcm_to_mel_with_state +
 * whisper_encode_qwen2_internal). Plain pointers and sizes only; no torch types.
 *
 * The reference-named API (whisper_init_from_file_with_params / whisper_full / whisper_pcm_to_mel /
 * whisper_print_emb_enc / whisper_free, include/qwen2-whisper.h:141,446,211,527,203) is layered on top of this
 * in include/q2a_whisper.h and exported from the same library.
 *
 * Threading: one q2a_engine per device per host thread (like one whisper_state, include/qwen2-whisper.h:44-45).
 * Errors: functions return 0 / a non-NULL handle on success; negative q2a_status codes otherwise, with a message
 * retrievable through q2a_last_error(). No call aborts the process.
 */
#ifndef Q2A_ENCODER_H
#define Q2A_ENCODER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct q2a_engine q2a_engine;

typedef enum {
    Q2A_OK = 0,
    Q2A_ERR_IO = -1,           /* model file missing / unreadable */
    Q2A_ERR_FORMAT = -2,       /* bad magic, bad tensor shapes, unsupported ftype */
    Q2A_ERR_HIP = -3,          /* HIP runtime error (no device, launch failure, ...) */
    Q2A_ERR_ARG = -4,          /* invalid argument (sizes, NULL pointers, batch too large) */
    Q2A_ERR_OOM = -5,          /* device allocation failed */
    Q2A_ERR_UNSUPPORTED = -6   /* model variant not implemented on this path */
} q2a_status;

/* per-clip result status written by the encode calls */
#define Q2A_CLIP_ENCODED 0
#define Q2A_CLIP_SKIPPED 1   /* < 1 s of audio after the offset: the reference returns 0 without encoding
                                (qwen2-whisper.cpp:2359-2365); the clip's output rows are left untouched */
#define Q2A_CLIP_FAILED 2    /* the call returned an error before this clip's output reached the caller (host API) */

typedef struct {
    int32_t n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer, n_mels;
    int32_t wtype;          /* ggml type of the linear weights: 1 F16, 12 Q4_K, 8 Q8_0, 2 Q4_0 */
    int32_t n_out;          /* output vectors per clip (n_audio_ctx / 2 = 750) */
    int32_t device;
    int64_t weight_bytes;   /* device bytes of the packed weight blob */
    int64_t workspace_bytes;
    int32_t act;            /* Q2A_ACT_REFERENCE or Q2A_ACT_BF16 (from the blob) */
    int32_t reserved;
} q2a_info;

const char * q2a_last_error(void);

/* Load a reference-format ggml model file (models/convert-pt-to-ggml.py layout) onto HIP device `device`. */
q2a_engine * q2a_open(const char * model_path, int device);

/* Activation contract of an engine (q2a_open_ex / q2a_pack_model_ex):
 *   Q2A_ACT_REFERENCE  the reference's own: activations converted per ggml's vec_dot_type before every weight
 *                      GEMM (fp16 / Q8_K / Q8_0, or the exact fp16 hi/lo split for F32 files), F32-class attention
 *   Q2A_ACT_BF16       mixed precision (BASELINE configs[4]): linear weights dequantized (ggml dequantize_row_*) to
 *                      bf16, inter-op activations (LN outputs, Q/K/V, attention probabilities and output, GELU
 *                      output) in bf16, bf16 MFMA with f32 accumulation; the residual stream, LN statistics,
 *                      softmax and the conv front end stay as in the reference contract. A different numerical
 *                      contract from the reference CPU path: its error is reported separately. */
#define Q2A_ACT_REFERENCE 0
#define Q2A_ACT_BF16 1
q2a_engine * q2a_open_ex(const char * model_path, int device, int act);
int64_t q2a_pack_model_ex(const char * model_path, int act, void ** host_blob);

/* Multi-GPU: pack the model into its device layout on the host (rank 0), move the bytes to every rank's device
 * (e.g. one RCCL broadcast over xGMI), then open an engine on the device copy. The blob is self-describing. */
int64_t q2a_pack_model(const char * model_path, void ** host_blob);   /* returns size in bytes, < 0 on error */
void q2a_free_host_blob(void * host_blob);
q2a_engine * q2a_open_device_blob(const void * device_blob, int64_t size, int device);  /* blob not owned */
/* The compact TRANSPORT form of the same blob (what rank 0 broadcasts): the small sections plus every
 * linear weight as the model file's own ggml rows (Q4_K: raw block_q4_K, 144 B per 256 weights, ggml-common.h:282-297)
 * instead of the device layout's expanded operands — 0.37 GB instead of 1.40 GB for the full-size Q4_K model.
 * q2a_open_device_blob accepts it too and expands it on the GPU into an engine-owned device layout that is byte for
 * byte what q2a_pack_model_ex writes on the host. */
int64_t q2a_pack_model_compact(const char * model_path, int act, void ** host_blob);
/* From a blob's first header_bytes (>= 32 KiB) on the host: the device-layout size (return) and the size of the
 * blob as given (*transport_bytes: the compact size for a compact blob). */
int64_t q2a_blob_device_size(const void * host_header, int64_t header_bytes, int64_t * transport_bytes);
/* Expand a compact blob already on device `device` into out_dev (out_bytes >= the device-layout size). */
int q2a_expand_blob(const void * device_blob, int64_t size, void * out_dev, int64_t out_bytes, int device, void * stream);

/* A second engine on the same device sharing `base`'s weights (its own workspace and stream): the analogue of a
 * second whisper_state on one whisper_context. `base` must outlive it. */
q2a_engine * q2a_open_shared(const q2a_engine * base);
/* Encode windows with under 1 s of audio after the offset too (default off: they are skipped, Q2A_CLIP_SKIPPED,
 * like the reference). whisper_full uses it when duration_ms overrides the length check (qwen2-whisper.cpp:2357). */
int q2a_set_force_encode(q2a_engine * e, int on);

void q2a_close(q2a_engine * e);
int q2a_get_info(const q2a_engine * e, q2a_info * info);

/* Reserve device workspace for up to max_clips clips of up to max_samples samples (optional; grown on demand). */
int q2a_reserve(q2a_engine * e, int max_clips, int64_t max_samples);

/* Encode n_clips independent clips whose PCM (16 kHz mono f32) is already in device memory:
 *   pcm_dev    [n_clips][pcm_stride] floats, clip c has n_samples[c] valid samples (host array)
 *   offset_ms  whisper_full_params.offset_ms (window start = offset_ms / 10 mel frames)
 *   out_dev    [n_clips][n_out][n_audio_state] f32 (embd_enc of each clip)
 *   status     host array [n_clips] (Q2A_CLIP_*), may be NULL
 *   stream     hipStream_t to run on, or NULL: the legacy default stream 0 itself (the work starts after everything
 *              queued there before the call, and work queued there afterwards starts after it) — the same rule for
 *              every device-pointer entry point below and q2a_projector_apply. The call is asynchronous w.r.t. the
 *              host except for the small per-batch metadata upload: synchronise (the given stream, or stream 0)
 *              before reading out_dev on the host.
 * Audio longer than 30 s is truncated to one 30 s window, as in the reference (qwen2-whisper.cpp:2366-2372). */
int q2a_encode_device(q2a_engine * e, const float * pcm_dev, int64_t pcm_stride, const int32_t * n_samples,
                      int n_clips, int offset_ms, float * out_dev, int32_t * status, void * stream);

/* Same with host buffers in and out (PCIe transfers included; synchronous). out_host [n_clips][n_out][D]. */
int q2a_encode_host(q2a_engine * e, const float * const * pcm, const int32_t * n_samples, int n_clips,
                    int offset_ms, float * out_host, int32_t * status);

/* Per-clip window offsets (milliseconds, host array [n_clips]) instead of one offset_ms: e.g. the consecutive 30 s
 * windows of a long recording passed as n_clips rows that all point at the same PCM (pcm_stride 0 on the device
 * variant). Each window's log-mel is normalised over the whole recording, exactly as whisper_full(offset_ms = k *
 * 30000) on that recording would (the reference itself only ever encodes the first window). */
int q2a_encode_device_ex(q2a_engine * e, const float * pcm_dev, int64_t pcm_stride, const int32_t * n_samples,
                         const int32_t * offsets_ms, int n_clips, float * out_dev, int32_t * status, void * stream);
int q2a_encode_host_ex(q2a_engine * e, const float * const * pcm, const int32_t * n_samples, const int32_t * offsets_ms,
                       int n_clips, int offset_ms, float * out_host, int32_t * status);

/* log-mel of one clip (whisper_pcm_to_mel semantics): writes [n_mels][n_len] into mel_out (capacity
 * mel_cap floats) and *n_len. Runs the same kernels as the encoder on the engine's device. */
int q2a_pcm_to_mel(q2a_engine * e, const float * pcm, int n_samples, float * mel_out, int64_t mel_cap, int * n_len);

/* ---- one process, several GPUs (ncclCommInitAll + a host thread per device) -----------------------
 * Replaces the single-device choice of whisper_backend_init_gpu (qwen2-whisper.cpp:1217-1279) for batches of
 * independent clips, and is what whisper_full_parallel (declared, never defined, include/qwen2-whisper.h:464-469)
 * runs on when more than one device is visible (include/q2a_whisper.h). */
typedef struct q2a_group q2a_group;
int q2a_device_count(void);   /* visible HIP devices (0 when none) */
/* Open one engine per device of devices[0..n_devices) (n_devices = 0: every visible device). The model is packed
 * once on the host into its compact transport form, uploaded to devices[0] and sent to the others by ONE
 * ncclBroadcast over xGMI (RCCL communicators from ncclCommInitAll); each device expands its copy into the device
 * layout. act: Q2A_ACT_REFERENCE / Q2A_ACT_BF16. NULL on error (q2a_last_error). */
q2a_group * q2a_group_open(const char * model_path, const int * devices, int n_devices, int act);
/* The same over an engine that is already open (its weights, activation contract and device): base's device must be
 * in devices[0..n_devices) (n_devices = 0: base's device first, then every other visible device). base's own
 * device-layout weights are the root of the ONE ncclBroadcast (no second pack of the model file, no second replica on
 * base's device: that device's group engine shares base's weights, q2a_open_shared); every other device keeps the
 * replica it received. base must outlive the group. NULL on error (q2a_last_error). */
q2a_group * q2a_group_open_with(q2a_engine * base, const int * devices, int n_devices);
void q2a_group_close(q2a_group * g);
int q2a_group_size(const q2a_group * g);
q2a_engine * q2a_group_engine(q2a_group * g, int i);   /* the engine of the group's i-th device (owned by the group) */
/* The contiguous clip range [*first, *first + *count) the group gives its i-th device out of n_clips: near-equal,
 * the first n_clips % n_devices ranges one clip longer. Pure host arithmetic. */
int q2a_group_split(int n_clips, int n_devices, int i, int * first, int * count);
/* q2a_encode_host_ex over the group: every device encodes its clip range on its own host thread (no collective on
 * the data path); outputs and statuses land at the clips' own positions. offsets_ms may be NULL (offset_ms for all).
 * On error the first failing device's code is returned; its clips and every clip whose output never reached
 * out_host report Q2A_CLIP_FAILED. */
int q2a_group_encode_host(q2a_group * g, const float * const * pcm, const int32_t * n_samples, const int32_t * offsets_ms,
                          int n_clips, int offset_ms, float * out_host, int32_t * status);
/* Start-up cost of q2a_group_open: host pack, H2D + broadcast, per-device expand (seconds), transport bytes
 * (q2a_group_open_with: pack 0, the broadcast, the engines' open; the device-layout bytes broadcast). */
int q2a_group_setup_times(const q2a_group * g, double * pack_s, double * broadcast_s, double * open_s, int64_t * blob_bytes);

/* ---- per-kernel timing (HIP events recorded on the launch stream around every kernel of a class) ---- */
enum {
    Q2A_PROF_MEL = 0, Q2A_PROF_CONV1, Q2A_PROF_CONV2, Q2A_PROF_LN, Q2A_PROF_GEMM_QKV, Q2A_PROF_ATTN,
    Q2A_PROF_QUANT, Q2A_PROF_GEMM_O, Q2A_PROF_GEMM_FC1, Q2A_PROF_GEMM_FC2, Q2A_PROF_POOL, Q2A_PROF_CLASSES
};
int q2a_profile_enable(q2a_engine * e, int on);
/* time only the classes whose bit (1 << Q2A_PROF_*) is set (0 = off): fewer event pairs in a timed loop */
int q2a_profile_enable_mask(q2a_engine * e, unsigned mask);
/* accumulated milliseconds and launch counts per class (waits for the recorded events); reset != 0 clears */
int q2a_profile_read(q2a_engine * e, double * ms, int64_t * counts, int n, int reset);

/* ---- kernel-level entry points (device pointers), used by the parity tests ------------------------------ */
/* Y[M][N] = X[M][K] . W[N][K]^T for one linear weight of the loaded model (layer `layer`, which = 0 qkv
 * (raw, no bias/scale), 1 out_proj, 2 fc1, 3 fc2), with ggml's activation conversion of X (fp16 / Q8_K / Q8_0). */
int q2a_test_linear(q2a_engine * e, int layer, int which, const float * x_dev, int M, float * y_dev, void * stream);
/* One encoder block in place on X [n_clips*T][D] (f32, device). */
int q2a_test_block(q2a_engine * e, int layer, float * x_dev, int n_clips, void * stream);
/* Same, also copying the four GEMM A operands of the block as the MFMA consumed them into taps[0..3] (device,
 * 2-byte elements, NULL entries skipped): LN1 -> QKV [M][D], attention -> O [M][D], LN2 -> fc1 [M][D], GELU -> fc2
 * [M][F] (fp16 values for F16 files; Q8_K / Q8_0 integer codes held in fp16 for quantized files). Per-layer
 * divergence trace against the reference's own intermediates (diag/layer_trace.py). */
int q2a_test_block_taps(q2a_engine * e, int layer, float * x_dev, int n_clips, void * const * taps, void * stream);
/* Front end only: PCM [n_clips][pcm_stride] (device) -> log-mel -> conv1 + GELU -> conv2 + GELU -> + positions, the
 * first block's input X [n_clips*T][D] f32 (device) — the reference's embd_conv + pe (qwen2-whisper.cpp:1892-2005). */
int q2a_test_frontend(q2a_engine * e, const float * pcm_dev, int64_t pcm_stride, const int32_t * n_samples, int n_clips,
                      float * x_dev, void * stream);
/* AvgPool1d(2) + final LayerNorm only: X [n_clips*T][D] f32 (device) -> out [n_clips][T/2][D] f32 (device)
 * (qwen2-whisper.cpp:2157-2181). */
int q2a_test_pool_ln(q2a_engine * e, const float * x_dev, int n_clips, float * out_dev, void * stream);
/* Q4_K files: how fc1's output reaches fc2 as Q8_K codes — 0 (default) fp16 pre-activation + GELU inside the
 * quantizer, 1 GELU in the fc1 epilogue + quantizer, 2 GELU + Q8_K fused into the fc1 epilogue. All three give
 * identical codes (tests/test_gpu_parity.py::test_deferred_gelu_equals_epilogue_gelu); a test hook, not a tuning knob. */
int q2a_test_fc1_path(q2a_engine * e, int path);
/* Attention only: q,k,v [n_clips*T][D] f32 (q already scaled), out [n_clips*T][D] f32. */
int q2a_test_attention(q2a_engine * e, const float * q_dev, const float * k_dev, const float * v_dev, int n_clips,
                       float * out_dev, void * stream);

/* ---- downstream consumer: the Qwen2-Audio multi-modal projector ------------------------
 * audio_features = Linear(d_model -> text hidden size, bias)(embd_enc) — transformers' Qwen2AudioMultiModalProjector
 * (modeling_qwen2_audio.py), the step after the reference's path ends at embd_enc (qwen2-whisper.cpp:2185; the
 * reference has no projector). Weights: a projector file in the ggml container (multi_modal_projector.linear.weight
 * [d_out][d_in] F16 / Q4_K / Q8_0 / Q4_0, .bias [d_out] F32; bin/q2a_tool gen-projector + quantize). Numerics: a ggml
 * MUL_MAT of that weight type (activations per vec_dot_type, exact products, fp32 accumulation) + bias in f32. */
typedef struct q2a_projector q2a_projector;
q2a_projector * q2a_projector_open(const char * path, int device);
void q2a_projector_close(q2a_projector * p);
int q2a_projector_get_dims(const q2a_projector * p, int * d_in, int * d_out, int * wtype);
/* y_dev [rows][d_out] f32 = x_dev [rows][d_in] f32 (device) projected; asynchronous on `stream` (NULL = own stream).
 * A projector handle owns ONE workspace (the quantized activation operand): calls on one handle must be ordered on one
 * stream (or the caller synchronises between streams); use one handle per stream for concurrent projections. */
int q2a_projector_apply(q2a_projector * p, const float * x_dev, int64_t rows, float * y_dev, void * stream);

#ifdef __cplusplus
}
#endif
#endif /* Q2A_ENCODER_H */
