/*
 * q2a_whisper.h — reference-named C API of the encoder path, layered on q2a_encoder.h (same libq2a.so).
 *
 * Source-compatible with the subset of include/qwen2-whisper.h that the reference's own driver uses on this path
 * (examples/main/main.cpp compiles unchanged against this header):
 *   whisper_init_from_file_with_params   qwen2-whisper.h:141   (-> q2a_open on params.gpu_device)
 *   whisper_full / whisper_full_with_state  :446 / :452       (mel -> window at offset_ms -> encode; embd_enc kept)
 *   whisper_full_parallel                :464   (declared but never defined by the reference; here: n_processors
 *                                                 contiguous chunks of the input, encoded as one batch — spread over
 *                                                 gpu_device and the other visible devices, at most
 *                                                 Q2A_PARALLEL_DEVICES of them, on one replica per device)
 *   whisper_pcm_to_mel / whisper_n_len   :211 / :288
 *   whisper_encode                        :245   (encode the stored mel at `offset` frames)
 *   whisper_print_emb_enc                 :527   (first 20 values of embd_enc, " %.3f" each)
 *   whisper_free / whisper_init_state / whisper_free_state, default-params, model-dimension getters, timings.
 * Return conventions follow the reference: 0 success, -2 mel failure, -1 encode failure (qwen2-whisper.cpp:
 * 2353, 2370); 0 without encoding for under 1 s of audio (:2362-2364); NULL from init on failure.
 * Additions (no reference counterpart, which exposes no output accessor): whisper_get_embd_enc*, the WAV reader.
 */
#ifndef Q2A_WHISPER_H
#define Q2A_WHISPER_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WHISPER_SAMPLE_RATE 16000
#define WHISPER_N_FFT 400
#define WHISPER_HOP_LENGTH 160
#define WHISPER_CHUNK_SIZE 30

/* the ggml types the reference header pulls in through ggml.h (only what the API below needs) */
#ifndef Q2A_NO_GGML_TYPES
enum ggml_log_level { GGML_LOG_LEVEL_NONE = 0, GGML_LOG_LEVEL_INFO = 1, GGML_LOG_LEVEL_WARN = 2,
                      GGML_LOG_LEVEL_ERROR = 3, GGML_LOG_LEVEL_DEBUG = 4, GGML_LOG_LEVEL_CONT = 5 };
typedef void (*ggml_log_callback)(enum ggml_log_level level, const char * text, void * user_data);
typedef bool (*ggml_abort_callback)(void * data);
#endif

struct whisper_context;
struct whisper_state;
typedef int32_t whisper_token;

/* alignment-head presets: accepted for source compatibility (token-level DTW is a decoder feature) */
enum whisper_alignment_heads_preset {
    WHISPER_AHEADS_NONE, WHISPER_AHEADS_N_TOP_MOST, WHISPER_AHEADS_CUSTOM, WHISPER_AHEADS_TINY_EN,
    WHISPER_AHEADS_TINY, WHISPER_AHEADS_BASE_EN, WHISPER_AHEADS_BASE, WHISPER_AHEADS_SMALL_EN, WHISPER_AHEADS_SMALL,
    WHISPER_AHEADS_MEDIUM_EN, WHISPER_AHEADS_MEDIUM, WHISPER_AHEADS_LARGE_V1, WHISPER_AHEADS_LARGE_V2,
    WHISPER_AHEADS_LARGE_V3, WHISPER_AHEADS_LARGE_V3_TURBO
};

struct whisper_context_params {
    bool use_gpu;             /* must be true: the path has no CPU fallback (init fails without a HIP device) */
    bool flash_attn;          /* ignored: attention is always the fused kernel */
    int gpu_device;           /* HIP device index */
    bool dtw_token_timestamps;
    enum whisper_alignment_heads_preset dtw_aheads_preset;
    int dtw_n_top;
    size_t dtw_mem_size;
};

typedef void (*whisper_new_segment_callback)(struct whisper_context * ctx, struct whisper_state * state, int n_new,
                                             void * user_data);
typedef void (*whisper_progress_callback)(struct whisper_context * ctx, struct whisper_state * state, int progress,
                                          void * user_data);
typedef bool (*whisper_encoder_begin_callback)(struct whisper_context * ctx, struct whisper_state * state,
                                               void * user_data);

enum whisper_sampling_strategy { WHISPER_SAMPLING_GREEDY, WHISPER_SAMPLING_BEAM_SEARCH };

/* The fields the encoder path reads are marked (*); the rest are accepted and ignored (decoder options). */
struct whisper_full_params {
    enum whisper_sampling_strategy strategy;
    int n_threads;                 /* host threads for the WAV/mel staging (the encoder itself runs on the GPU) */
    int n_max_text_ctx;
    int offset_ms;                 /* (*) start of the encoded 30 s window */
    int duration_ms;
    bool translate, no_context, no_timestamps, single_segment, print_special, print_progress, print_realtime,
        print_timestamps, token_timestamps;
    float thold_pt, thold_ptsum;
    int max_len;
    bool split_on_word;
    int max_tokens;
    bool debug_mode;
    int audio_ctx;
    bool tdrz_enable;
    const char * suppress_regex;
    const char * initial_prompt;
    const whisper_token * prompt_tokens;
    int prompt_n_tokens;
    const char * language;
    bool detect_language, suppress_blank, suppress_non_speech_tokens;
    float temperature, max_initial_ts, length_penalty, temperature_inc, entropy_thold, logprob_thold, no_speech_thold;
    struct { int best_of; } greedy;
    struct { int beam_size; float patience; } beam_search;
    whisper_new_segment_callback new_segment_callback;
    void * new_segment_callback_user_data;
    whisper_progress_callback progress_callback;          /* (*) called with 0 and 100 around the encode */
    void * progress_callback_user_data;
    whisper_encoder_begin_callback encoder_begin_callback; /* (*) returning false aborts before the encode (-1) */
    void * encoder_begin_callback_user_data;
    ggml_abort_callback abort_callback;                    /* (*) returning true aborts before the encode (-1) */
    void * abort_callback_user_data;
};

struct whisper_context_params whisper_context_default_params(void);
struct whisper_context_params * whisper_context_default_params_by_ref(void);
void whisper_free_context_params(struct whisper_context_params * params);
#ifdef __cplusplus
struct whisper_full_params whisper_full_default_params(enum whisper_sampling_strategy strategy = WHISPER_SAMPLING_GREEDY);
#else
struct whisper_full_params whisper_full_default_params(enum whisper_sampling_strategy strategy);
#endif
struct whisper_full_params * whisper_full_default_params_by_ref(enum whisper_sampling_strategy strategy);
void whisper_free_params(struct whisper_full_params * params);

struct whisper_context * whisper_init_from_file_with_params(const char * path_model, struct whisper_context_params params);
struct whisper_context * whisper_init_from_file(const char * path_model);
struct whisper_context * whisper_init_from_file_with_params_no_state(const char * path_model, struct whisper_context_params params);
struct whisper_state * whisper_init_state(struct whisper_context * ctx);
void whisper_free(struct whisper_context * ctx);
void whisper_free_state(struct whisper_state * state);

int whisper_pcm_to_mel(struct whisper_context * ctx, const float * samples, int n_samples, int n_threads);
int whisper_pcm_to_mel_with_state(struct whisper_context * ctx, struct whisper_state * state, const float * samples,
                                  int n_samples, int n_threads);
int whisper_encode(struct whisper_context * ctx, int offset, int n_threads);
int whisper_encode_with_state(struct whisper_context * ctx, struct whisper_state * state, int offset, int n_threads);

int whisper_full(struct whisper_context * ctx, struct whisper_full_params params, const float * samples, int n_samples);
int whisper_full_with_state(struct whisper_context * ctx, struct whisper_state * state, struct whisper_full_params params,
                            const float * samples, int n_samples);
int whisper_full_parallel(struct whisper_context * ctx, struct whisper_full_params params, const float * samples,
                          int n_samples, int n_processors);
int whisper_full_n_segments(struct whisper_context * ctx);   /* 0: the path ends at embd_enc */

int whisper_n_len(struct whisper_context * ctx);
int whisper_n_len_from_state(struct whisper_state * state);
int whisper_n_vocab(struct whisper_context * ctx);
int whisper_n_audio_ctx(struct whisper_context * ctx);
int whisper_is_multilingual(struct whisper_context * ctx);
int whisper_model_n_vocab(struct whisper_context * ctx);
int whisper_model_n_audio_ctx(struct whisper_context * ctx);
int whisper_model_n_audio_state(struct whisper_context * ctx);
int whisper_model_n_audio_head(struct whisper_context * ctx);
int whisper_model_n_audio_layer(struct whisper_context * ctx);
int whisper_model_n_mels(struct whisper_context * ctx);
int whisper_model_ftype(struct whisper_context * ctx);

int whisper_lang_max_id(void);
int whisper_lang_id(const char * lang);
const char * whisper_lang_str(int id);

void whisper_print_emb_enc(struct whisper_context * ctx);
void whisper_print_timings(struct whisper_context * ctx);
void whisper_reset_timings(struct whisper_context * ctx);
const char * whisper_print_system_info(void);
void whisper_log_set(ggml_log_callback log_callback, void * user_data);

/* ---- additions ---- */
/* embd_enc of the last whisper_full / whisper_encode call: [n_out = n_audio_ctx/2][n_audio_state] f32 host copy
 * (valid until the next call on the same state). NULL before the first encode. */
const float * whisper_get_embd_enc(struct whisper_context * ctx, int * n_out, int * n_state);
const float * whisper_get_embd_enc_from_state(struct whisper_state * state, int * n_out, int * n_state);
/* whisper_full_parallel results: chunk i's embd_enc (NULL if that chunk was under 1 s and skipped) */
int whisper_full_n_chunks(struct whisper_context * ctx);
const float * whisper_get_embd_enc_chunk(struct whisper_context * ctx, int i_chunk);

/* The engine that holds the context's weights (q2a_encoder.h), for callers that batch clips through the engine API
 * or open a q2a_group_open_with over it without loading the model again. Owned by the context. */
struct q2a_engine * q2a_whisper_context_engine(struct whisper_context * ctx);

/* Encode every 30 s window of a long recording in one batch (windows k = 0.. at offset_ms + k*30000 until the
 * audio ends; each window normalised over the whole recording, as whisper_full at that offset would). Writes
 * min(n_windows, max_windows) windows to out [window][n_out][n_state] and returns the number of windows, < 0 on
 * error. */
int q2a_whisper_encode_long(struct whisper_context * ctx, const float * samples, int n_samples, int offset_ms,
                            float * out, int max_windows);

/* WAV ingestion with examples/common.cpp read_wav semantics (examples/common.cpp:642-748): 16 kHz, 16-bit PCM,
 * mono or stereo; mono = s16/32768, stereo mixed as (l + r)/65536; "-" reads the file from stdin. On success
 * *pcm is malloc'ed (free with q2a_wav_free), *n_samples = frames, stereo channels optionally split into
 * *left / *right (may be NULL). Returns 0, or -1 (unreadable / not RIFF-WAVE) / -2 (unsupported format). */
int q2a_read_wav(const char * path, float ** pcm, int64_t * n_samples, float ** left, float ** right);
void q2a_wav_free(void * p);

#ifdef __cplusplus
}
#endif
#endif /* Q2A_WHISPER_H */
