// q2a_whisper.cpp — the reference-named API (include/q2a_whisper.h) over the engine's C ABI.
//
// A whisper_context owns the weights (one q2a_engine loaded from the ggml file) and a default state; every
// whisper_state is a second engine sharing those weights (q2a_open_shared) with its own workspace and stream,
// the analogue of the reference's per-state ggml_backend_sched on shared model buffers (qwen2-whisper.cpp:
// 3095-3140). whisper_full follows whisper_encoder_output_with_state (qwen2-whisper.cpp:2341-2375): mel of the
// whole input, the 1 s length rule, one 30 s window at offset_ms, abort callback checked after the encode.
#include "q2a_encoder.h"
#include "q2a_whisper.h"

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

struct whisper_state {
    q2a_engine * eng = nullptr;
    std::vector<float> pcm;       // last input (whisper_encode re-encodes it at a new offset)
    std::vector<float> mel;       // [n_mel][n_len] of the last whisper_pcm_to_mel
    int n_len = 0;                // frames in `mel`
    int n_len_org = 0;            // mel.n_len_org: frames that carry audio (qwen2-whisper.cpp:2613)
    std::vector<float> embd;      // [n_out][n_state]
    bool has_embd = false;
    std::vector<float> chunks;    // whisper_full_parallel: [n_chunks][n_out][n_state]
    std::vector<int32_t> chunk_status;
    double t_mel_us = 0, t_encode_us = 0;
    int n_mel_calls = 0, n_encode = 0;
    int n_out = 0, n_state = 0;
};

struct whisper_context {
    q2a_engine * eng = nullptr;   // owns the device weights (on params.gpu_device)
    q2a_group * group = nullptr;  // whisper_full_parallel on > 1 device (opened on first use, over eng's weights)
    bool group_failed = false;    // a group could not be opened: the single-device path from then on
    q2a_info info{};
    int n_vocab = 0, ftype = 0;
    whisper_state * state = nullptr;
    double t_load_us = 0;
    int64_t t_start_us = 0;
};

namespace {

ggml_log_callback g_log = nullptr;
void * g_log_ud = nullptr;

void wlog(ggml_log_level level, const char * fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (g_log) g_log(level, buf, g_log_ud);
    else fputs(buf, stderr);
}

int64_t now_us() {
    return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// hparams from the ggml file header (magic, then 11 int32: n_vocab, n_audio_ctx, ..., n_mels, ftype)
bool read_header(const char * path, int32_t (&hp)[11]) {
    FILE * f = fopen(path, "rb");
    if (!f) return false;
    uint32_t magic = 0;
    const bool ok = fread(&magic, 4, 1, f) == 1 && fread(hp, 4, 11, f) == 11;
    fclose(f);
    return ok;
}

int n_len_org_of(int n_samples) { return 1 + (n_samples + 200 - 400) / 160; }   // stage_2_pad / frame_size / step

whisper_state * new_state(whisper_context * ctx) {
    q2a_engine * e = q2a_open_shared(ctx->eng);
    if (!e) { wlog(GGML_LOG_LEVEL_ERROR, "whisper_init_state: %s\n", q2a_last_error()); return nullptr; }
    whisper_state * st = new whisper_state();
    st->eng = e;
    st->n_out = ctx->info.n_out;
    st->n_state = ctx->info.n_audio_state;
    return st;
}

// one 30 s window of `pcm` at offset_ms through the engine; status per the reference's length rule
int encode_window(whisper_context * ctx, whisper_state * st, const float * pcm, int n, int offset_ms, bool force) {
    const int32_t ns = n;
    int32_t status = Q2A_CLIP_ENCODED;
    const int64_t t0 = now_us();
    q2a_set_force_encode(st->eng, force ? 1 : 0);
    st->embd.resize((size_t) ctx->info.n_out * ctx->info.n_audio_state);
    int32_t off = offset_ms;
    const int rc = q2a_encode_host_ex(st->eng, &pcm, &ns, &off, 1, 0, st->embd.data(), &status);
    q2a_set_force_encode(st->eng, 0);
    if (rc != Q2A_OK) { wlog(GGML_LOG_LEVEL_ERROR, "whisper_full: failed to encode: %s\n", q2a_last_error()); return -1; }
    if (status == Q2A_CLIP_ENCODED) {
        st->has_embd = true;
        st->t_encode_us += (double) (now_us() - t0);
        st->n_encode++;
    }
    return 0;
}

const char * k_langs[] = {
    "en", "zh", "de", "es", "ru", "ko", "fr", "ja", "pt", "tr", "pl", "ca", "nl", "ar", "sv", "it", "id", "hi", "fi", "vi",
    "he", "uk", "el", "ms", "cs", "ro", "da", "hu", "ta", "no", "th", "ur", "hr", "bg", "lt", "la", "mi", "ml", "cy", "sk",
    "te", "fa", "lv", "bn", "sr", "az", "sl", "kn", "et", "mk", "br", "eu", "is", "hy", "ne", "mn", "bs", "kk", "sq", "sw",
    "gl", "mr", "pa", "si", "km", "sn", "yo", "so", "af", "oc", "ka", "be", "tg", "sd", "gu", "am", "yi", "lo", "uz", "fo",
    "ht", "ps", "tk", "nn", "mt", "sa", "lb", "my", "bo", "tl", "mg", "as", "tt", "haw", "ln", "ha", "ba", "jw", "su", "yue",
};
constexpr int k_n_langs = (int) (sizeof(k_langs) / sizeof(k_langs[0]));

}  // namespace

extern "C" {

struct whisper_context_params whisper_context_default_params(void) {
    whisper_context_params p;
    memset(&p, 0, sizeof(p));
    p.use_gpu = true;
    p.flash_attn = false;
    p.gpu_device = 0;
    p.dtw_aheads_preset = WHISPER_AHEADS_NONE;
    p.dtw_n_top = -1;
    p.dtw_mem_size = (size_t) 128 << 20;
    return p;
}

struct whisper_context_params * whisper_context_default_params_by_ref(void) {
    whisper_context_params * p = new whisper_context_params(whisper_context_default_params());
    return p;
}

void whisper_free_context_params(struct whisper_context_params * params) { delete params; }

// The reference's version falls off the end without a return statement (qwen2-whisper.cpp:4231-4295, UB);
// this one returns the documented defaults.
struct whisper_full_params whisper_full_default_params(enum whisper_sampling_strategy strategy) {
    whisper_full_params p;
    memset(&p, 0, sizeof(p));
    p.strategy = strategy;
    p.n_threads = 4;
    p.n_max_text_ctx = 16384;
    p.print_progress = true;
    p.print_timestamps = true;
    p.thold_pt = 0.01f;
    p.thold_ptsum = 0.01f;
    p.language = "en";
    p.suppress_blank = true;
    p.temperature_inc = 0.2f;
    p.entropy_thold = 2.4f;
    p.logprob_thold = -1.0f;
    p.no_speech_thold = 0.6f;
    p.max_initial_ts = 1.0f;
    p.length_penalty = -1.0f;
    p.greedy.best_of = 5;
    p.beam_search.beam_size = 5;
    p.beam_search.patience = -1.0f;
    return p;
}

struct whisper_full_params * whisper_full_default_params_by_ref(enum whisper_sampling_strategy strategy) {
    return new whisper_full_params(whisper_full_default_params(strategy));
}

void whisper_free_params(struct whisper_full_params * params) { delete params; }

struct whisper_context * whisper_init_from_file_with_params_no_state(const char * path_model, struct whisper_context_params params) {
    const int64_t t0 = now_us();
    if (!params.use_gpu) {
        wlog(GGML_LOG_LEVEL_ERROR, "whisper_init: use_gpu = false is not supported: this path runs on the GPU only\n");
        return nullptr;
    }
    int32_t hp[11];
    if (!path_model || !read_header(path_model, hp)) {
        wlog(GGML_LOG_LEVEL_ERROR, "whisper_init: failed to open '%s'\n", path_model ? path_model : "(null)");
        return nullptr;
    }
    wlog(GGML_LOG_LEVEL_INFO, "whisper_init_from_file_with_params_no_state: loading model from '%s'\n", path_model);
    // the reference API has no activation-precision knob: Q2A_ACT=bf16 selects the bf16-activation contract
    // (BASELINE configs[4]) for an unchanged caller such as examples/main
    const char * act_env = getenv("Q2A_ACT");
    const int act = act_env && !strcmp(act_env, "bf16") ? Q2A_ACT_BF16 : Q2A_ACT_REFERENCE;
    q2a_engine * e = q2a_open_ex(path_model, params.gpu_device, act);
    if (!e) { wlog(GGML_LOG_LEVEL_ERROR, "whisper_init: %s\n", q2a_last_error()); return nullptr; }
    whisper_context * ctx = new whisper_context();
    ctx->eng = e;
    q2a_get_info(e, &ctx->info);
    ctx->n_vocab = hp[0];
    ctx->ftype = hp[10];
    ctx->t_start_us = t0;
    ctx->t_load_us = (double) (now_us() - t0);
    return ctx;
}

struct whisper_context * whisper_init_from_file_with_params(const char * path_model, struct whisper_context_params params) {
    whisper_context * ctx = whisper_init_from_file_with_params_no_state(path_model, params);
    if (!ctx) return nullptr;
    ctx->state = new_state(ctx);
    if (!ctx->state) { whisper_free(ctx); return nullptr; }
    return ctx;
}

struct whisper_context * whisper_init_from_file(const char * path_model) {
    return whisper_init_from_file_with_params(path_model, whisper_context_default_params());
}

struct whisper_state * whisper_init_state(struct whisper_context * ctx) { return ctx ? new_state(ctx) : nullptr; }

void whisper_free_state(struct whisper_state * state) {
    if (!state) return;
    q2a_close(state->eng);
    delete state;
}

void whisper_free(struct whisper_context * ctx) {
    if (!ctx) return;
    whisper_free_state(ctx->state);   // states first: they share the context's weights
    q2a_group_close(ctx->group);
    q2a_close(ctx->eng);
    delete ctx;
}

int whisper_pcm_to_mel_with_state(struct whisper_context * ctx, struct whisper_state * state, const float * samples,
                                  int n_samples, int n_threads) {
    (void) n_threads;
    if (!ctx || !state || !samples || n_samples <= 200) return -1;
    const int64_t t0 = now_us();
    const int n_len = (int) (((int64_t) n_samples + 480000) / 160);
    state->mel.resize((size_t) ctx->info.n_mels * n_len);
    int got = 0;
    if (q2a_pcm_to_mel(state->eng, samples, n_samples, state->mel.data(), (int64_t) state->mel.size(), &got) != Q2A_OK) {
        wlog(GGML_LOG_LEVEL_ERROR, "whisper_pcm_to_mel: %s\n", q2a_last_error());
        return -1;
    }
    state->n_len = got;
    state->n_len_org = n_len_org_of(n_samples);
    state->pcm.assign(samples, samples + n_samples);
    state->t_mel_us += (double) (now_us() - t0);
    state->n_mel_calls++;
    return 0;
}

int whisper_pcm_to_mel(struct whisper_context * ctx, const float * samples, int n_samples, int n_threads) {
    return ctx ? whisper_pcm_to_mel_with_state(ctx, ctx->state, samples, n_samples, n_threads) : -1;
}

int whisper_encode_with_state(struct whisper_context * ctx, struct whisper_state * state, int offset, int n_threads) {
    (void) n_threads;
    if (!ctx || !state || state->pcm.empty() || offset < 0) return -1;
    return encode_window(ctx, state, state->pcm.data(), (int) state->pcm.size(), offset * 10, true);
}

int whisper_encode(struct whisper_context * ctx, int offset, int n_threads) {
    return ctx ? whisper_encode_with_state(ctx, ctx->state, offset, n_threads) : -1;
}

int whisper_full_with_state(struct whisper_context * ctx, struct whisper_state * state, struct whisper_full_params params,
                            const float * samples, int n_samples) {
    if (!ctx || !state) return -1;
    if (n_samples > 0) {
        if (!samples) {
            wlog(GGML_LOG_LEVEL_ERROR, "whisper_full: failed to compute log mel spectrogram\n");
            return -2;
        }
        state->pcm.assign(samples, samples + n_samples);
        state->n_len_org = n_len_org_of(n_samples);
    }
    if (state->pcm.empty()) return -2;
    // the 1 s rule (qwen2-whisper.cpp:2356-2364): duration_ms, when set, replaces the audio length
    const int seek_start = params.offset_ms / 10;
    const int seek_end = params.duration_ms == 0 ? state->n_len_org : seek_start + params.duration_ms / 10;
    if (seek_end < seek_start + 100) {
        wlog(GGML_LOG_LEVEL_WARN, "whisper_full: input is too short - %d ms < 1000 ms\n", (seek_end - seek_start) * 10);
        return 0;
    }
    if (state->pcm.size() <= 200) return 0;   // (not reachable with duration_ms unset: under 1 s)
    const int rc = encode_window(ctx, state, state->pcm.data(), (int) state->pcm.size(), params.offset_ms, params.duration_ms != 0);
    if (rc) return rc;
    if (params.abort_callback && params.abort_callback(params.abort_callback_user_data)) {
        wlog(GGML_LOG_LEVEL_ERROR, "whisper_full: failed to encode\n");
        return -1;
    }
    return 0;
}

int whisper_full(struct whisper_context * ctx, struct whisper_full_params params, const float * samples, int n_samples) {
    return ctx ? whisper_full_with_state(ctx, ctx->state, params, samples, n_samples) : -1;
}

int whisper_full_parallel(struct whisper_context * ctx, struct whisper_full_params params, const float * samples,
                          int n_samples, int n_processors) {
    if (!ctx || !samples || n_samples <= 0) return -1;
    if (n_processors <= 1) return whisper_full(ctx, params, samples, n_samples);
    whisper_state * st = ctx->state;
    const int off = (int) ((int64_t) params.offset_ms * WHISPER_SAMPLE_RATE / 1000);
    if (off >= n_samples) return 0;
    const int per = (n_samples - off) / n_processors;
    std::vector<const float *> ptr(n_processors);
    std::vector<int32_t> ns(n_processors);
    for (int i = 0; i < n_processors; ++i) {
        ptr[i] = samples + off + (int64_t) i * per;
        ns[i] = i == n_processors - 1 ? n_samples - off - i * per : per;
    }
    const size_t per_out = (size_t) ctx->info.n_out * ctx->info.n_audio_state;
    st->chunks.assign(per_out * n_processors, 0.0f);
    st->chunk_status.assign(n_processors, Q2A_CLIP_SKIPPED);
    // more than one device: the chunks are spread over the context's device (params.gpu_device, first) and the other
    // visible devices, up to Q2A_PARALLEL_DEVICES of them (q2a_group_open_with: ONE RCCL broadcast of the context's own
    // device-layout weights at first use, no second replica on the context's device, contiguous chunk ranges, a host
    // thread per device). One device, Q2A_PARALLEL_DEVICES=1, or a group that cannot be opened: one batch on the state.
    if (!ctx->group && !ctx->group_failed) {
        const char * lim = getenv("Q2A_PARALLEL_DEVICES");
        int ndev = q2a_device_count();
        if (lim && atoi(lim) > 0 && atoi(lim) < ndev) ndev = atoi(lim);
        if (ndev > 1) {
            std::vector<int> devs;
            devs.push_back(ctx->info.device);
            for (int d = 0; (int) devs.size() < ndev; ++d)
                if (d != ctx->info.device) devs.push_back(d);
            ctx->group = q2a_group_open_with(ctx->eng, devs.data(), (int) devs.size());
            if (ctx->group) {
                wlog(GGML_LOG_LEVEL_INFO, "whisper_full_parallel: %d devices\n", q2a_group_size(ctx->group));
            } else {
                wlog(GGML_LOG_LEVEL_WARN, "whisper_full_parallel: multi-device open failed (%s): running on device %d only\n",
                     q2a_last_error(), ctx->info.device);
                ctx->group_failed = true;
            }
        }
    }
    const int64_t t0 = now_us();
    const int erc = ctx->group ? q2a_group_encode_host(ctx->group, ptr.data(), ns.data(), nullptr, n_processors, 0,
                                                        st->chunks.data(), st->chunk_status.data())
                               : q2a_encode_host(st->eng, ptr.data(), ns.data(), n_processors, 0, st->chunks.data(),
                                                 st->chunk_status.data());
    if (erc != Q2A_OK) {
        wlog(GGML_LOG_LEVEL_ERROR, "whisper_full_parallel: failed to encode: %s\n", q2a_last_error());
        return -1;
    }
    st->t_encode_us += (double) (now_us() - t0);
    st->n_encode += n_processors;
    if (st->chunk_status[0] == Q2A_CLIP_ENCODED) {
        st->embd.assign(st->chunks.begin(), st->chunks.begin() + (ptrdiff_t) per_out);
        st->has_embd = true;
    }
    return 0;
}

int whisper_full_n_segments(struct whisper_context * ctx) { (void) ctx; return 0; }

int whisper_full_n_chunks(struct whisper_context * ctx) { return ctx && ctx->state ? (int) ctx->state->chunk_status.size() : 0; }

const float * whisper_get_embd_enc_chunk(struct whisper_context * ctx, int i) {
    if (!ctx || !ctx->state || i < 0 || i >= (int) ctx->state->chunk_status.size()) return nullptr;
    if (ctx->state->chunk_status[i] != Q2A_CLIP_ENCODED) return nullptr;
    return ctx->state->chunks.data() + (size_t) i * ctx->info.n_out * ctx->info.n_audio_state;
}

const float * whisper_get_embd_enc_from_state(struct whisper_state * state, int * n_out, int * n_state) {
    if (!state || !state->has_embd) return nullptr;
    if (n_out) *n_out = state->n_out;
    if (n_state) *n_state = state->n_state;
    return state->embd.data();
}

const float * whisper_get_embd_enc(struct whisper_context * ctx, int * n_out, int * n_state) {
    if (!ctx || !ctx->state || !ctx->state->has_embd) return nullptr;
    if (n_out) *n_out = ctx->info.n_out;
    if (n_state) *n_state = ctx->info.n_audio_state;
    return ctx->state->embd.data();
}

q2a_engine * q2a_whisper_context_engine(struct whisper_context * ctx) { return ctx ? ctx->eng : nullptr; }

int q2a_whisper_encode_long(struct whisper_context * ctx, const float * samples, int n_samples, int offset_ms, float * out,
                            int max_windows) {
    if (!ctx || !samples || n_samples <= 200 || offset_ms < 0 || max_windows < 0) return -1;
    const int n_len_org = n_len_org_of(n_samples);
    int nw = 0;
    for (int seek = offset_ms / 10; seek + 100 <= n_len_org; seek += 2 * ctx->info.n_audio_ctx) ++nw;
    const int nrun = nw < max_windows ? nw : max_windows;
    if (nrun == 0 || !out) return nw;
    std::vector<const float *> ptr(nrun, samples);
    std::vector<int32_t> ns(nrun, n_samples), offs(nrun);
    for (int k = 0; k < nrun; ++k) offs[k] = offset_ms + k * WHISPER_CHUNK_SIZE * 1000;
    std::vector<int32_t> status(nrun);
    if (q2a_encode_host_ex(ctx->state->eng, ptr.data(), ns.data(), offs.data(), nrun, 0, out, status.data()) != Q2A_OK) {
        wlog(GGML_LOG_LEVEL_ERROR, "q2a_whisper_encode_long: %s\n", q2a_last_error());
        return -1;
    }
    return nw;
}

int whisper_n_len_from_state(struct whisper_state * state) { return state ? state->n_len_org : 0; }
int whisper_n_len(struct whisper_context * ctx) { return ctx && ctx->state ? ctx->state->n_len_org : 0; }
int whisper_n_vocab(struct whisper_context * ctx) { return ctx ? ctx->n_vocab : 0; }
int whisper_n_audio_ctx(struct whisper_context * ctx) { return ctx ? ctx->info.n_audio_ctx : 0; }
int whisper_is_multilingual(struct whisper_context * ctx) { return ctx && ctx->n_vocab >= 51865 ? 1 : 0; }
int whisper_model_n_vocab(struct whisper_context * ctx) { return whisper_n_vocab(ctx); }
int whisper_model_n_audio_ctx(struct whisper_context * ctx) { return ctx ? ctx->info.n_audio_ctx : 0; }
int whisper_model_n_audio_state(struct whisper_context * ctx) { return ctx ? ctx->info.n_audio_state : 0; }
int whisper_model_n_audio_head(struct whisper_context * ctx) { return ctx ? ctx->info.n_audio_head : 0; }
int whisper_model_n_audio_layer(struct whisper_context * ctx) { return ctx ? ctx->info.n_audio_layer : 0; }
int whisper_model_n_mels(struct whisper_context * ctx) { return ctx ? ctx->info.n_mels : 0; }
int whisper_model_ftype(struct whisper_context * ctx) { return ctx ? ctx->ftype : 0; }

int whisper_lang_max_id(void) { return k_n_langs - 1; }

int whisper_lang_id(const char * lang) {
    if (!lang) return -1;
    for (int i = 0; i < k_n_langs; ++i)
        if (strcmp(lang, k_langs[i]) == 0) return i;
    return -1;
}

const char * whisper_lang_str(int id) { return id >= 0 && id < k_n_langs ? k_langs[id] : nullptr; }

// qwen2-whisper.cpp:4191-4203: the first 20 values of embd_enc
void whisper_print_emb_enc(struct whisper_context * ctx) {
    if (!ctx || !ctx->state || !ctx->state->has_embd) return;
    for (int i = 0; i < 20; ++i) printf(" %.3f", ctx->state->embd[i]);
    printf("\n");
}

void whisper_print_timings(struct whisper_context * ctx) {
    if (!ctx) return;
    const whisper_state * st = ctx->state;
    const double t_end = (double) now_us();
    wlog(GGML_LOG_LEVEL_INFO, "\n");
    wlog(GGML_LOG_LEVEL_INFO, "%s:     load time = %8.2f ms\n", __func__, ctx->t_load_us / 1000.0);
    if (st) {
        wlog(GGML_LOG_LEVEL_INFO, "%s:      mel time = %8.2f ms / %5d runs\n", __func__, st->t_mel_us / 1000.0, st->n_mel_calls);
        wlog(GGML_LOG_LEVEL_INFO, "%s:   encode time = %8.2f ms / %5d runs (%8.2f ms per run, mel + encoder on the GPU)\n",
             __func__, st->t_encode_us / 1000.0, st->n_encode, st->n_encode ? st->t_encode_us / 1000.0 / st->n_encode : 0.0);
    }
    wlog(GGML_LOG_LEVEL_INFO, "%s:    total time = %8.2f ms\n", __func__, (t_end - (double) ctx->t_start_us) / 1000.0);
}

void whisper_reset_timings(struct whisper_context * ctx) {
    if (!ctx || !ctx->state) return;
    ctx->state->t_mel_us = ctx->state->t_encode_us = 0;
    ctx->state->n_mel_calls = ctx->state->n_encode = 0;
    ctx->t_start_us = now_us();
}

const char * whisper_print_system_info(void) {
    return "HIP = 1 | GFX950 = 1 | MFMA = 1 | BACKEND = q2a (MI355X-native encoder path) | ";
}

void whisper_log_set(ggml_log_callback log_callback, void * user_data) {
    g_log = log_callback;
    g_log_ud = user_data;
}

}  // extern "C"
