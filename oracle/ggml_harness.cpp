// ggml_harness.cpp — TEST INFRASTRUCTURE ONLY: the reference's unmodified whisper_full() on the Q2A ggml backend.
//
// The reference selects its GPU backend in whisper_backend_init_gpu / whisper_default_buffer_type
// (src/qwen2-whisper.cpp:1217-1279, 1309-1337) under `#ifdef GGML_USE_<X>`. The integration patch a maintainer adds
// (INTEGRATION.md §"ggml backend") is one more such branch calling ggml_backend_q2a_init / _buffer_type. This
// harness reproduces that patch without touching the reference source: it compiles src/qwen2-whisper.cpp where it
// lies with the CUDA branch selected and its two entry points renamed to the Q2A backend's, so the reference's own
// model loader, graph builders (:1892-2203), ggml_backend_sched splitting and whisper_full drive our backend
// (lib/libggml-q2a.so). Unlike ref_harness.cpp there is NO conv shim: the graph's MUL_MAT(F32 im2col, F16 kernel)
// runs on the backend as built.
//
//   ggml_harness encode MODEL PCM OUT [reps] [device]   -> embd_enc f32 [750][1280] to OUT, JSON line on stdout

#define GGML_USE_CUDA
#define ggml_backend_cuda_init ggml_backend_q2a_init
#define ggml_backend_cuda_buffer_type ggml_backend_q2a_buffer_type
#include "qwen2-whisper.cpp"
#undef ggml_backend_cuda_init
#undef ggml_backend_cuda_buffer_type

#include "ggml-q2a.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

namespace {

std::vector<float> read_f32(const char * path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) { fprintf(stderr, "cannot open %s\n", path); exit(2); }
    const size_t n = (size_t) f.tellg();
    f.seekg(0);
    std::vector<float> v(n / sizeof(float));
    f.read((char *) v.data(), (std::streamsize) (v.size() * sizeof(float)));
    return v;
}

int cmd_encode(int argc, char ** argv) {
    if (argc < 5) { fprintf(stderr, "encode MODEL PCM OUT [reps] [device]\n"); return 1; }
    const int reps = argc > 5 ? atoi(argv[5]) : 1;
    whisper_context_params cp = whisper_context_default_params();
    cp.use_gpu = true;
    cp.gpu_device = argc > 6 ? atoi(argv[6]) : 0;
    whisper_context * ctx = whisper_init_from_file_with_params(argv[2], cp);
    if (!ctx) { fprintf(stderr, "model load failed: %s\n", argv[2]); return 3; }
    ggml_backend_t be = ctx->state->backends[0];
    if (!ggml_backend_is_q2a(be)) { fprintf(stderr, "backend 0 is %s, not Q2A\n", ggml_backend_name(be)); return 4; }
    std::vector<float> pcm = read_f32(argv[3]);
    // whisper_full_default_params() has no return statement in the reference (qwen2-whisper.cpp:4231-4295, UB):
    // zero-initialise and set what the path reads
    whisper_full_params p;
    memset(&p, 0, sizeof(p));
    p.n_threads = 4;
    double best = 1e30, total = 0, best_mel = 1e30, best_enc = 1e30;
    for (int r = 0; r < reps; ++r) {
        const int64_t mel0 = ctx->state->t_mel_us, enc0 = ctx->state->t_encode_us;
        auto t0 = std::chrono::steady_clock::now();
        const int rc = whisper_full(ctx, p, pcm.data(), (int) pcm.size());
        auto t1 = std::chrono::steady_clock::now();
        if (rc != 0) { fprintf(stderr, "whisper_full rc=%d\n", rc); return 5; }
        const double s = std::chrono::duration<double>(t1 - t0).count();
        total += s;
        best = std::min(best, s);
        // the reference's own phase clocks (qwen2-whisper.cpp:2335, 2651): CPU log-mel, then conv + encoder graphs
        best_mel = std::min(best_mel, 1e-6 * (double) (ctx->state->t_mel_us - mel0));
        best_enc = std::min(best_enc, 1e-6 * (double) (ctx->state->t_encode_us - enc0));
    }
    ggml_backend_q2a_stats st;
    memset(&st, 0, sizeof(st));
    ggml_backend_q2a_get_stats(be, &st);
    // how the sched split the encoder graph: every node should sit on the Q2A backend
    ggml_tensor * e = ctx->state->embd_enc;
    std::vector<float> out(ggml_nelements(e));
    ggml_backend_tensor_get(e, out.data(), 0, ggml_nbytes(e));
    FILE * f = fopen(argv[4], "wb");
    fwrite(out.data(), sizeof(float), out.size(), f);
    fclose(f);
    printf("{\"ne0\": %lld, \"ne1\": %lld, \"reps\": %d, \"best_s\": %.6f, \"mean_s\": %.6f, \"backend\": \"%s\", "
           "\"embd_buffer\": \"%s\", \"n_splits_encode\": %d, \"nodes\": %d, \"mul_mat_fast\": %d, \"mul_mat_f32\": %d, "
           "\"attn_fused\": %d, \"other\": %d, \"graph_replayed\": %d, \"fused\": %d, \"mm_grouped\": %d, \"mm_conv\": %d, \"best_mel_s\": %.6f, \"best_encode_s\": %.6f}\n",
           (long long) e->ne[0], (long long) e->ne[1], reps, best, total / reps, ggml_backend_name(be),
           ggml_backend_buffer_name(e->buffer), ggml_backend_sched_get_n_splits(ctx->state->sched_encode.sched),
           st.n_nodes, st.n_mul_mat_fast, st.n_mul_mat_f32, st.n_attn_fused, st.n_other, st.n_graph_replayed, st.n_fused, st.n_mm_grouped, st.n_mul_mat_conv, best_mel,
           best_enc);
    whisper_free(ctx);
    return 0;
}

}  // namespace

int main(int argc, char ** argv) {
    if (argc < 2) { fprintf(stderr, "usage: ggml_harness encode ...\n"); return 1; }
    whisper_log_set([](ggml_log_level lvl, const char * text, void *) { if (lvl == GGML_LOG_LEVEL_ERROR) fputs(text, stderr); }, nullptr);
    if (std::string(argv[1]) == "encode") return cmd_encode(argc, argv);
    fprintf(stderr, "unknown command %s\n", argv[1]);
    return 1;
}
