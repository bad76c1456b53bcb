// ref_harness.cpp — TEST INFRASTRUCTURE ONLY (oracle leg). Never linked into the product.
//
// Drives the *unmodified* reference CPU path compiled from the sources where they lie under
// /root/reference (see oracle/Makefile), to generate golden vectors and to time the CPU baseline.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may execute the binary built
// from this file.
//
// Reference anchors:
//   whisper_full                      src/qwen2-whisper.cpp:2377-2383
//   whisper_encoder_output_with_state src/qwen2-whisper.cpp:2341-2375
//   log_mel_spectrogram               src/qwen2-whisper.cpp:2575-2665
//   ggml_common_quantize_0            examples/common-ggml.cpp:41-244
//
// One harness shim is applied (SURVEY.md §8c "Required shim"): the unmodified graph feeds an F16
// conv kernel into MUL_MAT(F32 im2col, F16 kernel), which neither the CPU nor the CUDA backend
// supports (ggml-backend.cpp:1155-1156 / ggml-cuda.cu:2981-2983), so F16 / quantized model files abort.
// The shim upcasts the conv kernel to F32 exactly (ggml_cast), which is the arithmetic of the shipped
// all-F32 configuration; no other reference code is touched.

#include "ggml.h"

static struct ggml_tensor * q2a_harness_conv_1d_ph(struct ggml_context * ctx, struct ggml_tensor * a,
                                                   struct ggml_tensor * b, int s, int d) {
    if (a->type != GGML_TYPE_F32) {
        a = ggml_cast(ctx, a, GGML_TYPE_F32);
    }
    return ggml_conv_1d(ctx, a, b, s, (int) (a->ne[0] / 2), d);
}

#define ggml_conv_1d_ph q2a_harness_conv_1d_ph
#include "qwen2-whisper.cpp"
#undef ggml_conv_1d_ph

#include "common-ggml.h"

#include <chrono>
#include <cstdint>
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

void write_blob(const std::string & path, const void * data, size_t nbytes) {
    FILE * f = fopen(path.c_str(), "wb");
    if (!f) { fprintf(stderr, "cannot write %s\n", path.c_str()); exit(2); }
    fwrite(data, 1, nbytes, f);
    fclose(f);
}

// whisper_full_default_params() has no return statement in the reference (qwen2-whisper.cpp:4231-4295,
// undefined behaviour), so the harness zero-initialises the params and sets what the path reads
// (n_threads, offset_ms, duration_ms, abort_callback — qwen2-whisper.cpp:2351-2369).
whisper_full_params harness_params(int n_threads) {
    whisper_full_params p;
    memset(&p, 0, sizeof(p));
    p.n_threads = n_threads;
    return p;
}

whisper_context * open_ctx(const char * model) {
    whisper_context_params cp = whisper_context_default_params();
    cp.use_gpu = false;
    whisper_context * ctx = whisper_init_from_file_with_params(model, cp);
    if (!ctx) { fprintf(stderr, "model load failed: %s\n", model); exit(3); }
    return ctx;
}

// Dump every node output of the encoder graph whose layer index is 0 (first n_dump nodes), through the
// sched eval callback (ggml-backend.cpp:2306), which the reference itself uses for debugging (:2305).
// ndump < 0 selects the per-layer mode: every layer's block input (node 3 + 33 l), its LN1 output (+3), the merged
// attention output (+21), the post-attention residual (+24), the LN2 output (+27), the GELU output (+30), and the
// encoder's last block output — the tensors ggml re-quantizes before the next weight GEMM, for the cross-build /
// per-layer divergence trace (tests/golden/make_crossbuild.py). 33 nodes per layer: the graph of
// whisper_build_graph_encoder (qwen2-whisper.cpp:1999-2154) as ggml orders it.
struct dump_state {
    std::string dir;
    int idx = 0;
    int limit = 0;
    bool layers = false;
    FILE * index = nullptr;
};

bool dump_wanted(const dump_state * ds, int idx) {
    if (!ds->layers) return idx < ds->limit;
    if (idx < 3) return false;
    const int r = (idx - 3) % 33;
    return r == 0 || r == 3 || r == 21 || r == 24 || r == 27 || r == 30;
}

bool dump_cb(struct ggml_tensor * t, bool ask, void * ud) {
    dump_state * ds = (dump_state *) ud;
    if (ask) {
        return ds->layers || ds->idx < ds->limit;
    }
    if (!dump_wanted(ds, ds->idx)) { ds->idx++; return true; }
    if (t->type == GGML_TYPE_F32 && ggml_is_contiguous(t)) {
        std::vector<float> buf(ggml_nelements(t));
        ggml_backend_tensor_get(t, buf.data(), 0, ggml_nbytes(t));
        char name[64];
        snprintf(name, sizeof(name), "node%03d_%s.f32", ds->idx, ggml_op_desc(t));
        write_blob(ds->dir + "/" + name, buf.data(), ggml_nbytes(t));
        fprintf(ds->index, "%d %s %lld %lld %lld %lld %s\n", ds->idx, ggml_op_desc(t), (long long) t->ne[0],
                (long long) t->ne[1], (long long) t->ne[2], (long long) t->ne[3], name);
    }
    ds->idx++;
    return true;
}

int cmd_mel(int argc, char ** argv) {
    if (argc < 5) { fprintf(stderr, "mel MODEL PCM OUT [threads]\n"); return 1; }
    whisper_context * ctx = open_ctx(argv[2]);
    std::vector<float> pcm = read_f32(argv[3]);
    const int nt = argc > 5 ? atoi(argv[5]) : 4;
    if (whisper_pcm_to_mel(ctx, pcm.data(), (int) pcm.size(), nt) != 0) return 4;
    const whisper_mel & mel = ctx->state->mel;
    FILE * f = fopen(argv[4], "wb");
    int32_t hdr[2] = { mel.n_mel, mel.n_len };
    fwrite(hdr, sizeof(hdr), 1, f);
    fwrite(mel.data.data(), sizeof(float), mel.data.size(), f);
    fclose(f);
    whisper_free(ctx);
    return 0;
}

int cmd_encode(int argc, char ** argv) {
    if (argc < 5) { fprintf(stderr, "encode MODEL PCM OUT [threads] [reps] [dumpdir] [ndump]\n"); return 1; }
    whisper_context * ctx = open_ctx(argv[2]);
    std::vector<float> pcm = read_f32(argv[3]);
    const int nt   = argc > 5 ? atoi(argv[5]) : 4;
    const int reps = argc > 6 ? atoi(argv[6]) : 1;
    dump_state ds;
    if (argc > 7) {
        ds.dir = argv[7];
        ds.limit = argc > 8 ? atoi(argv[8]) : 48;
        ds.layers = ds.limit < 0;
        ds.index = fopen((ds.dir + "/index.txt").c_str(), "w");
        ggml_backend_sched_set_eval_callback(ctx->state->sched_encode.sched, dump_cb, &ds);
    }
    whisper_full_params p = harness_params(nt);
    double best = 1e30, total = 0;
    for (int r = 0; r < reps; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        const int rc = whisper_full(ctx, p, pcm.data(), (int) pcm.size());
        auto t1 = std::chrono::steady_clock::now();
        if (rc != 0) { fprintf(stderr, "whisper_full rc=%d\n", rc); return 5; }
        const double s = std::chrono::duration<double>(t1 - t0).count();
        total += s;
        if (s < best) best = s;
        if (r == 0 && ds.index) {
            ggml_backend_sched_set_eval_callback(ctx->state->sched_encode.sched, nullptr, nullptr);
            fclose(ds.index);
            ds.index = nullptr;
            // the conv output of the same call
            ggml_tensor * ec = ctx->state->embd_conv;
            std::vector<float> buf(ggml_nelements(ec));
            ggml_backend_tensor_get(ec, buf.data(), 0, ggml_nbytes(ec));
            write_blob(ds.dir + "/embd_conv.f32", buf.data(), ggml_nbytes(ec));
        }
    }
    ggml_tensor * e = ctx->state->embd_enc;
    std::vector<float> out(ggml_nelements(e));
    ggml_backend_tensor_get(e, out.data(), 0, ggml_nbytes(e));
    write_blob(argv[4], out.data(), out.size() * sizeof(float));
    printf("{\"ne0\": %lld, \"ne1\": %lld, \"reps\": %d, \"best_s\": %.6f, \"mean_s\": %.6f, \"threads\": %d}\n",
           (long long) e->ne[0], (long long) e->ne[1], reps, best, total / reps, nt);
    whisper_free(ctx);
    return 0;
}

int cmd_quantize_model(int argc, char ** argv) {
    if (argc < 5) { fprintf(stderr, "quantize-model IN OUT ftype\n"); return 1; }
    // whisper.cpp's quantize flow over this file layout: copy the header with
    // ftype = ftype + GGML_QNT_VERSION*GGML_QNT_VERSION_FACTOR, copy filters + vocab, then quantize 2-D tensors.
    std::ifstream fin(argv[2], std::ios::binary);
    std::ofstream fout(argv[3], std::ios::binary);
    const int ftype = atoi(argv[4]);
    uint32_t magic; fin.read((char *) &magic, 4); fout.write((char *) &magic, 4);
    int32_t hp[11]; fin.read((char *) hp, sizeof(hp));
    hp[10] = ftype + GGML_QNT_VERSION * GGML_QNT_VERSION_FACTOR;
    fout.write((char *) hp, sizeof(hp));
    int32_t nmel, nfft; fin.read((char *) &nmel, 4); fin.read((char *) &nfft, 4);
    fout.write((char *) &nmel, 4); fout.write((char *) &nfft, 4);
    std::vector<float> filt((size_t) nmel * nfft);
    fin.read((char *) filt.data(), (std::streamsize) (filt.size() * 4));
    fout.write((char *) filt.data(), (std::streamsize) (filt.size() * 4));
    int32_t nvocab; fin.read((char *) &nvocab, 4); fout.write((char *) &nvocab, 4);
    for (int i = 0; i < nvocab; ++i) {
        uint32_t len; fin.read((char *) &len, 4); fout.write((char *) &len, 4);
        std::string w(len, 0); fin.read(&w[0], len); fout.write(w.data(), len);
    }
    ggml_init_params ip = { 1 << 20, nullptr, false };
    ggml_context * gctx = ggml_init(ip);  // initialises the fp16 tables
    const bool ok = ggml_common_quantize_0(fin, fout, (ggml_ftype) ftype, { ".*" },
                                           { "embed_positions.weight", "conv1.bias", "conv2.bias" });
    ggml_free(gctx);
    return ok ? 0 : 6;
}

// Quantizer / dot-product known answers straight from ggml:
//   q4k    : ggml_quantize_chunk(Q4_K)       (quantize_row_q4_K_ref, ggml-quants.c:2483-2553)
//   q80    : ggml_quantize_chunk(Q8_0)       (quantize_row_q8_0_ref, ggml-quants.c:848-871)
//   act_q8k: type_traits[Q8_K].from_float    (quantize_row_q8_K, ggml-quants.c:3835 -> _ref :3785)
//   act_q80: type_traits[Q8_0].from_float    (quantize_row_q8_0, ggml-quants.c:873, x86 branch)
//   f16    : ggml_fp32_to_fp16_row
int cmd_qrow(int argc, char ** argv) {
    if (argc < 6) { fprintf(stderr, "qrow KIND IN_F32 NCOLS OUT\n"); return 1; }
    ggml_init_params ip = { 1 << 20, nullptr, false };
    ggml_context * gctx = ggml_init(ip);
    const std::string kind = argv[2];
    std::vector<float> x = read_f32(argv[3]);
    const int64_t ncols = atoll(argv[4]);
    const int64_t nrows = (int64_t) x.size() / ncols;
    std::vector<uint8_t> out;
    if (kind == "q4k" || kind == "q80") {
        const ggml_type t = kind == "q4k" ? GGML_TYPE_Q4_K : GGML_TYPE_Q8_0;
        out.resize(ggml_row_size(t, ncols) * nrows);
        ggml_quantize_chunk(t, x.data(), out.data(), 0, nrows, ncols, nullptr);
    } else if (kind == "act_q8k" || kind == "act_q80") {
        const ggml_type t = kind == "act_q8k" ? GGML_TYPE_Q8_K : GGML_TYPE_Q8_0;
        ggml_type_traits_t tr = ggml_internal_get_type_traits(t);
        const size_t rs = ggml_row_size(t, ncols);
        out.resize(rs * nrows);
        for (int64_t r = 0; r < nrows; ++r) tr.from_float(x.data() + r * ncols, out.data() + r * rs, ncols);
    } else if (kind == "f16") {
        out.resize(sizeof(ggml_fp16_t) * x.size());
        ggml_fp32_to_fp16_row(x.data(), (ggml_fp16_t *) out.data(), (int64_t) x.size());
    } else {
        fprintf(stderr, "unknown kind %s\n", kind.c_str());
        return 1;
    }
    write_blob(argv[5], out.data(), out.size());
    ggml_free(gctx);
    return 0;
}

// Dot-product known answers: weights row-quantized by ggml_quantize_chunk, activations by from_float,
// then the type's vec_dot (ggml_vec_dot_q4_K_q8_K ggml-quants.c:7713, ggml_vec_dot_q8_0_q8_0 :5518,
// ggml_vec_dot_f16 ggml.c:2250). Y[r][c] = dot(W row c, X row r).
int cmd_gemm(int argc, char ** argv) {
    if (argc < 7) { fprintf(stderr, "gemm KIND W_F32 X_F32 K OUT\n"); return 1; }
    ggml_init_params ip = { 1 << 20, nullptr, false };
    ggml_context * gctx = ggml_init(ip);
    const std::string kind = argv[2];
    std::vector<float> w = read_f32(argv[3]);
    std::vector<float> x = read_f32(argv[4]);
    const int64_t K = atoll(argv[5]);
    const int64_t N = (int64_t) w.size() / K, M = (int64_t) x.size() / K;
    ggml_type wt = kind == "q4k" ? GGML_TYPE_Q4_K : kind == "q80" ? GGML_TYPE_Q8_0 : GGML_TYPE_F16;
    ggml_type_traits_t trw = ggml_internal_get_type_traits(wt);
    const ggml_type vt = trw.vec_dot_type;
    ggml_type_traits_t trv = ggml_internal_get_type_traits(vt);
    const size_t wrs = ggml_row_size(wt, K), xrs = ggml_row_size(vt, K);
    std::vector<uint8_t> wq(wrs * N), xq(xrs * M);
    if (wt == GGML_TYPE_F16) {
        ggml_fp32_to_fp16_row(w.data(), (ggml_fp16_t *) wq.data(), (int64_t) w.size());
    } else {
        ggml_quantize_chunk(wt, w.data(), wq.data(), 0, N, K, nullptr);
    }
    for (int64_t r = 0; r < M; ++r) trv.from_float(x.data() + r * K, xq.data() + r * xrs, K);
    std::vector<float> y((size_t) (M * N));
    for (int64_t r = 0; r < M; ++r)
        for (int64_t c = 0; c < N; ++c)
            trw.vec_dot((int) K, &y[(size_t) (r * N + c)], 0, wq.data() + c * wrs, 0, xq.data() + r * xrs, 0, 1);
    write_blob(argv[6], y.data(), y.size() * sizeof(float));
    ggml_free(gctx);
    return 0;
}

}  // namespace

int main(int argc, char ** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: ref_harness {mel|encode|quantize-model|qrow|gemm} ...\n");
        return 1;
    }
    whisper_log_set([](ggml_log_level, const char *, void *) {}, nullptr);
    const std::string cmd = argv[1];
    if (cmd == "mel") return cmd_mel(argc, argv);
    if (cmd == "encode") return cmd_encode(argc, argv);
    if (cmd == "quantize-model") return cmd_quantize_model(argc, argv);
    if (cmd == "qrow") return cmd_qrow(argc, argv);
    if (cmd == "gemm") return cmd_gemm(argc, argv);
    fprintf(stderr, "unknown command %s\n", cmd.c_str());
    return 1;
}
