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
//   ggml_harness encode MODEL PCM OUT [reps] [device] [dumpdir] [ndump] [skip_lo-skip_hi]
//                                                       -> embd_enc f32 [750][1280] to OUT, JSON line on stdout; with
//                                                          dumpdir, the first ndump encoder-graph node outputs of the
//                                                          first call (per-node comparison with ref_harness's dumps)
//   ggml_harness graphs [device]                        -> HIP-graph capture vs scratch growth check, JSON line
//   ggml_harness hostbuf [device]                       -> pinned host buffer type / host registration check, JSON line

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

// first `limit` node outputs of the encoder graph through the sched eval callback (ggml-backend.cpp:2306), the same
// node numbering and file names as ref_harness's dumps. The sched stops after each observed node, so observed nodes
// run unfused (the fusion tests show fused == per-node bit for bit); nodes in [skip_lo, skip_hi] are not observed,
// so a span such as the attention chain still reaches the backend in one piece (its fused kernel)
struct dump_state {
    std::string dir;
    int asked = 0;      // nodes the sched has asked about (its asks come once per node, in graph order)
    int limit = 0;
    int skip_lo = -1, skip_hi = -1;
    FILE * index = nullptr;
};

bool dump_cb(struct ggml_tensor * t, bool ask, void * ud) {
    dump_state * ds = (dump_state *) ud;
    if (ask) {
        const int n = ds->asked++;
        return n < ds->limit && !(n >= ds->skip_lo && n <= ds->skip_hi);
    }
    const int n = ds->asked - 1;
    if (t->type == GGML_TYPE_F32 && ggml_is_contiguous(t)) {
        std::vector<float> buf(ggml_nelements(t));
        ggml_backend_tensor_get(t, buf.data(), 0, ggml_nbytes(t));
        char name[64];
        snprintf(name, sizeof(name), "node%03d_%s.f32", n, ggml_op_desc(t));
        FILE * f = fopen((ds->dir + "/" + name).c_str(), "wb");
        fwrite(buf.data(), 1, ggml_nbytes(t), f);
        fclose(f);
        fprintf(ds->index, "%d %s %lld %lld %lld %lld %s\n", n, ggml_op_desc(t), (long long) t->ne[0],
                (long long) t->ne[1], (long long) t->ne[2], (long long) t->ne[3], name);
    }
    return true;
}

int cmd_encode(int argc, char ** argv) {
    if (argc < 5) { fprintf(stderr, "encode MODEL PCM OUT [reps] [device] [dumpdir] [ndump] [skip_lo-skip_hi]\n"); return 1; }
    const int reps = argc > 5 ? atoi(argv[5]) : 1;
    whisper_context_params cp = whisper_context_default_params();
    cp.use_gpu = true;
    cp.gpu_device = argc > 6 ? atoi(argv[6]) : 0;
    whisper_context * ctx = whisper_init_from_file_with_params(argv[2], cp);
    if (!ctx) { fprintf(stderr, "model load failed: %s\n", argv[2]); return 3; }
    ggml_backend_t be = ctx->state->backends[0];
    if (!ggml_backend_is_q2a(be)) { fprintf(stderr, "backend 0 is %s, not Q2A\n", ggml_backend_name(be)); return 4; }
    std::vector<float> pcm = read_f32(argv[3]);
    dump_state ds;
    if (argc > 7) {
        ds.dir = argv[7];
        ds.limit = argc > 8 ? atoi(argv[8]) : 40;
        if (argc > 9) sscanf(argv[9], "%d-%d", &ds.skip_lo, &ds.skip_hi);
        ds.index = fopen((ds.dir + "/index.txt").c_str(), "w");
        ggml_backend_sched_set_eval_callback(ctx->state->sched_encode.sched, dump_cb, &ds);
    }
    // whisper_full_default_params() has no return statement in the reference (qwen2-whisper.cpp:4231-4295, UB):
    // zero-initialise and set what the path reads
    whisper_full_params p;
    memset(&p, 0, sizeof(p));
    p.n_threads = 4;
    double best = 1e30, total = 0, best_mel = 1e30, best_enc = 1e30, first = 0;
    for (int r = 0; r < reps; ++r) {
        const int64_t mel0 = ctx->state->t_mel_us, enc0 = ctx->state->t_encode_us;
        auto t0 = std::chrono::steady_clock::now();
        const int rc = whisper_full(ctx, p, pcm.data(), (int) pcm.size());
        auto t1 = std::chrono::steady_clock::now();
        if (rc != 0) { fprintf(stderr, "whisper_full rc=%d\n", rc); return 5; }
        const double s = std::chrono::duration<double>(t1 - t0).count();
        total += s;
        if (r == 0) first = s;
        best = std::min(best, s);
        // the reference's own phase clocks (qwen2-whisper.cpp:2335, 2651): CPU log-mel, then conv + encoder graphs
        best_mel = std::min(best_mel, 1e-6 * (double) (ctx->state->t_mel_us - mel0));
        best_enc = std::min(best_enc, 1e-6 * (double) (ctx->state->t_encode_us - enc0));
        if (r == 0 && ds.index) {
            ggml_backend_sched_set_eval_callback(ctx->state->sched_encode.sched, nullptr, nullptr);
            fclose(ds.index);
            ds.index = nullptr;
            ggml_tensor * ec = ctx->state->embd_conv;
            std::vector<float> buf(ggml_nelements(ec));
            ggml_backend_tensor_get(ec, buf.data(), 0, ggml_nbytes(ec));
            FILE * f = fopen((ds.dir + "/embd_conv.f32").c_str(), "wb");
            fwrite(buf.data(), 1, ggml_nbytes(ec), f);
            fclose(f);
        }
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
           "\"attn_fused\": %d, \"other\": %d, \"graph_replayed\": %d, \"fused\": %d, \"mm_grouped\": %d, \"mm_conv\": %d, \"mm_conv_total\": %d, \"repack_lazy\": %d, \"first_s\": %.6f, \"best_mel_s\": %.6f, \"best_encode_s\": %.6f}\n",
           (long long) e->ne[0], (long long) e->ne[1], reps, best, total / reps, ggml_backend_name(be),
           ggml_backend_buffer_name(e->buffer), ggml_backend_sched_get_n_splits(ctx->state->sched_encode.sched),
           st.n_nodes, st.n_mul_mat_fast, st.n_mul_mat_f32, st.n_attn_fused, st.n_other, st.n_graph_replayed, st.n_fused, st.n_mm_grouped, st.n_mul_mat_conv, st.n_mul_mat_conv_total, st.n_repack_lazy, first, best_mel,
           best_enc);
    whisper_free(ctx);
    return 0;
}

// A captured graph must never replay against a reallocated scratch: capture a small MUL_MAT graph (third compute =
// replay), grow the scratch with a larger graph on the same backend, then compute the small graph again — it must be
// re-run (not replayed from the stale capture) and give the same bytes.
int cmd_graphs(int argc, char ** argv) {
    const int device = argc > 2 ? atoi(argv[2]) : 0;
    ggml_backend_t be = ggml_backend_q2a_init(device);
    if (!be) { fprintf(stderr, "no Q2A backend\n"); return 3; }
    const int K = 256, N = 256;
    ggml_init_params ip = { 8 * ggml_tensor_overhead(), nullptr, true };
    ggml_context * cw = ggml_init(ip);
    ggml_tensor * w = ggml_new_tensor_2d(cw, GGML_TYPE_F16, K, N);
    ggml_backend_buffer_t bw = ggml_backend_alloc_ctx_tensors(cw, be);
    ggml_backend_buffer_set_usage(bw, GGML_BACKEND_BUFFER_USAGE_WEIGHTS);
    std::vector<ggml_fp16_t> wh((size_t) K * N);
    uint32_t st = 12345;
    auto rnd = [&]() { st = st * 1664525u + 1013904223u; return (float) ((st >> 8) & 0xFFFF) / 65536.0f - 0.5f; };
    for (auto & v : wh) v = ggml_fp32_to_fp16(rnd());
    ggml_backend_tensor_set(w, wh.data(), 0, wh.size() * 2);
    struct G { ggml_context * c; ggml_cgraph * g; ggml_tensor * x, * y; ggml_backend_buffer_t buf; };
    auto make = [&](int M) {
        ggml_init_params gp = { 16 * ggml_tensor_overhead() + ggml_graph_overhead(), nullptr, true };
        G r;
        r.c = ggml_init(gp);
        r.x = ggml_new_tensor_2d(r.c, GGML_TYPE_F32, K, M);
        r.y = ggml_mul_mat(r.c, w, r.x);
        r.g = ggml_new_graph(r.c);
        ggml_build_forward_expand(r.g, r.y);
        r.buf = ggml_backend_alloc_ctx_tensors(r.c, be);
        std::vector<float> xh((size_t) K * M);
        for (auto & v : xh) v = rnd();
        ggml_backend_tensor_set(r.x, xh.data(), 0, xh.size() * 4);
        return r;
    };
    auto run = [&](G & g, std::vector<float> * out) {
        if (ggml_backend_graph_compute(be, g.g) != GGML_STATUS_SUCCESS) { fprintf(stderr, "compute failed\n"); exit(5); }
        ggml_backend_q2a_stats s;
        memset(&s, 0, sizeof(s));
        ggml_backend_q2a_get_stats(be, &s);
        if (out) { out->resize((size_t) ggml_nelements(g.y)); ggml_backend_tensor_get(g.y, out->data(), 0, ggml_nbytes(g.y)); }
        return s;
    };
    G small = make(64), big = make(8192);
    std::vector<float> y0, y1, y2;
    run(small, &y0);
    run(small, nullptr);
    const ggml_backend_q2a_stats s3 = run(small, &y1);   // third sighting: replayed from the capture
    const ggml_backend_q2a_stats sb = run(big, nullptr);  // grows the scratch (drops the captures)
    const ggml_backend_q2a_stats s4 = run(small, &y2);    // must NOT replay the stale capture
    const ggml_backend_q2a_stats s5 = run(small, nullptr);
    const ggml_backend_q2a_stats s6 = run(small, &y2);    // captured again against the new scratch, replayed
    const bool eq = y0 == y1 && y1 == y2;
    printf("{\"replayed_third\": %d, \"reallocs_before_big\": %d, \"reallocs_after_big\": %d, \"replayed_after_grow\": %d, "
           "\"recaptured\": %d, \"replayed_again\": %d, \"equal\": %s}\n", s3.n_graph_replayed, s3.n_buffer_reallocs,
           sb.n_buffer_reallocs, s4.n_graph_replayed, s5.n_graph_replayed, s6.n_graph_replayed, eq ? "true" : "false");
    for (G * g : {&small, &big}) { ggml_backend_buffer_free(g->buf); ggml_free(g->c); }
    ggml_backend_buffer_free(bw);
    ggml_free(cw);
    ggml_backend_free(be);
    return eq ? 0 : 6;
}

// The conv MUL_MAT(F32 x, F16 w) of the backend (run_mm_conv_hilo) at conv2's shape: x all fp16 values (the GELU
// table's outputs) runs the one-part GEMM, x with one value that is not an fp16 value (a GELU passthrough x >= 10) the
// three-part one. The rows that hold only fp16 values must come out with the same bits either way; every output is
// checked against a double-precision dot product of the same operands.
int cmd_convgate(int argc, char ** argv) {
    const int device = argc > 2 ? atoi(argv[2]) : 0;
    ggml_backend_t be = ggml_backend_q2a_init(device);
    if (!be) { fprintf(stderr, "no Q2A backend\n"); return 3; }
    const int K = 3840, M = 1500, N = 1280, m_odd = 777, k_odd = 1234;
    ggml_init_params ip = { 8 * ggml_tensor_overhead(), nullptr, true };
    ggml_context * cw = ggml_init(ip);
    ggml_tensor * w = ggml_new_tensor_2d(cw, GGML_TYPE_F16, K, N);
    ggml_backend_buffer_t bw = ggml_backend_alloc_ctx_tensors(cw, be);
    ggml_backend_buffer_set_usage(bw, GGML_BACKEND_BUFFER_USAGE_WEIGHTS);
    uint32_t st = 4242;
    auto rnd = [&]() { st = st * 1664525u + 1013904223u; return (float) ((st >> 8) & 0xFFFF) / 65536.0f - 0.5f; };
    std::vector<ggml_fp16_t> wh((size_t) K * N);
    for (auto & v : wh) v = ggml_fp32_to_fp16(0.05f * rnd());
    ggml_backend_tensor_set(w, wh.data(), 0, wh.size() * 2);
    ggml_init_params gp = { 16 * ggml_tensor_overhead() + ggml_graph_overhead(), nullptr, true };
    ggml_context * c = ggml_init(gp);
    ggml_tensor * x = ggml_new_tensor_2d(c, GGML_TYPE_F32, K, M);
    ggml_tensor * y = ggml_mul_mat(c, x, w);   // [M][N] as the conv graph's node: src0 = im2col (F32), src1 = kernel
    ggml_cgraph * g = ggml_new_graph(c);
    ggml_build_forward_expand(g, y);
    ggml_backend_buffer_t bx = ggml_backend_alloc_ctx_tensors(c, be);
    std::vector<float> xh((size_t) K * M);
    for (auto & v : xh) v = ggml_fp16_to_fp32(ggml_fp32_to_fp16(4.0f * rnd()));   // fp16 values
    auto run = [&](std::vector<float> & out) {
        ggml_backend_tensor_set(x, xh.data(), 0, xh.size() * 4);
        if (ggml_backend_graph_compute(be, g) != GGML_STATUS_SUCCESS) { fprintf(stderr, "compute failed\n"); exit(5); }
        out.resize((size_t) M * N);
        ggml_backend_tensor_get(y, out.data(), 0, out.size() * 4);
    };
    // error against the f64 dot product, relative to sum |x w| (the scale of the summation's own rounding)
    auto rel = [&](const std::vector<float> & out, int m, int n) {
        double d = 0, a = 0;
        for (int k = 0; k < K; ++k) {
            const double p = (double) xh[(size_t) m * K + k] * (double) ggml_fp16_to_fp32(wh[(size_t) n * K + k]);
            d += p;
            a += fabs(p);
        }
        return fabs((double) out[(size_t) n * M + m] - d) / a;
    };
    auto err = [&](const std::vector<float> & out) {
        double worst = 0;
        for (int n = 0; n < N; n += 7)
            for (int m = 0; m < M; m += 3) worst = std::max(worst, rel(out, m, n));
        return worst;
    };
    std::vector<float> y1, y3;
    run(y1);
    const double e1 = err(y1);
    ggml_backend_q2a_stats s1;
    memset(&s1, 0, sizeof(s1));
    ggml_backend_q2a_get_stats(be, &s1);
    xh[(size_t) m_odd * K + k_odd] = 12.345678f;   // not an fp16 value: the three-part GEMM
    run(y3);
    const double e3 = err(y3);
    int64_t diff_other = 0, diff_odd = 0;
    for (int n = 0; n < N; ++n)
        for (int m = 0; m < M; ++m) {
            const bool same = memcmp(&y1[(size_t) n * M + m], &y3[(size_t) n * M + m], 4) == 0;
            if (m == m_odd) diff_odd += !same;
            else diff_other += !same;
        }
    double e_odd = 0;
    for (int n = 0; n < N; ++n) e_odd = std::max(e_odd, rel(y3, m_odd, n));
    printf("{\"mm_conv\": %d, \"max_rel_fp16_inputs\": %.3e, \"max_rel_with_odd_value\": %.3e, \"odd_row_rel\": %.3e, "
           "\"other_rows_differing\": %lld, \"odd_row_outputs_changed\": %lld}\n", s1.n_mul_mat_conv, e1, e3, e_odd,
           (long long) diff_other, (long long) diff_odd);
    ggml_backend_buffer_free(bx);
    ggml_free(c);
    ggml_backend_buffer_free(bw);
    ggml_free(cw);
    ggml_backend_free(be);
    return 0;
}

// The pinned host buffer type and host-memory registration (ggml-q2a.h; the reference's ggml-cuda.h:34, 40-41):
// a host-buffer tensor is ordinary CPU memory to ggml (is_host, written in place), copies between it and a device
// tensor carry the bytes unchanged, the device and the registry expose it the way ggml's generic code looks it up, and
// registration is opt-in (GGML_Q2A_REGISTER_HOST). Also times 64 MiB H2D from the pinned buffer vs pageable memory.
int cmd_hostbuf(int argc, char ** argv) {
    const int device = argc > 2 ? atoi(argv[2]) : 0;
    ggml_backend_t be = ggml_backend_q2a_init(device);
    if (!be) { fprintf(stderr, "no Q2A backend\n"); return 3; }
    ggml_backend_buffer_type_t hb = ggml_backend_q2a_host_buffer_type();
    ggml_backend_dev_t dev = ggml_backend_get_device(be);
    ggml_backend_dev_props props;
    ggml_backend_dev_get_props(dev, &props);
    ggml_backend_reg_t reg = ggml_backend_q2a_reg();
    typedef bool (*reg_fn)(void *, size_t);
    typedef void (*unreg_fn)(void *);
    reg_fn rf = (reg_fn) ggml_backend_reg_get_proc_address(reg, "ggml_backend_register_host_buffer");
    unreg_fn uf = (unreg_fn) ggml_backend_reg_get_proc_address(reg, "ggml_backend_unregister_host_buffer");
    const bool split_absent = ggml_backend_reg_get_proc_address(reg, "ggml_backend_split_buffer_type") == nullptr;

    const int64_t n = 16 << 20;   // 64 MiB of f32
    ggml_init_params ip = { 4 * ggml_tensor_overhead(), nullptr, true };
    ggml_context * ch = ggml_init(ip), * cd = ggml_init(ip);
    ggml_tensor * th = ggml_new_tensor_1d(ch, GGML_TYPE_F32, n);
    ggml_tensor * td = ggml_new_tensor_1d(cd, GGML_TYPE_F32, n);
    ggml_backend_buffer_t bh = ggml_backend_alloc_ctx_tensors_from_buft(ch, hb);
    ggml_backend_buffer_t bd = ggml_backend_alloc_ctx_tensors(cd, be);
    if (!bh || !bd) { fprintf(stderr, "allocation failed\n"); return 4; }
    const bool pinned = strcmp(ggml_backend_buffer_name(bh), GGML_Q2A_NAME "_Host") == 0;
    float * hp = (float *) th->data;   // host memory: written in place
    for (int64_t i = 0; i < n; ++i) hp[i] = (float) ((i * 2654435761u) % 1000003) * 1e-3f - 500.f;
    ggml_backend_tensor_copy(th, td);   // host -> device (dst->buffer set_tensor from the pinned bytes)
    std::vector<float> back((size_t) n);
    ggml_backend_tensor_get(td, back.data(), 0, (size_t) n * 4);
    bool eq = memcmp(back.data(), hp, (size_t) n * 4) == 0;
    memset(hp, 0, (size_t) n * 4);
    ggml_backend_tensor_copy(td, th);   // device -> host buffer
    eq = eq && memcmp(back.data(), hp, (size_t) n * 4) == 0;

    auto h2d_gbs = [&](const void * src) {
        double best = 1e30;
        for (int r = 0; r < 5; ++r) {
            auto t0 = std::chrono::steady_clock::now();
            ggml_backend_tensor_set(td, src, 0, (size_t) n * 4);
            auto t1 = std::chrono::steady_clock::now();
            best = std::min(best, std::chrono::duration<double>(t1 - t0).count());
        }
        return (double) n * 4 / best / 1e9;
    };
    std::vector<float> pageable(back);
    const double gbs_pinned = h2d_gbs(hp), gbs_pageable = h2d_gbs(pageable.data());

    // registration of caller-owned memory: refused unless opted in, then page-locked and released again
    const char * opt = getenv("GGML_Q2A_REGISTER_HOST");
    const bool reg_default = opt ? true : ggml_backend_q2a_register_host_buffer(pageable.data(), pageable.size() * 4);
    setenv("GGML_Q2A_REGISTER_HOST", "1", 1);
    const bool reg_optin = rf && rf(pageable.data(), pageable.size() * 4);
    const double gbs_registered = h2d_gbs(pageable.data());
    if (uf) uf(pageable.data());
    if (!opt) unsetenv("GGML_Q2A_REGISTER_HOST");

    printf("{\"host_buft_name\": \"%s\", \"is_host\": %s, \"buffer_name\": \"%s\", \"pinned\": %s, \"dev_host_buft_same\": %s, "
           "\"caps_host_buffer\": %s, \"buft_device_set\": %s, \"proc_register\": %s, \"proc_unregister\": %s, \"split_absent\": %s, "
           "\"copies_equal\": %s, \"register_without_optin\": %s, \"register_optin\": %s, \"h2d_gbs_pinned\": %.2f, "
           "\"h2d_gbs_pageable\": %.2f, \"h2d_gbs_registered\": %.2f}\n",
           ggml_backend_buft_name(hb), ggml_backend_buft_is_host(hb) ? "true" : "false", ggml_backend_buffer_name(bh),
           pinned ? "true" : "false", ggml_backend_dev_host_buffer_type(dev) == hb ? "true" : "false",
           props.caps.host_buffer ? "true" : "false", ggml_backend_buft_get_device(hb) != nullptr ? "true" : "false",
           rf == (reg_fn) ggml_backend_q2a_register_host_buffer ? "true" : "false",
           uf == (unreg_fn) ggml_backend_q2a_unregister_host_buffer ? "true" : "false", split_absent ? "true" : "false",
           eq ? "true" : "false", reg_default ? "true" : "false", reg_optin ? "true" : "false", gbs_pinned, gbs_pageable,
           gbs_registered);
    ggml_backend_buffer_free(bh);
    ggml_backend_buffer_free(bd);
    ggml_free(ch);
    ggml_free(cd);
    ggml_backend_free(be);
    return eq ? 0 : 6;
}

}  // namespace

int main(int argc, char ** argv) {
    if (argc < 2) { fprintf(stderr, "usage: ggml_harness encode ...\n"); return 1; }
    whisper_log_set([](ggml_log_level lvl, const char * text, void *) { if (lvl == GGML_LOG_LEVEL_ERROR) fputs(text, stderr); }, nullptr);
    if (std::string(argv[1]) == "encode") return cmd_encode(argc, argv);
    if (std::string(argv[1]) == "graphs") return cmd_graphs(argc, argv);
    if (std::string(argv[1]) == "hostbuf") return cmd_hostbuf(argc, argv);
    if (std::string(argv[1]) == "convgate") return cmd_convgate(argc, argv);
    fprintf(stderr, "unknown command %s\n", argv[1]);
    return 1;
}
