// q2a_main — command-line driver of the encoder path, the counterpart of the reference's examples/main
// (examples/main/main.cpp:455-580: read_wav -> whisper_full x N -> whisper_print_emb_enc -> timings), built on the
// reference-named API of include/q2a_whisper.h. Extras: a batched mode (all files in one encoder batch), long
// recordings as consecutive 30 s windows, and a raw dump of embd_enc.
//
//   q2a_main -m MODEL [options] file0.wav [file1.wav ...]
#include "q2a_encoder.h"
#include "q2a_whisper.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct cli {
    std::string model = "models/ggml-base.en.bin";
    std::vector<std::string> files;
    int threads = 4, offset_ms = 0, duration_ms = 0, reps = 1, device = 0, processors = 1, gpus = 0;
    bool no_prints = false, batch = false, long_audio = false, bf16 = false, device_set = false;
    std::string dump;
};

void usage(const char * argv0) {
    fprintf(stderr,
            "usage: %s [options] file0.wav file1.wav ...\n"
            "  -m FNAME,  --model FNAME    model path (reference ggml file: f16 / q4_k / q8_0 / q4_0)\n"
            "  -t N,      --threads N      host threads (staging only; the path runs on the GPU)\n"
            "  -ot N,     --offset-t N     window start in milliseconds\n"
            "  -d N,      --duration N     duration in milliseconds (reference length rule)\n"
            "  -r N,      --reps N         whisper_full repetitions per file (the reference main loops 100x)\n"
            "  -p N,      --processors N   whisper_full_parallel: N contiguous chunks per file, one batch\n"
            "  -b,        --batch          encode all files as one batch (one clip each)\n"
            "  -la,       --long-audio     encode every 30 s window of each file in one batch\n"
            "  -oemb F,   --output-emb F   write embd_enc (f32, [windows/files][750][1280]) to F\n"
            "  -dev N,    --device N       HIP device\n"
            "  -ng N,     --gpus N         -b: spread the batch over N devices, the -dev device first (default: every\n"
            "                              visible device unless -dev is given; one RCCL broadcast of the loaded\n"
            "                              weights, a host thread per device)\n"
            "  -bf16,     --bf16-act       bf16-activation contract (Q2A_ACT_BF16, BASELINE configs[4]); not the\n"
            "                              reference's numerics: see DESIGN.md\n"
            "  -np,       --no-prints      only print results\n",
            argv0);
}

bool parse(int argc, char ** argv, cli & c) {
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char * { return i + 1 < argc ? argv[++i] : nullptr; };
        const char * v = nullptr;
        if (a == "-h" || a == "--help") { usage(argv[0]); exit(0); }
        else if (a == "-m" || a == "--model") { if (!(v = next())) return false; c.model = v; }
        else if (a == "-f" || a == "--file") { if (!(v = next())) return false; c.files.push_back(v); }
        else if (a == "-t" || a == "--threads") { if (!(v = next())) return false; c.threads = atoi(v); }
        else if (a == "-ot" || a == "--offset-t") { if (!(v = next())) return false; c.offset_ms = atoi(v); }
        else if (a == "-d" || a == "--duration") { if (!(v = next())) return false; c.duration_ms = atoi(v); }
        else if (a == "-r" || a == "--reps") { if (!(v = next())) return false; c.reps = atoi(v); }
        else if (a == "-dev" || a == "--device") { if (!(v = next())) return false; c.device = atoi(v); c.device_set = true; }
        else if (a == "-p" || a == "--processors") { if (!(v = next())) return false; c.processors = atoi(v); }
        else if (a == "-ng" || a == "--gpus") { if (!(v = next())) return false; c.gpus = atoi(v); }
        else if (a == "-oemb" || a == "--output-emb") { if (!(v = next())) return false; c.dump = v; }
        else if (a == "-b" || a == "--batch") c.batch = true;
        else if (a == "-bf16" || a == "--bf16-act") c.bf16 = true;
        else if (a == "-la" || a == "--long-audio") c.long_audio = true;
        else if (a == "-np" || a == "--no-prints") c.no_prints = true;
        else if (a[0] == '-' && a != "-") { fprintf(stderr, "error: unknown argument: %s\n", a.c_str()); return false; }
        else c.files.push_back(a);
    }
    return !c.files.empty();
}

void print20(const float * e) {
    for (int i = 0; i < 20; ++i) printf(" %.3f", e[i]);
    printf("\n");
}

void quiet(enum ggml_log_level, const char *, void *) {}

}  // namespace

int main(int argc, char ** argv) {
    cli c;
    if (!parse(argc, argv, c)) { usage(argv[0]); return 1; }
    if (c.bf16) setenv("Q2A_ACT", "bf16", 1);   // the whisper_* paths read it in whisper_init
    if (c.no_prints) whisper_log_set(quiet, nullptr);
    whisper_context_params cp = whisper_context_default_params();
    cp.gpu_device = c.device;
    whisper_context * ctx = whisper_init_from_file_with_params(c.model.c_str(), cp);
    if (!ctx) { fprintf(stderr, "error: failed to initialize whisper context\n"); return 3; }
    const int n_out = ctx ? whisper_model_n_audio_ctx(ctx) / 2 : 0, n_state = whisper_model_n_audio_state(ctx);
    FILE * dump = c.dump.empty() ? nullptr : fopen(c.dump.c_str(), "wb");

    std::vector<std::vector<float>> pcms;
    for (const auto & f : c.files) {
        float * p = nullptr;
        int64_t n = 0;
        if (q2a_read_wav(f.c_str(), &p, &n, nullptr, nullptr) != 0) {
            fprintf(stderr, "error: failed to read WAV file '%s'\n", f.c_str());
            pcms.emplace_back();
            continue;
        }
        pcms.emplace_back(p, p + n);
        q2a_wav_free(p);
        if (!c.no_prints)
            fprintf(stderr, "%s: processing '%s' (%lld samples, %.1f sec) on HIP device %d\n", __func__, f.c_str(),
                    (long long) n, (double) n / WHISPER_SAMPLE_RATE, c.device);
    }

    int rc = 0;
    const auto t0 = std::chrono::steady_clock::now();
    if (c.batch) {
        // one batch: clip i = file i (the engine's native batched entry point)
        std::vector<const float *> ptr;
        std::vector<int32_t> ns;
        for (const auto & p : pcms) { ptr.push_back(p.data()); ns.push_back((int32_t) p.size()); }
        // more than one device: a q2a_group over the context's loaded weights (contiguous clip ranges, one host thread
        // per device; -ng N, or every visible device when -dev was not given); else the context's own engine
        q2a_engine * e = q2a_whisper_context_engine(ctx);
        const int ndev = c.gpus > 0 ? c.gpus : c.device_set ? 1 : q2a_device_count();
        q2a_group * grp = nullptr;
        if (c.gpus > 0 || ndev > 1) {   // (an explicit -ng always takes the group path, -ng 1 included)
            std::vector<int> devs{c.device};
            for (int d = 0; (int) devs.size() < ndev; ++d)
                if (d != c.device) devs.push_back(d);
            grp = q2a_group_open_with(e, devs.data(), ndev);
            if (!grp) { fprintf(stderr, "error: %s\n", q2a_last_error()); whisper_free(ctx); return 3; }
            if (!c.no_prints) fprintf(stderr, "%s: batch of %zu clips over %d devices\n", __func__, ptr.size(), ndev);
        }
        std::vector<float> out((size_t) ptr.size() * n_out * n_state);
        std::vector<int32_t> st(ptr.size());
        for (int r = 0; r < c.reps && rc == 0; ++r) {
            const int erc = grp ? q2a_group_encode_host(grp, ptr.data(), ns.data(), nullptr, (int) ptr.size(), c.offset_ms,
                                                        out.data(), st.data())
                                : q2a_encode_host(e, ptr.data(), ns.data(), (int) ptr.size(), c.offset_ms, out.data(), st.data());
            if (erc != Q2A_OK) {
                fprintf(stderr, "%s: failed to process audio: %s\n", argv[0], q2a_last_error());
                rc = 10;
            }
            for (size_t i = 0; i < ptr.size() && rc == 0; ++i)
                if (st[i] == Q2A_CLIP_ENCODED) print20(out.data() + i * n_out * n_state);
        }
        if (dump) fwrite(out.data(), 4, out.size(), dump);
        q2a_group_close(grp);
    } else {
        whisper_full_params wp = whisper_full_default_params(WHISPER_SAMPLING_GREEDY);
        wp.n_threads = c.threads;
        wp.offset_ms = c.offset_ms;
        wp.duration_ms = c.duration_ms;
        for (size_t f = 0; f < pcms.size() && rc == 0; ++f) {
            if (pcms[f].empty()) continue;
            if (c.long_audio) {
                const int nw = q2a_whisper_encode_long(ctx, pcms[f].data(), (int) pcms[f].size(), c.offset_ms, nullptr, 0);
                std::vector<float> out((size_t) (nw > 0 ? nw : 1) * n_out * n_state);
                if (nw < 0 || q2a_whisper_encode_long(ctx, pcms[f].data(), (int) pcms[f].size(), c.offset_ms, out.data(), nw) < 0) {
                    rc = 10;
                    break;
                }
                for (int w = 0; w < nw; ++w) print20(out.data() + (size_t) w * n_out * n_state);
                if (dump) fwrite(out.data(), 4, (size_t) nw * n_out * n_state, dump);
                continue;
            }
            if (c.processors > 1) {
                if (whisper_full_parallel(ctx, wp, pcms[f].data(), (int) pcms[f].size(), c.processors) != 0) { rc = 10; break; }
                for (int k = 0; k < whisper_full_n_chunks(ctx); ++k) {
                    const float * e = whisper_get_embd_enc_chunk(ctx, k);
                    if (!e) continue;
                    print20(e);
                    if (dump) fwrite(e, 4, (size_t) n_out * n_state, dump);
                }
                continue;
            }
            for (int r = 0; r < c.reps; ++r) {
                if (whisper_full(ctx, wp, pcms[f].data(), (int) pcms[f].size()) != 0) {
                    fprintf(stderr, "%s: failed to process audio\n", argv[0]);
                    rc = 10;
                    break;
                }
                whisper_print_emb_enc(ctx);
            }
            const float * emb = whisper_get_embd_enc(ctx, nullptr, nullptr);
            if (dump && emb) fwrite(emb, 4, (size_t) n_out * n_state, dump);
        }
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    fprintf(stderr, "%f\n", secs);
    if (dump) fclose(dump);
    if (!c.no_prints) whisper_print_timings(ctx);
    whisper_free(ctx);
    return rc;
}
