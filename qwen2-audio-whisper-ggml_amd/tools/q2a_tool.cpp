// q2a_tool — model-file tooling CLI ("the build's own loader and Q4_K/Q8_0 quantizer
// for the unchanged ggml file"; the reference ships no quantize executable).
//
//   q2a_tool gen-model OUT {tiny|full|L,D,H,M} {f32|f16} [seed] [threads]
//   q2a_tool quantize IN OUT {q4_k|q8_0|q4_0} [threads]
//   q2a_tool synth-clip OUT.f32 N_SAMPLES CLIP_INDEX
//   q2a_tool gen-projector OUT D_IN D_OUT {f32|f16} [seed]   (Qwen2-Audio multi-modal projector, q2a_format.cpp)
#include "../csrc/q2a_format.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

static int usage() {
    fprintf(stderr,
            "usage:\n  q2a_tool gen-model OUT {tiny|full|L,D,H,M} {f32|f16} [seed] [threads]\n"
            "  q2a_tool quantize IN OUT {q4_k|q8_0|q4_0} [threads]\n"
            "  q2a_tool synth-clip OUT.f32 N_SAMPLES CLIP_INDEX\n"
            "  q2a_tool gen-projector OUT D_IN D_OUT {f32|f16} [seed]\n");
    return 1;
}

int main(int argc, char ** argv) {
    if (argc < 2) return usage();
    const std::string cmd = argv[1];
    if (cmd == "gen-model" && argc >= 5) {
        q2a_hparams hp;
        memset(&hp, 0, sizeof(hp));
        hp.n_vocab = 51866; hp.n_audio_ctx = 1500; hp.n_text_ctx = 448; hp.n_text_layer = 0; hp.n_mels = 128;
        const std::string cfg = argv[3];
        if (cfg == "tiny") { hp.n_audio_layer = 2; hp.n_audio_state = 256; hp.n_audio_head = 4; }
        else if (cfg == "full") { hp.n_audio_layer = 32; hp.n_audio_state = 1280; hp.n_audio_head = 20; }
        else if (sscanf(cfg.c_str(), "%d,%d,%d,%d", &hp.n_audio_layer, &hp.n_audio_state, &hp.n_audio_head, &hp.n_mels) != 4) return usage();
        hp.n_text_state = hp.n_audio_state;
        hp.n_text_head = hp.n_audio_head;
        hp.ftype = std::string(argv[4]) == "f32" ? 0 : 1;
        const uint64_t seed = argc > 5 ? strtoull(argv[5], nullptr, 0) : 0x51A2;
        const int nt = argc > 6 ? atoi(argv[6]) : 8;
        return q2a_write_synthetic_model(argv[2], &hp, seed, nt);
    }
    if (cmd == "quantize" && argc >= 5) {
        const std::string t = argv[4];
        const int qt = t == "q4_k" ? Q2A_TYPE_Q4_K : t == "q8_0" ? Q2A_TYPE_Q8_0 : t == "q4_0" ? Q2A_TYPE_Q4_0 : -1;
        if (qt < 0) return usage();
        return q2a_quantize_model(argv[2], argv[3], qt, argc > 5 ? atoi(argv[5]) : 8);
    }
    if (cmd == "synth-clip" && argc >= 5) {
        const long n = atol(argv[3]);
        std::vector<float> v((size_t) n);
        q2a_synth_clip(v.data(), n, atoi(argv[4]));
        FILE * f = fopen(argv[2], "wb");
        if (!f) return 2;
        fwrite(v.data(), 4, v.size(), f);
        fclose(f);
        return 0;
    }
    if (cmd == "gen-projector" && argc >= 6) {
        const uint64_t seed = argc > 6 ? strtoull(argv[6], nullptr, 0) : 0x51A2;
        return q2a_write_synthetic_projector(argv[2], atoi(argv[3]), atoi(argv[4]), std::string(argv[5]) == "f32" ? 0 : 1, seed);
    }
    return usage();
}
