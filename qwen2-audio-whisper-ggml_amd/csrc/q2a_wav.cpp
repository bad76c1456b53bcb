// q2a_wav.cpp — RIFF/WAVE reader for the path's audio ingestion (host code).
//
// Mirrors the acceptance rules and the sample conversion of the reference's read_wav (examples/common.cpp:642-748,
// which uses dr_wav): 16 kHz, 16-bit integer PCM, one or two channels; mono samples are s16/32768, stereo is
// mixed as (l + r)/65536 with the per-channel signals optionally returned as s16/32768. "-" reads stdin.
// WAVE_FORMAT_EXTENSIBLE with a PCM sub-format is accepted like plain PCM.
#include "q2a_whisper.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

uint32_t rd32(const uint8_t * p) { return (uint32_t) p[0] | ((uint32_t) p[1] << 8) | ((uint32_t) p[2] << 16) | ((uint32_t) p[3] << 24); }
uint16_t rd16(const uint8_t * p) { return (uint16_t) (p[0] | (p[1] << 8)); }

bool slurp(const char * path, std::vector<uint8_t> & buf) {
    FILE * f = strcmp(path, "-") == 0 ? stdin : fopen(path, "rb");
    if (!f) return false;
    uint8_t tmp[65536];
    size_t n;
    while ((n = fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + n);
    if (f != stdin) fclose(f);
    return true;
}

}  // namespace

extern "C" int q2a_read_wav(const char * path, float ** pcm, int64_t * n_samples, float ** left, float ** right) {
    if (!path || !pcm || !n_samples) return -1;
    *pcm = nullptr;
    *n_samples = 0;
    if (left) *left = nullptr;
    if (right) *right = nullptr;
    std::vector<uint8_t> b;
    if (!slurp(path, b) || b.size() < 12 || memcmp(b.data(), "RIFF", 4) != 0 || memcmp(b.data() + 8, "WAVE", 4) != 0) {
        fprintf(stderr, "q2a_read_wav: '%s' is not a RIFF/WAVE file\n", path);
        return -1;
    }
    int channels = 0, rate = 0, bits = 0, fmt = -1;
    const uint8_t * data = nullptr;
    size_t data_len = 0;
    size_t pos = 12;
    while (pos + 8 <= b.size()) {
        const uint32_t len = rd32(b.data() + pos + 4);
        const uint8_t * c = b.data() + pos + 8;
        const size_t avail = b.size() - (pos + 8);
        if (memcmp(b.data() + pos, "fmt ", 4) == 0 && len >= 16 && avail >= 16) {
            fmt = rd16(c);
            channels = rd16(c + 2);
            rate = (int) rd32(c + 4);
            bits = rd16(c + 14);
            if (fmt == 0xFFFE && len >= 40 && avail >= 40) fmt = rd16(c + 24);   // extensible: sub-format GUID
        } else if (memcmp(b.data() + pos, "data", 4) == 0) {
            data = c;
            data_len = len <= avail ? len : avail;   // a truncated or streamed file: take what is there
            break;
        }
        pos += 8 + (size_t) len + (len & 1);
    }
    if (fmt < 0 || !data) {
        fprintf(stderr, "q2a_read_wav: '%s' has no fmt/data chunk\n", path);
        return -1;
    }
    if (fmt != 1 || bits != 16) {
        fprintf(stderr, "q2a_read_wav: WAV file '%s' must be 16-bit PCM\n", path);
        return -2;
    }
    if (channels != 1 && channels != 2) {
        fprintf(stderr, "q2a_read_wav: WAV file '%s' must be mono or stereo\n", path);
        return -2;
    }
    if (rate != WHISPER_SAMPLE_RATE) {
        fprintf(stderr, "q2a_read_wav: WAV file '%s' must be %i kHz\n", path, WHISPER_SAMPLE_RATE / 1000);
        return -2;
    }
    const int64_t n = (int64_t) (data_len / (2 * (size_t) channels));
    float * out = (float *) malloc((size_t) (n > 0 ? n : 1) * sizeof(float));
    if (!out) return -1;
    const int16_t * s = (const int16_t *) data;   // little-endian host
    if (channels == 1) {
        for (int64_t i = 0; i < n; ++i) out[i] = float(s[i]) / 32768.0f;
    } else {
        for (int64_t i = 0; i < n; ++i) out[i] = float(s[2 * i] + s[2 * i + 1]) / 65536.0f;
        if (left || right) {
            float * l = (float *) malloc((size_t) (n > 0 ? n : 1) * sizeof(float));
            float * r = (float *) malloc((size_t) (n > 0 ? n : 1) * sizeof(float));
            if (!l || !r) { free(l); free(r); free(out); return -1; }
            for (int64_t i = 0; i < n; ++i) { l[i] = float(s[2 * i]) / 32768.0f; r[i] = float(s[2 * i + 1]) / 32768.0f; }
            if (left) *left = l; else free(l);
            if (right) *right = r; else free(r);
        }
    }
    *pcm = out;
    *n_samples = n;
    return 0;
}

extern "C" void q2a_wav_free(void * p) { free(p); }
