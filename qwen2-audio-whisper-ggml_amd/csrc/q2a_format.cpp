// q2a_format.cpp — model-file tooling: synthetic generator, reader, byte-exact k-quant/Q8_0 quantizers.
// Compiled with -ffp-contract=off: the quantizers must round exactly like the reference build (the
// reference's shipped Debug build forms no FMAs), so that quantized bytes are identical.
#include "q2a_format.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

// ------------------------------------------------------------------------------------------------
// fp16 <-> fp32 (IEEE binary16, RNE) — same results as F16C vcvtps2ph imm=0 used by GGML_FP32_TO_FP16
// ------------------------------------------------------------------------------------------------
static inline uint32_t f32_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bits_f32(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

extern "C" uint16_t q2a_fp32_to_fp16(float f) {
    const uint32_t x = f32_bits(f);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) {                       // inf / nan
        return (uint16_t) (sign | 0x7c00u | (ax > 0x7f800000u ? 0x200u | ((ax >> 13) & 0x3ffu) : 0u));
    }
    if (ax >= 0x477ff000u) {                       // >= 65520 rounds to inf
        return (uint16_t) (sign | 0x7c00u);
    }
    if (ax < 0x38800000u) {                        // below the smallest normal half (2^-14): subnormal
        // value = ax as float; half subnormal unit = 2^-24
        const float v = bits_f32(ax);
        // exact scaling by 2^24 then RNE to integer (the magic-add trick keeps RNE)
        const float scaled = v * 16777216.0f;      // exact (power of two)
        const float r = scaled + 12582912.0f - 12582912.0f;  // RNE for |scaled| < 2^22
        return (uint16_t) (sign | (uint32_t) r);
    }
    // normal range: rebias exponent, RNE on the 13 dropped bits
    uint32_t m = ax + 0xc8000000u;                 // exponent -= 112 (127-15) << 23
    const uint32_t lsb = (m >> 13) & 1u;
    m += 0xfffu + lsb;
    return (uint16_t) (sign | (m >> 13));
}

extern "C" float q2a_fp16_to_fp32(uint16_t h) {
    const uint32_t sign = (uint32_t) (h & 0x8000u) << 16;
    const uint32_t exp = (h >> 10) & 0x1fu;
    const uint32_t man = h & 0x3ffu;
    if (exp == 0) {
        if (man == 0) return bits_f32(sign);
        const float v = (float) man * (1.0f / 16777216.0f);   // exact
        return sign ? -v : v;
    }
    if (exp == 31) return bits_f32(sign | 0x7f800000u | (man << 13));
    return bits_f32(sign | ((exp + 112u) << 23) | (man << 13));
}

extern "C" size_t q2a_row_size(int t, int64_t n) {
    switch (t) {
        case Q2A_TYPE_F32: return (size_t) n * 4;
        case Q2A_TYPE_F16: return (size_t) n * 2;
        case Q2A_TYPE_Q4_0: return (size_t) (n / 32) * sizeof(q2a_block_q4_0);
        case Q2A_TYPE_Q8_0: return (size_t) (n / 32) * sizeof(q2a_block_q8_0);
        case Q2A_TYPE_Q4_K: return (size_t) (n / 256) * sizeof(q2a_block_q4_K);
        case Q2A_TYPE_Q8_K: return (size_t) (n / 256) * sizeof(q2a_block_q8_K);
        default: return 0;
    }
}

static_assert(sizeof(q2a_block_q4_0) == 18, "q4_0");
static_assert(sizeof(q2a_block_q8_0) == 34, "q8_0");
static_assert(sizeof(q2a_block_q4_K) == 144, "q4_K");
static_assert(sizeof(q2a_block_q8_K) == 292, "q8_K");

// ------------------------------------------------------------------------------------------------
// deterministic generators
// ------------------------------------------------------------------------------------------------
extern "C" uint64_t q2a_splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

extern "C" double q2a_gauss(uint64_t seed, uint32_t stream, uint64_t index) {
    const uint64_t v = q2a_splitmix64(seed ^ ((uint64_t) stream << 40) ^ index);
    const double u1 = (double) ((v >> 40) + 1) / 16777217.0;          // (0, 1)
    const double u2 = (double) (v & 0xffffffull) / 16777216.0;        // [0, 1)
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
}

extern "C" void q2a_synth_clip(float * out, int64_t n, int c) {
    const double f1 = 220.0 + 37.0 * c, f2 = 1000.0 + 53.0 * c;
    const uint64_t seed = 0xA0D1000000000000ull + (uint64_t) c;
    for (int64_t t = 0; t < n; ++t) {
        const double tt = (double) t / 16000.0;
        const double v = 0.3 * std::sin(6.283185307179586 * f1 * tt) + 0.1 * std::sin(6.283185307179586 * f2 * tt) +
                         0.05 * q2a_gauss(seed, 0, (uint64_t) t);
        out[t] = (float) v;
    }
}

static double hz_to_mel_slaney(double f) {
    const double f_sp = 200.0 / 3.0, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
    const double logstep = std::log(6.4) / 27.0;
    return f >= min_log_hz ? min_log_mel + std::log(f / min_log_hz) / logstep : f / f_sp;
}
static double mel_to_hz_slaney(double m) {
    const double f_sp = 200.0 / 3.0, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
    const double logstep = std::log(6.4) / 27.0;
    return m >= min_log_mel ? min_log_hz * std::exp(logstep * (m - min_log_mel)) : f_sp * m;
}

extern "C" void q2a_mel_filters_slaney(float * out, int n_mel, int n_fft, int sr) {
    const int n_bins = n_fft / 2 + 1;
    std::vector<double> fftf(n_bins), melf(n_mel + 2);
    for (int k = 0; k < n_bins; ++k) fftf[k] = (double) k * (sr / 2.0) / (n_bins - 1);
    const double mlo = hz_to_mel_slaney(0.0), mhi = hz_to_mel_slaney(sr / 2.0);
    for (int i = 0; i < n_mel + 2; ++i) melf[i] = mel_to_hz_slaney(mlo + (mhi - mlo) * i / (n_mel + 1));
    for (int i = 0; i < n_mel; ++i) {
        const double fd0 = melf[i + 1] - melf[i], fd1 = melf[i + 2] - melf[i + 1];
        const double enorm = 2.0 / (melf[i + 2] - melf[i]);
        for (int k = 0; k < n_bins; ++k) {
            const double lower = -(melf[i] - fftf[k]) / fd0;
            const double upper = (melf[i + 2] - fftf[k]) / fd1;
            out[(size_t) i * n_bins + k] = (float) (std::max(0.0, std::min(lower, upper)) * enorm);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// quantizers (restated from ggml-quants.c; byte-exact with ggml_quantize_chunk)
// ------------------------------------------------------------------------------------------------
static inline int nearest_int(float fval) {               // ggml-quants.c:1639-1644
    float val = fval + 12582912.f;
    int i; memcpy(&i, &val, sizeof(int));
    return (i & 0x007fffff) - 0x00400000;
}

// make_qkx2_quants, ggml-quants.c:1817-1896 (weighted least squares search for scale/min)
static float make_qkx2(int n, int nmax, const float * x, const float * w, uint8_t * L, float * the_min,
                       uint8_t * Laux, float rmin, float rdelta, int nstep) {
    float mn = x[0], mx = x[0];
    float sum_w = w[0];
    float sum_x = sum_w * x[0];
    for (int i = 1; i < n; ++i) {
        if (x[i] < mn) mn = x[i];
        if (x[i] > mx) mx = x[i];
        sum_w += w[i];
        sum_x += w[i] * x[i];
    }
    if (mn > 0) mn = 0;
    if (mx == mn) {
        for (int i = 0; i < n; ++i) L[i] = 0;
        *the_min = -mn;
        return 0.f;
    }
    float iscale = nmax / (mx - mn);
    float scale = 1 / iscale;
    float best = 0;
    for (int i = 0; i < n; ++i) {
        int l = nearest_int(iscale * (x[i] - mn));
        L[i] = (uint8_t) std::max(0, std::min(nmax, l));
        float diff = scale * L[i] + mn - x[i];
        diff = diff * diff;
        best += w[i] * diff;
    }
    for (int is = 0; is <= nstep; ++is) {
        iscale = (rmin + rdelta * is + nmax) / (mx - mn);
        float sum_l = 0, sum_l2 = 0, sum_xl = 0;
        for (int i = 0; i < n; ++i) {
            int l = nearest_int(iscale * (x[i] - mn));
            l = std::max(0, std::min(nmax, l));
            Laux[i] = (uint8_t) l;
            const float wi = w[i];
            sum_l += wi * l;
            sum_l2 += wi * l * l;
            sum_xl += wi * l * x[i];
        }
        const float D = sum_w * sum_l2 - sum_l * sum_l;
        if (D > 0) {
            float this_scale = (sum_w * sum_xl - sum_x * sum_l) / D;
            float this_min = (sum_l2 * sum_x - sum_l * sum_xl) / D;
            if (this_min > 0) {
                this_min = 0;
                this_scale = sum_xl / sum_l2;
            }
            float mad = 0;
            for (int i = 0; i < n; ++i) {
                float diff = this_scale * Laux[i] + this_min - x[i];
                diff = diff * diff;
                mad += w[i] * diff;
            }
            if (mad < best) {
                for (int i = 0; i < n; ++i) L[i] = Laux[i];
                best = mad;
                scale = this_scale;
                mn = this_min;
            }
        }
    }
    *the_min = -mn;
    return scale;
}

static inline void scale_min_k4(int j, const uint8_t * q, uint8_t * d, uint8_t * m) {   // ggml-quants.c:1898
    if (j < 4) {
        *d = q[j] & 63;
        *m = q[j + 4] & 63;
    } else {
        *d = (uint8_t) ((q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4));
        *m = (uint8_t) ((q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4));
    }
}

extern "C" void q2a_quantize_row_q4_K(const float * x, void * vy, int64_t k) {
    q2a_block_q4_K * y = (q2a_block_q4_K *) vy;
    const int64_t nb = k / 256;
    uint8_t L[256], Laux[32];
    float weights[32], mins[8], scales[8];
    for (int64_t i = 0; i < nb; i++) {
        float max_scale = 0, max_min = 0;
        for (int j = 0; j < 8; ++j) {
            float sum_x2 = 0;
            for (int l = 0; l < 32; ++l) sum_x2 += x[32 * j + l] * x[32 * j + l];
            const float av_x = sqrtf(sum_x2 / 32);
            for (int l = 0; l < 32; ++l) weights[l] = av_x + fabsf(x[32 * j + l]);
            scales[j] = make_qkx2(32, 15, x + 32 * j, weights, L + 32 * j, &mins[j], Laux, -1.f, 0.1f, 20);
            if (scales[j] > max_scale) max_scale = scales[j];
            if (mins[j] > max_min) max_min = mins[j];
        }
        const float inv_scale = max_scale > 0 ? 63.f / max_scale : 0.f;
        const float inv_min = max_min > 0 ? 63.f / max_min : 0.f;
        memset(y[i].scales, 0, 12);
        for (int j = 0; j < 8; ++j) {
            uint8_t ls = (uint8_t) nearest_int(inv_scale * scales[j]);
            uint8_t lm = (uint8_t) nearest_int(inv_min * mins[j]);
            ls = std::min<uint8_t>(63, ls);
            lm = std::min<uint8_t>(63, lm);
            if (j < 4) {
                y[i].scales[j] = ls;
                y[i].scales[j + 4] = lm;
            } else {
                y[i].scales[j + 4] = (uint8_t) ((ls & 0xF) | ((lm & 0xF) << 4));
                y[i].scales[j - 4] |= (uint8_t) ((ls >> 4) << 6);
                y[i].scales[j - 0] |= (uint8_t) ((lm >> 4) << 6);
            }
        }
        y[i].d = q2a_fp32_to_fp16(max_scale / 63.f);
        y[i].dmin = q2a_fp32_to_fp16(max_min / 63.f);
        for (int j = 0; j < 8; ++j) {
            uint8_t sc, m;
            scale_min_k4(j, y[i].scales, &sc, &m);
            const float d = q2a_fp16_to_fp32(y[i].d) * sc;
            if (!d) continue;
            const float dm = q2a_fp16_to_fp32(y[i].dmin) * m;
            for (int ii = 0; ii < 32; ++ii) {
                int l = nearest_int((x[32 * j + ii] + dm) / d);
                L[32 * j + ii] = (uint8_t) std::max(0, std::min(15, l));
            }
        }
        uint8_t * q = y[i].qs;
        for (int j = 0; j < 256; j += 64) {
            for (int l = 0; l < 32; ++l) q[l] = (uint8_t) (L[j + l] | (L[j + l + 32] << 4));
            q += 32;
        }
        x += 256;
    }
}

extern "C" void q2a_quantize_row_q8_0(const float * x, void * vy, int64_t k) {
    q2a_block_q8_0 * y = (q2a_block_q8_0 *) vy;
    const int64_t nb = k / 32;
    for (int64_t i = 0; i < nb; i++) {
        float amax = 0.0f;
        for (int j = 0; j < 32; j++) amax = std::max(amax, fabsf(x[i * 32 + j]));
        const float d = amax / ((1 << 7) - 1);
        const float id = d ? 1.0f / d : 0.0f;
        y[i].d = q2a_fp32_to_fp16(d);
        for (int j = 0; j < 32; ++j) y[i].qs[j] = (int8_t) roundf(x[i * 32 + j] * id);
    }
}

extern "C" void q2a_quantize_row_q4_0(const float * x, void * vy, int64_t k) {
    q2a_block_q4_0 * y = (q2a_block_q4_0 *) vy;
    const int64_t nb = k / 32;
    for (int64_t i = 0; i < nb; i++) {
        float amax = 0.0f, mx = 0.0f;
        for (int j = 0; j < 32; j++) {
            const float v = x[i * 32 + j];
            if (amax < fabsf(v)) { amax = fabsf(v); mx = v; }
        }
        const float d = mx / -8;
        const float id = d ? 1.0f / d : 0.0f;
        y[i].d = q2a_fp32_to_fp16(d);
        for (int j = 0; j < 16; ++j) {
            const float x0 = x[i * 32 + j] * id;
            const float x1 = x[i * 32 + 16 + j] * id;
            const uint8_t xi0 = (uint8_t) std::min(15, (int) (int8_t) (x0 + 8.5f));
            const uint8_t xi1 = (uint8_t) std::min(15, (int) (int8_t) (x1 + 8.5f));
            y[i].qs[j] = (uint8_t) (xi0 | (xi1 << 4));
        }
    }
}

// ------------------------------------------------------------------------------------------------
// reference numerics tables
// ------------------------------------------------------------------------------------------------
extern "C" void q2a_make_gelu_table(uint16_t * tab) {
    const float GELU_COEF_A = 0.044715f;
    const float SQRT_2_OVER_PI = 0.79788456080286535587989211986876f;
    for (int i = 0; i < 65536; ++i) {
        const float x = q2a_fp16_to_fp32((uint16_t) i);
        const float g = 0.5f * x * (1.0f + tanhf(SQRT_2_OVER_PI * x * (1.0f + GELU_COEF_A * x * x)));
        tab[i] = q2a_fp32_to_fp16(g);
    }
}

extern "C" void q2a_make_mel_tables(float * t) {
    const int N = 400;
    for (int i = 0; i < N; i++) {
        const double theta = (2 * M_PI * i) / N;
        t[N + i] = cosf((float) theta);
        t[2 * N + i] = sinf((float) theta);
    }
    for (int i = 0; i < N; i++) t[i] = (float) (0.5 * (1.0 - cosf((float) ((2.0 * M_PI * i) / N))));
}

// ------------------------------------------------------------------------------------------------
// writer
// ------------------------------------------------------------------------------------------------
namespace {

struct out_file {
    FILE * f = nullptr;
    bool ok = true;
    void w(const void * p, size_t n) { if (fwrite(p, 1, n, f) != n) ok = false; }
    void i32(int32_t v) { w(&v, 4); }
};

void write_tensor_header(out_file & o, const std::string & name, int ttype, std::vector<int32_t> ne) {
    o.i32((int32_t) ne.size());
    o.i32((int32_t) name.size());
    o.i32(ttype);
    for (int32_t v : ne) o.i32(v);
    o.w(name.data(), name.size());
}

// fill v[i] = mean + stdev * N(0,1) for (seed, stream, i), parallel over index ranges
void fill_gauss(std::vector<float> & v, uint64_t seed, uint32_t stream, float mean, float stdev, int nt) {
    const size_t n = v.size();
    auto work = [&](size_t b, size_t e) {
        for (size_t i = b; i < e; ++i) v[i] = (float) (mean + stdev * q2a_gauss(seed, stream, i));
    };
    if (nt <= 1 || n < (1u << 16)) { work(0, n); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(work, n * t / nt, n * (t + 1) / nt);
    for (auto & x : th) x.join();
}

void emit(out_file & o, const std::string & name, std::vector<int32_t> ne_np /*numpy shape*/, bool big,
          int ftype, uint64_t seed, uint32_t stream, float mean, float stdev, int nt, const float * fixed = nullptr) {
    size_t n = 1;
    for (int32_t d : ne_np) n *= (size_t) d;
    std::vector<float> v(n);
    if (fixed) memcpy(v.data(), fixed, n * 4);
    else fill_gauss(v, seed, stream, mean, stdev, nt);
    std::vector<int32_t> ne(ne_np.rbegin(), ne_np.rend());
    const bool f16 = big && ftype == 1;
    write_tensor_header(o, name, f16 ? Q2A_TYPE_F16 : Q2A_TYPE_F32, ne);
    if (f16) {
        std::vector<uint16_t> h(n);
        for (size_t i = 0; i < n; ++i) h[i] = q2a_fp32_to_fp16(v[i]);
        o.w(h.data(), n * 2);
    } else {
        o.w(v.data(), n * 4);
    }
}

}  // namespace

extern "C" int q2a_write_synthetic_model(const char * path, const q2a_hparams * hp, uint64_t seed, int nt) {
    out_file o;
    o.f = fopen(path, "wb");
    if (!o.f) return -1;
    const int D = hp->n_audio_state, T = hp->n_audio_ctx, M = hp->n_mels, L = hp->n_audio_layer;
    const int ftype = hp->ftype;
    o.i32((int32_t) Q2A_FILE_MAGIC);
    o.w(hp, sizeof(q2a_hparams));
    // mel filters [n_mel][201]
    const int n_fft = 201;
    std::vector<float> filt((size_t) M * n_fft);
    q2a_mel_filters_slaney(filt.data(), M, 400, 16000);
    o.i32(M);
    o.i32(n_fft);
    o.w(filt.data(), filt.size() * 4);
    o.i32(0);  // empty vocab (the encoder path never reads tokens)
    const float sd = 0.02f;
    // tensor order follows the HF Qwen2AudioEncoder state dict (convert-pt-to-ggml.py:289 iterates it)
    emit(o, "conv1.weight", {D, M, 3}, true, ftype, seed, 0, 0.f, sd, nt);
    emit(o, "conv1.bias", {D, 1}, false, ftype, seed, 1, 0.f, sd, nt);
    emit(o, "conv2.weight", {D, D, 3}, true, ftype, seed, 2, 0.f, sd, nt);
    emit(o, "conv2.bias", {D, 1}, false, ftype, seed, 3, 0.f, sd, nt);
    {
        // exact sinusoids (whisper `sinusoids(length, channels)`), [T][D] = [sin | cos]
        std::vector<float> pe((size_t) T * D);
        const int half = D / 2;
        const double inc = std::log(10000.0) / (half - 1);
        for (int t = 0; t < T; ++t)
            for (int c = 0; c < half; ++c) {
                const double a = t * std::exp(-inc * c);
                pe[(size_t) t * D + c] = (float) std::sin(a);
                pe[(size_t) t * D + half + c] = (float) std::cos(a);
            }
        emit(o, "embed_positions.weight", {T, D}, false, ftype, seed, 5, 0.f, 0.f, nt, pe.data());
    }
    const int F = 4 * D;
    for (int l = 0; l < L; ++l) {
        const std::string p = "layers." + std::to_string(l) + ".";
        const uint32_t s = 16 + 16 * (uint32_t) l;
        emit(o, p + "self_attn.k_proj.weight", {D, D}, true, ftype, seed, s + 2, 0.f, sd, nt);
        emit(o, p + "self_attn.v_proj.weight", {D, D}, true, ftype, seed, s + 3, 0.f, sd, nt);
        emit(o, p + "self_attn.v_proj.bias", {D}, false, ftype, seed, s + 4, 0.f, sd, nt);
        emit(o, p + "self_attn.q_proj.weight", {D, D}, true, ftype, seed, s + 0, 0.f, sd, nt);
        emit(o, p + "self_attn.q_proj.bias", {D}, false, ftype, seed, s + 1, 0.f, sd, nt);
        emit(o, p + "self_attn.out_proj.weight", {D, D}, true, ftype, seed, s + 5, 0.f, sd, nt);
        emit(o, p + "self_attn.out_proj.bias", {D}, false, ftype, seed, s + 6, 0.f, sd, nt);
        emit(o, p + "self_attn_layer_norm.weight", {D}, false, ftype, seed, s + 7, 1.f, sd, nt);
        emit(o, p + "self_attn_layer_norm.bias", {D}, false, ftype, seed, s + 8, 0.f, sd, nt);
        emit(o, p + "fc1.weight", {F, D}, true, ftype, seed, s + 9, 0.f, sd, nt);
        emit(o, p + "fc1.bias", {F}, false, ftype, seed, s + 10, 0.f, sd, nt);
        emit(o, p + "fc2.weight", {D, F}, true, ftype, seed, s + 11, 0.f, sd, nt);
        emit(o, p + "fc2.bias", {D}, false, ftype, seed, s + 12, 0.f, sd, nt);
        emit(o, p + "final_layer_norm.weight", {D}, false, ftype, seed, s + 13, 1.f, sd, nt);
        emit(o, p + "final_layer_norm.bias", {D}, false, ftype, seed, s + 14, 0.f, sd, nt);
    }
    emit(o, "layer_norm.weight", {D}, false, ftype, seed, 4, 1.f, sd, nt);
    emit(o, "layer_norm.bias", {D}, false, ftype, seed, 6, 0.f, sd, nt);
    const bool ok = o.ok;
    fclose(o.f);
    return ok ? 0 : -2;
}

// The Qwen2-Audio multi-modal projector (transformers modeling_qwen2_audio.py Qwen2AudioMultiModalProjector: one
// nn.Linear(audio d_model, text hidden_size, bias=True) over the encoder's last_hidden_state) in the same ggml container:
// hparams with n_audio_state = d_in, n_text_state = d_out (every other field 0 but ftype), no filters, no vocab,
// tensors multi_modal_projector.linear.weight [d_out][d_in] (F16 or F32 by ftype, quantizable by q2a_quantize_model)
// and multi_modal_projector.linear.bias [d_out] F32. The reference's converter stops at the encoder
// (qwen2-whisper.cpp:2185 ends the path at embd_enc), so this is the layout a converter of the projector would emit.
extern "C" int q2a_write_synthetic_projector(const char * path, int d_in, int d_out, int ftype, uint64_t seed) {
    if (d_in <= 0 || d_out <= 0 || (ftype != 0 && ftype != 1)) return -3;
    out_file o;
    o.f = fopen(path, "wb");
    if (!o.f) return -1;
    q2a_hparams hp;
    memset(&hp, 0, sizeof(hp));
    hp.n_audio_state = d_in;
    hp.n_text_state = d_out;
    hp.ftype = ftype;
    o.i32((int32_t) Q2A_FILE_MAGIC);
    o.w(&hp, sizeof(hp));
    o.i32(0);   // n_mel
    o.i32(0);   // n_fft
    o.i32(0);   // vocab
    emit(o, "multi_modal_projector.linear.weight", {d_out, d_in}, true, ftype, seed, 1000, 0.f, 0.02f, 8);
    emit(o, "multi_modal_projector.linear.bias", {d_out}, false, ftype, seed, 1001, 0.f, 0.02f, 8);
    const bool ok = o.ok;
    fclose(o.f);
    return ok ? 0 : -2;
}

// ------------------------------------------------------------------------------------------------
// reader
// ------------------------------------------------------------------------------------------------
namespace {
struct in_file {
    FILE * f;
    bool r(void * p, size_t n) { return fread(p, 1, n, f) == n; }
};
void set_err(char * err, size_t len, const char * msg, const char * extra = "") {
    if (err && len) snprintf(err, len, "%s%s", msg, extra);
}
int ftype_to_wtype(int ft) {
    switch (ft) {
        case Q2A_FTYPE_ALL_F32: return Q2A_TYPE_F32;
        case Q2A_FTYPE_MOSTLY_F16: return Q2A_TYPE_F16;
        case Q2A_FTYPE_MOSTLY_Q4_0: return Q2A_TYPE_Q4_0;
        case Q2A_FTYPE_MOSTLY_Q8_0: return Q2A_TYPE_Q8_0;
        case Q2A_FTYPE_MOSTLY_Q4_K: return Q2A_TYPE_Q4_K;
        default: return -1;
    }
}
}  // namespace

extern "C" q2a_model_file * q2a_model_file_read(const char * path, char * err, size_t err_len) {
    in_file in{fopen(path, "rb")};
    if (!in.f) { set_err(err, err_len, "cannot open model file ", path); return nullptr; }
    q2a_model_file * mf = (q2a_model_file *) calloc(1, sizeof(q2a_model_file));
    auto fail = [&](const char * msg, const char * extra = "") {
        set_err(err, err_len, msg, extra);
        fclose(in.f);
        q2a_model_file_free(mf);
        return (q2a_model_file *) nullptr;
    };
    uint32_t magic = 0;
    if (!in.r(&magic, 4) || magic != Q2A_FILE_MAGIC) return fail("invalid model data (bad magic)");
    if (!in.r(&mf->hp, sizeof(q2a_hparams))) return fail("truncated hparams");
    mf->qntvr = mf->hp.ftype / Q2A_QNT_VERSION_FACTOR;
    const int ft = mf->hp.ftype % Q2A_QNT_VERSION_FACTOR;
    mf->wtype = ftype_to_wtype(ft);
    if (mf->wtype < 0) return fail("unsupported ftype");
    if (!in.r(&mf->n_mel_filt, 4) || !in.r(&mf->n_fft_filt, 4)) return fail("truncated filters");
    const size_t nf = (size_t) mf->n_mel_filt * mf->n_fft_filt;
    mf->filters = (float *) malloc(nf * 4);
    if (!in.r(mf->filters, nf * 4)) return fail("truncated filters");
    int32_t n_vocab = 0;
    if (!in.r(&n_vocab, 4)) return fail("truncated vocab");
    for (int i = 0; i < n_vocab; ++i) {
        uint32_t len;
        if (!in.r(&len, 4)) return fail("truncated vocab");
        if (len) fseek(in.f, (long) len, SEEK_CUR);
    }
    // tensors: first pass records descriptors and payloads
    std::vector<q2a_tensor_desc> descs;
    std::vector<uint8_t> data;
    while (true) {
        int32_t n_dims, len, ttype;
        if (!in.r(&n_dims, 4)) break;
        if (!in.r(&len, 4) || !in.r(&ttype, 4)) return fail("truncated tensor header");
        if (n_dims < 1 || n_dims > 4 || len <= 0 || len >= 96) return fail("bad tensor header");
        q2a_tensor_desc d;
        memset(&d, 0, sizeof(d));
        d.type = ttype;
        d.n_dims = n_dims;
        int64_t nel = 1;
        for (int i = 0; i < 4; ++i) d.ne[i] = 1;
        for (int i = 0; i < n_dims; ++i) {
            int32_t v;
            if (!in.r(&v, 4)) return fail("truncated tensor dims");
            d.ne[i] = v;
            nel *= v;
        }
        if (!in.r(d.name, (size_t) len)) return fail("truncated tensor name");
        d.nbytes = q2a_row_size(ttype, d.ne[0]) * (size_t) (nel / d.ne[0]);
        if (d.nbytes == 0) return fail("unsupported tensor type in ", d.name);
        d.offset = data.size();
        data.resize(data.size() + d.nbytes);
        if (!in.r(data.data() + d.offset, d.nbytes)) return fail("truncated tensor data ", d.name);
        descs.push_back(d);
    }
    fclose(in.f);
    mf->n_tensors = (int32_t) descs.size();
    mf->tensors = (q2a_tensor_desc *) malloc(descs.size() * sizeof(q2a_tensor_desc));
    memcpy(mf->tensors, descs.data(), descs.size() * sizeof(q2a_tensor_desc));
    mf->data_size = data.size();
    mf->data = (uint8_t *) malloc(data.size() ? data.size() : 1);
    memcpy(mf->data, data.data(), data.size());
    return mf;
}

extern "C" void q2a_model_file_free(q2a_model_file * mf) {
    if (!mf) return;
    free(mf->filters);
    free(mf->tensors);
    free(mf->data);
    free(mf);
}

extern "C" const q2a_tensor_desc * q2a_model_file_find(const q2a_model_file * mf, const char * name) {
    for (int i = 0; i < mf->n_tensors; ++i)
        if (strcmp(mf->tensors[i].name, name) == 0) return &mf->tensors[i];
    return nullptr;
}

// ------------------------------------------------------------------------------------------------
// quantize-model (examples/common-ggml.cpp:41-244 flow)
// ------------------------------------------------------------------------------------------------
extern "C" int q2a_quantize_model(const char * in_path, const char * out_path, int qtype, int nt) {
    char err[256];
    q2a_model_file * mf = q2a_model_file_read(in_path, err, sizeof(err));
    if (!mf) { fprintf(stderr, "q2a_quantize_model: %s\n", err); return -1; }
    int ftype;
    void (*qrow)(const float *, void *, int64_t);
    switch (qtype) {
        case Q2A_TYPE_Q4_K: ftype = Q2A_FTYPE_MOSTLY_Q4_K; qrow = q2a_quantize_row_q4_K; break;
        case Q2A_TYPE_Q8_0: ftype = Q2A_FTYPE_MOSTLY_Q8_0; qrow = q2a_quantize_row_q8_0; break;
        case Q2A_TYPE_Q4_0: ftype = Q2A_FTYPE_MOSTLY_Q4_0; qrow = q2a_quantize_row_q4_0; break;
        default: q2a_model_file_free(mf); return -2;
    }
    out_file o;
    o.f = fopen(out_path, "wb");
    if (!o.f) { q2a_model_file_free(mf); return -3; }
    q2a_hparams hp = mf->hp;
    hp.ftype = ftype + 2 * Q2A_QNT_VERSION_FACTOR;   // GGML_QNT_VERSION = 2 (ggml.h:215)
    o.i32((int32_t) Q2A_FILE_MAGIC);
    o.w(&hp, sizeof(hp));
    o.i32(mf->n_mel_filt);
    o.i32(mf->n_fft_filt);
    o.w(mf->filters, (size_t) mf->n_mel_filt * mf->n_fft_filt * 4);
    o.i32(0);
    for (int ti = 0; ti < mf->n_tensors; ++ti) {
        const q2a_tensor_desc & d = mf->tensors[ti];
        const std::string name = d.name;
        bool quantize = d.n_dims == 2 && name != "embed_positions.weight" && name != "conv1.bias" && name != "conv2.bias";
        std::vector<int32_t> ne;
        for (int i = 0; i < d.n_dims; ++i) ne.push_back((int32_t) d.ne[i]);
        const uint8_t * src = mf->data + d.offset;
        if (!quantize || (d.type != Q2A_TYPE_F32 && d.type != Q2A_TYPE_F16)) {
            write_tensor_header(o, name, d.type, ne);
            o.w(src, d.nbytes);
            continue;
        }
        const int64_t K = d.ne[0], R = d.ne[1];
        std::vector<float> f32((size_t) (K * R));
        if (d.type == Q2A_TYPE_F16) {
            const uint16_t * h = (const uint16_t *) src;
            for (size_t i = 0; i < f32.size(); ++i) f32[i] = q2a_fp16_to_fp32(h[i]);
        } else {
            memcpy(f32.data(), src, f32.size() * 4);
        }
        const size_t rs = q2a_row_size(qtype, K);
        std::vector<uint8_t> q(rs * (size_t) R);
        auto work = [&](int64_t b, int64_t e) {
            for (int64_t r = b; r < e; ++r) qrow(f32.data() + r * K, q.data() + (size_t) r * rs, K);
        };
        const int T = std::max(1, nt);
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back(work, R * t / T, R * (t + 1) / T);
        for (auto & x : th) x.join();
        write_tensor_header(o, name, qtype, ne);
        o.w(q.data(), q.size());
    }
    const bool ok = o.ok;
    fclose(o.f);
    q2a_model_file_free(mf);
    return ok ? 0 : -4;
}
