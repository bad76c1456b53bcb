// q2a_oracle.c — TEST INFRASTRUCTURE ONLY. Plain-C restatement of the reference hot path
// (log-mel + Conv1d frontend + encoder blocks + pool + LN) with ggml CPU numerics.
// It is the checker for the HIP path; it is never linked into, loaded by, or called from the product.
//
// Pinning: tests/test_oracle_golden.py checks this file against vectors produced by the real reference
// (oracle/_ref/ref_harness built from /root/reference sources) and committed under tests/golden/.
//
// Numerics contract:
//   F16 GEMM   : activations -> fp16 RNE (ggml_fp32_to_fp16_row), exact products, wide accumulation
//   Q4_K GEMM  : activations -> Q8_K (quantize_row_q8_K_ref), integer sub-block dots, ggml scale formula
//   Q8_0/Q4_0  : activations -> Q8_0 (x86 AVX2 quantize_row_q8_0: id = 127/amax, round-half-even)
//   attention, softmax, LN, conv, pool, mel : F32 with double accumulation where ggml uses ggml_float
//   GELU       : fp16 LUT semantics
// Dot products here accumulate in double (ggml accumulates in f32 SIMD lanes then reduces); the
// difference is ~1e-7 relative and summation order is free under the contract.
#include "q2a_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXF(a, b) ((a) > (b) ? (a) : (b))
#define MINF(a, b) ((a) < (b) ? (a) : (b))

// ---------------------------------------------------------------- fp16 (IEEE binary16, RNE)
static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

// restated from ggml_compute_fp32_to_fp16 (ggml-impl.h) — the FP16 conversion ggml falls back to without F16C
uint16_t oracle_fp32_to_fp16(float f) {
    const float scale_to_inf = bitsf(0x77800000u);
    const float scale_to_zero = bitsf(0x08800000u);
    float base = (fabsf(f) * scale_to_inf) * scale_to_zero;
    const uint32_t w = fbits(f);
    const uint32_t shl1_w = w + w;
    const uint32_t sign = w & 0x80000000u;
    uint32_t bias = shl1_w & 0xFF000000u;
    if (bias < 0x71000000u) bias = 0x71000000u;
    base = bitsf((bias >> 1) + 0x07800000u) + base;
    const uint32_t bits = fbits(base);
    const uint32_t exp_bits = (bits >> 13) & 0x00007C00u;
    const uint32_t mantissa_bits = bits & 0x00000FFFu;
    const uint32_t nonsign = exp_bits + mantissa_bits;
    return (uint16_t) ((sign >> 16) | (shl1_w > 0xFF000000u ? 0x7E00u : nonsign));
}

float oracle_fp16_to_fp32(uint16_t h) {
    const uint32_t w = (uint32_t) h << 16;
    const uint32_t sign = w & 0x80000000u;
    const uint32_t two_w = w + w;
    const uint32_t exp_offset = 0xE0u << 23;
    const float exp_scale = bitsf(0x7800000u);
    const float normalized_value = bitsf((two_w >> 4) + exp_offset) * exp_scale;
    const uint32_t magic_mask = 126u << 23;
    const float magic_bias = 0.5f;
    const float denormalized_value = bitsf((two_w >> 17) | magic_mask) - magic_bias;
    const uint32_t denormalized_cutoff = 1u << 27;
    const uint32_t result = sign | (two_w < denormalized_cutoff ? fbits(denormalized_value) : fbits(normalized_value));
    return bitsf(result);
}

static inline float f16r(float x) { return oracle_fp16_to_fp32(oracle_fp32_to_fp16(x)); }

// ---------------------------------------------------------------- mel (qwen2-whisper.cpp:2402-2665)
#define NFFT 400
static float g_sin[NFFT], g_cos[NFFT], g_hann[NFFT];
static int g_mel_init = 0;

static void mel_init(void) {   // whisper_global_cache, qwen2-whisper.cpp:2404-2437
    if (g_mel_init) return;
    for (int i = 0; i < NFFT; i++) {
        double theta = (2 * M_PI * i) / NFFT;
        g_sin[i] = sinf(theta);
        g_cos[i] = cosf(theta);
    }
    for (int i = 0; i < NFFT; i++) g_hann[i] = 0.5 * (1.0 - cosf((2.0 * M_PI * i) / (NFFT + 0)));
    g_mel_init = 1;
}

static void dft(const float * in, int N, float * out) {   // :2443-2459
    const int step = NFFT / N;
    for (int k = 0; k < N; k++) {
        float re = 0, im = 0;
        for (int n = 0; n < N; n++) {
            int idx = (k * n * step) % NFFT;
            re += in[n] * g_cos[idx];
            im -= in[n] * g_sin[idx];
        }
        out[k * 2 + 0] = re;
        out[k * 2 + 1] = im;
    }
}

static void fft(float * in, int N, float * out) {   // :2465-2507 (radix-2 recursion down to odd N)
    if (N == 1) { out[0] = in[0]; out[1] = 0; return; }
    const int half = N / 2;
    if (N - half * 2 == 1) { dft(in, N, out); return; }
    float * even = in + N;
    for (int i = 0; i < half; ++i) even[i] = in[2 * i];
    float * even_fft = out + 2 * N;
    fft(even, half, even_fft);
    float * odd = even;
    for (int i = 0; i < half; ++i) odd[i] = in[2 * i + 1];
    float * odd_fft = even_fft + N;
    fft(odd, half, odd_fft);
    const int step = NFFT / N;
    for (int k = 0; k < half; k++) {
        int idx = k * step;
        float re = g_cos[idx], im = -g_sin[idx];
        float ro = odd_fft[2 * k + 0], io = odd_fft[2 * k + 1];
        out[2 * k + 0] = even_fft[2 * k + 0] + re * ro - im * io;
        out[2 * k + 1] = even_fft[2 * k + 1] + re * io + im * ro;
        out[2 * (k + half) + 0] = even_fft[2 * k + 0] - re * ro + im * io;
        out[2 * (k + half) + 1] = even_fft[2 * k + 1] - re * io - im * ro;
    }
}

int oracle_log_mel(const float * samples, int n_samples, const float * filters, int n_mel, int n_fft,
                   int n_threads, float * out, int cap) {
    mel_init();
    const int pad2 = NFFT / 2, pad1 = 16000 * 30;
    const int64_t np = (int64_t) n_samples + pad1 + 2 * pad2;
    float * sp = (float *) calloc((size_t) np, sizeof(float));
    memcpy(sp + pad2, samples, (size_t) n_samples * sizeof(float));
    for (int i = 0; i < pad2; ++i) sp[i] = samples[pad2 - i];   // reverse_copy(samples+1, samples+1+200)
    const int n_len = (int) ((np - NFFT) / 160);
    if (n_len > cap) { free(sp); return -1; }
    const int n_s = n_samples + pad2;   // what the workers see as n_samples (:2621)
    const int n_fft_frames = MINF(n_s / 160 + 1, n_len);
    (void) n_threads;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n_len; ++i) {
        if (i >= n_fft_frames) {
            const double c = log10(1e-10);
            for (int j = 0; j < n_mel; ++j) out[(size_t) j * n_len + i] = (float) c;
            continue;
        }
        float fin[NFFT * 2], fout[NFFT * 8];
        memset(fin, 0, sizeof(fin));
        const int off = i * 160;
        const int lim = MINF(NFFT, n_s - off);
        for (int j = 0; j < lim; j++) fin[j] = g_hann[j] * sp[off + j];
        fft(fin, NFFT, fout);
        for (int j = 0; j < n_fft; j++) fout[j] = fout[2 * j] * fout[2 * j] + fout[2 * j + 1] * fout[2 * j + 1];
        for (int j = 0; j < n_mel; j++) {
            double sum = 0.0;
            const float * f = filters + (size_t) j * n_fft;
            int k = 0;
            for (k = 0; k < n_fft - 3; k += 4)
                sum += fout[k] * f[k] + fout[k + 1] * f[k + 1] + fout[k + 2] * f[k + 2] + fout[k + 3] * f[k + 3];
            for (; k < n_fft; k++) sum += fout[k] * f[k];
            sum = log10(MAXF(sum, 1e-10));
            out[(size_t) j * n_len + i] = (float) sum;
        }
    }
    double mmax = -1e20;
    for (int64_t i = 0; i < (int64_t) n_mel * n_len; i++)
        if (out[i] > mmax) mmax = out[i];
    mmax -= 8.0;
    for (int64_t i = 0; i < (int64_t) n_mel * n_len; i++) {
        if (out[i] < mmax) out[i] = (float) mmax;
        out[i] = (float) ((out[i] + 4.0) / 4.0);
    }
    free(sp);
    return n_len;
}

// ---------------------------------------------------------------- GELU LUT (ggml.c:2541-2570, 3797-3806)
static uint16_t g_gelu[65536];
static int g_gelu_init = 0;
static void gelu_init(void) {
    if (g_gelu_init) return;
    const float GELU_COEF_A = 0.044715f;
    const float SQRT_2_OVER_PI = 0.79788456080286535587989211986876f;
    for (int i = 0; i < 65536; ++i) {
        const float x = oracle_fp16_to_fp32((uint16_t) i);
        const float g = 0.5f * x * (1.0f + tanhf(SQRT_2_OVER_PI * x * (1.0f + GELU_COEF_A * x * x)));
        g_gelu[i] = oracle_fp32_to_fp16(g);
    }
    g_gelu_init = 1;
}

float oracle_gelu(float x) {
    gelu_init();
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    return oracle_fp16_to_fp32(g_gelu[oracle_fp32_to_fp16(x)]);
}

// ---------------------------------------------------------------- activation quantizers
typedef struct { uint16_t d; int8_t qs[32]; } blk_q8_0;
typedef struct { uint16_t d; uint8_t qs[16]; } blk_q4_0;
typedef struct { uint16_t d, dmin; uint8_t scales[12]; uint8_t qs[128]; } blk_q4_K;
typedef struct { float d; int8_t qs[256]; int16_t bsums[16]; } blk_q8_K;

static inline int nearest_int(float fval) {   // ggml-quants.c:1639
    float val = fval + 12582912.f;
    int i; memcpy(&i, &val, sizeof(int));
    return (i & 0x007fffff) - 0x00400000;
}

void oracle_quantize_act_q8_K(const float * x, void * vy, int64_t k) {   // ggml-quants.c:3785-3822
    blk_q8_K * y = (blk_q8_K *) vy;
    for (int64_t i = 0; i < k / 256; i++, x += 256) {
        float max = 0, amax = 0;
        for (int j = 0; j < 256; ++j) {
            float ax = fabsf(x[j]);
            if (ax > amax) { amax = ax; max = x[j]; }
        }
        if (!amax) {
            y[i].d = 0;
            memset(y[i].qs, 0, 256);
            memset(y[i].bsums, 0, sizeof(y[i].bsums));
            continue;
        }
        const float iscale = -127.f / max;
        for (int j = 0; j < 256; ++j) {
            int v = nearest_int(iscale * x[j]);
            y[i].qs[j] = (int8_t) MINF(127, v);
        }
        for (int j = 0; j < 16; ++j) {
            int sum = 0;
            for (int ii = 0; ii < 16; ++ii) sum += y[i].qs[j * 16 + ii];
            y[i].bsums[j] = (int16_t) sum;
        }
        y[i].d = 1 / iscale;
    }
}

// x86 AVX2 quantize_row_q8_0 (ggml-quants.c:943-1000): d = amax/127 -> fp16, id = 127/amax,
// q = round-half-even(x*id) (_mm256_round_ps(_MM_ROUND_NEAREST) + cvtps)
void oracle_quantize_act_q8_0(const float * x, void * vy, int64_t k) {
    blk_q8_0 * y = (blk_q8_0 *) vy;
    for (int64_t i = 0; i < k / 32; i++, x += 32) {
        float amax = 0.f;
        for (int j = 0; j < 32; ++j) amax = MAXF(amax, fabsf(x[j]));
        const float d = amax / 127.f;
        y[i].d = oracle_fp32_to_fp16(d);
        const float id = (amax != 0.0f) ? 127.f / amax : 0.0f;
        for (int j = 0; j < 32; ++j) y[i].qs[j] = (int8_t) nearbyintf(x[j] * id);
    }
}

// ---------------------------------------------------------------- GEMMs
static inline void scale_min_k4(int j, const uint8_t * q, uint8_t * d, uint8_t * m) {   // ggml-quants.c:1898
    if (j < 4) { *d = q[j] & 63; *m = q[j + 4] & 63; }
    else {
        *d = (uint8_t) ((q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4));
        *m = (uint8_t) ((q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4));
    }
}

// Y[M][N] = X[M][K] . W[N][K]^T with ggml_compute_forward_mul_mat semantics (ggml.c:12439-12652):
// src1 (X) converted to the weight type's vec_dot_type first.
void oracle_gemm(int wtype, const void * W, const float * X, int M, int N, int K, float * Y, int n_threads) {
    (void) n_threads;
    if (wtype == 0 || wtype == 1) {
        float * xf = (float *) malloc((size_t) M * K * sizeof(float));
        float * wf = (float *) malloc((size_t) N * K * sizeof(float));
        for (int64_t i = 0; i < (int64_t) M * K; ++i) xf[i] = wtype == 1 ? f16r(X[i]) : X[i];
        for (int64_t i = 0; i < (int64_t) N * K; ++i)
            wf[i] = wtype == 1 ? oracle_fp16_to_fp32(((const uint16_t *) W)[i]) : ((const float *) W)[i];
#pragma omp parallel for schedule(static)
        for (int m = 0; m < M; ++m) {
            const float * xr = xf + (size_t) m * K;
            for (int n = 0; n < N; ++n) {
                const float * wr = wf + (size_t) n * K;
                double s = 0;
                for (int k = 0; k < K; ++k) s += (double) (xr[k] * wr[k]);
                Y[(size_t) m * N + n] = (float) s;
            }
        }
        free(xf);
        free(wf);
        return;
    }
    if (wtype == 12) {   // Q4_K x Q8_K: ggml_vec_dot_q4_K_q8_K (ggml-quants.c:7713-8279)
        const int nb = K / 256;
        blk_q8_K * xq = (blk_q8_K *) malloc((size_t) M * nb * sizeof(blk_q8_K));
        for (int m = 0; m < M; ++m) oracle_quantize_act_q8_K(X + (size_t) m * K, xq + (size_t) m * nb, K);
        const blk_q4_K * wq = (const blk_q4_K *) W;
#pragma omp parallel for schedule(static)
        for (int m = 0; m < M; ++m) {
            for (int n = 0; n < N; ++n) {
                double acc = 0;
                for (int b = 0; b < nb; ++b) {
                    const blk_q4_K * x = wq + (size_t) n * nb + b;
                    const blk_q8_K * y = xq + (size_t) m * nb + b;
                    int sumi = 0, summ = 0;
                    for (int j = 0; j < 8; ++j) {
                        uint8_t sc, mn;
                        scale_min_k4(j, x->scales, &sc, &mn);
                        const uint8_t * q = x->qs + 32 * (j / 2);
                        int dot = 0;
                        for (int l = 0; l < 32; ++l) {
                            const int w = (j & 1) ? (q[l] >> 4) : (q[l] & 0xF);
                            dot += w * y->qs[32 * j + l];
                        }
                        sumi += sc * dot;
                        summ += mn * (y->bsums[2 * j] + y->bsums[2 * j + 1]);
                    }
                    const float d = y->d * oracle_fp16_to_fp32(x->d);
                    const float dmin = y->d * oracle_fp16_to_fp32(x->dmin);
                    acc += (double) d * sumi - (double) dmin * summ;
                }
                Y[(size_t) m * N + n] = (float) acc;
            }
        }
        free(xq);
        return;
    }
    if (wtype == 8 || wtype == 2) {   // Q8_0 / Q4_0 x Q8_0 (ggml-quants.c:5518 / ggml_vec_dot_q4_0_q8_0)
        const int nb = K / 32;
        blk_q8_0 * xq = (blk_q8_0 *) malloc((size_t) M * nb * sizeof(blk_q8_0));
        for (int m = 0; m < M; ++m) oracle_quantize_act_q8_0(X + (size_t) m * K, xq + (size_t) m * nb, K);
#pragma omp parallel for schedule(static)
        for (int m = 0; m < M; ++m) {
            for (int n = 0; n < N; ++n) {
                double acc = 0;
                for (int b = 0; b < nb; ++b) {
                    const blk_q8_0 * y = xq + (size_t) m * nb + b;
                    int sumi = 0;
                    float dx;
                    if (wtype == 8) {
                        const blk_q8_0 * x = (const blk_q8_0 *) W + (size_t) n * nb + b;
                        for (int l = 0; l < 32; ++l) sumi += x->qs[l] * y->qs[l];
                        dx = oracle_fp16_to_fp32(x->d);
                    } else {
                        const blk_q4_0 * x = (const blk_q4_0 *) W + (size_t) n * nb + b;
                        for (int l = 0; l < 16; ++l) {
                            sumi += ((x->qs[l] & 0xF) - 8) * y->qs[l];
                            sumi += ((x->qs[l] >> 4) - 8) * y->qs[l + 16];
                        }
                        dx = oracle_fp16_to_fp32(x->d);
                    }
                    acc += (double) (dx * oracle_fp16_to_fp32(y->d)) * sumi;
                }
                Y[(size_t) m * N + n] = (float) acc;
            }
        }
        free(xq);
        return;
    }
    abort();
}

// ---------------------------------------------------------------- LN (ggml.c:11941-11990 + mul + add)
static void layer_norm(const float * x, float * y, int T, int D, const float * g, const float * b) {
#pragma omp parallel for schedule(static)
    for (int t = 0; t < T; ++t) {
        const float * xr = x + (size_t) t * D;
        float * yr = y + (size_t) t * D;
        double sum = 0.0;
        for (int i = 0; i < D; ++i) sum += (double) xr[i];
        const float mean = (float) (sum / D);
        double sum2 = 0.0;
        for (int i = 0; i < D; ++i) {
            float v = xr[i] - mean;
            yr[i] = v;
            sum2 += (double) (v * v);
        }
        const float variance = (float) (sum2 / D);
        const float scale = 1.0f / sqrtf(variance + 1e-5f);
        for (int i = 0; i < D; ++i) yr[i] = (yr[i] * scale) * g[i] + b[i];
    }
}

// conv1d (ggml_conv_1d ggml.c:6635-6652 with the F32 upcast of the kernel): in [IC][IW] -> out [OW][OC]
static void conv1d(const float * in, int IC, int IW, const void * w, int wtype, const float * bias, int OC,
                   int stride, float * out /*[OW][OC]*/, int OW) {
    float * wf = (float *) malloc((size_t) OC * IC * 3 * sizeof(float));
    for (int64_t i = 0; i < (int64_t) OC * IC * 3; ++i)
        wf[i] = wtype == 1 ? oracle_fp16_to_fp32(((const uint16_t *) w)[i]) : ((const float *) w)[i];
#pragma omp parallel for schedule(static)
    for (int t = 0; t < OW; ++t) {
        float col[3 * 1280 * 2];
        for (int ic = 0; ic < IC; ++ic)
            for (int k = 0; k < 3; ++k) {
                const int iw = t * stride + k - 1;
                col[ic * 3 + k] = (iw < 0 || iw >= IW) ? 0.f : in[(size_t) ic * IW + iw];
            }
        for (int oc = 0; oc < OC; ++oc) {
            const float * wr = wf + (size_t) oc * IC * 3;
            double s = 0;
            for (int j = 0; j < IC * 3; ++j) s += (double) (col[j] * wr[j]);
            out[(size_t) t * OC + oc] = oracle_gelu((float) s + bias[oc]);
        }
    }
    free(wf);
}

// ---------------------------------------------------------------- encoder (qwen2-whisper.cpp:1892-2203)
int oracle_encode(const oracle_model * m, const float * mel, float * out, oracle_dump * dump, int n_threads) {
    const int D = m->d, T = m->n_ctx, H = m->n_head, dh = D / H, F = 4 * D, TM = 2 * T;
    if (m->n_mels * 3 > 2 * 1280 * 3 || D > 2 * 1280) return -1;
    gelu_init();
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#endif
    float * c1 = (float *) malloc((size_t) TM * D * sizeof(float));
    float * c1t = (float *) malloc((size_t) TM * D * sizeof(float));
    float * x = (float *) malloc((size_t) T * D * sizeof(float));
    // conv1 (k3 s1 p1) + bias + GELU: [TM][D]
    conv1d(mel, m->n_mels, TM, m->conv1_w, m->conv_type, m->conv1_b, D, 1, c1, TM);
    // conv2 takes [IC=D][IW=TM]: transpose
    for (int t = 0; t < TM; ++t)
        for (int c = 0; c < D; ++c) c1t[(size_t) c * TM + t] = c1[(size_t) t * D + c];
    conv1d(c1t, D, TM, m->conv2_w, m->conv_type, m->conv2_b, D, 2, x, T);
    // x = e_pe + cont(transpose(embd_conv))   (:2005)
    for (int64_t i = 0; i < (int64_t) T * D; ++i) x[i] = m->pe[i] + x[i];
    if (dump && dump->conv_out) memcpy(dump->conv_out, x, (size_t) T * D * 4);
    free(c1);
    free(c1t);

    float * cur = (float *) malloc((size_t) T * D * sizeof(float));
    float * q = (float *) malloc((size_t) T * D * sizeof(float));
    float * k = (float *) malloc((size_t) T * D * sizeof(float));
    float * v = (float *) malloc((size_t) T * D * sizeof(float));
    float * att = (float *) malloc((size_t) T * D * sizeof(float));
    float * tmp = (float *) malloc((size_t) T * D * sizeof(float));
    float * h = (float *) malloc((size_t) T * F * sizeof(float));
    const float kq_scale = 1.0f / sqrtf((float) dh);

    for (int il = 0; il < m->n_layer; ++il) {
        const int d0 = dump && il == 0;
        layer_norm(x, cur, T, D, m->ln1_w[il], m->ln1_b[il]);
        if (d0 && dump->ln1) memcpy(dump->ln1, cur, (size_t) T * D * 4);
        oracle_gemm(m->wtype, m->q_w[il], cur, T, D, D, q, n_threads);
        oracle_gemm(m->wtype, m->k_w[il], cur, T, D, D, k, n_threads);
        oracle_gemm(m->wtype, m->v_w[il], cur, T, D, D, v, n_threads);
        for (int t = 0; t < T; ++t)
            for (int c = 0; c < D; ++c) {
                q[(size_t) t * D + c] = (q[(size_t) t * D + c] + m->q_b[il][c]) * kq_scale;
                v[(size_t) t * D + c] = v[(size_t) t * D + c] + m->v_b[il][c];
            }
        if (d0 && dump->q) memcpy(dump->q, q, (size_t) T * D * 4);
        if (d0 && dump->k) memcpy(dump->k, k, (size_t) T * D * 4);
        if (d0 && dump->v) memcpy(dump->v, v, (size_t) T * D * 4);
        // attention per head: KQ = K.Q^T, softmax over keys (ggml.c:13854-13950), KQV = P.V
#pragma omp parallel
        {
            float * srow = (float *) malloc((size_t) T * sizeof(float));
#pragma omp for schedule(static) collapse(2)
            for (int hh = 0; hh < H; ++hh) {
                for (int i = 0; i < T; ++i) {
                    const float * qi = q + (size_t) i * D + hh * dh;
                    float mx = -INFINITY;
                    for (int j = 0; j < T; ++j) {
                        const float * kj = k + (size_t) j * D + hh * dh;
                        double s = 0;
                        for (int d = 0; d < dh; ++d) s += (double) (kj[d] * qi[d]);
                        srow[j] = (float) s;
                        if (srow[j] > mx) mx = srow[j];
                    }
                    double sum = 0;
                    for (int j = 0; j < T; ++j) {
                        srow[j] = expf(srow[j] - mx);
                        sum += (double) srow[j];
                    }
                    const float inv = (float) (1.0 / sum);
                    for (int j = 0; j < T; ++j) srow[j] *= inv;
                    for (int d = 0; d < dh; ++d) {
                        double o = 0;
                        for (int j = 0; j < T; ++j) o += (double) (v[(size_t) j * D + hh * dh + d] * srow[j]);
                        att[(size_t) i * D + hh * dh + d] = (float) o;
                    }
                }
            }
            free(srow);
        }
        if (d0 && dump->attn) memcpy(dump->attn, att, (size_t) T * D * 4);
        oracle_gemm(m->wtype, m->o_w[il], att, T, D, D, tmp, n_threads);
        for (int t = 0; t < T; ++t)
            for (int c = 0; c < D; ++c) {
                const size_t i = (size_t) t * D + c;
                x[i] = (tmp[i] + m->o_b[il][c]) + x[i];
            }
        if (d0 && dump->x1) memcpy(dump->x1, x, (size_t) T * D * 4);
        layer_norm(x, cur, T, D, m->ln2_w[il], m->ln2_b[il]);
        oracle_gemm(m->wtype, m->fc1_w[il], cur, T, F, D, h, n_threads);
        for (int t = 0; t < T; ++t)
            for (int c = 0; c < F; ++c) {
                const size_t i = (size_t) t * F + c;
                h[i] = oracle_gelu(h[i] + m->fc1_b[il][c]);
            }
        if (d0 && dump->gelu) memcpy(dump->gelu, h, (size_t) T * F * 4);
        oracle_gemm(m->wtype, m->fc2_w[il], h, T, D, F, tmp, n_threads);
        for (int t = 0; t < T; ++t)
            for (int c = 0; c < D; ++c) {
                const size_t i = (size_t) t * D + c;
                x[i] = (tmp[i] + m->fc2_b[il][c]) + x[i];
            }
        if (d0 && dump->x2) memcpy(dump->x2, x, (size_t) T * D * 4);
    }
    // AvgPool1d(2,2) over time (ggml.c:15077-15125) then LN (:2157-2181)
    const int TO = T / 2;
    for (int t = 0; t < TO; ++t)
        for (int c = 0; c < D; ++c) {
            float s = 0;
            s += x[(size_t) (2 * t) * D + c];
            s += x[(size_t) (2 * t + 1) * D + c];
            tmp[(size_t) t * D + c] = s / 2;
        }
    layer_norm(tmp, out, TO, D, m->ln_post_w, m->ln_post_b);
    free(cur); free(q); free(k); free(v); free(att); free(tmp); free(h); free(x);
    return 0;
}
