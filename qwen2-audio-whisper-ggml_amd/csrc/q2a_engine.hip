// q2a_engine.hip — host orchestration of the MI355X encoder path behind the C ABI (include/q2a_encoder.h).
//
// Replaces whisper_full -> whisper_encoder_output_with_state (src/qwen2-whisper.cpp:2341-2383):
// log_mel_spectrogram (:2575) + whisper_encode_qwen2_internal (:2241) with its conv graph (:1892) and encoder
// graph (:1954), for a BATCH of independent clips in one pass. No ggml graph build / sched split / allocator at
// run time: the model is packed once into a device blob and every intermediate lives in a workspace reserved
// for the batch size, so a batch is ~11 launches per layer on one stream (capturable into a hipGraph).
#include "q2a_encoder.h"
#include "q2a_format.h"
#include "q2a_internal.h"

#include <algorithm>
#include <cmath>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_err;

void set_err(const char * fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}

#define HIP_TRY(x)                                                                        \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            set_err("%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            return Q2A_ERR_HIP;                                                           \
        }                                                                                 \
    } while (0)

// ------------------------------------------------------------------------------------------------
// packed device blob: 16 KiB self-describing header + 256-B aligned sections
// ------------------------------------------------------------------------------------------------
constexpr uint32_t BLOB_MAGIC = 0x42413251u;   // "Q2AB"
// version 3: the Q4_K gamma array holds -(dmin/dx) (stored negated); a version-2 blob (positive gamma) is refused
constexpr uint32_t BLOB_VERSION = 5;   // 4: conv1 taps against the three-part mel operand; 5: compact transport form
constexpr int MAX_LAYERS = 64;
constexpr size_t HEADER_BYTES = 32768;

enum { G_CONV1_W, G_CONV1_B, G_CONV2_W, G_CONV2_B, G_PE, G_LNP_W, G_LNP_B, G_FILT, G_TAB, G_GELU, G_GELU_C, G_COUNT };
// per-matrix arrays: W (fp16 [N][K]); block-major DX, DMIN, BETA = DX_{b-1}/DX_b, GAMMA = DMIN_b/DX_b (f32 [nblk][N]),
// WEXT (fp16 [nblk][N][16])
enum { A_W, A_DX, A_DMIN, A_WEXT, A_BETA, A_GAMMA, A_COUNT };
enum { L_BQKV, L_BO, L_B1, L_B2, L_LN1W, L_LN1B, L_LN2W, L_LN2B, L_MAT0, L_COUNT = L_MAT0 + 4 * A_COUNT };

struct blob_header {
    uint32_t magic, version;
    q2a_hparams hp;
    int32_t wtype, blk, n_bins, act;   // act: Q2A_ACT_REFERENCE (0) or Q2A_ACT_BF16 (1)
    int32_t compact;                   // 1: the transport form (compact_of below); 0: the device layout
    uint64_t total;                    // bytes of the device layout (goff / loff address it)
    uint64_t goff[G_COUNT];
    uint64_t loff[MAX_LAYERS][L_COUNT];
};
static_assert(sizeof(blob_header) <= HEADER_BYTES, "header too large");

struct dims {
    int T, D, H, L, M, F, TM, TO;
};
dims dims_of(const q2a_hparams & hp) {
    dims d;
    d.T = hp.n_audio_ctx; d.D = hp.n_audio_state; d.H = hp.n_audio_head; d.L = hp.n_audio_layer; d.M = hp.n_mels;
    d.F = 4 * d.D; d.TM = 2 * d.T; d.TO = d.T / 2;
    return d;
}
void mat_dims(const dims & d, int which, int & N, int & K) {
    switch (which) {
        case 0: N = 3 * d.D; K = d.D; break;
        case 1: N = d.D; K = d.D; break;
        case 2: N = d.F; K = d.D; break;
        default: N = d.D; K = d.F; break;
    }
}
int blk_of(int wtype) { return wtype == Q2A_TYPE_Q4_K ? 256 : (wtype == Q2A_TYPE_Q8_0 || wtype == Q2A_TYPE_Q4_0) ? 32 : 0; }

bool plan(blob_header & h, const q2a_hparams & hp, int wtype, int act) {
    memset(&h, 0, sizeof(h));
    // bf16-activation mode: every linear weight dequantized to bf16 [N][K] (no block scales, no splits)
    h.magic = BLOB_MAGIC; h.version = BLOB_VERSION; h.hp = hp; h.wtype = wtype; h.blk = act ? 0 : blk_of(wtype); h.n_bins = 201;
    h.act = act;
    const dims d = dims_of(hp);
    if (d.L > MAX_LAYERS) return false;
    // all-F32 files: every fp16 operand is a [hi | .. ] split (SPLIT = 3 parts of K for the linears, conv1 taps of
    // 3 mel parts, conv2 taps of 2 parts), see expand_rows / pack
    const bool f32 = wtype == Q2A_TYPE_F32;
    const uint64_t kx = f32 && !act ? 3 : 1;
    uint64_t off = HEADER_BYTES;
    auto take = [&](uint64_t bytes) { const uint64_t o = off; off += (bytes + 255) & ~uint64_t(255); return o; };
    h.goff[G_CONV1_W] = take((uint64_t) d.D * 3 * 3 * d.M * 2);
    h.goff[G_CONV1_B] = take((uint64_t) d.D * 4);
    h.goff[G_CONV2_W] = take((uint64_t) d.D * 3 * (f32 ? 2 : 1) * d.D * 2);
    h.goff[G_CONV2_B] = take((uint64_t) d.D * 4);
    h.goff[G_PE] = take((uint64_t) d.T * d.D * 4);
    h.goff[G_LNP_W] = take((uint64_t) d.D * 4);
    h.goff[G_LNP_B] = take((uint64_t) d.D * 4);
    h.goff[G_FILT] = take((uint64_t) d.M * 201 * 4);
    h.goff[G_TAB] = take(1200 * 4);
    h.goff[G_GELU] = take(65536 * 2);
    h.goff[G_GELU_C] = take(Q2A_GELU_C_BYTES);
    for (int l = 0; l < d.L; ++l) {
        uint64_t * lo = h.loff[l];
        lo[L_BQKV] = take((uint64_t) 3 * d.D * 4);
        lo[L_BO] = take((uint64_t) d.D * 4);
        lo[L_B1] = take((uint64_t) d.F * 4);
        lo[L_B2] = take((uint64_t) d.D * 4);
        lo[L_LN1W] = take((uint64_t) d.D * 4);
        lo[L_LN1B] = take((uint64_t) d.D * 4);
        lo[L_LN2W] = take((uint64_t) d.D * 4);
        lo[L_LN2B] = take((uint64_t) d.D * 4);
        for (int w = 0; w < 4; ++w) {
            int N, K;
            mat_dims(d, w, N, K);
            uint64_t * a = lo + L_MAT0 + w * A_COUNT;
            a[A_W] = take((uint64_t) N * K * 2 * kx);
            if (h.blk) a[A_DX] = take((uint64_t) N * (K / h.blk) * 4);
            if (h.blk == 256) {
                a[A_DMIN] = take((uint64_t) N * (K / 256) * 4);
                a[A_WEXT] = take((uint64_t) N * (K / 256) * 16 * 2);
                a[A_BETA] = take((uint64_t) N * (K / 256) * 4);
                a[A_GAMMA] = take((uint64_t) N * (K / 256) * 4);
            }
        }
    }
    h.total = off;
    return true;
}

// The compact TRANSPORT form of a blob (what rank 0 broadcasts): the header (compact = 1, goff / loff
// still describing the device layout), the small sections verbatim as two kinds of runs — the global one
// [HEADER_BYTES, loff[0][L_BQKV]) and, per layer, the biases + LayerNorm run [loff[l][L_BQKV], loff[l][L_MAT0]) — then
// every linear weight as the model file's own ggml rows (QKV: the q | k | v rows), e.g. raw block_q4_K at 144 B per
// 256 weights instead of the 2-byte sc*q expansion plus its block-scale arrays. expand_blob rebuilds the device
// layout from it on the GPU, byte for byte what pack() writes on the host.
struct compact_layout {
    uint64_t g_off, g_len;
    uint64_t l_off[MAX_LAYERS], l_len[MAX_LAYERS];
    uint64_t raw_off[MAX_LAYERS][4], raw_len[MAX_LAYERS][4];
    uint64_t total;
};
compact_layout compact_of(const blob_header & h) {
    compact_layout c;
    memset(&c, 0, sizeof(c));
    const dims d = dims_of(h.hp);
    uint64_t off = HEADER_BYTES;
    auto take = [&](uint64_t bytes) { const uint64_t o = off; off += (bytes + 255) & ~uint64_t(255); return o; };
    c.g_len = h.loff[0][L_BQKV] - HEADER_BYTES;
    c.g_off = take(c.g_len);
    for (int l = 0; l < d.L; ++l) {
        c.l_len[l] = h.loff[l][L_MAT0 + A_W] - h.loff[l][L_BQKV];
        c.l_off[l] = take(c.l_len[l]);
    }
    for (int l = 0; l < d.L; ++l)
        for (int w = 0; w < 4; ++w) {
            int N, K;
            mat_dims(d, w, N, K);
            c.raw_len[l][w] = (uint64_t) N * q2a_row_size(h.wtype, K);
            c.raw_off[l][w] = take(c.raw_len[l][w]);
        }
    c.total = off;
    return c;
}

// A header that arrives from outside the packer (a device blob, an RCCL-broadcast buffer, a caller's host copy) is
// checked before anything is derived from it: compact_of and expand_blob index fixed [MAX_LAYERS] arrays by its layer
// count and address device memory by its offsets. Magic, version, the shape rules pack() enforces, and every offset
// equal to what plan() lays out for those hparams. nullptr = valid, else the reason.
const char * header_problem(const blob_header & h) {
    if (h.magic != BLOB_MAGIC || h.version != BLOB_VERSION) return "not a q2a weight blob";
    const dims d = dims_of(h.hp);
    if (d.L <= 0 || d.L > MAX_LAYERS) return "not a q2a weight blob (layer count out of range)";
    if (d.D <= 0 || d.D % 128 || d.D != d.H * 64 || d.T <= 0 || d.T % 2 || d.M <= 0 || d.M % 4 || d.T > (1 << 20) ||
        d.M > 4096)
        return "not a q2a weight blob (unsupported shapes)";
    if ((h.compact != 0 && h.compact != 1) || (h.act != Q2A_ACT_REFERENCE && h.act != Q2A_ACT_BF16) ||
        q2a_row_size(h.wtype, d.D) == 0 || (blk_of(h.wtype) == 256 && d.D % 256))
        return "not a q2a weight blob (bad type fields)";
    blob_header p;
    if (!plan(p, h.hp, h.wtype, h.act)) return "not a q2a weight blob (layout)";
    if (p.total != h.total || p.blk != h.blk || p.n_bins != h.n_bins || memcmp(p.goff, h.goff, sizeof(p.goff)) ||
        memcmp(p.loff, h.loff, sizeof(p.loff[0]) * d.L))
        return "not a q2a weight blob (inconsistent layout)";
    return nullptr;
}

inline void scale_min_k4(int j, const uint8_t * q, uint8_t * dd, uint8_t * mm) {   // ggml-quants.c:1898
    if (j < 4) { *dd = q[j] & 63; *mm = q[j + 4] & 63; }
    else {
        *dd = (uint8_t) ((q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4));
        *mm = (uint8_t) ((q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4));
    }
}

// Expand rows [r0, r1) of a ggml weight matrix into the blob arrays (rows offset by dst_row0).
// F16: copied. Q4_K: W' = sc_j * q (exact small integers), DX = d, DMIN = dmin, WEXT = (64 m_j, m_j).
// Q8_0: W' = q, DX = d. Q4_0: W' = q - 8, DX = d.
// one ggml row -> f32 values, as ggml's dequantize_row_* computes them (ggml-quants.c: q8_0 :1734, q4_0 :1694,
// q4_K :2555-2577 with d1 = d*sc, m1 = dmin*m, y = d1*q - m1)
void dequant_row(const uint8_t * row, int wtype, int K, float * y) {
    if (wtype == Q2A_TYPE_F32) { memcpy(y, row, (size_t) K * 4); return; }
    if (wtype == Q2A_TYPE_F16) { for (int k = 0; k < K; ++k) y[k] = q2a_fp16_to_fp32(((const uint16_t *) row)[k]); return; }
    if (wtype == Q2A_TYPE_Q8_0) {
        for (int b = 0; b < K / 32; ++b) {
            const q2a_block_q8_0 * x = (const q2a_block_q8_0 *) row + b;
            const float d = q2a_fp16_to_fp32(x->d);
            for (int l = 0; l < 32; ++l) y[b * 32 + l] = x->qs[l] * d;
        }
    } else if (wtype == Q2A_TYPE_Q4_0) {
        for (int b = 0; b < K / 32; ++b) {
            const q2a_block_q4_0 * x = (const q2a_block_q4_0 *) row + b;
            const float d = q2a_fp16_to_fp32(x->d);
            for (int l = 0; l < 16; ++l) {
                y[b * 32 + l] = ((x->qs[l] & 0xF) - 8) * d;
                y[b * 32 + 16 + l] = ((x->qs[l] >> 4) - 8) * d;
            }
        }
    } else if (wtype == Q2A_TYPE_Q4_K) {
        for (int b = 0; b < K / 256; ++b) {
            const q2a_block_q4_K * x = (const q2a_block_q4_K *) row + b;
            const float d = q2a_fp16_to_fp32(x->d), dmin = q2a_fp16_to_fp32(x->dmin);
            for (int j = 0; j < 8; ++j) {
                uint8_t sc, m;
                scale_min_k4(j, x->scales, &sc, &m);
                const float d1 = d * sc, m1 = dmin * m;
                const uint8_t * q = x->qs + 32 * (j / 2);
                for (int l = 0; l < 32; ++l) y[b * 256 + 32 * j + l] = d1 * ((j & 1) ? (q[l] >> 4) : (q[l] & 0xF)) - m1;
            }
        }
    }
}

uint16_t f32_to_bf16(float f) {   // round to nearest even (finite inputs)
    uint32_t u;
    memcpy(&u, &f, 4);
    return (uint16_t) ((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

void expand_rows(const uint8_t * src, int wtype, int K, int Ntot, int r0, int r1, uint8_t * blob, const uint64_t * a, int dst_row0,
                 int act = 0) {
    uint16_t * W = (uint16_t *) (blob + a[A_W]);
    const size_t rs = q2a_row_size(wtype, K);
    std::vector<float> tmp(act ? K : 0);
    for (int r = r0; r < r1; ++r) {
        const uint8_t * row = src + (size_t) r * rs;
        const int n = dst_row0 + r;
        uint16_t * wr = W + (size_t) n * K;
        if (act) {   // bf16-activation mode: dequantized weight, RNE to bf16
            dequant_row(row, wtype, K, tmp.data());
            for (int k = 0; k < K; ++k) wr[k] = f32_to_bf16(tmp[k]);
        } else if (wtype == Q2A_TYPE_F16) {
            memcpy(wr, row, (size_t) K * 2);
        } else if (wtype == Q2A_TYPE_F32) {
            // [Wh | Wh | Wl] against activations [Ah | Al | Ah]: Ah.Wh + Al.Wh + Ah.Wl, F32-class products
            const float * x = (const float *) row;
            uint16_t * w3 = W + (size_t) n * 3 * K;
            for (int k = 0; k < K; ++k) {
                const uint16_t hi = q2a_fp32_to_fp16(x[k]);
                w3[k] = hi;
                w3[K + k] = hi;
                w3[2 * K + k] = q2a_fp32_to_fp16(x[k] - q2a_fp16_to_fp32(hi));
            }
        } else if (wtype == Q2A_TYPE_Q4_K) {
            // block-major scale arrays: [nb][Ntot] / [nb][Ntot][16] so a tile's block scales are contiguous
            const int nb = K / 256;
            float * dx = (float *) (blob + a[A_DX]);
            float * dm = (float *) (blob + a[A_DMIN]);
            float * be = (float *) (blob + a[A_BETA]);
            float * ga = (float *) (blob + a[A_GAMMA]);
            uint16_t * we = (uint16_t *) (blob + a[A_WEXT]);
            float dprev = 1.0f;
            for (int b = 0; b < nb; ++b) {
                const q2a_block_q4_K * x = (const q2a_block_q4_K *) row + b;
                // d = 0: the block's d*sc*q terms vanish; store dx = 1 with zero weights instead (same products,
                // and the block-ratio rescaling of the 8-phase kernel never divides by zero)
                const float d = q2a_fp16_to_fp32(x->d);
                const float deff = d != 0.0f ? d : 1.0f;
                dx[(size_t) b * Ntot + n] = deff;
                dm[(size_t) b * Ntot + n] = q2a_fp16_to_fp32(x->dmin);
                be[(size_t) b * Ntot + n] = dprev / deff;
                ga[(size_t) b * Ntot + n] = -(q2a_fp16_to_fp32(x->dmin) / deff);   // negated: the kernels' fma addend
                dprev = deff;
                for (int j = 0; j < 8; ++j) {
                    uint8_t sc, m;
                    scale_min_k4(j, x->scales, &sc, &m);
                    we[((size_t) b * Ntot + n) * 16 + 2 * j + 0] = q2a_fp32_to_fp16(64.0f * m);
                    we[((size_t) b * Ntot + n) * 16 + 2 * j + 1] = q2a_fp32_to_fp16((float) m);
                    const uint8_t * q = x->qs + 32 * (j / 2);
                    for (int l = 0; l < 32; ++l) {
                        const int v = (j & 1) ? (q[l] >> 4) : (q[l] & 0xF);
                        wr[b * 256 + 32 * j + l] = q2a_fp32_to_fp16(d != 0.0f ? (float) (sc * v) : 0.0f);
                    }
                }
            }
        } else if (wtype == Q2A_TYPE_Q8_0) {
            const int nb = K / 32;
            float * dx = (float *) (blob + a[A_DX]);
            for (int b = 0; b < nb; ++b) {
                const q2a_block_q8_0 * x = (const q2a_block_q8_0 *) row + b;
                dx[(size_t) b * Ntot + n] = q2a_fp16_to_fp32(x->d);
                for (int l = 0; l < 32; ++l) wr[b * 32 + l] = q2a_fp32_to_fp16((float) x->qs[l]);
            }
        } else if (wtype == Q2A_TYPE_Q4_0) {
            const int nb = K / 32;
            float * dx = (float *) (blob + a[A_DX]);
            for (int b = 0; b < nb; ++b) {
                const q2a_block_q4_0 * x = (const q2a_block_q4_0 *) row + b;
                dx[(size_t) b * Ntot + n] = q2a_fp16_to_fp32(x->d);
                for (int l = 0; l < 16; ++l) {
                    wr[b * 32 + l] = q2a_fp32_to_fp16((float) ((x->qs[l] & 0xF) - 8));
                    wr[b * 32 + 16 + l] = q2a_fp32_to_fp16((float) ((x->qs[l] >> 4) - 8));
                }
            }
        }
    }
}

int pack(const char * path, std::vector<uint8_t> & out, int act = 0, bool compact = false) {
    char err[256];
    q2a_model_file * mf = q2a_model_file_read(path, err, sizeof(err));
    if (!mf) { set_err("%s", err); return errno == ENOENT ? Q2A_ERR_IO : Q2A_ERR_FORMAT; }
    struct guard { q2a_model_file * m; ~guard() { q2a_model_file_free(m); } } gd{mf};
    const q2a_hparams & hp = mf->hp;
    const int wtype = mf->wtype;
    const dims d = dims_of(hp);
    if (d.D % 128 || d.D != d.H * 64 || d.T % 2 || d.M % 4 || (blk_of(wtype) == 256 && d.D % 256)) {
        set_err("unsupported shapes: D=%d H=%d T=%d M=%d", d.D, d.H, d.T, d.M);
        return Q2A_ERR_UNSUPPORTED;
    }
    if (mf->n_mel_filt != d.M || mf->n_fft_filt != 201) { set_err("bad mel filter shape"); return Q2A_ERR_FORMAT; }
    blob_header h;
    if (!plan(h, hp, wtype, act)) { set_err("too many layers"); return Q2A_ERR_UNSUPPORTED; }
    // the compact transport form is written directly (its size, not the device layout's: 0.38 vs 1.40 GB for Q4_K)
    compact_layout c;
    if (compact) { h.compact = 1; c = compact_of(h); }
    out.assign(compact ? c.total : h.total, 0);
    uint8_t * blob = out.data();
    memcpy(blob, &h, sizeof(h));
    // a small section's device-layout offset -> its bytes in `out` (the compact form keeps the global run and each
    // layer's bias / LayerNorm run verbatim, packed one after the other)
    auto at = [&](uint64_t off) -> uint8_t * {
        if (!compact) return blob + off;
        if (off < h.loff[0][L_BQKV]) return blob + c.g_off + (off - HEADER_BYTES);
        int l = d.L - 1;
        while (l > 0 && off < h.loff[l][L_BQKV]) --l;
        return blob + c.l_off[l] + (off - h.loff[l][L_BQKV]);
    };

    auto T = [&](const std::string & name, int type, std::initializer_list<int64_t> ne) -> const uint8_t * {
        const q2a_tensor_desc * t = q2a_model_file_find(mf, name.c_str());
        if (!t) { set_err("tensor '%s' missing from model file", name.c_str()); return nullptr; }
        if (type >= 0 && t->type != type) { set_err("tensor '%s' has type %d, expected %d", name.c_str(), t->type, type); return nullptr; }
        int i = 0;
        for (int64_t v : ne) {
            if (t->ne[i] != v) { set_err("tensor '%s' has wrong shape", name.c_str()); return nullptr; }
            ++i;
        }
        return mf->data + t->offset;
    };
    auto cpy = [&](uint64_t off, const uint8_t * src, size_t n) { memcpy(at(off), src, n); };

    // conv kernels are F16 in every file but the all-F32 one (vtype, qwen2-whisper.cpp:1542-1543)
    const bool f32 = wtype == Q2A_TYPE_F32;
    const int ctype = f32 ? Q2A_TYPE_F32 : Q2A_TYPE_F16;
    const uint8_t * c1 = T("conv1.weight", ctype, {3, d.M, d.D});
    const uint8_t * c1b = T("conv1.bias", Q2A_TYPE_F32, {1, d.D});
    const uint8_t * c2 = T("conv2.weight", ctype, {3, d.D, d.D});
    const uint8_t * c2b = T("conv2.bias", Q2A_TYPE_F32, {1, d.D});
    const uint8_t * pe = T("embed_positions.weight", Q2A_TYPE_F32, {d.D, d.T});
    const uint8_t * lnw = T("layer_norm.weight", Q2A_TYPE_F32, {d.D});
    const uint8_t * lnb = T("layer_norm.bias", Q2A_TYPE_F32, {d.D});
    if (!c1 || !c1b || !c2 || !c2b || !pe || !lnw || !lnb) return Q2A_ERR_FORMAT;
    {
        // hi / lo fp16 halves of a conv kernel element (F16 kernels: the value itself, lo = 0)
        auto hl = [&](const uint8_t * src, size_t i, uint16_t & hi, uint16_t & lo) {
            if (!f32) { hi = ((const uint16_t *) src)[i]; lo = 0; return; }
            const float x = ((const float *) src)[i];
            hi = q2a_fp32_to_fp16(x);
            lo = q2a_fp32_to_fp16(x - q2a_fp16_to_fp32(hi));
        };
        // conv1: [oc][ic][k] -> k-major taps against the mel operand rows: F16 [w | w | w] x [mel_h | mel_m | mel_l]
        // (exact); F32 [wh | wh | wl] x [mel_h | mel_l | mel_h]
        const int P1 = 3;
        uint16_t * w = (uint16_t *) at(h.goff[G_CONV1_W]);
        for (int oc = 0; oc < d.D; ++oc)
            for (int ic = 0; ic < d.M; ++ic)
                for (int k = 0; k < 3; ++k) {
                    uint16_t hi, lo;
                    hl(c1, ((size_t) oc * d.M + ic) * 3 + k, hi, lo);
                    uint16_t * t = w + (size_t) oc * 3 * P1 * d.M + (size_t) k * P1 * d.M + ic;
                    t[0] = hi;
                    t[d.M] = hi;
                    t[2 * d.M] = f32 ? lo : hi;
                }
        // conv2: k-major taps over three consecutive conv1 output rows: F16 [w]; F32 [wh | wl] x rows [y | y]
        const int P2 = f32 ? 2 : 1;
        uint16_t * w2 = (uint16_t *) at(h.goff[G_CONV2_W]);
        for (int oc = 0; oc < d.D; ++oc)
            for (int ic = 0; ic < d.D; ++ic)
                for (int k = 0; k < 3; ++k) {
                    uint16_t hi, lo;
                    hl(c2, ((size_t) oc * d.D + ic) * 3 + k, hi, lo);
                    uint16_t * t = w2 + (size_t) oc * 3 * P2 * d.D + (size_t) k * P2 * d.D + ic;
                    t[0] = hi;
                    if (f32) t[d.D] = lo;
                }
    }
    cpy(h.goff[G_CONV1_B], c1b, (size_t) d.D * 4);
    cpy(h.goff[G_CONV2_B], c2b, (size_t) d.D * 4);
    cpy(h.goff[G_PE], pe, (size_t) d.T * d.D * 4);
    cpy(h.goff[G_LNP_W], lnw, (size_t) d.D * 4);
    cpy(h.goff[G_LNP_B], lnb, (size_t) d.D * 4);
    cpy(h.goff[G_FILT], (const uint8_t *) mf->filters, (size_t) d.M * 201 * 4);
    q2a_make_mel_tables((float *) at(h.goff[G_TAB]));
    q2a_make_gelu_table((uint16_t *) at(h.goff[G_GELU]));
    {   // compact |x| <= 10 image of the table for the LDS-resident epilogue lookups: [+0 .. +10] | [-0 .. -10]
        const uint16_t * t = (const uint16_t *) at(h.goff[G_GELU]);
        uint16_t * cg = (uint16_t *) at(h.goff[G_GELU_C]);
        memset(cg, 0, Q2A_GELU_C_BYTES);
        for (int i = 0; i < Q2A_GELU_C_HALF; ++i) { cg[i] = t[i]; cg[Q2A_GELU_C_HALF + i] = t[0x8000 + i]; }
    }

    struct job { const uint8_t * src; int K, Ntot, r0, r1; const uint64_t * a; int dst0; };
    std::vector<job> jobs;
    for (int l = 0; l < d.L; ++l) {
        const std::string p = "layers." + std::to_string(l) + ".";
        const uint64_t * lo = h.loff[l];
        const uint8_t * wq = T(p + "self_attn.q_proj.weight", wtype, {d.D, d.D});
        const uint8_t * bq = T(p + "self_attn.q_proj.bias", Q2A_TYPE_F32, {d.D});
        const uint8_t * wk = T(p + "self_attn.k_proj.weight", wtype, {d.D, d.D});
        const uint8_t * wv = T(p + "self_attn.v_proj.weight", wtype, {d.D, d.D});
        const uint8_t * bv = T(p + "self_attn.v_proj.bias", Q2A_TYPE_F32, {d.D});
        const uint8_t * wo = T(p + "self_attn.out_proj.weight", wtype, {d.D, d.D});
        const uint8_t * bo = T(p + "self_attn.out_proj.bias", Q2A_TYPE_F32, {d.D});
        const uint8_t * l1w = T(p + "self_attn_layer_norm.weight", Q2A_TYPE_F32, {d.D});
        const uint8_t * l1b = T(p + "self_attn_layer_norm.bias", Q2A_TYPE_F32, {d.D});
        const uint8_t * w1 = T(p + "fc1.weight", wtype, {d.D, d.F});
        const uint8_t * b1 = T(p + "fc1.bias", Q2A_TYPE_F32, {d.F});
        const uint8_t * w2 = T(p + "fc2.weight", wtype, {d.F, d.D});
        const uint8_t * b2 = T(p + "fc2.bias", Q2A_TYPE_F32, {d.D});
        const uint8_t * l2w = T(p + "final_layer_norm.weight", Q2A_TYPE_F32, {d.D});
        const uint8_t * l2b = T(p + "final_layer_norm.bias", Q2A_TYPE_F32, {d.D});
        if (!wq || !bq || !wk || !wv || !bv || !wo || !bo || !l1w || !l1b || !w1 || !b1 || !w2 || !b2 || !l2w || !l2b)
            return Q2A_ERR_FORMAT;
        float * bqkv = (float *) at(lo[L_BQKV]);
        memcpy(bqkv, bq, (size_t) d.D * 4);                 // q bias; k has no bias (qwen2-whisper.cpp:2037)
        memcpy(bqkv + 2 * d.D, bv, (size_t) d.D * 4);
        cpy(lo[L_BO], bo, (size_t) d.D * 4);
        cpy(lo[L_B1], b1, (size_t) d.F * 4);
        cpy(lo[L_B2], b2, (size_t) d.D * 4);
        cpy(lo[L_LN1W], l1w, (size_t) d.D * 4);
        cpy(lo[L_LN1B], l1b, (size_t) d.D * 4);
        cpy(lo[L_LN2W], l2w, (size_t) d.D * 4);
        cpy(lo[L_LN2B], l2b, (size_t) d.D * 4);
        const uint64_t * a0 = lo + L_MAT0;
        jobs.push_back({wq, d.D, 3 * d.D, 0, d.D, a0, 0});
        jobs.push_back({wk, d.D, 3 * d.D, 0, d.D, a0, d.D});
        jobs.push_back({wv, d.D, 3 * d.D, 0, d.D, a0, 2 * d.D});
        jobs.push_back({wo, d.D, d.D, 0, d.D, lo + L_MAT0 + A_COUNT, 0});
        jobs.push_back({w1, d.D, d.F, 0, d.F, lo + L_MAT0 + 2 * A_COUNT, 0});
        jobs.push_back({w2, d.F, d.D, 0, d.D, lo + L_MAT0 + 3 * A_COUNT, 0});
    }
    if (compact) {   // the transport form: small sections written above, linear weights as the file's ggml rows
        for (int l = 0; l < d.L; ++l)
            for (int w = 0; w < 4; ++w) {   // jobs[6l..6l+5] = q, k, v, o, fc1, fc2
                const int j0 = w == 0 ? 0 : w + 2, nj = w == 0 ? 3 : 1;
                uint64_t o = c.raw_off[l][w];
                for (int q = 0; q < nj; ++q) {
                    const job & jb = jobs[6 * l + j0 + q];
                    const size_t n = (size_t) (jb.r1 - jb.r0) * q2a_row_size(wtype, jb.K);
                    memcpy(blob + o, jb.src, n);
                    o += n;
                }
            }
        return Q2A_OK;
    }
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t]() {
            for (const job & j : jobs) {
                const int n = j.r1 - j.r0;
                expand_rows(j.src, wtype, j.K, j.Ntot, j.r0 + n * t / nt, j.r0 + n * (t + 1) / nt, blob, j.a, j.dst0, act);
            }
        });
    for (auto & x : th) x.join();
    return Q2A_OK;
}

}  // namespace

// One weight matrix on its own (the ggml-backend plugin's MUL_MAT weights): same arrays as a blob matrix,
// laid out in one allocation whose offsets go to off[A_W..A_GAMMA] (0 = absent).
uint64_t q2a_pack_layout(int wtype, int N, int K, uint64_t off[6]) {
    const int blk = blk_of(wtype);
    if ((wtype != Q2A_TYPE_F16 && !blk) || (blk && K % blk) || N <= 0 || K <= 0) return 0;
    uint64_t o = 0;
    auto take = [&](uint64_t bytes) { const uint64_t r = o; o += (bytes + 255) & ~uint64_t(255); return r; };
    for (int i = 0; i < A_COUNT; ++i) off[i] = 0;
    off[A_W] = take((uint64_t) N * K * 2);
    if (blk) off[A_DX] = take((uint64_t) N * (K / blk) * 4);
    if (blk == 256) {
        off[A_DMIN] = take((uint64_t) N * (K / 256) * 4);
        off[A_WEXT] = take((uint64_t) N * (K / 256) * 16 * 2);
        off[A_BETA] = take((uint64_t) N * (K / 256) * 4);
        off[A_GAMMA] = take((uint64_t) N * (K / 256) * 4);
    }
    return o;
}

int q2a_pack_linear(const uint8_t * raw, int wtype, int N, int K, std::vector<uint8_t> & out, uint64_t off[6]) {
    const uint64_t o = q2a_pack_layout(wtype, N, K, off);
    if (!o) return Q2A_ERR_UNSUPPORTED;
    out.assign(o, 0);
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t]() { expand_rows(raw, wtype, K, N, (int) ((int64_t) N * t / nt), (int) ((int64_t) N * (t + 1) / nt), out.data(), off, 0); });
    for (auto & x : th) x.join();
    return Q2A_OK;
}

namespace {

__global__ void k_split_hilo(const float * x, q2a_half * hi, q2a_half * lo, int64_t n, float scale) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = x[i] * scale;
    asm volatile("" : "+v"(v));   // rounded to f32 before the split, as the QKV epilogue (no one-step fp16 rounding)
    const _Float16 h = (_Float16) v;
    hi[i] = h;
    lo[i] = (_Float16) (v - (float) h);
}

__global__ void k_to_half(const float * x, q2a_half * y, int64_t n) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = (_Float16) x[i];
}

__global__ void k_to_bf16(const float * x, q2a_half * y, int64_t n) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = __builtin_bit_cast(_Float16, (__bf16) x[i]);
}

// F32-weight activation operand: x [M][K] f32 -> [hi | lo | hi] rows of 3K fp16
__global__ void k_split3(const float * x, q2a_half * y, int K, int64_t n) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t m = i / K;
    const int k = (int) (i - m * K);
    const float v = x[i];
    const _Float16 h = (_Float16) v;
    q2a_half * o = y + m * 3 * K + k;
    o[0] = h;
    o[K] = (_Float16) (v - (float) h);
    o[2 * K] = h;
}

// ---- compact blob -> device layout (expand_rows on the GPU: every value bit-identical to the host pack) ----
__device__ __forceinline__ float h2f(uint16_t u) { return (float) __builtin_bit_cast(_Float16, u); }
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16) f); }   // RNE
__device__ __forceinline__ uint16_t f2bf(float f) {   // RNE on the bits, as f32_to_bf16 (finite inputs)
    const uint32_t u = __builtin_bit_cast(uint32_t, f);
    return (uint16_t) ((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ void scale_min_k4_d(int j, const uint8_t * q, int & dd, int & mm) {   // ggml-quants.c:1898
    if (j < 4) { dd = q[j] & 63; mm = q[j + 4] & 63; }
    else { dd = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4); mm = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4); }
}

struct expand_args {
    const uint8_t * raw;    // ggml rows [nrows][row_size]
    uint8_t * blob;         // device layout
    uint64_t a[A_COUNT];    // the matrix's array offsets in the device layout
    int wtype, act, K, Ntot, kx;
};

// one workgroup = 256 consecutive weights of one row (blockIdx.x = row, blockIdx.y = 256-chunk of K); the float
// operations are expand_rows' / dequant_row's, uncontracted, so every byte equals the host pack
__global__ __launch_bounds__(256) void k_expand_rows(const expand_args p) {
#pragma clang fp contract(off)
    const int n = blockIdx.x, t = threadIdx.x, k = blockIdx.y * 256 + t;
    const size_t rs = p.wtype == Q2A_TYPE_Q4_K ? (size_t) p.K / 256 * 144 : p.wtype == Q2A_TYPE_Q8_0 ? (size_t) p.K / 32 * 34
                    : p.wtype == Q2A_TYPE_Q4_0 ? (size_t) p.K / 32 * 18 : p.wtype == Q2A_TYPE_F16 ? (size_t) p.K * 2 : (size_t) p.K * 4;
    const uint8_t * row = p.raw + (size_t) n * rs;
    uint16_t * W = (uint16_t *) (p.blob + p.a[A_W]);
    if (k >= p.K) return;
    float val = 0.0f;   // dequantized value (bf16 mode)
    if (p.wtype == Q2A_TYPE_Q4_K) {
        const int b = k / 256, j = (k % 256) / 32, l = k % 32;
        const q2a_block_q4_K * x = (const q2a_block_q4_K *) row + b;
        int sc, m;
        scale_min_k4_d(j, x->scales, sc, m);
        const int v = (j & 1) ? (x->qs[32 * (j / 2) + l] >> 4) : (x->qs[32 * (j / 2) + l] & 0xF);
        const float d = h2f(x->d), dmin = h2f(x->dmin);
        if (p.act) {
            const float d1 = d * (float) sc, m1 = dmin * (float) m;
            val = d1 * (float) v - m1;
        } else {
            W[(size_t) n * p.K + k] = d != 0.0f ? f2h((float) (sc * v)) : (uint16_t) 0;
            const size_t bi = (size_t) b * p.Ntot + n;
            const float deff = d != 0.0f ? d : 1.0f;
            if (t == 0) {
                float dprev = 1.0f;
                if (b > 0) { const float dp = h2f(((const q2a_block_q4_K *) row + b - 1)->d); dprev = dp != 0.0f ? dp : 1.0f; }
                ((float *) (p.blob + p.a[A_DX]))[bi] = deff;
                ((float *) (p.blob + p.a[A_DMIN]))[bi] = dmin;
                ((float *) (p.blob + p.a[A_BETA]))[bi] = dprev / deff;
                ((float *) (p.blob + p.a[A_GAMMA]))[bi] = -(dmin / deff);
            }
            if (t < 16) {
                int sj, mj;
                scale_min_k4_d(t / 2, x->scales, sj, mj);
                ((uint16_t *) (p.blob + p.a[A_WEXT]))[bi * 16 + t] = f2h((t & 1) ? (float) mj : 64.0f * (float) mj);
            }
            return;
        }
    } else if (p.wtype == Q2A_TYPE_Q8_0) {
        const q2a_block_q8_0 * x = (const q2a_block_q8_0 *) row + k / 32;
        const float d = h2f(x->d);
        if (p.act) val = x->qs[k % 32] * d;
        else {
            W[(size_t) n * p.K + k] = f2h((float) x->qs[k % 32]);
            if (k % 32 == 0) ((float *) (p.blob + p.a[A_DX]))[(size_t) (k / 32) * p.Ntot + n] = d;
            return;
        }
    } else if (p.wtype == Q2A_TYPE_Q4_0) {
        const q2a_block_q4_0 * x = (const q2a_block_q4_0 *) row + k / 32;
        const int l = k % 32, q = (l < 16 ? (x->qs[l] & 0xF) : (x->qs[l - 16] >> 4)) - 8;
        const float d = h2f(x->d);
        if (p.act) val = q * d;
        else {
            W[(size_t) n * p.K + k] = f2h((float) q);
            if (l == 0) ((float *) (p.blob + p.a[A_DX]))[(size_t) (k / 32) * p.Ntot + n] = d;
            return;
        }
    } else if (p.wtype == Q2A_TYPE_F16) {
        const uint16_t u = ((const uint16_t *) row)[k];
        if (p.act) val = h2f(u);
        else { W[(size_t) n * p.K + k] = u; return; }
    } else {   // F32
        const float x = ((const float *) row)[k];
        if (p.act) val = x;
        else {   // [Wh | Wh | Wl]
            uint16_t * w3 = W + (size_t) n * 3 * p.K;
            const uint16_t hi = f2h(x);
            w3[k] = hi;
            w3[p.K + k] = hi;
            w3[2 * p.K + k] = f2h(x - h2f(hi));
            return;
        }
    }
    W[(size_t) n * p.K + k] = f2bf(val);
}

// device layout of `h` (compact = 1) from the compact blob `cb` (both on the current device); `out` holds h.total bytes
int expand_blob(const uint8_t * cb, const blob_header & h, uint8_t * out, hipStream_t s) {
    const compact_layout c = compact_of(h);
    const dims d = dims_of(h.hp);
    std::vector<uint8_t> head(HEADER_BYTES, 0);
    // on every return (errors included) the stream drains before `head`, which an async copy may still read, is freed
    struct drain { hipStream_t s; ~drain() { (void) hipStreamSynchronize(s); } } dr{s};
    blob_header hx = h;
    hx.compact = 0;
    memcpy(head.data(), &hx, sizeof(hx));
    HIP_TRY(hipMemsetAsync(out, 0, h.total, s));
    HIP_TRY(hipMemcpyAsync(out, head.data(), HEADER_BYTES, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(out + HEADER_BYTES, cb + c.g_off, c.g_len, hipMemcpyDeviceToDevice, s));
    const int kx = h.wtype == Q2A_TYPE_F32 && !h.act ? 3 : 1;
    for (int l = 0; l < d.L; ++l) {
        HIP_TRY(hipMemcpyAsync(out + h.loff[l][L_BQKV], cb + c.l_off[l], c.l_len[l], hipMemcpyDeviceToDevice, s));
        for (int w = 0; w < 4; ++w) {
            int N, K;
            mat_dims(d, w, N, K);
            expand_args a;
            a.raw = cb + c.raw_off[l][w];
            a.blob = out;
            for (int i = 0; i < A_COUNT; ++i) a.a[i] = h.loff[l][L_MAT0 + w * A_COUNT + i];
            a.wtype = h.wtype; a.act = h.act; a.K = K; a.Ntot = N; a.kx = kx;
            hipLaunchKernelGGL(k_expand_rows, dim3((unsigned) N, (unsigned) ((K + 255) / 256)), dim3(256), 0, s, a);
            HIP_TRY(hipGetLastError());
        }
    }
    HIP_TRY(hipStreamSynchronize(s));   // (the header's host staging must outlive its copy)
    return Q2A_OK;
}

hipError_t launch_split3(const float * x, q2a_half * y, int K, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_split3, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, x, y, K, n);
    return hipGetLastError();
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// engine
// ------------------------------------------------------------------------------------------------
struct q2a_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    blob_header h;
    dims d;
    int wtype = 0, blk = 0;
    bool f32 = false;        // all-F32 model file: fp16 hi/lo split operands, GEMM K tripled (kx = 3)
    int kx = 1;
    bool bf16 = false;       // bf16-activation mode (Q2A_ACT_BF16): bf16 weights and inter-op activations
    int gblk = 0;            // the GEMM launcher's blk: blk, or Q2A_BLK_BF16
    uint8_t * blob = nullptr;
    bool own_blob = false;
    int64_t blob_size = 0;

    // workspace (capacity)
    int cap_clips = 0;
    int64_t cap_samples = 0;
    void * ws = nullptr;
    size_t ws_bytes = 0;
    // host API (q2a_encode_host*): a copy stream and two sets of pinned + device staging buffers, so the PCIe copies
    // of one chunk of clips run beside the encode of the neighbouring chunk (host_pipe)
    struct host_buf {
        float * pin_in = nullptr; float * pin_out = nullptr; float * d_in = nullptr; float * d_out = nullptr;
        size_t in_cap = 0, out_cap = 0;   // floats
        hipEvent_t h2d = nullptr, comp = nullptr, d2h = nullptr;
    };
    hipStream_t copy_stream = nullptr;
    host_buf hb[2];
    float * out_stage = nullptr;     // unused (outputs are written straight to the user buffer)
    int32_t * meta = nullptr;        // device: nsamp | seek | clip_ok | clip_max
    int32_t * meta_host = nullptr;   // pinned
    hipEvent_t meta_evt = nullptr;   // last async upload out of meta_host (host rewrites wait on it)
    float * mel = nullptr;
    q2a_half * xc1 = nullptr;
    q2a_half * y1 = nullptr;
    float * X = nullptr;
    q2a_half * actD = nullptr;
    q2a_half * actF = nullptr;
    float * dyD = nullptr;
    float * dyF = nullptr;
    q2a_half * aextD = nullptr;
    q2a_half * aextF = nullptr;
    q2a_half *qh = nullptr, *ql = nullptr, *kh = nullptr, *kl = nullptr, *vt = nullptr;
    q2a_half * vtl = nullptr;        // V^T lo image, when the attention build reads one (q2a_attention_wants_vlo)
    float * attF = nullptr;
    float * hF = nullptr;
    float * part = nullptr;          // split-K partials of the small-tile residual GEMMs (NULL: big batches)
    int2 * frange = nullptr;         // per mel filter: non-zero bin-group range (computed once from the blob)
    int TP = 0;
    int dy_ld = 0;
    bool force_encode = false;   // encode windows with under 1 s of audio too (whisper_full with duration_ms set)
    // Q4_K fc1 -> fc2 operand path (q2a_test_fc1_path; the three produce identical Q8_K codes):
    //   0 (default) fc1 writes its fp16 pre-activation, the Q8_K quantizer applies the GELU table on the way
    //   1 GELU in the fc1 epilogue, then the fp16-input quantizer
    //   2 GELU + Q8_K quantization fused into the fc1 epilogue (8-phase tiles only)
    int fc1_path = 0;
    // q2a_test_block_taps: device buffers receiving the GEMM A operands of one block (LN1 -> QKV, attention -> O,
    // LN2 -> fc1, GELU -> fc2) as they were fed to the MFMA, for the per-layer divergence trace (NULL: off)
    void * taps[4] = {nullptr, nullptr, nullptr, nullptr};

    // optional per-kernel-class timing with HIP events on the launch stream (q2a_profile_*)
    bool prof = false;
    struct rec { int cls; hipEvent_t a, b; };
    std::vector<rec> pending;
    std::vector<hipEvent_t> pool;
    unsigned prof_mask = ~0u;        // classes timed when prof is on (bit = Q2A_PROF_*)
    double prof_ms[Q2A_PROF_CLASSES] = {};
    int64_t prof_n[Q2A_PROF_CLASSES] = {};

    template <class P> P g(int i) const { return (P) (blob + h.goff[i]); }
    template <class P> P lv(int l, int i) const { return (P) (blob + h.loff[l][i]); }
    const uint64_t * mat(int l, int w) const { return h.loff[l] + L_MAT0 + w * A_COUNT; }
};

namespace {

// A NULL `stream` argument of the device-pointer entry points (q2a_encode_device*, q2a_test_*, q2a_projector_apply)
// means the caller's legacy default stream (stream 0, torch's default stream): the work is issued ON it, so it starts
// after everything already queued there and everything queued there afterwards starts after it; inputs written and
// outputs read on stream 0 need no extra synchronisation. (Round 5 ran it on the handle's own stream between two
// cross-stream events: 0.2 ms per encode at one clip, diag/null_stream_ab.py, profiles/r06e_null_stream.jsonl.)
inline hipStream_t call_stream(const void * stream) { return (hipStream_t) stream; }

int engine_init(q2a_engine * e, int device) {
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) { set_err("device %d not available (%d devices)", device, n); return Q2A_ERR_HIP; }
    e->device = device;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&e->meta_evt, hipEventDisableTiming));
    return Q2A_OK;
}

int engine_adopt_header(q2a_engine * e) {
    if (const char * why = header_problem(e->h)) { set_err("%s", why); return Q2A_ERR_FORMAT; }
    e->d = dims_of(e->h.hp);
    e->wtype = e->h.wtype;
    e->blk = e->h.blk;
    e->f32 = e->wtype == Q2A_TYPE_F32;
    e->bf16 = e->h.act == Q2A_ACT_BF16;
    e->kx = e->f32 && !e->bf16 ? 3 : 1;
    e->gblk = e->bf16 ? Q2A_BLK_BF16 : e->blk;
    e->TP = ((e->d.T + 63) / 64) * 64;
    return Q2A_OK;
}

void free_ws(q2a_engine * e) {
    if (e->ws) (void) hipFree(e->ws);
    if (e->meta_host) (void) hipHostFree(e->meta_host);
    e->ws = nullptr; e->meta_host = nullptr;
    e->cap_clips = 0; e->ws_bytes = 0;
}

void free_host_bufs(q2a_engine * e) {
    if (e->copy_stream) (void) hipStreamSynchronize(e->copy_stream);
    for (auto & b : e->hb) {
        if (b.pin_in) (void) hipHostFree(b.pin_in);
        if (b.pin_out) (void) hipHostFree(b.pin_out);
        if (b.d_in) (void) hipFree(b.d_in);
        if (b.d_out) (void) hipFree(b.d_out);
        for (hipEvent_t ev : {b.h2d, b.comp, b.d2h}) if (ev) (void) hipEventDestroy(ev);
        b = q2a_engine::host_buf{};
    }
    if (e->copy_stream) (void) hipStreamDestroy(e->copy_stream);
    e->copy_stream = nullptr;
}

// staging for host-API chunks of up to `clips` clips of `maxn` samples (grows; never shrinks)
int ensure_host_bufs(q2a_engine * e, int clips, int64_t maxn) {
    if (!e->copy_stream) HIP_TRY(hipStreamCreateWithFlags(&e->copy_stream, hipStreamNonBlocking));
    const size_t in = (size_t) clips * maxn, out = (size_t) clips * e->d.TO * e->d.D;
    for (auto & b : e->hb) {
        if (!b.h2d) {
            HIP_TRY(hipEventCreateWithFlags(&b.h2d, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&b.comp, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&b.d2h, hipEventDisableTiming));
        }
        if (in > b.in_cap || out > b.out_cap) {
            HIP_TRY(hipStreamSynchronize(e->copy_stream));
            HIP_TRY(hipStreamSynchronize(e->stream));
        }
        if (in > b.in_cap) {
            if (b.pin_in) (void) hipHostFree(b.pin_in);
            if (b.d_in) (void) hipFree(b.d_in);
            b.pin_in = nullptr; b.d_in = nullptr; b.in_cap = 0;
            HIP_TRY(hipHostMalloc((void **) &b.pin_in, in * 4, hipHostMallocDefault));
            HIP_TRY(hipMalloc((void **) &b.d_in, in * 4));
            b.in_cap = in;
        }
        if (out > b.out_cap) {
            if (b.pin_out) (void) hipHostFree(b.pin_out);
            if (b.d_out) (void) hipFree(b.d_out);
            b.pin_out = nullptr; b.d_out = nullptr; b.out_cap = 0;
            HIP_TRY(hipHostMalloc((void **) &b.pin_out, out * 4, hipHostMallocDefault));
            HIP_TRY(hipMalloc((void **) &b.d_out, out * 4));
            b.out_cap = out;
        }
    }
    return Q2A_OK;
}

int reserve(q2a_engine * e, int B) {
    if (B <= e->cap_clips) return Q2A_OK;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipDeviceSynchronize());   // earlier calls may have run on any caller stream (or stream 0)
    if (e->ws) { (void) hipFree(e->ws); e->ws = nullptr; }
    if (e->meta_host) { (void) hipHostFree(e->meta_host); e->meta_host = nullptr; }
    const dims & d = e->d;
    const int64_t BT = (int64_t) B * d.T;
    const bool quant = e->blk != 0;
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~size_t(255); return o; };
    const size_t o_meta = take((size_t) B * 4 * 4);
    const size_t o_mel = take((size_t) B * d.M * d.TM * 4);
    const size_t o_xc1 = take((size_t) B * (d.TM + 2) * 3 * d.M * 2);
    const size_t o_y1 = take((size_t) B * (d.TM + 1) * d.D * 2 * (e->f32 ? 2 : 1));
    const size_t o_X = take((size_t) BT * d.D * 4);
    const size_t o_actD = take((size_t) BT * d.D * 2 * e->kx);
    const size_t o_actF = take((size_t) BT * d.F * 2 * e->kx);
    const size_t o_qh = take((size_t) BT * d.D * 2);
    const size_t o_ql = take((size_t) BT * d.D * 2);
    const size_t o_kh = take((size_t) BT * d.D * 2);
    const size_t o_kl = take((size_t) BT * d.D * 2);
    const size_t o_vt = take((size_t) B * d.H * 64 * e->TP * 2);
    const bool vlo = !e->bf16 && q2a_attention_wants_vlo();
    const size_t o_vtl = vlo ? take((size_t) B * d.H * 64 * e->TP * 2) : 0;
    size_t o_dyD = 0, o_dyF = 0, o_aD = 0, o_aF = 0, o_att = 0, o_hF = 0, o_part = 0;
    // split-K partials of the small-tile residual GEMMs (O-proj, fc2): up to 4 x [rows][D] f32. Sized for every
    // row count that takes the small-tile path (M <= 26 112 at D = 1280), whatever the capacity, so whether a
    // batch splits never depends on what the engine encoded before
    const int64_t split_rows = std::min<int64_t>(BT, 32768);
    const bool split = !q2a_gemm_wide_tiles((int) split_rows, d.D, e->gblk);
    if (split) o_part = take((size_t) 4 * split_rows * d.D * 4);
    const int64_t MP = (BT + 255) / 256 * 256;   // padded row stride of the block-major scale arrays
    e->dy_ld = (int) MP;
    if (quant) {
        o_dyD = take((size_t) MP * (d.D / 32) * 4);
        o_dyF = take((size_t) MP * (d.F / 32) * 4);
        o_aD = take((size_t) MP * (d.D / 256 + 1) * 16 * 2);
        o_aF = take((size_t) MP * (d.F / 256 + 1) * 16 * 2);
        o_att = take((size_t) BT * d.D * 4);
        o_hF = take((size_t) BT * d.F * 4);
    } else if (e->f32) {
        o_att = take((size_t) BT * d.D * 4);
    }
    void * ws = nullptr;
    if (hipMalloc(&ws, off) != hipSuccess) {
        (void) hipGetLastError();
        set_err("workspace allocation of %.2f GB for %d clips failed", off / 1e9, B);
        return Q2A_ERR_OOM;
    }
    HIP_TRY(hipMemsetAsync(ws, 0, off, e->stream));   // zero pad rows (xc1 rows 0/last, y1 row 0, V^T tail)
    HIP_TRY(hipHostMalloc((void **) &e->meta_host, (size_t) B * 4 * 4, hipHostMallocDefault));
    uint8_t * b = (uint8_t *) ws;
    e->ws = ws; e->ws_bytes = off; e->cap_clips = B;
    e->meta = (int32_t *) (b + o_meta);
    e->mel = (float *) (b + o_mel);
    e->xc1 = (q2a_half *) (b + o_xc1);
    e->y1 = (q2a_half *) (b + o_y1);
    e->X = (float *) (b + o_X);
    e->actD = (q2a_half *) (b + o_actD);
    e->actF = (q2a_half *) (b + o_actF);
    e->qh = (q2a_half *) (b + o_qh); e->ql = (q2a_half *) (b + o_ql);
    e->kh = (q2a_half *) (b + o_kh); e->kl = (q2a_half *) (b + o_kl);
    e->vt = (q2a_half *) (b + o_vt);
    e->vtl = vlo ? (q2a_half *) (b + o_vtl) : nullptr;
    e->part = split ? (float *) (b + o_part) : nullptr;
    if (quant) {
        e->dyD = (float *) (b + o_dyD); e->dyF = (float *) (b + o_dyF);
        e->aextD = (q2a_half *) (b + o_aD); e->aextF = (q2a_half *) (b + o_aF);
        e->attF = (float *) (b + o_att); e->hF = (float *) (b + o_hF);
    } else if (e->f32) {
        e->attF = (float *) (b + o_att);
    }
    HIP_TRY(hipStreamSynchronize(e->stream));
    return Q2A_OK;
}

q2a_gemm_args gemm_base(const q2a_engine * e, int l, int which, const q2a_half * A, int M) {
    q2a_gemm_args a;
    memset(&a, 0, sizeof(a));
    int N, K;
    mat_dims(e->d, which, N, K);
    const uint64_t * m = e->mat(l, which);
    a.A = A; a.lda = (int64_t) K * e->kx; a.a_rpg = M; a.a_gstride = 0; a.a_step = 1;
    a.W = (const q2a_half *) (e->blob + m[A_W]); a.ldw = (int64_t) K * e->kx;
    a.M = M; a.N = N; a.K = K * e->kx;
    a.gelu_tab = e->g<const uint16_t *>(G_GELU);
    a.gelu_c = e->g<const uint16_t *>(G_GELU_C);
    a.T = e->d.T; a.D = e->d.D; a.H = e->d.H; a.TP = e->TP;
    if (e->blk) {
        a.nblk = K / e->blk;
        a.dx = (const float *) (e->blob + m[A_DX]);
        a.dy = K == e->d.D ? e->dyD : e->dyF;
        a.dy_ld = e->dy_ld;
        if (e->blk == 256) {
            a.dmin = (const float *) (e->blob + m[A_DMIN]);
            a.wext = (const q2a_half *) (e->blob + m[A_WEXT]);
            a.beta = (const float *) (e->blob + m[A_BETA]);
            a.gamma = (const float *) (e->blob + m[A_GAMMA]);
            a.aext = K == e->d.D ? e->aextD : e->aextF;
        }
    }
    return a;
}

hipEvent_t prof_event(q2a_engine * e) {
    if (!e->pool.empty()) { hipEvent_t ev = e->pool.back(); e->pool.pop_back(); return ev; }
    hipEvent_t ev = nullptr;
    (void) hipEventCreate(&ev);
    return ev;
}

// Launch `call` on stream s; when profiling, bracket it with an event pair attributed to class cls.
#define PLAUNCH(e, s, cls, call)                                                      \
    do {                                                                              \
        q2a_engine::rec r_{cls, nullptr, nullptr};                                    \
        const bool on_ = (e)->prof && (((e)->prof_mask >> (cls)) & 1);                 \
        if (on_) { r_.a = prof_event(e); r_.b = prof_event(e); (void) hipEventRecord(r_.a, s); } \
        hipError_t e_ = (call);                                                       \
        if (e_ != hipSuccess) {                                                       \
            set_err("%s: %s", #call, hipGetErrorString(e_));                        \
            return Q2A_ERR_HIP;                                                       \
        }                                                                             \
        if (on_) { (void) hipEventRecord(r_.b, s); (e)->pending.push_back(r_); }      \
    } while (0)

int ln_mode(const q2a_engine * e) { return e->bf16 ? 4 : e->f32 ? 3 : e->blk == 0 ? 0 : e->blk == 256 ? 1 : 2; }

#define LAUNCH(x)                                                                     \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            set_err("%s: %s", #x, hipGetErrorString(e_));                           \
            return Q2A_ERR_HIP;                                                       \
        }                                                                             \
    } while (0)

// one pre-LN encoder block on X [B*T][D] (qwen2-whisper.cpp:2014-2155)
int run_block(q2a_engine * e, int l, int B, hipStream_t s) {
    const dims & d = e->d;
    const int M = B * d.T;
    const int mode = ln_mode(e);
    auto tap = [&](int i, const q2a_half * src, int K) -> hipError_t {
        if (!e->taps[i]) return hipSuccess;
        return hipMemcpyAsync(e->taps[i], src, (size_t) M * K * e->kx * 2, hipMemcpyDeviceToDevice, s);
    };
    q2a_ln_args ln{e->X, M, d.D, e->lv<const float *>(l, L_LN1W), e->lv<const float *>(l, L_LN1B), mode, e->actD, e->dyD, e->aextD, e->dy_ld};
    PLAUNCH(e, s, Q2A_PROF_LN, q2a_launch_layernorm(ln, s));
    LAUNCH(tap(0, e->actD, d.D));
    {
        q2a_gemm_args a = gemm_base(e, l, 0, e->actD, M);
        a.bias = e->lv<const float *>(l, L_BQKV);
        a.qh = e->qh; a.ql = e->ql; a.kh = e->kh; a.kl = e->kl; a.vt = e->vt; a.vtl = e->vtl;
        a.v_rows = e->bf16 ? 0 : 1;   // reference contract: V hi / lo row-major like K (bf16 contract: V^T)
        // ggml_scale(Q, 1/sqrt(dh)) (:2054); the reference-contract attention also wants log2(e) folded in (its
        // softmax runs in log2 units): one f32 multiply by fl(log2 e)/8, 2^-3 being exact
        a.qscale = (1.0f / sqrtf((float) (d.D / d.H))) * (e->bf16 ? 1.0f : Q2A_LOG2E);
        PLAUNCH(e, s, Q2A_PROF_GEMM_QKV, q2a_launch_gemm(a, Q2A_EPI_QKV, e->gblk, s));
    }
    {
        q2a_attn_args at{e->qh, e->ql, e->kh, e->kl, e->vt, B, d.T, d.D, d.H, e->TP, nullptr, nullptr, e->bf16 ? 1 : 0};
        at.vtl = e->vtl;
        at.v_rows = e->bf16 ? 0 : 1;
        if (mode == 0 || mode == 4) at.outH = e->actD; else at.outF = e->attF;
        PLAUNCH(e, s, Q2A_PROF_ATTN, q2a_launch_attention(at, s));
        if (mode == 3) {
            const int64_t n = (int64_t) M * d.D;
            PLAUNCH(e, s, Q2A_PROF_QUANT, launch_split3(e->attF, e->actD, d.D, n, s));
        } else if (mode == 1 || mode == 2) {
            q2a_quant_args qa{e->attF, nullptr, M, d.D, mode, e->actD, e->dyD, e->aextD, e->dy_ld};
            PLAUNCH(e, s, Q2A_PROF_QUANT, q2a_launch_quant_act(qa, s));
        }
    }
    LAUNCH(tap(1, e->actD, d.D));
    {
        q2a_gemm_args a = gemm_base(e, l, 1, e->actD, M);
        a.bias = e->lv<const float *>(l, L_BO);
        a.outF = e->X; a.ldo = d.D;
        a.part = e->part; a.split_stride = (int64_t) M * d.D;
        PLAUNCH(e, s, Q2A_PROF_GEMM_O, q2a_launch_gemm(a, Q2A_EPI_RESID, e->gblk, s));
    }
    q2a_ln_args ln2{e->X, M, d.D, e->lv<const float *>(l, L_LN2W), e->lv<const float *>(l, L_LN2B), mode, e->actD, e->dyD, e->aextD, e->dy_ld};
    PLAUNCH(e, s, Q2A_PROF_LN, q2a_launch_layernorm(ln2, s));
    LAUNCH(tap(2, e->actD, d.D));
    {
        q2a_gemm_args a = gemm_base(e, l, 2, e->actD, M);
        a.bias = e->lv<const float *>(l, L_B1);
        if (mode == 0 || mode == 3 || mode == 4) {
            // F32 weights: the GELU output is exactly fp16 (LUT), so the fc2 operand is [h | 0 | h] (middle third
            // stays zero from the workspace memset) against [W2h | W2h | W2l]
            a.outH = e->actF; a.ldo = (int64_t) d.F * e->kx; a.o_rpg = M; a.o_gstride = 0; a.o_off = 0;
            a.o_dup = mode == 3 ? 2 * d.F : 0;
            PLAUNCH(e, s, Q2A_PROF_GEMM_FC1, q2a_launch_gemm(a, Q2A_EPI_GELU_H, e->gblk, s));
        } else if (mode == 1 && q2a_gemm_wide_tiles(M, d.F, e->blk) &&
                   e->fc1_path == 2 && q2a_gemm_pipe8(a, e->blk)) {
            // fused fc1 + GELU + Q8_K quantization of the fc2 input (one Q8_K block per 256-column tile)
            a.outH = e->actF; a.ldo = d.F; a.qdy = e->dyF; a.qaext = e->aextF;
            PLAUNCH(e, s, Q2A_PROF_GEMM_FC1, q2a_launch_gemm(a, Q2A_EPI_GELU_Q8K, e->blk, s));
        } else if (mode == 1 && e->fc1_path != 1) {
            // fc1 writes its fp16 pre-activation (plain stores); the Q8_K quantizer of the fc2 input applies the
            // GELU table from LDS on the way (same codes as the GELU epilogue + quantizer below)
            q2a_half * hH = (q2a_half *) e->hF;
            a.outH = hH; a.ldo = d.F; a.o_rpg = M; a.o_gstride = 0; a.o_off = 0;
            PLAUNCH(e, s, Q2A_PROF_GEMM_FC1, q2a_launch_gemm(a, Q2A_EPI_PRE_H, e->blk, s));
            PLAUNCH(e, s, Q2A_PROF_QUANT, q2a_launch_gelu_quant_q8k(hH, M, d.F, e->g<const uint16_t *>(G_GELU), e->actF,
                                                                   e->dyF, e->aextF, e->dy_ld, s));
        } else {
            // GELU output is exactly fp16-valued (LUT): keep it as fp16, then quantize for fc2
            q2a_half * hH = (q2a_half *) e->hF;
            a.outH = hH; a.ldo = d.F; a.o_rpg = M; a.o_gstride = 0; a.o_off = 0;
            PLAUNCH(e, s, Q2A_PROF_GEMM_FC1, q2a_launch_gemm(a, Q2A_EPI_GELU_H, e->blk, s));
            q2a_quant_args qa{nullptr, hH, M, d.F, mode, e->actF, e->dyF, e->aextF, e->dy_ld};
            PLAUNCH(e, s, Q2A_PROF_QUANT, q2a_launch_quant_act(qa, s));
        }
    }
    LAUNCH(tap(3, e->actF, d.F));
    {
        q2a_gemm_args a = gemm_base(e, l, 3, e->actF, M);
        a.bias = e->lv<const float *>(l, L_B2);
        a.outF = e->X; a.ldo = d.D;
        a.part = e->part; a.split_stride = (int64_t) M * d.D;
        PLAUNCH(e, s, Q2A_PROF_GEMM_FC2, q2a_launch_gemm(a, Q2A_EPI_RESID, e->gblk, s));
    }
    return Q2A_OK;
}

int ensure_frange(q2a_engine * e, hipStream_t s) {
    if (e->frange) return Q2A_OK;
    if (hipMalloc((void **) &e->frange, (size_t) e->d.M * sizeof(int2)) != hipSuccess) {
        (void) hipGetLastError();
        e->frange = nullptr;
        set_err("filter-range allocation failed");
        return Q2A_ERR_OOM;
    }
    LAUNCH(q2a_launch_filter_ranges(e->g<const float *>(G_FILT), e->d.M, 201, e->frange, s));
    return Q2A_OK;
}

// mel + conv frontend: PCM -> X [B*T][D] (conv graph qwen2-whisper.cpp:1892-1952 + pe add :2005)
int run_frontend(q2a_engine * e, const float * pcm, int64_t stride, int B, int max_frames, hipStream_t s) {
    const dims & d = e->d;
    int32_t * nsamp = e->meta;
    int32_t * seek = e->meta + B;
    int32_t * cmax = e->meta + 3 * B;
    LAUNCH(hipMemsetAsync(cmax, 0x80, (size_t) B * 4, s));
    q2a_mel_args ma;
    ma.pcm = pcm; ma.pcm_stride = stride; ma.n_samples = nsamp; ma.seek = seek; ma.n_clips = B;
    ma.n_mel = d.M; ma.n_bins = 201; ma.n_frames_win = d.TM; ma.max_frames = max_frames;
    ma.filters = e->g<const float *>(G_FILT); ma.tab = e->g<const float *>(G_TAB);
    if (int rc = ensure_frange(e, s)) return rc;
    ma.frange = e->frange;
    ma.mel = e->mel; ma.clip_max = cmax; ma.xc1 = e->xc1; ma.xc_f32 = e->f32 ? 1 : 0;
    PLAUNCH(e, s, Q2A_PROF_MEL, q2a_launch_mel(ma, s));
    const int P1 = 3, P2 = e->f32 ? 2 : 1;   // operand parts per mel row / per conv1 output row
    // both convs sum each 64-deep K-step's MFMA partial in f64 (Q2A_BLK_EXACT): within rounding of the exact dot
    // product, where a plain f32 MFMA chain carried twice the reference builds' own conv error
    {   // conv1: implicit GEMM, A row t = xc1 rows t..t+2 of its clip (3 x P1 x M halves), K = 3 P1 M
        q2a_gemm_args a;
        memset(&a, 0, sizeof(a));
        a.A = e->xc1; a.lda = P1 * d.M; a.a_rpg = d.TM; a.a_gstride = d.TM + 2; a.a_step = 1;
        a.W = e->g<const q2a_half *>(G_CONV1_W); a.ldw = 3 * P1 * d.M;
        a.M = B * d.TM; a.N = d.D; a.K = 3 * P1 * d.M;
        a.bias = e->g<const float *>(G_CONV1_B);
        a.outH = e->y1; a.ldo = (int64_t) P2 * d.D; a.o_rpg = d.TM; a.o_gstride = d.TM + 1; a.o_off = 1;
        a.o_dup = e->f32 ? d.D : 0;
        a.gelu_tab = e->g<const uint16_t *>(G_GELU);
        a.gelu_c = e->g<const uint16_t *>(G_GELU_C);
        PLAUNCH(e, s, Q2A_PROF_CONV1, q2a_launch_gemm(a, Q2A_EPI_GELU_H, Q2A_BLK_EXACT, s));
    }
    {   // conv2 (stride 2): A row t = y1 rows 2t..2t+2 (inputs 2t-1..2t+1), K = 3D; + pe
        q2a_gemm_args a;
        memset(&a, 0, sizeof(a));
        a.A = e->y1; a.lda = (int64_t) P2 * d.D; a.a_rpg = d.T; a.a_gstride = d.TM + 1; a.a_step = 2;
        a.W = e->g<const q2a_half *>(G_CONV2_W); a.ldw = 3 * P2 * d.D;
        a.M = B * d.T; a.N = d.D; a.K = 3 * P2 * d.D;
        a.bias = e->g<const float *>(G_CONV2_B);
        a.outF = e->X; a.ldo = d.D; a.pe = e->g<const float *>(G_PE); a.T = d.T;
        a.gelu_tab = e->g<const uint16_t *>(G_GELU);
        a.gelu_c = e->g<const uint16_t *>(G_GELU_C);
        PLAUNCH(e, s, Q2A_PROF_CONV2, q2a_launch_gemm(a, Q2A_EPI_CONV2, Q2A_BLK_EXACT, s));
    }
    return Q2A_OK;
}

// per-clip metadata (host): whisper_encoder_output_with_state's seek / too-short logic (:2356-2365)
int prepare_meta(q2a_engine * e, const int32_t * n_samples, int B, int offset_ms, const int32_t * offs, int32_t * status, int & max_frames,
                 int64_t max_valid, hipStream_t s) {
    int32_t * mh = e->meta_host;
    HIP_TRY(hipEventSynchronize(e->meta_evt));   // the previous call's upload out of mh may still be queued
    max_frames = 0;
    for (int c = 0; c < B; ++c) {
        const int seek = (offs ? offs[c] : offset_ms) / 10;
        if (seek < 0) { set_err("clip %d: negative offset", c); return Q2A_ERR_ARG; }
        const int n = n_samples[c];
        if (n < 0 || (max_valid >= 0 && n > max_valid)) { set_err("clip %d: bad n_samples %d", c, n); return Q2A_ERR_ARG; }
        const int n_len_org = 1 + (n + 200 - 400) / 160;   // mel.n_len_org (:2613), C truncation
        const bool ok = n > 200 && (e->force_encode || !(n_len_org < seek + 100));
        mh[c] = ok ? n : 0;
        mh[B + c] = seek;
        mh[2 * B + c] = ok ? 1 : 0;
        if (status) status[c] = ok ? Q2A_CLIP_ENCODED : Q2A_CLIP_SKIPPED;
        max_frames = std::max(max_frames, (int) (((int64_t) mh[c] + 480000) / 160));
    }
    HIP_TRY(hipMemcpyAsync(e->meta, mh, (size_t) B * 3 * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(e->meta_evt, s));
    return Q2A_OK;
}

int encode_impl(q2a_engine * e, const float * pcm, int64_t stride, const int32_t * n_samples, int B, int offset_ms,
                const int32_t * offs, float * out, int32_t * status, hipStream_t s) {
    if (B <= 0 || !pcm || !n_samples || !out) { set_err("invalid arguments"); return Q2A_ERR_ARG; }
    if (offset_ms < 0) { set_err("offset_ms must be >= 0"); return Q2A_ERR_ARG; }
    HIP_TRY(hipSetDevice(e->device));
    int rc = reserve(e, B);
    if (rc) return rc;
    int max_frames = 0;
    rc = prepare_meta(e, n_samples, B, offset_ms, offs, status, max_frames, stride > 0 ? stride : -1, s);   // stride 0: shared PCM
    if (rc) return rc;
    rc = run_frontend(e, pcm, stride, B, max_frames, s);
    if (rc) return rc;
    for (int l = 0; l < e->d.L; ++l) {
        rc = run_block(e, l, B, s);
        if (rc) return rc;
    }
    q2a_pool_args pa{e->X, B, e->d.T, e->d.D, e->g<const float *>(G_LNP_W), e->g<const float *>(G_LNP_B), out, e->meta + 2 * B};
    PLAUNCH(e, s, Q2A_PROF_POOL, q2a_launch_pool_ln(pa, s));
    return Q2A_OK;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------------
extern "C" {

const char * q2a_last_error(void) { return g_err.c_str(); }

// (q2a_internal.h) the calling thread's q2a_last_error text, for the library's other translation units
void q2a_internal_set_error(const char * msg) { g_err = msg ? msg : ""; }

int q2a_internal_engine_blob(const q2a_engine * e, const void ** blob, int64_t * bytes, int * device) {
    if (!e || !e->blob || e->h.compact) { set_err("engine holds no device-layout weights"); return Q2A_ERR_ARG; }
    if (blob) *blob = e->blob;
    if (bytes) *bytes = e->blob_size;
    if (device) *device = e->device;
    return Q2A_OK;
}

int64_t q2a_pack_model(const char * path, void ** host_blob) { return q2a_pack_model_ex(path, Q2A_ACT_REFERENCE, host_blob); }

int64_t q2a_pack_model_ex(const char * path, int act, void ** host_blob) {
    if (act != Q2A_ACT_REFERENCE && act != Q2A_ACT_BF16) { set_err("unknown activation mode %d", act); return Q2A_ERR_ARG; }
    std::vector<uint8_t> v;
    const int rc = pack(path, v, act);
    if (rc) return rc;
    void * p = malloc(v.size());
    if (!p) { set_err("host allocation failed"); return Q2A_ERR_OOM; }
    memcpy(p, v.data(), v.size());
    *host_blob = p;
    return (int64_t) v.size();
}

int64_t q2a_pack_model_compact(const char * path, int act, void ** host_blob) {
    if (act != Q2A_ACT_REFERENCE && act != Q2A_ACT_BF16) { set_err("unknown activation mode %d", act); return Q2A_ERR_ARG; }
    std::vector<uint8_t> v;
    const int rc = pack(path, v, act, true);
    if (rc) return rc;
    void * p = malloc(v.size());
    if (!p) { set_err("host allocation failed"); return Q2A_ERR_OOM; }
    memcpy(p, v.data(), v.size());
    *host_blob = p;
    return (int64_t) v.size();
}

int64_t q2a_blob_device_size(const void * host_header, int64_t header_bytes, int64_t * transport_bytes) {
    blob_header h;
    if (!host_header || header_bytes < (int64_t) sizeof(h)) { set_err("invalid arguments"); return Q2A_ERR_ARG; }
    memcpy(&h, host_header, sizeof(h));
    if (const char * why = header_problem(h)) { set_err("%s", why); return Q2A_ERR_FORMAT; }
    if (transport_bytes) *transport_bytes = h.compact ? (int64_t) compact_of(h).total : (int64_t) h.total;
    return (int64_t) h.total;
}

int q2a_expand_blob(const void * dev_blob, int64_t size, void * dev_out, int64_t out_bytes, int device, void * stream) {
    if (!dev_blob || !dev_out || size < (int64_t) HEADER_BYTES) { set_err("invalid arguments"); return Q2A_ERR_ARG; }
    int prev = -1;
    HIP_TRY(hipGetDevice(&prev));
    struct restore { int d; ~restore() { if (d >= 0) (void) hipSetDevice(d); } } rs{prev};   // the caller's device back
    HIP_TRY(hipSetDevice(device));
    blob_header h;
    HIP_TRY(hipMemcpy(&h, dev_blob, sizeof(h), hipMemcpyDeviceToHost));
    if (const char * why = header_problem(h)) { set_err("%s", why); return Q2A_ERR_FORMAT; }
    if (!h.compact) { set_err("not a compact q2a weight blob"); return Q2A_ERR_FORMAT; }
    if ((int64_t) compact_of(h).total != size || out_bytes < (int64_t) h.total) { set_err("blob size mismatch"); return Q2A_ERR_ARG; }
    return expand_blob((const uint8_t *) dev_blob, h, (uint8_t *) dev_out, stream ? (hipStream_t) stream : nullptr);
}

void q2a_free_host_blob(void * p) { free(p); }

q2a_engine * q2a_open(const char * model_path, int device) { return q2a_open_ex(model_path, device, Q2A_ACT_REFERENCE); }

q2a_engine * q2a_open_ex(const char * model_path, int device, int act) {
    if (act != Q2A_ACT_REFERENCE && act != Q2A_ACT_BF16) { set_err("unknown activation mode %d", act); return nullptr; }
    q2a_engine * e = new q2a_engine();
    std::vector<uint8_t> v;
    if (engine_init(e, device) || pack(model_path, v, act)) { q2a_close(e); return nullptr; }
    memcpy(&e->h, v.data(), sizeof(blob_header));
    if (engine_adopt_header(e)) { q2a_close(e); return nullptr; }
    if (hipMalloc((void **) &e->blob, v.size()) != hipSuccess) {
        (void) hipGetLastError();
        set_err("weight allocation of %.2f GB failed", v.size() / 1e9);
        q2a_close(e);
        return nullptr;
    }
    e->own_blob = true;
    e->blob_size = (int64_t) v.size();
    if (hipMemcpy(e->blob, v.data(), v.size(), hipMemcpyHostToDevice) != hipSuccess) {
        set_err("weight upload failed");
        q2a_close(e);
        return nullptr;
    }
    return e;
}

q2a_engine * q2a_open_device_blob(const void * dev_blob, int64_t size, int device) {
    if (!dev_blob || size < (int64_t) HEADER_BYTES) { set_err("invalid blob"); return nullptr; }
    q2a_engine * e = new q2a_engine();
    if (engine_init(e, device)) { q2a_close(e); return nullptr; }
    if (hipMemcpy(&e->h, dev_blob, sizeof(blob_header), hipMemcpyDeviceToHost) != hipSuccess) {
        set_err("cannot read blob header from device");
        q2a_close(e);
        return nullptr;
    }
    if (engine_adopt_header(e)) { q2a_close(e); return nullptr; }   // (validates before any size is derived)
    const int64_t want = e->h.compact ? (int64_t) compact_of(e->h).total : (int64_t) e->h.total;
    if (want != size) {
        set_err("blob size mismatch");
        q2a_close(e);
        return nullptr;
    }
    if (e->h.compact) {   // the transport form: expand into an engine-owned device layout
        const blob_header hc = e->h;
        e->h.compact = 0;
        if (hipMalloc((void **) &e->blob, e->h.total) != hipSuccess) {
            (void) hipGetLastError();
            set_err("weight allocation of %.2f GB failed", e->h.total / 1e9);
            q2a_close(e);
            return nullptr;
        }
        e->own_blob = true;
        e->blob_size = (int64_t) e->h.total;
        if (expand_blob((const uint8_t *) dev_blob, hc, e->blob, e->stream)) { q2a_close(e); return nullptr; }
        return e;
    }
    e->blob = (uint8_t *) dev_blob;
    e->own_blob = false;
    e->blob_size = size;
    return e;
}

q2a_engine * q2a_open_shared(const q2a_engine * base) {
    if (!base) { set_err("invalid arguments"); return nullptr; }
    return q2a_open_device_blob(base->blob, base->blob_size, base->device);
}

int q2a_set_force_encode(q2a_engine * e, int on) {
    if (!e) return Q2A_ERR_ARG;
    e->force_encode = on != 0;
    return Q2A_OK;
}

void q2a_close(q2a_engine * e) {
    if (!e) return;
    (void) hipSetDevice(e->device);
    (void) hipDeviceSynchronize();   // (calls may have run on caller streams or stream 0, not only e->stream)
    free_host_bufs(e);
    free_ws(e);
    for (auto & r : e->pending) { (void) hipEventDestroy(r.a); (void) hipEventDestroy(r.b); }
    for (auto ev : e->pool) (void) hipEventDestroy(ev);
    if (e->own_blob && e->blob) (void) hipFree(e->blob);
    if (e->frange) (void) hipFree(e->frange);
    if (e->meta_evt) (void) hipEventDestroy(e->meta_evt);
    if (e->stream) (void) hipStreamDestroy(e->stream);
    delete e;
}

int q2a_get_info(const q2a_engine * e, q2a_info * info) {
    if (!e || !info) return Q2A_ERR_ARG;
    info->n_audio_ctx = e->d.T; info->n_audio_state = e->d.D; info->n_audio_head = e->d.H;
    info->n_audio_layer = e->d.L; info->n_mels = e->d.M; info->wtype = e->wtype; info->n_out = e->d.TO;
    info->device = e->device; info->weight_bytes = e->blob_size; info->workspace_bytes = (int64_t) e->ws_bytes;
    info->act = e->bf16 ? Q2A_ACT_BF16 : Q2A_ACT_REFERENCE;
    info->reserved = 0;
    return Q2A_OK;
}

int q2a_reserve(q2a_engine * e, int max_clips, int64_t max_samples) {
    if (!e || max_clips <= 0) { set_err("invalid arguments"); return Q2A_ERR_ARG; }
    (void) max_samples;
    return reserve(e, max_clips);
}

int q2a_encode_device(q2a_engine * e, const float * pcm_dev, int64_t pcm_stride, const int32_t * n_samples,
                      int n_clips, int offset_ms, float * out_dev, int32_t * status, void * stream) {
    if (!e) return Q2A_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = call_stream(stream);
    return encode_impl(e, pcm_dev, pcm_stride, n_samples, n_clips, offset_ms, nullptr, out_dev, status, s);
}

int q2a_encode_device_ex(q2a_engine * e, const float * pcm_dev, int64_t pcm_stride, const int32_t * n_samples,
                         const int32_t * offsets_ms, int n_clips, float * out_dev, int32_t * status, void * stream) {
    if (!e || !offsets_ms) { set_err("invalid arguments"); return Q2A_ERR_ARG; }
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = call_stream(stream);
    return encode_impl(e, pcm_dev, pcm_stride, n_samples, n_clips, 0, offsets_ms, out_dev, status, s);
}

int q2a_encode_host(q2a_engine * e, const float * const * pcm, const int32_t * n_samples, int n_clips, int offset_ms,
                    float * out_host, int32_t * status) {
    return q2a_encode_host_ex(e, pcm, n_samples, nullptr, n_clips, offset_ms, out_host, status);
}

int q2a_encode_host_ex(q2a_engine * e, const float * const * pcm, const int32_t * n_samples, const int32_t * offsets_ms,
                       int n_clips, int offset_ms, float * out_host, int32_t * status) {
    if (!e || !pcm || !n_samples || !out_host || n_clips <= 0) { set_err("invalid arguments"); return Q2A_ERR_ARG; }
    for (int c = 0; c < n_clips; ++c)   // (checked before any copy: a negative count would be a huge memcpy)
        if (n_samples[c] < 0 || (n_samples[c] > 0 && !pcm[c])) {
            set_err("clip %d: bad samples (%d, %p)", c, n_samples[c], (const void *) pcm[c]);
            if (status) for (int k = 0; k < n_clips; ++k) status[k] = Q2A_CLIP_FAILED;
            return Q2A_ERR_ARG;
        }
    HIP_TRY(hipSetDevice(e->device));
    // Chunks of clips through two staging sets: chunk k's host->pinned copy and H2D (copy stream) run while chunk k-1
    // encodes (compute stream), and chunk k-1's D2H + pinned->host copy while chunk k encodes. One chunk below 32
    // clips (nothing to overlap with); else at least two, at most 64 clips each. Clips are independent and every
    // tile regime sums in one K order, so the chunking changes no output bit (batch invariance).
    // Outputs of skipped clips (< 1 s after the offset) are never copied back: the caller's contents stay untouched.
    const int nchunk = n_clips < 32 ? 1 : std::max(2, (n_clips + 63) / 64);
    const int C = (n_clips + nchunk - 1) / nchunk;
    int64_t maxn = 1;
    for (int c = 0; c < n_clips; ++c) maxn = std::max<int64_t>(maxn, n_samples[c]);
    maxn = (maxn + 63) & ~int64_t(63);
    if (int rc = ensure_host_bufs(e, C, maxn)) return rc;
    const size_t per_out = (size_t) e->d.TO * e->d.D;
    // st: what encode_impl reported per clip; pub: what the caller gets — a clip's status is published only once its
    // chunk's outputs reached out_host, so a failure part-way leaves every later clip (and a chunk whose copy-out
    // never ran) at Q2A_CLIP_FAILED rather than a stale "encoded"
    std::vector<int32_t> st(n_clips, Q2A_CLIP_FAILED), pub(n_clips, Q2A_CLIP_FAILED);
    hipStream_t cs = e->copy_stream, s = e->stream;
    int rc = Q2A_OK;
    auto copy_out = [&](int k) {   // chunk k's encoded outputs: pinned -> caller (after its D2H)
        const int c0 = k * C, n = std::min(C, n_clips - c0);
        q2a_engine::host_buf & b = e->hb[k & 1];
        if (hipEventSynchronize(b.d2h) != hipSuccess) return Q2A_ERR_HIP;
        for (int c = 0; c < n; ++c) {
            if (st[c0 + c] == Q2A_CLIP_ENCODED)
                memcpy(out_host + (c0 + c) * per_out, b.pin_out + c * per_out, per_out * 4);
            pub[c0 + c] = st[c0 + c];
        }
        return Q2A_OK;
    };
    for (int k = 0; k < nchunk && rc == Q2A_OK; ++k) {
        const int c0 = k * C, n = std::min(C, n_clips - c0);
        q2a_engine::host_buf & b = e->hb[k & 1];
        // staging set k&1 was last used by chunk k-2: its H2D must have left pin_in, its D2H must have left d_out
        if (hipEventSynchronize(b.h2d) != hipSuccess) { rc = Q2A_ERR_HIP; break; }
        for (int c = 0; c < n; ++c) {
            memcpy(b.pin_in + c * maxn, pcm[c0 + c], (size_t) n_samples[c0 + c] * 4);
        }
        if (hipStreamWaitEvent(cs, b.comp, 0) != hipSuccess ||   // chunk k-2's encode no longer reads d_in
            hipMemcpyAsync(b.d_in, b.pin_in, (size_t) n * maxn * 4, hipMemcpyHostToDevice, cs) != hipSuccess ||
            hipEventRecord(b.h2d, cs) != hipSuccess ||
            hipStreamWaitEvent(s, b.h2d, 0) != hipSuccess ||     // PCM landed
            hipStreamWaitEvent(s, b.d2h, 0) != hipSuccess) {     // chunk k-2's outputs left d_out
            rc = Q2A_ERR_HIP;
            break;
        }
        rc = encode_impl(e, b.d_in, maxn, n_samples + c0, n, offset_ms, offsets_ms ? offsets_ms + c0 : nullptr, b.d_out,
                         st.data() + c0, s);
        if (rc) break;
        if (hipEventRecord(b.comp, s) != hipSuccess || hipStreamWaitEvent(cs, b.comp, 0) != hipSuccess ||
            hipMemcpyAsync(b.pin_out, b.d_out, (size_t) n * per_out * 4, hipMemcpyDeviceToHost, cs) != hipSuccess ||
            hipEventRecord(b.d2h, cs) != hipSuccess) {
            rc = Q2A_ERR_HIP;
            break;
        }
        if (k >= 1) rc = copy_out(k - 1);   // runs while chunk k encodes
    }
    if (rc == Q2A_OK) rc = copy_out(nchunk - 1);
    if (hipStreamSynchronize(cs) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
        if (rc == Q2A_OK) { set_err("stream error"); rc = Q2A_ERR_HIP; }
    }
    if (rc == Q2A_ERR_HIP && g_err.empty()) set_err("host-path copy failed");
    if (status) for (int c = 0; c < n_clips; ++c) status[c] = pub[c];
    return rc;
}

int q2a_pcm_to_mel(q2a_engine * e, const float * pcm, int n_samples, float * mel_out, int64_t mel_cap, int * n_len_out) {
    if (!e || !pcm || !mel_out || !n_len_out || n_samples <= 200) { set_err("invalid arguments"); return Q2A_ERR_ARG; }
    HIP_TRY(hipSetDevice(e->device));
    const dims & d = e->d;
    const int n_len = (int) (((int64_t) n_samples + 480000) / 160);
    if (mel_cap < (int64_t) d.M * n_len) { set_err("mel buffer too small (%d frames)", n_len); return Q2A_ERR_ARG; }
    int rc = reserve(e, 1);
    if (rc) return rc;
    // run the mel kernel with a window covering every frame, in chunks of TM frames
    float * dpcm = nullptr;
    HIP_TRY(hipMalloc((void **) &dpcm, (size_t) n_samples * 4));
    std::vector<float> chunk((size_t) d.M * d.TM);
    hipStream_t s = e->stream;
    rc = Q2A_OK;
    if (hipMemcpy(dpcm, pcm, (size_t) n_samples * 4, hipMemcpyHostToDevice) != hipSuccess) rc = Q2A_ERR_HIP;
    int32_t cmax = 0;
    for (int f0 = 0; f0 < n_len && rc == Q2A_OK; f0 += d.TM) {
        int32_t * mh = e->meta_host;
        if (hipEventSynchronize(e->meta_evt) != hipSuccess) { rc = Q2A_ERR_HIP; break; }
        mh[0] = n_samples; mh[1] = f0; mh[2] = 1;
        if (hipMemcpyAsync(e->meta, mh, 12, hipMemcpyHostToDevice, s) != hipSuccess) { rc = Q2A_ERR_HIP; break; }
        if (hipEventRecord(e->meta_evt, s) != hipSuccess) { rc = Q2A_ERR_HIP; break; }
        if (hipMemsetAsync(e->meta + 3, 0x80, 4, s) != hipSuccess) { rc = Q2A_ERR_HIP; break; }
        q2a_mel_args ma;
        ma.pcm = dpcm; ma.pcm_stride = n_samples; ma.n_samples = e->meta; ma.seek = e->meta + 1; ma.n_clips = 1;
        ma.n_mel = d.M; ma.n_bins = 201; ma.n_frames_win = d.TM; ma.max_frames = n_len;
        ma.filters = e->g<const float *>(G_FILT); ma.tab = e->g<const float *>(G_TAB);
        if (int rc = ensure_frange(e, e->stream)) return rc;
        ma.frange = e->frange;
        ma.mel = e->mel; ma.clip_max = e->meta + 3; ma.xc1 = e->xc1; ma.xc_f32 = e->f32 ? 1 : 0;
        if (q2a_launch_mel(ma, s) != hipSuccess) { rc = Q2A_ERR_HIP; break; }
        if (hipMemcpyAsync(chunk.data(), e->mel, chunk.size() * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(&cmax, e->meta + 3, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) { rc = Q2A_ERR_HIP; break; }
        const int nf = std::min(d.TM, n_len - f0);
        for (int j = 0; j < d.M; ++j) memcpy(mel_out + (size_t) j * n_len + f0, chunk.data() + (size_t) j * d.TM, (size_t) nf * 4);
    }
    (void) hipFree(dpcm);
    if (rc) { set_err("mel computation failed"); return rc; }
    // clamp + normalise exactly as the reference (:2633-2649) on the host (the device path fuses this into conv1)
    const float mx_f = [&] { int32_t i = cmax; i = i >= 0 ? i : i ^ 0x7fffffff; float f; memcpy(&f, &i, 4); return f; }();
    const double mmax = (double) mx_f - 8.0;
    for (int64_t i = 0; i < (int64_t) d.M * n_len; ++i) {
        float v = mel_out[i];
        if (v < mmax) v = (float) mmax;
        mel_out[i] = (float) ((v + 4.0) / 4.0);
    }
    *n_len_out = n_len;
    return Q2A_OK;
}

int q2a_profile_enable(q2a_engine * e, int on) {
    if (!e) return Q2A_ERR_ARG;
    e->prof = on != 0;
    e->prof_mask = ~0u;
    return Q2A_OK;
}

int q2a_profile_enable_mask(q2a_engine * e, unsigned mask) {
    if (!e) return Q2A_ERR_ARG;
    e->prof = mask != 0;
    e->prof_mask = mask;
    return Q2A_OK;
}

int q2a_profile_read(q2a_engine * e, double * ms, int64_t * counts, int n, int reset) {
    if (!e || n < 0) return Q2A_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    for (auto & r : e->pending) {
        HIP_TRY(hipEventSynchronize(r.b));
        float t = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, r.a, r.b));
        e->prof_ms[r.cls] += t;
        e->prof_n[r.cls] += 1;
        e->pool.push_back(r.a);
        e->pool.push_back(r.b);
    }
    e->pending.clear();
    for (int i = 0; i < n && i < Q2A_PROF_CLASSES; ++i) {
        if (ms) ms[i] = e->prof_ms[i];
        if (counts) counts[i] = e->prof_n[i];
    }
    if (reset)
        for (int i = 0; i < Q2A_PROF_CLASSES; ++i) { e->prof_ms[i] = 0; e->prof_n[i] = 0; }
    return Q2A_OK;
}

int q2a_test_linear(q2a_engine * e, int layer, int which, const float * x, int M, float * y, void * stream) {
    if (!e || layer < 0 || layer >= e->d.L || which < 0 || which > 3 || M <= 0) return Q2A_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = call_stream(stream);
    const dims & d = e->d;
    int rc = reserve(e, (M + d.T - 1) / d.T);
    if (rc) return rc;
    int N, K;
    mat_dims(d, which, N, K);
    q2a_half * A = K == d.D ? e->actD : e->actF;
    const int mode = ln_mode(e);
    if (mode == 0 || mode == 4) {
        const int64_t n = (int64_t) M * K;
        if (mode == 0) hipLaunchKernelGGL(k_to_half, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, x, A, n);
        else hipLaunchKernelGGL(k_to_bf16, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, x, A, n);
        LAUNCH(hipGetLastError());
    } else if (mode == 3) {
        const int64_t n = (int64_t) M * K;
        hipLaunchKernelGGL(k_split3, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, x, A, K, n);
        LAUNCH(hipGetLastError());
    } else {
        q2a_quant_args qa{x, nullptr, M, K, mode, A, K == d.D ? e->dyD : e->dyF, K == d.D ? e->aextD : e->aextF, e->dy_ld};
        LAUNCH(q2a_launch_quant_act(qa, s));
    }
    q2a_gemm_args a = gemm_base(e, layer, which, A, M);
    a.outF = y; a.ldo = N;
    LAUNCH(q2a_launch_gemm(a, Q2A_EPI_STORE_F, e->gblk, s));
    return Q2A_OK;
}

int q2a_test_block(q2a_engine * e, int layer, float * x, int n_clips, void * stream) {
    if (!e || layer < 0 || layer >= e->d.L || n_clips <= 0) return Q2A_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = call_stream(stream);
    int rc = reserve(e, n_clips);
    if (rc) return rc;
    const size_t bytes = (size_t) n_clips * e->d.T * e->d.D * 4;
    HIP_TRY(hipMemcpyAsync(e->X, x, bytes, hipMemcpyDeviceToDevice, s));
    rc = run_block(e, layer, n_clips, s);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(x, e->X, bytes, hipMemcpyDeviceToDevice, s));
    return Q2A_OK;
}

int q2a_test_block_taps(q2a_engine * e, int layer, float * x, int n_clips, void * const * taps, void * stream) {
    if (!e || !taps) return Q2A_ERR_ARG;
    for (int i = 0; i < 4; ++i) e->taps[i] = taps[i];
    const int rc = q2a_test_block(e, layer, x, n_clips, stream);
    for (int i = 0; i < 4; ++i) e->taps[i] = nullptr;
    return rc;
}

int q2a_test_frontend(q2a_engine * e, const float * pcm_dev, int64_t pcm_stride, const int32_t * n_samples, int n_clips,
                      float * x_dev, void * stream) {
    if (!e || !pcm_dev || !n_samples || !x_dev || n_clips <= 0) return Q2A_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = call_stream(stream);
    int rc = reserve(e, n_clips);
    if (rc) return rc;
    int max_frames = 0;
    rc = prepare_meta(e, n_samples, n_clips, 0, nullptr, nullptr, max_frames, pcm_stride > 0 ? pcm_stride : -1, s);
    if (rc) return rc;
    rc = run_frontend(e, pcm_dev, pcm_stride, n_clips, max_frames, s);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(x_dev, e->X, (size_t) n_clips * e->d.T * e->d.D * 4, hipMemcpyDeviceToDevice, s));
    return Q2A_OK;
}

int q2a_test_pool_ln(q2a_engine * e, const float * x_dev, int n_clips, float * out_dev, void * stream) {
    if (!e || !x_dev || !out_dev || n_clips <= 0) return Q2A_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = call_stream(stream);
    int rc = reserve(e, n_clips);
    if (rc) return rc;
    HIP_TRY(hipEventSynchronize(e->meta_evt));
    for (int c = 0; c < n_clips; ++c) e->meta_host[2 * n_clips + c] = 1;   // every clip "encoded"
    HIP_TRY(hipMemcpyAsync(e->meta + 2 * n_clips, e->meta_host + 2 * n_clips, (size_t) n_clips * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(e->meta_evt, s));
    HIP_TRY(hipMemcpyAsync(e->X, x_dev, (size_t) n_clips * e->d.T * e->d.D * 4, hipMemcpyDeviceToDevice, s));
    q2a_pool_args pa{e->X, n_clips, e->d.T, e->d.D, e->g<const float *>(G_LNP_W), e->g<const float *>(G_LNP_B), out_dev,
                     e->meta + 2 * n_clips};
    LAUNCH(q2a_launch_pool_ln(pa, s));
    return Q2A_OK;
}

int q2a_test_fc1_path(q2a_engine * e, int path) {
    if (!e || path < 0 || path > 2) return Q2A_ERR_ARG;
    e->fc1_path = path;
    return Q2A_OK;
}

int q2a_test_attention(q2a_engine * e, const float * q, const float * k, const float * v, int n_clips, float * out,
                       void * stream) {
    if (!e || n_clips <= 0) return Q2A_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t s = call_stream(stream);
    int rc = reserve(e, n_clips);
    if (rc) return rc;
    const dims & d = e->d;
    const int64_t n = (int64_t) n_clips * d.T * d.D;
    const dim3 g((unsigned) ((n + 255) / 256)), b(256);
    hipLaunchKernelGGL(k_split_hilo, g, b, 0, s, q, e->qh, e->ql, n, Q2A_LOG2E);   // the kernel's log2 units
    hipLaunchKernelGGL(k_split_hilo, g, b, 0, s, k, e->kh, e->kl, n, 1.0f);
    hipLaunchKernelGGL(k_split_hilo, g, b, 0, s, v, e->vt, e->vtl, n, 1.0f);   // V hi / lo row-major (the engine's layout)
    LAUNCH(hipGetLastError());
    q2a_attn_args at{e->qh, e->ql, e->kh, e->kl, e->vt, n_clips, d.T, d.D, d.H, e->TP, nullptr, out};
    at.vtl = e->vtl;
    at.v_rows = 1;
    LAUNCH(q2a_launch_attention(at, s));
    return Q2A_OK;
}

// ---- downstream consumer: the Qwen2-Audio multi-modal projector ---------------------------
// audio_features = Linear(d_model -> text hidden, bias)(embd_enc) (transformers modeling_qwen2_audio.py,
// Qwen2AudioMultiModalProjector; the reference path ends at embd_enc, qwen2-whisper.cpp:2185). Weights from a projector
// file in the ggml container (q2a_write_synthetic_projector layout), run with the encoder's numerics contract for a
// ggml MUL_MAT of that weight type: activations converted per vec_dot_type (fp16 RNE for F16, Q8_K for Q4_K, Q8_0 for
// Q8_0 / Q4_0), exact products, fp32 accumulation in the canonical K order, then + bias in f32 — on the same GEMM.
struct q2a_projector {
    int device = 0;
    hipStream_t stream = nullptr;
    int d_in = 0, d_out = 0, wtype = 0, blk = 0;
    void * wdev = nullptr;          // q2a_pack_linear layout
    uint64_t off[A_COUNT] = {};
    float * bias = nullptr;
    void * ws = nullptr;            // A operand [rows][d_in] fp16 | dy [d_in/blk][MP] | aext [d_in/256][MP][16]
    size_t ws_bytes = 0;
    const uint16_t * gelu = nullptr;   // the GEMM's table argument (unused by STORE_F, kept valid)
};

q2a_projector * q2a_projector_open(const char * path, int device) {
    char err[256] = {0};
    q2a_model_file * mf = q2a_model_file_read(path, err, sizeof(err));
    if (!mf) { set_err("projector %s: %s", path ? path : "(null)", err); return nullptr; }
    const q2a_tensor_desc * wt = q2a_model_file_find(mf, "multi_modal_projector.linear.weight");
    const q2a_tensor_desc * bt = q2a_model_file_find(mf, "multi_modal_projector.linear.bias");
    auto fail = [&](int code, const char * msg) -> q2a_projector * {
        set_err("projector %s: %s", path, msg);
        q2a_model_file_free(mf);
        (void) code;
        return nullptr;
    };
    if (!wt || !bt || wt->n_dims != 2 || bt->type != Q2A_TYPE_F32 || bt->ne[0] != wt->ne[1]) return fail(Q2A_ERR_FORMAT, "missing or malformed tensors");
    const int K = (int) wt->ne[0], N = (int) wt->ne[1];
    if (N % 128 != 0 || K % 256 != 0) return fail(Q2A_ERR_UNSUPPORTED, "d_out must be a multiple of 128, d_in of 256");
    std::vector<uint8_t> packed;
    uint64_t off[A_COUNT];
    if (q2a_pack_linear(mf->data + wt->offset, wt->type, N, K, packed, off) != Q2A_OK)
        return fail(Q2A_ERR_UNSUPPORTED, "weight type not supported (F16, Q4_K, Q8_0, Q4_0)");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) { (void) hipGetLastError(); return fail(Q2A_ERR_HIP, "no such HIP device"); }
    q2a_projector * p = new q2a_projector();
    p->device = device; p->d_in = K; p->d_out = N; p->wtype = wt->type; p->blk = blk_of(wt->type);
    for (int i = 0; i < A_COUNT; ++i) p->off[i] = off[i];
    std::vector<uint16_t> gtab(65536);
    q2a_make_gelu_table(gtab.data());
    bool ok = hipSetDevice(device) == hipSuccess && hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) == hipSuccess &&
              hipMalloc(&p->wdev, packed.size()) == hipSuccess && hipMalloc((void **) &p->bias, (size_t) N * 4) == hipSuccess &&
              hipMalloc((void **) &p->gelu, 65536 * 2) == hipSuccess;
    ok = ok && hipMemcpy(p->wdev, packed.data(), packed.size(), hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(p->bias, mf->data + bt->offset, (size_t) N * 4, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy((void *) p->gelu, gtab.data(), 65536 * 2, hipMemcpyHostToDevice) == hipSuccess;
    q2a_model_file_free(mf);
    if (!ok) {
        (void) hipGetLastError();
        set_err("projector %s: device allocation / upload failed", path);
        q2a_projector_close(p);
        return nullptr;
    }
    return p;
}

void q2a_projector_close(q2a_projector * p) {
    if (!p) return;
    (void) hipSetDevice(p->device);
    if (p->stream) (void) hipStreamSynchronize(p->stream);
    if (p->wdev) (void) hipFree(p->wdev);
    if (p->bias) (void) hipFree(p->bias);
    if (p->gelu) (void) hipFree((void *) p->gelu);
    if (p->ws) (void) hipFree(p->ws);
    if (p->stream) (void) hipStreamDestroy(p->stream);
    delete p;
}

int q2a_projector_get_dims(const q2a_projector * p, int * d_in, int * d_out, int * wtype) {
    if (!p) return Q2A_ERR_ARG;
    if (d_in) *d_in = p->d_in;
    if (d_out) *d_out = p->d_out;
    if (wtype) *wtype = p->wtype;
    return Q2A_OK;
}

int q2a_projector_apply(q2a_projector * p, const float * x, int64_t rows, float * y, void * stream) {
    if (!p || !x || !y || rows <= 0 || rows > (1 << 30) / 4) return Q2A_ERR_ARG;
    HIP_TRY(hipSetDevice(p->device));
    hipStream_t s = call_stream(stream);
    const int M = (int) rows, K = p->d_in, N = p->d_out, blk = p->blk;
    const int64_t MP = (rows + 255) / 256 * 256;
    const size_t a_bytes = ((size_t) M * K * 2 + 255) & ~size_t(255);
    const size_t dy_bytes = blk ? ((size_t) (K / blk) * MP * 4 + 255) & ~size_t(255) : 0;
    const size_t ae_bytes = blk == 256 ? (size_t) (K / 256 + 1) * MP * 32 : 0;
    const size_t need = a_bytes + dy_bytes + ae_bytes;
    if (need > p->ws_bytes) {
        HIP_TRY(hipStreamSynchronize(s));
        if (p->ws) (void) hipFree(p->ws);
        p->ws = nullptr; p->ws_bytes = 0;
        if (hipMalloc(&p->ws, need) != hipSuccess) { (void) hipGetLastError(); set_err("projector workspace of %zu bytes", need); return Q2A_ERR_OOM; }
        p->ws_bytes = need;
    }
    q2a_half * A = (q2a_half *) p->ws;
    float * dy = (float *) ((char *) p->ws + a_bytes);
    q2a_half * aext = (q2a_half *) ((char *) p->ws + a_bytes + dy_bytes);
    if (blk == 0) {
        const int64_t n = (int64_t) M * K;
        hipLaunchKernelGGL(k_to_half, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, x, A, n);
        LAUNCH(hipGetLastError());
    } else {
        q2a_quant_args qa{x, nullptr, M, K, blk == 256 ? 1 : 2, A, dy, aext, (int) MP};
        LAUNCH(q2a_launch_quant_act(qa, s));
    }
    q2a_gemm_args a;
    memset(&a, 0, sizeof(a));
    const char * w = (const char *) p->wdev;
    a.A = A; a.lda = K; a.a_rpg = M; a.a_gstride = 0; a.a_step = 1;
    a.W = (const q2a_half *) (w + p->off[A_W]); a.ldw = K;
    a.M = M; a.N = N; a.K = K;
    a.outF = y; a.ldo = N;
    a.bias = p->bias; a.store_bias = 1;
    a.gelu_tab = p->gelu;
    if (blk) {
        a.nblk = K / blk;
        a.dx = (const float *) (w + p->off[A_DX]);
        a.dy = dy; a.dy_ld = (int) MP;
        if (blk == 256) {
            a.dmin = (const float *) (w + p->off[A_DMIN]);
            a.wext = (const q2a_half *) (w + p->off[A_WEXT]);
            a.beta = (const float *) (w + p->off[A_BETA]);
            a.gamma = (const float *) (w + p->off[A_GAMMA]);
            a.aext = aext;
        }
    }
    LAUNCH(q2a_launch_gemm(a, Q2A_EPI_STORE_F, blk, s));
    return Q2A_OK;
}

}  // extern "C"
