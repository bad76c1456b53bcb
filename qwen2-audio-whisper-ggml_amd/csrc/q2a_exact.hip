// q2a_exact.hip — kernels whose float operation order follows the reference op-for-op (compiled with
// -ffp-contract=off): log-mel frontend, LayerNorm (+ activation quantizers), AvgPool + final LayerNorm.
// All are HBM/latency-bound; they are fused so that each tensor is read once and written once.
#include "q2a_internal.h"
#include <algorithm>
#include <cstdlib>
#include "q2a_quant.h"

#include <math.h>

namespace {

constexpr int NFFT = 400;

// ------------------------------------------------------------------------------------------------
// log-mel (log_mel_spectrogram + worker, qwen2-whisper.cpp:2443-2665)
// One wave per frame. The radix-2 recursion of `fft` (:2465-2507) is unrolled by depth: 16 leaf 25-point
// DFTs (`dft`, :2443-2459) on the decimated inputs x[id + 16n], then 4 combine levels; every butterfly uses
// the reference's expression order, so the power spectrum is bit-identical to the CPU path.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int32_t f2ord(float f) {
    int32_t i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float ord2f(int32_t i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

__global__ __launch_bounds__(256) void k_mel_frames(const q2a_mel_args p) {
    __shared__ float s_in[4][NFFT];
    __shared__ float s_a[4][2 * NFFT];
    __shared__ float s_b[4][2 * NFFT];
    __shared__ float s_pow[4][208];
    __shared__ float s_tw[25][2];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < 25) {   // cos/sin cache entries 16 m (global_cache, qwen2-whisper.cpp:2402-2438)
        s_tw[threadIdx.x][0] = p.tab[NFFT + 16 * threadIdx.x];
        s_tw[threadIdx.x][1] = p.tab[2 * NFFT + 16 * threadIdx.x];
    }
    const int c = blockIdx.y;
    const int i = blockIdx.x * 4 + w;
    const int n = p.n_samples[c];
    const int n_len = (int) (((int64_t) n + 480000) / 160);         // (n + 30 s + 2*200 - 400) / 160 (:2611)
    const int n_s = n + 200;                                         // worker's n_samples (:2621)
    const int n_fft_frames = min(n_s / 160 + 1, n_len);               // (:2522)
    const bool active = i < n_len;
    const bool do_fft = active && i < n_fft_frames;
    const int win = i - p.seek[c];
    const bool in_win = active && win >= 0 && win < p.n_frames_win;
    float * mel_out = p.mel + (int64_t) c * p.n_mel * p.n_frames_win;
    const float * hann = p.tab;
    const float * cosv = p.tab + NFFT;
    const float * sinv = p.tab + 2 * NFFT;

    if (active && !do_fft) {                                         // constant frames (:2565-2571)
        const float v = (float) log10(1e-10);
        if (in_win)
            for (int j = lane; j < p.n_mel; j += 64) mel_out[(int64_t) j * p.n_frames_win + win] = v;
        // every constant frame has the same value: its first one alone enters the clip maximum (thousands of
        // same-address atomics per clip serialised at L2 were most of this kernel's time)
        if (lane == 0 && i == n_fft_frames) atomicMax(p.clip_max + c, f2ord(v));
    }
    // every wave reaches every barrier below; inactive waves just skip the work
    // windowed input: samples_padded = [reflect(200) | pcm | zeros], read up to n_s (:2526-2533)
    const float * pcm = p.pcm + (int64_t) c * p.pcm_stride;
    const int off = i * 160;
    if (do_fft) {
        // the frame's loads issued together at clamped (always readable) addresses, then selected: a load under the
        // reflect / range branches waited alone, seven serial round trips per frame
        constexpr int NT = (NFFT + 63) / 64;
        const float * srcp = n > 0 ? pcm : hann;
        const int imax = max(n - 1, 0);
        float raw[NT], hw[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int j = lane + 64 * t, x = off + j;
            const int src = x < 200 ? 200 - x : x - 200;
            raw[t] = srcp[min(max(src, 0), imax)];
            hw[t] = hann[min(j, NFFT - 1)];
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int j = lane + 64 * t, x = off + j;
            const float v = (x < n_s && (x >= 200 || 200 - x < n)) ? raw[t] : 0.f;
            if (j < NFFT) s_in[w][j] = x < n_s ? hw[t] * v : 0.f;
        }
    }
    __syncthreads();
    // leaves: node id (0..15) takes x[id + 16 n], n = 0..24; DFT step 400/25 = 16. The twiddle index
    // (k t 16) mod 400 = 16 ((k t) mod 25) is stepped incrementally (same index, no integer division) and the 25
    // twiddles it can take are read from an LDS copy of the reference's cos/sin cache entries
    float * cur = s_a[w];
    if (do_fft) {
        for (int o = lane; o < NFFT; o += 64) {
            const int id = o / 25, k = o - 25 * (o / 25);
            float re = 0, im = 0;
            int m = 0;
            for (int t = 0; t < 25; ++t) {
                const float x = s_in[w][id + 16 * t];
                re += x * s_tw[m][0];
                im -= x * s_tw[m][1];
                m += k;
                m = m >= 25 ? m - 25 : m;
            }
            cur[2 * o + 0] = re;
            cur[2 * o + 1] = im;
        }
    }
    __syncthreads();
    // combine levels: depth d has 2^d nodes of length 400/2^d; children of node id: id (even), id + 2^d (odd)
    float * nxt = s_b[w];
    for (int d = 3; d >= 0; --d) {
        const int nn = 1 << d, nc = NFFT >> (d + 1), step = NFFT / (2 * nc);
        if (do_fft) {
            for (int b = lane; b < nn * nc; b += 64) {
                const int id = b / nc, k = b % nc;
                const float * E = cur + 2 * (id * nc);
                const float * O = cur + 2 * ((id + nn) * nc);
                float * out = nxt + 2 * (id * 2 * nc);
                const int idx = k * step;
                const float re = cosv[idx], im = -sinv[idx];
                const float ro = O[2 * k + 0], io = O[2 * k + 1];
                out[2 * k + 0] = E[2 * k + 0] + re * ro - im * io;
                out[2 * k + 1] = E[2 * k + 1] + re * io + im * ro;
                out[2 * (k + nc) + 0] = E[2 * k + 0] - re * ro + im * io;
                out[2 * (k + nc) + 1] = E[2 * k + 1] - re * io - im * ro;
            }
        }
        __syncthreads();
        float * t = cur; cur = nxt; nxt = t;
    }
    // |X|^2 for bins 0..200 (:2540-2542)
    if (do_fft)
        for (int j = lane; j < p.n_bins; j += 64) s_pow[w][j] = cur[2 * j] * cur[2 * j] + cur[2 * j + 1] * cur[2 * j + 1];
    __syncthreads();
    // mel filterbank in double with the reference's 4-way unrolled float partial sums (:2545-2561)
    float lmax = -INFINITY;
    const float * P = s_pow[w];
    for (int j = lane; do_fft && j < p.n_mel; j += 64) {
        const float * f = p.filters + (int64_t) j * p.n_bins;
        double sum = 0.0;
        int k = 0;
        // only the 4-aligned groups holding non-zero filter weights (p.frange): an all-zero group adds exactly
        // +0.0 to a non-negative double sum, so skipping it leaves the reference's result bit for bit
        const int kb = p.frange ? p.frange[j].x : 0;
        const int ke = p.frange ? p.frange[j].y : p.n_bins - 3;
        for (k = kb; k < ke; k += 4) sum += P[k] * f[k] + P[k + 1] * f[k + 1] + P[k + 2] * f[k + 2] + P[k + 3] * f[k + 3];
        for (k = (p.n_bins - 3 + 3) / 4 * 4; k < p.n_bins; k++) sum += P[k] * f[k];   // the reference's tail
        const float v = (float) log10(fmax(sum, 1e-10));
        if (in_win) mel_out[(int64_t) j * p.n_frames_win + win] = v;
        lmax = fmaxf(lmax, v);
    }
    for (int o = 32; o > 0; o >>= 1) lmax = fmaxf(lmax, __shfl_xor(lmax, o));
    // one atomic per workgroup (its four frames' maximum) instead of one per frame
    __shared__ float s_wmax[4];
    if (lane == 0) s_wmax[w] = lmax;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float m4 = fmaxf(fmaxf(s_wmax[0], s_wmax[1]), fmaxf(s_wmax[2], s_wmax[3]));
        if (m4 != -INFINITY) atomicMax(p.clip_max + c, f2ord(m4));
    }
}

// clamp to (max - 8), (x + 4) / 4 (:2633-2649), then write the conv1 operand rows as three fp16 parts. F16 conv kernels:
// [hi | mid | lo] with hi + mid + lo = the f32 value exactly (24 significant bits in three 11-bit pieces; pieces below
// fp16's 2^-24 resolution are lost only for |x| < 2^-1, an absolute error < 2^-25), so the fp16 MFMA conv's products
// are the F32 im2col x F32-upcast-kernel products exactly. F32 kernels (all-F32 files): [hi | lo | hi] against
// [wh | wh | wl] (the product to 22 bits).
__global__ __launch_bounds__(256) void k_mel_norm(const q2a_mel_args p) {
    __shared__ float tile[128][65];
    const int c = blockIdx.y, t0 = blockIdx.x * 64;
    const double mmax = (double) ord2f(p.clip_max[c]) - 8.0;
    const float * mel = p.mel + (int64_t) c * p.n_mel * p.n_frames_win;
    for (int e = threadIdx.x; e < p.n_mel * 64; e += 256) {
        const int j = e / 64, tt = e % 64;
        float v = 0.f;
        if (t0 + tt < p.n_frames_win) {
            v = mel[(int64_t) j * p.n_frames_win + t0 + tt];
            if (v < mmax) v = (float) mmax;
            v = (float) ((v + 4.0) / 4.0);
        }
        tile[j][tt] = v;
    }
    __syncthreads();
    const int nm = p.n_mel;
    q2a_half * xc = p.xc1 + (int64_t) c * (p.n_frames_win + 2) * 3 * nm;
    for (int e = threadIdx.x; e < nm * 64; e += 256) {
        const int tt = e / nm, j = e % nm;
        if (t0 + tt >= p.n_frames_win) continue;
        const float v = tile[j][tt];
        const _Float16 h = (_Float16) v;
        const float r = v - (float) h;             // exact (|r| <= ulp_fp16(v) / 2)
        const _Float16 m = (_Float16) r;
        q2a_half * row = xc + (int64_t) (t0 + tt + 1) * 3 * nm;
        row[j] = h;
        row[nm + j] = m;
        row[2 * nm + j] = p.xc_f32 ? h : (_Float16) (r - (float) m);   // (r - m exact as well)
    }
}

// ------------------------------------------------------------------------------------------------
// LayerNorm (ggml_compute_forward_norm_f32 ggml.c:11941-11990: double sums, eps 1e-5) + affine (MUL, ADD),
// fused with the conversion ggml applies to the next MUL_MAT's src1 (ggml.c:12462-12475):
//   mode 0 fp16 RNE;  mode 1 Q8_K (quantize_row_q8_K_ref ggml-quants.c:3785-3822);
//   mode 2 Q8_0 (x86 quantize_row_q8_0 ggml-quants.c:943-1000: d = amax/127, id = 127/amax, round-half-even).
// One wave per row; lane l owns float4 chunks l, l+64, ... so a 256-block is one float4 per lane.
// ------------------------------------------------------------------------------------------------
// (the f64 steps stay on the LDS pipe: the same butterfly on DPP / permlane swaps, bit-identical, measured slower —
// 9.9 against 9.3 ms per step for the Q4_K LayerNorms, diag/gpurun_r06y.sh — it adds VALU to a VALU-heavy kernel)
__device__ __forceinline__ double wave_sum_d(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// NBQ > 0 (D = 256 NBQ, compile-time): 8 rows per workgroup (512 threads), the LayerNorm weight and bias staged in LDS
// once per workgroup. Q8_K (MODE 1): the NBQ blocks of a row quantized together; the rows' d and bsum operands are
// staged in LDS and stored by the workgroup as whole sectors (32 B of d, 256 B of bsums per block column) — one row's
// 4-B d and 32-B bsum pieces stored by its own wave reach HBM as partial writes (diag/bwbench.hip)
template <int MODE, bool LN, bool HIN, int NBQ>
__device__ __forceinline__ void rownorm_rows(const float * __restrict__ X, int M, int D, const float * __restrict__ g,
                                             const float * __restrict__ b, q2a_half * outH, float * dy, q2a_half * aext,
                                             int nseg, int ld) {
    const int lane = threadIdx.x & 63;
    constexpr int RPB = NBQ ? 8 : 4;   // rows per workgroup
    const int row0 = blockIdx.x * RPB;
    const int row_raw = row0 + (threadIdx.x >> 6);
    if constexpr (!NBQ) {
        if (row_raw >= M) return;
    }
    const int row = min(row_raw, M - 1);   // NBQ: every wave stays for the workgroup's barrier
    const float4 * x4 = (const float4 *) (X + (int64_t) row * D);
    const int nch = D / 4;
    constexpr int MAXC = NBQ ? NBQ : 8;   // float4 chunks per lane (D <= 2048)
    float4 v[MAXC];
    __shared__ float4 sgb[NBQ ? 2 * 64 * NBQ : 1];   // NBQ: LayerNorm weight | bias
    float mean = 0.f, scale = 1.f;
    if (LN) {
        // all of the row's loads first, then the sums: a load and its sum under one `c < nch` branch compiled to a
        // load + vmcnt(0) per chunk, i.e. five serial HBM round trips per row (the summation order is unchanged)
#pragma unroll
        for (int u = 0; u < MAXC; ++u) {
            const int c = lane + 64 * u;
            if (NBQ || c < nch) v[u] = x4[c];
        }
        if constexpr (NBQ > 0) {   // the affine operands into LDS once per workgroup, under the rows' loads
            for (int i = threadIdx.x; i < 2 * 64 * NBQ; i += 512)
                sgb[i] = i < 64 * NBQ ? ((const float4 *) g)[i] : ((const float4 *) b)[i - 64 * NBQ];
        }
        double s = 0.0;
#pragma unroll
        for (int u = 0; u < MAXC; ++u) {
            const int c = lane + 64 * u;
            if (NBQ || c < nch) s += (double) v[u].x + (double) v[u].y + (double) v[u].z + (double) v[u].w;
        }
        s = wave_sum_d(s);
        mean = (float) (s / D);
        double s2 = 0.0;
#pragma unroll
        for (int u = 0; u < MAXC; ++u) {
            const int c = lane + 64 * u;
            if (NBQ || c < nch) {
                v[u].x = v[u].x - mean; v[u].y = v[u].y - mean; v[u].z = v[u].z - mean; v[u].w = v[u].w - mean;
                s2 += (double) (v[u].x * v[u].x) + (double) (v[u].y * v[u].y) + (double) (v[u].z * v[u].z) +
                      (double) (v[u].w * v[u].w);
            }
        }
        s2 = wave_sum_d(s2);
        const float variance = (float) (s2 / D);
        scale = 1.0f / sqrtf(variance + 1e-5f);
    } else if (HIN) {   // fp16 rows (e.g. the GELU output, exactly fp16-valued by the LUT)
        typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
        const h4_t * xh = (const h4_t *) ((const q2a_half *) X + (int64_t) row * D);
        h4_t h[MAXC];   // loads first (see the LN branch), then the conversions
#pragma unroll
        for (int u = 0; u < MAXC; ++u) {
            const int c = lane + 64 * u;
            if (NBQ || c < nch) h[u] = xh[c];
        }
#pragma unroll
        for (int u = 0; u < MAXC; ++u) {
            const int c = lane + 64 * u;
            if (NBQ || c < nch) v[u] = make_float4((float) h[u][0], (float) h[u][1], (float) h[u][2], (float) h[u][3]);
        }
    } else {
#pragma unroll
        for (int u = 0; u < MAXC; ++u) {
            const int c = lane + 64 * u;
            if (NBQ || c < nch) v[u] = x4[c];
        }
    }
    if constexpr (NBQ > 0 && LN) __syncthreads();   // sgb filled
    if constexpr (MODE == 1 && NBQ > 0) {
        // whole row resident: the NBQ Q8_K blocks of the row quantized with interleaved reductions
        float4 y[NBQ];
#pragma unroll
        for (int u = 0; u < NBQ; ++u) {
            if (LN) {
                const float4 gg = sgb[lane + 64 * u], bb = sgb[64 * NBQ + lane + 64 * u];
                y[u].x = (v[u].x * scale) * gg.x + bb.x;
                y[u].y = (v[u].y * scale) * gg.y + bb.y;
                y[u].z = (v[u].z * scale) * gg.z + bb.z;
                y[u].w = (v[u].w * scale) * gg.w + bb.w;
            } else {
                y[u] = v[u];
            }
        }
        __shared__ float sd[8][NBQ];
        __shared__ __attribute__((aligned(16))) q2a_half sa[8][NBQ][16];
        const int r = threadIdx.x >> 6;
        // codes of a clamped duplicate row (past M) are the real last row's: rewriting them changes nothing
        quant_q8k_blocks<NBQ>(y, lane, outH + (int64_t) row * D + 4 * lane, 256, &sd[r][0], 1, &sa[r][0][0], 16);
        __syncthreads();
        const int t = threadIdx.x;
        if (t < NBQ * 8) {     // d: block column u, rows row0 .. row0 + 7 (32 B)
            const int u = t >> 3, rr = t & 7;
            if (row0 + rr < M) dy[(int64_t) u * ld + row0 + rr] = sd[rr][u];
        }
        if (t < NBQ * 64) {    // bsum operand: block column u, 8 rows x 32 B contiguous, 4 B per thread
            const int u = t >> 6, w = t & 63, rr = w >> 3, j2 = w & 7;
            if (row0 + rr < M) *(uint32_t *) (aext + ((int64_t) u * ld + row0 + rr) * 16 + 2 * j2) = *(const uint32_t *) &sa[rr][u][2 * j2];
        }
        return;
    }
    if (NBQ && row_raw >= M) return;   // (after the workgroup's barrier)
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
        const int c = lane + 64 * u;
        if (!NBQ && c >= nch) continue;
        float4 y = v[u];
        if (LN) {
            const float4 gg = NBQ ? sgb[c] : ((const float4 *) g)[c], bb = NBQ ? sgb[64 * NBQ + c] : ((const float4 *) b)[c];
            y.x = (y.x * scale) * gg.x + bb.x;
            y.y = (y.y * scale) * gg.y + bb.y;
            y.z = (y.z * scale) * gg.z + bb.z;
            y.w = (y.w * scale) * gg.w + bb.w;
        }
        q2a_half * o = outH + (int64_t) row * (MODE == 3 ? 3 * D : D) + 4 * c;
        const int m = row / nseg, seg = row - m * nseg;
        if (MODE == 0) {
            o[0] = (_Float16) y.x; o[1] = (_Float16) y.y; o[2] = (_Float16) y.z; o[3] = (_Float16) y.w;
        } else if (MODE == 4) {   // bf16-activation mode: RNE to bf16, bits in the fp16-typed slots
            o[0] = __builtin_bit_cast(_Float16, (__bf16) y.x); o[1] = __builtin_bit_cast(_Float16, (__bf16) y.y);
            o[2] = __builtin_bit_cast(_Float16, (__bf16) y.z); o[3] = __builtin_bit_cast(_Float16, (__bf16) y.w);
        } else if (MODE == 3) {
            const float yy[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const _Float16 h = (_Float16) yy[e];
                o[e] = h;
                o[D + e] = (_Float16) (yy[e] - (float) h);
                o[2 * D + e] = h;
            }
        } else if (MODE == 1) {
            const int bf = seg * (D / 256) + u;
            quant_q8k_block(y, lane, o, dy + (int64_t) bf * ld + m, aext + ((int64_t) bf * ld + m) * 16);
        } else {
            const int bf = seg * (D / 32) + (4 * c) / 32;
            quant_q80_block(y, lane, o, dy + (int64_t) bf * ld + m);
        }
    }
}

template <int MODE, bool LN, bool HIN = false>
__global__ __launch_bounds__(256) void k_rownorm(const float * __restrict__ X, int M, int D, const float * __restrict__ g,
                                                 const float * __restrict__ b, q2a_half * outH, float * dy, q2a_half * aext,
                                                 int nseg, int ld) {
    rownorm_rows<MODE, LN, HIN, 0>(X, M, D, g, b, outH, dy, aext, nseg, ld);
}

// rows of D = 1280 (the model width): compile-time row length, 8 rows per 512-thread workgroup
template <int MODE, bool LN>
__global__ __launch_bounds__(512) void k_rownorm5(
    const float * __restrict__ X, int M, int D, const float * __restrict__ g, const float * __restrict__ b, q2a_half * outH,
    float * dy, q2a_half * aext, int nseg, int ld) {
    rownorm_rows<MODE, LN, false, 5>(X, M, D, g, b, outH, dy, aext, nseg, ld);
}

// Q8_K quantizer for fp16 rows (the fc1 GELU output), 16 lanes per 256-block: a wave quantizes four blocks at
// once with 16-B loads and stores (quant_q8k_row16: the arithmetic of quant_q8k_block, shorter reduction chains)
__global__ __launch_bounds__(256) void k_quant_q8k_h16(const q2a_half * __restrict__ X, int64_t nblocks, int bpr,
                                                       q2a_half * outH, float * dy, q2a_half * aext, int ld) {
    const int lane = threadIdx.x & 63, sub = lane & 15;
    const int64_t blk = ((int64_t) blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + (lane >> 4);
    if (blk >= nblocks) return;
    const int64_t m = blk / bpr;
    const int bf = (int) (blk - m * bpr);
    typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
    const h8_t * src = (const h8_t *) (X + blk * 256 + sub * 16);
    const h8_t h0 = __builtin_nontemporal_load(src), h1 = __builtin_nontemporal_load(src + 1);
    float v[16];
#pragma unroll
    for (int e = 0; e < 8; ++e) { v[e] = (float) h0[e]; v[8 + e] = (float) h1[e]; }
    quant_q8k_row16(v, sub, outH + blk * 256 + sub * 16, dy + (int64_t) bf * ld + m, aext + ((int64_t) bf * ld + m) * 16);
}

// GELU + Q8_K of the fc1 pre-activation (Q2A_EPI_PRE_H output, fp16). Persistent workgroups of 8 waves stage ggml's
// whole 64 Ki-entry fp16 GELU table (128 KiB) into LDS once, so an element is one lookup at its own bits: entries for
// h >= 10 are h itself (ggml_vec_gelu_f32's x >= 10 branch: tanhf saturates to 1), entries for h <= -10 are -0 (the
// x <= -10 branch's +0 up to the sign, which the Q8_K codes do not see), and the -inf entry (NaN in the table) is
// patched to +0. The kernel is VALU-bound once its stores are whole
// sectors (~19 -> ~13 VALU per element with the direct index).
//
// Work unit = one block column bf of 16 consecutive rows, four wave-iterations of 4 rows (16 lanes per 256-block,
// 16 values per lane): every side store is whole sectors — the bsum operand 128 B (4 rows x 32 B) per iteration, d
// 64 B (16 rows) per unit. Scattered 4-B d / 32-B bsum stores (one block per lane group) went to HBM as single
// partial writes: 25 % of the kernel (diag/bwbench.hip). Input: the 2 KiB of an iteration arrive by LDS-DMA one
// iteration ahead (register prefetch cannot run ahead: vmcnt retires in order and counts the stores, and with loads
// and stores pending the compiler waits vmcnt(0), i.e. for the previous iteration's stores). Per iteration 2 DMA +
// 3 stores (+1 for d on the unit's last iteration).
// Measured alternative (diag/experiment_knobs_r05.patch, Q2A_GELU_COMPACT): the |x| < 10 image of the table only (75 KiB: +0..+10 | -0..-10, what the GEMM epilogues
// stage), ggml's two branches as selects (x >= 10 -> x; x <= -10 -> the table's own -0, +0 for -inf), NaN inputs from
// the full table in global memory (a wave-uniform branch that real data never takes) — and 16 waves per CU instead of
// 8 (twice the input DMA in flight) in the LDS the full 128 KiB table held. Measured round 5 (diag/gpurun_r05f.sh):
// bit-identical, quant_act 17.26 -> 19.2 ms per step (index arithmetic + selects cost more than the DMA depth gains);
// a timing build with conflict-free reads bounds the whole bank-conflict cost at 0.3 ms per step. Diagnostic only.
constexpr int GQ_THREADS = 512;
constexpr int GQ_WAVES = GQ_THREADS / 64;
typedef __attribute__((address_space(3))) void * lds_vptr_t;
__global__ __launch_bounds__(GQ_THREADS) void k_gelu_quant_q8k_h16(const q2a_half * __restrict__ X, int M, int bpr,
                                                                   const uint16_t * __restrict__ gelu_tab, q2a_half * outH,
                                                                   float * dy, q2a_half * aext, int ld) {
    __shared__ __attribute__((aligned(16))) uint16_t lut[65536];
    __shared__ __attribute__((aligned(16))) char stage[GQ_WAVES][2048];
    for (int i = threadIdx.x; i < 65536 / 8; i += GQ_THREADS) ((uint4 *) lut)[i] = ((const uint4 *) gelu_tab)[i];
    __syncthreads();
    if (threadIdx.x == 0) lut[0xFC00] = 0;   // -inf (x below the fp16 range) -> +0
    __syncthreads();
    const int lane = threadIdx.x & 63, sub = lane & 15, grp = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t K = (int64_t) bpr * 256;
    // work position of iteration t, wave-uniform: unit u = blockIdx * GQ_WAVES + wave + (t >> 2) * stride = block
    // column bf of the 16-row group c (u = c * bpr + bf), quarter q = t & 3. Advanced incrementally — a division per
    // iteration was a 64-bit divide expansion of ~170 scalar instructions, twice per iteration (M * K < 2^31: 32 bits)
    const int nunits = ((M + 15) / 16) * bpr;
    const int stride = (int) gridDim.x * GQ_WAVES;
    const int s_c = stride / bpr, s_bf = stride - s_c * bpr;
    const int c_last = (nunits - 1) / bpr, bf_last = nunits - 1 - c_last * bpr;
    struct pos_t { int u, c, bf, q; };
    auto advance = [&](pos_t & w) {
        if (++w.q == 4) {
            w.q = 0;
            w.u += stride;
            w.c += s_c;
            w.bf += s_bf;
            if (w.bf >= bpr) { w.bf -= bpr; ++w.c; }
        }
    };
    // rows r0 .. r0 + 3 of block column bf for a position (past the last unit: the last unit, a harmless re-load)
    auto place = [&](const pos_t & w, int & r0, int & bf) {
        const bool past = w.u > nunits - 1;
        bf = past ? bf_last : w.bf;
        r0 = (past ? c_last : w.c) * 16 + w.q * 4;
    };
    char * st = &stage[wave][0];
    // 2 x 1 KiB pieces: piece i = rows r0 + 2i (lanes 0-31) and r0 + 2i + 1 (lanes 32-63), 16 B per lane
    auto dma = [&](const pos_t & w) {
        int r0, bf;
        place(w, r0, bf);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int row = min(r0 + 2 * i + (lane >> 5), M - 1);   // past the end: harmless re-loads keep the counts
            __builtin_amdgcn_global_load_lds((const void *) (X + row * K + bf * 256 + (lane & 31) * 8), (lds_vptr_t) (st + i * 1024),
                                             16, 0, 0);
        }
    };
    const uint32_t st0 = (uint32_t) (uintptr_t) (const __attribute__((address_space(3))) char *) st;
    const uint32_t lut0 = (uint32_t) (uintptr_t) (const __attribute__((address_space(3))) char *) lut;
    typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
    typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
    pos_t cur;
    cur.u = (int) blockIdx.x * GQ_WAVES + wave;
    cur.c = cur.u / bpr;
    cur.bf = cur.u - cur.c * bpr;
    cur.q = 0;
    pos_t nxt = cur;
    advance(nxt);
    if (cur.u < nunits) dma(cur);
    bool wait_all = true;
    float dd = 0.f;   // lane L (0..15): d of row 16c + L, filled over the unit's four iterations
    for (; cur.u < nunits; cur = nxt, advance(nxt)) {
        // this iteration's DMA; the previous iteration's 3 or 4 stores may still be out (all of them after a ragged one)
        if (wait_all) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        // lane (grp, sub): values 16 sub .. 16 sub + 15 of row r0 + grp
        h8_t h0, h1;
        const uint32_t a = st0 + (uint32_t) (grp * 512 + sub * 32);
        asm volatile("ds_read_b128 %0, %1" : "=v"(h0) : "v"(a));
        asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(h1) : "v"(a));
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(h0), "+v"(h1) :: "memory");
        dma(nxt);                                            // the buffer's next fill (its data is in registers)
        // the vmcnt(3) at the top of the next iteration counts on this DMA being issued BEFORE this iteration's 3
        // stores: pin the order (no IR motion of memory ops across the fence, no machine scheduling across the barrier)
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        int r0, bf;
        place(cur, r0, bf);
        wait_all = r0 + 4 > M;
        // 16 table reads back to back behind one wait (a compiler-visible lookup is placed per element with its own
        // wait); the index is the element's own bits
        uint32_t g[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const _Float16 he = e < 8 ? h0[e] : h1[e - 8];
            uint16_t u;
            __builtin_memcpy(&u, &he, 2);
            const uint32_t ix = u;
            asm volatile("ds_read_u16 %0, %1" : "=v"(g[e]) : "v"(lut0 + ix * 2));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(g[0]), "+v"(g[1]), "+v"(g[2]), "+v"(g[3]), "+v"(g[4]), "+v"(g[5]), "+v"(g[6]),
                     "+v"(g[7]), "+v"(g[8]), "+v"(g[9]), "+v"(g[10]), "+v"(g[11]), "+v"(g[12]), "+v"(g[13]), "+v"(g[14]), "+v"(g[15]));
        float v[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const uint16_t gg = (uint16_t) g[e];
            _Float16 gh;
            __builtin_memcpy(&gh, &gg, 2);
            v[e] = (float) gh;
        }
        const int row = r0 + grp;
        float d;
        int sb;
        quant_q8k_row16c(v, sub, outH + row * K + bf * 256 + sub * 16, row < M, d, sb);
        if ((sub & 1) == 0 && row < M) {   // bsum32 of sub-block sub / 2 as (hi, lo): rows r0 .. r0 + 3 = 128 B
            const int hi = (sb >= 0) ? (sb >> 6) : -((-sb + 63) >> 6);   // floor(s / 64)
            const int lo = sb - 64 * hi;
            *(h2_t *) (aext + ((int64_t) bf * ld + row) * 16 + sub) = h2_t{(_Float16) (float) hi, (_Float16) (float) lo};
        }
        const int q = cur.q;
        const float dq = __shfl(d, (lane & 3) * 16);         // d of row r0 + (lane & 3)
        if ((lane >> 2) == q) dd = dq;
        if (q == 3) {   // d of the unit's 16 rows: one 64-B store
            const int r = r0 - 12 + lane;
            if (lane < 16 && r < M) dy[(int64_t) bf * ld + r] = dd;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the trailing re-load lands before the workgroup's LDS is freed
}

// AvgPool1d(k=2,s=2) over time (ggml.c:15077-15125: drow = 0; += a; += b; /= 2) + final LayerNorm -> f32
__global__ __launch_bounds__(256) void k_pool_ln(const q2a_pool_args p) {
    const int lane = threadIdx.x & 63;
    const int TO = p.T / 2;
    const int orow = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (orow >= p.n_clips * TO) return;
    const int c = orow / TO, t = orow % TO;
    if (!p.clip_ok[c]) return;
    const float4 * a4 = (const float4 *) (p.X + ((int64_t) c * p.T + 2 * t) * p.D);
    const float4 * b4 = (const float4 *) (p.X + ((int64_t) c * p.T + 2 * t + 1) * p.D);
    const int nch = p.D / 4;
    constexpr int MAXC = 8;
    float4 v[MAXC], bv[MAXC];
    // the rows' loads at clamped chunk indices (always readable) before any arithmetic: under the `ch < nch` branches
    // each chunk's loads waited alone
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
        const int ch = min(lane + 64 * u, nch - 1);
        v[u] = a4[ch];
        bv[u] = b4[ch];
    }
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
        const int ch = lane + 64 * u;
        if (ch < nch) {
            const float4 a = v[u], b = bv[u];
            v[u].x = ((0.f + a.x) + b.x) / 2; v[u].y = ((0.f + a.y) + b.y) / 2;
            v[u].z = ((0.f + a.z) + b.z) / 2; v[u].w = ((0.f + a.w) + b.w) / 2;
            s += (double) v[u].x + (double) v[u].y + (double) v[u].z + (double) v[u].w;
        }
    }
    s = wave_sum_d(s);
    const float mean = (float) (s / p.D);
    double s2 = 0.0;
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
        const int ch = lane + 64 * u;
        if (ch < nch) {
            v[u].x -= mean; v[u].y -= mean; v[u].z -= mean; v[u].w -= mean;
            s2 += (double) (v[u].x * v[u].x) + (double) (v[u].y * v[u].y) + (double) (v[u].z * v[u].z) +
                  (double) (v[u].w * v[u].w);
        }
    }
    s2 = wave_sum_d(s2);
    const float scale = 1.0f / sqrtf((float) (s2 / p.D) + 1e-5f);
    float4 * o4 = (float4 *) (p.out + ((int64_t) c * TO + t) * p.D);
    // affine operands likewise (clamped, all in flight), then the stores
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
        const int ch = min(lane + 64 * u, nch - 1);
        const float4 gg = ((const float4 *) p.g)[ch], bb = ((const float4 *) p.b)[ch];
        float4 y;
        y.x = (v[u].x * scale) * gg.x + bb.x;
        y.y = (v[u].y * scale) * gg.y + bb.y;
        y.z = (v[u].z * scale) * gg.z + bb.z;
        y.w = (v[u].w * scale) * gg.w + bb.w;
        v[u] = y;
    }
#pragma unroll
    for (int u = 0; u < MAXC; ++u) {
        const int ch = lane + 64 * u;
        if (ch < nch) o4[ch] = v[u];
    }
}

}  // namespace

// per mel filter: [first, end) of the 4-aligned bin groups of the reference's unrolled sum (k < n_bins - 3) that
// hold a non-zero weight (an empty range when none do)
__global__ void k_filter_ranges(const float * filters, int n_mel, int n_bins, int2 * out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_mel) return;
    const float * f = filters + (int64_t) j * n_bins;
    int first = -1, last = -1;
    const int kt = (n_bins - 3 + 3) / 4 * 4;   // bins covered by the 4-way groups (where that loop exits)
    for (int k = 0; k < kt; ++k)
        if (f[k] != 0.0f) { if (first < 0) first = k; last = k; }
    out[j] = first < 0 ? make_int2(0, 0) : make_int2(first / 4 * 4, last / 4 * 4 + 4);
}

hipError_t q2a_launch_filter_ranges(const float * filters, int n_mel, int n_bins, int2 * out, hipStream_t s) {
    hipLaunchKernelGGL(k_filter_ranges, dim3((n_mel + 127) / 128), dim3(128), 0, s, filters, n_mel, n_bins, out);
    return hipGetLastError();
}

hipError_t q2a_launch_mel(const q2a_mel_args & a, hipStream_t s) {
    if (a.n_bins > 208 || a.n_mel > 128 * 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_mel_frames, dim3((a.max_frames + 3) / 4, a.n_clips), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_mel_norm, dim3((a.n_frames_win + 63) / 64, a.n_clips), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t q2a_launch_layernorm(const q2a_ln_args & a, hipStream_t s) {
    if (a.D % 4 != 0 || a.D > 2048) return hipErrorInvalidValue;
    if (a.mode == 1 && a.D % 256) return hipErrorInvalidValue;
    if (a.mode == 2 && a.D % 32) return hipErrorInvalidValue;
    const dim3 grid((a.M + 3) / 4), blk(256), grid8((a.M + 7) / 8), blk8(512);
    const bool d1280 = a.D == 1280;   // the model width: compile-time row length (k_rownorm NBQ = 5)
    if (a.mode == 0 && d1280)
        hipLaunchKernelGGL((k_rownorm5<0, true>), grid8, blk8, 0, s, a.X, a.M, a.D, a.g, a.b, a.outH, a.dy, a.aext, 1, a.dy_ld);
    else if (a.mode == 4 && d1280)
        hipLaunchKernelGGL((k_rownorm5<4, true>), grid8, blk8, 0, s, a.X, a.M, a.D, a.g, a.b, a.outH, a.dy, a.aext, 1, a.dy_ld);
    else if (a.mode == 2 && d1280)
        hipLaunchKernelGGL((k_rownorm5<2, true>), grid8, blk8, 0, s, a.X, a.M, a.D, a.g, a.b, a.outH, a.dy, a.aext, 1, a.dy_ld);
    else if (a.mode == 0) hipLaunchKernelGGL((k_rownorm<0, true>), grid, blk, 0, s, a.X, a.M, a.D, a.g, a.b, a.outH, a.dy, a.aext, 1, a.dy_ld);
    else if (a.mode == 3) hipLaunchKernelGGL((k_rownorm<3, true>), grid, blk, 0, s, a.X, a.M, a.D, a.g, a.b, a.outH, a.dy, a.aext, 1, a.dy_ld);
    else if (a.mode == 4) hipLaunchKernelGGL((k_rownorm<4, true>), grid, blk, 0, s, a.X, a.M, a.D, a.g, a.b, a.outH, a.dy, a.aext, 1, a.dy_ld);
    else if (a.mode == 1 && d1280)
        hipLaunchKernelGGL((k_rownorm5<1, true>), grid8, blk8, 0, s, a.X, a.M, a.D, a.g, a.b, a.outH, a.dy, a.aext, 1, a.dy_ld);
    else if (a.mode == 1) hipLaunchKernelGGL((k_rownorm<1, true>), grid, blk, 0, s, a.X, a.M, a.D, a.g, a.b, a.outH, a.dy, a.aext, 1, a.dy_ld);
    else hipLaunchKernelGGL((k_rownorm<2, true>), grid, blk, 0, s, a.X, a.M, a.D, a.g, a.b, a.outH, a.dy, a.aext, 1, a.dy_ld);
    return hipGetLastError();
}

hipError_t q2a_launch_gelu_quant_q8k(const q2a_half * XH, int M, int K, const uint16_t * gelu_tab, q2a_half * outH,
                                     float * dy, q2a_half * aext, int dy_ld, hipStream_t s) {
    if (K % 256 != 0 || M <= 0 || (int64_t) M * K >= ((int64_t) 1 << 31)) return hipErrorInvalidValue;
    int dev = 0, ncu = 256;
    (void) hipGetDevice(&dev);
    (void) hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t units = (int64_t) ((M + 15) / 16) * (K / 256);
    const unsigned grid = (unsigned) std::min<int64_t>((units + GQ_WAVES - 1) / GQ_WAVES, (int64_t) ncu);   // 144 KiB each
    hipLaunchKernelGGL(k_gelu_quant_q8k_h16, dim3(grid), dim3(GQ_THREADS), 0, s, XH, M, K / 256, gelu_tab, outH, dy, aext, dy_ld);
    return hipGetLastError();
}

hipError_t q2a_launch_quant_act(const q2a_quant_args & a, hipStream_t s) {
    if (a.K % 256 != 0 || a.K > 8192) return hipErrorInvalidValue;
    // rows longer than 2048 (fc2 input, K = 4D) are processed as K/1024 independent 1024-wide segments
    const int seg = a.K > 2048 ? 1024 : a.K;
    const int nseg = a.K / seg;
    const dim3 grid((a.M * nseg + 3) / 4), blk(256);
    // view X as [M*nseg][seg]: contiguous, and the block structure (256 / 32) never straddles a segment
    const float * X = a.XH ? (const float *) a.XH : a.X;
    if (a.mode == 1 && a.XH) {
        const int64_t nb = (int64_t) a.M * (a.K / 256);
        hipLaunchKernelGGL(k_quant_q8k_h16, dim3((unsigned) ((nb + 15) / 16)), dim3(256), 0, s, a.XH, nb, a.K / 256, a.outH,
                           a.dy, a.aext, a.dy_ld);
    } else if (a.mode == 1 && a.XH) {
        hipLaunchKernelGGL((k_rownorm<1, false, true>), grid, blk, 0, s, X, a.M * nseg, seg, nullptr, nullptr, a.outH, a.dy, a.aext, nseg, a.dy_ld);
    } else if (a.mode == 2 && a.XH) {
        hipLaunchKernelGGL((k_rownorm<2, false, true>), grid, blk, 0, s, X, a.M * nseg, seg, nullptr, nullptr, a.outH, a.dy, a.aext, nseg, a.dy_ld);
    } else if (a.mode == 1 && seg == 1280 && nseg == 1) {   // f32 rows of D = 1280 (attention output): 5 blocks interleaved
        hipLaunchKernelGGL((k_rownorm5<1, false>), dim3((a.M + 7) / 8), dim3(512), 0, s, X, a.M, seg, nullptr, nullptr,
                           a.outH, a.dy, a.aext, 1, a.dy_ld);
    } else if (a.mode == 1) {
        hipLaunchKernelGGL((k_rownorm<1, false>), grid, blk, 0, s, X, a.M * nseg, seg, nullptr, nullptr, a.outH, a.dy, a.aext, nseg, a.dy_ld);
    } else if (a.mode == 2) {
        hipLaunchKernelGGL((k_rownorm<2, false>), grid, blk, 0, s, X, a.M * nseg, seg, nullptr, nullptr, a.outH, a.dy, a.aext, nseg, a.dy_ld);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t q2a_launch_pool_ln(const q2a_pool_args & a, hipStream_t s) {
    if (a.D % 4 != 0 || a.D > 2048) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_pool_ln, dim3((a.n_clips * (a.T / 2) + 3) / 4), dim3(256), 0, s, a);
    return hipGetLastError();
}
