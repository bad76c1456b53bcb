// ggml-q2a.hip — the MI355X ggml backend (include/ggml-q2a.h): buffer type, buffer, backend, device and registry
// vtables of ggml/src/ggml-backend-impl.h:15-224 over HIP device memory, and a graph executor that runs every node
// of the reference's conv and encoder graphs (src/qwen2-whisper.cpp:1892-2203) on gfx950.
//
// Node kinds and how they run here:
//   MUL_MAT, weight × activation (F16 / Q4_K / Q8_0 / Q4_0 weights, F32 rows): ggml's activation conversion
//       (fp16 RNE / Q8_K / Q8_0, the same quantizer kernels as the fused engine) + the engine's MFMA GEMM
//       (q2a_launch_gemm) on the weight repacked once into the GEMM layout (cached per weight tensor, dropped when
//       the tensor's bytes are written again).
//   MUL_MAT, everything else (conv im2col × F16/F32 kernel, per-head K·Q and V·softmax, F32 weights): an exact-f32
//       batched GEMM on v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate: ggml_vec_dot_f32 products, ggml.c:12348).
//       With an F16 src0, src1 is rounded to fp16 first (ggml's vec_dot_type conversion, ggml.c:12462-12475).
//   KQ -> SOFT_MAX -> KQV with K, Q, V views of the QKV projections: the fused flash kernel of the engine
//       (k_attn: F32-class scores from hi/lo fp16 halves, online softmax), when the chain matches exactly.
//   IM2COL (ggml.c:14717), NORM (:11941, double sums), SOFT_MAX (:13854, double sum), GELU (fp16 table,
//       :2556-2570), ADD / MUL with broadcast, SCALE, CONT/CPY/DUP (strided), POOL_1D avg (:15077): elementwise /
//       row kernels below, with the CPU kernels' float operation order.
// Views, reshapes, permutes and transposes are free. Compiled with -ffp-contract=off (exact op order).
#include "ggml-q2a.h"
#include "ggml-backend-impl.h"

#include "q2a_format.h"
#include "q2a_internal.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#define Q2A_HIP(x)                                                                                   \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) GGML_ABORT("ggml-q2a: %s failed: %s", #x, hipGetErrorString(e_));     \
    } while (0)

#define Q2A_LOG_ERROR(...) fprintf(stderr, __VA_ARGS__)

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------------
struct tview {            // a strided 4-D view: element (i0,i1,i2,i3) at base + i0*nb0 + i1*nb1 + i2*nb2 + i3*nb3
    char * base;
    int64_t ne[4];
    int64_t nb[4];
};

__device__ __forceinline__ int64_t voff(const tview & t, int64_t i0, int64_t i1, int64_t i2, int64_t i3) {
    return i0 * t.nb[0] + i1 * t.nb[1] + i2 * t.nb[2] + i3 * t.nb[3];
}

__device__ __forceinline__ float ld_as_f32(const char * p, int type) {
    if (type == GGML_TYPE_F16) return (float) *(const _Float16 *) p;
    return *(const float *) p;
}
__device__ __forceinline__ void st_from_f32(char * p, int type, float v) {
    if (type == GGML_TYPE_F16) *(_Float16 *) p = (_Float16) v;
    else *(float *) p = v;
}

// dst = src (any strides, F32/F16 either side), one thread per element of dst's logical shape. I = uint32_t when
// the element count fits (32-bit divisions: several times cheaper than the 64-bit ones)
template <typename I>
__global__ void k_copy(tview s, int st, tview d, int dt, int64_t n) {
    const I i = (I) ((int64_t) blockIdx.x * blockDim.x + threadIdx.x);
    if ((int64_t) i >= n) return;
    const I i0 = i % (I) d.ne[0], r = i / (I) d.ne[0];
    const I i1 = r % (I) d.ne[1], r2 = r / (I) d.ne[1];
    const I i2 = r2 % (I) d.ne[2], i3 = r2 / (I) d.ne[2];
    // ggml_dup walks both tensors in their own logical (row-major) element order; with equal element counts the
    // flat index i maps to the source's own (i0, i1, i2, i3)
    const I j0 = i % (I) s.ne[0], q = i / (I) s.ne[0];
    const I j1 = q % (I) s.ne[1], q2 = q / (I) s.ne[1];
    const I j2 = q2 % (I) s.ne[2], j3 = q2 / (I) s.ne[2];
    const char * sp = s.base + voff(s, j0, j1, j2, j3);
    char * dp = d.base + voff(d, i0, i1, i2, i3);
    if (st == dt && st == GGML_TYPE_F16) *(uint16_t *) dp = *(const uint16_t *) sp;
    else st_from_f32(dp, dt, ld_as_f32(sp, st));
}

// dst = a (op) b with b broadcast (ggml_can_repeat), F32. op 0 add, 1 mul
template <int OP>
__global__ void k_binary(tview a, tview b, tview d, int64_t n) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t i0 = i % d.ne[0], r = i / d.ne[0];
    const int64_t i1 = r % d.ne[1], r2 = r / d.ne[1];
    const int64_t i2 = r2 % d.ne[2], i3 = r2 / d.ne[2];
    const float x = *(const float *) (a.base + voff(a, i0, i1, i2, i3));
    const float y = *(const float *) (b.base + voff(b, i0 % b.ne[0], i1 % b.ne[1], i2 % b.ne[2], i3 % b.ne[3]));
    *(float *) (d.base + voff(d, i0, i1, i2, i3)) = OP == 0 ? x + y : x * y;
}

// unary F32: 0 scale (ggml_vec_scale_f32), 1 GELU (ggml_vec_gelu_f32 with GGML_GELU_FP16, ggml.c:2556-2570)
template <int OP>
__global__ void k_unary(tview a, tview d, int64_t n, float scale, const uint16_t * gelu_tab) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t i0 = i % d.ne[0], r = i / d.ne[0];
    const int64_t i1 = r % d.ne[1], r2 = r / d.ne[1];
    const int64_t i2 = r2 % d.ne[2], i3 = r2 / d.ne[2];
    const float x = *(const float *) (a.base + voff(a, i0, i1, i2, i3));
    float y;
    if (OP == 0) {
        y = x * scale;
    } else {
        if (x <= -10.0f) y = 0.0f;
        else if (x >= 10.0f) y = x;
        else {
            const _Float16 h = (_Float16) x;
            uint16_t u;
            __builtin_memcpy(&u, &h, 2);
            const uint16_t g = gelu_tab[u];
            _Float16 gh;
            __builtin_memcpy(&gh, &g, 2);
            y = (float) gh;
        }
    }
    *(float *) (d.base + voff(d, i0, i1, i2, i3)) = y;
}

// Row-wise fast path of ADD / MUL (b broadcast per ggml_can_repeat with b.ne0 == ne0 or 1), SCALE and GELU when
// every operand's rows are f32-contiguous: one wave per row, the row index decomposed once per wave in 32 bits (the
// generic kernels above pay six 64-bit divisions per element), float4 accesses when rows are 16-B aligned.
// OP: 0 add, 1 mul, 2 scale, 3 GELU. Same float operations as the generic kernels.
// (the table read unconditional, the range branches as selects: inside the branches each read waited alone)
__device__ __forceinline__ float gelu_tab_f(float x, const uint16_t * gelu_tab) {
    const _Float16 h = (_Float16) x;
    uint16_t u;
    __builtin_memcpy(&u, &h, 2);
    const uint16_t g = gelu_tab[u];
    _Float16 gh;
    __builtin_memcpy(&gh, &g, 2);
    return x <= -10.0f ? 0.0f : x >= 10.0f ? x : (float) gh;
}

template <int OP, bool V4>
__global__ __launch_bounds__(256) void k_rows(tview a, tview b, tview d, int nrows, float scale, const uint16_t * gelu_tab) {
    const int r = (int) blockIdx.x * 4 + (int) (threadIdx.x >> 6);
    if (r >= nrows) return;
    const int lane = threadIdx.x & 63;
    const int ne0 = (int) d.ne[0], ne1 = (int) d.ne[1], ne2 = (int) d.ne[2];
    const int i1 = r % ne1, t = r / ne1, i2 = t % ne2, i3 = t / ne2;
    const float * x = (const float *) (a.base + i1 * a.nb[1] + i2 * a.nb[2] + i3 * a.nb[3]);
    float * y = (float *) (d.base + i1 * d.nb[1] + i2 * d.nb[2] + i3 * d.nb[3]);
    const float * z = x;
    bool zs = false;
    if (OP < 2) {
        z = (const float *) (b.base + (i1 % (int) b.ne[1]) * b.nb[1] + (i2 % (int) b.ne[2]) * b.nb[2] +
                             (i3 % (int) b.ne[3]) * b.nb[3]);
        zs = b.ne[0] == 1;
    }
    auto f = [&](float u, float v) -> float {
        if (OP == 0) return u + v;
        if (OP == 1) return u * v;
        if (OP == 2) return u * scale;
        return gelu_tab_f(u, gelu_tab);
    };
    if (V4) {
        const int n4 = ne0 >> 2;
        for (int j = lane; j < n4; j += 64) {
            const f4 u = ((const f4 *) x)[j];
            f4 v = u;
            if (OP < 2) v = zs ? f4{z[0], z[0], z[0], z[0]} : ((const f4 *) z)[j];
            f4 o;
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] = f(u[k], v[k]);
            ((f4 *) y)[j] = o;
        }
    } else {
        for (int j = lane; j < ne0; j += 64) y[j] = f(x[j], OP < 2 ? z[zs ? 0 : j] : 0.0f);
    }
}

__device__ __forceinline__ double block_sum_d(double v, double * red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    double t = 0.0;
    for (int i = 0; i < (int) (blockDim.x >> 6); ++i) t += red[i];
    return t;
}
__device__ __forceinline__ float block_max_f(float v, float * red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    float t = -INFINITY;
    for (int i = 0; i < (int) (blockDim.x >> 6); ++i) t = fmaxf(t, red[i]);
    return t;
}

// NORM over ne0 (ggml_compute_forward_norm_f32, ggml.c:11941-11990): mean and variance with double sums,
// y = (x - mean) * (1/sqrtf(var + eps)). One block per row.
__global__ __launch_bounds__(256) void k_norm(tview a, tview d, float eps) {
    __shared__ double red[4];
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % a.ne[1], i2 = (r / a.ne[1]) % a.ne[2], i3 = r / (a.ne[1] * a.ne[2]);
    const float * x = (const float *) (a.base + voff(a, 0, i1, i2, i3));
    float * y = (float *) (d.base + voff(d, 0, i1, i2, i3));
    const int n = (int) a.ne[0];
    double s = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += (double) x[i];
    s = block_sum_d(s, red);
    const float mean = (float) (s / n);
    double s2 = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float v = x[i] - mean;
        s2 += (double) (v * v);
    }
    s2 = block_sum_d(s2, red);
    const float variance = (float) (s2 / n);
    const float scale = 1.0f / sqrtf(variance + eps);
    for (int i = threadIdx.x; i < n; i += blockDim.x) y[i] = (x[i] - mean) * scale;
}

// NORM (+ the MUL by the LayerNorm weight and ADD of its bias when the graph chains them, qwen2-whisper.cpp:2002-2006)
// with one wave per row and the row held in registers (ne0 <= 2048): one HBM read instead of three and no block
// barriers. Mean and variance are double sums (ggml.c:11941-11990); y = (x - mean) * scale, then y * w, then + b,
// each rounded to f32 (no contraction). V4: ne0 % 4 == 0 and 16-B aligned rows.
template <bool AFF, bool V4>
__global__ __launch_bounds__(256) void k_norm_row(tview a, tview d, float eps, const float * w, const float * bb, int nrows,
                                                  _Float16 * yh) {
    const int r = (int) blockIdx.x * 4 + (int) (threadIdx.x >> 6);
    if (r >= nrows) return;
    const int lane = threadIdx.x & 63;
    const int ne1 = (int) a.ne[1], ne2 = (int) a.ne[2];
    const int i1 = r % ne1, t = r / ne1, i2 = t % ne2, i3 = t / ne2;
    const float * x = (const float *) (a.base + i1 * a.nb[1] + i2 * a.nb[2] + i3 * a.nb[3]);
    float * y = (float *) (d.base + i1 * d.nb[1] + i2 * d.nb[2] + i3 * d.nb[3]);
    const int n = (int) a.ne[0];
    constexpr int C = V4 ? 8 : 32;           // per-lane chunks: float4s (V4) or floats
    constexpr int W = V4 ? 4 : 1;
    float v[C][W];
    // every load of the row first, then the sums (a load and its sum in one loop body compiled to a load + vmcnt(0)
    // per chunk: serial HBM round trips)
#pragma unroll
    for (int k = 0; k < C; ++k) {
        const int j = lane + 64 * k;
        const bool ok = j * W < n;
        if (V4) {
            const f4 u = ok ? ((const f4 *) x)[j] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < W; ++q) v[k][q] = u[q];
        } else {
            v[k][0] = ok ? x[j] : 0.0f;
        }
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < C; ++k) {
        const bool ok = (lane + 64 * k) * W < n;
        // (a float4's four terms summed first, then into the running sum: the grouping of the engine's LayerNorm,
        // q2a_exact.hip k_rownorm, so both give the same row bit for bit and the fused LN route below can use it)
        if (ok) {
            if (V4) s += (double) v[k][0] + (double) v[k][W > 1 ? 1 : 0] + (double) v[k][W > 2 ? 2 : 0] + (double) v[k][W > 3 ? 3 : 0];
            else s += (double) v[k][0];
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = (float) (s / n);
    double s2 = 0.0;
#pragma unroll
    for (int k = 0; k < C; ++k) {
        if ((lane + 64 * k) * W < n) {
            float c[W];
#pragma unroll
            for (int q = 0; q < W; ++q) c[q] = v[k][q] - mean;
            if (V4) s2 += (double) (c[0] * c[0]) + (double) (c[W > 1 ? 1 : 0] * c[W > 1 ? 1 : 0]) +
                          (double) (c[W > 2 ? 2 : 0] * c[W > 2 ? 2 : 0]) + (double) (c[W > 3 ? 3 : 0] * c[W > 3 ? 3 : 0]);
            else s2 += (double) (c[0] * c[0]);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
    const float variance = (float) (s2 / n);
    const float scale = 1.0f / sqrtf(variance + eps);
#pragma unroll
    for (int k = 0; k < C; ++k) {
        const int j = lane + 64 * k;
        if (j * W >= n) continue;
        float o[W];
#pragma unroll
        for (int q = 0; q < W; ++q) {
            o[q] = (v[k][q] - mean) * scale;
            if (AFF) {
                o[q] = o[q] * w[j * W + q];
                o[q] = o[q] + bb[j * W + q];
            }
        }
        if (V4) ((f4 *) y)[j] = f4{o[0], o[W > 1 ? 1 : 0], o[W > 2 ? 2 : 0], o[W > 3 ? 3 : 0]};
        else y[j] = o[0];
        if (yh) {   // fp16 (RNE) copy of the row for the F16-weight GEMMs that consume it: ggml's vec_dot_type conversion
#pragma unroll
            for (int q = 0; q < W; ++q) yh[(int64_t) r * n + j * W + q] = (_Float16) o[q];
        }
    }
}

// SOFT_MAX without mask (ggml.c:13854-13950): w = x*scale, max, e = exp(w - max) with a double sum,
// y = e * (float)(1/sum). One block per row.
__global__ __launch_bounds__(256) void k_softmax(tview a, tview d, float scale) {
    __shared__ double red[4];
    __shared__ float redf[4];
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % a.ne[1], i2 = (r / a.ne[1]) % a.ne[2], i3 = r / (a.ne[1] * a.ne[2]);
    const float * x = (const float *) (a.base + voff(a, 0, i1, i2, i3));
    float * y = (float *) (d.base + voff(d, 0, i1, i2, i3));
    const int n = (int) a.ne[0];
    float mx = -INFINITY;
    for (int i = threadIdx.x; i < n; i += blockDim.x) mx = fmaxf(mx, x[i] * scale);
    mx = block_max_f(mx, redf);
    double s = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float e = expf(x[i] * scale - mx);
        y[i] = e;
        s += (double) e;
    }
    s = block_sum_d(s, red);
    const float inv = (float) (1.0 / s);
    for (int i = threadIdx.x; i < n; i += blockDim.x) y[i] = y[i] * inv;
}

// IM2COL, 1-D (ggml.c:14717-14786): dst[n][ow][ic*KW + kw] = src[n][ic][ow*s0 + kw*d0 - p0] (0 outside)
__global__ void k_im2col1d(tview s, tview d, int dt, int IC, int IW, int KW, int OW, int s0, int p0, int d0, int64_t n) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int kw = (int) (i % KW);
    int64_t r = i / KW;
    const int ic = (int) (r % IC); r /= IC;
    const int ow = (int) (r % OW);
    const int64_t in = r / OW;
    const int64_t iw = (int64_t) ow * s0 + (int64_t) kw * d0 - p0;
    const float v = (iw < 0 || iw >= IW) ? 0.0f : *(const float *) (s.base + in * s.nb[2] + ic * s.nb[1] + iw * s.nb[0]);
    st_from_f32(d.base + voff(d, (int64_t) ic * KW + kw, ow, in, 0), dt, v);
}

// POOL_1D avg, kernel == stride, no padding (ggml_compute_forward_pool_1d_sk_p0, ggml.c:15077-15125):
// acc = 0; acc += x[j] for the k inputs; acc /= k
__global__ void k_pool1d_avg(tview s, tview d, int k, int64_t n) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t i0 = i % d.ne[0], r = i / d.ne[0];
    const int64_t i1 = r % d.ne[1], r2 = r / d.ne[1];
    const int64_t i2 = r2 % d.ne[2], i3 = r2 / d.ne[2];
    float acc = 0.0f;
    for (int ki = 0; ki < k; ++ki) acc += *(const float *) (s.base + voff(s, i0 * k + ki, i1, i2, i3));
    acc /= (float) k;
    *(float *) (d.base + voff(d, i0, i1, i2, i3)) = acc;
}

// POOL_1D(AVG, k) over time of [T][C] rows, read and written in that layout: o[t][c] = (sum_k x[k t + ki][c]) / k —
// the reference's PERMUTE -> CONT -> POOL_1D -> PERMUTE -> CONT (qwen2-whisper.cpp:2160-2172) in one pass, the same
// f32 operations as k_pool1d_avg (acc from 0, then the division); o must not overlap x
__global__ void k_pool_rows_avg(const float * x, float * o, int C, int k, int64_t n) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t t = i / C, c = i - t * C;
    float acc = 0.0f;
    for (int ki = 0; ki < k; ++ki) acc += x[(t * k + ki) * C + c];
    acc /= (float) k;
    o[i] = acc;
}

// fp32 -> fp16 (RNE) of a contiguous F32 activation block (ggml_fp32_to_fp16_row, the F16 vec_dot_type); 8 per
// thread (two 16-B loads, one 16-B store) when n % 8 == 0 and both ends are 16-B aligned
__global__ void k_f32_to_f16(const float * x, _Float16 * y, int64_t n) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = (_Float16) x[i];
}
__global__ void k_f32_to_f16_x8(const f4 * x, uint4 * y, int64_t n8) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n8) return;
    const f4 u = x[2 * i], v = x[2 * i + 1];
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    const h8 h = {(_Float16) u[0], (_Float16) u[1], (_Float16) u[2], (_Float16) u[3],
                  (_Float16) v[0], (_Float16) v[1], (_Float16) v[2], (_Float16) v[3]};
    uint4 o;
    __builtin_memcpy(&o, &h, 16);
    y[i] = o;
}

// Batched exact-f32 GEMM: dst[i3][i2][i1][i0] = sum_k src0[i3/r3][i2/r2][i0][k] * src1[i3][i2][i1][k]
// (ggml_compute_forward_mul_mat semantics for src0 F32/F16 x src1 F32/F16; R16 rounds src1 to fp16 first, the
// conversion ggml applies for an F16 src0). 64x64 tile per workgroup, 4 waves of 32x32, K-step 16 staged in LDS,
// v_mfma_f32_16x16x4_f32 (f32 operands, f32 accumulation).
struct mm_args {
    tview a, b, d;
    int ta, tb;
    int64_t K, r2, r3;
};
template <bool R16>
__global__ __launch_bounds__(256) void k_mm_f32(mm_args p) {
    __shared__ float As[64][17];
    __shared__ float Bs[64][17];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 1, wc = w & 1;
    const int64_t i0b = (int64_t) blockIdx.x * 64, i1b = (int64_t) blockIdx.y * 64;
    const int64_t z = blockIdx.z, i2 = z % p.d.ne[2], i3 = z / p.d.ne[2];
    const char * abase = p.a.base + (i2 / p.r2) * p.a.nb[2] + (i3 / p.r3) * p.a.nb[3];
    const char * bbase = p.b.base + i2 * p.b.nb[2] + i3 * p.b.nb[3];
    const int64_t M0 = p.a.ne[1], M1 = p.b.ne[1];
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    for (int64_t k0 = 0; k0 < p.K; k0 += 16) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int idx = tid + 256 * u, row = idx >> 4, kk = idx & 15;
            const int64_t k = k0 + kk;
            float va = 0.f, vb = 0.f;
            if (k < p.K && i0b + row < M0) va = ld_as_f32(abase + (i0b + row) * p.a.nb[1] + k * p.a.nb[0], p.ta);
            if (k < p.K && i1b + row < M1) {
                vb = ld_as_f32(bbase + (i1b + row) * p.b.nb[1] + k * p.b.nb[0], p.tb);
                if (R16) vb = (float) (_Float16) vb;
            }
            As[row][kk] = va;
            Bs[row][kk] = vb;
        }
        __syncthreads();
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
            const int k = k4 * 4 + (lane >> 4);
            float av[2], bv[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) av[i] = As[wr * 32 + i * 16 + (lane & 15)][k];
#pragma unroll
            for (int j = 0; j < 2; ++j) bv[j] = Bs[wc * 32 + j * 16 + (lane & 15)][k];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
    char * dbase = p.d.base + i2 * p.d.nb[2] + i3 * p.d.nb[3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int64_t c1 = i1b + wc * 32 + j * 16 + (lane & 15);
            if (c1 >= M1) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t c0 = i0b + wr * 32 + i * 16 + (lane >> 4) * 4 + r;
                if (c0 < M0) *(float *) (dbase + c1 * p.d.nb[1] + c0 * p.d.nb[0]) = acc[i][j][r];
            }
        }
}

// attention operands for the fused path: per-head fp16 hi/lo halves of Q (already scaled) and K, V^T
template <bool WITH_V>
__global__ void k_attn_prep(tview q, tview k, tview v, _Float16 * qh, _Float16 * ql, _Float16 * kh, _Float16 * kl,
                            _Float16 * vt, _Float16 * vtl, int T, int H, int TP, int64_t n) {
    // element (d, t, h): q/k/v views have ne = [64, T, H]; q,k -> [t][h*64+d], v -> vt[h][d][t]
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int d = (int) (i & 63);
    const int r = (int) (i >> 6);
    const int t = r % T, h = r / T;
    float qv = *(const float *) (q.base + voff(q, d, t, h, 0)) * Q2A_LOG2E;   // the attention's log2 units
    // the product rounded to f32 first, then split (as the QKV GEMM epilogue does): left to itself the compiler
    // rounds q * log2e to fp16 in one mixed-precision op, which at an f32 value on an fp16 tie picks the other half
    // (128 of 1.92 M Q elements of a full-size layer; diag/gpurun_r05m.sh)
    asm volatile("" : "+v"(qv));
    const float kv = *(const float *) (k.base + voff(k, d, t, h, 0));
    const int64_t o = (int64_t) t * H * 64 + h * 64 + d;
    const _Float16 a = (_Float16) qv, b = (_Float16) kv;
    qh[o] = a; ql[o] = (_Float16) (qv - (float) a);
    kh[o] = b; kl[o] = (_Float16) (kv - (float) b);
    if (WITH_V) {
        const float vv = *(const float *) (v.base + voff(v, t, d, h, 0));
        const _Float16 vh = (_Float16) vv;
        vt[((int64_t) h * 64 + d) * TP + t] = vh;
        if (vtl) vtl[((int64_t) h * 64 + d) * TP + t] = (_Float16) (vv - (float) vh);
    }
}

// V^T operand of the fused attention, produced at the graph's CONT(permute(V)) node (qwen2-whisper.cpp:2081-2089)
// from the CONT's source view (ne = [T, 64, H]; the CONT would copy it verbatim): vt[h][d][t] = fp16 V(t, d, h),
// zero for T <= t < TP, and (vtl != NULL: the reference-contract attention's V hi/lo split) the lo image
// fp16(v - fp16(v)). One 64(t) x 64(d) tile per workgroup through LDS: reads run along d, writes along t.
__global__ __launch_bounds__(256) void k_vt_tile(tview v, _Float16 * vt, _Float16 * vtl, int T, int TP) {
    __shared__ float tile[64][65];
    const int t0 = (int) blockIdx.x * 64, h = (int) blockIdx.y;
    for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
        const int tt = idx >> 6, dd = idx & 63, t = t0 + tt;
        tile[tt][dd] = t < T ? *(const float *) (v.base + voff(v, t, dd, h, 0)) : 0.0f;
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
        const int dd = idx >> 6, tt = idx & 63;
        const float x = tile[tt][dd];
        const _Float16 xh = (_Float16) x;
        vt[((int64_t) h * 64 + dd) * TP + t0 + tt] = xh;
        if (vtl) vtl[((int64_t) h * 64 + dd) * TP + t0 + tt] = (_Float16) (x - (float) xh);
    }
}

// fused attention output [t][h*64+d] (f32) -> the KQV node's layout dst (ne = [64, T, H])
__global__ void k_attn_out(const float * o, tview d, int T, int H, int64_t n) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int dd = (int) (i & 63);
    const int64_t r = i >> 6;
    const int t = (int) (r % T), h = (int) (r / T);
    *(float *) (d.base + voff(d, dd, t, h, 0)) = o[(int64_t) t * H * 64 + h * 64 + dd];
}

// MUL_MAT(F32 im2col, F16 conv kernel) on the fp16 MFMA GEMM (the conv graph nodes, qwen2-whisper.cpp:1926-1931 via
// ggml_conv_1d): every f32 activation x is written as P fp16 parts against the weight row repeated P times, operand rows
// [M][K] -> [M][PK] against [N][PK]. P = 3 (conv_parts): hi = fp16(x), mid = fp16(x - hi), lo = fp16(x - hi - mid)
// hold x exactly (24 bits in three 11-bit pieces), so every product is the f32 product exactly. Both conv nodes use
// it: conv2's input is mostly the GELU table's fp16 values (mid = lo = 0), but ggml_vec_gelu_f32 passes x >= 10
// through as f32 (ggml.c:2562), which two parts (22 bits) would round. *inexact is raised when any x is not an fp16
// value (r != 0, NaN and infinities included): while it stays 0 the mid and lo parts are all zero, and the GEMM over
// the hi part alone (same K-steps, the zero parts' partials are exact zeros) gives the same bits as the three-part one
__global__ __launch_bounds__(256) void k_hilo_rows(const float * x, _Float16 * a, int K, int P, int n, int * inexact) {
    const int i = (int) blockIdx.x * blockDim.x + threadIdx.x;
    bool nz = false;
    if (i < n) {
        const int m = i / K, k = i - m * K;
        const float v = x[i];
        const _Float16 h = (_Float16) v;
        const float r = v - (float) h;   // exact
        const _Float16 md = (_Float16) r;
        _Float16 * row = a + (int64_t) m * P * K;
        row[k] = h;
        row[K + k] = md;
        if (P == 3) row[2 * K + k] = (_Float16) (r - (float) md);
        nz = !(r == 0.0f);
    }
    // one atomic per wave that holds such a value (inexact is null for conv1, whose mel rows hold them everywhere)
    if (inexact && __any(nz) && (threadIdx.x & 63) == 0) atomicOr(inexact, 1);
}
__global__ void k_dup_rows(const _Float16 * w, _Float16 * o, int K, int P, int n) {
    const int i = (int) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int r = i / K, k = i - r * K;
    for (int q = 0; q < P; ++q) o[(int64_t) r * P * K + q * K + k] = w[i];
}
// t [R][C] -> o [C][R] (f32), 64x64 tiles through LDS
// with bias (the conv's ADD of its [1][C] bias row, then GELU): o[c][r] = gelu(t[r][c] + bias[c]), the f32 ADD and
// the table GELU of the two graph nodes (k_rows<0>, k_rows<3>) on the same values; with addend (an [C][R] f32 array,
// the encoder's positional rows): o[c][r] = addend[c][r] + t[r][c], the ADD node's one f32 addition
// (every caller's t, o, bias, table and addend are distinct buffers: the conv scratch, the node's output checked
// disjoint from the others, weights)
__global__ __launch_bounds__(256) void k_transpose_f32(const float * __restrict__ t, float * __restrict__ o, int R, int C,
                                                       const float * __restrict__ bias, const uint16_t * __restrict__ gelu_tab,
                                                       const float * __restrict__ addend = nullptr) {
    __shared__ float tile[64][65];
    const int r0 = (int) blockIdx.y * 64, c0 = (int) blockIdx.x * 64;
    // unrolled with clamped (always valid) addresses, so each thread's 16 loads are in flight together; a load under
    // the bounds branch waited alone
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int idx = (int) threadIdx.x + 256 * it, rr = idx >> 6, cc = idx & 63;
        tile[rr][cc] = t[(int64_t) min(r0 + rr, R - 1) * C + min(c0 + cc, C - 1)];
    }
    __syncthreads();
    // the operand mode is uniform: one unrolled loop per mode, so the loads of different elements are not split by
    // per-element branches
    // per-element branches (the conditional stores included: values first, then the stores). The GELU table reads are
    // asm loads behind one wait: as plain loads the compiler moved each into the x > -10 branch with its own wait
    auto out = [&](auto has_bias, auto has_addend) {
        float v[16];
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const int idx = (int) threadIdx.x + 256 * it, cc = idx >> 6, rr = idx & 63;
            v[it] = tile[rr][cc];
            if constexpr (decltype(has_bias)::value) v[it] = v[it] + bias[min(c0 + cc, C - 1)];
        }
        if constexpr (decltype(has_bias)::value) {
            uint32_t g[16];
#pragma unroll
            for (int it = 0; it < 16; ++it) {
                const _Float16 h = (_Float16) v[it];
                uint16_t u;
                __builtin_memcpy(&u, &h, 2);
                asm volatile("global_load_ushort %0, %1, off" : "=v"(g[it]) : "v"(gelu_tab + u) : "memory");
            }
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(g[0]), "+v"(g[1]), "+v"(g[2]), "+v"(g[3]), "+v"(g[4]), "+v"(g[5]), "+v"(g[6]),
                         "+v"(g[7]), "+v"(g[8]), "+v"(g[9]), "+v"(g[10]), "+v"(g[11]), "+v"(g[12]), "+v"(g[13]), "+v"(g[14]),
                         "+v"(g[15]) :: "memory");
#pragma unroll
            for (int it = 0; it < 16; ++it) {   // gelu_tab_f's ranges (ggml_vec_gelu_f32, GGML_GELU_FP16)
                const uint16_t gg = (uint16_t) g[it];
                _Float16 gh;
                __builtin_memcpy(&gh, &gg, 2);
                v[it] = v[it] <= -10.0f ? 0.0f : v[it] >= 10.0f ? v[it] : (float) gh;
            }
        }
        if constexpr (decltype(has_addend)::value) {
#pragma unroll
            for (int it = 0; it < 16; ++it) {
                const int idx = (int) threadIdx.x + 256 * it, cc = idx >> 6, rr = idx & 63;
                v[it] = addend[(int64_t) min(c0 + cc, C - 1) * R + min(r0 + rr, R - 1)] + v[it];
            }
        }
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const int idx = (int) threadIdx.x + 256 * it, cc = idx >> 6, rr = idx & 63;
            if (r0 + rr < R && c0 + cc < C) o[(int64_t) (c0 + cc) * R + r0 + rr] = v[it];
        }
    };
    if (bias && addend) out(std::true_type{}, std::true_type{});
    else if (bias) out(std::true_type{}, std::false_type{});
    else if (addend) out(std::false_type{}, std::true_type{});
    else out(std::false_type{}, std::false_type{});
}

// ------------------------------------------------------------------------------------------------
// devices, buffers, weight cache
// ------------------------------------------------------------------------------------------------
struct packed_w {
    const char * raw;        // the weight tensor's bytes in a Q2A buffer
    size_t raw_bytes;
    int type, N, K;
    void * dev;              // repacked GEMM operand (q2a_pack_linear layout)
    uint64_t off[6];
};

struct q2a_device_ctx {
    int device = 0;
    std::string name, desc;
    ggml_backend_buffer_type buft;
    ggml_backend_device dev;
    std::mutex mu;
    std::vector<packed_w> wcache;
    uint64_t wgen = 0;                 // bumped whenever a packed weight is evicted (captured graphs hold its pointer)
    std::atomic<int> n_captured{0};    // HIP graphs instantiated by the backends of this device so far
    uint16_t * gelu_tab = nullptr;     // device copy of the 64 Ki-entry fp16 GELU table (lazy)
};

struct q2a_reg_ctx {
    std::vector<q2a_device_ctx *> devs;
};

struct q2a_buffer_ctx {
    int device;
    void * ptr;
    size_t size;
    std::string name;
};

struct q2a_backend_ctx {
    int device;
    std::string name;
    hipStream_t stream = nullptr;
    void * scratch = nullptr;
    _Float16 * vt_buf = nullptr;       // V^T operand of the fused attention, written at the V CONT node
    size_t vt_bytes = 0;
    char * qkv_buf = nullptr;          // attention operands written by the fused Q|K|V GEMM (run_qkv_fused)
    size_t qkv_bytes = 0;
    _Float16 * pre16 = nullptr;        // fc1's fp16 pre-activation / GELU output on the way to fc2's operand (run_fc1_for_fc2)
    size_t pre16_bytes = 0;
    // fp16 shadows of f32 activations written by their producer (LayerNorm, fc1 GELU epilogue) for F16-weight
    // MUL_MATs that would otherwise convert them: two slots, a producer never writes the slot its own GEMM reads
    _Float16 * a16[2] = {nullptr, nullptr};
    size_t a16_bytes[2] = {0, 0};
    const ggml_tensor * a16_src[2] = {nullptr, nullptr};
    int a16_last = 1;
    const ggml_tensor * quant_src = nullptr;   // activation whose quantized image is in the scratch (see run_mm_fast)
    int quant_blk = 0;
    size_t scratch_bytes = 0;
    ggml_backend_q2a_stats stats{};
    // HIP graphs of recent graph_computes: the sched hands the same cgraphs (same nodes, buffers, parameters) on
    // every whisper_full — the conv graph, then the encoder graph — so a cgraph seen a second time has its launches
    // captured once and is replayed from then on
    struct captured { uint64_t sig; int seen; hipGraphExec_t exec; ggml_backend_q2a_stats stats; uint64_t used; };
    std::vector<captured> graphs;
    uint64_t graph_clock = 0;
    int n_buffer_reallocs = 0;         // scratch / V^T / shadow reallocations (each drops the captured graphs)
    bool capture_aborted = false;      // a reallocation ended an in-progress capture (graph_compute re-runs directly)
    int n_mul_mat_conv_total = 0;      // conv MUL_MATs run on the hi/lo path over the backend's lifetime
    int n_repack_lazy = 0;             // get_packed cache misses over the backend's lifetime
};

q2a_reg_ctx * reg_ctx();
ggml_backend_reg * the_reg();

q2a_device_ctx * dev_ctx(int device) {
    q2a_reg_ctx * r = reg_ctx();
    if (device < 0 || device >= (int) r->devs.size()) return nullptr;
    return r->devs[device];
}

// drop cached repacks whose source bytes overlap [p, p + n)
void invalidate(int device, const void * p, size_t n) {
    q2a_device_ctx * d = dev_ctx(device);
    if (!d) return;
    std::lock_guard<std::mutex> lk(d->mu);
    const char * a = (const char *) p;
    for (size_t i = 0; i < d->wcache.size();) {
        packed_w & w = d->wcache[i];
        if (w.raw < a + n && a < w.raw + w.raw_bytes) {
            (void) hipSetDevice(device);
            (void) hipFree(w.dev);
            ++d->wgen;
            d->wcache[i] = d->wcache.back();
            d->wcache.pop_back();
        } else {
            ++i;
        }
    }
}

const uint16_t * gelu_table(int device) {
    q2a_device_ctx * d = dev_ctx(device);
    std::lock_guard<std::mutex> lk(d->mu);
    if (!d->gelu_tab) {
        std::vector<uint16_t> t(65536);
        q2a_make_gelu_table(t.data());
        Q2A_HIP(hipMalloc((void **) &d->gelu_tab, 65536 * 2));
        Q2A_HIP(hipMemcpy(d->gelu_tab, t.data(), 65536 * 2, hipMemcpyHostToDevice));
    }
    return d->gelu_tab;
}

// ---- buffer -----------------------------------------------------------------------------------
const char * buf_get_name(ggml_backend_buffer_t b) { return ((q2a_buffer_ctx *) b->context)->name.c_str(); }
void buf_free(ggml_backend_buffer_t b) {
    q2a_buffer_ctx * c = (q2a_buffer_ctx *) b->context;
    invalidate(c->device, c->ptr, c->size);
    (void) hipSetDevice(c->device);
    (void) hipFree(c->ptr);
    delete c;
}
void * buf_get_base(ggml_backend_buffer_t b) { return ((q2a_buffer_ctx *) b->context)->ptr; }
void buf_memset_tensor(ggml_backend_buffer_t b, ggml_tensor * t, uint8_t v, size_t off, size_t n) {
    q2a_buffer_ctx * c = (q2a_buffer_ctx *) b->context;
    Q2A_HIP(hipSetDevice(c->device));
    invalidate(c->device, (char *) t->data + off, n);
    Q2A_HIP(hipMemset((char *) t->data + off, v, n));
}
// Upload-time repack: the model loader writes each weight whole from host memory (qwen2-whisper.cpp:1845-1849),
// before it marks the buffer WEIGHTS (:1867), so a whole write of a 2-D tensor that the fast MUL_MAT path could take
// (mm_fast_ok's shape rule) is packed here from the host bytes, and the first whisper_full finds it in the cache
// instead of paying a device->host copy + host repack per weight. Anything else is packed lazily by get_packed.
void prepack(int device, const ggml_tensor * t, const void * host, size_t off, size_t n) {
    if (off != 0 || n != ggml_nbytes(t) || t->view_src) return;
    // gallocr COMPUTE buffers hold activations (an F16 input set every step would be host-packed on every write, and
    // its cache entry would outlive a kernel's later overwrite of the same address): only weight-bearing buffers,
    // which are still ANY while the loader uploads (qwen2-whisper.cpp:1845-1867)
    if (t->buffer && ggml_backend_buffer_get_usage(t->buffer) == GGML_BACKEND_BUFFER_USAGE_COMPUTE) return;
    if (t->type != GGML_TYPE_F16 && t->type != GGML_TYPE_Q4_K && t->type != GGML_TYPE_Q8_0 && t->type != GGML_TYPE_Q4_0)
        return;
    if (t->ne[2] != 1 || t->ne[3] != 1 || !ggml_is_contiguous(t)) return;
    const int64_t K = t->ne[0], N = t->ne[1];
    if (N % 128 != 0 || K % 256 != 0 || K > 8192 || N > (1 << 30)) return;
    packed_w p;
    p.raw = (const char *) t->data; p.raw_bytes = n; p.type = t->type; p.N = (int) N; p.K = (int) K;
    std::vector<uint8_t> out;
    if (q2a_pack_linear((const uint8_t *) host, t->type, p.N, p.K, out, p.off) != 0) return;
    Q2A_HIP(hipMalloc(&p.dev, out.size()));
    Q2A_HIP(hipMemcpy(p.dev, out.data(), out.size(), hipMemcpyHostToDevice));
    q2a_device_ctx * d = dev_ctx(device);
    std::lock_guard<std::mutex> lk(d->mu);
    d->wcache.push_back(p);
}

void buf_set_tensor(ggml_backend_buffer_t b, ggml_tensor * t, const void * data, size_t off, size_t n) {
    q2a_buffer_ctx * c = (q2a_buffer_ctx *) b->context;
    Q2A_HIP(hipSetDevice(c->device));
    invalidate(c->device, (char *) t->data + off, n);
    Q2A_HIP(hipMemcpy((char *) t->data + off, data, n, hipMemcpyHostToDevice));
    prepack(c->device, t, data, off, n);
}
void buf_get_tensor(ggml_backend_buffer_t b, const ggml_tensor * t, void * data, size_t off, size_t n) {
    q2a_buffer_ctx * c = (q2a_buffer_ctx *) b->context;
    Q2A_HIP(hipSetDevice(c->device));
    Q2A_HIP(hipMemcpy(data, (const char *) t->data + off, n, hipMemcpyDeviceToHost));
}
bool is_q2a_buffer(ggml_backend_buffer_t b);
bool buf_cpy_tensor(ggml_backend_buffer_t b, const ggml_tensor * src, ggml_tensor * dst) {
    if (!src->buffer || !is_q2a_buffer(src->buffer)) return false;
    q2a_buffer_ctx * c = (q2a_buffer_ctx *) b->context;
    Q2A_HIP(hipSetDevice(c->device));
    invalidate(c->device, dst->data, ggml_nbytes(dst));
    Q2A_HIP(hipMemcpy(dst->data, src->data, ggml_nbytes(src), hipMemcpyDeviceToDevice));
    return true;
}
void buf_clear(ggml_backend_buffer_t b, uint8_t v) {
    q2a_buffer_ctx * c = (q2a_buffer_ctx *) b->context;
    Q2A_HIP(hipSetDevice(c->device));
    invalidate(c->device, c->ptr, c->size);
    Q2A_HIP(hipMemset(c->ptr, v, c->size));
}

const ggml_backend_buffer_i k_buffer_iface = {
    /* get_name      */ buf_get_name,
    /* free_buffer   */ buf_free,
    /* get_base      */ buf_get_base,
    /* init_tensor   */ nullptr,
    /* memset_tensor */ buf_memset_tensor,
    /* set_tensor    */ buf_set_tensor,
    /* get_tensor    */ buf_get_tensor,
    /* cpy_tensor    */ buf_cpy_tensor,
    /* clear         */ buf_clear,
    /* reset         */ nullptr,
};

bool is_q2a_buffer(ggml_backend_buffer_t b) { return b->iface.get_name == buf_get_name; }

// ---- buffer type --------------------------------------------------------------------------------
const char * buft_get_name(ggml_backend_buffer_type_t t) { return ((q2a_device_ctx *) t->context)->name.c_str(); }
ggml_backend_buffer_t buft_alloc(ggml_backend_buffer_type_t t, size_t size) {
    q2a_device_ctx * d = (q2a_device_ctx *) t->context;
    if (hipSetDevice(d->device) != hipSuccess) return nullptr;
    void * p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(size, 1)) != hipSuccess) {
        (void) hipGetLastError();
        Q2A_LOG_ERROR("ggml-q2a: allocating %.2f MB on device %d failed\n", size / 1e6, d->device);
        return nullptr;
    }
    q2a_buffer_ctx * c = new q2a_buffer_ctx{d->device, p, size, d->name};
    return ggml_backend_buffer_init(t, k_buffer_iface, c, size);
}
size_t buft_get_alignment(ggml_backend_buffer_type_t) { return 256; }
bool buft_is_host(ggml_backend_buffer_type_t) { return false; }

const ggml_backend_buffer_type_i k_buft_iface = {
    /* get_name       */ buft_get_name,
    /* alloc_buffer   */ buft_alloc,
    /* get_alignment  */ buft_get_alignment,
    /* get_max_size   */ nullptr,
    /* get_alloc_size */ nullptr,
    /* is_host        */ buft_is_host,
};

// ---- pinned host buffer type (ggml-cuda.h:34; the CPU-side buffers a caller stages its copies in) ------------------
// Page-locked host memory (hipHostMalloc, portable: every device of a q2a_group sees it as pinned), handed to ggml as
// a CPU buffer over that pointer, so the CPU backend computes in it and the DMA engines copy out of it directly instead
// of through the runtime's pageable staging. GGML_Q2A_NO_PINNED=1 (the reference's GGML_CUDA_NO_PINNED) or a failed
// pinning falls back to an ordinary CPU buffer.
const char * host_buft_get_name(ggml_backend_buffer_type_t) { return GGML_Q2A_NAME "_Host"; }
const char * host_buf_get_name(ggml_backend_buffer_t) { return GGML_Q2A_NAME "_Host"; }
void host_buf_free(ggml_backend_buffer_t b) {
    if (hipHostFree(b->context) != hipSuccess) (void) hipGetLastError();
}
bool pinned_allowed() { return getenv("GGML_Q2A_NO_PINNED") == nullptr; }
ggml_backend_buffer_t host_buft_alloc(ggml_backend_buffer_type_t t, size_t size) {
    void * p = nullptr;
    if (pinned_allowed()) {
        if (hipHostMalloc(&p, std::max<size_t>(size, 1), hipHostMallocPortable) != hipSuccess) {
            (void) hipGetLastError();
            Q2A_LOG_ERROR("ggml-q2a: pinning %.2f MB of host memory failed; using pageable memory\n", size / 1e6);
            p = nullptr;
        }
    }
    if (!p) return ggml_backend_buft_alloc_buffer(ggml_backend_cpu_buffer_type(), size);
    ggml_backend_buffer_t b = ggml_backend_cpu_buffer_from_ptr(p, size);
    b->buft = t;      // (a CPU buffer's context is its pointer: what host_buf_free releases)
    b->iface.get_name = host_buf_get_name;
    b->iface.free_buffer = host_buf_free;
    return b;
}
size_t host_buft_get_alignment(ggml_backend_buffer_type_t) {
    return ggml_backend_buft_get_alignment(ggml_backend_cpu_buffer_type());
}
size_t host_buft_get_alloc_size(ggml_backend_buffer_type_t, const ggml_tensor * t) {
    return ggml_backend_buft_get_alloc_size(ggml_backend_cpu_buffer_type(), const_cast<ggml_tensor *>(t));
}
bool host_buft_is_host(ggml_backend_buffer_type_t) { return true; }

const ggml_backend_buffer_type_i k_host_buft_iface = {
    /* get_name       */ host_buft_get_name,
    /* alloc_buffer   */ host_buft_alloc,
    /* get_alignment  */ host_buft_get_alignment,
    /* get_max_size   */ nullptr,
    /* get_alloc_size */ host_buft_get_alloc_size,
    /* is_host        */ host_buft_is_host,
};

// ------------------------------------------------------------------------------------------------
// graph execution
// ------------------------------------------------------------------------------------------------
tview tv(const ggml_tensor * t) {
    tview v;
    v.base = (char *) t->data;
    for (int i = 0; i < 4; ++i) { v.ne[i] = t->ne[i]; v.nb[i] = (int64_t) t->nb[i]; }
    return v;
}

dim3 grid1(int64_t n) { return dim3((unsigned) ((n + 255) / 256)); }

// Captured HIP graphs bake in the addresses of the scratch, V^T and fp16-shadow buffers: whenever one of them is
// reallocated, every captured exec is destroyed (its cgraph is re-captured on its next sightings against the new
// buffers), so no replay can touch freed memory.
// A buffer must grow while graph_compute is capturing (the second sighting of a cgraph whose node sequence needs more
// than its first run did): a capturing stream cannot be synchronised and the capture would bake in the buffer about
// to be freed. End the capture and discard it (nothing captured has run). The node that asked for the buffer would
// otherwise go on launching its kernels directly, on inputs that earlier nodes only captured and never computed, so
// once the buffer has grown a DISCARD capture is begun (resume_discard): whatever the rest of that node launches is
// captured into it and thrown away. run_nodes stops at the next node, and graph_compute ends the discard capture and
// runs the cgraph again directly, against the new buffers.
void abort_capture(q2a_backend_ctx * b) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(b->stream, &st) == hipSuccess && st == hipStreamCaptureStatusActive) {
        hipGraph_t gr = nullptr;
        (void) hipStreamEndCapture(b->stream, &gr);
        if (gr) (void) hipGraphDestroy(gr);
        (void) hipGetLastError();
        b->capture_aborted = true;
    }
}

// after the growth that abort_capture allowed: route the aborted node's remaining launches into a discarded capture
void resume_discard(q2a_backend_ctx * b) {
    if (b->capture_aborted && hipStreamBeginCapture(b->stream, hipStreamCaptureModeThreadLocal) != hipSuccess)
        (void) hipGetLastError();
}

// end (and drop) the discard capture, if one is open
void end_discard(q2a_backend_ctx * b) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(b->stream, &st) == hipSuccess && st == hipStreamCaptureStatusActive) {
        hipGraph_t gr = nullptr;
        (void) hipStreamEndCapture(b->stream, &gr);
        if (gr) (void) hipGraphDestroy(gr);
    }
    (void) hipGetLastError();
}

void drop_graphs(q2a_backend_ctx * b) {
    for (auto & e : b->graphs) {
        if (e.exec) (void) hipGraphExecDestroy(e.exec);
        e.exec = nullptr;
        e.seen = 1;
    }
    ++b->n_buffer_reallocs;
}

void * scratch(q2a_backend_ctx * b, size_t bytes) {
    if (bytes > b->scratch_bytes) {
        b->quant_src = nullptr;
        abort_capture(b);
        Q2A_HIP(hipStreamSynchronize(b->stream));
        if (b->scratch) Q2A_HIP(hipFree(b->scratch));
        b->scratch = nullptr;
        Q2A_HIP(hipMalloc(&b->scratch, bytes));
        b->scratch_bytes = bytes;
        drop_graphs(b);
        resume_discard(b);
    }
    return b->scratch;
}

bool is_weight_type(int t) {
    return t == GGML_TYPE_F16 || t == GGML_TYPE_Q4_K || t == GGML_TYPE_Q8_0 || t == GGML_TYPE_Q4_0;
}

// the fast MUL_MAT path: contiguous 2-D weight (ne00 = K, ne01 = N) x contiguous F32 rows
bool mm_fast_ok(const ggml_tensor * op) {
    const ggml_tensor * w = op->src[0];
    const ggml_tensor * x = op->src[1];
    if (!is_weight_type(w->type) || x->type != GGML_TYPE_F32 || op->type != GGML_TYPE_F32) return false;
    if (!ggml_is_contiguous(w) || !ggml_is_contiguous(x) || !ggml_is_contiguous(op)) return false;
    if (w->ne[2] != 1 || w->ne[3] != 1) return false;
    const int64_t K = w->ne[0], N = w->ne[1];
    return N % 128 == 0 && K % 256 == 0 && K <= 8192 && N <= (1 << 30);
}

// (returned by value: the cache vector may grow or swap-remove entries under another backend's lock)
packed_w get_packed(q2a_backend_ctx * b, const ggml_tensor * w) {
    q2a_device_ctx * d = dev_ctx(b->device);
    {
        std::lock_guard<std::mutex> lk(d->mu);
        for (const packed_w & p : d->wcache)
            if (p.raw == (const char *) w->data && p.type == w->type && p.N == w->ne[1] && p.K == w->ne[0]) return p;
    }
    // first use: repack on the host from the device bytes (one-time, per weight tensor)
    ++b->n_repack_lazy;
    const size_t nb = ggml_nbytes(w);
    std::vector<uint8_t> raw(nb);
    Q2A_HIP(hipStreamSynchronize(b->stream));
    Q2A_HIP(hipMemcpy(raw.data(), w->data, nb, hipMemcpyDeviceToHost));
    packed_w p;
    p.raw = (const char *) w->data; p.raw_bytes = nb; p.type = w->type; p.N = (int) w->ne[1]; p.K = (int) w->ne[0];
    std::vector<uint8_t> out;
    if (q2a_pack_linear(raw.data(), w->type, p.N, p.K, out, p.off) != 0) GGML_ABORT("ggml-q2a: cannot pack %s", w->name);
    Q2A_HIP(hipMalloc(&p.dev, out.size()));
    Q2A_HIP(hipMemcpy(p.dev, out.data(), out.size(), hipMemcpyHostToDevice));
    std::lock_guard<std::mutex> lk(d->mu);
    d->wcache.push_back(p);
    return p;
}

struct mm_chain {          // a fast MUL_MAT and the nodes its epilogue absorbs
    ggml_tensor * out;     // last node of the chain (where the result goes)
    int epi;
    const float * bias;
    const float * resid;
    float oscale;
    int last;              // graph index of `out`
    int nfused;            // nodes absorbed
};
struct mm_second {         // the second GEMM of a grouped launch (same activation, fp16 weight of the same shape)
    const ggml_tensor * w;
    ggml_tensor * out;
    const float * bias;
    float oscale;
};

// the activation operand of a fast MUL_MAT, in the scratch: fp16 rows (F16 weights; the producer's fp16 shadow when it
// wrote one) or Q8_K / Q8_0 codes with their block scales (dy [K/blk][MP], and for Q8_K the bsum operand aext
// [K/256][MP][16]); `extra` more scratch bytes follow it (returned in .extra)
struct act_operand {
    const q2a_half * A;
    float * dy;
    q2a_half * aext;
    int MP;
    char * extra;
};
// where an activation operand of M rows x K lives in the scratch (grown to hold it and `extra` bytes; nothing produced)
act_operand act_slots(q2a_backend_ctx * b, int M, int K, int blk, size_t extra) {
    const int MP = (M + 255) / 256 * 256;
    // scratch: A operand fp16 [M][K] | dy [K/blk][MP] | aext [K/256][MP][16] | extra
    const size_t a_bytes = ((size_t) M * K * 2 + 255) & ~size_t(255);
    const size_t dy_bytes = blk ? ((size_t) (K / blk) * MP * 4 + 255) & ~size_t(255) : 0;
    const size_t ae_bytes = blk == 256 ? (size_t) (K / 256) * MP * 32 : 0;
    char * s = (char *) scratch(b, a_bytes + dy_bytes + ae_bytes + extra);
    return {(const q2a_half *) s, (float *) (s + a_bytes), (q2a_half *) (s + a_bytes + dy_bytes), MP,
            s + a_bytes + dy_bytes + ae_bytes};
}

act_operand activation_operand(q2a_backend_ctx * b, const ggml_tensor * x, int M, int K, int blk, size_t extra) {
    const act_operand slots = act_slots(b, M, K, blk, extra);
    const int MP = slots.MP;
    q2a_half * A = (q2a_half *) slots.A;
    float * dy = slots.dy;
    q2a_half * aext = slots.aext;
    const _Float16 * shadow = nullptr;
    if (blk == 0)
        for (int k = 0; k < 2; ++k) if (b->a16_src[k] == x) shadow = b->a16[k];
    if (shadow) {
        A = (q2a_half *) shadow;   // the producer already wrote the fp16 operand
    } else if (blk == 0) {
        const int64_t n = (int64_t) M * K;
        if (n % 8 == 0 && ((uintptr_t) x->data & 15) == 0 && ((uintptr_t) A & 15) == 0)
            hipLaunchKernelGGL(k_f32_to_f16_x8, grid1(n / 8), dim3(256), 0, b->stream, (const f4 *) x->data, (uint4 *) A, n / 8);
        else
            hipLaunchKernelGGL(k_f32_to_f16, grid1(n), dim3(256), 0, b->stream, (const float *) x->data, A, n);
    } else if (b->quant_src != x || b->quant_blk != blk) {
        q2a_quant_args qa{(const float *) x->data, nullptr, M, K, blk == 256 ? 1 : 2, A, dy, aext, MP};
        Q2A_HIP(q2a_launch_quant_act(qa, b->stream));
    }
    // the scratch now holds x's quantized image (Q8_K / Q8_0 codes and scales): the next quantized-weight MUL_MAT of
    // the same activation (the Q, K, V projections) reuses it; an fp16 conversion overwrote it
    b->quant_src = blk ? x : nullptr;
    b->quant_blk = blk;
    return {A, dy, aext, MP, slots.extra};
}

int blk_of_type(int t) { return t == GGML_TYPE_Q4_K ? 256 : t == GGML_TYPE_F16 ? 0 : 32; }

// the split-K partial planes run_mm_fast needs past the activation operand (0 = no split)
size_t mm_part_bytes(int epi, int blk, int M, int N, int K, bool grouped) {
    const int nsplit = grouped || !(epi == Q2A_EPI_RESID || epi == Q2A_EPI_STORE_F) ? 0
                       : blk == 0 ? q2a_gemm_resid_ksplit(M, N, K, 0) : q2a_gemm_kq_ksplit(M, N, K, blk);
    return nsplit > 1 ? (size_t) nsplit * M * N * 4 : 0;
}

// epi: Q2A_EPI_STORE_F (bias optional), Q2A_EPI_GELU_F (bias, GELU), Q2A_EPI_RESID (bias, + resid rows); the result
// goes to `out` (op itself, or the last node of a fused MUL_MAT -> ADD [-> GELU | ADD] chain)
void run_mm_fast(q2a_backend_ctx * b, ggml_tensor * op, ggml_tensor * out = nullptr, int epi = Q2A_EPI_STORE_F,
                 const float * bias = nullptr, const float * resid = nullptr, float oscale = 0.0f,
                 _Float16 * out16 = nullptr, const mm_second * sec = nullptr) {
    if (!out) out = op;
    const ggml_tensor * w = op->src[0];
    const ggml_tensor * x = op->src[1];
    const int K = (int) w->ne[0], N = (int) w->ne[1];
    const int M = (int) (x->ne[1] * x->ne[2] * x->ne[3]);
    const int blk = blk_of_type(w->type);
    // fp16 small-tile GEMMs (a single clip) split K like the engine's residual GEMMs (q2a_gemm_resid_ksplit: up to
    // 4 partial [M][N] f32 planes, reduced in split order with the bias / residual / scale of the epilogue)
    const size_t part_bytes = mm_part_bytes(epi, blk, M, N, K, sec != nullptr);
    const bool split = part_bytes > 0;
    const act_operand ao = activation_operand(b, x, M, K, blk, part_bytes);
    q2a_gemm_args a;
    memset(&a, 0, sizeof(a));
    a.A = ao.A; a.lda = K; a.a_rpg = M; a.a_gstride = 0; a.a_step = 1;
    a.M = M; a.N = N; a.K = K; a.ldw = K;
    a.outF = (float *) out->data; a.ldo = N;
    a.bias = bias; a.store_bias = bias != nullptr; a.resid = resid; a.out_scale = oscale;
    if (epi == Q2A_EPI_GELU_F) a.outH = (q2a_half *) out16;
    if (epi == Q2A_EPI_GELU_H || epi == Q2A_EPI_PRE_H) {   // fp16 [M][N] only (no row remap)
        a.outH = (q2a_half *) out16;
        a.o_rpg = M; a.o_gstride = 0; a.o_off = 0;
    }
    if (sec) {
        a.ngroup = 2;
        a.W2 = (const q2a_half *) sec->w->data;
        a.bias2 = sec->bias; a.store_bias2 = sec->bias != nullptr;
        a.outF2 = (float *) sec->out->data; a.out_scale2 = sec->oscale;
        if (blk == 256) {   // the second weight's packed image: operand and block scales like the first's below
            const packed_w p2 = get_packed(b, sec->w);
            const char * base2 = (const char *) p2.dev;
            a.W2 = (const q2a_half *) (base2 + p2.off[0]);
            a.dx2 = (const float *) (base2 + p2.off[1]);
            a.dmin2 = (const float *) (base2 + p2.off[2]);
            a.wext2 = (const q2a_half *) (base2 + p2.off[3]);
            a.beta2 = (const float *) (base2 + p2.off[4]);
            a.gamma2 = (const float *) (base2 + p2.off[5]);
        }
    }
    if (split) {
        a.part = (float *) ao.extra;
        a.split_stride = (int64_t) M * N;
        a.split_store = 1;
        a.split_kq = 1;
    }
    a.gelu_tab = gelu_table(b->device);
    if (blk == 0) {
        a.W = (const q2a_half *) w->data;
    } else {
        const packed_w p = get_packed(b, w);
        const char * base = (const char *) p.dev;
        a.W = (const q2a_half *) (base + p.off[0]);
        a.nblk = K / blk;
        a.dx = (const float *) (base + p.off[1]);
        a.dy = ao.dy; a.dy_ld = ao.MP;
        if (blk == 256) {
            a.dmin = (const float *) (base + p.off[2]);
            a.wext = (const q2a_half *) (base + p.off[3]);
            a.beta = (const float *) (base + p.off[4]);
            a.gamma = (const float *) (base + p.off[5]);
            a.aext = ao.aext;
        }
    }
    Q2A_HIP(q2a_launch_gemm(a, epi, blk, b->stream));
}

_Float16 * claim_a16(q2a_backend_ctx * b, const ggml_tensor * t);

_Float16 * pre16_buffer(q2a_backend_ctx * b, size_t bytes) {
    if (bytes > b->pre16_bytes) {
        abort_capture(b);
        Q2A_HIP(hipStreamSynchronize(b->stream));
        if (b->pre16) Q2A_HIP(hipFree(b->pre16));
        b->pre16 = nullptr;
        Q2A_HIP(hipMalloc((void **) &b->pre16, bytes));
        b->pre16_bytes = bytes;
        drop_graphs(b);
        resume_discard(b);
    }
    return b->pre16;
}

// fc1 -> ADD(bias) -> GELU whose output only fc2 reads (qwen2-whisper.cpp:2136-2154): fc1's epilogue writes what fc2
// consumes instead of the f32 GELU rows — for an F16 fc2 the fp16 GELU values (exact: ggml's GELU table is fp16), for a
// Q4_K fc2 the fp16 pre-activation, which the engine's GELU + Q8_K kernel turns into fc2's operand, for a Q8_0 / Q4_0
// fc2 the fp16 GELU values quantized to Q8_0. fc2 then finds its operand in place (shadow / quant_src). Same values as
// GELU_F + conversion / quantizer (the engine's fc1 paths, q2a_engine.hip run_block).
void run_fc1_for_fc2(q2a_backend_ctx * b, ggml_tensor * op, const mm_chain & c, const ggml_tensor * fc2) {
    const ggml_tensor * gelu = c.out;
    const int M = (int) (op->src[1]->ne[1] * op->src[1]->ne[2] * op->src[1]->ne[3]), F = (int) op->src[0]->ne[1];
    const int blk2 = blk_of_type(fc2->src[0]->type);
    if (blk2 == 0) {
        run_mm_fast(b, op, c.out, Q2A_EPI_GELU_H, c.bias, nullptr, 0.0f, claim_a16(b, gelu));
        return;
    }
    // fc2's operand slots first: a scratch growth now loses nothing (fc1's own operand is produced after it)
    const int N2 = (int) fc2->src[0]->ne[1];
    (void) act_slots(b, M, F, blk2, mm_part_bytes(Q2A_EPI_RESID, blk2, M, N2, F, false));
    _Float16 * pre = pre16_buffer(b, (size_t) M * F * 2);
    run_mm_fast(b, op, c.out, blk2 == 256 ? Q2A_EPI_PRE_H : Q2A_EPI_GELU_H, c.bias, nullptr, 0.0f, pre);
    const act_operand d = act_slots(b, M, F, blk2, 0);
    if (blk2 == 256) {
        Q2A_HIP(q2a_launch_gelu_quant_q8k((const q2a_half *) pre, M, F, gelu_table(b->device), (q2a_half *) d.A, d.dy,
                                          d.aext, d.MP, b->stream));
    } else {
        q2a_quant_args qa{nullptr, (const q2a_half *) pre, M, F, 2, (q2a_half *) d.A, d.dy, d.aext, d.MP};
        Q2A_HIP(q2a_launch_quant_act(qa, b->stream));
    }
    b->quant_src = gelu;
    b->quant_blk = blk2;
}

// the conv kernel duplicated into [N][2K] (w | w), cached like the repacked weights (dropped when its bytes change);
// only for tensors in a WEIGHTS buffer (the model's, qwen2-whisper.cpp:1867): any other F16 tensor may be rewritten
// by a kernel at the same address, so run_mm_conv_hilo duplicates it into the scratch on every call instead
bool is_weight_buffer(const ggml_tensor * w) {
    const ggml_tensor * t = w->view_src ? w->view_src : w;
    return t->buffer && ggml_backend_buffer_get_usage(t->buffer) == GGML_BACKEND_BUFFER_USAGE_WEIGHTS;
}

packed_w get_dup16(q2a_backend_ctx * b, const ggml_tensor * w, int N, int K, int P) {
    const int DUP16 = -16 - P;   // cache tag (not a ggml type)
    q2a_device_ctx * d = dev_ctx(b->device);
    {
        std::lock_guard<std::mutex> lk(d->mu);
        for (const packed_w & p : d->wcache)
            if (p.raw == (const char *) w->data && p.type == DUP16 && p.N == N && p.K == K) return p;
    }
    packed_w p{};
    p.raw = (const char *) w->data; p.raw_bytes = ggml_nbytes(w); p.type = DUP16; p.N = N; p.K = K;
    Q2A_HIP(hipStreamSynchronize(b->stream));
    Q2A_HIP(hipMalloc(&p.dev, (size_t) N * P * K * 2));
    const int n = N * K;
    hipLaunchKernelGGL(k_dup_rows, grid1(n), dim3(256), 0, b->stream, (const _Float16 *) w->data, (_Float16 *) p.dev, K, P, n);
    Q2A_HIP(hipStreamSynchronize(b->stream));
    std::lock_guard<std::mutex> lk(d->mu);
    d->wcache.push_back(p);
    return p;
}

// The hi/lo split writes each f32 activation x as fp16 hi = fp16(x) plus fp16 lo = fp16(x - hi) (22 significant
// bits). It assumes |x| < 65504 and |x| above the fp16 normal range (6.1e-5) for the full precision: the conv inputs
// are the normalised log-mel ((x + 4) / 4 after the clamp: [-0.75, 1.5], qwen2-whisper.cpp:2633-2649) and conv1's
// GELU output (|x| of order 1-10 for trained and synthetic weights); smaller values lose relative precision in lo only
// (absolute error < 2^-25, far below the f32 rounding of the 384/3840-term dot products). Outside that range
// (GGML_Q2A_NO_CONV_HILO=1) the exact-f32 MFMA GEMM (run_mm_f32) computes the node.
bool conv_hilo_ok(const ggml_tensor * op) {
    static const bool off = [] { const char * v = getenv("GGML_Q2A_NO_CONV_HILO"); return v && atoi(v); }();
    const ggml_tensor * x = op->src[0];
    const ggml_tensor * w = op->src[1];
    if (off || x->type != GGML_TYPE_F32 || w->type != GGML_TYPE_F16 || op->type != GGML_TYPE_F32) return false;
    if (!ggml_is_contiguous(x) || !ggml_is_contiguous(w) || !ggml_is_contiguous(op)) return false;
    if (x->ne[2] != 1 || x->ne[3] != 1 || w->ne[2] != 1 || w->ne[3] != 1) return false;
    const int64_t K = x->ne[0], M = x->ne[1], N = w->ne[1];
    return K % 64 == 0 && N % 128 == 0 && 3 * K <= 16384 && M * K < (1ll << 30) && N * K < (1ll << 30);
}

// operand parts of a conv MUL_MAT: the exact three-part split for both nodes (conv1: K = 3 x 128 mel bins; conv2:
// K = 3 x 1280, where the GELU passthrough values x >= 10 need all 24 bits)
int conv_parts(int K) { (void) K; return 3; }

// out[n][m] = sum_k x[m][k] * w[n][k] (ggml MUL_MAT with src0 = x F32, src1 = w F16): GEMM [M][N] into the scratch,
// then one transpose into the node's [N][M] layout — or, with gelu_out, into that node's: gelu(out + bias[n]) (the
// conv's ADD(bias) and GELU nodes folded into the transpose)
void run_mm_conv_hilo(q2a_backend_ctx * b, ggml_tensor * op, ggml_tensor * gelu_out = nullptr, const float * bias = nullptr) {
    const ggml_tensor * x = op->src[0];
    const ggml_tensor * w = op->src[1];
    const int K = (int) x->ne[0], M = (int) x->ne[1], N = (int) w->ne[1];
    const int P = conv_parts(K);
    const bool cached = is_weight_buffer(w);
    const packed_w wd = cached ? get_dup16(b, w, N, K, P) : packed_w{};
    const int S = q2a_gemm_resid_ksplit(M, N, P * K, 0);
    const size_t a_bytes = ((size_t) M * P * K * 2 + 255) & ~size_t(255);
    const size_t t_bytes = ((size_t) M * N * 4 + 255) & ~size_t(255);
    const size_t p_bytes = S > 1 ? ((size_t) S * M * N * 4 + 255) & ~size_t(255) : 0;
    const size_t d_bytes = cached ? 0 : (size_t) N * P * K * 2;
    char * s = (char *) scratch(b, a_bytes + t_bytes + p_bytes + d_bytes + 256);
    int * inexact = (int *) (s + a_bytes + t_bytes + p_bytes + d_bytes);
    b->quant_src = nullptr;
    const _Float16 * wdup = (const _Float16 *) wd.dev;
    if (!cached) {   // not a model weight: duplicate this call's bytes into the scratch
        _Float16 * dst = (_Float16 *) (s + a_bytes + t_bytes + p_bytes);
        hipLaunchKernelGGL(k_dup_rows, grid1((int64_t) N * K), dim3(256), 0, b->stream, (const _Float16 *) w->data, dst, K, P, N * K);
        wdup = dst;
    }
    _Float16 * A = (_Float16 *) s;
    float * tmp = (float *) (s + a_bytes);
    const int n = M * K;
    // the one-part alternative only for deep K (conv2, K = 3 x 1280: its input is the GELU table's fp16 values);
    // conv1's normalised log-mel is never fp16-valued
    const bool gated = S <= 1 && K >= 1024;
    if (gated) Q2A_HIP(hipMemsetAsync(inexact, 0, sizeof(int), b->stream));
    hipLaunchKernelGGL(k_hilo_rows, grid1(n), dim3(256), 0, b->stream, (const float *) x->data, A, K, P, n,
                       gated ? inexact : nullptr);
    q2a_gemm_args a;
    memset(&a, 0, sizeof(a));
    a.A = (const q2a_half *) A; a.lda = P * K; a.a_rpg = M; a.a_gstride = 0; a.a_step = 1;
    a.M = M; a.N = N; a.K = P * K; a.ldw = P * K;
    a.W = (const q2a_half *) wdup;
    a.outF = tmp; a.ldo = N;
    a.gelu_tab = gelu_table(b->device);
    if (S > 1) {
        a.part = (float *) (s + a_bytes + t_bytes);
        a.split_stride = (int64_t) M * N;
        a.split_store = 1;
    }
    // two launches, one of which computes: over the hi part alone when every x is an fp16 value (conv2's GELU-table
    // input, unless a value >= 10 passed through), over all P parts otherwise — the same bits either way
    a.gate = gated ? inexact : nullptr;
    a.gate_on = 1;
    Q2A_HIP(q2a_launch_gemm(a, Q2A_EPI_STORE_F, Q2A_BLK_EXACT, b->stream));
    if (a.gate) {
        q2a_gemm_args a1 = a;
        a1.K = K;
        a1.gate_on = 0;
        Q2A_HIP(q2a_launch_gemm(a1, Q2A_EPI_STORE_F, Q2A_BLK_EXACT, b->stream));
    }
    hipLaunchKernelGGL(k_transpose_f32, dim3((unsigned) ((N + 63) / 64), (unsigned) ((M + 63) / 64)), dim3(256), 0, b->stream,
                       (const float *) tmp, (float *) (gelu_out ? gelu_out->data : op->data), M, N, gelu_out ? bias : nullptr,
                       gelu_table(b->device));
}

// diagnostic (GGML_Q2A_CONV_F64=1): the conv MUL_MAT(F32 x, F16 w) summed in double, one thread per output, rounded
// to f32 once — the conv without accumulation error, to measure how much of the path's distance to the reference
// builds comes from the conv's own summation (diag/backend_tiny_variants.py)
__global__ void k_conv_f64(const float * x, const _Float16 * w, float * out, int M, int N, int K) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t) M * N) return;
    const int m = (int) (i % M), n = (int) (i / M);
    const float * xr = x + (int64_t) m * K;
    const _Float16 * wr = w + (int64_t) n * K;
    double acc = 0.0;
    for (int k = 0; k < K; ++k) acc += (double) xr[k] * (double) (float) wr[k];
    out[(int64_t) n * M + m] = (float) acc;
}
bool conv_f64_diag(const ggml_tensor * op) {
    static const bool on = [] { const char * v = getenv("GGML_Q2A_CONV_F64"); return v && atoi(v); }();
    const ggml_tensor * x = op->src[0];
    const ggml_tensor * w = op->src[1];
    return on && x->type == GGML_TYPE_F32 && w->type == GGML_TYPE_F16 && op->type == GGML_TYPE_F32 &&
           ggml_is_contiguous(x) && ggml_is_contiguous(w) && ggml_is_contiguous(op) && x->ne[2] == 1 && x->ne[3] == 1 &&
           w->ne[2] == 1 && w->ne[3] == 1;
}
void run_mm_conv_f64(q2a_backend_ctx * b, ggml_tensor * op) {
    const ggml_tensor * x = op->src[0];
    const ggml_tensor * w = op->src[1];
    const int K = (int) x->ne[0], M = (int) x->ne[1], N = (int) w->ne[1];
    b->quant_src = nullptr;
    hipLaunchKernelGGL(k_conv_f64, grid1((int64_t) M * N), dim3(256), 0, b->stream, (const float *) x->data,
                       (const _Float16 *) w->data, (float *) op->data, M, N, K);
}

void run_mm_f32(q2a_backend_ctx * b, ggml_tensor * op) {
    const ggml_tensor * s0 = op->src[0];
    const ggml_tensor * s1 = op->src[1];
    mm_args p;
    p.a = tv(s0); p.b = tv(s1); p.d = tv(op);
    p.ta = s0->type; p.tb = s1->type;
    p.K = s0->ne[0];
    p.r2 = s1->ne[2] / s0->ne[2];
    p.r3 = s1->ne[3] / s0->ne[3];
    const dim3 g((unsigned) ((op->ne[0] + 63) / 64), (unsigned) ((op->ne[1] + 63) / 64), (unsigned) (op->ne[2] * op->ne[3]));
    if (s0->type == GGML_TYPE_F16) hipLaunchKernelGGL(k_mm_f32<true>, g, dim3(256), 0, b->stream, p);
    else hipLaunchKernelGGL(k_mm_f32<false>, g, dim3(256), 0, b->stream, p);
}

// KQ = MUL_MAT(K, Q) -> SOFT_MAX(KQ, no mask) -> KQV = MUL_MAT(V, KQ_soft_max), heads of 64 (qwen2-whisper.cpp:
// 2052-2106): when nodes i..i+2 form exactly this chain and KQ / KQ_soft_max feed nothing else, run it as the
// engine's flash kernel and skip the 20 x T x T score tensors. Returns the number of nodes consumed (0 = no match).
// KQ -> SOFT_MAX -> KQV at nodes i..i+2 with K, Q, V views the fused kernel accepts (no other consumer of the score
// tensors); returns the KQV node or null
ggml_tensor * match_attention(ggml_cgraph * g, int i) {
    static const bool off = [] { const char * v = getenv("GGML_Q2A_NO_FUSED_ATTN"); return v && atoi(v); }();
    if (off || i + 2 >= ggml_graph_n_nodes(g)) return nullptr;
    ggml_tensor * kq = ggml_graph_node(g, i);
    ggml_tensor * sm = ggml_graph_node(g, i + 1);
    ggml_tensor * kqv = ggml_graph_node(g, i + 2);
    if (kq->op != GGML_OP_MUL_MAT || sm->op != GGML_OP_SOFT_MAX || kqv->op != GGML_OP_MUL_MAT) return nullptr;
    if (sm->src[0] != kq || sm->src[1] != nullptr || kqv->src[1] != sm) return nullptr;
    float scale, max_bias;
    memcpy(&scale, (const float *) sm->op_params + 0, 4);
    memcpy(&max_bias, (const float *) sm->op_params + 1, 4);
    if (scale != 1.0f || max_bias != 0.0f) return nullptr;
    // the score tensors must be used by this chain only
    for (int j = 0; j < ggml_graph_n_nodes(g); ++j) {
        ggml_tensor * n = ggml_graph_node(g, j);
        if (n == sm || n == kqv) continue;
        for (int s = 0; s < GGML_MAX_SRC; ++s)
            if (n->src[s] == kq || n->src[s] == sm) return nullptr;
    }
    if ((kq->flags | sm->flags) & GGML_TENSOR_FLAG_OUTPUT) return nullptr;
    const ggml_tensor * K = kq->src[0];
    const ggml_tensor * Q = kq->src[1];
    const ggml_tensor * V = kqv->src[0];
    const int64_t T = Q->ne[1], H = Q->ne[2];
    auto f32 = [](const ggml_tensor * t) { return t->type == GGML_TYPE_F32 && t->nb[0] == 4 && t->ne[3] == 1; };
    if (!f32(K) || !f32(Q) || !f32(V) || kqv->type != GGML_TYPE_F32 || kqv->ne[3] != 1) return nullptr;
    if (Q->ne[0] != 64 || K->ne[0] != 64 || K->ne[1] != T || K->ne[2] != H) return nullptr;
    if (V->ne[0] != T || V->ne[1] != 64 || V->ne[2] != H) return nullptr;
    if (kqv->ne[0] != 64 || kqv->ne[1] != T || kqv->ne[2] != H) return nullptr;
    if (T * H * 64 >= (1ll << 31)) return nullptr;
    return kqv;
}

_Float16 * vt_buffer(q2a_backend_ctx * b, size_t bytes) {
    if (bytes > b->vt_bytes) {
        abort_capture(b);
        Q2A_HIP(hipStreamSynchronize(b->stream));
        if (b->vt_buf) Q2A_HIP(hipFree(b->vt_buf));
        b->vt_buf = nullptr;
        Q2A_HIP(hipMalloc((void **) &b->vt_buf, bytes));
        b->vt_bytes = bytes;
        drop_graphs(b);
        resume_discard(b);
    }
    return b->vt_buf;
}

// a shadow slot for the fp16 copy of tensor t (the slot not written last)
_Float16 * claim_a16(q2a_backend_ctx * b, const ggml_tensor * t) {
    const int k = 1 - b->a16_last;
    const size_t bytes = (size_t) ggml_nelements(t) * 2;
    if (bytes > b->a16_bytes[k]) {
        abort_capture(b);
        Q2A_HIP(hipStreamSynchronize(b->stream));
        if (b->a16[k]) Q2A_HIP(hipFree(b->a16[k]));
        b->a16[k] = nullptr;
        Q2A_HIP(hipMalloc((void **) &b->a16[k], bytes));
        b->a16_bytes[k] = bytes;
        drop_graphs(b);
        resume_discard(b);
    }
    b->a16_last = k;
    b->a16_src[k] = t;
    return b->a16[k];
}

// vt_ready: V^T was already written into b->vt_buf at V's CONT node. merged: the CONT of permute(KQV, 0,2,1,3)
// that follows (qwen2-whisper.cpp:2105-2107), whose [t][h*64+d] rows are exactly the fused kernel's output rows —
// the kernel writes them there directly. Returns the number of nodes consumed.
struct qkv_ops {                   // the attention operands as the fused Q|K|V GEMM wrote them (qkv_buffer layout)
    _Float16 *qh, *ql, *kh, *kl, *vt, *vtl;
};

// out16: the merged output's fp16 shadow (its only consumer an F16-weight MUL_MAT): written instead of the f32 rows
int run_fused_attention(q2a_backend_ctx * b, ggml_cgraph * g, int i, bool vt_ready, ggml_tensor * merged,
                        const qkv_ops * ready = nullptr, _Float16 * out16 = nullptr) {
    ggml_tensor * kq = ggml_graph_node(g, i);
    ggml_tensor * kqv = ggml_graph_node(g, i + 2);
    const ggml_tensor * K = kq->src[0];
    const ggml_tensor * Q = kq->src[1];
    const ggml_tensor * V = kqv->src[0];
    const int64_t T = Q->ne[1], H = Q->ne[2];
    const int TP = (int) ((T + 63) / 64 * 64);
    const int64_t D = H * 64, n = T * D;
    const size_t hb = ((size_t) n * 2 + 255) & ~size_t(255);
    const bool vlo = q2a_attention_wants_vlo();
    const size_t vb1 = ((size_t) H * 64 * TP * 2 + 255) & ~size_t(255);
    const size_t vb = vlo ? 2 * vb1 : vb1;   // V^T [| V^T lo]
#ifdef Q2A_DIAG_DUMP_ATTN   // diagnostic builds only: the first attention's operands of a process -> $Q2A_DUMP_ATTN
    auto dump = [&](const _Float16 * qh, const _Float16 * ql, const _Float16 * kh, const _Float16 * kl, const _Float16 * vt,
                    const _Float16 * vtl) {
        static bool done = false;
        const char * path = getenv("Q2A_DUMP_ATTN");
        if (done || !path) return;
        done = true;
        Q2A_HIP(hipStreamSynchronize(b->stream));
        FILE * f = fopen(path, "wb");
        const size_t nq = (size_t) n * 2, nv = (size_t) H * 64 * TP * 2;
        std::vector<char> h(std::max(nq, nv));
        for (const _Float16 * x : {qh, ql, kh, kl}) { Q2A_HIP(hipMemcpy(h.data(), x, nq, hipMemcpyDeviceToHost)); fwrite(h.data(), 1, nq, f); }
        for (const _Float16 * x : {vt, vtl}) { if (!x) continue; Q2A_HIP(hipMemcpy(h.data(), x, nv, hipMemcpyDeviceToHost)); fwrite(h.data(), 1, nv, f); }
        fclose(f);
    };
    if (ready) dump(ready->qh, ready->ql, ready->kh, ready->kl, ready->vt, ready->vtl);
    {   // the Q tensor the separate route feeds its operand pass (f32 [T][D]) -> $Q2A_DUMP_ATTN.q
        static bool qdone = false;
        const char * path = getenv("Q2A_DUMP_ATTN");
        if (!ready && !qdone && path) {
            qdone = true;
            Q2A_HIP(hipStreamSynchronize(b->stream));
            std::vector<float> h((size_t) n);
            Q2A_HIP(hipMemcpy(h.data(), Q->data, (size_t) n * 4, hipMemcpyDeviceToHost));
            FILE * f = fopen((std::string(path) + ".q").c_str(), "wb");
            fwrite(h.data(), 4, h.size(), f);
            fclose(f);
        }
    }
#define Q2A_DUMP_PREP() dump(qh, ql, kh, kl, vt, vtl)
#else
#define Q2A_DUMP_PREP() do { } while (0)
#endif
    if (ready) {   // operands already in place (run_qkv_fused): only the kernel (and the output re-layout) runs
        float * o = merged ? (float *) merged->data : (float *) scratch(b, (size_t) n * 4);
        if (!merged) b->quant_src = nullptr;
        q2a_attn_args at{(const q2a_half *) ready->qh, (const q2a_half *) ready->ql, (const q2a_half *) ready->kh,
                         (const q2a_half *) ready->kl, (const q2a_half *) ready->vt, 1, (int) T, (int) D, (int) H, TP, nullptr, o};
        at.vtl = ready->vtl;
        at.v_rows = 1;   // (run_qkv_fused writes V row-major)
        if (out16 && merged) { at.outH = (q2a_half *) out16; at.outF = nullptr; }
        Q2A_HIP(q2a_launch_attention(at, b->stream));
        if (!merged)
            hipLaunchKernelGGL(k_attn_out, grid1(n), dim3(256), 0, b->stream, (const float *) o, tv(kqv), (int) T, (int) H, n);
        b->stats.n_attn_fused++;
        return merged ? 5 : 3;
    }
    char * s = (char *) scratch(b, 4 * hb + vb + (size_t) n * 4);
    b->quant_src = nullptr;   // the attention operands overwrite the scratch
    _Float16 *qh = (_Float16 *) s, *ql = (_Float16 *) (s + hb), *kh = (_Float16 *) (s + 2 * hb), *kl = (_Float16 *) (s + 3 * hb);
    _Float16 * vt = vt_ready ? b->vt_buf : (_Float16 *) (s + 4 * hb);
    _Float16 * vtl = vlo ? (_Float16 *) ((char *) vt + vb1) : nullptr;
    float * o = merged ? (float *) merged->data : (float *) (s + 4 * hb + vb);
    if (vt_ready) {
        hipLaunchKernelGGL(k_attn_prep<false>, grid1(n), dim3(256), 0, b->stream, tv(Q), tv(K), tv(V), qh, ql, kh, kl, vt,
                           vtl, (int) T, (int) H, TP, n);
    } else {
        Q2A_HIP(hipMemsetAsync(vt, 0, vb, b->stream));   // V^T tail columns past T are read as zero weights
        hipLaunchKernelGGL(k_attn_prep<true>, grid1(n), dim3(256), 0, b->stream, tv(Q), tv(K), tv(V), qh, ql, kh, kl, vt,
                           vtl, (int) T, (int) H, TP, n);
    }
    Q2A_DUMP_PREP();
#undef Q2A_DUMP_PREP
    q2a_attn_args at{(const q2a_half *) qh, (const q2a_half *) ql, (const q2a_half *) kh, (const q2a_half *) kl,
                     (const q2a_half *) vt, 1, (int) T, (int) D, (int) H, TP, nullptr, o};
    at.vtl = vtl;
    if (out16 && merged) { at.outH = (q2a_half *) out16; at.outF = nullptr; }
    Q2A_HIP(q2a_launch_attention(at, b->stream));
    if (!merged)
        hipLaunchKernelGGL(k_attn_out, grid1(n), dim3(256), 0, b->stream, (const float *) o, tv(kqv), (int) T, (int) H, n);
    b->stats.n_attn_fused++;
    return merged ? 5 : 3;
}

// ---- the Q | K | V projections as ONE GEMM whose epilogue writes the fused attention's operands (the engine's
// Q2A_EPI_QKV: Q (+bias) * scale * log2 e and K as fp16 hi/lo pairs, V (+bias) as V^T [h][d][TP] hi (| lo)), replacing
// two launches (K|Q grouped, V), the V^T tile pass at V's CONT and the attention's operand pass
// (qwen2-whisper.cpp:2029-2054 projections, :2052-2089 the attention's K, Q, V views)
struct qkv_route {
    ggml_tensor * mm[3];            // Q, K, V MUL_MATs (same activation, same weight type and shape)
    const ggml_tensor * bq, * bv;   // bias rows of Q and V (the reference's K has none, :2039)
    float qscale;                   // ggml_scale after Q's bias (a power of two: KQscale = 1/8 for heads of 64)
};

// the weights as one [3N][K] operand: fp16 rows concatenated (F16), or the three packed images' sections concatenated
// along N (every section of q2a_pack_linear's layout is row- or block-major over N, so this IS the packed image of the
// concatenated rows). Cached with the repacks under a key spanning the three source tensors: a write to any drops it.
packed_w get_qkv_weight(q2a_backend_ctx * b, const ggml_tensor * const w[3]) {
    const int TAG = -64 - (int) w[0]->type;   // cache tag (not a ggml type)
    const int N = (int) w[0]->ne[1], K = (int) w[0]->ne[0];
    const char * lo = (const char *) w[0]->data, * hi = lo + ggml_nbytes(w[0]);
    for (int i = 1; i < 3; ++i) {
        lo = std::min(lo, (const char *) w[i]->data);
        hi = std::max(hi, (const char *) w[i]->data + ggml_nbytes(w[i]));
    }
    q2a_device_ctx * d = dev_ctx(b->device);
    {
        std::lock_guard<std::mutex> lk(d->mu);
        for (const packed_w & p : d->wcache)
            if (p.raw == lo && p.raw_bytes == (size_t) (hi - lo) && p.type == TAG && p.N == 3 * N && p.K == K) return p;
    }
    packed_w p{};
    p.raw = lo; p.raw_bytes = (size_t) (hi - lo); p.type = TAG; p.N = 3 * N; p.K = K;
    Q2A_HIP(hipStreamSynchronize(b->stream));
    if (w[0]->type == GGML_TYPE_F16) {
        const size_t rb = (size_t) N * K * 2;
        Q2A_HIP(hipMalloc(&p.dev, 3 * rb));
        for (int i = 0; i < 3; ++i) Q2A_HIP(hipMemcpyAsync((char *) p.dev + i * rb, w[i]->data, rb, hipMemcpyDeviceToDevice, b->stream));
    } else {
        const int blk = w[0]->type == GGML_TYPE_Q4_K ? 256 : 32, nblk = K / blk;
        const uint64_t bytes = q2a_pack_layout(w[0]->type, 3 * N, K, p.off);
        if (!bytes) GGML_ABORT("ggml-q2a: cannot pack the Q|K|V weights of %s", w[0]->name);
        Q2A_HIP(hipMalloc(&p.dev, bytes));
        char * dst = (char *) p.dev;
        for (int i = 0; i < 3; ++i) {
            const packed_w s = get_packed(b, w[i]);
            const char * src = (const char *) s.dev;
            Q2A_HIP(hipMemcpyAsync(dst + p.off[0] + (size_t) i * N * K * 2, src + s.off[0], (size_t) N * K * 2,
                                   hipMemcpyDeviceToDevice, b->stream));
            // block-major sections [nblk][N] x element bytes: dx (and dmin, wext (16 halves), beta, gamma for Q4_K)
            const int secs[5] = {1, 2, 3, 4, 5};
            const int esz[6] = {0, 4, 4, 32, 4, 4};
            for (int k = 0; k < (blk == 256 ? 5 : 1); ++k) {
                const int sc = secs[k];
                const size_t e = (size_t) esz[sc];
                Q2A_HIP(hipMemcpy2DAsync(dst + p.off[sc] + i * N * e, 3 * N * e, src + s.off[sc], N * e, N * e, nblk,
                                         hipMemcpyDeviceToDevice, b->stream));
            }
        }
    }
    Q2A_HIP(hipStreamSynchronize(b->stream));
    std::lock_guard<std::mutex> lk(d->mu);
    // the per-tensor images of Q, K and V (upload-time or lazy repacks) are not read again while the fused route is on:
    // released, so the expanded QKV weights are resident once (a graph that still needed one repacks it lazily; once any
    // graph has been captured on the device, the wgen bump keeps those that may hold their pointers from being replayed —
    // before that, nothing holds them and the capture schedule stays as it was)
    for (size_t j = 0; j < d->wcache.size();) {
        const packed_w & c = d->wcache[j];
        bool own = false;
        for (int i = 0; i < 3; ++i)
            own |= c.raw == (const char *) w[i]->data && c.type == w[i]->type && c.N == N && c.K == K;
        if (own) {
            (void) hipFree(c.dev);
            if (d->n_captured.load() > 0) ++d->wgen;
            d->wcache[j] = d->wcache.back();
            d->wcache.pop_back();
        } else {
            ++j;
        }
    }
    d->wcache.push_back(p);
    return p;
}

// [bq | 0 | bv] as one f32 bias row (cached like the weights)
const float * get_qkv_bias(q2a_backend_ctx * b, const ggml_tensor * bq, const ggml_tensor * bv, int N) {
    const int TAG = -200;
    const char * lo = std::min((const char *) bq->data, (const char *) bv->data);
    const char * hi = std::max((const char *) bq->data + ggml_nbytes(bq), (const char *) bv->data + ggml_nbytes(bv));
    q2a_device_ctx * d = dev_ctx(b->device);
    {
        std::lock_guard<std::mutex> lk(d->mu);
        for (const packed_w & p : d->wcache)
            if (p.raw == lo && p.raw_bytes == (size_t) (hi - lo) && p.type == TAG && p.N == 3 * N) return (const float *) p.dev;
    }
    packed_w p{};
    p.raw = lo; p.raw_bytes = (size_t) (hi - lo); p.type = TAG; p.N = 3 * N; p.K = 1;
    Q2A_HIP(hipStreamSynchronize(b->stream));
    Q2A_HIP(hipMalloc(&p.dev, (size_t) 3 * N * 4));
    Q2A_HIP(hipMemsetAsync(p.dev, 0, (size_t) 3 * N * 4, b->stream));
    Q2A_HIP(hipMemcpyAsync(p.dev, bq->data, (size_t) N * 4, hipMemcpyDeviceToDevice, b->stream));
    Q2A_HIP(hipMemcpyAsync((char *) p.dev + (size_t) 2 * N * 4, bv->data, (size_t) N * 4, hipMemcpyDeviceToDevice, b->stream));
    Q2A_HIP(hipStreamSynchronize(b->stream));
    std::lock_guard<std::mutex> lk(d->mu);
    d->wcache.push_back(p);
    return (const float *) p.dev;
}

// the operand buffer (zero-filled when it grows: V^T's columns t >= T are read as zero weights)
char * qkv_buffer(q2a_backend_ctx * b, size_t bytes) {
    if (bytes > b->qkv_bytes) {
        abort_capture(b);
        Q2A_HIP(hipStreamSynchronize(b->stream));
        if (b->qkv_buf) Q2A_HIP(hipFree(b->qkv_buf));
        b->qkv_buf = nullptr;
        Q2A_HIP(hipMalloc((void **) &b->qkv_buf, bytes));
        Q2A_HIP(hipMemsetAsync(b->qkv_buf, 0, bytes, b->stream));
        Q2A_HIP(hipStreamSynchronize(b->stream));
        b->qkv_bytes = bytes;
        drop_graphs(b);
        resume_discard(b);
    }
    return b->qkv_buf;
}

void run_qkv_fused(q2a_backend_ctx * b, const qkv_route & r, qkv_ops & ops) {
    const ggml_tensor * x = r.mm[0]->src[1];
    const int K = (int) x->ne[0], M = (int) x->ne[1], D = (int) r.mm[0]->src[0]->ne[1], H = D / 64, T = M;
    const int TP = (T + 63) / 64 * 64;
    const ggml_tensor * const w[3] = {r.mm[0]->src[0], r.mm[1]->src[0], r.mm[2]->src[0]};
    const int blk = w[0]->type == GGML_TYPE_Q4_K ? 256 : w[0]->type == GGML_TYPE_F16 ? 0 : 32;
    const packed_w pw = get_qkv_weight(b, w);
    const float * bias = get_qkv_bias(b, r.bq, r.bv, D);
    const bool vlo = q2a_attention_wants_vlo();
    const size_t hb = ((size_t) T * D * 2 + 255) & ~size_t(255);
    const size_t vb1 = ((size_t) D * TP * 2 + 255) & ~size_t(255);
    char * ob = qkv_buffer(b, 4 * hb + (vlo ? 2 : 1) * vb1);
    ops = {(_Float16 *) ob, (_Float16 *) (ob + hb), (_Float16 *) (ob + 2 * hb), (_Float16 *) (ob + 3 * hb),
           (_Float16 *) (ob + 4 * hb), vlo ? (_Float16 *) (ob + 4 * hb + vb1) : nullptr};
    const act_operand ao = activation_operand(b, x, M, K, blk, 0);
    // (V hi / lo row-major: no pad columns; the attention clamps its key rows to T - 1)
    q2a_gemm_args a;
    memset(&a, 0, sizeof(a));
    a.A = ao.A; a.lda = K; a.a_rpg = M; a.a_gstride = 0; a.a_step = 1;
    a.M = M; a.N = 3 * D; a.K = K; a.ldw = K;
    a.bias = bias;
    a.qh = (q2a_half *) ops.qh; a.ql = (q2a_half *) ops.ql; a.kh = (q2a_half *) ops.kh; a.kl = (q2a_half *) ops.kl;
    a.vt = (q2a_half *) ops.vt; a.vtl = (q2a_half *) ops.vtl;
    a.v_rows = 1;   // V hi / lo row-major [T][D] like K (the attention below reads it with k_attn_t<true>)
    a.T = T; a.D = D; a.H = H; a.TP = TP;
    // (x + b) * s then * log2 e in the unfused path; s = 2^-k makes one multiply by s * log2 e the same rounding
    a.qscale = r.qscale * Q2A_LOG2E;
    a.gelu_tab = gelu_table(b->device);
    const char * base = (const char *) pw.dev;
    a.W = (const q2a_half *) (base + pw.off[0]);
    if (blk) {
        a.nblk = K / blk;
        a.dx = (const float *) (base + pw.off[1]);
        a.dy = ao.dy; a.dy_ld = ao.MP;
        if (blk == 256) {
            a.dmin = (const float *) (base + pw.off[2]);
            a.wext = (const q2a_half *) (base + pw.off[3]);
            a.beta = (const float *) (base + pw.off[4]);
            a.gamma = (const float *) (base + pw.off[5]);
            a.aext = ao.aext;
        }
    }
    Q2A_HIP(q2a_launch_gemm(a, Q2A_EPI_QKV, blk, b->stream));
#ifdef Q2A_DIAG_DUMP_ATTN   // diagnostic builds only: (acc + bias) * qscale of the same GEMM as f32 -> $Q2A_DUMP_ATTN.q
    static bool qdone = false;
    const char * path = getenv("Q2A_DUMP_ATTN");
    if (!qdone && path) {
        qdone = true;
        float * y = nullptr;
        Q2A_HIP(hipMalloc((void **) &y, (size_t) M * 3 * D * 4));
        q2a_gemm_args c = a;
        c.outF = y; c.ldo = 3 * D; c.store_bias = 1; c.out_scale = r.qscale;
        Q2A_HIP(q2a_launch_gemm(c, Q2A_EPI_STORE_F, blk, b->stream));
        Q2A_HIP(hipStreamSynchronize(b->stream));
        std::vector<float> h((size_t) M * 3 * D);
        Q2A_HIP(hipMemcpy(h.data(), y, h.size() * 4, hipMemcpyDeviceToHost));
        FILE * f = fopen((std::string(path) + ".q").c_str(), "wb");
        for (int m = 0; m < M; ++m) fwrite(h.data() + (size_t) m * 3 * D, 4, D, f);
        fclose(f);
        Q2A_HIP(hipFree(y));
    }
#endif
}

bool op_supported(const ggml_tensor * op) {
    auto f32 = [](const ggml_tensor * t) { return t && t->type == GGML_TYPE_F32; };
    auto f = [](const ggml_tensor * t) { return t && (t->type == GGML_TYPE_F32 || t->type == GGML_TYPE_F16); };
    switch (op->op) {
        case GGML_OP_NONE: case GGML_OP_RESHAPE: case GGML_OP_VIEW: case GGML_OP_PERMUTE: case GGML_OP_TRANSPOSE:
            return true;
        case GGML_OP_MUL_MAT: {
            const ggml_tensor * a = op->src[0];
            const ggml_tensor * x = op->src[1];
            if (op->type != GGML_TYPE_F32 || a->ne[2] == 0 || a->ne[3] == 0) return false;
            if (x->ne[2] % a->ne[2] || x->ne[3] % a->ne[3]) return false;
            if (mm_fast_ok(op)) return true;
            return f(a) && f(x) && a->nb[0] == ggml_type_size(a->type) && x->nb[0] == ggml_type_size(x->type);
        }
        case GGML_OP_ADD: case GGML_OP_MUL:
            return f32(op) && f32(op->src[0]) && f32(op->src[1]) && ggml_can_repeat(op->src[1], op->src[0]);
        case GGML_OP_SCALE:
            return f32(op) && f32(op->src[0]);
        case GGML_OP_NORM: case GGML_OP_SOFT_MAX:
            if (op->op == GGML_OP_SOFT_MAX && op->src[1]) return false;   // masks / ALiBi are not on this path
            return f32(op) && f32(op->src[0]) && op->src[0]->nb[0] == 4 && op->nb[0] == 4;
        case GGML_OP_UNARY:
            return ggml_get_unary_op(op) == GGML_UNARY_OP_GELU && f32(op) && f32(op->src[0]);
        case GGML_OP_CONT: case GGML_OP_DUP: case GGML_OP_CPY:
            return f(op) && f(op->src[0]) && ggml_nelements(op) == ggml_nelements(op->src[0]);
        case GGML_OP_IM2COL:
            return ((const int32_t *) op->op_params)[6] == 0 && f32(op->src[1]) && op->src[1]->nb[0] == 4 && f(op) &&
                   ggml_is_contiguous(op);
        case GGML_OP_POOL_1D: {
            const int32_t * pp = (const int32_t *) op->op_params;
            return pp[0] == GGML_OP_POOL_AVG && pp[1] == pp[2] && pp[3] == 0 && f32(op) && f32(op->src[0]);
        }
        default:
            return false;
    }
}

// the launcher would take the 8-phase kernels, whose GELU epilogue reads a compact LDS table this backend does not build
bool mm_is_pipe8(const ggml_tensor * op) {
    const int64_t M = op->src[1]->ne[1] * op->src[1]->ne[2] * op->src[1]->ne[3];
    return q2a_gemm_wide_tiles((int) M, (int) op->src[0]->ne[1], 0);
}

bool is_view_op(const ggml_tensor * t) {
    return t->op == GGML_OP_NONE || t->op == GGML_OP_RESHAPE || t->op == GGML_OP_VIEW || t->op == GGML_OP_PERMUTE ||
           t->op == GGML_OP_TRANSPOSE || ggml_is_empty(t);
}

bool rows_f32(const ggml_tensor * t) { return t->type == GGML_TYPE_F32 && t->nb[0] == 4; }
bool row_vec_f32(const ggml_tensor * t, int64_t n) {
    return rows_f32(t) && t->ne[0] == n && t->ne[1] == 1 && t->ne[2] == 1 && t->ne[3] == 1 && ((uintptr_t) t->data & 15) == 0;
}
bool aligned16(const ggml_tensor * t) {
    return ((uintptr_t) t->data & 15) == 0 && t->nb[1] % 16 == 0 && t->nb[2] % 16 == 0 && t->nb[3] % 16 == 0;
}

// ADD / MUL / SCALE / GELU on the row kernel when the shapes allow it (true), else false (generic kernel)
bool launch_rows(q2a_backend_ctx * b, int op_kind, const ggml_tensor * a, const ggml_tensor * y, const ggml_tensor * z,
                 float scale) {
    if (!rows_f32(a) || !rows_f32(y) || (z && !rows_f32(z))) return false;
    for (int k = 0; k < 4; ++k) if (a->ne[k] != y->ne[k]) return false;
    const int64_t ne0 = y->ne[0], nrows = y->ne[1] * y->ne[2] * y->ne[3];
    if (ne0 <= 0 || nrows <= 0 || ne0 > (1 << 30) || nrows > (1ll << 30) * 2 - 4) return false;
    const bool zs = z && z->ne[0] == 1 && ne0 != 1;
    if (z && !zs && z->ne[0] != ne0) return false;
    const bool v4 = ne0 % 4 == 0 && aligned16(a) && aligned16(y) && (!z || zs || aligned16(z));
    const tview ta = tv(a), tz = z ? tv(z) : ta, ty = tv(y);
    const dim3 grid((unsigned) ((nrows + 3) / 4));
    const uint16_t * gt = op_kind == 3 ? gelu_table(b->device) : nullptr;
#define Q2A_ROWS(OP)                                                                                                  \
    do {                                                                                                              \
        if (v4) hipLaunchKernelGGL((k_rows<OP, true>), grid, dim3(256), 0, b->stream, ta, tz, ty, (int) nrows, scale, gt); \
        else hipLaunchKernelGGL((k_rows<OP, false>), grid, dim3(256), 0, b->stream, ta, tz, ty, (int) nrows, scale, gt);   \
    } while (0)
    switch (op_kind) {
        case 0: Q2A_ROWS(0); break;
        case 1: Q2A_ROWS(1); break;
        case 2: Q2A_ROWS(2); break;
        default: Q2A_ROWS(3); break;
    }
#undef Q2A_ROWS
    return true;
}

ggml_status run_nodes(q2a_backend_ctx * b, ggml_cgraph * g) {
    static const bool no_fuse = [] { const char * v = getenv("GGML_Q2A_NO_FUSE"); return v && atoi(v); }();
    b->stats = ggml_backend_q2a_stats{};
    const int nn = ggml_graph_n_nodes(g);
    // consumers per tensor within this graph: a node is folded into its producer's kernel only when it is the
    // producer's sole consumer (views count as consumers) and the producer is not a graph output
    std::unordered_map<const ggml_tensor *, int> uses;
    if (!no_fuse) {
        uses.reserve((size_t) nn * 2);
        for (int j = 0; j < nn; ++j) {
            const ggml_tensor * t = ggml_graph_node(g, j);
            for (int k = 0; k < GGML_MAX_SRC; ++k) if (t->src[k]) uses[t->src[k]]++;
        }
    }
    auto sole = [&](const ggml_tensor * producer, const ggml_tensor * consumer) {
        if (no_fuse || (producer->flags & GGML_TENSOR_FLAG_OUTPUT)) return false;
        auto it = uses.find(producer);
        if (it == uses.end() || it->second != 1) return false;
        for (int k = 0; k < GGML_MAX_SRC; ++k) if (consumer->src[k] == producer) return true;
        return false;
    };
    auto node = [&](int j) -> ggml_tensor * { return j < nn ? ggml_graph_node(g, j) : nullptr; };
    auto same_shape_rows = [](const ggml_tensor * x, const ggml_tensor * y) {
        for (int k = 0; k < 4; ++k) if (x->ne[k] != y->ne[k]) return false;
        return ggml_is_contiguous(x) && ggml_is_contiguous(y) && x->type == GGML_TYPE_F32 && y->type == GGML_TYPE_F32;
    };
    // the SCALE node fed by `prod` (directly or through one contiguous RESHAPE view) at node j, when every link is the
    // sole consumer of the one before: its bytes are prod's bytes times the scale
    auto scale_after = [&](ggml_tensor * prod, int j) -> ggml_tensor * {
        ggml_tensor * t = node(j);
        if (t && t->op == GGML_OP_RESHAPE && t->src[0] == prod && sole(prod, t)) {
            prod = t;
            t = node(j + 1);
        }
        if (!t || t->op != GGML_OP_SCALE || t->src[0] != prod || !sole(prod, t) || t->type != GGML_TYPE_F32 ||
            !ggml_is_contiguous(t) || !ggml_is_contiguous(prod) || ggml_nelements(t) != ggml_nelements(prod) ||
            ((uintptr_t) t->data & 15) != 0 || *(const float *) t->op_params == 0.0f)
            return nullptr;
        return t;
    };
    // V CONT nodes feeding a fused attention as its sole consumer: they produce the attention's V^T operand
    std::unordered_map<const ggml_tensor *, int> vprep;
    const ggml_tensor * vt_ready_for = nullptr;
    // f32 activations some F16-weight MUL_MAT converts to fp16: their producer also writes the fp16 copy
    std::unordered_map<const ggml_tensor *, int> want16;
    b->a16_src[0] = b->a16_src[1] = nullptr;
    b->a16_last = 1;   // slot assignment deterministic per cgraph: a replayed capture sees the same slots as its run
    b->quant_src = nullptr;
    if (!no_fuse) {
        for (int j = 0; j < nn; ++j) {
            const ggml_tensor * t = ggml_graph_node(g, j);
            if (t->op == GGML_OP_MUL_MAT && t->src[0]->type == GGML_TYPE_F16 && mm_fast_ok(t)) want16[t->src[1]] = j;
        }
        for (int j = 0; j + 2 < nn; ++j) {
            ggml_tensor * kqv = match_attention(g, j);
            if (!kqv) continue;
            ggml_tensor * V = kqv->src[0];
            if (V->op == GGML_OP_CONT && sole(V, kqv) && V->src[0] && V->src[0]->type == GGML_TYPE_F32 &&
                ggml_are_same_shape(V, V->src[0]) && V->ne[1] == 64)
                vprep[V] = j;
        }
    }
    // Q | K | V projections feeding a fused attention through exactly the reference's views (qwen2-whisper.cpp:
    // 2029-2089): K = PERMUTE(RESHAPE(MUL_MAT)), Q = PERMUTE(SCALE(RESHAPE(ADD(MUL_MAT, bq)))),
    // V = CONT(PERMUTE(RESHAPE(ADD(MUL_MAT, bv)))), every link its producer's sole consumer, the three MUL_MATs on one
    // activation with weights of one type and shape in a weights buffer: one GEMM (run_qkv_fused) then replaces
    // them, and the attention reads its operands from it
    static const bool no_qkv = [] { const char * v = getenv("GGML_Q2A_NO_FUSED_QKV"); return v && atoi(v); }();
    auto match_qkv = [&](ggml_tensor * kq, ggml_tensor * kqv, qkv_route & r, std::vector<const ggml_tensor *> & absorbed) {
        auto is = [](const ggml_tensor * t, ggml_op o) { return t && t->op == o; };
        ggml_tensor * kp = kq->src[0];
        if (!is(kp, GGML_OP_PERMUTE) || !sole(kp, kq)) return false;
        ggml_tensor * kr = kp->src[0];
        if (!is(kr, GGML_OP_RESHAPE) || !sole(kr, kp)) return false;
        ggml_tensor * km = kr->src[0];
        if (!is(km, GGML_OP_MUL_MAT) || !sole(km, kr)) return false;
        ggml_tensor * qp = kq->src[1];
        if (!is(qp, GGML_OP_PERMUTE) || !sole(qp, kq)) return false;
        ggml_tensor * qs = qp->src[0];
        if (!is(qs, GGML_OP_SCALE) || !sole(qs, qp)) return false;
        ggml_tensor * qr = qs->src[0];
        if (!is(qr, GGML_OP_RESHAPE) || !sole(qr, qs)) return false;
        ggml_tensor * qa = qr->src[0];
        if (!is(qa, GGML_OP_ADD) || !sole(qa, qr)) return false;
        ggml_tensor * qm = qa->src[0];
        if (!is(qm, GGML_OP_MUL_MAT) || !sole(qm, qa)) return false;
        ggml_tensor * vc = kqv->src[0];
        if (!is(vc, GGML_OP_CONT) || !sole(vc, kqv)) return false;
        ggml_tensor * vp = vc->src[0];
        if (!is(vp, GGML_OP_PERMUTE) || !sole(vp, vc)) return false;
        ggml_tensor * vr = vp->src[0];
        if (!is(vr, GGML_OP_RESHAPE) || !sole(vr, vp)) return false;
        ggml_tensor * va = vr->src[0];
        if (!is(va, GGML_OP_ADD) || !sole(va, vr)) return false;
        ggml_tensor * vm = va->src[0];
        if (!is(vm, GGML_OP_MUL_MAT) || !sole(vm, va)) return false;
        const ggml_tensor * x = qm->src[1];
        const ggml_tensor * wq = qm->src[0];
        if (km->src[1] != x || vm->src[1] != x) return false;
        for (const ggml_tensor * m : {qm, km, vm})
            if (!mm_fast_ok(m) || m->src[0]->type != wq->type || !ggml_are_same_shape(m->src[0], wq) ||
                !is_weight_buffer(m->src[0]) || ((uintptr_t) m->data & 15) != 0)
                return false;
        const int64_t D = wq->ne[1], T = x->ne[1], H = D / 64;
        // (any T: the fused GEMM writes V row-major, q2a_gemm_args.v_rows — the V^T epilogue's 4-t groups, which needed
        // T % 4 == 0, are not used on this route)
        if (wq->ne[0] != D || D % 64 != 0 || x->ne[2] != 1 || x->ne[3] != 1 || T * D >= (1ll << 31)) return false;
        if (!row_vec_f32(qa->src[1], D) || !row_vec_f32(va->src[1], D) || !is_weight_buffer(qa->src[1]) ||
            !is_weight_buffer(va->src[1]) || !same_shape_rows(qm, qa) || !same_shape_rows(vm, va))
            return false;
        float sc;
        memcpy(&sc, qs->op_params, 4);
        int ex;
        if (!(sc > 0.0f) || frexpf(sc, &ex) != 0.5f || !ggml_is_contiguous(qs) || qs->type != GGML_TYPE_F32) return false;
        // element (d, t, h) of the K / Q views and (t, d, h) of V's CONT source = row t, column 64 h + d of the
        // projection (the only layout the epilogue writes)
        auto hd = [&](const ggml_tensor * v, const ggml_tensor * base, int64_t n0, int64_t s0, int64_t s1) {
            return v->data == base->data && v->ne[0] == n0 && v->ne[1] == (n0 == 64 ? T : 64) && v->ne[2] == H &&
                   (int64_t) v->nb[0] == s0 && (int64_t) v->nb[1] == s1 && (int64_t) v->nb[2] == 256;
        };
        if (!hd(kp, km, 64, 4, D * 4) || !hd(qp, qs, 64, 4, D * 4) || !hd(vp, va, T, D * 4, 4)) return false;
        if (qr->data != qa->data) return false;
        r = qkv_route{{qm, km, vm}, qa->src[1], va->src[1], sc};
        absorbed = {qm, km, vm, qa, qs, va, vc};
        return true;
    };
    std::vector<qkv_route> qkv_routes;
    std::vector<const ggml_tensor *> qkv_route_kq;                         // [route] its attention's KQ node
    std::unordered_map<const ggml_tensor *, int> qkv_mm;                   // Q / K / V MUL_MAT -> route
    std::unordered_map<const ggml_tensor *, int> qkv_absorbed;             // nodes a route replaces -> route
    std::vector<char> qkv_done;
    std::unordered_map<const ggml_tensor *, qkv_ops> qkv_ready;            // KQ node -> operands written
    if (!no_fuse && !no_qkv) {
        for (int j = 0; j + 2 < nn; ++j) {
            ggml_tensor * kqv = match_attention(g, j);
            if (!kqv) continue;
            qkv_route r;
            std::vector<const ggml_tensor *> ab;
            if (!match_qkv(ggml_graph_node(g, j), kqv, r, ab)) continue;
            const int id = (int) qkv_routes.size();
            qkv_routes.push_back(r);
            qkv_route_kq.push_back(ggml_graph_node(g, j));
            for (int k = 0; k < 3; ++k) qkv_mm[r.mm[k]] = id;
            for (const ggml_tensor * t : ab) qkv_absorbed[t] = id;
        }
        qkv_done.assign(qkv_routes.size(), 0);
    }
    // the fast MUL_MAT after node `from` that reads t, when it is t's only consumer (null otherwise)
    auto sole_mm_consumer = [&](const ggml_tensor * t, int from) -> const ggml_tensor * {
        if (no_fuse) return nullptr;
        for (int j = from + 1; j < nn; ++j) {
            const ggml_tensor * n = ggml_graph_node(g, j);
            if (n->op == GGML_OP_MUL_MAT && n->src[1] == t)
                return sole(t, n) && mm_fast_ok(n) && !qkv_mm.count(n) && !match_attention(g, j) ? n : nullptr;
        }
        return nullptr;
    };
    // the epilogue chain that follows the fast MUL_MAT at node j (see the MUL_MAT case)
    auto chain_of = [&](int j) -> mm_chain {
        ggml_tensor * op = ggml_graph_node(g, j);
        mm_chain c{op, Q2A_EPI_STORE_F, nullptr, nullptr, 0.0f, j, 0};
        ggml_tensor * n1 = node(j + 1), * n2 = node(j + 2);
        if (no_fuse || !n1 || n1->op != GGML_OP_ADD || n1->src[0] != op || !sole(op, n1) ||
            !row_vec_f32(n1->src[1], op->ne[0]) || !same_shape_rows(op, n1) || ((uintptr_t) n1->data & 15) != 0)
            return c;
        c.bias = (const float *) n1->src[1]->data;
        c.out = n1; c.last = j + 1; c.nfused = 1;
        if (n2 && n2->op == GGML_OP_UNARY && ggml_get_unary_op(n2) == GGML_UNARY_OP_GELU && n2->src[0] == n1 &&
            sole(n1, n2) && same_shape_rows(n1, n2) && ((uintptr_t) n2->data & 15) == 0 && !mm_is_pipe8(op)) {
            c.epi = Q2A_EPI_GELU_F; c.out = n2; c.last = j + 2; c.nfused = 2;
        } else if (ggml_tensor * sc = scale_after(n1, j + 2)) {
            c.oscale = *(const float *) sc->op_params; c.out = sc; c.nfused = 2;
            c.last = j + 2;
            while (ggml_graph_node(g, c.last) != sc) ++c.last;
        } else if (n2 && n2->op == GGML_OP_ADD && sole(n1, n2) && same_shape_rows(n1, n2) && ((uintptr_t) n2->data & 15) == 0) {
            const ggml_tensor * r = n2->src[0] == n1 ? n2->src[1] : n2->src[0];
            if (r != n1 && same_shape_rows(n1, r) && ((uintptr_t) r->data & 15) == 0) {
                c.epi = Q2A_EPI_RESID; c.resid = (const float *) r->data; c.out = n2; c.last = j + 2; c.nfused = 2;
            }
        }
        return c;
    };
    for (int i = 0; i < nn; ++i) {
        if (b->capture_aborted) return GGML_STATUS_SUCCESS;   // graph_compute re-runs the whole cgraph directly
        ggml_tensor * op = ggml_graph_node(g, i);
        if (ggml_is_empty(op) || op->op == GGML_OP_NONE || op->op == GGML_OP_RESHAPE || op->op == GGML_OP_VIEW ||
            op->op == GGML_OP_PERMUTE || op->op == GGML_OP_TRANSPOSE)
            continue;
        if (!qkv_absorbed.empty()) {
            const auto ab = qkv_absorbed.find(op);
            if (ab != qkv_absorbed.end()) {
                // the first of a route's MUL_MATs in node order runs the fused GEMM; everything else it replaces is done
                if (qkv_mm.count(op) && !qkv_done[ab->second]) {
                    qkv_done[ab->second] = 1;
                    b->stats.n_nodes++;
                    qkv_ops ops;
                    run_qkv_fused(b, qkv_routes[ab->second], ops);
                    qkv_ready[qkv_route_kq[ab->second]] = ops;
                    b->stats.n_mul_mat_fast += 3;
                    b->stats.n_mm_grouped++;
                    b->stats.n_fused += 4;   // Q bias, Q scale, V bias, V CONT
                    const hipError_t e = hipGetLastError();
                    if (e != hipSuccess) {
                        Q2A_LOG_ERROR("ggml-q2a: fused Q|K|V (%s) launch failed: %s\n", op->name, hipGetErrorString(e));
                        return GGML_STATUS_FAILED;
                    }
                }
                continue;
            }
        }
        b->stats.n_nodes++;
        const ggml_tensor * s0 = op->src[0];
        const ggml_tensor * s1 = op->src[1];
        const int64_t n = ggml_nelements(op);
        hipStream_t st = b->stream;
        switch (op->op) {
            case GGML_OP_MUL_MAT: {
                if (ggml_tensor * kqv = match_attention(g, i)) {
                    ggml_tensor * merged = nullptr;
                    ggml_tensor * p = node(i + 3), * c = node(i + 4);
                    if (p && c && p->op == GGML_OP_PERMUTE && p->src[0] == kqv && sole(kqv, p) && c->op == GGML_OP_CONT &&
                        c->src[0] == p && sole(p, c)) {
                        const int32_t * ax = (const int32_t *) p->op_params;
                        if (ax[0] == 0 && ax[1] == 2 && ax[2] == 1 && ax[3] == 3 && c->type == GGML_TYPE_F32 &&
                            ggml_is_contiguous(c) && c->ne[0] == 64 * kqv->ne[2] && c->ne[1] == kqv->ne[1] &&
                            c->ne[2] == 1 && c->ne[3] == 1 && ((uintptr_t) c->data & 15) == 0)
                            merged = c;
                    }
                    const bool vt_ready = kqv->src[0] == vt_ready_for;
                    const auto rd = qkv_ready.find(op);
                    // the merged rows feeding only an F16 O-projection: written as its fp16 operand directly
                    const ggml_tensor * o_mm = merged ? sole_mm_consumer(merged, i + 4) : nullptr;
                    _Float16 * out16 = o_mm && o_mm->src[0]->type == GGML_TYPE_F16 ? claim_a16(b, merged) : nullptr;
                    const int used = run_fused_attention(b, g, i, vt_ready, merged, rd != qkv_ready.end() ? &rd->second : nullptr,
                                                         out16);
                    if (merged) b->stats.n_fused += 1;
                    if (vt_ready) vt_ready_for = nullptr;
                    i += used - 1;
                    break;
                }
                if (!mm_fast_ok(op) && conv_f64_diag(op)) { run_mm_conv_f64(b, op); b->stats.n_mul_mat_conv++; break; }
                if (!mm_fast_ok(op) && conv_hilo_ok(op)) {
                    // the conv graph's MUL_MAT -> RESHAPE -> ADD(bias [1][C]) -> GELU (ggml_conv_1d_ph, then
                    // qwen2-whisper.cpp's bias add and GELU), every link its producer's sole consumer: one transpose
                    // writes the GELU node
                    int last = i;
                    ggml_tensor * gout = nullptr;
                    const float * cbias = nullptr;
                    if (!no_fuse) {
                        int j = i + 1;
                        ggml_tensor * prod = op;
                        while (node(j) && (node(j)->op == GGML_OP_RESHAPE || node(j)->op == GGML_OP_VIEW) &&
                               node(j)->src[0] == prod && sole(prod, node(j)) && ggml_is_contiguous(node(j)) &&
                               node(j)->data == op->data && ggml_nelements(node(j)) == n)
                            prod = node(j++);
                        ggml_tensor * ad = node(j), * ge = node(j + 1);
                        const ggml_tensor * bs = ad ? ad->src[1] : nullptr;
                        if (ad && ge && ad->op == GGML_OP_ADD && ad->src[0] == prod && sole(prod, ad) && bs &&
                            bs->type == GGML_TYPE_F32 && ggml_is_contiguous(bs) && bs->ne[0] == 1 && bs->ne[1] == op->ne[1] &&
                            bs->ne[2] == 1 && bs->ne[3] == 1 && ad->type == GGML_TYPE_F32 && ggml_is_contiguous(ad) &&
                            ggml_nelements(ad) == n && ad->ne[0] == op->ne[0] && ad->ne[1] == op->ne[1] &&
                            ge->op == GGML_OP_UNARY && ggml_get_unary_op(ge) == GGML_UNARY_OP_GELU && ge->src[0] == ad &&
                            sole(ad, ge) && ge->type == GGML_TYPE_F32 && ggml_is_contiguous(ge) && ggml_are_same_shape(ad, ge)) {
                            gout = ge;
                            cbias = (const float *) bs->data;
                            last = j + 1;
                        }
                    }
                    run_mm_conv_hilo(b, op, gout, cbias);
                    b->stats.n_mul_mat_conv++;
                    b->n_mul_mat_conv_total++;
                    if (gout) b->stats.n_fused += 2;
                    i = last;
                    break;
                }
                if (!mm_fast_ok(op)) { run_mm_f32(b, op); b->stats.n_mul_mat_f32++; break; }
                // MUL_MAT -> ADD(bias row) [-> GELU | -> ADD(residual) | -> [RESHAPE] -> SCALE] on the GEMM epilogue
                // (qwen2-whisper.cpp:2029-2054, 2120-2154): same f32 operations, one kernel, no [N][M] round trips
                mm_chain c1 = chain_of(i);
                // two consecutive projections of the same activation with plain / bias / bias+scale epilogues (the K
                // and Q projections, :2029-2062) run as one grouped launch: twice the workgroups of either alone
                int j2 = c1.last + 1;   // the next node that executes (views in between are free)
                while (node(j2) && is_view_op(node(j2))) ++j2;
                ggml_tensor * m2 = node(j2);
                if (c1.epi == Q2A_EPI_STORE_F && !no_fuse && m2 && m2->op == GGML_OP_MUL_MAT && m2->src[1] == op->src[1] &&
                    (op->src[0]->type == GGML_TYPE_F16 || op->src[0]->type == GGML_TYPE_Q4_K) &&
                    m2->src[0]->type == op->src[0]->type && mm_fast_ok(m2) &&
                    !match_attention(g, j2) && ggml_are_same_shape(m2->src[0], op->src[0]) && !mm_is_pipe8(op)) {
                    const mm_chain c2 = chain_of(j2);
                    if (c2.epi == Q2A_EPI_STORE_F) {
                        mm_second sec{m2->src[0], c2.out, c2.bias, c2.oscale};
                        run_mm_fast(b, op, c1.out, Q2A_EPI_STORE_F, c1.bias, nullptr, c1.oscale, nullptr, &sec);
                        b->stats.n_fused += c1.nfused + c2.nfused;
                        b->stats.n_mul_mat_fast += 2;
                        b->stats.n_mm_grouped++;
                        i = c2.last;
                        break;
                    }
                }
                if (c1.epi == Q2A_EPI_GELU_F && ggml_is_contiguous(c1.out)) {
                    if (const ggml_tensor * f2 = sole_mm_consumer(c1.out, c1.last)) {
                        run_fc1_for_fc2(b, op, c1, f2);
                        b->stats.n_fused += c1.nfused;
                        b->stats.n_mul_mat_fast++;
                        i = c1.last;
                        break;
                    }
                }
                _Float16 * out16 = c1.epi == Q2A_EPI_GELU_F && want16.count(c1.out) && ggml_is_contiguous(c1.out)
                                       ? claim_a16(b, c1.out) : nullptr;
                run_mm_fast(b, op, c1.out, c1.epi, c1.bias, c1.resid, c1.oscale, out16);
                b->stats.n_fused += c1.nfused;
                b->stats.n_mul_mat_fast++;
                i = c1.last;
                break;
            }
            case GGML_OP_ADD: case GGML_OP_MUL:
                if (!launch_rows(b, op->op == GGML_OP_ADD ? 0 : 1, s0, op, s1, 1.0f)) {
                    if (op->op == GGML_OP_ADD)
                        hipLaunchKernelGGL(k_binary<0>, grid1(n), dim3(256), 0, st, tv(s0), tv(s1), tv(op), n);
                    else
                        hipLaunchKernelGGL(k_binary<1>, grid1(n), dim3(256), 0, st, tv(s0), tv(s1), tv(op), n);
                }
                b->stats.n_other++;
                break;
            case GGML_OP_SCALE: {
                float sc;
                memcpy(&sc, op->op_params, 4);
                if (!launch_rows(b, 2, s0, op, nullptr, sc))
                    hipLaunchKernelGGL(k_unary<0>, grid1(n), dim3(256), 0, st, tv(s0), tv(op), n, sc, (const uint16_t *) nullptr);
                b->stats.n_other++;
                break;
            }
            case GGML_OP_UNARY:
                if (!launch_rows(b, 3, s0, op, nullptr, 1.0f))
                    hipLaunchKernelGGL(k_unary<1>, grid1(n), dim3(256), 0, st, tv(s0), tv(op), n, 1.0f, gelu_table(b->device));
                b->stats.n_other++;
                break;
            case GGML_OP_NORM: {
                float eps;
                memcpy(&eps, op->op_params, 4);
                const unsigned rows = (unsigned) ggml_nrows(op);
                if (op->ne[0] > 2048 || ggml_nrows(op) > (1ll << 31) - 1) {
                    hipLaunchKernelGGL(k_norm, dim3(rows), dim3(256), 0, st, tv(s0), tv(op), eps);
                    b->stats.n_other++;
                    break;
                }
                // NORM -> MUL(weight row) -> ADD(bias row) (qwen2-whisper.cpp:2002-2006, 2124-2128, 2176-2180)
                ggml_tensor * n1 = node(i + 1), * n2 = node(i + 2);
                const bool aff = n1 && n2 && n1->op == GGML_OP_MUL && n1->src[0] == op && sole(op, n1) &&
                    row_vec_f32(n1->src[1], op->ne[0]) && n2->op == GGML_OP_ADD && n2->src[0] == n1 && sole(n1, n2) &&
                    row_vec_f32(n2->src[1], op->ne[0]) && rows_f32(n2) && n1->type == GGML_TYPE_F32 &&
                    ggml_are_same_shape(op, n2);
                ggml_tensor * out = aff ? n2 : op;
                const bool v4 = op->ne[0] % 4 == 0 && aligned16(s0) && aligned16(out);
                const float * w = aff ? (const float *) n1->src[1]->data : nullptr;
                const float * bb = aff ? (const float *) n2->src[1]->data : nullptr;
                // rows read only by fast MUL_MATs of one weight class (the Q|K|V projections; fc1): the engine's fused
                // LayerNorm writes their operand — fp16 rows, or Q8_K / Q8_0 codes and scales in the scratch —
                // instead of the f32 rows (the same rows: k_norm_row sums like it; q2a_engine.hip run_block)
                if (aff && v4 && eps == 1e-5f && !no_fuse && ggml_is_contiguous(s0) && ggml_is_contiguous(out) &&
                    !(out->flags & GGML_TENSOR_FLAG_OUTPUT)) {
                    const int D = (int) op->ne[0], M = (int) rows;
                    int blk = -1, found = 0, last = -1;
                    size_t extra = 0;
                    bool ok = true;
                    for (int j = i + 3; j < nn && ok; ++j) {
                        const ggml_tensor * c = ggml_graph_node(g, j);
                        bool reads = false;
                        for (int k = 0; k < GGML_MAX_SRC; ++k) reads = reads || c->src[k] == out;
                        if (reads) {
                            if (c->op != GGML_OP_MUL_MAT || c->src[1] != out || c->src[0] == out || !mm_fast_ok(c) ||
                                match_attention(g, j)) { ok = false; break; }
                            const int cb = blk_of_type(c->src[0]->type);
                            if (blk >= 0 && cb != blk) { ok = false; break; }
                            blk = cb;
                            ++found;
                            last = j;
                            extra = std::max(extra, mm_part_bytes(Q2A_EPI_STORE_F, cb, M, (int) c->src[0]->ne[1], D, false));
                        } else if (found < (uses.count(out) ? uses[out] : 0) && c->op == GGML_OP_MUL_MAT && !qkv_absorbed.count(c)) {
                            ok = false;   // another GEMM (scratch user) between the LayerNorm and its last reader
                        }
                        if (found == (uses.count(out) ? uses[out] : 0)) break;
                    }
                    if (ok && found > 0 && found == uses[out] && last > i && (blk == 0 || D % (blk == 256 ? 256 : 32) == 0)) {
                        q2a_ln_args la{(const float *) s0->data, M, D, w, bb, blk == 0 ? 0 : blk == 256 ? 1 : 2, nullptr, nullptr, nullptr, 0};
                        if (blk == 0) {
                            la.outH = (q2a_half *) claim_a16(b, out);
                        } else {
                            const act_operand d = act_slots(b, M, D, blk, extra);
                            la.outH = (q2a_half *) d.A; la.dy = d.dy; la.aext = d.aext; la.dy_ld = d.MP;
                        }
                        Q2A_HIP(q2a_launch_layernorm(la, st));
                        if (blk) { b->quant_src = out; b->quant_blk = blk; }
                        b->stats.n_fused += 2;
                        b->stats.n_other++;
                        i += 2;
                        break;
                    }
                }
                const dim3 grid((rows + 3) / 4);
                _Float16 * yh = want16.count(out) && ggml_is_contiguous(out) ? claim_a16(b, out) : nullptr;
                if (aff && v4) hipLaunchKernelGGL((k_norm_row<true, true>), grid, dim3(256), 0, st, tv(s0), tv(out), eps, w, bb, (int) rows, yh);
                else if (aff) hipLaunchKernelGGL((k_norm_row<true, false>), grid, dim3(256), 0, st, tv(s0), tv(out), eps, w, bb, (int) rows, yh);
                else if (v4) hipLaunchKernelGGL((k_norm_row<false, true>), grid, dim3(256), 0, st, tv(s0), tv(out), eps, w, bb, (int) rows, yh);
                else hipLaunchKernelGGL((k_norm_row<false, false>), grid, dim3(256), 0, st, tv(s0), tv(out), eps, w, bb, (int) rows, yh);
                if (aff) {
                    b->stats.n_fused += 2;
                    i += 2;
                }
                b->stats.n_other++;
                break;
            }
            case GGML_OP_SOFT_MAX: {
                float sc;
                memcpy(&sc, op->op_params, 4);
                hipLaunchKernelGGL(k_softmax, dim3((unsigned) ggml_nrows(op)), dim3(256), 0, st, tv(s0), tv(op), sc);
                b->stats.n_other++;
                break;
            }
            case GGML_OP_CONT: case GGML_OP_DUP: case GGML_OP_CPY: {
                // the encoder's head and tail (qwen2-whisper.cpp:2004, 2160-2172): CONT(TRANSPOSE(embd_conv)) read only
                // by ADD(positional rows, ·) -> one tiled transpose writing the ADD; CONT(PERMUTE(x)) read only by
                // POOL_1D AVG whose PERMUTE -> CONT restores x's layout -> one pass over x's rows, written into that
                // CONT, or — when the allocator gave the CONT x's block (rows read and written by different threads
                // must not overlap) — into the first CONT's own block and copied over
                if (op->op == GGML_OP_CONT && !no_fuse && !vprep.count(op) && op->type == GGML_TYPE_F32 && s0 &&
                    s0->type == GGML_TYPE_F32 && ggml_is_contiguous(op)) {
                    const ggml_tensor * x = s0->src[0];
                    const bool swap01 = (s0->op == GGML_OP_TRANSPOSE ||
                                         (s0->op == GGML_OP_PERMUTE && ((const int32_t *) s0->op_params)[0] == 1 &&
                                          ((const int32_t *) s0->op_params)[1] == 0 && ((const int32_t *) s0->op_params)[2] == 2 &&
                                          ((const int32_t *) s0->op_params)[3] == 3)) &&
                                        x && x->type == GGML_TYPE_F32 && ggml_is_contiguous(x) && x->ne[2] == 1 && x->ne[3] == 1 &&
                                        s0->data == x->data && s0->ne[0] == x->ne[1] && s0->ne[1] == x->ne[0];
                    auto disjoint = [](const ggml_tensor * u, const ggml_tensor * v) {
                        return (const char *) u->data + ggml_nbytes(u) <= (const char *) v->data ||
                               (const char *) v->data + ggml_nbytes(v) <= (const char *) u->data;
                    };
                    int j = i + 1;
                    while (node(j) && is_view_op(node(j)) && node(j)->src[0] != op) ++j;
                    ggml_tensor * nx = node(j);
                    if (swap01 && nx && nx->op == GGML_OP_ADD && sole(op, nx) && nx->type == GGML_TYPE_F32 &&
                        ggml_is_contiguous(nx) && ggml_are_same_shape(nx, op)) {
                        const ggml_tensor * pe = nx->src[0] == op ? nx->src[1] : nx->src[0];
                        if (pe != op && pe->type == GGML_TYPE_F32 && ggml_are_same_shape(pe, op) && pe->nb[0] == 4 &&
                            pe->nb[1] == (size_t) pe->ne[0] * 4 && nx->src[1] == op && disjoint(nx, x) && disjoint(nx, pe)) {
                            // x [C rows][T] -> nx [T rows][C]: R = C, C' = T
                            const int R = (int) x->ne[1], Cc = (int) x->ne[0];
                            hipLaunchKernelGGL(k_transpose_f32, dim3((unsigned) ((Cc + 63) / 64), (unsigned) ((R + 63) / 64)), dim3(256), 0,
                                               st, (const float *) x->data, (float *) nx->data, R, Cc, nullptr, nullptr,
                                               (const float *) pe->data);
                            b->stats.n_other++;
                            b->stats.n_fused += 1;
                            i = j;
                            break;
                        }
                    }
                    if (swap01 && nx && nx->op == GGML_OP_POOL_1D && nx->src[0] == op && sole(op, nx)) {
                        const int32_t * pp = (const int32_t *) nx->op_params;
                        ggml_tensor * p2 = node(j + 1), * c2 = node(j + 2);
                        if (pp[0] == GGML_OP_POOL_AVG && pp[1] == pp[2] && pp[3] == 0 && pp[1] >= 1 && nx->type == GGML_TYPE_F32 &&
                            p2 && c2 && p2->op == GGML_OP_PERMUTE && p2->src[0] == nx && sole(nx, p2) &&
                            ((const int32_t *) p2->op_params)[0] == 1 && ((const int32_t *) p2->op_params)[1] == 0 &&
                            c2->op == GGML_OP_CONT && c2->src[0] == p2 && sole(p2, c2) && c2->type == GGML_TYPE_F32 &&
                            ggml_is_contiguous(c2) && c2->ne[0] == x->ne[0] && c2->ne[1] == x->ne[1] / pp[1] &&
                            c2->ne[2] == 1 && c2->ne[3] == 1) {
                            const bool direct = disjoint(c2, x);
                            if (direct || (disjoint(op, x) && disjoint(op, c2))) {
                                const int64_t nn2 = ggml_nelements(c2);
                                float * dst = (float *) (direct ? c2->data : op->data);
                                hipLaunchKernelGGL(k_pool_rows_avg, grid1(nn2), dim3(256), 0, st, (const float *) x->data, dst,
                                                   (int) x->ne[0], (int) pp[1], nn2);
                                if (!direct) Q2A_HIP(hipMemcpyAsync(c2->data, dst, (size_t) nn2 * 4, hipMemcpyDeviceToDevice, st));
                                b->stats.n_other++;
                                b->stats.n_fused += 2;
                                i = j + 2;
                                break;
                            }
                        }
                    }
                }
                if (vprep.count(op) && !vt_ready_for) {   // V of a fused attention: its V^T operand instead of the f32 copy
                    // (one pending at a time: a second V before the first attention is copied normally)
                    const int T = (int) op->ne[0], H = (int) op->ne[2], TP = (T + 63) / 64 * 64;
                    const size_t vb1 = ((size_t) H * 64 * TP * 2 + 255) & ~size_t(255);
                    const bool vlo = q2a_attention_wants_vlo();   // (run_fused_attention finds the lo image at +vb1)
                    _Float16 * vt = vt_buffer(b, vlo ? 2 * vb1 : vb1);
                    hipLaunchKernelGGL(k_vt_tile, dim3((unsigned) (TP / 64), (unsigned) H), dim3(256), 0, st, tv(op->src[0]), vt,
                                       vlo ? (_Float16 *) ((char *) vt + vb1) : nullptr, T, TP);
                    vt_ready_for = op;
                    b->stats.n_other++;
                    break;
                }
                ggml_tensor * dst = op->op == GGML_OP_CPY ? op->src[1] : op;
                if (n < (1ll << 31))
                    hipLaunchKernelGGL(k_copy<uint32_t>, grid1(n), dim3(256), 0, st, tv(s0), (int) s0->type, tv(dst), (int) dst->type, n);
                else
                    hipLaunchKernelGGL(k_copy<int64_t>, grid1(n), dim3(256), 0, st, tv(s0), (int) s0->type, tv(dst), (int) dst->type, n);
                b->stats.n_other++;
                break;
            }
            case GGML_OP_IM2COL: {
                const int32_t * pp = (const int32_t *) op->op_params;
                const int IC = (int) s1->ne[1], IW = (int) s1->ne[0], KW = (int) s0->ne[0], OW = (int) op->ne[1];
                hipLaunchKernelGGL(k_im2col1d, grid1(n), dim3(256), 0, st, tv(s1), tv(op), (int) op->type, IC, IW, KW, OW,
                                   pp[0], pp[2], pp[4], n);
                b->stats.n_other++;
                break;
            }
            case GGML_OP_POOL_1D: {
                const int32_t * pp = (const int32_t *) op->op_params;
                hipLaunchKernelGGL(k_pool1d_avg, grid1(n), dim3(256), 0, st, tv(s0), tv(op), (int) pp[1], n);
                b->stats.n_other++;
                break;
            }
            default:
                Q2A_LOG_ERROR("ggml-q2a: unsupported op %s (%s)\n", ggml_op_desc(op), op->name);
                return GGML_STATUS_FAILED;
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            Q2A_LOG_ERROR("ggml-q2a: %s (%s) launch failed: %s\n", ggml_op_desc(op), op->name, hipGetErrorString(e));
            return GGML_STATUS_FAILED;
        }
    }
    return GGML_STATUS_SUCCESS;
}

// everything a captured launch depends on: per node its op, parameters, shape, strides and the addresses of the
// node and its sources; plus the weight-cache generation (packed weight pointers are baked into the graph)
uint64_t graph_signature(ggml_cgraph * g, uint64_t wgen) {
    uint64_t h = 1469598103934665603ull ^ wgen;
    auto mix = [&](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
    const int nn = ggml_graph_n_nodes(g);
    mix((uint64_t) nn);
    for (int i = 0; i < nn; ++i) {
        const ggml_tensor * t = ggml_graph_node(g, i);
        mix((uint64_t) t->op); mix((uint64_t) t->type); mix((uint64_t) (uintptr_t) t->data);
        for (int k = 0; k < 4; ++k) { mix((uint64_t) t->ne[k]); mix((uint64_t) t->nb[k]); }
        for (int k = 0; k < 8; ++k) mix((uint64_t) (uint32_t) t->op_params[k]);
        for (int s = 0; s < GGML_MAX_SRC && t->src[s]; ++s) {
            const ggml_tensor * u = t->src[s];
            mix((uint64_t) (uintptr_t) u->data); mix((uint64_t) u->type);
            for (int k = 0; k < 4; ++k) { mix((uint64_t) u->ne[k]); mix((uint64_t) u->nb[k]); }
        }
    }
    return h;
}

ggml_status graph_compute(ggml_backend_t backend, ggml_cgraph * g) {
    q2a_backend_ctx * b = (q2a_backend_ctx *) backend->context;
    Q2A_HIP(hipSetDevice(b->device));
    static const bool no_graph = [] { const char * v = getenv("GGML_Q2A_NO_GRAPH"); return v && atoi(v); }();
    if (no_graph) return run_nodes(b, g);
    constexpr size_t max_graphs = 8;
    q2a_device_ctx * d = dev_ctx(b->device);
    const uint64_t sig = graph_signature(g, d->wgen);
    q2a_backend_ctx::captured * c = nullptr;
    for (auto & e : b->graphs) if (e.sig == sig) c = &e;
    if (!c) {   // first sighting: run directly (packs weights, sizes the scratch), remember the signature
        if (b->graphs.size() == max_graphs) {
            auto lru = std::min_element(b->graphs.begin(), b->graphs.end(),
                                        [](const auto & x, const auto & y) { return x.used < y.used; });
            if (lru->exec) (void) hipGraphExecDestroy(lru->exec);
            b->graphs.erase(lru);
        }
        b->graphs.push_back({sig, 1, nullptr, {}, ++b->graph_clock});
        return run_nodes(b, g);
    }
    c->used = ++b->graph_clock;
    if (c->exec) {   // replay
        if (hipGraphLaunch(c->exec, b->stream) == hipSuccess) {
            b->stats = c->stats;
            b->stats.n_graph_replayed = 1;
            return GGML_STATUS_SUCCESS;
        }
        (void) hipGetLastError();
        (void) hipGraphExecDestroy(c->exec);
        c->exec = nullptr;
        return run_nodes(b, g);
    }
    if (++c->seen == 2) {   // second sighting (weights packed, scratch sized): capture once, then launch
        hipGraph_t graph = nullptr;
        b->capture_aborted = false;
        if (hipStreamBeginCapture(b->stream, hipStreamCaptureModeThreadLocal) == hipSuccess) {
            const ggml_status st = run_nodes(b, g);
            if (b->capture_aborted) {   // a buffer grew mid-capture: the capture is gone, nothing of it ran
                end_discard(b);         // (the aborted node's remaining launches, discarded)
                b->capture_aborted = false;
                c->seen = 1;            // captured again on its next sighting, against the grown buffers
                return run_nodes(b, g);
            }
            const hipError_t ec = hipStreamEndCapture(b->stream, &graph);
            hipGraphExec_t exec = nullptr;
            if (st == GGML_STATUS_SUCCESS && ec == hipSuccess && graph &&
                hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) == hipSuccess) {
                (void) hipGraphDestroy(graph);
                c->exec = exec;
                c->stats = b->stats;
                ++d->n_captured;
                if (hipGraphLaunch(exec, b->stream) == hipSuccess) return GGML_STATUS_SUCCESS;
                (void) hipGraphExecDestroy(exec);
                c->exec = nullptr;
            } else if (graph) {
                (void) hipGraphDestroy(graph);
            }
        }
        (void) hipGetLastError();   // capture refused or failed: nothing ran; run the nodes directly below
    }
    return run_nodes(b, g);
}

// ---- backend ------------------------------------------------------------------------------------
ggml_guid_t q2a_guid() {
    static ggml_guid guid = {0x51, 0x32, 0x41, 0x2d, 0x67, 0x66, 0x78, 0x39, 0x35, 0x30, 0x4d, 0x49, 0x33, 0x35, 0x35, 0x58};
    return &guid;
}

const char * be_get_name(ggml_backend_t be) { return ((q2a_backend_ctx *) be->context)->name.c_str(); }
void be_free(ggml_backend_t be) {
    q2a_backend_ctx * b = (q2a_backend_ctx *) be->context;
    (void) hipSetDevice(b->device);
    (void) hipStreamSynchronize(b->stream);
    if (b->scratch) (void) hipFree(b->scratch);
    if (b->vt_buf) (void) hipFree(b->vt_buf);
    if (b->qkv_buf) (void) hipFree(b->qkv_buf);
    if (b->pre16) (void) hipFree(b->pre16);
    for (int k = 0; k < 2; ++k) if (b->a16[k]) (void) hipFree(b->a16[k]);
    for (auto & e : b->graphs) if (e.exec) (void) hipGraphExecDestroy(e.exec);
    (void) hipStreamDestroy(b->stream);
    delete b;
    delete be;
}
ggml_backend_buffer_type_t be_get_default_buft(ggml_backend_t be) {
    return ggml_backend_q2a_buffer_type(((q2a_backend_ctx *) be->context)->device);
}
void be_set_tensor_async(ggml_backend_t be, ggml_tensor * t, const void * data, size_t off, size_t n) {
    q2a_backend_ctx * b = (q2a_backend_ctx *) be->context;
    ggml_backend_buffer_t buf = t->view_src ? t->view_src->buffer : t->buffer;
    GGML_ASSERT(buf && is_q2a_buffer(buf) && "unsupported buffer type");
    invalidate(b->device, (char *) t->data + off, n);
    Q2A_HIP(hipMemcpyAsync((char *) t->data + off, data, n, hipMemcpyHostToDevice, b->stream));
    prepack(b->device, t, data, off, n);   // reads the host bytes only (the pack does not wait for the copy)
}
void be_get_tensor_async(ggml_backend_t be, const ggml_tensor * t, void * data, size_t off, size_t n) {
    q2a_backend_ctx * b = (q2a_backend_ctx *) be->context;
    ggml_backend_buffer_t buf = t->view_src ? t->view_src->buffer : t->buffer;
    GGML_ASSERT(buf && is_q2a_buffer(buf) && "unsupported buffer type");
    Q2A_HIP(hipMemcpyAsync(data, (const char *) t->data + off, n, hipMemcpyDeviceToHost, b->stream));
}
void be_synchronize(ggml_backend_t be) {
    q2a_backend_ctx * b = (q2a_backend_ctx *) be->context;
    Q2A_HIP(hipSetDevice(b->device));
    Q2A_HIP(hipStreamSynchronize(b->stream));
}
bool dev_supports_op(ggml_backend_dev_t, const ggml_tensor * op) { return op_supported(op); }
bool dev_supports_buft(ggml_backend_dev_t dev, ggml_backend_buffer_type_t t) {
    return t->iface.get_name == buft_get_name && t->context == dev->context;
}
bool be_supports_op(ggml_backend_t, const ggml_tensor * op) { return op_supported(op); }
bool be_supports_buft(ggml_backend_t be, ggml_backend_buffer_type_t t) {
    return t->iface.get_name == buft_get_name && ((q2a_device_ctx *) t->context)->device == ((q2a_backend_ctx *) be->context)->device;
}
bool be_offload_op(ggml_backend_t, const ggml_tensor *) { return false; }

const ggml_backend_i k_backend_iface = {
    /* get_name                */ be_get_name,
    /* free                    */ be_free,
    /* get_default_buffer_type */ be_get_default_buft,
    /* set_tensor_async        */ be_set_tensor_async,
    /* get_tensor_async        */ be_get_tensor_async,
    /* cpy_tensor_async        */ nullptr,
    /* synchronize             */ be_synchronize,
    /* graph_plan_create       */ nullptr,
    /* graph_plan_free         */ nullptr,
    /* graph_plan_update       */ nullptr,
    /* graph_plan_compute      */ nullptr,
    /* graph_compute           */ graph_compute,
    /* supports_op             */ be_supports_op,
    /* supports_buft           */ be_supports_buft,
    /* offload_op              */ be_offload_op,
    /* event_record            */ nullptr,
    /* event_wait              */ nullptr,
};

// ---- device / registry --------------------------------------------------------------------------
const char * dev_get_name(ggml_backend_dev_t d) { return ((q2a_device_ctx *) d->context)->name.c_str(); }
const char * dev_get_desc(ggml_backend_dev_t d) { return ((q2a_device_ctx *) d->context)->desc.c_str(); }
void dev_get_memory(ggml_backend_dev_t d, size_t * free, size_t * total) {
    ggml_backend_q2a_get_device_memory(((q2a_device_ctx *) d->context)->device, free, total);
}
enum ggml_backend_dev_type dev_get_type(ggml_backend_dev_t) { return GGML_BACKEND_DEVICE_TYPE_GPU_FULL; }
void dev_get_props(ggml_backend_dev_t d, ggml_backend_dev_props * p) {
    p->name = dev_get_name(d);
    p->description = dev_get_desc(d);
    p->type = dev_get_type(d);
    dev_get_memory(d, &p->memory_free, &p->memory_total);
    p->caps = {/* async */ true, /* host_buffer */ pinned_allowed(), /* events */ false};
}
ggml_backend_t dev_init_backend(ggml_backend_dev_t d, const char *) {
    return ggml_backend_q2a_init(((q2a_device_ctx *) d->context)->device);
}
ggml_backend_buffer_type_t dev_get_buft(ggml_backend_dev_t d) { return &((q2a_device_ctx *) d->context)->buft; }
ggml_backend_buffer_type_t dev_get_host_buft(ggml_backend_dev_t) { return ggml_backend_q2a_host_buffer_type(); }
bool dev_offload_op(ggml_backend_dev_t, const ggml_tensor *) { return false; }

const ggml_backend_device_i k_device_iface = {
    /* get_name             */ dev_get_name,
    /* get_description      */ dev_get_desc,
    /* get_memory           */ dev_get_memory,
    /* get_type             */ dev_get_type,
    /* get_props            */ dev_get_props,
    /* init_backend         */ dev_init_backend,
    /* get_buffer_type      */ dev_get_buft,
    /* get_host_buffer_type */ dev_get_host_buft,
    /* buffer_from_host_ptr */ nullptr,
    /* supports_op          */ dev_supports_op,
    /* supports_buft        */ dev_supports_buft,
    /* offload_op           */ dev_offload_op,
    /* event_new            */ nullptr,
    /* event_free           */ nullptr,
    /* event_synchronize    */ nullptr,
};

const char * reg_get_name(ggml_backend_reg_t) { return GGML_Q2A_NAME; }
size_t reg_get_device_count(ggml_backend_reg_t) { return reg_ctx()->devs.size(); }
ggml_backend_dev_t reg_get_device(ggml_backend_reg_t, size_t i) {
    q2a_reg_ctx * r = reg_ctx();
    return i < r->devs.size() ? &r->devs[i]->dev : nullptr;
}

// the optional functions ggml_backend_reg_get_proc_address hands out (ggml-backend.h:169-178; the reference's CUDA
// registry answers the same two names, ggml-cuda.cu:3276-3288). No split buffer type: a model is replicated per
// device, never split by rows
void * reg_get_proc_address(ggml_backend_reg_t, const char * name) {
    if (strcmp(name, "ggml_backend_register_host_buffer") == 0) return (void *) ggml_backend_q2a_register_host_buffer;
    if (strcmp(name, "ggml_backend_unregister_host_buffer") == 0) return (void *) ggml_backend_q2a_unregister_host_buffer;
    return nullptr;
}

const ggml_backend_reg_i k_reg_iface = {
    /* get_name         */ reg_get_name,
    /* get_device_count */ reg_get_device_count,
    /* get_device       */ reg_get_device,
    /* get_proc_address */ reg_get_proc_address,
};

ggml_backend_reg * the_reg() {
    static ggml_backend_reg reg = {k_reg_iface, nullptr};
    return &reg;
}

q2a_reg_ctx * reg_ctx() {
    static q2a_reg_ctx * r = [] {
        q2a_reg_ctx * c = new q2a_reg_ctx();
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) { (void) hipGetLastError(); n = 0; }
        for (int i = 0; i < std::min(n, GGML_Q2A_MAX_DEVICES); ++i) {
            q2a_device_ctx * d = new q2a_device_ctx();
            d->device = i;
            d->name = std::string(GGML_Q2A_NAME) + std::to_string(i);
            hipDeviceProp_t prop;
            d->desc = hipGetDeviceProperties(&prop, i) == hipSuccess ? std::string(prop.name) + " (" + prop.gcnArchName + ")" : "HIP device";
            d->buft = {k_buft_iface, &d->dev, d};
            d->dev = {k_device_iface, the_reg(), d};
            c->devs.push_back(d);
        }
        return c;
    }();
    return r;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// public API (include/ggml-q2a.h)
// ------------------------------------------------------------------------------------------------
extern "C" {

ggml_backend_t ggml_backend_q2a_init(int device) {
    q2a_device_ctx * d = dev_ctx(device);
    if (!d) {
        Q2A_LOG_ERROR("ggml-q2a: invalid device %d\n", device);
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    q2a_backend_ctx * b = new q2a_backend_ctx();
    b->device = device;
    b->name = d->name;
    // a blocking stream: the buffers' synchronous copies on the null stream stay ordered with graph work
    if (hipStreamCreate(&b->stream) != hipSuccess) {
        delete b;
        return nullptr;
    }
    return new ggml_backend{q2a_guid(), k_backend_iface, &d->dev, b};
}

bool ggml_backend_is_q2a(ggml_backend_t backend) {
    return backend != nullptr && ggml_guid_matches(backend->guid, q2a_guid());
}

ggml_backend_buffer_type_t ggml_backend_q2a_buffer_type(int device) {
    q2a_device_ctx * d = dev_ctx(device);
    return d ? &d->buft : nullptr;
}

ggml_backend_buffer_type_t ggml_backend_q2a_host_buffer_type(void) {
    static ggml_backend_buffer_type host_buft = {k_host_buft_iface, nullptr, nullptr};
    static std::once_flag once;
    std::call_once(once, [] {
        q2a_reg_ctx * r = reg_ctx();
        host_buft.device = r->devs.empty() ? nullptr : &r->devs[0]->dev;
    });
    return &host_buft;
}

// Page-locks memory the caller already owns (e.g. a loaded model file or a PCM ring) so copies out of it run at DMA
// rate. Opt-in like the reference's (GGML_Q2A_REGISTER_HOST set; ggml-cuda.cu GGML_CUDA_REGISTER_HOST): false if not
// enabled or the runtime refuses; the buffer works either way
bool ggml_backend_q2a_register_host_buffer(void * buffer, size_t size) {
    if (getenv("GGML_Q2A_REGISTER_HOST") == nullptr || buffer == nullptr || size == 0) return false;
    if (hipHostRegister(buffer, size, hipHostRegisterPortable | hipHostRegisterReadOnly) != hipSuccess) {
        (void) hipGetLastError();
        Q2A_LOG_ERROR("ggml-q2a: registering %.2f MB of host memory failed\n", size / 1e6);
        return false;
    }
    return true;
}

void ggml_backend_q2a_unregister_host_buffer(void * buffer) {
    if (getenv("GGML_Q2A_REGISTER_HOST") == nullptr || buffer == nullptr) return;
    if (hipHostUnregister(buffer) != hipSuccess) (void) hipGetLastError();
}

int ggml_backend_q2a_get_device_count(void) { return (int) reg_ctx()->devs.size(); }

void ggml_backend_q2a_get_device_description(int device, char * description, size_t n) {
    q2a_device_ctx * d = dev_ctx(device);
    snprintf(description, n, "%s", d ? d->desc.c_str() : "");
}

void ggml_backend_q2a_get_device_memory(int device, size_t * free, size_t * total) {
    *free = 0;
    *total = 0;
    if (hipSetDevice(device) != hipSuccess) return;
    (void) hipMemGetInfo(free, total);
}

ggml_backend_reg_t ggml_backend_q2a_reg(void) {
    (void) reg_ctx();
    return the_reg();
}

void ggml_backend_q2a_get_stats(ggml_backend_t backend, ggml_backend_q2a_stats * stats) {
    if (ggml_backend_is_q2a(backend) && stats) {
        const q2a_backend_ctx * b = (const q2a_backend_ctx *) backend->context;
        *stats = b->stats;
        stats->n_buffer_reallocs = b->n_buffer_reallocs;
        stats->n_mul_mat_conv_total = b->n_mul_mat_conv_total;
        stats->n_repack_lazy = b->n_repack_lazy;
    }
}

}  // extern "C"
