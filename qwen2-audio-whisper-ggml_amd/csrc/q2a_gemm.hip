// q2a_gemm.hip — fused weight GEMM for gfx950: C[M][N] = A[M][K] . W[N][K]^T on fp16 MFMA
// (v_mfma_f32_16x16x32_f16, fp32 accumulation) with the reference's per-op epilogues fused in.
//
// Reference ops replaced: MUL_MAT (ggml_compute_forward_mul_mat ggml.c:12439-12652) plus the
// ADD (bias / residual), SCALE (Q*1/8), GELU, CONT/permute nodes around it (qwen2-whisper.cpp:2029-2154) and the
// IM2COL+MUL_MAT conv pair (ggml_conv_1d ggml.c:6635-6652, as an implicit GEMM with overlapping A rows).
//
// Exactness: every A/W operand fed here is exactly representable in fp16 (ggml rounds activations to fp16 for
// F16 weights; Q8_K/Q8_0 codes and sc*q weight products are small integers), products are exact in fp32 and
// only the fp32 summation order differs from ggml. For the k-quant formats the integer per-block sums are kept
// in a fresh accumulator per K-block and combined with ggml's scale formula (ggml-quants.c:7795-7858).
//
// Tiling: 128x128x64 per 256-thread workgroup (2x2 waves, 64x64 per wave = 4x4 MFMA tiles), LDS operand images
// filled by global_load_lds_dwordx4 (16 B/lane, lane-linear LDS destination) with the XOR swizzle applied on the
// global SOURCE address and undone on the ds_read (cdna_hip_programming.md §5.4 rule 21), two LDS stages.
// Workgroup -> tile order is XCD-aware (bijective remap; neighbouring N tiles of one A panel share an XCD L2).
#include "q2a_internal.h"

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void * lds_ptr_t;

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int ROWB = BK * 2;   // bytes per LDS row (64 halves)

__device__ __forceinline__ float gelu_lut(float x, const uint16_t * tab) {
    // ggml_vec_gelu_f32 with GGML_GELU_FP16 (ggml.c:2556-2570)
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    const _Float16 h = (_Float16) x;
    uint16_t u;
    __builtin_memcpy(&u, &h, 2);
    const uint16_t g = __ldg(tab + u);
    _Float16 gh;
    __builtin_memcpy(&gh, &g, 2);
    return (float) gh;
}

__device__ __forceinline__ int64_t a_row_off(const q2a_gemm_args & p, int m) {
    return ((int64_t) (m / p.a_rpg) * p.a_gstride + (int64_t) (m % p.a_rpg) * p.a_step) * p.lda;
}

template <int EPI>
__device__ __forceinline__ void epilogue_store(const q2a_gemm_args & p, int m, int n, float v) {
    if (EPI == Q2A_EPI_RESID) {
        float * o = p.outF + (int64_t) m * p.ldo + n;
        *o = (v + p.bias[n]) + *o;
    } else if (EPI == Q2A_EPI_GELU_H) {
        const int64_t row = (int64_t) (m / p.o_rpg) * p.o_gstride + (m % p.o_rpg) + p.o_off;
        p.outH[row * p.ldo + n] = (_Float16) gelu_lut(v + p.bias[n], p.gelu_tab);
    } else if (EPI == Q2A_EPI_GELU_F) {
        p.outF[(int64_t) m * p.ldo + n] = gelu_lut(v + p.bias[n], p.gelu_tab);
    } else if (EPI == Q2A_EPI_CONV2) {
        const float g = gelu_lut(v + p.bias[n], p.gelu_tab);
        p.outF[(int64_t) m * p.ldo + n] = p.pe[(int64_t) (m % p.T) * p.ldo + n] + g;
    } else if (EPI == Q2A_EPI_STORE_F) {
        p.outF[(int64_t) m * p.ldo + n] = v;
    } else if (EPI == Q2A_EPI_QKV) {
        const int part = n / p.D, c = n - part * p.D;
        const float val = v + p.bias[n];
        if (part == 0) {
            const float q = val * p.qscale;   // ggml_scale after the bias add (qwen2-whisper.cpp:2054); exact 2^-3
            const _Float16 hi = (_Float16) q;
            const _Float16 lo = (_Float16) (q - (float) hi);
            p.qh[(int64_t) m * p.D + c] = hi;
            p.ql[(int64_t) m * p.D + c] = lo;
        } else if (part == 1) {
            const _Float16 hi = (_Float16) val;
            const _Float16 lo = (_Float16) (val - (float) hi);
            p.kh[(int64_t) m * p.D + c] = hi;
            p.kl[(int64_t) m * p.D + c] = lo;
        } else {
            const int clip = m / p.T, t = m - clip * p.T;
            const int h = c >> 6, d = c & 63;
            p.vt[(((int64_t) clip * p.H + h) * 64 + d) * p.TP + t] = (_Float16) val;
        }
    }
}

// Stage one BM x BK A tile and one BN x BK W tile into LDS buffer `buf` (fp16 elements) for K offset k0.
__device__ __forceinline__ void stage(const q2a_gemm_args & p, char * lds_buf, const int64_t * arow, const int64_t * wrow,
                                      int k0, int wave, int lane) {
    const int c = lane & 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = wave * 32 + i * 8 + (lane >> 3);
        const int sc = c ^ (r & 7);
        const q2a_half * src = p.A + arow[i] + k0 + sc * 8;
        __builtin_amdgcn_global_load_lds((const void *) src, (lds_ptr_t) (lds_buf + (wave * 32 + i * 8) * ROWB), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = wave * 32 + i * 8 + (lane >> 3);
        const int sc = c ^ (r & 7);
        const q2a_half * src = p.W + wrow[i] + k0 + sc * 8;
        __builtin_amdgcn_global_load_lds((const void *) src, (lds_ptr_t) (lds_buf + (BM + wave * 32 + i * 8) * ROWB), 16, 0, 0);
    }
}

__device__ __forceinline__ half8 frag(const char * img, int row, int chunk) {
    return *(const half8 *) (img + row * ROWB + ((chunk ^ (row & 7)) << 4));
}

template <int EPI, int BLK>
__global__ __launch_bounds__(256, 2) void k_gemm(const q2a_gemm_args p) {
    __shared__ __attribute__((aligned(16))) char lds[2][(BM + BN) * ROWB];   // 2 x 32 KiB
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;

    // XCD-aware bijective remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective")
    const int nbn = p.N / BN, nbm = (p.M + BM - 1) / BM, nwg = nbn * nbm;
    const int bid = blockIdx.x, xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    const int tn = wgid % nbn, tm = wgid / nbn;
    const int m0 = tm * BM, n0 = tn * BN;

    // per-lane source rows for the 4+4 glds instructions of this wave (rows past M clamp to M-1: loaded, never stored)
    int64_t arow[4], wrow[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = wave * 32 + i * 8 + (lane >> 3);
        arow[i] = a_row_off(p, min(m0 + r, p.M - 1));
        wrow[i] = (int64_t) (n0 + r) * p.ldw;
    }

    f4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    f4 blk[4][4];
    if (BLK) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) blk[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    }

    const int nk = p.K / BK;
    stage(p, lds[0], arow, wrow, 0, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) stage(p, lds[cur ^ 1], arow, wrow, (kt + 1) * BK, wave, lane);
        const char * ia = lds[cur];
        const char * iw = lds[cur] + BM * ROWB;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int chunk = s * 4 + (lane >> 4);
            half8 a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = frag(ia, wm * 64 + i * 16 + (lane & 15), chunk);
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = frag(iw, wn * 64 + j * 16 + (lane & 15), chunk);
            if (BLK == 0) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) blk[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], blk[i][j], 0, 0, 0);
                const int kpos = kt * BK + (s + 1) * 32;   // K consumed so far
                if (kpos % BLK == 0) {
                    const int kb = kpos / BLK - 1;
                    float dy[4][4], dx[4], dm[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int m = min(m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r, p.M - 1);
                            dy[i][r] = p.dy[(int64_t) m * p.nblk + kb];
                        }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int n = n0 + wn * 64 + j * 16 + (lane & 15);
                        dx[j] = p.dx[(int64_t) n * p.nblk + kb];
                        if (BLK == 256) dm[j] = p.dmin[(int64_t) n * p.nblk + kb];
                    }
                    if (BLK == 256) {
                        // min term S2 = sum_j m_j * bsum32_j with one 16x16x16 MFMA per tile on (hi,lo) split bsums
                        half4 ae[4], we[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int m = min(m0 + wm * 64 + i * 16 + (lane & 15), p.M - 1);
                            ae[i] = *(const half4 *) (p.aext + ((int64_t) m * p.nblk + kb) * 16 + (lane >> 4) * 4);
                        }
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int n = n0 + wn * 64 + j * 16 + (lane & 15);
                            we[j] = *(const half4 *) (p.wext + ((int64_t) n * p.nblk + kb) * 16 + (lane >> 4) * 4);
                        }
#pragma unroll
                        for (int i = 0; i < 4; ++i)
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                f4 s2 = __builtin_amdgcn_mfma_f32_16x16x16f16(ae[i], we[j], f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    acc[i][j][r] += (dy[i][r] * dx[j]) * blk[i][j][r];
                                    acc[i][j][r] -= (dy[i][r] * dm[j]) * s2[r];
                                }
                                blk[i][j] = f4{0.f, 0.f, 0.f, 0.f};
                            }
                    } else {
#pragma unroll
                        for (int i = 0; i < 4; ++i)
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
#pragma unroll
                                for (int r = 0; r < 4; ++r) acc[i][j][r] += (dx[j] * dy[i][r]) * blk[i][j][r];
                                blk[i][j] = f4{0.f, 0.f, 0.f, 0.f};
                            }
                    }
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // epilogue: C layout of 16x16 tiles: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
            if (m >= p.M) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int n = n0 + wn * 64 + j * 16 + (lane & 15);
                epilogue_store<EPI>(p, m, n, acc[i][j][r]);
            }
        }
}

template <int EPI>
hipError_t launch_epi(const q2a_gemm_args & a, int blk, hipStream_t s) {
    const int nwg = (a.N / BN) * ((a.M + BM - 1) / BM);
    if (blk == 0) hipLaunchKernelGGL((k_gemm<EPI, 0>), dim3(nwg), dim3(256), 0, s, a);
    else if (blk == 256) hipLaunchKernelGGL((k_gemm<EPI, 256>), dim3(nwg), dim3(256), 0, s, a);
    else if (blk == 32) hipLaunchKernelGGL((k_gemm<EPI, 32>), dim3(nwg), dim3(256), 0, s, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace

hipError_t q2a_launch_gemm(const q2a_gemm_args & a, int epi, int blk, hipStream_t s) {
    if (a.N % BN != 0 || a.K % BK != 0 || a.M <= 0) return hipErrorInvalidValue;
    if (blk && (a.K % blk != 0)) return hipErrorInvalidValue;
    switch (epi) {
        case Q2A_EPI_QKV: return launch_epi<Q2A_EPI_QKV>(a, blk, s);
        case Q2A_EPI_RESID: return launch_epi<Q2A_EPI_RESID>(a, blk, s);
        case Q2A_EPI_GELU_H: return launch_epi<Q2A_EPI_GELU_H>(a, blk, s);
        case Q2A_EPI_CONV2: return launch_epi<Q2A_EPI_CONV2>(a, blk, s);
        case Q2A_EPI_GELU_F: return launch_epi<Q2A_EPI_GELU_F>(a, blk, s);
        case Q2A_EPI_STORE_F: return launch_epi<Q2A_EPI_STORE_F>(a, blk, s);
        default: return hipErrorInvalidValue;
    }
}
