// q2a_attn.hip — fused multi-head self-attention for gfx950 (flash-style, no T x T score tensor in HBM).
//
// Replaces, per layer (qwen2-whisper.cpp:2052-2107): KQ = mul_mat(K, Q) (F32, ggml.c:12439), SOFT_MAX
// (ggml.c:13854-13950, scale 1, no mask), KQV = mul_mat(cont(V^T), KQ_soft_max), the permutes and the merge.
// The reference materialises 20 x 1500 x 1500 F32 scores per layer (180 MB per clip).
//
// Numerics: the reference computes QK^T in F32. Here Q and K arrive as fp16 hi/lo pairs (x = hi + lo, 22
// significant bits) and S = Kh.Qh + Kl.Qh + Kh.Ql on fp16 MFMA with fp32 accumulation (the lo.lo term is below
// 2^-22 relative), i.e. F32-class scores. P (in [0,1]) and V are fp16 for the P.V product. Online softmax keeps
// a running max/sum per query; the 1/sum normalisation is applied once at the end.
//
// Structure: one 256-thread workgroup = 4 waves x 32 queries of one (clip, head); K/V tiles of 64 keys are
// register-staged into double-buffered LDS images (rows padded to 144 B / 136 B: conflict-free ds_read_b128 /
// ds_read_b64 for 32 distinct rows). S^T = K.Q^T is computed with v_mfma_f32_32x32x16_f16 so each lane owns one
// query column (softmax is lane-local plus one lane^32 exchange) and the S accumulator feeds the P.V MFMA as
// its B operand with no data movement (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand").
#include "q2a_internal.h"

#include <cstdlib>

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void * lds_ptr_t;

// 32x32x16 MFMA on fp16 operands, or on the same bits read as bf16 (bf16-activation mode)
template <bool BF>
__device__ __forceinline__ f16v mma32(half8 a, half8 b, f16v c) {
    if constexpr (BF) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, a), __builtin_bit_cast(bf8, b), c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
template <bool BF>
__device__ __forceinline__ _Float16 to16(float v) {
    if constexpr (BF) return __builtin_bit_cast(_Float16, (__bf16) v);
    else return (_Float16) v;
}

constexpr int KT = 64;            // keys per LDS tile
// LDS images per mode. F32-class (3 MFMAs per step, 174 VGPRs, 2 workgroups per CU): rows padded to 144 B (K) /
// 136 B (V^T). bf16 (one MFMA per step, fewer registers): unpadded 128-B rows, XOR-swizzled — the K image's 16-B
// chunk ch of row r at chunk ch ^ ((r >> 1) & 7), the V^T image's 8-B chunk c at c ^ ((r >> 1) & 15), conflict-free
// for ds_read_b128 (16-lane groups of distinct rows) and ds_read_b64 (32 distinct rows) — 48 KiB per workgroup, so
// three fit a CU (measured: padded 2/CU 33.4 ms/step, swizzled 3/CU 31.8; the swizzle alone costs address VALU)
#ifndef Q2A_ATTN_F32_OCC
#define Q2A_ATTN_F32_OCC 2
#endif
template <bool SW> struct attn_lds;
template <> struct attn_lds<false> {
    static constexpr int KROW = 144, VROW = 136;
    static __device__ __forceinline__ int k(int, int ch) { return ch << 4; }
    static __device__ __forceinline__ int v(int, int c8) { return c8 << 3; }
};
template <> struct attn_lds<true> {
    static constexpr int KROW = 128, VROW = 128;
    static __device__ __forceinline__ int k(int r, int ch) { return (ch ^ ((r >> 1) & 7)) << 4; }
    static __device__ __forceinline__ int v(int r, int c8) { return (c8 ^ ((r >> 1) & 15)) << 3; }
};
constexpr float L2E = 1.4426950408889634f;   // exp(x) = exp2(x * log2 e)

// BF: bf16-activation mode (Q, K, V^T, P and the output in bf16; S = K.Q^T is one MFMA per 16-deep step)
// QT: fp16 terms of S in the reference contract (3: Kh.Qh + Kl.Qh + Kh.Ql, the default; 2 / 1: precision experiments,
// Q2A_ATTN_TERMS, diag only)
template <bool BF, int QT = 3>
__global__ __launch_bounds__(256, BF ? 3 : Q2A_ATTN_F32_OCC) void k_attn(const q2a_attn_args p) {
    typedef attn_lds<BF || Q2A_ATTN_F32_OCC >= 3> LY;
    constexpr int KROW = LY::KROW, VROW = LY::VROW;
    constexpr int KIMG = KT * KROW, VIMG = 64 * VROW, STAGE = 2 * KIMG + VIMG;
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int T = p.T, D = p.D;
    // XCD-contiguous work order: workgroup L is dispatched to XCD L % 8, so work item w = (L % 8)·(total/8) + L/8
    // puts the q-tiles of one (clip, head) on ONE XCD at about the same time and its K/V are fetched into that
    // L2 once instead of into up to eight of them (bijective when total % 8 == 0, identity otherwise)
    const int nq = (T + 127) / 128, total = (int) gridDim.x;
    const int L = (int) blockIdx.x;
    const int w = (total & 7) ? L : (L & 7) * (total >> 3) + (L >> 3);
    const int qt = w % nq, h = (w / nq) % p.H, clip = w / (nq * p.H);
    const int q0 = qt * 128 + wave * 32;
    const int64_t rowbase = (int64_t) clip * T;
    const int hi = lane >> 5, col = lane & 31;

    // Q fragments (B operand of S^T = K.Q^T): lane holds Q[q0+col][16s + 8hi .. +7]
    half8 qh[4], ql[4];
    {
        const int q = min(q0 + col, T - 1);
        const q2a_half * sh = p.qh + (rowbase + q) * D + h * 64 + 8 * hi;
        const q2a_half * sl = p.ql + (rowbase + q) * D + h * 64 + 8 * hi;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            qh[s] = *(const half8 *) (sh + 16 * s);
            ql[s] = BF ? qh[s] : *(const half8 *) (sl + 16 * s);
        }
    }

    // staging: each thread moves 2 x 16 B of Kh, of Kl and of V^T per tile
    const q2a_half * vt_base = p.vt + ((int64_t) clip * p.H + h) * 64 * p.TP;
    uint4 rk_h0, rk_h1, rk_l0, rk_l1, rv0, rv1;
#define Q2A_LOAD_TILE(t_)                                                                           \
    do {                                                                                            \
        const int kb0_ = (t_) * KT;                                                                 \
        const int c0_ = tid, c1_ = tid + 256;                                                       \
        const int k0_ = min(kb0_ + (c0_ >> 3), T - 1), k1_ = min(kb0_ + (c1_ >> 3), T - 1);       \
        rk_h0 = *(const uint4 *) (p.kh + (rowbase + k0_) * D + h * 64 + (c0_ & 7) * 8);              \
        rk_h1 = *(const uint4 *) (p.kh + (rowbase + k1_) * D + h * 64 + (c1_ & 7) * 8);              \
        if (!BF) {                                                                                  \
            rk_l0 = *(const uint4 *) (p.kl + (rowbase + k0_) * D + h * 64 + (c0_ & 7) * 8);          \
            rk_l1 = *(const uint4 *) (p.kl + (rowbase + k1_) * D + h * 64 + (c1_ & 7) * 8);          \
        }                                                                                           \
        rv0 = *(const uint4 *) (vt_base + (int64_t) (c0_ >> 3) * p.TP + kb0_ + (c0_ & 7) * 8);      \
        rv1 = *(const uint4 *) (vt_base + (int64_t) (c1_ >> 3) * p.TP + kb0_ + (c1_ & 7) * 8);      \
    } while (0)
#define Q2A_STORE_ONE(st_, c_, kh_, kl_, v_)                                                        \
    do {                                                                                            \
        const int r_ = (c_) >> 3, ch_ = (c_) & 7;                                                   \
        *(uint4 *) ((st_) + r_ * KROW + LY::k(r_, ch_)) = (kh_);                                     \
        if (!BF) *(uint4 *) ((st_) + KIMG + r_ * KROW + LY::k(r_, ch_)) = (kl_);                     \
        char * vr_ = (st_) + 2 * KIMG + r_ * VROW;                                                  \
        *(uint2 *) (vr_ + LY::v(r_, 2 * ch_)) = make_uint2((v_).x, (v_).y);                          \
        *(uint2 *) (vr_ + LY::v(r_, 2 * ch_ + 1)) = make_uint2((v_).z, (v_).w);                      \
    } while (0)
#define Q2A_STORE_TILE(buf_)                                                                        \
    do {                                                                                            \
        char * st__ = lds + (buf_) * STAGE;                                                         \
        Q2A_STORE_ONE(st__, tid, rk_h0, rk_l0, rv0);                                                \
        Q2A_STORE_ONE(st__, tid + 256, rk_h1, rk_l1, rv1);                                          \
    } while (0)

    f16v o[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    float m_run = -1e30f, l_run = 0.f;

    const int ntiles = (T + KT - 1) / KT;
    Q2A_LOAD_TILE(0);
    Q2A_STORE_TILE(0);
    // the Q fragments must be complete before the loop (an asm "use" makes the waitcnt pass wait for them here):
    // otherwise their loads stay pending at the loop header, merge with the next-tile prefetch and every
    // iteration's QK^T MFMAs wait on that prefetch
    asm volatile("" :: "v"(qh[0]), "v"(qh[1]), "v"(qh[2]), "v"(qh[3]), "v"(ql[0]), "v"(ql[1]), "v"(ql[2]), "v"(ql[3]));
    __syncthreads();

    for (int t = 0; t < ntiles; ++t) {
        const int cur = t & 1;
        if (t + 1 < ntiles) Q2A_LOAD_TILE(t + 1);
        const char * kh_img = lds + cur * STAGE;
        const char * kl_img = kh_img + KIMG;
        const char * vt_img = kh_img + 2 * KIMG;
        // S^T for both 32-key halves of the tile (24 MFMAs), then ONE online-softmax update per 64 keys
        f16v sc[2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
            for (int r = 0; r < 16; ++r) sc[kb][r] = 0.f;
            const int krow = kb * 32 + col;
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const int off = krow * KROW + LY::k(krow, 2 * st + hi);
                const half8 ah = *(const half8 *) (kh_img + off);
                sc[kb] = mma32<BF>(ah, qh[st], sc[kb]);
                if (!BF) {
                    if (QT >= 3) {
                        const half8 al = *(const half8 *) (kl_img + off);
                        sc[kb] = mma32<BF>(al, qh[st], sc[kb]);
                    }
                    if (QT >= 2) sc[kb] = mma32<BF>(ah, ql[st], sc[kb]);
                }
            }
        }
        if (t == ntiles - 1) {   // keys >= T exist only in the last tile (row of reg r = (r&3) + 8(r>>2) + 4hi)
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (t * KT + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi >= T) sc[kb][r] = -1e30f;
        }
        float mx = sc[0][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sc[0][r]);
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[1][r]);
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float m_new = fmaxf(m_run, mx);
        const float nm = -m_new * L2E;
        const float alpha = __builtin_amdgcn_exp2f(fmaf(m_run, L2E, nm));
        float ls = 0.f;
        half8 pf[2][2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float pv = __builtin_amdgcn_exp2f(fmaf(sc[kb][r], L2E, nm));
                ls += pv;
                pf[kb][r >> 3][r & 7] = to16<BF>(pv);
            }
        l_run = l_run * alpha + ls;
        m_run = m_new;
        if (__any(alpha != 1.0f)) {   // the running max moved for some query of this wave
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
        }
        // O^T[d][q] += V^T[d][keys] . P^T[keys][q]
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
                const int vr = dt * 32 + col;
                const char * vrow = vt_img + vr * VROW;
#pragma unroll
                for (int sp = 0; sp < 2; ++sp) {
                    const int c8 = 8 * kb + 4 * sp + hi;   // 8-B chunk of keys 32kb + 16sp + 4hi .. +3
                    const half4 v0 = *(const half4 *) (vrow + LY::v(vr, c8));
                    const half4 v1 = *(const half4 *) (vrow + LY::v(vr, c8 + 2));
                    const half8 va = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
                    o[dt] = mma32<BF>(va, pf[kb][sp], o[dt]);
                }
            }
        // buffer cur^1 was last read in iteration t-1, before the barrier that ended it
        if (t + 1 < ntiles) Q2A_STORE_TILE(cur ^ 1);
        __syncthreads();
    }

    const float l_tot = l_run + __shfl_xor(l_run, 32);
    const float inv = 1.0f / l_tot;
    const int q = q0 + col;
    if (q < T) {
        const int64_t orow = (rowbase + q) * D + h * 64;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = dt * 32 + 8 * g + 4 * hi;
                const float v0 = o[dt][4 * g + 0] * inv, v1 = o[dt][4 * g + 1] * inv;
                const float v2 = o[dt][4 * g + 2] * inv, v3 = o[dt][4 * g + 3] * inv;
                if (p.outH) {
                    const half4 hv = {to16<BF>(v0), to16<BF>(v1), to16<BF>(v2), to16<BF>(v3)};
                    *(half4 *) (p.outH + orow + d) = hv;
                } else {
                    *(float4 *) (p.outF + orow + d) = make_float4(v0, v1, v2, v3);
                }
            }
    }
}

// ---- F32-class default (Q2A_ATTN_G=0: k_attn instead): k_attn's arithmetic op for op, but the next tile's K hi,
// K lo and V^T arrive by global_load_lds straight into the other of two LDS stages (two __shared__ arrays, the loop
// unrolled by two, so the compiler sees no alias between the stage it reads and the one in flight) instead of through
// 24 staging VGPRs: 48 KiB of LDS and < 168 VGPRs, i.e. three workgroups per CU instead of two. LDS images unpadded,
// 16-B granules XOR-swizzled by row (K: chunk ch of row r at ch ^ ((r >> 1) & 7); V^T: granule g at g ^ ((r >> 1) & 7),
// its two 8-B halves in order — the DMA moves whole granules, with the swizzle on the source address).
struct attn_lds_g {
    static constexpr int KROW = 128, VROW = 128;
    static __device__ __forceinline__ int k(int r, int ch) { return (ch ^ ((r >> 1) & 7)) << 4; }
    static __device__ __forceinline__ int vg(int r, int g) { return (g ^ ((r >> 1) & 7)) << 4; }
};
// K row loaded into row i of the QK^T A operand: i with bits 2 and 3 swapped. S^T's accumulator row for register r
// of lane half hi is (r&3) + 8(r>>2) + 4hi, so register r then holds key 16(r>>3) + 8hi + (r&7): the 8 keys a lane
// half feeds the P.V MFMA as one B fragment are contiguous, and their V^T operand is ONE 16-B LDS read instead of
// two 8-B reads and a register shuffle (softmax is order-free over the keys of a tile)
// exp2 of x <= 0 on the FMA pipe instead of the transcendental unit (v_exp_f32 is the softmax's bottleneck: ~17
// cycles per wave instruction, not overlapped with the MFMAs — profiles/r02q_attention_sq.json). x rounded to the
// nearest integer n by the 1.5*2^23 shift, f = x - n in [-0.5, 0.5], 2^f by a degree-5 polynomial (relative error
// 3.4e-7 in fp32 Horner, vs ~1 ulp for v_exp_f32), n added to the exponent bits. x is clamped at -125 (2^-125 is 0
// once P is rounded to fp16 and nothing against the row sum).
__device__ __forceinline__ float exp2_poly(float x) {
    x = fmaxf(x, -125.0f);
    const float t = x + 12582912.0f;
    const float f = x - (t - 12582912.0f);
    float p = __builtin_fmaf(0.0012915669940412045f, f, 0.009668530896306038f);
    p = __builtin_fmaf(p, f, 0.055516887456178665f);
    p = __builtin_fmaf(p, f, 0.24022264778614044f);
    p = __builtin_fmaf(p, f, 0.6931464672088623f);
    p = __builtin_fmaf(p, f, 1.0f);
    return __uint_as_float(__float_as_uint(p) + (__float_as_uint(t) << 23));
}
// Q2A_ATTN_POLY: how many of every 16 score exponentials of a lane go through exp2_poly (the rest v_exp_f32)
#ifndef Q2A_ATTN_POLY
#define Q2A_ATTN_POLY 0
#endif
__device__ __forceinline__ int kperm(int c) { return (c & ~12) | ((c & 4) << 1) | ((c & 8) >> 1); }
// max of x over lanes l and l ^ 32: v_permlane32_swap exchanges the two wave halves in a VALU slot (no LDS round
// trip as ds_bpermute, no lgkmcnt wait); one of the two results is the lane's own value (attention -1 %, same box)
#ifndef Q2A_ATTN_PERM32
#define Q2A_ATTN_PERM32 1
#endif
__device__ __forceinline__ float max_lane32(float x) {
#if Q2A_ATTN_PERM32
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
#else
    return fmaxf(x, __shfl_xor(x, 32));
#endif
}
// Q2A_ATTN_PRIO: 1 = s_setprio 1 around the QK^T MFMA cluster, 2 = around the QK^T and the P.V clusters (the wave
// with matrix work ready wins issue arbitration over the co-resident waves in their softmax)
#ifndef Q2A_ATTN_PRIO
#define Q2A_ATTN_PRIO 0
#endif
#ifndef Q2A_ATTN_LAZY
#define Q2A_ATTN_LAZY 1   // k_attn_g: lazy re-basing of the softmax max (0 = eager, every tile)
#endif
#ifndef Q2A_ATTN_LAZY_TAU
#define Q2A_ATTN_LAZY_TAU 5.0f
#endif
#ifndef Q2A_ATTN_KPF
#define Q2A_ATTN_KPF 1   // k_attn_g: both 32-key QK^T chains per 16-deep step (136 VGPRs; 0 = chain after chain, 163)
#endif
#ifndef Q2A_ATTN_DIAG_NOSM
#define Q2A_ATTN_DIAG_NOSM 0   // diagnostic builds only (diag/build_attn_variant.sh): no softmax VALU
#endif
#ifndef Q2A_ATTN_DIAG_NOEXP
#define Q2A_ATTN_DIAG_NOEXP 0  // diagnostic builds only: exp2 of the scores replaced by a multiply
#endif
#ifndef Q2A_ATTN_DIAG_NOPV
#define Q2A_ATTN_DIAG_NOPV 0   // diagnostic builds only: no P.V MFMAs
#endif
__global__ __launch_bounds__(256, 3) void k_attn_g(const q2a_attn_args p) {
    typedef attn_lds_g LY;
    constexpr int KROW = LY::KROW, VROW = LY::VROW;
    constexpr int KIMG = KT * KROW, VIMG = 64 * VROW, STAGE = 2 * KIMG + VIMG;
    __shared__ __attribute__((aligned(16))) char ldsA[STAGE];
    __shared__ __attribute__((aligned(16))) char ldsB[STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = p.T, D = p.D;
    const int nq = (T + 127) / 128, total = (int) gridDim.x;
    const int L = (int) blockIdx.x;
    const int w = (total & 7) ? L : (L & 7) * (total >> 3) + (L >> 3);   // XCD-contiguous work order (k_attn)
    const int qt = w % nq, h = (w / nq) % p.H, clip = w / (nq * p.H);
    const int q0 = qt * 128 + wave * 32;
    const int64_t rowbase = (int64_t) clip * T;
    const int hi = lane >> 5, col = lane & 31;

    half8 qh[4], ql[4];
    {
        const int q = min(q0 + col, T - 1);
        const q2a_half * sh = p.qh + (rowbase + q) * D + h * 64 + 8 * hi;
        const q2a_half * sl = p.ql + (rowbase + q) * D + h * 64 + 8 * hi;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            qh[s] = *(const half8 *) (sh + 16 * s);
            ql[s] = *(const half8 *) (sl + 16 * s);
        }
    }
    const q2a_half * vt_base = p.vt + ((int64_t) clip * p.H + h) * 64 * p.TP;
    // tile t -> stage: wave w's instruction i covers rows (2w + i) * 8 .. +7 of each image (1 KiB), lane l row
    // + l / 8, LDS granule l % 8 <- source granule (l % 8) ^ ((row >> 1) & 7)
    // sources as a uniform (clip, head) base + a 32-bit per-lane byte offset (the saddr form of the DMA: no 64-bit
    // address arithmetic per tile; a clip's K rows span T·D·2 B, its head's V^T 64·TP·2 B)
    const char * khb = (const char *) (p.kh + rowbase * D + h * 64);
    const char * klb = (const char *) (p.kl + rowbase * D + h * 64);
    const char * vtb = (const char *) vt_base;
    auto dma_tile = [&](char * st, int t) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int row = (2 * wave + i) * 8 + (lane >> 3), g = (lane & 7) ^ ((row >> 1) & 7);
            const int key = min(t * KT + row, T - 1);
            const uint32_t ko = (uint32_t) (key * D + g * 8) * 2u;
            const uint32_t vo = (uint32_t) (row * p.TP + t * KT + g * 8) * 2u;
            __builtin_amdgcn_global_load_lds((const void *) (khb + ko), (lds_ptr_t) (st + (2 * wave + i) * 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void *) (klb + ko), (lds_ptr_t) (st + KIMG + (2 * wave + i) * 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void *) (vtb + vo), (lds_ptr_t) (st + 2 * KIMG + (2 * wave + i) * 1024), 16, 0, 0);
        }
    };

    f16v o[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    float m_run = -1e30f, l_run = 0.f, nm_run = 0.f;
    const int ntiles = (T + KT - 1) / KT;

    auto tile = [&](const char * kh_img, int t) {
        const char * kl_img = kh_img + KIMG;
        const char * vt_img = kh_img + 2 * KIMG;
        f16v sc[2];
        if (Q2A_ATTN_PRIO >= 1) __builtin_amdgcn_s_setprio(1);
#if Q2A_ATTN_KPF
        // K fragments one 16-deep step ahead: the reads of step st+1 (both 32-key halves) are issued before the MFMAs
        // of step st, so each MFMA group waits only for its own reads (lgkmcnt(4), not 0); same MFMA order per chain
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) sc[kb][r] = 0.f;
        half8 fh[2], fl[2];
        auto rdk = [&](int st, int kb, half8 & h, half8 & l) {
            const int krow = kb * 32 + kperm(col);
            const int off = krow * KROW + LY::k(krow, 2 * st + hi);
            h = *(const half8 *) (kh_img + off);
            l = *(const half8 *) (kl_img + off);
        };
        rdk(0, 0, fh[0], fl[0]);
        rdk(0, 1, fh[1], fl[1]);
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            half8 nh[2], nl[2];
            if (st < 3) { rdk(st + 1, 0, nh[0], nl[0]); rdk(st + 1, 1, nh[1], nl[1]); }
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                sc[kb] = mma32<false>(fh[kb], qh[st], sc[kb]);
                sc[kb] = mma32<false>(fl[kb], qh[st], sc[kb]);
                sc[kb] = mma32<false>(fh[kb], ql[st], sc[kb]);
            }
            if (st < 3) { fh[0] = nh[0]; fh[1] = nh[1]; fl[0] = nl[0]; fl[1] = nl[1]; }
        }
#else
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
            for (int r = 0; r < 16; ++r) sc[kb][r] = 0.f;
            const int krow = kb * 32 + kperm(col);
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const int off = krow * KROW + LY::k(krow, 2 * st + hi);
                const half8 ah = *(const half8 *) (kh_img + off);
                sc[kb] = mma32<false>(ah, qh[st], sc[kb]);
                const half8 al = *(const half8 *) (kl_img + off);
                sc[kb] = mma32<false>(al, qh[st], sc[kb]);
                sc[kb] = mma32<false>(ah, ql[st], sc[kb]);
            }
        }
#endif
        if (Q2A_ATTN_PRIO >= 1) __builtin_amdgcn_s_setprio(0);
        if (t == ntiles - 1) {   // keys >= T exist only in the last tile (key of reg r: 16(r>>3) + 8hi + (r&7))
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (t * KT + kb * 32 + 16 * (r >> 3) + 8 * hi + (r & 7) >= T) sc[kb][r] = -1e30f;
        }
#if Q2A_ATTN_DIAG_NOSM   // diagnostic timing build: no max / exp (P = S / 64), wrong values on purpose
        half8 pf[2][2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) pf[kb][r >> 3][r & 7] = (_Float16) (sc[kb][r] * 0.015625f);
        l_run += 1.0f;
#else
        float mx = sc[0][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sc[0][r]);
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[1][r]);
        mx = max_lane32(mx);
#if Q2A_ATTN_LAZY && !Q2A_ATTN_DIAG_NOEXP && !Q2A_ATTN_POLY
        // lazy re-basing: the exponent's reference m_run moves only when some score of the wave's queries exceeds it
        // by more than Q2A_ATTN_LAZY_TAU (natural-log units: P <= e^TAU in between, well inside fp16), so most tiles
        // skip the alpha exponential and the O / l rescale (fma(m_run, L2E, -m_new L2E) is the product's rounding
        // error, not 0, when the max did not move: the eager form multiplied O by 1 + ulp on almost every tile)
        if (__any(mx > m_run + Q2A_ATTN_LAZY_TAU)) {
            const float m_new = fmaxf(m_run, mx);
            const float nm_new = -m_new * L2E;
            const float alpha = __builtin_amdgcn_exp2f(fmaf(m_run, L2E, nm_new));
            l_run *= alpha;
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
            m_run = m_new;
            nm_run = nm_new;
        }
        const float nm = nm_run;
        float ls = 0.f;
        half8 pf[2][2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float pv = __builtin_amdgcn_exp2f(fmaf(sc[kb][r], L2E, nm));
                ls += pv;
                pf[kb][r >> 3][r & 7] = (_Float16) pv;
            }
        l_run += ls;
#else
        const float m_new = fmaxf(m_run, mx);
        const float nm = -m_new * L2E;
        const float alpha = __builtin_amdgcn_exp2f(fmaf(m_run, L2E, nm));
        float ls = 0.f;
        half8 pf[2][2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
#if Q2A_ATTN_DIAG_NOEXP   // diagnostic: the transcendental replaced by a multiply (wrong values on purpose)
                const float pv = fmaf(sc[kb][r], L2E, nm) * 0.01f;
#else
                const float xr = fmaf(sc[kb][r], L2E, nm);
                const float pv = (r & 3) < Q2A_ATTN_POLY / 4 ? exp2_poly(xr) : __builtin_amdgcn_exp2f(xr);
#endif
                ls += pv;
                pf[kb][r >> 3][r & 7] = (_Float16) pv;
            }
        l_run = l_run * alpha + ls;
        m_run = m_new;
        if (__any(alpha != 1.0f)) {
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
        }
#endif
#endif
        if (Q2A_ATTN_PRIO >= 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
                const int vr = dt * 32 + col;
#pragma unroll
                for (int sp = 0; sp < 2; ++sp) {   // keys 32kb + 16sp + 8hi .. +7: one 16-B granule of the V^T row
                    const half8 va = *(const half8 *) (vt_img + vr * VROW + LY::vg(vr, 4 * kb + 2 * sp + hi));
                    if (!Q2A_ATTN_DIAG_NOPV) o[dt] = mma32<false>(va, pf[kb][sp], o[dt]);
                    else o[dt][0] += (float) pf[kb][sp][0] + (float) va[1];   // diagnostic: keep P and V live
                }
            }
        if (Q2A_ATTN_PRIO >= 2) __builtin_amdgcn_s_setprio(0);
    };

    dma_tile(ldsA, 0);
    asm volatile("" :: "v"(qh[0]), "v"(qh[1]), "v"(qh[2]), "v"(qh[3]), "v"(ql[0]), "v"(ql[1]), "v"(ql[2]), "v"(ql[3]));
    __syncthreads();   // (waits for the DMA: a pending LDS-DMA is a vmcnt event)
    for (int t = 0; t < ntiles; t += 2) {
        if (t + 1 < ntiles) dma_tile(ldsB, t + 1);
        tile(ldsA, t);
        __syncthreads();   // tile t + 1 landed (vmcnt(0) in the barrier), every wave done with A
        if (t + 1 >= ntiles) break;
        if (t + 2 < ntiles) dma_tile(ldsA, t + 2);
        tile(ldsB, t + 1);
        __syncthreads();
    }

    const float l_tot = l_run + __shfl_xor(l_run, 32);
    const float inv = 1.0f / l_tot;
    const int q = q0 + col;
    if (q < T) {
        const int64_t orow = (rowbase + q) * D + h * 64;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = dt * 32 + 8 * g + 4 * hi;
                const float v0 = o[dt][4 * g + 0] * inv, v1 = o[dt][4 * g + 1] * inv;
                const float v2 = o[dt][4 * g + 2] * inv, v3 = o[dt][4 * g + 3] * inv;
                if (p.outH) {
                    const half4 hv = {(_Float16) v0, (_Float16) v1, (_Float16) v2, (_Float16) v3};
                    *(half4 *) (p.outH + orow + d) = hv;
                } else {
                    *(float4 *) (p.outF + orow + d) = make_float4(v0, v1, v2, v3);
                }
            }
    }
}

// ---- F32-class, 32-key tiles (k_attn_g32): k_attn_g's arithmetic per 32-key half tile — the same three MFMAs per
// 16-deep step in the same order, the same exp2/fp16 P — with the online-softmax update once per 32 keys instead of
// once per 64, so only 16 score registers are live and the kernel fits 128 VGPRs: FOUR workgroups (16 waves) per CU
// instead of three, for latency hiding. A stage is 12 KiB (K hi, K lo: 32 rows x 128 B; V^T: 64 rows x 64 B), two
// stages 24 KiB, four workgroups 96 KiB of LDS. Per tile each wave DMAs one 1-KiB piece of each image. LDS layouts:
// K as k_attn_g (16-B chunk ch of row r at ch ^ ((r >> 1) & 7)); V^T granule g of row r at g ^ ((r >> 2) & 3), which
// makes the 16 rows of each ds_read_b128 lane group hit 16 distinct 16-B bank groups of the 64-B rows.
// NOTE: per-32-key updates change where the running max is re-based (m after 32 keys instead of 64): P values are
// exp2 of a different (equally valid) shift, so results are F32-class-equal to k_attn_g, not bit-identical.
constexpr int KT32 = 32;
__global__ __launch_bounds__(256, 4) void k_attn_g32(const q2a_attn_args p) {
    constexpr int KROW = 128, VROW = 64;
    constexpr int KIMG = KT32 * KROW, VIMG = 64 * VROW, STAGE = 2 * KIMG + VIMG;
    __shared__ __attribute__((aligned(16))) char ldsA[STAGE];
    __shared__ __attribute__((aligned(16))) char ldsB[STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = p.T, D = p.D;
    const int nq = (T + 127) / 128, total = (int) gridDim.x;
    const int L = (int) blockIdx.x;
    const int w = (total & 7) ? L : (L & 7) * (total >> 3) + (L >> 3);   // XCD-contiguous work order (k_attn)
    const int qt = w % nq, h = (w / nq) % p.H, clip = w / (nq * p.H);
    const int q0 = qt * 128 + wave * 32;
    const int64_t rowbase = (int64_t) clip * T;
    const int hi = lane >> 5, col = lane & 31;

    half8 qh[4], ql[4];
    {
        const int q = min(q0 + col, T - 1);
        const q2a_half * sh = p.qh + (rowbase + q) * D + h * 64 + 8 * hi;
        const q2a_half * sl = p.ql + (rowbase + q) * D + h * 64 + 8 * hi;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            qh[s] = *(const half8 *) (sh + 16 * s);
            ql[s] = *(const half8 *) (sl + 16 * s);
        }
    }
    const char * khb = (const char *) (p.kh + rowbase * D + h * 64);
    const char * klb = (const char *) (p.kl + rowbase * D + h * 64);
    const char * vtb = (const char *) (p.vt + ((int64_t) clip * p.H + h) * 64 * p.TP);
    // wave w: rows 8w .. 8w+7 of the K hi and K lo images (lane: row + lane / 8, LDS chunk lane % 8), rows
    // 16w .. 16w+15 of the V^T image (lane: row + lane / 4, LDS granule lane % 4); swizzles on the source address
    const int krow_d = 8 * wave + (lane >> 3), kg = (lane & 7) ^ ((krow_d >> 1) & 7);
    const int vrow_d = 16 * wave + (lane >> 2), vg = (lane & 3) ^ ((vrow_d >> 2) & 3);
    auto dma_tile = [&](char * st, int t) {
        const int key = min(t * KT32 + krow_d, T - 1);
        const uint32_t ko = (uint32_t) (key * D + kg * 8) * 2u;
        const uint32_t vo = (uint32_t) (vrow_d * p.TP + t * KT32 + vg * 8) * 2u;
        __builtin_amdgcn_global_load_lds((const void *) (khb + ko), (lds_ptr_t) (st + wave * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *) (klb + ko), (lds_ptr_t) (st + KIMG + wave * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *) (vtb + vo), (lds_ptr_t) (st + 2 * KIMG + wave * 1024), 16, 0, 0);
    };

    f16v o[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    float m_run = -1e30f, l_run = 0.f;
    const int ntiles = (T + KT32 - 1) / KT32;
    const int krow = kperm(col);

    auto tile = [&](const char * kh_img, int t) {
        const char * kl_img = kh_img + KIMG;
        const char * vt_img = kh_img + 2 * KIMG;
        f16v sc;
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[r] = 0.f;
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const int off = krow * KROW + attn_lds_g::k(krow, 2 * st + hi);
            const half8 ah = *(const half8 *) (kh_img + off);
            sc = mma32<false>(ah, qh[st], sc);
            const half8 al = *(const half8 *) (kl_img + off);
            sc = mma32<false>(al, qh[st], sc);
            sc = mma32<false>(ah, ql[st], sc);
        }
        if (t == ntiles - 1) {   // keys >= T exist only in the last tile (key of reg r: 16(r>>3) + 8hi + (r&7))
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (t * KT32 + 16 * (r >> 3) + 8 * hi + (r & 7) >= T) sc[r] = -1e30f;
        }
        float mx = sc[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sc[r]);
        mx = max_lane32(mx);
        const float m_new = fmaxf(m_run, mx);
        const float nm = -m_new * L2E;
        const float alpha = __builtin_amdgcn_exp2f(fmaf(m_run, L2E, nm));
        float ls = 0.f;
        half8 pf[2];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float pv = __builtin_amdgcn_exp2f(fmaf(sc[r], L2E, nm));
            ls += pv;
            pf[r >> 3][r & 7] = (_Float16) pv;
        }
        l_run = l_run * alpha + ls;
        m_run = m_new;
        if (__any(alpha != 1.0f)) {
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
        }
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
            const int vr = dt * 32 + col;
#pragma unroll
            for (int sp = 0; sp < 2; ++sp) {   // keys 16sp + 8hi .. +7: one 16-B granule of the V^T row
                const half8 va = *(const half8 *) (vt_img + vr * VROW + (((2 * sp + hi) ^ ((vr >> 2) & 3)) << 4));
                o[dt] = mma32<false>(va, pf[sp], o[dt]);
            }
        }
    };

    dma_tile(ldsA, 0);
    asm volatile("" :: "v"(qh[0]), "v"(qh[1]), "v"(qh[2]), "v"(qh[3]), "v"(ql[0]), "v"(ql[1]), "v"(ql[2]), "v"(ql[3]));
    __syncthreads();   // (waits for the DMA: a pending LDS-DMA is a vmcnt event)
    for (int t = 0; t < ntiles; t += 2) {
        if (t + 1 < ntiles) dma_tile(ldsB, t + 1);
        tile(ldsA, t);
        __syncthreads();   // tile t + 1 landed (vmcnt(0) in the barrier), every wave done with A
        if (t + 1 >= ntiles) break;
        if (t + 2 < ntiles) dma_tile(ldsA, t + 2);
        tile(ldsB, t + 1);
        __syncthreads();
    }

    float l_tot = l_run;
    {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_run), __float_as_uint(l_run), false, false);
        l_tot = __uint_as_float(r[0]) + __uint_as_float(r[1]);   // the lane's own sum plus its partner's
    }
    const float inv = 1.0f / l_tot;
    const int q = q0 + col;
    if (q < T) {
        const int64_t orow = (rowbase + q) * D + h * 64;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = dt * 32 + 8 * g + 4 * hi;
                const float v0 = o[dt][4 * g + 0] * inv, v1 = o[dt][4 * g + 1] * inv;
                const float v2 = o[dt][4 * g + 2] * inv, v3 = o[dt][4 * g + 3] * inv;
                if (p.outH) {
                    const half4 hv = {(_Float16) v0, (_Float16) v1, (_Float16) v2, (_Float16) v3};
                    *(half4 *) (p.outH + orow + d) = hv;
                } else {
                    *(float4 *) (p.outF + orow + d) = make_float4(v0, v1, v2, v3);
                }
            }
    }
}

// ---- F32-class, software-pipelined (k_attn_p32): k_attn_g32's per-32-key arithmetic, but iteration t issues the
// QK^T MFMAs of tile t+1 in the same scheduling region as the online-softmax VALU of tile t (independent, so the
// wave's own matrix pipe and VALU overlap: sched_group_barrier interleaves one MFMA with a group of VALU), then the
// P.V MFMAs of tile t. Three LDS stages (tile t's V^T, tile t+1's K, tile t+2 in flight), 36 KiB, one barrier per
// tile. The QK^T of the (non-existent) tile after the last one reads a stale stage; its scores are discarded.
#ifndef Q2A_ATTN_P32_OCC
#define Q2A_ATTN_P32_OCC 3
#endif
#ifndef Q2A_ATTN_P32_SCHED
#define Q2A_ATTN_P32_SCHED 1
#endif
__global__ __launch_bounds__(256, Q2A_ATTN_P32_OCC) void k_attn_p32(const q2a_attn_args p) {
    constexpr int KROW = 128, VROW = 64;
    constexpr int KIMG = KT32 * KROW, VIMG = 64 * VROW, STAGE = 2 * KIMG + VIMG;
    __shared__ __attribute__((aligned(16))) char ldsA[STAGE];
    __shared__ __attribute__((aligned(16))) char ldsB[STAGE];
    __shared__ __attribute__((aligned(16))) char ldsC[STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = p.T, D = p.D;
    const int nq = (T + 127) / 128, total = (int) gridDim.x;
    const int L = (int) blockIdx.x;
    const int w = (total & 7) ? L : (L & 7) * (total >> 3) + (L >> 3);   // XCD-contiguous work order (k_attn)
    const int qt = w % nq, h = (w / nq) % p.H, clip = w / (nq * p.H);
    const int q0 = qt * 128 + wave * 32;
    const int64_t rowbase = (int64_t) clip * T;
    const int hi = lane >> 5, col = lane & 31;

    half8 qh[4], ql[4];
    {
        const int q = min(q0 + col, T - 1);
        const q2a_half * sh = p.qh + (rowbase + q) * D + h * 64 + 8 * hi;
        const q2a_half * sl = p.ql + (rowbase + q) * D + h * 64 + 8 * hi;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            qh[s] = *(const half8 *) (sh + 16 * s);
            ql[s] = *(const half8 *) (sl + 16 * s);
        }
    }
    const char * khb = (const char *) (p.kh + rowbase * D + h * 64);
    const char * klb = (const char *) (p.kl + rowbase * D + h * 64);
    const char * vtb = (const char *) (p.vt + ((int64_t) clip * p.H + h) * 64 * p.TP);
    const int krow_d = 8 * wave + (lane >> 3), kg = (lane & 7) ^ ((krow_d >> 1) & 7);
    const int vrow_d = 16 * wave + (lane >> 2), vg = (lane & 3) ^ ((vrow_d >> 2) & 3);
    auto dma_tile = [&](char * st, int t) {
        const int key = min(t * KT32 + krow_d, T - 1);
        const uint32_t ko = (uint32_t) (key * D + kg * 8) * 2u;
        const uint32_t vo = (uint32_t) (vrow_d * p.TP + t * KT32 + vg * 8) * 2u;
        __builtin_amdgcn_global_load_lds((const void *) (khb + ko), (lds_ptr_t) (st + wave * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *) (klb + ko), (lds_ptr_t) (st + KIMG + wave * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *) (vtb + vo), (lds_ptr_t) (st + 2 * KIMG + wave * 1024), 16, 0, 0);
    };

    f16v o[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    float m_run = -1e30f, l_run = 0.f;
    const int ntiles = (T + KT32 - 1) / KT32;
    const int krow = kperm(col);

    auto qk = [&](const char * kh_img) {
        const char * kl_img = kh_img + KIMG;
        f16v s;
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const int off = krow * KROW + attn_lds_g::k(krow, 2 * st + hi);
            const half8 ah = *(const half8 *) (kh_img + off);
            s = mma32<false>(ah, qh[st], s);
            const half8 al = *(const half8 *) (kl_img + off);
            s = mma32<false>(al, qh[st], s);
            s = mma32<false>(ah, ql[st], s);
        }
        return s;
    };

    f16v sc;
    // iteration t: K of tile t+1 in sK, V^T of tile t in sV, tile t+2 DMA'd into sD
    auto iter = [&](const char * sK, const char * sV, char * sD, int t) {
        if (t + 2 < ntiles) dma_tile(sD, t + 2);
        if (t == ntiles - 1) {   // keys >= T exist only in the last tile (key of reg r: 16(r>>3) + 8hi + (r&7))
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (t * KT32 + 16 * (r >> 3) + 8 * hi + (r & 7) >= T) sc[r] = -1e30f;
        }
        // ---- one scheduling region: QK^T(t+1) MFMAs beside softmax(t) VALU
        const f16v sn = qk(sK);
        float mx = sc[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sc[r]);
        mx = max_lane32(mx);
        const float m_new = fmaxf(m_run, mx);
        const float nm = -m_new * L2E;
        const float alpha = __builtin_amdgcn_exp2f(fmaf(m_run, L2E, nm));
        float ls = 0.f;
        half8 pf[2];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float pv = __builtin_amdgcn_exp2f(fmaf(sc[r], L2E, nm));
            ls += pv;
            pf[r >> 3][r & 7] = (_Float16) pv;
        }
        l_run = l_run * alpha + ls;
        m_run = m_new;
        // P complete before the rescale branch below (otherwise the exp2 loop is sunk past it, out of the MFMAs' region)
        asm volatile("" :: "v"(pf[0]), "v"(pf[1]), "v"(l_run));
#if Q2A_ATTN_P32_SCHED
        // 8 K-fragment reads first, then 12 x {1 MFMA, 6 VALU}
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
        }
#endif
        if (__any(alpha != 1.0f)) {
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
        }
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
            const int vr = dt * 32 + col;
#pragma unroll
            for (int sp = 0; sp < 2; ++sp) {   // keys 16sp + 8hi .. +7: one 16-B granule of the V^T row
                const half8 va = *(const half8 *) (sV + 2 * KIMG + vr * VROW + (((2 * sp + hi) ^ ((vr >> 2) & 3)) << 4));
                o[dt] = mma32<false>(va, pf[sp], o[dt]);
            }
        }
        sc = sn;
        __syncthreads();   // tile t+2 landed (vmcnt(0) in the barrier); every wave done with tile t's stage
    };

    dma_tile(ldsA, 0);
    if (ntiles > 1) dma_tile(ldsB, 1);
    asm volatile("" :: "v"(qh[0]), "v"(qh[1]), "v"(qh[2]), "v"(qh[3]), "v"(ql[0]), "v"(ql[1]), "v"(ql[2]), "v"(ql[3]));
    __syncthreads();
    sc = qk(ldsA);
    for (int t = 0; t < ntiles; t += 3) {
        iter(ldsB, ldsA, ldsC, t);
        if (t + 1 >= ntiles) break;
        iter(ldsC, ldsB, ldsA, t + 1);
        if (t + 2 >= ntiles) break;
        iter(ldsA, ldsC, ldsB, t + 2);
    }

    float l_tot;
    {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_run), __float_as_uint(l_run), false, false);
        l_tot = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    const float inv = 1.0f / l_tot;
    const int q = q0 + col;
    if (q < T) {
        const int64_t orow = (rowbase + q) * D + h * 64;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = dt * 32 + 8 * g + 4 * hi;
                const float v0 = o[dt][4 * g + 0] * inv, v1 = o[dt][4 * g + 1] * inv;
                const float v2 = o[dt][4 * g + 2] * inv, v3 = o[dt][4 * g + 3] * inv;
                if (p.outH) {
                    const half4 hv = {(_Float16) v0, (_Float16) v1, (_Float16) v2, (_Float16) v3};
                    *(half4 *) (p.outH + orow + d) = hv;
                } else {
                    *(float4 *) (p.outF + orow + d) = make_float4(v0, v1, v2, v3);
                }
            }
    }
}

// ---- F32-class ping-pong on 32-key tiles (k_attn_pp32). The timing decomposition of k_attn_g (profiles/
// r02q_attention_sq.json) shows the online-softmax VALU adding its full time to the MFMA time: within one wave they
// are dependent, and the co-resident waves of other workgroups do not fill the gaps. Here one 512-thread workgroup =
// 8 waves x 32 queries (256 queries of one (clip, head)); waves w and w + 4 share a SIMD and run the same loop one
// segment apart (group B starts after one extra barrier), so in every segment one of them issues MFMAs
// (P.V of tile t-1 + QK^T of tile t: 16 MFMAs) while the other runs the softmax of its tile. k_attn_g32's per-32-key
// arithmetic (same MFMA order, same exp2 / fp16 P, max, row sums), so the output equals k_attn_g32's bit for bit.
// The 32-key tiles keep 16 score registers live: <= 128 VGPRs, two workgroups (16 waves) per CU. Three LDS stages of
// 12 KiB (36 KiB per workgroup): group A DMAs tile t+1 at the start of its MFMA segment t and waits for it before
// the barrier that ends its softmax segment t, two segments later. LDS reads use integer LDS addresses (the compiler
// would otherwise guard them with vmcnt(0) against the DMA in flight), barriers are raw s_barrier.
#ifndef Q2A_ATTN_PP32_PRIO
#define Q2A_ATTN_PP32_PRIO 1   // static s_setprio 1 for group B (MI355X_MICROARCH.md, two waves per SIMD, item 4)
#endif
__global__ __launch_bounds__(512, 2) void k_attn_pp32(const q2a_attn_args p) {
    constexpr int KROW = 128, VROW = 64;
    constexpr int KIMG = KT32 * KROW, VIMG = 64 * VROW, STAGE = 2 * KIMG + VIMG;
    __shared__ __attribute__((aligned(16))) char lds[3 * STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, gw = wave & 3;
    const int T = p.T, D = p.D;
    const int nq = (T + 255) / 256, total = (int) gridDim.x;
    const int L = (int) blockIdx.x;
    const int w = (total & 7) ? L : (L & 7) * (total >> 3) + (L >> 3);   // XCD-contiguous work order (k_attn)
    const int qt = w % nq, h = (w / nq) % p.H, clip = w / (nq * p.H);
    const int q0 = qt * 256 + wave * 32;
    const int64_t rowbase = (int64_t) clip * T;
    const int hi = lane >> 5, col = lane & 31;

    half8 qh[4], ql[4];
    {
        const int q = min(q0 + col, T - 1);
        const q2a_half * sh = p.qh + (rowbase + q) * D + h * 64 + 8 * hi;
        const q2a_half * sl = p.ql + (rowbase + q) * D + h * 64 + 8 * hi;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            qh[s] = *(const half8 *) (sh + 16 * s);
            ql[s] = *(const half8 *) (sl + 16 * s);
        }
    }
    const char * khb = (const char *) (p.kh + rowbase * D + h * 64);
    const char * klb = (const char *) (p.kl + rowbase * D + h * 64);
    const char * vtb = (const char *) (p.vt + ((int64_t) clip * p.H + h) * 64 * p.TP);
    // group A's wave gw DMAs rows 8gw .. +7 of the K hi / K lo images and rows 16gw .. +15 of the V^T image
    const int krow_d = 8 * gw + (lane >> 3), kg = (lane & 7) ^ ((krow_d >> 1) & 7);
    const int vrow_d = 16 * gw + (lane >> 2), vg = (lane & 3) ^ ((vrow_d >> 2) & 3);
    auto dma_tile = [&](int t) {
        char * st = lds + (t % 3) * STAGE;
        const int key = min(t * KT32 + krow_d, T - 1);
        const uint32_t ko = (uint32_t) (key * D + kg * 8) * 2u;
        const uint32_t vo = (uint32_t) (vrow_d * p.TP + t * KT32 + vg * 8) * 2u;
        __builtin_amdgcn_global_load_lds((const void *) (khb + ko), (lds_ptr_t) (st + gw * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *) (klb + ko), (lds_ptr_t) (st + KIMG + gw * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *) (vtb + vo), (lds_ptr_t) (st + 2 * KIMG + gw * 1024), 16, 0, 0);
    };
    typedef const __attribute__((address_space(3))) half8 * lds_h8p;
    const uint32_t lds0 = (uint32_t) (uintptr_t) (const __attribute__((address_space(3))) char *) lds;
    const int krow = kperm(col);

    f16v o[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    float m_run = -1e30f, l_run = 0.f;
    const int ntiles = (T + KT32 - 1) / KT32;
    f16v sc;
    half8 pf[2];

    auto barrier = [&]() {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    // MFMA segment t: P.V of tile t-1 (its V^T in stage (t-1)%3), QK^T of tile t (stage t%3)
    auto mfma_seg = [&](int t) {
        if (t >= 1) {
            const uint32_t sv = lds0 + ((t - 1) % 3) * STAGE + 2 * KIMG;
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
                const int vr = dt * 32 + col;
#pragma unroll
                for (int sp = 0; sp < 2; ++sp) {
                    const half8 va = *(lds_h8p) (uintptr_t) (sv + vr * VROW + (((2 * sp + hi) ^ ((vr >> 2) & 3)) << 4));
                    o[dt] = mma32<false>(va, pf[sp], o[dt]);
                }
            }
        }
        if (t < ntiles) {
            const uint32_t sk = lds0 + (t % 3) * STAGE;
#pragma unroll
            for (int r = 0; r < 16; ++r) sc[r] = 0.f;
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const uint32_t off = (uint32_t) (krow * KROW + attn_lds_g::k(krow, 2 * st + hi));
                const half8 ah = *(lds_h8p) (uintptr_t) (sk + off);
                sc = mma32<false>(ah, qh[st], sc);
                const half8 al = *(lds_h8p) (uintptr_t) (sk + KIMG + off);
                sc = mma32<false>(al, qh[st], sc);
                sc = mma32<false>(ah, ql[st], sc);
            }
        }
    };
    // VALU segment t: online-softmax update of tile t's scores (k_attn_g32's operations), P into pf
    auto valu_seg = [&](int t) {
        if (t == ntiles - 1) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (t * KT32 + 16 * (r >> 3) + 8 * hi + (r & 7) >= T) sc[r] = -1e30f;
        }
        float mx = sc[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sc[r]);
        mx = max_lane32(mx);
        const float m_new = fmaxf(m_run, mx);
        const float nm = -m_new * L2E;
        const float alpha = __builtin_amdgcn_exp2f(fmaf(m_run, L2E, nm));
        float ls = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float pv = __builtin_amdgcn_exp2f(fmaf(sc[r], L2E, nm));
            ls += pv;
            pf[r >> 3][r & 7] = (_Float16) pv;
        }
        l_run = l_run * alpha + ls;
        m_run = m_new;
        if (__any(alpha != 1.0f)) {
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
        }
    };

    if (grp == 0) dma_tile(0);
    asm volatile("" :: "v"(qh[0]), "v"(qh[1]), "v"(qh[2]), "v"(qh[3]), "v"(ql[0]), "v"(ql[1]), "v"(ql[2]), "v"(ql[3]));
    __syncthreads();
    if (Q2A_ATTN_PP32_PRIO && grp == 1) __builtin_amdgcn_s_setprio(1);
    if (grp == 1) barrier();   // group B runs one segment behind
    for (int t = 0; t <= ntiles; ++t) {
        if (grp == 0 && t + 1 < ntiles) dma_tile(t + 1);   // stage (t+1)%3: its last reader (B's P.V of t-2) is done
        mfma_seg(t);
        barrier();
        if (t < ntiles) valu_seg(t);
        if (grp == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tile t+1 landed before the next barrier
        barrier();
    }
    if (grp == 0) barrier();
    if (Q2A_ATTN_PP32_PRIO && grp == 1) __builtin_amdgcn_s_setprio(0);

    float l_tot;
    {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_run), __float_as_uint(l_run), false, false);
        l_tot = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    const float inv = 1.0f / l_tot;
    const int q = q0 + col;
    if (q < T) {
        const int64_t orow = (rowbase + q) * D + h * 64;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = dt * 32 + 8 * g + 4 * hi;
                const float v0 = o[dt][4 * g + 0] * inv, v1 = o[dt][4 * g + 1] * inv;
                const float v2 = o[dt][4 * g + 2] * inv, v3 = o[dt][4 * g + 3] * inv;
                if (p.outH) {
                    const half4 hv = {(_Float16) v0, (_Float16) v1, (_Float16) v2, (_Float16) v3};
                    *(half4 *) (p.outH + orow + d) = hv;
                } else {
                    *(float4 *) (p.outF + orow + d) = make_float4(v0, v1, v2, v3);
                }
            }
    }
}

// ---- ping-pong variant (default): one 512-thread workgroup = 8 waves x 32 queries (256 queries of one (clip, head)),
// the two waves that share a SIMD (w and w + 4) run the same loop one segment apart: while group A (waves 0-3) is in
// its MFMA segment (P.V of the previous tile + QK^T of this one, 32 MFMAs) group B (waves 4-7) is in its VALU segment
// (the online-softmax update of its scores), and the other way round after the next workgroup barrier — the matrix
// pipe and the VALU of each SIMD busy at once (MI355X_MICROARCH.md "Two waves per SIMD"). K/V tiles of 64 keys in
// three LDS stages: tile t is read from segment 2t (A's QK^T) to 2t+3 (B's P.V); tile t+3 is written into tile t's
// stage by A in its VALU segment 2t+5 and by B in its VALU segment 2t+4 (one half each), from registers loaded two
// segments earlier. Per element the arithmetic of k_attn: S = Kh.Qh + Kl.Qh + Kh.Ql in the same MFMA order, one
// online-softmax update per 64 keys, P and V fp16 (bf16 in the bf16-activation mode) into the P.V MFMA.
template <bool BF>
__global__ __launch_bounds__(512, 2) void k_attn_pp(const q2a_attn_args p) {
    typedef attn_lds<false> LY;
    // V^T rows padded to 144 B like K's (16-B granules in order: conflict-free for the 16-lane groups of a b128 read,
    // one base register + immediates; an XOR swizzle needs an address register per granule and costs the 4th wave)
    // so the 8 keys of a P.V B fragment (K rows permuted by kperm, as in k_attn_g) are ONE ds_read_b128
    constexpr int KROW = LY::KROW, VROW = LY::KROW;
    constexpr int KIMG = KT * KROW, VIMG = 64 * VROW;
    constexpr int NK = BF ? 1 : 2;                 // K images per stage (hi, lo)
    constexpr int STAGE = NK * KIMG + VIMG;
    constexpr int NST = 3;
    constexpr int CH = (NK + 1) * 512;             // 16-B chunks per tile: K images then V^T
    constexpr int CPT = CH / 512;                  // chunks per thread of one group's half tile (CH / 2 / 256)
    __shared__ __attribute__((aligned(16))) char lds[NST * STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = wave >> 2, gt = tid & 255;     // group A (0) / B (1), thread index within the group
    const int T = p.T, D = p.D;
    const int nq = (T + 255) / 256, total = (int) gridDim.x;
    const int L = (int) blockIdx.x;
    const int w = (total & 7) ? L : (L & 7) * (total >> 3) + (L >> 3);
    const int qt = w % nq, h = (w / nq) % p.H, clip = w / (nq * p.H);
    const int q0 = qt * 256 + wave * 32;
    const int64_t rowbase = (int64_t) clip * T;
    const int hi = lane >> 5, col = lane & 31;

    half8 qh[4], ql[4];
    {
        const int q = min(q0 + col, T - 1);
        const q2a_half * sh = p.qh + (rowbase + q) * D + h * 64 + 8 * hi;
        const q2a_half * sl = p.ql + (rowbase + q) * D + h * 64 + 8 * hi;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            qh[s] = *(const half8 *) (sh + 16 * s);
            ql[s] = BF ? qh[s] : *(const half8 *) (sl + 16 * s);
        }
    }
    const q2a_half * vt_base = p.vt + ((int64_t) clip * p.H + h) * 64 * p.TP;
    // staging: this group's half of a tile, CPT 16-B chunks per thread. Chunk c of the tile (0 .. CH-1): image
    // c / 512 (Kh, [Kl,] V^T), row (c % 512) / 8, 16-B piece c % 8.
    uint4 rg[CPT];
    auto chunk_of = [&](int u) __attribute__((always_inline)) { return grp * (CH / 2) + u * 256 + gt; };
    auto load_half = [&](int t) __attribute__((always_inline)) {
        const int kb0 = t * KT;
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            const int c = chunk_of(u), img = c >> 9, r = (c >> 3) & 63, pc = c & 7;
            if (img < NK) {
                const q2a_half * src = img == 0 ? p.kh : p.kl;
                rg[u] = *(const uint4 *) (src + (rowbase + min(kb0 + r, T - 1)) * D + h * 64 + pc * 8);
            } else {
                rg[u] = *(const uint4 *) (vt_base + (int64_t) r * p.TP + kb0 + pc * 8);
            }
        }
    };
    auto store_half = [&](int t) __attribute__((always_inline)) {
        char * st = lds + (t % NST) * STAGE;
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            const int c = chunk_of(u), img = c >> 9, r = (c >> 3) & 63, pc = c & 7;
            if (img < NK) {
                *(uint4 *) (st + img * KIMG + r * KROW + LY::k(r, pc)) = rg[u];
            } else {
                // (two 8-B stores: written as one uint4 here the compiler merges both branches and moves rg to scratch)
                char * vr = st + NK * KIMG + r * VROW + pc * 16;
                *(uint2 *) vr = make_uint2(rg[u].x, rg[u].y);
                *(uint2 *) (vr + 8) = make_uint2(rg[u].z, rg[u].w);
            }
        }
    };
    auto barrier = [&]() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // LDS writes done; global prefetch stays in flight
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    f16v o[2], sc[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    float m_run = -1e30f, l_run = 0.f, alpha = 1.f;
    half8 pf[2][2];

    // MFMA segment M(t): P.V(t-1) (t > 0) then S^T = K_t . Q^T
    auto mfma_seg = [&](int t, int ntiles) __attribute__((always_inline)) {
        if (t > 0) {
            if (__any(alpha != 1.0f)) {
#pragma unroll
                for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
            }
            const char * vt_img = lds + ((t - 1) % NST) * STAGE + NK * KIMG;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int dt = 0; dt < 2; ++dt) {
                    const int vr = dt * 32 + col;
#pragma unroll
                    for (int sp = 0; sp < 2; ++sp) {   // keys 32kb + 16sp + 8hi .. +7
                        const half8 va = *(const half8 *) (vt_img + vr * VROW + (4 * kb + 2 * sp + hi) * 16);
                        o[dt] = mma32<BF>(va, pf[kb][sp], o[dt]);
                    }
                }
        }
        if (t < ntiles) {
            const char * kh_img = lds + (t % NST) * STAGE;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                const int krow = kb * 32 + kperm(col);
#pragma unroll
                for (int r = 0; r < 16; ++r) sc[kb][r] = 0.f;
#pragma unroll
                for (int st = 0; st < 4; ++st) {
                    const int off = krow * KROW + LY::k(krow, 2 * st + hi);
                    const half8 ah = *(const half8 *) (kh_img + off);
                    sc[kb] = mma32<BF>(ah, qh[st], sc[kb]);
                    if (!BF) {
                        const half8 al = *(const half8 *) (kh_img + KIMG + off);
                        sc[kb] = mma32<BF>(al, qh[st], sc[kb]);
                        sc[kb] = mma32<BF>(ah, ql[st], sc[kb]);
                    }
                }
            }
        }
    };
    // VALU segment V(t): online-softmax update of tile t's scores -> pf, alpha (applied at the next P.V)
    auto valu_seg = [&](int t, int ntiles) __attribute__((always_inline)) {
        if (t == ntiles - 1) {   // keys >= T exist only in the last tile (key of reg r: 16(r>>3) + 8hi + (r&7))
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (t * KT + kb * 32 + 16 * (r >> 3) + 8 * hi + (r & 7) >= T) sc[kb][r] = -1e30f;
        }
        float mx0 = sc[0][0], mx1 = sc[1][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) { mx0 = fmaxf(mx0, sc[0][r]); mx1 = fmaxf(mx1, sc[1][r]); }
        float mx = fmaxf(mx0, mx1);
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float m_new = fmaxf(m_run, mx);
        const float nm = -m_new * L2E;
        alpha = __builtin_amdgcn_exp2f(fmaf(m_run, L2E, nm));
        float ls0 = 0.f, ls1 = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float pv = __builtin_amdgcn_exp2f(fmaf(sc[kb][r], L2E, nm));
                if (r & 1) ls1 += pv; else ls0 += pv;
                pf[kb][r >> 3][r & 7] = to16<BF>(pv);
            }
        l_run = l_run * alpha + (ls0 + ls1);
        m_run = m_new;
    };

    const int ntiles = (T + KT - 1) / KT;
    // prologue: tiles 0, 1, 2 into the three stages, every thread a share of each
    {
        // prologue staging by every thread: tile t's 2 halves = all CH chunks, 512 threads
#pragma unroll
        for (int t = 0; t < NST; ++t) {
            if (t >= ntiles) break;
            const int kb0 = t * KT;
            char * st = lds + t * STAGE;
#pragma unroll
            for (int u = 0; u < CH / 512; ++u) {
                const int c = u * 512 + tid, img = c >> 9, r = (c >> 3) & 63, pc = c & 7;
                if (img < NK) {
                    const q2a_half * src = img == 0 ? p.kh : p.kl;
                    *(uint4 *) (st + img * KIMG + r * KROW + LY::k(r, pc)) =
                        *(const uint4 *) (src + (rowbase + min(kb0 + r, T - 1)) * D + h * 64 + pc * 8);
                } else {
                    *(uint4 *) (st + NK * KIMG + r * VROW + pc * 16) =
                        *(const uint4 *) (vt_base + (int64_t) r * p.TP + kb0 + pc * 8);
                }
            }
        }
    }
    asm volatile("" :: "v"(qh[0]), "v"(qh[1]), "v"(qh[2]), "v"(qh[3]), "v"(ql[0]), "v"(ql[1]), "v"(ql[2]), "v"(ql[3]));
    __syncthreads();
    // group B starts one segment late; A ends with one extra barrier: every wave passes 2 * ntiles + 1 barriers
    if (grp == 0 && ntiles > 3) load_half(3);   // A stores its half of tile 3 in V(2)
    if (grp == 1) {
        if (ntiles > 3) load_half(3);           // B stores its half of tile 3 in V(1)
        barrier();
    }
    for (int t = 0; t < ntiles; ++t) {
        mfma_seg(t, ntiles);
        barrier();
        valu_seg(t, ntiles);
        // staging: tile t+1 (A) / t+2 (B) goes into the stage of tile t-2 / t-1, whose last reader (B's P.V) has
        // passed the previous barrier; then the registers load the group's half of the next tile it will store
        const int ts = grp == 0 ? t + 1 : t + 2;
        if (t >= (grp == 0 ? 2 : 1) && ts < ntiles && ts >= NST) {
            store_half(ts);
            if (ts + 1 < ntiles) load_half(ts + 1);
        }
        barrier();
    }
    mfma_seg(ntiles, ntiles);   // the last P.V
    if (grp == 0) barrier();

    const float l_tot = l_run + __shfl_xor(l_run, 32);
    const float inv = 1.0f / l_tot;
    const int q = q0 + col;
    if (q < T) {
        const int64_t orow = (rowbase + q) * D + h * 64;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = dt * 32 + 8 * g + 4 * hi;
                const float v0 = o[dt][4 * g + 0] * inv, v1 = o[dt][4 * g + 1] * inv;
                const float v2 = o[dt][4 * g + 2] * inv, v3 = o[dt][4 * g + 3] * inv;
                if (p.outH) {
                    const half4 hv = {to16<BF>(v0), to16<BF>(v1), to16<BF>(v2), to16<BF>(v3)};
                    *(half4 *) (p.outH + orow + d) = hv;
                } else {
                    *(float4 *) (p.outF + orow + d) = make_float4(v0, v1, v2, v3);
                }
            }
    }
}

}  // namespace

hipError_t q2a_launch_attention(const q2a_attn_args & a, hipStream_t s) {
    if (a.D != a.H * 64 || a.TP < ((a.T + KT - 1) / KT) * KT) return hipErrorInvalidValue;
    dim3 grid(((a.T + 127) / 128) * a.H * a.n_clips);
    // bf16 contract: the 8-wave ping-pong kernel (measured 33 -> 30 ms/step at 64 clips; Q2A_ATTN_V1=1 for the 4-wave
    // one). F32-class contract: the 4-wave kernel — the ping-pong form of its 3-term QK^T ran slower (61 vs 49 ms/step:
    // one 81 KiB workgroup per CU, barrier waits 46 % of wave cycles; Q2A_ATTN_PP=1 runs it, A/B only)
    static const bool v1 = [] { const char * v = getenv("Q2A_ATTN_V1"); return v && atoi(v); }();
    static const bool pp32 = [] { const char * v = getenv("Q2A_ATTN_PP"); return v && atoi(v); }();
    static const int terms = [] { const char * v = getenv("Q2A_ATTN_TERMS"); return v ? atoi(v) : 3; }();
    if (!v1 && (a.bf16 || (pp32 && terms == 3))) {
        const dim3 grid2(((a.T + 255) / 256) * a.H * a.n_clips);
        if (a.bf16) {
            if (!a.outH) return hipErrorInvalidValue;
            hipLaunchKernelGGL(k_attn_pp<true>, grid2, dim3(512), 0, s, a);
        } else {
            hipLaunchKernelGGL(k_attn_pp<false>, grid2, dim3(512), 0, s, a);
        }
        return hipGetLastError();
    }
    if (a.bf16) {
        if (!a.outH) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_attn<true>, grid, dim3(256), 0, s, a);
    } else {
        // F32-class default: k_attn_g (K/V by LDS-DMA, three workgroups per CU: 52 -> 49 ms/step at 64 clips);
        // Q2A_ATTN_G=0 runs the register-staged k_attn (A/B)
        static const bool g = [] { const char * v = getenv("Q2A_ATTN_G"); return !v || atoi(v); }();
        static const bool g32 = [] { const char * v = getenv("Q2A_ATTN_G32"); return v && atoi(v); }();
        static const bool p32 = [] { const char * v = getenv("Q2A_ATTN_P32"); return v && atoi(v); }();
        static const bool ppk32 = [] { const char * v = getenv("Q2A_ATTN_PP32"); return v && atoi(v); }();
        if (g && ppk32 && terms == 3) {
            hipLaunchKernelGGL(k_attn_pp32, dim3(((a.T + 255) / 256) * a.H * a.n_clips), dim3(512), 0, s, a);
            return hipGetLastError();
        }
        if (g && p32 && terms == 3) hipLaunchKernelGGL(k_attn_p32, grid, dim3(256), 0, s, a);
        else if (g && g32 && terms == 3) hipLaunchKernelGGL(k_attn_g32, grid, dim3(256), 0, s, a);
        else if (g && terms == 3) hipLaunchKernelGGL(k_attn_g, grid, dim3(256), 0, s, a);
        else if (terms == 2) hipLaunchKernelGGL((k_attn<false, 2>), grid, dim3(256), 0, s, a);
        else if (terms == 1) hipLaunchKernelGGL((k_attn<false, 1>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL(k_attn<false>, grid, dim3(256), 0, s, a);
    }
    return hipGetLastError();
}
