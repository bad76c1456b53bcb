// q2a_attn.hip — fused multi-head self-attention for gfx950 (flash-style, no T x T score tensor in HBM).
//
// Replaces, per layer (qwen2-whisper.cpp:2052-2107): KQ = mul_mat(K, Q) (F32, ggml.c:12439), SOFT_MAX
// (ggml.c:13854-13950, scale 1, no mask), KQV = mul_mat(cont(V^T), KQ_soft_max), the permutes and the merge.
// The reference materialises 20 x 1500 x 1500 F32 scores per layer (180 MB per clip).
//
// Numerics (reference contract): the reference computes QK^T, the softmax and P.V all in F32. Here Q and K arrive as
// fp16 hi/lo pairs (x = hi + lo, 22 significant bits) and S = Kh.Qh + Kl.Qh + Kh.Ql on fp16 MFMA with fp32
// accumulation (the lo.lo term is below 2^-22 relative), i.e. F32-class scores. The P.V product's precision is set
// by Q2A_ATTN_PHL / Q2A_ATTN_VHL below (hi/lo fp16 splits of P and of V: F32-class when both are on). Online softmax
// keeps a running max/sum per query; the 1/sum normalisation is applied once at the end.
//
// Kernels (the schedules measured and not adopted live in diag/attn_variants.hip, built only into diag libraries):
//   k_attn_g       reference contract: one 256-thread workgroup = 4 waves x 32 queries of one (clip, head), K/V tiles
//                  of 64 keys by LDS-DMA into two LDS stages
//   k_attn_pp<BF>  bf16-activation contract (BF = true): 8-wave ping-pong, one 512-thread workgroup = 256 queries
// S^T = K.Q^T is computed with v_mfma_f32_32x32x16_f16 so each lane owns one query column (softmax is lane-local plus
// one lane^32 exchange) and the S accumulator feeds the P.V MFMA as its B operand with no data movement
// (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand").
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
// padded LDS rows (k_attn_pp): K rows 144 B, V^T rows 136 B — conflict-free ds_read_b128 (16-lane groups of distinct
// rows) without per-granule address registers; swizzled unpadded 128-B rows (diag variants)
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

// ---- reference-contract kernel. The next tile's K hi, K lo and V^T (hi, lo) arrive by global_load_lds straight into
// the other of two LDS stages (two __shared__ arrays, the loop unrolled by two, so the compiler sees no alias between
// the stage it reads and the one in flight) instead of through staging VGPRs. LDS images unpadded, 16-B granules
// XOR-swizzled by row (K: chunk ch of row r at ch ^ ((r >> 1) & 7); V^T: granule g at g ^ ((r >> 1) & 7), its two 8-B
// halves in order — the DMA moves whole granules, with the swizzle on the source address).
struct attn_lds_g {
    static constexpr int KROW = 128, VROW = 128;
    static __device__ __forceinline__ int k(int r, int ch) { return (ch ^ ((r >> 1) & 7)) << 4; }
    static __device__ __forceinline__ int vg(int r, int g) { return (g ^ ((r >> 1) & 7)) << 4; }
};
// K row loaded into row i of the QK^T A operand: i with bits 2 and 3 swapped. S^T's accumulator row for register r
// of lane half hi is (r&3) + 8(r>>2) + 4hi, so register r then holds key 16(r>>3) + 8hi + (r&7): the 8 keys a lane
// half feeds the P.V MFMA as one B fragment are contiguous, and their V^T operand is ONE 16-B LDS read instead of
// two 8-B reads and a register shuffle (softmax is order-free over the keys of a tile)
__device__ __forceinline__ int kperm(int c) { return (c & ~12) | ((c & 4) << 1) | ((c & 8) >> 1); }
// max of x over lanes l and l ^ 32: v_permlane32_swap exchanges the two wave halves in a VALU slot (no LDS round
// trip as ds_bpermute, no lgkmcnt wait); one of the two results is the lane's own value
__device__ __forceinline__ float max_lane32(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// P.V precision of k_attn_g (reference: F32 P and V, qwen2-whisper.cpp:2088-2102):
//   Q2A_ATTN_PHL = 1: P = Ph + Pl, two fp16 halves (Ph = P truncated to fp16, Pl = the exact f32 remainder truncated
//                     to fp16: 22 significant bits), two P.V MFMAs per fragment
//   Q2A_ATTN_VHL = 1: V^T = Vh + Vl likewise (the QKV epilogue writes the lo image), one more MFMA per fragment
//                     (Vl.Ph; the Vl.Pl term is below 2^-22 relative) and a fourth LDS image per stage (two
//                     workgroups per CU instead of three)
// With PHL = 0 P is ONE fp16 value (truncated) and the softmax denominator is the sum of exactly those fp16 values
// (v_dot2 of the packed pairs against 1.0): the output is an exact weighted mean of V with the fp16 weights, so P's
// rounding does not bias the normalisation. With PHL = 1 the denominator is the f32 sum of P.
#ifndef Q2A_ATTN_PHL
#define Q2A_ATTN_PHL 1
#endif
#ifndef Q2A_ATTN_VHL
#define Q2A_ATTN_VHL 1
#endif
// QK^T terms of k_attn_g (diagnostic builds only): 3 = Kh.Qh + Kl.Qh + Kh.Ql (the contract); 21 = without Kl.Qh (K as
// fp16); 22 = without Kh.Ql (Q as fp16)
#ifndef Q2A_ATTN_QK_TERMS
#define Q2A_ATTN_QK_TERMS 3
#endif
// lazy re-basing threshold of the softmax reference point (k_attn_g): a lane re-bases when the 32 P of its tile sum to
// more than this (so each P <= 2^15 < 65504, inside fp16, between moves)
constexpr float PLIM = 32768.0f;
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ half2_t pk_rtz(float a, float b) {
    return __builtin_bit_cast(half2_t, __builtin_amdgcn_cvt_pkrtz(a, b));
}
// p - fp16 element (lo or hi half of h) in ONE v_fma_mix_f32 (the fp16 operand read in place, the product by -1 exact,
// one rounding of an exactly representable difference): hipcc otherwise emits a v_cvt_f32_f16 and a v_sub_f32
template <int HI>
__device__ __forceinline__ float sub_half(float p, half2_t h) {
    float r;
    if constexpr (HI) asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(p));
    else asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(p));
    return r;
}
// LDS: VHL = 0: two stages of K hi | K lo | V^T (24 KiB each), one barrier per tile. VHL = 1: two stages of K hi | K lo
// (16 KiB each) and ONE V^T hi | lo stage (16 KiB): 48 KiB, three workgroups per CU (a second V stage would make it
// 64 KiB and two per CU). Tile t's V^T is DMA'd at the start of its iteration beside K(t+1), lands under QK^T(t) and
// the softmax, and a second barrier per tile separates the P.V reads from the next overwrite.
#ifndef Q2A_ATTN_VDB
#define Q2A_ATTN_VDB 0     // 1: V^T hi | lo double-buffered beside K (64 KiB, one barrier per tile; diagnostic builds)
#endif
#ifndef Q2A_ATTN_G_OCC
#define Q2A_ATTN_G_OCC (Q2A_ATTN_VDB ? 2 : 3)   // workgroups per CU the register budget is sized for
#endif
__global__ __launch_bounds__(256, Q2A_ATTN_G_OCC) void k_attn_g(const q2a_attn_args p) {
    typedef attn_lds_g LY;
    constexpr bool VHL = Q2A_ATTN_VHL, PHL = Q2A_ATTN_PHL, VDB = VHL && Q2A_ATTN_VDB;
    constexpr int KROW = LY::KROW, VROW = LY::VROW;
    constexpr int KIMG = KT * KROW, VIMG = 64 * VROW, STAGE = 2 * KIMG + (VHL ? (VDB ? 2 * VIMG : 0) : VIMG);
    __shared__ __attribute__((aligned(16))) char ldsA[STAGE];
    __shared__ __attribute__((aligned(16))) char ldsB[STAGE];
    __shared__ __attribute__((aligned(16))) char ldsV[VHL && !VDB ? 2 * VIMG : 16];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = p.T, D = p.D;
    const int nq = (T + 127) / 128, total = (int) gridDim.x;
    const int L = (int) blockIdx.x;
    // XCD-contiguous work order: workgroup L is dispatched to XCD L % 8, so work item w = (L % 8)·(total/8) + L/8
    // puts the q-tiles of one (clip, head) on ONE XCD at about the same time and its K/V are fetched into that
    // L2 once instead of into up to eight of them (bijective when total % 8 == 0, identity otherwise)
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
            ql[s] = *(const half8 *) (sl + 16 * s);
        }
    }
    // tile t -> stage: wave w's instruction i covers rows (2w + i) * 8 .. +7 of each image (1 KiB), lane l row
    // + l / 8, LDS granule l % 8 <- source granule (l % 8) ^ ((row >> 1) & 7)
    // sources as a uniform (clip, head) base + a 32-bit per-lane byte offset (the saddr form of the DMA: no 64-bit
    // address arithmetic per tile; a clip's K rows span T·D·2 B, its head's V^T 64·TP·2 B)
    const int64_t vt_off = ((int64_t) clip * p.H + h) * 64 * p.TP;
    const char * khb = (const char *) (p.kh + rowbase * D + h * 64);
    const char * klb = (const char *) (p.kl + rowbase * D + h * 64);
    const char * vtb = (const char *) (p.vt + vt_off);
    const char * vlb = VHL ? (const char *) (p.vtl + vt_off) : nullptr;
    // st: the K hi | K lo stage of tile t; vst: where its V^T (hi [| lo]) goes (st + 2 KIMG, or the V stage)
    auto dma_tile = [&](char * st, char * vst, int t, bool with_k, bool with_v) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int row = (2 * wave + i) * 8 + (lane >> 3), g = (lane & 7) ^ ((row >> 1) & 7);
            const int key = min(t * KT + row, T - 1);
            const uint32_t ko = (uint32_t) (key * D + g * 8) * 2u;
            const uint32_t vo = (uint32_t) (row * p.TP + t * KT + g * 8) * 2u;
            const int pc = (2 * wave + i) * 1024;
            if (with_k) {
                __builtin_amdgcn_global_load_lds((const void *) (khb + ko), (lds_ptr_t) (st + pc), 16, 0, 0);
                __builtin_amdgcn_global_load_lds((const void *) (klb + ko), (lds_ptr_t) (st + pc + KIMG), 16, 0, 0);
            }
            if (with_v) {
                __builtin_amdgcn_global_load_lds((const void *) (vtb + vo), (lds_ptr_t) (vst + pc), 16, 0, 0);
                if (VHL) __builtin_amdgcn_global_load_lds((const void *) (vlb + vo), (lds_ptr_t) (vst + pc + VIMG), 16, 0, 0);
            }
        }
    };

    f16v o[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    // Online softmax in log2 units: Q arrives pre-multiplied by log2(e) (the QKV epilogue folds it into the 1/8
    // scale), so S' = log2(e)·S and P = exp2(S' - m'). The reference point m' of the lane's query enters the QK^T
    // MFMAs as their initial accumulator (negm = -m' in all 16 C registers of each chain's first MFMA), so the
    // accumulators hold S' - m' and feed v_exp_f32 directly: no subtraction per score. m' is set on the first tile (its
    // max) and moves (lazily) only when a tile's P would leave the range the fp16 P halves hold: a lane whose 32 P of
    // the tile sum to more than PLIM (then every one of them is <= PLIM < 65504) re-bases to the tile's max, so the
    // common path needs no per-score max either.
    float m_run = 0.f, l_run = 0.f;
    f16v negm;
#pragma unroll
    for (int r = 0; r < 16; ++r) negm[r] = 0.f;
    const int ntiles = (T + KT - 1) / KT;

    // P of the current tile, packed two per register (truncated to fp16); PHL: plus the truncated remainders
    half2_t ph[2][8], pl[2][8];
    // per-lane LDS byte offsets of the fragment reads, computed once: K (key row kperm(col), chunk 2st+hi, swizzled) per
    // step st for the first 32-key half (the second is +32 rows = +4096, the lo image +KIMG, the stage a constant);
    // V^T (row col, granule 4kb+2sp+hi, swizzled) per (kb, sp) for d-block 0 (d-block 1 is +32 rows = +4096). Kept
    // opaque (asm) so the compiler folds the constants into the ds_read immediate instead of re-deriving the swizzle
    uint32_t kofs[4], vofs[2][2];
    {
        const int kr = kperm(col);
#pragma unroll
        for (int st = 0; st < 4; ++st) kofs[st] = (uint32_t) (kr * KROW + LY::k(kr, 2 * st + hi));
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int sp = 0; sp < 2; ++sp) vofs[kb][sp] = (uint32_t) (col * VROW + LY::vg(col, 4 * kb + 2 * sp + hi));
    }
    auto launder_ofs = [&]() {
        asm volatile("" : "+v"(kofs[0]), "+v"(kofs[1]), "+v"(kofs[2]), "+v"(kofs[3]), "+v"(vofs[0][0]), "+v"(vofs[0][1]),
                          "+v"(vofs[1][0]), "+v"(vofs[1][1]));
    };
    // QK^T + online softmax of tile t (K hi | K lo image at kh_img) -> ph / pl, l_run, m_run, rescaled O
    auto qk_softmax = [&](const char * kh_img, int t) {
        const char * kl_img = kh_img + KIMG;
        f16v sc[2];
        // S'^T - m' for both 32-key halves of the tile (24 MFMAs, the two chains interleaved per 16-deep step, each
        // starting from negm); the K fragments of step st+1 are read before the MFMAs of step st, so each MFMA group
        // waits only for its own reads
        auto qk = [&]() {
            half8 fh[2], fl[2];
            launder_ofs();
            auto rdk = [&](int st, int kb, half8 & hh, half8 & ll) {
                const uint32_t off = kofs[st] + kb * 32 * KROW;   // (krow >> 1) & 7 does not depend on kb
                hh = *(const half8 *) (kh_img + off);
                ll = *(const half8 *) (kl_img + off);
            };
            rdk(0, 0, fh[0], fl[0]);
            rdk(0, 1, fh[1], fl[1]);
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                half8 nh[2], nl[2];
                if (st < 3) { rdk(st + 1, 0, nh[0], nl[0]); rdk(st + 1, 1, nh[1], nl[1]); }
#pragma unroll
                for (int kb = 0; kb < 2; ++kb) {
                    sc[kb] = mma32<false>(fh[kb], qh[st], st == 0 ? negm : sc[kb]);
                    if (Q2A_ATTN_QK_TERMS != 21) sc[kb] = mma32<false>(fl[kb], qh[st], sc[kb]);
                    if (Q2A_ATTN_QK_TERMS != 22) sc[kb] = mma32<false>(fh[kb], ql[st], sc[kb]);
                }
                if (st < 3) { fh[0] = nh[0]; fh[1] = nh[1]; fl[0] = nl[0]; fl[1] = nl[1]; }
            }
            if (t == ntiles - 1) {   // keys >= T exist only in the last tile (key of reg r: 16(r>>3) + 8hi + (r&7))
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        if (t * KT + kb * 32 + 16 * (r >> 3) + 8 * hi + (r & 7) >= T) sc[kb][r] = -1e30f;
            }
        };
        // re-base to the tile's max (per query: both lane halves): on the first tile m' := that max (O and l are 0);
        // later only for queries whose max exceeds m' (alpha = 1 for the others)
        auto rebase = [&](bool first) {
            float mx = fmaxf(sc[0][0], sc[1][0]);
#pragma unroll
            for (int r = 1; r < 16; ++r) mx = fmaxf(mx, fmaxf(sc[0][r], sc[1][r]));   // (v_max3_f32; -fno-honor-nans)
            mx = max_lane32(mx);
            const float sh = first ? mx : fmaxf(mx, 0.f);
            if (!first) {
                const float alpha = __builtin_amdgcn_exp2f(-sh);
                l_run *= alpha;
#pragma unroll
                for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
            }
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int r = 0; r < 16; ++r) sc[kb][r] -= sh;
            m_run += sh;
#pragma unroll
            for (int r = 0; r < 16; ++r) negm[r] = -m_run;
        };
        // P = exp2(S' - m') in place of the scores, and the lane's f32 sum of them
        float ls = 0.f;
        auto exps = [&]() {
            ls = 0.f;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    sc[kb][r] = __builtin_amdgcn_exp2f(sc[kb][r]);
                    ls += sc[kb][r];
                }
        };
        qk();
        if (t == 0) rebase(true);
        exps();
        if (t != 0 && __any(ls > PLIM)) {   // rare: some P of the tile may not fit fp16; the scores again (the K stage
            qk();                           // is still in place), re-based, and their P
            rebase(false);
            exps();
        }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
                const float p0 = sc[kb][r], p1 = sc[kb][r + 1];
                const half2_t hp = pk_rtz(p0, p1);
                ph[kb][r >> 1] = hp;
                if (PHL) {   // exact remainders p - fp16(p) (one v_fma_mix each: the fp16 operand read in place)
                    pl[kb][r >> 1] = pk_rtz(sub_half<0>(p0, hp), sub_half<1>(p1, hp));
                }
            }
        if (!PHL) {   // the denominator of fp16 P: the sum of exactly those fp16 values
            ls = 0.f;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int r = 0; r < 8; ++r) ls = __builtin_amdgcn_fdot2(ph[kb][r], half2_t{(_Float16) 1.0f, (_Float16) 1.0f}, ls, false);
        }
        l_run += ls;
    };
    // O^T[d][q] += V^T[d][keys] . P^T[keys][q] for the tile whose V^T (hi [| lo]) image is at vt_img
    auto pv = [&](const char * vt_img) {
        launder_ofs();
        auto frag8 = [](const half2_t (&v)[8], int sp) {
            return half8{v[4 * sp][0], v[4 * sp][1], v[4 * sp + 1][0], v[4 * sp + 1][1],
                         v[4 * sp + 2][0], v[4 * sp + 2][1], v[4 * sp + 3][0], v[4 * sp + 3][1]};
        };
        // O^T[d][q] += V^T[d][keys] . P^T[keys][q] (small terms first)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
                const int vr = dt * 32 + col;
#pragma unroll
                for (int sp = 0; sp < 2; ++sp) {   // keys 32kb + 16sp + 8hi .. +7: one 16-B granule of the V^T row
                    const uint32_t vo = vofs[kb][sp] + dt * 32 * VROW;   // (vr >> 1) & 7 does not depend on dt
                    const half8 va = *(const half8 *) (vt_img + vo);
                    const half8 pb = frag8(ph[kb], sp);
                    if (VHL) o[dt] = mma32<false>(*(const half8 *) (vt_img + VIMG + vo), pb, o[dt]);
                    if (PHL) o[dt] = mma32<false>(va, frag8(pl[kb], sp), o[dt]);
                    o[dt] = mma32<false>(va, pb, o[dt]);
                }
            }
    };

    dma_tile(ldsA, ldsA + 2 * KIMG, 0, true, !VHL || VDB);
    // the Q fragments must be complete before the loop (an asm "use" makes the waitcnt pass wait for them here):
    // otherwise their loads stay pending at the loop header, merge with the next-tile prefetch and every
    // iteration's QK^T MFMAs wait on that prefetch
    asm volatile("" :: "v"(qh[0]), "v"(qh[1]), "v"(qh[2]), "v"(qh[3]), "v"(ql[0]), "v"(ql[1]), "v"(ql[2]), "v"(ql[3]));
    __syncthreads();   // (waits for the DMA: a pending LDS-DMA is a vmcnt event)
    if constexpr (VHL && !VDB) {
        // iteration t: V(t) -> V stage and K(t+1) -> the other K stage; QK^T(t) + softmax; barrier (V(t) landed);
        // P.V(t); barrier (every wave done with the V stage and K(t)'s stage)
        for (int t = 0; t < ntiles; t += 2) {
            dma_tile(ldsB, ldsV, t + 1, t + 1 < ntiles, false);
            dma_tile(ldsA, ldsV, t, false, true);
            qk_softmax(ldsA, t);
            __syncthreads();
            pv(ldsV);
            __syncthreads();
            if (t + 1 >= ntiles) break;
            dma_tile(ldsA, ldsV, t + 2, t + 2 < ntiles, false);
            dma_tile(ldsB, ldsV, t + 1, false, true);
            qk_softmax(ldsB, t + 1);
            __syncthreads();
            pv(ldsV);
            __syncthreads();
        }
    } else {
        for (int t = 0; t < ntiles; t += 2) {
            if (t + 1 < ntiles) dma_tile(ldsB, ldsB + 2 * KIMG, t + 1, true, true);
            qk_softmax(ldsA, t);
            pv(ldsA + 2 * KIMG);
            __syncthreads();   // tile t + 1 landed (vmcnt(0) in the barrier), every wave done with A
            if (t + 1 >= ntiles) break;
            if (t + 2 < ntiles) dma_tile(ldsA, ldsA + 2 * KIMG, t + 2, true, true);
            qk_softmax(ldsB, t + 1);
            pv(ldsB + 2 * KIMG);
            __syncthreads();
        }
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
    constexpr float QL2E = BF ? L2E : 1.0f;   // reference-contract Q arrives pre-multiplied by log2(e)
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
        const float nm = -m_new * QL2E;
        alpha = __builtin_amdgcn_exp2f(fmaf(m_run, QL2E, nm));
        float ls0 = 0.f, ls1 = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float pv = __builtin_amdgcn_exp2f(fmaf(sc[kb][r], QL2E, nm));
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

// the QKV epilogue must write the V^T lo image (q2a_attn_args.vtl) for this build's reference-contract kernel
bool q2a_attention_wants_vlo() { return Q2A_ATTN_VHL != 0; }

#ifndef Q2A_ATTN_LAUNCH
#define Q2A_ATTN_LAUNCH q2a_launch_attention
#endif
hipError_t Q2A_ATTN_LAUNCH(const q2a_attn_args & a, hipStream_t s) {
    if (a.D != a.H * 64 || a.TP < ((a.T + KT - 1) / KT) * KT) return hipErrorInvalidValue;
    if (a.bf16) {
        // bf16 contract: the 8-wave ping-pong kernel (33 -> 30 ms/step at 64 clips against the 4-wave form)
        if (!a.outH) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_attn_pp<true>, dim3(((a.T + 255) / 256) * a.H * a.n_clips), dim3(512), 0, s, a);
    } else {
        if (Q2A_ATTN_VHL && !a.vtl) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_attn_g, dim3(((a.T + 127) / 128) * a.H * a.n_clips), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}
