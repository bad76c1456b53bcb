// q2a_attn.hip — fused multi-head self-attention for gfx950 (flash-style, no T x T score tensor in HBM).
//
// Replaces, per layer (qwen2-whisper.cpp:2052-2107): KQ = mul_mat(K, Q) (F32, ggml.c:12439), SOFT_MAX
// (ggml.c:13854-13950, scale 1, no mask), KQV = mul_mat(cont(V^T), KQ_soft_max), the permutes and the merge.
// The reference materialises 20 x 1500 x 1500 F32 scores per layer (180 MB per clip).
//
// Numerics (reference contract): the reference computes QK^T, the softmax and P.V all in F32. Here Q and K arrive as
// fp16 hi/lo pairs (x = hi + lo, 22 significant bits) and S = Kh.Qh + Kl.Qh + Kh.Ql on fp16 MFMA with fp32
// accumulation (the lo.lo term is below 2^-22 relative), i.e. F32-class scores; P and V^T enter the P.V MFMA as hi/lo
// pairs too (Vh.Ph + Vh.Pl + Vl.Ph). Online softmax keeps a running reference point and sum per query; the 1/sum
// normalisation is applied once at the end.
//
// Kernels (the schedules measured and not adopted live in diag/attn_variants.hip, built only into diag libraries):
//   k_attn_t       reference contract: one 256-thread workgroup = 4 waves x 32 queries of one (clip, head) (x 16 when
//                  that grid would leave CUs idle), K/V tiles of 32 keys by LDS-DMA into three LDS stages,
//                  software-pipelined, 16x16x32 MFMAs
//   k_attn_pp<BF>  bf16-activation contract (BF = true): 8-wave ping-pong, one 512-thread workgroup = 256 queries
// The S accumulator feeds the P.V MFMA as its B operand with no data movement (K rows permuted so a lane's scores are
// the keys of its P.V fragment; cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand").
#include "q2a_internal.h"

#include <cstdlib>

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v_t __attribute__((ext_vector_type(4)));
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
// P.V precision of the diagnostic k_attn_g (diag/attn_variants.hip; reference: F32 P and V, qwen2-whisper.cpp:2088-2102):
//   PHL = 1: P = Ph + Pl, two fp16 halves (Ph = P truncated to fp16, Pl = the exact f32 remainder truncated
//                     to fp16: 22 significant bits), two P.V MFMAs per fragment
//   VHL = 1: V^T = Vh + Vl likewise (the QKV epilogue writes the lo image), one more MFMA per fragment
//                     (Vl.Ph; the Vl.Pl term is below 2^-22 relative) and a fourth LDS image per stage (two
//                     workgroups per CU instead of three)
// With PHL = 0 P is ONE fp16 value (truncated) and the softmax denominator is the sum of exactly those fp16 values
// (v_dot2 of the packed pairs against 1.0): the output is an exact weighted mean of V with the fp16 weights, so P's
// rounding does not bias the normalisation. With PHL = 1 the denominator is the f32 sum of P.
// QK^T terms of k_attn_g (diagnostic builds only): 3 = Kh.Qh + Kl.Qh + Kh.Ql (the contract); 21 = without Kl.Qh (K as
// fp16); 22 = without Kh.Ql (Q as fp16)
// lazy re-basing threshold of the softmax reference point: a lane re-bases when the P of its tile (8 or 16 per lane) sum to
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
// ---- reference contract (k_attn_t): the QK^T MFMAs of tile t+1 in one scheduling region with the softmax VALU of
// tile t (exp2, row sum, P hi/lo split: independent of those MFMAs), then the P.V MFMAs of tile t; 32-key tiles, three
// LDS stages of 16 KiB (K hi | K lo | V^T hi | V^T lo): iteration t reads K(t+1) from one, V(t) (and, on the rare
// re-base path, K(t)) from another, and DMAs tile t+2 into the third; one barrier per tile. The re-base path (a lane's
// P of the tile sum past PLIM) recomputes tile t's scores from K(t), re-bases, and moves the already computed
// S(t+1) - m' by the same shift.
constexpr int KS = 32;   // keys per tile
// fp16 remainder pair p - h (h = the truncated fp16 pair of p0, p1) in two v_fma_mix{lo,hi}_f16: the exact f32
// difference rounded once to fp16 (RNE), written straight into the packed register
__device__ __forceinline__ half2_t rem_pair(float p0, float p1, half2_t h) {
    half2_t r;
    asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(p0));
    asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(r) : "v"(h), "v"(p1));
    return r;
}
// The matrix work is v_mfma_f32_16x16x32_f16, not 32x32x16 (same cycles per flop; the attention runs power-limited,
// ~1.6 GHz against the GEMMs' ~2.0, and the 16x16 form draws less per flop: MI355X_MICROARCH.md, "bare bf16 MFMA
// loops"; the same software pipeline on 32x32x16 tiles, diag k_attn_s, measured 58.9 vs 56.0 ms/step). A wave = 32 queries as two 16-query blocks qb. S^T tile of 16 keys x 16 queries: lane l holds query
// 16qb + (l&15) and accumulator rows 4(l>>4) + r; the K row loaded into MFMA row i of key block kb is key
// 8(i>>2) + 4kb + (i&3), so lane group g = l>>4 holds keys 8g..8g+3 (kb 0) and 8g+4..8g+7 (kb 1): exactly the 8
// contiguous keys of its P.V B fragment, whose V^T operand is granule g of the V^T row (one 16-B read).
__device__ __forceinline__ f4v_t mma16(half8 a, half8 b, f4v_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// x combined with the value of lane ^ 16 / lane ^ 32 (v_permlane16/32_swap: one of the two results is the lane's own)
__device__ __forceinline__ float max_lane16(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_lane16(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float sum_lane32(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// VR (round 6): V hi / lo arrive row-major [clips*T][D] like K (the QKV GEMM's staged or persistent epilogue writes
// them as whole 128-B rows, no transposing epilogue) and the P.V A operand V^T[d][keys] is read out of the [key][d] LDS
// image by ds_read_b64_tr_b16 (two 4-key reads per 8-key fragment); !VR: the V^T [clip][head][64][TP] image (the ggml
// backend's operands) read by ds_read_b128.
// NQB = 16-query blocks per wave: 2 (128 queries per workgroup) or 1 (64, for grids too small to fill the chip — one
// clip). A block's arithmetic does not depend on its wave-mates (the lazy re-base is decided per block), so both forms
// give every query the same bits.
template <bool VR, int NQB>
__global__ __launch_bounds__(256, 3) void k_attn_t(const q2a_attn_args p) {
    static_assert(NQB == 1 || NQB == 2, "16 or 32 queries per wave");
    constexpr int QWG = 64 * NQB;   // queries per workgroup
    constexpr int KROW = 128, VROW = 64;
    constexpr int KIMG = KS * KROW, VIMG = 64 * VROW;
    constexpr int STAGE = 2 * KIMG + 2 * VIMG;                   // Kh | Kl | Vh^T | Vl^T of 32 keys
    __shared__ __attribute__((aligned(16))) char ldsA[STAGE];
    __shared__ __attribute__((aligned(16))) char ldsB[STAGE];
    __shared__ __attribute__((aligned(16))) char ldsC[STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = p.T, D = p.D;
    const int nq = (T + QWG - 1) / QWG, total = (int) gridDim.x;
    const int L = (int) blockIdx.x;
    const int w = (total & 7) ? L : (L & 7) * (total >> 3) + (L >> 3);   // XCD-contiguous work order: the q-tiles of one (clip, head) on one XCD
    const int qt = w % nq, h = (w / nq) % p.H, clip = w / (nq * p.H);
    const int q0 = qt * QWG + wave * 16 * NQB;
    const int64_t rowbase = (int64_t) clip * T;
    const int c16 = lane & 15, g = lane >> 4;

    // Q fragments (B operand): query 16qb + c16, d = 32ds + 8g .. +7
    half8 qh[NQB][2], ql[NQB][2];
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) {
        const int q = min(q0 + 16 * qb + c16, T - 1);
        const q2a_half * sh = p.qh + (rowbase + q) * D + h * 64 + 8 * g;
        const q2a_half * sl = p.ql + (rowbase + q) * D + h * 64 + 8 * g;
#pragma unroll
        for (int ds = 0; ds < 2; ++ds) {
            qh[qb][ds] = *(const half8 *) (sh + 32 * ds);
            ql[qb][ds] = *(const half8 *) (sl + 32 * ds);
        }
    }
    const int64_t vt_off = ((int64_t) clip * p.H + h) * 64 * p.TP;
    const char * khb = (const char *) (p.kh + rowbase * D + h * 64);
    const char * klb = (const char *) (p.kl + rowbase * D + h * 64);
    const char * vtb = (const char *) (VR ? p.vt + rowbase * D + h * 64 : p.vt + vt_off);
    const char * vlb = (const char *) (VR ? p.vtl + rowbase * D + h * 64 : p.vtl + vt_off);
    // LDS images: K granule c of row r at position c ^ kswz(r), V^T granule c of row r at c ^ vswz(r). ds_read_b128 is
    // serviced in four groups of 16 lanes ({0-3,12-15,20-27}, {4-11,16-19,28-31}, and +32; MI355X_MICROARCH.md §LDS);
    // these swizzles give every group's 16-B reads 16 distinct bank quads (modelled per group, then measured): the
    // 32x32x16 kernels' (r >> 1) & 7 / (r >> 2) & 3 gave 2-way conflicts here (SQ_LDS_BANK_CONFLICT 0.08 per
    // wave-cycle, 1.7 ms/step)
    auto kswz = [](int r) { return ((r >> 1) & 1) | ((r >> 2) & 6); };
    auto vswz = [](int r) { return (r & 1) | ((r >> 1) & 2); };
    // VR: granule c of key row r at c ^ vrswz(r) (128-B rows as K). A transposed read's 32-lane half covers key rows
    // 8g + q (+4) for g = 2h, 2h + 1 and q = 0..3 in the same two granules 2db, 2db + 1: rows of one parity share a
    // 32-bank half, and the four of them (q >> 1, g & 1) land on four distinct granule pairs — conflict-free
    auto vrswz = [](int r) { return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2); };
    const int krow_d = 8 * wave + (lane >> 3), kg = (lane & 7) ^ kswz(krow_d);
    const int vrow_d = 16 * wave + (lane >> 2), vg = (lane & 3) ^ vswz(vrow_d);
    const int vrg = (lane & 7) ^ vrswz(krow_d);
    auto dma_tile = [&](char * st, int t) {   // (k_attn_s's DMA)
        const int key = min(t * KS + krow_d, T - 1);
        const uint32_t ko = (uint32_t) (key * D + kg * 8) * 2u;
        const uint32_t vo = VR ? (uint32_t) (key * D + vrg * 8) * 2u : (uint32_t) (vrow_d * p.TP + t * KS + vg * 8) * 2u;
        __builtin_amdgcn_global_load_lds((const void *) (khb + ko), (lds_ptr_t) (st + wave * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *) (klb + ko), (lds_ptr_t) (st + KIMG + wave * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *) (vtb + vo), (lds_ptr_t) (st + 2 * KIMG + wave * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *) (vlb + vo), (lds_ptr_t) (st + 2 * KIMG + VIMG + wave * 1024), 16, 0, 0);
    };

    f4v_t o[NQB][4];
    float m_run[NQB], l_run[NQB];
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) {
#pragma unroll
        for (int db = 0; db < 4; ++db) o[qb][db] = f4v_t{0.f, 0.f, 0.f, 0.f};
        m_run[qb] = 0.f;
        l_run[qb] = 0.f;
    }
    const int ntiles = (T + KS - 1) / KS;
    // LDS byte offsets: K row of (kb, i = c16), chunk 4ds + g (swizzled); V^T row c16 (+16db), granule g (swizzled)
    uint32_t kofs[2][2], vofs;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
        const int kr = 8 * (c16 >> 2) + 4 * kb + (c16 & 3);
#pragma unroll
        for (int ds = 0; ds < 2; ++ds) kofs[kb][ds] = (uint32_t) (kr * KROW + (((4 * ds + g) ^ kswz(kr)) << 4));
    }
    vofs = (uint32_t) (2 * KIMG + c16 * VROW + ((g ^ vswz(c16)) << 4));   // (row + 16db: same swizzle)
    // VR: lane 4q + pp of group g supplies key row 8g + q (+ 4 for the fragment's upper half), columns 16db + 4pp ..
    // + 3: granule 2db + (pp >> 1), 8-B half pp & 1; the row's swizzle 2 (q >> 1) + 4 (g & 1) XORs db's bits only
    if (VR) {
        const int q4 = c16 >> 2, pp = c16 & 3;
        const int sx = (q4 >> 1) | ((g & 1) << 1);
        vofs = (uint32_t) (2 * KIMG + (8 * g + q4) * KROW + 8 * pp + 32 * sx);   // db = 0; db's fragment at vofs ^ 32 db
    }
    auto launder_ofs = [&]() {
        asm volatile("" : "+v"(kofs[0][0]), "+v"(kofs[0][1]), "+v"(kofs[1][0]), "+v"(kofs[1][1]), "+v"(vofs));
    };
    typedef short s4_t __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) s4_t * lds_s4p;
    // the V^T fragment of d-block db (8 keys of lane group g) from the row-major image at stage offset img
    auto vr_frag = [&](const char * st, int img, int db) -> half8 {
        const uint32_t a = (uint32_t) (uintptr_t) (const __attribute__((address_space(3))) char *) st + img + (vofs ^ (32u * db));
        const s4_t lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p) (uintptr_t) a);
        const s4_t hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4p) (uintptr_t) (a + 4 * KROW));
        const short8_t v8 = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
        return __builtin_bit_cast(half8, v8);
    };
    typedef f4v_t sc_t[NQB][2];   // [qb][kb]
    auto splat = [&](sc_t & s) {
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
            float nm = -m_run[qb];
            asm volatile("" : "+v"(nm));
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) s[qb][kb] = f4v_t{nm, nm, nm, nm};
        }
    };
    // P of the tile: [qb] = B fragment of keys 8g .. 8g+7 (hi and lo halves)
    half8 ph[NQB], pl[NQB];
    typedef float ex_t[NQB][8];   // exp2 of one tile's scores, [qb][4kb + r]
    // P hi / lo pairs and the lane sums of one tile's exponentials
    auto split = [&](const ex_t & e, float (&ls)[NQB]) {
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
            float a = e[qb][0];
#pragma unroll
            for (int j = 1; j < 8; ++j) a += e[qb][j];
            ls[qb] = a;
            half2_t hp[4], lp[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                hp[j] = pk_rtz(e[qb][2 * j], e[qb][2 * j + 1]);
                lp[j] = rem_pair(e[qb][2 * j], e[qb][2 * j + 1], hp[j]);
            }
            ph[qb] = half8{hp[0][0], hp[0][1], hp[1][0], hp[1][1], hp[2][0], hp[2][1], hp[3][0], hp[3][1]};
            pl[qb] = half8{lp[0][0], lp[0][1], lp[1][0], lp[1][1], lp[2][0], lp[2][1], lp[3][0], lp[3][1]};
        }
    };
    auto exps = [&](const sc_t & sv, ex_t & e) {
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    e[qb][4 * kb + r] = __builtin_amdgcn_exp2f(sv[qb][kb][r]);
                }
    };
    // region A: S'^T - m' of the tile at stage st into s (initialised by the caller with the splat); with e: the
    // previous tile's P split and sums in the MFMA issue gaps
    auto qk = [&](const char * st, sc_t & s, const ex_t * e, float (&ls)[NQB]) {
        launder_ofs();
#pragma unroll
        for (int ds = 0; ds < 2; ++ds) {
            half8 kh[2], kl[2];
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                kh[kb] = *(const half8 *) (st + kofs[kb][ds]);
                kl[kb] = *(const half8 *) (st + KIMG + kofs[kb][ds]);
            }
#pragma unroll
            for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
                for (int kb = 0; kb < 2; ++kb) {
                    s[qb][kb] = mma16(kh[kb], qh[qb][ds], s[qb][kb]);
                    s[qb][kb] = mma16(kl[kb], qh[qb][ds], s[qb][kb]);
                    s[qb][kb] = mma16(kh[kb], ql[qb][ds], s[qb][kb]);
                }
        }
        if (e) {
            split(*e, ls);
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
            for (int i = 0; i < 6 * NQB; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
            for (int i = 0; i < 6 * NQB; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
            }
        }
    };
    auto mask = [&](sc_t & sv, int t) {   // keys >= T (last tile only): key of (kb, r) in lane group g is 8g + 4kb + r
        if (t == ntiles - 1) {
#pragma unroll
            for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (t * KS + 8 * g + 4 * kb + r >= T) sv[qb][kb][r] = -1e30f;
        }
    };
    // re-base query block qb to the tile's max over its 32 keys (4 lane groups): first tile m' := that max
    auto rebase = [&](sc_t & sv, int qb, bool first, bool on = true) {
        float mx = sv[qb][0][0];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 4; ++r) mx = fmaxf(mx, sv[qb][kb][r]);
        mx = max_lane32(max_lane16(mx));
        // (on = false: a shift of exactly 0 — alpha 1, every value unchanged)
        const float sh = first ? mx : on ? fmaxf(mx, 0.f) : 0.f;
        if (!first) {
            const float alpha = __builtin_amdgcn_exp2f(-sh);
            l_run[qb] *= alpha;
#pragma unroll
            for (int db = 0; db < 4; ++db) o[qb][db] *= alpha;
        }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) sv[qb][kb] -= sh;
        m_run[qb] += sh;
        return sh;
    };
    // region B: O^T[d][q] += V^T[d][keys] . P^T[keys][q] (small terms first), with the exponentials of the next
    // tile's scores sn and the next QK^T's initial accumulators (the splat) in the MFMA issue gaps
    auto pv = [&](const char * st, sc_t & init, const sc_t & sn, ex_t & e) {
        launder_ofs();
        half8 va[4], vl[4];
#pragma unroll
        for (int db = 0; db < 4; ++db) {
            if constexpr (VR) {
                va[db] = vr_frag(st, 0, db);
                vl[db] = vr_frag(st, VIMG, db);
            } else {
                va[db] = *(const half8 *) (st + vofs + db * 16 * VROW);
                vl[db] = *(const half8 *) (st + VIMG + vofs + db * 16 * VROW);
            }
        }
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
            for (int db = 0; db < 4; ++db) {
                o[qb][db] = mma16(vl[db], ph[qb], o[qb][db]);
                o[qb][db] = mma16(va[db], pl[qb], o[qb][db]);
                o[qb][db] = mma16(va[db], ph[qb], o[qb][db]);
            }
        exps(sn, e);
        splat(init);
        // both stay in this region (not sunk past the barrier into the next tile's head)
        if constexpr (NQB == 2) {
            asm volatile("" : "+v"(init[0][0]), "+v"(init[0][1]), "+v"(init[1][0]), "+v"(init[1][1]));
            asm volatile("" : "+v"(e[0][0]), "+v"(e[0][1]), "+v"(e[0][2]), "+v"(e[0][3]), "+v"(e[0][4]), "+v"(e[0][5]),
                              "+v"(e[0][6]), "+v"(e[0][7]), "+v"(e[1][0]), "+v"(e[1][1]), "+v"(e[1][2]), "+v"(e[1][3]),
                              "+v"(e[1][4]), "+v"(e[1][5]), "+v"(e[1][6]), "+v"(e[1][7]));
        } else {
            asm volatile("" : "+v"(init[0][0]), "+v"(init[0][1]));
            asm volatile("" : "+v"(e[0][0]), "+v"(e[0][1]), "+v"(e[0][2]), "+v"(e[0][3]), "+v"(e[0][4]), "+v"(e[0][5]),
                              "+v"(e[0][6]), "+v"(e[0][7]));
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
        for (int i = 0; i < 8 * NQB; ++i) {   // one exponential per MFMA gap (8 of the 16 cycles issue VALU)
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        }
#pragma unroll
        for (int i = 0; i < 4 * NQB; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x002, 8 * NQB, 0);
    };

    sc_t sn, init;
    ex_t ex;   // exp2 of the current tile's scores (computed in the previous iteration's region B)
    // iteration t: stage sK holds tile t+1, sV tile t (its V for P.V, its K for the rare re-base), tile t+2 -> sD
    auto iter = [&](const char * sK, const char * sV, char * sD, int t) {
        if (t + 2 < ntiles) dma_tile(sD, t + 2);
        float ls[NQB];
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) sn[qb][kb] = init[qb][kb];
        // region A: QK^T(t+1) beside the P split / sums of tile t. (After the last tile it reads a stage holding an
        // older tile; those scores are never used.)
        qk(sK, sn, &ex, ls);
        // rare: re-base from tile t's scores (K(t) in place), decided per 16-query block (a block whose lanes all stay
        // under PLIM keeps its reference point and its exponentials)
        bool rb[NQB], any_rb = false;
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) {
            rb[qb] = __any(ls[qb] > PLIM);
            any_rb |= rb[qb];
        }
        if (t != 0 && any_rb) {
            sc_t s2;
            splat(s2);
            float dummy[NQB];
            qk(sV, s2, nullptr, dummy);
            mask(s2, t);
#pragma unroll
            for (int qb = 0; qb < NQB; ++qb) {
                const float sh = rebase(s2, qb, false, rb[qb]);
#pragma unroll
                for (int kb = 0; kb < 2; ++kb) sn[qb][kb] -= sh;
            }
            // P of tile t again, against the new reference point — only for the re-based blocks: the others keep the
            // exponentials of S(t) - m' as first computed (a recomputation from the current m' can differ in the
            // last bit when m' moved in the previous iteration)
            ex_t e2;
            exps(s2, e2);
#pragma unroll
            for (int qb = 0; qb < NQB; ++qb)
#pragma unroll
                for (int j = 0; j < 8; ++j) ex[qb][j] = rb[qb] ? e2[qb][j] : ex[qb][j];
            split(ex, ls);
        }
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) l_run[qb] += ls[qb];
        mask(sn, t + 1);
        // region B: P.V(t) beside the exponentials of tile t+1
        pv(sV, init, sn, ex);
        __syncthreads();   // tile t+2 landed; every wave done with tile t's stage
    };

    dma_tile(ldsA, 0);
    if (ntiles > 1) dma_tile(ldsB, 1);
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) asm volatile("" :: "v"(qh[qb][0]), "v"(qh[qb][1]), "v"(ql[qb][0]), "v"(ql[qb][1]));
    __syncthreads();
    {
        float dummy[NQB];
        sc_t s0;
        splat(s0);
        qk(ldsA, s0, nullptr, dummy);   // tile 0 against m' = 0, then m' := its max
        mask(s0, 0);
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) rebase(s0, qb, true);
        exps(s0, ex);
        splat(init);
    }
    for (int t = 0; t < ntiles; t += 3) {
        iter(ldsB, ldsA, ldsC, t);
        if (t + 1 >= ntiles) break;
        iter(ldsC, ldsB, ldsA, t + 1);
        if (t + 2 >= ntiles) break;
        iter(ldsA, ldsC, ldsB, t + 2);
    }

#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) {
        const float l_tot = sum_lane32(sum_lane16(l_run[qb]));
        const float inv = 1.0f / l_tot;
        const int q = q0 + 16 * qb + c16;
        if (q < T) {
            const int64_t orow = (rowbase + q) * D + h * 64;
#pragma unroll
            for (int db = 0; db < 4; ++db) {
                const int d = 16 * db + 4 * g;
                f4v_t v = o[qb][db] * inv;
                if (p.outH) {
                    asm volatile("" : "+v"(v));   // f32 first: the fp16 output is the fp16 of the f32 output
                    const half4 hv = {(_Float16) v[0], (_Float16) v[1], (_Float16) v[2], (_Float16) v[3]};
                    *(half4 *) (p.outH + orow + d) = hv;
                } else {
                    *(float4 *) (p.outF + orow + d) = make_float4(v[0], v[1], v[2], v[3]);
                }
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
                float v0 = o[dt][4 * g + 0] * inv, v1 = o[dt][4 * g + 1] * inv;
                float v2 = o[dt][4 * g + 2] * inv, v3 = o[dt][4 * g + 3] * inv;
                if (p.outH) {
                    // rounded to f32 first (no one-step fp16 rounding of the product): the fp16 output is the fp16 of
                    // the f32 output, bit for bit
                    asm volatile("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
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
bool q2a_attention_wants_vlo() { return true; }

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
        if (!a.vtl) return hipErrorInvalidValue;
        // 32 queries per wave, or 16 when that grid would leave CUs idle (one clip: 240 workgroups of 128 queries on
        // 256 CUs, one wave per SIMD); the two forms give the same bits
        const int n2 = ((a.T + 127) / 128) * a.H * a.n_clips;
        const bool narrow = n2 < q2a_cu_count();
        const dim3 grid(narrow ? ((a.T + 63) / 64) * a.H * a.n_clips : n2);
        if (a.v_rows) {
            if (narrow) hipLaunchKernelGGL((k_attn_t<true, 1>), grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_attn_t<true, 2>), grid, dim3(256), 0, s, a);
        } else {
            if (narrow) hipLaunchKernelGGL((k_attn_t<false, 1>), grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_attn_t<false, 2>), grid, dim3(256), 0, s, a);
        }
    }
    return hipGetLastError();
}
