// diag/attn_variants.hip — attention schedules measured and NOT adopted, built only into diagnostic
// variant libraries (diag/build_attn_variant.sh), never into lib/libq2a.so. This translation unit is the product
// q2a_attn.hip (its launcher renamed) plus these kernels and a launcher that picks one at COMPILE time:
//   Q2A_ATTN_VARIANT 0 product launcher   1 k_attn (register-staged K/V)   2 k_attn_g32 (32-key tiles)
//                    3 k_attn_p32 (QK^T of tile t+1 interleaved with softmax t)   4 k_attn_pp32 (8-wave ping-pong)
//                    5 k_attn_pp<false> (F32-class ping-pong, 64-key tiles)   6 / 7 k_attn with 2 / 1 QK^T terms
//                    8 k_attn_g (64-key tiles, 32x32x16; its PHL / VHL / VDB / QK_TERMS switches)   9 k_attn_s
// (round 6: the product kernel's own precision / schedule switches moved to diag/experiment_knobs_r05.patch; the
// switches of k_attn_g below keep their product values unless a build sets them).
#define Q2A_ATTN_LAUNCH q2a_launch_attention_product
#include "../qwen2-audio-whisper-ggml_amd/csrc/q2a_attn.hip"
#ifndef Q2A_ATTN_PHL
#define Q2A_ATTN_PHL 1
#endif
#ifndef Q2A_ATTN_VHL
#define Q2A_ATTN_VHL 1
#endif
#ifndef Q2A_ATTN_QK_TERMS
#define Q2A_ATTN_QK_TERMS 3
#endif
#ifndef Q2A_ATTN_S_SCHED
#define Q2A_ATTN_S_SCHED 1
#endif

#ifndef Q2A_ATTN_VARIANT
#define Q2A_ATTN_VARIANT 0
#endif

namespace {

// the reference-contract producers fold log2(e) into Q (q2a_internal.h, Q2A_LOG2E): these kernels' scores are
// already in log2 units
constexpr float QL2E = 1.0f;

// ---- moved from the product (round 3): the 64-key 32x32x16 kernel k_attn_g (round-3 default until k_attn_t) with its
// P.V precision / occupancy switches (Q2A_ATTN_PHL, Q2A_ATTN_VHL, Q2A_ATTN_VDB, Q2A_ATTN_QK_TERMS), and k_attn_s, the
// software-pipelined 32-key form on 32x32x16 MFMAs (k_attn_t's schedule before the 16x16x32 rewrite)
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


__global__ __launch_bounds__(256, 3) void k_attn_s(const q2a_attn_args p) {
    constexpr int KROW = 128, VROW = 64;                         // K rows: 64 d (8 granules); V^T rows: 32 keys (4)
    constexpr int KIMG = KS * KROW, VIMG = 64 * VROW;            // 4 KiB each
    constexpr int STAGE = 2 * KIMG + 2 * VIMG;                   // Kh | Kl | Vh^T | Vl^T
    __shared__ __attribute__((aligned(16))) char ldsA[STAGE];
    __shared__ __attribute__((aligned(16))) char ldsB[STAGE];
    __shared__ __attribute__((aligned(16))) char ldsC[STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int T = p.T, D = p.D;
    const int nq = (T + 127) / 128, total = (int) gridDim.x;
    const int L = (int) blockIdx.x;
    const int w = (total & 7) ? L : (L & 7) * (total >> 3) + (L >> 3);   // XCD-contiguous work order (k_attn_g)
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
    // DMA of one tile: wave w moves rows 8w..8w+7 of each K image (granule l%8 <- source granule (l%8)^((row>>1)&7))
    // and rows 16w..16w+15 of each V^T image (granule l%4 <- source granule (l%4)^((row>>2)&3)): 1 KiB per image
    const int64_t vt_off = ((int64_t) clip * p.H + h) * 64 * p.TP;
    const char * khb = (const char *) (p.kh + rowbase * D + h * 64);
    const char * klb = (const char *) (p.kl + rowbase * D + h * 64);
    const char * vtb = (const char *) (p.vt + vt_off);
    const char * vlb = (const char *) (p.vtl + vt_off);
    const int krow_d = 8 * wave + (lane >> 3), kg = (lane & 7) ^ ((krow_d >> 1) & 7);
    const int vrow_d = 16 * wave + (lane >> 2), vg = (lane & 3) ^ ((vrow_d >> 2) & 3);
    auto dma_tile = [&](char * st, int t) {
        const int key = min(t * KS + krow_d, T - 1);
        const uint32_t ko = (uint32_t) (key * D + kg * 8) * 2u;
        const uint32_t vo = (uint32_t) (vrow_d * p.TP + t * KS + vg * 8) * 2u;
        __builtin_amdgcn_global_load_lds((const void *) (khb + ko), (lds_ptr_t) (st + wave * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *) (klb + ko), (lds_ptr_t) (st + KIMG + wave * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *) (vtb + vo), (lds_ptr_t) (st + 2 * KIMG + wave * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *) (vlb + vo), (lds_ptr_t) (st + 2 * KIMG + VIMG + wave * 1024), 16, 0, 0);
    };

    f16v o[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    float m_run = 0.f, l_run = 0.f;
    // -m' in all 16 registers of the next QK^T chain's accumulator: a splat of one scalar into the registers the chain
    // then accumulates in, written among the previous tile's P.V MFMAs (no live 16-register constant)
    auto splat = [&]() {
        float nm = -m_run;
        asm volatile("" : "+v"(nm));
        f16v s;
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = nm;
        return s;
    };
    const int ntiles = (T + KS - 1) / KS;
    // per-lane LDS byte offsets: K row kperm(col), chunk 2st+hi (swizzled); V^T row col, granule 2sp+hi (swizzled)
    uint32_t kofs[4], vofs[2];
    {
        const int kr = kperm(col);
#pragma unroll
        for (int st = 0; st < 4; ++st) kofs[st] = (uint32_t) (kr * KROW + (((2 * st + hi) ^ ((kr >> 1) & 7)) << 4));
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) vofs[sp] = (uint32_t) (2 * KIMG + col * VROW + (((2 * sp + hi) ^ ((col >> 2) & 3)) << 4));
    }
    auto launder_ofs = [&]() {
        asm volatile("" : "+v"(kofs[0]), "+v"(kofs[1]), "+v"(kofs[2]), "+v"(kofs[3]), "+v"(vofs[0]), "+v"(vofs[1]));
    };
    // S'^T - m' of the tile whose K images are at st (12 MFMAs on one chain, starting from the splat s); the K fragments of
    // step k+1 are read before the MFMAs of step k. With sm: the softmax of the previous tile's scores sm (4 scores
    // per 16-deep step, about 5 VALU instructions after each MFMA: one scheduling group each) -> ph, pl, ls
    half2_t ph[8], pl[8];
    auto qk = [&](const char * st, f16v s, const f16v * sm, float & ls) {
        launder_ofs();
        half8 fh = *(const half8 *) (st + kofs[0]), fl = *(const half8 *) (st + KIMG + kofs[0]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            half8 nh, nl;
            if (k < 3) {
                nh = *(const half8 *) (st + kofs[k + 1]);
                nl = *(const half8 *) (st + KIMG + kofs[k + 1]);
            }
            s = mma32<false>(fh, qh[k], s);
            float p0, p1, p2, p3;
            if (sm) {
                p0 = __builtin_amdgcn_exp2f((*sm)[4 * k]);
                p1 = __builtin_amdgcn_exp2f((*sm)[4 * k + 1]);
                ls = k ? ls + p0 : p0;
                ls += p1;
                ph[2 * k] = pk_rtz(p0, p1);
            }
            s = mma32<false>(fl, qh[k], s);
            if (sm) {
                p2 = __builtin_amdgcn_exp2f((*sm)[4 * k + 2]);
                p3 = __builtin_amdgcn_exp2f((*sm)[4 * k + 3]);
                pl[2 * k] = rem_pair(p0, p1, ph[2 * k]);
                ls += p2;
            }
            s = mma32<false>(fh, ql[k], s);
            if (sm) {
                ls += p3;
                ph[2 * k + 1] = pk_rtz(p2, p3);
                pl[2 * k + 1] = rem_pair(p2, p3, ph[2 * k + 1]);
            }
#if Q2A_ATTN_S_SCHED
            if (sm) {   // one group per step: its K reads, then MFMA / VALU alternating
                if (k < 3) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
#endif
            if (k < 3) { fh = nh; fl = nl; }
        }
        return s;
    };
    // mask keys >= T (only the last tile has them; key of reg r: 16(r>>3) + 8hi + (r&7))
    auto mask = [&](f16v & s, int t) {
        if (t == ntiles - 1) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (t * KS + 16 * (r >> 3) + 8 * hi + (r & 7) >= T) s[r] = -1e30f;
        }
    };
    // P = exp2(S' - m'), its f32 lane sum, the truncated fp16 pairs and their fp16 remainders (the re-base path)
    auto softmax = [&](f16v s, float & ls) {
        ls = 0.f;
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
            const float p0 = __builtin_amdgcn_exp2f(s[r]), p1 = __builtin_amdgcn_exp2f(s[r + 1]);
            ls += p0;
            ls += p1;
            const half2_t hp = pk_rtz(p0, p1);
            ph[r >> 1] = hp;
            pl[r >> 1] = rem_pair(p0, p1, hp);
        }
    };
    // re-base to the tile's max (per query: both lane halves): first tile m' := that max; later only upward
    auto rebase = [&](f16v & s, bool first) {
        float mx = s[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s[r]);
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
        for (int r = 0; r < 16; ++r) s[r] -= sh;
        m_run += sh;
        return sh;
    };
    // O^T[d][q] += V^T[d][keys] . P^T[keys][q] (small terms first), V images of stage st; returns the next QK^T
    // chain's initial accumulator (the splat, its 16 moves in the MFMA issue gaps)
    auto pv = [&](const char * st) {
        launder_ofs();
        half8 va[2][2], vl[2][2];
#pragma unroll
        for (int sp = 0; sp < 2; ++sp)
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
                va[sp][dt] = *(const half8 *) (st + vofs[sp] + dt * 32 * VROW);
                vl[sp][dt] = *(const half8 *) (st + VIMG + vofs[sp] + dt * 32 * VROW);
            }
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {   // keys 16sp + 8hi .. +7 = P registers 8sp .. 8sp+7
            const half8 pb = {ph[4 * sp][0], ph[4 * sp][1], ph[4 * sp + 1][0], ph[4 * sp + 1][1],
                              ph[4 * sp + 2][0], ph[4 * sp + 2][1], ph[4 * sp + 3][0], ph[4 * sp + 3][1]};
            const half8 pc = {pl[4 * sp][0], pl[4 * sp][1], pl[4 * sp + 1][0], pl[4 * sp + 1][1],
                              pl[4 * sp + 2][0], pl[4 * sp + 2][1], pl[4 * sp + 3][0], pl[4 * sp + 3][1]};
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
                o[dt] = mma32<false>(vl[sp][dt], pb, o[dt]);
                o[dt] = mma32<false>(va[sp][dt], pc, o[dt]);
                o[dt] = mma32<false>(va[sp][dt], pb, o[dt]);
            }
        }
        f16v init = splat();
        asm volatile("" : "+v"(init));   // the moves stay in this region (not sunk to the next tile's QK^T)
#if Q2A_ATTN_S_SCHED
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);   // sp = 0's V fragments
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);   // sp = 1's
#pragma unroll
        for (int i = 0; i < 11; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
#endif
        return init;
    };

    f16v sc, init;
    // iteration t: stage sK holds tile t+1, sV tile t (its V for P.V, its K for the rare re-base), tile t+2 -> sD
    auto iter = [&](const char * sK, const char * sV, char * sD, int t) {
        if (t + 2 < ntiles) dma_tile(sD, t + 2);
        mask(sc, t);
        // ---- QK^T(t+1) MFMAs interleaved with softmax(t) VALU. (After the last tile it reads a stage holding an
        // older tile; those scores are never used.)
        float ls;
        f16v sn = qk(sK, init, &sc, ls);
        if (t != 0 && __any(ls > PLIM)) {   // rare: re-base from tile t's scores (its K stage is still in place)
            float dummy;
            f16v s2 = qk(sV, splat(), nullptr, dummy);
            mask(s2, t);
            const float sh = rebase(s2, false);
#pragma unroll
            for (int r = 0; r < 16; ++r) sn[r] -= sh;
            softmax(s2, ls);
        }
        l_run += ls;
        init = pv(sV);
        sc = sn;
        __syncthreads();   // tile t+2 landed (vmcnt(0) in the barrier); every wave done with tile t's stage
    };

    dma_tile(ldsA, 0);
    if (ntiles > 1) dma_tile(ldsB, 1);
    asm volatile("" :: "v"(qh[0]), "v"(qh[1]), "v"(qh[2]), "v"(qh[3]), "v"(ql[0]), "v"(ql[1]), "v"(ql[2]), "v"(ql[3]));
    __syncthreads();
    float dummy;
    sc = qk(ldsA, splat(), nullptr, dummy);      // tile 0 against m' = 0, then m' := its max
    mask(sc, 0);
    rebase(sc, true);
    init = splat();
    for (int t = 0; t < ntiles; t += 3) {
        iter(ldsB, ldsA, ldsC, t);
        if (t + 1 >= ntiles) break;
        iter(ldsC, ldsB, ldsA, t + 1);
        if (t + 2 >= ntiles) break;
        iter(ldsA, ldsC, ldsB, t + 2);
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


#ifndef Q2A_ATTN_F32_OCC
#define Q2A_ATTN_F32_OCC 2
#endif
// BF: bf16-activation mode (Q, K, V^T, P and the output in bf16; S = K.Q^T is one MFMA per 16-deep step)
// QT: fp16 terms of S in the reference contract (3: Kh.Qh + Kl.Qh + Kh.Ql; 2 / 1: precision experiments)
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
        const float nm = -m_new * QL2E;
        const float alpha = __builtin_amdgcn_exp2f(fmaf(m_run, QL2E, nm));
        float ls = 0.f;
        half8 pf[2][2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float pv = __builtin_amdgcn_exp2f(fmaf(sc[kb][r], QL2E, nm));
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
        const float nm = -m_new * QL2E;
        const float alpha = __builtin_amdgcn_exp2f(fmaf(m_run, QL2E, nm));
        float ls = 0.f;
        half8 pf[2];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float pv = __builtin_amdgcn_exp2f(fmaf(sc[r], QL2E, nm));
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
        const float nm = -m_new * QL2E;
        const float alpha = __builtin_amdgcn_exp2f(fmaf(m_run, QL2E, nm));
        float ls = 0.f;
        half8 pf[2];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float pv = __builtin_amdgcn_exp2f(fmaf(sc[r], QL2E, nm));
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
        const float nm = -m_new * QL2E;
        const float alpha = __builtin_amdgcn_exp2f(fmaf(m_run, QL2E, nm));
        float ls = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float pv = __builtin_amdgcn_exp2f(fmaf(sc[r], QL2E, nm));
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
}  // namespace

hipError_t q2a_launch_attention(const q2a_attn_args & a, hipStream_t s) {
    if (Q2A_ATTN_VARIANT == 0 || a.bf16) return q2a_launch_attention_product(a, s);
    if (a.D != a.H * 64 || a.TP < ((a.T + KT - 1) / KT) * KT) return hipErrorInvalidValue;
    const dim3 grid(((a.T + 127) / 128) * a.H * a.n_clips), grid2(((a.T + 255) / 256) * a.H * a.n_clips);
    switch (Q2A_ATTN_VARIANT) {
        case 1: hipLaunchKernelGGL(k_attn<false>, grid, dim3(256), 0, s, a); break;
        case 2: hipLaunchKernelGGL(k_attn_g32, grid, dim3(256), 0, s, a); break;
        case 3: hipLaunchKernelGGL(k_attn_p32, grid, dim3(256), 0, s, a); break;
        case 4: hipLaunchKernelGGL(k_attn_pp32, grid2, dim3(512), 0, s, a); break;
        case 5: hipLaunchKernelGGL(k_attn_pp<false>, grid2, dim3(512), 0, s, a); break;
        case 6: hipLaunchKernelGGL((k_attn<false, 2>), grid, dim3(256), 0, s, a); break;
        case 7: hipLaunchKernelGGL((k_attn<false, 1>), grid, dim3(256), 0, s, a); break;
        case 8: hipLaunchKernelGGL(k_attn_g, grid, dim3(256), 0, s, a); break;
        case 9: hipLaunchKernelGGL(k_attn_s, grid, dim3(256), 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
