// Deep-scale conv family, device side (included by conv_deep.hip): the
// per-tile body and its LDS size.
#pragma once
#include <stdlib.h>

#include "common.h"
#include "conv_common.h"

namespace {

constexpr int DEEP_BM = 64;

// phase stamps for tools/probe/deep_stamps.hip (compiled out of the product)
#ifdef RNVP_DEEP_STAMPS
__device__ unsigned long long* g_deep_stamps;
#define DEEP_STAMP(i) \
    do { if (threadIdx.x == 0) g_deep_stamps[blockIdx.x * 8 + (i)] = wall_clock64(); } while (0)
#else
#define DEEP_STAMP(i) do {} while (0)
#endif
constexpr int DEEP_MAX_CS = 1024;    // prologue BN table capacity (channels)

template <typename T>
__host__ __device__ constexpr int deep_pitch(int cs) { return lds_mfma_pitch(cs, Mf<T>::CH); }

// bp: the BatchNorm-backward prologue's table (3 floats per channel, not 2)
template <typename T, int BN, int NW, int WK, int BM = DEEP_BM>
size_t deep_lds_bytes(int cs, int W, int ks, bool bp = false) {
    constexpr int TM = BM / 16, WM = NW / WK;
    constexpr int G = WK > 1 ? TM : WM;
    const int hal = (ks / 2) * (W + 1), R = BM + 2 * hal;
    const size_t head = 4 * (5 * (size_t)BN) + 8 * (2 * (size_t)G * BN) + 4 * (bp ? 3 : 2) * (size_t)cs;
    const size_t zrow = (size_t)deep_pitch<T>(cs) * sizeof(T);
    size_t act = (size_t)R * deep_pitch<T>(cs) * sizeof(T);
    const size_t red = WK > 1 ? (size_t)WK * BM * (BN + 4) * 4 : 0;
    return head + zrow + (act > red ? act : red);
}

// One 64-pixel x BN-channel output tile.  vb / nvb: the tile's virtual block
// index and the virtual grid (= the tile count); a standalone launch passes
// its blockIdx / gridDim, the persistent net chain (net_chain.hip) the tiles
// its resident workgroups loop over (vb % 8 is still the XCD when the
// resident grid is a multiple of 8).  Callers separate consecutive tiles of
// one workgroup with a barrier (the LDS is reused).
// FM: the weights come from the fragment-major image (rnvp_conv_args.w_frag,
// bf16): 16 output rows x 32 k per 1 KiB block, in MFMA lane order, so every
// weight load of a wave is one contiguous KiB (eight whole 128-B lines)
// instead of 64 B from each of 16 rows -- the row-major loads held the deep
// 3x3 tiles to ~37 GB/s of weights per CU (TA busy ~55 cycles per load)
// BM: pixels per tile (64; 128 for the 3x3 tiles of cfg 6, which read each
// weight slice for twice the pixels: half the weight stream per launch)
// BP: the BatchNorm-backward prologue (rnvp_conv_args.bp; data gradients, so
// never with PRO): the staged operand is dL/dt = coef (g - k1 - xhat k2) of
// the gradient g (a.x) and the BatchNorm input t (a.bp_x), formed in
// registers as the rows go to LDS; channel tile 0 also stores it (a.bp_out)
template <typename T, int BN, int KSZ, bool PRO, int NW, int WK, int DK, int NC, bool FM = false, int BM = DEEP_BM,
          bool BP = false>
__device__ __forceinline__ void deep_tile(const rnvp_conv_args& a, int shards, int xa, int xb, int vb, int nvb,
                                          char* lds) {
    constexpr int NT = 64 * NW;
    constexpr int CH = Mf<T>::CH, KS = 4 * CH;
    constexpr int TM = BM / 16, TN = BN / 16;
    constexpr int WM = NW / WK;
    constexpr int TMW = TM / WM;                 // 16-pixel fragment rows per wave
    static_assert(WM * WK == NW && TMW * WM == TM, "wave layout");
    constexpr int PAD = KSZ / 2;
    constexpr int RP = BN + 4;                   // partial-tile row pitch (floats)
    constexpr int G = WK > 1 ? TM : WM;          // stat partial groups per column
    constexpr int FR = WK > 1 ? (TM * TN) / NW : 1;
    static_assert(WK == 1 || FR * NW == TM * TN, "final tiles");
    // TALL: more 16-pixel row groups than waves (BM = 128 with 4 waves): wave
    // wid takes row groups wid, wid + NW, ... with all TN column tiles of each
    constexpr bool TALL = WK > 1 && TM > NW;
    static_assert(!TALL || TM % NW == 0, "row groups per wave");
    // the operand's channel stride is NC * WK * KS exactly (launcher): the BN
    // table needs ceil(cs / NT) channels per thread, not DEEP_MAX_CS's
    constexpr int CPT = (NC * WK * KS + NT - 1) / NT;
    static_assert(!(BP && PRO), "BatchNorm-backward prologue: data gradients only");
    constexpr int NSTEP = KSZ * KSZ * NC;        // k-steps of one wave (static: fully unrolled)
    const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wk = wid % WK, wm = wid / WK;
    const int M = a.B * a.H * a.W, W = a.W, H = a.H;
    const int N = a.n, cs = a.cs_in;
    const int gm = (M + BM - 1) / BM;
    // tiles of one channel block (same weights) are consecutive and share an XCD
    const int nb = nvb, b = vb;
    const int q8 = nb / 8, r8 = nb % 8, xcd = b % 8;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
    // consecutive t share an XCD; tile order: blocks of xa pixel tiles x xb
    // channel tiles (xa | gm, xb | gn), or channel-major (xa == 0: tiles of one
    // channel block together) / pixel-major (xa < 0)
    int mt, nt;
    if (xa > 0) {
        const int per = xa * xb, bi = t / per, w = t - bi * per, gmb = gm / xa;
        const int bm = bi % gmb, bn = bi / gmb;
        mt = bm * xa + w % xa;
        nt = bn * xb + w / xa;
    } else if (xa == 0) {
        nt = t / gm;
        mt = t - nt * gm;
    } else {
        const int gn = nvb / gm;
        mt = t / gn;
        nt = t - mt * gn;
    }
    const int m0 = mt * BM, n0 = nt * BN;
    const T* __restrict__ X = (const T*)a.x;
    const T* __restrict__ Wt = (const T*)(FM ? a.w_frag : a.w);
    const bool epi_bn = a.epi_relu_bn_bwd != 0;
    static_assert(BN <= NT, "bias / table loads: one channel per thread");

    const int hal = PAD * (W + 1);
    const int R = BM + 2 * hal;
    const int pitch = deep_pitch<T>(cs);
    float* etab = (float*)lds;                   // scale | shift | mean | rstd [BN each]
    float* btab = etab + 4 * BN;                 // bias [BN]
    double* sred = (double*)(btab + BN);         // [G][BN][2]
    float* bnp = (float*)(sred + G * BN * 2);    // prologue scale | shift [cs each] (BP: A | B | C)
    T* zrow = (T*)(bnp + (BP ? 3 : 2) * cs);     // [pitch] zeros
    T* act = zrow + pitch;                       // [R][pitch]; after the K loop: red [WK][BM][RP] f32

    // ---- prologue: every independent load at once (weight ring, BN-table
    // sums, activation rows), one wait, the transform into LDS ----
    // the channel stride is NC * WK * KS (launcher), so a row is CPR chunks
    // and NT % CPR == 0: a thread's chunk column is the same in every staged
    // row -- its BN coefficients are loaded into registers once, and its rows
    // advance by NT / CPR per slot
    constexpr int CPR = NC * WK * 4;
    static_assert(NT % CPR == 0, "fixed chunk column per thread");
    constexpr int RSTEP = NT / CPR;
    // staged chunks per thread per batch.  BP (two operands per chunk): the
    // slots one batch needs -- the 64 rows of a 1x1 tile, the rows of a 3x3
    // tile + halo up to 16 pixels wide (wider images loop) -- at most 12 (8
    // for the 4-wave tiles, whose 3x3 kernels otherwise pass 256 registers
    // and drop to one wave per SIMD: a second batch costs less)
    constexpr int SBP = KSZ == 1 ? (BM + RSTEP - 1) / RSTEP : (BM + 2 * 17 + RSTEP - 1) / RSTEP;
    constexpr int SBC = NT == 256 ? 8 : 12;
    constexpr int SB = BP ? (SBP < SBC ? SBP : SBC) : 20 * 256 / NT;
    const int cfix = tid % CPR, rbase = tid / CPR;
    u32x4 sv[SB];
    u32x4 sx[BP ? SB : 1];
    const T* __restrict__ XT = (const T*)a.bp_x;
    // loads past the staged rows are not issued at all (a uniform skip): at
    // 128 channels the rows fill ~6 of the SB slots, and every wasted load
    // counts against the 63 outstanding vector memory operations a wave can
    // have, serialising the prologue into extra memory round trips
    auto stage_load = [&](int r0) {
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            if (r0 + u * RSTEP >= R) break;
            const int r = r0 + rbase + u * RSTEP;
            const int p = m0 - hal + r;
            const bool ok = (r < R) & (p >= 0) & (p < M);
            const long long o = ok ? (long long)p * cs + cfix * CH : 0;
            sv[u] = *(const u32x4*)(X + o);
            if constexpr (BP) sx[u] = *(const u32x4*)(XT + o);
        }
    };
    float scv[CH], shv[CH];
    // BP coefficients of the thread's channels: dL/dt = A g - (B t + C) with
    // A = gamma rstd, B = A rstd k2, C = A (k1 - rstd k2 mean) (rnvp_bn_bwd_apply's
    // A (g - k1 - (t - mean) rstd k2), regrouped: three registers per channel)
    float bca[BP ? CH : 1], bcb[BP ? CH : 1], bcc[BP ? CH : 1];
    T* __restrict__ BPO = (T*)a.bp_out;
    const bool bp_store = BP && BPO != nullptr && nt == 0;
    auto stage_store = [&](int r0) {
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            const int r = r0 + rbase + u * RSTEP;
            if (r >= R) continue;
            const int p = m0 - hal + r;
            u32x4 w = sv[u];
            if (PRO) {
                if constexpr (sizeof(T) == 2) {
                    w = bn_relu_bf16x8(w, scv, shv);
                } else {
                    float f[CH];
                    unpack(w, f, T());
#pragma unroll
                    for (int e = 0; e < CH; ++e) f[e] = fmaxf(f[e] * scv[e] + shv[e], 0.f);
                    w = pack(f, T());
                }
            }
            if constexpr (BP) {
                float gv[CH], xv[CH], d[CH];
                unpack(w, gv, T());
                unpack(sx[u], xv, T());
#pragma unroll
                for (int e = 0; e < CH; ++e) d[e] = fmaf(bca[e], gv[e], -fmaf(bcb[e], xv[e], bcc[e]));
                w = pack(d, T());
                // each interior pixel once (its own tile's rows, channel tile 0)
                if (bp_store && r >= hal && r < hal + BM && p < M)
                    *(u32x4*)(BPO + (long long)p * cs + cfix * CH) = w;
            }
            const uint32_t keep = (p >= 0 && p < M) ? ~0u : 0u;
            *(u32x4*)(act + r * pitch + cfix * CH) = w & u32x4{keep, keep, keep, keep};
        }
    };
    DEEP_STAMP(0);
    // epilogue elements of this thread: (pixel m, tile column col) of element e
    constexpr int NE = WK > 1 ? FR : TMW * TN;
    auto elem = [&](int e, int& m, int& col) {
        if constexpr (TALL) {
            m = m0 + (wid + NW * (e / TN)) * 16 + li;
            col = (e % TN) * 16 + 4 * g;
        } else if constexpr (WK > 1) {
            m = m0 + (wid % TM) * 16 + li;
            col = ((wid / TM) * FR + e) * 16 + 4 * g;
        } else {
            m = m0 + (wm * TMW + e / TN) * 16 + li;
            col = (e % TN) * 16 + 4 * g;
        }
    };
    const int cso = a.cs_out;
    // issue order = wait order (vmcnt is in order): the small table / bias /
    // epilogue operands first, then the activation rows, then the weight ring
    BnTab<CPT> ptab;
    BnTab<1> etb;
    if (PRO) tab_issue<CPT, NT>(a.pro, a.cin, 0, cs, ptab);
    // BP: the BatchNorm's batch statistics and the gradient sums, as two
    // BatchNorm sources (a sums source with no affine reads nothing else)
    BnTab<BP ? CPT : 1> btb, gtb;
    rnvp_bn_src gsrc = {};
    if constexpr (BP) {
        gsrc.sums = a.bp_sums;
        gsrc.count = a.bp_bn.count;
        gsrc.shards = a.bp_shards;
        tab_issue<CPT, NT>(a.bp_bn, a.cin, 0, cs, btb);
        tab_issue<CPT, NT>(gsrc, a.cin, 0, cs, gtb);
    }
    if (epi_bn) tab_issue<1, NT>(a.epi, N, n0, BN, etb);
    const float bval = (tid < BN && a.bias && n0 + tid < N) ? a.bias[n0 + tid] : 0.f;
    EpiPre pre[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        int m, col;
        elem(e, m, col);
        epi_prefetch<T>(a, (long long)m * cso + n0 + col, m < M && n0 + col < cso, pre[e]);
    }
    stage_load(0);
    const T* wrow[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        if constexpr (FM) {
            static_assert(sizeof(T) == 2 && KS == 32, "fragment-major images are bf16");
            // row blocks >= ceil(N / 16) (clamped to block 0) only feed columns never stored
            const int nb = (n0 >> 4) + j, nbl = (N + 15) >> 4;
            wrow[j] = Wt + (long long)(nb < nbl ? nb : 0) * (a.kp >> 5) * 512 + (li + 16 * g) * CH;
        } else {
            // rows >= N (clamped to row 0) only feed output columns that are never stored
            const int row = n0 + j * 16 + li;
            wrow[j] = Wt + (long long)(row < N ? row : 0) * a.kp + g * CH;
        }
    }
    // wave wk's k-step s: tap s / NC, channel chunk (s % NC) * WK + wk of KS
    // (plain loads: buffer loads here measured slower -- the ring's waits)
    u32x4 rb[DK][TN];
    auto bload = [&](int st) {   // st is a compile-time constant after unrolling
        const int tp = st / NC, ch = st - (st / NC) * NC;
        const int k = tp * cs + (ch * WK + wk) * KS;
#pragma unroll
        for (int j = 0; j < TN; ++j) rb[st % DK][j] = *(const u32x4*)(wrow[j] + (FM ? (k >> 5) * 512 : k));
    };
#pragma unroll
    for (int u = 0; u < DK; ++u)
        if (u < NSTEP) bload(u);
    if (PRO) tab_finish<CPT, NT>(a.pro, a.cin, 0, cs, ptab, bnp, bnp + cs, nullptr, nullptr);
    if constexpr (BP) {
        // A | B | C per channel (padding channels: 0)
#pragma unroll
        for (int j = 0; j < CPT; ++j) {
            const int c = tid + NT * j;
            if (c >= cs) continue;
            float coef = 0.f, k1 = 0.f, k2 = 0.f, mo = 0.f, ro = 1.f;
            if (c < a.cin) {
                double mean, var;
                if (a.bp_bn.sums) {
                    const double s1 = btb.a1[j] + (a.bp_bn.shards > 1 ? btb.b1[j] : 0.0);
                    const double s2 = btb.a2[j] + (a.bp_bn.shards > 1 ? btb.b2[j] : 0.0);
                    mean = s1 / a.bp_bn.count;   // (rnvp_bn_bwd_apply's rounding)
                    var = s2 / a.bp_bn.count - mean * mean;
                    if (var < 0) var = 0;
                } else {
                    mean = btb.a1[j];
                    var = btb.a2[j];
                }
                ro = (float)(1.0 / sqrt(var + (double)a.bp_bn.eps));
                mo = (float)mean;
                coef = btb.gam[j] * ro;
                const double g1 = gtb.a1[j] + (a.bp_shards > 1 ? gtb.b1[j] : 0.0);
                const double g2 = gtb.a2[j] + (a.bp_shards > 1 ? gtb.b2[j] : 0.0);
                if (a.bp_bn.sums) {   // train mode: batch statistics carry gradient
                    k1 = (float)(g1 / a.bp_bn.count);
                    k2 = (float)(g2 / a.bp_bn.count);
                }
                if (vb == 0) {
                    if (a.bp_dbeta) a.bp_dbeta[c] = (float)g1;
                    if (a.bp_dgamma) a.bp_dgamma[c] = (float)g2;
                }
            }
            const double rk2 = (double)ro * (double)k2;
            bnp[c] = coef;
            bnp[cs + c] = (float)((double)coef * rk2);
            bnp[2 * cs + c] = (float)((double)coef * ((double)k1 - rk2 * (double)mo));
        }
    }
    if (epi_bn) tab_finish<1, NT>(a.epi, N, n0, BN, etb, etab, etab + BN, etab + 2 * BN, etab + 3 * BN);
    if (tid < BN) btab[tid] = bval;
    for (int c = tid * CH; c < pitch; c += NT * CH) *(u32x4*)(zrow + c) = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();
    DEEP_STAMP(1);
    if (PRO) {
#pragma unroll
        for (int e = 0; e < CH; ++e) {
            scv[e] = bnp[cfix * CH + e];
            shv[e] = bnp[cs + cfix * CH + e];
        }
    }
    if constexpr (BP) {
#pragma unroll
        for (int e = 0; e < CH; ++e) {
            bca[e] = bnp[cfix * CH + e];
            bcb[e] = bnp[cs + cfix * CH + e];
            bcc[e] = bnp[2 * cs + cfix * CH + e];
        }
    }

    // ---- act(x) rows [m0 - hal, m0 + BM + hal) -> LDS (transformed once) ----
    stage_store(0);
    for (int r0 = RSTEP * SB; r0 < R; r0 += RSTEP * SB) {
        stage_load(r0);
        stage_store(r0);
    }
    __syncthreads();
    DEEP_STAMP(2);

    // ---- per-lane pixel state of this wave's fragment rows ----
    int rowoff[TMW];     // LDS element offset of the pixel's own row (+ the lane's k-group)
    unsigned tvm[TMW];   // bit tap set iff that tap of this output pixel is inside the image
    const float rW = 1.0f / (float)W, rH = 1.0f / (float)H;
#pragma unroll
    for (int i = 0; i < TMW; ++i) {
        const int lp = (wm * TMW + i) * 16 + li, m = m0 + lp;
        rowoff[i] = (lp + hal) * pitch + g * CH;
        const int mm = m < M ? m : 0;
        const int row = fdiv_small(mm, rW);
        const int x = mm - row * W, y = row - fdiv_small(row, rH) * H;
        tvm[i] = tap_mask<KSZ>(x, y, W, H, m < M);
    }
    floatx4 acc[TMW][TN];
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    // The whole K sequence of the wave is static (taps x NC channel chunks):
    // ring slots, tap offsets and the per-tap zero-row select are resolved at
    // compile time.  DBUF: the A fragments are double-buffered -- step st+1's
    // LDS reads are issued before step st's MFMAs, and scheduling barriers
    // keep the compiler from sinking them (or the weight ring's refills) back
    // to their use; left alone it reused one fragment register, i.e. waited
    // for every LDS read right before its MFMAs.  The 8-wave 3x3 tiles with
    // the larger register footprints keep the single-buffered loop (the second
    // buffer would spill there), and so does the 4-wave 64-channel tile at
    // 1024 channels (its A double buffer spilled ~120 VGPRs into AGPRs).
    constexpr bool DBUF = KSZ == 1 || (NW == 4 ? (BN == 32 || NC <= 4) : (BN == 32 ? NC <= 2 : NC == 1));
    auto aload = [&](int st, u32x4* dst) {
        const int tp = st / NC, ch = st - (st / NC) * NC;
        const int toff = ((tp / KSZ - PAD) * W + (tp % KSZ - PAD)) * pitch + wk * KS + ch * WK * KS;
#pragma unroll
        for (int i = 0; i < TMW; ++i)
            dst[i] = *(const u32x4*)(((tvm[i] >> tp) & 1u) ? act + rowoff[i] + toff : zrow + ch * WK * KS);
    };
    if constexpr (DBUF) {
        u32x4 avb[2][TMW];
        aload(0, avb[0]);
#pragma unroll
        for (int st = 0; st < NSTEP; ++st) {
            if (st + 1 < NSTEP) aload(st + 1, avb[(st + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < TMW; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) Mf<T>::step(rb[st % DK][j], avb[st & 1][i], acc[i][j]);
            // refill this ring slot after its MFMAs (no register copies)
            if (st + DK < NSTEP) bload(st + DK);
            __builtin_amdgcn_sched_barrier(0);
        }
    } else {
#pragma unroll
        for (int st = 0; st < NSTEP; ++st) {
            u32x4 av[TMW];
            aload(st, av);
#pragma unroll
            for (int i = 0; i < TMW; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) Mf<T>::step(rb[st % DK][j], av[i], acc[i][j]);
            if (st + DK < NSTEP) bload(st + DK);
        }
    }

    DEEP_STAMP(3);
    // ---- epilogue ----
    const bool want_sums = a.out_sums || (epi_bn && a.epi_sums);
    constexpr int NS = (WK > 1 && !TALL) ? FR : TN;   // stat slots (distinct columns) per thread
    double s1[NS][4], s2[NS][4];
#pragma unroll
    for (int f = 0; f < NS; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) s1[f][r] = s2[f][r] = 0.0;
    const int grp = TALL ? wid : (WK > 1 ? wid % TM : wm);
    constexpr int GU = TALL ? NW : G;             // stat partial groups in use
    if constexpr (WK > 1) {
        // sum the WK partial tiles through LDS (aliases the activation tile)
        float* red = (float*)act;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < TMW; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                *(floatx4*)&red[(wk * BM + (wm * TMW + i) * 16 + li) * RP + j * 16 + 4 * g] = acc[i][j];
        __syncthreads();
        const int fi = wid % TM;
#pragma unroll
        for (int f = 0; f < FR; ++f) {
            int m, col;
            elem(f, m, col);
            const int n = n0 + col;
            if (m >= M || n >= cso) continue;
            const int ri = TALL ? wid + NW * (f / TN) : fi;   // the element's row group
            const int sl = TALL ? f % TN : f;                    // its stat slot
            floatx4 v = *(const floatx4*)&red[(ri * 16 + li) * RP + col];
#pragma unroll
            for (int w = 1; w < WK; ++w) v += *(const floatx4*)&red[(w * BM + ri * 16 + li) * RP + col];
            epi4p<T>(a, (long long)m * cso + n, v, btab + col, epi_bn, etab + col, BN, s1[sl], s2[sl], N - n, pre[f]);
        }
    } else {
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            int m, col;
            elem(e, m, col);
            const int n = n0 + col;
            if (m >= M || n >= cso) continue;
            epi4p<T>(a, (long long)m * cso + n, acc[e / TN][e % TN], btab + col, epi_bn, etab + col, BN, s1[e % TN],
                     s2[e % TN], N - n, pre[e]);
        }
    }
    DEEP_STAMP(4);
    if (want_sums) {
#pragma unroll
        for (int f = 0; f < NS; ++f)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double u1 = row_sum16(s1[f][r]), u2 = row_sum16(s2[f][r]);
                if (li == 0) {
                    const int cb = ((WK > 1 && !TALL) ? ((wid / TM) * FR + f) : f) * 16 + 4 * g;
                    sred[(grp * BN + cb + r) * 2] = u1;
                    sred[(grp * BN + cb + r) * 2 + 1] = u2;
                }
            }
        __syncthreads();
        double* sums = (epi_bn ? a.epi_sums : a.out_sums) + (long long)(vb % shards) * 2 * N;
        for (int col = tid; col < BN; col += NT) {
            const int n = n0 + col;
            if (n >= N) continue;
            double t1 = 0.0, t2 = 0.0;
#pragma unroll
            for (int q = 0; q < GU; ++q) {
                t1 += sred[(q * BN + col) * 2];
                t2 += sred[(q * BN + col) * 2 + 1];
            }
            atomicAdd(&sums[n], t1);
            atomicAdd(&sums[N + n], t2);
        }
    }
    DEEP_STAMP(5);
}

// Tile -> XCD order.  Every tile reads its pixel block's activation rows
// (+ halo) and its channel block's weight rows; the 8 XCD groups of
// consecutive tiles each hold ~grid/8 tiles, so pick the xa x xb block of
// pixel x channel tiles (xa | gm, xb | gn, xa * xb = grid / 8) whose unique
// bytes (xa activation tiles + xb weight slices) are smallest: that is what
// one XCD's L2 has to bring in.
inline void xcd_blocks(const rnvp_conv_args* a, int gm, int gn, int bn, int esz, int* xa, int* xb, int bm = DEEP_BM) {
    *xa = -1;
    *xb = 1;
    const long long per = (long long)gm * gn / 8;
    const int hal = (a->ks / 2) * (a->W + 1);
    const double act = (double)(bm + 2 * hal) * a->cs_in * esz;
    const double wsl = (double)bn * a->ks * a->ks * a->cs_in * esz;
    double best = 1e300;
    for (int x = 1; x <= gm; ++x) {
        if (gm % x || per % x) continue;
        const long long y = per / x;
        if (y < 1 || gn % y) continue;
        const double bytes = x * act + y * wsl;
        if (bytes < best) { best = bytes; *xa = x; *xb = (int)y; }
    }
}

}  // namespace
