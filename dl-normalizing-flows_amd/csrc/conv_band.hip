// Persistent band kernel for the wide-scale 3x3 convs (cs_in <= 64, 32 or 64
// outputs, M = 32k .. 2M pixels: scales 1-2 of the 64x64 flow).
// WeightNormConv2d (modules_realnvp.py:64-71) with the fused BN+ReLU
// prologue and the bias / residual / skip / next-BN-statistics (or dgrad
// ReLU/BN-backward) epilogue, as rnvp_conv2d's other families.
//
// One workgroup per CU walks a contiguous run of pixel bands (BM = 64*TM
// pixels, whole image rows at 64x64 / 32x32):
//   * the packed weights, the BatchNorm tables and the bias go to LDS ONCE per
//     workgroup (the one-band-per-workgroup kernel, conv.hip k_conv_band,
//     reloaded its 19-75 KB of weights for every band, in dependent rounds);
//   * bands are double buffered: band k+1's rows + halo are loaded into
//     registers before band k's MFMAs and written (BN+ReLU'd) into the other
//     LDS buffer after them -- no band load waits alone;
//   * band k's epilogue operands (residual, the previous skip sum, the dgrad
//     epilogue's pre-BN x) are loaded before its MFMAs;
//   * BatchNorm batch statistics accumulate in registers over all the
//     workgroup's bands: one fp64 atomic per channel and workgroup.
// MFMA: transposed product D[n][m] (a lane owns 4 consecutive output
// channels of one pixel), eight waves = 4 pixel groups x 2 channel halves.
#include <type_traits>

#include "common.h"
#include "conv_common.h"

namespace {

template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<N, I + 1>(f);
    }
}

// phase stamps for tools/probe/band_stamps.hip (compiled out of the product):
// [wg][16]: 0 start, 1 tables + weights in LDS, 2 first band in LDS, then per
// band k < 6: 3+2k MFMAs done, 4+2k epilogue done; 15 end
#ifdef RNVP_BAND_STAMPS
__device__ unsigned long long* g_band_stamps;
#define BAND_STAMP(i) \
    do { if (threadIdx.x == 0 && (i) < 16) g_band_stamps[blockIdx.x * 16 + (i)] = wall_clock64(); } while (0)
#else
#define BAND_STAMP(i) do {} while (0)
#endif

// HF channel groups x WPG = 8 / HF pixel groups of waves
template <typename T, int NT, int TM, int HF>
struct BandGeo {
    static constexpr int CH = Mf<T>::CH, KS = 4 * CH;
    static constexpr int NC = 16 * NT;          // output channels (padded)
    static constexpr int WPG = 8 / HF;          // pixel groups
    static constexpr int BM = 16 * TM * WPG;    // band pixels
};

template <typename T>
__host__ __device__ inline int band2_kpl(int cs) {
    constexpr int CH = Mf<T>::CH, KS = 4 * CH;
    const int nsteps = (9 * cs + KS - 1) / KS;
    return lds_mfma_pitch(nsteps * KS, CH);   // weight row pitch (conflict-free)
}

template <typename T, int NT, int TM, int HF>
size_t band2_lds_bytes(int cs, int W) {
    using G = BandGeo<T, NT, TM, HF>;
    const int ntmp = cs > G::NC ? cs : G::NC;
    const int R = G::BM + 2 * (W + 1);
    const int pitch = lds_mfma_pitch(cs, G::CH);
    return 16 * (size_t)ntmp + 8 * (size_t)cs + 20 * (size_t)G::NC + 16 * (size_t)G::WPG * G::NC +
           ((size_t)G::NC * band2_kpl<T>(cs) + (size_t)pitch + 2 * (size_t)R * pitch) * sizeof(T);
}

// raw epilogue operand of 4 channels (bf16: 8 B, f32: 16 B) and its unpack
template <typename T> struct Raw4;
template <> struct Raw4<bf16_t> {
    using type = uint2;
    __device__ static __forceinline__ void cvt(const uint2 u, float* f) {
        f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
        f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
    }
};
template <> struct Raw4<float> {
    using type = u32x4;
    __device__ static __forceinline__ void cvt(const u32x4 u, float* f) {
        f[0] = __uint_as_float(u.x); f[1] = __uint_as_float(u.y); f[2] = __uint_as_float(u.z); f[3] = __uint_as_float(u.w);
    }
};

// NOPS epilogue operand streams (residual, previous y for the skip
// accumulation, the dgrad epilogue's pre-BN x -- in that order, those present)
// CS: the input channel stride (a power of two, 8..64): the K sequence of a
// lane -- tap and channel of every k-step -- is static, the k-loop fully
// unrolled with the next step's fragments read before the current MFMAs.
// HF: channel groups of waves (1: every wave holds all NT channel tiles of
// its pixels; 2: wave pairs split them).  WREG: the wave's weight fragments
// of every k-step in registers (read from LDS once per workgroup), so the
// k-loop reads only activation fragments from LDS.
// BP: the BatchNorm-backward prologue of a data gradient (rnvp_conv_args.bp,
// conv_deep.h's form): x is the pre-apply gradient g, bp_x the BatchNorm input
// t; each staged chunk becomes dL/dt = A g - (B t + C) (coefficients from
// LDS), and a band's own rows (not its halo) are stored once to bp_out.  Half
// the staged chunks per thread per operand (the launcher checks the rows fit)
template <typename T, int NT, int TM, int CS, int HF, bool WREG, bool PRO, int NOPS, bool BP = false>
__global__ __launch_bounds__(512) void k_conv_band2(rnvp_conv_args a, int shards, int per) {
    using RT = typename Raw4<T>::type;
    using G = BandGeo<T, NT, TM, HF>;
    constexpr int CH = G::CH, KS = G::KS, NC = G::NC, BM = G::BM, WPG = G::WPG;
    static_assert((CS & (CS - 1)) == 0 && CS >= CH && CS <= 64, "channel stride");
    constexpr int NSTEP = (9 * CS + KS - 1) / KS;
    constexpr int KPL = lds_mfma_pitch(NSTEP * KS, CH);
    constexpr int NTW = NT / HF;                // channel tiles per wave
    constexpr int NTH = 512;
    static_assert(!(BP && PRO), "BatchNorm-backward prologue: data gradients only");
    constexpr int SB = BP ? 4 : 8;              // staged 16-B chunks per thread per band (checked by the launcher)
    constexpr int WB = 10;                      // weight chunks per thread (launcher: NC * kpl / CH <= WB * NTH)
    static_assert(NT % HF == 0 && (HF == 1 || HF == 2), "channel groups");
    extern __shared__ double dsm[];
    const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
    const int wid = (tid >> 6) % WPG, hf = (tid >> 6) / WPG;   // pixel group, channel group
    const int M = a.B * a.H * a.W, W = a.W, H = a.H;
    const int N = a.n;
    constexpr int cs = CS;
    constexpr int nsteps = NSTEP;
    constexpr int kpl = KPL;
    const bool epi_bn = a.epi_relu_bn_bwd != 0;
    const int ntmp = cs > NC ? cs : NC;
    const int hal = W + 1, R = BM + 2 * hal;
    constexpr int pitch = lds_mfma_pitch(CS, CH);   // band row pitch (conflict-free reads)
    const int nbands = (M + BM - 1) / BM;
    const int b0 = blockIdx.x * per, b1 = min(nbands, b0 + per);
    if (b0 >= b1) return;                       // (uniform: whole workgroup)

    double* tmp = dsm;
    float* bnp = (float*)(dsm + 2 * ntmp);      // scale | shift [cs each]
    float* etab = bnp + 2 * cs;                 // scale | shift | mean | rstd [NC each]
    float* btab = etab + 4 * NC;                // bias [NC]
    double* red = (double*)(btab + NC);         // [WPG pixel groups][NC][2]
    T* Wl = (T*)(red + 2 * WPG * NC);           // [NC][kpl]
    T* zrow = Wl + NC * kpl;                    // [pitch] zeros
    T* act0 = zrow + pitch;                     // [2][R][pitch]

    const T* __restrict__ X = (const T*)a.x;
    // cs <= 64: a row is cpr <= 16 chunks and NTH % cpr == 0 (launcher), so a
    // thread's chunk column is fixed: its BN coefficients live in registers
    constexpr int cpr = CS / CH;
    const int cfix = tid % cpr, rbase = tid / cpr;
    constexpr int rstep = NTH / cpr;
    u32x4 sv[SB];
    u32x4 sx[BP ? SB : 1];
    const T* __restrict__ XT = (const T*)a.bp_x;
    T* __restrict__ BPO = (T*)a.bp_out;
    const float* ctab = (const float*)tmp;      // BP: C [cs] (the table scratch, after the tables)
    auto stage_load = [&](int band) {
        const int m0 = band * BM;
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            if (u * rstep >= R) break;          // uniform: no thread has a row left
            const int r = rbase + u * rstep;
            const int p = m0 - hal + r;
            const bool ok = (r < R) & (p >= 0) & (p < M);
            const long long o = ok ? (long long)p * cs + cfix * CH : 0;
            sv[u] = *(const u32x4*)(X + o);
            if constexpr (BP) sx[u] = *(const u32x4*)(XT + o);
        }
    };
    float scv[CH], shv[CH];
    auto stage_store = [&](int band, T* act) {
        const int m0 = band * BM;
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            if (u * rstep >= R) break;
            const int r = rbase + u * rstep;
            if (r >= R) continue;
            const int p = m0 - hal + r;
            u32x4 w = sv[u];
            if constexpr (BP) {
                float gv[CH], tv[CH], d[CH];
                unpack(w, gv, T());
                unpack(sx[u], tv, T());
#pragma unroll
                for (int e = 0; e < CH; ++e) {
                    const int c = cfix * CH + e;
                    d[e] = fmaf(bnp[c], gv[e], -fmaf(bnp[cs + c], tv[e], ctab[c]));
                }
                w = pack(d, T());
                // the band's own rows, once (the halo rows are a neighbour band's)
                if (BPO && r >= hal && r < hal + BM && p < M) *(u32x4*)(BPO + (long long)p * cs + cfix * CH) = w;
            }
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
            const uint32_t keep = (p >= 0 && p < M) ? ~0u : 0u;
            *(u32x4*)(act + r * pitch + cfix * CH) = w & u32x4{keep, keep, keep, keep};
        }
    };

    // ---- prologue: the BN tables' shard sums first (their wait then does
    // not queue behind the bulk loads), the first band and all weights in
    // flight behind them ----
    BAND_STAMP(0);
    ShardLoads<2> pro_l, epi_l;
    const int pnv = min(cs, a.cin);
    const bool pro_pre = PRO && a.pro.sums && shard_fits(pnv, a.pro.shards, 2);
    const bool epi_pre = epi_bn && a.epi.sums && shard_fits(min(NC, N), a.epi.shards, 2);
    if (pro_pre) shard_issue<2>(a.pro.sums, a.cin, a.pro.shards, 0, pnv, pro_l);
    if (epi_pre) shard_issue<2>(a.epi.sums, N, a.epi.shards, 0, min(NC, N), epi_l);
    // BP: the BatchNorm's statistics and the gradient sums (launcher: both fit shard_issue<2>)
    ShardLoads<BP ? 2 : 1> bpb_l, bpg_l;
    if constexpr (BP) {
        shard_issue<2>(a.bp_bn.sums, a.cin, a.bp_bn.shards, 0, pnv, bpb_l);
        shard_issue<2>(a.bp_sums, a.cin, a.bp_shards, 0, pnv, bpg_l);
    }
    const BnAff bp_a = BP ? bn_aff_issue(a.bp_bn, a.cin, 0, a.w) : BnAff{1.f, 0.f};
    // the tables' affine parameters and the bias, in the same batch (no
    // global round trip left between the reductions and the first band)
    static_assert(NC <= NTH, "one table channel per thread");
    const BnAff pro_a = bn_aff_issue(a.pro, a.cin, 0, a.w);
    const BnAff epi_a = bn_aff_issue(a.epi, N, 0, a.w);
    const float bias_v = (a.bias ? a.bias : (const float*)a.w)[a.bias ? max(0, min(tid, N - 1)) : 0];
    stage_load(b0);
    const T* Wg = (const T*)a.w;
    constexpr int wcpr = KPL / CH, wtot = NC * wcpr, kv = NSTEP * KS;
    u32x4 wv[WB];
#pragma unroll
    for (int u = 0; u < WB; ++u) {
        const int q = u * NTH + tid;
        const int r = q / wcpr, c = q - r * wcpr;
        const bool ok = (q < wtot) & (r < N) & (c * CH < kv);
        wv[u] = *(const u32x4*)(Wg + (ok ? (long long)r * a.kp + c * CH : 0));
        if (!ok) wv[u] = u32x4{0u, 0u, 0u, 0u};
    }
    if (PRO) {
        if (pro_pre) {
            shard_finish<2>(pro_l, cs, tmp, tmp + cs);   // channels >= pnv stay zero (block_bn_finish pads them)
            block_bn_finish_aff(a.pro, a.cin, 0, cs, bnp, bnp + cs, nullptr, nullptr, tmp, pro_a);
        } else {
            block_bn_table(a.pro, a.cin, 0, cs, bnp, bnp + cs, nullptr, nullptr, tmp);
        }
    }
    if (epi_bn) {
        if (epi_pre) {
            shard_finish<2>(epi_l, NC, tmp, tmp + NC);
            block_bn_finish_aff(a.epi, N, 0, NC, etab, etab + NC, etab + 2 * NC, etab + 3 * NC, tmp, epi_a);
        } else {
            block_bn_table(a.epi, N, 0, NC, etab, etab + NC, etab + 2 * NC, etab + 3 * NC, tmp);
        }
    }
    if constexpr (BP) {
        // A | B -> bnp, C -> the table scratch (read by stage_store): dL/dt =
        // A g - (B t + C), A = gamma rstd, B = A rstd k2, C = A (k1 - rstd k2 mean)
        double* gsm = red;                       // [2][cs] gradient sums (red is free until the statistics)
        shard_finish<2>(bpb_l, cs, tmp, tmp + cs);
        shard_finish<2>(bpg_l, cs, gsm, gsm + cs);
        float A = 0.f, Bc = 0.f, Cc = 0.f;
        if (tid < pnv) {
            const double cnt = a.bp_bn.count, g1 = gsm[tid], g2 = gsm[cs + tid];
            const double mean = tmp[tid] / cnt;
            double var = tmp[cs + tid] / cnt - mean * mean;
            if (var < 0) var = 0;
            const float rstd = (float)(1.0 / sqrt(var + (double)a.bp_bn.eps));
            A = (a.bp_bn.gamma ? bp_a.g : 1.f) * rstd;
            const float k1 = (float)(g1 / cnt), k2 = (float)(g2 / cnt);
            const double rk2 = (double)rstd * (double)k2;
            Bc = (float)((double)A * rk2);
            Cc = (float)((double)A * ((double)k1 - rk2 * (double)(float)mean));
            if (blockIdx.x == 0) {
                if (a.bp_dbeta) a.bp_dbeta[tid] = (float)g1;
                if (a.bp_dgamma) a.bp_dgamma[tid] = (float)g2;
            }
        }
        __syncthreads();                         // every thread has read tmp / gsm
        if (tid < cs) {
            bnp[tid] = A;
            bnp[cs + tid] = Bc;
            ((float*)tmp)[tid] = Cc;
        }
    }
#pragma unroll
    for (int u = 0; u < WB; ++u) {
        const int q = u * NTH + tid;
        if (q < wtot) {
            const int r = q / wcpr, c = q - r * wcpr;
            *(u32x4*)(Wl + r * kpl + c * CH) = wv[u];
        }
    }
    if (tid < NC) btab[tid] = (a.bias && tid < N) ? bias_v : 0.f;
    for (int c = tid * CH; c < pitch; c += NTH * CH) *(u32x4*)(zrow + c) = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();
    BAND_STAMP(1);
    if (PRO) {
#pragma unroll
        for (int e = 0; e < CH; ++e) {
            scv[e] = bnp[cfix * CH + e];
            shv[e] = bnp[cs + cfix * CH + e];
        }
    }
    stage_store(b0, act0);
    const T* wl = Wl + (hf * NTW * 16 + li) * KPL + g * CH;
    u32x4 wr[WREG ? NSTEP : 1][NTW];
    if constexpr (WREG) {
#pragma unroll
        for (int st = 0; st < NSTEP; ++st)
#pragma unroll
            for (int j = 0; j < NTW; ++j) wr[st][j] = *(const u32x4*)(wl + j * 16 * KPL + st * KS);
    }
    __syncthreads();
    BAND_STAMP(2);

    const float rW = 1.0f / (float)W, rH = 1.0f / (float)H;
    const int cso = a.cs_out;
    // epilogue streams: role 0 residual, 1 previous y (skip accumulation), 2 pre-BN x
    const bool p0 = a.residual != nullptr, p1 = a.accumulate != 0;
    int role[3];
    role[0] = p0 ? 0 : (p1 ? 1 : 2);
    role[1] = (p0 && p1) ? 1 : 2;
    role[2] = 2;
    const T* opsrc[3];
#pragma unroll
    for (int q = 0; q < 3; ++q)
        opsrc[q] = role[q] == 0 ? (const T*)a.residual : (role[q] == 1 ? (const T*)a.y : (const T*)a.epi_x);
    T* __restrict__ Y = (T*)a.y;
    double s1[NTW][4], s2[NTW][4];
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) s1[j][r] = s2[j][r] = 0.0;
    // lane's K position of step st: k = st*KS + g*CH -> (tap, ci) (a chunk
    // never straddles a tap); its LDS offset from the pixel's own row and the
    // tap's bit in the in-image mask (31: K padding, never set)
    int toffl[NSTEP], tshl[NSTEP];
#pragma unroll
    for (int st = 0; st < NSTEP; ++st) {
        const int k = st * KS + g * CH, tap = k / CS, ci = k % CS;
        toffl[st] = tap < 9 ? ((tap / 3 - 1) * W + (tap % 3 - 1)) * pitch + ci : 0;
        tshl[st] = tap < 9 ? tap : 31;
    }

    for (int band = b0; band < b1; ++band) {
        const int cur = (band - b0) & 1;
        const T* act = act0 + cur * R * pitch;
        const bool more = band + 1 < b1;
        if (more) stage_load(band + 1);
        const int m0 = band * BM;
        // epilogue operands of this band, in flight under the MFMAs
        RT pre[NOPS > 0 ? NOPS : 1][TM][NTW];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < NTW; ++j) {
                const int m = m0 + wid * 16 * TM + i * 16 + li;
                const int n0 = (hf * NTW + j) * 16 + 4 * g;
                const long long o = (m < M && n0 < cso) ? (long long)m * cso + n0 : 0;
#pragma unroll
                for (int q = 0; q < NOPS; ++q) pre[q][i][j] = *(const RT*)(opsrc[q] + o);
            }
        // per-lane pixel state: LDS row of the pixel, in-image taps
        int rowoff[TM];
        unsigned tvm[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int lp = wid * 16 * TM + i * 16 + li, m = m0 + lp;
            rowoff[i] = (lp + hal) * pitch;
            const int mm = m < M ? m : 0;
            const int row = fdiv_small(mm, rW);
            const int x = mm - row * W, y = row - fdiv_small(row, rH) * H;
            tvm[i] = tap_mask<3>(x, y, W, H, m < M);
        }
        floatx4 acc[TM][NTW];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < NTW; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        // the static k-loop: step st's fragments are in registers before its
        // MFMAs, step st+1's reads issued ahead of them
        u32x4 wf[2][WREG ? 1 : NTW], av[2][TM];
        auto frag = [&](auto STC, int buf) {
            constexpr int st = decltype(STC)::value;
            if constexpr (!WREG) {
#pragma unroll
                for (int j = 0; j < NTW; ++j) wf[buf][j] = *(const u32x4*)(wl + j * 16 * KPL + st * KS);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const bool ok = (tvm[i] >> tshl[st]) & 1u;
                av[buf][i] = *(const u32x4*)(ok ? act + rowoff[i] + toffl[st] : zrow);
            }
        };
        frag(std::integral_constant<int, 0>{}, 0);
        static_for<NSTEP>([&](auto STC) {
            constexpr int st = decltype(STC)::value;
            if constexpr (st + 1 < NSTEP) frag(std::integral_constant<int, st + 1>{}, (st + 1) & 1);
            // keep the reads ahead: unfenced, the scheduler sank them to their
            // MFMAs (an LDS drain before ~40 % of the MFMAs)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < NTW; ++j) {
                    if constexpr (WREG) Mf<T>::step(wr[st][j], av[st & 1][i], acc[i][j]);
                    else Mf<T>::step(wf[st & 1][j], av[st & 1][i], acc[i][j]);
                }
            __builtin_amdgcn_sched_barrier(0);
        });
        if ((band - b0) < 6) BAND_STAMP(3 + 2 * (band - b0));
        // epilogue: lane owns channels j*16 + 4g .. +3 of its pixels
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int m = m0 + wid * 16 * TM + i * 16 + li;
            if (m >= M) continue;
#pragma unroll
            for (int j = 0; j < NTW; ++j) {
                const int n0 = (hf * NTW + j) * 16 + 4 * g;
                if (n0 >= cso) continue;
                float v[4], xv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + btab[n0 + r];
#pragma unroll
                for (int q = 0; q < NOPS; ++q) {
                    float f[4];
                    Raw4<T>::cvt(pre[q][i][j], f);
                    if (role[q] == 2) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) xv[r] = f[r];
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] += f[r];
                    }
                }
                if (epi_bn) {
                    const float* et = etab + n0;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        if (xv[r] * et[r] + et[NC + r] <= 0.f) v[r] = 0.f;
                        s1[j][r] += v[r];
                        s2[j][r] += v[r] * (xv[r] - et[2 * NC + r]) * et[3 * NC + r];
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        s1[j][r] += v[r];
                        s2[j][r] += (double)v[r] * v[r];
                    }
                }
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (n0 + r >= N) v[r] = 0.f;
                st4(Y + (long long)m * cso + n0, v);
            }
        }
        if ((band - b0) < 6) BAND_STAMP(4 + 2 * (band - b0));
        if (more) stage_store(band + 1, act0 + (cur ^ 1) * R * pitch);
        __syncthreads();
    }

    // ---- batch statistics: DPP row sums, LDS across pixel groups, sharded fp64 atomics ----
    const bool want_sums = a.out_sums || (epi_bn && a.epi_sums);
    if (want_sums) {
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double u1 = row_sum16(s1[j][r]), u2 = row_sum16(s2[j][r]);
                const int col = (hf * NTW + j) * 16 + 4 * g + r;
                if (li == 0) {
                    red[(wid * NC + col) * 2] = u1;
                    red[(wid * NC + col) * 2 + 1] = u2;
                }
            }
        __syncthreads();
        double* sums = shard_ptr(epi_bn ? a.epi_sums : a.out_sums, shards, N);
        for (int n = tid; n < N; n += NTH) {
            double t1 = 0.0, t2 = 0.0;
#pragma unroll
            for (int w = 0; w < WPG; ++w) {
                t1 += red[(w * NC + n) * 2];
                t2 += red[(w * NC + n) * 2 + 1];
            }
            atomicAdd(&sums[n], t1);
            atomicAdd(&sums[N + n], t2);
        }
    }
    BAND_STAMP(15);
}

template <typename T, int NT, int TM, int CS, int HF, bool WREG>
int launch_band2(const rnvp_conv_args* a, hipStream_t s, bool dry) {
    using G = BandGeo<T, NT, TM, HF>;
    const long long M = (long long)a->B * a->H * a->W;
    const size_t shm = band2_lds_bytes<T, NT, TM, HF>(a->cs_in, a->W);
    if (shm > 160 * 1024) return RNVP_E_UNSUPPORTED;
    // every staged row of a band in SB chunks per thread (BP: 4 per operand), every weight chunk in WB
    const int cpr = a->cs_in / G::CH;
    const int R = G::BM + 2 * (a->W + 1);
    if ((long long)R * cpr > (a->bp ? 4LL : 8LL) * 512) return RNVP_E_UNSUPPORTED;
    if ((long long)G::NC * (band2_kpl<T>(a->cs_in) / G::CH) > 10LL * 512) return RNVP_E_UNSUPPORTED;
    const long long nbands = (M + G::BM - 1) / G::BM;
    const long long grid = nbands < 256 ? nbands : 256;
    const int per = (int)((nbands + grid - 1) / grid);
    const unsigned ng = (unsigned)((nbands + per - 1) / per);
    const int sh = rnvp_stat_shards(M);
    const int nops = (a->residual ? 1 : 0) + (a->accumulate ? 1 : 0) + (a->epi_relu_bn_bwd ? 1 : 0);
    if (a->bp) {
        // a data gradient with the ReLU/BN epilogue only; the tables' shards fit shard_issue<2>
        const int pnv = a->cs_in < a->cin ? a->cs_in : a->cin;
        auto fits = [&](int sh_) { return (long long)pnv * (sh_ < 1 ? 1 : sh_) <= 2LL * 512; };
        if (a->pro_bn_relu || !a->epi_relu_bn_bwd || nops != 1 || !a->bp_bn.sums || !a->bp_sums ||
            !fits(a->bp_bn.shards) || !fits(a->bp_shards) || (a->cs_in > G::NC ? a->cs_in : G::NC) * 2 > 2 * G::WPG * G::NC)
            return RNVP_E_UNSUPPORTED;
        if (dry) return RNVP_OK;
        k_conv_band2<T, NT, TM, CS, HF, WREG, false, 1, true><<<ng, 512, shm, s>>>(*a, sh, per);
        RNVP_LAUNCH_CHECK();
        return RNVP_OK;
    }
    if (dry) return RNVP_OK;
    if (a->pro_bn_relu) {
        switch (nops) {
            case 0: k_conv_band2<T, NT, TM, CS, HF, WREG, true, 0><<<ng, 512, shm, s>>>(*a, sh, per); break;
            case 1: k_conv_band2<T, NT, TM, CS, HF, WREG, true, 1><<<ng, 512, shm, s>>>(*a, sh, per); break;
            case 2: k_conv_band2<T, NT, TM, CS, HF, WREG, true, 2><<<ng, 512, shm, s>>>(*a, sh, per); break;
            default: return RNVP_E_UNSUPPORTED;
        }
    } else {
        switch (nops) {
            case 0: k_conv_band2<T, NT, TM, CS, HF, WREG, false, 0><<<ng, 512, shm, s>>>(*a, sh, per); break;
            case 1: k_conv_band2<T, NT, TM, CS, HF, WREG, false, 1><<<ng, 512, shm, s>>>(*a, sh, per); break;
            case 2: k_conv_band2<T, NT, TM, CS, HF, WREG, false, 2><<<ng, 512, shm, s>>>(*a, sh, per); break;
            default: k_conv_band2<T, NT, TM, CS, HF, WREG, false, 3><<<ng, 512, shm, s>>>(*a, sh, per); break;
        }
    }
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

template <typename T, int CS>
int dispatch_band2_cs(const rnvp_conv_args* a, hipStream_t s, bool dry) {
    const long long M = (long long)a->B * a->H * a->W;
    const long long b256 = (M + 255) / 256;
    if (a->bp) {   // the prologue's staging at half width per operand: the weights stay in registers
        constexpr bool WRB = CS <= 32;
        if (a->n <= 32) {
            if (b256 >= 512) return launch_band2<T, 2, 2, CS, 1, WRB>(a, s, dry);
            return launch_band2<T, 2, 1, CS, 1, WRB>(a, s, dry);
        }
        return launch_band2<T, 4, 2, CS, 2, false>(a, s, dry);
    }
    // <= 32 outputs: every wave holds both channel tiles of its pixels and
    // the weights in registers (k-loop LDS reads: the activation fragments
    // only); 256-pixel bands while that leaves >= 2 bands per workgroup.
    // 64 outputs: wave pairs split the channels, weights read from LDS per
    // step (in registers they would take 144 VGPRs).
    constexpr bool WR = CS <= 32;   // 36-72 VGPRs of weights (64 channels: 144)
    if (a->n <= 32) {
        if (b256 >= 512) return launch_band2<T, 2, 2, CS, 1, WR>(a, s, dry);
        return launch_band2<T, 2, 1, CS, 1, WR>(a, s, dry);
    }
    return launch_band2<T, 4, 2, CS, 2, false>(a, s, dry);
}

template <typename T>
int dispatch_band2(const rnvp_conv_args* a, hipStream_t s, bool dry) {
    switch (a->cs_in) {
        case 8: return dispatch_band2_cs<T, 8>(a, s, dry);
        case 16: return dispatch_band2_cs<T, 16>(a, s, dry);
        case 32: return dispatch_band2_cs<T, 32>(a, s, dry);
        case 64: return dispatch_band2_cs<T, 64>(a, s, dry);
        default: return RNVP_E_UNSUPPORTED;
    }
}

}  // namespace

// 3x3, 17..64 outputs, cs_in <= 64 with a fixed chunk column per thread,
// 32k <= M < 2^21: the persistent band kernel (RNVP_E_UNSUPPORTED otherwise)
int rnvp_conv_band2_launch(const rnvp_conv_args* a, hipStream_t s, bool dry) {
    const long long M = (long long)a->B * a->H * a->W;
    if (a->ks != 3 || a->n <= 16 || a->n > 64 || a->cs_in > 64 || a->cs_out > 64) return RNVP_E_UNSUPPORTED;
    if (M < 32768 || M >= (1ll << 21)) return RNVP_E_UNSUPPORTED;
    // bf16 (the fp32 parity mode keeps the one-band-per-workgroup kernel)
    if (a->dtype != RNVP_BF16) return RNVP_E_UNSUPPORTED;
    return dispatch_band2<bf16_t>(a, s, dry);
}
