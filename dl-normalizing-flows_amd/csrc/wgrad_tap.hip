// Grouped weight gradients of one coupling's s/t-net convs, bf16, tap-shared
// (modules_realnvp.py:36-71 WeightNormConv2d backward, for every conv of a
// ResidualModule in one launch).
//
//   dW[co][t*cs_in + ci] = sum_p dy[p][co] * act(x)[p + off(t)][ci]     (+ bias: sum_p dy[p][co])
//
// The round-2 kernel (conv.hip k_wgrad_grouped) gave every tap of a 3x3 its own
// 64x64 (co x k) tile: the activation rows were re-read, re-decoded and
// re-transformed (BN+ReLU) once per tap and per co tile, and each 64-pixel
// stage cost ~350 VALU instructions against 8 MFMAs (PMC: 4.7 % MFMA busy).
// Here a workgroup owns a (co tile) x (ci tile) x ALL taps block:
//   * per stage of 128 output pixels (whole image rows) the dy rows and the
//     activation rows + halo are staged ONCE in LDS, the activations BN+ReLU'd
//     once and laid out as zero-padded image rows ((W+2) columns, a zero row
//     above and below every image): every tap reads its operand at a fixed
//     row offset with no border masks;
//   * MFMA operands come from LDS by ds_read_b64_tr_b16 (8 pixels of one
//     channel per lane), one A fragment (dy^T) serving all 9 taps;
//   * the next stage's global loads are in flight under the current stage's
//     MFMAs (register staging, one stage ahead; one barrier per stage);
//   * the bias gradient rides on the MFMAs (dy^T x a ones fragment).
// Output: the same packed fp32 slabs / replicas as k_wgrad_grouped (plain
// stores when every slab has its replica, atomics otherwise), summed by the
// weight-norm backward.
#include "common.h"
#include "conv_common.h"

#include <type_traits>

namespace {

// compile-time loop: f(std::integral_constant<int, i>) for i = 0 .. N-1
template <int I, int N, typename F>
__device__ __forceinline__ void static_for_impl(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for_impl<I + 1, N>(f);
    }
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) { static_for_impl<0, N>(f); }

constexpr int WT_NT = 512;     // 8 waves
#ifndef WT_C0_DEPTH
#define WT_C0_DEPTH 1   // 2 (per-tap B fragments, a second stage in flight) measured slower: profiles/r3_experiments.txt
#endif
constexpr int WT_SP = 128;     // output pixels per stage: 4 MFMA k-steps of 32
constexpr int WT_KST = WT_SP / 32;

// tile classes: (co tile, ci tile, kernel size, waves over co, waves over ci,
template <int C> struct WtCfg;
// tap groups, x chunks per thread per stage, stages of global loads in flight)
// BALL: every B fragment of a k-step read before its MFMAs (one LDS wait) or
// each tap's fragment right before that tap's MFMAs (32 fewer VGPRs for the
// 3x3 class, spent on a second stage of global loads in flight)
template <> struct WtCfg<0> { static constexpr int TCO = 64, TCI = 64, KS = 3, WCO = 2, WCI = 4, WTG = 1, NX = 5, DEPTH = WT_C0_DEPTH, BALL = WT_C0_DEPTH == 1; };
template <> struct WtCfg<1> { static constexpr int TCO = 128, TCI = 128, KS = 1, WCO = 2, WCI = 4, WTG = 1, NX = 4, DEPTH = 1, BALL = 1; };
#ifndef WT_SMALL_DEPTH
// stages of loads in flight for the wide scales' 32 / 64-channel classes (3
// measured no step change: 19.60 vs 19.58 ms, gpurun_out/r6_wgd3 -- the stage
// loop is not load-latency bound)
#define WT_SMALL_DEPTH 2
#endif
#ifndef WT_BALANCE
// one-class launches in atomic mode re-slab for the device's slots (wt_balance)
#define WT_BALANCE 1
#endif
#ifndef WT_WG_OVERHEAD
#define WT_WG_OVERHEAD 2    // a workgroup's table prologue + epilogue, in stages
#endif
#ifndef WT_MIN_STAGES
#define WT_MIN_STAGES 4
#endif
#ifndef WT_SPLIT_MIN_M
// mixed-class groups over at least this many pixels launch per class (below;
// config 1: scales 1-2, 19.35 -> 19.11 ms/step; from 262144: 19.16; every
// size: 19.80 -- the deep scales' small launches lose, gpurun_out/splitab)
#define WT_SPLIT_MIN_M 65536
#endif
template <> struct WtCfg<2> { static constexpr int TCO = 32, TCI = 32, KS = 3, WCO = 2, WCI = 2, WTG = 2, NX = 4, DEPTH = WT_SMALL_DEPTH, BALL = 1; };
template <> struct WtCfg<3> { static constexpr int TCO = 64, TCI = 64, KS = 1, WCO = 2, WCI = 4, WTG = 1, NX = 2, DEPTH = WT_SMALL_DEPTH, BALL = 1; };

inline int wt_class_base(int ks, int cs_in, int cs_dy) {
    if (ks == 3) return (cs_in <= 32 && cs_dy <= 32) ? 2 : 0;
    return (cs_in <= 64 && cs_dy <= 64) ? 3 : 1;
}
__host__ __device__ inline int wt_tco(int c) { return c == 1 ? 128 : (c == 2 ? 32 : 64); }
__host__ __device__ inline int wt_tci(int c) { return c == 1 ? 128 : (c == 2 ? 32 : 64); }
__host__ __device__ inline int wt_ks(int c) { return (c == 0 || c == 2) ? 3 : 1; }
// bytes per LDS row.  KO (the consecutive-row k order, wt_krow): an odd
// number of 32-byte granules, so that the 8 consecutive rows one
// ds_read_b64_tr_b16 half-wave reads land in 8 distinct 32-byte bank groups
// for any starting row; otherwise (the identity order, when the wider rows do
// not fit LDS) +16 B
__host__ __device__ inline int wt_pitch(int t, bool ko) { return t * 2 + (ko ? 32 : 16); }
// padded rows a stage of rs output rows can touch (image boundaries add 2 each)
__host__ __device__ inline int wt_npr(int rs, int H) { return rs + 2 + 2 * ((rs - 1 + H - 1) / H); }

__host__ __device__ inline size_t wt_stage_bytes(int c, int H, int W, bool ko) {
    const int tco = wt_tco(c), tci = wt_tci(c);
    const size_t dy = (size_t)WT_SP * wt_pitch(tco, ko);
    size_t x;
    if (wt_ks(c) == 1) x = (size_t)WT_SP * wt_pitch(tci, ko);
    else x = (size_t)wt_npr(WT_SP / W, H) * (W + 2) * wt_pitch(tci, ko);
    return dy + x;
}
// 2 stages; the prologue's BN table + fp64 scratch (24 B per ci) alias the
// second stage buffer, which is first written after the barrier that follows
// every thread's table read (so the 1x1 64-channel class fits two
// workgroups per CU: 2 x 80 KB)
#ifndef WT_TABLE_ALIAS
#define WT_TABLE_ALIAS 1
#endif
__host__ __device__ inline size_t wt_lds_bytes(int c, int H, int W, bool ko) {
    return 2 * wt_stage_bytes(c, H, W, ko) + (WT_TABLE_ALIAS ? 0 : 24 * (size_t)wt_tci(c));
}

// the k -> pixel order of one 32-pixel k-step: lane group gq's B/A fragment
// takes k = 8gq .. 8gq+7 as two transposed 4-row reads (lo, hi); k is any
// permutation of the step's pixels as long as both operands use the same one.
// KO: a half-wave's lo read covers 8 CONSECUTIVE pixel rows (pixels
// 16*(gq/2) + 4*(gq%2) + 0..3) and its hi read the next 8 (+8) -- with an odd
// granule pitch (wt_pitch) every read is bank-conflict-free; the identity
// order (rows r..r+3 and r+8..r+11 per half-wave) is 2-way on any linear pitch
template <bool KO>
__device__ __forceinline__ int wt_krow(int gq, int qq) { return KO ? 16 * (gq >> 1) + 4 * (gq & 1) + qq : 8 * gq + qq; }
template <bool KO>
constexpr int wt_khi() { return KO ? 8 : 4; }   // rows from a lane's lo read to its hi read

template <bool KO>
__device__ __forceinline__ u32x4 tr_pair(const RNVP_LDS char* base, int pitch) {
    const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RNVP_LDS i16x4*)base);
    const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RNVP_LDS i16x4*)(base + wt_khi<KO>() * pitch));
    const uint2 l = __builtin_bit_cast(uint2, lo), h = __builtin_bit_cast(uint2, hi);
    return u32x4{l.x, l.y, h.x, h.y};
}

// the fields of one conv a block needs, by value (a reference into the
// by-value group argument would be indexed dynamically from scratch)
struct WtConv {
    const void* x; const void* dy; float* ws; float* wsb;
    rnvp_bn_src pro;
    int cs_in, cin, cs_dy, n, kp, pro_bn_relu, nz, nrep, B, H, W;
    long long m_per_slab;
};

template <int CLS, bool KO>
__device__ __forceinline__ void wt_body(const WtConv& cv, int cot, int cit, int z, char* lds) {
    using Cfg = WtCfg<CLS>;
    constexpr int TCO = Cfg::TCO, TCI = Cfg::TCI, KS = Cfg::KS, T = KS * KS;
    constexpr int WCO = Cfg::WCO, WCI = Cfg::WCI, WTG = Cfg::WTG, NX = Cfg::NX, DEPTH = Cfg::DEPTH;
    constexpr int FCO = TCO / (16 * WCO), FCI = TCI / (16 * WCI);
    constexpr int TPW = (T + WTG - 1) / WTG;                    // taps per wave
    constexpr int DP = TCO * 2 + (KO ? 32 : 16), XP = TCI * 2 + (KO ? 32 : 16);   // LDS row pitches (bytes, wt_pitch)
    constexpr int CPO = TCO / 8, CPI = TCI / 8;                 // 16-byte chunks per row
    constexpr int NDY = WT_SP * CPO / WT_NT;
    static_assert(WCO * WCI * WTG * 64 == WT_NT, "wave layout");
    static_assert(NDY * WT_NT == WT_SP * CPO && WT_NT % CPI == 0, "chunk layout");

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wg = wid % WTG, wci = (wid / WTG) % WCI, wco = wid / (WTG * WCI);
    const int gq = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
    const int H = cv.H, W = cv.W, Bn = cv.B;
    const long long M = (long long)Bn * H * W;
    const int cs = cv.cs_in, csd = cv.cs_dy, N = cv.n;
    const int co0 = cot * TCO, ci0 = cit * TCI;
    const long long mb = (long long)z * cv.m_per_slab;
    const long long me = (mb + cv.m_per_slab < M) ? mb + cv.m_per_slab : M;
    const int ns = mb < me ? (int)((me - mb + WT_SP - 1) / WT_SP) : 0;
    const int PW = KS == 3 ? W + 2 : 0;
    const int RS = WT_SP / W;                                   // output rows per stage (launcher: W | 128)
    // stage alignment (uniform; 3x3 classes): 1 = every stage lies inside one
    // image (H*W % WT_SP == 0), 2 = every stage is whole images (WT_SP %
    // H*W == 0), 0 = general.  Aligned stages have one padded layout: a
    // chunk's pixel offset from the stage start and its column validity are
    // stage-invariant (computed once below), and so are the lanes' LDS
    // positions in compute(); they also stage exactly the rows they read (RS
    // + 2 per image), wt_npr's bound covers any stage
    const int HWi = H * W;
    const int al = KS == 3 ? (HWi % WT_SP == 0 ? 1 : (WT_SP % HWi == 0 ? 2 : 0)) : 0;
    const int NPR = KS == 3 ? (al == 1 ? RS + 2 : (al == 2 ? RS + 2 * (RS / H) : wt_npr(RS, H))) : 0;
    const int xrows = KS == 3 ? NPR * PW : WT_SP;               // staged x positions per stage
    const int xtot = xrows * CPI;                               // x chunks per stage
    const unsigned sbytes = (unsigned)wt_stage_bytes(CLS, H, W, KO);
    float* bnp = (float*)(lds + (WT_TABLE_ALIAS ? 1 : 2) * sbytes);                      // scale [TCI] | shift [TCI] | fp64 scratch [2 TCI] (stage buffer 1)
    // LDS-space base: stage addresses in 32-bit arithmetic (generic-pointer
    // offsets compiled to 64-bit multiply-adds per operand read)
    RNVP_LDS char* const L3 = (RNVP_LDS char*)lds;
    const bool pro = cv.pro_bn_relu != 0;

    // ---- BN+ReLU table of this ci tile (channels >= cin: scale = shift = 0) ----
    if (pro) block_bn_table(cv.pro, cv.cin, ci0, TCI, bnp, bnp + TCI, nullptr, nullptr, (double*)(bnp + 2 * TCI));
    __syncthreads();
    const int cch = tid % CPI;                                  // this thread's x channel chunk (fixed)
    float sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        sc[e] = pro ? bnp[cch * 8 + e] : 1.f;
        sh[e] = pro ? bnp[TCI + cch * 8 + e] : 0.f;
    }
    const bool xcol_ok = ci0 + cch * 8 < cs;
    const int dch = tid % CPO;                                  // this thread's dy channel chunk (fixed)
    const bool dcol_ok = co0 + dch * 8 < csd;
    const float rPW = KS == 3 ? 1.0f / (float)PW : 0.f, rH2 = 1.0f / (float)(H + 2);   // PW, H+2 > 0
    const float rW = 1.0f / (float)W, rH = 1.0f / (float)H;

    // buffer resources: an out-of-range offset (invalid pixel / channel chunk)
    // returns zeros without a memory access
    const __amdgpu_buffer_rsrc_t XR = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(cv.x), 0, (int)((long long)M * cs * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t DR = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(cv.dy), 0, (int)((long long)M * csd * 2), 0x00020000);
    constexpr int OOB = 0x7ffffff0;
    u32x4 rx[DEPTH][NX], rd[DEPTH][NDY];
    unsigned xm[DEPTH];                                         // x chunk validity (the transform of 0 is not 0)
    // stage-invariant part of this thread's x chunks: padded (row slot, column)
    int xjp[NX];
#pragma unroll
    for (int u = 0; u < NX; ++u) {
        const int q = tid + u * WT_NT, pos = q / CPI;
        if constexpr (KS == 3) {
            const int j = fdiv_small(pos, rPW);
            xjp[u] = (q < xtot) ? (j << 8) | (pos - j * PW) : -1;      // PW <= 130
        } else {
            xjp[u] = (q < xtot) ? pos : -1;
        }
    }

    int xrel[NX], xrow[NX];
    unsigned xinv = 0;                                          // al 1: column ok; al 2: slot holds a pixel
    if constexpr (KS == 3) {
#pragma unroll
        for (int u = 0; u < NX; ++u) {
            const int j = xjp[u] >> 8, pc = xjp[u] & 255;
            const bool colok = (xjp[u] >= 0) & (pc >= 1) & (pc <= W) & xcol_ok;
            if (al == 1) {
                xrel[u] = (j - 1) * W + pc - 1;
                xrow[u] = j - 1;                                // image row = stage's first row + xrow
                xinv |= (unsigned)colok << u;
            } else {
                const int bb = fdiv_small(j, rH2), yy = j - bb * (H + 2) - 1;
                xrel[u] = (bb * H + yy) * W + pc - 1;
                xrow[u] = 0;
                xinv |= (unsigned)(colok & (yy >= 0) & (yy < H)) << u;
            }
        }
    }

    // global loads of stage s into register slot SL
    auto gload = [&](int s, auto SLC) {
        constexpr int SL = decltype(SLC)::value;
        const int p0 = (int)(mb + (long long)s * WT_SP);
#pragma unroll
        for (int u = 0; u < NDY; ++u) {
            const int p = p0 + (tid + u * WT_NT) / CPO;
            const bool ok = (p < me) & dcol_ok;
            rd[SL][u] = __builtin_amdgcn_raw_buffer_load_b128(DR, ok ? (p * csd + co0 + dch * 8) * 2 : OOB, 0, 0);
        }
        unsigned m = 0;
        if constexpr (KS == 1) {
#pragma unroll
            for (int u = 0; u < NX; ++u) {
                const int p = p0 + xjp[u];
                const bool ok = (xjp[u] >= 0) & (p < me) & xcol_ok;
                rx[SL][u] = __builtin_amdgcn_raw_buffer_load_b128(XR, ok ? (p * cs + ci0 + cch * 8) * 2 : OOB, 0, 0);
                m |= (unsigned)ok << u;
            }
        } else if (al) {
            // aligned stages: p0 + the chunk's invariant offset; al 1 also
            // checks the row against the image (first / last stage of an
            // image).  The halo rows are bounded by the tensor, not by the
            // slab: a slab may end inside an image, and the row below its
            // last stage belongs to the next slab's pixels (bounding it by
            // the slab's end dropped that row's tap contributions: ~7 % of
            // the 3x3 weight gradient at 64x64 images, 2048-pixel slabs)
            const int om = (p0 / W) % H;
#pragma unroll
            for (int u = 0; u < NX; ++u) {
                const bool rowok = al == 2 || (unsigned)(om + xrow[u]) < (unsigned)H;
                const bool ok = ((xinv >> u) & 1u) & rowok & (p0 + xrel[u] < M);
                rx[SL][u] = __builtin_amdgcn_raw_buffer_load_b128(XR, ok ? ((p0 + xrel[u]) * cs + ci0 + cch * 8) * 2 : OOB,
                                                                  0, 0);
                m |= (unsigned)ok << u;
            }
        } else {
            // padded row G of slot j: G = gs + j, gs = G(o0) - 1 where G(o) =
            // o + 2 (o / H) + 1 is the padded row of output row o (a zero row
            // above and below every image; p0 is row aligned)
            const int o0 = p0 / W;
            const int gs = o0 + 2 * fdiv_small(o0, rH);
#pragma unroll
            for (int u = 0; u < NX; ++u) {
                const int j = xjp[u] >> 8, pc = xjp[u] & 255;
                const int G = gs + j;                             // < 2^22 (launcher)
                const int bb = fdiv_small(G, rH2);
                const int yy = G - bb * (H + 2) - 1, xx = pc - 1;
                const bool ok = (xjp[u] >= 0) & (bb < Bn) & (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W) & xcol_ok;
                const int pix = (bb * H + yy) * W + xx;
                rx[SL][u] = __builtin_amdgcn_raw_buffer_load_b128(XR, ok ? (pix * cs + ci0 + cch * 8) * 2 : OOB, 0, 0);
                m |= (unsigned)ok << u;
            }
        }
        xm[SL] = m;
    };
    // transform + store of register slot SL into LDS buffer buf
    auto lstore = [&](int buf, auto SLC) {
        constexpr int SL = decltype(SLC)::value;
        RNVP_LDS char* dyL = L3 + buf * sbytes;
        RNVP_LDS char* xL = dyL + WT_SP * DP;
#pragma unroll
        for (int u = 0; u < NDY; ++u) {
            const int r = (tid + u * WT_NT) / CPO;
            *(RNVP_LDS u32x4*)(dyL + r * DP + dch * 16) = rd[SL][u];
        }
#pragma unroll
        for (int u = 0; u < NX; ++u) {
            if (xjp[u] < 0) continue;
            const int pos = (tid + u * WT_NT) / CPI;
            u32x4 v = rx[SL][u];
            if (pro) {
                v = bn_relu_bf16x8(v, sc, sh);
                const uint32_t k = ((xm[SL] >> u) & 1u) ? ~0u : 0u;
                v &= u32x4{k, k, k, k};
            }
            *(RNVP_LDS u32x4*)(xL + pos * XP + cch * 16) = v;
        }
    };

    floatx4 acc[FCO][FCI][TPW];
    floatx4 bacc[FCO];
#pragma unroll
    for (int a = 0; a < FCO; ++a) {
        bacc[a] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b = 0; b < FCI; ++b)
#pragma unroll
            for (int t = 0; t < TPW; ++t) acc[a][b][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    const bool do_bias = cv.wsb != nullptr && cit == 0 && wci == 0 && wg == 0;
    const u32x4 ones = u32x4{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};   // bf16 1.0 x 8
    // per-tap LDS row offsets (positions) of this wave's taps
    int toff[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        const int tap = wg * TPW + t;
        toff[t] = KS == 3 ? ((tap / 3 - 1) * PW + (tap % 3 - 1)) : 0;
    }

    // this lane's LDS x positions (pixel rows lo, hi = lo + wt_khi) per k-step
    // of a stage whose first output row is o0: pixel j sits in output row
    // o0 + j / W, column j % W; its slot = rows since o0 + 2 per image
    // boundary crossed + 1 (aligned stages: the same for every stage)
    auto positions = [&](int o0, int* plo, int* phi) {
        if constexpr (KS == 1) {
#pragma unroll
            for (int kk = 0; kk < WT_KST; ++kk) {
                plo[kk] = kk * 32 + wt_krow<KO>(gq, qq);
                phi[kk] = plo[kk] + wt_khi<KO>();
            }
        } else {
            const int ob0 = fdiv_small(o0, rH);
            auto posof = [&](int j) {
                const int jr = fdiv_small(j, rW), xx = j - jr * W;
                const int ob = fdiv_small(o0 + jr, rH);
                return (jr + 2 * (ob - ob0) + 1) * PW + xx + 1;
            };
#pragma unroll
            for (int kk = 0; kk < WT_KST; ++kk) {
                plo[kk] = posof(kk * 32 + wt_krow<KO>(gq, qq));
                phi[kk] = posof(kk * 32 + wt_krow<KO>(gq, qq) + wt_khi<KO>());
            }
        }
    };
    int plo_a[WT_KST], phi_a[WT_KST];
    positions(0, plo_a, phi_a);   // aligned (al != 0) and 1x1 stages

    // MFMAs of the stage in LDS buffer cur (stage s)
    auto compute = [&](int s, int cur) {
        const RNVP_LDS char* dyL = L3 + cur * sbytes;
        const RNVP_LDS char* xL = dyL + WT_SP * DP;
        int plo[WT_KST], phi[WT_KST];
        if (KS == 1 || al) {
#pragma unroll
            for (int kk = 0; kk < WT_KST; ++kk) {
                plo[kk] = plo_a[kk];
                phi[kk] = phi_a[kk];
            }
        } else {
            positions((int)((mb + (long long)s * WT_SP) / W), plo, phi);
        }
#pragma unroll
        for (int kk = 0; kk < WT_KST; ++kk) {
            const int jl = kk * 32 + wt_krow<KO>(gq, qq);         // dy pixel rows of this lane (lo; hi = + wt_khi)
            u32x4 af[FCO];
#pragma unroll
            for (int a = 0; a < FCO; ++a)
                af[a] = tr_pair<KO>(dyL + jl * DP + (wco * FCO * 16 + a * 16 + 4 * pp) * 2, DP);
            // per k-step lane bases; taps add a uniform offset
            const RNVP_LDS char* xlo = xL + plo[kk] * XP + (wci * FCI * 16 + 4 * pp) * 2;
            const RNVP_LDS char* xhi = xL + phi[kk] * XP + (wci * FCI * 16 + 4 * pp) * 2;
            auto bfrag = [&](int b, int t) {
                const int off = toff[t] * XP + b * 32;
                const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RNVP_LDS i16x4*)(xlo + off));
                const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RNVP_LDS i16x4*)(xhi + off));
                const uint2 l = __builtin_bit_cast(uint2, lo), h = __builtin_bit_cast(uint2, hi);
                return u32x4{l.x, l.y, h.x, h.y};
            };
            if (do_bias) {
#pragma unroll
                for (int a = 0; a < FCO; ++a) Mf<bf16_t>::step(af[a], ones, bacc[a]);
            }
            if constexpr (Cfg::BALL) {
                // every B fragment of the k-step is read before the MFMAs (one LDS wait)
                u32x4 bfr[FCI][TPW];
#pragma unroll
                for (int b = 0; b < FCI; ++b)
#pragma unroll
                    for (int t = 0; t < TPW; ++t)
                        if (wg * TPW + t < T) bfr[b][t] = bfrag(b, t);
#pragma unroll
                for (int b = 0; b < FCI; ++b)
#pragma unroll
                    for (int t = 0; t < TPW; ++t) {
                        if (wg * TPW + t >= T) continue;
#pragma unroll
                        for (int a = 0; a < FCO; ++a) Mf<bf16_t>::step(af[a], bfr[b][t], acc[a][b][t]);
                    }
            } else {
#pragma unroll
                for (int b = 0; b < FCI; ++b)
#pragma unroll
                    for (int t = 0; t < TPW; ++t) {
                        if (wg * TPW + t >= T) continue;
                        const u32x4 bf = bfrag(b, t);
#pragma unroll
                        for (int a = 0; a < FCO; ++a) Mf<bf16_t>::step(af[a], bf, acc[a][b][t]);
                    }
            }
        }
    };

    // stage pipeline: DEPTH stages of global loads in flight (register slots
    // s % DEPTH), LDS double buffer (s & 1), one barrier per stage
    using I0 = std::integral_constant<int, 0>;
    static_for<DEPTH>([&](auto D) {
        constexpr int d = decltype(D)::value;
        if (d < ns) gload(d, D);
    });
    if (ns > 0) lstore(0, I0{});
    __syncthreads();
    auto iter = [&](int s, auto SLC) {
        constexpr int SL = decltype(SLC)::value;                   // slot of stage s (free: stored already)
        constexpr int SN = (SL + 1) % DEPTH;                       // slot of stage s + 1
        if (s + DEPTH < ns) gload(s + DEPTH, std::integral_constant<int, SL>{});
        compute(s, s & 1);
        if (s + 1 < ns) lstore((s + 1) & 1, std::integral_constant<int, SN>{});
        __syncthreads();
    };
    for (int s = 0; s < ns; s += DEPTH) {
        static_for<DEPTH>([&](auto D) {
            constexpr int d = decltype(D)::value;
            if (s + d < ns) iter(s + d, D);
        });
    }

    // ---- epilogue: D rows = co, cols = ci; k = tap * cs_in + ci ----
    const int rep = z % cv.nrep;
    const bool atomic = cv.nrep < cv.nz;
    float* out = cv.ws + (long long)rep * N * cv.kp;
#pragma unroll
    for (int a = 0; a < FCO; ++a)
#pragma unroll
        for (int b = 0; b < FCI; ++b)
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
                const int tap = wg * TPW + t;
                if (tap >= T) continue;
                const int ci = ci0 + wci * FCI * 16 + b * 16 + li;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int co = co0 + wco * FCO * 16 + a * 16 + gq * 4 + r;
                    if (co < N && ci < cs) {
                        float* o = out + (long long)co * cv.kp + tap * cs + ci;
                        if (atomic) atomicAdd(o, acc[a][b][t][r]);
                        else *o = acc[a][b][t][r];
                    }
                }
            }
    if (do_bias && li == 0) {
        float* bo = cv.wsb + (long long)rep * N;
#pragma unroll
        for (int a = 0; a < FCO; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = co0 + wco * FCO * 16 + a * 16 + gq * 4 + r;
                if (co < N) {
                    if (atomic) atomicAdd(bo + co, bacc[a][r]);
                    else bo[co] = bacc[a][r];
                }
            }
    }
}

// block -> (conv, slab, co tile, ci tile); consecutive tasks (one slab's tiles,
// which share the slab's pixels through L2) go to one XCD.  One kernel per
// tile class (every conv of the launch has class CLS): each class gets its
// own register allocation (the 1x1 classes fit more waves per SIMD than the
// 3x3 ones; one kernel over all classes took the largest class's 207 VGPRs)
template <int CLS, bool KO>
__global__ __launch_bounds__(WT_NT) void k_wgrad_tap(rnvp_wgrad_group g) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int nb = gridDim.x, b = blockIdx.x;
    const int q = nb / 8, r = nb % 8, xcd = b % 8;
    const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
    int c = 0;
    while (c + 1 < g.n_conv && g.conv[c + 1].task0 <= t) ++c;
    const rnvp_wgrad_conv& gc = g.conv[c];
    const WtConv cv{gc.x, gc.dy, gc.ws, gc.wsb, gc.pro, gc.cs_in, gc.cin, gc.cs_dy, gc.n, gc.kp, gc.pro_bn_relu,
                    gc.nz, gc.nrep, g.B, g.H, g.W, gc.m_per_slab};
    const int cls = CLS >= 0 ? CLS : gc.cls;
    const int tco = (gc.n + wt_tco(cls) - 1) / wt_tco(cls), tci = gc.tk;
    const int local = t - gc.task0;
    const int per = tco * tci;
    const int z = local / per, rr = local - z * per;
    const int cot = rr / tci, cit = rr - cot * tci;
    if constexpr (CLS >= 0) {
        wt_body<CLS, KO>(cv, cot, cit, z, lds);
    } else {
        switch (cls) {
            case 0: wt_body<0, KO>(cv, cot, cit, z, lds); break;
            case 1: wt_body<1, KO>(cv, cot, cit, z, lds); break;
            case 2: wt_body<2, KO>(cv, cot, cit, z, lds); break;
            default: wt_body<3, KO>(cv, cot, cit, z, lds); break;
        }
    }
}

using WtKernel = void (*)(rnvp_wgrad_group);
WtKernel wt_kernel(int cls, bool ko) {
    switch (cls) {
        case 0: return ko ? k_wgrad_tap<0, true> : k_wgrad_tap<0, false>;
        case 1: return ko ? k_wgrad_tap<1, true> : k_wgrad_tap<1, false>;
        case 2: return ko ? k_wgrad_tap<2, true> : k_wgrad_tap<2, false>;
        case 3: return ko ? k_wgrad_tap<3, true> : k_wgrad_tap<3, false>;
        default: return ko ? k_wgrad_tap<-1, true> : k_wgrad_tap<-1, false>;
    }
}

// x staging of a 3x3 class fits its NX chunks per thread
bool wt_stage_fits(int cls, int H, int W) {
    if (wt_ks(cls) != 3) return true;
    const int npr = wt_npr(WT_SP / W, H);
    const int cpi = wt_tci(cls) / 8;
    const int nx = cls == 0 ? WtCfg<0>::NX : WtCfg<2>::NX;   // class 0: W = 128 (config 4 scale 1) falls back
    return (long long)npr * (W + 2) * cpi <= (long long)nx * WT_NT;
}

long long wt_tasks(const rnvp_wgrad_conv& v, int cls) {
    return (long long)v.nz * ((v.n + wt_tco(cls) - 1) / wt_tco(cls)) * ((v.cs_in + wt_tci(cls) - 1) / wt_tci(cls));
}

// tile class of a conv: by channel count (the widest tiles, fewest operand
// re-reads; the 32 x 32 / 64 x 64 tiles for the deep scales' small convs
// were faster alone and slower in the grouped step launch,
// profiles/r4_wgrad_ab.txt)
int wt_class(const rnvp_wgrad_conv& v, int H, int W) { return wt_class_base(v.ks, v.cs_in, v.cs_dy); }

// compute units of the current device (queried once, before any capture: the
// first launch is a warm-up step)
int wt_cus() {
    static int n = 0;
    if (n == 0) {
        int d = 0, v = 0;
        n = (hipGetDevice(&d) == hipSuccess &&
             hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && v > 0) ? v : 256;
    }
    return n;
}

// workgroups of a class kernel resident per CU: registers (the 3x3 and
// 128-wide classes take > 128 VGPRs: 2 waves per SIMD = one 8-wave
// workgroup; the 1x1 64-wide class 108) and LDS
int wt_wg_per_cu(int cls, size_t lds) {
    const int reg = cls == 3 ? 2 : 1;
    const int l = lds > 0 ? (int)((160 * 1024) / lds) : reg;
    return l < reg ? (l < 1 ? 1 : l) : reg;
}

// Slab size of a one-class launch whose convs accumulate atomically into
// their replicas (nrep < nz: the slab count is then free): the stages per
// slab that minimise rounds x (stages + WT_WG_OVERHEAD) over the device's
// resident-workgroup slots.  The engine's 2048-pixel slabs leave scale 2's
// 3x3 launch at 160 workgroups on 256 CUs and scale 1's at 2.5 rounds.
void wt_balance(rnvp_wgrad_group& sg, int cls, long long M, size_t lds) {
    long long t1 = 0;
    int nrep = 1, sps0 = 1;
    for (int c = 0; c < sg.n_conv; ++c) {
        const rnvp_wgrad_conv& v = sg.conv[c];
        if (v.nrep >= v.nz) return;                                   // plain stores: one slab per replica
        t1 += (long long)((v.n + wt_tco(cls) - 1) / wt_tco(cls)) * v.tk;
        nrep = v.nrep > nrep ? v.nrep : nrep;
        sps0 = (int)(v.m_per_slab / WT_SP) > sps0 ? (int)(v.m_per_slab / WT_SP) : sps0;
    }
    const long long S = (M + WT_SP - 1) / WT_SP;
    const long long slots = (long long)wt_cus() * wt_wg_per_cu(cls, lds);
    long long best = -1, best_cost = 0;
    for (long long sps = 2ll * sps0 < S ? 2ll * sps0 : S; sps >= WT_MIN_STAGES; --sps) {
        const long long nz = (S + sps - 1) / sps;
        if (nz <= nrep || nz * t1 > (1ll << 28)) continue;           // stay atomic
        const long long cost = ((nz * t1 + slots - 1) / slots) * (sps + WT_WG_OVERHEAD);
        if (best < 0 || cost < best_cost) { best = sps; best_cost = cost; }
    }
    if (best < 0) return;
    for (int c = 0; c < sg.n_conv; ++c) {
        sg.conv[c].nz = (int)((S + best - 1) / best);
        sg.conv[c].m_per_slab = best * WT_SP;
    }
}

}  // namespace

// Launch of the tap-shared kernel for a bf16 group; RNVP_E_UNSUPPORTED when a
// conv's shape is outside what it stages (the caller then uses the per-tap
// kernel).  Fills task0 / tk (= ci tiles) / m_per_slab of the group's copy.
int rnvp_wgrad_tap_launch(rnvp_wgrad_group* g, hipStream_t s) {
    if (g->dtype != RNVP_BF16) return RNVP_E_UNSUPPORTED;
    const long long M = (long long)g->B * g->H * g->W;
    const int H = g->H, W = g->W;
    if (W > WT_SP || WT_SP % W) return RNVP_E_UNSUPPORTED;            // stages are whole rows
    if ((long long)g->B * (H + 2) >= (1ll << 22) || M >= (1ll << 31)) return RNVP_E_UNSUPPORTED;
    // validate every conv and pick its class before launching anything
    for (int c = 0; c < g->n_conv; ++c) {
        rnvp_wgrad_conv& v = g->conv[c];
        // 32-bit buffer offsets (bytes)
        if (M * v.cs_in * 2 >= (1ll << 31) || M * v.cs_dy * 2 >= (1ll << 31)) return RNVP_E_UNSUPPORTED;
        const int cls = wt_class(v, H, W);
        if (wt_lds_bytes(cls, H, W, false) > 160 * 1024 || !wt_stage_fits(cls, H, W)) return RNVP_E_UNSUPPORTED;
        // slabs of whole stages; the slab count must stay v.nz (the replica
        // workspace and the weight-norm backward are sized by it)
        const long long stages = (M + WT_SP - 1) / WT_SP;
        v.m_per_slab = ((stages + v.nz - 1) / v.nz) * WT_SP;
        if ((M + v.m_per_slab - 1) / v.m_per_slab != v.nz) return RNVP_E_UNSUPPORTED;
        v.cls = cls;
        v.tk = (v.cs_in + wt_tci(cls) - 1) / wt_tci(cls);
        if (wt_tasks(v, cls) <= 0 || wt_tasks(v, cls) > (1ll << 28)) return RNVP_E_INVALID;
    }
    // ONE launch for the group -- the class kernel (its own register budget)
    // when every conv has the same class, else the all-class kernel (the
    // largest class's VGPRs for every task) -- or, from WT_SPLIT_MIN_M pixels
    // up, one class kernel per class present, back to back: at the wide
    // scales the all-class kernel's register budget costs more than the
    // extra launch (scale 1: 290 us grouped vs 134 + 94 us per class,
    // tools/conv_microbench.py "wgrad s1 group"); at the deep scales one
    // launch per class measured 0.3 ms/step slower (profiles/r4_wgrad_split.txt).
    // The conflict-free k order where every conv's wider rows fit LDS.
    bool one_class = true;
    for (int c = 1; c < g->n_conv; ++c) one_class = one_class && g->conv[c].cls == g->conv[0].cls;
    if (M >= WT_SPLIT_MIN_M) {    // (a one-class group takes this path too: its slabs re-balanced)
        for (int cls = 0; cls < 4; ++cls) {
            rnvp_wgrad_group sg = *g;
            sg.n_conv = 0;
            for (int c = 0; c < g->n_conv; ++c)
                if (g->conv[c].cls == cls) sg.conv[sg.n_conv++] = g->conv[c];
            if (sg.n_conv == 0) continue;
            const bool ko = wt_lds_bytes(cls, H, W, true) <= 160 * 1024;
            if (WT_BALANCE) wt_balance(sg, cls, M, wt_lds_bytes(cls, H, W, ko));
            long long tasks = 0;
            for (int c = 0; c < sg.n_conv; ++c) {
                sg.conv[c].task0 = (int)tasks;
                tasks += wt_tasks(sg.conv[c], cls);
            }
            if (tasks > (1ll << 30)) return RNVP_E_INVALID;
            hipLaunchKernelGGL(wt_kernel(cls, ko), dim3((unsigned)tasks), dim3(WT_NT), wt_lds_bytes(cls, H, W, ko), s, sg);
            RNVP_LAUNCH_CHECK();
        }
        return RNVP_OK;
    }
    bool ko = true;
    for (int c = 0; c < g->n_conv; ++c) ko = ko && wt_lds_bytes(g->conv[c].cls, H, W, true) <= 160 * 1024;
    long long tasks = 0;
    size_t shm = 0;
    for (int c = 0; c < g->n_conv; ++c) {
        rnvp_wgrad_conv& v = g->conv[c];
        v.task0 = (int)tasks;
        tasks += wt_tasks(v, v.cls);
        shm = wt_lds_bytes(v.cls, H, W, ko) > shm ? wt_lds_bytes(v.cls, H, W, ko) : shm;
    }
    if (tasks > (1ll << 30)) return RNVP_E_INVALID;
    hipLaunchKernelGGL(wt_kernel(one_class ? g->conv[0].cls : -1, ko), dim3((unsigned)tasks), dim3(WT_NT), shm, s, *g);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}
