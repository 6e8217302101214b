// Streaming 1x1 conv for the wide scales (bf16; N <= 64 outputs, cs_in <= 64):
// WeightNormConv2d (modules_realnvp.py:64-71) with the fused BatchNorm+ReLU
// prologue and the bias / residual / skip / next-BN-statistics (or the
// dgrad ReLU/BN-backward) epilogue, as rnvp_conv2d's other families.
//
// At 64x64 / 32x32 pixels with 32-64 channels a 1x1 conv is a pure stream:
// read x (and the residual / previous skip sum), write y, ~16 FLOP per byte.
// The round-2 streaming kernel issued a tile's loads only after the previous
// tile's epilogue (one memory latency per 64-pixel tile: ~1.7-2.8 TB/s).
// Here every lane keeps its weights (an MFMA A fragment per 16 outputs and
// k-step) and its BN prologue coefficients in registers, and each wave walks
// its tiles with the NEXT tile's pixel chunks and epilogue operands already in
// flight (register ring of two tiles): no LDS on the data path, no barrier.
// Product D[n][m] = W[n][k] X[m][k]^T: a lane owns 4 consecutive output
// channels of one pixel (8-byte epilogue vectors).
#include "common.h"
#include <map>
#include <mutex>

#include "conv_common.h"

#include <type_traits>

namespace {

// phase stamps for tools/probe/s1_stamps.hip (compiled out of the product)
#ifdef RNVP_S1_STAMPS
__device__ unsigned long long* g_s1_stamps;
#define S1_STAMP(i) \
    do { if (threadIdx.x == 0) g_s1_stamps[blockIdx.x * 8 + (i)] = wall_clock64(); } while (0)
#else
#define S1_STAMP(i) do {} while (0)
#endif

// NOPS epilogue operand streams per element (residual, previous y, the dgrad
// epilogue's pre-BN x -- in that order, those present)
// two waves per SIMD (<= 256 registers) unless that would spill
template <int NT, int NKS, int NOPS>
constexpr int s1_min_blocks() { return (NKS == 2 && (NOPS == 3 || (NT == 4 && NOPS == 2))) ? 1 : 2; }

// TP: every BN table of the launch comes from batch sums whose shards fit
// shard_issue<4> (checked on the host): the tables' shard loads go out first
// and are summed by shard_sum_tab, and the kernel holds no other table path
// -- with both paths in one function the compiler's wait tracking merges
// them and waits for every load in flight (the first tile's included)
// before the table sums.
// BP: the BatchNorm-backward prologue of a data gradient (rnvp_conv_args.bp):
// x is the pre-apply gradient g, bp_x the BatchNorm input t; each chunk becomes
// dL/dt = A g - (B t + C) in registers (the deep tiles' form, conv_deep.h) and
// is stored once to bp_out (a workgroup covers every output channel, so every
// pixel chunk is transformed exactly once)
template <int NT, int NKS, int TW, int NOPS, bool TP, bool BP = false>
__global__ __launch_bounds__(256, (s1_min_blocks<NT, NKS, NOPS>())) void k_conv_s1(rnvp_conv_args a, int shards) {
    constexpr int CH = 8, KS = 32;            // bf16: 8 channels per 16-B chunk, 32 per k-step
    constexpr int NC = 16 * NT;
    // shard table of the BN prologue / epilogue tables (shard_sum_tab), and
    // the per-wave statistic partials at the end: one buffer
    __shared__ double tabred[(2 * 4 * 256 > 4 * NC * 2) ? 2 * 4 * 256 : 4 * NC * 2];
    double (*red)[NC][2] = (double (*)[NC][2])tabred;
    __shared__ double tmp[2 * 64];
    __shared__ __attribute__((aligned(16))) float bnp[3 * 64];   // pro: scale | shift; BP: A | B | C
    __shared__ float etab[4 * NC];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, li = lane & 15;
    const int M = a.B * a.H * a.W;             // < 2^31 (host)
    const int N = a.n, cs = a.cs_in, cso = a.cs_out;
    const bool pro = a.pro_bn_relu != 0, epi_bn = a.epi_relu_bn_bwd != 0;
    const bool has_acc = a.accumulate != 0;
    S1_STAMP(0);

    // the BN tables' shard sums first: their wait does not queue behind the
    // weight and tile loads (vmcnt completes in issue order)
    ShardLoads<4> pro_l, epi_l;
    const int pnv = min(cs, a.cin);
    const bool pro_pre = TP && pro;
    const bool epi_pre = TP && epi_bn;
    if (pro_pre) shard_issue<4>(a.pro.sums, a.cin, a.pro.shards, 0, pnv, pro_l);
    if (epi_pre) shard_issue<4>(a.epi.sums, N, a.epi.shards, 0, min(NC, N), epi_l);
    ShardLoads<BP ? 4 : 1> bpb_l, bpg_l;
    if constexpr (BP) {
        shard_issue<4>(a.bp_bn.sums, a.cin, a.bp_bn.shards, 0, pnv, bpb_l);
        shard_issue<4>(a.bp_sums, a.cin, a.bp_shards, 0, pnv, bpg_l);
    }
    const BnAff bp_a = BP ? bn_aff_issue(a.bp_bn, a.cin, 0, a.w) : BnAff{1.f, 0.f};
    // the tables' affine parameters in the same batch (cs, NC <= 64 < 256)
    const BnAff pro_a = bn_aff_issue(a.pro, a.cin, 0, a.w);
    const BnAff epi_a = bn_aff_issue(a.epi, N, 0, a.w);

    // ---- per-lane constants: weights, prologue coefficients, bias ----
    const bf16_t* __restrict__ Wg = (const bf16_t*)a.w;
    u32x4 wv[NKS][NT];
#pragma unroll
    for (int s = 0; s < NKS; ++s)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int n = j * 16 + li, k = s * KS + g * CH;
            wv[s][j] = (n < N && k < cs) ? *(const u32x4*)(Wg + (long long)n * a.kp + k) : u32x4{0u, 0u, 0u, 0u};
        }
    float bias[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = j * 16 + 4 * g + r;
            bias[j][r] = (a.bias && n < N) ? a.bias[n] : 0.f;
        }

    // buffer resources: out-of-range offsets read zeros without a memory access
    const __amdgpu_buffer_rsrc_t XR = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0,
                                                                        (int)((long long)M * cs * 2), 0x00020000);
    // epilogue streams: role 0 residual, 1 previous y (skip accumulation), 2 pre-BN x
    // (stream q takes the q-th present role; the host picked NOPS = their count)
    const bool p0 = a.residual != nullptr, p1 = has_acc;
    int role[3];
    role[0] = p0 ? 0 : (p1 ? 1 : 2);
    role[1] = (p0 && p1) ? 1 : 2;
    role[2] = 2;
    __amdgpu_buffer_rsrc_t OR[NOPS > 0 ? NOPS : 1];
#pragma unroll
    for (int q = 0; q < NOPS; ++q) {
        const void* src = role[q] == 0 ? a.residual : (role[q] == 1 ? (const void*)a.y : a.epi_x);
        OR[q] = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(src), 0, (int)((long long)M * cso * 2),
                                                  0x00020000);
    }
    constexpr int OOB = 0x7ffffff0;
    const __amdgpu_buffer_rsrc_t TR = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(BP ? a.bp_x : a.x), 0,
                                                                        (int)((long long)M * cs * 2), 0x00020000);
    bf16_t* __restrict__ BPO = (bf16_t*)a.bp_out;

    // ---- tile ring: pixel chunks + epilogue operands of two tiles ----
    struct Tile {
        u32x4 x[TW][NKS];
        u32x4 t[BP ? TW : 1][BP ? NKS : 1];
        uint2 o[NOPS > 0 ? NOPS : 1][TW][NT];
    };
    Tile ring[2];
    const int ntiles = (M + 16 * TW - 1) / (16 * TW);
    const int nwaves = gridDim.x * 4;
    const int w0 = blockIdx.x * 4 + wid;
    auto load = [&](int t, auto SLC) __attribute__((always_inline)) {
        constexpr int SL = decltype(SLC)::value;
        Tile& T = ring[SL];
#pragma unroll
        for (int i = 0; i < TW; ++i) {
            const int m = t * (16 * TW) + i * 16 + li;
            const bool okm = (t < ntiles) & (m < M);
#pragma unroll
            for (int s = 0; s < NKS; ++s) {
                const int k = s * KS + g * CH;
                const int off = (okm & (k < cs)) ? (m * cs + k) * 2 : OOB;
                T.x[i][s] = __builtin_amdgcn_raw_buffer_load_b128(XR, off, 0, 0);
                if constexpr (BP) T.t[i][s] = __builtin_amdgcn_raw_buffer_load_b128(TR, off, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int n0 = j * 16 + 4 * g;
                const int off = (okm & (n0 < cso)) ? (m * cso + n0) * 2 : OOB;
#pragma unroll
                for (int q = 0; q < NOPS; ++q)
                    T.o[q][i][j] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(OR[q], off, 0, 0));
            }
        }
    };

    // per-lane partial statistics in fp32 (a lane adds TW values per tile over a
    // few tiles); the cross-lane and cross-block sums are fp64
    float s1[NT][4], s2[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) s1[j][r] = s2[j][r] = 0.f;
    bf16_t* __restrict__ Y = (bf16_t*)a.y;

    auto run = [&](int t, auto SLC) __attribute__((always_inline)) {
        constexpr int SL = decltype(SLC)::value;
        const Tile& T = ring[SL];
        floatx4 acc[TW][NT];
#pragma unroll
        for (int i = 0; i < TW; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < TW; ++i)
#pragma unroll
            for (int s = 0; s < NKS; ++s) {
                u32x4 v = T.x[i][s];
                if constexpr (BP) {
                    const int c0 = s * KS + g * CH;
                    const int m = t * (16 * TW) + i * 16 + li, k = c0;
                    float gv[CH], tv[CH], d[CH];
                    unpack(v, gv, bf16_t());
                    unpack(T.t[i][s], tv, bf16_t());
                    const float4 qa = *(const float4*)&bnp[c0], qb = *(const float4*)&bnp[c0 + 4];
                    const float4 ra = *(const float4*)&bnp[64 + c0], rb = *(const float4*)&bnp[64 + c0 + 4];
                    const float4 ua = *(const float4*)&bnp[128 + c0], ub = *(const float4*)&bnp[128 + c0 + 4];
                    const float A[CH] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
                    const float Bv[CH] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
                    const float Cv[CH] = {ua.x, ua.y, ua.z, ua.w, ub.x, ub.y, ub.z, ub.w};
#pragma unroll
                    for (int e = 0; e < CH; ++e) d[e] = fmaf(A[e], gv[e], -fmaf(Bv[e], tv[e], Cv[e]));
                    v = pack(d, bf16_t());
                    const bool in = (m < M) & (k < cs);
                    if (in && BPO) *(u32x4*)(BPO + (long long)m * cs + k) = v;
                    const uint32_t keep = in ? ~0u : 0u;
                    v &= u32x4{keep, keep, keep, keep};
                } else if (pro) {
                    // prologue coefficients from LDS (registers go to the tile ring)
                    const int c0 = s * KS + g * CH;
                    const float4 sa = *(const float4*)&bnp[c0], sb = *(const float4*)&bnp[c0 + 4];
                    const float4 ha = *(const float4*)&bnp[64 + c0], hb = *(const float4*)&bnp[64 + c0 + 4];
                    const float sc[CH] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
                    const float sh[CH] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
                    v = bn_relu_bf16x8(v, sc, sh);
                    // a pixel outside the image / a channel chunk beyond cs stays zero
                    const int m = t * (16 * TW) + i * 16 + li, k = s * KS + g * CH;
                    const uint32_t keep = ((m < M) & (k < cs)) ? ~0u : 0u;
                    v &= u32x4{keep, keep, keep, keep};
                }
#pragma unroll
                for (int j = 0; j < NT; ++j) Mf<bf16_t>::step(wv[s][j], v, acc[i][j]);
            }
        // epilogue: lane owns channels j*16 + 4g .. +3 of pixel t*16*TW + i*16 + li
#pragma unroll
        for (int i = 0; i < TW; ++i) {
            const int m = t * (16 * TW) + i * 16 + li;
            if (m >= M) continue;
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int n0 = j * 16 + 4 * g;
                if (n0 >= cso) continue;
                float v[4], xv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[j][r];
#pragma unroll
                for (int q = 0; q < NOPS; ++q) {
                    const uint2 u = T.o[q][i][j];
                    const float f[4] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                        __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
                    if (role[q] == 2) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) xv[r] = f[r];
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] += f[r];
                    }
                }
                if (epi_bn) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int n = n0 + r;
                        if (xv[r] * etab[n] + etab[NC + n] <= 0.f) v[r] = 0.f;
                        s1[j][r] += v[r];
                        s2[j][r] += v[r] * (xv[r] - etab[2 * NC + n]) * etab[3 * NC + n];
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        s1[j][r] += v[r];
                        s2[j][r] += v[r] * v[r];
                    }
                }
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (n0 + r >= N) v[r] = 0.f;
                st4(Y + (long long)m * cso + n0, v);
            }
        }
    };

    // walk this wave's tiles w0, w0 + nwaves, ... with the next one in flight
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    int t = w0;
    if (t < ntiles) load(t, I0{});

    // ---- tables (every thread: block-wide reductions), their loads in flight
    // behind the weights and the first tile's ----
    if constexpr (BP) {
        // dL/dt = A g - (B t + C): A = gamma rstd, B = A rstd k2, C = A (k1 - rstd k2 mean)
        // (rnvp_bn_bwd_apply's A (g - k1 - (t - mean) rstd k2) regrouped)
        shard_sum_tab<4>(bpb_l, pnv, a.bp_bn.shards, tabred, tmp, tmp + cs);
        const double S1 = tid < pnv ? tmp[tid] : 0.0, S2 = tid < pnv ? tmp[cs + tid] : 0.0;
        __syncthreads();
        shard_sum_tab<4>(bpg_l, pnv, a.bp_shards, tabred, tmp, tmp + cs);
        if (tid < cs) {
            float A = 0.f, Bc = 0.f, Cc = 0.f;
            if (tid < pnv) {
                const double g1 = tmp[tid], g2 = tmp[cs + tid], cnt = a.bp_bn.count;
                const double mean = S1 / cnt;
                double var = S2 / cnt - mean * mean;
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
            bnp[tid] = A;
            bnp[64 + tid] = Bc;
            bnp[128 + tid] = Cc;
        }
        __syncthreads();
    }
    if constexpr (TP) {
        if (pro) {
            shard_sum_tab<4>(pro_l, pnv, a.pro.shards, tabred, tmp, tmp + cs);
            block_bn_finish_aff(a.pro, a.cin, 0, cs, bnp, bnp + 64, nullptr, nullptr, tmp, pro_a);
        }
        if (epi_bn) {
            shard_sum_tab<4>(epi_l, min(NC, N), a.epi.shards, tabred, tmp, tmp + NC);
            block_bn_finish_aff(a.epi, N, 0, NC, etab, etab + NC, etab + 2 * NC, etab + 3 * NC, tmp, epi_a);
        }
    } else {
        if (pro) block_bn_table(a.pro, a.cin, 0, cs, bnp, bnp + 64, nullptr, nullptr, tmp);
        if (epi_bn) block_bn_table(a.epi, N, 0, NC, etab, etab + NC, etab + 2 * NC, etab + 3 * NC, tmp);
    }
    __syncthreads();
    S1_STAMP(1);

    while (t < ntiles) {
        if (t + nwaves < ntiles) load(t + nwaves, I1{});
        run(t, I0{});
        t += nwaves;
        if (t >= ntiles) break;
        if (t + nwaves < ntiles) load(t + nwaves, I0{});
        run(t, I1{});
        t += nwaves;
    }
    S1_STAMP(2);

    // ---- batch statistics: DPP row sums, LDS across waves, sharded fp64 atomics ----
    const bool want_sums = a.out_sums || (epi_bn && a.epi_sums);
    if (want_sums) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double u1 = row_sum16((double)s1[j][r]), u2 = row_sum16((double)s2[j][r]);
                if (li == 0) {
                    red[wid][j * 16 + 4 * g + r][0] = u1;
                    red[wid][j * 16 + 4 * g + r][1] = u2;
                }
            }
        __syncthreads();
        double* sums = shard_ptr(epi_bn ? a.epi_sums : a.out_sums, shards, N);
        for (int n = tid; n < N; n += 256) {
            double t1 = 0.0, t2 = 0.0;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                t1 += red[w][n][0];
                t2 += red[w][n][1];
            }
            atomicAdd(&sums[n], t1);
            atomicAdd(&sums[N + n], t2);
        }
    }
    S1_STAMP(3);
}

template <int NT, int NKS, int TW, int NOPS, bool TP, bool BP = false>
int launch_s1(const rnvp_conv_args* a, hipStream_t s, bool dry) {
    if (dry) return RNVP_OK;
    const long long M = (long long)a->B * a->H * a->W;
    const long long ntiles = (M + 16 * TW - 1) / (16 * TW);
    // one resident wave of workgroups, one tile per wave and step with the
    // next one in flight (a second round of workgroups would restart the
    // pipeline; more tiles per wave measured slower, profiles/r4_step_ab.txt)
    static const int per_cu = [] {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_conv_s1<NT, NKS, TW, NOPS, TP, BP>, 256, 0) != hipSuccess ||
            n < 1)
            n = 1;
        return n;
    }();
    long long grid = (ntiles + 3) / 4;
    if (grid > 256LL * per_cu) grid = 256LL * per_cu;
    k_conv_s1<NT, NKS, TW, NOPS, TP, BP><<<(unsigned)grid, 256, 0, s>>>(*a, rnvp_stat_shards(M));
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

// every BN table from batch sums whose shards fit shard_issue<4> (256 threads)
inline bool s1_tables_pre(const rnvp_conv_args* a, int NC) {
    auto fits = [](int nc, int shards) { return (long long)nc * (shards < 1 ? 1 : shards) <= 4LL * 256; };
    if (a->bp) {
        const int nc = a->cs_in < a->cin ? a->cs_in : a->cin;
        if (!a->bp_bn.sums || !a->bp_sums || !fits(nc, a->bp_bn.shards) || !fits(nc, a->bp_shards)) return false;
    }
    if (a->pro_bn_relu && !(a->pro.sums && fits(a->cs_in < a->cin ? a->cs_in : a->cin, a->pro.shards))) return false;
    if (a->epi_relu_bn_bwd && !(a->epi.sums && fits(NC < a->n ? NC : a->n, a->epi.shards))) return false;
    return true;
}

template <int NT, int NKS, int TW, int NOPS>
int launch_s1(const rnvp_conv_args* a, hipStream_t s, bool dry) {
    if (a->bp) return RNVP_E_UNSUPPORTED;
    return s1_tables_pre(a, 16 * NT) ? launch_s1<NT, NKS, TW, NOPS, true>(a, s, dry)
                                     : launch_s1<NT, NKS, TW, NOPS, false>(a, s, dry);
}

// the BatchNorm-backward prologue: a data gradient with the ReLU/BN epilogue
// as its one operand stream, every table in a shard table
template <int NT, int NKS, int TW>
int launch_s1_bp(const rnvp_conv_args* a, hipStream_t s, bool dry) {
    if (!a->epi_relu_bn_bwd || a->residual || a->accumulate || !s1_tables_pre(a, 16 * NT)) return RNVP_E_UNSUPPORTED;
    return launch_s1<NT, NKS, TW, 1, true, true>(a, s, dry);
}

template <int NT, int NKS, int TW>
int launch_s1_ops(const rnvp_conv_args* a, hipStream_t s, bool dry) {
    const int nops = (a->residual ? 1 : 0) + (a->accumulate ? 1 : 0) + (a->epi_relu_bn_bwd ? 1 : 0);
    switch (nops) {
        case 0: return launch_s1<NT, NKS, TW, 0>(a, s, dry);
        case 1: return launch_s1<NT, NKS, TW, 1>(a, s, dry);
        case 2: return launch_s1<NT, NKS, TW, 2>(a, s, dry);
        default: return launch_s1<NT, NKS, TW, 3>(a, s, dry);
    }
}

// ---------------------------------------------------------------------------
// Fan-out: several independent 1x1 convs of one net that read the SAME input
// (wide scales, M > 16k pixels): each input tile is loaded once and feeds
// every member's MFMAs and epilogue.  The forward pairs core_skips[i] with the
// next block's first 1x1 (both read x1_{i+1}; in_skip with block 0's, both
// read x1_0) and the backward runs the data gradients of in_skip and every
// core_skips[i] (all read d out) -- modules_realnvp.py:175-194.  Members:
// optional BN+ReLU prologue (their own table), bias, skip accumulation, next-
// BN statistics (at most one member), no residual / dgrad epilogue
// (rnvp_net_group_prepare checks).  Weights of all members in LDS.
constexpr int FAN_MAX = 8;

template <int NT, int NKS, int TW>
__global__ __launch_bounds__(256, 2) void k_s1_fanout(const rnvp_group_kargs gk) {
    constexpr int CH = 8, KS = 32, NC = 16 * NT, KL = lds_mfma_pitch(NKS * KS, CH);   // LDS weight row pitch
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int nm = gk.n;
    bf16_t* Wl = (bf16_t*)lds;                                   // [nm][NC][KL]
    float* bnp = (float*)(Wl + nm * NC * KL);                    // [nm][2][64] prologue scale | shift
    float* btab = bnp + nm * 128;                                // [nm][NC] bias
    double* red = (double*)(btab + nm * NC);                     // [4 waves][NC][2]
    double* tmp = red + 4 * NC * 2;                              // [128] BN-table scratch
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, li = lane & 15;
    const rnvp_conv_args& a0 = gk.conv[0];
    const int M = a0.B * a0.H * a0.W;
    const int cs = a0.cs_in;
    int sm = -1;                                                 // the member with statistics
    for (int c = 0; c < nm; ++c)
        if (gk.conv[c].out_sums) sm = c;

    // ---- weights, bias, prologue tables -> LDS (once per workgroup) ----
    for (int c = 0; c < nm; ++c) {
        const rnvp_conv_args& a = gk.conv[c];
        const bf16_t* Wg = (const bf16_t*)a.w;
        for (int q = tid; q < NC * (NKS * KS / CH); q += 256) {
            const int r = q / (NKS * KS / CH), ch = q - r * (NKS * KS / CH);
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            if (r < a.n && ch * CH < cs) v = *(const u32x4*)(Wg + (long long)r * a.kp + ch * CH);
            *(u32x4*)(Wl + (c * NC + r) * KL + ch * CH) = v;
        }
        for (int n = tid; n < NC; n += 256) btab[c * NC + n] = (a.bias && n < a.n) ? a.bias[n] : 0.f;
        if (a.pro_bn_relu) block_bn_table(a.pro, a.cin, 0, cs, bnp + c * 128, bnp + c * 128 + 64, nullptr, nullptr, tmp);
    }
    __syncthreads();

    const __amdgpu_buffer_rsrc_t XR = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a0.x), 0,
                                                                        (int)((long long)M * cs * 2), 0x00020000);
    constexpr int OOB = 0x7ffffff0;
    const int ntiles = (M + 16 * TW - 1) / (16 * TW);
    const int nwaves = gridDim.x * 4;
    float s1[NT][4], s2[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) s1[j][r] = s2[j][r] = 0.f;
    u32x4 xr[2][TW][NKS];
    auto load = [&](int t, u32x4 (&X)[TW][NKS]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < TW; ++i) {
            const int m = t * (16 * TW) + i * 16 + li;
            const bool okm = (t < ntiles) & (m < M);
#pragma unroll
            for (int s = 0; s < NKS; ++s) {
                const int k = s * KS + g * CH;
                X[i][s] = __builtin_amdgcn_raw_buffer_load_b128(XR, (okm & (k < cs)) ? (m * cs + k) * 2 : OOB, 0, 0);
            }
        }
    };
    auto run = [&](int t, const u32x4 (&X)[TW][NKS]) __attribute__((always_inline)) {
        for (int c = 0; c < nm; ++c) {
            const rnvp_conv_args& a = gk.conv[c];
            const bool pro = a.pro_bn_relu != 0;
            const int cso = a.cs_out, N = a.n;
            floatx4 acc[TW][NT];
#pragma unroll
            for (int i = 0; i < TW; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < NKS; ++s) {
                u32x4 wf[NT];
#pragma unroll
                for (int j = 0; j < NT; ++j) wf[j] = *(const u32x4*)(Wl + (c * NC + j * 16 + li) * KL + s * KS + g * CH);
#pragma unroll
                for (int i = 0; i < TW; ++i) {
                    u32x4 v = X[i][s];
                    if (pro) {
                        const int c0 = s * KS + g * CH;
                        const float* sc = bnp + c * 128 + c0;
                        const float* sh = sc + 64;
                        v = bn_relu_bf16x8(v, sc, sh);
                        const int m = t * (16 * TW) + i * 16 + li;
                        const uint32_t keep = ((m < M) & (c0 < cs)) ? ~0u : 0u;
                        v &= u32x4{keep, keep, keep, keep};
                    }
#pragma unroll
                    for (int j = 0; j < NT; ++j) Mf<bf16_t>::step(wf[j], v, acc[i][j]);
                }
            }
            bf16_t* __restrict__ Y = (bf16_t*)a.y;
            const bool accu = a.accumulate != 0, st = c == sm;
#pragma unroll
            for (int i = 0; i < TW; ++i) {
                const int m = t * (16 * TW) + i * 16 + li;
                if (m >= M) continue;
#pragma unroll
                for (int j = 0; j < NT; ++j) {
                    const int n0 = j * 16 + 4 * g;
                    if (n0 >= cso) continue;
                    float v[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + btab[c * NC + n0 + r];
                    if (accu) {
                        float o[4];
                        ld4(Y + (long long)m * cso + n0, o);
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] += o[r];
                    }
                    if (st) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            s1[j][r] += v[r];
                            s2[j][r] += v[r] * v[r];
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (n0 + r >= N) v[r] = 0.f;
                    st4(Y + (long long)m * cso + n0, v);
                }
            }
        }
    };
    // walk this wave's tiles with the next one in flight (static ring slots)
    int t = blockIdx.x * 4 + wid;
    if (t < ntiles) load(t, xr[0]);
    while (t < ntiles) {
        if (t + nwaves < ntiles) load(t + nwaves, xr[1]);
        run(t, xr[0]);
        t += nwaves;
        if (t >= ntiles) break;
        if (t + nwaves < ntiles) load(t + nwaves, xr[0]);
        run(t, xr[1]);
        t += nwaves;
    }
    if (sm >= 0) {
        const rnvp_conv_args& a = gk.conv[sm];
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double u1 = row_sum16((double)s1[j][r]), u2 = row_sum16((double)s2[j][r]);
                if (li == 0) {
                    red[(wid * NC + j * 16 + 4 * g + r) * 2] = u1;
                    red[(wid * NC + j * 16 + 4 * g + r) * 2 + 1] = u2;
                }
            }
        __syncthreads();
        double* sums = shard_ptr(a.out_sums, gk.shards[sm], a.n);
        for (int n = tid; n < a.n; n += 256) {
            double t1 = 0.0, t2 = 0.0;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                t1 += red[(w * NC + n) * 2];
                t2 += red[(w * NC + n) * 2 + 1];
            }
            atomicAdd(&sums[n], t1);
            atomicAdd(&sums[a.n + n], t2);
        }
    }
}

using FanKernel = void (*)(const rnvp_group_kargs);

FanKernel fan_kernel(int nt, int nks) {
    if (nt == 1) return nks == 1 ? k_s1_fanout<1, 1, 4> : k_s1_fanout<1, 2, 4>;
    if (nt == 2) return nks == 1 ? k_s1_fanout<2, 1, 4> : k_s1_fanout<2, 2, 4>;
    return nks == 1 ? k_s1_fanout<4, 1, 2> : k_s1_fanout<4, 2, 2>;
}

}  // namespace

// fan-out group of the wide scales (rnvp_net_group_prepare's M > 16k branch):
// validates, fills the members' shard counts and returns klass = 1 << 12 |
// NT << 4 | NKS, the grid and the LDS bytes (RNVP_E_UNSUPPORTED: no such form)
int rnvp_s1_fanout_prepare(rnvp_net_step* steps, int n, int* klass, int* grid, int* lds_bytes) {
    if (n < 2 || n > FAN_MAX) return RNVP_E_UNSUPPORTED;
    const rnvp_conv_args& a0 = steps[0].conv;
    const long long M = (long long)a0.B * a0.H * a0.W;
    if (a0.dtype != RNVP_BF16 || M <= 16384 || M * 64 * 2 >= (1ll << 31)) return RNVP_E_UNSUPPORTED;
    if (a0.cs_in > 64 || (a0.cs_in & 7) || ((uintptr_t)a0.x & 15)) return RNVP_E_UNSUPPORTED;
    int nmax = 0, nstats = 0;
    for (int i = 0; i < n; ++i) {
        const rnvp_net_step& st = steps[i];
        const rnvp_conv_args& a = st.conv;
        if (st.kind != RNVP_STEP_CONV || a.ks != 1 || a.dtype != RNVP_BF16) return RNVP_E_UNSUPPORTED;
        if (a.x != a0.x || a.cs_in != a0.cs_in || a.B != a0.B || a.H != a0.H || a.W != a0.W) return RNVP_E_UNSUPPORTED;
        if (a.residual || a.epi_relu_bn_bwd || a.n <= 0 || a.n > 64 || a.cs_out > 64 || a.cs_out < a.n) return RNVP_E_UNSUPPORTED;
        if (!a.w || !a.y || (a.kp & 63) || a.kp < a.cs_in || ((uintptr_t)a.y & 7) || ((uintptr_t)a.w & 15))
            return RNVP_E_UNSUPPORTED;
        if (a.pro_bn_relu && a.pro.sums && a.pro.shards > 32) return RNVP_E_UNSUPPORTED;
        nstats += a.out_sums != nullptr;
        nmax = a.n > nmax ? a.n : nmax;
    }
    if (nstats > 1) return RNVP_E_UNSUPPORTED;
    const int nt = nmax <= 16 ? 1 : (nmax <= 32 ? 2 : 4), nks = a0.cs_in <= 32 ? 1 : 2;
    for (int i = 0; i < n; ++i) steps[i].shards = rnvp_stat_shards(M);
    const int NC = 16 * nt, KL = lds_mfma_pitch(nks * 32, 8);
    const size_t lds = (size_t)n * NC * KL * 2 + (size_t)n * 128 * 4 + (size_t)n * NC * 4 + 4 * NC * 2 * 8 + 128 * 8;
    if (lds > 64 * 1024) return RNVP_E_UNSUPPORTED;
    // host-only (no HIP call): the grid is one wave per tile here; the
    // launch caps it to one resident round of workgroups (occupancy queried
    // there, once per kernel)
    const int tw = nt == 4 ? 2 : 4;
    const long long ntiles = (M + 16 * tw - 1) / (16 * tw);
    const long long gr = (ntiles + 3) / 4;
    if (gr >= (1ll << 31)) return RNVP_E_UNSUPPORTED;
    *klass = (1 << 12) | (nt << 4) | nks;
    *grid = (int)gr;
    *lds_bytes = (int)lds;
    return RNVP_OK;
}

int rnvp_s1_fanout_launch(const rnvp_group_kargs& g, int klass, int grid, int lds_bytes, hipStream_t s) {
    const int nt = (klass >> 4) & 15, nks = klass & 15;
    const FanKernel k = fan_kernel(nt, nks);
    // resident workgroups per CU of this kernel at this LDS size: one runtime
    // query per (kernel, LDS size) -- the members' weights make the LDS size
    // vary -- cached behind a lock (launches may come from several threads;
    // the query is not a stream operation, so a capture in progress is fine)
    static std::mutex mu;
    static std::map<long long, int> occ;
    const long long key = ((long long)klass << 32) | (unsigned)lds_bytes;
    int per_cu;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = occ.find(key);
        if (it == occ.end()) {
            int q = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&q, k, 256, lds_bytes) != hipSuccess || q < 1) q = 1;
            it = occ.emplace(key, q).first;
        }
        per_cu = it->second;
    }
    const long long cap = 256LL * per_cu;
    hipLaunchKernelGGL(k, dim3((unsigned)(grid < cap ? grid : cap)), dim3(256), lds_bytes, s, g);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

// 1x1, bf16, N <= 64, cs_in <= 64, M >= 16k: the register-pipelined stream
int rnvp_conv_s1_launch(const rnvp_conv_args* a, hipStream_t s, bool dry) {
    if (a->dtype != RNVP_BF16 || a->ks != 1 || a->n > 64 || a->cs_in > 64 || a->cs_out > 64) return RNVP_E_UNSUPPORTED;
    const long long M = (long long)a->B * a->H * a->W;
    if (M < 16384 || M * 64 * 2 >= (1ll << 31)) return RNVP_E_UNSUPPORTED;
    if (((uintptr_t)a->y & 7) || (a->residual && ((uintptr_t)a->residual & 7)) ||
        (a->epi_relu_bn_bwd && ((uintptr_t)a->epi_x & 7)))
        return RNVP_E_UNSUPPORTED;
    if (a->bp && a->pro_bn_relu) return RNVP_E_UNSUPPORTED;
    const bool k1 = a->cs_in <= 32;
    if (a->bp) {   // the prologue's second operand stream: half-width tiles (registers)
        if (a->n <= 16) return k1 ? launch_s1_bp<1, 1, 2>(a, s, dry) : launch_s1_bp<1, 2, 2>(a, s, dry);
        if (a->n <= 32) return k1 ? launch_s1_bp<2, 1, 2>(a, s, dry) : launch_s1_bp<2, 2, 2>(a, s, dry);
        return k1 ? launch_s1_bp<4, 1, 1>(a, s, dry) : launch_s1_bp<4, 2, 1>(a, s, dry);
    }
    if (a->n <= 16) return k1 ? launch_s1_ops<1, 1, 4>(a, s, dry) : launch_s1_ops<1, 2, 4>(a, s, dry);
    if (a->n <= 32) return k1 ? launch_s1_ops<2, 1, 4>(a, s, dry) : launch_s1_ops<2, 2, 4>(a, s, dry);
    return k1 ? launch_s1_ops<4, 1, 2>(a, s, dry) : launch_s1_ops<4, 2, 2>(a, s, dry);
}
