// Coupling links: the training step's flow program between two couplings
// (flow_realnvp.py:252-327) without a permuted copy and without a separate
// reduction pass.
//
// A link joins coupling a to what consumes its output z:
//   SAME      the next coupling of the same combo (z is its input as is)
//   SQUEEZE   checkerboard -> channelwise, the input is squeeze(z)        (flow_realnvp.py:260)
//   UNFACTOR  channelwise -> the next scale, (x', off) =
//             factor_out(undo_squeeze(z)): a channel gather at the same
//             pixels, the off half goes to the prior                     (264-267)
//   FINAL     the last scale's z goes to the prior                      (312-327, 336-338)
//
// Forward, per coupling: k_out_u (a's u = x*exp(lr)+shift reduced to sums
// per pixel class and channel, no u stored) and k_link_fwd (z = out_bn(u)
// recomputed from x and the net output, written straight to the consumer's
// input at its permuted address, the consumer's in_bn statistics in closed
// form from a's class sums, its net input h0, the prior of what leaves the
// flow).  The closed form works because every class of a's pixels is wholly
// transformed or wholly kept by a (checkerboard parity, channel halves) and
// each in_bn channel of the consumer reads exactly one such class.
//
// Backward, per coupling: k_link_bwd forms dL/dz of a (the consumer's direct
// input gradient + its in_bn backward from its net-input gradient gh0, or the
// prior's -z*g_lp) and runs a's out part with it.  The out_bn backward sums
// (sum dL/dz and sum dL/dz * xhat over a's transformed positions) are closed
// forms of sums the consumer's own passes already reduced, so they are ready
// before the pass starts.  a's in part backward stays in coupling.hip
// (k_in_bwd_red with the extra kept-position sums this file's closed forms use).
#include "coupling_common.h"

// phase stamps for tools/probe/link_stamps.hip (compiled out of the product)
#ifdef RNVP_LINK_STAMPS
__device__ unsigned long long* g_link_stamps;
#define LINK_STAMP(i) \
    do { if (threadIdx.x == 0) g_link_stamps[blockIdx.x * 8 + (i)] = wall_clock64(); } while (0)
#else
#define LINK_STAMP(i) do {} while (0)
#endif

namespace {

constexpr float LOG_SQRT_2PI = 0.91893853320467274178f;

// pixel class of p (= i*W + j) under class mode nc: 1 = one class,
// 2 = (i+j)&1, 4 = (i&1)*2 + (j&1)
__device__ __forceinline__ int pcls(int nc, const Geo& g, int p) {
    if (nc == 1) return 0;
    const int i = p / g.W, j = p - i * g.W;
    return nc == 2 ? ((i + j) & 1) : ((i & 1) * 2 + (j & 1));
}

// positions per sample in class q
__device__ __forceinline__ double cls_count(int nc, const Geo& g, int q) {
    const long long H = g.H, W = g.W;
    if (nc == 1) return (double)(H * W);
    if (nc == 2) {
        const long long even = ((H & 1) && (W & 1)) ? (H * W + 1) / 2 : H * W / 2;
        return (double)(q == 0 ? even : H * W - even);
    }
    const long long hi = (q >> 1) ? H / 2 : (H + 1) / 2, wj = (q & 1) ? W / 2 : (W + 1) / 2;
    return (double)(hi * wj);
}

// (channel c, class q) transformed by coupling g: checkerboard (cfg + i + j)
// even (classes by parity), channelwise the "on" half
__device__ __forceinline__ bool cls_tr(const Geo& g, int nc, int c, int q) {
    if (g.kind == 1) return c >= g.on_base && c < g.on_base + g.Cb;
    const int par = nc == 2 ? q : (((q >> 1) + (q & 1)) & 1);
    return ((g.cfg + par) & 1) == 0;
}

// out[i] = sum over the shards of entry i (LDS), spread over the block
__device__ __forceinline__ void lds_shard_reduce(const double* sums, int width, double* out) {
    for (int i = threadIdx.x; i < width; i += blockDim.x) out[i] = csum(sums, width, i);
}

// the same over several arrays at once: their entries share one flat index
// space over the block, so every thread's loads go out together (one memory
// round trip for up to blockDim entries, not one per array)
struct ShardArr {
    const double* p;
    int w;
    double* out;
};
template <int N>
__device__ __forceinline__ void lds_shard_reduce_multi(const ShardArr (&a)[N]) {
    constexpr int K = 2;   // entries per thread per round: K * shards loads in flight (registers: occupancy)
    int total = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) total += a[i].w;
    for (int f0 = 0; f0 < total; f0 += K * (int)blockDim.x) {
        const double* p[K];
        double* o[K];
        int w[K], off[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int f = f0 + k * (int)blockDim.x + (int)threadIdx.x;
            int r = f < total ? f : 0;
            p[k] = a[0].p;
            o[k] = f < total ? a[0].out : nullptr;
            w[k] = a[0].w;
#pragma unroll
            for (int i = 1; i < N; ++i) {
                if (r >= w[k]) {
                    r -= w[k];
                    p[k] = a[i].p;
                    if (o[k]) o[k] = a[i].out;
                    w[k] = a[i].w;
                }
            }
            off[k] = r;
        }
        double v[K][RNVP_COUPLING_SHARDS];
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int h = 0; h < RNVP_COUPLING_SHARDS; ++h) v[k][h] = p[k][(long long)h * w[k] + off[k]];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double t = 0.0;
#pragma unroll
            for (int h = 0; h < RNVP_COUPLING_SHARDS; ++h) t += v[k][h];
            if (o[k]) o[k][off[k]] = t;
        }
    }
}

// block-wide sums of two values (one pair of barriers); every thread gets them
__device__ __forceinline__ void block_sum2(double& x, double& y, double* red /* >= 32 entries of LDS */) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    x = wave_sum(x);
    y = wave_sum(y);
    __syncthreads();
    if (lane == 0) {
        red[wid] = x;
        red[16 + wid] = y;
    }
    __syncthreads();
    double tx = 0.0, ty = 0.0;
    for (int i = 0; i < nw; ++i) {
        tx += red[i];
        ty += red[16 + i];
    }
    x = tx;
    y = ty;
}

// a's out_bn batch statistics of out_bn channel cb from the reduced class sums
// (the same reduction order in the forward and backward passes)
__device__ __forceinline__ void cls_out_stats(const double* cs, const Geo& g, int nc, int cb, float eps, double& mean,
                                              double& var) {
    const int ca = g.kind == 0 ? cb : g.on_base + cb;
    double s1 = 0.0, s2 = 0.0;
    for (int q = 0; q < nc; ++q) {
        s1 += cs[(2 * q) * g.C + ca];
        s2 += cs[(2 * q + 1) * g.C + ca];
    }
    const double cnt = (double)g.B * g.HW;
    mean = s1 / cnt;
    var = s2 / cnt - mean * mean;
    if (var < 0) var = 0;
    (void)eps;
}

// the (a channel, a class) that in_bn channel cbn of the consumer reads
template <int LT>
__device__ __forceinline__ void link_src(const Geo& gn, int cbn, int& ca, int& q) {
    if (LT == RNVP_LINK_SAME) {
        if (gn.kind == 0) {        // n's kept squares = a's transformed ones: parity (cfg_n + 1) & 1
            ca = cbn;
            q = (gn.cfg + 1) & 1;
        } else {                   // n's conditioning half = a's transformed half
            ca = gn.off_base + cbn;
            q = 0;
        }
    } else if (LT == RNVP_LINK_SQUEEZE) {   // squeezed channel k = 4c + 2i + j
        const int k = gn.off_base + cbn;
        ca = k >> 2;
        q = k & 3;
    } else {                                // UNFACTOR: n channel c <- z channel 4c / 4(c-K)+3, n's kept squares
        const int K = gn.C / 2;
        ca = cbn < K ? 4 * cbn : 4 * (cbn - K) + 3;
        q = (gn.cfg + 1) & 1;
    }
}

// where element (channel ca, pixel pa) of a's z goes: the consumer's input
// element (c, p) or (to_prior) the prior
struct Dst {
    bool to_prior;
    int c, p;
};
template <int LT>
__device__ __forceinline__ Dst link_dst(const Geo& ga, const Geo& gn, int ca, int pa) {
    Dst d;
    d.to_prior = false;
    d.c = ca;
    d.p = pa;
    if (LT == RNVP_LINK_SQUEEZE) {
        const int i = pa / ga.W, j = pa - i * ga.W;
        d.c = 4 * ca + 2 * (i & 1) + (j & 1);
        d.p = (i >> 1) * gn.W + (j >> 1);
    } else if (LT == RNVP_LINK_UNFACTOR) {
        const int r = ca & 3, c = ca >> 2, K = gn.C / 2;
        if (r == 0 || r == 3) {
            d.c = r == 0 ? c : K + c;
        } else {                    // the factored-out half: off channel c (r = 1) / K + c (r = 2)
            d.to_prior = true;
            d.c = r == 1 ? c : K + c;
        }
    } else if (LT == RNVP_LINK_FINAL) {
        d.to_prior = true;
    }
    return d;
}

// in_bn channel of the consumer's input channel c (-1: not normalised)
__device__ __forceinline__ int in_bn_channel(const Geo& gn, int c) {
    if (gn.kind == 0) return c;
    return (c >= gn.off_base && c < gn.off_base + gn.Cb) ? c - gn.off_base : -1;
}

// one s/t-net BatchNorm running-stat update (the link's extra workgroups)
__device__ __forceinline__ void net_running_block(const rnvp_coupling_args& a, int i, double* tmp) {
    const rnvp_bn_running r = a.net_running[i];
    block_shard_sums(r.sums, r.C, r.shards, 0, r.C, tmp, tmp + r.C);
    const float mom = a.momentum;
    for (int c = threadIdx.x; c < r.C; c += blockDim.x) {
        double mean = tmp[c] / r.count;
        double var = tmp[r.C + c] / r.count - mean * mean;
        if (var < 0) var = 0;
        double unb = r.count > 1 ? var * r.count / (r.count - 1) : var;
        r.rmean[c] = (1.f - mom) * r.rmean[c] + mom * (float)mean;
        r.rvar[c] = (1.f - mom) * r.rvar[c] + mom * (float)unb;
    }
    if (threadIdx.x == 0 && r.nbt) r.nbt[0] += 1;
}

// ---------------------------------------------------------------------------
// forward: u's class sums (the out part's reduction pass)
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_out_u(rnvp_coupling_args a, int TP, int seg) {
    extern __shared__ double dsm[];
    __shared__ float redl[16];
    const Geo g = geo(a);
    const Tile t = tile_of(g, TP);
    const int lane = threadIdx.x & 63;
    const int nc = a.nclass, W2 = nc * 2 * g.C;
    double* red = dsm;          // [nc][2][C]
    T* st = (T*)(dsm + W2);     // [tp][cs_st]  (W2 even: 16-B aligned)
    const int total = g.C * t.tp;
    auto xidx = [&](int e) {
        const int c = e / t.tp, pl = e - c * t.tp;
        return ((long long)t.b * g.C + c) * g.HW + t.p0 + pl;
    };
    float xp[CP_K];
#pragma unroll
    for (int k = 0; k < CP_K; ++k) {
        const int e = k * 256 + threadIdx.x;
        const float v = a.x[xidx(e < total ? e : 0)];   // unconditional (clamped) load
        xp[k] = e < total ? v : 0.f;
    }
    const float sc = a.scale[0], ss = a.scale_shift[0];
    lds_zero(red, W2);
    tile_copy_in<T>(a.st, t.m0, t.tp, a.cs_st, st);
    __syncthreads();
    float sl = 0.f;
    auto body = [&](int e0, float xv) {
        const int e = e0 + threadIdx.x;
        const bool ok = e < total;
        const int c = ok ? e / t.tp : 0, pl = ok ? e - c * t.tp : 0, p = t.p0 + pl;
        const bool tr = ok && (g.kind == 0 ? !ckbd_m(g, p) : (c >= g.on_base && c < g.on_base + g.Cb));
        const int cb = g.kind == 0 ? c : c - g.on_base;
        float u = ok ? xv : 0.f;
        if (tr) {
            float lr, th, ex;
            u = coupling_u(u, ldv(&st[pl * a.cs_st + cb]), ldv(&st[pl * a.cs_st + g.Cb + cb]), sc, ss, lr, th, ex);
            sl += lr;
        }
        const int q = pcls(nc, g, p);
        for (int k = 0; k < nc; ++k) {   // nc is uniform: every lane takes part in the segment sums
            const double s1 = seg_red(q == k ? (double)u : 0.0, seg), s2 = seg_red(q == k ? (double)u * u : 0.0, seg);
            if (ok && (lane & seg_mask(seg)) == 0) {
                atomicAdd(&red[(2 * k) * g.C + c], s1);
                atomicAdd(&red[(2 * k + 1) * g.C + c], s2);
            }
        }
    };
#pragma unroll
    for (int k = 0; k < CP_K; ++k)
        if (k * 256 < total) body(k * 256, xp[k]);
    for (int e0 = CP_K * 256; e0 < total; e0 += 256) {
        const int e = e0 + threadIdx.x;
        const float v = a.x[xidx(e < total ? e : 0)];
        body(e0, e < total ? v : 0.f);
    }
    const float dl = block_sum(sl, redl);   // (barriers also publish red)
    if (threadIdx.x == 0 && dl != 0.f) atomicAdd(&a.ldj_sample[t.b], dl);
    double* dst = cshard(a.cls_sums, W2);
    for (int i = threadIdx.x; i < W2; i += blockDim.x) atomicAdd(&dst[i], red[i]);
}

// ---------------------------------------------------------------------------
// forward: z, the consumer's input / in_bn / h0, the prior
// ---------------------------------------------------------------------------
template <typename T, int LT>
__global__ __launch_bounds__(256) void k_link_fwd(rnvp_coupling_args a, rnvp_coupling_args n, rnvp_link_args l,
                                                  int TP, int seg, int main_grid) {
    extern __shared__ double dsm[];
    __shared__ double redp[16];
    if ((int)blockIdx.x >= main_grid) {
        net_running_block(a, blockIdx.x - main_grid, dsm);
        return;
    }
    constexpr bool TO_N = LT != RNVP_LINK_FINAL;
    constexpr bool PRIOR = LT == RNVP_LINK_UNFACTOR || LT == RNVP_LINK_FINAL;
    const Geo ga = geo(a);
    const Geo gn = TO_N ? geo(n) : ga;
    const Tile t = tile_of(ga, TP);
    const int lane = threadIdx.x & 63;
    const int nc = a.nclass, W2 = nc * 2 * ga.C, W2p = PRIOR ? W2 : 0;
    const int Cba = ga.Cb, Cra = r4(Cba);
    const int Cbn = TO_N ? gn.Cb : 0, Crn = r4(Cbn);
    double* cs = dsm;                // a's class sums, reduced [nc][2][C]
    double* pred = cs + W2;          // this block's prior sums [nc][2][C]
    float* ot = (float*)(pred + W2p);   // a's out_bn: mean | rstd | half log var [Cra each]
    float* it = ot + 3 * Cra;           // n's in_bn: scale | shift [Crn each]
    T* sta = (T*)(it + 2 * Crn);        // a's net output tile [tp][cs_st]
    T* h = sta + TP * a.cs_st;          // n's h0 tile [tpn][cs_h0]
    const int pn0 = LT == RNVP_LINK_SQUEEZE ? t.p0 / 4 : t.p0;   // the tile's first pixel of n
    const int tpn = LT == RNVP_LINK_SQUEEZE ? t.tp / 4 : t.tp;
    const int csn = TO_N ? n.cs_h0 : 0;
    const int total = ga.C * t.tp;
    const double cnt_a = (double)ga.B * ga.HW, cnt_n = (double)gn.B * gn.HW;
    auto xidx = [&](int e) {
        const int c = e / t.tp, pl = e - c * t.tp;
        return ((long long)t.b * ga.C + c) * ga.HW + t.p0 + pl;
    };
    float xp[CP_K];
#pragma unroll
    for (int k = 0; k < CP_K; ++k) {
        const int e = k * 256 + threadIdx.x;
        const float v = a.x[xidx(e < total ? e : 0)];
        xp[k] = e < total ? v : 0.f;
    }
    const float glp = (PRIOR && l.g_lp) ? l.g_lp[t.b] : 0.f;   // the prior's gradient weight
    const float sc = a.scale[0], ss = a.scale_shift[0];
    const int ci = (int)threadIdx.x;   // this thread's in_bn channel of n in the table phase (Cbn <= 256 here)
    const float gam0 = (TO_N && ci < Cbn && n.in_gamma) ? n.in_gamma[ci] : 1.f;
    const float bet0 = (TO_N && ci < Cbn && n.in_beta) ? n.in_beta[ci] : 0.f;
    // the tile's loads go out with the class sums' (one round trip), LDS stores after
    TileRegs<2> rst;
    tile_issue<T, 2>(a.st, t.m0, t.tp, a.cs_st, rst);
    {
        const ShardArr arrs[1] = {{a.cls_sums, W2, cs}};
        lds_shard_reduce_multi(arrs);
    }
    tile_commit<T, 2>(rst, a.st, t.m0, a.cs_st, sta);
    if (PRIOR) lds_zero(pred, W2p);
    if constexpr (TO_N) {   // n's padding / mask channels of the h0 tile
        for (int e = threadIdx.x; e < tpn * csn; e += blockDim.x) {
            const int pl = e / csn, ch = e - pl * csn;
            if (ch >= 2 * Cbn) stv(&h[e], (gn.kind == 0 && ch == 2 * Cbn) ? (float)ckbd_m(gn, pn0 + pl) : 0.f);
        }
    }
    __syncthreads();
    // a's out_bn statistics; in the same phase n's in_bn statistics in closed form (the
    // class it reads is wholly transformed -- z = (u - mean) * rstd with a's fp32 mean /
    // rstd, recomputed here from the same sums -- or wholly kept: z = u)
    for (int cb = threadIdx.x; cb < Cba; cb += blockDim.x) {
        double mean, var;
        cls_out_stats(cs, ga, nc, cb, a.eps, mean, var);
        const float rstd = (float)(1.0 / sqrt(var + (double)a.eps));
        ot[cb] = (float)mean;
        ot[Cra + cb] = rstd;
        ot[2 * Cra + cb] = (float)(0.5 * log(var + (double)a.eps));
        if (blockIdx.x == 0) {
            if (a.out_tab) {   // for the link backward
                a.out_tab[cb] = (float)mean;
                a.out_tab[Cba + cb] = rstd;
            }
            if (a.out_rmean) {
                const double unb = cnt_a > 1 ? var * cnt_a / (cnt_a - 1) : var;
                a.out_rmean[cb] = (1.f - a.momentum) * a.out_rmean[cb] + a.momentum * (float)mean;
                a.out_rvar[cb] = (1.f - a.momentum) * a.out_rvar[cb] + a.momentum * (float)unb;
            }
        }
    }
    if (TO_N) {
        for (int cb = threadIdx.x; cb < Cbn; cb += blockDim.x) {
            int ca, q;
            link_src<LT>(gn, cb, ca, q);
            const double S1 = cs[(2 * q) * ga.C + ca], S2 = cs[(2 * q + 1) * ga.C + ca];
            double D1 = S1, D2 = S2;
            if (cls_tr(ga, nc, ca, q)) {
                const int cba = ga.kind == 0 ? ca : ca - ga.on_base;
                double am, av;
                cls_out_stats(cs, ga, nc, cba, a.eps, am, av);
                const double N = (double)ga.B * cls_count(nc, ga, q);
                const double m = (double)(float)am, r = (double)(float)(1.0 / sqrt(av + (double)a.eps));
                D1 = r * (S1 - N * m);
                D2 = r * r * (S2 - 2.0 * m * S1 + N * m * m);
                if (D2 < 0) D2 = 0;
            }
            const double mean = D1 / cnt_n;
            double var = D2 / cnt_n - mean * mean;
            if (var < 0) var = 0;
            const float rstd = (float)(1.0 / sqrt(var + (double)n.eps));
            const float gam = cb == ci ? gam0 : (n.in_gamma ? n.in_gamma[cb] : 1.f);
            const float bet = cb == ci ? bet0 : (n.in_beta ? n.in_beta[cb] : 0.f);
            it[cb] = gam * rstd;
            it[Crn + cb] = bet - (float)mean * gam * rstd;
            if (blockIdx.x == 0) {   // n's in_sums (shard 0 = the closed form; the others are zero) and running stats
                n.in_sums[cb] = D1;
                n.in_sums[Cbn + cb] = D2;
                if (n.in_tab) {   // for n's in part backward and the link backward
                    n.in_tab[cb] = gam * rstd;
                    n.in_tab[Cbn + cb] = bet - (float)mean * gam * rstd;
                    n.in_tab[2 * Cbn + cb] = (float)mean;
                    n.in_tab[3 * Cbn + cb] = rstd;
                }
                if (n.in_rmean) {
                    const double iu = cnt_n > 1 ? var * cnt_n / (cnt_n - 1) : var;
                    n.in_rmean[cb] = (1.f - n.momentum) * n.in_rmean[cb] + n.momentum * (float)mean;
                    n.in_rvar[cb] = (1.f - n.momentum) * n.in_rvar[cb] + n.momentum * (float)iu;
                }
            }
        }
    }
    __syncthreads();
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            if (a.out_nbt) a.out_nbt[0] += 1;
            if (TO_N && n.in_nbt) n.in_nbt[0] += 1;
        }
        // per-sample constant of a: -sum_c 0.5*log(var_c+eps) * (#transformed positions per channel)
        float k = 0.f;
        for (int cb = 0; cb < Cba; ++cb) k += ot[2 * Cra + cb];
        k = -k * (float)n_transformed(ga);
        for (int b = threadIdx.x; b < ga.B; b += blockDim.x) a.ldj_sample[b] += k;
    }
    double pacc = 0.0;
    float* nx = TO_N ? (float*)n.x : nullptr;
    auto body = [&](int e0, float xv) {
        const int e = e0 + threadIdx.x;
        const bool ok = e < total;
        const int c = ok ? e / t.tp : 0, pl = ok ? e - c * t.tp : 0, p = t.p0 + pl;
        const bool tr = ok && (ga.kind == 0 ? !ckbd_m(ga, p) : (c >= ga.on_base && c < ga.on_base + Cba));
        const int cb = ga.kind == 0 ? c : c - ga.on_base;
        float v = xv;
        if (tr) {
            float lr, th, ex;
            const float u = coupling_u(xv, ldv(&sta[pl * a.cs_st + cb]), ldv(&sta[pl * a.cs_st + Cba + cb]), sc, ss, lr,
                                       th, ex);
            v = (u - ot[cb]) * ot[Cra + cb];
        }
        const Dst d = link_dst<LT>(ga, gn, c, p);
        if (ok) {
            if (!d.to_prior) {
                nx[((long long)t.b * gn.C + d.c) * gn.HW + d.p] = v;
                const int cbn = in_bn_channel(gn, d.c);
                if (cbn >= 0) {
                    const float xm = (gn.kind == 0 && !ckbd_m(gn, d.p)) ? 0.f : v;
                    const float xa = xm * it[cbn] + it[Crn + cbn];
                    const int pnl = d.p - pn0;
                    stv(&h[pnl * csn + cbn], fmaxf(xa, 0.f));
                    stv(&h[pnl * csn + Cbn + cbn], fmaxf(-xa, 0.f));
                }
            } else {
                pacc += (double)(-0.5f * v * v - LOG_SQRT_2PI);
                if (LT == RNVP_LINK_UNFACTOR && l.off) l.off[((long long)t.b * gn.C + d.c) * gn.HW + d.p] = v;
                if (LT == RNVP_LINK_FINAL && l.z) l.z[((long long)t.b * ga.C + c) * ga.HW + p] = v;
            }
        }
        if (PRIOR) {   // dL/dz = -z * g_lp[b] of what goes to the prior: its sums for a's backward
            const int q = pcls(nc, ga, p);
            for (int k = 0; k < nc; ++k) {
                const bool m = ok && d.to_prior && q == k;
                const double s1 = seg_red(m ? -(double)v * glp : 0.0, seg);
                const double s2 = seg_red(m ? -(double)v * v * glp : 0.0, seg);
                if (ok && d.to_prior && (lane & seg_mask(seg)) == 0) {
                    atomicAdd(&pred[(2 * k) * ga.C + c], s1);
                    atomicAdd(&pred[(2 * k + 1) * ga.C + c], s2);
                }
            }
        }
    };
#pragma unroll
    for (int k = 0; k < CP_K; ++k)
        if (k * 256 < total) body(k * 256, xp[k]);
    for (int e0 = CP_K * 256; e0 < total; e0 += 256) {
        const int e = e0 + threadIdx.x;
        const float v = a.x[xidx(e < total ? e : 0)];
        body(e0, e < total ? v : 0.f);
    }
    if (PRIOR) {
        const double ps = block_sum(pacc, redp);   // (barriers also publish pred)
        if (threadIdx.x == 0) atomicAdd(&l.prior[t.b], ps);
        double* dst = cshard(a.prior_sums, W2p);
        for (int i = threadIdx.x; i < W2p; i += blockDim.x)
            if (pred[i] != 0.0) atomicAdd(&dst[i], pred[i]);
    }
    if (TO_N) {
        __syncthreads();
        tile_copy_out<T>(h, (long long)t.b * gn.HW + pn0, tpn, csn, n.h0);
    }
}

// ---------------------------------------------------------------------------
// backward: dL/dz of a from the consumer, then a's out part
// ---------------------------------------------------------------------------
template <typename T, int LT>
__global__ __launch_bounds__(256) void k_link_bwd(rnvp_coupling_args a, rnvp_coupling_args n, rnvp_link_args l, int TP,
                                                  int seg) {
    extern __shared__ double dsm[];
    __shared__ double redl[32];
    __shared__ double gls_sh;
    constexpr bool TO_N = LT != RNVP_LINK_FINAL;
    constexpr bool PRIOR = LT == RNVP_LINK_UNFACTOR || LT == RNVP_LINK_FINAL;
    LINK_STAMP(0);
    const Geo ga = geo(a);
    const Geo gn = TO_N ? geo(n) : ga;
    const Tile t = tile_of(ga, TP);
    const int lane = threadIdx.x & 63;
    const int nc = a.nclass, W2 = nc * 2 * ga.C, W2p = PRIOR ? W2 : 0;
    const int Cn = TO_N ? gn.C : 0, Cbn = TO_N ? gn.Cb : 0;
    const int Cba = ga.Cb, Cra = r4(Cba), Crn = r4(Cbn);
    double* psa = dsm;               // a's prior sums [nc][2][Ca]
    double* osn = psa + W2p;         // n's direct-gradient sums [2][2][Cn]
    double* ibn = osn + 4 * Cn;      // n's in_bwd_sums [2][Cbn]
    double* iex = ibn + 2 * Cbn;     // n's in_bwd_ext [2][Cbn]
    double* isn = iex + 2 * Cbn;     // n's in_sums, shard 0 (the closed form of the forward) [2][Cbn]
    double* red = isn + 2 * Cbn;     // this block's direct-gradient sums of a [2][2][Ca]
    float* ta = (float*)(red + 4 * ga.C);   // a: mean | rstd | kA | kB [Cra each]
    float* tn = ta + 4 * Cra;               // n: scale | shift | mean | rstd | k1 | k2 [Crn each]
    T* sta = (T*)(tn + 6 * Crn);            // a's net output tile [tp][cs_st]
    T* gs = sta + TP * a.cs_st;             // a's net output gradient tile [tp][cs_gst]
    T* gh = gs + TP * a.cs_gst;             // n's net input gradient tile [tpn][cs_gh0]
    const int pn0 = LT == RNVP_LINK_SQUEEZE ? t.p0 / 4 : t.p0;
    const int tpn = LT == RNVP_LINK_SQUEEZE ? t.tp / 4 : t.tp;
    const int csg = TO_N ? n.cs_gh0 : 0;
    const int total = ga.C * t.tp;
    const double cnt_a = (double)ga.B * ga.HW, cnt_n = (double)gn.B * gn.HW;
    auto aidx = [&](int e) {
        const int c = e / t.tp, pl = e - c * t.tp;
        return ((long long)t.b * ga.C + c) * ga.HW + t.p0 + pl;
    };
    // the consumer's direct gradient of element e (clamped, unconditional: no branch around the load)
    auto gn_ld = [&](int e) -> float {
        if (!TO_N) return 0.f;
        const int c = e / t.tp, pl = e - c * t.tp;
        const Dst d = link_dst<LT>(ga, gn, c, t.p0 + pl);
        const long long i = ((long long)t.b * gn.C + (d.to_prior ? 0 : d.c)) * gn.HW + (d.to_prior ? 0 : d.p);
        const float v = n.gx[i];
        return d.to_prior ? 0.f : v;
    };
    // ---- phase 1: every global load of the table phase in flight together
    float xp[CP_K], gp[CP_K];
#pragma unroll
    for (int k = 0; k < CP_K; ++k) {
        const int e = k * 256 + threadIdx.x;
        const int ec = e < total ? e : 0;
        xp[k] = a.x[aidx(ec)];
        gp[k] = gn_ld(ec);
    }
    const int tid = (int)threadIdx.x;
    const float glp = a.gl_sample ? a.gl_sample[t.b] : 0.f;           // log-det gradient of sample b
    const float gpr = (PRIOR && l.g_lp) ? l.g_lp[t.b] : 0.f;         // the prior's gradient weight
    const float sc = a.scale[0], ss = a.scale_shift[0];
    float glv[4];   // wave 0: the per-sample log-det gradients (summed after the round trip)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int b = tid + 64 * k;
        const float v = a.gl_sample ? a.gl_sample[b < ga.B ? b : 0] : 0.f;
        glv[k] = (tid < 64 && b < ga.B) ? v : 0.f;
    }
    // the forward's tables: a's out_bn (mean, rstd), n's in_bn (scale, shift, mean, rstd),
    // n's closed-form in_sums (shard 0); up to 2 / 4 / 2 entries per thread
    const int nta = 2 * Cba, ntn = 4 * Cbn, nsn = 2 * Cbn;
    float tav[2], tnv[2];
    double snv[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int i = tid + 256 * k;
        tav[k] = a.out_tab[i < nta ? i : 0];
        tnv[k] = TO_N ? n.in_tab[i < ntn ? i : 0] : 0.f;
        snv[k] = TO_N ? n.in_sums[i < nsn ? i : 0] : 0.0;
    }
    TileRegs<2> rst, rgh;
    tile_issue<T, 2>(a.st, t.m0, t.tp, a.cs_st, rst);
    if (TO_N) tile_issue<T, 2>(n.gh0, (long long)t.b * gn.HW + pn0, tpn, csg, rgh);
    {
        const ShardArr arrs[4] = {{PRIOR ? a.prior_sums : a.cls_sums, W2p, psa},
                                  {TO_N ? n.outp_sums : a.cls_sums, 4 * Cn, osn},
                                  {TO_N ? n.in_bwd_sums : a.cls_sums, 2 * Cbn, ibn},
                                  {TO_N ? n.in_bwd_ext : a.cls_sums, 2 * Cbn, iex}};
        lds_shard_reduce_multi(arrs);
    }
    // (every load above has returned: commit to LDS)
    tile_commit<T, 2>(rst, a.st, t.m0, a.cs_st, sta);
    if (TO_N) tile_commit<T, 2>(rgh, n.gh0, (long long)t.b * gn.HW + pn0, csg, gh);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int i = tid + 256 * k;
        if (i < nta) ta[(i / Cba) * Cra + i % Cba] = tav[k];
        if constexpr (TO_N) {
            if (i < ntn) tn[(i / Cbn) * Crn + i % Cbn] = tnv[k];
        }
        if (i < nsn) isn[i] = snv[k];
    }
    if constexpr (TO_N) {
        for (int i = tid + 512; i < ntn; i += blockDim.x) tn[(i / Cbn) * Crn + i % Cbn] = n.in_tab[i];   // > 128 ch.
    }
    if (tid < 64) {   // sum_b dL/dlog_prob[b]: the log-det gradient of every transformed position
        double s = (double)glv[0] + (double)glv[1] + (double)glv[2] + (double)glv[3];
        if (a.gl_sample)
            for (int b = tid + 256; b < ga.B; b += 64) s += (double)a.gl_sample[b];
        s = wave_sum(s);
        if (tid == 0) gls_sh = s;
    }
    lds_zero(red, 4 * ga.C);
    for (int e = tid; e < t.tp * a.cs_gst; e += blockDim.x) stv(&gs[e], 0.f);
    __syncthreads();
    LINK_STAMP(1);
    // ---- phase 2: n's in_bn backward coefficients; a's out_bn backward coefficients from
    // closed-form sums of dL/dz and dL/dz * xhat over a's transformed positions (what
    // k_out_bwd_red would reduce); k1 / k2 as the in part rounds them
    for (int cb = tid; cb < Cbn; cb += blockDim.x) {
        tn[4 * Crn + cb] = (float)(ibn[cb] / cnt_n);
        tn[5 * Crn + cb] = (float)(ibn[Cbn + cb] / cnt_n);
        if (blockIdx.x == 0) {   // n's in_bn affine gradients (k_in_bwd_apply's block 0)
            if (n.g_in_beta) n.g_in_beta[cb] = (float)ibn[cb];
            if (n.g_in_gamma) n.g_in_gamma[cb] = (float)ibn[Cbn + cb];
        }
    }
    for (int cb = tid; cb < Cba; cb += blockDim.x) {
        const int ca = ga.kind == 0 ? cb : ga.on_base + cb;
        double A = 0.0, Bs = 0.0;
        for (int q = 0; q < nc; ++q) {
            if (!cls_tr(ga, nc, ca, q)) continue;
            const Dst d = link_dst<LT>(ga, gn, ca, 0);   // channel routing only (pixel 0)
            const bool prior_cls = PRIOR && (LT == RNVP_LINK_FINAL || d.to_prior);
            if (prior_cls) {
                A += psa[(2 * q) * ga.C + ca];
                Bs += psa[(2 * q + 1) * ga.C + ca];
                continue;
            }
            int cn, qn;   // the consumer's channel and parity class (-1 = both) of class (ca, q)
            if (LT == RNVP_LINK_SAME) {
                cn = ca;
                qn = gn.kind == 0 ? q : -1;
            } else if (LT == RNVP_LINK_SQUEEZE) {
                cn = 4 * ca + q;
                qn = -1;
            } else {
                cn = (ca & 3) == 0 ? (ca >> 2) : gn.C / 2 + (ca >> 2);
                qn = q;
            }
            for (int k = 0; k < 2; ++k)
                if (qn < 0 || qn == k) {
                    A += osn[(2 * k) * Cn + cn];
                    Bs += osn[(2 * k + 1) * Cn + cn];
                }
            const int cbn = in_bn_channel(gn, cn);
            if (cbn >= 0 && (gn.kind == 1 || qn == ((gn.cfg + 1) & 1))) {
                // n's in_bn backward over its whole normalised set S (= this class)
                const double NS = (double)gn.B * (gn.kind == 0 ? (double)gn.HW - n_transformed(gn) : (double)gn.HW);
                const double GA = iex[cbn], GAV = iex[Cbn + cbn], SV = isn[cbn], SV2 = isn[Cbn + cbn];
                const double coef = tn[cbn], mi = tn[2 * Crn + cbn], ri = tn[3 * Crn + cbn];
                const double k1 = (float)(ibn[cbn] / cnt_n), k2 = (float)(ibn[Cbn + cbn] / cnt_n);
                const double Sxh = ri * (SV - NS * mi), Sxhv = ri * (SV2 - mi * SV);
                A += coef * (GA - NS * k1 - k2 * Sxh);
                Bs += coef * (GAV - k1 * SV - k2 * Sxhv);
            }
        }
        const double G = gls_sh * n_transformed(ga);
        ta[2 * Cra + cb] = (float)(A / cnt_a);
        ta[3 * Cra + cb] = (float)((Bs + G) / cnt_a);
    }
    __syncthreads();
    LINK_STAMP(2);
    double gsc = 0.0, gss = 0.0;
    auto body = [&](int e0, float xv, float gnv) {
        const int e = e0 + threadIdx.x;
        const bool ok = e < total;
        const int c = ok ? e / t.tp : 0, pl = ok ? e - c * t.tp : 0, p = t.p0 + pl;
        const bool chan_on = ga.kind == 1 && c >= ga.on_base && c < ga.on_base + Cba;
        const int cb = ga.kind == 0 ? c : (chan_on ? c - ga.on_base : 0);
        const bool has_bn = ga.kind == 0 || chan_on;
        const bool tr = ok && (ga.kind == 0 ? !ckbd_m(ga, p) : chan_on);
        float v = xv, th = 0.f, ex = 1.f;
        if (tr) {
            float lr;
            const float u = coupling_u(xv, ldv(&sta[pl * a.cs_st + cb]), ldv(&sta[pl * a.cs_st + Cba + cb]), sc, ss, lr,
                                       th, ex);
            v = (u - ta[cb]) * ta[Cra + cb];
        }
        // dL/dz
        float gz = 0.f;
        if (ok) {
            const Dst d = link_dst<LT>(ga, gn, c, p);
            if (d.to_prior) {
                gz = -v * gpr;
            } else {
                gz = gnv;
                const int cbn = in_bn_channel(gn, d.c);
                if (cbn >= 0 && (gn.kind != 0 || ckbd_m(gn, d.p))) {   // n's in_bn backward (k_in_bwd_apply)
                    const int pnl = d.p - pn0;
                    const float xa = v * tn[cbn] + tn[Crn + cbn];
                    const float g1 = ldv(&gh[pnl * csg + cbn]), g2 = ldv(&gh[pnl * csg + Cbn + cbn]);
                    const float gxa = (xa > 0.f ? g1 : 0.f) - (xa < 0.f ? g2 : 0.f);
                    const float xh = (v - tn[2 * Crn + cbn]) * tn[3 * Crn + cbn];
                    gz = gnv + tn[cbn] * (gxa - tn[4 * Crn + cbn] - xh * tn[5 * Crn + cbn]);
                }
            }
        }
        // a's out part (k_out_bwd_apply)
        float gu = gz;
        if (has_bn) {
            const float fm = ta[cb], rstd = ta[Cra + cb], kA = ta[2 * Cra + cb], kB = ta[3 * Cra + cb];
            if (!tr) gu = gz + rstd * (-kA - (xv - fm) * rstd * kB);   // kept square: z = u, but u moves the stats
            else gu = rstd * (gz - kA - v * kB);
        }
        float gxo = gu;
        if (tr) {
            gxo = gu * ex;
            const float glr = gu * xv * ex + glp;
            stv(&gs[pl * a.cs_gst + cb], gu);
            stv(&gs[pl * a.cs_gst + Cba + cb], glr * sc * (1.f - th * th));
            gsc += (double)glr * th;
            gss += glr;
        }
        if (ok) a.gx[((long long)t.b * ga.C + c) * ga.HW + p] = gxo;
        // sums of a's direct input gradient for the previous link's closed form
        const int q2 = pcls(2, ga, p);
        for (int k = 0; k < 2; ++k) {
            const bool m = ok && q2 == k;
            const double s1 = seg_red(m ? (double)gxo : 0.0, seg), s2 = seg_red(m ? (double)gxo * xv : 0.0, seg);
            if (ok && (lane & seg_mask(seg)) == 0) {
                atomicAdd(&red[(2 * k) * ga.C + c], s1);
                atomicAdd(&red[(2 * k + 1) * ga.C + c], s2);
            }
        }
    };
#pragma unroll
    for (int k = 0; k < CP_K; ++k)
        if (k * 256 < total) body(k * 256, xp[k], gp[k]);
    for (int e0 = CP_K * 256; e0 < total; e0 += 256) {
        const int e = e0 + threadIdx.x;
        const int ec = e < total ? e : 0;
        const float xv = a.x[aidx(ec)], gv = gn_ld(ec);
        body(e0, e < total ? xv : 0.f, e < total ? gv : 0.f);
    }
    LINK_STAMP(3);
    block_sum2(gsc, gss, redl);   // (barriers also publish gs and red)
    const float dsc = (float)gsc, dss = (float)gss;
    LINK_STAMP(4);
    tile_copy_out<T>(gs, t.m0, t.tp, a.cs_gst, a.gst);
    if (threadIdx.x == 0 && (dsc != 0.f || dss != 0.f)) {
        double* sp = a.gscale_part + 2 * (blockIdx.x % RNVP_COUPLING_SHARDS);
        atomicAdd(sp, (double)dsc);
        atomicAdd(sp + 1, (double)dss);
    }
    if (a.outp_sums) {
        double* dst = cshard(a.outp_sums, 4 * ga.C);
        for (int i = threadIdx.x; i < 4 * ga.C; i += blockDim.x) atomicAdd(&dst[i], red[i]);
    }
    __syncthreads();
    LINK_STAMP(5);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
int link_nclass(int type, int kind) {
    switch (type) {
        case RNVP_LINK_SAME: return kind == 0 ? 2 : 1;
        case RNVP_LINK_SQUEEZE: return 4;
        case RNVP_LINK_UNFACTOR: return 2;
        case RNVP_LINK_FINAL: return kind == 0 ? 2 : 1;
    }
    return -1;
}

int base_check(const rnvp_coupling_args* a) {
    if (!a || !a->x || a->B < 0 || a->C <= 0 || a->H <= 0 || a->W <= 0) return RNVP_E_INVALID;
    if (a->kind != 0 && a->kind != 1) return RNVP_E_INVALID;
    if (a->kind == 1 && (a->C & 1)) return RNVP_E_INVALID;
    if (a->dtype != RNVP_F32 && a->dtype != RNVP_BF16) return RNVP_E_INVALID;
    if (!a->training || !a->coupling_bn) return RNVP_E_INVALID;
    if (a->nclass != 1 && a->nclass != 2 && a->nclass != 4) return RNVP_E_INVALID;
    if (!a->st || !a->cls_sums || !a->scale || !a->scale_shift || a->cs_st < 2 * (a->kind == 0 ? a->C : a->C / 2))
        return RNVP_E_INVALID;
    return RNVP_OK;
}

// a -> n geometry of the link type
int link_check(const rnvp_coupling_args* a, const rnvp_coupling_args* n, const rnvp_link_args* l) {
    if (!l || base_check(a)) return RNVP_E_INVALID;
    if (a->nclass != link_nclass(l->type, a->kind)) return RNVP_E_INVALID;
    if (l->type == RNVP_LINK_FINAL) return n == nullptr ? RNVP_OK : RNVP_E_INVALID;
    if (!n || !n->x || n->B != a->B || n->dtype != a->dtype || !n->training) return RNVP_E_INVALID;
    if (n->kind != 0 && n->kind != 1) return RNVP_E_INVALID;
    switch (l->type) {
        case RNVP_LINK_SAME:
            if (n->kind != a->kind || n->C != a->C || n->H != a->H || n->W != a->W) return RNVP_E_INVALID;
            if ((n->mask_config ? 1 : 0) == (a->mask_config ? 1 : 0)) return RNVP_E_INVALID;
            return RNVP_OK;
        case RNVP_LINK_SQUEEZE:
            if (a->kind != 0 || n->kind != 1 || n->C != 4 * a->C || (a->H & 1) || (a->W & 1)) return RNVP_E_INVALID;
            if (n->H != a->H / 2 || n->W != a->W / 2) return RNVP_E_INVALID;
            return RNVP_OK;
        case RNVP_LINK_UNFACTOR:
            if (a->kind != 1 || n->kind != 0 || (a->C & 3) || n->C != a->C / 2) return RNVP_E_INVALID;
            if (n->H != a->H || n->W != a->W) return RNVP_E_INVALID;
            return RNVP_OK;
    }
    return RNVP_E_INVALID;
}

struct LinkTile {
    int TP, seg, grid;
};
// pixel tiles of a: <= 256 px, the NHWC tiles within ~48 KB of LDS, >= 512
// workgroups where the image allows; a squeeze link's tile is whole pairs of
// a's rows (= whole rows of n's pixels) and divides H*W
LinkTile link_tile(const rnvp_coupling_args* a, int cs_sum, bool squeeze) {
    const int HW = a->H * a->W;
    const int esz = a->dtype == RNVP_F32 ? 4 : 2;
    if (cs_sum < 8) cs_sum = 8;
    LinkTile c;
    c.TP = HW < 256 ? HW : 256;
    while (c.TP > 16 && (long long)c.TP * cs_sum * esz > 48 * 1024) c.TP /= 2;
    while (c.TP > 4 && c.TP % 2 == 0 && (long long)a->B * ((HW + c.TP - 1) / c.TP) < 512) c.TP /= 2;
    if (squeeze) {
        const int q = 2 * a->W;
        int tp = c.TP < q ? q : c.TP / q * q;
        while (tp > q && HW % tp) tp -= q;
        c.TP = tp;
    }
    int seg = 1;
    while (seg < 64 && c.TP % (2 * seg) == 0 && HW % (2 * seg) == 0) seg *= 2;
    c.seg = seg;
    c.grid = a->B * ((HW + c.TP - 1) / c.TP);
    return c;
}

template <int LT>
void launch_fwd(const rnvp_coupling_args* a, const rnvp_coupling_args* n, const rnvp_link_args* l, const LinkTile& tc,
                int nrun, size_t shm, hipStream_t s) {
    const rnvp_coupling_args nn = n ? *n : *a;
    if (a->dtype == RNVP_F32) k_link_fwd<float, LT><<<tc.grid + nrun, 256, shm, s>>>(*a, nn, *l, tc.TP, tc.seg, tc.grid);
    else k_link_fwd<bf16_t, LT><<<tc.grid + nrun, 256, shm, s>>>(*a, nn, *l, tc.TP, tc.seg, tc.grid);
}

template <int LT>
void launch_bwd(const rnvp_coupling_args* a, const rnvp_coupling_args* n, const rnvp_link_args* l, const LinkTile& tc,
                size_t shm, hipStream_t s) {
    const rnvp_coupling_args nn = n ? *n : *a;
    if (a->dtype == RNVP_F32) k_link_bwd<float, LT><<<tc.grid, 256, shm, s>>>(*a, nn, *l, tc.TP, tc.seg);
    else k_link_bwd<bf16_t, LT><<<tc.grid, 256, shm, s>>>(*a, nn, *l, tc.TP, tc.seg);
}

}  // namespace

extern "C" int rnvp_link_nclass(int type, int kind) { return link_nclass(type, kind); }

extern "C" int rnvp_coupling_out_u(const rnvp_coupling_args* a, void* stream) {
    if (base_check(a) || !a->ldj_sample) return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    const LinkTile tc = link_tile(a, a->cs_st, false);
    const int esz = a->dtype == RNVP_F32 ? 4 : 2;
    const size_t shm = 8 * (size_t)(a->nclass * 2 * a->C) + (size_t)tc.TP * a->cs_st * esz;
    hipStream_t s = (hipStream_t)stream;
    if (a->dtype == RNVP_F32) k_out_u<float><<<tc.grid, 256, shm, s>>>(*a, tc.TP, tc.seg);
    else k_out_u<bf16_t><<<tc.grid, 256, shm, s>>>(*a, tc.TP, tc.seg);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_coupling_link_fwd(const rnvp_coupling_args* a, const rnvp_coupling_args* n,
                                      const rnvp_link_args* l, void* stream) {
    if (link_check(a, n, l)) return RNVP_E_INVALID;
    const bool to_n = l->type != RNVP_LINK_FINAL, prior = l->type == RNVP_LINK_UNFACTOR || l->type == RNVP_LINK_FINAL;
    if (!a->ldj_sample || !a->out_tab || (prior && (!l->prior || !a->prior_sums))) return RNVP_E_INVALID;
    if (to_n && (!n->h0 || !n->in_sums || !n->in_tab || n->cs_h0 < (n->kind == 0 ? 2 * n->C + 1 : n->C)))
        return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    const int nrun = a->net_running ? a->n_net_running : 0;
    if (nrun < 0 || (nrun > 0 && a->net_running_cmax <= 0)) return RNVP_E_INVALID;
    const bool sq = l->type == RNVP_LINK_SQUEEZE;
    const LinkTile tc = link_tile(a, a->cs_st + (to_n ? n->cs_h0 : 0), sq);
    const int esz = a->dtype == RNVP_F32 ? 4 : 2;
    const int Cba = a->kind == 0 ? a->C : a->C / 2, Cbn = to_n ? (n->kind == 0 ? n->C : n->C / 2) : 0;
    const int W2 = a->nclass * 2 * a->C;
    const int tpn = sq ? tc.TP / 4 : tc.TP;
    size_t shm = 8 * (size_t)(W2 + (prior ? W2 : 0)) + 4 * (size_t)(3 * r4(Cba) + 2 * r4(Cbn)) +
                 (size_t)tc.TP * a->cs_st * esz + (to_n ? (size_t)tpn * n->cs_h0 * esz : 0);
    if (nrun > 0 && 16 * (size_t)a->net_running_cmax > shm) shm = 16 * (size_t)a->net_running_cmax;
    if (shm > 160 * 1024) return RNVP_E_UNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    switch (l->type) {
        case RNVP_LINK_SAME: launch_fwd<RNVP_LINK_SAME>(a, n, l, tc, nrun, shm, s); break;
        case RNVP_LINK_SQUEEZE: launch_fwd<RNVP_LINK_SQUEEZE>(a, n, l, tc, nrun, shm, s); break;
        case RNVP_LINK_UNFACTOR: launch_fwd<RNVP_LINK_UNFACTOR>(a, n, l, tc, nrun, shm, s); break;
        default: launch_fwd<RNVP_LINK_FINAL>(a, n, l, tc, nrun, shm, s); break;
    }
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_coupling_link_bwd(const rnvp_coupling_args* a, const rnvp_coupling_args* n,
                                      const rnvp_link_args* l, void* stream) {
    if (link_check(a, n, l)) return RNVP_E_INVALID;
    const bool to_n = l->type != RNVP_LINK_FINAL, prior = l->type == RNVP_LINK_UNFACTOR || l->type == RNVP_LINK_FINAL;
    const int Cba = a->kind == 0 ? a->C : a->C / 2;
    if (!a->gx || !a->gst || a->cs_gst < 2 * Cba || !a->gscale_part || (prior && !a->prior_sums) || !a->out_tab)
        return RNVP_E_INVALID;
    if (to_n && (!n->gx || !n->gh0 || !n->in_sums || !n->in_tab || !n->in_bwd_sums || !n->in_bwd_ext || !n->outp_sums ||
                 n->cs_gh0 < (n->kind == 0 ? 2 * n->C : n->C)))
        return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    const bool sq = l->type == RNVP_LINK_SQUEEZE;
    const LinkTile tc = link_tile(a, a->cs_st + a->cs_gst + (to_n ? n->cs_gh0 : 0), sq);
    const int esz = a->dtype == RNVP_F32 ? 4 : 2;
    const int Cn = to_n ? n->C : 0, Cbn = to_n ? (n->kind == 0 ? n->C : n->C / 2) : 0;
    const int W2 = a->nclass * 2 * a->C;
    const int tpn = sq ? tc.TP / 4 : tc.TP;
    const size_t shm = 8 * (size_t)((prior ? W2 : 0) + 4 * Cn + 6 * Cbn + 4 * a->C) +
                       4 * (size_t)(4 * r4(Cba) + 6 * r4(Cbn)) + (size_t)tc.TP * (a->cs_st + a->cs_gst) * esz +
                       (to_n ? (size_t)tpn * n->cs_gh0 * esz : 0);
    if (shm > 160 * 1024) return RNVP_E_UNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    switch (l->type) {
        case RNVP_LINK_SAME: launch_bwd<RNVP_LINK_SAME>(a, n, l, tc, shm, s); break;
        case RNVP_LINK_SQUEEZE: launch_bwd<RNVP_LINK_SQUEEZE>(a, n, l, tc, shm, s); break;
        case RNVP_LINK_UNFACTOR: launch_bwd<RNVP_LINK_UNFACTOR>(a, n, l, tc, shm, s); break;
        default: launch_bwd<RNVP_LINK_FINAL>(a, n, l, tc, shm, s); break;
    }
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}
