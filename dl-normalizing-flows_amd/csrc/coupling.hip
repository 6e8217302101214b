// Affine coupling layers (modules_realnvp.py:239-370) around the s/t ResNet.
//
// "in"  part: mask apply + in_bn (batch stats) + CReLU/mask concat  -> net input h0 (NHWC)
// "out" part: scale*tanh+shift, masked affine, out_bn with the batch-variance
//             log|det J| term, per-sample log-det accumulation       -> z, ldj[b]
// plus the exact inverse (reverse=True, running out_bn stats) and the
// backward of both parts, including the cross-sample batch-variance gradient.
//
// Flow tensors are NCHW fp32, net tensors NHWC; the reductions and the
// NHWC-touching passes run on pixel tiles (see "pixel tiles" below), the
// purely elementwise NCHW passes grid-stride.
#include "coupling_common.h"

namespace {

// ---------------------------------------------------------------------------
// in part, forward
// ---------------------------------------------------------------------------
// sums of xm and xm^2 per in_bn channel
__global__ __launch_bounds__(256) void k_in_stats(rnvp_coupling_args a, int TP, int seg) {
    extern __shared__ double red[];   // [2*Cb]
    const Geo g = geo(a);
    const Tile t = tile_of(g, TP);
    const int lane = threadIdx.x & 63;
    const int total = g.Cb * t.tp;
    auto xidx = [&](int e) {
        const int cb = e / t.tp, p = t.p0 + (e - cb * t.tp);
        const int c = (g.kind == 0) ? cb : g.off_base + cb;
        return ((long long)t.b * g.C + c) * g.HW + p;
    };
    float xp[CP_K];
#pragma unroll
    for (int k = 0; k < CP_K; ++k) {
        const int e = k * 256 + threadIdx.x;
        { const float v = a.x[xidx(e < total ? e : 0)]; xp[k] = e < total ? v : 0.f; }   // unconditional (clamped) load: no branch, no wait
    }
    lds_zero(red, 2 * g.Cb);
    __syncthreads();
    auto body = [&](int e0, float xv) {
        const int e = e0 + threadIdx.x;
        const bool ok = e < total;
        const int cb = ok ? e / t.tp : 0, p = t.p0 + (ok ? e - cb * t.tp : 0);
        float v = ok ? xv : 0.f;
        if (g.kind == 0 && !ckbd_m(g, p)) v = 0.f;
        const double s1 = seg_red((double)v, seg), s2 = seg_red((double)v * v, seg);
        if (ok && (lane & seg_mask(seg)) == 0) {
            atomicAdd(&red[cb], s1);
            atomicAdd(&red[g.Cb + cb], s2);
        }
    };
#pragma unroll
    for (int k = 0; k < CP_K; ++k)
        if (k * 256 < total) body(k * 256, xp[k]);
    for (int e0 = CP_K * 256; e0 < total; e0 += 256) {
        const int e = e0 + threadIdx.x;
        { const float v = a.x[xidx(e < total ? e : 0)]; body(e0, e < total ? v : 0.f); }
    }
    __syncthreads();
    double* dst = cshard(a.in_sums, 2 * g.Cb);
    for (int c = threadIdx.x; c < 2 * g.Cb; c += blockDim.x) atomicAdd(&dst[c], red[c]);
}

// h0[m][ch] NHWC: relu(xa), relu(-xa) [, mask], zero pad; built in LDS, stored
// as one contiguous region.  Block 0 updates the in_bn running stats.
template <typename T>
__global__ __launch_bounds__(256) void k_in_apply(rnvp_coupling_args a, int TP, int seg) {
    extern __shared__ double dsm[];
    const Geo g = geo(a);
    const Tile t = tile_of(g, TP);
    float* tab = (float*)dsm;                   // [4*Cb]
    T* h = (T*)(tab + 4 * ((g.Cb + 3) / 4 * 4));  // [tp][cs_h0] (16-B aligned)
    const int cs = a.cs_h0;
    const int total = g.Cb * t.tp;
    auto xidx = [&](int e) {
        const int cb = e / t.tp, p = t.p0 + (e - cb * t.tp);
        const int c = (g.kind == 0) ? cb : g.off_base + cb;
        return ((long long)t.b * g.C + c) * g.HW + p;
    };
    float xp[CP_K];
#pragma unroll
    for (int k = 0; k < CP_K; ++k) {
        const int e = k * 256 + threadIdx.x;
        { const float v = a.x[xidx(e < total ? e : 0)]; xp[k] = e < total ? v : 0.f; }   // unconditional (clamped) load: no branch, no wait
    }
    in_bn_table(a, g, tab);
    if (blockIdx.x == 0 && a.training && a.in_tab) {   // the in_bn table for the backward (coupling links)
        for (int c = threadIdx.x; c < g.Cb; c += blockDim.x) {
            float sc, sf, mean, rstd;
            rnvp_bn_src s;
            s.shards = RNVP_COUPLING_SHARDS;
            s.sums = a.in_sums;
            s.count = (double)g.B * g.HW;
            s.mean = a.in_rmean; s.var = a.in_rvar;
            s.gamma = a.in_gamma; s.beta = a.in_beta; s.eps = a.eps;
            bn_affine(s, g.Cb, c, sc, sf, &mean, &rstd);
            a.in_tab[c] = sc;
            a.in_tab[g.Cb + c] = sf;
            a.in_tab[2 * g.Cb + c] = mean;
            a.in_tab[3 * g.Cb + c] = rstd;
        }
    }
    if (blockIdx.x == 0 && a.training && a.in_rmean) {
        const double cnt = (double)g.B * g.HW;
        for (int c = threadIdx.x; c < g.Cb; c += blockDim.x) {
            double mean = csum(a.in_sums, 2 * g.Cb, c) / cnt;
            double var = csum(a.in_sums, 2 * g.Cb, g.Cb + c) / cnt - mean * mean;
            if (var < 0) var = 0;
            double unb = cnt > 1 ? var * cnt / (cnt - 1) : var;
            a.in_rmean[c] = (1.f - a.momentum) * a.in_rmean[c] + a.momentum * (float)mean;
            a.in_rvar[c] = (1.f - a.momentum) * a.in_rvar[c] + a.momentum * (float)unb;
        }
        if (threadIdx.x == 0 && a.in_nbt) a.in_nbt[0] += 1;
    }
    // padding channels (and the mask channel) first
    for (int e = threadIdx.x; e < t.tp * cs; e += blockDim.x) {
        const int pl = e / cs, ch = e - pl * cs;
        if (ch >= 2 * g.Cb) {
            float out = 0.f;
            if (g.kind == 0 && ch == 2 * g.Cb) out = (float)ckbd_m(g, t.p0 + pl);   // relu(mask) = mask
            stv(&h[e], out);
        }
    }
    __syncthreads();
    auto body = [&](int e, float v) {
        const int cb = e / t.tp, pl = e - cb * t.tp, p = t.p0 + pl;
        if (g.kind == 0 && !ckbd_m(g, p)) v = 0.f;
        const float xa = v * tab[cb] + tab[g.Cb + cb];
        stv(&h[pl * cs + cb], fmaxf(xa, 0.f));
        stv(&h[pl * cs + g.Cb + cb], fmaxf(-xa, 0.f));
    };
#pragma unroll
    for (int k = 0; k < CP_K; ++k) {
        const int e = k * 256 + threadIdx.x;
        if (e < total) body(e, xp[k]);
    }
    for (int e = CP_K * 256 + threadIdx.x; e < total; e += 256) body(e, a.x[xidx(e)]);
    __syncthreads();
    tile_copy_out<T>(h, t.m0, t.tp, cs, a.h0);
}

// ---------------------------------------------------------------------------
// out part, forward
// ---------------------------------------------------------------------------
// u = x*exp(lr)+shift on transformed positions (x elsewhere); stats of u over
// the out_bn channels; ldj_sample[b] += sum lr.
template <typename T>
__global__ __launch_bounds__(256) void k_out1(rnvp_coupling_args a, int TP, int seg) {
    extern __shared__ double dsm[];
    const Geo g = geo(a);
    const Tile t = tile_of(g, TP);
    const int lane = threadIdx.x & 63;
    double* red = dsm;                          // [2*Cb] (+ pad to 16 B): out_bn sums
    __shared__ float redl[16];
    T* st = (T*)(dsm + 2 * ((g.Cb + 1) / 2 * 2));   // [tp][cs_st]
    const int total = g.C * t.tp;
    auto xidx = [&](int e) {
        const int c = e / t.tp, pl = e - c * t.tp;
        return ((long long)t.b * g.C + c) * g.HW + t.p0 + pl;
    };
    float xp[CP_K];
#pragma unroll
    for (int k = 0; k < CP_K; ++k) {
        const int e = k * 256 + threadIdx.x;
        { const float v = a.x[xidx(e < total ? e : 0)]; xp[k] = e < total ? v : 0.f; }   // unconditional (clamped) load: no branch, no wait
    }
    lds_zero(red, 2 * g.Cb);
    tile_copy_in<T>(a.st, t.m0, t.tp, a.cs_st, st);
    __syncthreads();
    const float sc = a.scale[0], ss = a.scale_shift[0];
    float sl = 0.f;
    auto body = [&](int e0, float xv) {
        const int e = e0 + threadIdx.x;
        const bool ok = e < total;
        const int c = ok ? e / t.tp : 0, pl = ok ? e - c * t.tp : 0, p = t.p0 + pl;
        const long long idx = ((long long)t.b * g.C + c) * g.HW + p;
        const bool chan_on = g.kind == 1 && c >= g.on_base && c < g.on_base + g.Cb;
        const int cb = g.kind == 0 ? c : c - g.on_base;
        const bool tr = ok && (g.kind == 0 ? !ckbd_m(g, p) : chan_on);
        float u = ok ? xv : 0.f;
        if (tr) {
            const float sh = ldv(&st[pl * a.cs_st + cb]);
            const float r = ldv(&st[pl * a.cs_st + g.Cb + cb]);
            const float lr = sc * tanhf(r) + ss;
            u = u * expf(lr) + sh;
            sl += lr;
        }
        if (ok) a.u[idx] = u;
        const double s1 = seg_red((double)u, seg), s2 = seg_red((double)u * u, seg);
        if (ok && (g.kind == 0 || chan_on) && (lane & seg_mask(seg)) == 0) {
            atomicAdd(&red[cb], s1);
            atomicAdd(&red[g.Cb + cb], s2);
        }
    };
    // e0 is block-uniform (seg_sum shuffles need every lane)
#pragma unroll
    for (int k = 0; k < CP_K; ++k)
        if (k * 256 < total) body(k * 256, xp[k]);
    for (int e0 = CP_K * 256; e0 < total; e0 += 256) {
        const int e = e0 + threadIdx.x;
        { const float v = a.x[xidx(e < total ? e : 0)]; body(e0, e < total ? v : 0.f); }
    }
    const float dl = block_sum(sl, redl);   // (barriers also publish red)
    if (threadIdx.x == 0 && dl != 0.f) atomicAdd(&a.ldj_sample[t.b], dl);
    if (a.out_sums) {
        double* dst = cshard(a.out_sums, 2 * g.Cb);
        for (int c = threadIdx.x; c < 2 * g.Cb; c += blockDim.x) atomicAdd(&dst[c], red[c]);
    }
}

// z = out_bn(u) on transformed positions; ldj var term; running stats.
template <typename T>
__global__ void k_out2(rnvp_coupling_args a, int main_grid) {
    extern __shared__ float sh[];   // mean[Cb], rstd[Cb], half_log_var[Cb]
    if ((int)blockIdx.x >= main_grid) {
        // extra workgroups: one s/t-net BatchNorm running-stat update each
        // (the net's batch sums are complete: every conv ran before this launch)
        const rnvp_bn_running r = a.net_running[blockIdx.x - main_grid];
        double* tmp = (double*)sh;   // [2*C]
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
        return;
    }
    const Geo g = geo(a);
    const double cnt = (double)g.B * g.HW;
    const long long n = (long long)g.B * g.C * g.HW;
    const long long e_first = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    const float u_first = a.u[e_first < n ? e_first : 0];   // in flight under the table (clamped: no branch)
    for (int cb = threadIdx.x; cb < g.Cb; cb += blockDim.x) {
        double mean = 0, var = 1;
        if (a.coupling_bn) {
            if (a.training) {
                mean = csum(a.out_sums, 2 * g.Cb, cb) / cnt;
                var = csum(a.out_sums, 2 * g.Cb, g.Cb + cb) / cnt - mean * mean;
                if (var < 0) var = 0;
            } else {
                mean = a.out_rmean[cb];
                var = a.out_rvar[cb];
            }
        }
        sh[cb] = (float)mean;
        sh[g.Cb + cb] = (float)(1.0 / sqrt(var + (double)a.eps));
        sh[2 * g.Cb + cb] = a.coupling_bn ? (float)(0.5 * log(var + (double)a.eps)) : 0.f;
        if (blockIdx.x == 0 && a.training && a.coupling_bn && a.out_rmean) {
            double unb = cnt > 1 ? var * cnt / (cnt - 1) : var;
            a.out_rmean[cb] = (1.f - a.momentum) * a.out_rmean[cb] + a.momentum * (float)mean;
            a.out_rvar[cb] = (1.f - a.momentum) * a.out_rvar[cb] + a.momentum * (float)unb;
        }
    }
    __syncthreads();
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0 && a.training && a.coupling_bn && a.out_nbt) a.out_nbt[0] += 1;
        if (a.coupling_bn) {
            // per-sample constant: -sum_c 0.5*log(var_c+eps) * (#transformed positions per channel)
            float k = 0.f;
            for (int cb = 0; cb < g.Cb; ++cb) k += sh[2 * g.Cb + cb];
            k = -k * (float)n_transformed(g);
            for (int b = threadIdx.x; b < g.B; b += blockDim.x) a.ldj_sample[b] += k;
        }
    }
    const T* st = cptr<T>(a.st);
    const float sc = a.scale[0], ss = a.scale_shift[0];
    for (long long e = e_first; e < n; e += (long long)main_grid * blockDim.x) {
        const int p = (int)(e % g.HW);
        const long long t = e / g.HW;
        const int c = (int)(t % g.C);
        const long long b = t / g.C;
        bool tr;
        int cb;
        if (g.kind == 0) {
            tr = !ckbd_m(g, p);
            cb = c;
        } else {
            tr = c >= g.on_base && c < g.on_base + g.Cb;
            cb = c - g.on_base;
        }
        float u = e == e_first ? u_first : a.u[e];
        float zv = u;
        if (tr && a.coupling_bn) zv = (u - sh[cb]) * sh[g.Cb + cb];
        a.z[e] = zv;
        if (a.ldj_full) {
            float l = 0.f;
            if (tr) {
                const long long m = b * g.HW + p;
                float r = ldv(&st[m * a.cs_st + g.Cb + cb]);
                l = sc * tanhf(r) + ss - sh[2 * g.Cb + cb];
            }
            a.ldj_full[e] = l;
        }
    }
}

// ---------------------------------------------------------------------------
// inverse (reverse=True): running out_bn stats, (x - shift) * exp(-lr)
// ---------------------------------------------------------------------------
template <typename T>
__global__ void k_reverse(rnvp_coupling_args a) {
    const Geo g = geo(a);
    const T* st = cptr<T>(a.st);
    const float sc = a.scale[0], ss = a.scale_shift[0];
    const long long n = (long long)g.B * g.C * g.HW;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
        const int p = (int)(e % g.HW);
        const long long t = e / g.HW;
        const int c = (int)(t % g.C);
        const long long b = t / g.C;
        bool tr;
        int cb;
        if (g.kind == 0) {
            tr = !ckbd_m(g, p);
            cb = c;
        } else {
            tr = c >= g.on_base && c < g.on_base + g.Cb;
            cb = c - g.on_base;
        }
        float v = a.x[e];
        float lr = 0.f;
        if (tr) {
            if (a.coupling_bn) {
                float rv = a.out_rvar[cb], rm = a.out_rmean[cb];
                v = v * expf(0.5f * logf(rv + a.eps)) + rm;
            }
            const long long m = b * g.HW + p;
            float sh = ldv(&st[m * a.cs_st + cb]);
            float r = ldv(&st[m * a.cs_st + g.Cb + cb]);
            lr = sc * tanhf(r) + ss;
            v = (v - sh) * expf(-lr);
        }
        a.z[e] = v;
        if (a.ldj_full) a.ldj_full[e] = lr;   // the reference returns the masked log_rescale
    }
}

// backward of k_reverse (the inverse is differentiable in the reference:
// modules_realnvp.py:284-291): for a transformed element y = (v' - sh) E with
// v' = v sd + rm (running out_bn statistics, sd = sqrt(rv + eps)), E =
// exp(-lr), lr = scale tanh(r) + shift:  dv = gy sd E, d sh = -gy E,
// d lr = -gy y + gl (gl: the gradient of the returned log_diag_J = lr), d r =
// d lr scale (1 - tanh^2 r); kept elements pass gy through.  d sh / d r go to
// the net's output gradient (a.gst, NHWC), the scale / shift partials to the
// sharded gscale_part (folded by the in part's reduction, k_in_bwd_red).
template <typename T>
__global__ __launch_bounds__(256) void k_reverse_bwd(rnvp_coupling_args a, int TP) {
    extern __shared__ double dsm[];
    __shared__ double redl[16];
    const Geo g = geo(a);
    const Tile t = tile_of(g, TP);
    T* st = (T*)dsm;                                  // [tp][cs_st]
    T* gs = st + t.tp * a.cs_st;                      // [tp][cs_gst]
    const int total = g.C * t.tp;
    tile_copy_in<T>(a.st, t.m0, t.tp, a.cs_st, st);
    for (int e = threadIdx.x; e < t.tp * a.cs_gst; e += blockDim.x) stv(&gs[e], 0.f);
    __syncthreads();
    const float sc = a.scale[0], ss = a.scale_shift[0];
    double gsc = 0.0, gss = 0.0;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
        const int c = e / t.tp, pl = e - c * t.tp, p = t.p0 + pl;
        const long long idx = ((long long)t.b * g.C + c) * g.HW + p;
        bool tr;
        int cb;
        if (g.kind == 0) {
            tr = !ckbd_m(g, p);
            cb = c;
        } else {
            tr = c >= g.on_base && c < g.on_base + g.Cb;
            cb = c - g.on_base;
        }
        const float gy = a.gz[idx];
        if (!tr) {
            a.gx[idx] = gy;
            continue;
        }
        float v = a.x[idx], sd = 1.f;
        if (a.coupling_bn) {
            sd = expf(0.5f * logf(a.out_rvar[cb] + a.eps));
            v = v * sd + a.out_rmean[cb];
        }
        const float sh = ldv(&st[pl * a.cs_st + cb]), r = ldv(&st[pl * a.cs_st + g.Cb + cb]);
        const float th = tanhf(r);
        const float ex = expf(-(sc * th + ss));
        const float y = (v - sh) * ex;
        const float gl = a.gl_full ? a.gl_full[idx] : 0.f;
        const float glr = -gy * y + gl;
        a.gx[idx] = gy * sd * ex;
        stv(&gs[pl * a.cs_gst + cb], -gy * ex);
        stv(&gs[pl * a.cs_gst + g.Cb + cb], glr * sc * (1.f - th * th));
        gsc += (double)glr * th;
        gss += glr;
    }
    const float dsc = (float)block_sum(gsc, redl);   // (barriers also publish gs)
    const float dss = (float)block_sum(gss, redl);
    tile_copy_out<T>(gs, t.m0, t.tp, a.cs_gst, a.gst);
    if (threadIdx.x == 0 && (dsc != 0.f || dss != 0.f)) {
        double* sp = a.gscale_part + 2 * (blockIdx.x % RNVP_COUPLING_SHARDS);
        atomicAdd(sp, (double)dsc);
        atomicAdd(sp + 1, (double)dss);
    }
}

// ---------------------------------------------------------------------------
// out part, backward
// ---------------------------------------------------------------------------
__device__ __forceinline__ float gl_at(const rnvp_coupling_args& a, long long e, long long b) {
    return a.gl_full ? a.gl_full[e] : (a.gl_sample ? a.gl_sample[b] : 0.f);
}
// the same operand as one unconditional load (uniform base / index choice;
// with neither gradient present a valid dummy address, weighted 0): a
// prefetch without branches, so no wait is forced at the branch join
struct GlOp {
    const float* base;
    bool full;
    float w;
};
__device__ __forceinline__ GlOp gl_op(const rnvp_coupling_args& a) {
    GlOp o;
    o.full = a.gl_full != nullptr;
    o.base = a.gl_full ? a.gl_full : (a.gl_sample ? a.gl_sample : a.gz);
    o.w = (a.gl_full || a.gl_sample) ? 1.f : 0.f;
    return o;
}
__device__ __forceinline__ float gl_ld(const GlOp& o, long long e, long long b) { return o.w * o.base[o.full ? e : b]; }

// out_bn statistics of the forward (train) or running (eval) for channel cb
__device__ __forceinline__ void out_bn_stats(const rnvp_coupling_args& a, const Geo& g, int cb, float& fm, float& rstd) {
    const double cnt = (double)g.B * g.HW;
    double mean, var;
    if (a.training) {
        mean = csum(a.out_sums, 2 * g.Cb, cb) / cnt;
        var = csum(a.out_sums, 2 * g.Cb, g.Cb + cb) / cnt - mean * mean;
        if (var < 0) var = 0;
    } else {
        mean = a.out_rmean[cb];
        var = a.out_rvar[cb];
    }
    fm = (float)mean;
    rstd = (float)(1.0 / sqrt(var + (double)a.eps));
}

// per-channel A = sum t*gz, Bs = sum t*gz*xhat, G = sum t*gl over all (b, pos)
__global__ __launch_bounds__(256) void k_out_bwd_red(rnvp_coupling_args a, int TP, int seg) {
    extern __shared__ double dsm[];
    const Geo g = geo(a);
    const Tile t = tile_of(g, TP);
    const int lane = threadIdx.x & 63;
    double* red = dsm;                           // [3*Cb]
    float* tab = (float*)(dsm + 3 * g.Cb);       // mean | rstd [Cb each]
    const int total = g.Cb * t.tp;
    auto eidx = [&](int e) {
        const int cb = e / t.tp, p = t.p0 + (e - cb * t.tp);
        const int c = g.kind == 0 ? cb : g.on_base + cb;
        return ((long long)t.b * g.C + c) * g.HW + p;
    };
    float gzp[CP_K], up[CP_K], glp[CP_K];
    const GlOp glo = gl_op(a);
#pragma unroll
    for (int k = 0; k < CP_K; ++k) {
        const int e = k * 256 + threadIdx.x;
        const long long idx = eidx(e < total ? e : 0);   // unconditional (clamped) loads
        const float gz = a.gz[idx], uv = a.u[idx], gl = gl_ld(glo, idx, t.b);
        gzp[k] = e < total ? gz : 0.f;
        up[k] = e < total ? uv : 0.f;
        glp[k] = e < total ? gl : 0.f;
    }
    lds_zero(red, 3 * g.Cb);
    for (int cb = threadIdx.x; cb < g.Cb; cb += blockDim.x) out_bn_stats(a, g, cb, tab[cb], tab[g.Cb + cb]);
    __syncthreads();
    auto body = [&](int e0, float gz, float uv, float glv) {
        const int e = e0 + threadIdx.x;
        const bool ok = e < total;
        const int cb = ok ? e / t.tp : 0, p = t.p0 + (ok ? e - cb * t.tp : 0);
        const bool tr = ok && (g.kind == 0 ? !ckbd_m(g, p) : true);
        float vA = 0.f, vB = 0.f, vG = 0.f;
        if (tr) {
            vA = gz;
            vB = gz * (uv - tab[cb]) * tab[g.Cb + cb];
            vG = glv;
        }
        const double dA = seg_red((double)vA, seg), dB = seg_red((double)vB, seg), dG = seg_red((double)vG, seg);
        if (ok && (lane & seg_mask(seg)) == 0) {
            atomicAdd(&red[cb], dA);
            atomicAdd(&red[g.Cb + cb], dB);
            atomicAdd(&red[2 * g.Cb + cb], dG);
        }
    };
#pragma unroll
    for (int k = 0; k < CP_K; ++k)
        if (k * 256 < total) body(k * 256, gzp[k], up[k], glp[k]);
    for (int e0 = CP_K * 256; e0 < total; e0 += 256) {
        const int e = e0 + threadIdx.x;
        const long long idx = eidx(e < total ? e : 0);
        const float gz = a.gz[idx], uv = a.u[idx], gl = gl_ld(glo, idx, t.b);
        body(e0, e < total ? gz : 0.f, e < total ? uv : 0.f, e < total ? gl : 0.f);
    }
    __syncthreads();
    double* dst = cshard(a.bwd_sums, 3 * g.Cb);
    for (int c = threadIdx.x; c < 3 * g.Cb; c += blockDim.x) atomicAdd(&dst[c], red[c]);
}

// gx (direct part), gst = [g_shift | g_r] (built in LDS, stored as one
// region incl. zero padding), g_scale, g_scale_shift (one atomic per block).
template <typename T>
__global__ __launch_bounds__(256) void k_out_bwd_apply(rnvp_coupling_args a, int TP, int seg) {
    extern __shared__ double dsm[];
    __shared__ double redl[16];
    const Geo g = geo(a);
    const Tile t = tile_of(g, TP);
    float* tab = (float*)dsm;                         // fm | rstd | kA | kB [Cb each]
    const int tabn = 4 * ((g.Cb + 3) / 4 * 4);
    T* st = (T*)(tab + tabn);                         // [tp][cs_st]
    T* gs = st + t.tp * a.cs_st;                      // [tp][cs_gst]
    const double cnt = (double)g.B * g.HW;
    const int total = g.C * t.tp;
    auto eidx = [&](int e) {
        const int c = e / t.tp, pl = e - c * t.tp;
        return ((long long)t.b * g.C + c) * g.HW + t.p0 + pl;
    };
    float gzp[CP_K], up[CP_K], xp[CP_K], glp[CP_K];
    const GlOp glo = gl_op(a);
#pragma unroll
    for (int k = 0; k < CP_K; ++k) {
        const int e = k * 256 + threadIdx.x;
        const long long idx = eidx(e < total ? e : 0);   // unconditional (clamped) loads
        gzp[k] = a.gz[idx];
        up[k] = a.u[idx];
        xp[k] = a.x[idx];
        glp[k] = gl_ld(glo, idx, t.b);
    }
    for (int cb = threadIdx.x; cb < g.Cb; cb += blockDim.x) {
        float fm = 0.f, rstd = 1.f, kA = 0.f, kB = 0.f;
        if (a.coupling_bn) {
            out_bn_stats(a, g, cb, fm, rstd);
            if (a.training) {
                kA = (float)(csum(a.bwd_sums, 3 * g.Cb, cb) / cnt);
                kB = (float)((csum(a.bwd_sums, 3 * g.Cb, g.Cb + cb) + csum(a.bwd_sums, 3 * g.Cb, 2 * g.Cb + cb)) / cnt);
            }
        }
        tab[cb] = fm; tab[g.Cb + cb] = rstd; tab[2 * g.Cb + cb] = kA; tab[3 * g.Cb + cb] = kB;
    }
    tile_copy_in<T>(a.st, t.m0, t.tp, a.cs_st, st);
    for (int e = threadIdx.x; e < t.tp * a.cs_gst; e += blockDim.x) stv(&gs[e], 0.f);
    __syncthreads();
    const float sc = a.scale[0], ss = a.scale_shift[0];
    double gsc = 0.0, gss = 0.0;
    auto body = [&](int e, float gz, float uv, float xv, float glv) {
        const int c = e / t.tp, pl = e - c * t.tp, p = t.p0 + pl;
        const long long idx = ((long long)t.b * g.C + c) * g.HW + p;
        const bool chan_on = g.kind == 1 && c >= g.on_base && c < g.on_base + g.Cb;
        const int cb = g.kind == 0 ? c : c - g.on_base;
        const bool has_bn_chan = g.kind == 0 || chan_on;
        const bool tr = g.kind == 0 ? !ckbd_m(g, p) : chan_on;
        float gu;
        if (!a.coupling_bn || !has_bn_chan) {
            gu = gz;
        } else {
            const float fm = tab[cb], rstd = tab[g.Cb + cb], kA = tab[2 * g.Cb + cb], kB = tab[3 * g.Cb + cb];
            if (!tr) {   // ckbd kept position: z = u, but u still moves the batch stats
                gu = gz;
                if (a.training) gu += rstd * (-kA - (uv - fm) * rstd * kB);
            } else {
                gu = rstd * gz;
                if (a.training) gu = rstd * (gz - kA - (uv - fm) * rstd * kB);
            }
        }
        if (tr) {
            const float r = ldv(&st[pl * a.cs_st + g.Cb + cb]);
            const float th = tanhf(r);
            const float ex = expf(sc * th + ss);
            a.gx[idx] = gu * ex;
            const float glr = gu * xv * ex + glv;
            stv(&gs[pl * a.cs_gst + cb], gu);
            stv(&gs[pl * a.cs_gst + g.Cb + cb], glr * sc * (1.f - th * th));
            gsc += (double)glr * th;
            gss += glr;
        } else {
            a.gx[idx] = gu;
        }
    };
#pragma unroll
    for (int k = 0; k < CP_K; ++k) {
        const int e = k * 256 + threadIdx.x;
        if (e < total) body(e, gzp[k], up[k], xp[k], glp[k]);
    }
    for (int e = CP_K * 256 + threadIdx.x; e < total; e += 256) {
        const long long idx = eidx(e);
        body(e, a.gz[idx], a.u[idx], a.x[idx], gl_ld(glo, idx, t.b));
    }
    const float dsc = (float)block_sum(gsc, redl);   // (barriers also publish gs)
    const float dss = (float)block_sum(gss, redl);
    tile_copy_out<T>(gs, t.m0, t.tp, a.cs_gst, a.gst);
    if (threadIdx.x == 0 && (dsc != 0.f || dss != 0.f)) {
        if (a.gscale_part) {   // sharded: bounded same-address atomic depth
            double* sp = a.gscale_part + 2 * (blockIdx.x % RNVP_COUPLING_SHARDS);
            atomicAdd(sp, (double)dsc);
            atomicAdd(sp + 1, (double)dss);
        } else {
            atomicAdd(a.g_scale, dsc);
            atomicAdd(a.g_scale_shift, dss);
        }
    }
}

// ---------------------------------------------------------------------------
// in part, backward (through CReLU and in_bn)
// ---------------------------------------------------------------------------
// fold the out part's sharded scale / scale_shift partials into g_scale /
// g_scale_shift (+=) and leave them zero (wave 0 of block 0; every partial
// was written by an earlier launch)
__device__ __forceinline__ void fold_gscale(const rnvp_coupling_args& a) {
    const int l = threadIdx.x;
    double v0 = 0.0, v1 = 0.0;
    if (l < RNVP_COUPLING_SHARDS) {
        v0 = a.gscale_part[2 * l];
        v1 = a.gscale_part[2 * l + 1];
        a.gscale_part[2 * l] = 0.0;
        a.gscale_part[2 * l + 1] = 0.0;
    }
    v0 = wave_sum(v0);
    v1 = wave_sum(v1);
    if (l == 0) {
        *a.g_scale += (float)v0;
        *a.g_scale_shift += (float)v1;
    }
}

// gxa = d/dxa of [relu(xa), relu(-xa)] . [g1, g2]; gh: LDS tile [tp][cs_gh0]
template <typename T>
__device__ __forceinline__ void in_bwd_vals(const rnvp_coupling_args& a, const Geo& g, const Tile& t, const T* gh,
                                            const float* tab, int cb, int pl, float v, float& gxa, float& xh) {
    const int p = t.p0 + pl;
    if (g.kind == 0 && !ckbd_m(g, p)) v = 0.f;
    const float xa = v * tab[cb] + tab[g.Cb + cb];
    const float g1 = ldv(&gh[pl * a.cs_gh0 + cb]);
    const float g2 = ldv(&gh[pl * a.cs_gh0 + g.Cb + cb]);
    gxa = (xa > 0.f ? g1 : 0.f) - (xa < 0.f ? g2 : 0.f);
    xh = (v - tab[2 * g.Cb + cb]) * tab[3 * g.Cb + cb];
}

template <typename T>
__global__ __launch_bounds__(256) void k_in_bwd_red(rnvp_coupling_args a, int TP, int seg) {
    extern __shared__ double dsm[];
    const Geo g = geo(a);
    const Tile t = tile_of(g, TP);
    const int lane = threadIdx.x & 63;
    const bool ext = a.in_bwd_ext != nullptr;
    double* red = dsm;                                   // [2*Cb] (+ [2*Cb] ext)
    float* tab = (float*)(dsm + (ext ? 4 : 2) * g.Cb);   // [4*Cb]
    T* gh = (T*)(tab + 4 * ((g.Cb + 3) / 4 * 4));        // [tp][cs_gh0]
    const int total = g.Cb * t.tp;
    auto xidx = [&](int e) {
        const int cb = e / t.tp, p = t.p0 + (e - cb * t.tp);
        const int c = (g.kind == 0) ? cb : g.off_base + cb;
        return ((long long)t.b * g.C + c) * g.HW + p;
    };
    float xp[CP_K];
#pragma unroll
    for (int k = 0; k < CP_K; ++k) {
        const int e = k * 256 + threadIdx.x;
        { const float v = a.x[xidx(e < total ? e : 0)]; xp[k] = e < total ? v : 0.f; }   // unconditional (clamped) load: no branch, no wait
    }
    tile_copy_in<T>(a.gh0, t.m0, t.tp, a.cs_gh0, gh);   // in flight under the table's loads
    lds_zero(red, (ext ? 4 : 2) * g.Cb);
    if (a.training && a.in_tab) {   // the forward's table (coupling links): 4*Cb loads instead of the shard sums
        for (int i = threadIdx.x; i < 4 * g.Cb; i += blockDim.x) tab[i] = a.in_tab[i];
    } else {
        in_bn_table(a, g, tab);
    }
    if (blockIdx.x == 0 && a.gscale_part && threadIdx.x < 64) fold_gscale(a);
    __syncthreads();
    auto body = [&](int e0, float xv) {
        const int e = e0 + threadIdx.x;
        const bool ok = e < total;
        const int cb = ok ? e / t.tp : 0, pl = ok ? e - cb * t.tp : 0;
        float gxa = 0.f, xh = 0.f;
        if (ok) in_bwd_vals<T>(a, g, t, gh, tab, cb, pl, xv, gxa, xh);
        const double s1 = seg_red((double)gxa, seg), s2 = seg_red((double)gxa * xh, seg);
        if (ok && (lane & seg_mask(seg)) == 0) {
            atomicAdd(&red[cb], s1);
            atomicAdd(&red[g.Cb + cb], s2);
        }
        if (ext) {   // over the positions in_bn normalises (coupling links' closed forms)
            const bool kept = ok && (g.kind != 0 || ckbd_m(g, t.p0 + pl));
            const double e1 = seg_red(kept ? (double)gxa : 0.0, seg), e2 = seg_red(kept ? (double)gxa * xv : 0.0, seg);
            if (ok && (lane & seg_mask(seg)) == 0) {
                atomicAdd(&red[2 * g.Cb + cb], e1);
                atomicAdd(&red[3 * g.Cb + cb], e2);
            }
        }
    };
#pragma unroll
    for (int k = 0; k < CP_K; ++k)
        if (k * 256 < total) body(k * 256, xp[k]);
    for (int e0 = CP_K * 256; e0 < total; e0 += 256) {
        const int e = e0 + threadIdx.x;
        { const float v = a.x[xidx(e < total ? e : 0)]; body(e0, e < total ? v : 0.f); }
    }
    __syncthreads();
    double* dst = cshard(a.in_bwd_sums, 2 * g.Cb);
    for (int c = threadIdx.x; c < 2 * g.Cb; c += blockDim.x) atomicAdd(&dst[c], red[c]);
    if (ext) {
        double* dx = cshard(a.in_bwd_ext, 2 * g.Cb);
        for (int c = threadIdx.x; c < 2 * g.Cb; c += blockDim.x) atomicAdd(&dx[c], red[2 * g.Cb + c]);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_in_bwd_apply(rnvp_coupling_args a, int TP, int seg) {
    extern __shared__ double dsm[];
    const Geo g = geo(a);
    const Tile t = tile_of(g, TP);
    float* tab = (float*)dsm;                            // sc | sf | mean | rstd | coef | k1 | k2 [Cb each]
    const int tabn = 8 * ((g.Cb + 3) / 4 * 4);
    T* gh = (T*)(tab + tabn);
    const int total = g.Cb * t.tp;
    auto xidx = [&](int e) {
        const int cb = e / t.tp, p = t.p0 + (e - cb * t.tp);
        const int c = (g.kind == 0) ? cb : g.off_base + cb;
        return ((long long)t.b * g.C + c) * g.HW + p;
    };
    float xp[CP_K], gxp[CP_K];
#pragma unroll
    for (int k = 0; k < CP_K; ++k) {
        const int e = k * 256 + threadIdx.x;
        const long long idx = xidx(e < total ? e : 0);   // unconditional (clamped) loads
        xp[k] = a.x[idx];
        gxp[k] = a.gx[idx];
    }
    in_bn_table(a, g, tab);
    const double cnt = (double)g.B * g.HW;
    for (int cb = threadIdx.x; cb < g.Cb; cb += blockDim.x) {
        const float gam = a.in_gamma ? a.in_gamma[cb] : 1.f;
        tab[4 * g.Cb + cb] = gam * tab[3 * g.Cb + cb];
        const double s1 = a.in_bwd_sums ? csum(a.in_bwd_sums, 2 * g.Cb, cb) : 0.0;
        const double s2 = a.in_bwd_sums ? csum(a.in_bwd_sums, 2 * g.Cb, g.Cb + cb) : 0.0;
        tab[5 * g.Cb + cb] = a.training ? (float)(s1 / cnt) : 0.f;
        tab[6 * g.Cb + cb] = a.training ? (float)(s2 / cnt) : 0.f;
        if (blockIdx.x == 0) {   // the affine grads, once
            if (a.g_in_beta) a.g_in_beta[cb] = (float)s1;
            if (a.g_in_gamma) a.g_in_gamma[cb] = (float)s2;
        }
    }
    if (blockIdx.x == 0 && a.gscale_part && threadIdx.x < 64) fold_gscale(a);   // (no-op after k_in_bwd_red)
    tile_copy_in<T>(a.gh0, t.m0, t.tp, a.cs_gh0, gh);
    __syncthreads();
    auto body = [&](int e, float xv, float gxv) {
        const int cb = e / t.tp, pl = e - cb * t.tp, p = t.p0 + pl;
        const int c = (g.kind == 0) ? cb : g.off_base + cb;
        const long long idx = ((long long)t.b * g.C + c) * g.HW + p;
        float gxa, xh;
        in_bwd_vals<T>(a, g, t, gh, tab, cb, pl, xv, gxa, xh);
        float gxm = tab[4 * g.Cb + cb] * (gxa - tab[5 * g.Cb + cb] - xh * tab[6 * g.Cb + cb]);
        if (g.kind == 0 && !ckbd_m(g, p)) gxm = 0.f;   // xm = x * mask
        a.gx[idx] = gxv + gxm;
    };
#pragma unroll
    for (int k = 0; k < CP_K; ++k) {
        const int e = k * 256 + threadIdx.x;
        if (e < total) body(e, xp[k], gxp[k]);
    }
    for (int e = CP_K * 256 + threadIdx.x; e < total; e += 256) {
        const long long idx = xidx(e);
        body(e, a.x[idx], a.gx[idx]);
    }
}

int check(const rnvp_coupling_args* a) {
    if (!a || !a->x || a->B < 0 || a->C <= 0 || a->H <= 0 || a->W <= 0) return RNVP_E_INVALID;
    if (a->kind != 0 && a->kind != 1) return RNVP_E_INVALID;
    if (a->kind == 1 && (a->C & 1)) return RNVP_E_INVALID;
    if (a->dtype != RNVP_F32 && a->dtype != RNVP_BF16) return RNVP_E_INVALID;
    return RNVP_OK;
}

inline int cb_of(const rnvp_coupling_args* a) { return a->kind == 0 ? a->C : a->C / 2; }

// pixel-tile geometry: TP pixels per workgroup (<= 256, LDS-bounded by the
// widest NHWC tile), seg = lanes sharing a channel in the reductions
struct TileCfg {
    int TP, seg, grid;
};
inline TileCfg tile_cfg(const rnvp_coupling_args* a) {
    const int HW = a->H * a->W;
    const int esz = a->dtype == RNVP_F32 ? 4 : 2;
    int cs = a->cs_h0;
    if (a->cs_st + a->cs_gst > cs) cs = a->cs_st + a->cs_gst;
    if (a->cs_gh0 > cs) cs = a->cs_gh0;
    if (cs < 8) cs = 8;
    TileCfg c;
    // largest power-of-2-ish tile (<= 256 px) that still gives >= 512
    // workgroups (each thread then touches <= ~3 elements per pass)
    c.TP = HW < 256 ? HW : 256;
    while (c.TP > 16 && (long long)c.TP * cs * esz > 32 * 1024) c.TP /= 2;
    while (c.TP > 4 && c.TP % 2 == 0 && (long long)a->B * ((HW + c.TP - 1) / c.TP) < 512) c.TP /= 2;
    int seg = 1;
    while (seg < 64 && c.TP % (2 * seg) == 0 && HW % (2 * seg) == 0) seg *= 2;
    c.seg = seg;
    c.grid = a->B * ((HW + c.TP - 1) / c.TP);
    return c;
}
}  // namespace

extern "C" int rnvp_coupling_in_fwd(const rnvp_coupling_args* a, void* stream) {
    int st = check(a);
    if (st) return st;
    if (!a->h0 || (a->training && !a->in_sums) || (!a->training && (!a->in_rmean || !a->in_rvar))) return RNVP_E_INVALID;
    const int Cb = cb_of(a);
    if (a->cs_h0 < (a->kind == 0 ? 2 * Cb + 1 : 2 * Cb)) return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    hipStream_t s = (hipStream_t)stream;
    const TileCfg tc = tile_cfg(a);
    const int esz = a->dtype == RNVP_F32 ? 4 : 2;
    if (a->training) {
        k_in_stats<<<tc.grid, 256, 16 * Cb, s>>>(*a, tc.TP, tc.seg);
        RNVP_LAUNCH_CHECK();
    }
    const size_t shm = 16 * r4(Cb) + (size_t)tc.TP * a->cs_h0 * esz;
    if (a->dtype == RNVP_F32) k_in_apply<float><<<tc.grid, 256, shm, s>>>(*a, tc.TP, tc.seg);
    else k_in_apply<bf16_t><<<tc.grid, 256, shm, s>>>(*a, tc.TP, tc.seg);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_coupling_in_apply(const rnvp_coupling_args* a, void* stream) {
    int st = check(a);
    if (st) return st;
    if (!a->h0 || (a->training && !a->in_sums) || (!a->training && (!a->in_rmean || !a->in_rvar))) return RNVP_E_INVALID;
    const int Cb = cb_of(a);
    if (a->cs_h0 < (a->kind == 0 ? 2 * Cb + 1 : 2 * Cb)) return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    const TileCfg tc = tile_cfg(a);
    const int esz = a->dtype == RNVP_F32 ? 4 : 2;
    const size_t shm = 16 * r4(Cb) + (size_t)tc.TP * a->cs_h0 * esz;
    hipStream_t s = (hipStream_t)stream;
    if (a->dtype == RNVP_F32) k_in_apply<float><<<tc.grid, 256, shm, s>>>(*a, tc.TP, tc.seg);
    else k_in_apply<bf16_t><<<tc.grid, 256, shm, s>>>(*a, tc.TP, tc.seg);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_coupling_out_fwd(const rnvp_coupling_args* a, void* stream) {
    int st = check(a);
    if (st) return st;
    if (!a->st || !a->u || !a->z || !a->ldj_sample || !a->scale || !a->scale_shift) return RNVP_E_INVALID;
    if (a->coupling_bn && ((a->training && !a->out_sums) || (!a->training && (!a->out_rmean || !a->out_rvar))))
        return RNVP_E_INVALID;
    const int Cb = cb_of(a);
    if (a->cs_st < 2 * Cb) return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    hipStream_t s = (hipStream_t)stream;
    const TileCfg tc = tile_cfg(a);
    const int esz = a->dtype == RNVP_F32 ? 4 : 2;
    const size_t shm1 = 16 * ((Cb + 1) / 2 * 2) + (size_t)tc.TP * a->cs_st * esz;
    if (a->dtype == RNVP_F32) k_out1<float><<<tc.grid, 256, shm1, s>>>(*a, tc.TP, tc.seg);
    else k_out1<bf16_t><<<tc.grid, 256, shm1, s>>>(*a, tc.TP, tc.seg);
    RNVP_LAUNCH_CHECK();
    long long n = (long long)a->B * a->C * a->H * a->W;
    size_t shm = 3 * Cb * sizeof(float);
    const int nrun = (a->training && a->net_running) ? a->n_net_running : 0;
    if (nrun < 0 || (nrun > 0 && a->net_running_cmax <= 0)) return RNVP_E_INVALID;
    if (nrun > 0 && 16 * (size_t)a->net_running_cmax > shm) shm = 16 * (size_t)a->net_running_cmax;
    const int g2 = rnvp_grid(n, 256, 2048);
    if (a->dtype == RNVP_F32) k_out2<float><<<g2 + nrun, 256, shm, s>>>(*a, g2);
    else k_out2<bf16_t><<<g2 + nrun, 256, shm, s>>>(*a, g2);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_coupling_reverse(const rnvp_coupling_args* a, void* stream) {
    int st = check(a);
    if (st) return st;
    if (!a->st || !a->z || !a->scale || !a->scale_shift) return RNVP_E_INVALID;
    if (a->coupling_bn && (!a->out_rmean || !a->out_rvar)) return RNVP_E_INVALID;
    if (a->cs_st < 2 * cb_of(a)) return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    long long n = (long long)a->B * a->C * a->H * a->W;
    hipStream_t s = (hipStream_t)stream;
    if (a->dtype == RNVP_F32) k_reverse<float><<<rnvp_grid(n, 256, 2048), 256, 0, s>>>(*a);
    else k_reverse<bf16_t><<<rnvp_grid(n, 256, 2048), 256, 0, s>>>(*a);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_coupling_reverse_bwd(const rnvp_coupling_args* a, void* stream) {
    int st = check(a);
    if (st) return st;
    if (!a->st || !a->gz || !a->gx || !a->gst || !a->gscale_part || !a->scale || !a->scale_shift) return RNVP_E_INVALID;
    const int Cb = cb_of(a);
    if (a->cs_gst < 2 * Cb || a->cs_st < 2 * Cb) return RNVP_E_INVALID;
    if (a->coupling_bn && (!a->out_rmean || !a->out_rvar)) return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    const TileCfg tc = tile_cfg(a);
    const int esz = a->dtype == RNVP_F32 ? 4 : 2;
    const size_t shm = (size_t)tc.TP * (a->cs_st + a->cs_gst) * esz;
    hipStream_t s = (hipStream_t)stream;
    if (a->dtype == RNVP_F32) k_reverse_bwd<float><<<tc.grid, 256, shm, s>>>(*a, tc.TP);
    else k_reverse_bwd<bf16_t><<<tc.grid, 256, shm, s>>>(*a, tc.TP);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_coupling_out_bwd(const rnvp_coupling_args* a, void* stream) {
    int st = check(a);
    if (st) return st;
    if (!a->st || !a->u || !a->gz || !a->gx || !a->gst || !a->g_scale || !a->g_scale_shift) return RNVP_E_INVALID;
    const int Cb = cb_of(a);
    if (a->cs_gst < 2 * Cb || a->cs_st < 2 * Cb) return RNVP_E_INVALID;
    const bool stats = a->coupling_bn && a->training;
    if (stats && (!a->out_sums || !a->bwd_sums)) return RNVP_E_INVALID;
    if (a->coupling_bn && !a->training && (!a->out_rmean || !a->out_rvar)) return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    hipStream_t s = (hipStream_t)stream;
    const TileCfg tc = tile_cfg(a);
    const int esz = a->dtype == RNVP_F32 ? 4 : 2;
    if (stats) {
        k_out_bwd_red<<<tc.grid, 256, 24 * Cb + 8 * Cb, s>>>(*a, tc.TP, tc.seg);
        RNVP_LAUNCH_CHECK();
    }
    const size_t shm = 16 * r4(Cb) + (size_t)tc.TP * (a->cs_st + a->cs_gst) * esz;
    if (a->dtype == RNVP_F32) k_out_bwd_apply<float><<<tc.grid, 256, shm, s>>>(*a, tc.TP, tc.seg);
    else k_out_bwd_apply<bf16_t><<<tc.grid, 256, shm, s>>>(*a, tc.TP, tc.seg);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_coupling_in_bwd(const rnvp_coupling_args* a, void* stream) {
    int st = check(a);
    if (st) return st;
    // gx NULL: the reduction pass only (coupling links: the in_bn backward apply
    // is folded into the previous coupling's rnvp_coupling_link_bwd)
    if (!a->gh0 || (!a->gx && !(a->in_bwd_ext && a->training))) return RNVP_E_INVALID;
    if (a->training && (!a->in_sums || !a->in_bwd_sums)) return RNVP_E_INVALID;
    if (!a->training && (!a->in_rmean || !a->in_rvar)) return RNVP_E_INVALID;
    const int Cb = cb_of(a);
    if (a->cs_gh0 < 2 * Cb) return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    hipStream_t s = (hipStream_t)stream;
    const TileCfg tc = tile_cfg(a);
    const int esz = a->dtype == RNVP_F32 ? 4 : 2;
    const size_t gsh = (size_t)tc.TP * a->cs_gh0 * esz;
    if (a->training || a->g_in_gamma || a->g_in_beta) {
        if (!a->in_bwd_sums) return RNVP_E_INVALID;
        const size_t shm = (a->in_bwd_ext ? 32 : 16) * Cb + 16 * r4(Cb) + gsh;
        if (a->dtype == RNVP_F32) k_in_bwd_red<float><<<tc.grid, 256, shm, s>>>(*a, tc.TP, tc.seg);
        else k_in_bwd_red<bf16_t><<<tc.grid, 256, shm, s>>>(*a, tc.TP, tc.seg);
        RNVP_LAUNCH_CHECK();
    }
    if (!a->gx) return RNVP_OK;
    const size_t shm = 32 * r4(Cb) + gsh;
    if (a->dtype == RNVP_F32) k_in_bwd_apply<float><<<tc.grid, 256, shm, s>>>(*a, tc.TP, tc.seg);
    else k_in_bwd_apply<bf16_t><<<tc.grid, 256, shm, s>>>(*a, tc.TP, tc.seg);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}
