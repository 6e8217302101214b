// Affine coupling layers (modules_realnvp.py:239-370) around the s/t ResNet.
//
// "in"  part: mask apply + in_bn (batch stats) + CReLU/mask concat  -> net input h0 (NHWC)
// "out" part: scale*tanh+shift, masked affine, out_bn with the batch-variance
//             log|det J| term, per-sample log-det accumulation       -> z, ldj[b]
// plus the exact inverse (reverse=True, running out_bn stats) and the
// backward of both parts, including the cross-sample batch-variance gradient.
//
// Flow tensors are NCHW fp32; one block per (b, c) plane for the reductions
// (coalesced over H*W), grid-stride elementwise passes otherwise.
#include <math.h>

#include "common.h"

namespace {

struct Geo {
    int kind, B, C, H, W, HW, Cb, cfg, on_base, off_base;
};

__device__ __forceinline__ Geo geo(const rnvp_coupling_args& a) {
    Geo g;
    g.kind = a.kind; g.B = a.B; g.C = a.C; g.H = a.H; g.W = a.W; g.HW = a.H * a.W;
    g.cfg = a.mask_config ? 1 : 0;
    if (a.kind == 0) {
        g.Cb = a.C; g.on_base = 0; g.off_base = 0;
    } else {
        g.Cb = a.C / 2;
        // mask_config truthy: (on, off) = (top, bottom) halves (modules_realnvp.py:333-336)
        g.on_base = g.cfg ? 0 : g.Cb;
        g.off_base = g.cfg ? g.Cb : 0;
    }
    return g;
}

// checkerboard mask at pixel p (= h*W + w): 1 = kept ("masked in") position
__device__ __forceinline__ int ckbd_m(const Geo& g, int p) { return (g.cfg + p / g.W + p % g.W) & 1; }

// number of transformed (mask == 0) positions per (sample, channel)
__device__ __forceinline__ double n_transformed(const Geo& g) {
    if (g.kind == 1) return (double)g.HW;
    const long long total = (long long)g.H * g.W;
    // positions with (i + j) even
    const long long even = ((g.H & 1) && (g.W & 1)) ? (total + 1) / 2 : total / 2;
    // mask == 0  <=>  (cfg + i + j) even
    return (double)(g.cfg ? total - even : even);
}

template <typename T>
__device__ __forceinline__ const T* cptr(const void* p) { return (const T*)p; }

// ---------------------------------------------------------------------------
// in part, forward
// ---------------------------------------------------------------------------
// one block per (b, cb) plane of the in_bn input: sums of xm and xm^2
__global__ void k_in_stats(rnvp_coupling_args a) {
    __shared__ double red[16];
    const Geo g = geo(a);
    const int b = blockIdx.x / g.Cb, cb = blockIdx.x % g.Cb;
    const int c = (g.kind == 0) ? cb : g.off_base + cb;
    const float* xp = a.x + ((long long)b * g.C + c) * g.HW;
    float s = 0.f, s2 = 0.f;
    for (int p = threadIdx.x; p < g.HW; p += blockDim.x) {
        float v = xp[p];
        if (g.kind == 0 && !ckbd_m(g, p)) v = 0.f;
        s += v;
        s2 += v * v;
    }
    double ds = block_sum((double)s, red);
    double ds2 = block_sum((double)s2, red);
    if (threadIdx.x == 0) {
        atomicAdd(&a.in_sums[cb], ds);
        atomicAdd(&a.in_sums[g.Cb + cb], ds2);
    }
}

// h0[m][ch] NHWC: relu(xa), relu(-xa) [, mask], zero pad.  One thread per (m, ch).
template <typename T>
__global__ void k_in_apply(rnvp_coupling_args a) {
    extern __shared__ float sh[];   // 2*Cb floats: scale, shift
    const Geo g = geo(a);
    const double cnt = (double)g.B * g.HW;
    for (int c = threadIdx.x; c < g.Cb; c += blockDim.x) {
        rnvp_bn_src s;
        s.shards = 1;
        s.sums = a.training ? a.in_sums : nullptr;
        s.count = cnt;
        s.mean = a.in_rmean; s.var = a.in_rvar;
        s.gamma = a.in_gamma; s.beta = a.in_beta; s.eps = a.eps;
        float sc, sf;
        bn_affine(s, g.Cb, c, sc, sf);
        sh[c] = sc;
        sh[g.Cb + c] = sf;
        if (blockIdx.x == 0 && a.training && a.in_rmean) {
            double mean = a.in_sums[c] / cnt;
            double var = a.in_sums[g.Cb + c] / cnt - mean * mean;
            if (var < 0) var = 0;
            double unb = cnt > 1 ? var * cnt / (cnt - 1) : var;
            a.in_rmean[c] = (1.f - a.momentum) * a.in_rmean[c] + a.momentum * (float)mean;
            a.in_rvar[c] = (1.f - a.momentum) * a.in_rvar[c] + a.momentum * (float)unb;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.training && a.in_nbt) a.in_nbt[0] += 1;
    __syncthreads();
    T* h0 = (T*)a.h0;
    const int cs = a.cs_h0;
    const long long n = (long long)g.B * g.HW * cs;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
        const int ch = (int)(e % cs);
        const long long m = e / cs;
        const int p = (int)(m % g.HW);
        const long long b = m / g.HW;
        float out = 0.f;
        if (ch < 2 * g.Cb) {
            const int cb = ch < g.Cb ? ch : ch - g.Cb;
            const int c = (g.kind == 0) ? cb : g.off_base + cb;
            float v = a.x[(b * g.C + c) * g.HW + p];
            if (g.kind == 0 && !ckbd_m(g, p)) v = 0.f;
            float xa = v * sh[cb] + sh[g.Cb + cb];
            out = ch < g.Cb ? fmaxf(xa, 0.f) : fmaxf(-xa, 0.f);
        } else if (g.kind == 0 && ch == 2 * g.Cb) {
            out = (float)ckbd_m(g, p);   // relu(mask) = mask
        }
        stv(&h0[e], out);
    }
}

// ---------------------------------------------------------------------------
// out part, forward
// ---------------------------------------------------------------------------
// u = x*exp(lr)+shift on transformed positions (x elsewhere); stats of u over
// the out_bn channels; ldj_sample[b] += sum lr.  One block per (b, c) plane.
template <typename T>
__global__ void k_out1(rnvp_coupling_args a) {
    __shared__ double red[16];
    const Geo g = geo(a);
    const int b = blockIdx.x / g.C, c = blockIdx.x % g.C;
    const long long plane = ((long long)b * g.C + c) * g.HW;
    const T* st = cptr<T>(a.st);
    const bool chan_on = g.kind == 1 && c >= g.on_base && c < g.on_base + g.Cb;
    const int cb = g.kind == 0 ? c : c - g.on_base;
    const float sc = a.scale[0], ss = a.scale_shift[0];
    float s = 0.f, s2 = 0.f, sl = 0.f;
    for (int p = threadIdx.x; p < g.HW; p += blockDim.x) {
        float xv = a.x[plane + p];
        float u = xv;
        bool tr = g.kind == 0 ? !ckbd_m(g, p) : chan_on;
        if (tr) {
            const long long m = (long long)b * g.HW + p;
            float sh = ldv(&st[m * a.cs_st + cb]);
            float r = ldv(&st[m * a.cs_st + g.Cb + cb]);
            float lr = sc * tanhf(r) + ss;
            u = xv * expf(lr) + sh;
            sl += lr;
        }
        a.u[plane + p] = u;
        s += u;
        s2 += u * u;
    }
    double ds = block_sum((double)s, red);
    double ds2 = block_sum((double)s2, red);
    double dl = block_sum((double)sl, red);
    if (threadIdx.x == 0) {
        if ((g.kind == 0 || chan_on) && a.out_sums) {
            atomicAdd(&a.out_sums[cb], ds);
            atomicAdd(&a.out_sums[g.Cb + cb], ds2);
        }
        if (dl != 0.0) atomicAdd(&a.ldj_sample[b], (float)dl);
    }
}

// z = out_bn(u) on transformed positions; ldj var term; running stats.
template <typename T>
__global__ void k_out2(rnvp_coupling_args a) {
    extern __shared__ float sh[];   // mean[Cb], rstd[Cb], half_log_var[Cb]
    const Geo g = geo(a);
    const double cnt = (double)g.B * g.HW;
    for (int cb = threadIdx.x; cb < g.Cb; cb += blockDim.x) {
        double mean = 0, var = 1;
        if (a.coupling_bn) {
            if (a.training) {
                mean = a.out_sums[cb] / cnt;
                var = a.out_sums[g.Cb + cb] / cnt - mean * mean;
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
        float u = a.u[e];
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

// ---------------------------------------------------------------------------
// out part, backward
// ---------------------------------------------------------------------------
__device__ __forceinline__ float gl_at(const rnvp_coupling_args& a, long long e, long long b) {
    return a.gl_full ? a.gl_full[e] : (a.gl_sample ? a.gl_sample[b] : 0.f);
}

// per-channel A = sum t*gz, Bs = sum t*gz*xhat, G = sum t*gl over all (b, pos)
__global__ void k_out_bwd_red(rnvp_coupling_args a) {
    __shared__ double red[16];
    const Geo g = geo(a);
    const int b = blockIdx.x / g.Cb, cb = blockIdx.x % g.Cb;
    const int c = g.kind == 0 ? cb : g.on_base + cb;
    const long long plane = ((long long)b * g.C + c) * g.HW;
    const double cnt = (double)g.B * g.HW;
    double mean = a.out_sums[cb] / cnt;
    double var = a.out_sums[g.Cb + cb] / cnt - mean * mean;
    if (var < 0) var = 0;
    const float fm = (float)mean, rstd = (float)(1.0 / sqrt(var + (double)a.eps));
    float sA = 0.f, sB = 0.f, sG = 0.f;
    for (int p = threadIdx.x; p < g.HW; p += blockDim.x) {
        bool tr = g.kind == 0 ? !ckbd_m(g, p) : true;
        if (!tr) continue;
        const long long e = plane + p;
        float gz = a.gz[e];
        float xh = (a.u[e] - fm) * rstd;
        sA += gz;
        sB += gz * xh;
        sG += gl_at(a, e, b);
    }
    double dA = block_sum((double)sA, red);
    double dB = block_sum((double)sB, red);
    double dG = block_sum((double)sG, red);
    if (threadIdx.x == 0) {
        atomicAdd(&a.bwd_sums[cb], dA);
        atomicAdd(&a.bwd_sums[g.Cb + cb], dB);
        atomicAdd(&a.bwd_sums[2 * g.Cb + cb], dG);
    }
}

// gx (direct part), gst = [g_shift | g_r], g_scale, g_scale_shift.  One block
// per (b, c) plane so the scale reductions stay block-local.
template <typename T>
__global__ void k_out_bwd_apply(rnvp_coupling_args a) {
    __shared__ double red[16];
    const Geo g = geo(a);
    const int b = blockIdx.x / g.C, c = blockIdx.x % g.C;
    const long long plane = ((long long)b * g.C + c) * g.HW;
    const bool chan_on = g.kind == 1 && c >= g.on_base && c < g.on_base + g.Cb;
    const int cb = g.kind == 0 ? c : c - g.on_base;
    const bool has_bn_chan = g.kind == 0 || chan_on;
    const double cnt = (double)g.B * g.HW;
    float fm = 0.f, rstd = 1.f, kA = 0.f, kB = 0.f;
    if (a.coupling_bn && has_bn_chan) {
        double mean, var;
        if (a.training) {
            mean = a.out_sums[cb] / cnt;
            var = a.out_sums[g.Cb + cb] / cnt - mean * mean;
            if (var < 0) var = 0;
        } else {
            mean = a.out_rmean[cb];
            var = a.out_rvar[cb];
        }
        fm = (float)mean;
        rstd = (float)(1.0 / sqrt(var + (double)a.eps));
        if (a.training) {
            kA = (float)(a.bwd_sums[cb] / cnt);
            kB = (float)((a.bwd_sums[g.Cb + cb] + a.bwd_sums[2 * g.Cb + cb]) / cnt);
        }
    }
    const T* st = cptr<T>(a.st);
    T* gst = (T*)a.gst;
    const float sc = a.scale[0], ss = a.scale_shift[0];
    float gsc = 0.f, gss = 0.f;
    for (int p = threadIdx.x; p < g.HW; p += blockDim.x) {
        const long long e = plane + p;
        const long long m = (long long)b * g.HW + p;
        bool tr = g.kind == 0 ? !ckbd_m(g, p) : chan_on;
        float gz = a.gz[e];
        float gu;
        if (!a.coupling_bn || !has_bn_chan) {
            gu = gz;
        } else if (!tr) {
            // ckbd kept position: z = u, but u still moves the batch stats
            gu = gz;
            if (a.training) gu += rstd * (-kA - (a.u[e] - fm) * rstd * kB);
        } else {
            gu = rstd * gz;
            if (a.training) gu = rstd * (gz - kA - (a.u[e] - fm) * rstd * kB);
        }
        if (tr) {
            float r = ldv(&st[m * a.cs_st + g.Cb + cb]);
            float th = tanhf(r);
            float lr = sc * th + ss;
            float ex = expf(lr);
            float xv = a.x[e];
            a.gx[e] = gu * ex;
            float glr = gu * xv * ex + gl_at(a, e, b);
            stv(&gst[m * a.cs_gst + cb], gu);
            stv(&gst[m * a.cs_gst + g.Cb + cb], glr * sc * (1.f - th * th));
            gsc += glr * th;
            gss += glr;
        } else {
            a.gx[e] = gu;
            if (g.kind == 0) {   // masked position: st gradients are zero
                stv(&gst[m * a.cs_gst + cb], 0.f);
                stv(&gst[m * a.cs_gst + g.Cb + cb], 0.f);
            }
        }
        if (c == 0) {   // zero the padded channels of gst once per pixel
            for (int ch = 2 * g.Cb; ch < a.cs_gst; ++ch) stv(&gst[m * a.cs_gst + ch], 0.f);
        }
    }
    double dsc = block_sum((double)gsc, red);
    double dss = block_sum((double)gss, red);
    if (threadIdx.x == 0 && (dsc != 0.0 || dss != 0.0)) {
        atomicAdd(a.g_scale, (float)dsc);
        atomicAdd(a.g_scale_shift, (float)dss);
    }
}

// ---------------------------------------------------------------------------
// in part, backward (through CReLU and in_bn)
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void in_bwd_vals(const rnvp_coupling_args& a, const Geo& g, long long b, int cb, int p,
                                            float sc, float sf, float mean, float rstd, float& gxa, float& xh,
                                            float& xm) {
    const int c = (g.kind == 0) ? cb : g.off_base + cb;
    float v = a.x[(b * g.C + c) * g.HW + p];
    if (g.kind == 0 && !ckbd_m(g, p)) v = 0.f;
    xm = v;
    float xa = v * sc + sf;
    const long long m = b * g.HW + p;
    const T* gh = cptr<T>(a.gh0);
    float g1 = ldv(&gh[m * a.cs_gh0 + cb]);
    float g2 = ldv(&gh[m * a.cs_gh0 + g.Cb + cb]);
    gxa = (xa > 0.f ? g1 : 0.f) - (xa < 0.f ? g2 : 0.f);
    xh = (v - mean) * rstd;
}

__device__ __forceinline__ void in_bn_params(const rnvp_coupling_args& a, const Geo& g, int cb, float& sc, float& sf,
                                             float& mean, float& rstd) {
    rnvp_bn_src s;
    s.shards = 1;
    s.sums = a.training ? a.in_sums : nullptr;
    s.count = (double)g.B * g.HW;
    s.mean = a.in_rmean; s.var = a.in_rvar;
    s.gamma = a.in_gamma; s.beta = a.in_beta; s.eps = a.eps;
    bn_affine(s, g.Cb, cb, sc, sf, &mean, &rstd);
}

template <typename T>
__global__ void k_in_bwd_red(rnvp_coupling_args a) {
    __shared__ double red[16];
    const Geo g = geo(a);
    const int b = blockIdx.x / g.Cb, cb = blockIdx.x % g.Cb;
    float sc, sf, mean, rstd;
    in_bn_params(a, g, cb, sc, sf, mean, rstd);
    float s1 = 0.f, s2 = 0.f;
    for (int p = threadIdx.x; p < g.HW; p += blockDim.x) {
        float gxa, xh, xm;
        in_bwd_vals<T>(a, g, b, cb, p, sc, sf, mean, rstd, gxa, xh, xm);
        s1 += gxa;
        s2 += gxa * xh;
    }
    double d1 = block_sum((double)s1, red);
    double d2 = block_sum((double)s2, red);
    if (threadIdx.x == 0) {
        atomicAdd(&a.in_bwd_sums[cb], d1);
        atomicAdd(&a.in_bwd_sums[g.Cb + cb], d2);
    }
}

template <typename T>
__global__ void k_in_bwd_apply(rnvp_coupling_args a) {
    const Geo g = geo(a);
    const int b = blockIdx.x / g.Cb, cb = blockIdx.x % g.Cb;
    float sc, sf, mean, rstd;
    in_bn_params(a, g, cb, sc, sf, mean, rstd);
    const double cnt = (double)g.B * g.HW;
    const float gam = a.in_gamma ? a.in_gamma[cb] : 1.f;
    const float k1 = a.training ? (float)(a.in_bwd_sums[cb] / cnt) : 0.f;
    const float k2 = a.training ? (float)(a.in_bwd_sums[g.Cb + cb] / cnt) : 0.f;
    const int c = (g.kind == 0) ? cb : g.off_base + cb;
    if (blockIdx.x == cb && threadIdx.x == 0) {   // b == 0 block writes the affine grads
        if (a.g_in_beta) a.g_in_beta[cb] = (float)a.in_bwd_sums[cb];
        if (a.g_in_gamma) a.g_in_gamma[cb] = (float)a.in_bwd_sums[g.Cb + cb];
    }
    for (int p = threadIdx.x; p < g.HW; p += blockDim.x) {
        float gxa, xh, xm;
        in_bwd_vals<T>(a, g, b, cb, p, sc, sf, mean, rstd, gxa, xh, xm);
        float gxm = gam * rstd * (gxa - k1 - xh * k2);
        if (g.kind == 0 && !ckbd_m(g, p)) gxm = 0.f;   // xm = x * mask
        a.gx[((long long)b * g.C + c) * g.HW + p] += gxm;
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

}  // namespace

extern "C" int rnvp_coupling_in_fwd(const rnvp_coupling_args* a, void* stream) {
    int st = check(a);
    if (st) return st;
    if (!a->h0 || (a->training && !a->in_sums) || (!a->training && (!a->in_rmean || !a->in_rvar))) return RNVP_E_INVALID;
    const int Cb = cb_of(a);
    if (a->cs_h0 < (a->kind == 0 ? 2 * Cb + 1 : 2 * Cb)) return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    hipStream_t s = (hipStream_t)stream;
    if (a->training) {
        k_in_stats<<<a->B * Cb, 256, 0, s>>>(*a);
        RNVP_LAUNCH_CHECK();
    }
    long long n = (long long)a->B * a->H * a->W * a->cs_h0;
    size_t shm = 2 * Cb * sizeof(float);
    if (a->dtype == RNVP_F32) k_in_apply<float><<<rnvp_grid(n, 256, 2048), 256, shm, s>>>(*a);
    else k_in_apply<bf16_t><<<rnvp_grid(n, 256, 2048), 256, shm, s>>>(*a);
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
    if (a->dtype == RNVP_F32) k_out1<float><<<a->B * a->C, 256, 0, s>>>(*a);
    else k_out1<bf16_t><<<a->B * a->C, 256, 0, s>>>(*a);
    RNVP_LAUNCH_CHECK();
    long long n = (long long)a->B * a->C * a->H * a->W;
    size_t shm = 3 * Cb * sizeof(float);
    if (a->dtype == RNVP_F32) k_out2<float><<<rnvp_grid(n, 256, 2048), 256, shm, s>>>(*a);
    else k_out2<bf16_t><<<rnvp_grid(n, 256, 2048), 256, shm, s>>>(*a);
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
    if (stats) {
        k_out_bwd_red<<<a->B * Cb, 256, 0, s>>>(*a);
        RNVP_LAUNCH_CHECK();
    }
    if (a->dtype == RNVP_F32) k_out_bwd_apply<float><<<a->B * a->C, 256, 0, s>>>(*a);
    else k_out_bwd_apply<bf16_t><<<a->B * a->C, 256, 0, s>>>(*a);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_coupling_in_bwd(const rnvp_coupling_args* a, void* stream) {
    int st = check(a);
    if (st) return st;
    if (!a->gh0 || !a->gx) return RNVP_E_INVALID;
    if (a->training && (!a->in_sums || !a->in_bwd_sums)) return RNVP_E_INVALID;
    if (!a->training && (!a->in_rmean || !a->in_rvar)) return RNVP_E_INVALID;
    const int Cb = cb_of(a);
    if (a->cs_gh0 < 2 * Cb) return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    hipStream_t s = (hipStream_t)stream;
    if (a->training || a->g_in_gamma || a->g_in_beta) {
        if (!a->in_bwd_sums) return RNVP_E_INVALID;
        if (a->dtype == RNVP_F32) k_in_bwd_red<float><<<a->B * Cb, 256, 0, s>>>(*a);
        else k_in_bwd_red<bf16_t><<<a->B * Cb, 256, 0, s>>>(*a);
        RNVP_LAUNCH_CHECK();
    }
    if (a->dtype == RNVP_F32) k_in_bwd_apply<float><<<a->B * Cb, 256, 0, s>>>(*a);
    else k_in_bwd_apply<bf16_t><<<a->B * Cb, 256, 0, s>>>(*a);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}
