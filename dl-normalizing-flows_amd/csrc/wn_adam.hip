// Row-local parameter pass: weight-norm backward + Adam + the next step's
// weight norm and packed weight images, in ONE launch per coupling.
//
// Replaces, for every WeightNormConv2d (modules_realnvp.py:53-71) of the
// s/t network, the chain
//     k_wn_bwd (dv, dg, dbias from the wgrad slabs)            -- per coupling
//     k_adam   (torch.optim.Adam step, train.py:134, 200)      -- whole arena
//     k_wn_norm + k_wn_pack (||v|| and both packed images)     -- next step
// which streamed the 120 M conv parameters four times per step.  Everything
// a row of v needs is local to that output channel co: the slab sums of dW,
// <dW, v>, ||v||, g[co], the bias, Adam's element-wise update and the new
// ||v'|| -- so one workgroup owns RB consecutive output rows of one conv,
// keeps them in LDS (fp32, packed-k order) and writes the next step's
// forward image wf[co][tap*cs_in+ci] row by row.  The transposed
// data-gradient image wd[ci][tp*cs_out+co] spans all output channels of a
// conv per row: it is derived from wf by rnvp_weight_norm_transpose, once
// per step for the whole model (RB-channel runs of wd written from here
// measured a third of the launch: 49 of 143 us at config 1's scale 5).
//
// from_slabs = 1 (single process): dW is the sum of the grouped wgrad's nz
// replica slabs (rnvp_conv2d_wgrad_grouped); dv/dg/dbias are computed here
// (and also stored in the gradient arena).  from_slabs = 0 (data parallel):
// dv/dg/dbias are read from the gradient arena after the all-reduce.
#include "common.h"
#include "conv_common.h"

namespace {

typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int WA_THREADS = 512;
#ifndef WA_LDS_KB
#define WA_LDS_KB 38
#endif
#ifndef WA_U
#define WA_U 2
#endif
#ifndef WA_UV
#define WA_UV 1
#endif
#ifndef WA_UD
#define WA_UD 4
#endif
#ifndef WA_SKIP
#define WA_SKIP 0
#endif
#ifndef WA_WPE
#define WA_WPE 6
#endif
constexpr int WA_LDS = WA_LDS_KB * 1024;   // four workgroups per CU

// LDS floats per tap: a 3x3 row keeps its taps cs_in + 4 apart (banks of the
// v-order accesses tap*P + ci skew by 4 per tap; rows stay 16-byte aligned)
__host__ __device__ inline int wa_pitch(int cs_in, int kk) { return kk == 1 ? cs_in : cs_in + 4; }
__host__ __device__ inline int wa_row(int cs_in, int kk) { return kk * wa_pitch(cs_in, kk); }
// output rows per workgroup: 8 (one wave per row) down to 1 (8 waves per row)
__host__ __device__ inline int wa_rb(int cs_in, int kk) {
    const int row = 4 * wa_row(cs_in, kk);
    for (int rb = 8; rb >= 1; rb >>= 1)
        if (rb * row <= WA_LDS) return rb;
    return 0;
}

__device__ __forceinline__ int find_blk(const rnvp_wn_desc* d, int n, int b) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (d[mid].blk0 <= b) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

template <typename T, bool SLABS>
__global__ __launch_bounds__(WA_THREADS) __attribute__((amdgpu_waves_per_eu(WA_WPE, 8))) void k_wn_adam(const rnvp_wn_desc* __restrict__ descs, int n_desc,
                                                        rnvp_adam_args ad, int nblk, double* z0, long long n0,
                                                        double* z1, long long n1) {
    if ((int)blockIdx.x >= nblk) {   // extra workgroups: zero the caller's sums ranges
        const long long stride = (long long)(gridDim.x - nblk) * blockDim.x;
        const long long i0 = (long long)(blockIdx.x - nblk) * blockDim.x + threadIdx.x;
        for (long long i = i0; i < n0; i += stride) z0[i] = 0.0;
        for (long long i = i0; i < n1; i += stride) z1[i] = 0.0;
        return;
    }
    extern __shared__ float tile[];
    __shared__ double red[8 * 4];
    __shared__ float scl[8];
    __shared__ float coef[2];
    // logical block order: XCD x (hardware block b runs on XCD b % 8) owns a
    // contiguous run of row blocks
    const int nb = nblk, b = blockIdx.x;
    const int q8 = nb / 8, r8 = nb % 8, xcd = b % 8;
    const int lb = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
    const rnvp_wn_desc d = descs[find_blk(descs, n_desc, lb)];
    const int kk = d.ks * d.ks, kr = d.cin * kk;
    const int P = wa_pitch(d.cs_in, kk), RP = kk * P;
    const int rb = wa_rb(d.cs_in, kk), wpr = 8 / rb, tpr = 64 * wpr;
    const int co0 = (lb - d.blk0) * rb, nr = min(rb, d.cout - co0);
    const int r = (threadIdx.x >> 6) / wpr, tr = threadIdx.x % tpr;
    const int co = co0 + r;
    const bool live = r < nr;
    float* trow = tile + r * RP;
    if (threadIdx.x == 0) {
        const double t = (double)(ad.step[0] + ad.step_add);
        const double bc1 = 1.0 - pow((double)ad.beta1, t), bc2 = 1.0 - pow((double)ad.beta2, t);
        coef[0] = (float)(ad.lr / bc1);
        coef[1] = (float)(1.0 / sqrt(bc2));
    }
    const long long vrow = d.dv_off + (long long)co * kr;
    RNVP_GLOBAL float* pv = (RNVP_GLOBAL float*)ad.param + vrow;
    RNVP_GLOBAL float* gv = (RNVP_GLOBAL float*)ad.grad + vrow;
    RNVP_GLOBAL float* mv = (RNVP_GLOBAL float*)ad.exp_avg + vrow;
    RNVP_GLOBAL float* sv = (RNVP_GLOBAL float*)ad.exp_avg_sq + vrow;
    const float rkk = 1.0f / (float)kk;
    const int nz = d.nz > 0 ? d.nz : 1;
    const long long zs = (long long)d.cout * d.kp_f;
    // ---- phase 0: dW row (sum of the nz replica slabs) into LDS, packed-k order.
    // Loops below issue U iterations' loads before using any of them (loads
    // past the end are clamped to the iteration's first element and their
    // results -- identical -- stored twice), so every lane keeps several
    // memory round trips in flight; no load sits under a branch.
    constexpr int U = WA_U;
    if (SLABS && live && WA_SKIP != 2) {
        const int K4 = kk * d.cs_in / 4;           // cs_in % 8 == 0: a chunk never straddles a tap
        const float rcs = 1.0f / (float)d.cs_in;
        const RNVP_GLOBAL floatx4* src = (const RNVP_GLOBAL floatx4*)(d.dw + (long long)co * d.kp_f);
        for (int q0 = tr; q0 < K4; q0 += U * tpr) {
            floatx4 t[U];
#pragma unroll
            for (int u = 0; u < U; ++u) t[u] = src[q0 + u * tpr < K4 ? q0 + u * tpr : q0];
            for (int z = 1; z < nz; ++z) {
#pragma unroll
                for (int u = 0; u < U; ++u) t[u] += src[(q0 + u * tpr < K4 ? q0 + u * tpr : q0) + z * zs / 4];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int q4 = q0 + u * tpr < K4 ? q0 + u * tpr : q0;
                const int k = 4 * q4, tap = fdiv_small(k, rcs), ci = k - tap * d.cs_in;
                *(floatx4*)(trow + tap * P + ci) = t[u];
            }
        }
    }
    __syncthreads();
    const float step_size = coef[0], inv_bc2s = coef[1];
    const float nrm = (d.g && live) ? ((const RNVP_GLOBAL float*)d.norm)[co] : 1.f;
    const float gold = (d.g && live) ? ((const RNVP_GLOBAL float*)d.g)[co] : 1.f;
    // ---- phase 1a: <dW, v> (weight-norm backward needs it before dv).
    // Summed in k_wn_bwd's order: 256 virtual threads vt = lane + 64 vw take
    // i = vt + 256 j (j ascending), a butterfly per virtual wave, the four
    // wave sums added in order -- so the fused and the separate passes agree
    // bitwise (a near-cancelling <dW, v> is order-sensitive in its last bits)
    const int lane = threadIdx.x & 63, pw = (threadIdx.x >> 6) % wpr;
    double dot = 0.0;
    if (SLABS && d.g && WA_SKIP != 3) {
        constexpr int UD = WA_UD;
        for (int vw = pw; vw < 4; vw += wpr) {
            double acc = 0.0;
            if (live) {
                for (int i0 = lane + 64 * vw; i0 < kr; i0 += 256 * UD) {
                    float x[UD];
#pragma unroll
                    for (int u = 0; u < UD; ++u) x[u] = pv[i0 + 256 * u < kr ? i0 + 256 * u : i0];
#pragma unroll
                    for (int u = 0; u < UD; ++u) {
                        const int i = i0 + 256 * u < kr ? i0 + 256 * u : i0;
                        const int ci = fdiv_small(i, rkk), tap = i - ci * kk;
                        const double t = fma((double)trow[tap * P + ci], (double)x[u], acc);
                        acc = i0 + 256 * u < kr ? t : acc;
                    }
                }
            }
            acc = wave_sum(acc);
            if (lane == 0) red[r * 4 + vw] = acc;
        }
        __syncthreads();
        dot = 0.0;
        for (int vw = 0; vw < 4; ++vw) dot += red[r * 4 + vw];
    }
    // ---- phase 1b: dv, Adam, v' into LDS.  Element-wise (any mapping gives
    // the same bits): the 16-byte-aligned body of the row in float4 chunks,
    // the 0-3 element head and tail (the arenas' rows need not be aligned)
    // one element per lane
    if (live && WA_SKIP != 4) {
        const float gs = gold / nrm;
        const float proj = (float)(dot / ((double)nrm * nrm));
        auto elem = [&](int i, float p, float gin, float& m, float& v2, float dwv, float& g) {
            g = SLABS ? (d.g ? gs * fmaf(-proj, p, dwv) : dwv) : gin;
            return adam_elem(p, g, m, v2, 1, ad.beta1, ad.beta2, ad.eps, ad.weight_decay, ad.reg_coef, step_size,
                             inv_bc2s);
        };
        auto lds_at = [&](int i) {
            const int ci = fdiv_small(i, rkk), tap = i - ci * kk;
            return tap * P + ci;
        };
        const int h = min(kr, (int)((4 - (vrow & 3)) & 3));
        const int nb4 = (kr - h) >> 2, t0 = h + 4 * nb4;
        if (tr < h + (kr - t0)) {     // head / tail: at most 6 scalar elements
            const int i = tr < h ? tr : t0 + (tr - h);
            const int l = lds_at(i);
            float m = mv[i], v2 = sv[i], g = SLABS ? 0.f : gv[i];
            const float pn = elem(i, pv[i], g, m, v2, SLABS ? trow[l] : 0.f, g);
            if (SLABS) gv[i] = g;
            pv[i] = pn;
            mv[i] = m;
            sv[i] = v2;
            trow[l] = pn;
        }
        RNVP_GLOBAL floatx4* p4 = (RNVP_GLOBAL floatx4*)(pv + h);
        RNVP_GLOBAL floatx4* g4 = (RNVP_GLOBAL floatx4*)(gv + h);
        RNVP_GLOBAL floatx4* m4 = (RNVP_GLOBAL floatx4*)(mv + h);
        RNVP_GLOBAL floatx4* s4 = (RNVP_GLOBAL floatx4*)(sv + h);
        constexpr int UV = WA_UV;
        for (int c0 = tr; c0 < nb4; c0 += UV * tpr) {
            // every operand (LDS dW included) is read before the first store:
            // a clamped duplicate must see the old values
            floatx4 P4[UV], M4[UV], S4[UV], G4[UV];
            float DW[UV][4];
#pragma unroll
            for (int u = 0; u < UV; ++u) {
                const int c = c0 + u * tpr < nb4 ? c0 + u * tpr : c0;
                P4[u] = p4[c];
                M4[u] = m4[c];
                S4[u] = s4[c];
                if (!SLABS) G4[u] = g4[c];
            }
            if (SLABS) {
#pragma unroll
                for (int u = 0; u < UV; ++u) {
                    const int c = c0 + u * tpr < nb4 ? c0 + u * tpr : c0;
#pragma unroll
                    for (int e = 0; e < 4; ++e) DW[u][e] = trow[lds_at(h + 4 * c + e)];
                }
            }
#pragma unroll
            for (int u = 0; u < UV; ++u) {
                const int c = c0 + u * tpr < nb4 ? c0 + u * tpr : c0;
                floatx4 pn, go;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float m = M4[u][e], v2 = S4[u][e], g;
                    pn[e] = elem(h + 4 * c + e, P4[u][e], SLABS ? 0.f : G4[u][e], m, v2, SLABS ? DW[u][e] : 0.f, g);
                    M4[u][e] = m;
                    S4[u][e] = v2;
                    go[e] = g;
                }
                if (SLABS) g4[c] = go;
                p4[c] = pn;
                m4[c] = M4[u];
                s4[c] = S4[u];
#pragma unroll
                for (int e = 0; e < 4; ++e) trow[lds_at(h + 4 * c + e)] = pn[e];
            }
        }
    }
    __syncthreads();
    // ---- per-row scalars, by the first wave of the row group: ||v'|| in
    // k_wn_norm's order (lane l sums i = l + 64 u ascending, then a
    // butterfly), the bias gradient in k_wn_bwd's (one replica per lane,
    // butterfly), g (weight_g) and the bias through Adam
    if (live && pw == 0) {
        double ss = 0.0;
        for (int i = lane; i < kr; i += 64) {
            const int ci = fdiv_small(i, rkk), tap = i - ci * kk;
            const float x = trow[tap * P + ci];
            ss = fma((double)x, (double)x, ss);
        }
        ss = wave_sum(ss);
        float db = 0.f;
        if (d.db_off >= 0) {
            if (SLABS) {
                for (int z = lane; z < nz; z += 64) db += ((const RNVP_GLOBAL float*)d.dbp)[(long long)z * d.cout + co];
                db = wave_sum(db);
            }
        }
        if (lane == 0) {
            RNVP_GLOBAL float* P0 = (RNVP_GLOBAL float*)ad.param;
            RNVP_GLOBAL float* G0 = (RNVP_GLOBAL float*)ad.grad;
            RNVP_GLOBAL float* M0 = (RNVP_GLOBAL float*)ad.exp_avg;
            RNVP_GLOBAL float* S0 = (RNVP_GLOBAL float*)ad.exp_avg_sq;
            const RNVP_GLOBAL uint8_t* K0 = (const RNVP_GLOBAL uint8_t*)ad.mask;
            const float nn = (float)sqrt(ss);
            float gnew = gold;
            if (d.g && d.dg_off >= 0) {
                const long long o = d.dg_off + co;
                float dg;
                if (SLABS) {
                    dg = (float)(dot / nrm);
                    G0[o] = dg;
                } else {
                    dg = G0[o];
                }
                const int f = K0 ? K0[o] : 1;
                if (f) {
                    float m = M0[o], s = S0[o];
                    gnew = adam_elem(gold, dg, m, s, f, ad.beta1, ad.beta2, ad.eps, ad.weight_decay, ad.reg_coef,
                                     step_size, inv_bc2s);
                    P0[o] = gnew;
                    M0[o] = m;
                    S0[o] = s;
                }
            }
            if (d.g) ((RNVP_GLOBAL float*)d.norm)[co] = nn;
            scl[r] = d.g ? gnew / nn : 1.f;
            if (d.db_off >= 0) {
                const long long o = d.db_off + co;
                if (SLABS) G0[o] = db;
                else db = G0[o];
                const int f = K0 ? K0[o] : 1;
                if (f) {
                    float m = M0[o], s = S0[o];
                    P0[o] = adam_elem(P0[o], db, m, s, f, ad.beta1, ad.beta2, ad.eps, ad.weight_decay,
                                      ad.reg_coef, step_size, inv_bc2s);
                    M0[o] = m;
                    S0[o] = s;
                }
            }
        }
    }
    // leave the replica slabs zero for the next step's atomic accumulation
    if (SLABS && d.zero_after && live) {
        RNVP_GLOBAL float* dwz = (RNVP_GLOBAL float*)(d.dw + (long long)co * d.kp_f);
        const int K4 = kk * d.cs_in / 4;
        for (int z = 0; z < nz; ++z)
            for (int q4 = tr; q4 < K4; q4 += tpr)
                *(RNVP_GLOBAL floatx4*)(dwz + z * zs + 4 * q4) = floatx4{0.f, 0.f, 0.f, 0.f};
        if (d.dbp && tr < nz) ((RNVP_GLOBAL float*)d.dbp)[(long long)tr * d.cout + co] = 0.f;
    }
    __syncthreads();
    // ---- phase 2: the next step's packed images from the LDS rows
    if (live && WA_SKIP != 1) {   // forward image: row co, CH consecutive ci per store
        constexpr int CH = 16 / sizeof(T);
        const int ng = (d.cin + CH - 1) / CH;
        const float rng = 1.0f / (float)ng;
        const float sc = scl[r];
        T* wrow = (T*)d.wf + (long long)co * d.kp_f;
        for (int q = tr; q < kk * ng; q += tpr) {
            const int tap = fdiv_small(q, rng), c0 = (q - tap * ng) * CH;
            const float* src = trow + tap * P + c0;
            T* dst = wrow + tap * d.cs_in + c0;
            if (c0 + CH <= d.cin) {
                float v[CH];
#pragma unroll
                for (int e = 0; e < CH; e += 4) {
                    const floatx4 t = *(const floatx4*)(src + e);
                    v[e] = sc * t.x; v[e + 1] = sc * t.y; v[e + 2] = sc * t.z; v[e + 3] = sc * t.w;
                }
                *(RNVP_GLOBAL u32x4*)dst = pack(v, T());
            } else {
                for (int e = 0; c0 + e < d.cin; ++e) stg(dst + e, sc * src[e]);
            }
        }
    }
    // (the data-gradient image follows from the forward image:
    // rnvp_weight_norm_transpose, one launch for the whole model)
}

// zero a table of byte ranges (8-byte multiples): blockIdx.y = range
__global__ void k_zero_ranges(const rnvp_range* __restrict__ r) {
    const rnvp_range q = r[blockIdx.y];
    RNVP_GLOBAL double* p = (RNVP_GLOBAL double*)q.p;
    const long long n = q.bytes / 8;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        p[i] = 0.0;
}

// leftover trainable elements (BatchNorm affines, coupling scales, ...)
__global__ void k_adam_gather(rnvp_adam_args ad, const long long* __restrict__ idx, long long n) {
    __shared__ float coef[2];
    if (threadIdx.x == 0) {
        const double t = (double)(ad.step[0] + ad.step_add);
        const double bc1 = 1.0 - pow((double)ad.beta1, t), bc2 = 1.0 - pow((double)ad.beta2, t);
        coef[0] = (float)(ad.lr / bc1);
        coef[1] = (float)(1.0 / sqrt(bc2));
    }
    __syncthreads();
    for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < n; q += (long long)gridDim.x * blockDim.x) {
        const long long o = idx[q];
        const int f = ad.mask ? ad.mask[o] : 1;
        if (!f) continue;
        float m = ad.exp_avg[o], s = ad.exp_avg_sq[o];
        ad.param[o] = adam_elem(ad.param[o], ad.grad[o], m, s, f, ad.beta1, ad.beta2, ad.eps, ad.weight_decay,
                                ad.reg_coef, coef[0], coef[1]);
        ad.exp_avg[o] = m;
        ad.exp_avg_sq[o] = s;
    }
}

}  // namespace

extern "C" int rnvp_weight_norm_opt_blocks(int cout, int cin, int ks) {
    if (cout <= 0 || cin <= 0 || (ks != 1 && ks != 3)) return RNVP_E_INVALID;
    const int rb = wa_rb((cin + 7) / 8 * 8, ks * ks);
    if (rb == 0) return RNVP_E_UNSUPPORTED;
    return (cout + rb - 1) / rb;
}

extern "C" int rnvp_weight_norm_bwd_adam(const rnvp_wn_desc* d, int n_desc, int total_blocks, int from_slabs,
                                         int dtype, const rnvp_adam_args* ad, void* zero0, long long zero0_bytes,
                                         void* zero1, long long zero1_bytes, void* stream) {
    if (!d || !ad || n_desc <= 0 || total_blocks <= 0) return RNVP_E_INVALID;
    if (!ad->param || !ad->grad || !ad->exp_avg || !ad->exp_avg_sq || !ad->step) return RNVP_E_INVALID;
    if (dtype != RNVP_F32 && dtype != RNVP_BF16) return RNVP_E_INVALID;
    if (zero0_bytes < 0 || zero1_bytes < 0 || (zero0_bytes & 7) || (zero1_bytes & 7)) return RNVP_E_INVALID;
    if ((zero0_bytes && (!zero0 || ((uintptr_t)zero0 & 7))) || (zero1_bytes && (!zero1 || ((uintptr_t)zero1 & 7))))
        return RNVP_E_INVALID;
    const long long nzr = (zero0_bytes > zero1_bytes ? zero0_bytes : zero1_bytes) / 8;
    const int extra = nzr > 0 ? (int)((nzr + 511) / 512 < 16 ? (nzr + 511) / 512 : 16) : 0;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid(total_blocks + extra);
    double* a0 = (double*)zero0;
    double* a1 = (double*)zero1;
    const long long c0 = zero0_bytes / 8, c1 = zero1_bytes / 8;
    if (dtype == RNVP_BF16) {
        if (from_slabs) k_wn_adam<bf16_t, true><<<grid, WA_THREADS, WA_LDS, s>>>(d, n_desc, *ad, total_blocks, a0, c0, a1, c1);
        else k_wn_adam<bf16_t, false><<<grid, WA_THREADS, WA_LDS, s>>>(d, n_desc, *ad, total_blocks, a0, c0, a1, c1);
    } else {
        if (from_slabs) k_wn_adam<float, true><<<grid, WA_THREADS, WA_LDS, s>>>(d, n_desc, *ad, total_blocks, a0, c0, a1, c1);
        else k_wn_adam<float, false><<<grid, WA_THREADS, WA_LDS, s>>>(d, n_desc, *ad, total_blocks, a0, c0, a1, c1);
    }
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_adam_gather(const rnvp_adam_args* ad, const long long* idx, long long n, void* stream) {
    if (!ad || n < 0 || (n > 0 && !idx)) return RNVP_E_INVALID;
    if (!ad->param || !ad->grad || !ad->exp_avg || !ad->exp_avg_sq || !ad->step) return RNVP_E_INVALID;
    if (n == 0) return RNVP_OK;
    k_adam_gather<<<rnvp_grid(n, 256, 1024), 256, 0, (hipStream_t)stream>>>(*ad, idx, n);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_zero_ranges(const rnvp_range* ranges_device, int n, long long max_bytes, void* stream) {
    if (n < 0 || max_bytes < 0 || (n > 0 && !ranges_device)) return RNVP_E_INVALID;
    if (n == 0 || max_bytes == 0) return RNVP_OK;
    if (n > 65535) return RNVP_E_UNSUPPORTED;
    const long long per = (max_bytes / 8 + 255) / 256;
    const unsigned bx = (unsigned)(per < 16 ? per : 16);
    k_zero_ranges<<<dim3(bx, (unsigned)n), 256, 0, (hipStream_t)stream>>>(ranges_device);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}
