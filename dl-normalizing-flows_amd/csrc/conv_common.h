// Device helpers shared by the conv kernel translation units (conv.hip,
// conv_deep.hip): MFMA step per operand type, LDS swizzle, BN-statistics
// shards, the fused 4-channel epilogue, register BN tables, fast division.
// Included inside each file's anonymous namespace.
#pragma once
#include <math.h>

#include "common.h"

namespace {

template <typename T> struct Mf;
template <> struct Mf<bf16_t> {
    static constexpr int CH = 8;
    __device__ static __forceinline__ void step(const u32x4& a, const u32x4& b, floatx4& c) {
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
    }
};
template <> struct Mf<float> {
    static constexpr int CH = 4;
    // lane group g supplies k = 4g + s at sub-step s (same mapping for A and B)
    __device__ static __forceinline__ void step(const u32x4& a, const u32x4& b, floatx4& c) {
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), c, 0, 0, 0);
    }
};

// [row][8 chunks of 16 B]; XOR swizzle spreads the 16 rows one ds_read_b128
// lane group reads over all 64 banks (rows r, r+1 differ in bank half, r>>1
// picks the chunk).
__device__ __forceinline__ int sw8(int row, int c) { return row * 8 + (c ^ ((row >> 1) & 7)); }

__device__ __forceinline__ double* shard_ptr(double* sums, int shards, int N) {
    return sums ? sums + (long long)(blockIdx.x % shards) * 2 * N : nullptr;
}

// 4-channel epilogue in the transposed layout: y = acc + bias (+ residual)
// (+ y), or the dgrad ReLU/BN-backward form; BN statistics into s1/s2.
// et: LDS epilogue table at channel n0 (scale | shift | mean | rstd, pitch).
template <typename T>
__device__ __forceinline__ void epi4(const rnvp_conv_args& a, long long o, const floatx4& acc, const float* bias,
                                     bool epi_bn, const float* et, int pitch, double* s1, double* s2, int nvalid) {
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = acc[r] + bias[r];
    if (a.residual) {
        float t[4];
        ld4((const T*)a.residual + o, t);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += t[r];
    }
    if (a.accumulate) {
        float t[4];
        ld4((const T*)a.y + o, t);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += t[r];
    }
    if (epi_bn) {
        float xv[4];
        ld4((const T*)a.epi_x + o, xv);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (xv[r] * et[r] + et[pitch + r] <= 0.f) v[r] = 0.f;
            s1[r] += v[r];
            s2[r] += v[r] * (xv[r] - et[2 * pitch + r]) * et[3 * pitch + r];
        }
    } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            s1[r] += v[r];
            s2[r] += (double)v[r] * v[r];
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (r >= nvalid) v[r] = 0.f;
    st4((T*)a.y + o, v);
}

// the epilogue operands of one 4-channel element (residual, previous y for
// the skip accumulation, the dgrad epilogue's pre-BN x), loaded at kernel
// start so the epilogue waits on no global round trip
struct EpiPre {
    float r[4], y[4], x[4];
};

template <typename T>
__device__ __forceinline__ void epi_prefetch(const rnvp_conv_args& a, long long o, bool live, EpiPre& p) {
    const long long oo = live ? o : 0;
    if (a.residual) ld4((const T*)a.residual + oo, p.r);
    if (a.accumulate) ld4((const T*)a.y + oo, p.y);
    if (a.epi_relu_bn_bwd) ld4((const T*)a.epi_x + oo, p.x);
}

// epi4 over prefetched operands
template <typename T>
__device__ __forceinline__ void epi4p(const rnvp_conv_args& a, long long o, const floatx4& acc, const float* bias,
                                      bool epi_bn, const float* et, int pitch, double* s1, double* s2, int nvalid,
                                      const EpiPre& p) {
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = acc[r] + bias[r];
    if (a.residual) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += p.r[r];
    }
    if (a.accumulate) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += p.y[r];
    }
    if (epi_bn) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (p.x[r] * et[r] + et[pitch + r] <= 0.f) v[r] = 0.f;
            s1[r] += v[r];
            s2[r] += v[r] * (p.x[r] - et[2 * pitch + r]) * et[3 * pitch + r];
        }
    } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            s1[r] += v[r];
            s2[r] += (double)v[r] * v[r];
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (r >= nvalid) v[r] = 0.f;
    st4((T*)a.y + o, v);
}

// in-image tap mask of an output pixel at column x, row y (0 <= x < W,
// 0 <= y < H): bit ky*KSZ + kx is set iff tap (ky, kx) of the KSZ x KSZ
// (pad KSZ/2) window reads inside the image -- the outer product of three
// row bits and three column bits (~8 VALU instead of 9 taps x 5 compares)
template <int KSZ>
__device__ __forceinline__ unsigned tap_mask(int x, int y, int W, int H, bool valid) {
    static_assert(KSZ == 1 || KSZ == 3, "1x1 / 3x3");
    if constexpr (KSZ == 1) {
        return valid ? 1u : 0u;
    } else {
        const unsigned cb = (x > 0 ? 1u : 0u) | 2u | (x < W - 1 ? 4u : 0u);
        const unsigned mk = (y > 0 ? cb : 0u) | (cb << 3) | (y < H - 1 ? cb << 6 : 0u);
        return valid ? mk : 0u;
    }
}

// BN+ReLU of 8 bf16 channels (one 16-B chunk), scale / shift per channel:
// packed fp32 FMAs, the bf16 rounding, then ReLU as a packed signed-16-bit
// max against 0 on the rounded pair (a bf16 with its sign bit set is a
// negative int16; relu commutes with the monotone rounding, so the bits equal
// rounding max(x*sc+sh, 0)).  20 VALU per chunk instead of 28.
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef short i16x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x4 bn_relu_bf16x8(const u32x4& c, const float* sc, const float* sh) {
    const uint32_t w[4] = {c.x, c.y, c.z, c.w};
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f32x2_t x = {__uint_as_float(w[i] << 16), __uint_as_float(w[i] & 0xffff0000u)};
        const f32x2_t y = __builtin_elementwise_fma(x, f32x2_t{sc[2 * i], sc[2 * i + 1]}, f32x2_t{sh[2 * i], sh[2 * i + 1]});
        const uint32_t p = __builtin_bit_cast(uint32_t, __builtin_convertvector(y, bf16x2_t));
        o[i] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(i16x2_t, p), i16x2_t{0, 0}));
    }
    return u32x4{o[0], o[1], o[2], o[3]};
}

// Row pitch (elements) of an LDS image read by MFMA operand loads: lane l
// reads 16 B at row (l & 15) (+ a common row offset), 16-B column (l >> 4)
// (+ a common column).  ds_read_b128 serves lanes {0-3,12-15,20-27},
// {4-11,16-19,28-31}, ... as one bank group each (MI355X_MICROARCH.md SS LDS),
// so a row pitch of 16-B units == 2 (mod 4) puts every group on 16 distinct
// 16-B bank slots for ANY row / column offset; the former "+16 B" pitches
// (units odd) were 2-way conflicted on every read.
__host__ __device__ constexpr int lds_mfma_pitch(int elems, int ch) {
    return (elems / ch + ((2 - elems / ch) & 3)) * ch;
}
template <typename T>
__host__ __device__ constexpr int halo_pitch(int cs) { return lds_mfma_pitch(cs, Mf<T>::CH); }


// BN table for channels [c0, c0+nc) of a source with <= 2 stat shards, in
// registers (CPT channels per thread of NT, no LDS atomics): tab_issue loads
// (unconditional, clamped addresses, so the loads can stay in flight behind
// later ones), tab_finish forms scale/shift (+ mean, rstd) into LDS.
template <int CPT>
struct BnTab {
    double a1[CPT], a2[CPT], b1[CPT], b2[CPT];
    float gam[CPT], bet[CPT];
};

template <int CPT, int NT = 256>
__device__ __forceinline__ void tab_issue(const rnvp_bn_src& s, int C, int c0, int nc, BnTab<CPT>& t) {
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
        const int c = threadIdx.x + NT * j;
        const int cc = (c < nc && c0 + c < C) ? c0 + c : 0;
        if (s.sums) {
            t.a1[j] = s.sums[cc];
            t.a2[j] = s.sums[C + cc];
            if (s.shards > 1) {   // uniform: the second shard's loads only when it exists
                t.b1[j] = s.sums[2 * (long long)C + cc];
                t.b2[j] = s.sums[3 * (long long)C + cc];
            } else {
                t.b1[j] = t.b2[j] = 0.0;
            }
        } else {
            t.a1[j] = s.mean[cc];
            t.a2[j] = s.var[cc];
            t.b1[j] = t.b2[j] = 0.0;
        }
        t.gam[j] = s.gamma ? s.gamma[cc] : 1.f;
        t.bet[j] = s.beta ? s.beta[cc] : 0.f;
    }
}

template <int CPT, int NT = 256>
__device__ __forceinline__ void tab_finish(const rnvp_bn_src& s, int C, int c0, int nc, const BnTab<CPT>& t,
                                           float* scale, float* shift, float* mean_out, float* rstd_out) {
    const double inv = s.sums ? 1.0 / s.count : 0.0;
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
        const int c = threadIdx.x + NT * j;
        if (c >= nc) continue;
        float sc = 0.f, sf = 0.f, mo = 0.f, ro = 1.f;
        if (c0 + c < C) {
            double mean, var;
            if (s.sums) {
                const double s1 = t.a1[j] + (s.shards > 1 ? t.b1[j] : 0.0);
                const double s2 = t.a2[j] + (s.shards > 1 ? t.b2[j] : 0.0);
                mean = s1 * inv;
                var = s2 * inv - mean * mean;
                if (var < 0) var = 0;
            } else {
                mean = t.a1[j];
                var = t.a2[j];
            }
            const float rstd = (float)(1.0 / sqrt(var + (double)s.eps));
            sc = t.gam[j] * rstd;
            sf = t.bet[j] - (float)mean * t.gam[j] * rstd;
            mo = (float)mean;
            ro = rstd;
        }
        scale[c] = sc;
        shift[c] = sf;
        if (mean_out) mean_out[c] = mo;
        if (rstd_out) rstd_out[c] = ro;
    }
}

// floor(q / d) for 0 <= q < 2^22 from a float reciprocal r = 1/d: q + 0.5 is
// >= 0.5 away from any multiple of d, far more than the rounding error.
__device__ __forceinline__ int fdiv_small(int q, float r) { return (int)(((float)q + 0.5f) * r); }

// floor(q / d) for 0 <= q < 2^31 with q / d < 2^22 (r = 1/d): the float
// quotient is within 0.75 of the true one, one correction step each way.
__device__ __forceinline__ int fdiv_exact(int q, int d, float r) {
    int t = (int)((float)q * r);
    t -= (t * d > q) ? 1 : 0;
    t += ((t + 1) * d <= q) ? 1 : 0;
    return t;
}

// BatchNorm backward apply over the blocks blk = 0..nblk-1 of a (virtual)
// grid: every block reduces the statistic shards into its LDS table, then
// grid-strides over the 16-byte chunks.  dsm: 68*cs bytes of LDS
// (tmp [2*cs] | gsum [2*cs] fp64 | p [5*cs] f32 | table [4*cs] f32).
// GAM: gamma present -- its values for the thread's first two channels are
// loaded ahead of the shard reduction, so no global round trip sits between
// the reduction and the streaming loop (mean / rstd / coef follow
// block_bn_finish's arithmetic exactly).
template <typename T, bool GAM>
__device__ __forceinline__ void bn_bwd_run(const rnvp_bn_bwd_args& a, double* dsm, int blk, int nblk) {
    constexpr int CH = Mf<T>::CH;
    const int cs = a.cs, C = a.C;
    const double cnt = (double)a.M;
    double* gs = dsm + 2 * cs;
    float* p = (float*)(dsm + 4 * cs);   // per channel: coef, k1, k2, mean, rstd
    float gpre[2] = {1.f, 1.f};
    if constexpr (GAM) {
#pragma unroll
        for (int j = 0; j < 2; ++j) gpre[j] = a.bn.gamma[min((int)threadIdx.x + j * (int)blockDim.x, C - 1)];
    }
    // the thread's first data chunk is loaded before the statistic tables, so
    // its latency overlaps theirs instead of following the reduction (at the
    // deep scales that is every chunk of the thread); the optional operands
    // through a pointer select -- no branch around the loads
    const T* G = (const T*)a.g;
    const T* X = (const T*)a.x;
    const T* R = (const T*)a.residual;
    T* DX = (T*)a.dx;
    const int cpr = cs / CH;
    const long long nch = a.M * cpr;
    const long long q0 = blk * (long long)blockDim.x + threadIdx.x, qs = (long long)nblk * blockDim.x;
    const long long of = (q0 < nch ? q0 : 0) * CH;
    const u32x4 fg = *(const u32x4*)(G + of), fx = *(const u32x4*)(X + of);
    const u32x4 fr = *(const u32x4*)((R ? R : G) + of), fd = *(const u32x4*)((a.accumulate ? (const T*)DX : G) + of);
    // both shard reductions (forward BN stats, backward g-sums): every load
    // issued up front, without branches, when the tables fit one pass
    // (ShardLoads); otherwise the looping block reduction
    const bool two = a.bn.sums != nullptr;
    if (shard_fits(C, a.sum_shards, 4) && shard_fits(C, two ? a.bn.shards : 1, 4)) {
        ShardLoads<4> lg, lb;
        shard_issue<4>(a.sums, C, a.sum_shards, 0, C, lg);
        shard_issue<4>(two ? a.bn.sums : a.sums, C, two ? a.bn.shards : a.sum_shards, 0, C, lb);
        for (int i = threadIdx.x; i < C; i += blockDim.x) {
            gs[i] = gs[cs + i] = 0.0;
            dsm[i] = dsm[cs + i] = 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (lg.cc[u] >= 0) {
                atomicAdd(&gs[lg.cc[u]], lg.v1[u]);
                atomicAdd(&gs[cs + lg.cc[u]], lg.v2[u]);
            }
            if (two && lb.cc[u] >= 0) {
                atomicAdd(&dsm[lb.cc[u]], lb.v1[u]);
                atomicAdd(&dsm[cs + lb.cc[u]], lb.v2[u]);
            }
        }
        __syncthreads();
    } else if (two) {
        const ShardSrc src[2] = {{a.sums, C, a.sum_shards, 0, C, gs, gs + cs},
                                 {a.bn.sums, C, a.bn.shards, 0, C, dsm, dsm + cs}};
        block_shard_sums_n<2>(src);
    } else {
        const ShardSrc src[1] = {{a.sums, C, a.sum_shards, 0, C, gs, gs + cs}};
        block_shard_sums_n<1>(src);
    }
    auto entry = [&](int c, float gam) {
        float coef = 0.f, k1 = 0.f, k2 = 0.f, mean = 0.f, rstd = 1.f;
        if (c < C) {
            double mn, var;
            if (a.bn.sums) {
                mn = dsm[c] / a.bn.count;
                var = dsm[cs + c] / a.bn.count - mn * mn;
                if (var < 0) var = 0;
            } else {
                mn = a.bn.mean[c];
                var = a.bn.var[c];
            }
            rstd = (float)(1.0 / sqrt(var + (double)a.bn.eps));
            mean = (float)mn;
            coef = gam * rstd;
            const double g1 = gs[c], g2 = gs[cs + c];
            if (a.bn.sums) {   // train mode: batch statistics carry gradient
                k1 = (float)(g1 / cnt);
                k2 = (float)(g2 / cnt);
            }
            if (blk == 0) {
                if (a.dbeta) a.dbeta[c] = (float)g1;
                if (a.dgamma) a.dgamma[c] = (float)g2;
            }
        }
        p[5 * c] = coef; p[5 * c + 1] = k1; p[5 * c + 2] = k2; p[5 * c + 3] = mean; p[5 * c + 4] = rstd;
    };
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int c = threadIdx.x + j * blockDim.x;
        if (c < cs) entry(c, gpre[j]);
    }
    for (int c = threadIdx.x + 2 * blockDim.x; c < cs; c += blockDim.x) entry(c, GAM ? a.bn.gamma[c] : 1.f);
    __syncthreads();
    // the grid stride is a multiple of the chunks per pixel in practice: the
    // channel chunk of a thread is then fixed (no 64-bit modulo per chunk)
    const bool fixed = qs % cpr == 0;
    int c0 = (int)(q0 % cpr) * CH;
    auto apply = [&](long long o, const u32x4& vg, const u32x4& vx, const u32x4& vr, const u32x4& vd) {
        float g[CH], x[CH], d[CH];
        unpack(vg, g, T());
        unpack(vx, x, T());
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            const float* pp = p + 5 * (c0 + j);
            const float xh = (x[j] - pp[3]) * pp[4];
            d[j] = pp[0] * (g[j] - pp[1] - xh * pp[2]);
        }
        if (R) {
            float r[CH];
            unpack(vr, r, T());
#pragma unroll
            for (int j = 0; j < CH; ++j) d[j] += r[j];
        }
        if (a.accumulate) {
            float r[CH];
            unpack(vd, r, T());
#pragma unroll
            for (int j = 0; j < CH; ++j) d[j] += r[j];
        }
        *(u32x4*)(DX + o) = pack(d, T());
    };
    if (q0 < nch) apply(q0 * CH, fg, fx, fr, fd);
    for (long long q = q0 + qs; q < nch; q += qs) {
        const long long o = q * CH;
        if (!fixed) c0 = (int)(q % cpr) * CH;
        const u32x4 vg = *(const u32x4*)(G + o), vx = *(const u32x4*)(X + o);
        const u32x4 vr = R ? *(const u32x4*)(R + o) : vg;
        const u32x4 vd = a.accumulate ? *(const u32x4*)(DX + o) : vg;
        apply(o, vg, vx, vr, vd);
    }
}

template <typename T>
__device__ __forceinline__ void bn_bwd_body(const rnvp_bn_bwd_args& a, double* dsm, int blk, int nblk) {
    if (a.bn.gamma) bn_bwd_run<T, true>(a, dsm, blk, nblk);
    else bn_bwd_run<T, false>(a, dsm, blk, nblk);
}

}  // namespace

// deep-scale conv family (conv_deep.hip): number of configurations and the
// launcher of configuration cfg (RNVP_E_UNSUPPORTED when it does not apply)
constexpr int RNVP_DEEP_CFGS = 7;
int rnvp_deep_launch(const rnvp_conv_args* a, hipStream_t s, int cfg, bool dry = false);
int rnvp_deep_auto_cfg(const rnvp_conv_args* a);

// tap-shared bf16 weight gradients (wgrad_tap.hip): RNVP_E_UNSUPPORTED when a
// conv of the group is outside its staging limits (the caller falls back)
int rnvp_wgrad_tap_launch(rnvp_wgrad_group* g, hipStream_t s);

// register-pipelined streaming 1x1 conv (conv_s1.hip): RNVP_E_UNSUPPORTED
// outside bf16 / 1x1 / <= 64 channels / M >= 16k; dry: checks only
int rnvp_conv_s1_launch(const rnvp_conv_args* a, hipStream_t s, bool dry = false);

// fan-out groups of 1x1 convs sharing one input at the wide scales (conv_s1.hip):
// the M > 16k branch of rnvp_net_group_prepare / rnvp_net_group (klass bit 12)
// A group's members travel BY VALUE in the kernel arguments (2.2 KB):
// pointers a kernel reads from its argument segment are known to address
// global memory (global_load / global_store).  Read from a device table they
// were generic -- flat operations, which count on lgkmcnt as well as vmcnt, so
// every LDS wait of a tile also waited for its global loads and stores.
struct rnvp_group_kargs {
    rnvp_conv_args conv[RNVP_NET_GROUP_MAX];
    int shards[RNVP_NET_GROUP_MAX], tiles[RNVP_NET_GROUP_MAX], xa[RNVP_NET_GROUP_MAX], xb[RNVP_NET_GROUP_MAX];
    int n;
};
rnvp_group_kargs group_kargs(const rnvp_net_step* steps, int n);
int rnvp_s1_fanout_prepare(rnvp_net_step* steps, int n, int* klass, int* grid, int* lds_bytes);
int rnvp_s1_fanout_launch(const rnvp_group_kargs& g, int klass, int grid, int lds_bytes, hipStream_t s);

// persistent band kernel for the wide-scale 3x3 convs (conv_band.hip):
// RNVP_E_UNSUPPORTED outside 3x3 / 17..64 outputs / cs_in <= 64 / 32k <= M < 2^21
int rnvp_conv_band2_launch(const rnvp_conv_args* a, hipStream_t s, bool dry = false);
