// Shared device helpers for the RealNVP MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "realnvp_hip.h"

typedef uint16_t bf16_t;                                        // bf16 storage
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));      // MFMA operand
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define RNVP_LDS __attribute__((address_space(3)))
// global-memory view of a pointer read from memory (a descriptor table):
// accesses through it compile to global_* instead of flat_* operations (a
// flat operation also counts on lgkmcnt, so LDS waits wait for it as well)
#define RNVP_GLOBAL __attribute__((address_space(1)))

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

// scalar load/store of a net-activation element as float
__device__ __forceinline__ float ldv(const float* p) { return *p; }
__device__ __forceinline__ float ldv(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ void stv(float* p, float v) { *p = v; }
__device__ __forceinline__ void stv(bf16_t* p, float v) { *p = f2bf(v); }

// elements per 16-byte chunk
template <typename T> struct Chunk;
template <> struct Chunk<float> { static constexpr int N = 4; };
template <> struct Chunk<bf16_t> { static constexpr int N = 8; };

// unpack / pack one 16-byte chunk
__device__ __forceinline__ void unpack(const u32x4& c, float* v, float) {
    v[0] = __uint_as_float(c.x); v[1] = __uint_as_float(c.y);
    v[2] = __uint_as_float(c.z); v[3] = __uint_as_float(c.w);
}
__device__ __forceinline__ void unpack(const u32x4& c, float* v, bf16_t) {
    uint32_t w[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}
__device__ __forceinline__ u32x4 pack(const float* v, float) {
    u32x4 c;
    c.x = __float_as_uint(v[0]); c.y = __float_as_uint(v[1]);
    c.z = __float_as_uint(v[2]); c.w = __float_as_uint(v[3]);
    return c;
}
__device__ __forceinline__ u32x4 pack(const float* v, bf16_t) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
    u32x4 c;
    c.x = w[0]; c.y = w[1]; c.z = w[2]; c.w = w[3];
    return c;
}

// 4 consecutive elements (8 B of bf16 / 16 B of f32) <-> float[4]
__device__ __forceinline__ void ld4(const float* p, float* v) {
    const floatx4 t = *(const floatx4*)p;
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
}
__device__ __forceinline__ void ld4(const bf16_t* p, float* v) {
    const uint2 t = *(const uint2*)p;
    v[0] = __uint_as_float(t.x << 16); v[1] = __uint_as_float(t.x & 0xffff0000u);
    v[2] = __uint_as_float(t.y << 16); v[3] = __uint_as_float(t.y & 0xffff0000u);
}
__device__ __forceinline__ void st4(float* p, const float* v) { *(floatx4*)p = floatx4{v[0], v[1], v[2], v[3]}; }
__device__ __forceinline__ void st4(bf16_t* p, const float* v) {
    uint2 t;
    t.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    t.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *(uint2*)p = t;
}

// load / store through a global-memory view (pointers read from descriptor tables)
__device__ __forceinline__ float ldg(const RNVP_GLOBAL float* p) { return *p; }
__device__ __forceinline__ float ldg(const RNVP_GLOBAL bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ void stg(float* p, float v) { *(RNVP_GLOBAL float*)p = v; }
__device__ __forceinline__ void stg(bf16_t* p, float v) { *(RNVP_GLOBAL bf16_t*)p = f2bf(v); }

// one element of torch.optim.Adam (single-tensor form, coupled L2 weight
// decay, train.py:134); f = 2 adds the 5e-5 * weight_scale regulariser's
// gradient 2*reg*p (train.py:194).  m, v updated in place; returns p'.
// step_size = lr / (1 - b1^t), inv_bc2s = 1 / sqrt(1 - b2^t).
// Every multiply-add is an explicit fmaf and no other product feeds an
// addition, so no FMA contraction is left to the compiler: the kernels that
// inline this (k_adam, k_adam_gather, k_wn_adam) compute bitwise the same
// update from the same operands.
__device__ __forceinline__ float adam_elem(float p, float g, float& m, float& v, int f, float b1, float b2, float eps,
                                           float wd, float reg, float step_size, float inv_bc2s) {
    float gr = fmaf(wd, p, g);
    if (f == 2) gr = fmaf(2.f * reg, p, gr);
    m = fmaf(1.f - b1, gr - m, m);
    const float t = (1.f - b2) * gr;
    v = fmaf(v, b2, t * gr);
    const float den = fmaf(sqrtf(v), inv_bc2s, eps);
    return p - (step_size * m) / den;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Sum over the 16 lanes of a DPP row (lanes 16r .. 16r+15 = one MFMA column
// group); every lane of the row gets the result.  row_ror butterfly on the
// VALU (no LDS round trip: __shfl_xor lowers to ds_bpermute).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ float row_sum16(float v) {
    v += dpp_f<0x128>(v); v += dpp_f<0x124>(v); v += dpp_f<0x122>(v); v += dpp_f<0x121>(v);
    return v;
}
__device__ __forceinline__ double row_sum16(double v) {
    v += dpp_d<0x128>(v); v += dpp_d<0x124>(v); v += dpp_d<0x122>(v); v += dpp_d<0x121>(v);
    return v;
}

// block-wide sum (blockDim.x multiple of 64, <= 1024); every thread gets the result
template <typename F>
__device__ __forceinline__ F block_sum(F v, F* red /* >= 16 entries of LDS */) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    F t = 0;
    for (int i = 0; i < nw; ++i) t += red[i];
    return t;
}

// per-channel BN affine (scale, shift) such that bn(x) = x*scale + shift:
// the alpha/beta form ATen's batch_norm applies (the reference's own
// arithmetic; a centred (x - mean)*scale + beta form was measured further
// from the fp64 truth on the deep goldens, whose near-degenerate channels
// make ReLU decisions rounding-sensitive)
__device__ __forceinline__ void bn_affine(const rnvp_bn_src& s, int C, int c, float& scale, float& shift,
                                          float* mean_out = nullptr, float* rstd_out = nullptr) {
    double mean, var;
    if (s.sums) {
        // shards <= 32 (rnvp_stat_shards, RNVP_COUPLING_SHARDS): every load is
        // issued up front (clamped address, masked contribution), then added in
        // shard order -- one memory round trip instead of one per shard
        double v1[32], v2[32];
        const int ns = s.shards > 0 ? s.shards : 1;
#pragma unroll
        for (int h = 0; h < 32; ++h) {
            const long long o = (long long)(h < ns ? h : 0) * 2 * C;
            v1[h] = s.sums[o + c];
            v2[h] = s.sums[o + C + c];
        }
        double s1 = 0, s2 = 0;
#pragma unroll
        for (int h = 0; h < 32; ++h) {
            if (h < ns) {
                s1 += v1[h];
                s2 += v2[h];
            }
        }
        mean = s1 / s.count;
        var = s2 / s.count - mean * mean;
        if (var < 0) var = 0;
    } else {
        mean = s.mean[c];
        var = s.var[c];
    }
    float rstd = (float)(1.0 / sqrt(var + (double)s.eps));
    float g = s.gamma ? s.gamma[c] : 1.f;
    float b = s.beta ? s.beta[c] : 0.f;
    scale = g * rstd;
    shift = b - (float)mean * g * rstd;
    if (mean_out) *mean_out = (float)mean;
    if (rstd_out) *rstd_out = rstd;
}

// Whole-block reduction of sharded BN sums ([shards][2*C] fp64) for channels
// [c0, c0+nc) into LDS s1[nc], s2[nc]; up to two independent sources in one
// pass.  Every (channel, shard) pair is a separate load spread over the block;
// a thread issues up to 4 pairs' loads at once (the first round before the
// barrier that zeroes the outputs), then accumulates them with LDS fp64
// atomics (ds_add_f64).  Must be reached by every thread of the block.
struct ShardSrc {
    const double* sums; int C, shards, c0, nc; double* s1; double* s2;
};

template <int NS>
__device__ __forceinline__ void block_shard_sums_n(const ShardSrc (&src)[NS]) {
    constexpr int U = 4;
    int total[NS], tmax = 0;
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        total[q] = src[q].sums ? src[q].nc * (src[q].shards < 1 ? 1 : src[q].shards) : 0;
        tmax = max(tmax, total[q]);
    }
    auto zero = [&]() {
#pragma unroll
        for (int q = 0; q < NS; ++q)
            for (int i = threadIdx.x; i < src[q].nc; i += blockDim.x) {
                src[q].s1[i] = 0.0;
                src[q].s2[i] = 0.0;
            }
        __syncthreads();
    };
    if (tmax <= 0) zero();
    for (int t0 = 0; t0 < tmax; t0 += U * blockDim.x) {
        double v1[NS][U], v2[NS][U];
        int cc[NS][U];
#pragma unroll
        for (int q = 0; q < NS; ++q)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = t0 + u * blockDim.x + threadIdx.x;
                cc[q][u] = -1;
                v1[q][u] = v2[q][u] = 0.0;
                if (t < total[q]) {
                    const int c = t % src[q].nc, h = t / src[q].nc;
                    const double* p = src[q].sums + (long long)h * 2 * src[q].C + src[q].c0 + c;
                    v1[q][u] = p[0];
                    v2[q][u] = p[src[q].C];
                    cc[q][u] = c;
                }
            }
        if (t0 == 0) zero();
#pragma unroll
        for (int q = 0; q < NS; ++q)
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (cc[q][u] >= 0) {
                    atomicAdd(&src[q].s1[cc[q][u]], v1[q][u]);
                    atomicAdd(&src[q].s2[cc[q][u]], v2[q][u]);
                }
    }
    __syncthreads();
}

__device__ __forceinline__ void block_shard_sums(const double* sums, int C, int shards, int c0, int nc, double* s1,
                                                 double* s2) {
    const ShardSrc src[1] = {{sums, C, shards, c0, nc, s1, s2}};
    block_shard_sums_n<1>(src);
}

// block_shard_sums split in two: shard_issue loads a thread's entries into
// registers (first thing in a kernel, ahead of its bulk loads: vmcnt waits in
// issue order), shard_finish folds them into s1 / s2 (LDS fp64 atomics, as
// block_shard_sums).  Needs nc * shards <= U * blockDim.x (shard_fits).
template <int U>
struct ShardLoads {
    double v1[U], v2[U];
    int cc[U];
};
__device__ __forceinline__ bool shard_fits(int nc, int shards, int U) {
    return (long long)nc * (shards < 1 ? 1 : shards) <= (long long)U * blockDim.x;
}
template <int U>
__device__ __forceinline__ void shard_issue(const double* sums, int C, int shards, int c0, int nc, ShardLoads<U>& L) {
    const int total = nc * (shards < 1 ? 1 : shards);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        // unconditional loads (an index past the table reads entry 0 and is
        // marked unused): no branch, so no wait is forced at its join
        const int t = u * blockDim.x + threadIdx.x;
        const bool ok = t < total;
        const int tt = ok ? t : 0;
        const int c = tt % nc, h = tt / nc;
        const double* p = sums + (long long)h * 2 * C + c0 + c;
        L.v1[u] = p[0];
        L.v2[u] = p[C];
        L.cc[u] = ok ? c : -1;
    }
}
template <int U>
__device__ __forceinline__ void shard_finish(const ShardLoads<U>& L, int nc, double* s1, double* s2) {
    for (int i = threadIdx.x; i < nc; i += blockDim.x) {
        s1[i] = 0.0;
        s2[i] = 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (L.cc[u] >= 0) {
            atomicAdd(&s1[L.cc[u]], L.v1[u]);
            atomicAdd(&s2[L.cc[u]], L.v2[u]);
        }
    __syncthreads();
}

// shard_finish without zeroing and without LDS atomics: every thread parks
// its loaded entries in tab (2 * U * blockDim.x doubles of LDS) at their
// entry index h * nc + c, ONE barrier, then thread c < nc adds channel c's
// shards in shard order into s1[c] / s2[c] (deterministic).  No branch and no
// loop sits between the shard loads and their first use, so the wait for
// them counts only the loads issued before them (the tile loads a kernel
// issued after them stay in flight).  The sums are left for the SAME thread
// (block_bn_finish_aff reads entry threadIdx.x): no trailing barrier.
// Needs nc <= blockDim.x and shard_fits(nc, shards, U).
template <int U>
__device__ __forceinline__ void shard_sum_tab(const ShardLoads<U>& L, int nc, int shards, double* tab, double* s1,
                                              double* s2) {
    const int n = U * blockDim.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int t = u * blockDim.x + threadIdx.x;
        tab[t] = L.v1[u];
        tab[n + t] = L.v2[u];
    }
    __syncthreads();
    const int i = threadIdx.x;
    if (i < nc) {
        const int hs = shards < 1 ? 1 : shards;
        double a = 0.0, b = 0.0;
        for (int h = 0; h < hs; ++h) {
            a += tab[h * nc + i];
            b += tab[n + h * nc + i];
        }
        s1[i] = a;
        s2[i] = b;
    }
}

// Affine parameters of channel c0 + threadIdx.x, loaded into registers with
// a prologue's other loads (bn_aff_issue) so that the table finish below
// waits on no global load.  No branch: an absent gamma / beta reads `any` (a
// valid global address of the same launch, value unused) and the finish
// applies the default 1 / 0.
struct BnAff { float g, b; };
__device__ __forceinline__ BnAff bn_aff_issue(const rnvp_bn_src& s, int C, int c0, const void* any) {
    const int c = max(0, min(c0 + (int)threadIdx.x, C - 1));
    const float* gp = s.gamma ? s.gamma : (const float*)any;
    const float* bp = s.beta ? s.beta : (const float*)any;
    return BnAff{gp[s.gamma ? c : 0], bp[s.beta ? c : 0]};
}

// one channel of the BN table (i < nv: a real channel; else padding)
__device__ __forceinline__ void bn_finish_entry(const rnvp_bn_src& s, int c, int i, int nc, int nv, const double* tmp,
                                                float g, float b, float* scale, float* shift, float* mean_out,
                                                float* rstd_out) {
    float sc = 0.f, sf = 0.f, mo = 0.f, ro = 1.f;
    if (i < nv) {
        double mean, var;
        if (s.sums) {
            mean = tmp[i] / s.count;
            var = tmp[nc + i] / s.count - mean * mean;
            if (var < 0) var = 0;
        } else {
            mean = s.mean[c];
            var = s.var[c];
        }
        const float rstd = (float)(1.0 / sqrt(var + (double)s.eps));
        sc = g * rstd;
        sf = b - (float)mean * g * rstd;
        mo = (float)mean;
        ro = rstd;
    }
    scale[i] = sc;
    shift[i] = sf;
    if (mean_out) mean_out[i] = mo;
    if (rstd_out) rstd_out[i] = ro;
}

// BN table for channels [c0, c0+nc) from already-reduced sums tmp[0..nc) /
// tmp[nc..2nc) (train) or the running stats (eval): scale/shift such that
// bn(x) = x*scale + shift, plus mean / rstd when requested.  Channels >= C
// (padding) get scale = shift = 0, mean = 0, rstd = 1.
__device__ __forceinline__ void block_bn_finish(const rnvp_bn_src& s, int C, int c0, int nc, float* scale, float* shift,
                                                float* mean_out, float* rstd_out, const double* tmp) {
    const int nv = max(0, min(nc, C - c0));
    for (int i = threadIdx.x; i < nc; i += blockDim.x) {
        const int c = c0 + i;
        const float g = (i < nv && s.gamma) ? s.gamma[c] : 1.f;
        const float b = (i < nv && s.beta) ? s.beta[c] : 0.f;
        bn_finish_entry(s, c, i, nc, nv, tmp, g, b, scale, shift, mean_out, rstd_out);
    }
    __syncthreads();
}

// block_bn_finish for nc <= blockDim.x with the affine parameters in
// registers (bn_aff_issue(s, C, c0, ...))
__device__ __forceinline__ void block_bn_finish_aff(const rnvp_bn_src& s, int C, int c0, int nc, float* scale,
                                                    float* shift, float* mean_out, float* rstd_out, const double* tmp,
                                                    BnAff A) {
    const int nv = max(0, min(nc, C - c0));
    const int i = threadIdx.x;
    if (i < nc)
        bn_finish_entry(s, c0 + i, i, nc, nv, tmp, s.gamma ? A.g : 1.f, s.beta ? A.b : 0.f, scale, shift, mean_out,
                        rstd_out);
    __syncthreads();
}

// Whole-block BN table (shard reduction + finish).  tmp: 2*nc doubles of LDS.
// Must be reached by every thread of the block.
__device__ __forceinline__ void block_bn_table(const rnvp_bn_src& s, int C, int c0, int nc, float* scale, float* shift,
                                               float* mean_out, float* rstd_out, double* tmp) {
    const int nv = max(0, min(nc, C - c0));
    if (s.sums) block_shard_sums(s.sums, C, s.shards, c0, nv, tmp, tmp + nc);
    block_bn_finish(s, C, c0, nc, scale, shift, mean_out, rstd_out, tmp);
}

static inline int rnvp_grid(long long n, int block, int cap = 4096) {
    long long g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

#define RNVP_LAUNCH_CHECK() do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)
