// Shared device helpers of the affine-coupling kernels (coupling.hip,
// coupling_link.hip): coupling geometry, pixel tiles, per-channel segment
// reductions and the sharded fp64 statistic tables.
#pragma once
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
// pixel tiles
// ---------------------------------------------------------------------------
// A workgroup owns TP consecutive pixels of one image (all channels): NCHW
// flow-tensor planes are read/written as coalesced TP-runs per channel, the
// NHWC net tensors (h0, st and their gradients) as one contiguous
// [TP][cs] region staged through LDS, per-channel reductions are wave
// segment sums (seg = min(TP, 64) lanes share a channel) folded into LDS and
// then one global atomic per channel per workgroup.
struct Tile {
    int b, p0, tp;
    long long m0;
};

__device__ __forceinline__ Tile tile_of(const Geo& g, int TP) {
    const int tpi = (g.HW + TP - 1) / TP;
    Tile t;
    t.b = blockIdx.x / tpi;
    t.p0 = (blockIdx.x - t.b * tpi) * TP;
    t.tp = min(TP, g.HW - t.p0);
    t.m0 = (long long)t.b * g.HW + t.p0;
    return t;
}

// Elements of a block's first CP_K passes (e0 = 256 k) whose global operands
// are loaded at kernel entry, before the BN tables / LDS tiles: their memory
// round trip overlaps the table's (one exposed latency instead of two or
// three per launch; at the deep scales every thread has <= 2 elements)
constexpr int CP_K = 4;

// sum over groups of `seg` lanes (power of 2 <= 64; 1 = no reduction)
__device__ __forceinline__ float seg_sum(float v, int seg) {
    for (int o = 1; o < seg; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double seg_sum(double v, int seg) {
    for (int o = 1; o < seg; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// per-channel sums of doubles over a lane segment: seg >= 16 (the wide
// scales) -> DPP row sums on the VALU, every 16-lane row's lane 0 then adds
// its row (rows never straddle a segment); shorter segments -> ds_bpermute
// shuffles.  The shuffles were the coupling passes' bottleneck at the wide
// scales (6 steps x 2 bpermutes per double and quantity).  seg_mask: a lane
// with (lane & seg_mask(seg)) == 0 holds a sum to add.
__device__ __forceinline__ double seg_red(double v, int seg) { return seg >= 16 ? row_sum16(v) : seg_sum(v, seg); }
__device__ __forceinline__ int seg_mask(int seg) { return seg >= 16 ? 15 : seg - 1; }

template <typename T>
__device__ __forceinline__ void tile_copy_in(const void* src, long long m0, int tp, int cs, T* lds) {
    const int n16 = tp * cs * (int)sizeof(T) / 16;
    const u32x4* s = (const u32x4*)((const T*)src + m0 * cs);
    u32x4* d = (u32x4*)lds;
    for (int i = threadIdx.x; i < n16; i += blockDim.x) d[i] = s[i];
}

template <typename T>
__device__ __forceinline__ void tile_copy_out(const T* lds, long long m0, int tp, int cs, void* dst) {
    const int n16 = tp * cs * (int)sizeof(T) / 16;
    const u32x4* s = (const u32x4*)lds;
    u32x4* d = (u32x4*)((T*)dst + m0 * cs);
    for (int i = threadIdx.x; i < n16; i += blockDim.x) d[i] = s[i];
}

// an NHWC tile's 16-B chunks loaded into registers (R per thread, clamped
// unconditional loads) and stored to LDS later: the loads of several tiles
// and tables go out together, one memory round trip for all of them
template <int R>
struct TileRegs {
    u32x4 v[R];
    int n16;
};
template <typename T, int R>
__device__ __forceinline__ void tile_issue(const void* src, long long m0, int tp, int cs, TileRegs<R>& r) {
    r.n16 = tp * cs * (int)sizeof(T) / 16;
    const u32x4* s = (const u32x4*)((const T*)src + m0 * cs);
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int i = (int)threadIdx.x + k * (int)blockDim.x;
        r.v[k] = s[i < r.n16 ? i : 0];
    }
}
template <typename T, int R>
__device__ __forceinline__ void tile_commit(const TileRegs<R>& r, const void* src, long long m0, int cs, T* lds) {
    u32x4* d = (u32x4*)lds;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int i = (int)threadIdx.x + k * (int)blockDim.x;
        if (i < r.n16) d[i] = r.v[k];
    }
    const u32x4* s = (const u32x4*)((const T*)src + m0 * cs);
    for (int i = (int)threadIdx.x + R * (int)blockDim.x; i < r.n16; i += blockDim.x) d[i] = s[i];
}

__device__ __forceinline__ void lds_zero(double* p, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0.0;
}

// coupling reductions: [RNVP_COUPLING_SHARDS][k*Cb] fp64, this block's shard
__device__ __forceinline__ double* cshard(double* sums, int width) {
    return sums + (long long)(blockIdx.x % RNVP_COUPLING_SHARDS) * width;
}
// sum over the shards of entry i of a [shards][width] reduction.  Fully
// unrolled: all RNVP_COUPLING_SHARDS loads are independent and go out
// together (one memory round trip, not one per unroll group), then are
// added in shard order.
__device__ __forceinline__ double csum(const double* sums, int width, int i) {
    double v[RNVP_COUPLING_SHARDS];
#pragma unroll
    for (int h = 0; h < RNVP_COUPLING_SHARDS; ++h) v[h] = sums[(long long)h * width + i];
    double t = 0.0;
#pragma unroll
    for (int h = 0; h < RNVP_COUPLING_SHARDS; ++h) t += v[h];
    return t;
}

// per-channel in_bn table of the in part: scale, shift, mean, rstd [Cb each]
__device__ __forceinline__ void in_bn_table(const rnvp_coupling_args& a, const Geo& g, float* t) {
    for (int cb = threadIdx.x; cb < g.Cb; cb += blockDim.x) {
        rnvp_bn_src s;
        s.shards = RNVP_COUPLING_SHARDS;
        s.sums = a.training ? a.in_sums : nullptr;
        s.count = (double)g.B * g.HW;
        s.mean = a.in_rmean; s.var = a.in_rvar;
        s.gamma = a.in_gamma; s.beta = a.in_beta; s.eps = a.eps;
        float sc, sf, mean, rstd;
        bn_affine(s, g.Cb, cb, sc, sf, &mean, &rstd);
        t[cb] = sc;
        t[g.Cb + cb] = sf;
        t[2 * g.Cb + cb] = mean;
        t[3 * g.Cb + cb] = rstd;
    }
}

// the coupling's affine transform of one transformed element (modules_realnvp.py:278, 293):
// lr = scale*tanh(r) + scale_shift, u = x*exp(lr) + shift.  Explicit FMAs: every kernel that
// (re)computes u gets the same bits.
__device__ __forceinline__ float coupling_u(float x, float sh, float r, float sc, float ss, float& lr, float& th,
                                            float& ex) {
    th = tanhf(r);
    lr = fmaf(sc, th, ss);
    ex = expf(lr);
    return fmaf(x, ex, sh);
}

__host__ __device__ inline int r4(int x) { return (x + 3) / 4 * 4; }

}  // namespace
