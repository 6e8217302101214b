// Deep-scale s/t-network convolutions (scales 3-5 of the 64x64 flow, every
// scale of the 32x32 / config-3 flow): M = B*H*W <= 16k pixels, 128..1024
// channels, K = ks*ks*cs up to 9216.  Same fused operation as rnvp_conv2d's
// other families (conv.hip): BatchNorm+ReLU of the operand, bias / residual /
// skip accumulation, the next BatchNorm's batch sums, or the data-gradient
// ReLU/BN-backward epilogue.
//
// What bounds these shapes is latency, not bytes: a 3x3 at 4x4..16x16 is
// ~4.8 GFLOP over 1-5 MB.  A workgroup owns a 64-pixel x BN-channel output
// tile; its activation rows plus the 3x3 halo are loaded ONCE, BN+ReLU'd
// once into LDS (every tap then reads its A fragment from LDS: no per-tap or
// per-channel-tile re-fetch of pixels), and only the weights stream from
// L2/HBM, through a register ring of DK k-steps per wave.  NW waves (4 or 8)
// are laid out WM (pixel sub-tiles) x WK (interleaved k-steps); the WK
// partial tiles are summed through LDS (aliasing the activation tile) before
// the epilogue.  With WK = NW a wave owns the whole tile and a 1/NW share of
// K (deep K: 3x3 at 256..1024 channels); with WK = 1 the waves split the
// pixels and each walks all of K (1x1 at small K).  Per-shape configuration:
// rnvp_deep_auto_cfg, measured with tools/conv_microbench.py.
#include "conv_deep.h"

namespace {

template <typename T, int BN, int KSZ, bool PRO, int NW, int WK, int DK, int NC, bool FM = false, int BM = DEEP_BM,
          bool BP = false>
__global__ __launch_bounds__(64 * NW) void k_conv_deep(rnvp_conv_args a, int shards, int xa, int xb) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    deep_tile<T, BN, KSZ, PRO, NW, WK, DK, NC, FM, BM, BP>(a, shards, xa, xb, blockIdx.x, gridDim.x, lds);
}

// the BatchNorm-backward prologue (a->bp) is compiled for the data-gradient
// configurations only: 32-channel tiles, whole tile per wave, 64 pixels
// (rnvp_deep_auto_cfg's cfg 0 / 4)
template <int BN, int NW, int WK, int BM>
constexpr bool bp_cfg() { return BN == 32 && WK == NW && BM == DEEP_BM; }

// dry: every check, nothing launched (rnvp_conv2d_check)
template <typename T, int BN, int NW, int WK, int DK, int NC, int KSZ, int BM = DEEP_BM>
int launch_deep_nc(const rnvp_conv_args* a, hipStream_t s, bool dry) {
    const long long M = (long long)a->B * a->H * a->W;
    const size_t shm = deep_lds_bytes<T, BN, NW, WK, BM>(a->cs_in, a->W, a->ks, a->bp != 0);
    if (shm > 160 * 1024) return RNVP_E_UNSUPPORTED;
    const long long gm = (M + BM - 1) / BM, gn = (a->n + BN - 1) / BN;
    const unsigned grid = (unsigned)(gm * gn);
    const int sh = rnvp_stat_shards(M);
    const dim3 blk(64 * NW);
    int xa, xb;
    xcd_blocks(a, (int)gm, (int)gn, BN, sizeof(T), &xa, &xb, BM);
    if (a->bp) {
        if constexpr (bp_cfg<BN, NW, WK, BM>()) {
            if (dry) return RNVP_OK;
            if constexpr (sizeof(T) == 2 && NC <= 4) {
                if (a->w_frag) {
                    k_conv_deep<T, BN, KSZ, false, NW, WK, DK, NC, true, BM, true><<<grid, blk, shm, s>>>(*a, sh, xa, xb);
                    RNVP_LAUNCH_CHECK();
                    return RNVP_OK;
                }
            }
            k_conv_deep<T, BN, KSZ, false, NW, WK, DK, NC, false, BM, true><<<grid, blk, shm, s>>>(*a, sh, xa, xb);
            RNVP_LAUNCH_CHECK();
            return RNVP_OK;
        } else {
            return RNVP_E_UNSUPPORTED;
        }
    }
    if (dry) return RNVP_OK;
    // the fragment-major weight image where the caller provides one (bf16)
    if constexpr (sizeof(T) == 2 && NC <= 4) {
        if (a->w_frag) {
            if (a->pro_bn_relu) k_conv_deep<T, BN, KSZ, true, NW, WK, DK, NC, true, BM><<<grid, blk, shm, s>>>(*a, sh, xa, xb);
            else k_conv_deep<T, BN, KSZ, false, NW, WK, DK, NC, true, BM><<<grid, blk, shm, s>>>(*a, sh, xa, xb);
            RNVP_LAUNCH_CHECK();
            return RNVP_OK;
        }
    }
    if (a->pro_bn_relu) k_conv_deep<T, BN, KSZ, true, NW, WK, DK, NC, false, BM><<<grid, blk, shm, s>>>(*a, sh, xa, xb);
    else k_conv_deep<T, BN, KSZ, false, NW, WK, DK, NC, false, BM><<<grid, blk, shm, s>>>(*a, sh, xa, xb);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

// channel chunks per wave NC = cs / (WK * KS), a template parameter (the
// k-step sequence is unrolled): the channel strides of the RealNVP nets
template <typename T, int BN, int NW, int WK, int DK>
int launch_deep(const rnvp_conv_args* a, hipStream_t s, bool dry) {
    constexpr int KS = 4 * Mf<T>::CH;
    const long long M = (long long)a->B * a->H * a->W;
    if (M > 65536 || a->n < BN / 2 || a->cs_in % (WK * KS)) return RNVP_E_UNSUPPORTED;
    if (a->pro_bn_relu && a->pro.sums && a->pro.shards > 2) return RNVP_E_UNSUPPORTED;
    if (a->epi_relu_bn_bwd && a->epi.sums && a->epi.shards > 2) return RNVP_E_UNSUPPORTED;
    if (a->cs_in > DEEP_MAX_CS) return RNVP_E_UNSUPPORTED;
    if (a->bp && (a->pro_bn_relu || (a->bp_bn.sums && a->bp_bn.shards > 2) || a->bp_shards > 2)) return RNVP_E_UNSUPPORTED;
    const int nc = a->cs_in / (WK * KS);
    if (a->ks == 1) {
        switch (nc) {
            case 1: return launch_deep_nc<T, BN, NW, WK, DK, 1, 1>(a, s, dry);
            case 2: return launch_deep_nc<T, BN, NW, WK, DK, 2, 1>(a, s, dry);
            case 4: return launch_deep_nc<T, BN, NW, WK, DK, 4, 1>(a, s, dry);
            case 8: return launch_deep_nc<T, BN, NW, WK, DK, 8, 1>(a, s, dry);
            case 16: return launch_deep_nc<T, BN, NW, WK, DK, 16, 1>(a, s, dry);
        }
        return RNVP_E_UNSUPPORTED;
    }
    if constexpr (WK == NW) {   // 3x3: whole-tile-per-wave configurations only
        switch (nc) {
            case 1: return launch_deep_nc<T, BN, NW, WK, DK, 1, 3>(a, s, dry);
            case 2: return launch_deep_nc<T, BN, NW, WK, DK, 2, 3>(a, s, dry);
            case 4: return launch_deep_nc<T, BN, NW, WK, DK, 4, 3>(a, s, dry);
            case 8: return launch_deep_nc<T, BN, NW, WK, DK, 8, 3>(a, s, dry);
        }
    }
    return RNVP_E_UNSUPPORTED;
}

// 128-pixel 3x3 tiles (bf16, <= 4 channel chunks per wave): each weight
// slice serves twice the pixels of the 64-pixel tiles
template <typename T, int BN, int NW, int WK, int DK>
int launch_deep_tall(const rnvp_conv_args* a, hipStream_t s, bool dry) {
    constexpr int KS = 4 * Mf<T>::CH;
    if constexpr (sizeof(T) != 2) {
        return RNVP_E_UNSUPPORTED;
    } else {
        const long long M = (long long)a->B * a->H * a->W;
        if (a->ks != 3 || M > 65536 || a->n < BN / 2 || a->cs_in % (WK * KS)) return RNVP_E_UNSUPPORTED;
        if (a->pro_bn_relu && a->pro.sums && a->pro.shards > 2) return RNVP_E_UNSUPPORTED;
        if (a->epi_relu_bn_bwd && a->epi.sums && a->epi.shards > 2) return RNVP_E_UNSUPPORTED;
        switch (a->cs_in / (WK * KS)) {
            case 1: return launch_deep_nc<T, BN, NW, WK, DK, 1, 3, 128>(a, s, dry);
            case 2: return launch_deep_nc<T, BN, NW, WK, DK, 2, 3, 128>(a, s, dry);
            case 4: return launch_deep_nc<T, BN, NW, WK, DK, 4, 3, 128>(a, s, dry);
        }
        return RNVP_E_UNSUPPORTED;
    }
}

//                       BN  NW  WK  DK
// cfg 0                 32   4   4   8   whole 64x32 tile per wave, K / 4 (deep K)
// cfg 1                 64   4   4   6   whole 64x64 tile per wave, K / 4
// cfg 2                 64   4   1   8   16-pixel quarters, all of K (1x1, small K)
// cfg 3                 32   4   2   8   32-pixel halves x K / 2
// cfg 4                 32   8   8   8   cfg 0 with 8 waves (two per SIMD: one's memory waits under the other's MFMAs)
// cfg 5                 64   8   8   6   cfg 1 with 8 waves
// cfg 6                 32   4   4   8   cfg 0 on 128-pixel tiles (bf16 3x3)
template <typename T>
int launch_cfg(const rnvp_conv_args* a, hipStream_t s, int cfg, bool dry) {
    switch (cfg) {
        case 0: return launch_deep<T, 32, 4, 4, 8>(a, s, dry);
        case 1: return launch_deep<T, 64, 4, 4, 6>(a, s, dry);
        case 2: return a->ks == 1 ? launch_deep<T, 64, 4, 1, 8>(a, s, dry) : RNVP_E_UNSUPPORTED;
        case 3: return a->ks == 1 ? launch_deep<T, 32, 4, 2, 8>(a, s, dry) : RNVP_E_UNSUPPORTED;
        case 4: return launch_deep<T, 32, 8, 8, 8>(a, s, dry);
        case 5: return launch_deep<T, 64, 8, 8, 6>(a, s, dry);
        case 6: return launch_deep_tall<T, 32, 4, 4, 8>(a, s, dry);
    }
    return RNVP_E_INVALID;
}

// ---------------------------------------------------------------------------
// grouped independent 1x1 convs: one launch, the convs' tiles concatenated
// (block b -> the conv whose tile range holds b; every conv keeps its own
// XCD-aware tile order).  Both prologue forms are compiled in.
template <typename T, int BN, int NW, int WK, int DK, int NC, bool FM = false>
__global__ __launch_bounds__(64 * NW) void k_net_group(const rnvp_group_kargs g) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    int b = blockIdx.x, c = 0;
    while (c + 1 < g.n && b >= g.tiles[c]) {   // uniform scan over <= RNVP_NET_GROUP_MAX tile counts
        b -= g.tiles[c];
        ++c;
    }
    if (g.conv[c].pro_bn_relu)
        deep_tile<T, BN, 1, true, NW, WK, DK, NC, FM>(g.conv[c], g.shards[c], g.xa[c], g.xb[c], b, g.tiles[c], lds);
    else
        deep_tile<T, BN, 1, false, NW, WK, DK, NC, FM>(g.conv[c], g.shards[c], g.xa[c], g.xb[c], b, g.tiles[c], lds);
}

using GroupKernel = void (*)(const rnvp_group_kargs);

template <typename T, int BN, int NW, int WK, int DK>
GroupKernel group_kernel_nc(int nc, bool fm) {
    if constexpr (sizeof(T) == 2) {
        if (fm) {   // every member carries a fragment-major weight image
            switch (nc) {
                case 1: return k_net_group<T, BN, NW, WK, DK, 1, true>;
                case 2: return k_net_group<T, BN, NW, WK, DK, 2, true>;
                case 4: return k_net_group<T, BN, NW, WK, DK, 4, true>;
            }
            return nullptr;
        }
    }
    if (fm) return nullptr;
    switch (nc) {
        case 1: return k_net_group<T, BN, NW, WK, DK, 1>;
        case 2: return k_net_group<T, BN, NW, WK, DK, 2>;
        case 4: return k_net_group<T, BN, NW, WK, DK, 4>;
        case 8: return k_net_group<T, BN, NW, WK, DK, 8>;
        case 16: return k_net_group<T, BN, NW, WK, DK, 16>;
    }
    return nullptr;
}

// the configuration table of launch_cfg (cfg 0 / 1 / 4 / 5)
template <typename T>
GroupKernel group_kernel_t(int cfg, int nc, bool fm) {
    switch (cfg) {
        case 0: return group_kernel_nc<T, 32, 4, 4, 8>(nc, fm);
        case 1: return group_kernel_nc<T, 64, 4, 4, 6>(nc, fm);
        case 4: return group_kernel_nc<T, 32, 8, 8, 8>(nc, fm);
        case 5: return group_kernel_nc<T, 64, 8, 8, 6>(nc, fm);
    }
    return nullptr;
}

// klass = cfg | nc << 4 | fm << 11 (fm: the members' fragment-major weight images)
constexpr int GROUP_FM = 1 << 11;
GroupKernel group_kernel(int dtype, int klass) {
    const int cfg = klass & 15, nc = (klass >> 4) & 127;
    const bool fm = (klass & GROUP_FM) != 0;
    return dtype == RNVP_F32 ? group_kernel_t<float>(cfg, nc, fm) : group_kernel_t<bf16_t>(cfg, nc, fm);
}

struct GroupCfg { int bn, nw, wk; };
inline GroupCfg group_cfg_shape(int cfg) {
    switch (cfg) {
        case 0: return {32, 4, 4};
        case 1: return {64, 4, 4};
        case 4: return {32, 8, 8};
        default: return {64, 8, 8};
    }
}

}  // namespace

// Grouped 1x1 convs: the group's configuration follows the single-launch
// choice (rnvp_deep_auto_cfg's policy, extended to M <= 16384 for 1x1)
extern "C" int rnvp_net_group_prepare(rnvp_net_step* steps, int n, int* klass, int* grid, int* lds_bytes) {
    if (!steps || n <= 0 || n > RNVP_NET_GROUP_MAX || !klass || !grid || !lds_bytes) return RNVP_E_INVALID;
    const rnvp_conv_args& a0 = steps[0].conv;
    const long long M = (long long)a0.B * a0.H * a0.W;
    // the grouped tiles have no BatchNorm-backward prologue
    for (int i = 0; i < n; ++i)
        if (steps[i].conv.bp) return RNVP_E_UNSUPPORTED;
    // wide scales: convs sharing one input run as a fan-out (conv_s1.hip)
    if (M > 16384) return rnvp_s1_fanout_prepare(steps, n, klass, grid, lds_bytes);
    if (M <= 0) return RNVP_E_UNSUPPORTED;
    if (a0.dtype != RNVP_F32 && a0.dtype != RNVP_BF16) return RNVP_E_INVALID;
    const int kc = a0.dtype == RNVP_F32 ? 16 : 32;   // channels per k-step
    int cfg = -1, nc = -1;
    long long tiles = 0;
    size_t lds = 0;
    for (int i = 0; i < n; ++i) {
        rnvp_net_step& st = steps[i];
        const rnvp_conv_args& a = st.conv;
        if (st.kind != RNVP_STEP_CONV || a.ks != 1) return RNVP_E_UNSUPPORTED;
        if (a.dtype != a0.dtype || a.B != a0.B || a.H != a0.H || a.W != a0.W) return RNVP_E_UNSUPPORTED;
        if (!a.x || !a.w || !a.y || a.n <= 0 || a.cin <= 0 || (a.cs_in & 7) || (a.cs_out & 7)) return RNVP_E_INVALID;
        if (a.cs_in < a.cin || a.cs_out < a.n || (a.kp & 63) || a.kp < a.cs_in) return RNVP_E_INVALID;
        if (((uintptr_t)a.x & 15) || ((uintptr_t)a.w & 15)) return RNVP_E_INVALID;
        if (a.epi_relu_bn_bwd && !a.epi_x) return RNVP_E_INVALID;
        if (a.pro_bn_relu && a.pro.sums && a.pro.shards > 2) return RNVP_E_UNSUPPORTED;
        if (a.epi_relu_bn_bwd && a.epi.sums && a.epi.shards > 2) return RNVP_E_UNSUPPORTED;
        // one configuration for the whole group: the single-launch choice of
        // its first conv (rnvp_deep_auto_cfg, incl. its RNVP_DEEP_MAXM1 limit)
        const int c = rnvp_deep_auto_cfg(&steps[0].conv);
        if (c < 0) return RNVP_E_UNSUPPORTED;
        const GroupCfg g = group_cfg_shape(c);
        if (a.cs_in % (g.wk * kc) || a.cs_in > DEEP_MAX_CS || a.n < g.bn / 2) return RNVP_E_UNSUPPORTED;
        const int ncv = a.cs_in / (g.wk * kc);
        if (ncv != 1 && ncv != 2 && ncv != 4 && ncv != 8 && ncv != 16) return RNVP_E_UNSUPPORTED;
        if (i == 0) {
            cfg = c;
            nc = ncv;
        } else if (c != cfg || ncv != nc) {
            return RNVP_E_UNSUPPORTED;
        }
        const size_t shm = a0.dtype == RNVP_F32
                               ? (g.nw == 8 ? (g.bn == 32 ? deep_lds_bytes<float, 32, 8, 8>(a.cs_in, a.W, 1)
                                                          : deep_lds_bytes<float, 64, 8, 8>(a.cs_in, a.W, 1))
                                            : (g.bn == 32 ? deep_lds_bytes<float, 32, 4, 4>(a.cs_in, a.W, 1)
                                                          : deep_lds_bytes<float, 64, 4, 4>(a.cs_in, a.W, 1)))
                               : (g.nw == 8 ? (g.bn == 32 ? deep_lds_bytes<bf16_t, 32, 8, 8>(a.cs_in, a.W, 1)
                                                          : deep_lds_bytes<bf16_t, 64, 8, 8>(a.cs_in, a.W, 1))
                                            : (g.bn == 32 ? deep_lds_bytes<bf16_t, 32, 4, 4>(a.cs_in, a.W, 1)
                                                          : deep_lds_bytes<bf16_t, 64, 4, 4>(a.cs_in, a.W, 1)));
        if (shm > 160 * 1024) return RNVP_E_UNSUPPORTED;
        if (shm > lds) lds = shm;
        const long long gm = (M + DEEP_BM - 1) / DEEP_BM, gn = (a.n + g.bn - 1) / g.bn;
        st.cfg = c;
        st.nc = ncv;
        st.shards = rnvp_stat_shards(M);
        st.tiles = (int)(gm * gn);
        xcd_blocks(&a, (int)gm, (int)gn, g.bn, a0.dtype == RNVP_F32 ? 4 : 2, &st.xa, &st.xb);
        tiles += st.tiles;
    }
    if (tiles <= 0 || tiles >= (1ll << 31)) return RNVP_E_INVALID;
    bool fm = a0.dtype == RNVP_BF16 && nc <= 4;
    for (int i = 0; i < n; ++i) fm = fm && steps[i].conv.w_frag != nullptr && (((uintptr_t)steps[i].conv.w_frag) & 15) == 0;
    *klass = cfg | (nc << 4) | (fm ? GROUP_FM : 0);
    *grid = (int)tiles;
    *lds_bytes = (int)lds;
    return group_kernel(a0.dtype, *klass) ? RNVP_OK : RNVP_E_UNSUPPORTED;
}

rnvp_group_kargs group_kargs(const rnvp_net_step* steps, int n) {
    rnvp_group_kargs g = {};
    for (int i = 0; i < n; ++i) {
        g.conv[i] = steps[i].conv;
        g.shards[i] = steps[i].shards;
        g.tiles[i] = steps[i].tiles;
        g.xa[i] = steps[i].xa;
        g.xb[i] = steps[i].xb;
    }
    g.n = n;
    return g;
}

extern "C" int rnvp_net_group(const rnvp_net_step* steps, int n, int dtype, int klass, int grid, int lds_bytes,
                              void* stream) {
    if (!steps || n <= 0 || n > RNVP_NET_GROUP_MAX || grid <= 0 || lds_bytes < 0 || lds_bytes > 160 * 1024)
        return RNVP_E_INVALID;
    if (dtype != RNVP_F32 && dtype != RNVP_BF16) return RNVP_E_INVALID;
    const rnvp_group_kargs g = group_kargs(steps, n);
    if (klass & (1 << 12)) {
        if (dtype != RNVP_BF16 || n < 2) return RNVP_E_INVALID;
        return rnvp_s1_fanout_launch(g, klass, grid, lds_bytes, (hipStream_t)stream);
    }
    const GroupKernel k = group_kernel(dtype, klass);
    if (!k) return RNVP_E_INVALID;
    const int nw = group_cfg_shape(klass & 15).nw;
    hipLaunchKernelGGL(k, dim3(grid), dim3(64 * nw), lds_bytes, (hipStream_t)stream, g);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

// measured (tools/conv_microbench.py --deep, profiles/r2_deep_microbench.txt):
// the deep family beats the other families at M <= 1024 (every shape:
// whole-tile-per-wave, K / 4) and for the 3x3 at M <= 4096 (64-channel
// tiles); elsewhere -1 (the caller's other families).
// Round 3 (prologue loads trimmed): 1x1 up to M = 4096 and 3x3 up to
// M = 16384 as well -- step 26.47 -> 26.03 ms (profiles/r3_dispatch_ab.txt);
// 1x1 up to 16384 later (23.70 -> 23.64 ms, three alternating pairs).
// The family takes 1x1 and 3x3 convs up to M = 16384 pixels.
int rnvp_deep_auto_cfg(const rnvp_conv_args* a) {
    const long long M = (long long)a->B * a->H * a->W;
    if (M > 16384) return -1;
    // per-shape choice from tools/conv_microbench.py --deep
    // (profiles/r3_deep_microbench_cfgs.txt): the 8-wave tiles at M <= 1024;
    // 32-channel tiles for the data gradients above (more workgroups); the
    // 8-wave 64-channel tile for the forward convs at 256+ channels
    const bool dgrad = a->epi_relu_bn_bwd || (!a->pro_bn_relu && !a->out_sums);
    const int kc = a->dtype == RNVP_F32 ? 16 : 32;   // channels per k-step
    if (M <= 1024) return a->cs_in % (8 * kc) == 0 ? 4 : 0;
    if (dgrad) return 0;
    // 128-pixel tiles for the bf16 3x3 forward convs at 128 channels (scale 3:
    // 21.8 vs 22.6-23.1 us with fragment-major weights; data gradients and the
    // wider channels measured slower, gpurun_out/r5_tall)
    if (a->ks == 3 && a->dtype == RNVP_BF16 && M > 4096 && a->cs_in == 128) return 6;
    // (32-channel tiles for the forward convs as well measured slower in the
    // step, profiles/r4_step_ab.txt)
    return a->cs_in % (8 * kc) == 0 ? 5 : 1;
}

int rnvp_deep_launch(const rnvp_conv_args* a, hipStream_t s, int cfg, bool dry) {
    if (cfg < 0 || cfg >= RNVP_DEEP_CFGS) return RNVP_E_INVALID;
    return a->dtype == RNVP_F32 ? launch_cfg<float>(a, s, cfg, dry) : launch_cfg<bf16_t>(a, s, cfg, dry);
}
