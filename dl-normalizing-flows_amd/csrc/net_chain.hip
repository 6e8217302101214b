// Persistent net chain: the deep-scale s/t-net steps of one coupling in ONE
// launch.
//
// At M <= 4096 pixels a coupling's forward is 18 dependent convs and its
// backward 18 data-gradient convs + 13 BatchNorm-backward applies, each a
// few microseconds of work behind a kernel boundary (dispatch, ramp, drain,
// cache write-back): the chain, not the arithmetic, sets the time.  Here the
// workgroups stay resident (one or two per CU, the grid the occupancy
// guarantees) and meet at a grid barrier between steps.  Each step is the
// same per-tile body the standalone launches run (deep_tile, conv_deep.h;
// bn_bwd_body, conv_common.h): a resident workgroup loops over the step's
// tiles (virtual block ids, so the XCD-aware tile order still holds when the
// grid is a multiple of 8).
//
// Barrier: generation / count words (the last arriver resets the count and
// bumps the generation, so the words are reusable by the next launch without
// a reset node); agent-scope release before arriving (writes back this XCD's
// L2 so other XCDs see the step's outputs) and acquire after leaving
// (invalidates it).  The spin is bounded: a grid that is not co-resident
// times out, sets the abort word, and every workgroup leaves -- wrong
// results, reported through the barrier words, never a hang.
#include "conv_deep.h"

namespace {

struct ChainBar {
    unsigned count, gen, abort, pad;
};

constexpr unsigned long long CHAIN_TIMEOUT_TICKS = 200000000ull;   // 2 s at the 100 MHz wall clock

// false when the chain was aborted (time-out here or in another workgroup)
__device__ __forceinline__ bool chain_sync(ChainBar* bar, unsigned nb) {
    __shared__ unsigned ok;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned good = 1;
        const unsigned g = __hip_atomic_load(&bar->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned old = __hip_atomic_fetch_add(&bar->count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == nb - 1) {
            __hip_atomic_store(&bar->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&bar->gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const unsigned long long t0 = wall_clock64();
            while (__hip_atomic_load(&bar->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (__hip_atomic_load(&bar->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                    wall_clock64() - t0 > CHAIN_TIMEOUT_TICKS) {
                    __hip_atomic_store(&bar->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    good = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        ok = good;
    }
    __syncthreads();
    return ok != 0;
}

// deep configurations the chain instantiates (conv_deep.hip's table):
//   cfg 0: BN 32, whole 64x32 tile per wave, K / 4   (M <= 1024)
//   cfg 1: BN 64, whole 64x64 tile per wave, K / 4   (M <= 4096)
// One kernel per (dtype, cfg, NC): its conv steps differ only in tap size and
// prologue, so the kernel holds four tile bodies (a kernel holding every
// configuration spills: one register allocation over all of them).
template <int CFG> struct ChainCfg;
template <> struct ChainCfg<0> { static constexpr int BN = 32, NW = 4, WK = 4, DK = 8; };
template <> struct ChainCfg<1> { static constexpr int BN = 64, NW = 4, WK = 4, DK = 6; };

// tile bodies a chain kernel holds (bit set): the forward chain needs 1x1
// and 3x3 with the BN prologue and 1x1 without (the skip convs); the backward
// chain 1x1 and 3x3 without (data gradients) and the BN-backward apply.  One
// register allocation covers the bodies of a kernel, so each kernel holds
// only the three its direction uses.
enum { TB_1N = 1, TB_1P = 2, TB_3N = 4, TB_3P = 8, TB_BN = 16 };
constexpr int CHAIN_FWD = TB_1N | TB_1P | TB_3P;
constexpr int CHAIN_BWD = TB_1N | TB_3N | TB_BN;

__host__ __device__ constexpr int tile_body(int ks, bool pro) {
    return ks == 1 ? (pro ? TB_1P : TB_1N) : (pro ? TB_3P : TB_3N);
}

template <typename T, int CFG, int NC, int BODIES>
__global__ __launch_bounds__(256) void k_net_chain(const rnvp_net_step* __restrict__ steps, int n, ChainBar* bar,
                                                   float* grad_base) {
    using C = ChainCfg<CFG>;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    for (int i = 0; i < n; ++i) {
        const rnvp_net_step& st = steps[i];
        if (st.kind == RNVP_STEP_CONV) {
            const rnvp_conv_args& a = st.conv;
            const int body = tile_body(a.ks, a.pro_bn_relu != 0);
            for (int v = blockIdx.x; v < st.tiles; v += gridDim.x) {
                if ((BODIES & TB_1N) && body == TB_1N)
                    deep_tile<T, C::BN, 1, false, C::NW, C::WK, C::DK, NC>(a, st.shards, st.xa, st.xb, v, st.tiles, lds);
                if ((BODIES & TB_1P) && body == TB_1P)
                    deep_tile<T, C::BN, 1, true, C::NW, C::WK, C::DK, NC>(a, st.shards, st.xa, st.xb, v, st.tiles, lds);
                if ((BODIES & TB_3N) && body == TB_3N)
                    deep_tile<T, C::BN, 3, false, C::NW, C::WK, C::DK, NC>(a, st.shards, st.xa, st.xb, v, st.tiles, lds);
                if ((BODIES & TB_3P) && body == TB_3P)
                    deep_tile<T, C::BN, 3, true, C::NW, C::WK, C::DK, NC>(a, st.shards, st.xa, st.xb, v, st.tiles, lds);
                __syncthreads();
            }
        } else if (BODIES & TB_BN) {
            rnvp_bn_bwd_args b = st.bn;
            b.dgamma = st.dgamma_off >= 0 ? grad_base + st.dgamma_off : nullptr;
            b.dbeta = st.dbeta_off >= 0 ? grad_base + st.dbeta_off : nullptr;
            bn_bwd_body<T>(b, (double*)lds, blockIdx.x, gridDim.x);
        }
        if (i + 1 < n && !chain_sync(bar, gridDim.x)) return;
    }
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// the chain configuration of a conv step
int chain_cfg(const rnvp_conv_args& a) {
    const long long M = (long long)a.B * a.H * a.W;
    return M <= 1024 ? 0 : 1;
}

template <typename T, int CFG>
int prepare_conv(rnvp_net_step& st, size_t* lds) {
    using C = ChainCfg<CFG>;
    constexpr int KS = 4 * Mf<T>::CH;
    const rnvp_conv_args& a = st.conv;
    const long long M = (long long)a.B * a.H * a.W;
    if (a.n < C::BN / 2 || a.cs_in % (C::WK * KS) || a.cs_in > DEEP_MAX_CS) return RNVP_E_UNSUPPORTED;
    if (a.pro_bn_relu && a.pro.sums && a.pro.shards > 2) return RNVP_E_UNSUPPORTED;
    if (a.epi_relu_bn_bwd && a.epi.sums && a.epi.shards > 2) return RNVP_E_UNSUPPORTED;
    const int nc = a.cs_in / (C::WK * KS);
    if (nc != 1 && nc != 2 && nc != 4 && nc != 8) return RNVP_E_UNSUPPORTED;
    const size_t shm = deep_lds_bytes<T, C::BN, C::NW, C::WK>(a.cs_in, a.W, a.ks);
    if (shm > 160 * 1024) return RNVP_E_UNSUPPORTED;
    const long long gm = (M + DEEP_BM - 1) / DEEP_BM, gn = (a.n + C::BN - 1) / C::BN;
    st.cfg = CFG;
    st.nc = nc;
    st.shards = rnvp_stat_shards(M);
    st.tiles = (int)(gm * gn);
    xcd_blocks(&a, (int)gm, (int)gn, C::BN, sizeof(T), &st.xa, &st.xb);
    if (shm > *lds) *lds = shm;
    return RNVP_OK;
}

template <typename T>
int prepare_step(rnvp_net_step& st, size_t* lds) {
    if (st.kind == RNVP_STEP_CONV) {
        const rnvp_conv_args& a = st.conv;
        if (!a.x || !a.w || !a.y || a.dtype != st.conv.dtype) return RNVP_E_INVALID;
        if (a.ks != 1 && a.ks != 3) return RNVP_E_UNSUPPORTED;
        if (a.B <= 0 || a.H <= 0 || a.W <= 0 || a.n <= 0 || a.cin <= 0) return RNVP_E_INVALID;
        if ((a.cs_in & 7) || (a.cs_out & 7) || a.cs_in < a.cin || a.cs_out < a.n) return RNVP_E_INVALID;
        if ((a.kp & 63) || a.kp < a.ks * a.ks * a.cs_in) return RNVP_E_INVALID;
        if (!al16(a.x) || !al16(a.w)) return RNVP_E_INVALID;
        if (a.epi_relu_bn_bwd && !a.epi_x) return RNVP_E_INVALID;
        if ((long long)a.B * a.H * a.W > 4096) return RNVP_E_UNSUPPORTED;
        return chain_cfg(a) == 0 ? prepare_conv<T, 0>(st, lds) : prepare_conv<T, 1>(st, lds);
    }
    if (st.kind == RNVP_STEP_BN_BWD) {
        const rnvp_bn_bwd_args& b = st.bn;
        if (!b.g || !b.x || !b.dx || !b.sums || b.M <= 0 || b.C <= 0 || (b.cs & 7) || b.cs < b.C) return RNVP_E_INVALID;
        if (b.sum_shards < 1) return RNVP_E_INVALID;
        if (!al16(b.g) || !al16(b.x) || !al16(b.dx) || (b.residual && !al16(b.residual))) return RNVP_E_INVALID;
        const size_t shm = 68 * (size_t)b.cs;
        if (shm > 160 * 1024) return RNVP_E_UNSUPPORTED;
        st.cfg = st.nc = st.xa = st.xb = 0;
        st.shards = 1;
        st.tiles = 0;
        if (shm > *lds) *lds = shm;
        return RNVP_OK;
    }
    return RNVP_E_INVALID;
}

using ChainKernel = void (*)(const rnvp_net_step*, int, ChainBar*, float*);

template <typename T, int CFG, int BODIES>
ChainKernel chain_kernel_nc(int nc) {
    switch (nc) {
        case 1: return k_net_chain<T, CFG, 1, BODIES>;
        case 2: return k_net_chain<T, CFG, 2, BODIES>;
        case 4: return k_net_chain<T, CFG, 4, BODIES>;
        case 8: return k_net_chain<T, CFG, 8, BODIES>;
    }
    return nullptr;
}

template <typename T, int BODIES>
ChainKernel chain_kernel_cfg(int cfg, int nc) {
    return cfg == 0 ? chain_kernel_nc<T, 0, BODIES>(nc) : chain_kernel_nc<T, 1, BODIES>(nc);
}

// klass = cfg | nc << 4 | (0 forward bodies, 1 backward bodies) << 12
ChainKernel chain_kernel(int dtype, int klass) {
    const int cfg = klass & 15, nc = (klass >> 4) & 255, dir = klass >> 12;
    if (cfg > 1 || dir > 1) return nullptr;
    if (dtype == RNVP_F32)
        return dir ? chain_kernel_cfg<float, CHAIN_BWD>(cfg, nc) : chain_kernel_cfg<float, CHAIN_FWD>(cfg, nc);
    return dir ? chain_kernel_cfg<bf16_t, CHAIN_BWD>(cfg, nc) : chain_kernel_cfg<bf16_t, CHAIN_FWD>(cfg, nc);
}

// resident grid: one or two workgroups per CU (what the occupancy
// guarantees; RNVP_CHAIN_WGS_PER_CU caps it), a multiple of 8 so that the
// virtual block -> XCD mapping of the tiles holds
int chain_grid(ChainKernel k, size_t lds, int* grid) {
    static const int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess) return 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
        return n;
    }();
    static const int cap = [] { const char* e = getenv("RNVP_CHAIN_WGS_PER_CU"); return e ? atoi(e) : 2; }();
    int occ = 0;
    if (cus <= 0 || !k) return RNVP_E_UNSUPPORTED;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, 256, lds) != hipSuccess || occ < 1)
        return RNVP_E_UNSUPPORTED;
    const int per = occ < cap ? occ : (cap < 1 ? 1 : cap);
    *grid = cus * per;
    return RNVP_OK;
}

}  // namespace

// the chain's kernel class: every conv step must share (cfg, nc), and the
// tile bodies must all be forward ones or all backward ones
extern "C" int rnvp_net_chain_prepare(rnvp_net_step* steps, int n, int* klass, int* grid, int* lds_bytes) {
    if (!steps || n <= 0 || !klass || !grid || !lds_bytes) return RNVP_E_INVALID;
    const int dt = steps[0].kind == RNVP_STEP_CONV ? steps[0].conv.dtype : steps[0].bn.dtype;
    if (dt != RNVP_F32 && dt != RNVP_BF16) return RNVP_E_INVALID;
    size_t lds = 0;
    int cfg = -1, nc = -1, bodies = 0;
    for (int i = 0; i < n; ++i) {
        const int sdt = steps[i].kind == RNVP_STEP_CONV ? steps[i].conv.dtype : steps[i].bn.dtype;
        if (sdt != dt) return RNVP_E_INVALID;
        const int rc = dt == RNVP_F32 ? prepare_step<float>(steps[i], &lds) : prepare_step<bf16_t>(steps[i], &lds);
        if (rc != RNVP_OK) return rc;
        if (steps[i].kind == RNVP_STEP_CONV) {
            bodies |= tile_body(steps[i].conv.ks, steps[i].conv.pro_bn_relu != 0);
            if (cfg < 0) {
                cfg = steps[i].cfg;
                nc = steps[i].nc;
            } else if (steps[i].cfg != cfg || steps[i].nc != nc) {
                return RNVP_E_UNSUPPORTED;
            }
        } else {
            bodies |= TB_BN;
        }
    }
    int dir;
    if ((bodies & ~CHAIN_FWD) == 0) dir = 0;
    else if ((bodies & ~CHAIN_BWD) == 0) dir = 1;
    else return RNVP_E_UNSUPPORTED;
    if (cfg < 0) {
        cfg = 0;
        nc = 1;
    }
    for (int i = 0; i < n; ++i) {
        steps[i].cfg = cfg;
        steps[i].nc = nc;
    }
    const int k = cfg | (nc << 4) | (dir << 12);
    const int rc = chain_grid(chain_kernel(dt, k), lds, grid);
    if (rc != RNVP_OK) return rc;
    *klass = k;
    *lds_bytes = (int)lds;
    return RNVP_OK;
}

extern "C" int rnvp_net_chain(const rnvp_net_step* steps, int n, int dtype, int klass, int grid, int lds_bytes,
                              float* grad_base, void* barrier, void* stream) {
    if (!steps || n <= 0 || grid <= 0 || lds_bytes < 0 || lds_bytes > 160 * 1024 || !barrier) return RNVP_E_INVALID;
    if (dtype != RNVP_F32 && dtype != RNVP_BF16) return RNVP_E_INVALID;
    const ChainKernel k = chain_kernel(dtype, klass);
    if (!k) return RNVP_E_INVALID;
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds_bytes, (hipStream_t)stream, steps, n, (ChainBar*)barrier,
                       grad_base);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}
