// s/t ResNet convolutions on the MFMA matrix cores (gfx950).
//
// Implicit GEMM over NHWC activations: M = B*H*W pixels, N = output channels,
// K = ks*ks*cs_in (tap-major, channel-minor).  BatchNorm+ReLU of the operand is
// applied while staging the A tile (global -> registers -> LDS), bias /
// residual / skip accumulation and the next BatchNorm's batch statistics are
// fused into the epilogue.  The data gradient is the same kernel on the
// flipped/transposed weight image with a ReLU+BN-backward epilogue; the
// weight gradient reduces over pixels with both operands transposed through
// LDS by ds_read_b64_tr_b16.
//
// MFMA: bf16 -> v_mfma_f32_16x16x32_bf16 (fp32 accumulate);
//       f32  -> v_mfma_f32_16x16x4_f32 (exact fp32, parity mode).
// A 16-byte chunk holds 8 bf16 / 4 f32; one LDS tile row is 4 chunks = 64 B.
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

__device__ __forceinline__ int swz(int row, int c4) { return row * 4 + (c4 ^ ((row >> 2) & 3)); }

// ---------------------------------------------------------------------------
// forward / data-gradient conv
// ---------------------------------------------------------------------------
template <typename T, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void k_conv(rnvp_conv_args a) {
    constexpr int CH = Mf<T>::CH;
    constexpr int BK = 4 * CH;
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
    constexpr int A_PER = (BM * 4) / 256;
    constexpr int B_CHUNKS = BN * 4;
    static_assert(WM * WN == 4, "4 waves");
    static_assert(A_PER >= 1, "BM >= 64");

    __shared__ u32x4 As[BM * 4];
    __shared__ u32x4 Bs[BN * 4];
    __shared__ float red[WM * BN * 2];
    extern __shared__ float bnp[];   // [2 * cs_in] prologue scale / shift

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const long long M = (long long)a.B * a.H * a.W;
    const int N = a.n, cs = a.cs_in, ks = a.ks, pad = a.ks >> 1;
    const int K = ks * ks * cs;
    const long long m0 = (long long)blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const T* __restrict__ X = (const T*)a.x;
    const T* __restrict__ Wt = (const T*)a.w;

    if (a.pro_bn_relu) {
        for (int c = tid; c < cs; c += 256) {
            float sc = 0.f, sf = 0.f;
            if (c < a.cin) bn_affine(a.pro, a.cin, c, sc, sf);
            bnp[c] = sc;
            bnp[cs + c] = sf;
        }
    }

    // per-thread A rows (fixed over the K loop)
    const int c4 = tid & 3;
    long long arow_m[A_PER];
    int arow_y[A_PER], arow_x[A_PER];
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
        const int r = (tid + i * 256) >> 2;
        const long long m = m0 + r;
        arow_m[i] = m < M ? m : -1;
        const long long mm = m < M ? m : 0;
        arow_x[i] = (int)(mm % a.W);
        arow_y[i] = (int)((mm / a.W) % a.H);
    }

    floatx4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    __syncthreads();
    const int nk = (K + BK - 1) / BK;
    for (int kt = 0; kt < nk; ++kt) {
        // ---- stage A (implicit im2col + BN/ReLU prologue) ----
        const int k = kt * BK + c4 * CH;
        const int tap = k / cs, ci = k - tap * cs;
        const int dy = tap / ks - pad, dx = tap % ks - pad;
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const int r = (tid + i * 256) >> 2;
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            const int yy = arow_y[i] + dy, xx = arow_x[i] + dx;
            if (arow_m[i] >= 0 && k < K && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) {
                const long long off = (arow_m[i] + (long long)dy * a.W + dx) * cs + ci;
                v = *(const u32x4*)(X + off);
                if (a.pro_bn_relu) {
                    float f[CH];
                    unpack(v, f, T());
#pragma unroll
                    for (int j = 0; j < CH; ++j) f[j] = fmaxf(f[j] * bnp[ci + j] + bnp[cs + ci + j], 0.f);
                    v = pack(f, T());
                }
            }
            As[swz(r, c4)] = v;
        }
        // ---- stage B (packed weights [n][kp]) ----
        for (int q = tid; q < B_CHUNKS; q += 256) {
            const int nr = q >> 2, cc = q & 3;
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            if (n0 + nr < N) v = *(const u32x4*)(Wt + (long long)(n0 + nr) * a.kp + kt * BK + cc * CH);
            Bs[swz(nr, cc)] = v;
        }
        __syncthreads();
        // ---- MFMA ----
        const int g = lane >> 4, li = lane & 15;
        u32x4 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = As[swz(wm * WTM + i * 16 + li, g)];
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = Bs[swz(wn * WTN + j * 16 + li, g)];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) Mf<T>::step(af[i], bfr[j], acc[i][j]);
        __syncthreads();
    }

    // ---- epilogue ----
    T* __restrict__ Y = (T*)a.y;
    const T* __restrict__ R = (const T*)a.residual;
    const T* __restrict__ EX = (const T*)a.epi_x;
    const int cso = a.cs_out;
    const bool want_sums = a.out_sums || (a.epi_relu_bn_bwd && a.epi_sums);
    float s1[TN], s2[TN];
    float e_sc[TN], e_sf[TN], e_mean[TN], e_rstd[TN], bias[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WTN + j * 16 + (lane & 15);
        s1[j] = 0.f;
        s2[j] = 0.f;
        bias[j] = (a.bias && n < N) ? a.bias[n] : 0.f;
        e_sc[j] = e_sf[j] = e_mean[j] = 0.f;
        e_rstd[j] = 1.f;
        if (a.epi_relu_bn_bwd && n < N) bn_affine(a.epi, N, n, e_sc[j], e_sf[j], &e_mean[j], &e_rstd[j]);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const long long m = m0 + wm * WTM + i * 16 + (lane >> 4) * 4 + r;
            if (m >= M) continue;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = n0 + wn * WTN + j * 16 + (lane & 15);
                if (n >= cso) continue;
                const long long o = m * cso + n;
                float v = 0.f;
                if (n < N) {
                    v = acc[i][j][r] + bias[j];
                    if (R) v += ldv(&R[o]);
                    if (a.accumulate) v += ldv(&Y[o]);
                    if (a.epi_relu_bn_bwd) {
                        const float xv = ldv(&EX[o]);
                        if (xv * e_sc[j] + e_sf[j] <= 0.f) v = 0.f;
                        s1[j] += v;
                        s2[j] += v * (xv - e_mean[j]) * e_rstd[j];
                    } else {
                        s1[j] += v;
                        s2[j] += v * v;
                    }
                }
                stv(&Y[o], v);
            }
        }
    }
    if (want_sums) {
        double* sums = a.epi_relu_bn_bwd ? a.epi_sums : a.out_sums;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            s1[j] += __shfl_xor(s1[j], 16, 64);
            s1[j] += __shfl_xor(s1[j], 32, 64);
            s2[j] += __shfl_xor(s2[j], 16, 64);
            s2[j] += __shfl_xor(s2[j], 32, 64);
            if (lane < 16) {
                const int col = wn * WTN + j * 16 + lane;
                red[(wm * BN + col) * 2] = s1[j];
                red[(wm * BN + col) * 2 + 1] = s2[j];
            }
        }
        __syncthreads();
        for (int col = tid; col < BN; col += 256) {
            const int n = n0 + col;
            if (n >= N) continue;
            float t1 = 0.f, t2 = 0.f;
#pragma unroll
            for (int w = 0; w < WM; ++w) {
                t1 += red[(w * BN + col) * 2];
                t2 += red[(w * BN + col) * 2 + 1];
            }
            atomicAdd(&sums[n], (double)t1);
            atomicAdd(&sums[N + n], (double)t2);
        }
    }
}

template <typename T, int BM, int BN, int WM, int WN>
int launch_conv(const rnvp_conv_args* a, hipStream_t s) {
    const long long M = (long long)a->B * a->H * a->W;
    dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)((a->n + BN - 1) / BN));
    size_t shm = a->pro_bn_relu ? 2 * (size_t)a->cs_in * sizeof(float) : 0;
    k_conv<T, BM, BN, WM, WN><<<grid, 256, shm, s>>>(*a);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

template <typename T>
int dispatch_conv(const rnvp_conv_args* a, hipStream_t s) {
    const long long M = (long long)a->B * a->H * a->W;
    if (a->n <= 16) return launch_conv<T, 128, 16, 4, 1>(a, s);
    if (a->n <= 32) return launch_conv<T, 128, 32, 4, 1>(a, s);
    if (a->n <= 64) return launch_conv<T, 128, 64, 2, 2>(a, s);
    if (M >= 16384) return launch_conv<T, 128, 128, 2, 2>(a, s);
    return launch_conv<T, 64, 128, 1, 4>(a, s);
}

// ---------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------
// Output tile [64 co][64 k]; 4 waves as 2x2 of 32x32.  Per stage BKM pixels
// (32 bf16 / 16 f32) of dy (P) and act(x) (Q) are staged row-major [m][col];
// MFMA operands are columns, read transposed.
template <typename T>
__global__ __launch_bounds__(256) void k_wgrad(rnvp_wgrad_args a, long long m_per_block) {
    constexpr int CH = Mf<T>::CH;
    constexpr int BKM = (sizeof(T) == 2) ? 32 : 16;
    constexpr int CPR = 64 / CH;           // chunks per 64-element row
    constexpr int ROWB = 64 * sizeof(T) + 16;   // padded row bytes
    __shared__ __attribute__((aligned(16))) char Ps[BKM * ROWB];
    __shared__ __attribute__((aligned(16))) char Qs[BKM * ROWB];
    __shared__ float dbs[64];
    extern __shared__ float bnp[];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wc = wid >> 1, wk = wid & 1;
    const long long M = (long long)a.B * a.H * a.W;
    const int N = a.n, cs = a.cs_in, ks = a.ks, pad = ks >> 1;
    const int K = ks * ks * cs;
    const int co0 = blockIdx.x * 64, k0 = blockIdx.y * 64;
    const long long mb = (long long)blockIdx.z * m_per_block;
    const long long me = (mb + m_per_block < M) ? mb + m_per_block : M;
    const T* __restrict__ X = (const T*)a.x;
    const T* __restrict__ DY = (const T*)a.dy;
    const bool do_bias = a.dbias && blockIdx.y == 0;

    if (a.pro_bn_relu) {
        for (int c = tid; c < cs; c += 256) {
            float sc = 0.f, sf = 0.f;
            if (c < a.cin) bn_affine(a.pro, a.cin, c, sc, sf);
            bnp[c] = sc;
            bnp[cs + c] = sf;
        }
    }
    if (tid < 64) dbs[tid] = 0.f;
    // staging coordinates: row r (pixel), chunk c (column group)
    const int sr = tid / CPR, sc = tid % CPR;
    const int pk = k0 + sc * CH;                 // Q column
    const int ptap = pk / cs, pci = pk - ptap * cs;
    const int pdy = ptap / ks - pad, pdx = ptap % ks - pad;
    const int pco = co0 + sc * CH;               // P column

    floatx4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();

    for (long long mt = mb; mt < me; mt += BKM) {
        const long long m = mt + sr;
        // P: dy[m][co]
        {
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            if (m < me && pco < N) v = *(const u32x4*)(DY + m * a.cs_dy + pco);
            *(u32x4*)(Ps + sr * ROWB + sc * 16) = v;
        }
        // Q: act(x)[m + tap][ci]
        {
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            if (m < me && pk < K) {
                const int xx = (int)(m % a.W), yy = (int)((m / a.W) % a.H);
                const int y2 = yy + pdy, x2 = xx + pdx;
                if (y2 >= 0 && y2 < a.H && x2 >= 0 && x2 < a.W) {
                    v = *(const u32x4*)(X + (m + (long long)pdy * a.W + pdx) * cs + pci);
                    if (a.pro_bn_relu) {
                        float f[CH];
                        unpack(v, f, T());
#pragma unroll
                        for (int j = 0; j < CH; ++j) f[j] = fmaxf(f[j] * bnp[pci + j] + bnp[cs + pci + j], 0.f);
                        v = pack(f, T());
                    }
                }
            }
            *(u32x4*)(Qs + sr * ROWB + sc * 16) = v;
        }
        __syncthreads();
        if (do_bias && tid < 64) {
            float t = 0.f;
            for (int r = 0; r < BKM; ++r) t += ldv((const T*)(Ps + r * ROWB) + tid);
            dbs[tid] += t;
        }
        const int g = lane >> 4, li = lane & 15;
        if constexpr (sizeof(T) == 2) {
            const int q = li >> 2, p = li & 3;
            u32x4 af[2], bfr[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int c0 = wc * 32 + i * 16 + 4 * p;
                i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RNVP_LDS i16x4*)(Ps + (8 * g + q) * ROWB + c0 * 2));
                i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RNVP_LDS i16x4*)(Ps + (8 * g + 4 + q) * ROWB + c0 * 2));
                af[i].x = (uint32_t)(uint16_t)lo.x | ((uint32_t)(uint16_t)lo.y << 16);
                af[i].y = (uint32_t)(uint16_t)lo.z | ((uint32_t)(uint16_t)lo.w << 16);
                af[i].z = (uint32_t)(uint16_t)hi.x | ((uint32_t)(uint16_t)hi.y << 16);
                af[i].w = (uint32_t)(uint16_t)hi.z | ((uint32_t)(uint16_t)hi.w << 16);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int c0 = wk * 32 + j * 16 + 4 * p;
                i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RNVP_LDS i16x4*)(Qs + (8 * g + q) * ROWB + c0 * 2));
                i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RNVP_LDS i16x4*)(Qs + (8 * g + 4 + q) * ROWB + c0 * 2));
                bfr[j].x = (uint32_t)(uint16_t)lo.x | ((uint32_t)(uint16_t)lo.y << 16);
                bfr[j].y = (uint32_t)(uint16_t)lo.z | ((uint32_t)(uint16_t)lo.w << 16);
                bfr[j].z = (uint32_t)(uint16_t)hi.x | ((uint32_t)(uint16_t)hi.y << 16);
                bfr[j].w = (uint32_t)(uint16_t)hi.z | ((uint32_t)(uint16_t)hi.w << 16);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) Mf<bf16_t>::step(af[i], bfr[j], acc[i][j]);
        } else {
            u32x4 af[2], bfr[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const float* pcol = (const float*)Ps + wc * 32 + i * 16 + li;
                af[i].x = __float_as_uint(*(const float*)((const char*)pcol + (4 * g + 0) * ROWB));
                af[i].y = __float_as_uint(*(const float*)((const char*)pcol + (4 * g + 1) * ROWB));
                af[i].z = __float_as_uint(*(const float*)((const char*)pcol + (4 * g + 2) * ROWB));
                af[i].w = __float_as_uint(*(const float*)((const char*)pcol + (4 * g + 3) * ROWB));
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const float* qcol = (const float*)Qs + wk * 32 + j * 16 + li;
                bfr[j].x = __float_as_uint(*(const float*)((const char*)qcol + (4 * g + 0) * ROWB));
                bfr[j].y = __float_as_uint(*(const float*)((const char*)qcol + (4 * g + 1) * ROWB));
                bfr[j].z = __float_as_uint(*(const float*)((const char*)qcol + (4 * g + 2) * ROWB));
                bfr[j].w = __float_as_uint(*(const float*)((const char*)qcol + (4 * g + 3) * ROWB));
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) Mf<float>::step(af[i], bfr[j], acc[i][j]);
        }
        __syncthreads();
    }
    // D rows = co, cols = k
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = co0 + wc * 32 + i * 16 + (lane >> 4) * 4 + r;
                const int k = k0 + wk * 32 + j * 16 + (lane & 15);
                if (co < N && k < K) atomicAdd(&a.dw[(long long)co * a.kp + k], acc[i][j][r]);
            }
    if (do_bias && tid < 64 && co0 + tid < N) atomicAdd(&a.dbias[co0 + tid], dbs[tid]);
}

template <typename T>
int launch_wgrad(const rnvp_wgrad_args* a, hipStream_t s) {
    constexpr int BKM = (sizeof(T) == 2) ? 32 : 16;
    const long long M = (long long)a->B * a->H * a->W;
    const int K = a->ks * a->ks * a->cs_in;
    const int tco = (a->n + 63) / 64, tk = (K + 63) / 64;
    long long steps = (M + BKM - 1) / BKM;
    long long z = 1024 / (tco * tk);
    if (z < 1) z = 1;
    if (z > steps) z = steps;
    long long mpb = ((steps + z - 1) / z) * BKM;
    z = (M + mpb - 1) / mpb;
    dim3 grid((unsigned)tco, (unsigned)tk, (unsigned)z);
    size_t shm = a->pro_bn_relu ? 2 * (size_t)a->cs_in * sizeof(float) : 0;
    k_wgrad<T><<<grid, 256, shm, s>>>(*a, mpb);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

// ---------------------------------------------------------------------------
// BN backward apply
// ---------------------------------------------------------------------------
template <typename T>
__global__ void k_bn_bwd(rnvp_bn_bwd_args a) {
    constexpr int CH = Mf<T>::CH;
    extern __shared__ float p[];   // per channel: coef, k1, k2, mean, rstd
    const int cs = a.cs, C = a.C;
    const double cnt = (double)a.M;
    for (int c = threadIdx.x; c < cs; c += blockDim.x) {
        float coef = 0.f, k1 = 0.f, k2 = 0.f, mean = 0.f, rstd = 1.f;
        if (c < C) {
            float sc, sf;
            bn_affine(a.bn, C, c, sc, sf, &mean, &rstd);
            const float gam = a.bn.gamma ? a.bn.gamma[c] : 1.f;
            coef = gam * rstd;
            if (a.bn.sums) {   // train mode: batch statistics carry gradient
                k1 = (float)(a.sums[c] / cnt);
                k2 = (float)(a.sums[C + c] / cnt);
            }
            if (blockIdx.x == 0) {
                if (a.dbeta) a.dbeta[c] = (float)a.sums[c];
                if (a.dgamma) a.dgamma[c] = (float)a.sums[C + c];
            }
        }
        p[5 * c] = coef; p[5 * c + 1] = k1; p[5 * c + 2] = k2; p[5 * c + 3] = mean; p[5 * c + 4] = rstd;
    }
    __syncthreads();
    const T* G = (const T*)a.g;
    const T* X = (const T*)a.x;
    const T* R = (const T*)a.residual;
    T* DX = (T*)a.dx;
    const long long nch = a.M * (cs / CH);
    for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < nch; q += (long long)gridDim.x * blockDim.x) {
        const long long o = q * CH;
        const int c0 = (int)(o % cs);
        float g[CH], x[CH], d[CH];
        unpack(*(const u32x4*)(G + o), g, T());
        unpack(*(const u32x4*)(X + o), x, T());
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            const float* pp = p + 5 * (c0 + j);
            const float xh = (x[j] - pp[3]) * pp[4];
            d[j] = pp[0] * (g[j] - pp[1] - xh * pp[2]);
        }
        if (R) {
            float r[CH];
            unpack(*(const u32x4*)(R + o), r, T());
#pragma unroll
            for (int j = 0; j < CH; ++j) d[j] += r[j];
        }
        if (a.accumulate) {
            float r[CH];
            unpack(*(const u32x4*)(DX + o), r, T());
#pragma unroll
            for (int j = 0; j < CH; ++j) d[j] += r[j];
        }
        *(u32x4*)(DX + o) = pack(d, T());
    }
}

// ---------------------------------------------------------------------------
// weight normalisation
// ---------------------------------------------------------------------------
__device__ __forceinline__ int find_desc(const rnvp_wn_desc* d, int n, int row) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (d[mid].row0 <= row) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

template <typename T>
__global__ void k_wn_fwd(const rnvp_wn_desc* __restrict__ descs, int n_desc) {
    __shared__ double red[16];
    const int row = blockIdx.x;
    const rnvp_wn_desc d = descs[find_desc(descs, n_desc, row)];
    const int co = row - d.row0;
    const int kk = d.ks * d.ks, kr = d.cin * kk;
    const float* v = d.v + (long long)co * kr;
    double ss = 0;
    for (int i = threadIdx.x; i < kr; i += blockDim.x) ss += (double)v[i] * v[i];
    ss = block_sum(ss, red);
    const float nrm = (float)sqrt(ss);
    const float scale = d.g ? d.g[co] / nrm : 1.f;
    if (threadIdx.x == 0 && d.norm) d.norm[co] = nrm;
    T* wf = (T*)d.wf + (long long)co * d.kp_f;
    for (int k = threadIdx.x; k < d.kp_f; k += blockDim.x) {
        const int tap = k / d.cs_in, ci = k - tap * d.cs_in;
        float w = 0.f;
        if (tap < kk && ci < d.cin) w = scale * v[ci * kk + tap];
        stv(&wf[k], w);
    }
    if (d.wd) {
        T* wd = (T*)d.wd;
        for (int i = threadIdx.x; i < kr; i += blockDim.x) {
            const int ci = i / kk, tp = i - ci * kk;     // dgrad tap tp reads w tap kk-1-tp
            stv(&wd[(long long)ci * d.kp_d + tp * d.cs_out + co], scale * v[ci * kk + (kk - 1 - tp)]);
        }
    }
}

__global__ void k_wn_bwd(const rnvp_wn_desc* __restrict__ descs, int n_desc, float* gbase) {
    __shared__ double red[16];
    const int row = blockIdx.x;
    const rnvp_wn_desc d = descs[find_desc(descs, n_desc, row)];
    const int co = row - d.row0;
    const int kk = d.ks * d.ks, kr = d.cin * kk;
    const float* v = d.v + (long long)co * kr;
    const float* dw = d.dw + (long long)co * d.kp_f;
    double dot = 0;
    for (int i = threadIdx.x; i < kr; i += blockDim.x) {
        const int ci = i / kk, tap = i - ci * kk;
        dot += (double)dw[tap * d.cs_in + ci] * v[i];
    }
    dot = block_sum(dot, red);
    float* dv = gbase + d.dv_off + (long long)co * kr;
    if (d.g) {
        const float nrm = d.norm[co];
        const float gs = d.g[co] / nrm;
        const float proj = (float)(dot / ((double)nrm * nrm));
        for (int i = threadIdx.x; i < kr; i += blockDim.x) {
            const int ci = i / kk, tap = i - ci * kk;
            dv[i] = gs * (dw[tap * d.cs_in + ci] - proj * v[i]);
        }
        if (threadIdx.x == 0 && d.dg_off >= 0) gbase[d.dg_off + co] = (float)(dot / nrm);
    } else {
        for (int i = threadIdx.x; i < kr; i += blockDim.x) {
            const int ci = i / kk, tap = i - ci * kk;
            dv[i] = dw[tap * d.cs_in + ci];
        }
    }
}

inline bool al16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

}  // namespace

extern "C" int rnvp_conv2d(const rnvp_conv_args* a, void* stream) {
    if (!a || !a->x || !a->w || !a->y) return RNVP_E_INVALID;
    if (a->dtype != RNVP_F32 && a->dtype != RNVP_BF16) return RNVP_E_INVALID;
    if (a->ks != 1 && a->ks != 3) return RNVP_E_UNSUPPORTED;
    if (a->B < 0 || a->H <= 0 || a->W <= 0 || a->n <= 0 || a->cin <= 0) return RNVP_E_INVALID;
    if ((a->cs_in & 7) || (a->cs_out & 7) || a->cs_in < a->cin || a->cs_out < a->n) return RNVP_E_INVALID;
    if ((a->kp & 31) || a->kp < a->ks * a->ks * a->cs_in) return RNVP_E_INVALID;
    if (!al16(a->x) || !al16(a->w)) return RNVP_E_INVALID;
    if (a->epi_relu_bn_bwd && !a->epi_x) return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    hipStream_t s = (hipStream_t)stream;
    return a->dtype == RNVP_F32 ? dispatch_conv<float>(a, s) : dispatch_conv<bf16_t>(a, s);
}

extern "C" int rnvp_conv2d_wgrad(const rnvp_wgrad_args* a, void* stream) {
    if (!a || !a->x || !a->dy || !a->dw) return RNVP_E_INVALID;
    if (a->dtype != RNVP_F32 && a->dtype != RNVP_BF16) return RNVP_E_INVALID;
    if (a->ks != 1 && a->ks != 3) return RNVP_E_UNSUPPORTED;
    if (a->B < 0 || a->H <= 0 || a->W <= 0 || a->n <= 0 || a->cin <= 0) return RNVP_E_INVALID;
    if ((a->cs_in & 7) || (a->cs_dy & 7) || a->cs_in < a->cin || a->cs_dy < a->n) return RNVP_E_INVALID;
    if (a->kp < a->ks * a->ks * a->cs_in) return RNVP_E_INVALID;
    if (!al16(a->x) || !al16(a->dy)) return RNVP_E_INVALID;
    if (a->B == 0) return RNVP_OK;
    hipStream_t s = (hipStream_t)stream;
    return a->dtype == RNVP_F32 ? launch_wgrad<float>(a, s) : launch_wgrad<bf16_t>(a, s);
}

extern "C" int rnvp_bn_bwd_apply(const rnvp_bn_bwd_args* a, void* stream) {
    if (!a || !a->g || !a->x || !a->dx || !a->sums || a->M < 0 || a->C <= 0 || (a->cs & 7) || a->cs < a->C)
        return RNVP_E_INVALID;
    if (a->dtype != RNVP_F32 && a->dtype != RNVP_BF16) return RNVP_E_INVALID;
    if (!al16(a->g) || !al16(a->x) || !al16(a->dx) || (a->residual && !al16(a->residual))) return RNVP_E_INVALID;
    if (a->M == 0) return RNVP_OK;
    hipStream_t s = (hipStream_t)stream;
    const int CH = a->dtype == RNVP_F32 ? 4 : 8;
    const long long nch = a->M * (a->cs / CH);
    size_t shm = 5 * (size_t)a->cs * sizeof(float);
    if (a->dtype == RNVP_F32) k_bn_bwd<float><<<rnvp_grid(nch, 256, 2048), 256, shm, s>>>(*a);
    else k_bn_bwd<bf16_t><<<rnvp_grid(nch, 256, 2048), 256, shm, s>>>(*a);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_weight_norm_fwd(const rnvp_wn_desc* d, int n_desc, int total_rows, int dtype, void* stream) {
    if (!d || n_desc <= 0 || total_rows <= 0) return RNVP_E_INVALID;
    hipStream_t s = (hipStream_t)stream;
    if (dtype == RNVP_F32) k_wn_fwd<float><<<total_rows, 256, 0, s>>>(d, n_desc);
    else if (dtype == RNVP_BF16) k_wn_fwd<bf16_t><<<total_rows, 256, 0, s>>>(d, n_desc);
    else return RNVP_E_INVALID;
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_weight_norm_bwd(const rnvp_wn_desc* d, int n_desc, int total_rows, float* grad_base, void* stream) {
    if (!d || !grad_base || n_desc <= 0 || total_rows <= 0) return RNVP_E_INVALID;
    k_wn_bwd<<<total_rows, 256, 0, (hipStream_t)stream>>>(d, n_desc, grad_base);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}
