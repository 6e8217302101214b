// s/t ResNet convolutions on the MFMA matrix cores (gfx950).
//
// Implicit GEMM over NHWC activations: M = B*H*W pixels, N = output channels,
// K = ks*ks*cs_in (tap-major, channel-minor).  BatchNorm+ReLU of the operand is
// applied while staging the A tile (global -> registers -> LDS); bias /
// residual / skip accumulation and the next BatchNorm's batch statistics are
// fused into the epilogue.  The data gradient is the same kernel on the
// flipped/transposed weight image with a ReLU+BN-backward epilogue; the
// weight gradient reduces over pixels with both operands transposed through
// LDS by ds_read_b64_tr_b16.
//
// Pipeline: a stage is 128 B of K per tile row (64 bf16 / 32 f32), double
// buffered in LDS; the global loads of stage k+1 are issued before the MFMAs
// of stage k and land in registers, the BN/ReLU transform and the LDS store
// happen after the MFMAs -> one barrier per stage, load latency under compute.
// Small grids (deep scales: M = 1024..4096 pixels, K up to 4608) split K over
// workgroups into an fp32 workspace reduced by a second, epilogue kernel.
// BN statistics go to rnvp_stat_shards(M) shards (bounded atomic contention).
//
// MFMA: bf16 -> v_mfma_f32_16x16x32_bf16 (fp32 accumulate);
//       f32  -> v_mfma_f32_16x16x4_f32 (exact fp32, parity mode).
#include <math.h>
#include <stdlib.h>

#include "common.h"
#include "conv_common.h"

#ifndef RNVP_SHARD_PX
#define RNVP_SHARD_PX 8192
#endif
extern "C" int rnvp_stat_shards(long long M) {
    long long s = M / RNVP_SHARD_PX;
    int r = 1;
    while (r < 32 && r * 2 <= s) r *= 2;
    return r;
}

namespace {

// ---------------------------------------------------------------------------
// forward / data-gradient conv
// ---------------------------------------------------------------------------
template <typename T, int BM, int BN, int WM, int WN, bool PARTIAL>
__global__ __launch_bounds__(256) void k_conv(rnvp_conv_args a, int kt_per_split, int shards) {
    constexpr int CH = Mf<T>::CH;
    constexpr int BKS = 8 * CH;                        // K elements per stage
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
    constexpr int A_PER = (BM * 8) / 256;
    constexpr int B_CH = BN * 8;
    constexpr int B_PER = (B_CH + 255) / 256;
    static_assert(WM * WN == 4, "4 waves");
    static_assert(A_PER >= 1, "BM >= 32");

    __shared__ u32x4 As[2][BM * 8];
    __shared__ u32x4 Bs[2][BN * 8];
    __shared__ double red[WM * BN * 2];
    extern __shared__ double dsm[];   // tmp [2*max(cs,BN)] fp64 | bnp [2*cs] | etab [4*BN]

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const long long M = (long long)a.B * a.H * a.W;
    const int N = a.n, cs = a.cs_in, ks = a.ks, pad = a.ks >> 1;
    const int K = ks * ks * cs;
    const long long m0 = (long long)blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const T* __restrict__ X = (const T*)a.x;
    const T* __restrict__ Wt = (const T*)a.w;
    const bool pro = a.pro_bn_relu != 0;
    const bool epi_bn = a.epi_relu_bn_bwd != 0;

    double* tmp = dsm;
    float* bnp = (float*)(dsm + 2 * max(cs, BN));   // prologue scale [cs] | shift [cs]
    float* etab = bnp + 2 * cs;                      // epilogue scale | shift | mean | rstd [BN each]
    float* btab = etab + 4 * BN;                     // bias [BN]

    // per-thread A rows (fixed over K) and chunk column
    const int cA = tid & 7;
    long long arow_m[A_PER];
    int arow_y[A_PER], arow_x[A_PER];
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
        const int r = (tid + i * 256) >> 3;
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

    const int nk = (K + BKS - 1) / BKS;
    const int kt0 = blockIdx.z * kt_per_split;
    const int kt1 = min(nk, kt0 + kt_per_split);

    u32x4 ra[A_PER], rb[B_PER];
    unsigned amask = 0;
    int aci = 0;

    auto gload = [&](int kt) {
        const int k = kt * BKS + cA * CH;
        const int tap = k / cs, ci = k - tap * cs;
        const int dy = tap / ks - pad, dx = tap % ks - pad;
        aci = ci;
        amask = 0;
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const int yy = arow_y[i] + dy, xx = arow_x[i] + dx;
            ra[i] = u32x4{0u, 0u, 0u, 0u};
            if (arow_m[i] >= 0 && k < K && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) {
                ra[i] = *(const u32x4*)(X + (arow_m[i] + (long long)dy * a.W + dx) * cs + ci);
                amask |= 1u << i;
            }
        }
#pragma unroll
        for (int i = 0; i < B_PER; ++i) {
            const int q = tid + i * 256;
            rb[i] = u32x4{0u, 0u, 0u, 0u};
            if (q < B_CH) {
                const int nr = q >> 3, cc = q & 7;
                if (n0 + nr < N) rb[i] = *(const u32x4*)(Wt + (long long)(n0 + nr) * a.kp + kt * BKS + cc * CH);
            }
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const int r = (tid + i * 256) >> 3;
            u32x4 v = ra[i];
            if (pro) {
                if (amask & (1u << i)) {
                    float f[CH];
                    unpack(v, f, T());
#pragma unroll
                    for (int j = 0; j < CH; ++j) f[j] = fmaxf(f[j] * bnp[aci + j] + bnp[cs + aci + j], 0.f);
                    v = pack(f, T());
                } else {
                    v = u32x4{0u, 0u, 0u, 0u};
                }
            }
            As[buf][sw8(r, cA)] = v;
        }
#pragma unroll
        for (int i = 0; i < B_PER; ++i) {
            const int q = tid + i * 256;
            if (q < B_CH) Bs[buf][sw8(q >> 3, q & 7)] = rb[i];
        }
    };

    // the first stage's loads are in flight while the BN tables are built
    if (kt0 < kt1) gload(kt0);
    if (pro) block_bn_table(a.pro, a.cin, 0, cs, bnp, bnp + cs, nullptr, nullptr, tmp);
    if (epi_bn && !PARTIAL)
        block_bn_table(a.epi, N, n0, BN, etab, etab + BN, etab + 2 * BN, etab + 3 * BN, tmp);
    for (int c = tid; c < BN; c += 256) btab[c] = (a.bias && n0 + c < N) ? a.bias[n0 + c] : 0.f;
    __syncthreads();   // bnp / etab / btab ready
    if (kt0 < kt1) lstore(0);
    __syncthreads();
    const int g = lane >> 4, li = lane & 15;
    for (int kt = kt0; kt < kt1; ++kt) {
        const int cur = (kt - kt0) & 1;
        const bool more = kt + 1 < kt1;
        if (more) gload(kt + 1);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            u32x4 af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = As[cur][sw8(wm * WTM + i * 16 + li, s * 4 + g)];
#pragma unroll
            for (int j = 0; j < TN; ++j) bfr[j] = Bs[cur][sw8(wn * WTN + j * 16 + li, s * 4 + g)];
            // transposed product: acc[i][j] = D[n][m], a lane owns 4 channels of one pixel
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) Mf<T>::step(bfr[j], af[i], acc[i][j]);
        }
        if (more) lstore(cur ^ 1);
        __syncthreads();
    }

    const int cso = a.cs_out;
    if constexpr (PARTIAL) {
        float* ws = a.ws + (long long)blockIdx.z * M * cso;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const long long m = m0 + wm * WTM + i * 16 + li;
            if (m >= M) continue;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = n0 + wn * WTN + j * 16 + 4 * g;
                if (n < cso) *(floatx4*)(ws + m * cso + n) = acc[i][j];
            }
        }
        return;
    } else {
        // ---- fused epilogue (4 channels of one pixel per lane) ----
        const bool want_sums = a.out_sums || (a.epi_relu_bn_bwd && a.epi_sums);
        double s1[TN][4], s2[TN][4];
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) s1[j][r] = s2[j][r] = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const long long m = m0 + wm * WTM + i * 16 + li;
            if (m >= M) continue;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int col = wn * WTN + j * 16 + 4 * g;
                const int n = n0 + col;
                if (n >= cso) continue;
                epi4<T>(a, m * cso + n, acc[i][j], btab + col, epi_bn, etab + col, BN, s1[j], s2[j], N - n);
            }
        }
        if (want_sums) {
            double* sums = shard_ptr(a.epi_relu_bn_bwd ? a.epi_sums : a.out_sums, shards, N);
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double u1 = row_sum16(s1[j][r]), u2 = row_sum16(s2[j][r]);
                    if (li == 0) {
                        const int col = wn * WTN + j * 16 + 4 * g + r;
                        red[(wm * BN + col) * 2] = u1;
                        red[(wm * BN + col) * 2 + 1] = u2;
                    }
                }
            __syncthreads();
            for (int col = tid; col < BN; col += 256) {
                const int n = n0 + col;
                if (n >= N) continue;
                double t1 = 0.0, t2 = 0.0;
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
}

// split-K reduction + epilogue: block = [16 pixels][64 channels], thread =
// 4 channels of one pixel; partials ws[z][m][cs_out] (fp32).
constexpr int MAX_SPLITS = 8;

template <typename T>
__global__ __launch_bounds__(256) void k_splitk_epi(rnvp_conv_args a, int splits, int shards) {
    __shared__ double red[16][64][2];
    __shared__ double tmp[128];
    __shared__ float etab[4 * 64];
    __shared__ float btab[64];
    const int tid = threadIdx.x, c4 = tid & 15, row = tid >> 4;
    const long long M = (long long)a.B * a.H * a.W;
    const int N = a.n, cso = a.cs_out;
    const int n0 = blockIdx.y * 64;
    const long long m = (long long)blockIdx.x * 16 + row;
    const int col = 4 * c4, n = n0 + col;
    const bool epi_bn = a.epi_relu_bn_bwd != 0;
    // partial loads first (independent of the tables)
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
    const bool live = m < M && n < cso;
    if (live) {
        const float* wz = a.ws + m * cso + n;
#pragma unroll
        for (int z = 0; z < MAX_SPLITS; ++z)
            if (z < splits) acc += *(const floatx4*)(wz + (long long)z * M * cso);
    }
    if (epi_bn) block_bn_table(a.epi, N, n0, 64, etab, etab + 64, etab + 128, etab + 192, tmp);
    if (tid < 64) btab[tid] = (a.bias && n0 + tid < N) ? a.bias[n0 + tid] : 0.f;
    __syncthreads();
    double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
    if (live) epi4<T>(a, m * cso + n, acc, btab + col, epi_bn, etab + col, 64, s1, s2, N - n);
    const bool want_sums = a.out_sums || (epi_bn && a.epi_sums);
    if (want_sums) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            red[row][col + r][0] = s1[r];
            red[row][col + r][1] = s2[r];
        }
        __syncthreads();
        if (tid < 64 && n0 + tid < N) {
            double t1 = 0.0, t2 = 0.0;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                t1 += red[r][tid][0];
                t2 += red[r][tid][1];
            }
            double* sums = shard_ptr(epi_bn ? a.epi_sums : a.out_sums, shards, N);
            atomicAdd(&sums[n0 + tid], (double)t1);
            atomicAdd(&sums[N + n0 + tid], (double)t2);
        }
    }
}

// ---------------------------------------------------------------------------
// register-streaming conv for small channel counts (scales 1-2)
// ---------------------------------------------------------------------------
// For K <= ~600 and N <= 64 the whole packed weight matrix fits in LDS, and an
// MFMA B-fragment column (lane&15) x k-group (lane>>4) is exactly one pixel's
// 16-byte channel chunk: waves stream pixel fragments from global/L2 straight
// into registers (BN+ReLU applied there), no LDS round trip and no barrier in
// the main loop.  The product is formed transposed, D[n][m] = W[n][k] X[m][k]^T,
// so a lane ends up owning 4 consecutive output channels of one pixel: the
// epilogue reads/writes 8-byte (bf16) / 16-byte (f32) vectors.  Each wave owns
// 64-pixel tiles (4 MFMA column tiles); the next k-step's (or the next tile's)
// fragments are loaded before the current MFMAs, and the first tile's loads
// are issued before the BN-table / weight prologue.

template <typename T, int NT, int TW>
__global__ __launch_bounds__(256) void k_conv_stream(rnvp_conv_args a, int shards) {
    constexpr int CH = Mf<T>::CH;
    constexpr int KS = 4 * CH;             // K per step call (bf16: one 16x16x32, f32: four 16x16x4)
    constexpr int NC = 16 * NT;            // columns held by a wave
    extern __shared__ double dsm[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, li = lane & 15;
    const long long M = (long long)a.B * a.H * a.W;
    const int N = a.n, cs = a.cs_in, ks = a.ks, pad = ks >> 1;
    const int K = ks * ks * cs;
    const int nsteps = (K + KS - 1) / KS;
    const int kpl = lds_mfma_pitch(nsteps * KS, CH);   // LDS row pitch (conflict-free row reads)
    const bool pro = a.pro_bn_relu != 0;
    const bool epi_bn = a.epi_relu_bn_bwd != 0;
    const int ntmp = cs > NC ? cs : NC;

    double* tmp = dsm;
    float* bnp = (float*)(dsm + 2 * ntmp);
    float* etab = bnp + 2 * cs;            // scale | shift | mean | rstd [NC each]
    float* btab = etab + 4 * NC;           // bias [NC]
    double* red = (double*)(btab + NC);    // [4 waves][NC][2]
    T* Wl = (T*)(red + 4 * NC * 2);

    // pixel decode of this wave's tile (4 column tiles of 16 pixels); M < 2^31
    const int ntiles = (int)((M + 16 * TW - 1) / (16 * TW));
    const int tstride = gridDim.x * 4;
    int mrow[TW], yr[TW], xr[TW];
    auto decode = [&](int t) {
#pragma unroll
        for (int i = 0; i < TW; ++i) {
            const int m = t * (16 * TW) + i * 16 + li;
            mrow[i] = (t < ntiles && m < M) ? m : -1;
            const int mm = mrow[i] >= 0 ? m : 0;
            xr[i] = mm % a.W;
            yr[i] = (mm / a.W) % a.H;
        }
    };
    const T* __restrict__ X = (const T*)a.x;
    u32x4 ra[TW];
    unsigned msk = 0;
    int cur_ci = 0;
    auto load = [&](int s) {
        const int k = s * KS + g * CH;
        const int tap = k / cs, ci = k - tap * cs;
        const int dy = tap / ks - pad, dx = tap % ks - pad;
        cur_ci = ci;
        msk = 0;
#pragma unroll
        for (int i = 0; i < TW; ++i) {
            ra[i] = u32x4{0u, 0u, 0u, 0u};
            const int yy = yr[i] + dy, xx = xr[i] + dx;
            if (mrow[i] >= 0 && k < K && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) {
                ra[i] = *(const u32x4*)(X + (long long)(mrow[i] + dy * a.W + dx) * cs + ci);
                msk |= 1u << i;
            }
        }
    };
    // first tile's fragments in flight while the prologue runs
    int t = blockIdx.x * 4 + wid;
    decode(t);
    load(0);

    if (pro) block_bn_table(a.pro, a.cin, 0, cs, bnp, bnp + cs, nullptr, nullptr, tmp);
    if (epi_bn) block_bn_table(a.epi, N, 0, NC, etab, etab + NC, etab + 2 * NC, etab + 3 * NC, tmp);
    // weights -> LDS (rows >= N and k >= K zero), bias -> LDS
    {
        const T* Wg = (const T*)a.w;
        const int cpr = kpl / CH;
        for (int q = tid; q < NC * cpr; q += 256) {
            const int r = q / cpr, c = q - r * cpr;
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            if (r < N && c * CH < nsteps * KS) v = *(const u32x4*)(Wg + (long long)r * a.kp + c * CH);
            *(u32x4*)(Wl + r * kpl + c * CH) = v;
        }
        for (int n = tid; n < NC; n += 256) btab[n] = (a.bias && n < N) ? a.bias[n] : 0.f;
    }
    __syncthreads();

    const int cso = a.cs_out;
    double s1[NT][4], s2[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) s1[j][r] = s2[j][r] = 0.f;

    for (; t < ntiles; t += tstride) {
        floatx4 acc[TW][NT];
#pragma unroll
        for (int i = 0; i < TW; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

        for (int s = 0; s < nsteps; ++s) {
            u32x4 av[TW];
            const int ci = cur_ci;
            const unsigned mk = msk;
#pragma unroll
            for (int i = 0; i < TW; ++i) av[i] = ra[i];
            if (s + 1 < nsteps) load(s + 1);   // next k-step in flight under these MFMAs
            if (pro) {
#pragma unroll
                for (int i = 0; i < TW; ++i) {
                    if (mk & (1u << i)) {
                        float f[CH];
                        unpack(av[i], f, T());
#pragma unroll
                        for (int j = 0; j < CH; ++j) f[j] = fmaxf(f[j] * bnp[ci + j] + bnp[cs + ci + j], 0.f);
                        av[i] = pack(f, T());
                    }
                }
            }
            u32x4 wv[NT];
#pragma unroll
            for (int j = 0; j < NT; ++j) wv[j] = *(const u32x4*)(Wl + (j * 16 + li) * kpl + s * KS + g * CH);
#pragma unroll
            for (int i = 0; i < TW; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j) Mf<T>::step(wv[j], av[i], acc[i][j]);
        }
        // epilogue: lane owns channels j*16 + 4g .. +3 of pixel t*64 + i*16 + li
#pragma unroll
        for (int i = 0; i < TW; ++i) {
            const long long m = mrow[i];
            if (m < 0) continue;
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int n0 = j * 16 + 4 * g;
                if (n0 >= cso) continue;
                epi4<T>(a, m * cso + n0, acc[i][j], btab + n0, epi_bn, etab + n0, NC, s1[j], s2[j], N - n0);
            }
        }
        if (t + tstride < ntiles) {
            decode(t + tstride);
            load(0);
        }
    }
    const bool want_sums = a.out_sums || (epi_bn && a.epi_sums);
    if (want_sums) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double u1 = row_sum16(s1[j][r]), u2 = row_sum16(s2[j][r]);
                if (li == 0) {
                    red[(wid * NC + j * 16 + 4 * g + r) * 2] = u1;
                    red[(wid * NC + j * 16 + 4 * g + r) * 2 + 1] = u2;
                }
            }
        __syncthreads();
        double* sums = shard_ptr(epi_bn ? a.epi_sums : a.out_sums, shards, N);
        for (int n = tid; n < N; n += 256) {
            double t1 = 0.0, t2 = 0.0;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                t1 += red[(w * NC + n) * 2];
                t2 += red[(w * NC + n) * 2 + 1];
            }
            atomicAdd(&sums[n], (double)t1);
            atomicAdd(&sums[N + n], (double)t2);
        }
    }
}

template <typename T>
size_t stream_lds_bytes(const rnvp_conv_args* a, int nt) {
    constexpr int CH = Mf<T>::CH, KS = 4 * CH;
    const int K = a->ks * a->ks * a->cs_in;
    const int kpl = lds_mfma_pitch(((K + KS - 1) / KS) * KS, CH);
    const int nc = 16 * nt, ntmp = a->cs_in > nc ? a->cs_in : nc;
    return 16 * (size_t)ntmp + 8 * (size_t)a->cs_in + 16 * (size_t)nc + 4 * (size_t)nc + 64 * (size_t)nc +
           (size_t)nc * kpl * sizeof(T);
}

template <typename T, int NT, int TW>
int launch_stream(const rnvp_conv_args* a, hipStream_t s) {
    const long long M = (long long)a->B * a->H * a->W;
    const long long ntiles = (M + 16 * TW - 1) / (16 * TW);
    long long grid = (ntiles + 3) / 4;
    // two workgroups per CU, each walking several tiles: the next tile's
    // fragments load under the current tile's epilogue (measured: 10-20 %
    // faster than one tile per wave at scale 1, equal at scale 2)
    if (grid > 512) grid = 512;
    k_conv_stream<T, NT, TW><<<(unsigned)grid, 256, stream_lds_bytes<T>(a, NT), s>>>(*a, rnvp_stat_shards(M));
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

// pixels per wave (16 * TW), picked per pixel count from measurements
template <typename T, int NT>
int launch_stream_tw(const rnvp_conv_args* a, hipStream_t s) {
    const long long M = (long long)a->B * a->H * a->W;
    const int tw = M >= 4 * 64 * 1024 ? 4 : (M >= 32 * 1024 ? 2 : 1);   // measured: s1 4, s2 2
    if (tw == 1) return launch_stream<T, NT, 1>(a, s);
    if (tw == 2) return launch_stream<T, NT, 2>(a, s);
    return launch_stream<T, NT, 4>(a, s);
}

// true when the streaming kernel handles this conv (N <= 64, weights fit LDS)
template <typename T>
bool stream_ok(const rnvp_conv_args* a) {
    if (a->n > 64 || a->cs_in > 64) return false;
    const int nt = a->n <= 16 ? 1 : (a->n <= 32 ? 2 : 4);
    return stream_lds_bytes<T>(a, nt) <= 48 * 1024;
}

template <typename T>
int dispatch_stream(const rnvp_conv_args* a, hipStream_t s) {
    if (a->n <= 16) return launch_stream_tw<T, 1>(a, s);
    if (a->n <= 32) return launch_stream_tw<T, 2>(a, s);
    return launch_stream_tw<T, 4>(a, s);
}

template <typename T, int BM, int BN, int WM, int WN>
int launch_conv(const rnvp_conv_args* a, hipStream_t s) {
    constexpr int BKS = 8 * Mf<T>::CH;
    const long long M = (long long)a->B * a->H * a->W;
    const int K = a->ks * a->ks * a->cs_in;
    const int nk = (K + BKS - 1) / BKS;
    const long long gm = (M + BM - 1) / BM, gn = (a->n + BN - 1) / BN;
    const long long grid = gm * gn;
    const int shards = rnvp_stat_shards(M);
    const int cs = a->cs_in;
    const size_t shm = 16 * (size_t)(cs > BN ? cs : BN) + 8 * (size_t)cs + 20 * (size_t)BN;
    int splits = 1;
    if (a->ws && grid < 384 && nk >= 8) {
        splits = (int)((512 + grid - 1) / grid);
        if (splits > MAX_SPLITS) splits = MAX_SPLITS;
        if (splits > nk / 4) splits = nk / 4;
        while (splits > 1 && (long long)splits * M * a->cs_out > a->ws_elems) --splits;
    }
    if (splits > 1) {
        const int kps = (nk + splits - 1) / splits;
        splits = (nk + kps - 1) / kps;
        dim3 g1((unsigned)gm, (unsigned)gn, (unsigned)splits);
        k_conv<T, BM, BN, WM, WN, true><<<g1, 256, shm, s>>>(*a, kps, shards);
        RNVP_LAUNCH_CHECK();
        dim3 g2((unsigned)((M + 15) / 16), (unsigned)((a->cs_out + 63) / 64));
        k_splitk_epi<T><<<g2, 256, 0, s>>>(*a, splits, shards);
        RNVP_LAUNCH_CHECK();
        return RNVP_OK;
    }
    dim3 g1((unsigned)gm, (unsigned)gn, 1);
    k_conv<T, BM, BN, WM, WN, false><<<g1, 256, shm, s>>>(*a, nk, shards);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}


// prologue BN table capacity of the halo-tile kernel (channels)
constexpr int DK_MAX_CS = 1024;

// ---------------------------------------------------------------------------
// halo-tile conv (deep scales): act(x) staged ONCE per workgroup in LDS
// ---------------------------------------------------------------------------
// A workgroup owns 64 consecutive output pixels (NHW order: a band of image
// rows, or several whole 4x4 / 8x8 images) x BN channels.  Its input rows
// [m0 - hal, m0 + 64 + hal) (hal = one image row + 1 for 3x3) are loaded
// once, BN+ReLU'd once and kept in LDS; every tap of the 3x3 then reads its
// A fragments from LDS (tap validity from a per-pixel 9-bit mask, invalid
// taps read a zero row), so the transform and the activation traffic are not
// repeated per tap and per channel tile.  Only the weights stream from global
// memory (register ring, DK k-steps ahead; every load unconditional).  The
// four waves split K (interleaved k-steps) and their partial tiles are summed
// through LDS for the fused epilogue.

template <typename T, int BN>
size_t halo_lds_bytes(int cs, int W, int ks) {
    constexpr int BM = 64, TM = BM / 16;
    const int pad = ks / 2, hal = pad * (W + 1), R = BM + 2 * hal;
    const size_t head = 4 * (4 * BN + BN) + 8 * (2 * TM * BN);
    const size_t zrow = (size_t)halo_pitch<T>(cs) * sizeof(T);
    size_t act = (size_t)R * halo_pitch<T>(cs) * sizeof(T);
    const size_t red = 4 * (size_t)BM * (BN + 4) * 4;
    if (red > act) act = red;
    const size_t tail = 8 * 2 * (size_t)(cs > BN ? cs : BN) + 4 * 2 * (size_t)cs;
    return head + zrow + act + tail;
}

template <typename T, int BN, int KSZ, bool PRO, int DK, bool UNI>
__global__ __launch_bounds__(256) void k_conv_halo(rnvp_conv_args a, int shards) {
    constexpr int BM = 64;
    constexpr int CH = Mf<T>::CH, KS = 4 * CH;
    constexpr int TM = BM / 16, TN = BN / 16;
    constexpr int PAD = KSZ / 2;
    constexpr int RP = BN + 4;
    constexpr int FR = TM * TN / 4;
    extern __shared__ __attribute__((aligned(16))) char lds[];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, li = lane & 15;
    const int M = a.B * a.H * a.W, W = a.W, H = a.H;
    const int N = a.n, cs = a.cs_in;
    const int K = KSZ * KSZ * cs;
    const int nsteps = (K + KS - 1) / KS;
    const int gm = (M + BM - 1) / BM;
    const int nb = gridDim.x, b = blockIdx.x;
    const int q8 = nb / 8, r8 = nb % 8, xcd = b % 8;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
    const int nt = t / gm, mt = t - nt * gm;
    const int m0 = mt * BM, n0 = nt * BN;
    const T* __restrict__ X = (const T*)a.x;
    const T* __restrict__ Wt = (const T*)a.w;
    const bool epi_bn = a.epi_relu_bn_bwd != 0;

    const int hal = PAD * (W + 1);
    const int R = BM + 2 * hal;
    const int pitch = halo_pitch<T>(cs);
    float* etab = (float*)lds;                 // scale | shift | mean | rstd [BN each]
    float* btab = etab + 4 * BN;
    double* sred = (double*)(btab + BN);       // [TM][BN][2]
    T* zrow = (T*)(sred + TM * BN * 2);
    T* act = zrow + pitch;
    size_t act_bytes = (size_t)R * pitch * sizeof(T);
    if (act_bytes < 4 * (size_t)BM * RP * 4) act_bytes = 4 * (size_t)BM * RP * 4;
    double* tmp = (double*)((char*)act + act_bytes);
    float* bnp = (float*)(tmp + 2 * (cs > BN ? cs : BN));
    float* red = (float*)act;                  // [4][BM][RP], after the K loop

    // ---- prologue, ordered for the in-order vmcnt: staging loads, then the
    // BN-table loads (the table code waits for both), then the weight ring
    // (stays in flight across the transform and the barrier) ----
    const int cpr = cs / CH;
    const int total = R * cpr;
    const float rcpr = 1.0f / (float)cpr;
    constexpr int SB = 20;                     // chunks per thread per batch (deep scales: one batch)
    u32x4 sv[SB];
    auto stage_load = [&](int q0) {
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            const int q = q0 + u * 256 + tid;
            const int r = fdiv_small(q, rcpr), c = q - r * cpr;
            const int p = m0 - hal + r;
            const bool ok = (q < total) & (p >= 0) & (p < M);
            sv[u] = *(const u32x4*)(X + (ok ? (long long)p * cs + c * CH : 0));
        }
    };
    auto stage_store = [&](int q0) {
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            const int q = q0 + u * 256 + tid;
            if (q >= total) continue;
            const int r = fdiv_small(q, rcpr), c = q - r * cpr;
            const int p = m0 - hal + r;
            u32x4 w = sv[u];
            if (PRO) {
                float f[CH];
                unpack(w, f, T());
                const int c0 = c * CH;
#pragma unroll
                for (int e = 0; e < CH; e += 4) {
                    const floatx4 sc = *(const floatx4*)&bnp[c0 + e];
                    const floatx4 sh = *(const floatx4*)&bnp[cs + c0 + e];
                    f[e] = fmaxf(f[e] * sc.x + sh.x, 0.f);
                    f[e + 1] = fmaxf(f[e + 1] * sc.y + sh.y, 0.f);
                    f[e + 2] = fmaxf(f[e + 2] * sc.z + sh.z, 0.f);
                    f[e + 3] = fmaxf(f[e + 3] * sc.w + sh.w, 0.f);
                }
                w = pack(f, T());
            }
            const uint32_t keep = (p >= 0 && p < M) ? ~0u : 0u;
            *(u32x4*)(act + r * pitch + c * CH) = w & u32x4{keep, keep, keep, keep};
        }
    };
    BnTab<DK_MAX_CS / 256> ptab;
    BnTab<1> etb;
    if (PRO) tab_issue(a.pro, a.cin, 0, cs, ptab);
    if (epi_bn) tab_issue(a.epi, N, n0, BN, etb);
    stage_load(0);
    if (PRO) tab_finish(a.pro, a.cin, 0, cs, ptab, bnp, bnp + cs, nullptr, nullptr);
    if (epi_bn) tab_finish(a.epi, N, n0, BN, etb, etab, etab + BN, etab + 2 * BN, etab + 3 * BN);
    for (int c = tid; c < BN; c += 256) btab[c] = (a.bias && n0 + c < N) ? a.bias[n0 + c] : 0.f;
    for (int c = tid * CH; c < pitch; c += 256 * CH) *(u32x4*)(zrow + c) = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();

    const T* wrow[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        // rows >= N (clamped to row 0) only feed output columns that are never stored
        const int row = n0 + j * 16 + li;
        wrow[j] = Wt + (long long)(row < N ? row : 0) * a.kp + g * CH;
    }
    const int wv = __builtin_amdgcn_readfirstlane(wid);     // wave-uniform: step math on the SALU
    const int my_steps = wv < nsteps ? (nsteps - wv + 3) / 4 : 0;
    u32x4 rb[DK][TN];
    auto bload = [&](int u, int it) {
        const int st = wv + 4 * (it < my_steps ? it : 0);
#pragma unroll
        for (int j = 0; j < TN; ++j) rb[u][j] = *(const u32x4*)(wrow[j] + st * KS);
    };
#pragma unroll
    for (int u = 0; u < DK; ++u) bload(u, u);

    // ---- act(x) rows [m0 - hal, m0 + BM + hal) -> LDS (transformed once) ----
    stage_store(0);
    for (int q0 = 256 * SB; q0 < total; q0 += 256 * SB) {   // wide channels only
        stage_load(q0);
        stage_store(q0);
    }
    __syncthreads();

    // ---- per-lane pixel state ----
    int rowoff[TM];      // LDS element offset of the pixel's own row
    unsigned tvm[TM];    // bit tap set iff that tap of this output pixel is inside the image
    const float rW = 1.0f / (float)W, rH = 1.0f / (float)H;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int lp = i * 16 + li, m = m0 + lp;
        rowoff[i] = (lp + hal) * pitch;
        const int mm = m < M ? m : 0;
        const int row = fdiv_small(mm, rW);
        const int x = mm - row * W, y = row - fdiv_small(row, rH) * H;
        tvm[i] = tap_mask<KSZ>(x, y, W, H, m < M);
    }
    // K position of k = (wid + 4 it) * KS (+ g * CH for this lane).  UNI
    // (cs % KS == 0): a k-step never straddles a tap, so (tap, ci) are
    // wave-uniform (SALU) and the lane offset g * CH folds into rowoff.
    int tap, ci;
    {
        const int k = wv * KS + (UNI ? 0 : g * CH);
        tap = k / cs;
        ci = k - tap * cs;
    }
    if (UNI) {
#pragma unroll
        for (int i = 0; i < TM; ++i) rowoff[i] += g * CH;
    }
    const int zoff = UNI ? 0 : 0;

    floatx4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    for (int it0 = 0; it0 < my_steps; it0 += DK) {
#pragma unroll
        for (int u = 0; u < DK; ++u) {
            const int it = it0 + u;
            const int dy = tap / KSZ - PAD, dx = tap - (tap / KSZ) * KSZ - PAD;
            const int toff = (dy * W + dx) * pitch + ci;
            const bool live = it < my_steps;
            const int tsh = live ? tap : 31;   // bit 31 of tvm is never set
            u32x4 av[TM];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const bool ok = (tvm[i] >> tsh) & 1u;
                const T* src = ok ? act + rowoff[i] + toff : zrow + zoff;
                av[i] = *(const u32x4*)src;
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) Mf<T>::step(rb[u][j], av[i], acc[i][j]);
            // refill this ring slot after its MFMAs (no register copies)
            bload(u, it + DK);
            // advance (tap, ci) by 4 k-steps; cs >= 2 * 4 * KS / 2 -> at most two wraps
            ci += 4 * KS;
            if (ci >= cs) { ci -= cs; ++tap; }
            if (ci >= cs) { ci -= cs; ++tap; }
        }
    }

    // ---- reduce the four partial tiles through LDS (aliases the act tile) ----
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) *(floatx4*)&red[(wid * BM + i * 16 + li) * RP + j * 16 + 4 * g] = acc[i][j];
    __syncthreads();

    const int fi = wid % TM, fj0 = (wid / TM) * FR;
    const int m = m0 + fi * 16 + li;
    const int cso = a.cs_out;
    double s1[FR][4], s2[FR][4];
#pragma unroll
    for (int f = 0; f < FR; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) s1[f][r] = s2[f][r] = 0.f;
    if (m < M) {
#pragma unroll
        for (int f = 0; f < FR; ++f) {
            const int col = (fj0 + f) * 16 + 4 * g;
            const int n = n0 + col;
            if (n >= cso) continue;
            floatx4 v = *(const floatx4*)&red[(fi * 16 + li) * RP + col];
#pragma unroll
            for (int w = 1; w < 4; ++w) v += *(const floatx4*)&red[(w * BM + fi * 16 + li) * RP + col];
            epi4<T>(a, (long long)m * cso + n, v, btab + col, epi_bn, etab + col, BN, s1[f], s2[f], N - n);
        }
    }
    const bool want_sums = a.out_sums || (epi_bn && a.epi_sums);
    if (want_sums) {
#pragma unroll
        for (int f = 0; f < FR; ++f)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double u1 = row_sum16(s1[f][r]), u2 = row_sum16(s2[f][r]);
                if (li == 0) {
                    const int col = (fj0 + f) * 16 + 4 * g + r;
                    sred[(fi * BN + col) * 2] = u1;
                    sred[(fi * BN + col) * 2 + 1] = u2;
                }
            }
        __syncthreads();
        double* sums = (epi_bn ? a.epi_sums : a.out_sums) + (long long)(blockIdx.x % shards) * 2 * N;
        for (int col = tid; col < BN; col += 256) {
            const int n = n0 + col;
            if (n >= N) continue;
            double t1 = 0.0, t2 = 0.0;
#pragma unroll
            for (int w = 0; w < TM; ++w) {
                t1 += sred[(w * BN + col) * 2];
                t2 += sred[(w * BN + col) * 2 + 1];
            }
            atomicAdd(&sums[n], (double)t1);
            atomicAdd(&sums[N + n], (double)t2);
        }
    }
}

template <typename T, int BN, int KSZ>
int launch_halo(const rnvp_conv_args* a, hipStream_t s) {
    const long long M = (long long)a->B * a->H * a->W;
    const long long gm = (M + 63) / 64, gn = (a->n + BN - 1) / BN;
    const size_t shm = halo_lds_bytes<T, BN>(a->cs_in, a->W, KSZ);
    const int sh = rnvp_stat_shards(M);
    const bool uni = a->cs_in % (4 * Mf<T>::CH) == 0;
    constexpr int DK = BN >= 64 ? 6 : 8;      // weight k-steps in flight per wave
    const unsigned grid = (unsigned)(gm * gn);
    if (a->pro_bn_relu) {
        if (uni) k_conv_halo<T, BN, KSZ, true, DK, true><<<grid, 256, shm, s>>>(*a, sh);
        else k_conv_halo<T, BN, KSZ, true, DK, false><<<grid, 256, shm, s>>>(*a, sh);
    } else {
        if (uni) k_conv_halo<T, BN, KSZ, false, DK, true><<<grid, 256, shm, s>>>(*a, sh);
        else k_conv_halo<T, BN, KSZ, false, DK, false><<<grid, 256, shm, s>>>(*a, sh);
    }
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

// deep scales: few pixels, wide channels, the halo tile fits LDS
template <typename T>
bool halo_ok(const rnvp_conv_args* a) {
    const long long M = (long long)a->B * a->H * a->W;
    // measured against the LDS-tiled kernel: the halo tile wins at M <= 1024
    // (every shape) and for 3x3 at M <= 4096, loses above
    if (M > 4096 || (M > 1024 && a->ks != 3)) return false;
    if (a->cs_in < 64 || a->cs_in > DK_MAX_CS || a->n <= 16) return false;
    if (a->pro_bn_relu && a->pro.sums && a->pro.shards > 2) return false;
    if (a->epi_relu_bn_bwd && a->epi.sums && a->epi.shards > 2) return false;
    return halo_lds_bytes<T, 64>(a->cs_in, a->W, a->ks) <= 150 * 1024;
}

template <typename T>
int dispatch_halo(const rnvp_conv_args* a, hipStream_t s) {
    const long long M = (long long)a->B * a->H * a->W;
    // 64-channel tiles when that still gives >= 256 workgroups
    const bool wide = ((M + 63) / 64) * ((a->n + 63) / 64) >= 256;
    if (a->ks == 3) return wide ? launch_halo<T, 64, 3>(a, s) : launch_halo<T, 32, 3>(a, s);
    return wide ? launch_halo<T, 64, 1>(a, s) : launch_halo<T, 32, 1>(a, s);
}

// ---------------------------------------------------------------------------
// Band kernel for the wide scales (cs_in <= 64, N <= 64; M = 32k .. 262k
// pixels).  A workgroup owns a band of BM = 256 consecutive pixels (whole
// image rows at 64x64 / 32x32); the band plus its halo (pad*(W+1) pixels on
// either side) is read from HBM once, BN+ReLU applied, into LDS, next to the
// packed weights.  Each wave owns 64 pixels x all N channels and walks the
// whole K from LDS: no split-K, no partial-tile reduction, and no per-tap
// re-fetch of pixels (k_conv_stream re-reads every tap of every pixel from
// L1/L2 with one k-step in flight).  Transposed product, epilogue as in
// k_conv_stream (lane = 4 consecutive channels of one pixel).
template <typename T>
size_t band_lds_bytes(int cs, int n, int W, int ks) {
    constexpr int CH = Mf<T>::CH, KS = 4 * CH, BM = 256;
    const int nc = n <= 16 ? 16 : (n <= 32 ? 32 : 64);
    const int K = ks * ks * cs;
    const int kpl = lds_mfma_pitch(((K + KS - 1) / KS) * KS, CH);
    const int R = BM + 2 * (ks / 2) * (W + 1);
    const int ntmp = cs > nc ? cs : nc;
    return 16 * (size_t)ntmp + 8 * (size_t)cs + 20 * (size_t)nc + 64 * (size_t)nc +
           ((size_t)nc * kpl + (size_t)(R + 1) * lds_mfma_pitch(cs, CH)) * sizeof(T);
}

// NH = 2: eight waves, wave pairs split the output channels (each wave 64
// pixels x NT/2 channel tiles): two waves per SIMD when the band and the
// weights hold the CU to one workgroup (64-channel 3x3 at 32x32)
template <typename T, int NT, int KSZ, bool PRO, int NH>
__global__ __launch_bounds__(256 * NH) void k_conv_band(rnvp_conv_args a, int shards) {
    constexpr int CH = Mf<T>::CH, KS = 4 * CH;
    constexpr int NC = 16 * NT;
    constexpr int TM = 4, BM = 64 * TM;        // 4 waves x 64 pixels
    constexpr int PAD = KSZ / 2;
    constexpr int SB = 12 / NH;                // staged 16-B chunks per thread per batch
    constexpr int NTH = 256 * NH, NTW = NT / NH;
    static_assert(NT % NH == 0, "channel tiles split evenly");
    extern __shared__ double dsm[];
    const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, li = lane & 15;
    const int wid = (tid >> 6) & 3, hf = tid >> 8;   // pixel group, channel half
    const int M = a.B * a.H * a.W, W = a.W, H = a.H;
    const int N = a.n, cs = a.cs_in;
    const int K = KSZ * KSZ * cs;
    const int nsteps = (K + KS - 1) / KS;
    const int kpl = lds_mfma_pitch(nsteps * KS, CH);   // weight row pitch (conflict-free)
    const bool epi_bn = a.epi_relu_bn_bwd != 0;
    const int ntmp = cs > NC ? cs : NC;
    const int hal = PAD * (W + 1), R = BM + 2 * hal;
    const int pitch = lds_mfma_pitch(cs, CH);  // band row pitch (conflict-free reads)

    double* tmp = dsm;
    float* bnp = (float*)(dsm + 2 * ntmp);     // scale | shift [cs each]
    float* etab = bnp + 2 * cs;                // scale | shift | mean | rstd [NC each]
    float* btab = etab + 4 * NC;               // bias [NC]
    double* red = (double*)(btab + NC);        // [4 waves][NC][2]
    T* Wl = (T*)(red + 8 * NC);                // [NC][kpl]
    T* zrow = Wl + NC * kpl;                   // [pitch] zeros
    T* act = zrow + pitch;                     // [R][pitch]

    // consecutive bands (which share halo rows) on one XCD (bijective remap)
    const int nb = gridDim.x, b = blockIdx.x;
    const int q8 = nb / 8, r8 = nb % 8, xcd = b % 8;
    const int m0 = ((xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8) * BM;

    // ---- band + halo loads first: in flight under the table / weight prologue
    const T* __restrict__ X = (const T*)a.x;
    // cs <= 64 channels: a row is cpr <= 16 chunks (bf16: <= 8) and 256 % cpr
    // == 0 (launcher), so a thread's chunk column is the same in every staged
    // row: its BN coefficients go to registers once (no per-chunk LDS table
    // reads or divisions), its rows advance by 256 / cpr per slot, and no
    // load is issued past the band
    const int cpr = cs / CH;
    const int cfix = tid % cpr, rbase = tid / cpr, rstep = NTH / cpr;
    u32x4 sv[SB];
    auto stage_load = [&](int r0) {
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            if (r0 + u * rstep >= R) break;
            const int r = r0 + rbase + u * rstep;
            const int p = m0 - hal + r;
            const bool ok = (r < R) & (p >= 0) & (p < M);
            sv[u] = *(const u32x4*)(X + (ok ? (long long)p * cs + cfix * CH : 0));
        }
    };
    float scv[CH], shv[CH];
    auto stage_store = [&](int r0) {
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            const int r = r0 + rbase + u * rstep;
            if (r >= R) continue;
            const int p = m0 - hal + r;
            u32x4 w = sv[u];
            if (PRO) {
                if constexpr (sizeof(T) == 2) {
                    w = bn_relu_bf16x8(w, scv, shv);
                } else {
                    float f[CH];
                    unpack(w, f, T());
#pragma unroll
                    for (int e = 0; e < CH; ++e) f[e] = fmaxf(f[e] * scv[e] + shv[e], 0.f);
                    w = pack(f, T());
                }
            }
            const uint32_t keep = (p >= 0 && p < M) ? ~0u : 0u;
            *(u32x4*)(act + r * pitch + cfix * CH) = w & u32x4{keep, keep, keep, keep};
        }
    };
    stage_load(0);

    // ---- BN tables, packed weights (rows >= N and k >= K zero) and bias -> LDS
    if (PRO) block_bn_table(a.pro, a.cin, 0, cs, bnp, bnp + cs, nullptr, nullptr, tmp);
    if (epi_bn) block_bn_table(a.epi, N, 0, NC, etab, etab + NC, etab + 2 * NC, etab + 3 * NC, tmp);
    {
        const T* Wg = (const T*)a.w;
        const int wcpr = kpl / CH, wtot = NC * wcpr, kv = nsteps * KS;
        const float rw = 1.0f / (float)wcpr;
        for (int q0 = 0; q0 < wtot; q0 += 4 * NTH) {
            u32x4 v[4];
            unsigned okm = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = q0 + u * NTH + tid;
                const int r = fdiv_small(q, rw), c = q - r * wcpr;
                const bool ok = (q < wtot) & (r < N) & (c * CH < kv);
                v[u] = *(const u32x4*)(Wg + (ok ? (long long)r * a.kp + c * CH : 0));
                okm |= (unsigned)ok << u;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = q0 + u * NTH + tid;
                if (q < wtot) {
                    const int r = fdiv_small(q, rw), c = q - r * wcpr;
                    const uint32_t keep = ((okm >> u) & 1u) ? ~0u : 0u;
                    *(u32x4*)(Wl + r * kpl + c * CH) = v[u] & u32x4{keep, keep, keep, keep};
                }
            }
        }
        for (int n = tid; n < NC; n += NTH) btab[n] = (a.bias && n < N) ? a.bias[n] : 0.f;
        for (int c = tid * CH; c < pitch; c += NTH * CH) *(u32x4*)(zrow + c) = u32x4{0u, 0u, 0u, 0u};
    }
    __syncthreads();
    if (PRO) {
#pragma unroll
        for (int e = 0; e < CH; ++e) {
            scv[e] = bnp[cfix * CH + e];
            shv[e] = bnp[cs + cfix * CH + e];
        }
    }

    // ---- act(x) band -> LDS (transformed once) ----
    stage_store(0);
    for (int r0 = rstep * SB; r0 < R; r0 += rstep * SB) {
        stage_load(r0);
        stage_store(r0);
    }
    __syncthreads();

    // ---- per-lane pixel state ----
    int rowoff[TM];      // LDS element offset of the pixel's own band row
    unsigned tvm[TM];    // bit tap set iff that tap of this output pixel is inside the image
    const float rW = 1.0f / (float)W, rH = 1.0f / (float)H;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int lp = wid * 64 + i * 16 + li, m = m0 + lp;
        rowoff[i] = (lp + hal) * pitch;
        const int mm = m < M ? m : 0;
        const int row = fdiv_small(mm, rW);
        const int x = mm - row * W, y = row - fdiv_small(row, rH) * H;
        tvm[i] = tap_mask<KSZ>(x, y, W, H, m < M);
    }

    floatx4 acc[TM][NTW];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    // lane's K position k = s*KS + g*CH -> (tap, ci); a 16-B chunk never
    // straddles a tap (cs % CH == 0); KS / cs <= 4 wraps per step
    int tap = 0, ci = g * CH;
#pragma unroll
    for (int w = 0; w < 4; ++w)
        if (ci >= cs) { ci -= cs; ++tap; }
    const T* wl = Wl + (hf * NTW * 16 + li) * kpl + g * CH;
    for (int st = 0; st < nsteps; ++st) {
        const int ty = tap / KSZ;
        const int toff = ((ty - PAD) * W + (tap - ty * KSZ - PAD)) * pitch + ci;
        const int tsh = tap < KSZ * KSZ ? tap : 31;   // bit 31 of tvm is never set
        u32x4 wv[NTW], av[TM];
#pragma unroll
        for (int j = 0; j < NTW; ++j) wv[j] = *(const u32x4*)(wl + j * 16 * kpl + st * KS);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const bool ok = (tvm[i] >> tsh) & 1u;
            av[i] = *(const u32x4*)(ok ? act + rowoff[i] + toff : zrow);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < NTW; ++j) Mf<T>::step(wv[j], av[i], acc[i][j]);
        ci += KS;
#pragma unroll
        for (int w = 0; w < 4; ++w)
            if (ci >= cs) { ci -= cs; ++tap; }
    }

    // ---- epilogue: lane owns channels j*16 + 4g .. +3 of its pixels ----
    const int cso = a.cs_out;
    double s1[NTW][4], s2[NTW][4];
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) s1[j][r] = s2[j][r] = 0.0;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + wid * 64 + i * 16 + li;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const int n0 = (hf * NTW + j) * 16 + 4 * g;
            if (n0 >= cso) continue;
            epi4<T>(a, (long long)m * cso + n0, acc[i][j], btab + n0, epi_bn, etab + n0, NC, s1[j], s2[j], N - n0);
        }
    }
    const bool want_sums = a.out_sums || (epi_bn && a.epi_sums);
    if (want_sums) {
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double u1 = row_sum16(s1[j][r]), u2 = row_sum16(s2[j][r]);
                const int col = (hf * NTW + j) * 16 + 4 * g + r;
                if (li == 0) {
                    red[(wid * NC + col) * 2] = u1;
                    red[(wid * NC + col) * 2 + 1] = u2;
                }
            }
        __syncthreads();
        double* sums = shard_ptr(epi_bn ? a.epi_sums : a.out_sums, shards, N);
        for (int n = tid; n < N; n += NTH) {
            double t1 = 0.0, t2 = 0.0;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                t1 += red[(w * NC + n) * 2];
                t2 += red[(w * NC + n) * 2 + 1];
            }
            atomicAdd(&sums[n], t1);
            atomicAdd(&sums[N + n], t2);
        }
    }
}

template <typename T, int NT, int KSZ>
int launch_band(const rnvp_conv_args* a, hipStream_t s) {
    const long long M = (long long)a->B * a->H * a->W;
    const unsigned grid = (unsigned)((M + 255) / 256);
    const size_t shm = band_lds_bytes<T>(a->cs_in, a->n, a->W, KSZ);
    const int sh = rnvp_stat_shards(M);
    // eight waves for the 3x3 (64 channels: 23.76 vs 24.03 ms per step; 32
    // channels: 23.71 vs 23.79)
    if constexpr ((NT == 4 || NT == 2) && KSZ == 3) {
        if (a->pro_bn_relu) k_conv_band<T, NT, KSZ, true, 2><<<grid, 512, shm, s>>>(*a, sh);
        else k_conv_band<T, NT, KSZ, false, 2><<<grid, 512, shm, s>>>(*a, sh);
        RNVP_LAUNCH_CHECK();
        return RNVP_OK;
    }
    if (a->pro_bn_relu) k_conv_band<T, NT, KSZ, true, 1><<<grid, 256, shm, s>>>(*a, sh);
    else k_conv_band<T, NT, KSZ, false, 1><<<grid, 256, shm, s>>>(*a, sh);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

// wide scales: few channels, many pixels (fp32 reciprocal pixel decode: M < 2^21)
template <typename T>
bool band_ok(const rnvp_conv_args* a) {
    const long long M = (long long)a->B * a->H * a->W;
    // 3x3 only: for 1x1 the streaming kernel (no halo to share) is faster
    if (a->n > 64 || a->cs_in > 64 || a->ks != 3) return false;
    if (256 % (a->cs_in / Mf<T>::CH) != 0) return false;   // fixed chunk column per thread
    if (M < 32768 || M >= (1ll << 21)) return false;
    return band_lds_bytes<T>(a->cs_in, a->n, a->W, a->ks) <= 150 * 1024;
}

template <typename T>
int dispatch_band(const rnvp_conv_args* a, hipStream_t s) {
    if (a->ks == 3) {
        if (a->n <= 16) return launch_band<T, 1, 3>(a, s);
        if (a->n <= 32) return launch_band<T, 2, 3>(a, s);
        return launch_band<T, 4, 3>(a, s);
    }
    if (a->n <= 16) return launch_band<T, 1, 1>(a, s);
    if (a->n <= 32) return launch_band<T, 2, 1>(a, s);
    return launch_band<T, 4, 1>(a, s);
}

template <typename T>
int dispatch_conv(const rnvp_conv_args* a, hipStream_t s) {
    const long long M = (long long)a->B * a->H * a->W;
    // forced deep-scale configuration (A/B and parity tests): no fallback
    if (a->variant >= RNVP_VARIANT_DEEP0) return rnvp_deep_launch(a, s, a->variant - RNVP_VARIANT_DEEP0);
    if (a->variant == 0 || a->variant == RNVP_VARIANT_DEEP) {
        const int cfg = rnvp_deep_auto_cfg(a);
        if (cfg >= 0) {
            const int r = rnvp_deep_launch(a, s, cfg);
            if (r != RNVP_E_UNSUPPORTED) return r;
        }
    }
    const bool tuned = a->variant != 1;
    // bf16 1x1 convs of the wide scales: the register-pipelined stream kernel (conv_s1.hip)
    if (tuned && a->dtype == RNVP_BF16 && a->ks == 1) {
        const int r = rnvp_conv_s1_launch(a, s);
        if (r != RNVP_E_UNSUPPORTED) return r;
    }
    if (tuned && band_ok<T>(a)) {
        // the persistent band kernel (conv_band.hip) where it applies
        const int r = rnvp_conv_band2_launch(a, s);
        if (r != RNVP_E_UNSUPPORTED) return r;
        return dispatch_band<T>(a, s);
    }
    if (stream_ok<T>(a)) return dispatch_stream<T>(a, s);
    if (tuned && halo_ok<T>(a)) return dispatch_halo<T>(a, s);
    // largest tile that still gives >= 512 workgroups (2 per CU); small grids
    // fall through to 64x64 tiles and split K
    if (a->n <= 16) return launch_conv<T, 128, 16, 4, 1>(a, s);
    if (a->n <= 32) return M >= 512 * 128 ? launch_conv<T, 128, 32, 4, 1>(a, s) : launch_conv<T, 64, 32, 4, 1>(a, s);
    if (a->n <= 64) return M >= 512 * 128 ? launch_conv<T, 128, 64, 2, 2>(a, s) : launch_conv<T, 64, 64, 2, 2>(a, s);
    const long long g128 = ((M + 127) / 128) * ((a->n + 127) / 128);
    if (g128 >= 512) return launch_conv<T, 128, 128, 2, 2>(a, s);
    return launch_conv<T, 64, 64, 2, 2>(a, s);
}

// ---------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------
// Output tile [64 co][64 k]; 4 waves as 2x2 of 32x32.  A stage is STG pixels
// (64 bf16 / 32 f32) of dy (P) and act(x) (Q), staged row-major [m][col] in
// double-buffered LDS; MFMA operands are columns, read transposed
// (ds_read_b64_tr_b16 for bf16).
struct WgView {
    const void* x; const void* dy; rnvp_bn_src pro;
    int H, W, ks, cs_in, cin, cs_dy, n, kp, pro_bn_relu;
};

// one [TC co] x [TC k] tile (TC = 64 or 128) over pixels [mb, me): result to out[co*kp + k]
// (fp32 atomics or plain stores) and, when bias_out, the bias sums of the
// tile's co columns to bias_out[co] (atomic or plain).
template <typename T, int TC>
__device__ __forceinline__ void wgrad_tile(const WgView& a, int co0, int k0, long long mb, long long me,
                                           long long M, float* out, bool atomic, float* bias_out, bool bias_atomic) {
    constexpr int CH = Mf<T>::CH;
    constexpr int STG = (sizeof(T) == 2) ? 64 : 32;   // pixels per stage (two MFMA K-steps)
    constexpr int CPR = TC / CH;                      // chunks per TC-column row
    constexpr int ROWB = TC * sizeof(T) + 16;         // padded row bytes
    constexpr int PER = STG * CPR / 256;              // chunks per thread per operand (2 / 4)
    constexpr int D = TC == 64 ? 4 : 2;               // stages of global loads in flight per thread
    constexpr int WT = TC / 2, FT = WT / 16;          // per-wave tile (2 x 2 waves), its 16x16 fragments
    __shared__ __attribute__((aligned(16))) char Ps[2][STG * ROWB];
    __shared__ __attribute__((aligned(16))) char Qs[2][STG * ROWB];
    __shared__ float dbs[TC];
    extern __shared__ double dsm[];   // tmp [2*cs] fp64 | bnp scale [cs] | shift [cs]

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wc = wid >> 1, wk = wid & 1;
    const int N = a.n, cs = a.cs_in, ks = a.ks, pad = ks >> 1;
    const int K = ks * ks * cs;
    const int H = a.H, W = a.W;
    const T* __restrict__ X = (const T*)a.x;
    const T* __restrict__ DY = (const T*)a.dy;
    const bool do_bias = bias_out != nullptr;
    const bool pro = a.pro_bn_relu != 0;

    float* bnp = (float*)(dsm + 2 * cs);
    if (tid < TC) dbs[tid] = 0.f;
    const int sc_ = tid % CPR;
    const int pk = k0 + sc_ * CH;                // Q column
    const int ptap = pk / cs, pci = pk - ptap * cs;
    const int pdy = ptap / ks - pad, pdx = ptap % ks - pad;
    const int pco = co0 + sc_ * CH;              // P column
    const bool colp = pco < N, colq = pk < K;
    const float rW = 1.0f / (float)W, rH = 1.0f / (float)H;   // pixel decode (M / W < 2^22, host-checked)
    const int nst = mb < me ? (int)((me - mb + STG - 1) / STG) : 0;
    const int mfirst = nst > 0 ? (int)mb : 0;

    floatx4 acc[FT][FT];
#pragma unroll
    for (int i = 0; i < FT; ++i)
#pragma unroll
        for (int j = 0; j < FT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    // D-deep ring of register stages.  Loads are unconditional (clamped
    // addresses) so none of them sits under a branch (which would make the
    // compiler drain the queue); validity travels as bit masks applied when
    // the stage is written to LDS.
    u32x4 rp[D][PER], rq[D][PER];
    unsigned pm[D], qm[D];
    auto gload = [&](int u, long long mt) {
        unsigned bp = 0, bq = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int r = (tid + i * 256) / CPR;
            const long long m = mt + r;
            const bool inm = m < me;
            const int mi = inm ? (int)m : mfirst;
            const int row = fdiv_exact(mi, W, rW);
            const int xx = mi - row * W, yy = row - fdiv_exact(row, H, rH) * H;
            const int y2 = yy + pdy, x2 = xx + pdx;
            const bool okq = inm & colq & (y2 >= 0) & (y2 < H) & (x2 >= 0) & (x2 < W);
            rp[u][i] = *(const u32x4*)(DY + (long long)mi * a.cs_dy + (colp ? pco : 0));
            rq[u][i] = *(const u32x4*)(X + (okq ? ((long long)mi + pdy * W + pdx) * cs + pci : 0));
            bp |= (unsigned)(inm & colp) << i;
            bq |= (unsigned)okq << i;
        }
        pm[u] = bp;
        qm[u] = bq;
    };
    auto lstore = [&](int u, int buf) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int r = (tid + i * 256) / CPR;
            const uint32_t kp = ((pm[u] >> i) & 1u) ? ~0u : 0u;
            const uint32_t kq = ((qm[u] >> i) & 1u) ? ~0u : 0u;
            u32x4 v = rq[u][i];
            if (pro) {
                float f[CH];
                unpack(v, f, T());
#pragma unroll
                for (int j = 0; j < CH; ++j) f[j] = fmaxf(f[j] * bnp[pci + j] + bnp[cs + pci + j], 0.f);
                v = pack(f, T());
            }
            *(u32x4*)(Ps[buf] + r * ROWB + sc_ * 16) = rp[u][i] & u32x4{kp, kp, kp, kp};
            *(u32x4*)(Qs[buf] + r * ROWB + sc_ * 16) = v & u32x4{kq, kq, kq, kq};
        }
    };

    if (nst > 0) {   // the first D stages in flight while the BN table settles
#pragma unroll
        for (int u = 0; u < D; ++u) gload(u, mb + (long long)u * STG);
    }
    if (pro) block_bn_table(a.pro, a.cin, 0, cs, bnp, bnp + cs, nullptr, nullptr, dsm);
    __syncthreads();
    if (nst > 0) lstore(0, 0);
    __syncthreads();
    const int g = lane >> 4, li = lane & 15;
    float bpart = 0.f;   // bias partial: column tid % TC, rows (tid / TC) * STG*TC/256 .. of every stage
    for (int it0 = 0; it0 < nst; it0 += D) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
            const int it = it0 + u;
            if (it >= nst) break;
            const int cur = it & 1;
            // ring slot u (stage it) is in LDS already: refill it with stage it + D
            gload(u, mb + (long long)(it + D) * STG);
            if (do_bias) {
                constexpr int RB = STG * TC / 256;
                const int c = tid % TC, r0 = (tid / TC) * RB;
#pragma unroll
                for (int r = 0; r < RB; ++r) bpart += ldv((const T*)(Ps[cur] + (r0 + r) * ROWB) + c);
            }
            if constexpr (sizeof(T) == 2) {
                const int q = li >> 2, p = li & 3;
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    u32x4 af[FT], bfr[FT];
#pragma unroll
                    for (int i = 0; i < FT; ++i) {
                        const int c0 = wc * WT + i * 16 + 4 * p;
                        const char* base = Ps[cur] + (32 * s + 8 * g + q) * ROWB + c0 * 2;
                        i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RNVP_LDS i16x4*)base);
                        i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RNVP_LDS i16x4*)(base + 4 * ROWB));
                        af[i].x = (uint32_t)(uint16_t)lo.x | ((uint32_t)(uint16_t)lo.y << 16);
                        af[i].y = (uint32_t)(uint16_t)lo.z | ((uint32_t)(uint16_t)lo.w << 16);
                        af[i].z = (uint32_t)(uint16_t)hi.x | ((uint32_t)(uint16_t)hi.y << 16);
                        af[i].w = (uint32_t)(uint16_t)hi.z | ((uint32_t)(uint16_t)hi.w << 16);
                    }
#pragma unroll
                    for (int j = 0; j < FT; ++j) {
                        const int c0 = wk * WT + j * 16 + 4 * p;
                        const char* base = Qs[cur] + (32 * s + 8 * g + q) * ROWB + c0 * 2;
                        i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RNVP_LDS i16x4*)base);
                        i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RNVP_LDS i16x4*)(base + 4 * ROWB));
                        bfr[j].x = (uint32_t)(uint16_t)lo.x | ((uint32_t)(uint16_t)lo.y << 16);
                        bfr[j].y = (uint32_t)(uint16_t)lo.z | ((uint32_t)(uint16_t)lo.w << 16);
                        bfr[j].z = (uint32_t)(uint16_t)hi.x | ((uint32_t)(uint16_t)hi.y << 16);
                        bfr[j].w = (uint32_t)(uint16_t)hi.z | ((uint32_t)(uint16_t)hi.w << 16);
                    }
#pragma unroll
                    for (int i = 0; i < FT; ++i)
#pragma unroll
                        for (int j = 0; j < FT; ++j) Mf<bf16_t>::step(af[i], bfr[j], acc[i][j]);
                }
            } else {
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    u32x4 af[FT], bfr[FT];
#pragma unroll
                    for (int i = 0; i < FT; ++i) {
                        const char* pcol = Ps[cur] + (16 * s + 4 * g) * ROWB + (wc * WT + i * 16 + li) * 4;
                        af[i].x = *(const uint32_t*)(pcol);
                        af[i].y = *(const uint32_t*)(pcol + ROWB);
                        af[i].z = *(const uint32_t*)(pcol + 2 * ROWB);
                        af[i].w = *(const uint32_t*)(pcol + 3 * ROWB);
                    }
#pragma unroll
                    for (int j = 0; j < FT; ++j) {
                        const char* qcol = Qs[cur] + (16 * s + 4 * g) * ROWB + (wk * WT + j * 16 + li) * 4;
                        bfr[j].x = *(const uint32_t*)(qcol);
                        bfr[j].y = *(const uint32_t*)(qcol + ROWB);
                        bfr[j].z = *(const uint32_t*)(qcol + 2 * ROWB);
                        bfr[j].w = *(const uint32_t*)(qcol + 3 * ROWB);
                    }
#pragma unroll
                    for (int i = 0; i < FT; ++i)
#pragma unroll
                        for (int j = 0; j < FT; ++j) Mf<float>::step(af[i], bfr[j], acc[i][j]);
                }
            }
            if (it + 1 < nst) lstore((u + 1) % D, cur ^ 1);
            __syncthreads();
        }
    }
    // D rows = co, cols = k
#pragma unroll
    for (int i = 0; i < FT; ++i)
#pragma unroll
        for (int j = 0; j < FT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = co0 + wc * WT + i * 16 + (lane >> 4) * 4 + r;
                const int k = k0 + wk * WT + j * 16 + (lane & 15);
                if (co < N && k < K) {
                    float* o = out + (long long)co * a.kp + k;
                    if (atomic) atomicAdd(o, acc[i][j][r]);
                    else *o = acc[i][j][r];
                }
            }
    if (do_bias) atomicAdd(&dbs[tid % TC], bpart);
    __syncthreads();
    if (do_bias && tid < TC && co0 + tid < N) {
        if (bias_atomic) atomicAdd(&bias_out[co0 + tid], dbs[tid]);
        else bias_out[co0 + tid] = dbs[tid];
    }
}

// grouped: block -> (conv, slab z, co tile, k tile).  Consecutive tasks (the
// tiles of one slab, which re-read the same pixels through L2) are placed on
// one XCD: dispatch hands block b to XCD b % 8, so task = bijective remap.
template <typename T, int TC>
__global__ __launch_bounds__(256) void k_wgrad_grouped(rnvp_wgrad_group g) {
    const int nb = gridDim.x, b = blockIdx.x;
    const int q = nb / 8, r = nb % 8, xcd = b % 8;
    const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
    int c = 0;
    while (c + 1 < g.n_conv && g.conv[c + 1].task0 <= t) ++c;
    const rnvp_wgrad_conv& cv = g.conv[c];
    const int tco = (cv.n + TC - 1) / TC;
    const int local = t - cv.task0;
    const int per = tco * cv.tk;
    const int z = local / per, rr = local - z * per;
    const int cot = rr / cv.tk, kt = rr - cot * cv.tk;
    const long long M = (long long)g.B * g.H * g.W;
    const long long mb = (long long)z * cv.m_per_slab;
    const long long me = (mb + cv.m_per_slab < M) ? mb + cv.m_per_slab : M;
    const WgView v{cv.x, cv.dy, cv.pro, g.H, g.W, cv.ks, cv.cs_in, cv.cin, cv.cs_dy, cv.n, cv.kp, cv.pro_bn_relu};
    const int rep = z % cv.nrep;
    const bool atomic = cv.nrep < cv.nz;
    wgrad_tile<T, TC>(v, cot * TC, kt * TC, mb, me, M, cv.ws + (long long)rep * cv.n * cv.kp, atomic,
                  (cv.wsb && kt == 0) ? cv.wsb + (long long)rep * cv.n : nullptr, atomic);
}

// ---------------------------------------------------------------------------
// BN backward apply
// ---------------------------------------------------------------------------
template <typename T>
__global__ void k_bn_bwd(rnvp_bn_bwd_args a) {
    extern __shared__ double dsm[];
    bn_bwd_body<T>(a, dsm, blockIdx.x, gridDim.x);
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

__device__ __forceinline__ int find_tile(const rnvp_wn_desc* d, int n, int t) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (d[mid].tile0 <= t) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

constexpr int WN_ROW_LDS = 4608;

// Weight-norm forward, pass 1: ||v|| of every output row, one wave per row
// (coalesced 4-byte loads, 8 in flight per lane; v rows need not be 16-B
// aligned inside the parameter arena).  16-B loads (an aligned body between
// scalar head and tail) measured slower: 184 vs 147 us for config 1's rows.
__global__ __launch_bounds__(256) void k_wn_norm(const rnvp_wn_desc* __restrict__ descs, int n_desc, int rows) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= rows) return;
    const rnvp_wn_desc& d = descs[find_desc(descs, n_desc, row)];
    const int co = row - d.row0;
    const int kr = d.cin * d.ks * d.ks;
    const float* v = d.v + (long long)co * kr;
    double ss = 0.0;
    int i = lane;
    for (; i + 7 * 64 < kr; i += 8 * 64) {
        float x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = v[i + u * 64];
#pragma unroll
        for (int u = 0; u < 8; ++u) ss = fma((double)x[u], (double)x[u], ss);
    }
    for (; i < kr; i += 64) ss = fma((double)v[i], (double)v[i], ss);
    ss = wave_sum(ss);
    if (lane == 0) d.norm[co] = (float)sqrt(ss);
}

// Pass 2: w = g v / ||v|| on tiles of WN_TCO output x WN_TCI input channels
// (all taps): the v tile is read once (runs of WN_TCI*ks*ks contiguous floats
// per output channel) into LDS, then written as both packed images in
// 4-element stores -- wf[co][tap*cs_in + ci] and the flipped, transposed
// wd[ci][tp*cs_out + co] = w[co][ci][ks*ks-1-tp].  The images' padding
// (ci >= cin, co >= cout, k >= ks*ks*cs) is zero from allocation and never
// written.
// A 1x1 conv's tile spans WN_TCI1 input channels (the same LDS row, ks*ks = 1
// float per channel): 8x fewer, 8x larger blocks than 32-channel tiles, with
// 512-byte forward-image runs.  With the XCD-contiguous tile order and
// float-reciprocal index math below, config 1's large refresh went from 376
// to 284 us (profiles/r2_small_kernel_sweeps.txt).
constexpr int WN_TCO = 32, WN_TCI = 32, WN_TCI1 = 256;

__host__ __device__ constexpr int wn_tci(int ks) { return ks == 1 ? WN_TCI1 : WN_TCI; }

// The fragment-major copies (rnvp_wn_desc.wf_frag / wd_frag, read by the deep
// tiles through rnvp_conv_args.w_frag) of one k_wn_pack / k_wn_wd tile
// ([32 co] x [32 ci] x 3x3, or [32 co] x [256 ci] for 1x1): block (row / 16,
// k / 32) of 512 elements, lane L = row % 16 + 16 * (k % 32 / 8) holding
// k % 8 = 0..7.  With cs_in, cs_out, co0 and ci0 multiples of 32 every block
// the tile touches lies wholly in it (per tap: 16 rows x 32 ci, resp. 16 ci x
// 32 co) and is written whole: 16-byte stores, 1 KiB per block.
// val(c, ci, tap) is the tile's value of w[co0 + c][ci0 + ci][tap] as the
// row-major image holds it (0 outside the conv's rows / channels).
template <typename T, typename F>
__device__ __forceinline__ void wn_frag_tile(const rnvp_wn_desc& d, int co0, int ci0, int nco, int ncc, F val) {
    if constexpr (sizeof(T) != 2) return;   // the deep tiles read fragment-major images in bf16 only
    const int kk = d.ks * d.ks;
    const int rbo = (nco + 15) >> 4, rbi = (ncc + 15) >> 4, nkb = (ncc + 31) >> 5;
    if (d.wf_frag) {
        for (int q = threadIdx.x; q < rbo * kk * nkb * 64; q += blockDim.x) {
            const int L = q & 63, r = q >> 6, kb = r % nkb, r2 = r / nkb, tap = r2 % kk, rb = r2 / kk;
            const int c = rb * 16 + (L & 15), ci = kb * 32 + (L >> 4) * 8;
            float f[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = (c < nco && ci + e < ncc) ? val(c, ci + e, tap) : 0.f;
            T* dst = (T*)d.wf_frag +
                     ((long long)((co0 >> 4) + rb) * (d.kp_f >> 5) + ((tap * d.cs_in + ci0) >> 5) + kb) * 512 + L * 8;
            *(RNVP_GLOBAL u32x4*)dst = pack(f, T());
        }
    }
    if (d.wd_frag) {
        for (int q = threadIdx.x; q < rbi * kk * 64; q += blockDim.x) {
            const int L = q & 63, r = q >> 6, tp = r % kk, rb = r / kk;
            const int ci = rb * 16 + (L & 15), co = (L >> 4) * 8;
            float f[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = (ci < ncc && co + e < nco) ? val(co + e, ci, kk - 1 - tp) : 0.f;
            T* dst = (T*)d.wd_frag + ((long long)((ci0 >> 4) + rb) * (d.kp_d >> 5) + ((tp * d.cs_out + co0) >> 5)) * 512 + L * 8;
            *(RNVP_GLOBAL u32x4*)dst = pack(f, T());
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_wn_pack(const rnvp_wn_desc* __restrict__ descs, int n_desc) {
    constexpr int TP = WN_TCI * 9 + 1;                      // LDS row pitch (floats), odd
    static_assert(WN_TCI1 < TP, "1x1 tile row must fit the LDS row");
    __shared__ float tile[WN_TCO * TP];
    __shared__ float scl[WN_TCO];
    // consecutive tiles (the two halves of a 128-byte line of either image)
    // on one XCD: block b runs on XCD b % 8, so remap b bijectively
    const int nb = gridDim.x, b = blockIdx.x;
    const int q8 = nb / 8, r8 = nb % 8, xcd = b % 8;
    const int tg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
    const rnvp_wn_desc& d = descs[find_tile(descs, n_desc, tg)];
    const int t = tg - d.tile0;
    const int tci = wn_tci(d.ks);
    const int nci = (d.cin + tci - 1) / tci;
    const int co0 = (t / nci) * WN_TCO, ci0 = (t % nci) * tci;
    const int kk = d.ks * d.ks, kr = d.cin * kk;
    const int nco = min(WN_TCO, d.cout - co0), ncc = min(tci, d.cin - ci0);
    const int run = ncc * kk;                               // contiguous floats per output channel
    if (threadIdx.x < WN_TCO) {
        const int co = co0 + threadIdx.x;
        scl[threadIdx.x] = (threadIdx.x < nco && d.g) ? d.g[co] / d.norm[co] : 1.f;
    }
    // item indices stay < 2^17: float-reciprocal divisions (fdiv_small)
    const float r_run = 1.0f / (float)run;
    for (int q = threadIdx.x; q < nco * run; q += 256) {
        const int c = fdiv_small(q, r_run), j = q - c * run;
        tile[c * TP + j] = d.v[(long long)(co0 + c) * kr + (long long)ci0 * kk + j];
    }
    __syncthreads();
    // forward image: 4 consecutive ci per item
    const int ng = (ncc + 3) / 4;
    const float r_kng = 1.0f / (float)(kk * ng), r_ng = 1.0f / (float)ng;
    for (int q = threadIdx.x; q < nco * kk * ng; q += 256) {
        const int c = fdiv_small(q, r_kng), r = q - c * (kk * ng), tap = fdiv_small(r, r_ng), c4 = (r - tap * ng) * 4;
        float w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = c4 + e < ncc ? scl[c] * tile[c * TP + (c4 + e) * kk + tap] : 0.f;
        T* dst = (T*)d.wf + (long long)(co0 + c) * d.kp_f + tap * d.cs_in + ci0 + c4;
        if (c4 + 4 <= ncc) {
            st4(dst, w);
        } else {
            for (int e = 0; e < 4 && c4 + e < ncc; ++e) stv(dst + e, w[e]);
        }
    }
    wn_frag_tile<T>(d, co0, ci0, nco, ncc, [&](int c, int ci, int tap) { return scl[c] * tile[c * TP + ci * kk + tap]; });
    if (!d.wd) return;
    // data-gradient image: 4 consecutive co per item
    const int mg = (nco + 3) / 4;
    const float r_kmg = 1.0f / (float)(kk * mg), r_mg = 1.0f / (float)mg;
    for (int q = threadIdx.x; q < ncc * kk * mg; q += 256) {
        const int ci = fdiv_small(q, r_kmg), r = q - ci * (kk * mg), tp = fdiv_small(r, r_mg), o4 = (r - tp * mg) * 4;
        const int tap = kk - 1 - tp;
        float w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = o4 + e < nco ? scl[o4 + e] * tile[(o4 + e) * TP + ci * kk + tap] : 0.f;
        T* dst = (T*)d.wd + (long long)(ci0 + ci) * d.kp_d + tp * d.cs_out + co0 + o4;
        if (o4 + 4 <= nco) {
            st4(dst, w);
        } else {
            for (int e = 0; e < 4 && o4 + e < nco; ++e) stv(dst + e, w[e]);
        }
    }
}

// The data-gradient image from the forward image: wd[ci][tp*cs_out + co] =
// wf[co][(ks*ks-1-tp)*cs_in + ci], on k_wn_pack's tiles (the same XCD order
// and LDS tile, read from the forward image instead of v -- the values are
// already g v / ||v|| rounded to T, so the two images stay bitwise what
// k_wn_pack writes).  Used after the fused parameter pass (wn_adam.hip),
// which writes the forward image row by row: a row of wd spans every output
// channel, so writing it from one row block would be RB-element scatter.
template <typename T>
__global__ __launch_bounds__(256) void k_wn_wd(const rnvp_wn_desc* __restrict__ descs, int n_desc) {
    constexpr int TP = WN_TCI * 9 + 1;
    __shared__ float tile[WN_TCO * TP];
    const int nb = gridDim.x, b = blockIdx.x;
    const int q8 = nb / 8, r8 = nb % 8, xcd = b % 8;
    const int tg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
    const rnvp_wn_desc& d = descs[find_tile(descs, n_desc, tg)];
    if (!d.wd) return;
    const int t = tg - d.tile0;
    const int tci = wn_tci(d.ks);
    const int nci = (d.cin + tci - 1) / tci;
    const int co0 = (t / nci) * WN_TCO, ci0 = (t % nci) * tci;
    const int kk = d.ks * d.ks;
    const int nco = min(WN_TCO, d.cout - co0), ncc = min(tci, d.cin - ci0);
    // tile[c][ci * kk + tap] (k_wn_pack's layout) from the forward image rows,
    // 8 input channels per item: ci0 and cs_in are multiples of 8 and a row's
    // channel padding (up to cs_in) is in bounds, so every group is one
    // aligned 16-byte (bf16) or two (fp32) loads
    const int ng = (ncc + 7) / 8;
    const float r_kg = 1.0f / (float)(kk * ng), r_g = 1.0f / (float)ng;
    const RNVP_GLOBAL T* wf = (const RNVP_GLOBAL T*)d.wf;
    // WD_U items' loads issued before any is used (a latency-bound loop
    // otherwise: one 16-byte load in flight per thread); a clamped duplicate
    // past the end reloads the thread's first item and is not stored
    constexpr int WD_U = 4, NV = sizeof(T) == 4 ? 2 : 1;
    const int nit = nco * kk * ng;
    for (int q0 = threadIdx.x; q0 < nit; q0 += WD_U * 256) {
        u32x4 v[WD_U][NV];
#pragma unroll
        for (int u = 0; u < WD_U; ++u) {
            const int q = q0 + u * 256 < nit ? q0 + u * 256 : q0;
            const int c = fdiv_small(q, r_kg), r = q - c * (kk * ng), tap = fdiv_small(r, r_g), c8 = (r - tap * ng) * 8;
            const RNVP_GLOBAL T* src = wf + (long long)(co0 + c) * d.kp_f + tap * d.cs_in + ci0 + c8;
#pragma unroll
            for (int h = 0; h < NV; ++h) v[u][h] = *(const RNVP_GLOBAL u32x4*)(src + 4 * h);
        }
#pragma unroll
        for (int u = 0; u < WD_U; ++u) {
            const int q = q0 + u * 256;
            if (q >= nit) break;
            const int c = fdiv_small(q, r_kg), r = q - c * (kk * ng), tap = fdiv_small(r, r_g), c8 = (r - tap * ng) * 8;
            float f[8];
            unpack(v[u][0], f, T());
            if constexpr (NV == 2) unpack(v[u][1], f + 4, T());
#pragma unroll
            for (int e = 0; e < 8; ++e)
                if (c8 + e < ncc) tile[c * TP + (c8 + e) * kk + tap] = f[e];
        }
    }
    __syncthreads();
    wn_frag_tile<T>(d, co0, ci0, nco, ncc, [&](int c, int ci, int tap) { return tile[c * TP + ci * kk + tap]; });
    // 8 consecutive output channels per item: one 16-byte store (bf16)
    const int mg = (nco + 7) / 8;
    const float r_kmg = 1.0f / (float)(kk * mg), r_mg = 1.0f / (float)mg;
    for (int q = threadIdx.x; q < ncc * kk * mg; q += 256) {
        const int ci = fdiv_small(q, r_kmg), r = q - ci * (kk * mg), tp = fdiv_small(r, r_mg), o8 = (r - tp * mg) * 8;
        const int tap = kk - 1 - tp;
        float w[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) w[e] = o8 + e < nco ? tile[(o8 + e) * TP + ci * kk + tap] : 0.f;
        T* dst = (T*)d.wd + (long long)(ci0 + ci) * d.kp_d + tp * d.cs_out + co0 + o8;
        if (o8 + 8 <= nco) {
            if constexpr (sizeof(T) == 2) {
                *(RNVP_GLOBAL u32x4*)dst = pack(w, T());
            } else {
                *(RNVP_GLOBAL u32x4*)dst = pack(w, T());
                *(RNVP_GLOBAL u32x4*)(dst + 4) = pack(w + 4, T());
            }
        } else {
            for (int e = 0; e < 8 && o8 + e < nco; ++e) stg(dst + e, w[e]);
        }
    }
}

// one block per output row co: dW row = sum of the nz partial slabs, gathered
// into LDS in v's [ci][tap] order (coalesced over the packed k), then the
// weight-norm backward and the bias partial sum.

// bias sum over the replicas, and re-zeroing of the replicas (zero_after)
__device__ __forceinline__ void wn_bwd_tail(const rnvp_wn_desc& d, float* gbase, int co, int nz, long long zs,
                                            double* red) {
    if (d.dbp) {
        float bs = 0.f;
        for (int z = threadIdx.x; z < nz; z += blockDim.x) bs += d.dbp[(long long)z * d.cout + co];
        bs = block_sum(bs, (float*)red);
        if (threadIdx.x == 0) gbase[d.db_off + co] = bs;
        if (d.zero_after) {
            __syncthreads();
            for (int z = threadIdx.x; z < nz; z += blockDim.x) d.dbp[(long long)z * d.cout + co] = 0.f;
        }
    }
    if (d.zero_after) {   // leave the replicas zero for the next atomic accumulation
        __syncthreads();
        RNVP_GLOBAL float* dwz = (RNVP_GLOBAL float*)(d.dw + (long long)co * d.kp_f);
        const int K = d.ks * d.ks * d.cs_in;
        if ((K & 3) == 0 && (zs & 3) == 0 && (((uintptr_t)dwz) & 15) == 0) {
            for (int z = 0; z < nz; ++z)
                for (int k = 4 * threadIdx.x; k < K; k += 4 * blockDim.x)
                    *(RNVP_GLOBAL floatx4*)(dwz + z * zs + k) = floatx4{0.f, 0.f, 0.f, 0.f};
        } else {
            for (int z = 0; z < nz; ++z)
                for (int k = threadIdx.x; k < K; k += blockDim.x) dwz[z * zs + k] = 0.f;
        }
    }
}

__global__ void k_wn_bwd(const rnvp_wn_desc* __restrict__ descs, int n_desc, float* gbase, int rows, double* z0,
                         long long n0, double* z1, long long n1) {
    if ((int)blockIdx.x >= rows) {   // extra workgroups: zero the caller's sums ranges
        const long long stride = (long long)(gridDim.x - rows) * blockDim.x;
        const long long i0 = (long long)(blockIdx.x - rows) * blockDim.x + threadIdx.x;
        for (long long i = i0; i < n0; i += stride) z0[i] = 0.0;
        for (long long i = i0; i < n1; i += stride) z1[i] = 0.0;
        return;
    }
    __shared__ double red[16];
    __shared__ float rowbuf[WN_ROW_LDS];
    const int row = blockIdx.x;
    const rnvp_wn_desc d = descs[find_desc(descs, n_desc, row)];
    const int co = row - d.row0;
    const int kk = d.ks * d.ks, kr = d.cin * kk;
    const int nz = d.nz > 0 ? d.nz : 1;
    const long long zs = (long long)d.cout * d.kp_f;
    const float* v = d.v + (long long)co * kr;
    const float* dw = d.dw + (long long)co * d.kp_f;
    const bool in_lds = kr <= WN_ROW_LDS;
    auto dw_at = [&](int k) {
        float t = 0.f;
        for (int z = 0; z < nz; ++z) t += dw[z * zs + k];
        return t;
    };
    if (in_lds && blockDim.x == 256 && nz <= 8 && kk * d.cs_in <= WN_ROW_LDS) {
        // one memory round trip: every load of the row is issued up front --
        // this thread's v elements (kept in registers for both passes) and its
        // float4 chunks of the packed dW row, summed over the nz replicas --
        // then the dW row is gathered into v's [ci][tap] order in LDS
        constexpr int PT = WN_ROW_LDS / 256, P4 = (WN_ROW_LDS / 4 + 255) / 256;
        const int K4 = kk * d.cs_in / 4;            // cs_in % 8 == 0: a chunk never straddles a tap
        const float rcs = 1.0f / (float)d.cs_in;
        const RNVP_GLOBAL float* vg = (const RNVP_GLOBAL float*)v;
        float vr[PT];
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const int i = threadIdx.x + j * 256;
            vr[j] = vg[i < kr ? i : 0];
        }
        float4 cw[P4];
#pragma unroll
        for (int j = 0; j < P4; ++j) {
            const int q4 = threadIdx.x + j * 256;
            const RNVP_GLOBAL floatx4* src = (const RNVP_GLOBAL floatx4*)dw + (q4 < K4 ? q4 : 0);
            floatx4 t = src[0];
#pragma unroll
            for (int z = 1; z < 8; ++z) {
                if (z < nz) t += src[z * zs / 4];
            }
            cw[j] = float4{t.x, t.y, t.z, t.w};
        }
#pragma unroll
        for (int j = 0; j < P4; ++j) {
            const int q4 = threadIdx.x + j * 256;
            if (q4 < K4) {
                const int k = 4 * q4, tap = fdiv_small(k, rcs), ci = k - tap * d.cs_in;
                const float e[4] = {cw[j].x, cw[j].y, cw[j].z, cw[j].w};
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (ci + u < d.cin) rowbuf[(ci + u) * kk + tap] = e[u];
            }
        }
        __syncthreads();
        float dr[PT];
        double dot = 0;
#pragma unroll
        for (int j = 0; j < PT; ++j) {
            const int i = threadIdx.x + j * 256;
            dr[j] = i < kr ? rowbuf[i] : 0.f;
            dot = fma((double)dr[j], (double)vr[j], dot);
        }
        dot = block_sum(dot, red);
        RNVP_GLOBAL float* dv = (RNVP_GLOBAL float*)(gbase + d.dv_off + (long long)co * kr);
        if (d.g) {
            const float nrm = d.norm[co];
            const float gs = d.g[co] / nrm;
            const float proj = (float)(dot / ((double)nrm * nrm));
#pragma unroll
            for (int j = 0; j < PT; ++j) {
                const int i = threadIdx.x + j * 256;
                if (i < kr) dv[i] = gs * fmaf(-proj, vr[j], dr[j]);
            }
            if (threadIdx.x == 0 && d.dg_off >= 0) gbase[d.dg_off + co] = (float)(dot / nrm);
        } else {
#pragma unroll
            for (int j = 0; j < PT; ++j) {
                const int i = threadIdx.x + j * 256;
                if (i < kr) dv[i] = dr[j];
            }
        }
        wn_bwd_tail(d, gbase, co, nz, zs, red);
        return;
    }
    if (in_lds) {
        const int K = kk * d.cs_in;
        const float rcs = 1.0f / (float)d.cs_in;
        for (int k = threadIdx.x; k < K; k += blockDim.x) {
            const int tap = fdiv_small(k, rcs), ci = k - tap * d.cs_in;
            if (ci < d.cin) rowbuf[ci * kk + tap] = dw_at(k);
        }
        __syncthreads();
    }
    auto dwv = [&](int i) {
        if (in_lds) return rowbuf[i];
        const int ci = i / kk, tap = i - ci * kk;
        return dw_at(tap * d.cs_in + ci);
    };
    double dot = 0;
    for (int i = threadIdx.x; i < kr; i += blockDim.x) dot = fma((double)dwv(i), (double)v[i], dot);
    dot = block_sum(dot, red);
    float* dv = gbase + d.dv_off + (long long)co * kr;
    if (d.g) {
        const float nrm = d.norm[co];
        const float gs = d.g[co] / nrm;
        const float proj = (float)(dot / ((double)nrm * nrm));
        for (int i = threadIdx.x; i < kr; i += blockDim.x) dv[i] = gs * fmaf(-proj, v[i], dwv(i));
        if (threadIdx.x == 0 && d.dg_off >= 0) gbase[d.dg_off + co] = (float)(dot / nrm);
    } else {
        for (int i = threadIdx.x; i < kr; i += blockDim.x) dv[i] = dwv(i);
    }
    wn_bwd_tail(d, gbase, co, nz, zs, red);
}

inline bool al16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

// argument checks shared by rnvp_conv2d and rnvp_conv2d_check
int conv_args_status(const rnvp_conv_args* a) {
    if (!a || !a->x || !a->w || !a->y) return RNVP_E_INVALID;
    if (a->variant < 0 || (a->variant > RNVP_VARIANT_DEEP && a->variant < RNVP_VARIANT_DEEP0) ||
        a->variant >= RNVP_VARIANT_DEEP0 + RNVP_DEEP_CFGS)
        return RNVP_E_INVALID;
    if (a->w_frag && !al16(a->w_frag)) return RNVP_E_INVALID;
    if (a->dtype != RNVP_F32 && a->dtype != RNVP_BF16) return RNVP_E_INVALID;
    if (a->ks != 1 && a->ks != 3) return RNVP_E_UNSUPPORTED;
    if (a->B < 0 || a->H <= 0 || a->W <= 0 || a->n <= 0 || a->cin <= 0) return RNVP_E_INVALID;
    if ((a->cs_in & 7) || (a->cs_out & 7) || a->cs_in < a->cin || a->cs_out < a->n) return RNVP_E_INVALID;
    if ((a->kp & 63) || a->kp < a->ks * a->ks * a->cs_in) return RNVP_E_INVALID;
    if (!al16(a->x) || !al16(a->w)) return RNVP_E_INVALID;
    if (a->epi_relu_bn_bwd && !a->epi_x) return RNVP_E_INVALID;
    if ((long long)a->B * a->H * a->W >= (1ll << 31)) return RNVP_E_UNSUPPORTED;
    if (a->bp) {
        if (!a->bp_x || !al16(a->bp_x) || (a->bp_out && !al16(a->bp_out))) return RNVP_E_INVALID;
        if (a->bp_bn.sums && (!a->bp_sums || a->bp_shards < 1 || a->bp_bn.count <= 0)) return RNVP_E_INVALID;
        if (!a->bp_bn.sums && (!a->bp_bn.mean || !a->bp_bn.var)) return RNVP_E_INVALID;
        if (a->pro_bn_relu) return RNVP_E_INVALID;
    }
    return RNVP_OK;
}

// the configuration a BatchNorm-backward prologue runs on: the deep family's
// data-gradient tiles only (the other families have no such prologue).  The
// tuned dispatch folds where that measured faster than the apply's launch +
// the plain conv (tools/probe/deep_stamps.py bp / bp8, profiles/r6_bnfold.txt):
// the 3x3 tiles, the 8-wave tiles and the 4-wave 1x1 tiles up to 4096 pixels
// (+2.8 us against a ~5.7 us apply); at 16384 pixels the 4-wave 1x1 tile loses
// a wave per SIMD to the prologue's registers (+7.8 us) and keeps the apply (a
// forced deep configuration still runs it)
int bp_cfg_of(const rnvp_conv_args* a) {
    if (a->variant >= RNVP_VARIANT_DEEP0) {
        const int cfg = a->variant - RNVP_VARIANT_DEEP0;
        return (cfg == 0 || cfg == 4) ? cfg : -1;
    }
    if (a->variant != 0 && a->variant != RNVP_VARIANT_DEEP) return -1;
    const int cfg = rnvp_deep_auto_cfg(a);
    const long long M = (long long)a->B * a->H * a->W;
    if (cfg == 4 || (cfg == 0 && (a->ks == 3 || M <= 4096))) return cfg;
    return -1;
}

}  // namespace

extern "C" int rnvp_conv2d(const rnvp_conv_args* a, void* stream) {
    const int st = conv_args_status(a);
    if (st != RNVP_OK) return st;
    if (a->B == 0) return RNVP_OK;
    hipStream_t s = (hipStream_t)stream;
    if (a->bp) {
        const int cfg = bp_cfg_of(a);
        if (cfg >= 0) return rnvp_deep_launch(a, s, cfg);
        // the wide scales' streaming 1x1 and band 3x3 (bf16) have the prologue too
        if (a->variant != 0) return RNVP_E_UNSUPPORTED;
        const int r = rnvp_conv_s1_launch(a, s);
        return r != RNVP_E_UNSUPPORTED ? r : rnvp_conv_band2_launch(a, s);
    }
    return a->dtype == RNVP_F32 ? dispatch_conv<float>(a, s) : dispatch_conv<bf16_t>(a, s);
}

extern "C" int rnvp_conv2d_check(const rnvp_conv_args* a) {
    const int st = conv_args_status(a);
    if (st != RNVP_OK || a->B == 0) return st;
    if (a->bp) {
        const int cfg = bp_cfg_of(a);
        if (cfg >= 0) return rnvp_deep_launch(a, nullptr, cfg, true);
        if (a->variant != 0) return RNVP_E_UNSUPPORTED;
        const int r = rnvp_conv_s1_launch(a, nullptr, true);
        return r != RNVP_E_UNSUPPORTED ? r : rnvp_conv_band2_launch(a, nullptr, true);
    }
    return RNVP_OK;   // the dispatch has a family for every shape that passes the checks
}

#ifndef RNVP_SLAB_PX
#define RNVP_SLAB_PX 2048
#endif
extern "C" int rnvp_wgrad_slabs(long long M) {
    // ~2048 pixels per slab (32 stages of 64), at most 128 slabs
    long long z = M / RNVP_SLAB_PX;
    if (z > 128) z = 128;
    if (z < 1) z = 1;
    return (int)z;
}

extern "C" int rnvp_wgrad_replicas(int nz) { return nz < 8 ? (nz < 1 ? 1 : nz) : 8; }

extern "C" int rnvp_conv2d_wgrad_grouped(const rnvp_wgrad_group* gin, void* stream) {
    if (!gin || gin->n_conv <= 0 || gin->n_conv > RNVP_WGRAD_GROUP_MAX) return RNVP_E_INVALID;
    if (gin->dtype != RNVP_F32 && gin->dtype != RNVP_BF16) return RNVP_E_INVALID;
    if (gin->B < 0 || gin->H <= 0 || gin->W <= 0) return RNVP_E_INVALID;
    if (gin->B == 0) return RNVP_OK;
    // bf16: the tap-shared kernel (wgrad_tap.hip) where it applies
    if (gin->dtype == RNVP_BF16) {
        for (int c = 0; c < gin->n_conv; ++c) {
            const rnvp_wgrad_conv& v = gin->conv[c];
            if (!v.x || !v.dy || !v.ws) return RNVP_E_INVALID;
            if (v.ks != 1 && v.ks != 3) return RNVP_E_UNSUPPORTED;
            if (v.n <= 0 || v.cin <= 0 || v.nz <= 0 || v.nrep <= 0 || v.nrep > v.nz) return RNVP_E_INVALID;
            if ((v.cs_in & 7) || (v.cs_dy & 7) || v.cs_in < v.cin || v.cs_dy < v.n) return RNVP_E_INVALID;
            if (v.kp < v.ks * v.ks * v.cs_in) return RNVP_E_INVALID;
            if (!al16(v.x) || !al16(v.dy)) return RNVP_E_INVALID;
        }
        rnvp_wgrad_group gt = *gin;
        const int rc = rnvp_wgrad_tap_launch(&gt, (hipStream_t)stream);
        if (rc != RNVP_E_UNSUPPORTED) return rc;
    }
    rnvp_wgrad_group g = *gin;
    const long long M = (long long)g.B * g.H * g.W;
    const int STG = g.dtype == RNVP_BF16 ? 64 : 32;
    if (M >= (1ll << 31) || M / g.W >= (1ll << 22)) return RNVP_E_UNSUPPORTED;
    // 64 x 64 output tiles (128 x 128 halves the operand re-reads but was
    // measured slower at every scale of config 1: 5.0 vs 4.3 ms per step)
    const int TC = 64;
    long long tasks = 0;
    int max_cs = 8;
    for (int c = 0; c < g.n_conv; ++c) {
        rnvp_wgrad_conv& v = g.conv[c];
        if (!v.x || !v.dy || !v.ws) return RNVP_E_INVALID;
        if (v.ks != 1 && v.ks != 3) return RNVP_E_UNSUPPORTED;
        if (v.n <= 0 || v.cin <= 0 || v.nz <= 0 || v.nrep <= 0 || v.nrep > v.nz) return RNVP_E_INVALID;
        if ((v.cs_in & 7) || (v.cs_dy & 7) || v.cs_in < v.cin || v.cs_dy < v.n) return RNVP_E_INVALID;
        if (v.kp < v.ks * v.ks * v.cs_in) return RNVP_E_INVALID;
        if (!al16(v.x) || !al16(v.dy)) return RNVP_E_INVALID;
        const long long steps = (M + STG - 1) / STG;
        v.m_per_slab = ((steps + v.nz - 1) / v.nz) * STG;
        if ((M + v.m_per_slab - 1) / v.m_per_slab > v.nz) return RNVP_E_INVALID;
        v.tk = (v.ks * v.ks * v.cs_in + TC - 1) / TC;
        v.task0 = (int)tasks;
        tasks += (long long)v.nz * ((v.n + TC - 1) / TC) * v.tk;
        if (v.cs_in > max_cs) max_cs = v.cs_in;
    }
    if (tasks <= 0 || tasks > (1ll << 30)) return RNVP_E_INVALID;
    hipStream_t s = (hipStream_t)stream;
    const size_t shm = 24 * (size_t)max_cs;
    if (g.dtype == RNVP_F32) {
        if (TC == 128) k_wgrad_grouped<float, 128><<<(unsigned)tasks, 256, shm, s>>>(g);
        else k_wgrad_grouped<float, 64><<<(unsigned)tasks, 256, shm, s>>>(g);
    } else {
        if (TC == 128) k_wgrad_grouped<bf16_t, 128><<<(unsigned)tasks, 256, shm, s>>>(g);
        else k_wgrad_grouped<bf16_t, 64><<<(unsigned)tasks, 256, shm, s>>>(g);
    }
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_bn_bwd_apply(const rnvp_bn_bwd_args* a, void* stream) {
    if (!a || !a->g || !a->x || !a->dx || !a->sums || a->M < 0 || a->C <= 0 || (a->cs & 7) || a->cs < a->C)
        return RNVP_E_INVALID;
    if (a->sum_shards < 1) return RNVP_E_INVALID;
    if (a->dtype != RNVP_F32 && a->dtype != RNVP_BF16) return RNVP_E_INVALID;
    if (!al16(a->g) || !al16(a->x) || !al16(a->dx) || (a->residual && !al16(a->residual))) return RNVP_E_INVALID;
    if (a->M == 0) return RNVP_OK;
    hipStream_t s = (hipStream_t)stream;
    const int CH = a->dtype == RNVP_F32 ? 4 : 8;
    const long long nch = a->M * (a->cs / CH);
    size_t shm = 68 * (size_t)a->cs;   // 4*cs fp64 + 9*cs f32 (see k_bn_bwd)
    // every workgroup first reduces the fp64 statistic shards: 1024 groups
    // (4 per CU) amortise that best (sweep 512-4096, profiles/r2_small_kernel_sweeps.txt)
    if (a->dtype == RNVP_F32) k_bn_bwd<float><<<rnvp_grid(nch, 256, 1024), 256, shm, s>>>(*a);
    else k_bn_bwd<bf16_t><<<rnvp_grid(nch, 256, 1024), 256, shm, s>>>(*a);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_weight_norm_tiles(int cout, int cin, int ks) {
    if (cout <= 0 || cin <= 0 || (ks != 1 && ks != 3)) return RNVP_E_INVALID;
    return ((cout + WN_TCO - 1) / WN_TCO) * ((cin + wn_tci(ks) - 1) / wn_tci(ks));
}

extern "C" int rnvp_weight_norm_fwd(const rnvp_wn_desc* d, int n_desc, int total_rows, int total_tiles, int dtype,
                                    void* stream) {
    if (!d || n_desc <= 0 || total_rows <= 0 || total_tiles <= 0) return RNVP_E_INVALID;
    if (dtype != RNVP_F32 && dtype != RNVP_BF16) return RNVP_E_INVALID;
    hipStream_t s = (hipStream_t)stream;
    k_wn_norm<<<(total_rows + 3) / 4, 256, 0, s>>>(d, n_desc, total_rows);
    RNVP_LAUNCH_CHECK();
    if (dtype == RNVP_F32) k_wn_pack<float><<<total_tiles, 256, 0, s>>>(d, n_desc);
    else k_wn_pack<bf16_t><<<total_tiles, 256, 0, s>>>(d, n_desc);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_weight_norm_transpose(const rnvp_wn_desc* d, int n_desc, int total_tiles, int dtype, void* stream) {
    if (!d || n_desc <= 0 || total_tiles <= 0) return RNVP_E_INVALID;
    if (dtype != RNVP_F32 && dtype != RNVP_BF16) return RNVP_E_INVALID;
    hipStream_t s = (hipStream_t)stream;
    if (dtype == RNVP_F32) k_wn_wd<float><<<total_tiles, 256, 0, s>>>(d, n_desc);
    else k_wn_wd<bf16_t><<<total_tiles, 256, 0, s>>>(d, n_desc);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

extern "C" int rnvp_weight_norm_bwd(const rnvp_wn_desc* d, int n_desc, int total_rows, float* grad_base, void* zero0,
                                    long long zero0_bytes, void* zero1, long long zero1_bytes, void* stream) {
    if (!d || !grad_base || n_desc <= 0 || total_rows <= 0) return RNVP_E_INVALID;
    if (zero0_bytes < 0 || zero1_bytes < 0 || (zero0_bytes & 7) || (zero1_bytes & 7)) return RNVP_E_INVALID;
    if ((zero0_bytes && (!zero0 || ((uintptr_t)zero0 & 7))) || (zero1_bytes && (!zero1 || ((uintptr_t)zero1 & 7))))
        return RNVP_E_INVALID;
    const long long nz = (zero0_bytes > zero1_bytes ? zero0_bytes : zero1_bytes) / 8;
    const int extra = nz > 0 ? (int)((nz + 255) / 256 < 16 ? (nz + 255) / 256 : 16) : 0;
    k_wn_bwd<<<total_rows + extra, 256, 0, (hipStream_t)stream>>>(d, n_desc, grad_base, total_rows, (double*)zero0,
                                                                  zero0_bytes / 8, (double*)zero1, zero1_bytes / 8);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}
