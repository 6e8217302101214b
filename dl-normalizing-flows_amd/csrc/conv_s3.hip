// Row-streaming 3x3 conv for the wide scales (bf16; image rows of 32 or 64
// pixels, cs_in <= 64, N <= 64): WeightNormConv2d (modules_realnvp.py:64-71)
// with the fused BatchNorm+ReLU prologue and the bias / residual / skip /
// next-BN-statistics (or the dgrad ReLU/BN-backward) epilogue, as
// rnvp_conv2d's other families.
//
// At 64x64 / 32x32 pixels a 3x3 over 32-64 channels is a stream (~140 FLOP
// per byte against a ridge of ~300): read x once, write y once.  The round-2
// band kernel staged a 256-pixel band plus a (W+1)-row halo per workgroup and
// re-derived BN tables and weights per band (~1.2 TB/s).  Here a workgroup
// walks a run of image rows four at a time (one output row per wave):
//   * input rows live in an LDS ring of 10 zero-padded rows ((W+2) columns,
//     BN+ReLU applied once); the rows above/below an image are a zero row;
//   * the next TWO iterations' input rows are in flight in registers while the
//     current one computes (one barrier per iteration);
//   * packed weights and BN tables are loaded once per workgroup;
//   * product D[n][m] = W[n][k] X[m][k]^T: a lane owns 4 consecutive output
//     channels of one pixel (8-byte epilogue vectors).
#include "common.h"
#include "conv_common.h"

#include <type_traits>

namespace {

constexpr int S3_NR = 10;        // ring rows: o-1 .. o+8 of an iteration at rows o .. o+3
constexpr int S3_RPI = 4;        // output rows per iteration (one per wave)

__host__ __device__ inline int s3_csp(int cs) { return (cs + 31) / 32 * 32; }    // LDS channel pitch
__host__ __device__ inline int s3_xp(int cs) { return s3_csp(cs) * 2 + 16; }     // bytes per position
__host__ __device__ inline int s3_kp(int cs) { return 9 * s3_csp(cs) * 2 + 16; } // bytes per weight row
__host__ __device__ inline size_t s3_lds(int cs, int n, int W) {
    const int nc = n <= 16 ? 16 : (n <= 32 ? 32 : 64);
    return (size_t)(S3_NR + 1) * (W + 2) * s3_xp(cs) + (size_t)nc * s3_kp(cs);
}

// TW: 16-pixel fragments per output row (W / 16); NOPS epilogue streams
template <int NT, int TW, int NOPS>
__global__ __launch_bounds__(256) void k_conv_s3(rnvp_conv_args a, int shards, int groups_per_wg) {
    constexpr int CH = 8, KS = 32;
    constexpr int NC = 16 * NT;
    constexpr int W = 16 * TW, PW = W + 2;
    constexpr int CPT = (S3_RPI * W * 8) / 256;              // max 16-B chunks per thread per iteration (csp 64)
    extern __shared__ __attribute__((aligned(16))) char lds[];
    __shared__ double red[4][NC][2];
    __shared__ double tmp[2 * 64];
    __shared__ float bnp[2 * 64];
    __shared__ float etab[4 * NC];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, li = lane & 15;
    const int H = a.H, N = a.n, cs = a.cs_in, cso = a.cs_out;
    const int rows = a.B * H;                                // output rows (b, y)
    const int M = rows * W;
    const int csp = s3_csp(cs), XP = s3_xp(cs), KPB = s3_kp(cs);
    const int ncs = csp / 32;                                // 32-channel chunks per tap
    const int nsteps = 9 * ncs;
    const int cpp = csp / 8;                                 // 16-B chunks per position
    const bool pro = a.pro_bn_relu != 0, epi_bn = a.epi_relu_bn_bwd != 0;
    char* ring = lds;                                        // [NR][PW][XP]; row NR = zeros
    char* wl = lds + (size_t)(S3_NR + 1) * PW * XP;          // [NC][9*csp] bf16 (+16 B pitch)

    // ---- tables and weights (once per workgroup) ----
    if (pro) block_bn_table(a.pro, a.cin, 0, cs, bnp, bnp + cs, nullptr, nullptr, tmp);
    if (epi_bn) block_bn_table(a.epi, N, 0, NC, etab, etab + NC, etab + 2 * NC, etab + 3 * NC, tmp);
    {
        // packed wf[n][(ky*3+kx)*cs + ci] -> LDS [n][tap*csp + ci] (zero beyond N / cs)
        const bf16_t* Wg = (const bf16_t*)a.w;
        const int wcpr = 9 * cpp;
        for (int q = tid; q < NC * wcpr; q += 256) {
            const int n = q / wcpr, c = q - n * wcpr, tap = c / cpp, ci = (c - tap * cpp) * 8;
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            if (n < N && ci < cs) v = *(const u32x4*)(Wg + (long long)n * a.kp + tap * cs + ci);
            *(u32x4*)(wl + n * KPB + (tap * csp + ci) * 2) = v;
        }
        for (int q = tid; q < PW * cpp; q += 256)            // the zero row
            *(u32x4*)(ring + (size_t)S3_NR * PW * XP + (q / cpp) * XP + (q % cpp) * 16) = u32x4{0u, 0u, 0u, 0u};
        for (int q = tid; q < S3_NR * 2 * cpp; q += 256) {   // padding columns of every ring row
            const int r = q / (2 * cpp), side = (q / cpp) & 1, c = q % cpp;
            *(u32x4*)(ring + ((size_t)r * PW + (side ? PW - 1 : 0)) * XP + c * 16) = u32x4{0u, 0u, 0u, 0u};
        }
    }
    __syncthreads();
    // this thread's prologue coefficients: chunk column cch of every staged row
    // (256 threads over W * cpp chunks of a row: the chunk index is fixed)
    const int cch = tid % cpp;
    float psc[CH], psh[CH];
#pragma unroll
    for (int e = 0; e < CH; ++e) {
        const int c = cch * 8 + e;
        psc[e] = (pro && c < cs) ? bnp[c] : 1.f;
        psh[e] = (pro && c < cs) ? bnp[cs + c] : 0.f;
    }
    float bias[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = j * 16 + 4 * g + r;
            bias[j][r] = (a.bias && n < N) ? a.bias[n] : 0.f;
        }

    const __amdgpu_buffer_rsrc_t XR = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0,
                                                                        (int)((long long)M * cs * 2), 0x00020000);
    const bool p0 = a.residual != nullptr, p1 = a.accumulate != 0;
    int role[3];
    role[0] = p0 ? 0 : (p1 ? 1 : 2);
    role[1] = (p0 && p1) ? 1 : 2;
    role[2] = 2;
    __amdgpu_buffer_rsrc_t OR[NOPS > 0 ? NOPS : 1];
#pragma unroll
    for (int q = 0; q < NOPS; ++q) {
        const void* src = role[q] == 0 ? a.residual : (role[q] == 1 ? (const void*)a.y : a.epi_x);
        OR[q] = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(src), 0, (int)((long long)M * cso * 2),
                                                  0x00020000);
    }
    constexpr int OOB = 0x7ffffff0;

    // this workgroup's output rows [r0, r1), walked S3_RPI at a time
    const int ngroups = (rows + S3_RPI - 1) / S3_RPI;
    const int gq0 = blockIdx.x * groups_per_wg;
    const int r0 = gq0 * S3_RPI;
    int r1 = (gq0 + groups_per_wg) * S3_RPI;
    if (r1 > rows) r1 = rows;
    const int nit = r0 < r1 ? (r1 - r0 + S3_RPI - 1) / S3_RPI : 0;
    (void)ngroups;

    // staging of input rows [rb, rb + nr) (global row index; rows outside
    // [0, rows) are never needed: image borders read the zero row)
    const int chunks_per_row = W * cpp;
    u32x4 stg[2][CPT];
    auto sload = [&](int rb, int nr, auto SLC) __attribute__((always_inline)) {
        constexpr int SL = decltype(SLC)::value;
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            const int q = tid + u * 256;
            const int rr = q / chunks_per_row, rem = q - rr * chunks_per_row;
            const int px = rem / cpp, c = rem - px * cpp;
            const int row = rb + rr;
            const bool ok = (rr < nr) & (row >= 0) & (row < rows) & (c * 8 < cs);
            stg[SL][u] = __builtin_amdgcn_raw_buffer_load_b128(XR, ok ? ((row * W + px) * cs + c * 8) * 2 : OOB, 0, 0);
        }
    };
    auto sstore = [&](int rb, int nr, auto SLC) __attribute__((always_inline)) {
        constexpr int SL = decltype(SLC)::value;
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            const int q = tid + u * 256;
            const int rr = q / chunks_per_row, rem = q - rr * chunks_per_row;
            const int px = rem / cpp, c = rem - px * cpp;
            const int row = rb + rr;
            if (rr >= nr || row < 0) continue;
            u32x4 v = stg[SL][u];
            if (pro) {
                float f[CH];
                unpack(v, f, bf16_t());
#pragma unroll
                for (int e = 0; e < CH; ++e) f[e] = fmaxf(f[e] * psc[e] + psh[e], 0.f);
                v = pack(f, bf16_t());
                const uint32_t keep = ((row < rows) & (c * 8 < cs)) ? ~0u : 0u;
                v &= u32x4{keep, keep, keep, keep};
            }
            *(u32x4*)(ring + ((size_t)(row % S3_NR) * PW + px + 1) * XP + c * 16) = v;
        }
    };

    double s1[NT][4], s2[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) s1[j][r] = s2[j][r] = 0.0;
    bf16_t* __restrict__ Y = (bf16_t*)a.y;

    // one iteration: output row o = rbase + wid of this wave
    auto compute = [&](int rbase) __attribute__((always_inline)) {
        const int o = rbase + wid;
        const bool live = o < r1;
        const int y = o % H;
        // ring rows of taps dy = -1, 0, +1 (the zero row across an image border)
        const int rw0 = ((y > 0) ? ((o - 1) % S3_NR) : S3_NR) * PW * XP;
        const int rw1 = (o % S3_NR) * PW * XP;
        const int rw2 = ((y < H - 1) ? ((o + 1) % S3_NR) : S3_NR) * PW * XP;
        // epilogue operands in flight under the MFMAs
        uint2 eo[NOPS > 0 ? NOPS : 1][TW][NT];
#pragma unroll
        for (int i = 0; i < TW; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int m = o * W + i * 16 + li, n0 = j * 16 + 4 * g;
                const int off = (live & (n0 < cso)) ? (m * cso + n0) * 2 : OOB;
#pragma unroll
                for (int q = 0; q < NOPS; ++q)
                    eo[q][i][j] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(OR[q], off, 0, 0));
            }
        floatx4 acc[TW][NT];
#pragma unroll
        for (int i = 0; i < TW; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        for (int st = 0; st < nsteps; ++st) {
            const int tap = st / ncs, ch = st - tap * ncs;
            const int dy = tap / 3, dx = tap - dy * 3;            // dx: column offset 0..2 in the padded row
            const int rw = dy == 0 ? rw0 : (dy == 1 ? rw1 : rw2);     // selects, not an indexed array
            const char* rp = ring + rw + dx * XP + (ch * 32 + g * 8) * 2;
            u32x4 wv[NT], xv[TW];
#pragma unroll
            for (int j = 0; j < NT; ++j)
                wv[j] = *(const u32x4*)(wl + (j * 16 + li) * KPB + (st * 32 + g * 8) * 2);
#pragma unroll
            for (int i = 0; i < TW; ++i) xv[i] = *(const u32x4*)(rp + (i * 16 + li) * XP);
#pragma unroll
            for (int i = 0; i < TW; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j) Mf<bf16_t>::step(wv[j], xv[i], acc[i][j]);
        }
        if (!live) return;
#pragma unroll
        for (int i = 0; i < TW; ++i) {
            const int m = o * W + i * 16 + li;
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int n0 = j * 16 + 4 * g;
                if (n0 >= cso) continue;
                float v[4], xv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[j][r];
#pragma unroll
                for (int q = 0; q < NOPS; ++q) {
                    const uint2 u = eo[q][i][j];
                    const float f[4] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                        __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
                    if (role[q] == 2) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) xv[r] = f[r];
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] += f[r];
                    }
                }
                if (epi_bn) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int n = n0 + r;
                        if (xv[r] * etab[n] + etab[NC + n] <= 0.f) v[r] = 0.f;
                        s1[j][r] += v[r];
                        s2[j][r] += v[r] * (xv[r] - etab[2 * NC + n]) * etab[3 * NC + n];
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        s1[j][r] += v[r];
                        s2[j][r] += (double)v[r] * v[r];
                    }
                }
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (n0 + r >= N) v[r] = 0.f;
                st4(Y + (long long)m * cso + n0, v);
            }
        }
    };

    // pipeline: the ring holds rows o-1 .. o+4 of the current iteration (rows
    // o .. o+3); registers hold rows o+5 .. o+8 (next iteration) and o+9 ..
    // o+12 (the one after, issued here)
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    if (nit > 0) {
        sload(r0 - 1, 3, I0{});                 // rows r0-1 .. r0+1
        sload(r0 + 2, 3, I1{});                 // rows r0+2 .. r0+4
        sstore(r0 - 1, 3, I0{});
        sstore(r0 + 2, 3, I1{});
        sload(r0 + 5, 4, I0{});                 // next iteration's new rows
    }
    __syncthreads();
    auto iter = [&](int it, auto SLC) __attribute__((always_inline)) {
        constexpr int SL = decltype(SLC)::value;                 // slot holding rows of iteration it + 1
        const int rb = r0 + it * S3_RPI;
        if (it + 2 < nit) sload(rb + 9, 4, std::integral_constant<int, 1 - SL>{});
        compute(rb);
        sstore(rb + 5, 4, std::integral_constant<int, SL>{});
        __syncthreads();
    };
    for (int it = 0; it < nit; it += 2) {
        iter(it, I0{});
        if (it + 1 < nit) iter(it + 1, I1{});
    }

    // ---- batch statistics ----
    const bool want_sums = a.out_sums || (epi_bn && a.epi_sums);
    if (want_sums) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double u1 = row_sum16(s1[j][r]), u2 = row_sum16(s2[j][r]);
                if (li == 0) {
                    red[wid][j * 16 + 4 * g + r][0] = u1;
                    red[wid][j * 16 + 4 * g + r][1] = u2;
                }
            }
        __syncthreads();
        double* sums = shard_ptr(epi_bn ? a.epi_sums : a.out_sums, shards, N);
        for (int n = tid; n < N; n += 256) {
            double t1 = 0.0, t2 = 0.0;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                t1 += red[w][n][0];
                t2 += red[w][n][1];
            }
            atomicAdd(&sums[n], t1);
            atomicAdd(&sums[N + n], t2);
        }
    }
}

template <int NT, int TW, int NOPS>
int launch_s3(const rnvp_conv_args* a, hipStream_t s) {
    const int rows = a->B * a->H;
    const int ngroups = (rows + S3_RPI - 1) / S3_RPI;
    const size_t shm = s3_lds(a->cs_in, a->n, a->W);
    static const int per_cu = [&] {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_conv_s3<NT, TW, NOPS>, 256, shm) != hipSuccess || n < 1)
            n = 1;
        return n;
    }();
    long long nwg = 256LL * per_cu;
    if (nwg > ngroups) nwg = ngroups;
    const int gpw = (int)((ngroups + nwg - 1) / nwg);
    nwg = (ngroups + gpw - 1) / gpw;
    k_conv_s3<NT, TW, NOPS><<<(unsigned)nwg, 256, shm, s>>>(*a, rnvp_stat_shards((long long)rows * a->W), gpw);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

template <int NT, int TW>
int launch_s3_ops(const rnvp_conv_args* a, hipStream_t s) {
    const int nops = (a->residual ? 1 : 0) + (a->accumulate ? 1 : 0) + (a->epi_relu_bn_bwd ? 1 : 0);
    switch (nops) {
        case 0: return launch_s3<NT, TW, 0>(a, s);
        case 1: return launch_s3<NT, TW, 1>(a, s);
        case 2: return launch_s3<NT, TW, 2>(a, s);
        default: return launch_s3<NT, TW, 3>(a, s);
    }
}

}  // namespace

// 3x3, bf16, W in {32, 64}, cs_in <= 64, N <= 64, M >= 16k: the row stream
int rnvp_conv_s3_launch(const rnvp_conv_args* a, hipStream_t s) {
    if (a->dtype != RNVP_BF16 || a->ks != 3 || a->n > 64 || a->cs_in > 64 || a->cs_out > 64) return RNVP_E_UNSUPPORTED;
    if (a->W != 32 && a->W != 64) return RNVP_E_UNSUPPORTED;
    const long long M = (long long)a->B * a->H * a->W;
    if (M < 16384 || M * 64 * 2 >= (1ll << 31)) return RNVP_E_UNSUPPORTED;
    if (s3_lds(a->cs_in, a->n, a->W) > 150 * 1024) return RNVP_E_UNSUPPORTED;
    if (((uintptr_t)a->y & 7) || (a->residual && ((uintptr_t)a->residual & 7)) ||
        (a->epi_relu_bn_bwd && ((uintptr_t)a->epi_x & 7)))
        return RNVP_E_UNSUPPORTED;
    const bool w64 = a->W == 64;
    if (a->n <= 16) return w64 ? launch_s3_ops<1, 4>(a, s) : launch_s3_ops<1, 2>(a, s);
    if (a->n <= 32) return w64 ? launch_s3_ops<2, 4>(a, s) : launch_s3_ops<2, 2>(a, s);
    return w64 ? launch_s3_ops<4, 4>(a, s) : launch_s3_ops<4, 2>(a, s);
}
