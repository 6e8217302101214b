"""One-off source edit: band kernel for the wide scales (cs_in <= 64, N <= 64)."""
import sys

p = "/root/repo/dl-normalizing-flows_amd/csrc/conv.hip"
s = open(p).read()
anchor = "template <typename T>\nint dispatch_conv(const rnvp_conv_args* a, hipStream_t s) {"
if s.count(anchor) != 1:
    sys.exit("anchor")
band = r'''// ---------------------------------------------------------------------------
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
    const int kpl = ((K + KS - 1) / KS) * KS + CH;
    const int R = BM + 2 * (ks / 2) * (W + 1);
    const int ntmp = cs > nc ? cs : nc;
    return 16 * (size_t)ntmp + 8 * (size_t)cs + 20 * (size_t)nc + 64 * (size_t)nc +
           ((size_t)nc * kpl + (size_t)(R + 1) * (cs + CH)) * sizeof(T);
}

template <typename T, int NT, int KSZ, bool PRO>
__global__ __launch_bounds__(256) void k_conv_band(rnvp_conv_args a, int shards) {
    constexpr int CH = Mf<T>::CH, KS = 4 * CH;
    constexpr int NC = 16 * NT;
    constexpr int TM = 4, BM = 64 * TM;        // 4 waves x 64 pixels
    constexpr int PAD = KSZ / 2;
    constexpr int SB = 12;                     // staged 16-B chunks per thread per batch
    extern __shared__ double dsm[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, li = lane & 15;
    const int M = a.B * a.H * a.W, W = a.W, H = a.H;
    const int N = a.n, cs = a.cs_in;
    const int K = KSZ * KSZ * cs;
    const int nsteps = (K + KS - 1) / KS;
    const int kpl = nsteps * KS + CH;          // weight row pitch (+16 B)
    const bool epi_bn = a.epi_relu_bn_bwd != 0;
    const int ntmp = cs > NC ? cs : NC;
    const int hal = PAD * (W + 1), R = BM + 2 * hal;
    const int pitch = cs + CH;                 // band row pitch (+16 B)

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
    const int cpr = cs / CH;
    const int total = R * cpr;
    const float rcpr = 1.0f / (float)cpr;
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
    stage_load(0);

    // ---- BN tables, packed weights (rows >= N and k >= K zero) and bias -> LDS
    if (PRO) block_bn_table(a.pro, a.cin, 0, cs, bnp, bnp + cs, nullptr, nullptr, tmp);
    if (epi_bn) block_bn_table(a.epi, N, 0, NC, etab, etab + NC, etab + 2 * NC, etab + 3 * NC, tmp);
    {
        const T* Wg = (const T*)a.w;
        const int wcpr = kpl / CH, wtot = NC * wcpr, kv = nsteps * KS;
        const float rw = 1.0f / (float)wcpr;
        for (int q0 = 0; q0 < wtot; q0 += 4 * 256) {
            u32x4 v[4];
            unsigned okm = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = q0 + u * 256 + tid;
                const int r = fdiv_small(q, rw), c = q - r * wcpr;
                const bool ok = (q < wtot) & (r < N) & (c * CH < kv);
                v[u] = *(const u32x4*)(Wg + (ok ? (long long)r * a.kp + c * CH : 0));
                okm |= (unsigned)ok << u;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = q0 + u * 256 + tid;
                if (q < wtot) {
                    const int r = fdiv_small(q, rw), c = q - r * wcpr;
                    const uint32_t keep = ((okm >> u) & 1u) ? ~0u : 0u;
                    *(u32x4*)(Wl + r * kpl + c * CH) = v[u] & u32x4{keep, keep, keep, keep};
                }
            }
        }
        for (int n = tid; n < NC; n += 256) btab[n] = (a.bias && n < N) ? a.bias[n] : 0.f;
        for (int c = tid * CH; c < pitch; c += 256 * CH) *(u32x4*)(zrow + c) = u32x4{0u, 0u, 0u, 0u};
    }
    __syncthreads();

    // ---- act(x) band -> LDS (transformed once) ----
    stage_store(0);
    for (int q0 = 256 * SB; q0 < total; q0 += 256 * SB) {
        stage_load(q0);
        stage_store(q0);
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
        unsigned bits = 0;
#pragma unroll
        for (int tp = 0; tp < KSZ * KSZ; ++tp) {
            const int yy = y + tp / KSZ - PAD, xx = x + tp % KSZ - PAD;
            bits |= (unsigned)((m < M) & (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)) << tp;
        }
        tvm[i] = bits;
    }

    floatx4 acc[TM][NT];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    // lane's K position k = s*KS + g*CH -> (tap, ci); a 16-B chunk never
    // straddles a tap (cs % CH == 0); KS / cs <= 4 wraps per step
    int tap = 0, ci = g * CH;
#pragma unroll
    for (int w = 0; w < 4; ++w)
        if (ci >= cs) { ci -= cs; ++tap; }
    const T* wl = Wl + li * kpl + g * CH;
    for (int st = 0; st < nsteps; ++st) {
        const int ty = tap / KSZ;
        const int toff = ((ty - PAD) * W + (tap - ty * KSZ - PAD)) * pitch + ci;
        const int tsh = tap < KSZ * KSZ ? tap : 31;   // bit 31 of tvm is never set
        u32x4 wv[NT], av[TM];
#pragma unroll
        for (int j = 0; j < NT; ++j) wv[j] = *(const u32x4*)(wl + j * 16 * kpl + st * KS);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const bool ok = (tvm[i] >> tsh) & 1u;
            av[i] = *(const u32x4*)(ok ? act + rowoff[i] + toff : zrow);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) Mf<T>::step(wv[j], av[i], acc[i][j]);
        ci += KS;
#pragma unroll
        for (int w = 0; w < 4; ++w)
            if (ci >= cs) { ci -= cs; ++tap; }
    }

    // ---- epilogue: lane owns channels j*16 + 4g .. +3 of its pixels ----
    const int cso = a.cs_out;
    double s1[NT][4], s2[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) s1[j][r] = s2[j][r] = 0.0;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + wid * 64 + i * 16 + li;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int n0 = j * 16 + 4 * g;
            if (n0 >= cso) continue;
            epi4<T>(a, (long long)m * cso + n0, acc[i][j], btab + n0, epi_bn, etab + n0, NC, s1[j], s2[j], N - n0);
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
    if (a->pro_bn_relu) k_conv_band<T, NT, KSZ, true><<<grid, 256, shm, s>>>(*a, sh);
    else k_conv_band<T, NT, KSZ, false><<<grid, 256, shm, s>>>(*a, sh);
    RNVP_LAUNCH_CHECK();
    return RNVP_OK;
}

// wide scales: few channels, many pixels (fp32 reciprocal pixel decode: M < 2^21)
template <typename T>
bool band_ok(const rnvp_conv_args* a) {
    const long long M = (long long)a->B * a->H * a->W;
    if (a->n > 64 || a->cs_in > 64 || (a->ks != 1 && a->ks != 3)) return false;
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

'''
s = s.replace(anchor, band + anchor)
old = "    if (stream_ok<T>(a)) return dispatch_stream<T>(a, s);\n    if (rnvp_conv_legacy == 0 && halo_ok<T>(a))"
if s.count(old) != 1:
    sys.exit("dispatch")
s = s.replace(old, "    if (rnvp_conv_legacy == 0 && band_ok<T>(a)) return dispatch_band<T>(a, s);\n" + old)
s = s.replace("static int rnvp_conv_legacy = 0;",
              "// (also the register-streaming kernel instead of the band kernel at the wide scales)\nstatic int rnvp_conv_legacy = 0;")
open(p, "w").write(s)
print("ok")
