"""Kernel-level parity of rnvp_conv2d (every kernel family it dispatches to:
band, register-streaming, halo tile, deep-K, LDS-tiled + split-K) against a float64 torch CPU
restatement of the same fused op:

    y[m, n] = sum_k act(x)[m + tap(k), ci(k)] * w[n, k] + bias[n] (+ residual) (+ y)
    act     = relu(bn(x)) (batch statistics from the given sharded sums) or x
    stats   = {sum y, sum y^2} per channel           (forward epilogue)
    dgrad   = y * [relu(bn(epi_x)) > 0], stats {sum, sum * xhat}

which is what WeightNormConv2d inside ResidualBlock computes
(modules_realnvp.py:64-114) once BatchNorm/ReLU and the residual/skip adds are
fused.  Tolerances: fp32 1e-5 relative (normwise); bf16 operands are rounded
the way the kernels round them (act -> bf16 before the product), 4e-3.
"""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
EPS = 1e-5


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def bf16_round(t):
    return t.to(torch.bfloat16).to(torch.float64)


def run_case(B, H, W, cin, cout, ks, dtype, pro=False, residual=False, acc=False, stats=False, dgrad=False,
             bias=True, variant=0, seed=0, rows=None, fm=False):
    """rows: compute the float64 reference only at these output pixels
    (config 4's M = 2^22 shapes, whose full float64 conv is too slow on the
    host); the statistics are then checked against the float64 sums of the
    kernel's own output (the epilogue reduction), the values row by row."""
    from realnvp_hip import _lib
    from realnvp_hip._lib import BNSrc, ConvArgs
    from realnvp_hip.engine import splitk_workspace, stat_shards
    from realnvp_hip.net import chan_stride, round_up
    g = torch.Generator().manual_seed(seed)
    tdt = torch.float32 if dtype == "fp32" else torch.bfloat16
    M = B * H * W
    csi, cso = chan_stride(cin), chan_stride(cout)
    kp = round_up(ks * ks * csi, 64)
    x = torch.randn(M, cin, generator=g, dtype=torch.float64)
    w = torch.randn(cout, ks, ks, cin, generator=g, dtype=torch.float64) / np.sqrt(ks * ks * cin)
    bvec = torch.randn(cout, generator=g, dtype=torch.float64) if bias else torch.zeros(cout, dtype=torch.float64)
    rnd = (lambda t: t.float().double()) if dtype == "fp32" else bf16_round
    # operands the flags do not use are not drawn (config 4's M = 2^22 cases)
    zero = torch.zeros(1, cout, dtype=torch.float64)
    res = rnd(torch.randn(M, cout, generator=g, dtype=torch.float64)) if residual else zero
    yold = rnd(torch.randn(M, cout, generator=g, dtype=torch.float64)) if acc else zero
    ex = rnd(torch.randn(M, cout, generator=g, dtype=torch.float64)) if dgrad else zero
    x, w, bvec = rnd(x), rnd(w), bvec.float().double()

    def nhwc(t, cs):
        out = torch.zeros(t.shape[0], cs, dtype=tdt)
        out[:, :t.shape[1]] = t.to(tdt)
        return out.to(DEV)

    # packed weights: wf[n][(ky*ks+kx)*cs_in + ci]
    wp = torch.zeros(cout, kp, dtype=tdt)
    for ky in range(ks):
        for kx in range(ks):
            base = (ky * ks + kx) * csi
            wp[:, base:base + cin] = w[:, ky, kx, :].to(tdt)
    dx, dw = nhwc(x, csi), wp.to(DEV)
    dwf = None
    if fm:   # the fragment-major image (w_frag): 16 x 32 blocks in MFMA lane order; w = zeros, so a
        # kernel reading w instead of w_frag fails the float64 comparison
        npad = (cout + 15) // 16 * 16
        wpad = torch.zeros(npad, kp, dtype=tdt, device=DEV)
        wpad[:cout] = dw
        dwf = wpad.view(npad // 16, 16, kp // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
        dw = torch.zeros_like(dw)
    dy = nhwc(yold, cso) if acc else torch.zeros(M, cso, dtype=tdt, device=DEV)
    dres, dex = nhwc(res, cso), nhwc(ex, cso)      # 1-row placeholders when unused
    db = bvec.float().to(DEV)

    # BN statistics for the prologue / dgrad epilogue, as sharded fp64 sums
    def bn_src(t, C_):
        sh = stat_shards(M)
        s1 = t.sum(0)
        s2 = (t * t).sum(0)
        sums = torch.zeros(sh, 2, C_, dtype=torch.float64)
        sums[0, 0], sums[0, 1] = s1, s2   # shard 0 holds everything, others zero
        gam = (torch.rand(C_, generator=g, dtype=torch.float64) + 0.5).float().double()
        bet = (torch.randn(C_, generator=g, dtype=torch.float64) * 0.3).float().double()
        dsums = sums.to(DEV)
        dg, dbt = gam.float().to(DEV), bet.float().to(DEV)
        src = BNSrc(dsums.data_ptr(), float(M), None, None, dg.data_ptr(), dbt.data_ptr(), EPS, sh)
        mean = s1 / M
        var = (s2 / M - mean * mean).clamp_min(0)
        rstd = (1.0 / torch.sqrt(var + EPS)).float().double()
        return src, (dsums, dg, dbt), gam, bet, mean, rstd

    keep = []
    a = ConvArgs()
    a.dtype = 0 if dtype == "fp32" else 1
    a.B, a.H, a.W, a.ks = B, H, W, ks
    a.x, a.cs_in, a.cin = dx.data_ptr(), csi, cin
    a.w, a.kp = dw.data_ptr(), kp
    a.w_frag = dwf.data_ptr() if dwf is not None else None
    a.y, a.cs_out, a.n = dy.data_ptr(), cso, cout
    a.bias = db.data_ptr() if bias else None
    a.residual = dres.data_ptr() if residual else None
    a.accumulate = int(acc)
    act = x
    if pro:
        src, k1, gam, bet, mean, rstd = bn_src(x, cin)
        keep.append(k1)
        a.pro_bn_relu, a.pro = 1, src
        # the kernels form fp32 scale/shift, then round act to the operand type
        scale = (gam * rstd).float().double()
        shift = (bet - mean.float().double() * gam * rstd).float().double()
        act = rnd(torch.relu(x * scale + shift))
    sh = stat_shards(M)
    osums = torch.zeros(sh, 2, cout, dtype=torch.float64, device=DEV)
    if stats and not dgrad:
        a.out_sums = osums.data_ptr()
    if dgrad:
        src, k2, egam, ebet, emean, erstd = bn_src(ex, cout)
        keep.append(k2)
        a.epi_relu_bn_bwd, a.epi_x, a.epi, a.epi_sums = 1, dex.data_ptr(), src, osums.data_ptr()
    ws = splitk_workspace(DEV, 8 * M * max(cso, csi) if M <= 16384 else 1)
    a.ws, a.ws_elems = ws.data_ptr(), ws.numel()
    a.variant = variant
    L = _lib.lib()
    L.conv2d(C.byref(a), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    full = dy.float().cpu()
    got = full.double()[:, :cout]
    assert torch.count_nonzero(full[:, cout:]) == 0, "channel padding must stay zero"

    # float64 reference
    if rows is None:
        a4 = act.reshape(B, H, W, cin).permute(0, 3, 1, 2)
        w4 = w.permute(0, 3, 1, 2)
        ref = torch.nn.functional.conv2d(a4, w4, bias=bvec, padding=ks // 2).permute(0, 2, 3, 1).reshape(M, cout)
        sel = slice(None)
    else:
        sel = rows
        pb, rem = rows // (H * W), rows % (H * W)
        py, px = rem // W, rem % W
        ref = bvec.view(1, -1).expand(len(rows), cout).clone()
        for ky in range(ks):
            for kx in range(ks):
                yy, xx = py + ky - ks // 2, px + kx - ks // 2
                ok = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
                src = (pb * H + yy.clamp(0, H - 1)) * W + xx.clamp(0, W - 1)
                ref = ref + (act[src] * ok.view(-1, 1).double()) @ w[:, ky, kx, :].T
    if residual:
        ref = ref + res[sel]
    if acc:
        ref = ref + yold[sel]
    s1 = s2 = None
    out = ref if rows is None else got
    if dgrad:
        escale = (egam * erstd).float().double()
        eshift = (ebet - emean.float().double() * egam * erstd).float().double()
        ref = ref * ((ex[sel] * escale + eshift) > 0)
        out = ref if rows is None else got
        xhat = (ex - emean.float().double()) * erstd
        s1, s2 = out.sum(0), (out * xhat).sum(0)
    elif stats:
        s1, s2 = out.sum(0), (out * out).sum(0)
    sums = osums.sum(0).cpu() if (stats or dgrad) else None
    if rows is not None:
        got = got[rows]
    return got, ref, sums, s1, s2


CASES = [
    # name, B, H, W, cin, cout, ks, flags            (kernel family at this size)
    ("s5_3x3_pro_stats", 8, 4, 4, 512, 512, 3, dict(pro=True, stats=True, bias=False)),   # deep-K, 32-pixel tiles
    ("s5_1x1_pro_res", 8, 4, 4, 512, 512, 1, dict(pro=True, residual=True, stats=True)),
    ("s5_in_3x3", 8, 4, 4, 97, 512, 3, dict(stats=True)),                                 # cin 97 (cs 104)
    ("s5_out_1x1", 8, 4, 4, 512, 96, 1, dict(pro=True)),
    ("s5_skip_acc", 8, 4, 4, 512, 512, 1, dict(acc=True, stats=True)),
    ("s5_3x3_dgrad", 8, 4, 4, 512, 512, 3, dict(dgrad=True, bias=False)),
    ("s4_3x3_dgrad_res_acc", 16, 8, 8, 256, 256, 3, dict(dgrad=True, residual=True, acc=True, bias=False)),
    ("s3_3x3_pro_stats", 16, 16, 16, 128, 128, 3, dict(pro=True, stats=True)),            # deep-K, 64-pixel tiles
    ("s3_1x1_odd", 4, 16, 16, 120, 200, 1, dict(pro=True, stats=True)),                   # ragged N / K
    ("s2_3x3_stream", 4, 32, 32, 64, 64, 3, dict(pro=True, stats=True)),                  # streaming kernel
    ("s1_in_3x3_stream", 2, 64, 64, 7, 32, 3, dict(stats=True)),
    ("big_m_n128", 8, 64, 64, 64, 128, 3, dict(pro=True, stats=True)),                    # LDS-tiled kernel
    # band kernel (M >= 32768, cs_in <= 64, N <= 64)
    ("s2_3x3_band", 32, 32, 32, 64, 64, 3, dict(pro=True, stats=True)),
    ("s1_3x3_band_dgrad", 8, 64, 64, 32, 32, 3, dict(dgrad=True, residual=True, acc=True, bias=False)),
    ("s1_1x1_band_res", 8, 64, 64, 32, 32, 1, dict(pro=True, residual=True, stats=True)),
    ("s1_in_band", 8, 64, 64, 7, 32, 3, dict(stats=True)),
    ("s1_out_band", 8, 64, 64, 32, 6, 1, dict(pro=True)),
    ("s2_1x1_band_odd", 32, 32, 32, 60, 40, 1, dict(pro=True, stats=True)),
    ("band_ragged_m", 9, 61, 61, 24, 16, 3, dict(pro=True, stats=True)),                 # M % 256 != 0, odd W
    # the persistent band kernel (bf16, 17-64 outputs, 32k <= M < 2^21): a
    # partial last band, odd / non-power-of-2 widths (halo crossing rows), N
    # not a multiple of 16 (zeroed padding channels, sums for n < N)
    ("band2_ragged_n24", 9, 61, 61, 24, 24, 3, dict(pro=True, stats=True)),
    ("band2_ragged_n40", 9, 61, 61, 24, 40, 3, dict(pro=True, stats=True)),
    ("band2_dgrad_res_acc_ragged", 9, 61, 61, 40, 40, 3, dict(dgrad=True, residual=True, acc=True, bias=False)),
    ("band2_w48_n20_cs16", 16, 48, 48, 13, 20, 3, dict(pro=True, stats=True)),
    # config 3's widest convs (mid 1024 at 2x2 / 4x4)
    ("c3_1024_3x3_pro_stats", 16, 2, 2, 1024, 1024, 3, dict(pro=True, stats=True, bias=False)),
    ("c3_1024_1x1_pro_res", 16, 4, 4, 1024, 1024, 1, dict(pro=True, residual=True, stats=True)),
    ("c3_1024_3x3_dgrad", 16, 2, 2, 1024, 1024, 3, dict(dgrad=True, bias=False)),
    ("c3_1024_out_1x1", 16, 2, 2, 1024, 192, 1, dict(pro=True)),
    # config 1 at its benchmarked batch: scale-1 shapes, M = 64*64*64 = 262,144
    ("c1_full_in_3x3", 64, 64, 64, 7, 32, 3, dict(stats=True)),
    ("c1_full_3x3_pro_stats", 64, 64, 64, 32, 32, 3, dict(pro=True, stats=True, bias=False)),
    ("c1_full_1x1_pro", 64, 64, 64, 32, 32, 1, dict(pro=True, stats=True, bias=False)),
    ("c1_full_1x1_res", 64, 64, 64, 32, 32, 1, dict(pro=True, residual=True, stats=True)),
    ("c1_full_skip_acc", 64, 64, 64, 32, 32, 1, dict(acc=True, stats=True)),
    ("c1_full_out_1x1", 64, 64, 64, 32, 6, 1, dict(pro=True)),
    ("c1_full_3x3_dgrad", 64, 64, 64, 32, 32, 3, dict(dgrad=True, residual=True, acc=True, bias=False)),
    ("c1_full_1x1_dgrad", 64, 64, 64, 32, 32, 1, dict(dgrad=True, bias=False)),
    ("c1_full_in_dgrad", 64, 64, 64, 32, 7, 3, dict(bias=False)),
    # 3x3 shapes of the band family and the 1x1 stream family (conv_s1.hip):
    # ragged channel counts, N < 16, every epilogue stream mix,
    # an image height that is not a multiple of the 4-row iteration
    ("st3_w32_odd", 16, 32, 32, 40, 48, 3, dict(pro=True, stats=True)),
    ("st3_w64_n6", 8, 64, 64, 32, 6, 3, dict(pro=True)),
    ("st3_w32_cs16", 16, 32, 32, 13, 24, 3, dict(stats=True)),
    ("st3_h37_res", 7, 37, 64, 32, 32, 3, dict(pro=True, stats=True, residual=True)),
    ("st3_w32_dgrad_res", 16, 32, 32, 64, 64, 3, dict(dgrad=True, residual=True, bias=False)),
    ("st1_odd", 16, 32, 32, 40, 48, 1, dict(pro=True, residual=True, stats=True)),
    ("st1_acc", 8, 64, 64, 32, 32, 1, dict(acc=True, stats=True)),
    ("st1_n6", 8, 64, 64, 32, 6, 1, dict(pro=True)),
    ("st1_dgrad_res_acc", 8, 64, 64, 32, 32, 1, dict(dgrad=True, residual=True, acc=True, bias=False)),
    ("st1_ragged_m", 5, 61, 61, 24, 16, 1, dict(pro=True, stats=True)),
    # config 4's widest convs: scale 6 of the 128x128 / 6-scale / D64 flow, mid
    # 2048 at 4x4 (beyond the deep family's 1024-channel table: generic path)
    ("c4_s6_3x3_pro_stats", 16, 4, 4, 2048, 2048, 3, dict(pro=True, stats=True, bias=False)),
    ("c4_s6_3x3_plain", 16, 4, 4, 2048, 2048, 3, dict(stats=True, bias=False)),
    ("c4_s6_1x1_pro_res", 16, 4, 4, 2048, 2048, 1, dict(pro=True, residual=True, stats=True)),
    ("c4_s6_1x1_plain", 16, 4, 4, 2048, 2048, 1, dict(stats=True)),
    ("c4_s6_skip_acc", 16, 4, 4, 2048, 2048, 1, dict(acc=True, stats=True)),
    ("c4_s6_3x3_dgrad", 16, 4, 4, 2048, 2048, 3, dict(dgrad=True, bias=False)),
    ("c4_s6_1x1_dgrad_res", 16, 4, 4, 2048, 2048, 1, dict(dgrad=True, residual=True, bias=False)),
    ("c4_s6_3x3_plain_dgrad", 16, 4, 4, 2048, 2048, 3, dict(bias=False)),
    ("c4_s6_in_3x3", 16, 4, 4, 193, 2048, 3, dict(stats=True)),
    ("c4_s6_out_1x1", 16, 4, 4, 2048, 192, 1, dict(pro=True)),
    ("c4_s6_1x1_full_batch", 256, 4, 4, 2048, 2048, 1, dict(pro=True, stats=True)),
]

# config 4 scale 1 at its per-GPU batch (B = 256, 128 x 128: M = 2^22), mid 64;
# float64 reference on 4,096 sampled output pixels (run_case rows=)
C4_S1 = [
    ("c4_s1_in_3x3", 256, 128, 128, 7, 64, 3, dict(stats=True)),
    ("c4_s1_3x3_pro_stats", 256, 128, 128, 64, 64, 3, dict(pro=True, stats=True, bias=False)),
    ("c4_s1_1x1_pro_res", 256, 128, 128, 64, 64, 1, dict(pro=True, residual=True, stats=True)),
    ("c4_s1_skip_acc", 256, 128, 128, 64, 64, 1, dict(acc=True, stats=True)),
    ("c4_s1_out_1x1", 256, 128, 128, 64, 6, 1, dict(pro=True)),
    ("c4_s1_3x3_dgrad", 256, 128, 128, 64, 64, 3, dict(dgrad=True, residual=True, acc=True, bias=False)),
    ("c4_s1_1x1_dgrad", 256, 128, 128, 64, 64, 1, dict(dgrad=True, bias=False)),
]


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", C4_S1, ids=[c[0] for c in C4_S1])
def test_conv_c4_scale1_sampled(case, dtype):
    name, B, H, W, cin, cout, ks, fl = case
    M = B * H * W
    rows = torch.from_numpy(np.random.default_rng(7).choice(M, 4096, replace=False)).long()
    rows = torch.cat([rows, torch.tensor([0, W - 1, M - W, M - 1])])   # image corners (padding taps)
    got, ref, sums, s1, s2 = run_case(B, H, W, cin, cout, ks, dtype, rows=rows, **fl)
    tol = 1e-5 if dtype == "fp32" else 4e-3
    assert rel(got, ref) < tol, rel(got, ref)
    if s1 is not None:     # the epilogue's sums against the float64 sums of its own output
        stol = 1e-5 if dtype == "fp32" else 10 * tol    # bf16: sums of the unrounded values
        assert rel(sums[0], s1) < stol, rel(sums[0], s1)
        assert rel(sums[1], s2) < stol, rel(sums[1], s2)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_conv_vs_float64(case, dtype):
    name, B, H, W, cin, cout, ks, fl = case
    got, ref, sums, s1, s2 = run_case(B, H, W, cin, cout, ks, dtype, **fl)
    tol = 1e-5 if dtype == "fp32" else 4e-3
    assert rel(got, ref) < tol, rel(got, ref)
    if s1 is not None:
        assert rel(sums[0], s1) < 10 * tol, rel(sums[0], s1)
        assert rel(sums[1], s2) < 10 * tol, rel(sums[1], s2)


DEEP = [c for c in CASES if c[0].startswith(("s5", "s4", "s3", "c3_"))]


@pytest.mark.parametrize("case", DEEP, ids=[c[0] for c in DEEP])
def test_conv_variants_agree(case):
    """the small-pixel-count kernel families (halo tile: default; LDS-tiled
    split-K + reduce launch: variant 1) give the same fp32 result"""
    name, B, H, W, cin, cout, ks, fl = case
    a, ref, _, _, _ = run_case(B, H, W, cin, cout, ks, "fp32", variant=0, **fl)
    b, _, _, _, _ = run_case(B, H, W, cin, cout, ks, "fp32", variant=1, **fl)
    assert rel(a, b) < 2e-6
    assert rel(b, ref) < 1e-5


BAND = [c for c in CASES if "band" in c[0]]


@pytest.mark.parametrize("case", BAND, ids=[c[0] for c in BAND])
def test_band_matches_stream(case):
    """band kernel (default at the wide scales) vs the register-streaming
    kernel (variant 1), fp32"""
    name, B, H, W, cin, cout, ks, fl = case
    a, ref, _, _, _ = run_case(B, H, W, cin, cout, ks, "fp32", variant=0, **fl)
    b, _, _, _, _ = run_case(B, H, W, cin, cout, ks, "fp32", variant=1, **fl)
    assert rel(a, b) < 2e-6
    assert rel(b, ref) < 1e-5


@pytest.mark.parametrize("case", BAND, ids=[c[0] for c in BAND])
def test_band_bf16_matches_generic(case):
    """bf16: the default wide-scale 3x3 path (the persistent band kernel where
    it applies) vs the generic LDS-tiled kernel (variant 1), both against the
    float64 restatement"""
    name, B, H, W, cin, cout, ks, fl = case
    a, ref, _, _, _ = run_case(B, H, W, cin, cout, ks, "bf16", variant=0, **fl)
    b, _, _, _, _ = run_case(B, H, W, cin, cout, ks, "bf16", variant=1, **fl)
    assert rel(a, ref) < 4e-3 and rel(b, ref) < 4e-3, (rel(a, ref), rel(b, ref))
    assert rel(a, b) < 6e-3, rel(a, b)


# deep-scale family (conv_deep.hip): every configuration against the float64
# restatement, both dtypes; configurations that do not apply to a shape
# (channel stride not a multiple of the k-step, LDS too small) are skipped
DEEP_FAMILY = DEEP + [
    ("s3_1x1_pro_stats", 64, 16, 16, 128, 128, 1, dict(pro=True, stats=True)),
    ("s3_3x3_dgrad_res", 16, 16, 16, 128, 128, 3, dict(dgrad=True, residual=True, bias=False)),
    ("s4_1x1_skip_acc", 16, 8, 8, 256, 256, 1, dict(acc=True, stats=True)),
    ("s4_3x3_ragged_m", 3, 7, 9, 256, 200, 3, dict(pro=True, stats=True)),                # M % 64 != 0, N % 64 != 0
    ("s2_1x1_64", 8, 32, 32, 64, 64, 1, dict(pro=True, residual=True, stats=True)),
]
DEEP_CFGS = 7
VARIANT_DEEP0 = 16


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("cfg", range(DEEP_CFGS))
@pytest.mark.parametrize("case", DEEP_FAMILY, ids=[c[0] for c in DEEP_FAMILY])
def test_deep_family_vs_float64(case, cfg, dtype):
    name, B, H, W, cin, cout, ks, fl = case
    try:
        got, ref, sums, s1, s2 = run_case(B, H, W, cin, cout, ks, dtype, variant=VARIANT_DEEP0 + cfg, **fl)
    except RuntimeError as e:
        if "unsupported" in str(e):
            pytest.skip("configuration %d does not apply" % cfg)
        raise
    tol = 1e-5 if dtype == "fp32" else 4e-3
    assert rel(got, ref) < tol, rel(got, ref)
    if s1 is not None:
        assert rel(sums[0], s1) < 10 * tol, rel(sums[0], s1)
        assert rel(sums[1], s2) < 10 * tol, rel(sums[1], s2)


# fragment-major weight images (rnvp_conv_args.w_frag, bf16 deep tiles): the
# same MFMAs in the same order from another weight layout -- bitwise equal
# outputs to the row-major image, every configuration (w itself is zeros in
# the w_frag run: a kernel that read it would miss the float64 reference)
@pytest.mark.parametrize("cfg", range(DEEP_CFGS))
@pytest.mark.parametrize("case", DEEP_FAMILY, ids=[c[0] for c in DEEP_FAMILY])
def test_deep_frag_major_weights(case, cfg):
    name, B, H, W, cin, cout, ks, fl = case
    if (cin + 7) // 8 * 8 // ((4, 4, 1, 2, 8, 8, 4)[cfg] * 32) > 4:
        pytest.skip("no fragment-major kernel beyond 4 channel chunks per wave (the row-major image is used)")
    try:
        a = run_case(B, H, W, cin, cout, ks, "bf16", variant=VARIANT_DEEP0 + cfg, **fl)
    except RuntimeError as e:
        if "unsupported" in str(e):
            pytest.skip("configuration %d does not apply" % cfg)
        raise
    b = run_case(B, H, W, cin, cout, ks, "bf16", variant=VARIANT_DEEP0 + cfg, fm=True, **fl)
    assert torch.equal(a[0], b[0])
    if a[2] is not None:
        assert torch.allclose(a[2], b[2], rtol=1e-12, atol=1e-9)
    assert rel(b[0], b[1]) < 4e-3
