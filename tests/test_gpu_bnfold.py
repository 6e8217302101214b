"""BatchNorm-backward applies folded into their consumer's data-gradient
operand staging (rnvp_conv_args.bp, csrc/conv_deep.h; engine.FOLD_BN).

At the deep scales a BatchNorm's backward apply (modules_realnvp.py:36-52's
res_block.1 / res_block.4 in the backward, rnvp_bn_bwd_apply) is followed
directly by the data gradient of the conv that produced its input; the fold
computes dL/dt = gamma rstd (g - k1 - xhat k2) while that conv stages its
operand tile, stores it once for the weight gradient and writes the
BatchNorm's parameter gradients, so the apply's launch and its dL/dt round
trip disappear.

* test_bp_conv_matches_apply_then_conv: through the C ABI, the folded conv
  against rnvp_bn_bwd_apply + the plain conv on the same inputs -- output,
  side output (dL/dt), the epilogue's BatchNorm sums and the parameter
  gradients; 1x1 and 3x3, both data-gradient tile configurations, fp32 and
  bf16 (bf16 with and without the fragment-major weight image), and the wide
  scales' streaming 1x1 and band 3x3 (bf16).
* test_coupling_fold_matches_unfolded: whole deep-scale couplings (drop-in
  module, forward + backward) with the fold on and off: the fold really
  happened (fewer BatchNorm-apply launches), outputs and every gradient agree
  to rounding, and each schedule is pinned to the CPU oracle with
  test_gpu_group's allowance.
"""
import ctypes as C

import pytest
import torch

from test_gpu_group import _check_vs_oracle, _inputs, rel

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _frag_major(w):
    n, kp = w.shape
    npad = (n + 15) // 16 * 16
    wp = torch.zeros(npad, kp, dtype=w.dtype, device=w.device)
    wp[:n] = w
    return wp.view(npad // 16, 16, kp // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()


# (B, H, W, channels in (= the BatchNorm's), channels out, ks, cfg): cfg 4 =
# 8-wave tiles (M <= 1024), cfg 0 = 4-wave tiles, -1 = the tuned dispatch
# (the wide scales' streaming 1x1, conv_s1.hip)
BP_CASES = [
    (64, 4, 4, 512, 512, 1, 4),
    (64, 4, 4, 512, 512, 3, 4),
    (64, 8, 8, 256, 256, 3, 0),
    (64, 16, 16, 128, 128, 3, 0),
    (64, 16, 16, 128, 64, 1, 0),
    # the wide scales' streaming 1x1 and band 3x3 (tuned dispatch, bf16)
    (64, 32, 32, 64, 64, 1, -1),
    (16, 64, 64, 32, 32, 1, -1),
    (64, 32, 32, 64, 64, 3, -1),
    (16, 64, 64, 32, 32, 3, -1),
]


@pytest.mark.parametrize("frag", [False, True])
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", BP_CASES, ids=["m%d_c%d_k%d" % (c[0] * c[1] * c[2], c[3], c[5]) for c in BP_CASES])
def test_bp_conv_matches_apply_then_conv(case, dtype, frag):
    from realnvp_hip import _lib
    from realnvp_hip._lib import BNBwdArgs, BNSrc, ConvArgs
    from realnvp_hip.engine import stat_shards
    if frag and dtype == "fp32":
        pytest.skip("fragment-major weight images are bf16")
    if case[6] < 0 and (frag or dtype == "fp32"):
        pytest.skip("the streaming 1x1 / band 3x3 are bf16, row-major weights")
    L = _lib.lib()
    B, H, W, Ci, Co, ks, cfg = case
    M = B * H * W
    dt, tdt = (0, torch.float32) if dtype == "fp32" else (1, torch.bfloat16)
    torch.manual_seed(11)
    t = (torch.randn(M, Ci, device=DEV) * 1.5 + 0.3).to(tdt)          # BatchNorm input (saved activation)
    g = torch.randn(M, Ci, device=DEV).to(tdt)                          # gradient of the BatchNorm output
    ex = torch.randn(M, Co, device=DEV).to(tdt)                         # the epilogue BatchNorm's input
    kp = (ks * ks * Ci + 63) // 64 * 64
    w = torch.zeros(Co, kp, device=DEV)
    w[:, :ks * ks * Ci] = torch.randn(Co, ks * ks * Ci, device=DEV) * (1.0 / (ks * ks * Ci) ** 0.5)
    w = w.to(tdt)
    wf = _frag_major(w) if frag else None
    sh = stat_shards(M)
    td, gd = t.double(), g.double()
    tsum = torch.zeros(sh, 2, Ci, device=DEV, dtype=torch.float64)
    tsum[0, 0], tsum[0, 1] = td.sum(0), (td * td).sum(0)
    mean = tsum[0, 0] / M
    xhat = (td - mean) / torch.sqrt(tsum[0, 1] / M - mean * mean + 1e-5)
    gsum = torch.zeros(sh, 2, Ci, device=DEV, dtype=torch.float64)
    gsum[0, 0], gsum[0, 1] = gd.sum(0), (gd * xhat).sum(0)
    gam = torch.rand(Ci, device=DEV) + 0.5
    bet = torch.randn(Ci, device=DEV) * 0.1
    esum = torch.zeros(sh, 2, Co, device=DEV, dtype=torch.float64)
    esum[0, 0], esum[0, 1] = ex.double().sum(0), (ex.double() ** 2).sum(0)
    egam = torch.rand(Co, device=DEV) + 0.5
    ebet = torch.randn(Co, device=DEV) * 0.1
    s = torch.cuda.current_stream().cuda_stream
    bn = BNSrc(tsum.data_ptr(), float(M), None, None, gam.data_ptr(), bet.data_ptr(), 1e-5, sh)

    def conv(xp, y, epi_sums):
        a = ConvArgs()
        a.dtype, a.B, a.H, a.W, a.ks = dt, B, H, W, ks
        a.x, a.cs_in, a.cin, a.w, a.kp = xp, Ci, Ci, w.data_ptr(), kp
        a.w_frag = wf.data_ptr() if frag else None
        a.y, a.cs_out, a.n = y.data_ptr(), Co, Co
        a.epi_relu_bn_bwd, a.epi_x = 1, ex.data_ptr()
        a.epi = BNSrc(esum.data_ptr(), float(M), None, None, egam.data_ptr(), ebet.data_ptr(), 1e-5, sh)
        a.epi_sums = epi_sums.data_ptr()
        a.variant = 16 + cfg if cfg >= 0 else 0   # RNVP_VARIANT_DEEP0 + cfg, or the tuned dispatch
        return a

    dummy = torch.zeros(64, device=DEV)
    probe = conv(g.data_ptr(), dummy, dummy)
    probe.bp, probe.bp_x, probe.bp_bn, probe.bp_sums, probe.bp_shards = 1, t.data_ptr(), bn, gsum.data_ptr(), sh
    if dtype == "fp32" and L.conv2d_check(C.byref(probe)) == -2:
        pytest.skip("fp32 tile + the fold's table exceed the LDS (the engine keeps this apply)")
    # unfolded: apply, then the conv
    dx = torch.zeros(M, Ci, device=DEV, dtype=tdt)
    dg0, db0 = torch.zeros(Ci, device=DEV), torch.zeros(Ci, device=DEV)
    b = BNBwdArgs()
    b.dtype, b.M, b.C, b.cs = dt, M, Ci, Ci
    b.g, b.x, b.bn, b.sums, b.sum_shards = g.data_ptr(), t.data_ptr(), bn, gsum.data_ptr(), sh
    b.dx, b.dgamma, b.dbeta = dx.data_ptr(), dg0.data_ptr(), db0.data_ptr()
    L.bn_bwd_apply(C.byref(b), s)
    y0 = torch.zeros(M, Co, device=DEV, dtype=tdt)
    es0 = torch.zeros(sh, 2, Co, device=DEV, dtype=torch.float64)
    L.conv2d(C.byref(conv(dx.data_ptr(), y0, es0)), s)
    # folded
    y1 = torch.zeros(M, Co, device=DEV, dtype=tdt)
    es1 = torch.zeros(sh, 2, Co, device=DEV, dtype=torch.float64)
    side = torch.full((M, Ci), 7.0, device=DEV, dtype=tdt)
    dg1, db1 = torch.zeros(Ci, device=DEV), torch.zeros(Ci, device=DEV)
    a = conv(g.data_ptr(), y1, es1)
    a.bp, a.bp_x, a.bp_bn, a.bp_sums, a.bp_shards = 1, t.data_ptr(), bn, gsum.data_ptr(), sh
    a.bp_out, a.bp_dgamma, a.bp_dbeta = side.data_ptr(), dg1.data_ptr(), db1.data_ptr()
    assert L.conv2d_check(C.byref(a)) == 0
    L.conv2d(C.byref(a), s)
    torch.cuda.synchronize()
    assert torch.equal(dg1, dg0) and torch.equal(db1, db0)
    # the fold evaluates the apply as A g - (B t + C) (three coefficients per
    # channel, fp64-formed): fp32 rounding differences, which a bf16 store
    # turns into one-ulp flips at a few elements
    tol = 1e-5 if dtype == "fp32" else 2e-3
    # (the epilogue's sums compared over shards: a launch's shard of a
    # workgroup follows its grid, which the fold may change)
    r_side, r_y, r_e = rel(side.float(), dx.float()), rel(y1.float(), y0.float()), rel(es1.sum(0), es0.sum(0))
    frac = float((side != dx).float().mean())
    print("side %.3g (%.2g%% differ)  y %.3g  epi sums %.3g" % (r_side, 100 * frac, r_y, r_e))
    assert r_side < tol and r_y < tol and r_e < tol
    if dtype == "bf16":
        assert frac < 1e-2
    # and the truth: torch's BatchNorm backward formula in float64
    k1, k2 = gsum[0, 0] / M, gsum[0, 1] / M
    rstd = 1.0 / torch.sqrt(tsum[0, 1] / M - mean * mean + 1e-5)
    ref = gam.double() * rstd * (gd - k1 - xhat * k2)
    assert rel(side.double(), ref) < (1e-5 if dtype == "fp32" else 1e-2)


DEEP_CASES = [
    # name, kind, in_out_dim, mid, size, batch (as test_gpu_group)
    ("s5_ckbd_m1024", "ckbd", 48, 512, 4, 64),
    ("s4_chan_m1024", "chan", 96, 512, 4, 64),
    ("s4_ckbd_m4096", "ckbd", 24, 256, 8, 64),
    ("s3_ckbd_m16384", "ckbd", 12, 128, 16, 64),
    # wide scales: the streaming 1x1 and band 3x3 data gradients fold (bf16)
    ("s2_ckbd_m65536", "ckbd", 6, 64, 32, 64),
    ("s1_ckbd_m65536", "ckbd", 3, 32, 64, 16),
]


def _run(case, dtype, fold):
    from realnvp_hip import engine
    _, kind, cio, mid, size, B = case
    old = engine.FOLD_BN
    engine.FOLD_BN = fold
    try:
        mod, x, gy, gl = _inputs(kind, cio, mid, size, B)
        mod = mod.to(DEV).train()
        mod.compute_dtype = dtype
        x = x.to(DEV).requires_grad_(True)
        y, ldj = mod(x)
        (y * gy.to(DEV) + ldj * gl.to(DEV)).sum().backward()
        torch.cuda.synchronize()
        grads = {n: p.grad.clone() for n, p in mod.named_parameters() if p.grad is not None}
        eng = mod.engine()
        sv = [sv for pool in eng._saved_pool.values() for sv in pool][0]
        items = sv["bwd_plan"][1][0]
        n_apply = sum(it[0] == "bn" for it in items)
        n_fold = sum(it[0] == "dgrad" and it[4] is not None for it in items)
        return (y.detach(), ldj.detach(), x.grad.clone(), grads), n_apply, n_fold
    finally:
        engine.FOLD_BN = old


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", DEEP_CASES, ids=[c[0] for c in DEEP_CASES])
def test_coupling_fold_matches_unfolded(case, dtype):
    r0, a0, f0 = _run(case, dtype, False)
    r1, a1, f1 = _run(case, dtype, True)
    assert f0 == 0 and a1 == a0 - f1, (a0, a1, f1)
    # per residual block (4), deep scales: res_block.4 into the 3x3's data
    # gradient, and res_block.1 into the first 1x1's up to 4096 pixels (the
    # tuned dispatch keeps the apply before the 16384-pixel 1x1 tiles); fp32 3x3
    # tiles at 512 channels exceed the LDS with the fold's table
    _, _, _, mid, size, B = case
    M = B * size * size
    small = M <= 1024
    if M > 16384:   # wide: res_block.1 / .4 into the streaming 1x1 / band 3x3 (bf16 only)
        want = 8 if dtype == "bf16" else 0
    else:
        want = 4 * (int(M <= 4096) + int(not (small and dtype == "fp32")))
    assert f1 == want, (f1, want)
    y0, l0, gx0, g0 = r0
    y1, l1, gx1, g1 = r1
    assert torch.equal(y0, y1) and torch.equal(l0, l1)   # the forward is untouched
    tol = 1e-4 if dtype == "fp32" else 3e-2
    worst = max([rel(gx1, gx0)] + [rel(g1[n], g0[n]) for n in g0 if float(g0[n].norm()) > 0])
    print("largest folded-vs-unfolded gradient difference %.3g" % worst)
    for r in (r0, r1):
        _check_vs_oracle(case, dtype, r)
    assert rel(gx1, gx0) < tol
