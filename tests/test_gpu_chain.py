"""Persistent net chain (rnvp_net_chain, csrc/net_chain.hip) against the same
steps launched one by one.

The chain runs each step's tiles with the same per-tile bodies as the
standalone launches (conv_deep.h / bn_bwd_body), so a chained forward and
backward must reproduce the per-launch results up to the order of the fp64
BatchNorm-sum atomics: checked on the deep-scale couplings of config 1
(scale-4 channelwise, scale-5 checkerboard: the chained shapes) in fp32 and
bf16, on the whole config-1 training step at B = 64 (the benchmarked path),
and through the C ABI on a hand-built two-conv chain.  The barrier words must
come back clean (no time-out abort).
"""
import ctypes as C

import numpy as np
import pytest
import torch

from formula_init import formula_state

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _hp(bd, rb):
    import utils
    return utils.Hyperparameters(bd, rb, True, True, True, True)


def rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _barriers_clean():
    from realnvp_hip import engine
    for t in engine._BARRIERS.values():
        w = t.cpu().tolist()
        assert w[2] == 0, "net chain barrier timed out: %s" % w[:4]
        assert w[0] == 0, "net chain barrier count left non-zero: %s" % w[:4]


def _run_coupling(kind, cio, mid, size, B, dtype, chain, seed=0):
    import modules_realnvp as MR
    from realnvp_hip import engine
    old = engine.NET_CHAIN
    engine.NET_CHAIN = int(chain)
    try:
        torch.manual_seed(seed)
        hp = _hp(32, 4)
        mod = MR.CheckerboardAffineCoupling(cio, mid, size, 1.0, hp) if kind == "ckbd" else \
            MR.ChannelwiseAffineCoupling(cio, mid, 0.0, hp)
        mod.load_state_dict(formula_state(mod, style="chirp"))
        mod = mod.to(DEV).train()
        mod.compute_dtype = dtype
        g = torch.Generator().manual_seed(seed + 1)
        x = torch.randn(B, cio, size, size, generator=g).to(DEV).requires_grad_(True)
        gy = torch.randn(B, cio, size, size, generator=g).to(DEV)
        gl = torch.randn(B, cio, size, size, generator=g).to(DEV)
        y, ldj = mod(x)
        (y * gy + ldj * gl).sum().backward()
        torch.cuda.synchronize()
        grads = {n: p.grad.clone() for n, p in mod.named_parameters() if p.grad is not None}
        return y.detach(), ldj.detach(), x.grad.clone(), grads, mod.engine()
    finally:
        engine.NET_CHAIN = old


DEEP = [
    # config 1 scale-5 checkerboard (4x4, 48 channels, mid 512), scale-4
    # channelwise (4x4, 96 channels, mid 512): M = 1024; scale-4 checkerboard
    # (8x8, 24 channels, mid 256): M = 4096.  The single launches use other
    # tile configurations than the chain (8-wave tiles, grouped skip convs:
    # another fp32 summation order), so the ReLU-kink floor of the data
    # gradient, ~1e-3, applies
    ("s5_ckbd", "ckbd", 48, 512, 4, 3e-3),
    ("s4_chan", "chan", 96, 512, 4, 3e-3),
    ("s4_ckbd", "ckbd", 24, 256, 8, 3e-3),
]


@pytest.mark.parametrize("case", DEEP, ids=[c[0] for c in DEEP])
def test_chain_coupling_matches_single_launches(case):
    _, kind, cio, mid, size, tol = case
    y0, l0, gx0, g0, _ = _run_coupling(kind, cio, mid, size, 64, "fp32", chain=False)
    y1, l1, gx1, g1, eng = _run_coupling(kind, cio, mid, size, 64, "fp32", chain=True)
    _barriers_clean()
    assert rel(y1, y0) < 1e-6 and rel(l1, l0) < 1e-6, (rel(y1, y0), rel(l1, l0))
    assert rel(gx1, gx0) < tol, rel(gx1, gx0)
    # biases of convs that feed only a BatchNorm (in_skip, core_skips: their
    # sum goes through out_bn) have a zero gradient in exact arithmetic, so
    # theirs is rounding noise: errors are measured against the largest norm
    gmax = max(float(g0[n].norm()) for n in g0)
    worst = max((float((g1[n] - g0[n]).norm()) / (float(g0[n].norm()) + 1e-3 * gmax), n) for n in g0)
    assert worst[0] < 10 * tol, worst


def test_chain_is_used_at_the_deep_scales():
    """the engine plans chains for the scale-5 coupling: forward 18 convs ->
    one chain (the in-conv's 97-channel operand is not chainable), backward
    one chain over all but the first data gradient"""
    from realnvp_hip import engine
    _, _, _, _, eng = _run_coupling("ckbd", 48, 512, 4, 64, "fp32", chain=True)
    svs = [sv for pool in eng._saved_pool.values() for sv in pool]
    assert svs, "no saved arena"
    # (grouped launches of independent 1x1 convs are planned first; the chain
    # takes the rest)
    fwd = svs[0]["fwd_plan"][2]
    covered = sum(gr[2] - gr[1] for gr in fwd if gr[0] in ("chain", "group"))
    assert covered == 18 and any(gr[0] == "chain" for gr in fwd), [g[:3] for g in fwd]
    bwd = svs[0]["bwd_plan"][2]
    nb = sum(gr[2] - gr[1] for gr in bwd if gr[0] in ("chain", "group"))
    assert nb >= 28 and any(gr[0] == "chain" for gr in bwd), [g[:3] for g in bwd]


def test_chain_trainer_step_config1():
    """the benchmarked step (config 1, B = 64) with and without chains: fp32
    per-sample log-prob and the whole gradient arena agree, bf16 within its
    rounding (the chained bf16 tiles round exactly as the single launches;
    only the fp64 sum order differs)."""
    import flow_realnvp
    from realnvp_hip import engine
    from realnvp_hip.trainer import FlowTrainer
    from test_gpu_deep import make_model, model_inputs
    out = {}
    for dtype in ("fp32", "bf16"):
        for chain in (0, 1):
            old = engine.NET_CHAIN
            engine.NET_CHAIN = chain
            try:
                model = make_model(64, 32, 4)
                tr = FlowTrainer(model, 64, dtype=dtype)
                x, logdet = model_inputs(64, 64)
                tr.set_input(x.to(DEV), logdet.to(DEV))
                tr.step_eager()
                torch.cuda.synchronize()
                out[(dtype, chain)] = (tr.lp.clone(), tr.grad.clone())
            finally:
                engine.NET_CHAIN = old
    _barriers_clean()
    lp0, g0 = out[("fp32", 0)]
    lp1, g1 = out[("fp32", 1)]
    # the M = 4096 couplings' single 1x1 launches use the generic family
    # (another fp32 summation order): the ReLU-kink floor, as in the coupling test
    assert float(((lp1 - lp0).abs() / lp0.abs()).max()) < 1e-6
    assert rel(g1, g0) < 3e-3, rel(g1, g0)
    lp0, g0 = out[("bf16", 0)]
    lp1, g1 = out[("bf16", 1)]
    # bf16: the per-sample log-prob floor of two correct bf16 evaluations is
    # 4.2e-4 (test_gpu_deep.test_trainer_config1_full_batch_bf16)
    assert float(((lp1 - lp0).abs() / lp0.abs()).max()) < 5e-4
    assert rel(g1, g0) < 2e-2, rel(g1, g0)


def test_chain_c_abi_two_convs():
    """a hand-built chain through the C ABI: 1x1 (with batch sums) then a 3x3
    with the BN+ReLU prologue reading those sums, at scale-5 shape, against
    the two rnvp_conv2d launches"""
    from realnvp_hip import _lib
    from realnvp_hip._lib import BNSrc, ConvArgs, NetStep
    from realnvp_hip.engine import stat_shards, upload
    L = _lib.lib()
    B, H, W, Cc = 64, 4, 4, 512
    M = B * H * W
    torch.manual_seed(3)
    x = torch.randn(M, Cc, device=DEV)
    w1 = torch.randn(Cc, Cc, device=DEV) * 0.05
    w2 = torch.randn(Cc, 9 * Cc, device=DEV) * 0.02
    gam = torch.rand(Cc, device=DEV) + 0.5
    bet = torch.randn(Cc, device=DEV) * 0.1
    sh = stat_shards(M)
    s = torch.cuda.current_stream().cuda_stream

    def run(chain):
        t1 = torch.zeros(M, Cc, device=DEV)
        y = torch.zeros(M, Cc, device=DEV)
        sums = torch.zeros(sh, 2, Cc, device=DEV, dtype=torch.float64)
        a1 = ConvArgs()
        a1.dtype, a1.B, a1.H, a1.W, a1.ks = 0, B, H, W, 1
        a1.x, a1.cs_in, a1.cin, a1.w, a1.kp = x.data_ptr(), Cc, Cc, w1.data_ptr(), Cc
        a1.y, a1.cs_out, a1.n = t1.data_ptr(), Cc, Cc
        a1.out_sums = sums.data_ptr()
        a2 = ConvArgs()
        a2.dtype, a2.B, a2.H, a2.W, a2.ks = 0, B, H, W, 3
        a2.x, a2.cs_in, a2.cin, a2.w, a2.kp = t1.data_ptr(), Cc, Cc, w2.data_ptr(), 9 * Cc
        a2.y, a2.cs_out, a2.n = y.data_ptr(), Cc, Cc
        a2.pro_bn_relu = 1
        a2.pro = BNSrc(sums.data_ptr(), float(M), None, None, gam.data_ptr(), bet.data_ptr(), 1e-5, sh)
        if chain:
            steps = (NetStep * 2)()
            for st, a in zip(steps, (a1, a2)):
                st.kind, st.conv, st.dgamma_off, st.dbeta_off = 0, a, -1, -1
            k, g, lb = C.c_int(), C.c_int(), C.c_int()
            rc = L.net_chain_prepare(steps, 2, C.byref(k), C.byref(g), C.byref(lb))
            assert rc == 0, rc
            assert g.value % 8 == 0 and g.value >= 256, g.value
            tab = upload(bytes(steps), DEV)
            bar = torch.zeros(16, dtype=torch.int32, device=DEV)
            L.net_chain(tab.data_ptr(), 2, 0, k.value, g.value, lb.value, None, bar.data_ptr(), s)
            torch.cuda.synchronize()
            assert bar[2].item() == 0 and bar[0].item() == 0, bar[:4].tolist()
            assert bar[1].item() == 1, bar[:4].tolist()   # one barrier between the two steps
        else:
            L.conv2d(C.byref(a1), s)
            L.conv2d(C.byref(a2), s)
        torch.cuda.synchronize()
        return t1, y, sums.sum(0)

    t0, y0, s0 = run(False)
    t1, y1, s1 = run(True)
    # the single 1x1 launch runs the 8-wave tile configuration (K split 8
    # ways), the chain's class the 4-wave one: fp32 summation order only
    assert rel(t1, t0) < 1e-6
    assert rel(s1, s0) < 1e-6
    assert rel(y1, y0) < 1e-6, rel(y1, y0)
    # and against torch: relu(bn(t1)) conv 3x3
    mean = s0[0] / M
    var = s0[1] / M - mean * mean
    a = torch.relu((t1 - mean.float()) / torch.sqrt(var.float() + 1e-5) * gam + bet)
    a = a.view(B, H, W, Cc).permute(0, 3, 1, 2)
    wt = w2.view(Cc, 3, 3, Cc).permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(a, wt, padding=1).permute(0, 2, 3, 1).reshape(M, Cc)
    assert rel(y1, ref) < 1e-4, rel(y1, ref)


def test_chain_prepare_rejects_unchainable():
    """a step outside the chain's forms (97-channel operand, M > 4096) is
    RNVP_E_UNSUPPORTED, so the engine launches it on its own"""
    from realnvp_hip import _lib
    from realnvp_hip._lib import ConvArgs, NetStep
    L = _lib.lib()
    buf = torch.empty(1 << 22, device=DEV)
    for (B, H, W, cs, ks) in [(64, 4, 4, 104, 3), (64, 16, 16, 128, 1)]:
        a = ConvArgs()
        a.dtype, a.B, a.H, a.W, a.ks = 0, B, H, W, ks
        a.x, a.cs_in, a.cin, a.w = buf.data_ptr(), cs, cs, buf.data_ptr()
        a.kp = (ks * ks * cs + 63) // 64 * 64
        a.y, a.cs_out, a.n = buf.data_ptr(), 128, 128
        steps = (NetStep * 2)()
        for st in steps:
            st.kind, st.conv = 0, a
        k, g, lb = C.c_int(), C.c_int(), C.c_int()
        assert L.net_chain_prepare(steps, 2, C.byref(k), C.byref(g), C.byref(lb)) == -2
