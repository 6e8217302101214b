"""Grouped launches of independent 1x1 convs (rnvp_net_group, csrc/conv_deep.hip)
against the same convs launched one by one (engine.NET_GROUP = False).

The engine groups each core_skips[i] forward with the next block's first 1x1
and the data gradients of in_skip + every core_skips[i]
(modules_realnvp.py:175-194).  A grouped tile runs the same deep_tile body as
the single launch, in the configuration its first conv would get alone
(rnvp_deep_auto_cfg, so the dispatch knobs reach groups too), so forward
outputs, the data gradient and every parameter gradient must agree up to
summation order: checked on bottleneck+skip couplings at M = 256, 1024,
4096 and 16384 pixels (both sides of the 8-wave / 4-wave boundary at 1024 and
the deep family's 16384-pixel limit), fp32 and bf16, the wide scales' fan-out
launches (M = 65536, bf16: one input tile feeds every member), and through
the C ABI.
"""
import ctypes as C

import numpy as np

import pytest
import torch

from formula_init import formula_state

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _inputs(kind, cio, mid, size, B, seed=0):
    """the coupling module (formula weights, chirp style) and its x, gy, gl on the host"""
    import modules_realnvp as MR
    import utils
    torch.manual_seed(seed)
    hp = utils.Hyperparameters(32, 4, True, True, True, True)
    mod = MR.CheckerboardAffineCoupling(cio, mid, size, 1.0, hp) if kind == "ckbd" else \
        MR.ChannelwiseAffineCoupling(cio, mid, 0.0, hp)
    mod.load_state_dict(formula_state(mod, style="chirp"))
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(B, cio, size, size, generator=g)
    gy = torch.randn(B, cio, size, size, generator=g)
    gl = torch.randn(B, cio, size, size, generator=g)
    return mod, x, gy, gl


_ORACLE = {}


def _oracle(case, mode, training=True, reverse=False):
    """The CPU oracle of the same coupling step: mode "f64" (the truth),
    "f32" (the reference's own precision), "emu" / "emu_wide" (the engine's
    bf16 rounding points, fp32 / fp64 conv accumulation); training / reverse
    as the coupling's own arguments.  Returns (y, ldj, dL/dx, {name:
    gradient}) in float64."""
    key = (case, mode, training, reverse)
    if key not in _ORACLE:
        import realnvp_oracle as O
        from realnvp_bf16emu import Emu, _R
        _, kind, cio, mid, size, B = case
        mod, x, gy, gl = _inputs(kind, cio, mid, size, B)
        dt = torch.float64 if mode == "f64" else torch.float32
        S = {k: (v.to(dt) if v.is_floating_point() else v) for k, v in mod.state_dict().items()}
        names = [n for n, p in mod.named_parameters() if p.requires_grad]
        for n in names:
            S[n].requires_grad_(True)
        hp = O.HP(32, 4)
        saved = O.residual_module
        if mode.startswith("emu"):
            emu = Emu(mode == "emu_wide")
            O.residual_module = lambda S_, p, h, tr, rb, bn, sk: emu.module(S_, p, _R.apply(h), tr, hp)
        try:
            xx = x.to(dt).requires_grad_(True)
            fn = O.checkerboard_coupling if kind == "ckbd" else O.channelwise_coupling
            y, ldj = fn(S, "", xx, 1.0 if kind == "ckbd" else 0.0, hp, training=training, reverse=reverse)
            grads = torch.autograd.grad((y * gy.to(dt) + ldj * gl.to(dt)).sum(), [xx] + [S[n] for n in names],
                                        allow_unused=True)
        finally:
            O.residual_module = saved
        gd = {n: (g if g is not None else torch.zeros_like(S[n])).detach().double() for g, n in zip(grads[1:], names)}
        _ORACLE[key] = (y.detach().double(), ldj.detach().double(), grads[0].double(), gd)
    return _ORACLE[key]


def _check_vs_oracle(case, dtype, got, training=True, reverse=False):
    """Every gradient tensor and dL/dx of one launch schedule against the
    oracle, with test_deep_coupling_vs_reference's allowance: fp32 -- within
    5e-3 of the float64 truth or 3x the fp32 reference's own error, at most
    5 % of the tensors beyond (ReLU-kink decisions), none 10x; bf16 -- the
    bf16 emulation as the target and twice the largest scatter of the three
    CPU references (fp32 oracle, emulation with fp32 / fp64 conv sums: the
    engine keeps the BN statistics of the unrounded conv outputs, the
    emulation those of the stored bf16 values) as the allowance, the rule of
    test_trainer_config1_full_batch_bf16, same exception rule.
    Zero-expectation gradients (a bias feeding a BatchNorm) are measured
    against 1e-3 (bf16: 1e-2) of the largest gradient norm."""
    y, ldj, gx, grads = got
    o = lambda mode: _oracle(case, mode, training, reverse)  # noqa: E731
    if dtype == "fp32":
        tgt, others, k, floor = o("f64"), [o("f32")], 3.0, 1e-3
    else:
        tgt, others, k, floor = o("emu"), [o("emu_wide"), o("f32")], 2.0, 1e-2
    ty, tl, tgx, tg = tgt
    gmax = max(float(v.norm()) for v in tg.values())
    ratio, info = [], []
    pairs = [("dL/dx", gx, tgx, [o[2] for o in others])] + [(n, grads[n], tg[n], [o[3][n] for o in others])
                                                            for n in tg]
    for n, a, t, os_ in pairs:
        a = a.detach().double().cpu()
        err, tn = float((a - t).norm()), float(t.norm())
        oerr = max(float((o - t).norm()) for o in os_)
        if len(os_) > 1:
            oerr = max(oerr, float((os_[0] - os_[1]).norm()))
        ratio.append(err / max(5e-3 * tn + floor * (gmax if n != "dL/dx" else tn), k * oerr))
        info.append((n, err / max(tn, 1e-30), oerr / max(tn, 1e-30)))
    ratio = np.array(ratio)
    for i in np.argsort(-ratio)[:6]:
        print("%.2f  %-45s ours %.3g  other %.3g" % ((ratio[i],) + info[i]))
    assert (ratio > 1).mean() <= 0.05 and ratio.max() < 10, (float((ratio > 1).mean()), float(ratio.max()))
    fy = float((y.detach().double().cpu() - ty).norm() / ty.norm())
    assert fy < (1e-5 if dtype == "fp32" else 1e-2), fy


def _run_coupling(kind, cio, mid, size, B, dtype, group, seed=0):
    import modules_realnvp as MR
    import utils
    from realnvp_hip import engine
    old = engine.NET_GROUP
    engine.NET_GROUP = int(group)
    try:
        mod, x, gy, gl = _inputs(kind, cio, mid, size, B, seed)
        mod = mod.to(DEV).train()
        mod.compute_dtype = dtype
        x = x.to(DEV).requires_grad_(True)
        gy, gl = gy.to(DEV), gl.to(DEV)
        y, ldj = mod(x)
        (y * gy + ldj * gl).sum().backward()
        torch.cuda.synchronize()
        grads = {n: p.grad.clone() for n, p in mod.named_parameters() if p.grad is not None}
        return y.detach(), ldj.detach(), x.grad.clone(), grads, mod.engine()
    finally:
        engine.NET_GROUP = old


CASES = [
    # name, kind, in_out_dim, mid, size, batch: M = batch * size^2
    ("s5_ckbd_m256", "ckbd", 48, 512, 4, 16),
    ("s5_ckbd_m1024", "ckbd", 48, 512, 4, 64),
    ("s4_chan_m1024", "chan", 96, 512, 4, 64),
    ("s4_ckbd_m4096", "ckbd", 24, 256, 8, 64),
    ("s3_ckbd_m16384", "ckbd", 12, 128, 16, 64),
    # wide scales (M > 16k): fan-out launches (conv_s1.hip k_s1_fanout, bf16),
    # members sharing one input tile
    ("s2_ckbd_m65536", "ckbd", 6, 64, 32, 64),
    ("s1_ckbd_m65536", "ckbd", 3, 32, 64, 16),
    ("s1_ckbd_m262144", "ckbd", 3, 32, 64, 64),    # config 1's scale 1 at its full batch
    ("s1_chan_m65536", "chan", 12, 64, 32, 64),     # ... and its channelwise couplings
]


def _plans(eng):
    svs = [sv for pool in eng._saved_pool.values() for sv in pool]
    assert svs, "no saved arena"
    return svs[0]["fwd_plan"][2], svs[0]["bwd_plan"][2]


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_grouped_matches_single_launches(case, dtype):
    _, kind, cio, mid, size, B = case
    if B * size * size > 16384 and dtype == "fp32":
        pytest.skip("fan-out groups are bf16 only (fp32 runs single launches at the wide scales)")
    y0, l0, gx0, g0, e0 = _run_coupling(kind, cio, mid, size, B, dtype, group=False)
    y1, l1, gx1, g1, e1 = _run_coupling(kind, cio, mid, size, B, dtype, group=True)
    f0, b0 = _plans(e0)
    f1, b1 = _plans(e1)
    assert all(p[0] == "single" for p in f0 + b0)
    # grouping really happened: R = 4 skip convs -> 3 forward groups (skip i
    # beside block i+1's first 1x1), one backward group (in_skip + 4 skips)
    assert sum(p[0] == "group" for p in f1) >= 3, [p[:3] for p in f1]
    assert any(p[0] == "group" and p[2] - p[1] >= 5 for p in b1), [p[:3] for p in b1]
    # a group runs its first conv's tile configuration for every member, so
    # a member can sum K in another order than its single launch: the
    # forward agrees to rounding (bf16: flipped bf16 roundings of stored
    # activations); the backward of EACH schedule is pinned to the oracle
    fw = 1e-5 if dtype == "fp32" else 1e-2
    assert rel(y1, y0) < fw and rel(l1, l0) < fw, (rel(y1, y0), rel(l1, l0))
    for y, l, gx, g in ((y0, l0, gx0, g0), (y1, l1, gx1, g1)):
        _check_vs_oracle(case, dtype, (y, l, gx, g))


def test_group_c_abi_two_skip_convs():
    """two independent 1x1 convs (one with a BN+ReLU prologue) through
    rnvp_net_group_prepare / rnvp_net_group against two rnvp_conv2d launches
    and torch"""
    from realnvp_hip import _lib
    from realnvp_hip._lib import BNSrc, ConvArgs, NetStep
    from realnvp_hip.engine import stat_shards
    L = _lib.lib()
    B, H, W, Cc = 64, 4, 4, 512
    M = B * H * W
    torch.manual_seed(3)
    x = torch.randn(M, Cc, device=DEV)
    w1 = torch.randn(Cc, Cc, device=DEV) * 0.05
    w2 = torch.randn(Cc, Cc, device=DEV) * 0.05
    sh = stat_shards(M)
    bsum = torch.zeros(sh, 2, Cc, device=DEV, dtype=torch.float64)
    bsum[0, 0] = x.double().sum(0)
    bsum[0, 1] = (x.double() ** 2).sum(0)
    gam = torch.rand(Cc, device=DEV) + 0.5
    bet = torch.randn(Cc, device=DEV) * 0.1
    s = torch.cuda.current_stream().cuda_stream

    def run(grouped):
        y1 = torch.zeros(M, Cc, device=DEV)
        y2 = torch.zeros(M, Cc, device=DEV)
        a1 = ConvArgs()
        a1.dtype, a1.B, a1.H, a1.W, a1.ks = 0, B, H, W, 1
        a1.x, a1.cs_in, a1.cin, a1.w, a1.kp = x.data_ptr(), Cc, Cc, w1.data_ptr(), Cc
        a1.y, a1.cs_out, a1.n = y1.data_ptr(), Cc, Cc
        a2 = ConvArgs()
        a2.dtype, a2.B, a2.H, a2.W, a2.ks = 0, B, H, W, 1
        a2.x, a2.cs_in, a2.cin, a2.w, a2.kp = x.data_ptr(), Cc, Cc, w2.data_ptr(), Cc
        a2.y, a2.cs_out, a2.n = y2.data_ptr(), Cc, Cc
        a2.pro_bn_relu = 1
        a2.pro = BNSrc(bsum.data_ptr(), float(M), None, None, gam.data_ptr(), bet.data_ptr(), 1e-5, sh)
        if grouped:
            steps = (NetStep * 2)()
            for st, a in zip(steps, (a1, a2)):
                st.kind, st.conv, st.dgamma_off, st.dbeta_off = 0, a, -1, -1
            k, g, lb = C.c_int(), C.c_int(), C.c_int()
            assert L.net_group_prepare(steps, 2, C.byref(k), C.byref(g), C.byref(lb)) == 0
            L.net_group(C.addressof(steps), 2, 0, k.value, g.value, lb.value, s)
        else:
            L.conv2d(C.byref(a1), s)
            L.conv2d(C.byref(a2), s)
        torch.cuda.synchronize()
        return y1, y2

    y1s, y2s = run(False)
    y1g, y2g = run(True)
    assert rel(y1g, y1s) < 1e-6 and rel(y2g, y2s) < 1e-6
    mean = bsum[0, 0] / M
    var = bsum[0, 1] / M - mean * mean
    act = torch.relu((x - mean.float()) / torch.sqrt(var.float() + 1e-5) * gam + bet)
    assert rel(y1g, x @ w1.t()) < 1e-5
    assert rel(y2g, act @ w2.t()) < 1e-5


def _frag_major(w):
    """[n][kp] -> the fragment-major image of rnvp_conv_args.w_frag"""
    n, kp = w.shape
    npad = (n + 15) // 16 * 16
    wp = torch.zeros(npad, kp, dtype=w.dtype, device=w.device)
    wp[:n] = w
    return wp.view(npad // 16, 16, kp // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()


def test_group_frag_major_members():
    """bf16 grouped 1x1 convs whose members carry fragment-major weight images
    (rnvp_conv_args.w_frag; their row-major w zeroed): bitwise the row-major
    single launches"""
    from realnvp_hip import _lib
    from realnvp_hip._lib import BNSrc, ConvArgs, NetStep
    from realnvp_hip.engine import stat_shards
    L = _lib.lib()
    B, H, W, Cc = 64, 4, 4, 512
    M = B * H * W
    torch.manual_seed(5)
    x = torch.randn(M, Cc, device=DEV).to(torch.bfloat16)
    ws = [(torch.randn(Cc, Cc, device=DEV) * 0.05).to(torch.bfloat16) for _ in range(2)]
    wfs = [_frag_major(w) for w in ws]
    zero = torch.zeros(Cc, Cc, device=DEV, dtype=torch.bfloat16)
    sh = stat_shards(M)
    bsum = torch.zeros(sh, 2, Cc, device=DEV, dtype=torch.float64)
    bsum[0, 0] = x.double().sum(0)
    bsum[0, 1] = (x.double() ** 2).sum(0)
    gam = torch.rand(Cc, device=DEV) + 0.5
    bet = torch.randn(Cc, device=DEV) * 0.1
    s = torch.cuda.current_stream().cuda_stream

    def run(grouped):
        ys = [torch.zeros(M, Cc, device=DEV, dtype=torch.bfloat16) for _ in range(2)]
        args = []
        for i in range(2):
            a = ConvArgs()
            a.dtype, a.B, a.H, a.W, a.ks = 1, B, H, W, 1
            a.x, a.cs_in, a.cin, a.kp = x.data_ptr(), Cc, Cc, Cc
            a.w = zero.data_ptr() if grouped else ws[i].data_ptr()
            a.w_frag = wfs[i].data_ptr() if grouped else None
            a.y, a.cs_out, a.n = ys[i].data_ptr(), Cc, Cc
            if i == 1:
                a.pro_bn_relu = 1
                a.pro = BNSrc(bsum.data_ptr(), float(M), None, None, gam.data_ptr(), bet.data_ptr(), 1e-5, sh)
            args.append(a)
        if grouped:
            steps = (NetStep * 2)()
            for st, a in zip(steps, args):
                st.kind, st.conv, st.dgamma_off, st.dbeta_off = 0, a, -1, -1
            k, g, lb = C.c_int(), C.c_int(), C.c_int()
            assert L.net_group_prepare(steps, 2, C.byref(k), C.byref(g), C.byref(lb)) == 0
            assert k.value & (1 << 11), "the fragment-major group kernel"
            L.net_group(C.addressof(steps), 2, 1, k.value, g.value, lb.value, s)
        else:
            for a in args:
                L.conv2d(C.byref(a), s)
        torch.cuda.synchronize()
        return ys

    single, grouped = run(False), run(True)
    for a, b in zip(single, grouped):
        assert torch.equal(a, b)
    assert rel(grouped[0].float(), x.float() @ ws[0].float().t()) < 1e-2
