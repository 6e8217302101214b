"""Parity of the HIP path (through the C ABI) against golden vectors produced by
the reference and against the CPU oracle.  Runs on the MI355X box.

Tolerances (fp32 parity mode):
  * index maps: bit-exact (== comparison, so +0/-0 compare equal)
  * per-sample log-prob: 1e-5 relative (BASELINE.json north star)
  * coupling outputs: rtol 1e-4 / atol 2e-5 elementwise
  * eval reconstruction ||g(f(x)) - x||_inf / ||x||_inf <= 1e-5
  * gradients: global relative L2 of dL/dx <= 1e-2 and of the per-tensor norm
    vector <= 5e-3 (fp32 noise floor measured in tests/test_oracle_golden.py)
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from formula_init import formula_state, pixels, uniform_noise

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _hp(bd, rb, bottleneck=True, skip=True, weight_norm=True, coupling_bn=True):
    import utils
    return utils.Hyperparameters(bd, rb, bottleneck, skip, weight_norm, coupling_bn)


# ---------------------------------------------------------------------------
def test_index_maps_bit_exact():
    from realnvp_hip import functions as Fn
    from realnvp_hip import _lib
    from realnvp_hip.engine import stream_ptr
    g = load_golden("index_maps.npz")
    for size in (2, 4, 8, 16, 32, 64, 128):
        for cfg in (0, 1):
            m = torch.empty(size * size, device=DEV)
            _lib.lib().checkerboard_mask(m.data_ptr(), size, cfg, stream_ptr())
            assert np.array_equal(m.cpu().numpy().reshape(1, 1, size, size), g["mask_%d_%d" % (size, cfg)])
    for shp in ((2, 3, 8, 8), (1, 6, 4, 4), (2, 12, 16, 16), (3, 24, 2, 2), (1, 3, 64, 64)):
        tag = "x".join(map(str, shp))
        x = T(g["squeeze_in_" + tag])
        assert np.array_equal(Fn.squeeze(x).cpu().numpy(), g["squeeze_out_" + tag])
        assert np.array_equal(Fn.undo_squeeze(Fn.squeeze(x)).cpu().numpy(), g["undo_out_" + tag])
        assert np.array_equal(Fn.undo_squeeze(T(g["undo_direct_in_" + tag])).cpu().numpy(), g["undo_direct_out_" + tag])
        on, off = Fn.factor_out(x)
        assert np.array_equal(on.cpu().numpy(), g["factor_on_" + tag])
        assert np.array_equal(off.cpu().numpy(), g["factor_off_" + tag])
        assert np.array_equal(Fn.restore(on, off).cpu().numpy(), g["restore_out_" + tag])


def test_permutations_large_roundtrip():
    from realnvp_hip import functions as Fn
    x = torch.randn(64, 3, 64, 64, device=DEV)
    assert torch.equal(Fn.undo_squeeze(Fn.squeeze(x)), x)
    on, off = Fn.factor_out(x)
    assert torch.equal(Fn.restore(on, off), x)
    # a permutation preserves the multiset: checksum of sorted values
    assert torch.equal(torch.sort(Fn.squeeze(x).flatten())[0], torch.sort(x.flatten())[0])


def test_logit_transform():
    import utils
    g = load_golden("logit.npz")
    lx, ld = utils.logit_transform(T(g["x"]), noise=T(g["noise"]))
    np.testing.assert_allclose(lx.cpu().numpy(), g["logit"], rtol=1e-6, atol=2e-6)
    np.testing.assert_allclose(ld.cpu().numpy(), g["logdet"], rtol=1e-6)
    inv, _ = utils.logit_transform(T(g["inv_in"]), reverse=True)
    np.testing.assert_allclose(inv.cpu().numpy(), g["inv_out"], rtol=1e-6, atol=1e-7)
    # device Philox noise: in [0,1), reproducible for a seed
    x = T(g["x"])
    a, la = utils.logit_transform(x, seed=123)
    b, lb = utils.logit_transform(x, seed=123)
    assert torch.equal(a, b) and torch.equal(la, lb)
    lo, _ = utils.logit_transform(x, noise=torch.zeros_like(x))
    hi, _ = utils.logit_transform(x, noise=torch.full_like(x, 0.999999))
    assert bool(((a >= lo - 1e-5) & (a <= hi + 1e-5)).all())


# ---------------------------------------------------------------------------
COUPLINGS = [
    ("ckbd_c3_m32_s32_cfg1", "ckbd", 3, 32, 32, 1.0, dict(bd=32, rb=2)),
    ("ckbd_c3_m32_s32_cfg0", "ckbd", 3, 32, 32, 0.0, dict(bd=32, rb=2)),
    ("chan_c12_m64_s16_cfg0", "chan", 12, 64, 16, 0.0, dict(bd=32, rb=2)),
    ("chan_c12_m64_s16_cfg1", "chan", 12, 64, 16, 1.0, dict(bd=32, rb=2)),
    ("ckbd_c48_m64_s4_cfg0", "ckbd", 48, 64, 4, 0.0, dict(bd=32, rb=1)),
    ("ckbd_nobott_cfg1", "ckbd", 3, 16, 8, 1.0, dict(bd=16, rb=2, bottleneck=False)),
    ("ckbd_r0_bott_cfg0", "ckbd", 3, 16, 8, 0.0, dict(bd=16, rb=0)),
    ("ckbd_r0_nobott_cfg1", "ckbd", 3, 16, 8, 1.0, dict(bd=16, rb=0, bottleneck=False)),
    ("chan_noskip_cfg1", "chan", 12, 16, 8, 1.0, dict(bd=16, rb=2, skip=False)),
    ("ckbd_nownorm_cfg1", "ckbd", 3, 16, 8, 1.0, dict(bd=16, rb=1, weight_norm=False)),
    ("chan_nocbn_cfg0", "chan", 12, 16, 8, 0.0, dict(bd=16, rb=1, coupling_bn=False)),
]


def make_coupling(kind, cio, mid, size, cfg, hk):
    import modules_realnvp as MR
    hp = _hp(**hk)
    if kind == "ckbd":
        return MR.CheckerboardAffineCoupling(cio, mid, size, cfg, hp)
    return MR.ChannelwiseAffineCoupling(cio, mid, cfg, hp)


def close(a, b, rtol=1e-4, atol=2e-5):
    np.testing.assert_allclose(a.detach().cpu().numpy(), b, rtol=rtol, atol=atol)


@pytest.mark.parametrize("case", COUPLINGS, ids=[c[0] for c in COUPLINGS])
def test_coupling_vs_reference(case):
    name, kind, cio, mid, size, cfg, hk = case
    g = load_golden("coupling_%s.npz" % name)
    mod = make_coupling(kind, cio, mid, size, cfg, hk)
    mod.load_state_dict(formula_state(mod))
    mod = mod.to(DEV).train()
    x = T(g["x"]).requires_grad_(True)
    y, ldj = mod(x)
    close(y, g["train_y"])
    close(ldj, g["train_ldj"])
    (y * T(g["gy"]) + ldj * T(g["gl"])).sum().backward()
    assert rel(x.grad.cpu().numpy(), g["grad_x"]) < 1e-4
    gn = np.sqrt(sum(float((g[k].astype(np.float64) ** 2).sum()) for k in g.files if k.startswith("grad.")))
    for n, p in mod.named_parameters():
        if not p.requires_grad:
            assert p.grad is None
            continue
        ref = g["grad." + n]
        got = p.grad.cpu().numpy()
        err = np.linalg.norm(got.astype(np.float64) - ref)
        assert err <= 1e-4 * np.linalg.norm(ref) + 1e-6 * gn, n
    sd = mod.state_dict()
    for k in g.files:
        if k.startswith("after_train."):
            kk = k[len("after_train."):]
            np.testing.assert_allclose(sd[kk].cpu().numpy(), g[k], rtol=1e-4, atol=1e-6, err_msg=kk)
    with torch.no_grad():
        xr, _ = mod(T(g["x"]), reverse=True)
    close(xr, g["train_rev"])
    sd = mod.state_dict()
    for k in g.files:
        if k.startswith("after_train_rev."):
            kk = k[len("after_train_rev."):]
            np.testing.assert_allclose(sd[kk].cpu().numpy(), g[k], rtol=1e-4, atol=1e-6, err_msg=kk)
    mod.eval()
    with torch.no_grad():
        ye, le = mod(T(g["x"]))
        xe, _ = mod(ye, reverse=True)
    close(ye, g["eval_y"])
    close(le, g["eval_ldj"])
    close(xe, g["eval_rec"])


# ---------------------------------------------------------------------------
MODELS = [("m32_d8_r1", 32, 8, 1), ("m32_d32_r2", 32, 32, 2), ("m64_d32_r4", 64, 32, 4)]


def make_model(size, bd, rb):
    import flow_realnvp
    prior = torch.distributions.Normal(torch.tensor(0.0, device=DEV), torch.tensor(1.0, device=DEV),
                                       validate_args=False)
    m = flow_realnvp.RealNVP(3, size, prior, _hp(bd, rb))
    m.load_state_dict(formula_state(m))
    return m.to(DEV)


def oracle_grads64(size, bd, rb, x, logdet, names):
    """fp64 CPU oracle gradients of the train.py loss at the formula init
    (test infrastructure: the truth the fp32 paths are measured against)."""
    import realnvp_oracle as O
    from formula_init import formula_value
    spec = O.FlowSpec(3, size, O.HP(bd, rb))
    e = O.flow_spec_entries(spec)
    S = {k: (v.double() if v.is_floating_point() else v) for k, v in O.build_state(e, formula_value).items()}
    trainable = set(O.trainable_names(e))
    for n in names:
        S[n] = S[n].requires_grad_(True)
    x64 = torch.from_numpy(np.asarray(x)).double()
    ld64 = torch.from_numpy(np.asarray(logdet)).double()
    lp = O.log_prob(S, spec, x64, training=True)
    ws = O.weight_scale(S, O.param_names(e), lambda n: n in trainable)
    loss = -(lp + ld64).mean() + 5e-5 * ws
    grads = torch.autograd.grad(loss, [S[n] for n in names])
    return {n: gr.numpy() for n, gr in zip(names, grads)}


@pytest.mark.parametrize("case", MODELS, ids=[c[0] for c in MODELS])
def test_model_vs_reference(case):
    name, size, bd, rb = case
    g = load_golden("model_%s.npz" % name)
    model = make_model(size, bd, rb).train()
    x = T(g["x"]).requires_grad_(True)
    logdet = T(g["logdet"])
    lp, ws = model(x)
    np.testing.assert_allclose(lp.detach().cpu().numpy(), g["train_logprob"], rtol=1e-5)
    np.testing.assert_allclose(float(ws.detach()), float(g["weight_scale"]), rtol=1e-5)
    loss = -(lp + logdet).mean() + 5e-5 * ws
    np.testing.assert_allclose(float(loss), float(g["loss"]), rtol=1e-5)
    loss.backward()
    # fp32 floor of dL/dx through 28 batch-stat couplings: the CPU oracle in
    # fp32 vs fp64 differs by 2.9e-3 (m32_d32_r2) and 1.4e-2 (m64_d32_r4, B=2)
    assert rel(x.grad.cpu().numpy(), g["grad_x"]) < 3e-2
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    assert names == list(g["grad_names"])
    params = dict(model.named_parameters())
    norms = np.array([float(params[n].grad.norm()) for n in names])
    assert rel(norms, g["grad_norms"]) < 5e-3
    big = g["grad_norms"] > 1e-4 * np.linalg.norm(g["grad_norms"])
    # single tensors near cancellation (conv biases / BN affine feeding a batch
    # statistic) are ill-conditioned in fp32 (oracle fp32 vs fp64 up to 3.9e-2
    # at m32, larger at m64 B=2): allow a 2% tail beyond 8%
    off = np.abs(norms[big] - g["grad_norms"][big]) > 8e-2 * g["grad_norms"][big]
    assert off.mean() <= 0.02, (off.sum(), big.sum())
    # full tensors stored for scale / scale_shift / in_bn grads: sums over the
    # whole batch that nearly cancel, so fp32 summation order alone moves them
    # by several percent (the reference itself is 2.4e-2 off fp64 in norm on
    # s3_ckbd.2.in_bn.weight).  Anchor on the fp64 oracle: ours must be within
    # the fixed band of the fp64 value, or within 3x the reference's own fp32
    # error for that tensor.
    gkeys = [k[5:] for k in g.files if k.startswith("grad.")]
    g64 = oracle_grads64(size, bd, rb, g["x"], g["logdet"], gkeys)
    tol = 1e-1 if size == 32 else 2.5e-1
    for n in gkeys:
        ours, ref, truth = params[n].grad.cpu().numpy(), g["grad." + n], g64[n]
        assert rel(ours, truth) < max(tol, 3 * rel(ref, truth)), (n, rel(ours, truth), rel(ref, truth))
    with torch.no_grad():
        z, ldj = model.f(T(g["x"]))
    np.testing.assert_allclose(z.cpu().numpy(), g["train_z"], rtol=1e-3, atol=1e-4)
    assert rel(ldj.sum((1, 2, 3)).cpu().numpy(), g["train_ldj"].sum((1, 2, 3))) < 1e-5
    sd = model.state_dict()
    for k in g.files:
        if k.startswith("after_train."):
            kk = k[len("after_train."):]
            np.testing.assert_allclose(sd[kk].cpu().numpy(), g[k], rtol=1e-4, atol=1e-5, err_msg=kk)
    model.eval()
    with torch.no_grad():
        lpe, _ = model(T(g["x"]))
        ze, _ = model.f(T(g["x"]))
        xrec = model.g(ze)
        xs = model.g(T(g["sample_z"]))
    np.testing.assert_allclose(lpe.cpu().numpy(), g["eval_logprob"], rtol=1e-5)
    assert np.abs(xrec.cpu().numpy() - g["eval_rec"]).max() / np.abs(g["eval_rec"]).max() < 1e-5
    x0 = g["x"]
    assert np.abs(xrec.cpu().numpy() - x0).max() / np.abs(x0).max() < 1e-5
    assert rel(xs.cpu().numpy(), g["sample_x"]) < 1e-4


def test_reference_training_loop_trajectory():
    """train.py:176-200 with torch.optim.Adam around the drop-in model."""
    import utils
    name, size, bd, rb = MODELS[0]
    g = load_golden("model_%s.npz" % name)
    model = make_model(size, bd, rb).train()
    opt = torch.optim.Adam(model.parameters(), lr=5e-4, weight_decay=5e-5)
    B = g["x"].shape[0]
    for s in range(len(g["traj_loss"])):
        x, ld = utils.logit_transform(pixels(B, 3, size, seed=100 + s), noise=uniform_noise(B, 3, size, seed=200 + s))
        opt.zero_grad()
        lp, ws = model(x)
        ll = (lp + ld).mean()
        loss = -ll + 5e-5 * ws
        loss.backward()
        opt.step()
        # step 1 is a pure forward of the same weights (<= 2e-5); later steps
        # carry Adam-amplified fp32 noise of near-zero gradients
        np.testing.assert_allclose(float(loss), g["traj_loss"][s], rtol=2e-5 if s == 0 else 1e-4)
    model.eval()
    with torch.no_grad():
        lp, _ = model(T(g["x"]))
    # after 3 Adam steps: Adam's m/sqrt(v) turns the fp32 noise of near-zero
    # gradients (conv biases feeding a BatchNorm, ...) into +-lr updates, so
    # the weights differ at the 1e-4 level -> 5e-4 on the resulting log-prob
    np.testing.assert_allclose(lp.cpu().numpy(), g["traj_eval_logprob_after"], rtol=5e-4)


def test_bf16_mode_close_to_fp32():
    name, size, bd, rb = MODELS[2]
    g = load_golden("model_%s.npz" % name)
    model = make_model(size, bd, rb).train().set_precision("bf16")
    x = T(g["x"])
    lp, ws = model(x)
    # bf16 s/t network (fp32 accumulate, fp32 couplings / log-det): bounded drift
    r = np.abs(lp.detach().cpu().numpy() - g["train_logprob"]) / np.abs(g["train_logprob"])
    assert r.max() < 2e-3, r
    (-lp.mean()).backward()
    assert all(torch.isfinite(p.grad).all() for p in model.parameters() if p.grad is not None)
