"""Deep and large configurations on the MI355X, against reference goldens
(tools/make_goldens.py) and the CPU oracle:

  * R=8 couplings (BASELINE config 3 and the reference CLI default R8/D64,
    main.py:231-240; modules_realnvp.py:136-152 builds any R): 4R+3 = 35 convs,
    more than one grouped weight-gradient launch; the mid-1024 channelwise
    coupling of config 3's scale 4;
  * the whole config-3 model (32x32x3, R8, D64, 923.6 M parameters) at B=2;
  * config 1 (64x64x3, R4, D32) at its benchmarked batch B=64: the drop-in and
    the fused trainer (the path bench.py times) in fp32 to the north star's
    1e-5, and the bf16 mode against the same golden;
  * config 4's generalised 6-scale flow at 128x128 against the oracle (the
    reference hard-codes 5 scales, flow_realnvp.py:46-95, so there is no
    reference golden for it: layer goldens + composition);
  * grouped weight gradients at >= 2^22 pixels (config 4's scale 1 at B=256).
"""
import ctypes as C

import numpy as np
import pytest
import torch

from conftest import load_golden
from formula_init import formula_state, formula_value, pixels, uniform_noise

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


def model_inputs(B, size):
    """tools/make_goldens.py:model_inputs (the same torch-CPU formula)."""
    pix = pixels(B, 3, size, seed=10)
    noise = uniform_noise(B, 3, size, seed=11)
    x = (pix * 255.0 + noise) / 256.0
    x = ((x * 2.0 - 1.0) * 0.9 + 1.0) / 2.0
    x_in = torch.log(x) - torch.log(1.0 - x)
    pre = torch.tensor(np.log(0.9) - np.log(0.1))
    logdet = (torch.nn.functional.softplus(x_in) + torch.nn.functional.softplus(-x_in)
              - torch.nn.functional.softplus(-pre)).sum(dim=(1, 2, 3))
    return x_in, logdet


def make_model_chirp(size, bd, rb):
    """formula init with full-rank (chirp) weights, as tools/make_bf16_golden.py"""
    m = make_model(size, bd, rb)
    m.load_state_dict(formula_state(m, style="chirp"))
    return m


def make_model(size, bd, rb, n_scales=5, device_init=False):
    import flow_realnvp
    prior = torch.distributions.Normal(torch.tensor(0.0, device=DEV), torch.tensor(1.0, device=DEV),
                                       validate_args=False)
    m = flow_realnvp.RealNVP(3, size, prior, _hp(bd, rb), n_scales=n_scales)
    if device_init:
        m = m.to(DEV)
        m.load_state_dict(formula_state(m, device=DEV))
        return m
    m.load_state_dict(formula_state(m))
    return m.to(DEV)


# ---------------------------------------------------------------------------
BIG_COUPLINGS = [
    ("ckbd_c3_m64_s32_r8_cfg1", "ckbd", 3, 64, 32, 1.0, dict(bd=64, rb=8)),
    ("chan_c96_m1024_s2_r8_cfg0", "chan", 96, 1024, 2, 0.0, dict(bd=64, rb=8)),
]


@pytest.mark.parametrize("case", BIG_COUPLINGS, ids=[c[0] for c in BIG_COUPLINGS])
def test_deep_coupling_vs_reference(case):
    import modules_realnvp as MR
    name, kind, cio, mid, size, cfg, hk = case
    g = load_golden("coupling_%s.npz" % name)
    hp = _hp(**hk)
    mod = MR.CheckerboardAffineCoupling(cio, mid, size, cfg, hp) if kind == "ckbd" else \
        MR.ChannelwiseAffineCoupling(cio, mid, cfg, hp)
    mod.load_state_dict(formula_state(mod, style="chirp"))   # full-rank weights (formula_init.chirp_value)
    mod = mod.to(DEV).train()
    eng = mod.engine()
    assert len(eng.P.convs) == 4 * hk["rb"] + 3 > 24   # spans two grouped-wgrad launches
    x = T(g["x"]).requires_grad_(True)
    y, ldj = mod(x)
    np.testing.assert_allclose(y.detach().cpu().numpy(), g["train_y"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(ldj.detach().cpu().numpy(), g["train_ldj"], rtol=1e-4, atol=2e-5)
    (y * T(g["gy"]) + ldj * T(g["gl"])).sum().backward()
    # gradients: anchored on the fp64 oracle (tools/make_fp64_refs.py).  Deep
    # nets put a few of their 10^5-10^6 BatchNorm outputs within fp32 rounding
    # of the ReLU kink; such a decision can come out either way in any fp32
    # evaluation, and one flip moves dL/dx by ~1e-3 normwise (measured with
    # tools/coupling_diag.py --trace: a single element of g:out of ckbd R4 mid32
    # decides 1.4e-3, every other element agrees to 1e-6).  Tolerance: 5e-3, or
    # 3x the reference's own fp32 error when that is larger.
    t = load_golden("fp64_coupling_%s.npz" % name)
    gx = x.grad.cpu().numpy()
    assert rel(gx, t["grad_x"]) < max(5e-3, 3 * rel(g["grad_x"], t["grad_x"])), (rel(gx, t["grad_x"]),
                                                                                 rel(g["grad_x"], t["grad_x"]))
    params = dict(mod.named_parameters())
    names = [n for n, p in mod.named_parameters() if p.requires_grad]
    assert names == list(g["grad_names"]) == list(t["grad_names"])
    norms = np.array([float(params[n].grad.double().norm()) for n in names])
    gn = float(np.linalg.norm(t["grad_norms"]))
    ratio, info = [], []   # error / allowance: within 5e-3 of the fp64 truth or 3x the reference's own error
    for n, ref_n, true_n, got_n in zip(names, g["grad_norms"], t["grad_norms"], norms):
        ratio.append(abs(got_n - true_n) / max(5e-3 * true_n + 1e-6 * gn, 3 * abs(ref_n - true_n)))
        info.append(("norm " + n, abs(got_n - true_n) / true_n, abs(ref_n - true_n) / true_n, true_n))
        if "grad." + n in t.files:      # full tensors
            truth = t["grad." + n]
            tn = np.linalg.norm(truth)
            err = np.linalg.norm(params[n].grad.cpu().numpy().astype(np.float64) - truth)
            ref_err = np.linalg.norm(g["grad." + n].astype(np.float64) - truth)
            ratio.append(err / max(5e-3 * tn + 1e-6 * gn, 3 * ref_err))
            info.append(("full " + n, err / tn, ref_err / tn, tn))
    ratio = np.array(ratio)
    for i in np.argsort(-ratio)[:12]:
        print("%.2f  %s  ours %.3g  ref %.3g  |truth| %.3g" % ((ratio[i],) + info[i]))
    # ReLU-kink decisions (above) and summation-order noise of batch-stat
    # gradients: at most 5 % of the checks beyond the allowance, none 10x
    assert (ratio > 1).mean() <= 0.05 and ratio.max() < 10, (float((ratio > 1).mean()), float(ratio.max()))
    sd = mod.state_dict()
    for k in g.files:
        if k.startswith("after_train."):
            kk = k[len("after_train."):]
            np.testing.assert_allclose(sd[kk].cpu().numpy(), g[k], rtol=1e-4, atol=1e-6, err_msg=kk)
    with torch.no_grad():
        xr, _ = mod(T(g["x"]), reverse=True)
    np.testing.assert_allclose(xr.cpu().numpy(), g["train_rev"], rtol=1e-4, atol=2e-5)
    mod.eval()
    with torch.no_grad():
        ye, le = mod(T(g["x"]))
        xe, _ = mod(ye, reverse=True)
    np.testing.assert_allclose(ye.cpu().numpy(), g["eval_y"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(le.cpu().numpy(), g["eval_ldj"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(xe.cpu().numpy(), g["eval_rec"], rtol=1e-4, atol=2e-5)


# ---------------------------------------------------------------------------
def check_norms_vs_truth(norms, g, t, band=8e-2, tail=0.02):
    """per-tensor gradient norms against the fp64 truth t, with the
    reference's own fp32 error (g) as the yardstick (x3); see
    tools/make_fp64_refs.py."""
    ref, truth = g["grad_norms"], t["grad_norms"]
    assert rel(norms, truth) < max(5e-3, 3 * rel(ref, truth)), (rel(norms, truth), rel(ref, truth))
    big = truth > 1e-4 * np.linalg.norm(truth)
    off = np.abs(norms[big] - truth[big]) > np.maximum(band * truth[big], 3 * np.abs(ref[big] - truth[big]))
    assert off.mean() <= tail, (off.sum(), big.sum())


def _lite_model_check(model, g, t, x, logdet, lp_tol=1e-5):
    lp, ws = model(x)
    np.testing.assert_allclose(lp.detach().cpu().numpy(), g["train_logprob"], rtol=lp_tol)
    np.testing.assert_allclose(float(ws.detach()), float(g["weight_scale"]), rtol=1e-5)
    loss = -(lp + logdet).mean() + 5e-5 * ws
    np.testing.assert_allclose(float(loss.detach()), float(g["loss"]), rtol=lp_tol)
    loss.backward()
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    assert names == list(g["grad_names"]) == list(t["grad_names"])
    params = dict(model.named_parameters())
    norms = np.array([float(params[n].grad.double().norm()) for n in names])
    check_norms_vs_truth(norms, g, t)
    return names, norms


def test_model_config3_r8_d64_vs_reference():
    """BASELINE config 3 (923.6 M parameters) through the drop-in at B=2:
    training log-prob within 1e-5 of the reference, gradients, running
    statistics, eval log-prob and eval reconstruction."""
    g = load_golden("model_m32_d64_r8.npz")
    t = load_golden("fp64_model_m32_d64_r8.npz")
    model = make_model(32, 64, 8, device_init=True).train()
    x, logdet = model_inputs(2, 32)
    x, logdet = x.to(DEV).requires_grad_(True), logdet.to(DEV)
    _lite_model_check(model, g, t, x, logdet)
    sd = model.state_dict()
    for k in g.files:
        if k.startswith("after_train."):
            kk = k[len("after_train."):]
            np.testing.assert_allclose(sd[kk].cpu().numpy(), g[k], rtol=1e-4, atol=1e-5, err_msg=kk)
    model.eval()
    with torch.no_grad():
        lpe, _ = model(x.detach())
        ze, _ = model.f(x.detach())
        xrec = model.g(ze)
    np.testing.assert_allclose(lpe.cpu().numpy(), g["eval_logprob"], rtol=1e-5)
    err = float((xrec - x.detach()).abs().max() / x.detach().abs().max())
    assert err < 1e-5, err


def test_model_config1_full_batch_fp32_drop_in():
    """config 1 at B=64 (the benchmarked batch), drop-in fp32 path."""
    g = load_golden("model_m64_d32_r4_b64.npz")
    t = load_golden("fp64_model_m64_d32_r4_b64.npz")
    model = make_model(64, 32, 4).train()
    x, logdet = model_inputs(64, 64)
    x, logdet = x.to(DEV), logdet.to(DEV)
    _lite_model_check(model, g, t, x, logdet)
    sd = model.state_dict()
    for k in g.files:
        if k.startswith("after_train."):
            kk = k[len("after_train."):]
            np.testing.assert_allclose(sd[kk].cpu().numpy(), g[k], rtol=1e-4, atol=1e-5, err_msg=kk)
    model.eval()
    with torch.no_grad():
        lpe, _ = model(x)
    np.testing.assert_allclose(lpe.cpu().numpy(), g["eval_logprob"], rtol=1e-5)


_ORACLE_STEPS = {}


def oracle_step(style, emu=None):
    """The CPU oracle's training step on the config-1 golden batch (B = 64,
    formula weights of `style`), run here on the host: (per-tensor gradients,
    dL/dx).  emu: None = plain fp32 oracle, else the engine's bf16 emulation
    (oracle/realnvp_bf16emu.py).  Cached per session (~10-30 s each)."""
    key = (style, None if emu is None else emu.wide)
    if key not in _ORACLE_STEPS:
        import realnvp_oracle as O
        from formula_init import chirp_value
        from realnvp_bf16emu import run
        spec = O.FlowSpec(3, 64, O.HP(32, 4))
        entries = O.flow_spec_entries(spec)
        S0 = O.build_state(entries, chirp_value if style == "chirp" else formula_value)
        x, ld = model_inputs(64, 64)
        r = run(S0, spec, O.trainable_names(entries), x, ld, emu, full=True)
        _ORACLE_STEPS[key] = (r[4], r[5])
    return _ORACLE_STEPS[key]


def trainer_grads(tr, model, p0):
    """The fused trainer's parameter gradients (the arena plus the
    regulariser term its Adam folds in) per tensor, and dL/dx of the step's
    input (the first coupling's input gradient)."""
    grad = tr.grad + (tr.mask == 2).float() * (2 * 5e-5) * p0
    out = {n: grad[tr.offsets[n]:tr.offsets[n] + p.numel()].view_as(p) for n, p in model.named_parameters()}
    return out, tr._g(tr.xl)


def trel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm())


def check_projections_vs_truth(P, Pref, Ptrue, band=8e-2, tail=0.02):
    """projection checksums (tests/formula_init.py:projections) of every
    trainable tensor against the fp64 truth, the reference's own fp32 error
    as the yardstick (x3), as check_norms_vs_truth does for the norms: the
    whole [tensors x 4] matrix, then tensor by tensor with a 2 % tail for
    ReLU-kink decisions (none beyond 10x its allowance)"""
    assert rel(P, Ptrue) < max(5e-3, 3 * rel(Pref, Ptrue)), (rel(P, Ptrue), rel(Pref, Ptrue))
    tn = np.linalg.norm(Ptrue, axis=1)
    big = tn > 1e-4 * np.linalg.norm(Ptrue)
    err = np.linalg.norm(P - Ptrue, axis=1)[big]
    allow = np.maximum(band * tn[big], 3 * np.linalg.norm(Pref - Ptrue, axis=1)[big])
    assert (err > allow).mean() <= tail and (err / allow).max() < 10, (int((err > allow).sum()), int(big.sum()),
                                                                         float((err / allow).max()))


def _trainer(model, B, dtype, chain):
    """FlowTrainer over coupling links (the default, rnvp_coupling_link_fwd /
    _link_bwd) or every coupling's in and out
    parts launched on their own (chain=0)"""
    from realnvp_hip import trainer as TM
    tr = TM.FlowTrainer(model, B, dtype=dtype, chain=bool(chain))
    assert (tr.links is not None) == bool(chain)
    return tr


def _trainer_step_check(dtype, lp_tol, norm_tol=None, chain=1):
    """One fused-trainer step (the code bench.py times) on the golden batch:
    per-sample log-prob, loss and the gradient arena (+ the regulariser term
    the fused Adam folds in) against the reference -- norms, projection
    checksums of every tensor, the 10 largest tensors element by element and
    dL/dx."""
    from formula_init import projection_matrix
    g = load_golden("model_m64_d32_r4_b64.npz")
    model = make_model(64, 32, 4)
    tr = _trainer(model, 64, dtype, chain)
    x, logdet = model_inputs(64, 64)
    tr.set_input(x.to(DEV), logdet.to(DEV))
    p0 = tr.param.clone()
    tr.step_eager()
    torch.cuda.synchronize()
    lp = tr.lp.cpu().numpy()
    r = np.abs(lp - g["train_logprob"]) / np.abs(g["train_logprob"])
    assert r.max() < lp_tol, r.max()
    ll = tr.mean_logll(1)
    np.testing.assert_allclose(-ll, float(g["loss"]) - 5e-5 * float(g["weight_scale"]), rtol=lp_tol)
    grads, gx = trainer_grads(tr, model, p0)
    names = list(g["grad_names"])
    norms = np.array([float(grads[n].double().norm()) for n in names])
    if dtype == "fp32":
        check_norms_vs_truth(norms, g, load_golden("fp64_model_m64_d32_r4_b64.npz"))
        # gradient VALUES (tools/make_goldens.py:grads_golden): projection
        # checksums against the reference (fp32) and the float64 truth ...
        v = load_golden("grads_m64_d32_r4_b64.npz")
        assert list(v["grad_names"]) == names
        P = projection_matrix([grads[n] for n in names])
        check_projections_vs_truth(P, v["ref_grad_proj"], v["truth_grad_proj"])
        # ... and the 10 largest tensors and dL/dx element by element against
        # the fp32 oracle re-run here: within 5e-3 or 3x the reference's own
        # error of the truth, plus the oracle's own error (its distance to the
        # truth, stored): |ours - truth| <= allowance  =>  |ours - oracle| <=
        # allowance + |oracle - truth|
        og, ogx = oracle_step("wave")
        for n, ref_err, or_err in zip(v["full_names"], v["ref_full_err"], v["oracle_full_err"]):
            e = trel(grads[n], og[n])
            assert e < max(5e-3, 3 * ref_err) + or_err, (n, e, ref_err, or_err)
        e = trel(gx, ogx)
        assert e < max(5e-3, 3 * float(v["ref_grad_x_err"])) + float(v["oracle_grad_x_err"]), e
    else:
        assert rel(norms, g["grad_norms"]) < norm_tol, rel(norms, g["grad_norms"])
    return r.max(), rel(norms, g["grad_norms"])


@pytest.mark.parametrize("chain", [1, 0], ids=["chained", "unchained"])
def test_trainer_config1_full_batch_fp32(chain):
    """both coupling schedules pinned to the float64 truth (the chained one is
    the default; each is held to the same allowance, not to the other)"""
    _trainer_step_check("fp32", 1e-5, chain=chain)


@pytest.mark.parametrize("chain", [1, 0], ids=["chained", "unchained"])
def test_trainer_config1_full_batch_bf16(chain):
    """The benchmarked step itself (config 1, B = 64, bf16 s/t net) pinned to
    a bf16-faithful CPU golden (tools/make_bf16_golden.py): the oracle with
    the engine's bf16 rounding points (stored conv outputs, packed operands
    and weights, stored activation gradients), computed twice with different
    conv summation orders (fp32 vs fp64-accumulated), beside the fp32 oracle.
    The model has full-rank weights (formula init, chirp style).

    The three CPU references are as far from each other as bf16 itself
    scatters (measured: per-sample log-prob L2 1.7e-4 / max 4.2e-4, mean
    3.5e-5; per-tensor gradient-norm vector 0.023, per-tensor 90th percentile
    0.066): two correct bf16 implementations differ by that floor.  The HIP
    step must land within 3x the floor of EACH reference.  (Against the
    round-2 bound -- 2e-3 log-prob, 0.5 norm vector on rank-2 weights -- the
    norm-vector bound is 7x tighter; a kernel error of a few percent in any
    large gradient tensor moves the vector past it.)"""
    from formula_init import projection_matrix
    from realnvp_bf16emu import Emu
    g = load_golden("bf16emu_model_m64_d32_r4_b64.npz")
    refs = ("fp32", "emu", "emu_wide")
    model = make_model_chirp(64, 32, 4)
    tr = _trainer(model, 64, "bf16", chain)
    x, logdet = model_inputs(64, 64)
    tr.set_input(x.to(DEV), logdet.to(DEV))
    p0 = tr.param.clone()
    ws = sum(float(p.detach().double().pow(2).sum()) for n, p in model.named_parameters()
             if p.requires_grad and n.split(".")[-1] in ("weight_g", "scale"))
    tr.step_eager()
    torch.cuda.synchronize()
    lp = tr.lp.double().cpu().numpy()
    loss = -tr.mean_logll(1) + 5e-5 * ws
    grads, gx = trainer_grads(tr, model, p0)
    names = list(g["grad_names"])
    norms = np.array([float(grads[n].double().norm()) for n in names])
    proj = projection_matrix([grads[n] for n in names])

    def metrics(lp_a, loss_a, n_a, p_a, lp_b, loss_b, n_b, p_b):
        big = n_b > 1e-4 * np.linalg.norm(n_b)
        per = np.abs(n_a[big] - n_b[big]) / n_b[big]
        return np.array([rel(lp_a, lp_b), np.max(np.abs(lp_a - lp_b) / np.abs(lp_b)),
                         abs(loss_a - loss_b) / abs(loss_b), rel(n_a, n_b), np.percentile(per, 90), rel(p_a, p_b)])
    floor = np.max([metrics(g[a + "_logprob"], float(g[a + "_loss"]), g[a + "_grad_norms"], g[a + "_grad_proj"],
                            g[b + "_logprob"], float(g[b + "_loss"]), g[b + "_grad_norms"], g[b + "_grad_proj"])
                    for a in refs for b in refs if a != b], axis=0)
    labels = ("log-prob L2", "log-prob max", "loss", "grad-norm vector", "per-tensor p90", "projection matrix")
    for r in refs:
        m = metrics(lp, loss, norms, proj, g[r + "_logprob"], float(g[r + "_loss"]), g[r + "_grad_norms"],
                    g[r + "_grad_proj"])
        print("HIP bf16 vs %-8s " % r + "  ".join("%s %.3g (floor %.3g)" % (k, v, f)
                                                  for k, v, f in zip(labels, m, floor)))
        # the loss floor is a difference of near-equal means: floor it at 1e-4
        bound = 3 * np.maximum(floor, [0, 0, 1e-4, 0, 0, 0])
        assert np.all(m < bound), (r, dict(zip(labels, m)), dict(zip(labels, bound)))
    # element by element: the 10 largest tensors and dL/dx against the bf16
    # emulation re-run here.  bf16 storage makes these elementwise values
    # noisy -- two valid emulations (fp32 vs fp64 conv accumulation) differ by
    # ~0.55-0.65 relative L2 (tools/make_bf16_golden.py, "full_floor"), the
    # gradient direction, not its norm, carrying that noise.  The bound is 2x
    # that floor rather than 3x: a correct bf16 step lands about one floor
    # from the emulation, and 2x stays below sqrt(2), the distance of a
    # scrambled (permuted / mis-scattered) tensor, so such an error still fails.
    eg, egx = oracle_step("chirp", Emu(False))
    pair = list(g["full_pairs"]).index("emu~emu_wide")
    for n, fl in zip(g["full_names"], g["full_floor"][:, pair]):
        e = trel(grads[n], eg[n])
        print("full %s: %.3g (floor %.3g)" % (n, e, fl))
        assert e < min(2 * fl, 1.3), (n, e, fl)
    e, fl = trel(gx, egx), float(g["grad_x_floor"][pair])
    print("dL/dx: %.3g (floor %.3g)" % (e, fl))
    assert e < min(2 * fl, 1.3), (e, fl)


# ---------------------------------------------------------------------------
def test_six_scale_128_vs_oracle():
    """config 4's shape family: 128x128x3 with n_scales=6 (scales down to
    4x4) against the CPU oracle's generalised flow (which the goldens pin at
    n_scales=5): train log-prob 1e-5, eval log-prob, reconstruction 1e-5,
    dL/dx; plus a graph-captured bf16 trainer step stays finite."""
    import realnvp_oracle as O
    size, bd, rb, B = 128, 4, 1, 2
    model = make_model(size, bd, rb, n_scales=6).train()
    x, logdet = model_inputs(B, size)
    spec = O.FlowSpec(3, size, O.HP(bd, rb), n_scales=6)
    S = O.build_state(O.flow_spec_entries(spec), formula_value)
    xo = x.clone().requires_grad_(True)
    lpo = O.log_prob(S, spec, xo, training=True)
    (-(lpo + logdet).mean()).backward()
    # float64 truth of dL/dx: held to 5e-3 or 3x the fp32 oracle's own error
    S64 = {k: (v.double() if v.is_floating_point() else v) for k, v in S.items()}
    x64 = x.clone().double().requires_grad_(True)
    (-(O.log_prob(S64, spec, x64, training=True) + logdet.double()).mean()).backward()
    xd = x.to(DEV).requires_grad_(True)
    lp, ws = model(xd)
    np.testing.assert_allclose(lp.detach().cpu().numpy(), lpo.detach().numpy(), rtol=1e-5)
    (-(lp + logdet.to(DEV)).mean()).backward()
    own = rel(xo.grad.numpy(), x64.grad.numpy())
    assert rel(xd.grad.cpu().numpy(), x64.grad.numpy()) < max(5e-3, 3 * own), (
        rel(xd.grad.cpu().numpy(), x64.grad.numpy()), own)
    assert all(torch.isfinite(p.grad).all() for p in model.parameters() if p.grad is not None)
    model.eval()
    with torch.no_grad():
        lpe, _ = model(x.to(DEV))
        z, _ = model.f(x.to(DEV))
        xr = model.g(z)
    lpeo = O.log_prob(S, spec, x, training=False)
    np.testing.assert_allclose(lpe.cpu().numpy(), lpeo.detach().numpy(), rtol=1e-5)
    assert float((xr.cpu() - x).abs().max() / x.abs().max()) < 1e-5
    from realnvp_hip.trainer import FlowTrainer
    model.train()
    tr = FlowTrainer(model, B, dtype="bf16")
    tr.set_pixels(pixels(B, 3, size, seed=4).to(DEV))
    tr.capture(warmup=1)
    tr.reset_metrics()
    for _ in range(2):
        tr.step()
    assert np.isfinite(tr.mean_logll(2))


# ---------------------------------------------------------------------------
def _wgrad_case(B, H, W, cin, cout, ks, dtype, pro, seed=0):
    """rnvp_conv2d_wgrad_grouped for one conv vs torch's weight gradient of
    the same (BN+ReLU'd) input."""
    from realnvp_hip import _lib
    from realnvp_hip._lib import BNSrc, WgradGroup
    from realnvp_hip.engine import stat_shards
    from realnvp_hip.net import chan_stride, round_up
    gen = torch.Generator(device=DEV).manual_seed(seed)
    tdt = torch.float32 if dtype == "fp32" else torch.bfloat16
    M = B * H * W
    csi, cso = chan_stride(cin), chan_stride(cout)
    kp = round_up(ks * ks * csi, 64)
    x = torch.zeros(M, csi, device=DEV, dtype=tdt)
    x[:, :cin] = torch.randn(M, cin, device=DEV, generator=gen).to(tdt)
    dy = torch.zeros(M, cso, device=DEV, dtype=tdt)
    dy[:, :cout] = torch.randn(M, cout, device=DEV, generator=gen).to(tdt)
    L = _lib.lib()
    nz = int(L.wgrad_slabs(M))
    nrep = int(L.wgrad_replicas(nz))
    ws = torch.zeros(nrep, cout, kp, device=DEV)
    wsb = torch.zeros(nrep, cout, device=DEV)
    grp = WgradGroup()
    grp.dtype, grp.B, grp.H, grp.W, grp.n_conv = (0 if dtype == "fp32" else 1), B, H, W, 1
    c = grp.conv[0]
    c.x, c.cs_in, c.cin, c.ks = x.data_ptr(), csi, cin, ks
    act = x[:, :cin].double()
    keep = []
    if pro:
        xf = x[:, :cin].double()
        sh = stat_shards(M)
        sums = torch.zeros(sh, 2, cin, dtype=torch.float64, device=DEV)
        sums[0, 0], sums[0, 1] = xf.sum(0), (xf * xf).sum(0)
        gam = torch.rand(cin, device=DEV, generator=gen) + 0.5
        bet = torch.randn(cin, device=DEV, generator=gen) * 0.3
        keep += [sums, gam, bet]
        c.pro_bn_relu = 1
        c.pro = BNSrc(sums.data_ptr(), float(M), None, None, gam.data_ptr(), bet.data_ptr(), 1e-5, sh)
        mean = sums[0, 0] / M
        var = (sums[0, 1] / M - mean * mean).clamp_min(0)
        rstd = (1.0 / torch.sqrt(var + 1e-5)).float().double()
        scale = (gam.double() * rstd).float().double()
        shift = (bet.double() - mean.float().double() * gam.double() * rstd).float().double()
        act = torch.relu(xf * scale + shift).to(tdt).double()
    c.dy, c.cs_dy, c.n = dy.data_ptr(), cso, cout
    c.ws, c.wsb, c.kp, c.nz, c.nrep = ws.data_ptr(), wsb.data_ptr(), kp, nz, nrep
    L.conv2d_wgrad_grouped(C.byref(grp), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = ws.sum(0).double()
    gotb = wsb.sum(0).double()
    a4 = act.reshape(B, H, W, cin).permute(0, 3, 1, 2)
    d4 = dy[:, :cout].double().reshape(B, H, W, cout).permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(a4, (cout, cin, ks, ks), d4, padding=ks // 2)   # [co, ci, ky, kx]
    refp = torch.zeros(cout, kp, dtype=torch.float64, device=DEV)
    for ky in range(ks):
        for kx in range(ks):
            base = (ky * ks + kx) * csi
            refp[:, base:base + cin] = ref[:, :, ky, kx]
    return got, refp, gotb, d4.sum((0, 2, 3))


WGRAD_CASES = [
    ("small_pro", 4, 16, 16, 24, 40, 3, True),
    # the wide scales' 32-channel 3x3 tile class at config 1's image widths
    ("s1_3x3_w64", 16, 64, 64, 32, 32, 3, True),
    ("s1_3x3_w64_b64", 64, 64, 64, 32, 32, 3, True),
    ("s1_3x3_w32", 16, 32, 32, 32, 32, 3, True),
    ("s1_3x3_w64_nopro", 16, 64, 64, 32, 32, 3, False),
    # every config-1 scale at its full batch (slabs ending inside an image at
    # s1 / s2), config 4's 128-channel 3x3 at 64x64, and the unaligned stage
    # layout (H*W = 320: stages straddle images, a slab ends mid-image)
    ("c1_s1_1x1", 64, 64, 64, 32, 32, 1, True),
    ("c1_s1_in_3x3", 64, 64, 64, 7, 32, 3, False),
    ("c1_s2_3x3", 64, 32, 32, 64, 64, 3, True),
    ("c1_s2_1x1", 64, 32, 32, 64, 64, 1, True),
    ("c1_s3_3x3", 64, 16, 16, 128, 128, 3, True),
    ("c1_s4_3x3", 64, 8, 8, 256, 256, 3, True),
    ("c1_s5_3x3", 64, 4, 4, 512, 512, 3, True),
    ("c4_s2_3x3_w64", 64, 64, 64, 128, 128, 3, True),
    ("unaligned_slab_mid", 13, 5, 64, 32, 32, 3, True),
    ("unaligned_h3", 8, 3, 32, 32, 32, 3, True),
    ("deep_1024", 16, 2, 2, 1024, 1024, 3, True),
    ("m_2pow22", 256, 128, 128, 8, 8, 3, False),      # config 4 scale 1: M = 2^22
    ("m_above_2pow22", 257, 128, 128, 8, 16, 1, True),
    # 128 x 128 tiles (nets with mid >= 128)
    ("s4_256_3x3", 16, 8, 8, 256, 256, 3, True),
    ("s5_512_1x1", 64, 4, 4, 512, 512, 1, False),
    ("ragged_128", 4, 16, 16, 136, 200, 3, True),
    # config 4's widest nets (scale 6: mid 2048 at 4x4; in-conv 193 -> 2048)
    ("c4_s6_2048_1x1", 16, 4, 4, 2048, 2048, 1, True),
    ("c4_s6_2048_3x3", 16, 4, 4, 2048, 2048, 3, True),
    ("c4_s6_in_193", 16, 4, 4, 193, 2048, 3, False),
]


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", WGRAD_CASES, ids=[c[0] for c in WGRAD_CASES])
def test_grouped_wgrad_vs_torch(case, dtype):
    name, B, H, W, cin, cout, ks, pro = case
    got, ref, gotb, refb = _wgrad_case(B, H, W, cin, cout, ks, dtype, pro)
    tol = 1e-5 if dtype == "fp32" else 1e-4
    assert rel(got.cpu(), ref.cpu()) < tol, rel(got.cpu(), ref.cpu())
    # the bias gradient is a plain sum of M fp32 terms (~N(0,1) here): its
    # rounding error grows ~sqrt(M) (measured 1.25e-5 at M = 2^22 in fp32)
    M = B * H * W
    tolb = tol * max(1.0, (M / 2.0 ** 18) ** 0.5)
    assert rel(gotb.cpu(), refb.cpu()) < tolb, rel(gotb.cpu(), refb.cpu())


MIXED_WGRAD = [
    # B, H, W, [(ks, cin, cout, pro)] -- one grouped launch over tile classes
    (16, 64, 64, [(3, 32, 32, True), (1, 32, 32, True), (1, 32, 6, True), (3, 7, 32, False), (1, 64, 64, True)]),
    (64, 32, 32, [(3, 64, 64, True), (1, 64, 64, True), (1, 64, 12, False)]),
    (64, 8, 8, [(3, 256, 256, True), (1, 256, 256, True), (1, 32, 32, True)]),
]


@pytest.mark.parametrize("case", MIXED_WGRAD, ids=["m65536_s1", "m65536_s2", "m4096_deep"])
def test_grouped_wgrad_mixed_classes(case):
    """One rnvp_conv2d_wgrad_grouped call over convs of different tile
    classes (3x3 / 1x1, 32 / 64 / 128+ channels), bf16: from 65536 pixels up
    the launcher runs one class kernel per class (wgrad_tap.hip
    WT_SPLIT_MIN_M), below it the all-class kernel -- every conv's dW and
    bias gradient against torch's weight gradient in float64."""
    from realnvp_hip import _lib
    from realnvp_hip._lib import BNSrc, WgradGroup
    from realnvp_hip.engine import stat_shards
    from realnvp_hip.net import chan_stride, round_up
    B, H, W, convs = case
    gen = torch.Generator(device=DEV).manual_seed(5)
    M = B * H * W
    L = _lib.lib()
    nz = int(L.wgrad_slabs(M))
    nrep = int(L.wgrad_replicas(nz))
    grp = WgradGroup()
    grp.dtype, grp.B, grp.H, grp.W, grp.n_conv = 1, B, H, W, len(convs)
    keep, refs = [], []
    for i, (ks, cin, cout, pro) in enumerate(convs):
        csi, cso = chan_stride(cin), chan_stride(cout)
        kp = round_up(ks * ks * csi, 64)
        x = torch.zeros(M, csi, device=DEV, dtype=torch.bfloat16)
        x[:, :cin] = torch.randn(M, cin, device=DEV, generator=gen).to(torch.bfloat16)
        dy = torch.zeros(M, cso, device=DEV, dtype=torch.bfloat16)
        dy[:, :cout] = torch.randn(M, cout, device=DEV, generator=gen).to(torch.bfloat16)
        ws = torch.zeros(nrep, cout, kp, device=DEV)
        wsb = torch.zeros(nrep, cout, device=DEV)
        c = grp.conv[i]
        c.x, c.cs_in, c.cin, c.ks = x.data_ptr(), csi, cin, ks
        act = x[:, :cin].double()
        if pro:
            xf = x[:, :cin].double()
            sh = stat_shards(M)
            sums = torch.zeros(sh, 2, cin, dtype=torch.float64, device=DEV)
            sums[0, 0], sums[0, 1] = xf.sum(0), (xf * xf).sum(0)
            gam = torch.rand(cin, device=DEV, generator=gen) + 0.5
            bet = torch.randn(cin, device=DEV, generator=gen) * 0.3
            keep += [sums, gam, bet]
            c.pro_bn_relu = 1
            c.pro = BNSrc(sums.data_ptr(), float(M), None, None, gam.data_ptr(), bet.data_ptr(), 1e-5, sh)
            mean = sums[0, 0] / M
            var = (sums[0, 1] / M - mean * mean).clamp_min(0)
            rstd = (1.0 / torch.sqrt(var + 1e-5)).float().double()
            scale = (gam.double() * rstd).float().double()
            shift = (bet.double() - mean.float().double() * gam.double() * rstd).float().double()
            act = torch.relu(xf * scale + shift).to(torch.bfloat16).double()
        c.dy, c.cs_dy, c.n = dy.data_ptr(), cso, cout
        c.ws, c.wsb, c.kp, c.nz, c.nrep = ws.data_ptr(), wsb.data_ptr(), kp, nz, nrep
        keep += [x, dy]
        refs.append((ws, wsb, act, dy, ks, cin, cout, csi, kp))
    L.conv2d_wgrad_grouped(C.byref(grp), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    errs = []
    for i, (ws, wsb, act, dy, ks, cin, cout, csi, kp) in enumerate(refs):
        a4 = act.reshape(B, H, W, cin).permute(0, 3, 1, 2)
        d4 = dy[:, :cout].double().reshape(B, H, W, cout).permute(0, 3, 1, 2)
        ref = torch.nn.grad.conv2d_weight(a4, (cout, cin, ks, ks), d4, padding=ks // 2)
        refp = torch.zeros(cout, kp, dtype=torch.float64, device=DEV)
        for ky in range(ks):
            for kx in range(ks):
                base = (ky * ks + kx) * csi
                refp[:, base:base + cin] = ref[:, :, ky, kx]
        errs.append((i, rel(ws.sum(0).double().cpu(), refp.cpu()), rel(wsb.sum(0).double().cpu(), d4.sum((0, 2, 3)).cpu())))
    print(errs)
    assert all(e < 1e-4 and eb < 1e-4 for _, e, eb in errs), errs
