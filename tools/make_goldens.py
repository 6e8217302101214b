"""Generate golden vectors by importing the REFERENCE (build container only).

    python tools/make_goldens.py            # writes tests/golden/*.npz

The reference lives at /root/reference (read-only; absent on the GPU box).  It
is imported as-is; the only harness shim is ``torch.Tensor.cuda`` raising
AssertionError so the reference takes its *own* CPU fallback
(modules_realnvp.py:251-254, flow_realnvp.py:53-93) on this GPU-less ROCm
torch, where ``.cuda()`` would otherwise raise RuntimeError.  Nothing from the
reference is copied into the repo: only inputs and outputs are stored.

Parameters come from ``tests/formula_init.py`` (closed form), so the tests can
rebuild identical weights anywhere without a checkpoint.
"""
import os
import sys
import time
import warnings
import zlib

sys.dont_write_bytecode = True
warnings.filterwarnings("ignore")
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributions as D  # noqa: E402


def _no_cuda(*a, **k):
    raise AssertionError("harness shim: force the reference's CPU fallback")


torch.Tensor.cuda = _no_cuda

import flow_realnvp  # noqa: E402
import modules_realnvp  # noqa: E402
import utils as ref_utils  # noqa: E402
from formula_init import formula_state, pixels, uniform_noise  # noqa: E402

torch.set_num_threads(8)


def hps(base_dim, res_blocks, bottleneck=True, skip=True, weight_norm=True, coupling_bn=True):
    return ref_utils.Hyperparameters(base_dim=base_dim, res_blocks=res_blocks, bottleneck=bottleneck,
                                     skip=skip, weight_norm=weight_norm, coupling_bn=coupling_bn)


def f32(t):
    return t.detach().cpu().numpy()


def save(name, d):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **d)
    print("wrote", path, "%.1f KB" % (os.path.getsize(path) / 1024))


# ---------------------------------------------------------------------------
def index_maps():
    d = {}
    for size in (2, 4, 8, 16, 32, 64, 128):
        for cfg in (0.0, 1.0):
            c = modules_realnvp.AbstractCoupling.__new__(modules_realnvp.AbstractCoupling)
            d["mask_%d_%d" % (size, int(cfg))] = f32(modules_realnvp.AbstractCoupling.build_mask(c, size, cfg))
    R = flow_realnvp.RealNVP
    for shp in ((2, 3, 8, 8), (1, 6, 4, 4), (2, 12, 16, 16), (3, 24, 2, 2), (1, 3, 64, 64)):
        B, C, H, W = shp
        x = torch.arange(B * C * H * W, dtype=torch.float32).reshape(shp)
        tag = "x".join(map(str, shp))
        d["squeeze_in_" + tag] = f32(x)
        d["squeeze_out_" + tag] = f32(R.squeeze(None, x))
        d["undo_out_" + tag] = f32(R.undo_squeeze(None, R.squeeze(None, x)))
        if C * 4 % 4 == 0:
            xs = x.reshape(B, C * 4, H // 2, W // 2)
            d["undo_direct_in_" + tag] = f32(xs)
            d["undo_direct_out_" + tag] = f32(R.undo_squeeze(None, xs))
        om = R.order_matrix(None, C)
        d["order_matrix_%d" % C] = f32(om)
        on, off = R.factor_out(None, x, om)
        d["factor_on_" + tag] = f32(on)
        d["factor_off_" + tag] = f32(off)
        d["restore_out_" + tag] = f32(R.restore(None, on, off, om))
    save("index_maps.npz", d)


# ---------------------------------------------------------------------------
def logit_golden():
    d = {}
    x = pixels(4, 3, 16, seed=5)
    torch.manual_seed(1234)
    lx, ld = ref_utils.logit_transform(x.clone())
    torch.manual_seed(1234)
    noise = D.Uniform(0.0, 1.0).sample((4, 3, 16, 16))
    d.update(x=f32(x), noise=f32(noise), logit=f32(lx), logdet=f32(ld))
    z = torch.linspace(-6, 6, 4 * 3 * 16 * 16).reshape(4, 3, 16, 16)
    inv, _ = ref_utils.logit_transform(z.clone(), reverse=True)
    d.update(inv_in=f32(z), inv_out=f32(inv))
    save("logit.npz", d)


# ---------------------------------------------------------------------------
COUPLING_CASES = [
    # name, kind, in_out, mid, size, cfg, hps kwargs, B
    ("ckbd_c3_m32_s32_cfg1", "ckbd", 3, 32, 32, 1.0, dict(base_dim=32, res_blocks=2), 4),
    ("ckbd_c3_m32_s32_cfg0", "ckbd", 3, 32, 32, 0.0, dict(base_dim=32, res_blocks=2), 4),
    ("chan_c12_m64_s16_cfg0", "chan", 12, 64, 16, 0.0, dict(base_dim=32, res_blocks=2), 4),
    ("chan_c12_m64_s16_cfg1", "chan", 12, 64, 16, 1.0, dict(base_dim=32, res_blocks=2), 4),
    ("ckbd_c48_m64_s4_cfg0", "ckbd", 48, 64, 4, 0.0, dict(base_dim=32, res_blocks=1), 8),
    ("ckbd_nobott_cfg1", "ckbd", 3, 16, 8, 1.0, dict(base_dim=16, res_blocks=2, bottleneck=False), 4),
    ("ckbd_r0_bott_cfg0", "ckbd", 3, 16, 8, 0.0, dict(base_dim=16, res_blocks=0), 4),
    ("ckbd_r0_nobott_cfg1", "ckbd", 3, 16, 8, 1.0, dict(base_dim=16, res_blocks=0, bottleneck=False), 4),
    ("chan_noskip_cfg1", "chan", 12, 16, 8, 1.0, dict(base_dim=16, res_blocks=2, skip=False), 4),
    ("ckbd_nownorm_cfg1", "ckbd", 3, 16, 8, 1.0, dict(base_dim=16, res_blocks=1, weight_norm=False), 4),
    ("chan_nocbn_cfg0", "chan", 12, 16, 8, 0.0, dict(base_dim=16, res_blocks=1, coupling_bn=False), 4),
]


# deep nets (BASELINE config 3 / the reference CLI default R8 D64,
# main.py:231-240), with full-rank chirped formula weights
# (tests/formula_init.py:chirp_value): an R=8 coupling crosses the 24-conv grouped-wgrad chunk
# (4R+3 = 35 convs); the mid-1024 channelwise coupling is c3's scale-4 shape
# (C = 96 at 2x2), ~100 M parameters, so only per-tensor gradient norms and the
# small tensors' full gradients are stored (weights come from formula_init).
BIG_COUPLING_CASES = [
    # name, kind, in_out, mid, size, cfg, hps kwargs, B, full gradients
    ("ckbd_c3_m64_s32_r8_cfg1", "ckbd", 3, 64, 32, 1.0, dict(base_dim=64, res_blocks=8), 4, True),
    ("chan_c96_m1024_s2_r8_cfg0", "chan", 96, 1024, 2, 0.0, dict(base_dim=64, res_blocks=8), 4, False),
]


def make_coupling(kind, cio, mid, size, cfg, hp):
    if kind == "ckbd":
        return modules_realnvp.CheckerboardAffineCoupling(cio, mid, size, cfg, hp)
    return modules_realnvp.ChannelwiseAffineCoupling(cio, mid, cfg, hp)


def coupling_goldens(cases=None):
    cases = cases if cases is not None else [c + (True,) for c in COUPLING_CASES]
    for name, kind, cio, mid, size, cfg, hk, B, full in cases:
        t0 = time.time()
        hp = hps(**hk)
        mod = make_coupling(kind, cio, mid, size, cfg, hp)
        mod.load_state_dict(formula_state(mod, style="chirp" if "_r8_" in name else "wave"))
        g = torch.Generator().manual_seed(zlib.crc32(name.encode()) % 1000)
        x = torch.randn(B, cio, size, size, generator=g)
        gy = torch.randn(B, cio, size, size, generator=g)
        gl = torch.randn(B, cio, size, size, generator=g)
        d = dict(x=f32(x), gy=f32(gy), gl=f32(gl))
        mod.train()
        xr = x.clone().requires_grad_(True)
        y, ldj = mod(xr)
        (y * gy + ldj * gl).sum().backward()
        d.update(train_y=f32(y), train_ldj=f32(ldj), grad_x=f32(xr.grad))
        names, norms = [], []
        for n, p in mod.named_parameters():
            if p.grad is not None:
                names.append(n)
                norms.append(float(p.grad.double().norm()))
                if full or p.numel() <= 4096:
                    d["grad." + n] = f32(p.grad)
        d["grad_names"] = np.array(names)
        d["grad_norms"] = np.array(norms, dtype=np.float64)
        for k, v in mod.state_dict().items():
            if "running" in k or "num_batches" in k:
                d["after_train." + k] = v.clone().numpy()
        # train-mode reverse (batch-stat in_bn / net BNs; running out_bn)
        with torch.no_grad():
            xrev, _ = mod(x.clone(), reverse=True)
        d["train_rev"] = f32(xrev)
        for k, v in mod.state_dict().items():
            if "running" in k or "num_batches" in k:
                d["after_train_rev." + k] = v.clone().numpy()
        mod.eval()
        with torch.no_grad():
            ye, le = mod(x.clone())
            xe, _ = mod(ye.clone(), reverse=True)
        d.update(eval_y=f32(ye), eval_ldj=f32(le), eval_rec=f32(xe))
        save("coupling_%s.npz" % name, d)
        print(name, "took %.1fs" % (time.time() - t0))


# ---------------------------------------------------------------------------
MODEL_CASES = [
    # name, size, base_dim, res_blocks, B, adam steps
    ("m32_d8_r1", 32, 8, 1, 4, 3),
    ("m32_d32_r2", 32, 32, 2, 4, 3),
    ("m64_d32_r4", 64, 32, 4, 2, 3),
]
# BASELINE config 3 (32x32x3, R8, D64: 923.6 M parameters) at B=2, and config 1
# at its full benchmarked batch B=64.  "lite" goldens keep the per-sample and
# per-tensor outputs only (inputs are regenerated from the pixel / noise seeds).
BIG_MODEL_CASES = [
    ("m32_d64_r8", 32, 64, 8, 2, 0),
    ("m64_d32_r4_b64", 64, 32, 4, 64, 0),
]


def model_inputs(B, size):
    """the logit-transformed synthetic batch every model golden uses
    (utils.py:44-72 with explicit noise)."""
    pix = pixels(B, 3, size, seed=10)
    noise = uniform_noise(B, 3, size, seed=11)
    x = (pix * 255.0 + noise) / 256.0
    x = ((x * 2.0 - 1.0) * 0.9 + 1.0) / 2.0
    x_in = torch.log(x) - torch.log(1.0 - x)
    pre = torch.tensor(np.log(0.9) - np.log(0.1))
    logdet = (torch.nn.functional.softplus(x_in) + torch.nn.functional.softplus(-x_in)
              - torch.nn.functional.softplus(-pre)).sum(dim=(1, 2, 3))
    return pix, noise, x_in, logdet


def lite_model_golden(name, size, bd, rb, B):
    t0 = time.time()
    prior = D.Normal(torch.tensor(0.0), torch.tensor(1.0), validate_args=False)
    model = flow_realnvp.RealNVP(3, size, prior, hps(bd, rb))
    model.load_state_dict(formula_state(model))
    print(name, "built in %.1fs" % (time.time() - t0))
    _, _, x_in, logdet = model_inputs(B, size)
    d = dict(batch=np.array(B), logdet=f32(logdet))
    model.train()
    xr = x_in.clone().requires_grad_(True)
    lp, ws = model(xr)
    loss = -(lp + logdet).mean() + 5e-5 * ws
    loss.backward()
    d.update(train_logprob=f32(lp), weight_scale=f32(ws), loss=f32(loss),
             grad_x_norm=np.array(float(xr.grad.double().norm())), grad_x_sum=np.array(float(xr.grad.double().sum())))
    names, norms = [], []
    for n, p in model.named_parameters():
        if p.grad is not None:
            names.append(n)
            norms.append(float(p.grad.double().norm()))
            if n.endswith("scale") or n.endswith("scale_shift"):
                d["grad." + n] = f32(p.grad)
    d["grad_names"] = np.array(names)
    d["grad_norms"] = np.array(norms, dtype=np.float64)
    for k, v in model.state_dict().items():
        if "running" in k:
            d["after_train." + k] = v.clone().numpy()
    model.eval()
    with torch.no_grad():
        lpe, _ = model(x_in.clone())
        ze, _ = model.f(x_in.clone())
        xrec = model.g(ze.clone())
    d.update(eval_logprob=f32(lpe),
             eval_rec_err=np.array(float((xrec - x_in).abs().max() / x_in.abs().max())))
    save("model_%s.npz" % name, d)
    print(name, "took %.1fs" % (time.time() - t0))


def model_goldens():
    for name, size, bd, rb, B, steps in MODEL_CASES:
        t0 = time.time()
        prior = D.Normal(torch.tensor(0.0), torch.tensor(1.0), validate_args=False)
        model = flow_realnvp.RealNVP(3, size, prior, hps(bd, rb))
        model.load_state_dict(formula_state(model))
        pix = pixels(B, 3, size, seed=10)
        noise = uniform_noise(B, 3, size, seed=11)
        # logit_transform with explicit noise: seed the global RNG the reference draws from
        x = (pix * 255.0 + noise) / 256.0
        x = ((x * 2.0 - 1.0) * 0.9 + 1.0) / 2.0
        x_in = torch.log(x) - torch.log(1.0 - x)
        pre = torch.tensor(np.log(0.9) - np.log(0.1))
        logdet = (torch.nn.functional.softplus(x_in) + torch.nn.functional.softplus(-x_in)
                  - torch.nn.functional.softplus(-pre)).sum(dim=(1, 2, 3))
        d = dict(pixels=f32(pix), noise=f32(noise), x=f32(x_in), logdet=f32(logdet))
        model.train()
        xr = x_in.clone().requires_grad_(True)
        lp, ws = model(xr)
        logll = (lp + logdet).mean()
        loss = -logll + 5e-5 * ws
        loss.backward()
        d.update(train_logprob=f32(lp), weight_scale=f32(ws), loss=f32(loss), grad_x=f32(xr.grad))
        names, norms = [], []
        for n, p in model.named_parameters():
            if p.grad is not None:
                names.append(n)
                norms.append(float(p.grad.norm()))
        d["grad_names"] = np.array(names)
        d["grad_norms"] = np.array(norms, dtype=np.float64)
        # a few full gradient tensors
        for n in names:
            if n.endswith("scale") or n.endswith("scale_shift") or ".in_bn." in n:
                d["grad." + n] = f32(dict(model.named_parameters())[n].grad)
        with torch.no_grad():
            z, ldj = model.f(x_in.clone())
        d.update(train_z=f32(z), train_ldj=f32(ldj))
        rs = {k: v.clone() for k, v in model.state_dict().items() if "running" in k}
        for k, v in rs.items():
            d["after_train." + k] = v.clone().numpy()
        model.eval()
        with torch.no_grad():
            lpe, _ = model(x_in.clone())
            ze, le = model.f(x_in.clone())
            xrec = model.g(ze.clone())
            z0 = torch.randn(B, 3, size, size, generator=torch.Generator().manual_seed(7))
            xs = model.g(z0)
        d.update(eval_logprob=f32(lpe), eval_z=f32(ze), eval_ldj=f32(le), eval_rec=f32(xrec),
                 sample_z=f32(z0), sample_x=f32(xs))
        # 3-step trajectory of the train.py:176-200 loop from a fresh formula init
        model.load_state_dict(formula_state(model))
        model.train()
        opt = torch.optim.Adam(model.parameters(), lr=5e-4, weight_decay=5e-5)
        losses, lls = [], []
        for s in range(steps):
            pix_s = pixels(B, 3, size, seed=100 + s)
            noise_s = uniform_noise(B, 3, size, seed=200 + s)
            xs_ = (pix_s * 255.0 + noise_s) / 256.0
            xs_ = ((xs_ * 2.0 - 1.0) * 0.9 + 1.0) / 2.0
            xl = torch.log(xs_) - torch.log(1.0 - xs_)
            ldt = (torch.nn.functional.softplus(xl) + torch.nn.functional.softplus(-xl)
                   - torch.nn.functional.softplus(-pre)).sum(dim=(1, 2, 3))
            opt.zero_grad()
            lp_s, ws_s = model(xl)
            ll = (lp_s + ldt).mean()
            ls = -ll + 5e-5 * ws_s
            ls.backward()
            opt.step()
            losses.append(float(ls))
            lls.append(float(ll))
        d["traj_loss"] = np.array(losses)
        d["traj_logll"] = np.array(lls)
        with torch.no_grad():
            model.eval()
            lp_after, _ = model(x_in.clone())
        d["traj_eval_logprob_after"] = f32(lp_after)
        save("model_%s.npz" % name, d)
        print(name, "took %.1fs" % (time.time() - t0))


def grads_golden(name="m64_d32_r4_b64", size=64, bd=32, rb=4, B=64):
    """Gradient VALUES of the benchmarked configuration (config 1, B=64,
    formula weights, the lite golden's batch and loss): per-tensor projection
    checksums (tests/formula_init.py:projections) of the reference's fp32
    gradients and of the oracle's float64 truth, and for the 10 largest
    tensors and dL/dx the element-wise fp32 error floors (relative L2 against
    the truth) of the reference and of the fp32 oracle, which the GPU test
    re-runs to compare those tensors element by element."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import realnvp_oracle as O
    from formula_init import formula_value, largest, projection_matrix
    t0 = time.time()
    prior = D.Normal(torch.tensor(0.0), torch.tensor(1.0), validate_args=False)
    model = flow_realnvp.RealNVP(3, size, prior, hps(bd, rb))
    model.load_state_dict(formula_state(model))
    _, _, x_in, logdet = model_inputs(B, size)
    model.train()
    xr = x_in.clone().requires_grad_(True)
    lp, ws = model(xr)
    (-(lp + logdet).mean() + 5e-5 * ws).backward()
    names = [n for n, p in model.named_parameters() if p.grad is not None]
    params = dict(model.named_parameters())
    ref = {n: params[n].grad.detach().clone() for n in names}
    ref_gx = xr.grad.detach().clone()
    print(name, "reference step %.1fs" % (time.time() - t0), flush=True)

    def oracle(dtype):
        spec = O.FlowSpec(3, size, O.HP(bd, rb))
        entries = O.flow_spec_entries(spec)
        S = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in O.build_state(entries, formula_value).items()}
        train = O.trainable_names(entries)
        assert train == names
        for n in train:
            S[n].requires_grad_(True)
        x = x_in.clone().to(dtype).requires_grad_(True)
        lpo = O.log_prob(S, spec, x, training=True)
        wso = O.weight_scale(S, O.param_names(entries), lambda n: n in set(train))
        loss = -(lpo + logdet.to(dtype)).mean() + O.SCALE_REG * wso
        g = torch.autograd.grad(loss, [x] + [S[n] for n in train])
        return dict(zip(train, g[1:])), g[0]
    truth, truth_gx = oracle(torch.float64)
    o32, o32_gx = oracle(torch.float32)
    print(name, "oracle fp64 + fp32 %.1fs" % (time.time() - t0), flush=True)

    def trel(a, b):
        a, b = a.double(), b.double()
        return float((a - b).norm() / b.norm())
    big = largest(names, [ref[n].numel() for n in names])
    d = dict(grad_names=np.array(names), ref_grad_proj=projection_matrix([ref[n] for n in names]),
             truth_grad_proj=projection_matrix([truth[n] for n in names]),
             oracle_grad_proj=projection_matrix([o32[n] for n in names]),
             full_names=np.array(big),
             ref_full_err=np.array([trel(ref[n], truth[n]) for n in big]),
             oracle_full_err=np.array([trel(o32[n], truth[n]) for n in big]),
             ref_grad_x_err=np.float64(trel(ref_gx, truth_gx)), oracle_grad_x_err=np.float64(trel(o32_gx, truth_gx)),
             oracle_vs_ref_full=np.array([trel(o32[n], ref[n]) for n in big]))
    print("full-tensor errors vs fp64: reference", np.round(d["ref_full_err"], 5), "oracle",
          np.round(d["oracle_full_err"], 5), "dL/dx", float(d["ref_grad_x_err"]), float(d["oracle_grad_x_err"]))
    save("grads_%s.npz" % name, d)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    which = sys.argv[1:2] or ["index", "logit", "coupling", "model"]
    if "grads" in which:
        grads_golden()
    if "index" in which:
        index_maps()
    if "logit" in which:
        logit_golden()
    if "coupling" in which:
        coupling_goldens()
    if "model" in which:
        model_goldens()
    if "big_coupling" in which:
        coupling_goldens(BIG_COUPLING_CASES)
    if "big_model" in which:
        for c in BIG_MODEL_CASES:
            if not sys.argv[2:] or c[0] in sys.argv[2:]:
                lite_model_golden(*c[:5])


def init_golden():
    """Per-key checksums of the reference's default init under torch.manual_seed(0)."""
    d = {}
    for name, size, bd, rb in (("m32_d8_r1", 32, 8, 1), ("m16_d4_r2_nobott", 16, 4, 2)):
        hp = hps(bd, rb, bottleneck=(name.find("nobott") < 0))
        torch.manual_seed(0)
        prior = D.Normal(torch.tensor(0.0), torch.tensor(1.0), validate_args=False)
        model = flow_realnvp.RealNVP(3, size, prior, hp)
        keys = list(model.state_dict().keys())
        d[name + ".keys"] = np.array(keys)
        d[name + ".sum"] = np.array([float(v.double().sum()) for v in model.state_dict().values()])
        d[name + ".sumsq"] = np.array([float(v.double().pow(2).sum()) for v in model.state_dict().values()])
    save("init_seed0.npz", d)


if __name__ == "__main__" and "init" in sys.argv[1:]:
    init_golden()
