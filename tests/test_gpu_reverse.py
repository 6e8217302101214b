"""The differentiable inverse pass (modules_realnvp.py:284-291 / 345-351 are
plain torch in the reference, so `reverse=True` carries gradients): the
engine's rnvp_coupling_reverse + rnvp_coupling_reverse_bwd + the net's and the
in part's backward against torch autograd through the CPU oracle's reverse in
float64 -- the output, log_diag_J, dL/dx and every parameter gradient, for
both coupling kinds, training (in_bn batch statistics) and eval mode, deep and
wide shapes, fp32 and bf16; and RealNVP.g (the whole inverse flow) at a small
model.  Tolerances are test_gpu_group._check_vs_oracle's (the forward step's
rule): fp32 -- per tensor within 5e-3 of the float64 truth (plus 1e-3 of the
largest gradient norm) or 3x the fp32 oracle's own error, at most 5 % of the
tensors beyond, none 10x; bf16 -- the bf16 emulation (realnvp_bf16emu, the
engine's rounding points) as the target, twice the scatter of the CPU
references as the allowance.  The inverse amplifies rounding through
exp(-log_scale): the bf16 emulation itself sits 5-7 % (dL/dx, training) and
10-14 % (parameters, eval) from the float64 truth, which is why bf16 is held to
the emulation and not to fp64.
"""
import pytest
import torch

from test_gpu_group import _check_vs_oracle, _inputs, _oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [
    # kind, in_out_dim, mid, size, batch
    ("ckbd", 3, 32, 64, 16),     # wide-scale kernels (M = 65536: band / stream families)
    ("ckbd", 12, 128, 16, 16),   # deep family
    ("chan", 12, 64, 16, 8),
    ("ckbd", 3, 32, 64, 64),     # config 1's scale 1 at its full batch (M = 262144)
]


@pytest.mark.parametrize("training", [True, False], ids=["train", "eval"])
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", CASES, ids=["%s_c%d_m%d" % (c[0], c[1], c[4] * c[3] ** 2) for c in CASES])
def test_coupling_reverse_gradients(case, dtype, training):
    kind, cio, mid, size, B = case
    mod, x, gy, gl = _inputs(kind, cio, mid, size, B)
    mod = mod.to(DEV).train(training)
    mod.compute_dtype = dtype
    xg = x.to(DEV).requires_grad_(True)
    y, ldj = mod(xg, reverse=True)
    (y * gy.to(DEV) + ldj * gl.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    grads = {n: (p.grad if p.grad is not None else torch.zeros_like(p)) for n, p in mod.named_parameters()}
    ocase = ("rev",) + tuple(case)
    _check_vs_oracle(ocase, dtype, (y, ldj, xg.grad, grads), training=training, reverse=True)
    tl = _oracle(ocase, "f64" if dtype == "fp32" else "emu", training, True)[1]
    el = float((ldj.detach().double().cpu() - tl).norm() / tl.norm())
    assert el < (1e-5 if dtype == "fp32" else 1e-2), el


def test_flow_inverse_is_differentiable():
    """RealNVP.g (flow_realnvp.py:196-249: the inverse couplings, undo
    squeeze / factor-out restores) end to end: dL/dz and the coupling
    parameters' gradients against the oracle's inverse flow in float64."""
    import realnvp_oracle as O
    from test_gpu_trainer import make_model
    model = make_model(32, 8, 1).eval()
    torch.manual_seed(3)
    z = torch.randn(2, 3, 32, 32)
    w = torch.randn(2, 3, 32, 32)
    zg = z.to(DEV).requires_grad_(True)
    x = model.g(zg)
    (x * w.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    spec = O.FlowSpec(3, 32, O.HP(8, 1))
    S = {k: (v.detach().double().cpu() if v.is_floating_point() else v.cpu()) for k, v in model.state_dict().items()}
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    for n in names:
        S[n].requires_grad_(True)
    zz = z.double().requires_grad_(True)
    xr = O.flow_g(S, spec, zz, training=False)
    grads = torch.autograd.grad((xr * w.double()).sum(), [zz] + [S[n] for n in names], allow_unused=True)

    def rel(a, b):
        return float((a.detach().double().cpu() - b).norm() / max(float(b.norm()), 1e-30))
    assert rel(x, xr.detach()) < 1e-4
    assert rel(zg.grad, grads[0]) < 1e-3, rel(zg.grad, grads[0])
    pg = dict(model.named_parameters())
    big = max(float(g.norm()) for g in grads[1:] if g is not None)
    for n, g in zip(names, grads[1:]):
        if g is None or float(g.norm()) < 1e-3 * big:
            continue
        got = pg[n].grad if pg[n].grad is not None else torch.zeros_like(pg[n])
        assert rel(got, g) < 1e-3, (n, rel(got, g))
