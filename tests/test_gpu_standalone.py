"""Standalone calls of the s/t-network submodules (modules_realnvp.py:36-194):
WeightNormConv2d through the HIP kernels one at a time
(realnvp_hip.standalone), ResidualBlock / ResidualModule composed as the
reference composes them, each against the oracle's restatement
(oracle/realnvp_oracle.py: conv / residual_block / residual_module) in
float64 on the CPU.  Inside a coupling these modules never run standalone
(the engine fuses them); this is the API the reference also exposes."""
import numpy as np
import pytest
import torch

import realnvp_oracle as O

DEV = "cuda"


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _state64(mod):
    return {k: v.detach().cpu().double().clone() for k, v in mod.state_dict().items()}


def test_standalone_conv_refuses_cpu():
    import modules_realnvp as M
    conv = M.WeightNormConv2d(4, 8, (3, 3), padding=1)
    with pytest.raises(RuntimeError):
        conv(torch.zeros(1, 4, 4, 4))
    rm = M.ResidualModule(4, 8, 4, 1, True, True, True)
    with pytest.raises(RuntimeError):
        rm(torch.zeros(1, 4, 4, 4))


CONVS = [
    # cin, cout, k, bias, weight_norm, scale, B, H, W
    (7, 32, 3, True, True, False, 4, 16, 16),      # the net's in conv (frozen g)
    (32, 32, 1, True, True, True, 4, 16, 16),      # skip / out-of-block 1x1 (trainable g)
    (64, 64, 3, False, True, False, 2, 8, 8),      # bottleneck 3x3, no bias
    (24, 40, 3, True, False, False, 3, 9, 7),      # plain nn.Conv2d (weight_norm=False), ragged shape
    (256, 96, 1, True, True, True, 8, 4, 4),       # deep-scale out conv
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CONVS, ids=["c%d_%d_k%d_b%d_wn%d_s%d" % c[:6] for c in CONVS])
def test_weightnorm_conv_standalone_vs_float64(case):
    import modules_realnvp as M
    cin, cout, k, bias, wn, scale, B, H, W = case
    torch.manual_seed(0)
    conv = M.WeightNormConv2d(cin, cout, (k, k), padding=k // 2, bias=bias, weight_norm=wn, scale=scale).to(DEV)
    if wn and scale:
        with torch.no_grad():
            conv.conv.weight_g.mul_(torch.linspace(0.5, 1.5, cout, device=DEV).view(-1, 1, 1, 1))
    x = torch.randn(B, cin, H, W, device=DEV, requires_grad=True)
    y = conv(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    # float64 restatement (oracle.conv = WeightNormConv2d.forward, modules_realnvp.py:64-71)
    S = {"" + n: t.requires_grad_(True) if t.is_floating_point() else t for n, t in _state64(conv).items()}
    xr = x.detach().cpu().double().requires_grad_(True)
    yr = O.conv(S, "", xr)
    yr.backward(gy.cpu().double())
    assert rel(y.detach().cpu(), yr.detach()) < 1e-5
    assert rel(x.grad.cpu(), xr.grad) < 1e-5
    for n, p in conv.named_parameters():
        if p.requires_grad:
            assert p.grad is not None, n
            assert rel(p.grad.cpu(), S[n].grad) < 2e-5, n
        else:
            assert p.grad is None, n


@pytest.mark.gpu
@pytest.mark.parametrize("bottleneck", [True, False])
def test_residual_block_standalone_vs_oracle(bottleneck):
    import modules_realnvp as M
    torch.manual_seed(1)
    blk = M.ResidualBlock(32, bottleneck, True).to(DEV).train()
    S = _state64(blk)
    x = torch.randn(4, 32, 8, 8, device=DEV, requires_grad=True)
    y = blk(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    xr = x.detach().cpu().double().requires_grad_(True)
    yr = O.residual_block(S, "", xr, True, bottleneck)
    yr.backward(gy.cpu().double())
    assert rel(y.detach().cpu(), yr.detach()) < 5e-5
    assert rel(x.grad.cpu(), xr.grad) < 1e-4
    # running statistics moved like the reference's (train-mode BatchNorm2d)
    for n, b in blk.state_dict().items():
        if "running" in n:
            assert rel(b.cpu(), S[n]) < 1e-5, n


@pytest.mark.gpu
@pytest.mark.parametrize("res_blocks,bottleneck,skip", [(2, True, True), (1, False, False), (0, True, True)])
def test_residual_module_standalone_vs_oracle(res_blocks, bottleneck, skip):
    """ResidualModule(in, dim, out) standalone, train and eval mode, incl. the
    res_blocks = 0 variant (modules_realnvp.py:153-173)."""
    import modules_realnvp as M
    torch.manual_seed(2)
    rm = M.ResidualModule(13, 32, 12, res_blocks, bottleneck, skip, True).to(DEV).train()
    S = _state64(rm)
    x = torch.randn(4, 13, 8, 8, device=DEV, requires_grad=True)
    y = rm(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    xr = x.detach().cpu().double().requires_grad_(True)
    yr = O.residual_module(S, "", xr, True, res_blocks, bottleneck, skip)
    yr.backward(gy.cpu().double())
    assert rel(y.detach().cpu(), yr.detach()) < 5e-5
    assert rel(x.grad.cpu(), xr.grad) < 1e-4
    rm.eval()
    with torch.no_grad():
        ye = rm(x)
    ys = O.residual_module(S, "", x.detach().cpu().double(), False, res_blocks, bottleneck, skip)
    assert rel(ye.cpu(), ys) < 5e-5
