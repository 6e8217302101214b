"""bf16 emulation of the HIP engine's s/t network (test infrastructure only:
imported by tools/make_bf16_golden.py and by tests/test_gpu_deep.py, which
re-runs it on the GPU box's host CPU to compare the benchmarked bf16 step's
largest gradient tensors element by element).  Nothing in the product path
imports this module.

The fp32 oracle (realnvp_oracle.py) with the engine's bf16 roundings at the
places its kernels round (stored conv outputs and their gradients, packed
BatchNorm+ReLU operands, packed weights in the forward, the net input and the
s/t output); BatchNorm statistics, couplings, log-det, prior and weight norm
stay fp32.  As in the engine, a BatchNorm's batch statistics are those of the
UNROUNDED conv output (the conv epilogue reduces its fp32 accumulators
before the bf16 store), applied to the stored bf16 values; its backward is
the usual formula on the stored values, rounded once (_BNStat).
Emu(wide=True) accumulates every conv in fp64 (a second, equally valid
summation order: the spread between the two is the floor any bf16
implementation is held to).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import realnvp_oracle as O  # noqa: E402
from formula_init import projection_matrix  # noqa: E402


class _R(torch.autograd.Function):
    """bf16 storage of a value and of the gradient flowing back into it."""
    @staticmethod
    def forward(ctx, t):
        return t.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g.bfloat16().float()


class _RF(torch.autograd.Function):
    """bf16 operand in the forward only (packed weights)."""
    @staticmethod
    def forward(ctx, t):
        return t.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g


class _BNStat(torch.autograd.Function):
    """Training-mode BatchNorm (realnvp_oracle.batch_norm semantics) that
    normalises the stored values `xs` with the batch statistics of the raw,
    unrounded values `xr` they were rounded from (the engine's rounding
    point).  Backward: dL/dxs by the BatchNorm formula on the stored values
    (the engine's BN-backward apply / dgrad epilogue), nothing to xr (the
    rounding is straight-through: the caller's _R passes dL/dxs back to xr,
    rounded once)."""
    @staticmethod
    def forward(ctx, xs, xr, w, b):
        mean = xr.mean(dim=(0, 2, 3))
        var = (xr - mean.view(1, -1, 1, 1)).pow(2).mean(dim=(0, 2, 3))
        rstd = 1.0 / torch.sqrt(var + O.BN_EPS)
        xhat = (xs - mean.view(1, -1, 1, 1)) * rstd.view(1, -1, 1, 1)
        ctx.save_for_backward(xhat, rstd, w)
        ctx.stats = (mean.detach(), var.detach())
        return xhat * w.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)

    @staticmethod
    def backward(ctx, dy):
        xhat, rstd, w = ctx.saved_tensors
        n = dy.numel() // dy.shape[1]
        db = dy.sum(dim=(0, 2, 3))
        dw = (dy * xhat).sum(dim=(0, 2, 3))
        dxs = (w * rstd).view(1, -1, 1, 1) * (dy - (db / n).view(1, -1, 1, 1) - xhat * (dw / n).view(1, -1, 1, 1))
        return dxs, None, dw, db


def _bn_stat(S, p, xs, xr, training):
    """ReLU-less BatchNorm of stored xs with xr's batch statistics; running
    statistics updated from them as nn.BatchNorm2d does."""
    if not training:
        return O.batch_norm(S, p, xs, training)
    y = _BNStat.apply(xs, xr, S[p + "weight"], S[p + "bias"])
    n = xr.numel() // xr.shape[1]
    with torch.no_grad():
        mean = xr.detach().mean(dim=(0, 2, 3))
        var = (xr.detach() - mean.view(1, -1, 1, 1)).pow(2).mean(dim=(0, 2, 3))
        S[p + "running_mean"].mul_(1 - O.BN_MOMENTUM).add_(O.BN_MOMENTUM * mean)
        S[p + "running_var"].mul_(1 - O.BN_MOMENTUM).add_(O.BN_MOMENTUM * var * (n / max(n - 1, 1)))
        S[p + "num_batches_tracked"].add_(1)
    return y


class Emu:
    """The oracle's residual module with the engine's bf16 rounding points;
    wide=True accumulates every conv in fp64 (the summation-order variant)."""

    def __init__(self, wide):
        self.wide = wide

    def conv_raw(self, S, p, x):
        w = _RF.apply(O.wn_weight(S, p + "conv."))
        b = S.get(p + "conv.bias")
        pad = w.shape[-1] // 2
        if self.wide:
            return _Wide.apply(x, w, pad) + (b.view(1, -1, 1, 1) if b is not None else 0.0)
        return F.conv2d(x, w, b, padding=pad)

    def operand(self, S, p, x, xr, training):
        """ReLU(BN(x)) as the MFMA operand (rounded when packed); x the stored
        bf16 activation, xr the unrounded value whose statistics the engine's
        producing epilogue reduced"""
        return _R.apply(F.relu(_bn_stat(S, p, x, xr, training)))

    def block(self, S, p, x, xr, training, bottleneck, skip_in, skip_p):
        r = p + "res_block."
        h = self.operand(S, p + "in_block.0.", x, xr, training)
        if bottleneck:
            hr = self.conv_raw(S, r + "0.", h)
            h = self.operand(S, r + "1.", _R.apply(hr), hr, training)
            hr = self.conv_raw(S, r + "3.", h)
            h = self.operand(S, r + "4.", _R.apply(hr), hr, training)
            yr = self.conv_raw(S, r + "6.", h) + x        # residual in the epilogue
        else:
            hr = self.conv_raw(S, r + "0.", h)
            h = self.operand(S, r + "1.", _R.apply(hr), hr, training)
            yr = self.conv_raw(S, r + "3.", h) + x
        y = _R.apply(yr)
        out = outr = None
        if skip_in is not None:
            outr = skip_in + self.conv_raw(S, skip_p, y)   # skip accumulation
            out = _R.apply(outr)
        return y, yr, out, outr

    def module(self, S, p, h0, training, hp):
        assert hp.res_blocks > 0 and hp.skip, "config-1 net (skip, res_blocks > 0)"
        xr = self.conv_raw(S, p + "in_block.", h0)
        x = _R.apply(xr)
        outr = self.conv_raw(S, p + "in_skip.", x)
        out = _R.apply(outr)
        for i in range(hp.res_blocks):
            x, xr, out, outr = self.block(S, p + "core_block.%d." % i, x, xr, training, hp.bottleneck, out,
                                          p + "core_skips.%d." % i)
        h = self.operand(S, p + "out_block.0.", out, outr, training)
        return _R.apply(self.conv_raw(S, p + "out_block.2.", h))


class _Wide(torch.autograd.Function):
    """conv2d accumulated in fp64, result rounded to fp32 (forward and both
    backward products): an fp32-grade conv with a different summation."""
    @staticmethod
    def forward(ctx, x, w, pad):
        ctx.save_for_backward(x, w)
        ctx.pad = pad
        return F.conv2d(x.double(), w.double(), padding=pad).float()

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        gd = g.double()
        gx = torch.nn.grad.conv2d_input(x.shape, w.double(), gd, padding=ctx.pad).float()
        gw = torch.nn.grad.conv2d_weight(x.double(), w.shape, gd, padding=ctx.pad).float()
        return gx, gw, None


def run(S0, spec, train, x, ld, emu, full=False):
    """(log-prob [B], loss, per-tensor gradient norms, projection checksums
    [n, K]) of one training step; full=True also returns the gradient
    tensors and dL/dx."""
    S = {k: v.clone() for k, v in S0.items()}
    for n in train:
        S[n].requires_grad_(True)
    saved = O.residual_module
    if emu is not None:
        def rm(S_, p, h, training, res_blocks, bottleneck, skip):
            return emu.module(S_, p, _R.apply(h), training, spec.hp)
        O.residual_module = rm
    try:
        xr = x.clone().requires_grad_(True)
        lp = O.log_prob(S, spec, xr, training=True)
        names = O.param_names(O.flow_spec_entries(spec))
        ws = O.weight_scale(S, names, lambda n: n in train)
        loss = -(lp + ld).mean() + 5e-5 * ws
        grads = torch.autograd.grad(loss, [xr] + [S[n] for n in train], allow_unused=True)
    finally:
        O.residual_module = saved
    gx, grads = grads[0], [g if g is not None else torch.zeros_like(S[n]) for g, n in zip(grads[1:], train)]
    norms = np.array([float(g.double().norm()) for g in grads])
    out = (lp.detach().numpy().astype(np.float64), float(loss), norms, projection_matrix(grads))
    return out + ((dict(zip(train, grads)), gx) if full else ())
