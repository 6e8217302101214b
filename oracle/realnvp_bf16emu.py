"""bf16 emulation of the HIP engine's s/t network (test infrastructure only:
imported by tools/make_bf16_golden.py and by tests/test_gpu_deep.py, which
re-runs it on the GPU box's host CPU to compare the benchmarked bf16 step's
largest gradient tensors element by element).  Nothing in the product path
imports this module.

The fp32 oracle (realnvp_oracle.py) with the engine's bf16 roundings at the
places its kernels round (stored conv outputs and their gradients, packed
BatchNorm+ReLU operands, packed weights in the forward, the net input and the
s/t output); BatchNorm statistics, couplings, log-det, prior and weight norm
stay fp32.  Emu(wide=True) accumulates every conv in fp64 (a second,
equally valid summation order: the spread between the two is the floor any
bf16 implementation is held to).
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

    def operand(self, S, p, x, training):
        """ReLU(BN(x)) as the MFMA operand (rounded when packed)."""
        return _R.apply(F.relu(O.batch_norm(S, p, x, training)))

    def block(self, S, p, x, training, bottleneck, skip_in, skip_p):
        r = p + "res_block."
        h = self.operand(S, p + "in_block.0.", x, training)
        if bottleneck:
            h = _R.apply(self.conv_raw(S, r + "0.", h))
            h = self.operand(S, r + "1.", h, training)
            h = _R.apply(self.conv_raw(S, r + "3.", h))
            h = self.operand(S, r + "4.", h, training)
            y = _R.apply(self.conv_raw(S, r + "6.", h) + x)       # residual in the epilogue
        else:
            h = _R.apply(self.conv_raw(S, r + "0.", h))
            h = self.operand(S, r + "1.", h, training)
            y = _R.apply(self.conv_raw(S, r + "3.", h) + x)
        out = None
        if skip_in is not None:
            out = _R.apply(skip_in + self.conv_raw(S, skip_p, y))  # skip accumulation
        return y, out

    def module(self, S, p, h0, training, hp):
        assert hp.res_blocks > 0 and hp.skip, "config-1 net (skip, res_blocks > 0)"
        x = _R.apply(self.conv_raw(S, p + "in_block.", h0))
        out = _R.apply(self.conv_raw(S, p + "in_skip.", x))
        for i in range(hp.res_blocks):
            x, out = self.block(S, p + "core_block.%d." % i, x, training, hp.bottleneck, out,
                                p + "core_skips.%d." % i)
        h = self.operand(S, p + "out_block.0.", out, training)
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
