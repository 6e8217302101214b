"""What bf16 activations cost the gradient, independent of the HIP kernels
(CPU; test infrastructure): the fp32 oracle with the engine's bf16
roundings emulated in torch -- conv operands rounded to bf16, conv outputs
(stored activations) and their gradients rounded to bf16, weights rounded in
the forward only, accumulation / BatchNorm / couplings in fp32 -- against
the plain fp32 oracle on the same random-init model and batch.

    python tools/bf16_emulation.py [--size 64 --base-dim 32 --res-blocks 4 --batch 16]

Measured here: 64x64 R4 D32 B=16: log-prob 3.2e-4, gradient 0.28 (relative
L2 over all parameters); 32x32 R1 D8 B=16: 2.2e-4 / 0.063.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import realnvp_oracle as O  # noqa: E402
from formula_init import formula_value, pixels, uniform_noise  # noqa: E402


class _Round(torch.autograd.Function):
    """bf16 storage of a value and of its gradient."""
    @staticmethod
    def forward(ctx, t):
        return t.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g.bfloat16().float()


class _RoundFwd(torch.autograd.Function):
    """bf16 operand in the forward only (packed weights; fp32 weight gradient)."""
    @staticmethod
    def forward(ctx, t):
        return t.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g


def bf16_conv(S, p, x):
    w = O.wn_weight(S, p + "conv.")
    b = S.get(p + "conv.bias")
    y = torch.nn.functional.conv2d(_Round.apply(x), _RoundFwd.apply(w), b, padding=w.shape[-1] // 2)
    return _Round.apply(y)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--base-dim", type=int, default=32)
    ap.add_argument("--res-blocks", type=int, default=4)
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    torch.manual_seed(0)
    spec = O.FlowSpec(3, a.size, O.HP(a.base_dim, a.res_blocks))
    entries = O.flow_spec_entries(spec)

    def value(name, shape, trainable):      # random weights (the formula init is rank 2)
        leaf = name.split(".")[-1]
        if leaf == "weight_v":
            return torch.randn(shape) * 0.1
        if leaf == "bias":
            return torch.randn(shape) * 0.05
        return formula_value(name, shape, trainable)

    S0 = O.build_state(entries, value)
    train = O.trainable_names(entries)
    x, ld = O.logit_transform(pixels(a.batch, 3, a.size, seed=10), uniform_noise(a.batch, 3, a.size, seed=11))
    fp32_conv = O.conv

    def run(emulate):
        S = {k: v.clone() for k, v in S0.items()}
        for n in train:
            S[n].requires_grad_(True)
        O.conv = bf16_conv if emulate else fp32_conv
        try:
            lp = O.log_prob(S, spec, x.clone(), training=True)
            grads = torch.autograd.grad(-(lp + ld).mean(), [S[n] for n in train])
        finally:
            O.conv = fp32_conv
        return lp.detach(), torch.cat([gr.reshape(-1) for gr in grads])

    l32, g32 = run(False)
    l16, g16 = run(True)
    print("log-prob max rel %.3g, gradient rel L2 %.3g" % (float(((l16 - l32).abs() / l32.abs()).max()),
                                                          float((g16 - g32).norm() / g32.norm())))


if __name__ == "__main__":
    main()
