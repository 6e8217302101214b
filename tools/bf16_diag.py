"""bf16 vs fp32 gradient agreement of the fused step, per coupling and per
parameter kind (GPU box diagnostic).

    python tools/bf16_diag.py [--batch 64] [--size 64] [--res-blocks 4] [--base-dim 32]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dl-normalizing-flows_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from formula_init import formula_state, pixels, uniform_noise  # noqa: E402


def run(dtype, a):
    import flow_realnvp
    import utils
    from realnvp_hip.trainer import FlowTrainer, arena_blocks
    dev = "cuda"
    prior = torch.distributions.Normal(torch.tensor(0.0, device=dev), torch.tensor(1.0, device=dev))
    torch.manual_seed(0)
    m = flow_realnvp.RealNVP(3, a.size, prior, utils.Hyperparameters(a.base_dim, a.res_blocks, True, True, True, True))
    if a.init == "formula":      # closed-form goldens init: rank-2 sinusoid weights (ill-conditioned)
        m.load_state_dict(formula_state(m))
    m = m.to(dev)
    tr = FlowTrainer(m, a.batch, dtype=dtype)
    pix = pixels(a.batch, 3, a.size, seed=10)
    noise = uniform_noise(a.batch, 3, a.size, seed=11)
    x, ld = utils.logit_transform(pix, noise=noise)
    tr.set_input(x, ld)
    tr.step_eager()
    torch.cuda.synchronize()
    return tr, m, arena_blocks(m)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--size", type=int, default=64)
    p.add_argument("--res-blocks", type=int, default=4)
    p.add_argument("--base-dim", type=int, default=32)
    p.add_argument("--init", default="default", choices=["default", "formula"])
    a = p.parse_args()
    t32, m32, blocks = run("fp32", a)
    t16, m16, _ = run("bf16", a)
    g32, g16 = t32.grad.double(), t16.grad.double()
    lp = (t16.lp - t32.lp).abs().max() / t32.lp.abs().max()
    print("batch %d: log-prob max rel diff %.3g; whole grad rel %.3g" % (a.batch, float(lp),
                                                                        float((g16 - g32).norm() / g32.norm())))
    names = {id(mm): n for n, mm in m32.named_modules()}
    for (off, n), mod in zip(blocks, m32.couplings()):
        s32, s16 = g32[off:off + n], g16[off:off + n]
        print("%-12s %9d params  |g| %.3e  rel %.3g" % (names[id(mod)], n, float(s32.norm()),
                                                        float((s16 - s32).norm() / s32.norm())))
    kinds = {}
    for name, prm in m32.named_parameters():
        if not prm.requires_grad:
            continue
        k = name.split(".")[-1]
        if ".in_bn." in name:
            k = "in_bn." + k
        o = t32.offsets[name]
        s32, s16 = g32[o:o + prm.numel()], g16[o:o + prm.numel()]
        d = kinds.setdefault(k, [0.0, 0.0])
        d[0] += float(((s16 - s32) ** 2).sum())
        d[1] += float((s32 ** 2).sum())
    for k, (e, n) in sorted(kinds.items()):
        print("kind %-16s |g| %.3e rel %.3g" % (k, n ** 0.5, (e / max(n, 1e-300)) ** 0.5))
    # worst single tensors among the large ones
    rows = []
    gn = float(g32.norm())
    for name, prm in m32.named_parameters():
        if not prm.requires_grad:
            continue
        o = t32.offsets[name]
        s32, s16 = g32[o:o + prm.numel()], g16[o:o + prm.numel()]
        n32 = float(s32.norm())
        if n32 > 1e-3 * gn:
            rows.append((float((s16 - s32).norm()) / n32, n32, name))
    rows.sort(reverse=True)
    for r in rows[:25]:
        print("  %.3g  |g| %.3e  %s" % r)


if __name__ == "__main__":
    main()
