"""One coupling through the HIP engine (fp32) against the float64 CPU oracle
(GPU box diagnostic): relative errors of y, log_diag_J, dL/dx (upstream
gradient on y only, on log_diag_J only, both) and the parameter gradients,
over a sweep of depths / widths.  Weights: formula_init.chirp_value
(full rank).

    python tools/coupling_diag.py [--kind ckbd] [--C 3] [--size 32] [--B 4]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("dl-normalizing-flows_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import realnvp_oracle as O  # noqa: E402
from formula_init import chirp_value, formula_state  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def run(kind, C, mid, size, R, B, cfg, bottleneck=True, skip=True):
    import modules_realnvp as MR
    import utils
    hp = utils.Hyperparameters(mid, R, bottleneck, skip, True, True)
    mod = MR.CheckerboardAffineCoupling(C, mid, size, cfg, hp) if kind == "ckbd" else \
        MR.ChannelwiseAffineCoupling(C, mid, cfg, hp)
    mod.load_state_dict(formula_state(mod, style="chirp"))
    mod = mod.cuda().train()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, C, size, size, generator=g)
    gy = torch.randn(B, C, size, size, generator=g)
    gl = torch.randn(B, C, size, size, generator=g)
    # oracle fp64
    ohp = O.HP(mid, R, bottleneck, skip)
    entries = O.coupling_spec("", kind, C, mid, ohp)
    S = {k: (v.double() if v.is_floating_point() else v) for k, v in O.build_state(entries, chirp_value).items()}
    train = O.trainable_names(entries)
    fn = O.checkerboard_coupling if kind == "ckbd" else O.channelwise_coupling
    res = {}
    for tag, wy, wl in (("gy", 1.0, 0.0), ("gl", 0.0, 1.0), ("both", 1.0, 1.0)):
        S2 = {k: v.clone() for k, v in S.items()}
        for n in train:
            S2[n].requires_grad_(True)
        xo = x.double().requires_grad_(True)
        yo, lo = fn(S2, "", xo, cfg, ohp, training=True)
        loss = (yo * gy.double() * wy + lo * gl.double() * wl).sum()
        go = torch.autograd.grad(loss, [xo] + [S2[n] for n in train])
        mod.load_state_dict(formula_state(mod, style="chirp"))
        mod.zero_grad()
        xd = x.cuda().requires_grad_(True)
        y, l = mod(xd)
        (y * gy.cuda() * wy + l * gl.cuda() * wl).sum().backward()
        params = dict(mod.named_parameters())
        pg = np.concatenate([params[n].grad.double().cpu().numpy().ravel() for n in train])
        pgo = np.concatenate([t.numpy().ravel() for t in go[1:]])
        res[tag] = (rel(xd.grad.cpu().numpy(), go[0].numpy()), rel(pg, pgo))
        if tag == "both":
            res["y"] = rel(y.detach().cpu().numpy(), yo.detach().numpy())
            res["ldj"] = rel(l.detach().cpu().numpy(), lo.detach().numpy())
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="ckbd")
    ap.add_argument("--C", type=int, default=3)
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--cfg", type=float, default=1.0)
    a = ap.parse_args()
    print("%-22s %9s %9s | %9s %9s | %9s %9s | %9s %9s" % ("case", "y", "ldj", "gx|gy", "gp|gy", "gx|gl", "gp|gl",
                                                          "gx|both", "gp|both"))
    for mid in (32, 64):
        for R in (0, 1, 2, 4, 8):
            r = run(a.kind, a.C, mid, a.size, R, a.B, a.cfg)
            print("%-22s %9.2e %9.2e | %9.2e %9.2e | %9.2e %9.2e | %9.2e %9.2e" % (
                "%s mid%d R%d" % (a.kind, mid, R), r["y"], r["ldj"], *r["gy"], *r["gl"], *r["both"]), flush=True)


if __name__ == "__main__" and "--trace" not in sys.argv:
    main()


def trace(kind, C, mid, size, R, B, cfg):
    """per-buffer data gradients of the s/t net (engine scratch g:<buffer>)
    against the fp64 oracle's autograd gradients of the same tensors"""
    import modules_realnvp as MR
    import utils
    import torch.nn.functional as F
    from realnvp_hip.net import chan_stride
    rec = {}

    def keep(name, t):
        t.retain_grad()
        rec[name] = t
        return t

    def res_module(S, p, x, training, res_blocks, bottleneck, skip):
        keep("h0", x)
        x = keep("x1_0", O.conv(S, p + "in_block.", x))
        out = O.conv(S, p + "in_skip.", x)
        for i in range(res_blocks):
            q = p + "core_block.%d." % i
            h = F.relu(O.batch_norm(S, q + "in_block.0.", x, training))
            r = q + "res_block."
            t1 = keep("t1_%d" % i, O.conv(S, r + "0.", h))
            h = F.relu(O.batch_norm(S, r + "1.", t1, training))
            t2 = keep("t2_%d" % i, O.conv(S, r + "3.", h))
            h = F.relu(O.batch_norm(S, r + "4.", t2, training))
            x = keep("x1_%d" % (i + 1), x + O.conv(S, r + "6.", h))
            out = out + O.conv(S, p + "core_skips.%d." % i, x)
        keep("out", out)
        h = F.relu(O.batch_norm(S, p + "out_block.0.", out, training))
        return keep("st", O.conv(S, p + "out_block.2.", h))

    hp = utils.Hyperparameters(mid, R, True, True, True, True)
    mod = MR.CheckerboardAffineCoupling(C, mid, size, cfg, hp) if kind == "ckbd" else \
        MR.ChannelwiseAffineCoupling(C, mid, cfg, hp)
    mod.load_state_dict(formula_state(mod, style="chirp"))
    mod = mod.cuda().train()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, C, size, size, generator=g)
    gy = torch.randn(B, C, size, size, generator=g)
    ohp = O.HP(mid, R)
    entries = O.coupling_spec("", kind, C, mid, ohp)
    S = {k: (v.double() if v.is_floating_point() else v) for k, v in O.build_state(entries, chirp_value).items()}
    fn = O.checkerboard_coupling if kind == "ckbd" else O.channelwise_coupling
    orig = O.residual_module
    O.residual_module = res_module
    try:
        xo = x.double().requires_grad_(True)
        yo, lo = fn(S, "", xo, cfg, ohp, training=True)
        (yo * gy.double()).sum().backward()
    finally:
        O.residual_module = orig
    xd = x.cuda().requires_grad_(True)
    y, l = mod(xd)
    (y * gy.cuda()).sum().backward()
    torch.cuda.synchronize()
    eng = mod.engine()
    sc = next(iter(eng._scratch.values()))
    ar = sc["arena"]
    Hs = rec["h0"].shape[2]
    for name in ["st", "out"] + sum([["x1_%d" % (i + 1), "t2_%d" % i, "t1_%d" % i] for i in reversed(range(R))],
                                      []) + ["x1_0", "h0"]:
        t = rec[name]
        ch = t.shape[1]
        cs = chan_stride(ch)
        got = ar.view("g:" + name, torch.float32, (B, Hs, Hs, cs))[..., :ch].permute(0, 3, 1, 2).double().cpu()
        d = got.numpy() - t.grad.numpy()
        rms = np.sqrt((t.grad.numpy() ** 2).mean())
        big = np.abs(d) > 1e-3 * rms
        print("  g:%-6s rel %.3e  elems>1e-3rms %d/%d  max|d|/rms %.3e  per-channel rel max %.3e" % (
            name, rel(got.numpy(), t.grad.numpy()), big.sum(), d.size, np.abs(d).max() / rms,
            max(rel(got.numpy()[:, c], t.grad.numpy()[:, c]) for c in range(ch))), flush=True)
        if name == "out":
            # where: channel / position of the largest deviations
            idx = np.argsort(-np.abs(d).ravel())[:8]
            for k in idx:
                b_, c_, y_, x_ = np.unravel_index(k, d.shape)
                print("     b%d c%d (%d,%d)  ours %.6e  truth %.6e" % (b_, c_, y_, x_, got.numpy()[b_, c_, y_, x_],
                                                                    t.grad.numpy()[b_, c_, y_, x_]))


if __name__ == "__main__" and "--trace" in sys.argv:
    # python tools/coupling_diag.py --trace kind C mid size R B
    k, c, m, sz, r, b = sys.argv[sys.argv.index("--trace") + 1:][:6]
    trace(k, int(c), int(m), int(sz), int(r), int(b), 1.0)
