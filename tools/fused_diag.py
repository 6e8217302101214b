"""GPU diagnostic: the fused parameter pass against the separate launches, one
step at a time, per named parameter and per packed image.

    python3 tools/fused_diag.py [size bd rb dtype steps [graph]]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "dl-normalizing-flows_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import flow_realnvp  # noqa: E402
import utils  # noqa: E402
from formula_init import formula_state, pixels  # noqa: E402
from realnvp_hip.trainer import FlowTrainer  # noqa: E402

DEV = "cuda"


def make(size, bd, rb, dtype, mode):
    prior = torch.distributions.Normal(torch.tensor(0.0, device=DEV), torch.tensor(1.0, device=DEV))
    m = flow_realnvp.RealNVP(3, size, prior, utils.Hyperparameters(bd, rb, True, True, True, True))
    m.load_state_dict(formula_state(m))
    tr = FlowTrainer(m.to(DEV), 4, dtype=dtype, param_pass=mode)
    tr.set_pixels(pixels(4, 3, size, seed=5).to(DEV))
    return tr


def images(tr):
    out = {}
    for st in tr.stages:
        if st[0] != "coupling":
            continue
        ws = st[2].weights(tr.dtype)
        dt = torch.bfloat16 if tr.dtype == "bf16" else torch.float32
        for name in ws["geo"]:
            for kind in ("wf:", "wd:"):
                out[(id(st[2]), kind + name)] = ws["arena"].view(kind + name, dt).float().clone()
            out[(id(st[2]), "norm:" + name)] = ws["arena"].view("norm:" + name, torch.float32).clone()
    return out


def main():
    size, bd, rb = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (64, 32, 4)
    dtype = sys.argv[4] if len(sys.argv) > 4 else "bf16"
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    graph = len(sys.argv) > 6 and sys.argv[6] == "graph"
    fu, se = make(size, bd, rb, dtype, "fused"), make(size, bd, rb, dtype, "separate")
    if graph:
        fu.capture(warmup=1)
        se.capture(warmup=1)
    names = [n for n, _ in fu.model.named_parameters()]
    for step in range(steps):
        fu.step()
        se.step()
        torch.cuda.synchronize()
        print("== after step", step + 1)
        for arena in ("param", "grad", "exp_avg", "exp_avg_sq"):
            a, b = getattr(fu, arena), getattr(se, arena)
            bad = []
            for n in names:
                o = fu.offsets[n]
                k = dict(fu.model.named_parameters())[n].numel()
                d = float((a[o:o + k] - b[o:o + k]).abs().max())
                if d > 0:
                    bad.append((d, n, int((a[o:o + k] != b[o:o + k]).sum()), k))
            bad.sort(reverse=True)
            print("%-10s %d tensors differ" % (arena, len(bad)))
            for d, n, c, k in bad[:8]:
                print("    %.3e  %6d/%-8d %s" % (d, c, k, n))
        imf = images(fu)
        for t in fu.wn_tables:
            fu._wn_fwd(t)
        torch.cuda.synchronize()
        imr = images(fu)
        ims = images(se)
        nd = sum(1 for k, (a, b) in enumerate(zip(imr.values(), ims.values())) if not torch.equal(a, b))
        print("images: wn_fwd(fused params) vs separate's own:", nd, "differ")
        nb = 0
        for key in imf:
            d = (imf[key] - imr[key]).abs()
            if float(d.max()) > 0:
                nb += 1
                if nb <= 12:
                    i = int(d.argmax())
                    print("  image %-60s max %.3e  n %d  at %d (fused %.6g ref %.6g)" % (
                        key[1], float(d.max()), int((d > 0).sum()), i, float(imf[key][i]), float(imr[key][i])))
        print("images differing:", nb, "of", len(imf))


if __name__ == "__main__":
    main()
