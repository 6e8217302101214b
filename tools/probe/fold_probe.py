"""Where do the folded and unfolded backward schedules first differ?  Runs one
deep-scale coupling (drop-in module) with engine.FOLD_BN on and off and
compares every gradient / BatchNorm-sum buffer of the two engines' scratch
arenas in backward-program order.  Usage: fold_probe.py [case] [dtype]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "dl-normalizing-flows_amd"), os.path.join(ROOT, "oracle")]

from test_gpu_group import _inputs  # noqa: E402
from realnvp_hip import engine  # noqa: E402

CASES = {"s4": ("ckbd", 24, 256, 8, 64), "s3": ("ckbd", 12, 128, 16, 64), "s5": ("ckbd", 48, 512, 4, 64)}


def run(case, dtype, fold):
    kind, cio, mid, size, B = CASES[case]
    engine.FOLD_BN = fold
    mod, x, gy, gl = _inputs(kind, cio, mid, size, B)
    mod = mod.cuda().train()
    mod.compute_dtype = dtype
    x = x.cuda().requires_grad_(True)
    y, ldj = mod(x)
    (y * gy.cuda() + ldj * gl.cuda()).sum().backward()
    torch.cuda.synchronize()
    eng = mod.engine()
    sc = list(eng._scratch.values())[0]
    ar = sc["arena"]
    bufs = {n: ar.view(n, torch.uint8).clone() for n in ar.slots}
    sv = [sv for pool in eng._saved_pool.values() for sv in pool][0]
    return eng, bufs, sv["bwd_plan"][1][0]


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "s4"
    dtype = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    tdt = torch.float32 if dtype == "fp32" else torch.bfloat16
    e0, b0, it0 = run(case, dtype, False)
    e1, b1, it1 = run(case, dtype, True)
    print("items unfolded %d, folded %d" % (len(it0), len(it1)))
    for kind, c, nb, fl, bn, rw in it1:
        print("  %-5s %-40s reads %s writes %s" % (kind, bn or "", sorted(rw[0]), sorted(rw[1])))
    for n in b0:
        if n in ("gtmp", "gtmp2"):
            continue
        a, b = b0[n], b1[n]
        if n.startswith("e:") or n.endswith("_sums") or n in ("in_bwd_ext", "gscale_part"):
            a, b = a.view(torch.float64), b.view(torch.float64)
        else:
            a, b = a.view(tdt).float(), b.view(tdt).float()
        d = float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-30))
        print("%-40s rel %.3g  |unfolded| %.4g" % (n, d, float(a.double().norm())))


if __name__ == "__main__":
    main()
