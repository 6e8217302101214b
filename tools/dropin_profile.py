"""GPU profile of the drop-in loop train.py:176-200 drives (model(x),
loss.backward(), torch.optim.Adam): host time of each call vs device time of
each phase, fp32 and bf16, config 1 (64x64x3, R4, D32, B=64).

    python3 tools/dropin_profile.py [steps] [fused]

"fused": realnvp_hip.FusedAdam in place of torch.optim.Adam (train.py:134 changed).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "dl-normalizing-flows_amd"), ROOT):
    sys.path.insert(0, p)

import torch  # noqa: E402

import utils  # noqa: E402
from bench import build_model, synthetic_pixels  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    pix = synthetic_pixels(64, 3, 64, seed=0).to(dev)
    for dtype in ("fp32", "bf16"):
        model = build_model(64, 4, 32, 5, dev, 0)
        model.set_precision(dtype)
        model.train()
        if len(sys.argv) > 2 and sys.argv[2] == "fused":
            import realnvp_hip
            opt = realnvp_hip.FusedAdam(model.parameters(), lr=5e-4, weight_decay=5e-5)
        else:
            opt = torch.optim.Adam(model.parameters(), lr=5e-4, weight_decay=5e-5)
        ev = {k: [torch.cuda.Event(enable_timing=True) for _ in range(2)] for k in ("fwd", "bwd", "opt")}
        host = {k: 0.0 for k in ("fwd", "bwd", "opt")}
        dev_t = {k: 0.0 for k in ("fwd", "bwd", "opt")}
        total = 0.0
        for it in range(steps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            x, ld = utils.logit_transform(pix)
            opt.zero_grad()
            h0 = time.perf_counter()
            ev["fwd"][0].record()
            lp, ws = model(x)
            loss = -(lp + ld).mean() + 5e-5 * ws
            ev["fwd"][1].record()
            h1 = time.perf_counter()
            ev["bwd"][0].record()
            loss.backward()
            ev["bwd"][1].record()
            h2 = time.perf_counter()
            ev["opt"][0].record()
            opt.step()
            ev["opt"][1].record()
            h3 = time.perf_counter()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if it == 0:
                continue
            total += t1 - t0
            for k, (a, b) in (("fwd", (h0, h1)), ("bwd", (h1, h2)), ("opt", (h2, h3))):
                host[k] += b - a
                dev_t[k] += ev[k][0].elapsed_time(ev[k][1]) * 1e-3
        print("%s: %.1f ms/step (%.0f img/s) | host fwd %.1f bwd %.1f opt %.1f ms | device fwd %.1f bwd %.1f opt %.1f ms"
              % (dtype, total / steps * 1e3, 64 * steps / total, host["fwd"] / steps * 1e3, host["bwd"] / steps * 1e3,
                 host["opt"] / steps * 1e3, dev_t["fwd"] / steps * 1e3, dev_t["bwd"] / steps * 1e3,
                 dev_t["opt"] / steps * 1e3), flush=True)
        del opt, model
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
