"""Host-side profile (cProfile) of the drop-in loop with FusedAdam: where the
eager path spends its Python time per step (config 1, fp32).

    python3 tools/dropin_hostprof.py [steps]
"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "dl-normalizing-flows_amd"), ROOT):
    sys.path.insert(0, p)

import torch  # noqa: E402

import realnvp_hip  # noqa: E402
import utils  # noqa: E402
from bench import build_model, synthetic_pixels  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    pix = synthetic_pixels(64, 3, 64, seed=0).to(dev)
    model = build_model(64, 4, 32, 5, dev, 0)
    model.train()
    opt = realnvp_hip.FusedAdam(model.parameters(), lr=5e-4, weight_decay=5e-5)

    def step():
        x, ld = utils.logit_transform(pix)
        opt.zero_grad()
        lp, ws = model(x)
        loss = -(lp + ld).mean() + 5e-5 * ws
        loss.backward()
        opt.step()
    step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(30)


if __name__ == "__main__":
    main()
