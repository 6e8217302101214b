"""GPU probe: torch.optim.Adam over the config-1 drop-in model's 1,960
parameter tensors -- default / foreach / fused implementations, and the
implementation torch picks by default."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "dl-normalizing-flows_amd"), ROOT):
    sys.path.insert(0, p)

import torch  # noqa: E402
from torch.optim.optimizer import _default_to_fused_or_foreach  # noqa: E402

from bench import build_model  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = build_model(64, 4, 32, 5, dev, 0)
    params = [p for p in model.parameters() if p.requires_grad]
    for p in params:
        p.grad = torch.randn_like(p) * 1e-3
    print("params", len(params), "default (fused, foreach) =", _default_to_fused_or_foreach(params, False, False))
    for kw in ({}, {"foreach": True}, {"foreach": False}, {"fused": True}):
        opt = torch.optim.Adam(params, lr=5e-4, weight_decay=5e-5, **kw)
        for _ in range(2):
            opt.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            opt.step()
        e1.record()
        h = (time.perf_counter() - t0) / 5 * 1e3
        torch.cuda.synchronize()
        print("%-18s device %.2f ms/step, host %.2f ms/step" % (kw or "default", e0.elapsed_time(e1) / 5, h),
              flush=True)
        del opt


if __name__ == "__main__":
    main()
