"""Would one launch covering k convs' tiles beat k launches?  Per-launch time
of a deep-family conv at M = 1024 * k (k = 1, 2, 5) against k x the M = 1024
time (same channels, same kernel configuration): the grouped-launch upper
bound for independent convs of one coupling (skip convs / first 1x1 of the
next block)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from conv_microbench import conv_case  # noqa: E402

for (name, H, W, c, ks, kw) in [("s5 1x1", 4, 4, 512, 1, dict(pro=True, stats=True)),
                                ("s5 1x1 skip", 4, 4, 512, 1, dict(acc=True)),
                                ("s5 1x1 dgrad", 4, 4, 512, 1, dict(dgrad_epi=True)),
                                ("s5 3x3", 4, 4, 512, 3, dict(pro=True, stats=True)),
                                ("s4 1x1", 8, 8, 256, 1, dict(pro=True, stats=True)),
                                ("s4 3x3", 8, 8, 256, 3, dict(pro=True, stats=True))]:
    base = None
    for k in (1, 2, 5):
        us, gbs, tf = conv_case(64 * k, H, W, c, c, ks, variant=2, **kw)
        if k == 1:
            base = us
        print("%-14s k=%d  M=%6d  %7.2f us  (k x single: %7.2f us)" % (name, k, 64 * k * H * W, us, k * base),
              flush=True)
