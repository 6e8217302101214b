"""MI355X-native RealNVP coupling-layer engine (host side).

Layout:
  _lib.py        ctypes binding of include/realnvp_hip.h (librealnvp_hip.so)
  net.py         the s/t ResNet as a conv program (forward + derived backward)
  engine.py      per-coupling executor (workspaces, kernel sequencing)
  functions.py   autograd Functions for the drop-in modules
  trainer.py     fused NLL training step (flat parameter arena, fused Adam,
                 HIP-graph capture, RCCL data parallelism)
  optim.py       FusedAdam: torch.optim.Adam drop-in for the reference loop
"""
from ._lib import LIB_PATH, lib  # noqa: F401
from .optim import FusedAdam  # noqa: F401
