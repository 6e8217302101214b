"""Drop-in for the reference ``utils`` module (utils.py:33-113): the
``Hyperparameters`` holder, ``logit_transform`` and ``weights_init`` (the
DCGAN initialiser train.py:37-41 imports next to them).

logit_transform runs as one fused HIP kernel (dequantisation noise, affine
squash to [0.05, 0.95], logit, per-sample log-det).  Differences from the
reference, by design:
  * the noise is drawn on the device (counter-based Philox keyed by a seed
    taken from torch's default CPU generator, so torch.manual_seed still
    makes it reproducible) instead of torch's CPU Uniform sampler; pass
    ``noise=`` to supply it explicitly (the parity tests do);
  * a CPU input is moved to the current HIP device and the results are
    returned there (the reference moves them right after, train.py:188-189).
"""
import torch

from realnvp_hip import _lib
from realnvp_hip.engine import stream_ptr

__all__ = ["Hyperparameters", "logit_transform", "weights_init"]


class Hyperparameters():
    """utils.py:78-93."""

    def __init__(self, base_dim, res_blocks, bottleneck, skip, weight_norm, coupling_bn):
        self.base_dim = base_dim
        self.res_blocks = res_blocks
        self.bottleneck = bottleneck
        self.skip = skip
        self.weight_norm = weight_norm
        self.coupling_bn = coupling_bn


def _to_device(x):
    if x.is_cuda:
        return x
    if not torch.cuda.is_available():
        raise RuntimeError("logit_transform: no HIP device available; the MI355X engine has no CPU path")
    return x.to(torch.device("cuda", torch.cuda.current_device()))


def logit_transform(x, constraint=0.9, reverse=False, noise=None, seed=None):
    """utils.py:33-72.  Forward returns (logit_x, per-sample log-det [B]);
    reverse returns (x, 0) like the reference."""
    x = _to_device(x).contiguous().float()
    L = _lib.lib()
    if reverse:
        y = torch.empty_like(x)
        L.logit_inv(x.data_ptr(), y.data_ptr(), float(constraint), x.numel(), stream_ptr())
        return y, 0
    B = x.shape[0]
    n = x.numel() // max(B, 1)
    y = torch.empty_like(x)
    logdet = torch.empty(B, device=x.device, dtype=torch.float32)
    nptr = None
    if noise is not None:
        noise = noise.to(x.device).contiguous().float()
        if noise.shape != x.shape:
            raise ValueError("noise must have the shape of x")
        nptr = noise.data_ptr()
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    L.logit_fwd(x.data_ptr(), nptr, seed, 0, None, float(constraint), y.data_ptr(), logdet.data_ptr(), B, n,
                stream_ptr())
    return y, logdet


def weights_init(m):
    """utils.py:98-113 (DCGAN initialiser, kept so train.py's import line
    works unchanged): N(0, 0.02) conv weights, N(1, 0.02) / 0 BatchNorm
    affine parameters.  Plain torch init on the module's own device (the
    reference's trailing .cuda() calls return copies that are discarded)."""
    import torch.nn as nn
    classname = m.__class__.__name__
    if classname.find("Conv") != -1:
        nn.init.normal_(m.weight.data, 0.0, 0.02)
    elif classname.find("BatchNorm") != -1:
        nn.init.normal_(m.weight.data, 1.0, 0.02)
        nn.init.constant_(m.bias.data, 0)
