"""Drop-in for the reference ``modules_realnvp`` (affine coupling layers).

Same class names, constructor signatures, module tree, parameter
registration order and ``state_dict`` keys as modules_realnvp.py:36-370, so
reference checkpoints load unchanged and ``torch.manual_seed(s)`` followed by
construction draws the same initial weights.  A coupling's forward / inverse /
backward do NOT run through its children: they are executed, fused, by
``realnvp_hip.engine.CouplingEngine`` on the MI355X (HIP kernels behind
include/realnvp_hip.h).  The s/t-network submodules are still callable on
their own as in the reference: WeightNormConv2d runs the same HIP kernels one
at a time (``realnvp_hip.standalone``), ResidualBlock / ResidualModule
compose their children like modules_realnvp.py:107-114, 175-194.  Inputs
must live on a HIP device; there is no CPU path.
"""
import math

import numpy as np
import torch
import torch.nn as nn

from realnvp_hip.functions import coupling_apply, coupling_reverse
from realnvp_hip.standalone import wn_conv2d

__all__ = ["WeightNormConv2d", "ResidualBlock", "ResidualModule", "AbstractCoupling",
           "CheckerboardAffineCoupling", "ChannelwiseAffineCoupling", "AffineCoupling"]


class _ConvParams(nn.Module):
    """Parameter holder with the key layout of nn.utils.weight_norm(nn.Conv2d)
    (bias, weight_g, weight_v) or of a plain nn.Conv2d (weight, bias).
    Initialisation follows nn.Conv2d.reset_parameters (same RNG draws) and
    weight_norm's g = ||v|| (modules_realnvp.py:53-62)."""

    def __init__(self, in_dim, out_dim, kernel_size, bias, weight_norm, scale, padding=None):
        super().__init__()
        k = kernel_size if isinstance(kernel_size, int) else kernel_size[0]
        self.padding = k // 2 if padding is None else (padding if isinstance(padding, int) else padding[0])
        w = torch.empty(out_dim, in_dim, k, k)
        nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        b = None
        if bias:
            bound = 1.0 / math.sqrt(in_dim * k * k)
            b = torch.empty(out_dim)
            nn.init.uniform_(b, -bound, bound)
        self.kernel_size = (k, k)
        self.in_channels, self.out_channels = in_dim, out_dim
        if weight_norm:
            if b is not None:
                self.bias = nn.Parameter(b)
            else:
                self.register_parameter("bias", None)
            g = w.pow(2).sum(dim=(1, 2, 3), keepdim=True).sqrt()
            if not scale:
                self.weight_g = nn.Parameter(torch.ones_like(g), requires_grad=False)   # frozen, 57-59
            else:
                self.weight_g = nn.Parameter(g)
            self.weight_v = nn.Parameter(w)
        else:
            self.weight = nn.Parameter(w)
            if b is not None:
                self.bias = nn.Parameter(b)
            else:
                self.register_parameter("bias", None)

    def forward(self, x):
        """The weight-normalised nn.Conv2d on its own (HIP kernels, fp32)."""
        return wn_conv2d(self, x)


class WeightNormConv2d(nn.Module):
    """modules_realnvp.py:36-71 (parameter container; executed by the engine)."""

    def __init__(self, in_dim, out_dim, kernel_size, stride=1, padding=0, bias=True, weight_norm=True, scale=False):
        super().__init__()
        if stride != 1:
            raise NotImplementedError("only stride 1 occurs on the RealNVP path")
        self.conv = _ConvParams(in_dim, out_dim, kernel_size, bias, weight_norm, scale, padding)
        self.padding, self.scale = padding, scale

    def forward(self, x):
        """modules_realnvp.py:64-71 (standalone call: realnvp_hip.standalone)."""
        return self.conv(x)


class ResidualBlock(nn.Module):
    """modules_realnvp.py:73-114."""

    def __init__(self, dim, bottleneck, weight_norm):
        super().__init__()
        self.in_block = nn.Sequential(nn.BatchNorm2d(dim), nn.ReLU())
        if bottleneck:
            self.res_block = nn.Sequential(
                WeightNormConv2d(dim, dim, (1, 1), stride=1, padding=0, bias=False, weight_norm=weight_norm, scale=False),
                nn.BatchNorm2d(dim), nn.ReLU(),
                WeightNormConv2d(dim, dim, (3, 3), stride=1, padding=1, bias=False, weight_norm=weight_norm, scale=False),
                nn.BatchNorm2d(dim), nn.ReLU(),
                WeightNormConv2d(dim, dim, (1, 1), stride=1, padding=0, bias=True, weight_norm=weight_norm, scale=True))
        else:
            self.res_block = nn.Sequential(
                WeightNormConv2d(dim, dim, (3, 3), stride=1, padding=1, bias=False, weight_norm=weight_norm, scale=False),
                nn.BatchNorm2d(dim), nn.ReLU(),
                WeightNormConv2d(dim, dim, (3, 3), stride=1, padding=1, bias=True, weight_norm=weight_norm, scale=True))

    def forward(self, x):
        """modules_realnvp.py:107-114 (standalone call; inside a coupling the
        engine runs it fused)."""
        return x + self.res_block(self.in_block(x))


class ResidualModule(nn.Module):
    """modules_realnvp.py:116-194."""

    def __init__(self, in_dim, dim, out_dim, res_blocks, bottleneck, skip, weight_norm):
        super().__init__()
        self.res_blocks = res_blocks
        self.skip = skip
        if res_blocks > 0:
            self.in_block = WeightNormConv2d(in_dim, dim, (3, 3), stride=1, padding=1, bias=True,
                                             weight_norm=weight_norm, scale=False)
            self.core_block = nn.ModuleList([ResidualBlock(dim, bottleneck, weight_norm) for _ in range(res_blocks)])
            self.out_block = nn.Sequential(
                nn.BatchNorm2d(dim), nn.ReLU(),
                WeightNormConv2d(dim, out_dim, (1, 1), stride=1, padding=0, bias=True, weight_norm=weight_norm,
                                 scale=True))
            if skip:
                self.in_skip = WeightNormConv2d(dim, dim, (1, 1), stride=1, padding=0, bias=True,
                                                weight_norm=weight_norm, scale=True)
                self.core_skips = nn.ModuleList([
                    WeightNormConv2d(dim, dim, (1, 1), stride=1, padding=0, bias=True, weight_norm=weight_norm,
                                     scale=True) for _ in range(res_blocks)])
        else:
            if bottleneck:
                self.block = nn.Sequential(
                    WeightNormConv2d(in_dim, dim, (1, 1), stride=1, padding=0, bias=False, weight_norm=weight_norm,
                                     scale=False),
                    nn.BatchNorm2d(dim), nn.ReLU(),
                    WeightNormConv2d(dim, dim, (3, 3), stride=1, padding=1, bias=False, weight_norm=weight_norm,
                                     scale=False),
                    nn.BatchNorm2d(dim), nn.ReLU(),
                    WeightNormConv2d(dim, out_dim, (1, 1), stride=1, padding=0, bias=True, weight_norm=weight_norm,
                                     scale=True))
            else:
                self.block = nn.Sequential(
                    WeightNormConv2d(in_dim, dim, (3, 3), stride=1, padding=1, bias=False, weight_norm=weight_norm,
                                     scale=False),
                    nn.BatchNorm2d(dim), nn.ReLU(),
                    WeightNormConv2d(dim, out_dim, (3, 3), stride=1, padding=1, bias=True, weight_norm=weight_norm,
                                     scale=True))

    def forward(self, x):
        """modules_realnvp.py:175-194 (standalone call; inside a coupling the
        engine runs it fused)."""
        if self.res_blocks > 0:
            x = self.in_block(x)
            out = self.in_skip(x) if self.skip else None
            for i in range(len(self.core_block)):
                x = self.core_block[i](x)
                if self.skip:
                    out = out + self.core_skips[i](x)
            if self.skip:
                x = out
            return self.out_block(x)
        return self.block(x)


class AbstractCoupling(nn.Module):
    """modules_realnvp.py:196-237."""

    KIND = None

    def __init__(self, mask_config, hps):
        super().__init__()
        self.mask_config = mask_config
        self.res_blocks = hps.res_blocks
        self.bottleneck = hps.bottleneck
        self.skip = hps.skip
        self.weight_norm = hps.weight_norm
        self.coupling_bn = hps.coupling_bn
        self.hps = hps
        self.compute_dtype = "fp32"
        object.__setattr__(self, "_engine", None)

    def build_mask(self, size, config=1.):
        """Binary checkerboard mask (modules_realnvp.py:211-226): mask[i,j] =
        (config + i + j) mod 2, as a [1,1,S,S] float32 tensor."""
        i = np.arange(size)
        mask = np.mod(config + i.reshape(-1, 1) + i, 2).reshape(-1, 1, size, size)
        return torch.tensor(mask.astype("float32"))

    def batch_stat(self, x):
        """modules_realnvp.py:228-237 (kept for API parity; the engine fuses it)."""
        mean = torch.mean(x, dim=(0, 2, 3), keepdim=True)
        var = torch.mean((x - mean) ** 2, dim=(0, 2, 3), keepdim=True)
        return mean, var

    def engine(self):
        if self._engine is None:
            from realnvp_hip.engine import CouplingEngine
            object.__setattr__(self, "_engine", CouplingEngine(self))
        return self._engine

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        object.__setattr__(self, "_engine", None)   # storage moved: rebuild descriptor tables
        return out

    def forward(self, x, reverse=False):
        """Returns (y, log_diag_J) like the reference (modules_realnvp.py:264-302, 324-370)."""
        if reverse:
            return coupling_reverse(self, x)
        return coupling_apply(self, x, full_ldj=True)


class CheckerboardAffineCoupling(AbstractCoupling):
    """modules_realnvp.py:239-302."""

    KIND = "ckbd"

    def __init__(self, in_out_dim, mid_dim, size, mask_config, hps):
        super().__init__(mask_config, hps)
        self.in_out_dim, self.mid_dim, self.size = in_out_dim, mid_dim, size
        self.mask = self.build_mask(size, config=mask_config)   # plain attribute, as in the reference
        self.scale = nn.Parameter(torch.zeros(1), requires_grad=True)
        self.scale_shift = nn.Parameter(torch.zeros(1), requires_grad=True)
        self.in_bn = nn.BatchNorm2d(in_out_dim)
        self.block = nn.Sequential(
            nn.ReLU(),
            ResidualModule(2 * in_out_dim + 1, mid_dim, 2 * in_out_dim, self.res_blocks, self.bottleneck, self.skip,
                           self.weight_norm))
        self.out_bn = nn.BatchNorm2d(in_out_dim, affine=False)


class ChannelwiseAffineCoupling(AbstractCoupling):
    """modules_realnvp.py:304-370."""

    KIND = "chan"

    def __init__(self, in_out_dim, mid_dim, mask_config, hps):
        super().__init__(mask_config, hps)
        self.in_out_dim, self.mid_dim = in_out_dim, mid_dim
        self.scale = nn.Parameter(torch.zeros(1), requires_grad=True)
        self.scale_shift = nn.Parameter(torch.zeros(1), requires_grad=True)
        self.in_bn = nn.BatchNorm2d(in_out_dim // 2)
        self.block = nn.Sequential(
            nn.ReLU(),
            ResidualModule(in_out_dim, mid_dim, in_out_dim, self.res_blocks, self.bottleneck, self.skip,
                           self.weight_norm))
        self.out_bn = nn.BatchNorm2d(in_out_dim // 2, affine=False)


# BASELINE.json's north star names "modules_realnvp.AffineCoupling", which the
# reference does not define; alias the checkerboard coupling (the first layer
# type of every scale).
AffineCoupling = CheckerboardAffineCoupling
