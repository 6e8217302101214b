"""Drop-in for the reference ``flow_realnvp.RealNVP`` (flow_realnvp.py:35-370).

Same constructor, attributes (s{k}_ckbd / s{k}_chan / order_matrix_{k} /
prior / channels / image_size), methods (f, g, log_prob, sample, forward,
squeeze, undo_squeeze, order_matrix, factor_out, restore) and state_dict
keys.  The scale count is generalised by the optional ``n_scales`` argument
(default 5 = the reference's hard-coded stack, flow_realnvp.py:46-95).

Compute runs on the MI355X through realnvp_hip (HIP kernels behind
include/realnvp_hip.h): couplings, permutations, the N(0,1) prior term and
the weight_scale regulariser.  ``log_prob``/``forward`` accumulate the
log-determinant per sample (the only quantity the reference consumes,
flow_realnvp.py:338); ``f`` still returns the elementwise log_diag_J.
"""
import numpy as np
import torch
import torch.nn as nn

from modules_realnvp import ChannelwiseAffineCoupling, CheckerboardAffineCoupling
from realnvp_hip import functions as Fn

__all__ = ["RealNVP"]


class RealNVP(nn.Module):
    def __init__(self, channels, image_size, prior, hps, n_scales=5):
        super().__init__()
        if n_scales < 2:
            raise ValueError("n_scales must be >= 2")
        if image_size % (1 << (n_scales - 1)):
            raise ValueError("image_size must be divisible by 2**(n_scales-1)")
        self.prior = prior
        self.channels = channels
        self.image_size = image_size
        self.n_scales = n_scales
        chan, size, dim = channels, image_size, hps.base_dim
        # construction order (and therefore RNG draws) follows flow_realnvp.py:51-95
        for s in range(1, n_scales):
            setattr(self, "s%d_ckbd" % s, self.checkerboard_combo(chan, dim, size, hps))
            setattr(self, "s%d_chan" % s, self.channelwise_combo(chan * 4, dim * 2, hps))
            setattr(self, "order_matrix_%d" % s, self.order_matrix(chan))
            chan, size, dim = chan * 2, size // 2, dim * 2
        setattr(self, "s%d_ckbd" % n_scales, self.checkerboard_combo(chan, dim, size, hps, final=True))

    # ---------------------------------------------------------------- builders
    def checkerboard_combo(self, in_out_dim, mid_dim, size, hps, final=False):
        """flow_realnvp.py:98-109: masks 1,0,1(,0)."""
        cfgs = [1., 0., 1., 0.] if final else [1., 0., 1.]
        return nn.ModuleList([CheckerboardAffineCoupling(in_out_dim, mid_dim, size, c, hps) for c in cfgs])

    def channelwise_combo(self, in_out_dim, mid_dim, hps):
        """flow_realnvp.py:112-116: masks 0,1,0."""
        return nn.ModuleList([ChannelwiseAffineCoupling(in_out_dim, mid_dim, c, hps) for c in (0., 1., 0.)])

    def couplings(self):
        for s in range(1, self.n_scales + 1):
            for m in getattr(self, "s%d_ckbd" % s):
                yield m
            if s < self.n_scales:
                for m in getattr(self, "s%d_chan" % s):
                    yield m

    def set_precision(self, dtype):
        """'fp32' (parity mode, default) or 'bf16' (s/t network in bf16 with
        fp32 accumulation; couplings, log-det and BN statistics stay fp32)."""
        if dtype not in ("fp32", "bf16"):
            raise ValueError(dtype)
        for m in self.couplings():
            m.compute_dtype = dtype
        return self

    # ------------------------------------------------------------ permutations
    def squeeze(self, x):
        """flow_realnvp.py:121-126 (HIP gather kernel)."""
        return Fn.squeeze(x)

    def undo_squeeze(self, x):
        """flow_realnvp.py:130-135."""
        return Fn.undo_squeeze(x)

    def order_matrix(self, channel):
        """flow_realnvp.py:139-165: the 0/1 [4C, C, 2, 2] kernel describing the
        factor-out ordering (kept for API parity; factor_out/restore implement
        the permutation it encodes directly)."""
        weights = np.zeros((channel * 4, channel, 2, 2), dtype=np.float32)
        picks = [(0, 0), (1, 1), (0, 1), (1, 0)]   # on = (0,0),(1,1); off = (0,1),(1,0)
        for r, (i, j) in enumerate(picks):
            for c in range(channel):
                weights[r * channel + c, c, i, j] = 1.0
        return torch.tensor(weights)

    def _check_om(self, x, order_matrix):
        """The reference convolves with whatever 0/1 kernel it is handed
        (flow_realnvp.py:167-193); the HIP path implements the permutation of
        the canonical order_matrix(C) -- the only one the reference itself
        passes (order_matrix_k, flow_realnvp.py:60-93).  Any other matrix is
        refused rather than silently giving a different result."""
        if order_matrix is None:
            return
        C = x.shape[1]
        if tuple(order_matrix.shape) != (4 * C, C, 2, 2):
            raise ValueError("order_matrix shape does not match the input channels")
        canon = self.order_matrix(C).to(device=order_matrix.device, dtype=order_matrix.dtype)
        if not torch.equal(order_matrix, canon):
            raise ValueError("factor_out / restore implement the canonical order_matrix(%d) only "
                             "(flow_realnvp.py:139-165); got another 0/1 kernel" % C)

    def factor_out(self, x, order_matrix=None):
        """flow_realnvp.py:167-180 -> (on, off), each [B, 2C, H/2, W/2]."""
        self._check_om(x, order_matrix)
        return Fn.factor_out(x)

    def restore(self, on, off, order_matrix=None):
        """flow_realnvp.py:182-193."""
        if order_matrix is not None:
            self._check_om(on.new_empty(on.shape[0], on.shape[1] // 2, 1, 1), order_matrix)
        return Fn.restore(on, off)

    # ------------------------------------------------------------------- flow
    def _scale_mods(self, s):
        return getattr(self, "s%d_ckbd" % s), (getattr(self, "s%d_chan" % s) if s < self.n_scales else None)

    def f(self, x):
        """flow_realnvp.py:252-327: x -> (z, elementwise log_diag_J)."""
        z, ldj = x, torch.zeros_like(x)
        offs = []
        for s in range(1, self.n_scales):
            ckbd, chan = self._scale_mods(s)
            for m in ckbd:
                z, inc = m(z)
                ldj = ldj + inc
            z, ldj = Fn.squeeze(z), Fn.squeeze(ldj)
            for m in chan:
                z, inc = m(z)
                ldj = ldj + inc
            z, ldj = Fn.undo_squeeze(z), Fn.undo_squeeze(ldj)
            z, z_off = Fn.factor_out(z)
            ldj, l_off = Fn.factor_out(ldj)
            offs.append((z_off, l_off))
        for m in self._scale_mods(self.n_scales)[0]:
            z, inc = m(z)
            ldj = ldj + inc
        for z_off, l_off in reversed(offs):
            z = Fn.restore(z, z_off)
            ldj = Fn.restore(ldj, l_off)
        return z, ldj

    def _f_sample(self, x):
        """Hot path of log_prob: z plus the per-sample log-det sum [B]."""
        z = x
        parts = []
        offs = []
        for s in range(1, self.n_scales):
            ckbd, chan = self._scale_mods(s)
            for m in ckbd:
                z, l = Fn.coupling_apply(m, z, full_ldj=False)
                parts.append(l)
            z = Fn.squeeze(z)
            for m in chan:
                z, l = Fn.coupling_apply(m, z, full_ldj=False)
                parts.append(l)
            z = Fn.undo_squeeze(z)
            z, z_off = Fn.factor_out(z)
            offs.append(z_off)
        for m in self._scale_mods(self.n_scales)[0]:
            z, l = Fn.coupling_apply(m, z, full_ldj=False)
            parts.append(l)
        for z_off in reversed(offs):
            z = Fn.restore(z, z_off)
        return z, torch.stack(parts, 0).sum(0)

    def g(self, z):
        """flow_realnvp.py:196-249: z -> x (exact inverse)."""
        x = z
        offs = []
        for s in range(1, self.n_scales):
            x, off = Fn.factor_out(x)
            offs.append(off)
        for m in reversed(self._scale_mods(self.n_scales)[0]):
            x, _ = m(x, reverse=True)
        for s in reversed(range(1, self.n_scales)):
            ckbd, chan = self._scale_mods(s)
            x = Fn.restore(x, offs[s - 1])
            x = Fn.squeeze(x)
            for m in reversed(chan):
                x, _ = m(x, reverse=True)
            x = Fn.undo_squeeze(x)
            for m in reversed(ckbd):
                x, _ = m(x, reverse=True)
        return x

    def log_prob(self, x):
        """flow_realnvp.py:329-340."""
        z, ldj = self._f_sample(x)
        if Fn.is_std_normal(self.prior):
            return Fn.std_normal_logprob(z, ldj)
        return torch.sum(self.prior.log_prob(z), dim=(1, 2, 3)) + ldj

    def sample(self, size):
        """flow_realnvp.py:342-352."""
        C = self.channels
        H = W = self.image_size
        z = self.prior.sample((size, C, H, W))
        if not z.is_cuda:
            z = z.to(self._device())
        return self.g(z)

    def _device(self):
        return next(self.parameters()).device

    def weight_scale_params(self):
        # the (module dict, key) slots of every weight_g / scale, walked once
        # (a named_parameters() walk per forward cost ~8 ms of host time)
        slots = self.__dict__.get("_ws_slots")
        if slots is None:
            slots = [(m._parameters, k) for _, m in self.named_modules() for k, v in m._parameters.items()
                     if v is not None and k in ("weight_g", "scale")]
            object.__setattr__(self, "_ws_slots", slots)
        return [p for p in (d[k] for d, k in slots) if p is not None and p.requires_grad]

    def forward(self, x):
        """flow_realnvp.py:354-370: (log_prob(x), sum of squares of trainable
        weight_g / scale parameters)."""
        ps = self.weight_scale_params()
        weight_scale = Fn.sum_of_squares(ps) if ps else None
        return self.log_prob(x), weight_scale
