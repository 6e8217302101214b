"""CPU oracle for the RealNVP coupling-layer training path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline -- never as the thing measured or shipped.
The product path (``dl-normalizing-flows_amd``) never imports it.

This is a clean-room, functional fp32 restatement of the reference algorithm
(alisher-turubayev/dl-normalizing-flows) written against torch *CPU* ops.  It
operates on a flat ``state`` dict whose keys are exactly the reference
``state_dict`` keys, so the same dict can be loaded into the reference, into
this oracle and into the MI355X engine.  Every function cites the reference
file:line it restates.

Pinning: checked against golden vectors produced by importing the reference
itself in the build container (``tools/make_goldens.py`` -> ``tests/golden``),
see ``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn.functional as F

BN_EPS = 1e-5          # torch BatchNorm2d default (modules_realnvp.py:84,257,262)
BN_MOMENTUM = 0.1      # torch BatchNorm2d default
LDJ_EPS = 1e-5         # modules_realnvp.py:289,301

State = Dict[str, torch.Tensor]


# ---------------------------------------------------------------------------
# index maps (bit-exact)
# ---------------------------------------------------------------------------
def checkerboard_mask(size: int, config: float) -> torch.Tensor:
    """modules_realnvp.py:211-226: mask[i,j] = (config + i + j) mod 2, [1,1,S,S] f32."""
    i = np.arange(size)
    m = np.mod(int(config) + i[:, None] + i[None, :], 2).astype(np.float32)
    return torch.from_numpy(m).reshape(1, 1, size, size)


def squeeze(x: torch.Tensor) -> torch.Tensor:
    """flow_realnvp.py:121-126: [B,C,H,W] -> [B,4C,H/2,W/2], out ch 4c+2i+j = x[c,2h+i,2w+j]."""
    B, C, H, W = x.shape
    return x.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 3, 5, 2, 4).reshape(B, 4 * C, H // 2, W // 2)


def undo_squeeze(x: torch.Tensor) -> torch.Tensor:
    """flow_realnvp.py:130-135 (inverse of squeeze)."""
    B, C, H, W = x.shape
    return x.reshape(B, C // 4, 2, 2, H, W).permute(0, 1, 4, 2, 5, 3).reshape(B, C // 4, 2 * H, 2 * W)


def factor_out(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """flow_realnvp.py:139-180.  The reference does a stride-2 conv with the 0/1
    ``order_matrix`` kernel; that kernel is the permutation
    on  = cat(x[..,0::2,0::2], x[..,1::2,1::2]),  off = cat(x[..,0::2,1::2], x[..,1::2,0::2])."""
    on = torch.cat((x[:, :, 0::2, 0::2], x[:, :, 1::2, 1::2]), dim=1)
    off = torch.cat((x[:, :, 0::2, 1::2], x[:, :, 1::2, 0::2]), dim=1)
    return on, off


def restore(on: torch.Tensor, off: torch.Tensor) -> torch.Tensor:
    """flow_realnvp.py:182-193 (conv_transpose2d with the order matrix == inverse permutation)."""
    B, C2, h, w = on.shape
    C = C2 // 2
    x = on.new_empty(B, C, 2 * h, 2 * w)
    x[:, :, 0::2, 0::2] = on[:, :C]
    x[:, :, 1::2, 1::2] = on[:, C:]
    x[:, :, 0::2, 1::2] = off[:, :C]
    x[:, :, 1::2, 0::2] = off[:, C:]
    return x


# ---------------------------------------------------------------------------
# layers
# ---------------------------------------------------------------------------
def wn_weight(S: State, p: str) -> torch.Tensor:
    """torch.nn.utils.weight_norm(dim=0) as used at modules_realnvp.py:53-59:
    w = g * v / ||v||, norm over every dim but 0.  Plain conv when no weight_v."""
    if p + "weight_v" not in S:
        return S[p + "weight"]
    v, g = S[p + "weight_v"], S[p + "weight_g"]
    n = v.pow(2).sum(dim=(1, 2, 3), keepdim=True).sqrt()
    return v * (g / n)


def conv(S: State, p: str, x: torch.Tensor) -> torch.Tensor:
    """WeightNormConv2d.forward (modules_realnvp.py:64-71); padding = k//2, stride 1."""
    w = wn_weight(S, p + "conv.")
    b = S.get(p + "conv.bias")
    return F.conv2d(x, w, b, stride=1, padding=w.shape[-1] // 2)


def batch_norm(S: State, p: str, x: torch.Tensor, training: bool, affine: bool = True) -> torch.Tensor:
    """nn.BatchNorm2d semantics (torch defaults, modules_realnvp.py:84,90,93,257,262).
    Train: biased batch var to normalise, running stats momentum 0.1 with the
    unbiased var, num_batches_tracked += 1.  Eval: running stats."""
    rm, rv = S[p + "running_mean"], S[p + "running_var"]
    if training:
        n = x.numel() // x.shape[1]
        mean = x.mean(dim=(0, 2, 3))
        var = (x - mean.view(1, -1, 1, 1)).pow(2).mean(dim=(0, 2, 3))
        with torch.no_grad():
            rm.mul_(1 - BN_MOMENTUM).add_(BN_MOMENTUM * mean.detach())
            rv.mul_(1 - BN_MOMENTUM).add_(BN_MOMENTUM * var.detach() * (n / max(n - 1, 1)))
            S[p + "num_batches_tracked"].add_(1)
    else:
        mean, var = rm, rv
    y = (x - mean.view(1, -1, 1, 1)) / torch.sqrt(var.view(1, -1, 1, 1) + BN_EPS)
    if affine:
        y = y * S[p + "weight"].view(1, -1, 1, 1) + S[p + "bias"].view(1, -1, 1, 1)
    return y


def residual_block(S: State, p: str, x, training, bottleneck):
    """ResidualBlock.forward (modules_realnvp.py:73-114): x + res_block(ReLU(BN(x)))."""
    h = F.relu(batch_norm(S, p + "in_block.0.", x, training))
    r = p + "res_block."
    if bottleneck:
        h = conv(S, r + "0.", h)
        h = F.relu(batch_norm(S, r + "1.", h, training))
        h = conv(S, r + "3.", h)
        h = F.relu(batch_norm(S, r + "4.", h, training))
        h = conv(S, r + "6.", h)
    else:
        h = conv(S, r + "0.", h)
        h = F.relu(batch_norm(S, r + "1.", h, training))
        h = conv(S, r + "3.", h)
    return x + h


def residual_module(S: State, p: str, x, training, res_blocks, bottleneck, skip):
    """ResidualModule.forward (modules_realnvp.py:116-194)."""
    if res_blocks > 0:
        x = conv(S, p + "in_block.", x)
        out = conv(S, p + "in_skip.", x) if skip else None
        for i in range(res_blocks):
            x = residual_block(S, p + "core_block.%d." % i, x, training, bottleneck)
            if skip:
                out = out + conv(S, p + "core_skips.%d." % i, x)
        if skip:
            x = out
        h = F.relu(batch_norm(S, p + "out_block.0.", x, training))
        return conv(S, p + "out_block.2.", h)
    b = p + "block."
    if bottleneck:
        h = conv(S, b + "0.", x)
        h = F.relu(batch_norm(S, b + "1.", h, training))
        h = conv(S, b + "3.", h)
        h = F.relu(batch_norm(S, b + "4.", h, training))
        return conv(S, b + "6.", h)
    h = conv(S, b + "0.", x)
    h = F.relu(batch_norm(S, b + "1.", h, training))
    return conv(S, b + "3.", h)


class HP:
    """utils.Hyperparameters (utils.py:78-93)."""

    def __init__(self, base_dim, res_blocks, bottleneck=True, skip=True, weight_norm=True, coupling_bn=True):
        self.base_dim, self.res_blocks = base_dim, res_blocks
        self.bottleneck, self.skip = bottleneck, skip
        self.weight_norm, self.coupling_bn = weight_norm, coupling_bn


def _out_bn_var(S, p, y, training):
    if training:
        mean = y.mean(dim=(0, 2, 3), keepdim=True)
        return (y - mean).pow(2).mean(dim=(0, 2, 3), keepdim=True)   # batch_stat, modules_realnvp.py:228-237
    return S[p + "out_bn.running_var"].view(1, -1, 1, 1)


def checkerboard_coupling(S: State, p: str, x, mask_config, hp: HP, training, reverse=False):
    """CheckerboardAffineCoupling.forward (modules_realnvp.py:264-302).  Returns (y, log_diag_J)."""
    B, C, H, W = x.shape
    m = checkerboard_mask(H, mask_config).expand(B, 1, H, W)
    xa = batch_norm(S, p + "in_bn.", x * m, training)
    h = F.relu(torch.cat((xa, -xa, m), dim=1))          # block = Seq(ReLU, ResidualModule), 258-261
    st = residual_module(S, p + "block.1.", h, training, hp.res_blocks, hp.bottleneck, hp.skip)
    shift, lr = st[:, :C], st[:, C:]
    lr = S[p + "scale"] * torch.tanh(lr) + S[p + "scale_shift"]
    inv = 1.0 - m
    shift = shift * inv
    lr = lr * inv
    ldj = lr
    if reverse:
        if hp.coupling_bn:
            rm = S[p + "out_bn.running_mean"].view(1, -1, 1, 1)
            rv = S[p + "out_bn.running_var"].view(1, -1, 1, 1)
            x = x * torch.exp(0.5 * torch.log(rv + LDJ_EPS) * inv) + rm * inv
        return (x - shift) * torch.exp(-lr), ldj
    y = x * torch.exp(lr) + shift
    if hp.coupling_bn:
        var = _out_bn_var(S, p, y, training)
        y = batch_norm(S, p + "out_bn.", y, training, affine=False) * inv + y * m
        ldj = ldj - 0.5 * torch.log(var + LDJ_EPS) * inv
    return y, ldj


def channelwise_coupling(S: State, p: str, x, mask_config, hp: HP, training, reverse=False):
    """ChannelwiseAffineCoupling.forward (modules_realnvp.py:324-370)."""
    C = x.shape[1]
    a, b = x[:, :C // 2], x[:, C // 2:]
    on, off = (a, b) if mask_config else (b, a)
    oa = batch_norm(S, p + "in_bn.", off, training)
    h = F.relu(torch.cat((oa, -oa), dim=1))
    st = residual_module(S, p + "block.1.", h, training, hp.res_blocks, hp.bottleneck, hp.skip)
    shift, lr = st[:, :C // 2], st[:, C // 2:]
    lr = S[p + "scale"] * torch.tanh(lr) + S[p + "scale_shift"]
    ldj = lr
    if reverse:
        if hp.coupling_bn:
            rm = S[p + "out_bn.running_mean"].view(1, -1, 1, 1)
            rv = S[p + "out_bn.running_var"].view(1, -1, 1, 1)
            on = on * torch.exp(0.5 * torch.log(rv + LDJ_EPS)) + rm
        on = (on - shift) * torch.exp(-lr)
    else:
        on = on * torch.exp(lr) + shift
        if hp.coupling_bn:
            var = _out_bn_var(S, p, on, training)
            on = batch_norm(S, p + "out_bn.", on, training, affine=False)
            ldj = ldj - 0.5 * torch.log(var + LDJ_EPS)
    z = torch.zeros_like(ldj)
    if mask_config:
        return torch.cat((on, off), dim=1), torch.cat((ldj, z), dim=1)
    return torch.cat((off, on), dim=1), torch.cat((z, ldj), dim=1)


# ---------------------------------------------------------------------------
# multi-scale flow
# ---------------------------------------------------------------------------
CKBD_CFGS = [1.0, 0.0, 1.0]        # flow_realnvp.py:106-109
CKBD_FINAL_CFGS = [1.0, 0.0, 1.0, 0.0]   # flow_realnvp.py:99-104
CHAN_CFGS = [0.0, 1.0, 0.0]        # flow_realnvp.py:112-116


def default_scales(image_size: int) -> int:
    """The reference hard-codes 5 scales (flow_realnvp.py:46-95)."""
    return 5


class FlowSpec:
    """Static description of the RealNVP stack (flow_realnvp.py:36-95), with the
    scale count generalised (``n_scales`` = 5 reproduces the reference)."""

    def __init__(self, channels, image_size, hp: HP, n_scales: int = 5):
        self.channels, self.image_size, self.hp, self.n_scales = channels, image_size, hp, n_scales
        self.scales = []   # (chan, size, dim) for scale s = 1..n_scales
        c, s, d = channels, image_size, hp.base_dim
        for i in range(n_scales):
            self.scales.append((c, s, d))
            c, s, d = c * 2, s // 2, d * 2


def coupling_forward(S, spec: FlowSpec, kind, scale_idx, j, x, training, reverse=False):
    c, s, d = spec.scales[scale_idx]
    last = scale_idx == spec.n_scales - 1
    p = "s%d_%s.%d." % (scale_idx + 1, kind, j)
    if kind == "ckbd":
        cfg = (CKBD_FINAL_CFGS if last else CKBD_CFGS)[j]
        return checkerboard_coupling(S, p, x, cfg, spec.hp, training, reverse)
    cfg = CHAN_CFGS[j]
    return channelwise_coupling(S, p, x, cfg, spec.hp, training, reverse)


def flow_f(S, spec: FlowSpec, x, training):
    """RealNVP.f (flow_realnvp.py:252-327): x -> (z, elementwise log_diag_J)."""
    z, ldj = x, torch.zeros_like(x)
    offs = []
    for si in range(spec.n_scales - 1):
        for j in range(3):
            z, inc = coupling_forward(S, spec, "ckbd", si, j, z, training)
            ldj = ldj + inc
        z, ldj = squeeze(z), squeeze(ldj)
        for j in range(3):
            z, inc = coupling_forward(S, spec, "chan", si, j, z, training)
            ldj = ldj + inc
        z, ldj = undo_squeeze(z), undo_squeeze(ldj)
        z, z_off = factor_out(z)
        ldj, l_off = factor_out(ldj)
        offs.append((z_off, l_off))
    for j in range(4):
        z, inc = coupling_forward(S, spec, "ckbd", spec.n_scales - 1, j, z, training)
        ldj = ldj + inc
    for z_off, l_off in reversed(offs):
        z = restore(z, z_off)
        ldj = restore(ldj, l_off)
    return z, ldj


def flow_g(S, spec: FlowSpec, z, training):
    """RealNVP.g (flow_realnvp.py:196-249): z -> x."""
    offs = []
    x = z
    for si in range(spec.n_scales - 1):
        x, off = factor_out(x)
        offs.append(off)
    for j in reversed(range(4)):
        x, _ = coupling_forward(S, spec, "ckbd", spec.n_scales - 1, j, x, training, reverse=True)
    for si in reversed(range(spec.n_scales - 1)):
        x = restore(x, offs[si])
        x = squeeze(x)
        for j in reversed(range(3)):
            x, _ = coupling_forward(S, spec, "chan", si, j, x, training, reverse=True)
        x = undo_squeeze(x)
        for j in reversed(range(3)):
            x, _ = coupling_forward(S, spec, "ckbd", si, j, x, training, reverse=True)
    return x


HALF_LOG_2PI = 0.5 * math.log(2 * math.pi)


def log_prob(S, spec: FlowSpec, x, training):
    """RealNVP.log_prob (flow_realnvp.py:329-340) with a N(0,1) prior (train.py:109)."""
    z, ldj = flow_f(S, spec, x, training)
    prior = (-0.5 * z * z - HALF_LOG_2PI).sum(dim=(1, 2, 3))
    return prior + ldj.sum(dim=(1, 2, 3))


def weight_scale(S, param_names: List[str], trainable) -> torch.Tensor:
    """RealNVP.forward regulariser (flow_realnvp.py:362-369): sum of squares of every
    trainable parameter whose last name component is weight_g or scale."""
    tot = None
    for n in param_names:
        if n.split(".")[-1] in ("weight_g", "scale") and trainable(n):
            t = S[n].pow(2).sum()
            tot = t if tot is None else tot + t
    return tot


def logit_transform(x: torch.Tensor, noise: torch.Tensor, constraint: float = 0.9):
    """utils.py:33-72 (forward), with the dequantisation noise passed in explicitly."""
    y = (x * 255.0 + noise) / 256.0
    y = ((y * 2.0 - 1.0) * constraint + 1.0) / 2.0
    lx = torch.log(y) - torch.log(1.0 - y)
    pre = torch.tensor(np.log(constraint) - np.log(1.0 - constraint))
    ld = F.softplus(lx) + F.softplus(-lx) - F.softplus(-pre)
    return lx, ld.sum(dim=(1, 2, 3))


def logit_inverse(x: torch.Tensor, constraint: float = 0.9):
    """utils.py:34-42."""
    y = 1.0 / (torch.exp(-x) + 1.0)
    return ((y * 2.0 - 1.0) / constraint + 1.0) / 2.0


def bits_per_dim(mean_logll: float, image_size: int, channels: int) -> float:
    """train.py:203-204."""
    D = image_size * image_size * channels
    return (-mean_logll + np.log(256.0) * D) / (D * np.log(2.0))


# ---------------------------------------------------------------------------
# one NLL training step (train.py:176-200)
# ---------------------------------------------------------------------------
SCALE_REG = 5e-5   # train.py:158


class OracleTrainer:
    """Restates train.py:176-200 around the functional flow: loss =
    -mean(log_prob + logdet) + 5e-5 * weight_scale, torch Adam(lr, wd) semantics
    (coupled L2 weight decay), model in train mode."""

    def __init__(self, S: State, spec: FlowSpec, param_names: List[str], trainable_names,
                 lr=5e-4, weight_decay=5e-5, betas=(0.9, 0.999), eps=1e-8):
        self.S, self.spec = S, spec
        self.names = [n for n in param_names if n in trainable_names]
        self.all_names = param_names
        self.trainable = set(trainable_names)
        self.lr, self.wd, self.betas, self.eps = lr, weight_decay, betas, eps
        self.m = {n: torch.zeros_like(S[n]) for n in self.names}
        self.v = {n: torch.zeros_like(S[n]) for n in self.names}
        self.t = 0

    def step(self, x: torch.Tensor, logdet: torch.Tensor):
        S = self.S
        for n in self.names:
            S[n] = S[n].detach().requires_grad_(True)
        lp = log_prob(S, self.spec, x, training=True)
        ws = weight_scale(S, self.all_names, lambda n: n in self.trainable)
        logll = (lp + logdet).mean()
        loss = -logll + SCALE_REG * ws
        grads = torch.autograd.grad(loss, [S[n] for n in self.names], allow_unused=True)
        self.t += 1
        b1, b2 = self.betas
        with torch.no_grad():
            for n, g in zip(self.names, grads):
                if g is None:
                    continue
                p = S[n].detach()
                g = g + self.wd * p
                self.m[n].mul_(b1).add_(g, alpha=1 - b1)
                self.v[n].mul_(b2).addcmul_(g, g, value=1 - b2)
                bc1 = 1 - b1 ** self.t
                bc2 = 1 - b2 ** self.t
                denom = (self.v[n].sqrt() / math.sqrt(bc2)).add_(self.eps)
                S[n] = p.addcdiv(self.m[n], denom, value=-self.lr / bc1)
        return float(loss.detach()), float(logll.detach())


# ---------------------------------------------------------------------------
# state layout in reference registration order
# ---------------------------------------------------------------------------
# Each entry: (key, shape, role) with role in {"param", "frozen", "buffer"};
# the list order is the reference state_dict order, and filtering the
# param/frozen entries gives named_parameters() order.
def _conv_spec(p, cin, cout, k, bias, scale, wn):
    """WeightNormConv2d (modules_realnvp.py:36-62).  weight_norm re-registers
    ``weight`` as weight_g/weight_v after ``bias``; weight_g is frozen when
    scale=False (57-59)."""
    out = []
    if wn:
        if bias:
            out.append((p + "conv.bias", (cout,), "param"))
        out.append((p + "conv.weight_g", (cout, 1, 1, 1), "param" if scale else "frozen"))
        out.append((p + "conv.weight_v", (cout, cin, k, k), "param"))
    else:
        out.append((p + "conv.weight", (cout, cin, k, k), "param"))
        if bias:
            out.append((p + "conv.bias", (cout,), "param"))
    return out


def _bn_spec(p, c, affine=True):
    out = [(p + "weight", (c,), "param"), (p + "bias", (c,), "param")] if affine else []
    return out + [(p + "running_mean", (c,), "buffer"), (p + "running_var", (c,), "buffer"),
                  (p + "num_batches_tracked", (), "buffer")]


def residual_module_spec(p, cin, dim, cout, hp: HP):
    """ResidualModule / ResidualBlock ctor order (modules_realnvp.py:73-173)."""
    wn, out = hp.weight_norm, []
    if hp.res_blocks > 0:
        out += _conv_spec(p + "in_block.", cin, dim, 3, True, False, wn)
        for i in range(hp.res_blocks):
            q = p + "core_block.%d." % i
            out += _bn_spec(q + "in_block.0.", dim)
            r = q + "res_block."
            if hp.bottleneck:
                out += _conv_spec(r + "0.", dim, dim, 1, False, False, wn) + _bn_spec(r + "1.", dim)
                out += _conv_spec(r + "3.", dim, dim, 3, False, False, wn) + _bn_spec(r + "4.", dim)
                out += _conv_spec(r + "6.", dim, dim, 1, True, True, wn)
            else:
                out += _conv_spec(r + "0.", dim, dim, 3, False, False, wn) + _bn_spec(r + "1.", dim)
                out += _conv_spec(r + "3.", dim, dim, 3, True, True, wn)
        out += _bn_spec(p + "out_block.0.", dim) + _conv_spec(p + "out_block.2.", dim, cout, 1, True, True, wn)
        if hp.skip:
            out += _conv_spec(p + "in_skip.", dim, dim, 1, True, True, wn)
            for i in range(hp.res_blocks):
                out += _conv_spec(p + "core_skips.%d." % i, dim, dim, 1, True, True, wn)
        return out
    b = p + "block."
    if hp.bottleneck:
        out += _conv_spec(b + "0.", cin, dim, 1, False, False, wn) + _bn_spec(b + "1.", dim)
        out += _conv_spec(b + "3.", dim, dim, 3, False, False, wn) + _bn_spec(b + "4.", dim)
        out += _conv_spec(b + "6.", dim, cout, 1, True, True, wn)
    else:
        out += _conv_spec(b + "0.", cin, dim, 3, False, False, wn) + _bn_spec(b + "1.", dim)
        out += _conv_spec(b + "3.", dim, cout, 3, True, True, wn)
    return out


def coupling_spec(p, kind, in_out, mid, hp: HP):
    """Checkerboard (modules_realnvp.py:249-262) / Channelwise (313-322) ctor order."""
    if kind == "ckbd":
        c_bn, cin, cout = in_out, 2 * in_out + 1, 2 * in_out
    else:
        c_bn, cin, cout = in_out // 2, in_out, in_out
    return ([(p + "scale", (1,), "param"), (p + "scale_shift", (1,), "param")] + _bn_spec(p + "in_bn.", c_bn)
            + residual_module_spec(p + "block.1.", cin, mid, cout, hp) + _bn_spec(p + "out_bn.", c_bn, affine=False))


def flow_spec_entries(spec: FlowSpec):
    """RealNVP.__init__ registration order (flow_realnvp.py:51-95)."""
    out = []
    for si in range(spec.n_scales - 1):
        c, _, d = spec.scales[si]
        for j in range(3):
            out += coupling_spec("s%d_ckbd.%d." % (si + 1, j), "ckbd", c, d, spec.hp)
        for j in range(3):
            out += coupling_spec("s%d_chan.%d." % (si + 1, j), "chan", 4 * c, 2 * d, spec.hp)
    c, _, d = spec.scales[-1]
    for j in range(4):
        out += coupling_spec("s%d_ckbd.%d." % (spec.n_scales, j), "ckbd", c, d, spec.hp)
    return out


def build_state(entries, value_fn):
    """state dict from entries; value_fn(key, shape, trainable) -> tensor."""
    S = {}
    for k, shp, role in entries:
        S[k] = value_fn(k, shp, role == "param")
    return S


def param_names(entries):
    return [k for k, _, r in entries if r != "buffer"]


def trainable_names(entries):
    return [k for k, _, r in entries if r == "param"]
