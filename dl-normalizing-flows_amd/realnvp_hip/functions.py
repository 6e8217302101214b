"""autograd bindings of the HIP engine (one torch.autograd.Function per fused op).

Parameters are passed to the Functions only so that autograd routes their
gradients; the kernels read them by device pointer.  Each backward returns
fresh gradient tensors (views into one flat block per call), so torch's
accumulation / set_to_none semantics are unchanged.
"""
import ctypes as C
import warnings

import torch

from . import _lib
from ._lib import TensorRef
from .engine import stream_ptr, upload


def _check_device(x, what):
    if not x.is_cuda:
        raise RuntimeError("%s: the MI355X engine needs tensors on a HIP device (got %s); "
                           "there is no CPU path" % (what, x.device))
    if x.dtype != torch.float32:
        raise RuntimeError("%s: expected float32, got %s" % (what, x.dtype))


# ---------------------------------------------------------------------------
# coupling
# ---------------------------------------------------------------------------
class _Coupling(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, training, dtype, full, *params):
        eng = mod.engine()
        B, _, H, W = x.shape
        sv = eng.saved(B, H, W, dtype, x.device, training)
        z, ldj, sv = eng.forward(x, training, dtype, full, saved=sv)
        if any(ctx.needs_input_grad):
            ctx.eng, ctx.sv, ctx.full = eng, sv, full
        else:   # no backward will read it
            eng.release(sv)
            ctx.eng, ctx.sv, ctx.full = eng, None, full
        ctx.mark_non_differentiable()
        return z, ldj

    @staticmethod
    def backward(ctx, gz, gl):
        eng, sv = ctx.eng, ctx.sv
        x = sv["x"]
        if gz is None:
            gz = torch.zeros_like(x)
        if gl is None:
            gl = torch.zeros((x.shape[0],) if not ctx.full else x.shape, device=x.device)
        gz = gz.contiguous()
        gl = gl.contiguous()
        grad_block = torch.zeros(eng.n_params, device=x.device, dtype=torch.float32)
        gx = eng.backward(sv, gz, gl if ctx.full else None, None if ctx.full else gl, grad_block)
        grads = []
        for (off, cnt), p in zip(eng.layout.values(), eng.params()):
            grads.append(grad_block[off:off + cnt].view_as(p) if p.requires_grad else None)
        ctx.sv = None
        eng.release(sv)
        return (gx, None, None, None, None) + tuple(grads)


def coupling_apply(mod, x, full_ldj):
    """(z, ldj) of one coupling; ldj elementwise [B,C,H,W] (full_ldj) or the
    per-sample sum [B]."""
    _check_device(x, type(mod).__name__)
    x = x.contiguous()
    params = tuple(mod.engine().params())
    return _Coupling.apply(x, mod, mod.training, mod.compute_dtype, full_ldj, *params)




class _CouplingReverse(torch.autograd.Function):
    """The inverse pass with a backward (modules_realnvp.py:284-291 is plain
    torch in the reference, so differentiable): the forward keeps its saved
    arena (net activations, in_bn batch sums) for rnvp_coupling_reverse_bwd +
    the net's and the in part's backward."""
    @staticmethod
    def forward(ctx, x, mod, training, dtype, *params):
        eng = mod.engine()
        B, _, H, W = x.shape
        sv = eng.saved(B, H, W, dtype, x.device, training)
        out, ldj = eng.reverse(x, training, dtype, saved=sv)
        ctx.eng, ctx.sv = eng, sv
        ctx.mark_non_differentiable()
        return out, ldj

    @staticmethod
    def backward(ctx, gz, gl):
        eng, sv = ctx.eng, ctx.sv
        x = sv["x"]
        gz = torch.zeros_like(x) if gz is None else gz.contiguous()
        gl = None if gl is None else gl.contiguous()
        grad_block = torch.zeros(eng.n_params, device=x.device, dtype=torch.float32)
        gx = eng.backward(sv, gz, gl, None, grad_block, reverse=True)
        grads = []
        for (off, cnt), p in zip(eng.layout.values(), eng.params()):
            grads.append(grad_block[off:off + cnt].view_as(p) if p.requires_grad else None)
        ctx.sv = None
        eng.release(sv)
        return (gx, None, None, None) + tuple(grads)


def coupling_reverse(mod, x):
    """Inverse pass (modules_realnvp.py:284-291, 345-351).  Returns (x, log_diag_J)
    where log_diag_J is the masked log_rescale, as the reference returns.
    Differentiable (x and the parameters) when autograd wants it; under
    torch.no_grad() (the sampling path, train.py:253-259) it keeps no state."""
    _check_device(x, type(mod).__name__)
    x = x.contiguous()
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in mod.engine().params())):
        params = tuple(mod.engine().params())
        return _CouplingReverse.apply(x, mod, mod.training, mod.compute_dtype, *params)
    with torch.no_grad():
        out, ldj = mod.engine().reverse(x, mod.training, mod.compute_dtype)
    return out, ldj


# ---------------------------------------------------------------------------
# permutations
# ---------------------------------------------------------------------------
def _sq(x):
    B, Cc, H, W = x.shape
    y = torch.empty(B, 4 * Cc, H // 2, W // 2, device=x.device, dtype=x.dtype)
    _lib.lib().squeeze(x.data_ptr(), y.data_ptr(), B, Cc, H, W, stream_ptr())
    return y


def _usq(y):
    B, C4, h, w = y.shape
    x = torch.empty(B, C4 // 4, 2 * h, 2 * w, device=y.device, dtype=y.dtype)
    _lib.lib().undo_squeeze(y.data_ptr(), x.data_ptr(), B, C4 // 4, 2 * h, 2 * w, stream_ptr())
    return x


def _fo(x):
    B, Cc, H, W = x.shape
    on = torch.empty(B, 2 * Cc, H // 2, W // 2, device=x.device, dtype=x.dtype)
    off = torch.empty_like(on)
    _lib.lib().factor_out(x.data_ptr(), on.data_ptr(), off.data_ptr(), B, Cc, H, W, stream_ptr())
    return on, off


def _rs(on, off):
    B, C2, h, w = on.shape
    x = torch.empty(B, C2 // 2, 2 * h, 2 * w, device=on.device, dtype=on.dtype)
    _lib.lib().restore(on.data_ptr(), off.data_ptr(), x.data_ptr(), B, C2 // 2, 2 * h, 2 * w, stream_ptr())
    return x


class _Squeeze(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _sq(x)

    @staticmethod
    def backward(ctx, g):
        return _usq(g.contiguous())


class _UndoSqueeze(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y):
        return _usq(y)

    @staticmethod
    def backward(ctx, g):
        return _sq(g.contiguous())


class _FactorOut(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _fo(x)

    @staticmethod
    def backward(ctx, gon, goff):
        if gon is None:
            gon = torch.zeros_like(goff)
        if goff is None:
            goff = torch.zeros_like(gon)
        return _rs(gon.contiguous(), goff.contiguous())


class _Restore(torch.autograd.Function):
    @staticmethod
    def forward(ctx, on, off):
        return _rs(on, off)

    @staticmethod
    def backward(ctx, g):
        return _fo(g.contiguous())


def _perm_check(x, what):
    _check_device(x, what)
    if x.dim() != 4 or x.shape[2] % 2 or x.shape[3] % 2:
        raise ValueError("%s: expected [B,C,H,W] with even H and W, got %s" % (what, tuple(x.shape)))


def squeeze(x):
    _perm_check(x, "squeeze")
    return _Squeeze.apply(x.contiguous())


def undo_squeeze(x):
    _check_device(x, "undo_squeeze")
    if x.dim() != 4 or x.shape[1] % 4:
        raise ValueError("undo_squeeze: channels must be a multiple of 4, got %s" % (tuple(x.shape),))
    return _UndoSqueeze.apply(x.contiguous())


def factor_out(x):
    _perm_check(x, "factor_out")
    return _FactorOut.apply(x.contiguous())


def restore(on, off):
    _check_device(on, "restore")
    if on.shape != off.shape or on.shape[1] % 2:
        raise ValueError("restore: on/off must match with an even channel count")
    return _Restore.apply(on.contiguous(), off.contiguous())


# ---------------------------------------------------------------------------
# N(0,1) prior log-prob + per-sample log-det (flow_realnvp.py:329-340)
# ---------------------------------------------------------------------------
class _StdNormalLogProb(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, ldj):
        B = z.shape[0]
        n = z.numel() // B
        out = torch.empty(B, device=z.device, dtype=torch.float32)
        _lib.lib().prior_logprob(z.data_ptr(), ldj.data_ptr(), out.data_ptr(), B, n, stream_ptr())
        ctx.save_for_backward(z)
        return out

    @staticmethod
    def backward(ctx, g):
        (z,) = ctx.saved_tensors
        B = z.shape[0]
        gz = torch.empty_like(z)
        g = g.contiguous()
        _lib.lib().prior_logprob_bwd(z.data_ptr(), g.data_ptr(), gz.data_ptr(), B, z.numel() // B, stream_ptr())
        return gz, g


def std_normal_logprob(z, ldj):
    return _StdNormalLogProb.apply(z.contiguous(), ldj.contiguous())


_STD_NORMAL = {}


def is_std_normal(prior):
    """True for torch.distributions.Normal(0, 1) (train.py:109), checked once
    per prior: the check reads device tensors (a host sync), so its result is
    cached against the loc / scale storage and version counters."""
    d = torch.distributions
    if not isinstance(prior, d.Normal):
        return False
    try:
        loc, scale = prior.loc, prior.scale
        key = (loc.data_ptr(), scale.data_ptr(), loc._version, scale._version, tuple(loc.shape))
        hit = _STD_NORMAL.get(id(prior))
        if hit is not None and hit[0] is prior and hit[1] == key:
            return hit[2]
        v = loc.dim() == 0 and bool((loc == 0).all()) and bool((scale == 1).all())
        _STD_NORMAL[id(prior)] = (prior, key, v)
        return v
    except Exception:
        return False


# ---------------------------------------------------------------------------
# weight_scale regulariser (flow_realnvp.py:362-369)
# ---------------------------------------------------------------------------
def _refs_table(params, grads, device):
    rows = [TensorRef(p.data_ptr(), g.data_ptr() if g is not None else None, p.numel())
            for p, g in zip(params, grads)]
    tab = (TensorRef * len(rows))(*rows)
    return upload(bytes(tab), device)


class _SumSq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *params):
        dev = params[0].device
        out = torch.zeros(1, device=dev, dtype=torch.float32)
        tab = _refs_table(params, [None] * len(params), dev)
        _lib.lib().sumsq_multi(tab.data_ptr(), len(params), out.data_ptr(), stream_ptr())
        ctx.save_for_backward(*params)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        params = ctx.saved_tensors
        dev = params[0].device
        sizes = [p.numel() for p in params]
        flat = torch.zeros(sum(sizes), device=dev, dtype=torch.float32)
        grads = list(torch.split(flat, sizes))
        tab = _refs_table(params, grads, dev)
        g1 = g.reshape(1).contiguous().float()
        _lib.lib().sumsq_bwd_multi(tab.data_ptr(), len(params), g1.data_ptr(), 1.0, stream_ptr())
        return tuple(gr.view_as(p) for gr, p in zip(grads, params))


def sum_of_squares(params):
    params = [p for p in params]
    for p in params:
        _check_device(p, "weight_scale")
    return _SumSq.apply(*params)
