"""Standalone calls of the s/t-network convolution (modules_realnvp.py:36-71).

On the training path a WeightNormConv2d never runs by itself: the coupling
engine (engine.py) fuses it with its neighbours' BatchNorm / ReLU / residual
work over NHWC activations.  The reference's submodules are nonetheless
callable on their own (WeightNormConv2d.forward, ResidualBlock.forward,
ResidualModule.forward: modules_realnvp.py:64-71, 107-114, 175-194), so the
drop-in keeps that API: a standalone WeightNormConv2d call runs the same HIP
kernels one at a time --

    forward : rnvp_weight_norm_fwd (w = g v / ||v||, packed fwd / dgrad
              images) -> rnvp_nchw_to_nhwc -> rnvp_conv2d (+ bias) ->
              rnvp_nhwc_to_nchw
    backward: rnvp_conv2d on the flipped image (data gradient),
              rnvp_conv2d_wgrad_grouped (one conv) -> rnvp_weight_norm_bwd
              (dv, dg, dbias)

in fp32 (exact-f32 MFMA, the reference's precision).  ResidualBlock and
ResidualModule compose their children exactly as the reference does, with
BatchNorm2d / ReLU as ordinary torch device modules.  Layout moves per call:
this is the API path, not the hot one.
"""
import ctypes as C

import torch

from . import _lib
from ._lib import RNVP_F32, ConvArgs, WgradGroup, WNDesc
from .engine import splitk_elems, splitk_workspace, stream_ptr, upload, wn_tiles
from .net import chan_stride, round_up


def _params(cp):
    """(v, g, bias, names) of a _ConvParams holder: weight-normalised
    (weight_v / weight_g) or plain (weight)."""
    if hasattr(cp, "weight_v"):
        return cp.weight_v, cp.weight_g, cp.bias, True
    return cp.weight, None, cp.bias, False


class _Geo:
    def __init__(self, cp, x):
        v, g, b, wn = _params(cp)
        self.cout, self.cin, self.ks = int(v.shape[0]), int(v.shape[1]), int(v.shape[2])
        self.B, _, self.H, self.W = (int(d) for d in x.shape)
        self.M = self.B * self.H * self.W
        self.cs_in, self.cs_out = chan_stride(self.cin), chan_stride(self.cout)
        self.kp_f = round_up(self.ks * self.ks * self.cs_in, 64)
        self.kp_d = round_up(self.ks * self.ks * self.cs_out, 64)


def _grad_layout(cp):
    """offset of each parameter in a flat fp32 block (named_parameters order)"""
    lay, off = {}, 0
    for n, p in cp.named_parameters():
        lay[n] = off
        off += p.numel()
    return lay, off


def _desc(cp, geo, wf, wd, norm):
    v, g, b, wn = _params(cp)
    lay, _ = _grad_layout(cp)
    d = WNDesc()
    d.v = v.data_ptr()
    d.g = g.data_ptr() if wn else None
    d.wf, d.wd, d.norm = wf.data_ptr(), wd.data_ptr(), norm.data_ptr()
    d.dw = None
    d.dv_off = lay["weight_v" if wn else "weight"]
    d.dg_off = lay["weight_g"] if (wn and g.requires_grad) else -1
    d.cout, d.cin, d.ks, d.cs_in, d.kp_f = geo.cout, geo.cin, geo.ks, geo.cs_in, geo.kp_f
    d.cs_out, d.kp_d, d.row0, d.tile0, d.nz = geo.cs_out, geo.kp_d, 0, 0, 1
    d.dbp, d.db_off, d.zero_after = None, (lay["bias"] if b is not None else 0), 0
    return d


def _table(d, dev):
    return upload(bytes(d), dev)


def _conv_args(geo, x, cs_in, cin, w, kp, y, cs_out, n, bias, dev):
    a = ConvArgs()
    a.dtype, a.B, a.H, a.W, a.ks = RNVP_F32, geo.B, geo.H, geo.W, geo.ks
    a.x, a.cs_in, a.cin = x.data_ptr(), cs_in, cin
    a.w, a.kp = w.data_ptr(), kp
    a.y, a.cs_out, a.n = y.data_ptr(), cs_out, n
    a.bias = bias.data_ptr() if bias is not None else None
    wse = splitk_elems(geo.M, max(geo.cs_in, geo.cs_out))
    if wse:
        ws = splitk_workspace(dev, wse)
        a.ws, a.ws_elems = ws.data_ptr(), wse
    a.variant = 0
    return a


class _WNConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cp, *params):
        L = _lib.lib()
        s = stream_ptr()
        dev = x.device
        geo = _Geo(cp, x)
        f32 = dict(device=dev, dtype=torch.float32)
        # packed images (their K padding must stay zero: allocated zeroed)
        wf = torch.zeros(geo.cout * geo.kp_f, **f32)
        wd = torch.zeros(geo.cin * geo.kp_d, **f32)
        norm = torch.empty(geo.cout, **f32)
        d = _desc(cp, geo, wf, wd, norm)
        tab = _table(d, dev)
        L.weight_norm_fwd(tab.data_ptr(), 1, geo.cout, wn_tiles(geo.cout, geo.cin, geo.ks), RNVP_F32, s)
        xh = torch.empty(geo.M * geo.cs_in, **f32)
        L.nchw_to_nhwc(x.data_ptr(), xh.data_ptr(), geo.B, geo.cin, geo.H, geo.W, geo.cs_in, RNVP_F32, s)
        yh = torch.empty(geo.M * geo.cs_out, **f32)
        _, _, bias, _ = _params(cp)
        a = _conv_args(geo, xh, geo.cs_in, geo.cin, wf, geo.kp_f, yh, geo.cs_out, geo.cout, bias, dev)
        L.conv2d(C.byref(a), s)
        y = torch.empty(geo.B, geo.cout, geo.H, geo.W, **f32)
        L.nhwc_to_nchw(yh.data_ptr(), y.data_ptr(), geo.B, geo.cout, geo.H, geo.W, geo.cs_out, RNVP_F32, s)
        ctx.cp, ctx.geo, ctx.desc = cp, geo, d
        ctx.save_for_backward(xh, wd, norm)
        return y

    @staticmethod
    def backward(ctx, gy):
        L = _lib.lib()
        s = stream_ptr()
        cp, geo, d = ctx.cp, ctx.geo, ctx.desc
        xh, wd, norm = ctx.saved_tensors
        dev = xh.device
        f32 = dict(device=dev, dtype=torch.float32)
        gy = gy.contiguous()
        gyh = torch.empty(geo.M * geo.cs_out, **f32)
        L.nchw_to_nhwc(gy.data_ptr(), gyh.data_ptr(), geo.B, geo.cout, geo.H, geo.W, geo.cs_out, RNVP_F32, s)
        gx = None
        if ctx.needs_input_grad[0]:
            gxh = torch.empty(geo.M * geo.cs_in, **f32)
            a = _conv_args(geo, gyh, geo.cs_out, geo.cout, wd, geo.kp_d, gxh, geo.cs_in, geo.cin, None, dev)
            L.conv2d(C.byref(a), s)
            gx = torch.empty(geo.B, geo.cin, geo.H, geo.W, **f32)
            L.nhwc_to_nchw(gxh.data_ptr(), gx.data_ptr(), geo.B, geo.cin, geo.H, geo.W, geo.cs_in, RNVP_F32, s)
        # weight (and bias) gradient: one-conv grouped launch into zeroed
        # partial slabs, summed by the weight-norm backward
        _, _, bias, _ = _params(cp)
        nz = int(L.wgrad_slabs(geo.M))
        nrep = int(L.wgrad_replicas(nz))
        nw = nrep * geo.cout * geo.kp_f
        ws = torch.zeros(nw + (nrep * geo.cout if bias is not None else 0), **f32)
        grp = WgradGroup()
        grp.dtype, grp.B, grp.H, grp.W, grp.n_conv = RNVP_F32, geo.B, geo.H, geo.W, 1
        c = grp.conv[0]
        c.x, c.cs_in, c.cin, c.ks = xh.data_ptr(), geo.cs_in, geo.cin, geo.ks
        c.dy, c.cs_dy, c.n = gyh.data_ptr(), geo.cs_out, geo.cout
        c.ws, c.kp, c.nz, c.nrep = ws.data_ptr(), geo.kp_f, nz, nrep
        c.wsb = ws.data_ptr() + 4 * nw if bias is not None else None
        L.conv2d_wgrad_grouped(C.byref(grp), s)
        e = WNDesc()
        C.memmove(C.addressof(e), C.addressof(d), C.sizeof(WNDesc))
        e.norm = norm.data_ptr()
        e.dw, e.nz = ws.data_ptr(), nrep
        e.dbp = ws.data_ptr() + 4 * nw if bias is not None else None
        _, n_params = _grad_layout(cp)
        block = torch.zeros(n_params, **f32)
        tab = _table(e, dev)
        L.weight_norm_bwd(tab.data_ptr(), 1, geo.cout, block.data_ptr(), None, 0, None, 0, s)
        lay, _ = _grad_layout(cp)
        grads = []
        for n, p in cp.named_parameters():
            grads.append(block[lay[n]:lay[n] + p.numel()].view_as(p) if p.requires_grad else None)
        return (gx, None) + tuple(grads)


def wn_conv2d(cp, x):
    """WeightNormConv2d / its weight-normalised nn.Conv2d applied to x
    ([B, cin, H, W] fp32 on a HIP device), 'same' padding, stride 1."""
    if not x.is_cuda:
        raise RuntimeError("WeightNormConv2d: the MI355X engine needs tensors on a HIP device (got %s); there is no "
                           "CPU path" % x.device)
    if x.dtype != torch.float32 or x.dim() != 4:
        raise RuntimeError("WeightNormConv2d: expected a 4-d float32 tensor, got %s %s" % (x.dtype, tuple(x.shape)))
    v, g, b, wn = _params(cp)
    if x.shape[1] != v.shape[1]:
        raise RuntimeError("WeightNormConv2d: expected %d input channels, got %d" % (v.shape[1], x.shape[1]))
    if cp.padding != v.shape[2] // 2:
        raise NotImplementedError("only 'same' padding (kernel_size // 2) occurs on the RealNVP path")
    return _WNConv.apply(x.contiguous(), cp, *tuple(cp.parameters()))
