"""Per-coupling executor: sequences the C-ABI kernels of one affine coupling
(modules_realnvp.py:239-370) and its s/t ResNet (36-194), forward, backward
and inverse.

Memory (all device, owned by torch tensors):
  * WeightSet  (per engine x dtype, persistent): packed weight images wf/wd,
    per-row norms, weight-norm descriptor table.
  * Saved      (per forward call, or persistent in the trainer): net input h0,
    every activation the backward needs, pre-out_bn u, fp64 BN batch sums.
  * Scratch    (per engine x shape, persistent): activation gradients, the
    pre-BN-apply temp, packed fp32 weight gradients, backward reductions.
Parameter gradients go to a flat fp32 "grad block" laid out like the
coupling's named_parameters() (frozen weight_g included, never written).
"""
import ctypes as C
from collections import OrderedDict

import torch

from . import _lib
from ._lib import (BNBwdArgs, BNRunning, BNSrc, ConvArgs, CouplingArgs, NetStep, WgradConv, WgradGroup, WNDesc,
                   NET_GROUP_MAX, RNVP_BF16, RNVP_F32, RNVP_STEP_BN_BWD, RNVP_STEP_CONV, WGRAD_GROUP_MAX)
from .net import backward_program, build_program, chan_stride, round_up

BN_EPS = 1e-5
COUPLING_SHARDS = 16      # RNVP_COUPLING_SHARDS (include/realnvp_hip.h; tests/test_boundary_cpu.py)
BN_MOMENTUM = 0.1

DTYPES = {"fp32": (RNVP_F32, 4, torch.float32), "bf16": (RNVP_BF16, 2, torch.bfloat16)}
# conv kernel family override for A/B diagnostics (rnvp_conv_args.variant; set
# programmatically by tests / tools, never from the environment):
# 0 = per-shape tuned dispatch, 1 = generic LDS-tiled kernels only
CONV_VARIANT = 0
# grouped launches of independent 1x1 convs (rnvp_net_group); False launches
# them one by one (tests/test_gpu_group.py compares the two)
NET_GROUP = True
# BatchNorm-backward applies folded into their consumer's data-gradient
# operand staging where the library supports it (rnvp_conv_args.bp, deep
# scales); False keeps every apply a launch of its own (tests compare the two)
FOLD_BN = True


def stream_ptr():
    return torch.cuda.current_stream().cuda_stream


def upload(raw, device):
    """A host descriptor table (bytes) -> a device uint8 tensor, copied on the
    current stream from pinned memory: a pageable copy would synchronise the
    stream and serialise the host's launches behind the GPU (the drop-in
    path builds some tables per call).  The caching host allocator keeps the
    pinned block until the copy has run."""
    host = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
    device = torch.device(device)
    if device.type != "cuda":
        return host
    return host.pin_memory().to(device, non_blocking=True)


# Optional launch timing (bench.py's per-kernel roofline): when PROFILE is a
# list, every engine launch appends (family, algorithmic bytes, flops,
# start event, end event), events recorded on the launch stream.
PROFILE = None
# When MARKERS is set (with PROFILE), an empty marker dispatch precedes and
# follows every engine launch so a per-dispatch PMC trace can be split by family
# (tools/pmc_traffic.py); MARKER_FAMILIES records the order.
MARKERS = False
MARKER_FAMILIES = []


def _launch(family, nbytes, flops, fn, *args):
    """One engine launch.  MARKERS alone (no PROFILE) also works under graph
    capture: the markers are captured with the step, so a rocprofv3 kernel
    trace of the replayed graph splits by family too (tools/trace_families.py)."""
    if PROFILE is None and not MARKERS:
        return fn(*args)
    if MARKERS:
        _lib.lib().marker(len(MARKER_FAMILIES), stream_ptr())
        MARKER_FAMILIES.append(family)
    if PROFILE is None:
        fn(*args)
    else:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn(*args)
        e1.record()
        PROFILE.append((family, nbytes, flops, e0, e1))
    if MARKERS:
        _lib.lib().marker(-1, stream_ptr())


class Arena:
    """Bump allocator over one device tensor (256-B aligned slots)."""

    def __init__(self):
        self.slots = OrderedDict()
        self.total = 0
        self.buf = None

    def add(self, name, nbytes):
        assert name not in self.slots, name
        self.slots[name] = (self.total, int(nbytes))
        self.total = round_up(self.total + int(nbytes), 256)

    def alloc(self, device, zero=False):
        n = max(self.total, 256)
        self.buf = (torch.zeros if zero else torch.empty)(n, dtype=torch.uint8, device=device)
        self.base = self.buf.data_ptr()
        return self

    def ptr(self, name):
        return self.base + self.slots[name][0]

    def has(self, name):
        return name in self.slots

    def view(self, name, dtype, shape=None):
        off, nb = self.slots[name]
        t = self.buf[off:off + nb].view(dtype)
        return t.view(shape) if shape is not None else t

    def range_bytes(self, first, last):
        """[start, end) byte range spanning slots first..last (in insertion order)."""
        s = self.slots[first][0]
        o, nb = self.slots[last]
        return s, o + nb


def _bn_src(sums, count, mean, var, gamma, beta, shards=1):
    return BNSrc(sums or None, float(count), mean or None, var or None, gamma or None, beta or None, BN_EPS,
                 int(shards))


def stat_shards(M):
    return int(_lib.lib().stat_shards(int(M)))


def wn_tiles(cout, cin, ks):
    """pack tiles of one conv in rnvp_weight_norm_fwd (rnvp_weight_norm_tiles)"""
    n = int(_lib.lib().weight_norm_tiles(int(cout), int(cin), int(ks)))
    if n <= 0:
        raise RuntimeError("rnvp_weight_norm_tiles: invalid conv shape %d x %d x %d" % (cout, cin, ks))
    return n


_SPLITK_WS = {}


def splitk_workspace(device, elems):
    """Per-device fp32 split-K workspace shared by every conv launch (all
    engine launches are ordered on the caller's stream)."""
    key = str(device)
    t = _SPLITK_WS.get(key)
    if t is None or t.numel() < elems:
        t = torch.empty(max(elems, 1 << 16), dtype=torch.float32, device=device)
        _SPLITK_WS[key] = t
    return t


def splitk_elems(M, nmax):
    return 8 * M * nmax if M <= 16384 else 0


def _independent(rw, members, j):
    """step j neither reads nor writes what the group members write, and
    writes nothing they read"""
    rj, wj = rw[j]
    for m in members:
        rm, wm = rw[m]
        if (wj & (rm | wm)) or (rj & wm):
            return False
    return True


def plan_launches(steps, device, rw=None):
    """Plan the launches of consecutive net steps (host NetStep structs):
    a run of mutually independent 1x1 convs (rw[i] = (buffers read, buffers
    written) of step i) that rnvp_net_group_prepare accepts becomes one
    grouped launch (rnvp_net_group); the rest stay single launches.
    Returns [("group", i0, i1, klass, grid, lds, host table) | ("single", i)];
    the host table (a NetStep array) travels by value in the kernel arguments."""
    L = _lib.lib()
    out = []
    n = len(steps)
    i = 0
    grouping = NET_GROUP and CONV_VARIANT == 0 and torch.device(device).type == "cuda" and rw is not None
    while i < n:
        if grouping:
            members = [i]
            best = None
            j = i + 1
            while j < n and len(members) < NET_GROUP_MAX and _independent(rw, members, j):
                arr = (NetStep * (j + 1 - i))(*steps[i:j + 1])
                k, g, lb = C.c_int(), C.c_int(), C.c_int()
                if L.net_group_prepare(arr, j + 1 - i, C.byref(k), C.byref(g), C.byref(lb)) != 0:
                    break
                members.append(j)
                best = (j + 1, arr, k.value, g.value, lb.value)
                j += 1
            if best is not None:
                j, arr, k, g, lb = best
                out.append(("group", i, j, k, g, lb, arr))
                i = j
                continue
        out.append(("single", i))
        i += 1
    return out


class CouplingEngine:
    """Executor for one Checkerboard/Channelwise affine coupling module."""

    def __init__(self, mod):
        self.mod = mod
        self.kind = 0 if mod.KIND == "ckbd" else 1
        self.C = mod.in_out_dim
        self.Cb = self.C if self.kind == 0 else self.C // 2
        cin = 2 * self.C + 1 if self.kind == 0 else self.C
        cout = 2 * self.Cb
        hp = mod.hps
        self.hp = hp
        self.P = build_program("block.1.", cin, mod.mid_dim, cout, hp.res_blocks, hp.bottleneck, hp.skip,
                               hp.weight_norm)
        self.steps = backward_program(self.P)
        self.cfg = 1 if mod.mask_config else 0
        # grad-block layout == named_parameters() order
        self.layout = OrderedDict()
        off = 0
        for n, p in mod.named_parameters():
            self.layout[n] = (off, p.numel())
            off += p.numel()
        self.n_params = off
        # (name, the owning module's _parameters / _buffers dict, key) of every
        # parameter and buffer, walked once: the per-call lookups are plain
        # dict reads (named_parameters() / named_buffers() recursed the module
        # tree on every call: ~30 % of the drop-in loop's host time)
        self._pslots = [(pre + ("." if pre else "") + k, m._parameters, k)
                        for pre, m in mod.named_modules() for k, v in m._parameters.items() if v is not None]
        self._bslots = [(pre + ("." if pre else "") + k, m._buffers, k)
                        for pre, m in mod.named_modules() for k, v in m._buffers.items() if v is not None]
        assert [n for n, _, _ in self._pslots] == list(self.layout), "parameter walk order"
        self._weights = {}
        self._scratch = {}
        self._saved_pool = {}

    # ------------------------------------------------------------------ params
    def _tensors(self):
        d = {n: dd[k] for n, dd, k in self._pslots}
        d.update({n: dd[k] for n, dd, k in self._bslots})
        return d

    def params(self):
        """the module's parameters in named_parameters() order (as _tensors)"""
        return [dd[k] for _, dd, k in self._pslots]

    def _conv_names(self, spec):
        p = spec.name + "conv."
        if spec.wn:
            return p + "weight_v", p + "weight_g", (p + "bias" if spec.bias else None)
        return p + "weight", None, (p + "bias" if spec.bias else None)

    def weights(self, dtype):
        """WeightSet for dtype, (re)built when parameter storage moved."""
        T = self._tensors()
        key = tuple(T[n].data_ptr() for n in self.layout)
        ws = self._weights.get(dtype)
        if ws is not None and ws["key"] == key:
            return ws
        dt, esz, _ = DTYPES[dtype]
        dev = next(iter(T.values())).device
        ar = Arena()
        geo = OrderedDict()
        for name, spec in self.P.convs.items():
            cs_in, cs_out = chan_stride(spec.cin), chan_stride(spec.cout)
            kp_f = round_up(spec.ks * spec.ks * cs_in, 64)
            kp_d = round_up(spec.ks * spec.ks * cs_out, 64)
            geo[name] = (cs_in, cs_out, kp_f, kp_d)
            ar.add("wf:" + name, spec.cout * kp_f * esz)
            ar.add("wd:" + name, spec.cin * kp_d * esz)
            ar.add("norm:" + name, spec.cout * 4)
            # bf16 3x3: fragment-major copies for the deep-scale tiles (rnvp_conv_args.w_frag),
            # written beside the row-major images by the weight-norm pack / transpose kernels.
            # (The 1x1 tiles and groups read them too, but their weight slices are small:
            # copies for them measured a wash -- 0.1 ms of tile time against 0.05 ms more
            # transpose traffic, gpurun_out/r5_fm1x1.)
            if dtype == "bf16" and spec.ks == 3:
                if cs_in % 32 == 0:
                    ar.add("wff:" + name, round_up(spec.cout, 16) * kp_f * esz)
                if cs_out % 32 == 0:
                    ar.add("wdf:" + name, round_up(spec.cin, 16) * kp_d * esz)
        ar.alloc(dev, zero=True)   # zero padding of the packed images, once
        descs = []
        row0 = tile0 = blk0 = 0
        for name, spec in self.P.convs.items():
            cs_in, cs_out, kp_f, kp_d = geo[name]
            vn, gn, _ = self._conv_names(spec)
            d = WNDesc()
            d.v = T[vn].data_ptr()
            d.g = T[gn].data_ptr() if gn else None
            d.wf, d.wd, d.norm = ar.ptr("wf:" + name), ar.ptr("wd:" + name), ar.ptr("norm:" + name)
            d.wf_frag = ar.ptr("wff:" + name) if ar.has("wff:" + name) else None
            d.wd_frag = ar.ptr("wdf:" + name) if ar.has("wdf:" + name) else None
            d.dw = None
            d.dv_off = self.layout[vn][0]
            d.dg_off = self.layout[gn][0] if (gn and spec.scale) else -1
            d.cout, d.cin, d.ks, d.cs_in, d.kp_f, d.cs_out, d.kp_d, d.row0 = (
                spec.cout, spec.cin, spec.ks, cs_in, kp_f, cs_out, kp_d, row0)
            d.nz = 1
            d.tile0 = tile0
            _, _, bname = self._conv_names(spec)
            d.db_off = self.layout[bname][0] if bname else -1
            d.blk0 = blk0
            # the fused pass's row blocks assume the packed row stride round_up(cin, 8)
            assert cs_in == round_up(spec.cin, 8), (name, cs_in, spec.cin)
            nb = int(_lib.lib().weight_norm_opt_blocks(spec.cout, spec.cin, spec.ks))
            blk0 = blk0 + nb if (nb > 0 and blk0 >= 0) else -1
            row0 += spec.cout
            tile0 += wn_tiles(spec.cout, spec.cin, spec.ks)
            descs.append(d)
        table = (WNDesc * len(descs))(*descs)
        dtab = upload(bytes(table), dev)
        # blocks < 0: some conv's rows do not fit the fused parameter pass
        ws = dict(key=key, arena=ar, geo=geo, descs=descs, table=dtab, rows=row0, tiles=tile0, dtype=dtype,
                  blocks=blk0)
        self._weights[dtype] = ws
        return ws

    def prepare_weights(self, dtype):
        ws = self.weights(dtype)
        _lib.lib().weight_norm_fwd(ws["table"].data_ptr(), len(ws["descs"]), ws["rows"], ws["tiles"],
                                   DTYPES[dtype][0], stream_ptr())
        return ws

    # ------------------------------------------------------------ workspaces
    def alloc_saved(self, B, H, W, dtype, device, training):
        esz = DTYPES[dtype][1]
        M = B * H * W
        ar = Arena()
        ar.add("h0", M * chan_stride(self.P.buf_ch["h0"]) * esz)
        for b, ch in self.P.buf_ch.items():
            if b != "h0":
                ar.add(b, M * chan_stride(ch) * esz)
        ar.add("u", B * self.C * H * W * 4)
        ar.add("in_sums", COUPLING_SHARDS * 2 * self.Cb * 8)
        ar.add("out_sums", COUPLING_SHARDS * 2 * self.Cb * 8)
        # coupling links (rnvp_coupling_out_u / _link_fwd): u's sums per pixel class, the prior's sums
        ar.add("cls_sums", COUPLING_SHARDS * 4 * 2 * self.C * 8)
        ar.add("prior_sums", COUPLING_SHARDS * 4 * 2 * self.C * 8)
        ar.add("out_tab", 2 * self.Cb * 4)     # the forward's out_bn / in_bn tables for the link backward
        ar.add("in_tab", 4 * self.Cb * 4)
        sh = stat_shards(M)
        for bn, spec in self.P.bns.items():
            ar.add("s:" + bn, sh * 2 * spec.c * 8)
        ar.alloc(device, zero=True)   # the sums start zero (persistent arenas keep them zero between steps)
        sv = dict(arena=ar, B=B, H=H, W=W, dtype=dtype, training=training, shards=sh)
        # running-stat update table for the net BNs
        if training and self.P.bns:
            T = self._tensors()
            rows = []
            for bn, spec in self.P.bns.items():
                r = BNRunning(ar.ptr("s:" + bn), float(M), spec.c, sh, T[bn + "running_mean"].data_ptr(),
                              T[bn + "running_var"].data_ptr(), T[bn + "num_batches_tracked"].data_ptr())
                rows.append(r)
            tab = (BNRunning * len(rows))(*rows)
            sv["bn_table"] = upload(bytes(tab), device)
            sv["bn_n"] = len(rows)
            sv["bn_cmax"] = max(spec.c for spec in self.P.bns.values())
        return sv

    def _pool_key(self, B, H, W, dtype, device, training):
        return (B, H, W, dtype, str(device), bool(training))

    def saved(self, B, H, W, dtype, device, training):
        """A saved-activation arena of this shape: a released one when
        available (the drop-in's autograd path returns them after backward), so
        an eager training loop neither reallocates nor re-zeroes the whole
        arena every call (forward zeroes the batch sums it accumulates)."""
        pool = self._saved_pool.get(self._pool_key(B, H, W, dtype, device, training))
        if pool:
            return pool.pop()
        return self.alloc_saved(B, H, W, dtype, device, training)

    def release(self, sv):
        """Hand an arena back (stream-ordered: later users run after the
        kernels that read it)."""
        sv.pop("x", None)
        key = self._pool_key(sv["B"], sv["H"], sv["W"], sv["dtype"], sv["arena"].buf.device, sv["training"])
        pool = self._saved_pool.setdefault(key, [])
        if len(pool) < 2:
            pool.append(sv)

    def param_pass_info(self, sv, dtype):
        """(host weight-norm descs with this coupling's wgrad slabs, [(ptr,
        bytes)] ranges its deferred parameter pass must leave zero: the
        forward batch sums of the saved arena sv and the backward reductions
        of the scratch) -- what backward(opt="defer") skips."""
        B, H, W = sv["B"], sv["H"], sv["W"]
        sc = self.scratch_checked(B, H, W, dtype, sv["arena"].buf.device)
        ar, sar = sv["arena"], sc["arena"]
        f0, f1 = ar.range_bytes("in_sums", list(ar.slots)[-1])
        z0, z1 = sc["zero"]
        return sc["wn_descs"], [(ar.base + f0, f1 - f0), (sar.base + z0, z1 - z0)]

    def scratch_checked(self, B, H, W, dtype, device):
        """scratch() rebuilt when the weight set moved since it was made (its
        weight-norm table points into the packed-weight arena)."""
        sc = self.scratch(B, H, W, dtype, device)
        if sc["wn_key"] != self.weights(dtype)["key"]:
            self._scratch.pop((B, H, W, dtype, str(device)))
            sc = self.scratch(B, H, W, dtype, device)
        return sc

    def scratch(self, B, H, W, dtype, device):
        key = (B, H, W, dtype, str(device))
        sc = self._scratch.get(key)
        if sc is not None:
            return sc
        esz = DTYPES[dtype][1]
        M = B * H * W
        ar = Arena()
        # zeroed every backward: the reductions (kept contiguous)
        wsz = self.weights(dtype)
        ar.add("bwd_sums", COUPLING_SHARDS * 3 * self.Cb * 8)
        # coupling links (rnvp_coupling_link_bwd): direct input-gradient sums, in_bn kept-position sums
        ar.add("outp_sums", COUPLING_SHARDS * 2 * 2 * self.C * 8)
        ar.add("in_bwd_ext", COUPLING_SHARDS * 2 * self.Cb * 8)
        ar.add("in_bwd_sums", COUPLING_SHARDS * 2 * self.Cb * 8)
        ar.add("gscale_part", COUPLING_SHARDS * 2 * 8)   # left zero by coupling_in_bwd
        first, last = "bwd_sums", "in_bwd_sums"
        sh = stat_shards(M)
        for bn, spec in self.P.bns.items():
            ar.add("e:" + bn, sh * 2 * spec.c * 8)
            last = "e:" + bn
        zr = ar.range_bytes(first, last)
        for b, ch in self.P.buf_ch.items():
            ar.add("g:" + b, M * chan_stride(ch) * esz)
        cmax = max([chan_stride(s.cin) for s in self.P.convs.values()])
        ar.add("gtmp", M * cmax * esz)
        ar.add("gtmp2", M * cmax * esz)     # the other pre-apply temp of a folded BatchNorm backward
        ar.alloc(device, zero=True)
        # grouped weight-gradient partial sums: [nrep][cout][kp_f] (+ bias [nrep][cout])
        nz = int(_lib.lib().wgrad_slabs(M))
        nrep = int(_lib.lib().wgrad_replicas(nz))
        wg = {}
        off = 0
        for name, spec in self.P.convs.items():
            kp_f = wsz["geo"][name][2]
            ow = off
            off += nrep * spec.cout * kp_f
            ob = None
            if spec.bias:
                ob = off
                off += nrep * spec.cout
            wg[name] = (ow, ob)
            off = round_up(off, 64)
        # per-coupling (zeroed once): replica regions are re-zeroed by the
        # weight-norm backward, plain-store regions are fully overwritten
        wgws = torch.zeros(max(off, 64), dtype=torch.float32, device=device)
        wbase = wgws.data_ptr()
        # weight-norm backward table (sums the slabs, writes dv / dg / dbias)
        descs = []
        for d, (name, spec) in zip(wsz["descs"], self.P.convs.items()):
            e = WNDesc()
            C.memmove(C.addressof(e), C.addressof(d), C.sizeof(WNDesc))
            ow, ob = wg[name]
            e.dw = wbase + 4 * ow
            e.nz = nrep
            _, _, bname = self._conv_names(spec)
            e.dbp = wbase + 4 * ob if ob is not None else None
            e.db_off = self.layout[bname][0] if ob is not None else -1
            e.zero_after = int(nrep < nz)
            descs.append(e)
        tab = (WNDesc * len(descs))(*descs)
        nmax = max(max(chan_stride(s.cin), chan_stride(s.cout)) for s in self.P.convs.values())
        wse = splitk_elems(M, nmax)
        sc = dict(arena=ar, zero=zr, wn_table=upload(bytes(tab), device), wn_descs=descs,
                  wn_key=wsz["key"], wn_rows=wsz["rows"], wn_blocks=wsz["blocks"], n_wn=len(descs), shards=sh,
                  ws=splitk_workspace(device, wse) if wse else None, ws_elems=wse,
                  wg=wg, wg_nz=nz, wg_nrep=nrep, wg_ws=wgws)
        self._scratch[key] = sc
        return sc

    # --------------------------------------------------------------- helpers
    def _coupling_args(self, T, x, B, H, W, dtype, training):
        a = CouplingArgs()
        a.kind, a.B, a.C, a.H, a.W = self.kind, B, self.C, H, W
        a.mask_config, a.coupling_bn, a.training = self.cfg, int(self.hp.coupling_bn), int(training)
        a.dtype = DTYPES[dtype][0]
        a.momentum, a.eps = BN_MOMENTUM, BN_EPS
        a.x = x.data_ptr()
        a.in_gamma, a.in_beta = T["in_bn.weight"].data_ptr(), T["in_bn.bias"].data_ptr()
        a.in_rmean, a.in_rvar = T["in_bn.running_mean"].data_ptr(), T["in_bn.running_var"].data_ptr()
        a.in_nbt = T["in_bn.num_batches_tracked"].data_ptr()
        a.scale, a.scale_shift = T["scale"].data_ptr(), T["scale_shift"].data_ptr()
        a.out_rmean, a.out_rvar = T["out_bn.running_mean"].data_ptr(), T["out_bn.running_var"].data_ptr()
        a.out_nbt = T["out_bn.num_batches_tracked"].data_ptr()
        a.cs_h0 = chan_stride(self.P.buf_ch["h0"])
        a.cs_st = chan_stride(self.P.buf_ch["st"])
        return a

    def _bn(self, T, bn, training, sums_ptr, M):
        return _bn_src(sums_ptr if training else None, M, T[bn + "running_mean"].data_ptr(),
                       T[bn + "running_var"].data_ptr(), T[bn + "weight"].data_ptr(), T[bn + "bias"].data_ptr(),
                       stat_shards(M))

    def _net_forward(self, T, sv, ws, training, s):
        """The s/t net's conv launches.  Their argument structs depend only on
        the saved arena, the weight set, the scratch and the parameters'
        storage, so they are built once per arena (re-built when the weights
        move) and replayed: per-call host work is the ctypes calls alone."""
        L = _lib.lib()
        key = (ws["key"], bool(training))
        plan = sv.get("fwd_plan")
        if plan is None or plan[0] != key:
            args = self._fwd_args(T, sv, ws, training)
            steps, rw = [], []
            for (a, _, _), op in zip(args, self.P.ops):
                st = NetStep()
                st.kind = RNVP_STEP_CONV
                st.conv = a
                steps.append(st)
                reads = {op.x} | ({op.residual} if op.residual else set()) | ({op.y} if op.accumulate else set())
                reads |= {"s:" + op.pro_bn} if op.pro_bn else set()
                rw.append((reads, {op.y} | ({"s:" + op.stats_bn} if op.stats_bn else set())))
            plan = (key, args, plan_launches(steps, sv["arena"].buf.device, rw))
            sv["fwd_plan"] = plan
        args = plan[1]
        dt = DTYPES[sv["dtype"]][0]
        for g in plan[2]:
            if g[0] == "single":
                a, nb, fl = args[g[1]]
                _launch("conv_fwd", nb, fl, L.conv2d, C.byref(a), s)
            else:
                _, i0, i1, klass, grid, lds, tab = g
                nb = sum(args[i][1] for i in range(i0, i1))
                fl = sum(args[i][2] for i in range(i0, i1))
                _launch("conv_fwd", nb, fl, L.net_group, C.addressof(tab), i1 - i0, dt, klass, grid, lds, s)

    def _fwd_args(self, T, sv, ws, training):
        ar = sv["arena"]
        B, H, W = sv["B"], sv["H"], sv["W"]
        M = B * H * W
        dt = DTYPES[sv["dtype"]][0]
        war = ws["arena"]
        sc = self.scratch(B, H, W, sv["dtype"], ar.buf.device)
        out = []
        for op in self.P.ops:
            spec = self.P.convs[op.conv]
            cs_in, cs_out, kp_f, _ = ws["geo"][op.conv]
            a = ConvArgs()
            a.dtype, a.B, a.H, a.W, a.ks = dt, B, H, W, spec.ks
            a.x, a.cs_in, a.cin = ar.ptr(op.x), cs_in, spec.cin
            a.w, a.kp = war.ptr("wf:" + op.conv), kp_f
            a.w_frag = war.ptr("wff:" + op.conv) if war.has("wff:" + op.conv) else None
            a.y, a.cs_out, a.n = ar.ptr(op.y), cs_out, spec.cout
            _, _, bn_ = self._conv_names(spec)
            a.bias = T[bn_].data_ptr() if bn_ else None
            a.residual = ar.ptr(op.residual) if op.residual else None
            a.accumulate = int(op.accumulate)
            if op.pro_bn:
                a.pro_bn_relu = 1
                a.pro = self._bn(T, op.pro_bn, training, ar.ptr("s:" + op.pro_bn), M)
            a.out_sums = ar.ptr("s:" + op.stats_bn) if (op.stats_bn and training) else None
            if sc["ws"] is not None:
                a.ws, a.ws_elems = sc["ws"].data_ptr(), sc["ws_elems"]
            a.variant = CONV_VARIANT
            esz = DTYPES[sv["dtype"]][1]
            nb = esz * (M * cs_in + spec.cout * kp_f + M * cs_out * (1 + int(bool(op.residual)) + int(op.accumulate)))
            out.append((a, nb, 2.0 * M * spec.cout * spec.ks * spec.ks * spec.cin))
        return out

    # ---------------------------------------------------------------- forward
    def chains_into(self, nxt):
        """True when coupling `nxt` directly consumes this coupling's output
        as the next coupling of the same combo (a RNVP_LINK_SAME link): same
        kind and shape, the opposite mask, out_bn with batch statistics."""
        return (nxt.kind == self.kind and nxt.C == self.C and nxt.cfg != self.cfg and
                bool(self.hp.coupling_bn))

    def forward(self, x, training, dtype, full_ldj, saved=None, prepare=True, ldj_sample=None, z_out=None,
                zero_sums=True):
        """x: [B,C,H,W] fp32 device tensor.  Returns (z, ldj, saved) where ldj
        is the elementwise log_diag_J [B,C,H,W] (full_ldj) or this coupling's
        per-sample sum [B] (accumulated into ldj_sample when given).
        zero_sums=False: the batch-statistic sums of `saved` are already zero
        (the previous step's backward left them so: backward(zero_at_end=True))."""
        L = _lib.lib()
        B, Cc, H, W = x.shape
        assert Cc == self.C, "channel mismatch"
        dev = x.device
        s = stream_ptr()
        ws = self.prepare_weights(dtype) if prepare else self.weights(dtype)
        sv = saved if saved is not None else self.alloc_saved(B, H, W, dtype, dev, training)
        ar = sv["arena"]
        T = self._tensors()
        z = torch.empty_like(x) if z_out is None else z_out
        if ldj_sample is None:
            ldj_sample = torch.zeros(B, device=dev, dtype=torch.float32)
        ldj_full = torch.empty_like(x) if full_ldj else None
        if training and zero_sums:
            s0, e0 = ar.range_bytes("in_sums", list(ar.slots)[-1])
            ar.buf[s0:e0].zero_()
        a = self._coupling_args(T, x, B, H, W, dtype, training)
        a.in_sums = ar.ptr("in_sums")
        a.h0 = ar.ptr("h0")
        n_el, esz = x.numel(), DTYPES[dtype][1]
        cs_h0, cs_st = chan_stride(self.P.buf_ch["h0"]), chan_stride(self.P.buf_ch["st"])
        # algorithmic bytes: x read by the stats and the apply pass, h0 written
        _launch("coupling", (8 if training else 4) * n_el + esz * B * H * W * cs_h0, 0.0, L.coupling_in_fwd,
                C.byref(a), s)
        self._net_forward(T, sv, ws, training, s)
        if training and "bn_table" in sv:
            # the net BNs' running-stat updates ride on the out launch
            a.net_running, a.n_net_running, a.net_running_cmax = (sv["bn_table"].data_ptr(), sv["bn_n"],
                                                                  sv["bn_cmax"])
        a.st = ar.ptr("st")
        a.u, a.z = ar.ptr("u"), z.data_ptr()
        a.out_sums = ar.ptr("out_sums")
        a.ldj_sample = ldj_sample.data_ptr()
        a.ldj_full = ldj_full.data_ptr() if full_ldj else None
        _launch("coupling", 16 * n_el + esz * B * H * W * cs_st, 0.0, L.coupling_out_fwd, C.byref(a), s)
        sv["x"] = x
        return z, (ldj_full if full_ldj else ldj_sample), sv

    # ---------------------------------------------------------------- inverse
    def reverse(self, x, training, dtype, saved=None, out=None, want_ldj=True, prepare=True):
        """Inverse pass (modules_realnvp.py:284-291, 345-351).  saved / out:
        persistent buffers (graph-captured sampling); prepare=False when the
        packed weights are already current."""
        L = _lib.lib()
        B, Cc, H, W = x.shape
        s = stream_ptr()
        ws = self.prepare_weights(dtype) if prepare else self.weights(dtype)
        sv = saved if saved is not None else self.alloc_saved(B, H, W, dtype, x.device, training)
        ar = sv["arena"]
        T = self._tensors()
        if training:
            s0, e0 = ar.range_bytes("in_sums", list(ar.slots)[-1])
            ar.buf[s0:e0].zero_()
        a = self._coupling_args(T, x, B, H, W, dtype, training)
        a.in_sums = ar.ptr("in_sums")
        a.h0 = ar.ptr("h0")
        L.coupling_in_fwd(C.byref(a), s)
        self._net_forward(T, sv, ws, training, s)
        if training and "bn_table" in sv:
            L.bn_running_update(sv["bn_table"].data_ptr(), sv["bn_n"], sv["bn_cmax"], BN_MOMENTUM, s)
        if out is None:
            out = torch.empty_like(x)
        ldj = torch.empty_like(x) if want_ldj else None
        a.st = ar.ptr("st")
        a.z = out.data_ptr()
        a.ldj_full = ldj.data_ptr() if want_ldj else None
        L.coupling_reverse(C.byref(a), s)
        sv["x"] = x          # (the input, for a backward through the inverse)
        return out, ldj


    def _net_backward(self, sv, sc, ws, T, training, gp, s):
        """The net's data-gradient chain: conv data gradients and BatchNorm
        backward applies (single or grouped launches) from d st to d h0."""
        L = _lib.lib()
        x = sv["x"]
        dt = DTYPES[sv["dtype"]][0]
        # the net's data-gradient chain and grouped weight gradients: argument
        # structs cached per (saved arena, scratch, weight set); only the
        # BatchNorm-affine gradient pointers follow this call's grad block
        key = (ws["key"], id(sc), bool(training), FOLD_BN)
        plan = sv.get("bwd_plan")
        if plan is None or plan[0] != key:
            plan = (key, self._bwd_args(T, sv, sc, ws, training))
            sv["bwd_plan"] = plan
        items, groups, wg_bytes, wg_flops = plan[1]
        if len(plan) < 3:
            steps = []
            for kind, c, nb, fl, bn, rw in items:
                st = NetStep()
                st.dgamma_off = st.dbeta_off = -1
                if kind == "dgrad":
                    st.kind = RNVP_STEP_CONV
                    st.conv = c
                else:
                    st.kind = RNVP_STEP_BN_BWD
                    st.bn = c
                    st.dgamma_off = self.layout[bn + "weight"][0]
                    st.dbeta_off = self.layout[bn + "bias"][0]
                steps.append(st)
            plan = plan + (plan_launches(steps, x.device, [it[5] for it in items]),)
            sv["bwd_plan"] = plan
        for g in plan[2]:
            if g[0] == "single":
                kind, c, nb, fl, bn, _ = items[g[1]]
                if kind == "dgrad":
                    if bn is not None:      # folded BatchNorm backward: its parameter gradients
                        c.bp_dgamma, c.bp_dbeta = gp(bn + "weight"), gp(bn + "bias")
                    _launch("conv_dgrad", nb, fl, L.conv2d, C.byref(c), s)
                else:
                    c.dgamma, c.dbeta = gp(bn + "weight"), gp(bn + "bias")
                    _launch("bn_bwd", nb, 0.0, L.bn_bwd_apply, C.byref(c), s)
            else:
                _, i0, i1, klass, grid, lds, tab = g
                nb = sum(items[i][2] for i in range(i0, i1))
                fl = sum(items[i][3] for i in range(i0, i1))
                _launch("conv_dgrad", nb, fl, L.net_group, C.addressof(tab), i1 - i0, dt, klass, grid, lds, s)

    def _weight_grads(self, sv, sc, ws, zero_at_end, opt, after, gbase):
        """The closure issuing the net's grouped weight gradients (+ the
        weight-norm backward or the fused parameter pass, see backward)."""
        L = _lib.lib()
        ar, sar = sv["arena"], sc["arena"]
        z0, z1 = sc["zero"]
        dt = DTYPES[sv["dtype"]][0]
        items, groups, wg_bytes, wg_flops = sv["bwd_plan"][1]

        # the weight gradients (grouped wgrad + weight-norm backward)
        # only feed the optimizer: on a side stream they overlap the backward
        # of the couplings before this one.  They read this coupling's saved
        # activations and gradient scratch, which nothing later in the step
        # rewrites; `after` runs behind them on the same stream (per-coupling
        # optimizer update).
        def weight_grads():
            ss = stream_ptr()
            for grp in groups:
                _launch("conv_wgrad", wg_bytes / len(groups), wg_flops / len(groups), L.conv2d_wgrad_grouped,
                        C.byref(grp), ss)
            # the backward reductions live in the scratch shared by every
            # caller of this shape (trainer and drop-in autograd alike): it is
            # ALWAYS left zero, so whichever path runs next finds it clean
            # (the drop-in also zeroes it on entry).  The forward's batch sums
            # belong to the saved arena: left zero only for the trainer's
            # persistent arenas (zero_at_end).
            if zero_at_end:
                f0, f1 = ar.range_bytes("in_sums", list(ar.slots)[-1])
                zr = (ar.base + f0, f1 - f0, sar.base + z0, z1 - z0)
            else:
                zr = (None, 0, sar.base + z0, z1 - z0)
            if isinstance(opt, str):
                pass    # "defer": the caller's model-wide parameter pass reads the slabs
            elif opt is not None:
                L.weight_norm_bwd_adam(sc["wn_table"].data_ptr(), sc["n_wn"], sc["wn_blocks"], 1, dt, C.byref(opt),
                                       *zr, ss)
            else:
                L.weight_norm_bwd(sc["wn_table"].data_ptr(), sc["n_wn"], sc["wn_rows"], gbase, *zr, ss)
            if after is not None:
                after()

        return weight_grads

    # --------------------------------------------------------------- backward
    def _bwd_args(self, T, sv, sc, ws, training):
        """(items, wgrad groups, wgrad bytes, wgrad flops) of the net backward:
        items are ("dgrad", ConvArgs, bytes, flops, folded bn name or None, rw)
        or ("bn", BNBwdArgs, bytes, 0, bn name, rw) in launch order, rw =
        (buffers read, buffers written); grouped weight gradients: one launch
        per WGRAD_GROUP_MAX convs (the group travels as a by-value kernel
        argument); R >= 6 nets have more."""
        B, H, W, dtype = sv["B"], sv["H"], sv["W"], sv["dtype"]
        M = B * H * W
        dt = DTYPES[dtype][0]
        esz = DTYPES[dtype][1]
        ar, sar, war = sv["arena"], sc["arena"], ws["arena"]
        items, groups = [], []
        ent = []        # [kind, args, bytes, flops, bn, reads, writes, BwdStep, tmp name]
        wg_bytes = wg_flops = 0.0
        wbase = sc["wg_ws"].data_ptr()
        for st in self.steps:
            op = st.op
            spec = self.P.convs[op.conv]
            cs_in, cs_out, kp_f, kp_d = ws["geo"][op.conv]
            if st.kind == "dgrad":
                c = ConvArgs()
                c.dtype, c.B, c.H, c.W, c.ks = dt, B, H, W, spec.ks
                c.x, c.cs_in, c.cin = sar.ptr(st.gy), cs_out, spec.cout
                c.w, c.kp = war.ptr("wd:" + op.conv), kp_d
                c.w_frag = war.ptr("wdf:" + op.conv) if war.has("wdf:" + op.conv) else None
                c.y = sar.ptr(st.tmp if st.tmp else st.gx)
                c.cs_out, c.n = cs_in, spec.cin
                c.residual = sar.ptr(st.residual) if st.residual else None
                c.accumulate = int(st.accumulate)
                if op.pro_bn:
                    c.epi_relu_bn_bwd = 1
                    c.epi_x = ar.ptr(op.x)
                    c.epi = self._bn(T, op.pro_bn, training, ar.ptr("s:" + op.pro_bn), M)
                    c.epi_sums = sar.ptr("e:" + op.pro_bn)
                if sc["ws"] is not None:
                    c.ws, c.ws_elems = sc["ws"].data_ptr(), sc["ws_elems"]
                c.variant = CONV_VARIANT
                nb = esz * (M * cs_out + spec.cin * kp_d + M * cs_in * (1 + int(bool(op.pro_bn)) + int(bool(
                    st.residual)) + int(st.accumulate)))
                dst = st.tmp if st.tmp else st.gx
                reads = {st.gy} | ({op.x} if op.pro_bn else set()) | ({st.residual} if st.residual else set()) | (
                    {dst} if st.accumulate else set())
                writes = {dst} | ({"e:" + op.pro_bn} if op.pro_bn else set())
                ent.append(["dgrad", c, nb, 2.0 * M * spec.cout * spec.ks * spec.ks * spec.cin, None, reads, writes, st,
                            st.tmp])
            elif st.kind == "bn_apply":
                bn = op.pro_bn
                c = BNBwdArgs()
                c.dtype, c.M, c.C, c.cs = dt, M, spec.cin, cs_in
                c.g, c.x = sar.ptr(st.tmp), ar.ptr(op.x)
                c.bn = self._bn(T, bn, training, ar.ptr("s:" + bn), M)
                c.sums = sar.ptr("e:" + bn)
                c.sum_shards = sc["shards"]
                c.dx = sar.ptr(st.gx)
                c.residual = sar.ptr(st.residual) if st.residual else None
                c.accumulate = int(st.accumulate)
                reads = {st.tmp, op.x, "e:" + bn} | ({st.residual} if st.residual else set()) | (
                    {st.gx} if st.accumulate else set())
                ent.append(["bn", c, esz * M * cs_in * (3 + int(bool(st.residual)) + int(st.accumulate)), 0.0, bn,
                            reads, {st.gx}, st, st.tmp])
            else:
                if not groups or groups[-1].n_conv >= WGRAD_GROUP_MAX:
                    grp = WgradGroup()
                    grp.dtype, grp.B, grp.H, grp.W = dt, B, H, W
                    groups.append(grp)
                grp = groups[-1]
                c = grp.conv[grp.n_conv]
                grp.n_conv += 1
                ow, ob = sc["wg"][op.conv]
                c.x, c.cs_in, c.cin, c.ks = ar.ptr(op.x), cs_in, spec.cin, spec.ks
                if op.pro_bn:
                    c.pro_bn_relu = 1
                    c.pro = self._bn(T, op.pro_bn, training, ar.ptr("s:" + op.pro_bn), M)
                c.dy, c.cs_dy, c.n = sar.ptr(st.gy), cs_out, spec.cout
                c.ws, c.kp, c.nz, c.nrep = wbase + 4 * ow, kp_f, sc["wg_nz"], sc["wg_nrep"]
                c.wsb = wbase + 4 * ob if ob is not None else None
                wg_bytes += esz * (M * cs_in + M * cs_out) + 4 * sc["wg_nz"] * spec.cout * spec.ks * spec.ks * cs_in
                wg_flops += 2.0 * M * spec.cout * spec.ks * spec.ks * spec.cin
        if FOLD_BN and training:
            self._fold_bn(ent, sar, esz * M)
        items = [(e[0], e[1], e[2], e[3], e[4], (e[5], e[6])) for e in ent if e[0] != "folded"]
        return items, groups, wg_bytes, wg_flops

    @staticmethod
    def _fold_bn(ent, sar, m_bytes):
        """Fold each BatchNorm-backward apply whose only data-gradient reader
        is the very next conv (a plain write: no accumulation, no residual)
        into that conv's operand staging (rnvp_conv_args.bp) where the library
        supports it (rnvp_conv2d_check).  The conv reads the apply's input
        temp and the BatchNorm input instead of the applied gradient, stores
        the applied gradient as a side output (the weight gradient reads it)
        and writes the BatchNorm's parameter gradients; its own pre-apply
        output moves to the other temp (gtmp / gtmp2) when it would overwrite
        the one it reads."""
        L = _lib.lib()
        other = {"gtmp": "gtmp2", "gtmp2": "gtmp"}
        for i in range(len(ent) - 1):
            e, d = ent[i], ent[i + 1]
            if e[0] != "bn" or d[0] != "dgrad" or e[7].accumulate or e[7].residual or d[7].gy != e[7].gx:
                continue
            if any(e[7].gx in ent[k][5] for k in range(i + 2, len(ent))):
                continue    # more data-gradient readers (the skip convs of d out): they stay grouped
            b, c = e[1], d[1]
            tin = e[8]
            assert b.g == sar.ptr(tin)
            retarget = d[8] is not None and d[8] == tin
            if retarget:
                nxt = ent[i + 2]
                assert nxt[0] == "bn" and nxt[7].op is d[7].op and nxt[8] == tin
            old_x, old_y = c.x, c.y
            c.bp, c.bp_x, c.bp_bn, c.bp_sums, c.bp_shards = 1, b.x, b.bn, b.sums, b.sum_shards
            c.bp_out, c.x = old_x, b.g
            if retarget:
                c.y = sar.ptr(other[tin])
            if L.conv2d_check(C.byref(c)) != 0:
                c.bp, c.bp_x, c.bp_sums, c.bp_out, c.x, c.y = 0, None, None, None, old_x, old_y
                continue
            if retarget:
                tn = other[tin]
                nxt[1].g = sar.ptr(tn)
                nxt[5] = (nxt[5] - {tin}) | {tn}
                nxt[8] = tn
                d[6] = (d[6] - {tin}) | {tn}
                d[8] = tn
            d[4] = e[4]
            d[5] = (d[5] - {e[7].gx}) | {tin} | (e[5] - {tin})
            d[6] = d[6] | {e[7].gx}
            d[2] += 2 * m_bytes * c.cs_in
            e[0] = "folded"

    def backward(self, sv, gz, gl_full, gl_sample, grad_block, gx=None, side=None, after=None, zero_at_end=False,
                 defer=None, opt=None, reverse=False):
        """Returns dL/dx; parameter gradients are written into grad_block
        (flat fp32, zeroed by the caller; scale/shift grads accumulate).

        The data-gradient chain (dgrad -> BN apply per conv) runs first; the
        weight gradients of all the net's convs only need their (complete,
        never rewritten) output gradients and saved inputs, so they run as
        ONE grouped launch afterwards (partial slabs, no atomics), followed by
        the weight-norm backward that sums the slabs.

        defer: a list that receives the weight-gradient closure instead of
        running it (it must run before anything rewrites this coupling's
        scratch, i.e. before its next backward).

        zero_at_end: the backward sums are zero on entry (not re-zeroed here)
        and the weight-norm backward launch leaves the forward's batch sums
        zero for the next step too (persistent arenas).  Either way the
        shared backward scratch is left zero.

        opt: an AdamArgs over this coupling's block of the trainer's arenas:
        the weight-norm backward becomes the fused row-local parameter pass
        (rnvp_weight_norm_bwd_adam: dv/dg/dbias, Adam on every conv row, the
        new norms and the next step's packed images); "defer": only the
        weight gradients run here -- the caller runs the parameter pass over
        this coupling's slabs later (param_pass_info) and zeroes its sums.

        reverse: sv comes from reverse(..., saved=sv): the backward of the
        inverse pass (rnvp_coupling_reverse_bwd in place of the out part's
        backward; gl_full is the gradient of the returned log_diag_J)."""
        L = _lib.lib()
        x = sv["x"]
        B, H, W, dtype, training = sv["B"], sv["H"], sv["W"], sv["dtype"], sv["training"]
        s = stream_ptr()
        T = self._tensors()
        ws = self.weights(dtype)
        sc = self.scratch_checked(B, H, W, dtype, x.device)
        ar, sar = sv["arena"], sc["arena"]
        z0, z1 = sc["zero"]
        if not zero_at_end:
            sar.buf[z0:z1].zero_()
        gbase = grad_block.data_ptr()

        def gp(name):
            return gbase + 4 * self.layout[name][0]

        if gx is None:
            gx = torch.empty_like(x)
        a = self._coupling_args(T, x, B, H, W, dtype, training)
        a.in_sums = ar.ptr("in_sums")
        a.st = ar.ptr("st")
        a.u = ar.ptr("u")
        a.out_sums = ar.ptr("out_sums")
        a.gz = gz.data_ptr()
        a.gl_full = gl_full.data_ptr() if gl_full is not None else None
        a.gl_sample = gl_sample.data_ptr() if gl_sample is not None else None
        a.gx = gx.data_ptr()
        a.gst, a.cs_gst = sar.ptr("g:st"), chan_stride(self.P.buf_ch["st"])
        a.bwd_sums = sar.ptr("bwd_sums")
        a.g_scale, a.g_scale_shift = gp("scale"), gp("scale_shift")
        a.gscale_part = sar.ptr("gscale_part")
        n_el, esz = x.numel(), DTYPES[dtype][1]
        cs_st = chan_stride(self.P.buf_ch["st"])
        if reverse:
            # gz, x (, gl) read, gx written; st read, gst written
            _launch("coupling", (16 if gl_full is not None else 12) * n_el + esz * B * H * W * 2 * cs_st, 0.0,
                    L.coupling_reverse_bwd, C.byref(a), s)
        else:
            # (reduction: gz, u) + apply: gz, u, x read, gx written; st read, gst written
            _launch("coupling", 24 * n_el + esz * B * H * W * 2 * cs_st, 0.0, L.coupling_out_bwd, C.byref(a), s)

        self._net_backward(sv, sc, ws, T, training, gp, s)
        # in_bn backward closes the critical path (dL/dx of the coupling) ...
        a.gh0, a.cs_gh0 = sar.ptr("g:h0"), chan_stride(self.P.buf_ch["h0"])
        a.in_bwd_sums = sar.ptr("in_bwd_sums")
        a.g_in_gamma, a.g_in_beta = gp("in_bn.weight"), gp("in_bn.bias")
        _launch("coupling", 16 * n_el + 2 * esz * B * H * W * a.cs_gh0, 0.0, L.coupling_in_bwd, C.byref(a), s)

        # ... while the weight gradients only feed the optimizer
        self._issue_weight_grads(self._weight_grads(sv, sc, ws, zero_at_end, opt, after, gbase), defer, side)
        return gx

    @staticmethod
    def _issue_weight_grads(weight_grads, defer, side):
        if defer is not None:
            # the caller issues the weight gradients later (e.g. after the
            # previous coupling's link backward has read this one's sums)
            defer.append(weight_grads)
        elif side is None:
            weight_grads()
        else:
            ev = torch.cuda.Event()
            ev.record()
            side.wait_event(ev)
            with torch.cuda.stream(side):
                weight_grads()

    # ------------------------------------------------------------ coupling links
    def link_args(self, sv, x, grad_block=None, gx=None):
        """CouplingArgs of this coupling for the link kernels (rnvp_coupling_out_u,
        rnvp_coupling_link_fwd / _bwd) over the saved arena sv (the trainer's,
        persistent) and this shape's scratch: forward sums, backward sums and,
        with grad_block / gx, the gradient outputs."""
        B, H, W, dtype = sv["B"], sv["H"], sv["W"], sv["dtype"]
        T = self._tensors()
        ar = sv["arena"]
        sar = self.scratch_checked(B, H, W, dtype, x.device)["arena"]
        a = self._coupling_args(T, x, B, H, W, dtype, True)
        a.in_sums, a.h0, a.st = ar.ptr("in_sums"), ar.ptr("h0"), ar.ptr("st")
        a.cls_sums, a.prior_sums = ar.ptr("cls_sums"), ar.ptr("prior_sums")
        a.out_tab, a.in_tab = ar.ptr("out_tab"), ar.ptr("in_tab")
        a.gst, a.cs_gst = sar.ptr("g:st"), chan_stride(self.P.buf_ch["st"])
        a.gh0, a.cs_gh0 = sar.ptr("g:h0"), chan_stride(self.P.buf_ch["h0"])
        a.in_bwd_sums, a.in_bwd_ext = sar.ptr("in_bwd_sums"), sar.ptr("in_bwd_ext")
        a.outp_sums, a.gscale_part = sar.ptr("outp_sums"), sar.ptr("gscale_part")
        if grad_block is not None:
            gb = grad_block.data_ptr()
            gp = lambda n: gb + 4 * self.layout[n][0]  # noqa: E731
            a.g_scale, a.g_scale_shift = gp("scale"), gp("scale_shift")
            a.g_in_gamma, a.g_in_beta = gp("in_bn.weight"), gp("in_bn.bias")
        if gx is not None:
            a.gx = gx.data_ptr()
        return a

    def forward_link(self, x, sv, ldj_sample, link):
        """Training forward of this coupling inside the trainer's flow program:
        the s/t net (its input h0 and in_bn statistics were produced by the
        previous link, or rnvp_flow_in_fwd + rnvp_coupling_in_apply for the
        first coupling), then u's class sums and the link to the consumer
        (rnvp_coupling_link_fwd: z at the consumer's permuted address, its in_bn
        statistics / h0, the prior).  link: dict(type, args=LinkArgs, nxt=(engine,
        saved arena, input tensor) or None)."""
        L = _lib.lib()
        s = stream_ptr()
        dtype = sv["dtype"]
        ws = self.weights(dtype)
        T = self._tensors()
        B, H, W = sv["B"], sv["H"], sv["W"]
        self._net_forward(T, sv, ws, True, s)
        a = self.link_args(sv, x)
        a.nclass = link["nclass"]
        a.ldj_sample = ldj_sample.data_ptr()
        a.gl_sample = link["args"].g_lp
        if "bn_table" in sv:   # the net BNs' running-stat updates ride on the link launch
            a.net_running, a.n_net_running, a.net_running_cmax = sv["bn_table"].data_ptr(), sv["bn_n"], sv["bn_cmax"]
        n_el, esz = x.numel(), DTYPES[dtype][1]
        cs_st = chan_stride(self.P.buf_ch["st"])
        # x and st read (u's class sums)
        _launch("coupling", 4 * n_el + esz * B * H * W * cs_st, 0.0, L.coupling_out_u, C.byref(a), s)
        nb = 8 * n_el + esz * B * H * W * cs_st        # x, st read; z written
        if link["nxt"] is not None:
            neng, nsv, nx = link["nxt"]
            n = neng.link_args(nsv, nx)
            nb += esz * nsv["B"] * nsv["H"] * nsv["W"] * chan_stride(neng.P.buf_ch["h0"])   # n's h0 written
            _launch("coupling", nb, 0.0, L.coupling_link_fwd, C.byref(a), C.byref(n), C.byref(link["args"]), s)
        else:
            _launch("coupling", nb, 0.0, L.coupling_link_fwd, C.byref(a), None, C.byref(link["args"]), s)
        sv["x"] = x

    def backward_link(self, sv, link, grad_block, gx, gl_sample, first, defer, opt=None, after=None):
        """Training backward of this coupling inside the trainer's flow program
        (after the consumer's): the link backward (dL/dz from the consumer's
        direct gradient + its in_bn backward, or the prior; then this coupling's
        out part, rnvp_coupling_link_bwd), the net's data-gradient chain and the
        in part's reduction pass (+ its apply pass for the first coupling:
        dL/dx of the flow input).  gx receives this coupling's direct input
        gradient (the full dL/dx for the first).  The weight-gradient closure
        goes to `defer`: the caller runs it once the previous link's backward
        has read this coupling's sums (the weight-norm backward zeroes them)."""
        L = _lib.lib()
        x = sv["x"]
        B, H, W, dtype = sv["B"], sv["H"], sv["W"], sv["dtype"]
        s = stream_ptr()
        T = self._tensors()
        ws = self.weights(dtype)
        sc = self.scratch_checked(B, H, W, dtype, x.device)
        gbase = grad_block.data_ptr()

        def gp(name):
            return gbase + 4 * self.layout[name][0]

        a = self.link_args(sv, x, grad_block, gx)
        a.nclass = link["nclass"]
        a.gl_sample = gl_sample.data_ptr()
        n_el, esz = x.numel(), DTYPES[dtype][1]
        cs_st = chan_stride(self.P.buf_ch["st"])
        nb = 12 * n_el + 2 * esz * B * H * W * cs_st   # x, consumer's gx read, gx written; st read, gst written
        if link["nxt"] is not None:
            neng, nsv, nx, ngx, nblock = link["nxt"]
            n = neng.link_args(nsv, nx, nblock, ngx)
            nb += esz * nsv["B"] * nsv["H"] * nsv["W"] * chan_stride(neng.P.buf_ch["h0"])   # consumer's gh0 read
            _launch("coupling", nb, 0.0, L.coupling_link_bwd, C.byref(a), C.byref(n), C.byref(link["args"]), s)
        else:
            _launch("coupling", nb, 0.0, L.coupling_link_bwd, C.byref(a), None, C.byref(link["args"]), s)
        self._net_backward(sv, sc, ws, T, True, gp, s)
        if not first:
            a.gx = None     # the reduction pass only; the apply is part of the previous link's backward
        cs_h0 = chan_stride(self.P.buf_ch["h0"])
        _launch("coupling", (8 if first else 4) * n_el + (2 if first else 1) * esz * B * H * W * cs_h0, 0.0,
                L.coupling_in_bwd, C.byref(a), s)
        self._issue_weight_grads(self._weight_grads(sv, sc, ws, True, opt, after, gbase), defer, None)
