"""Fused RealNVP NLL training step (train.py:176-200) on the MI355X.

One step = logit_transform of a uint8-valued pixel batch (device Philox
noise), RealNVP forward with per-sample log-det accumulation, N(0,1) prior,
loss = -mean(log_prob + logdet) + 5e-5 * weight_scale, explicit backward
through every coupling / permutation, and a fused Adam update (coupled L2
weight decay, train.py:134) over ONE flat fp32 parameter arena.

MI355X-specific structure:
  * parameters, gradients and both Adam moments are flat arenas; the
    drop-in modules' nn.Parameters are views into the parameter arena, so
    state_dict / load_state_dict / torch optimizers keep working;
  * every buffer is allocated once; the whole step is captured into a HIP
    graph and replayed (no per-kernel host cost);
  * data parallel: one process per GPU, batch slice per rank, gradient
    arena averaged over RCCL in ~25 MB buckets that are issued on a
    communication stream as soon as backward has finished them (the deep
    scales, 86 % of the parameters, finish first), overlapping the
    remaining backward; optionally reduced in bf16.  BatchNorm statistics
    stay per rank (= the reference's semantics for each 64-image shard).
  * optimizer state converts to / from torch.optim.Adam.state_dict() format
    (train.py:139-154, 249-250 checkpoints).
"""
import ctypes as C
import gc
import math

import numpy as np
import torch

from . import _lib
from .engine import _launch, stream_ptr


def wn_table(engines, dtype, dev):
    """One weight-norm descriptor table over the convs of several couplings
    (rnvp_weight_norm_fwd refreshes all their packed weight images in two
    launches: row norms, then both images on tiles).  None when there are no convs."""
    import ctypes as C
    from ._lib import WNDesc
    from .engine import wn_tiles
    descs = []
    row0 = tile0 = 0
    for eng in engines:
        for d in eng.weights(dtype)["descs"]:
            e = WNDesc()
            C.memmove(C.addressof(e), C.addressof(d), C.sizeof(WNDesc))
            e.row0, e.tile0 = row0, tile0
            row0 += e.cout
            tile0 += wn_tiles(e.cout, e.cin, e.ks)
            descs.append(e)
    if not descs:
        return None
    tab = (WNDesc * len(descs))(*descs)
    from .engine import upload
    t = upload(bytes(tab), dev)
    return (t, len(descs), row0, tile0)


def weights_key(engines, dtype):
    """Identity of the packed-weight arenas of these couplings: changes when
    a coupling's parameter storage moved (e.g. a FlowTrainer re-pointed the
    parameters into its flat arena), which makes CouplingEngine.weights()
    rebuild -- and free -- the arena a weight-norm table or a captured graph
    points into."""
    return tuple(e.weights(dtype)["key"] for e in engines)


def wn_forward(table, dtype):
    t, n, rows, tiles = table
    _lib.lib().weight_norm_fwd(t.data_ptr(), n, rows, tiles, 1 if dtype == "bf16" else 0, stream_ptr())


def arena_blocks(model):
    """(offset, numel) of each coupling's parameters in the flat arena
    (named_parameters() order), couplings in forward order."""
    offs = {}
    off = 0
    for n, p in model.named_parameters():
        offs[n] = off
        off += p.numel()
    names = {id(m): n for n, m in model.named_modules()}
    out = []
    for mod in model.couplings():
        pre = names[id(mod)] + "."
        first = next(n for n, _ in mod.named_parameters())
        out.append((offs[pre + first], sum(p.numel() for p in mod.parameters())))
    return out


def bucket_plan(model, bucket_elems, n_total):
    """The trainer's all-reduce buckets for this model (dist.bucket_schedule
    over the coupling blocks in backward order)."""
    from .dist import bucket_schedule
    return bucket_schedule(list(reversed(arena_blocks(model))), bucket_elems, n_total)


class FlowTrainer:
    def __init__(self, model, batch_size, lr=5e-4, weight_decay=5e-5, betas=(0.9, 0.999), eps=1e-8,
                 scale_reg=5e-5, dtype="bf16", seed=0, process_group=None, bucket_mb=25, overlap=False,
                 comm="overlap", reduce_dtype="fp32", param_pass=None, chain=True):
        self.model = model
        self.dev = next(model.parameters()).device
        if self.dev.type != "cuda":
            raise RuntimeError("FlowTrainer needs the model on a HIP device")
        self.B = batch_size
        self.lr, self.wd, self.betas, self.eps, self.reg = lr, weight_decay, betas, eps, scale_reg
        self.dtype = dtype
        self.seed = seed
        self.pg = process_group
        self.rank = 0
        if process_group is not None:
            import torch.distributed as dist
            self.rank = dist.get_rank(process_group)
        model.set_precision(dtype)
        model.train()
        self._build_arenas()
        self._build_plan(chain)
        self.graph = None
        self.graph_opt = None
        self.graph_input = None
        self.external_input = False
        self.bucket_elems = max(1, int(bucket_mb * 2 ** 20 // 4))
        if comm not in ("overlap", "split"):
            raise ValueError("comm must be 'overlap' or 'split'")
        if reduce_dtype not in ("fp32", "bf16"):
            raise ValueError("reduce_dtype must be 'fp32' or 'bf16'")
        self.comm, self.reduce_dtype = comm, reduce_dtype
        self._reduce_pg = None
        self._comm_off = False
        self.comm_events = None
        self.comm_stream = None
        if self.pg is not None and comm == "overlap":
            self.comm_stream = torch.cuda.Stream(device=self.dev)
        # side stream: weight gradients, weight-norm of the late couplings and
        # (single process) the per-coupling optimizer update run beside the
        # critical path (the forward/data-gradient chain)
        self.overlap = overlap
        self.side = torch.cuda.Stream(device=self.dev) if overlap else None
        if param_pass not in (None, "fused", "separate"):
            raise ValueError("param_pass must be None (fused when possible), 'fused' or 'separate'")
        self._build_param_pass("separate" if param_pass == "separate" else "fused")
        if param_pass == "fused" and not self.fused:
            raise ValueError("param_pass='fused' is not possible for this model: %s" % self.param_pass_reason)
        self._build_adam_ranges()
        self._build_buckets()
        self._cap_pg = self._capture_group()

    # ----------------------------------------------------------------- arenas
    def _build_arenas(self):
        named = list(self.model.named_parameters())
        n = sum(p.numel() for _, p in named)
        n_pad = (n + 3) // 4 * 4
        dev = self.dev
        self.n = n_pad
        self.param = torch.zeros(n_pad, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(n_pad, device=dev, dtype=torch.float32)
        self.exp_avg = torch.zeros(n_pad, device=dev, dtype=torch.float32)
        self.exp_avg_sq = torch.zeros(n_pad, device=dev, dtype=torch.float32)
        mask = np.zeros(n_pad, dtype=np.uint8)
        self.offsets = {}
        off = 0
        with torch.no_grad():
            for name, p in named:
                k = p.numel()
                self.param[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.param[off:off + k].view_as(p)
                if p.requires_grad:
                    mask[off:off + k] = 2 if name.split(".")[-1] in ("weight_g", "scale") else 1
                self.offsets[name] = off
                off += k
        self.mask = torch.from_numpy(mask).to(dev)
        self.step_t = torch.zeros(1, device=dev, dtype=torch.int64)
        self.n_trainable = int((mask > 0).sum())

    # ------------------------------------------------------------------- plan
    def _build_plan(self, chain=True):
        m = self.model
        B, C, S = self.B, m.channels, m.image_size
        dev = self.dev
        f32 = dict(device=dev, dtype=torch.float32)
        self.pix = torch.zeros(B, C, S, S, **f32)
        self.xl = torch.empty(B, C, S, S, **f32)
        self.logdet = torch.zeros(B, **f32)
        self.ldj = torch.zeros(B, **f32)
        self.prior = torch.zeros(B, dtype=torch.float64, device=dev)
        self.lp = torch.empty(B, **f32)
        self.g_lp = torch.full((B,), -1.0 / B, **f32)
        self.ll_acc = torch.zeros(1, dtype=torch.float64, device=dev)
        self.stages = []   # forward program: ("coupling", mod, eng, in, out, sv, block) | perm ops
        cur = self.xl
        c, s = C, S
        offs = []
        for si in range(1, m.n_scales):
            ckbd, chan = m._scale_mods(si)
            for mod in ckbd:
                cur = self._add_coupling(mod, cur)
            sq = torch.empty(B, 4 * c, s // 2, s // 2, **f32)
            self.stages.append(("squeeze", cur, sq))
            cur = sq
            for mod in chan:
                cur = self._add_coupling(mod, cur)
            un = torch.empty(B, c, s, s, **f32)
            self.stages.append(("undo", cur, un))
            on = torch.empty(B, 2 * c, s // 2, s // 2, **f32)
            off = torch.empty_like(on)
            self.stages.append(("factor_out", un, on, off))
            offs.append(off)
            cur = on
            c, s = 2 * c, s // 2
        for mod in m._scale_mods(m.n_scales)[0]:
            cur = self._add_coupling(mod, cur)
        for off in reversed(offs):
            full = torch.empty(B, off.shape[1] // 2, off.shape[2] * 2, off.shape[3] * 2, **f32)
            self.stages.append(("restore", cur, off, full))
            cur = full
        self.z = cur
        # backward buffers: a gradient buffer per forward tensor
        self.gbuf = {}
        self._build_links(chain)
        self._build_wn_table()

    def _build_links(self, chain):
        """The flow program as coupling links (rnvp_coupling_link_fwd / _bwd,
        include/realnvp_hip.h): what sits between coupling k and the next one
        in the stage list -- nothing (the next coupling of the same combo),
        a squeeze, undo_squeeze + factor_out (the next scale), or the end of
        the flow (restores only).  The permutations then live in the links'
        addressing and the next coupling's in part in the previous coupling's
        link launch.  chain=False (or a model whose couplings do not link,
        e.g. without out_bn) keeps every coupling's in / out parts, the
        permutation kernels and the prior as separate launches."""
        from ._lib import LinkArgs, RNVP_LINK_FINAL, RNVP_LINK_SAME, RNVP_LINK_SQUEEZE, RNVP_LINK_UNFACTOR
        self.cidx = [i for i, st in enumerate(self.stages) if st[0] == "coupling"]
        self.links = None
        if not chain:
            return
        types = []
        for k, i in enumerate(self.cidx):
            j = self.cidx[k + 1] if k + 1 < len(self.cidx) else len(self.stages)
            between = [self.stages[m][0] for m in range(i + 1, j)]
            a = self.stages[i][2]
            if not a.hp.coupling_bn:
                return
            if k + 1 == len(self.cidx):
                if any(b != "restore" for b in between):
                    return
                types.append(RNVP_LINK_FINAL)
                continue
            n = self.stages[j][2]
            if between == [] and a.chains_into(n):
                types.append(RNVP_LINK_SAME)
            elif between == ["squeeze"] and a.kind == 0 and n.kind == 1:
                types.append(RNVP_LINK_SQUEEZE)
            elif between == ["undo", "factor_out"] and a.kind == 1 and n.kind == 0:
                types.append(RNVP_LINK_UNFACTOR)
            else:
                return
        self.links = types
        self.link_fwd, self.link_bwd = [], []
        for k, (i, lt) in enumerate(zip(self.cidx, types)):
            _, mod, eng, x, z, sv, block = self.stages[i]
            la = LinkArgs(lt, self.g_lp.data_ptr(), self.prior.data_ptr(), None, None)
            nc = int(_lib.lib().link_nclass(lt, eng.kind))
            if lt == RNVP_LINK_FINAL:
                nf = nb = None
            else:
                _, _, neng, nx, _, nsv, nblock = self.stages[self.cidx[k + 1]]
                nf = (neng, nsv, nx)
                nb = (neng, nsv, nx, self._g(nx), nblock)
            self.link_fwd.append(dict(nclass=nc, args=la, nxt=nf))
            self.link_bwd.append(dict(nclass=nc, args=la, nxt=nb))

    def _build_wn_table(self):
        """Weight-norm descriptor tables over the model's convs: the packed
        bf16/fp32 weight images are refreshed by two forward weight-norm calls
        per step (2 launches each) instead of one per coupling.  The first
        table covers the early couplings (few parameters, needed at once), the
        second the late, deep couplings (most of the parameters), which the
        side stream prepares while the early couplings run."""
        engines = [st[2] for st in self.stages if st[0] == "coupling"]
        self.wn_split = min(len(engines), max(1, len(engines) * 3 // 7))
        self.wn_tables = [t for t in (wn_table(engines[:self.wn_split], self.dtype, self.dev),
                                      wn_table(engines[self.wn_split:], self.dtype, self.dev)) if t is not None]

    def _wn_fwd(self, table):
        wn_forward(table, self.dtype)

    # ------------------------------------------------------- parameter pass
    def _build_param_pass(self, mode):
        """The fused row-local parameter pass (rnvp_weight_norm_bwd_adam).

        Single process: each coupling's weight-norm backward launch also runs
        Adam on its conv rows (v, g, bias) and writes the new norms and both
        packed weight images, so the step has no separate Adam pass over the
        convs and no weight-norm forward (the images the forward reads were
        written by the previous step).  Data parallel: the per-coupling
        weight-norm backward stays (the all-reduce comes between it and Adam)
        and ONE model-wide launch does Adam + norms + images after the
        all-reduce.  The arena elements outside the convs (BatchNorm affines,
        coupling scales: 0.3 % of config 1's parameters) get a gather-Adam.
        The images are re-derived eagerly (two weight-norm launches) when the
        parameters changed outside the trainer's own kernels (_packed_token).
        mode 'separate' keeps weight_norm_fwd + weight_norm_bwd + adam_step."""
        self.fused = False
        self._packed_token = None
        self.param_pass_mode, self.param_pass_reason = "separate", "requested"
        if mode != "fused":
            return
        from ._lib import Range, WNDesc
        import ctypes as C
        mask = self.mask.cpu().numpy()
        covered = np.zeros(self.n, dtype=bool)
        base = self.grad.data_ptr()
        model_descs, blk0 = [], 0
        slab_descs, ranges = [], []

        def rebased(d, off, b0):
            e = WNDesc()
            C.memmove(C.addressof(e), C.addressof(d), C.sizeof(WNDesc))
            e.dv_off += off
            e.dg_off = e.dg_off + off if e.dg_off >= 0 else -1
            e.db_off = e.db_off + off if e.db_off >= 0 else -1
            e.blk0 += b0
            return e
        for st in self.stages:
            if st[0] != "coupling":
                continue
            eng, sv, block = st[2], st[5], st[6]
            off = (block.data_ptr() - base) // 4
            ws = eng.weights(self.dtype)
            if ws["blocks"] < 0:
                self.param_pass_reason = "a conv row of %s does not fit the fused pass's LDS" % self._module_name(
                    st[1])
                return
            if self.pg is None:
                # single process: every coupling's pass is deferred to ONE launch
                # at the end of the backward over the couplings' (persistent)
                # weight-gradient slabs
                sdescs, rg = eng.param_pass_info(sv, self.dtype)
                slab_descs += [rebased(d, off, blk0) for d in sdescs]
                ranges += rg
            for d in ws["descs"]:
                kr = d.cin * d.ks * d.ks
                a = off + d.dv_off
                if not (mask[a:a + d.cout * kr] == 1).all():
                    self.param_pass_reason = "a conv of %s has frozen or regularised weight_v" % self._module_name(
                        st[1])
                    return
                covered[a:a + d.cout * kr] = True
                if d.g and d.dg_off >= 0:
                    covered[off + d.dg_off:off + d.dg_off + d.cout] = True
                if d.db_off >= 0:
                    covered[off + d.db_off:off + d.db_off + d.cout] = True
                model_descs.append(rebased(d, off, blk0))
            blk0 += ws["blocks"]
        from .engine import upload
        self._opt_table = (upload(bytes((WNDesc * len(model_descs))(*model_descs)), self.dev), len(model_descs),
                           blk0)
        # algorithmic bytes of the parameter pass (bench.py kernel families):
        # dW replicas + v twice + m + v^2 read, grad + v + m + v^2 + wf written
        esz = 2 if self.dtype == "bf16" else 4
        n_w = sum(d.cout * d.cin * d.ks * d.ks for d in model_descs)
        nrep = sum(d.cout * d.cin * d.ks * d.ks * max(d.nz, 1) for d in slab_descs) if slab_descs else 0
        # the transposes also write the fragment-major copies (engine.weights: bf16 3x3 convs)
        n_frag = sum(d.cout * d.cin * d.ks * d.ks * (int(bool(d.wf_frag)) + int(bool(d.wd_frag))) for d in model_descs)
        self._param_bytes = (4 * (nrep if slab_descs else n_w) + 32 * n_w + esz * n_w, 2 * esz * n_w + esz * n_frag)
        self._slab_table = None
        if slab_descs:
            self._slab_table = (upload(bytes((WNDesc * len(slab_descs))(*slab_descs)), self.dev), len(slab_descs),
                                blk0)
            rt = (Range * len(ranges))(*[Range(p, b) for p, b in ranges])
            self._zero_table = (upload(bytes(rt), self.dev), len(ranges), max(b for _, b in ranges))
        rest = np.nonzero((mask > 0) & ~covered)[0].astype(np.int64)
        self._opt_rest = torch.from_numpy(rest).to(self.dev)
        self._opt_all = self._adam_args(0)
        self._vparams = [p for _, p in self.model.named_parameters()]
        self.fused = True
        self.param_pass_mode, self.param_pass_reason = "fused", None

    def _adam_args(self, off):
        from ._lib import AdamArgs
        a = AdamArgs()
        a.param, a.grad = self.param.data_ptr() + 4 * off, self.grad.data_ptr() + 4 * off
        a.exp_avg, a.exp_avg_sq = self.exp_avg.data_ptr() + 4 * off, self.exp_avg_sq.data_ptr() + 4 * off
        a.mask, a.step, a.step_add = self.mask.data_ptr() + off, self.step_t.data_ptr(), 1
        a.lr, a.beta1, a.beta2, a.eps = self.lr, self.betas[0], self.betas[1], self.eps
        a.weight_decay, a.reg_coef = self.wd, self.reg
        return a

    def _refresh_adam_args(self):
        """lr / betas / eps / weight decay changed (load_optimizer_state_dict)"""
        if not self.fused:
            return
        for a in (self._opt_all,):
            a.lr, a.beta1, a.beta2, a.eps = self.lr, self.betas[0], self.betas[1], self.eps
            a.weight_decay, a.reg_coef = self.wd, self.reg

    def _token(self):
        return (self.param._version, sum(p._version for p in self._vparams))

    def invalidate_packed(self):
        """Declare the parameters changed outside the trainer: the next step
        re-derives the packed weight images (fused parameter pass).  Writes
        through the parameters themselves (p.mul_, load_state_dict, ...) are
        seen on their own; writes through `p.data` (e.g. nn.init on
        `.data`, the reference's utils.py:103-113 style) or through the
        arena tensor's storage by other means are NOT -- call this after them."""
        self._packed_token = None

    def _ensure_packed(self):
        """Fused pass: the packed weight images and norms are the previous
        step's output; re-derive them (eagerly) when the parameters were
        changed by anything else (first step, capture's restore,
        load_state_dict, a caller writing the parameters: their version
        counters move; writes through `.data` need invalidate_packed())."""
        if not self.fused:
            return
        tok = self._token()
        if tok != self._packed_token:
            for t in self.wn_tables:
                self._wn_fwd(t)
            self._packed_token = tok

    def _build_adam_ranges(self):
        """Per-coupling optimizer ranges [ru4(off_i), ru4(off_next)) of the flat
        arena (float4 granules).  A granule straddling two couplings belongs to
        the range of the coupling at the LOWER offset, whose update runs after
        the other's in backward order -- so every gradient in a range is final
        when its update runs.  Disabled (one update at the end) unless the
        backward visits couplings in descending arena offset."""
        self.adam_ranges = None
        if self.pg is not None or not self.overlap or self.fused or self.links is not None:
            return
        blocks = [st[6] for st in self.stages if st[0] == "coupling"]
        base = self.grad.data_ptr()
        offs = [(b.data_ptr() - base) // 4 for b in blocks]
        if offs != sorted(offs) or offs[0] != 0:
            return
        ru = lambda v: (v + 3) // 4 * 4  # noqa: E731
        ends = offs[1:] + [self.n]
        self.adam_ranges = [(ru(o), (ru(e) if e < self.n else self.n)) for o, e in zip(offs, ends)]

    def _build_buckets(self):
        """All-reduce buckets in backward order (dist.bucket_schedule over the
        couplings' gradient blocks); bucket k is issued right after coupling
        bucket_after[k]'s backward has been scheduled."""
        blocks = [st[6] for st in self.stages if st[0] == "coupling"]
        base = self.grad.data_ptr()
        spans = [((b.data_ptr() - base) // 4, b.numel()) for b in blocks]
        if spans != arena_blocks(self.model):
            raise RuntimeError("coupling gradient blocks do not follow the parameter arena")
        self.buckets = bucket_plan(self.model, self.bucket_elems, self.n)
        self.bucket_after = {}
        for lo, hi, k in self.buckets:
            self.bucket_after.setdefault(k, []).append((lo, hi))
        self.reduce_buf = None
        if self.pg is not None and self.reduce_dtype == "bf16":
            self.reduce_buf = torch.empty(self.n, device=self.dev, dtype=torch.bfloat16)

    def _reduce_bucket(self, lo, hi):
        """Average grad[lo:hi) over the process group (on the current stream).
        No-op during capture()'s warm-up steps (see capture)."""
        if self._comm_off:
            return
        from .dist import average_slice
        pg = self._reduce_pg if self._reduce_pg is not None else self.pg
        average_slice(self.grad, lo, hi, pg, self.reduce_buf)

    def _capture_group(self):
        """The process group the captured step all-reduces over.

        RCCL's process group hands every eager collective to a watchdog
        thread that polls the collective's completion event on the group's
        communication stream until it retires it.  Inside a capture that
        stream joins the graph, and an event poll on a capturing stream is a
        fatal HIP error (it aborted the world-1 test twice in round 2, when a
        warm-up all-reduce was still on the watchdog's list).  So the capture
        uses a second group over the same ranks, created at construction
        (every rank of the trainer's group constructs its trainer; local
        synchronisation, so a process_group that is a subgroup of a larger
        world does not need the ranks outside it), connected eagerly (no
        collective) and used ONLY inside captures: its watchdog list is empty
        by construction, and the warm-up group's stream never captures.
        Collectives issued while capturing are not handed to any watchdog.
        gloo (CPU tests) needs no second group."""
        if self.pg is None or self.comm_stream is None:
            return None
        import torch.distributed as dist
        if dist.get_backend(self.pg) != "nccl":
            return self.pg
        ranks = dist.get_process_group_ranks(self.pg)
        g = dist.new_group(ranks=ranks, backend="nccl", use_local_synchronization=True)
        g._get_backend(self.dev).eager_connect_single_device(self.dev)
        return g

    def _add_coupling(self, mod, x):
        eng = mod.engine()
        B, C, H, W = x.shape
        sv = eng.alloc_saved(B, H, W, self.dtype, self.dev, True)
        z = torch.empty_like(x)
        first = next(n for n, _ in mod.named_parameters())
        name = self._module_name(mod) + "." + first
        block = self.grad[self.offsets[name]:self.offsets[name] + eng.n_params]
        self.stages.append(("coupling", mod, eng, x, z, sv, block))
        return z

    def _module_name(self, mod):
        if not hasattr(self, "_names"):
            self._names = {id(m): n for n, m in self.model.named_modules()}
        return self._names[id(mod)]

    def _g(self, t):
        """gradient buffer shaped like forward tensor t"""
        k = t.data_ptr()
        g = self.gbuf.get(k)
        if g is None:
            g = torch.empty_like(t)
            self.gbuf[k] = g
        return g

    # ------------------------------------------------------------------- step
    def _wn_prepare(self):
        """the packed weight images of this step (separate parameter pass:
        the weight-norm forward; fused: the previous step's, _ensure_packed)"""
        late_ready = None
        if self.fused:
            pass
        elif len(self.wn_tables) > 1 and self.side is not None:
            ev = torch.cuda.Event()
            ev.record()
            self.side.wait_event(ev)
            with torch.cuda.stream(self.side):
                self._wn_fwd(self.wn_tables[1])
                late_ready = torch.cuda.Event()
                late_ready.record()
            self._wn_fwd(self.wn_tables[0])
        else:
            for t in self.wn_tables:
                self._wn_fwd(t)
        return late_ready

    def _forward(self):
        if self.links is not None:
            return self._forward_links()
        L = _lib.lib()
        s = stream_ptr()
        B = self.B
        n = self.pix[0].numel()
        if not self.external_input:
            L.logit_fwd(self.pix.data_ptr(), None, self.seed, 0, self.step_t.data_ptr(), 0.9, self.xl.data_ptr(),
                        self.logdet.data_ptr(), B, n, s)
        self.ldj.zero_()
        late_ready = self._wn_prepare()
        ci = 0
        for i, st in enumerate(self.stages):
            if st[0] == "coupling":
                if ci == self.wn_split and late_ready is not None:
                    torch.cuda.current_stream().wait_event(late_ready)
                ci += 1
                _, mod, eng, x, z, sv, _ = st
                eng.forward(x, True, self.dtype, False, saved=sv, prepare=False, ldj_sample=self.ldj, z_out=z,
                            zero_sums=False)
            elif st[0] == "squeeze":
                _, a, b = st
                L.squeeze(a.data_ptr(), b.data_ptr(), *a.shape, s)
            elif st[0] == "undo":
                _, a, b = st
                L.undo_squeeze(a.data_ptr(), b.data_ptr(), *b.shape, s)
            elif st[0] == "factor_out":
                _, a, on, off = st
                L.factor_out(a.data_ptr(), on.data_ptr(), off.data_ptr(), *a.shape, s)
            else:
                _, on, off, full = st
                L.restore(on.data_ptr(), off.data_ptr(), full.data_ptr(), *full.shape, s)
        L.prior_logprob(self.z.data_ptr(), self.ldj.data_ptr(), self.lp.data_ptr(), B, self.z[0].numel(), s)
        self.ll_acc += (self.lp + self.logdet).mean().double()

    def _forward_links(self):
        """The flow program over coupling links: the input pass (logit
        transform + the first coupling's in_bn sums), the first coupling's in
        part, then per coupling its net, u's class sums and the link, and the
        per-sample log-likelihood.  No permutation kernel, no prior pass:
        the prior of the factored-out halves and of the last scale is added
        by the links."""
        L = _lib.lib()
        s = stream_ptr()
        B = self.B
        _, _, eng0, x0, _, sv0, _ = self.stages[self.cidx[0]]
        a0 = eng0.link_args(sv0, x0)
        n_el, esz = x0.numel(), 2 if self.dtype == "bf16" else 4
        cs_h0 = a0.cs_h0
        if not self.external_input:
            _launch("logit", 8 * n_el, 0.0, L.flow_in_fwd, self.pix.data_ptr(), self.seed, self.step_t.data_ptr(),
                    0.9, self.xl.data_ptr(), self.logdet.data_ptr(), C.byref(a0), B, *x0.shape[1:], s)
            _launch("coupling", 4 * n_el + esz * x0[:, 0].numel() * cs_h0, 0.0, L.coupling_in_apply, C.byref(a0), s)
        else:
            _launch("coupling", 8 * n_el + esz * x0[:, 0].numel() * cs_h0, 0.0, L.coupling_in_fwd, C.byref(a0), s)
        late_ready = self._wn_prepare()
        for k, i in enumerate(self.cidx):
            if k == self.wn_split and late_ready is not None:
                torch.cuda.current_stream().wait_event(late_ready)
            _, mod, eng, x, z, sv, _ = self.stages[i]
            eng.forward_link(x, sv, self.ldj, self.link_fwd[k])
        L.flow_lp_finish(self.prior.data_ptr(), self.ldj.data_ptr(), self.logdet.data_ptr(),
                         0 if self.external_input else 1, self.lp.data_ptr(), self.ll_acc.data_ptr(), B, s)

    def _issue_buckets(self, ci, n_coupling):
        """the all-reduce buckets that coupling ci's gradients complete"""
        if self.comm_stream is None:
            return
        for lo, hi in self.bucket_after.get(n_coupling - 1 - ci, ()):
            # the bucket's weight gradients were written on the side
            # stream (overlap) or the current one
            ev = torch.cuda.Event()
            ev.record(self.side if self.side is not None else torch.cuda.current_stream())
            self.comm_stream.wait_event(ev)
            with torch.cuda.stream(self.comm_stream):
                if self.comm_events is not None:     # bench.py: per-bucket timing (eager)
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                self._reduce_bucket(lo, hi)
                if self.comm_events is not None:
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record()
                    self.comm_events.append((hi - lo, e0, e1))

    def _backward(self):
        if self.links is not None:
            return self._backward_links()
        L = _lib.lib()
        s = stream_ptr()
        B = self.B
        gz = self._g(self.z)
        L.prior_logprob_bwd(self.z.data_ptr(), self.g_lp.data_ptr(), gz.data_ptr(), B, self.z[0].numel(), s)
        n_coupling = len(self.cidx)
        ci = n_coupling
        for i in reversed(range(len(self.stages))):
            st = self.stages[i]
            if st[0] == "coupling":
                ci -= 1
                _, mod, eng, x, z, sv, block = st
                after = None
                if self.adam_ranges is not None:
                    lo, hi = self.adam_ranges[ci]
                    after = (lambda lo=lo, hi=hi: self._adam_range(lo, hi))
                opt = "defer" if (self.fused and self.pg is None) else None
                eng.backward(sv, self._g(z), None, self.g_lp, block, gx=self._g(x), side=self.side, after=after,
                             zero_at_end=True, opt=opt)
                self._issue_buckets(ci, n_coupling)
            elif st[0] == "squeeze":
                _, a, b = st
                L.undo_squeeze(self._g(b).data_ptr(), self._g(a).data_ptr(), *a.shape, s)
            elif st[0] == "undo":
                _, a, b = st
                L.squeeze(self._g(b).data_ptr(), self._g(a).data_ptr(), *b.shape, s)
            elif st[0] == "factor_out":
                _, a, on, off = st
                L.restore(self._g(on).data_ptr(), self._g(off).data_ptr(), self._g(a).data_ptr(), *a.shape, s)
            else:
                _, on, off, full = st
                L.factor_out(self._g(full).data_ptr(), self._g(on).data_ptr(), self._g(off).data_ptr(),
                             *full.shape, s)

    def _backward_links(self):
        """Backward over the coupling links, last coupling first: its link
        backward (dL/dz from the consumer or the prior, then its out part),
        its net's data gradients and its in part's reduction pass.  A
        coupling's weight gradients (and, outside the fused single-process
        pass, its weight-norm backward, which leaves its sums zero) run after
        the previous coupling's link backward has read those sums; its
        all-reduce buckets follow them."""
        n_coupling = len(self.cidx)
        opt = "defer" if (self.fused and self.pg is None) else None
        pending, pending_ci = [], None
        for k in reversed(range(n_coupling)):
            _, mod, eng, x, z, sv, block = self.stages[self.cidx[k]]
            mine = []
            eng.backward_link(sv, self.link_bwd[k], block, self._g(x), self.g_lp, k == 0, mine, opt=opt)
            self._run_pending(pending, pending_ci, n_coupling)
            pending, pending_ci = mine, k
        self._run_pending(pending, pending_ci, n_coupling)

    def _run_pending(self, pending, ci, n_coupling):
        if not pending:
            return
        if self.side is not None:
            self._flush_side(pending)
        else:
            for f in pending:
                f()
            pending.clear()
        self._issue_buckets(ci, n_coupling)

    def _flush_side(self, pending):
        """fork the deferred weight-gradient closures onto the side stream"""
        ev = torch.cuda.Event()
        ev.record()
        self.side.wait_event(ev)
        with torch.cuda.stream(self.side):
            for f in pending:
                f()
        pending.clear()

    def _adam_range(self, lo, hi):
        b1, b2 = self.betas
        if hi <= lo:
            return
        _lib.lib().adam_update(self.param.data_ptr() + 4 * lo, self.grad.data_ptr() + 4 * lo,
                               self.exp_avg.data_ptr() + 4 * lo, self.exp_avg_sq.data_ptr() + 4 * lo, hi - lo,
                               self.step_t.data_ptr(), 1, self.lr, b1, b2, self.eps, self.wd,
                               self.mask.data_ptr() + lo, self.reg, stream_ptr())

    def _optimizer(self):
        if self.fused:
            from .engine import _launch
            L = _lib.lib()
            s = stream_ptr()
            import ctypes as C
            dt = 1 if self.dtype == "bf16" else 0
            pb, tb = self._param_bytes
            if self.pg is not None:
                # data parallel: the conv rows' Adam + norms + images, after the all-reduce
                t, n, nblk = self._opt_table
                _launch("param", pb, 0.0, L.weight_norm_bwd_adam, t.data_ptr(), n, nblk, 0, dt,
                        C.byref(self._opt_all), None, 0, None, 0, s)
            else:
                # single process: every coupling's slabs -> dv / dg / dbias, Adam,
                # norms and forward images in ONE launch (small couplings' rows fill
                # the big ones' gaps), then their batch sums left zero
                t, n, nblk = self._slab_table
                _launch("param", pb, 0.0, L.weight_norm_bwd_adam, t.data_ptr(), n, nblk, 1, dt,
                        C.byref(self._opt_all), None, 0, None, 0, s)
                zt, nz, zb = self._zero_table
                L.zero_ranges(zt.data_ptr(), nz, zb, s)
            # the data-gradient images from the forward images the row kernels wrote
            for t, n, _, tiles in self.wn_tables:
                _launch("param", tb / len(self.wn_tables), 0.0, L.weight_norm_transpose, t.data_ptr(), n, tiles, dt,
                        s)
            L.adam_gather(C.byref(self._opt_all), self._opt_rest.data_ptr(), self._opt_rest.numel(), s)
            L.step_increment(self.step_t.data_ptr(), s)
            return
        if self.adam_ranges is not None:
            # the per-coupling updates already ran (side stream, t = step + 1)
            _lib.lib().step_increment(self.step_t.data_ptr(), stream_ptr())
            return
        b1, b2 = self.betas
        _lib.lib().adam_step(self.param.data_ptr(), self.grad.data_ptr(), self.exp_avg.data_ptr(),
                             self.exp_avg_sq.data_ptr(), self.n, self.step_t.data_ptr(), self.lr, b1, b2, self.eps,
                             self.wd, self.mask.data_ptr(), self.reg, stream_ptr())

    def _allreduce(self):
        """Whole-arena bucketed average ("split" mode: between the captured
        forward/backward graph and the optimizer graph)."""
        if self.pg is None or self.comm_stream is not None:
            return
        for lo, hi, _ in self.buckets:
            self._reduce_bucket(lo, hi)

    def _fwd_bwd(self):
        if self.fused:
            # every conv gradient (v, g, bias) is written, not accumulated, by
            # the row kernels and every BatchNorm affine gradient by its
            # backward apply: only the accumulated ones (coupling scale /
            # scale_shift, +=) need zeroing -- the 0.3 % outside the convs
            self.grad.index_fill_(0, self._opt_rest, 0.0)
        else:
            self.grad.zero_()
        self._forward()
        self._backward()
        if self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)
        if self.comm_stream is not None:
            torch.cuda.current_stream().wait_stream(self.comm_stream)

    def step_eager(self):
        self._ensure_packed()
        self._fwd_bwd()
        self._allreduce()
        self._optimizer()

    # --------------------------------------------------------------- graphs
    def _snapshot(self):
        bufs = {n: b.detach().clone() for n, b in self.model.named_buffers()}
        return (self.param.clone(), self.exp_avg.clone(), self.exp_avg_sq.clone(), self.step_t.clone(),
                self.ll_acc.clone(), bufs)

    def _restore(self, snap):
        p, m, v, t, ll, bufs = snap
        with torch.no_grad():
            self.param.copy_(p)
            self.exp_avg.copy_(m)
            self.exp_avg_sq.copy_(v)
            self.step_t.copy_(t)
            self.ll_acc.copy_(ll)
            for n, b in self.model.named_buffers():
                b.copy_(bufs[n])

    def capture(self, warmup=2, restore=True, before_capture=None):
        """Warm up eagerly on a side stream, then capture the step into HIP
        graphs.  The warm-up steps move the parameters, Adam moments, step
        counter (and with it the dequantisation noise) and BN running stats;
        with restore=True (default) all of that is put back afterwards, so
        the first replay is the caller's first training step.  The input mode
        (set_pixels: logit transform inside the graph, or set_input: an
        already transformed batch) is fixed at capture.

        Single process, and data parallel with comm="overlap": ONE graph
        holds forward, backward, the bucketed all-reduces on the
        communication stream and Adam.  comm="split": forward/backward graph,
        eager all-reduce, optimizer graph.

        Nothing but the captured step's own work runs while a capture is
        open (the round-4 abort: SIGABRT from a thread without a Python
        frame in the middle of a capture):
          * the warm-up steps issue no collective (their state is restored,
            so with a process group restore must be True);
          * the captured all-reduces use a capture-only group (_capture_group);
          * unreachable objects are collected and their HIP teardown drained
            before the capture, and the garbage collector is off during it,
            so no graph / event / stream of another object is destroyed
            mid-capture.
        tools/probe/capture_watchdog.py showed that a c10d watchdog polling a
        finished eager all-reduce during a thread-local capture does NOT
        abort on this stack, so a pending watchdog entry alone is not the
        cause; the construction above removes every other thread-visible
        event of the window."""
        if self.pg is not None and not restore:
            raise ValueError("with a process group, capture() must restore the warm-up state: its warm-up "
                             "steps issue no all-reduce (see capture)")
        snap = self._snapshot() if restore else None
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        # The warm-up steps issue NO collective: their state is discarded
        # (restore) and a collective issued here would sit on its group's
        # watchdog list when the capture opens (see _wait_collectives_retired)
        self._comm_off = True
        try:
            with torch.cuda.stream(side):
                for _ in range(warmup):
                    self.step_eager()
        finally:
            self._comm_off = False
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        # Destroy unreachable objects (earlier trainers' graphs, events,
        # streams) NOW and let the HIP work their destruction queues drain,
        # and run no garbage collection while the capture is open: a cyclic
        # collection triggered by any allocation inside the capture would
        # otherwise destroy HIP graphs / events / streams of other objects in
        # the middle of it (see capture's note on the round-4 abort)
        gc.collect()
        torch.cuda.synchronize()
        # the captured all-reduces go through a group of their own (see
        # _capture_group); eager collectives stay on self.pg
        if before_capture is not None:
            before_capture()
        self.graph = torch.cuda.CUDAGraph()
        self.graph_opt = None
        self.graph_input = self.external_input
        # thread-local capture: other threads' HIP calls are not checked
        # against our capture (HIP still refuses an event query meanwhile,
        # hence the drain above)
        mode = "thread_local"
        gc_on = gc.isenabled()
        gc.disable()
        try:
            if self.pg is None or self.comm_stream is not None:
                try:
                    self._reduce_pg = self._cap_pg
                    with torch.cuda.graph(self.graph, capture_error_mode=mode):
                        self._fwd_bwd()
                        self._optimizer()
                finally:
                    self._reduce_pg = None
            else:
                with torch.cuda.graph(self.graph, capture_error_mode=mode):
                    self._fwd_bwd()
                self.graph_opt = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph_opt, capture_error_mode=mode):
                    self._optimizer()
        finally:
            if gc_on:
                gc.enable()
        torch.cuda.synchronize()
        if snap is not None:
            self._restore(snap)
            torch.cuda.synchronize()
        return warmup

    def drop_graph(self):
        self.graph = self.graph_opt = self.graph_input = None

    def step(self):
        if self.graph is None:
            return self.step_eager()
        self._ensure_packed()
        self.graph.replay()
        if self.graph_opt is not None:
            self._allreduce()
            self.graph_opt.replay()

    def _check_mode(self, external):
        if self.graph is not None and self.graph_input != external:
            raise RuntimeError("the captured step reads %s; call drop_graph() (or capture again) before feeding "
                               "%s" % ("set_input() batches" if self.graph_input else "set_pixels() pixels",
                                       "set_input() batches" if external else "set_pixels() pixels"))

    def set_pixels(self, pix):
        """Raw pixels in [0, 1]; the step applies logit_transform on the device."""
        self._check_mode(False)
        if self.external_input:
            self.logdet.zero_()   # the input pass adds the log-det (rnvp_flow_in_fwd)
        self.external_input = False
        self.pix.copy_(pix)

    def set_input(self, x, logdet):
        """Feed an already logit-transformed batch (parity tests)."""
        self._check_mode(True)
        self.external_input = True
        self.xl.copy_(x)
        self.logdet.copy_(logdet)

    # ------------------------------------------------------- checkpointing
    def _param_list(self):
        return list(self.model.named_parameters())

    def optimizer_state_dict(self):
        """The fused Adam's state as torch.optim.Adam(model.parameters(),
        lr, betas, eps, weight_decay).state_dict() would hold it (the
        reference's realnvp_state_optim.pt, train.py:250): per trainable
        parameter index exp_avg / exp_avg_sq / step; frozen parameters (no
        gradient, skipped by torch's Adam) carry no state."""
        step = float(self.step_t.item())
        state = {}
        named = self._param_list()
        for i, (n, p) in enumerate(named):
            if not p.requires_grad or step == 0:
                continue
            off, k = self.offsets[n], p.numel()
            state[i] = {"step": torch.tensor(step),
                        "exp_avg": self.exp_avg[off:off + k].view_as(p).clone(),
                        "exp_avg_sq": self.exp_avg_sq[off:off + k].view_as(p).clone()}
        group = {"lr": self.lr, "betas": tuple(self.betas), "eps": self.eps, "weight_decay": self.wd,
                 "amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                 "differentiable": False, "fused": None, "decoupled_weight_decay": False,
                 "params": list(range(len(named)))}
        return {"state": state, "param_groups": [group]}

    def load_optimizer_state_dict(self, sd):
        """Inverse of optimizer_state_dict (accepts what torch.optim.Adam
        saved for model.parameters(); train.py:149-154)."""
        named = self._param_list()
        groups = sd["param_groups"]
        idx = [i for g in groups for i in g["params"]]
        if len(idx) != len(named):
            raise ValueError("optimizer state has %d parameters, the model %d" % (len(idx), len(named)))
        g0 = groups[0]
        if g0.get("amsgrad") or g0.get("maximize") or g0.get("decoupled_weight_decay"):
            raise ValueError("only plain Adam with coupled weight decay is supported (train.py:134)")
        steps = set()
        with torch.no_grad():
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            for pos, (n, p) in zip(idx, named):
                st = sd["state"].get(pos)
                if st is None:
                    continue
                off, k = self.offsets[n], p.numel()
                self.exp_avg[off:off + k].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(float(st["step"]))
        if len(steps) > 1:
            raise ValueError("per-parameter Adam step counts differ: %s" % sorted(steps))
        self.step_t.fill_(int(steps.pop()) if steps else 0)
        self.lr, self.betas, self.eps, self.wd = g0["lr"], tuple(g0["betas"]), g0["eps"], g0["weight_decay"]
        self._refresh_adam_args()
        if self.graph is not None:
            self.drop_graph()    # lr / betas are baked into the captured launches

    def rng_state(self):
        """The dequantisation noise stream: k_logit_fwd draws step t's noise
        from Philox(seed, counter = t), so (seed, t) is the whole RNG state
        (the reference saves none, train.py:249-250).  The
        saving rank is recorded: data-parallel ranks draw from seeds of their
        own."""
        return {"seed": int(self.seed), "rank": int(self.rank), "step": int(self.step_t.item())}

    def state_dict(self):
        """{'model': model.state_dict(), 'optimizer': torch-Adam-format state,
        'rng': rng_state()} (the two files train.py:249-250 writes, plus the
        noise stream so a resumed run draws the same noise as an unbroken one)."""
        return {"model": self.model.state_dict(), "optimizer": self.optimizer_state_dict(),
                "rng": self.rng_state()}

    def load_state_dict(self, sd):
        with torch.no_grad():
            self.model.load_state_dict(sd["model"])
        self.load_optimizer_state_dict(sd["optimizer"])
        rng = sd.get("rng")
        if rng is not None:
            # a checkpoint of THIS rank resumes its noise stream exactly; one
            # saved by another rank (usually rank 0 for all) restores only the
            # step counter, so every replica keeps drawing its own noise
            own = int(rng.get("rank", 0)) == self.rank
            if own and int(rng["seed"]) != self.seed:
                self.seed = int(rng["seed"])
                self.drop_graph()    # the seed is a captured launch argument
            self.step_t.fill_(int(rng["step"]))

    def reset_optimizer(self):
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()
        self.step_t.zero_()

    def reset_metrics(self):
        self.ll_acc.zero_()

    def mean_logll(self, steps):
        return float(self.ll_acc.item()) / max(steps, 1)

    def bits_per_dim(self, mean_ll):
        """train.py:203-204."""
        D = self.model.image_size ** 2 * self.model.channels
        return (-mean_ll + math.log(256.0) * D) / (D * math.log(2.0))
