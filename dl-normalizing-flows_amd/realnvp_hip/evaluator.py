"""Validation loop of the training script (train.py:214-233) on the device.

Per batch the reference runs, in eval mode under no_grad:
    x, logdet = logit_transform(x); logll, weight_scale = model(x)
    logll = (logll + logdet).mean(); running_logll += logll.item()
and reports bits/dim = (-mean_logll + ln 256 * D) / (D ln 2) over the batches.

``FlowEvaluator`` holds persistent eval-mode buffers for one batch size (BN
running statistics, so every shape is fixed) and captures logit transform
(device Philox noise, a fresh counter per batch), the forward flow with
per-sample log-det accumulation, the N(0, 1) prior and the running sum into
one HIP graph; the host reads the sum once per pass instead of once per batch
(the reference's per-batch .item()).  The weight-norm refresh runs once per
pass (weights do not change inside a validation loop).
"""
import math

import torch

from . import _lib
from .engine import stream_ptr
from .trainer import weights_key, wn_forward, wn_table


class FlowEvaluator:
    def __init__(self, model, batch_size, dtype=None, constraint=0.9, seed=0, graph=True):
        self.model = model
        self.dev = next(model.parameters()).device
        if self.dev.type != "cuda":
            raise RuntimeError("FlowEvaluator needs the model on a HIP device")
        self.B = batch_size
        self.dtype = dtype or next(model.couplings()).compute_dtype
        self.constraint, self.seed = constraint, seed
        C, S = model.channels, model.image_size
        f32 = dict(device=self.dev, dtype=torch.float32)
        self.pix = torch.zeros(batch_size, C, S, S, **f32)
        self.xl = torch.empty_like(self.pix)
        self.logdet = torch.empty(batch_size, **f32)
        self.ldj = torch.zeros(batch_size, **f32)
        self.lp = torch.empty(batch_size, **f32)
        self.ll_sum = torch.zeros(1, dtype=torch.float64, device=self.dev)
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.n_batches = 0
        self._plan(f32)
        self.engines = list(dict.fromkeys(st[1].engine() for st in self.ops if st[0] == "coupling"))
        self.table = wn_table(self.engines, self.dtype, self.dev)
        self._wkey = weights_key(self.engines, self.dtype)
        self.graph = None
        self.use_graph = graph

    def _check_weights(self):
        """Rebuild the weight-norm table and drop the captured graph when the
        parameters moved since they were built (their packed-weight arenas
        were re-allocated): both hold raw arena pointers."""
        k = weights_key(self.engines, self.dtype)
        if k != self._wkey:
            self.table = wn_table(self.engines, self.dtype, self.dev)
            self._wkey = k
            self.graph = None

    def _plan(self, f32):
        """the op list of flow_realnvp.RealNVP.f (flow_realnvp.py:252-327) with
        persistent buffers and per-sample log-det accumulation"""
        m = self.model
        B = self.B
        ops = []
        cur = self.xl
        c, s = m.channels, m.image_size
        offs = []

        def coupling(mod, x):
            eng = mod.engine()
            sv = eng.alloc_saved(B, x.shape[2], x.shape[3], self.dtype, self.dev, False)
            z = torch.empty_like(x)
            ops.append(("coupling", mod, x, z, sv))
            return z

        for si in range(1, m.n_scales):
            ckbd, chan = m._scale_mods(si)
            for mod in ckbd:
                cur = coupling(mod, cur)
            sq = torch.empty(B, 4 * c, s // 2, s // 2, **f32)
            ops.append(("squeeze", cur, sq))
            cur = sq
            for mod in chan:
                cur = coupling(mod, cur)
            un = torch.empty(B, c, s, s, **f32)
            ops.append(("undo", cur, un))
            on = torch.empty(B, 2 * c, s // 2, s // 2, **f32)
            off = torch.empty_like(on)
            ops.append(("factor_out", un, on, off))
            offs.append(off)
            cur = on
            c, s = 2 * c, s // 2
        for mod in m._scale_mods(m.n_scales)[0]:
            cur = coupling(mod, cur)
        for off in reversed(offs):
            full = torch.empty(B, off.shape[1] // 2, off.shape[2] * 2, off.shape[3] * 2, **f32)
            ops.append(("restore", cur, off, full))
            cur = full
        self.z = cur
        self.ops = ops

    def _batch(self):
        L = _lib.lib()
        s = stream_ptr()
        B = self.B
        n = self.pix[0].numel()
        L.logit_fwd(self.pix.data_ptr(), None, self.seed, 0, self.counter.data_ptr(), float(self.constraint),
                    self.xl.data_ptr(), self.logdet.data_ptr(), B, n, s)
        self.ldj.zero_()
        for op in self.ops:
            k = op[0]
            if k == "coupling":
                _, mod, x, z, sv = op
                mod.engine().forward(x, False, self.dtype, False, saved=sv, prepare=False, ldj_sample=self.ldj,
                                     z_out=z)
            elif k == "squeeze":
                _, a, b = op
                L.squeeze(a.data_ptr(), b.data_ptr(), *a.shape, s)
            elif k == "undo":
                _, a, b = op
                L.undo_squeeze(a.data_ptr(), b.data_ptr(), *b.shape, s)
            elif k == "factor_out":
                _, a, on, off = op
                L.factor_out(a.data_ptr(), on.data_ptr(), off.data_ptr(), *a.shape, s)
            else:
                _, on, off, full = op
                L.restore(on.data_ptr(), off.data_ptr(), full.data_ptr(), *full.shape, s)
        L.prior_logprob(self.z.data_ptr(), self.ldj.data_ptr(), self.lp.data_ptr(), B, self.z[0].numel(), s)
        self.ll_sum += (self.lp + self.logdet).mean().double()
        L.step_increment(self.counter.data_ptr(), s)

    def _capture(self):
        snap = (self.ll_sum.clone(), self.counter.clone())
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self._batch()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self._batch()
        torch.cuda.synchronize()
        self.ll_sum.copy_(snap[0])
        self.counter.copy_(snap[1])

    def begin(self):
        """Start a validation pass: refresh the packed weights, zero the sum."""
        self._check_weights()
        if self.table is not None:
            wn_forward(self.table, self.dtype)
        self.ll_sum.zero_()
        self.n_batches = 0

    def add_batch(self, pix):
        """One validation batch of raw pixels in [0, 1] ([B, C, S, S])."""
        if tuple(pix.shape) != tuple(self.pix.shape):
            raise ValueError("FlowEvaluator batch is %s, got %s" % (tuple(self.pix.shape), tuple(pix.shape)))
        with torch.no_grad():
            self.pix.copy_(pix)
            if self.use_graph:
                if self.graph is None:
                    self._capture()
                self.graph.replay()
            else:
                self._batch()
        self.n_batches += 1

    def mean_logll(self):
        """running_logll / n_batches (one host read per pass)."""
        return float(self.ll_sum.item()) / max(self.n_batches, 1)

    def bits_per_dim(self, mean_ll=None):
        """train.py:230."""
        if mean_ll is None:
            mean_ll = self.mean_logll()
        D = self.model.image_size ** 2 * self.model.channels
        return (-mean_ll + math.log(256.0) * D) / (D * math.log(2.0))

    def evaluate(self, batches):
        """A full validation pass over an iterable of pixel batches (e.g.
        data.DeviceLoader(valid_set, B, dev, drop_last=True)); returns
        (mean log-likelihood, bits/dim)."""
        self.begin()
        for pix in batches:
            if isinstance(pix, (tuple, list)):
                pix = pix[0]
            self.add_batch(pix)
        ll = self.mean_logll()
        return ll, self.bits_per_dim(ll)
