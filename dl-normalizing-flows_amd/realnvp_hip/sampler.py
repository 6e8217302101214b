"""Graph-replayed generation: RealNVP.sample(n) followed by
logit_transform(reverse=True), as train.py:253-259 draws its 100 samples
(flow_realnvp.py:342-352 -> g, 196-249; utils.py:34-42).

Eval mode (BatchNorm running statistics), so every buffer has a fixed
shape: z, the factor-out halves, each coupling's saved activations and the
output are allocated once, the N(0,1) draw, the weight-norm refresh (two
launches for the whole model) and every inverse kernel are captured into one
HIP graph and replayed per call.
"""
import torch

from . import _lib
from .engine import stream_ptr
from .trainer import weights_key, wn_forward, wn_table


class FlowSampler:
    def __init__(self, model, n, dtype=None, logit_reverse=True, constraint=0.9, graph=True):
        if model.training:
            raise RuntimeError("FlowSampler samples in eval mode (train.py:253-259 runs after model.eval())")
        self.model = model
        self.dev = next(model.parameters()).device
        if self.dev.type != "cuda":
            raise RuntimeError("FlowSampler needs the model on a HIP device")
        self.n = n
        self.dtype = dtype or next(model.couplings()).compute_dtype
        self.logit_reverse, self.constraint = logit_reverse, constraint
        C, S = model.channels, model.image_size
        f32 = dict(device=self.dev, dtype=torch.float32)
        self.z = torch.empty(n, C, S, S, **f32)
        self.out = torch.empty(n, C, S, S, **f32)
        self._plan(f32)
        self.engines = list(dict.fromkeys(st[1].engine() for st in self.ops if st[0] == "coupling"))
        self.table = wn_table(self.engines, self.dtype, self.dev)
        self._wkey = weights_key(self.engines, self.dtype)
        self.graph = None
        self.use_graph = graph
        if graph:
            self._capture()

    def _check_weights(self):
        """Rebuild the weight-norm table (and the graph) when the parameters
        moved since capture: both hold raw packed-weight arena pointers, and
        the old arena has been freed (e.g. a FlowTrainer built after this
        sampler re-pointed the parameters into its flat arena)."""
        k = weights_key(self.engines, self.dtype)
        if k != self._wkey:
            self.table = wn_table(self.engines, self.dtype, self.dev)
            self._wkey = k
            self.graph = None
            if self.use_graph:
                self._capture()

    def _plan(self, f32):
        """the op list of flow_realnvp.RealNVP.g with persistent buffers"""
        m = self.model
        n = self.n
        ops = []
        shapes = []
        c, s = m.channels, m.image_size
        for _ in range(1, m.n_scales):
            shapes.append((c, s))
            c, s = 2 * c, s // 2
        x = self.z
        offs = []
        cc, ss = m.channels, m.image_size
        for _ in range(1, m.n_scales):        # factor_out x4 (flow_realnvp.py:197-200)
            on = torch.empty(n, 2 * cc, ss // 2, ss // 2, **f32)
            off = torch.empty_like(on)
            ops.append(("factor_out", x, on, off))
            offs.append(off)
            x = on
            cc, ss = 2 * cc, ss // 2

        def coupling(mod, x):
            eng = mod.engine()
            B, Cc, H, W = x.shape
            sv = eng.alloc_saved(B, H, W, self.dtype, self.dev, False)
            y = torch.empty_like(x)
            ops.append(("coupling", mod, x, y, sv))
            return y

        for mod in reversed(list(m._scale_mods(m.n_scales)[0])):
            x = coupling(mod, x)
        for si in reversed(range(1, m.n_scales)):
            ckbd, chan = m._scale_mods(si)
            c, s = shapes[si - 1]
            full = torch.empty(n, c, s, s, **f32)
            ops.append(("restore", x, offs[si - 1], full))
            sq = torch.empty(n, 4 * c, s // 2, s // 2, **f32)
            ops.append(("squeeze", full, sq))
            x = sq
            for mod in reversed(list(chan)):
                x = coupling(mod, x)
            un = torch.empty(n, c, s, s, **f32)
            ops.append(("undo", x, un))
            x = un
            for mod in reversed(list(ckbd)):
                x = coupling(mod, x)
        self.x = x
        self.ops = ops

    def _run(self, draw=True):
        L = _lib.lib()
        s = stream_ptr()
        if draw:
            self.z.normal_()      # prior N(0, 1) (flow_realnvp.py:342-352)
        if self.table is not None:
            wn_forward(self.table, self.dtype)
        for op in self.ops:
            k = op[0]
            if k == "coupling":
                _, mod, x, y, sv = op
                mod.engine().reverse(x, False, self.dtype, saved=sv, out=y, want_ldj=False, prepare=False)
            elif k == "factor_out":
                _, a, on, off = op
                L.factor_out(a.data_ptr(), on.data_ptr(), off.data_ptr(), *a.shape, s)
            elif k == "restore":
                _, on, off, full = op
                L.restore(on.data_ptr(), off.data_ptr(), full.data_ptr(), *full.shape, s)
            elif k == "squeeze":
                _, a, b = op
                L.squeeze(a.data_ptr(), b.data_ptr(), *a.shape, s)
            else:
                _, a, b = op
                L.undo_squeeze(a.data_ptr(), b.data_ptr(), *b.shape, s)
        if self.logit_reverse:
            L.logit_inv(self.x.data_ptr(), self.out.data_ptr(), float(self.constraint), self.x.numel(), s)
        else:
            self.out.copy_(self.x)

    def _capture(self):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self._run()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self._run()
        torch.cuda.synchronize()

    def sample(self, z=None):
        """n images in [0, 1] (or the flow's x when logit_reverse=False).
        z: an optional [n, C, H, W] latent to invert instead of a fresh draw
        (eager path; used by the parity test)."""
        self._check_weights()
        if z is not None:
            with torch.no_grad():
                self.z.copy_(z)
                self._run(draw=False)
            return self.out
        if self.graph is not None:
            self.graph.replay()
        else:
            self._run()
        return self.out
