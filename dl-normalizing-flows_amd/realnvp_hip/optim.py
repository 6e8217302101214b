"""A fused Adam for the reference's own training loop (train.py:134, 198-200).

    optimizer = realnvp_hip.FusedAdam(model.parameters(), lr=5e-4, weight_decay=5e-5)

is a drop-in for torch.optim.Adam(model.parameters(), lr, weight_decay=...)
in train.py: same update (coupled L2 weight decay, bias corrections, eps
outside the square root), same state_dict format (the reference's
realnvp_state_optim.pt, train.py:139-154, 249-250), zero_grad / param_groups as
torch's.  The parameters are moved once into ONE flat fp32 arena (their
.data become views of it, so the model, its state_dict and the engine's
packed-weight caches keep working), with Adam's two moments beside it; a step
is one gather of the gradients into a flat gradient arena
(torch._foreach_copy_) and one HIP launch over the whole arena
(rnvp_adam_step), instead of torch's foreach Adam over the model's 1,960
parameter tensors (~12.8 ms per step at config 1, tools/probe/adam_probe.py).
Parameters whose .grad is None are left untouched, as torch does (that step
falls back to the per-tensor update for the others).
"""
import math

import torch

from . import _lib
from .engine import stream_ptr


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False):
        if amsgrad:
            raise ValueError("FusedAdam implements plain Adam (train.py:134 uses amsgrad=False)")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None,
                        decoupled_weight_decay=False)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("FusedAdam takes one parameter group (the reference's optimizer has one)")
        ps = self.param_groups[0]["params"]
        if not ps:
            raise ValueError("FusedAdam got an empty parameter list")
        dev = ps[0].device
        if dev.type != "cuda" or any(p.device != dev or p.dtype != torch.float32 for p in ps):
            raise RuntimeError("FusedAdam needs float32 parameters on one HIP device")
        n = sum(p.numel() for p in ps)
        self.n = (n + 3) // 4 * 4
        self.param = torch.zeros(self.n, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(self.n, device=dev, dtype=torch.float32)
        self.exp_avg = torch.zeros(self.n, device=dev, dtype=torch.float32)
        self.exp_avg_sq = torch.zeros(self.n, device=dev, dtype=torch.float32)
        mask = torch.zeros(self.n, dtype=torch.uint8)
        self.offsets = []
        off = 0
        with torch.no_grad():
            for p in ps:
                k = p.numel()
                self.param[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.param[off:off + k].view_as(p)
                if p.requires_grad:
                    mask[off:off + k] = 1
                self.offsets.append(off)
                off += k
        self.mask = mask.to(dev)
        self.step_t = torch.zeros(1, device=dev, dtype=torch.int64)
        self._train = [i for i, p in enumerate(ps) if p.requires_grad]
        self._gdst = [self.grad[self.offsets[i]:self.offsets[i] + ps[i].numel()].view_as(ps[i]) for i in self._train]

    # ----------------------------------------------------------------- update
    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g = self.param_groups[0]
        ps = g["params"]
        grads = [ps[i].grad for i in self._train]
        if any(x is None for x in grads):
            self._step_some(ps)
            return loss
        torch._foreach_copy_(self._gdst, grads)
        b1, b2 = g["betas"]
        _lib.lib().adam_step(self.param.data_ptr(), self.grad.data_ptr(), self.exp_avg.data_ptr(),
                             self.exp_avg_sq.data_ptr(), self.n, self.step_t.data_ptr(), g["lr"], b1, b2, g["eps"],
                             g["weight_decay"], self.mask.data_ptr(), 0.0, stream_ptr())
        return loss

    def _step_some(self, ps):
        """Some trainable parameter has no gradient this step: torch.optim.Adam
        skips it (no moment update); the ones with a gradient are updated per
        tensor, with the shared step count."""
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        t = int(self.step_t.item()) + 1
        bc1, bc2 = 1.0 - b1 ** t, 1.0 - b2 ** t
        for i in self._train:
            p = ps[i]
            if p.grad is None:
                continue
            o, k = self.offsets[i], p.numel()
            m = self.exp_avg[o:o + k].view_as(p)
            v = self.exp_avg_sq[o:o + k].view_as(p)
            gr = p.grad
            if g["weight_decay"]:
                gr = gr.add(p, alpha=g["weight_decay"])
            m.mul_(b1).add_(gr, alpha=1 - b1)
            v.mul_(b2).addcmul_(gr, gr, value=1 - b2)
            den = (v.sqrt() / math.sqrt(bc2)).add_(g["eps"])
            p.addcdiv_(m, den, value=-g["lr"] / bc1)
        self.step_t.add_(1)

    # ------------------------------------------------------------ checkpoint
    def state_dict(self):
        """torch.optim.Adam's format: per trainable parameter index
        step / exp_avg / exp_avg_sq, and the group's hyperparameters."""
        g = self.param_groups[0]
        ps = g["params"]
        step = float(self.step_t.item())
        state = {}
        if step > 0:
            for i in self._train:
                o, k = self.offsets[i], ps[i].numel()
                state[i] = {"step": torch.tensor(step),
                            "exp_avg": self.exp_avg[o:o + k].view_as(ps[i]).clone(),
                            "exp_avg_sq": self.exp_avg_sq[o:o + k].view_as(ps[i]).clone()}
        group = {k: v for k, v in g.items() if k != "params"}
        group["params"] = list(range(len(ps)))
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd):
        """Inverse of state_dict; accepts what torch.optim.Adam saved for the
        same parameter list (train.py:149-154)."""
        g = self.param_groups[0]
        ps = g["params"]
        groups = sd["param_groups"]
        idx = [i for gr in groups for i in gr["params"]]
        if len(idx) != len(ps):
            raise ValueError("optimizer state has %d parameters, this optimizer %d" % (len(idx), len(ps)))
        g0 = groups[0]
        if g0.get("amsgrad") or g0.get("maximize") or g0.get("decoupled_weight_decay"):
            raise ValueError("only plain Adam with coupled weight decay is supported (train.py:134)")
        steps = set()
        with torch.no_grad():
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            for pos, i in zip(idx, range(len(ps))):
                st = sd["state"].get(pos)
                if st is None:
                    continue
                o, k = self.offsets[i], ps[i].numel()
                self.exp_avg[o:o + k].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[o:o + k].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(float(st["step"]))
        if len(steps) > 1:
            raise ValueError("per-parameter Adam step counts differ: %s" % sorted(steps))
        self.step_t.fill_(int(steps.pop()) if steps else 0)
        for k in ("lr", "betas", "eps", "weight_decay"):
            g[k] = tuple(g0[k]) if k == "betas" else g0[k]
