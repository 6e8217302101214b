"""GPU microbenchmark: the fused row-local parameter pass (k_wn_adam) of one
coupling against the separate launches it replaces, at config 1's shapes.

    python3 tools/param_pass_bench.py [coupling-index ...]

Per coupling (backward order index into the trainer's couplings): conv
parameters, the fused launch's time and achieved GB/s over its algorithmic
bytes (36 B per conv parameter: dW slab, v twice, m, v^2 read; grad, v, m,
v^2 written; both bf16 images written), and the separate chain
(k_wn_bwd + Adam over the same range + k_wn_norm/k_wn_pack of its table).
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "dl-normalizing-flows_amd"), ROOT):
    sys.path.insert(0, p)

import torch  # noqa: E402

from bench import build_model  # noqa: E402
from realnvp_hip import _lib  # noqa: E402
from realnvp_hip.engine import stream_ptr  # noqa: E402
from realnvp_hip.trainer import FlowTrainer, wn_table  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3   # us


def main():
    dev = torch.device("cuda", 0)
    model = build_model(64, 4, 32, 5, dev, 0)
    tr = FlowTrainer(model, 4, dtype="bf16")
    tr.set_pixels(torch.rand(4, 3, 64, 64, device=dev))
    tr.step()
    torch.cuda.synchronize()
    L = _lib.lib()
    st = [s for s in tr.stages if s[0] == "coupling"][::-1]
    which = [int(a) for a in sys.argv[1:]] or [0, 7, 13, 19, 25]
    for ci in which:
        _, mod, eng, x, z, sv, block = st[ci]
        B, Cc, H, W = x.shape
        sc = eng.scratch_checked(B, H, W, "bf16", dev)
        ws = eng.weights("bf16")
        nparam = sum(d.cout * d.cin * d.ks * d.ks for d in ws["descs"])
        opt = tr._adam_args((block.data_ptr() - tr.grad.data_ptr()) // 4)
        fused = timeit(lambda: L.weight_norm_bwd_adam(sc["wn_table"].data_ptr(), sc["n_wn"], sc["wn_blocks"], 1, 1,
                                                      C.byref(opt), None, 0, None, 0, stream_ptr()))
        off = ((block.data_ptr() - tr.grad.data_ptr()) // 4 + 3) // 4 * 4
        n = (block.numel() - 4) // 4 * 4
        gb = block.data_ptr()
        t_bwd = timeit(lambda: L.weight_norm_bwd(sc["wn_table"].data_ptr(), sc["n_wn"], sc["wn_rows"], gb, None, 0,
                                                 None, 0, stream_ptr()))
        b1, b2 = tr.betas
        t_adam = timeit(lambda: L.adam_update(tr.param.data_ptr() + 4 * off, tr.grad.data_ptr() + 4 * off,
                                              tr.exp_avg.data_ptr() + 4 * off, tr.exp_avg_sq.data_ptr() + 4 * off, n,
                                              tr.step_t.data_ptr(), 1, tr.lr, b1, b2, tr.eps, tr.wd,
                                              tr.mask.data_ptr() + off, tr.reg, stream_ptr()))
        tab = wn_table([eng], "bf16", dev)
        t_fwd = timeit(lambda: _lib.lib().weight_norm_fwd(tab[0].data_ptr(), tab[1], tab[2], tab[3], 1, stream_ptr()))
        alg = 36.0 * nparam
        print("coupling %2d  %-10s params %9d  fused %7.1f us  %6.0f GB/s  | separate bwd %6.1f + adam %6.1f + "
              "fwd %6.1f = %6.1f us" % (ci, "x".join(map(str, x.shape[1:])), nparam, fused, alg / fused / 1e3,
                                         t_bwd, t_adam, t_fwd, t_bwd + t_adam + t_fwd), flush=True)


if __name__ == "__main__":
    main()
