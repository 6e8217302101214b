"""Phase timing of the coupling-link backward (tools/probe/link_stamps.hip:
coupling_link.hip built with per-workgroup stamps).  Builds the config-1
trainer (bf16, B = 64), runs two eager steps, then launches each coupling's
rnvp_coupling_link_bwd through the probe library on the same arguments and
reports the spread of workgroup start times and the median / max of each
phase across workgroups (us, 100 MHz stamps).  Timing only: the repeated
launches accumulate into the step's sums, so values are not meaningful."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dl-normalizing-flows_amd"))
sys.path.insert(0, ROOT)

PH = ["loads+tables", "closed form", "body", "block sums", "tile out+atomics"]


def main():
    import bench
    from realnvp_hip.engine import stream_ptr
    from realnvp_hip.trainer import FlowTrainer
    probe = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblink_stamps.so"))
    probe.probe_link_bwd.restype = C.c_int
    probe.probe_link_bwd.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    dev = torch.device("cuda")
    model = bench.build_model(64, 4, 32, 5, dev, 0)
    tr = FlowTrainer(model, 64, dtype="bf16", seed=1)
    tr.set_pixels(bench.synthetic_pixels(64, 3, 64, 0).to(dev))
    tr.step_eager()
    tr.step_eager()
    torch.cuda.synchronize()
    st = torch.zeros(8192 * 8, dtype=torch.int64, device=dev)
    names = {id(m): n for n, m in model.named_modules()}
    for k in reversed(range(len(tr.cidx))):
        _, mod, eng, x, z, sv, block = tr.stages[tr.cidx[k]]
        link = tr.link_bwd[k]
        a = eng.link_args(sv, x, block, tr._g(x))
        a.nclass = link["nclass"]
        a.gl_sample = tr.g_lp.data_ptr()
        n = None
        if link["nxt"] is not None:
            neng, nsv, nx, ngx, nblock = link["nxt"]
            n = neng.link_args(nsv, nx, nblock, ngx)
        rows = []
        for rep in range(4):
            st.zero_()
            torch.cuda.synchronize()
            r = probe.probe_link_bwd(C.addressof(a), C.addressof(n) if n is not None else None,
                                     C.addressof(link["args"]), stream_ptr(), st.data_ptr())
            torch.cuda.synchronize()
            assert r == 0, r
        s = st.view(-1, 8).cpu().numpy().astype(np.int64)
        s = s[s[:, 0] > 0]
        t0 = s[:, 0].min()
        start = (s[:, 0] - t0) / 100.0
        ph = np.diff(s[:, :6], axis=1) / 100.0
        total = (s[:, 5].max() - t0) / 100.0
        out = "%-10s type %d grid %4d  start spread %.2f  wall %.2f |" % (names[id(mod)], link["args"].type, len(s),
                                                                            start.max(), total)
        for i in range(ph.shape[1]):
            out += " %s %.2f/%.2f" % (PH[i], np.median(ph[:, i]), ph[:, i].max())
        print(out, flush=True)


if __name__ == "__main__":
    main()
