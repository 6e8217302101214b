"""Phase timing of the wide-scale streaming 1x1 conv (k_conv_s1) from
in-kernel stamps (tools/probe/s1_stamps.hip).  Per case: 5 synchronised
launches; for the last one the spread of workgroup start times, the last end,
and the median / max of each phase across workgroups (us): prologue (weights,
BN tables, first tile issued), tiles (the tile walk incl. its loads' latency),
stats (batch-statistic reduction + fp64 atomics)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "dl-normalizing-flows_amd"))
from realnvp_hip._lib import BNSrc, ConvArgs  # noqa: E402
from realnvp_hip.engine import stat_shards  # noqa: E402
from realnvp_hip.net import chan_stride, round_up  # noqa: E402

LIBNAME = os.environ.get("S1_PROBE_LIB", "libs1_stamps.so")
lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), LIBNAME))
lib.probe_s1.restype = C.c_int
lib.probe_s1.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
PH = ["prologue", "tiles", "stats"]


def case(name, B, H, W, cin, cout, pro=False, stats=False, residual=False, acc=False, dgrad=False, bp=False):
    dev = "cuda"
    M = B * H * W
    csi, cso = chan_stride(cin), chan_stride(cout)
    kp = round_up(csi, 64)
    x = torch.randn(M, csi, device=dev).to(torch.bfloat16)
    w = (torch.randn(cout, kp, device=dev) * 0.05).to(torch.bfloat16)
    y = torch.zeros(M, cso, device=dev).to(torch.bfloat16)
    r = torch.randn(M, cso, device=dev).to(torch.bfloat16)
    sh = stat_shards(M)
    sums_in = torch.rand(sh, 2, max(cin, cout), device=dev, dtype=torch.float64) * M / sh
    sums_in[:, 1] += 2 * M / sh
    sums_out = torch.zeros(sh, 2, cout, device=dev, dtype=torch.float64)
    gam = torch.ones(max(cin, cout), device=dev)
    bet = torch.zeros(max(cin, cout), device=dev)
    a = ConvArgs()
    a.dtype = 1
    a.B, a.H, a.W, a.ks = B, H, W, 1
    a.x, a.cs_in, a.cin = x.data_ptr(), csi, cin
    a.w, a.kp = w.data_ptr(), kp
    a.y, a.cs_out, a.n = y.data_ptr(), cso, cout
    a.residual = r.data_ptr() if residual else None
    a.accumulate = int(acc)
    if pro:
        a.pro_bn_relu = 1
        a.pro = BNSrc(sums_in.data_ptr(), float(M), None, None, gam.data_ptr(), bet.data_ptr(), 1e-5, sh)
    if stats:
        a.out_sums = sums_out.data_ptr()
    if dgrad:
        a.epi_relu_bn_bwd = 1
        a.epi_x = r.data_ptr()
        a.epi = BNSrc(sums_in.data_ptr(), float(M), None, None, gam.data_ptr(), bet.data_ptr(), 1e-5, sh)
        a.epi_sums = sums_out.data_ptr()
    if bp:   # BatchNorm-backward prologue: x is the pre-apply gradient, t the BatchNorm input
        t = torch.randn(M, csi, device=dev).to(torch.bfloat16)
        side = torch.zeros(M, csi, device=dev).to(torch.bfloat16)
        dgb = torch.zeros(2, cin, device=dev)
        a.bp, a.bp_x, a.bp_sums, a.bp_shards = 1, t.data_ptr(), sums_in.data_ptr(), sh
        a.bp_bn = BNSrc(sums_in.data_ptr(), float(M), None, None, gam.data_ptr(), bet.data_ptr(), 1e-5, sh)
        a.bp_out, a.bp_dgamma, a.bp_dbeta = side.data_ptr(), dgb[0].data_ptr(), dgb[1].data_ptr()
    st = torch.zeros(8192 * 8, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        st.zero_()
        rc = lib.probe_s1(C.byref(a), s, st.data_ptr())
        assert rc == 0, rc
        torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        lib.probe_s1(C.byref(a), s, st.data_ptr())
    e1.record()
    torch.cuda.synchronize()
    per = e0.elapsed_time(e1) / 20 * 1000
    nwg = int((st.view(-1, 8)[:, 0] != 0).sum())
    v = st.view(-1, 8)[:nwg].cpu().numpy().astype(np.float64) / 100.0
    t0 = v[:, 0].min()
    d = np.diff(v[:, :4], axis=1)
    nb = 2 * M * (csi * (1 + 2 * int(bp)) + cso * (1 + int(residual) + int(acc) + int(dgrad)))
    print("%-26s %4d WGs  %6.2f us/launch (%5.0f GB/s)  start spread %5.2f  last end %6.2f | " %
          (name, nwg, per, nb / per / 1e3, (v[:, 0] - t0).max(), (v[:, 3] - t0).max()) +
          "  ".join("%s %5.2f/%5.2f" % (PH[i], np.median(d[:, i]), d[:, i].max()) for i in range(3)), flush=True)


CASES = [
    ("s2 64->64 pro+stats", 64, 32, 32, 64, 64, dict(pro=True, stats=True)),
    ("s2 64->64 pro+res", 64, 32, 32, 64, 64, dict(pro=True, residual=True)),
    ("s2 64->64 dgrad", 64, 32, 32, 64, 64, dict(dgrad=True)),
    ("s2 64->64 dgrad+bp", 64, 32, 32, 64, 64, dict(dgrad=True, bp=True)),
    ("s2 64->64 plain", 64, 32, 32, 64, 64, dict()),
    ("s1 32->32 pro+stats", 64, 64, 64, 32, 32, dict(pro=True, stats=True)),
    ("s1 32->32 dgrad", 64, 64, 64, 32, 32, dict(dgrad=True)),
    ("s1 32->32 dgrad+bp", 64, 64, 64, 32, 32, dict(dgrad=True, bp=True)),
    ("s1 32->32 plain", 64, 64, 64, 32, 32, dict()),
]

if __name__ == "__main__":
    for name, B, H, W, ci, co, fl in CASES:
        case(name, B, H, W, ci, co, **fl)
