"""Phase timing of the persistent band kernel from in-kernel stamps
(tools/probe/band_stamps.hip).  Per case: 5 synchronised launches; for the
last one, the spread of workgroup start times and the median / max duration
of each phase across workgroups (us)."""
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

lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libband_stamps.so"))
lib.probe_band.restype = C.c_int
lib.probe_band.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]


def case(name, B, H, W, cin, cout, pro=False, stats=False, dgrad=False):
    dev = "cuda"
    M = B * H * W
    csi, cso = chan_stride(cin), chan_stride(cout)
    kp = round_up(9 * csi, 64)
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
    a.dtype, a.B, a.H, a.W, a.ks = 1, B, H, W, 3
    a.x, a.cs_in, a.cin, a.w, a.kp = x.data_ptr(), csi, cin, w.data_ptr(), kp
    a.y, a.cs_out, a.n = y.data_ptr(), cso, cout
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
    st = torch.zeros(256 * 16, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        st.zero_()
        assert lib.probe_band(C.byref(a), s, st.data_ptr()) == 0
        torch.cuda.synchronize()
    v = st.view(-1, 16).cpu().numpy().astype(np.float64) / 100.0   # 100 MHz -> us
    v = v[v[:, 0] != 0]
    t0 = v[:, 0].min()
    print("%-26s %3d WGs  start spread %5.2f  end %6.2f | tables+w %5.2f  band0 st %5.2f" % (
        name, len(v), (v[:, 0] - t0).max(), (v[:, 15] - t0).max(), np.median(v[:, 1] - v[:, 0]),
        np.median(v[:, 2] - v[:, 1])), end="")
    prev = v[:, 2]
    for k in range(6):
        m, e = v[:, 3 + 2 * k], v[:, 4 + 2 * k]
        if not (m != 0).all():
            break
        print(" | b%d mfma %5.2f epi %5.2f" % (k, np.median(m - prev), np.median(e - m)), end="")
        nxt = v[:, 5 + 2 * k] if k < 5 else None
        prev = e
    print(" | stats %5.2f" % np.median(v[:, 15] - prev), flush=True)


if __name__ == "__main__":
    case("s1 3x3 32 pro+stats", 64, 64, 64, 32, 32, pro=True, stats=True)
    case("s1 3x3 32 dgrad", 64, 64, 64, 32, 32, dgrad=True)
    case("s2 3x3 64 pro+stats", 64, 32, 32, 64, 64, pro=True, stats=True)
    case("s2 3x3 64 dgrad", 64, 32, 32, 64, 64, dgrad=True)
