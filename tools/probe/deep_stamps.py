"""Phase timing of the deep-scale conv kernels from in-kernel stamps
(tools/probe/deep_stamps.hip).  Per case: launches the kernel 5 times
(synchronised), reports for the last launch the spread of workgroup start
times and the median / max duration of each phase across workgroups (us)."""
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

lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdeep_stamps.so"))
lib.probe_deep.restype = C.c_int
lib.probe_deep.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
PH = ["tab+stage ld", "ring+act st", "k-loop", "reduce+epi", "stats", ]


def case(name, B, H, W, cin, cout, ks, cfg, pro=False, stats=False, residual=False, acc=False, dgrad=False, bp=False):
    dev = "cuda"
    M = B * H * W
    csi, cso = chan_stride(cin), chan_stride(cout)
    kp = round_up(ks * ks * csi, 64)
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
    a.B, a.H, a.W, a.ks = B, H, W, ks
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
    if bp:   # BatchNorm-backward prologue (rnvp_conv_args.bp): x is the pre-apply gradient
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
        rc = lib.probe_deep(C.byref(a), s, cfg, st.data_ptr())
        assert rc == 0, rc
        torch.cuda.synchronize()
    nwg = int((st.view(-1, 8)[:, 0] != 0).sum())
    v = st.view(-1, 8)[:nwg].cpu().numpy().astype(np.float64) / 100.0   # 100 MHz -> us
    t0 = v[:, 0].min()
    start = v[:, 0] - t0
    end = v[:, 5] - t0
    d = np.diff(v[:, :6], axis=1)
    print("%-28s cfg %d: %4d WGs  start spread %5.2f  last end %6.2f  | " % (name, cfg, nwg, start.max(), end.max()) +
          "  ".join("%s %5.2f/%5.2f" % (PH[i], np.median(d[:, i]), d[:, i].max()) for i in range(5)), flush=True)


CASES = [
    ("s5 1x1 pro+stats", 64, 4, 4, 512, 512, 1, dict(pro=True, stats=True)),
    ("s5 1x1 skip acc", 64, 4, 4, 512, 512, 1, dict(acc=True, stats=True)),
    ("s5 3x3 pro+stats", 64, 4, 4, 512, 512, 3, dict(pro=True, stats=True)),
    ("s5 3x3 dgrad", 64, 4, 4, 512, 512, 3, dict(dgrad=True)),
    ("s4 3x3 pro+stats", 64, 8, 8, 256, 256, 3, dict(pro=True, stats=True)),
    ("s4 1x1 pro+stats", 64, 8, 8, 256, 256, 1, dict(pro=True, stats=True)),
    ("s3 1x1 pro+stats", 64, 16, 16, 128, 128, 1, dict(pro=True, stats=True)),
    ("s3 3x3 pro+stats", 64, 16, 16, 128, 128, 3, dict(pro=True, stats=True)),
]

BP_CASES = [
    ("s5 1x1 dgrad", 64, 4, 4, 512, 512, 1, dict(dgrad=True)),
    ("s5 1x1 dgrad+bp", 64, 4, 4, 512, 512, 1, dict(dgrad=True, bp=True)),
    ("s5 3x3 dgrad", 64, 4, 4, 512, 512, 3, dict(dgrad=True)),
    ("s5 3x3 dgrad+bp", 64, 4, 4, 512, 512, 3, dict(dgrad=True, bp=True)),
    ("s4 3x3 dgrad", 64, 8, 8, 256, 256, 3, dict(dgrad=True)),
    ("s4 3x3 dgrad+bp", 64, 8, 8, 256, 256, 3, dict(dgrad=True, bp=True)),
    ("s3 3x3 dgrad", 64, 16, 16, 128, 128, 3, dict(dgrad=True)),
    ("s3 3x3 dgrad+bp", 64, 16, 16, 128, 128, 3, dict(dgrad=True, bp=True)),
    ("s3 1x1 dgrad", 64, 16, 16, 128, 128, 1, dict(dgrad=True)),
    ("s3 1x1 dgrad+bp", 64, 16, 16, 128, 128, 1, dict(dgrad=True, bp=True)),
]

if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "bp":
        for name, B, H, W, ci, co, ks, fl in BP_CASES:
            case(name, B, H, W, ci, co, ks, 4 if B * H * W <= 1024 else 0, **fl)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "bp8":
        # the 8-wave tile (cfg 4) for the 1x1 data gradients above 1024 pixels
        for name, B, H, W, ci, co, ks, fl in [("s4 1x1 dgrad", 64, 8, 8, 256, 256, 1, dict(dgrad=True)),
                                                ("s4 1x1 dgrad+bp", 64, 8, 8, 256, 256, 1, dict(dgrad=True, bp=True)),
                                                ("s3 1x1 dgrad", 64, 16, 16, 128, 128, 1, dict(dgrad=True)),
                                                ("s3 1x1 dgrad+bp", 64, 16, 16, 128, 128, 1, dict(dgrad=True, bp=True))]:
            for cfg in (0, 4):
                try:
                    case(name, B, H, W, ci, co, ks, cfg, **fl)
                except AssertionError:
                    print("%-28s cfg %d: unsupported" % (name, cfg), flush=True)
        sys.exit(0)
    for name, B, H, W, ci, co, ks, fl in CASES:
        for cfg in (0, 1, 2, 3, 4, 5):
            try:
                case(name, B, H, W, ci, co, ks, cfg, **fl)
            except AssertionError:
                pass
