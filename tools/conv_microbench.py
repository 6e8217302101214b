"""Microbenchmark of the MFMA conv kernels in isolation (GPU box).

    python tools/conv_microbench.py [--quick]

For each config: median time of repeated launches (HIP events on the launch
stream), algorithmic bytes (x read once, w, y written, + residual/accumulate
and the dgrad epilogue's x read) and FLOPs, achieved GB/s and TFLOP/s.
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dl-normalizing-flows_amd"))

import torch  # noqa: E402

from realnvp_hip import _lib  # noqa: E402
from realnvp_hip._lib import BNSrc, ConvArgs, WgradGroup  # noqa: E402
from realnvp_hip.engine import splitk_workspace, stat_shards  # noqa: E402
from realnvp_hip.net import chan_stride, round_up  # noqa: E402


def bench(fn, iters=20, reps=5):
    """Per-launch time inside a captured graph of `iters` back-to-back
    launches (no per-launch host or event cost; includes the dependent-kernel
    boundary, as in the training step).  Median over `reps` replays."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    s = torch.cuda.current_stream()
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        g.replay()
        e1.record(s)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / iters)
    ts.sort()
    return ts[len(ts) // 2] * 1e3   # us


def frag_major(w):
    """[n][kp] -> the fragment-major image (rnvp_conv_args.w_frag): 16-row x 32-k
    blocks in MFMA lane order (lane = n % 16 + 16 * (k % 32 // 8))."""
    n, kp = w.shape
    npad = (n + 15) // 16 * 16
    wp = torch.zeros(npad, kp, dtype=w.dtype, device=w.device)
    wp[:n] = w
    return wp.view(npad // 16, 16, kp // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()


def conv_case(B, H, W, cin, cout, ks, pro=False, stats=False, residual=False, acc=False, dgrad_epi=False,
              dtype="bf16", wgrad=False, variant=0, fm=False, group=None):
    """group (wgrad only): the kernel sizes of a grouped launch's convs (each
    its own dW slabs, same x / dy) -- e.g. a scale-1 coupling's 5 3x3 + 14 1x1"""
    dev = "cuda"
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    esz = 2 if dtype == "bf16" else 4
    M = B * H * W
    csi, cso = chan_stride(cin), chan_stride(cout)
    kp = round_up(ks * ks * csi, 64)
    x = torch.randn(M, csi, device=dev).to(tdt)
    w = (torch.randn(cout, kp, device=dev) * 0.05).to(tdt)
    y = torch.zeros(M, cso, device=dev).to(tdt)
    r = torch.randn(M, cso, device=dev).to(tdt)
    sh = stat_shards(M)
    sums_in = torch.rand(sh, 2, cin, device=dev, dtype=torch.float64) * M / sh
    sums_in[:, 1] += 2 * M / sh
    sums_out = torch.zeros(sh, 2, cout, device=dev, dtype=torch.float64)
    gam = torch.ones(max(cin, cout), device=dev)
    bet = torch.zeros(max(cin, cout), device=dev)
    ws = splitk_workspace(dev, 8 * M * cso if M <= 16384 else 1)
    L = _lib.lib()
    s = torch.cuda.current_stream().cuda_stream
    if wgrad:
        nz = int(L.wgrad_slabs(M))
        nrep = int(L.wgrad_replicas(nz))
        kss = list(group) if group else [ks]
        dws = []
        a = WgradGroup()
        a.dtype = 1 if dtype == "bf16" else 0
        a.B, a.H, a.W, a.n_conv = B, H, W, len(kss)
        for i, k in enumerate(kss):
            kpk = round_up(k * k * csi, 64)
            dws.append(torch.zeros(nrep, cout, kpk, device=dev))
            c = a.conv[i]
            c.x, c.cs_in, c.cin, c.ks = x.data_ptr(), csi, cin, k
            if pro:
                c.pro_bn_relu = 1
                c.pro = BNSrc(sums_in.data_ptr(), float(M), None, None, gam.data_ptr(), bet.data_ptr(), 1e-5, sh)
            c.dy, c.cs_dy, c.n = y.data_ptr(), cso, cout
            c.ws, c.kp, c.nz, c.nrep = dws[-1].data_ptr(), kpk, nz, nrep
        fn = lambda: L.conv2d_wgrad_grouped(C.byref(a), torch.cuda.current_stream().cuda_stream)  # noqa: E731
        nbytes = sum(esz * M * (csi + cso) + 4 * cout * k * k * cin for k in kss)
        flops = sum(2.0 * M * cout * k * k * cin for k in kss)
        us = bench(fn)
        return us, nbytes / us / 1e3, flops / us / 1e6
    else:
        a = ConvArgs()
        a.dtype = 1 if dtype == "bf16" else 0
        a.B, a.H, a.W, a.ks = B, H, W, ks
        a.x, a.cs_in, a.cin = x.data_ptr(), csi, cin
        a.w, a.kp = w.data_ptr(), kp
        if fm:
            wfm = frag_major(w)
            a.w_frag = wfm.data_ptr()
        a.y, a.cs_out, a.n = y.data_ptr(), cso, cout
        a.residual = r.data_ptr() if residual else None
        a.accumulate = int(acc)
        if pro:
            a.pro_bn_relu = 1
            a.pro = BNSrc(sums_in.data_ptr(), float(M), None, None, gam.data_ptr(), bet.data_ptr(), 1e-5, sh)
        if stats:
            a.out_sums = sums_out.data_ptr()
        if dgrad_epi:
            a.epi_relu_bn_bwd = 1
            a.epi_x = r.data_ptr()
            a.epi = BNSrc(sums_in.data_ptr(), float(M), None, None, gam.data_ptr(), bet.data_ptr(), 1e-5, sh)
            a.epi_sums = sums_out.data_ptr()
        a.ws, a.ws_elems = ws.data_ptr(), ws.numel()
        a.variant = variant
        if dgrad_epi:
            sums_out.zero_()
        fn = lambda: L.conv2d(C.byref(a), torch.cuda.current_stream().cuda_stream)  # noqa: E731
        nbytes = esz * (M * csi + cout * kp + M * cso * (1 + int(residual) + int(acc) + int(dgrad_epi)))
    us = bench(fn)
    flops = 2.0 * M * cout * ks * ks * cin
    return us, nbytes / us / 1e3, flops / us / 1e6


CASES = [
    # name, B, H, W, cin, cout, ks, flags
    ("s1 1x1 32->32 plain", 64, 64, 64, 32, 32, 1, {}),
    ("s1 1x1 32->32 pro", 64, 64, 64, 32, 32, 1, dict(pro=True)),
    ("s1 1x1 32->32 pro+stats", 64, 64, 64, 32, 32, 1, dict(pro=True, stats=True)),
    ("s1 1x1 32->32 pro+stats+res", 64, 64, 64, 32, 32, 1, dict(pro=True, stats=True, residual=True)),
    ("s1 1x1 32->32 skip acc", 64, 64, 64, 32, 32, 1, dict(acc=True)),
    ("s1 3x3 32->32 pro+stats", 64, 64, 64, 32, 32, 3, dict(pro=True, stats=True)),
    ("s1 3x3 32->32 dgrad", 64, 64, 64, 32, 32, 3, dict(dgrad_epi=True)),
    ("s1 3x3 7->32 in", 64, 64, 64, 7, 32, 3, dict(stats=True)),
    ("s1 1x1 32->6 out", 64, 64, 64, 32, 6, 1, dict(pro=True)),
    ("s2 1x1 64->64 pro+stats", 64, 32, 32, 64, 64, 1, dict(pro=True, stats=True)),
    ("s2 3x3 64->64 pro+stats", 64, 32, 32, 64, 64, 3, dict(pro=True, stats=True)),
    ("s3 3x3 128->128 pro+stats", 64, 16, 16, 128, 128, 3, dict(pro=True, stats=True)),
    ("s4 3x3 256->256 pro+stats", 64, 8, 8, 256, 256, 3, dict(pro=True, stats=True)),
    ("s5 3x3 512->512 pro+stats", 64, 4, 4, 512, 512, 3, dict(pro=True, stats=True)),
    ("s5 1x1 512->512 pro+stats", 64, 4, 4, 512, 512, 1, dict(pro=True, stats=True)),
    ("s5 3x3 512->512 dgrad", 64, 4, 4, 512, 512, 3, dict(dgrad_epi=True)),
    ("s5 1x1 512->512 pro+stats+res", 64, 4, 4, 512, 512, 1, dict(pro=True, stats=True, residual=True)),
    ("s5 1x1 512->96 out", 64, 4, 4, 512, 96, 1, dict(pro=True)),
    ("s5 3x3 97->512 in", 64, 4, 4, 97, 512, 3, dict(stats=True)),
    ("s4 1x1 256->256 pro+stats", 64, 8, 8, 256, 256, 1, dict(pro=True, stats=True)),
    ("s4 3x3 256->256 dgrad", 64, 8, 8, 256, 256, 3, dict(dgrad_epi=True)),
    ("s3 1x1 128->128 pro+stats", 64, 16, 16, 128, 128, 1, dict(pro=True, stats=True)),
    ("s3 3x3 128->128 dgrad", 64, 16, 16, 128, 128, 3, dict(dgrad_epi=True)),
    ("s3 1x1 128->128 pro+stats+res", 64, 16, 16, 128, 128, 1, dict(pro=True, stats=True, residual=True)),
    ("s3 1x1 128->128 skip acc", 64, 16, 16, 128, 128, 1, dict(acc=True, stats=True)),
    ("s3 1x1 128->128 dgrad", 64, 16, 16, 128, 128, 1, dict(dgrad_epi=True)),
    ("s4 1x1 256->256 dgrad", 64, 8, 8, 256, 256, 1, dict(dgrad_epi=True)),
    ("s4 1x1 256->256 skip acc", 64, 8, 8, 256, 256, 1, dict(acc=True, stats=True)),
    ("s5 1x1 512->512 dgrad", 64, 4, 4, 512, 512, 1, dict(dgrad_epi=True)),
    ("s5 1x1 512->512 skip acc", 64, 4, 4, 512, 512, 1, dict(acc=True, stats=True)),
    ("s2c 1x1 64->64 pro+stats", 64, 32, 32, 64, 64, 1, dict(pro=True, stats=True)),
    ("wgrad s1 1x1 32", 64, 64, 64, 32, 32, 1, dict(pro=True, wgrad=True)),
    ("wgrad s1 3x3 32", 64, 64, 64, 32, 32, 3, dict(pro=True, wgrad=True)),
    ("wgrad s1 group 1x1 x14", 64, 64, 64, 32, 32, 1, dict(pro=True, wgrad=True, group=[1] * 14)),
    ("wgrad s1 group 3x3 x5", 64, 64, 64, 32, 32, 3, dict(pro=True, wgrad=True, group=[3] * 5)),
    ("wgrad s1 group 5 3x3 + 14 1x1", 64, 64, 64, 32, 32, 3, dict(pro=True, wgrad=True, group=[3] * 5 + [1] * 14)),
    ("wgrad s2 group 5 3x3 + 14 1x1", 64, 32, 32, 64, 64, 3, dict(pro=True, wgrad=True, group=[3] * 5 + [1] * 14)),
    ("wgrad s2 3x3 64", 64, 32, 32, 64, 64, 3, dict(pro=True, wgrad=True)),
    ("wgrad s3 3x3 128", 64, 16, 16, 128, 128, 3, dict(pro=True, wgrad=True)),
    ("wgrad s5 3x3 512", 64, 4, 4, 512, 512, 3, dict(pro=True, wgrad=True)),
    ("wgrad s5 1x1 512", 64, 4, 4, 512, 512, 1, dict(pro=True, wgrad=True)),
]


def main():
    torch.manual_seed(0)
    variants = [0, 1] if "--v01" in sys.argv else [0]
    fms = [False, True] if "--fm" in sys.argv else [False]
    if "--deep" in sys.argv:   # the deep-scale family's configurations (RNVP_VARIANT_DEEP0 + c)
        variants = [0] + [16 + c for c in range(7)]
    only = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--case=")]
    print("%-32s %3s %9s %9s %9s" % ("case", "var", "us", "GB/s", "TFLOP/s"))
    for name, B, H, W, ci, co, ks, fl in CASES:
        if only and not any(o in name for o in only):
            continue
        for v in variants:
            for fm in fms:
                if (fl.get("wgrad") and (v or fm)) or (fm and ks != 3):
                    continue
                try:
                    us, gbs, tfs = conv_case(B, H, W, ci, co, ks, variant=v, fm=fm, **fl)
                except RuntimeError:
                    continue   # configuration does not apply to this shape
                print("%-32s %3d%s %9.1f %9.1f %9.1f" % (name, v, "f" if fm else " ", us, gbs, tfs), flush=True)


if __name__ == "__main__":
    main()
