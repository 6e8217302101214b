"""CPU-side checks of the drop-in boundary (no GPU needed)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, load_golden

HEADER = os.path.join(ROOT, "include", "realnvp_hip.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(rnvp_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_declared_symbol():
    from realnvp_hip._lib import LIB_PATH, EXPORTED
    assert os.path.exists(LIB_PATH), "build the HIP library first (__graft_entry__.build())"
    dll = ctypes.CDLL(LIB_PATH)
    decl = declared_symbols()
    assert len(decl) >= 25
    for s in decl:
        assert hasattr(dll, s), s
    # the ctypes binding covers exactly the declared ABI
    assert sorted(EXPORTED) == decl
    assert dll.rnvp_version() >= 100


def test_invalid_arguments_return_status_without_launch():
    from realnvp_hip._lib import LIB_PATH
    dll = ctypes.CDLL(LIB_PATH)
    dll.rnvp_squeeze.restype = ctypes.c_int
    # NULL pointers / odd sizes are rejected before any HIP call
    assert dll.rnvp_squeeze(None, None, 1, 1, 2, 2, None) == -1
    x = ctypes.c_float(0)
    assert dll.rnvp_squeeze(ctypes.byref(x), ctypes.byref(x), 1, 1, 3, 2, None) == -1
    dll.rnvp_status_string.restype = ctypes.c_char_p
    assert dll.rnvp_status_string(-1) == b"invalid argument"


def test_stale_library_is_refused(monkeypatch):
    """A library whose argument structs differ from the binding's mirrors
    (built from another header revision) is refused at load time: reading a
    descriptor table at the wrong stride faulted the GPU in round 5
    (gpurun_out/r5_fm2)."""
    from realnvp_hip import _lib

    class Grown(ctypes.Structure):
        _fields_ = list(_lib.CouplingArgs._fields_) + [("extra", ctypes.c_int)]
    monkeypatch.setattr(_lib, "CouplingArgs", Grown)
    with pytest.raises(RuntimeError, match="stale build"):
        _lib._Lib()
    monkeypatch.undo()
    _lib._Lib()   # the real mirrors load


def test_link_arguments_checked_without_launch():
    """rnvp_coupling_link_fwd / _bwd / rnvp_coupling_out_u reject inconsistent
    links before any HIP call: the class mode must be the link's, the
    geometry must be the link type's (a squeeze quadruples the channels and
    halves the size, a factor-out halves the channels), training with out_bn."""
    from realnvp_hip import _lib
    L = _lib._Lib()
    assert [L.link_nclass(t, k) for t in range(4) for k in (0, 1)] == [2, 1, 4, 4, 2, 2, 2, 1]
    f = ctypes.c_float(0.0)
    d = ctypes.c_double(0.0)

    def args(kind, C, S, cfg, nclass):
        a = _lib.CouplingArgs()
        a.kind, a.B, a.C, a.H, a.W, a.mask_config, a.coupling_bn, a.training, a.dtype = kind, 2, C, S, S, cfg, 1, 1, 1
        a.x = a.st = a.scale = a.scale_shift = a.ldj_sample = ctypes.addressof(f)
        a.h0 = a.in_sums = a.cls_sums = a.prior_sums = ctypes.addressof(d)
        a.cs_st, a.cs_h0, a.nclass = 8 * ((2 * C + 7) // 8), 8 * ((2 * C + 8) // 8), nclass
        return a
    la = _lib.LinkArgs(_lib.RNVP_LINK_SQUEEZE, ctypes.addressof(f), ctypes.addressof(d), None, None)
    a, n = args(0, 3, 8, 1, 4), args(1, 12, 4, 0, 1)
    bad = [
        (args(0, 3, 8, 1, 2), n),        # wrong class mode for a squeeze
        (a, args(1, 12, 8, 0, 1)),       # consumer not half the size
        (a, args(1, 6, 4, 0, 1)),        # consumer not 4x the channels
        (args(1, 6, 8, 0, 4), n),        # a squeeze starts at a checkerboard coupling
    ]
    for x, y in bad:
        st = L.dll.rnvp_coupling_link_fwd(ctypes.byref(x), ctypes.byref(y), ctypes.byref(la), None)
        assert st == -1, st
    a.training = 0
    assert L.dll.rnvp_coupling_out_u(ctypes.byref(a), None) == -1


def test_bn_fold_support_query_without_launch():
    """rnvp_conv2d_check answers the engine's fold question on the host: a
    BatchNorm-backward prologue (bp) runs on the deep family's data-gradient
    tiles and the wide scales' streaming 1x1 and band 3x3 -- accepted where
    it pays, refused (UNSUPPORTED) for the 16384-pixel 4-wave 1x1 tiles or a
    forced non-deep variant, INVALID without the
    BatchNorm input; the coupling shard count mirrors the header's."""
    from realnvp_hip import _lib, engine
    L = _lib._Lib()
    hdr = open(os.path.join(ROOT, "include", "realnvp_hip.h")).read()
    assert int(re.search(r"#define RNVP_COUPLING_SHARDS (\d+)", hdr).group(1)) == engine.COUPLING_SHARDS
    buf = (ctypes.c_double * 64)()
    p = ctypes.addressof(buf)

    def args(B, S, c, ks, bp=1, bp_x=True, variant=0, epi=False):
        a = _lib.ConvArgs()
        a.dtype, a.B, a.H, a.W, a.ks = 1, B, S, S, ks
        a.x, a.cs_in, a.cin, a.w, a.kp = p, c, c, p, (ks * ks * c + 63) // 64 * 64
        a.y, a.cs_out, a.n = p, c, c
        a.variant = variant
        a.bp, a.bp_x, a.bp_sums, a.bp_shards = bp, p if bp_x else None, p, 1
        a.bp_bn = _lib.BNSrc(p, float(B * S * S), None, None, None, None, 1e-5, 1)
        if epi:   # the data gradient's ReLU/BN epilogue
            a.epi_relu_bn_bwd, a.epi_x, a.epi_sums = 1, p, p
            a.epi = _lib.BNSrc(p, float(B * S * S), None, None, None, None, 1e-5, 1)
        return a
    ok = [args(64, 4, 512, 1), args(64, 4, 512, 3), args(64, 8, 256, 3), args(64, 8, 256, 1), args(64, 16, 128, 3),
          args(64, 16, 128, 1, variant=16)]          # a forced 4-wave 1x1 tile (RNVP_VARIANT_DEEP0)
    for a in ok:
        assert L.conv2d_check(ctypes.byref(a)) == 0
    # the tuned dispatch keeps the apply before the 16384-pixel 1x1 tiles (measured slower folded)
    assert L.conv2d_check(ctypes.byref(args(64, 16, 128, 1))) == -2
    # wide scales: the streaming 1x1 (bf16) folds a data gradient with the ReLU/BN epilogue
    assert L.conv2d_check(ctypes.byref(args(64, 32, 64, 1, epi=True))) == 0
    assert L.conv2d_check(ctypes.byref(args(64, 32, 64, 1))) == -2
    assert L.conv2d_check(ctypes.byref(args(64, 32, 64, 3, epi=True))) == 0    # the band 3x3
    assert L.conv2d_check(ctypes.byref(args(64, 32, 64, 3))) == -2             # (with the ReLU/BN epilogue only)
    assert L.conv2d_check(ctypes.byref(args(64, 8, 256, 3, variant=1))) == -2
    assert L.conv2d_check(ctypes.byref(args(64, 8, 256, 3, bp_x=False))) == -1
    assert L.conv2d_check(ctypes.byref(args(64, 32, 64, 1, bp=0))) == 0


def _hp(bd, rb, bott=True, skip=True, wn=True, cbn=True):
    import utils
    return utils.Hyperparameters(bd, rb, bott, skip, wn, cbn)


def test_state_dict_layout_matches_reference_spec():
    import flow_realnvp
    import realnvp_oracle as O
    for size, bd, rb in ((32, 8, 1), (64, 32, 4), (32, 4, 0)):
        m = flow_realnvp.RealNVP(3, size, torch.distributions.Normal(torch.tensor(0.), torch.tensor(1.)), _hp(bd, rb))
        e = O.flow_spec_entries(O.FlowSpec(3, size, O.HP(bd, rb)))
        sd = m.state_dict()
        assert list(sd.keys()) == [k for k, _, _ in e]
        assert all(tuple(sd[k].shape) == tuple(s) for k, s, _ in e)
        assert [n for n, _ in m.named_parameters()] == O.param_names(e)
        assert [n for n, p in m.named_parameters() if p.requires_grad] == O.trainable_names(e)


def test_default_init_draws_like_reference():
    import flow_realnvp
    g = load_golden("init_seed0.npz")
    for name, size, bd, rb, bott in (("m32_d8_r1", 32, 8, 1, True), ("m16_d4_r2_nobott", 16, 4, 2, False)):
        torch.manual_seed(0)
        m = flow_realnvp.RealNVP(3, size, torch.distributions.Normal(torch.tensor(0.), torch.tensor(1.)),
                                 _hp(bd, rb, bott))
        sd = m.state_dict()
        assert list(sd.keys()) == list(g[name + ".keys"])
        s = np.array([float(v.double().sum()) for v in sd.values()])
        s2 = np.array([float(v.double().pow(2).sum()) for v in sd.values()])
        np.testing.assert_allclose(s, g[name + ".sum"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(s2, g[name + ".sumsq"], rtol=1e-5, atol=1e-6)


def test_order_matrix_and_mask_match_reference():
    import flow_realnvp
    import modules_realnvp
    g = load_golden("index_maps.npz")
    m = flow_realnvp.RealNVP.__new__(flow_realnvp.RealNVP)
    for C in (3, 6, 12, 24):
        assert np.array_equal(flow_realnvp.RealNVP.order_matrix(m, C).numpy(), g["order_matrix_%d" % C])
    c = modules_realnvp.CheckerboardAffineCoupling(3, 8, 8, 1., _hp(8, 1))
    for size in (2, 4, 8, 64):
        for cfg in (0, 1):
            assert np.array_equal(c.build_mask(size, float(cfg)).numpy(), g["mask_%d_%d" % (size, cfg)])


def test_cpu_tensors_fail_loudly():
    import modules_realnvp
    c = modules_realnvp.CheckerboardAffineCoupling(3, 8, 8, 1., _hp(8, 1))
    with pytest.raises(RuntimeError, match="HIP device"):
        c(torch.zeros(2, 3, 8, 8))


def test_backward_program_is_well_formed():
    from realnvp_hip.net import backward_program, build_program
    for rb in (0, 1, 4):
        for bott in (True, False):
            for skip in (True, False):
                P = build_program("block.1.", 7, 32, 6, rb, bott, skip, True)
                steps = backward_program(P)
                # every conv gets one wgrad and one dgrad
                assert sum(s.kind == "wgrad" for s in steps) == len(P.ops)
                assert sum(s.kind == "dgrad" for s in steps) == len(P.ops)
                # every gradient buffer is written before it is read as dy
                written = {"g:st"}
                for s in steps:
                    if s.kind in ("dgrad", "wgrad"):
                        assert s.gy in written, (rb, bott, skip, s)
                    if s.gx:
                        written.add(s.gx)
                assert "g:h0" in written
                # ... and COMPLETE: every contribution to d b (the data
                # gradient of each op reading b, the identity path of each
                # residual add onto b) is in before any step reads it (the skip
                # data gradients run early, block residuals fold into later writes)
                want = {}
                for op in P.ops:
                    want["g:" + op.x] = want.get("g:" + op.x, 0) + 1
                    if op.residual:
                        want["g:" + op.residual] = want.get("g:" + op.residual, 0) + 1
                have = {"g:st": 0}
                want["g:st"] = 0
                for s in steps:
                    for src in ([s.gy] if s.kind in ("dgrad", "wgrad") else []) + ([s.residual] if s.residual else []):
                        assert have.get(src, 0) == want.get(src, 0), (rb, bott, skip, src, s)
                    if s.gx and s.kind in ("dgrad", "bn_apply"):
                        have[s.gx] = have.get(s.gx, 0) + 1 + (1 if s.residual else 0)
                assert have["g:h0"] == want["g:h0"]


def test_reference_train_py_import_line():
    """train.py:37-41 imports these names from the drop-in modules unchanged."""
    import torch.nn as nn
    from flow_realnvp import RealNVP  # noqa: F401
    from modules_realnvp import ChannelwiseAffineCoupling, CheckerboardAffineCoupling  # noqa: F401
    from utils import Hyperparameters, logit_transform, weights_init  # noqa: F401
    torch.manual_seed(0)
    conv, bn = nn.Conv2d(3, 4, 3), nn.BatchNorm2d(4)
    weights_init(conv)
    weights_init(bn)
    assert abs(float(conv.weight.std()) - 0.02) < 0.01
    assert float(bn.bias.abs().max()) == 0.0 and abs(float(bn.weight.mean()) - 1.0) < 0.02


def test_net_group_prepare_rejections():
    """rnvp_net_group_prepare is host-only validation (no HIP call): it groups
    independent deep-scale 1x1 convs and refuses what has no grouped form
    (RNVP_E_UNSUPPORTED = -2: the engine then launches them one by one) or is
    malformed (RNVP_E_INVALID = -1).  Pointers are never dereferenced here."""
    from realnvp_hip import _lib
    from realnvp_hip._lib import ConvArgs, NetStep
    L = _lib.lib()
    fake = 1 << 20     # 16-B aligned, never dereferenced

    def step(B=64, H=4, W=4, cs=512, n=512, ks=1, dtype=0, kind=0, x=fake):
        st = NetStep()
        st.kind = kind
        a = st.conv
        a.dtype, a.B, a.H, a.W, a.ks = dtype, B, H, W, ks
        a.x, a.cs_in, a.cin, a.w, a.kp = x, cs, cs, fake, (ks * ks * cs + 63) // 64 * 64
        a.y, a.cs_out, a.n = fake, n, n
        return st

    def prep(*steps):
        arr = (NetStep * len(steps))(*steps)
        k, g, lb = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        rc = L.net_group_prepare(arr, len(steps), ctypes.byref(k), ctypes.byref(g), ctypes.byref(lb))
        return rc, k.value, g.value, lb.value, arr

    rc, k, g, lb, arr = prep(step(), step())
    assert rc == 0 and g == 2 * arr[0].tiles and 0 < lb <= 160 * 1024
    assert rc == 0 and arr[0].tiles == arr[1].tiles > 0
    assert prep(step(), step(ks=3))[0] == -2                     # a 3x3 member
    assert prep(step(), step(kind=1))[0] == -2                   # a BN-backward step
    assert prep(step(), step(B=32))[0] == -2                     # other pixels
    assert prep(step(B=64, H=32, W=32), step(B=64, H=32, W=32))[0] == -2   # M = 65536 > 16384
    assert prep(step(), step(dtype=1))[0] == -2                  # mixed dtypes
    assert prep(step(), step(x=fake + 4))[0] == -1               # misaligned operand
    assert prep(step(), step(x=0))[0] == -1                      # NULL operand
    assert prep(*[step() for _ in range(_lib.NET_GROUP_MAX + 1)])[0] == -1   # too many members
    # the wide-scale fan-out form (bf16, M > 16384, <= 64 channels, members
    # read the same input) -- also host-only: its grid is one wave per
    # 32-pixel tile, capped to the resident workgroups at launch
    wide = dict(B=64, H=32, W=32, cs=64, n=64, dtype=1)
    rc, k, g, lb, arr = prep(step(**wide), step(**wide))
    assert rc == 0 and k >> 12 == 1 and g == 64 * 32 * 32 // 128 and 0 < lb <= 64 * 1024
    assert prep(step(**wide), step(**dict(wide, x=fake + 256)))[0] == -2   # members read different inputs


def test_factor_out_refuses_non_canonical_order_matrix():
    """factor_out / restore implement order_matrix(C)'s permutation; another
    0/1 kernel (which the reference would convolve with,
    flow_realnvp.py:167-193) is refused instead of silently differing"""
    import flow_realnvp
    m = flow_realnvp.RealNVP(3, 16, torch.distributions.Normal(torch.tensor(0.), torch.tensor(1.)), _hp(4, 1))
    x = torch.zeros(2, 3, 16, 16)
    bad = m.order_matrix_1.clone()
    bad[0, 0, 0, 0], bad[0, 0, 1, 1] = 0.0, 1.0
    with pytest.raises(ValueError, match="canonical"):
        m.factor_out(x, bad)
    half = torch.zeros(2, 6, 8, 8)
    with pytest.raises(ValueError, match="canonical"):
        m.restore(half, half, bad)
    with pytest.raises(ValueError, match="shape"):
        m.factor_out(x, m.order_matrix(6))
    # the canonical matrix passes the check (then the CPU tensor is refused)
    with pytest.raises(RuntimeError, match="HIP device"):
        m.factor_out(x, m.order_matrix_1)
