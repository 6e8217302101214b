"""The BatchNorm-backward fold's launch plan, built on the host (no GPU): the
engine's data-gradient program with engine.FOLD_BN on and off
(realnvp_hip/engine.py _bwd_args / _fold_bn; rnvp_conv2d_check answers the
library's side without launching).

Checks, per coupling shape: which applies fold (the residual blocks'
res_block.1 / res_block.4 where the consumer's kernel has the prologue, never
an accumulating or multi-reader apply), that a folded conv is wired to the
apply's operands (g -> x, the BatchNorm input -> bp_x, its statistics and
gradient sums, the applied gradient's buffer -> bp_out), and that the two
pre-apply temps alternate safely: no launch reads and writes the same temp,
every temp read sees the write issued for it, and the applied gradients that
other launches read are still produced (by the apply or as the side output).
"""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dl-normalizing-flows_amd"))

CASES = [
    # kind, in_out_dim, mid, size, batch, dtype, expected folds (4 residual blocks)
    ("ckbd", 48, 512, 4, 64, "bf16", 8),     # s5: 8-wave tiles, 1x1 and 3x3
    ("ckbd", 48, 512, 4, 64, "fp32", 4),     # fp32 3x3 at 512 channels: no LDS for the fold's table
    ("ckbd", 24, 256, 8, 64, "bf16", 8),     # s4: 3x3 + 4-wave 1x1 (M = 4096)
    ("chan", 96, 512, 4, 64, "bf16", 8),
    ("ckbd", 12, 128, 16, 64, "bf16", 4),    # s3: 3x3 only (16384-pixel 1x1 keeps its apply)
    ("ckbd", 6, 64, 32, 64, "bf16", 8),      # s2: the streaming 1x1 and the band 3x3
    ("ckbd", 6, 64, 32, 64, "fp32", 0),      # (bf16 only)
    ("ckbd", 3, 32, 64, 16, "bf16", 8),      # s1
]


def _plan(kind, cio, mid, size, B, dtype, fold):
    import modules_realnvp as MR
    import utils
    from realnvp_hip import engine as E
    hp = utils.Hyperparameters(32, 4, True, True, True, True)
    torch.manual_seed(0)
    mod = MR.CheckerboardAffineCoupling(cio, mid, size, 1.0, hp) if kind == "ckbd" else \
        MR.ChannelwiseAffineCoupling(cio, mid, 0.0, hp)
    eng = mod.engine()
    cpu = torch.device("cpu")
    ws = eng.weights(dtype)
    sv = eng.alloc_saved(B, size, size, dtype, cpu, True)
    sc = eng.scratch(B, size, size, dtype, cpu)
    old = E.FOLD_BN
    E.FOLD_BN = fold
    try:
        items = eng._bwd_args(eng._tensors(), sv, sc, ws, True)[0]
    finally:
        E.FOLD_BN = old
    return eng, sv, sc, items


@pytest.mark.parametrize("case", CASES, ids=["%s_c%d_m%d_%s" % (c[0], c[1], c[4] * c[3] ** 2, c[5]) for c in CASES])
def test_fold_plan(case):
    kind, cio, mid, size, B, dtype, want = case
    eng, sv, sc, items0 = _plan(kind, cio, mid, size, B, dtype, False)
    _, sv1, sc1, items = _plan(kind, cio, mid, size, B, dtype, True)
    folded = [it for it in items if it[0] == "dgrad" and it[4] is not None]
    assert len(folded) == want, [it[4] for it in folded]
    assert len(items) == len(items0) - want
    assert all(it[0] != "dgrad" or it[4] is None for it in items0)
    # only the residual blocks' inner BatchNorms fold
    assert all(it[4].split(".")[-2] in ("1", "4") and "res_block" in it[4] for it in folded)
    sar = sc1["arena"]
    tmps = {sar.ptr("gtmp"): "gtmp", sar.ptr("gtmp2"): "gtmp2"}
    applied = {n for it in items0 if it[0] == "bn" for n in it[5][1]}
    produced = set()
    pending = {}                                  # temp -> written and not yet read
    for kind_, c, nb, fl, bn, (reads, writes) in items:
        if kind_ == "dgrad":
            r_t = {t for t in ("gtmp", "gtmp2") if t in reads}
            w_t = {t for t in ("gtmp", "gtmp2") if t in writes}
            assert not (r_t & w_t), (bn, reads, writes)
            if bn is not None:
                assert c.bp == 1 and c.x in tmps and tmps[c.x] in reads
                assert c.bp_out and c.bp_out not in tmps and c.bp_x and c.bp_sums
                assert c.y not in (c.x,)
                # its side output is the applied gradient the unfolded apply wrote
                assert len(writes & applied) == 1
            else:
                assert c.bp == 0
            for t in r_t:
                assert pending.pop(t, None) is not None, ("temp read before its write", t, bn)
            for t in w_t:
                pending[t] = True
            if c.y in tmps:
                assert tmps[c.y] in writes
        else:
            t = tmps[c.g]
            assert t in reads and pending.pop(t, None) is not None, ("apply reads a stale temp", bn)
        produced |= writes
    assert not pending
    # every applied gradient of the unfolded program is still produced
    assert applied <= produced
