"""Static description of one coupling's s/t ResNet as a conv program.

Mirrors ResidualModule / ResidualBlock / WeightNormConv2d
(modules_realnvp.py:36-194): which convs exist, their shapes, the BatchNorm
that precedes each conv (fused into its operand load), residual adds and
skip accumulations (fused into its epilogue), and which BatchNorm's batch
statistics each epilogue produces.  The backward program is derived from the
forward one by reverse-mode over this small op graph.
"""
from dataclasses import dataclass, field
from typing import Dict, List, Optional


def round_up(x, m):
    return (x + m - 1) // m * m


def chan_stride(c):
    """NHWC channel stride: multiple of 8 (16 B of bf16 / 32 B of fp32)."""
    return round_up(max(c, 1), 8)


@dataclass
class ConvSpec:
    name: str          # param prefix, e.g. "block.1.in_block."
    cin: int
    cout: int
    ks: int
    bias: bool
    scale: bool        # trainable weight_g
    wn: bool           # weight-normalised (weight_g/weight_v) or plain weight


@dataclass
class BNSpec:
    name: str          # param prefix of the BatchNorm2d, e.g. "block.1.out_block.0."
    c: int


@dataclass
class ConvOp:
    conv: str                  # ConvSpec.name
    x: str                     # input activation buffer
    y: str                     # output activation buffer
    pro_bn: Optional[str]      # BN (+ReLU) applied to x on load
    residual: Optional[str]    # y = conv(...) + residual
    accumulate: bool           # y += conv(...)
    stats_bn: Optional[str]    # BN whose batch stats are taken from y's epilogue


@dataclass
class NetProgram:
    convs: Dict[str, ConvSpec] = field(default_factory=dict)
    bns: Dict[str, BNSpec] = field(default_factory=dict)
    ops: List[ConvOp] = field(default_factory=list)
    buf_ch: Dict[str, int] = field(default_factory=dict)   # activation buffer -> channels
    input: str = "h0"
    output: str = "st"

    def add_conv(self, name, cin, cout, ks, bias, scale, wn):
        self.convs[name] = ConvSpec(name, cin, cout, ks, bias, scale, wn)

    def add_bn(self, name, c):
        self.bns[name] = BNSpec(name, c)


def build_program(p: str, cin: int, dim: int, cout: int, res_blocks: int, bottleneck: bool, skip: bool,
                  weight_norm: bool) -> NetProgram:
    """ResidualModule(in_dim=cin, dim, out_dim=cout, ...) with param prefix p."""
    P = NetProgram()
    P.buf_ch["h0"] = cin
    wn = weight_norm

    def op(conv, x, y, pro=None, res=None, acc=False, stats=None):
        P.ops.append(ConvOp(conv, x, y, pro, res, acc, stats))

    if res_blocks > 0:
        P.add_conv(p + "in_block.", cin, dim, 3, True, False, wn)
        if skip:
            P.add_conv(p + "in_skip.", dim, dim, 1, True, True, wn)
        for i in range(res_blocks):
            q = p + "core_block.%d." % i
            P.add_bn(q + "in_block.0.", dim)
            r = q + "res_block."
            if bottleneck:
                P.add_conv(r + "0.", dim, dim, 1, False, False, wn)
                P.add_bn(r + "1.", dim)
                P.add_conv(r + "3.", dim, dim, 3, False, False, wn)
                P.add_bn(r + "4.", dim)
                P.add_conv(r + "6.", dim, dim, 1, True, True, wn)
            else:
                P.add_conv(r + "0.", dim, dim, 3, False, False, wn)
                P.add_bn(r + "1.", dim)
                P.add_conv(r + "3.", dim, dim, 3, True, True, wn)
            if skip:
                P.add_conv(p + "core_skips.%d." % i, dim, dim, 1, True, True, wn)
        P.add_bn(p + "out_block.0.", dim)
        P.add_conv(p + "out_block.2.", dim, cout, 1, True, True, wn)

        bn_a = lambda i: p + "core_block.%d.in_block.0." % i  # noqa: E731
        out_bn = p + "out_block.0."
        for i in range(res_blocks + 1):
            P.buf_ch["x1_%d" % i] = dim
        P.buf_ch["out"] = dim
        P.buf_ch["st"] = cout
        op(p + "in_block.", "h0", "x1_0", stats=bn_a(0))
        if skip:
            op(p + "in_skip.", "x1_0", "out")
        for i in range(res_blocks):
            q = p + "core_block.%d." % i
            r = q + "res_block."
            last = i == res_blocks - 1
            nxt = out_bn if (last and not skip) else (bn_a(i + 1) if not last else None)
            P.buf_ch["t1_%d" % i] = dim
            if bottleneck:
                P.buf_ch["t2_%d" % i] = dim
                op(r + "0.", "x1_%d" % i, "t1_%d" % i, pro=bn_a(i), stats=r + "1.")
                op(r + "3.", "t1_%d" % i, "t2_%d" % i, pro=r + "1.", stats=r + "4.")
                op(r + "6.", "t2_%d" % i, "x1_%d" % (i + 1), pro=r + "4.", res="x1_%d" % i, stats=nxt)
            else:
                op(r + "0.", "x1_%d" % i, "t1_%d" % i, pro=bn_a(i), stats=r + "1.")
                op(r + "3.", "t1_%d" % i, "x1_%d" % (i + 1), pro=r + "1.", res="x1_%d" % i, stats=nxt)
            if skip:
                op(p + "core_skips.%d." % i, "x1_%d" % (i + 1), "out", acc=True, stats=out_bn if last else None)
        src = "out" if skip else "x1_%d" % res_blocks
        op(p + "out_block.2.", src, "st", pro=out_bn)
        if not skip:
            del P.buf_ch["out"]
    else:
        b = p + "block."
        P.buf_ch["t1"] = dim
        P.buf_ch["st"] = cout
        if bottleneck:
            P.add_conv(b + "0.", cin, dim, 1, False, False, wn)
            P.add_bn(b + "1.", dim)
            P.add_conv(b + "3.", dim, dim, 3, False, False, wn)
            P.add_bn(b + "4.", dim)
            P.add_conv(b + "6.", dim, cout, 1, True, True, wn)
            P.buf_ch["t2"] = dim
            op(b + "0.", "h0", "t1", stats=b + "1.")
            op(b + "3.", "t1", "t2", pro=b + "1.", stats=b + "4.")
            op(b + "6.", "t2", "st", pro=b + "4.")
        else:
            P.add_conv(b + "0.", cin, dim, 3, False, False, wn)
            P.add_bn(b + "1.", dim)
            P.add_conv(b + "3.", dim, cout, 3, True, True, wn)
            op(b + "0.", "h0", "t1", stats=b + "1.")
            op(b + "3.", "t1", "st", pro=b + "1.")
    return P


@dataclass
class BwdStep:
    kind: str                      # "dgrad" | "bn_apply" | "wgrad"
    op: ConvOp
    gy: str                        # gradient buffer of op.y
    gx: Optional[str] = None       # destination gradient buffer (dgrad/bn_apply)
    tmp: Optional[str] = None      # pre-BN-apply gradient (dgrad with relu+BN epilogue)
    accumulate: bool = False
    residual: Optional[str] = None  # pending residual gradient folded into this write


def backward_program(P: NetProgram) -> List[BwdStep]:
    """Reverse-mode over P.ops.  Gradient buffers are named "g:" + buffer.
    Handles: residual adds (folded into the next write of the residual's
    gradient), skip accumulations (identity), BN+ReLU prologues (dgrad with a
    relu/BN-statistics epilogue into "gtmp", then BN apply)."""
    steps: List[BwdStep] = []
    written = set()
    pending: Dict[str, str] = {}

    def write(dst):
        """(accumulate, residual) flags for the next write into dst."""
        acc = dst in written
        res = pending.pop(dst, None)
        written.add(dst)
        return acc, res

    order = list(reversed(P.ops))
    if "out" in P.buf_ch:
        # skip architecture: once the out_block's backward has made d out
        # complete, the data gradients of in_skip and every core_skips[i]
        # (all read d out) come next -- independent of each other, so the
        # engine runs them as one grouped launch; the blocks' chain follows
        # and accumulates onto what they wrote
        head = [op for op in order if op.x == "out"]
        skips = [op for op in order if op.y == "out"]
        order = head + skips + [op for op in order if op.x != "out" and op.y != "out"]
    for op in order:
        gy = "g:" + op.y
        gx = "g:" + op.x
        if op.residual is not None:
            # folded into the NEXT write of the residual's gradient (a first
            # write or an accumulation: with the skip data gradients hoisted,
            # g:x1_i already holds core_skips[i-1]'s part when block i's
            # residual is registered); gy is complete by then
            gr = "g:" + op.residual
            if gr in pending:
                raise NotImplementedError("two residuals into one gradient")
            pending[gr] = gy
        if op.pro_bn is not None:
            steps.append(BwdStep("dgrad", op, gy, gx=None, tmp="gtmp"))
            acc, res = write(gx)
            steps.append(BwdStep("bn_apply", op, gy, gx=gx, tmp="gtmp", accumulate=acc, residual=res))
        else:
            acc, res = write(gx)
            steps.append(BwdStep("dgrad", op, gy, gx=gx, accumulate=acc, residual=res))
        steps.append(BwdStep("wgrad", op, gy))
    if pending:
        raise NotImplementedError("unconsumed residual gradients: %s" % pending)
    return steps
