"""ctypes binding of include/realnvp_hip.h (the C ABI of the HIP engine).

The shared object is built in-tree (``csrc/Makefile`` -> ``librealnvp_hip.so``
next to this file).  There is no fallback: if the library is missing or a
call fails, a RuntimeError is raised.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RNVP_LIB_PATH: a probe build of the same library (tools/, timing experiments);
# announced on stderr, and refused at load when its structs differ (rnvp_struct_size)
LIB_PATH = os.environ.get("RNVP_LIB_PATH") or os.path.join(_HERE, "librealnvp_hip.so")
if os.environ.get("RNVP_LIB_PATH"):
    import sys as _sys
    print("realnvp_hip: RNVP_LIB_PATH=%s replaces the in-tree library" % LIB_PATH, file=_sys.stderr)

RNVP_F32, RNVP_BF16 = 0, 1

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_longlong
f32 = C.c_float
f64 = C.c_double


class BNSrc(C.Structure):
    _fields_ = [("sums", vp), ("count", f64), ("mean", vp), ("var", vp), ("gamma", vp), ("beta", vp), ("eps", f32),
                ("shards", i32)]


class BNRunning(C.Structure):
    _fields_ = [("sums", vp), ("count", f64), ("C", i32), ("shards", i32), ("rmean", vp), ("rvar", vp), ("nbt", vp)]


class ConvArgs(C.Structure):
    _fields_ = [("dtype", i32), ("B", i32), ("H", i32), ("W", i32), ("ks", i32),
                ("x", vp), ("cs_in", i32), ("cin", i32),
                ("w", vp), ("kp", i32),
                ("y", vp), ("cs_out", i32), ("n", i32),
                ("bias", vp), ("residual", vp), ("accumulate", i32),
                ("pro_bn_relu", i32), ("pro", BNSrc),
                ("out_sums", vp),
                ("epi_relu_bn_bwd", i32), ("epi_x", vp), ("epi", BNSrc), ("epi_sums", vp),
                ("ws", vp), ("ws_elems", i64), ("variant", i32), ("w_frag", vp),
                ("bp", i32), ("bp_x", vp), ("bp_bn", BNSrc), ("bp_sums", vp), ("bp_shards", i32),
                ("bp_out", vp), ("bp_dgamma", vp), ("bp_dbeta", vp)]


class BNBwdArgs(C.Structure):
    _fields_ = [("dtype", i32), ("M", i64), ("C", i32), ("cs", i32),
                ("g", vp), ("x", vp), ("bn", BNSrc), ("sums", vp), ("sum_shards", i32),
                ("dx", vp), ("residual", vp), ("accumulate", i32),
                ("dgamma", vp), ("dbeta", vp)]


RNVP_STEP_CONV, RNVP_STEP_BN_BWD = 0, 1
NET_GROUP_MAX = 8


class NetStep(C.Structure):
    _fields_ = [("kind", i32), ("conv", ConvArgs), ("bn", BNBwdArgs), ("dgamma_off", i64), ("dbeta_off", i64),
                ("cfg", i32), ("nc", i32), ("shards", i32), ("xa", i32), ("xb", i32), ("tiles", i32)]


class WNDesc(C.Structure):
    _fields_ = [("v", vp), ("g", vp), ("wf", vp), ("wd", vp), ("norm", vp),
                ("dw", vp), ("dv_off", i64), ("dg_off", i64),
                ("cout", i32), ("cin", i32), ("ks", i32), ("cs_in", i32), ("kp_f", i32),
                ("cs_out", i32), ("kp_d", i32), ("row0", i32), ("tile0", i32),
                ("nz", i32), ("dbp", vp), ("db_off", i64), ("zero_after", i32), ("blk0", i32),
                ("wf_frag", vp), ("wd_frag", vp)]


class Range(C.Structure):
    _fields_ = [("p", vp), ("bytes", i64)]


class AdamArgs(C.Structure):
    _fields_ = [("param", vp), ("grad", vp), ("exp_avg", vp), ("exp_avg_sq", vp), ("mask", vp),
                ("step", vp), ("step_add", i64),
                ("lr", f32), ("beta1", f32), ("beta2", f32), ("eps", f32), ("weight_decay", f32),
                ("reg_coef", f32)]


WGRAD_GROUP_MAX = 24


class WgradConv(C.Structure):
    _fields_ = [("x", vp), ("dy", vp), ("ws", vp), ("wsb", vp), ("pro", BNSrc),
                ("cs_in", i32), ("cin", i32), ("ks", i32), ("cs_dy", i32), ("n", i32), ("kp", i32),
                ("pro_bn_relu", i32), ("nz", i32), ("nrep", i32), ("m_per_slab", i64), ("task0", i32),
                ("tk", i32), ("cls", i32)]


class WgradGroup(C.Structure):
    _fields_ = [("dtype", i32), ("B", i32), ("H", i32), ("W", i32), ("n_conv", i32),
                ("conv", WgradConv * WGRAD_GROUP_MAX)]


class CouplingArgs(C.Structure):
    _fields_ = [("kind", i32), ("B", i32), ("C", i32), ("H", i32), ("W", i32), ("mask_config", i32),
                ("coupling_bn", i32), ("training", i32), ("dtype", i32),
                ("momentum", f32), ("eps", f32),
                ("x", vp),
                ("in_gamma", vp), ("in_beta", vp), ("in_rmean", vp), ("in_rvar", vp), ("in_nbt", vp),
                ("in_sums", vp),
                ("h0", vp), ("cs_h0", i32),
                ("st", vp), ("cs_st", i32),
                ("scale", vp), ("scale_shift", vp),
                ("u", vp), ("z", vp), ("out_sums", vp),
                ("out_rmean", vp), ("out_rvar", vp), ("out_nbt", vp),
                ("ldj_sample", vp), ("ldj_full", vp),
                ("gz", vp), ("gl_full", vp), ("gl_sample", vp), ("gx", vp),
                ("gst", vp), ("cs_gst", i32),
                ("bwd_sums", vp), ("g_scale", vp), ("g_scale_shift", vp),
                ("gh0", vp), ("cs_gh0", i32),
                ("in_bwd_sums", vp), ("g_in_gamma", vp), ("g_in_beta", vp),
                ("net_running", vp), ("n_net_running", i32), ("net_running_cmax", i32),
                ("gscale_part", vp),
                ("nclass", i32), ("cls_sums", vp), ("prior_sums", vp), ("outp_sums", vp), ("in_bwd_ext", vp),
                ("out_tab", vp), ("in_tab", vp)]


RNVP_LINK_SAME, RNVP_LINK_SQUEEZE, RNVP_LINK_UNFACTOR, RNVP_LINK_FINAL = 0, 1, 2, 3


class LinkArgs(C.Structure):
    _fields_ = [("type", i32), ("g_lp", vp), ("prior", vp), ("off", vp), ("z", vp)]


class TensorRef(C.Structure):
    _fields_ = [("p", vp), ("g", vp), ("n", i64)]


_SIGS = {
    "rnvp_version": (i32, []),
    "rnvp_struct_size": (i32, [i32]),
    "rnvp_status_string": (C.c_char_p, [i32]),
    "rnvp_marker": (i32, [i32, vp]),
    "rnvp_checkerboard_mask": (i32, [vp, i32, i32, vp]),
    "rnvp_squeeze": (i32, [vp, vp, i32, i32, i32, i32, vp]),
    "rnvp_undo_squeeze": (i32, [vp, vp, i32, i32, i32, i32, vp]),
    "rnvp_factor_out": (i32, [vp, vp, vp, i32, i32, i32, i32, vp]),
    "rnvp_restore": (i32, [vp, vp, vp, i32, i32, i32, i32, vp]),
    "rnvp_logit_fwd": (i32, [vp, vp, C.c_uint64, C.c_uint64, vp, f32, vp, vp, i32, i32, vp]),
    "rnvp_logit_inv": (i32, [vp, vp, f32, i64, vp]),
    "rnvp_u8_to_unit": (i32, [vp, vp, i64, vp]),
    "rnvp_nchw_to_nhwc": (i32, [vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "rnvp_nhwc_to_nchw": (i32, [vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "rnvp_prior_logprob": (i32, [vp, vp, vp, i32, i32, vp]),
    "rnvp_prior_logprob_bwd": (i32, [vp, vp, vp, i32, i32, vp]),
    "rnvp_bn_running_update": (i32, [vp, i32, i32, f32, vp]),
    "rnvp_stat_shards": (i32, [i64]),
    "rnvp_conv2d": (i32, [C.POINTER(ConvArgs), vp]),
    "rnvp_conv2d_check": (i32, [C.POINTER(ConvArgs)]),
    "rnvp_wgrad_slabs": (i32, [i64]),
    "rnvp_wgrad_replicas": (i32, [i32]),
    "rnvp_conv2d_wgrad_grouped": (i32, [C.POINTER(WgradGroup), vp]),
    "rnvp_bn_bwd_apply": (i32, [C.POINTER(BNBwdArgs), vp]),
    "rnvp_weight_norm_fwd": (i32, [vp, i32, i32, i32, i32, vp]),
    "rnvp_weight_norm_tiles": (i32, [i32, i32, i32]),
    "rnvp_weight_norm_bwd": (i32, [vp, i32, i32, vp, vp, i64, vp, i64, vp]),
    "rnvp_weight_norm_opt_blocks": (i32, [i32, i32, i32]),
    "rnvp_weight_norm_bwd_adam": (i32, [vp, i32, i32, i32, i32, C.POINTER(AdamArgs), vp, i64, vp, i64, vp]),
    "rnvp_adam_gather": (i32, [C.POINTER(AdamArgs), vp, i64, vp]),
    "rnvp_weight_norm_transpose": (i32, [vp, i32, i32, i32, vp]),
    "rnvp_zero_ranges": (i32, [vp, i32, i64, vp]),
    "rnvp_coupling_in_fwd": (i32, [C.POINTER(CouplingArgs), vp]),
    "rnvp_coupling_out_fwd": (i32, [C.POINTER(CouplingArgs), vp]),
    "rnvp_coupling_reverse": (i32, [C.POINTER(CouplingArgs), vp]),
    "rnvp_coupling_reverse_bwd": (i32, [C.POINTER(CouplingArgs), vp]),
    "rnvp_coupling_out_bwd": (i32, [C.POINTER(CouplingArgs), vp]),
    "rnvp_coupling_in_bwd": (i32, [C.POINTER(CouplingArgs), vp]),
    "rnvp_link_nclass": (i32, [i32, i32]),
    "rnvp_coupling_out_u": (i32, [C.POINTER(CouplingArgs), vp]),
    "rnvp_coupling_link_fwd": (i32, [C.POINTER(CouplingArgs), C.POINTER(CouplingArgs), C.POINTER(LinkArgs), vp]),
    "rnvp_coupling_link_bwd": (i32, [C.POINTER(CouplingArgs), C.POINTER(CouplingArgs), C.POINTER(LinkArgs), vp]),
    "rnvp_coupling_in_apply": (i32, [C.POINTER(CouplingArgs), vp]),
    "rnvp_flow_in_fwd": (i32, [vp, C.c_uint64, vp, f32, vp, vp, C.POINTER(CouplingArgs), i32, i32, i32, i32, vp]),
    "rnvp_flow_lp_finish": (i32, [vp, vp, vp, i32, vp, vp, i32, vp]),
    "rnvp_sumsq_multi": (i32, [vp, i32, vp, vp]),
    "rnvp_sumsq_bwd_multi": (i32, [vp, i32, vp, f32, vp]),
    "rnvp_adam_step": (i32, [vp, vp, vp, vp, i64, vp, f32, f32, f32, f32, f32, vp, f32, vp]),
    "rnvp_adam_update": (i32, [vp, vp, vp, vp, i64, vp, i64, f32, f32, f32, f32, f32, vp, f32, vp]),
    "rnvp_step_increment": (i32, [vp, vp]),
    "rnvp_fill_f64": (i32, [vp, i64, f64, vp]),
    "rnvp_net_group_prepare": (i32, [vp, i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]),
    "rnvp_net_group": (i32, [vp, i32, i32, i32, i32, i32, vp]),
}

EXPORTED = sorted(_SIGS)


class _Lib:
    def __init__(self, path=LIB_PATH):
        if not os.path.exists(path):
            raise RuntimeError("librealnvp_hip.so not built (%s); run __graft_entry__.build()" % path)
        self.dll = C.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(self.dll, name)
            fn.restype = res
            fn.argtypes = args
            raw = name in ("rnvp_version", "rnvp_struct_size", "rnvp_stat_shards", "rnvp_wgrad_slabs", "rnvp_wgrad_replicas",
                           "rnvp_link_nclass", "rnvp_conv2d_check",
                           "rnvp_weight_norm_tiles", "rnvp_weight_norm_opt_blocks",
                           "rnvp_net_group_prepare") or res is not i32
            setattr(self, name[len("rnvp_"):], fn if raw else self._wrap(name, fn))
        # the struct mirrors must match the library's layouts (rnvp_struct_size): a
        # table read at another stride would address arbitrary device memory
        mirrors = (BNSrc, BNRunning, ConvArgs, WgradConv, WgradGroup, BNBwdArgs, WNDesc, AdamArgs, CouplingArgs,
                   NetStep, Range, LinkArgs)
        for i, m in enumerate(mirrors):
            if self.dll.rnvp_struct_size(i) != C.sizeof(m):
                raise RuntimeError("%s: struct %s is %d bytes in the library, %d in the binding (stale build?)"
                                   % (path, m.__name__, self.dll.rnvp_struct_size(i), C.sizeof(m)))

    def _wrap(self, name, fn):
        dll = self.dll

        def call(*args):
            st = fn(*args)
            if st != 0:
                msg = dll.rnvp_status_string(st)
                raise RuntimeError("%s failed: status %d (%s)" % (name, st, msg.decode() if msg else "?"))
        call.__name__ = name
        return call


_lib = None


def lib() -> _Lib:
    global _lib
    if _lib is None:
        _lib = _Lib()
    return _lib
