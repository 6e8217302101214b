"""float64 truths for the deep / large goldens (build container; test infrastructure).

    python tools/make_fp64_refs.py [name ...]   # writes tests/golden/fp64_<name>.npz

The reference runs in fp32; through R=8 nets and 923 M parameters its own
rounding noise on gradients is larger than the fp32 tolerances used for the
shallow goldens.  The tests therefore anchor gradients on the CPU oracle
evaluated in float64 (oracle/realnvp_oracle.py, pinned to the reference by
tests/test_oracle_golden.py) and accept the engine's fp32 result when it is
as close to that truth as the reference's own fp32 result is (x3), as
tests/test_gpu_parity.py does for the shallow models.  Inputs and weights
are the goldens' (formula init, same seeds).
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import realnvp_oracle as O  # noqa: E402
from formula_init import chirp_value, formula_value, pixels, uniform_noise  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
torch.set_num_threads(8)


def f64_state(entries, value=formula_value):
    return {k: (v.double() if v.is_floating_point() else v) for k, v in O.build_state(entries, value).items()}


def coupling(name, kind, cio, mid, hk):
    g = np.load(os.path.join(OUT, "coupling_%s.npz" % name))
    hp = O.HP(**hk)
    entries = O.coupling_spec("", kind, cio, mid, hp)
    S = f64_state(entries, chirp_value if "_r8_" in name else formula_value)
    train = O.trainable_names(entries)
    for n in train:
        S[n].requires_grad_(True)
    fn = O.checkerboard_coupling if kind == "ckbd" else O.channelwise_coupling
    x = torch.from_numpy(g["x"]).double().requires_grad_(True)
    y, ldj = fn(S, "", x, float(name.endswith("cfg1")), hp, training=True)
    loss = (y * torch.from_numpy(g["gy"]).double() + ldj * torch.from_numpy(g["gl"]).double()).sum()
    grads = torch.autograd.grad(loss, [x] + [S[n] for n in train])
    d = dict(grad_x=grads[0].numpy(), grad_names=np.array(train),
             grad_norms=np.array([float(t.norm()) for t in grads[1:]]))
    for n, t in zip(train, grads[1:]):
        if "grad." + n in g.files:      # the golden's full tensors, in fp64
            d["grad." + n] = t.float().numpy()   # fp64 truth rounded to fp32 (6e-8)
    np.savez_compressed(os.path.join(OUT, "fp64_coupling_%s.npz" % name), **d)


def model(name, size, bd, rb, B):
    t0 = time.time()
    spec = O.FlowSpec(3, size, O.HP(bd, rb))
    entries = O.flow_spec_entries(spec)
    S = f64_state(entries)
    train = O.trainable_names(entries)
    names = O.param_names(entries)
    for n in train:
        S[n].requires_grad_(True)
    pix = pixels(B, 3, size, seed=10)
    noise = uniform_noise(B, 3, size, seed=11)
    x, logdet = O.logit_transform(pix, noise)
    x = x.double().requires_grad_(True)
    lp = O.log_prob(S, spec, x, training=True)
    ws = O.weight_scale(S, names, lambda n: n in set(train))
    loss = -(lp + logdet.double()).mean() + O.SCALE_REG * ws
    grads = torch.autograd.grad(loss, [x] + [S[n] for n in train])
    d = dict(train_logprob=lp.detach().numpy(), grad_x_norm=np.array(float(grads[0].norm())),
             grad_names=np.array(train), grad_norms=np.array([float(t.norm()) for t in grads[1:]]))
    np.savez_compressed(os.path.join(OUT, "fp64_model_%s.npz" % name), **d)
    print(name, "took %.1fs" % (time.time() - t0))


CASES = {
    "ckbd_c3_m64_s32_r8_cfg1": lambda: coupling("ckbd_c3_m64_s32_r8_cfg1", "ckbd", 3, 64, dict(base_dim=64, res_blocks=8)),
    "chan_c96_m1024_s2_r8_cfg0": lambda: coupling("chan_c96_m1024_s2_r8_cfg0", "chan", 96, 1024,
                                                  dict(base_dim=64, res_blocks=8)),
    "m64_d32_r4_b64": lambda: model("m64_d32_r4_b64", 64, 32, 4, 64),
    "m32_d64_r8": lambda: model("m32_d64_r8", 32, 64, 8, 2),
}

if __name__ == "__main__":
    for k in (sys.argv[1:] or list(CASES)):
        CASES[k]()
