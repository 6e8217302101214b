"""Graph-replayed generation (realnvp_hip.sampler.FlowSampler) against the
reference's sampling path: RealNVP.g on a fixed latent (golden sample_x,
flow_realnvp.py:196-249) and the drop-in's own eager g + logit reverse
(train.py:253-259)."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from formula_init import formula_state

pytestmark = pytest.mark.gpu
DEV = "cuda"


def make_model(size, bd, rb):
    import flow_realnvp
    import utils
    prior = torch.distributions.Normal(torch.tensor(0.0, device=DEV), torch.tensor(1.0, device=DEV))
    m = flow_realnvp.RealNVP(3, size, prior, utils.Hyperparameters(bd, rb, True, True, True, True))
    m.load_state_dict(formula_state(m))
    return m.to(DEV)


@pytest.mark.parametrize("name,size,bd,rb", [("m32_d8_r1", 32, 8, 1), ("m64_d32_r4", 64, 32, 4)])
def test_sampler_matches_reference_g(name, size, bd, rb):
    from realnvp_hip.sampler import FlowSampler
    g = load_golden("model_%s.npz" % name)
    model = make_model(size, bd, rb)
    # the golden's eval-mode g ran after two train-mode passes (forward and f:
    # running statistics updated twice, tools/make_goldens.py:model_goldens)
    model.train()
    with torch.no_grad():
        model(torch.from_numpy(g["x"]).to(DEV))
        model.f(torch.from_numpy(g["x"]).to(DEV))
    model.eval()
    z = torch.from_numpy(g["sample_z"]).to(DEV)
    s = FlowSampler(model, z.shape[0], logit_reverse=False)
    x = s.sample(z=z).cpu().numpy()
    rel = np.linalg.norm(x - g["sample_x"]) / np.linalg.norm(g["sample_x"])
    assert rel < 1e-4, rel


def test_sampler_graph_replay_equals_eager_path():
    import utils
    from realnvp_hip.sampler import FlowSampler
    model = make_model(32, 8, 1).eval()
    s = FlowSampler(model, 16)
    a = s.sample().clone()
    za = s.z.clone()
    b = s.sample().clone()
    assert not torch.equal(s.z, za)            # a fresh N(0,1) draw per replay
    # logit reverse maps sigmoid's (0, 1) onto ((1 - 1/0.9)/2, (1 + 1/0.9)/2) (utils.py:34-42)
    lo, hi = (1 - 1 / 0.9) / 2, (1 + 1 / 0.9) / 2
    assert bool(((a > lo) & (a < hi)).all()) and bool(torch.isfinite(b).all())
    with torch.no_grad():
        ref, _ = utils.logit_transform(model.g(za), reverse=True)
    assert float((a - ref).abs().max()) < 1e-5
    with pytest.raises(RuntimeError):
        FlowSampler(model.train(), 4)


def test_sampler_built_before_trainer_follows_moved_weights():
    """a FlowSampler captured before a FlowTrainer re-points the
    parameters into its flat arena (which makes the engines rebuild, and free,
    their packed-weight arenas) rebuilds its weight-norm table and graph on
    the next call instead of writing into freed memory; its samples then
    match the eager inverse of the current weights."""
    import utils
    from realnvp_hip.sampler import FlowSampler
    from realnvp_hip.trainer import FlowTrainer
    model = make_model(32, 8, 1).eval()
    s = FlowSampler(model, 8)
    s.sample()
    key0 = s._wkey
    model.train()
    tr = FlowTrainer(model, 4, dtype="fp32")
    from formula_init import pixels
    tr.set_pixels(pixels(4, 3, 32, seed=2).to(DEV))
    tr.step()
    model.eval()
    model.set_precision(s.dtype)
    a = s.sample().clone()
    assert s._wkey != key0
    with torch.no_grad():
        ref, _ = utils.logit_transform(model.g(s.z.clone()), reverse=True)
    assert float((a - ref).abs().max()) < 1e-5


def test_reverse_without_no_grad_on_a_trainable_model():
    """The reference's g() works without torch.no_grad() on a model whose
    parameters require grad, and is differentiable there (plain torch,
    modules_realnvp.py:284-291): the engine's inverse too -- same values as
    under no_grad, outputs that carry a gradient, an input that requires grad
    accepted (the gradients themselves: tests/test_gpu_reverse.py)."""
    model = make_model(32, 8, 1).eval()
    z = torch.randn(2, 3, 32, 32, device=DEV)
    x = model.g(z)
    with torch.no_grad():
        ref = model.g(z)
    assert x.requires_grad and torch.equal(x.detach(), ref)
    mod = next(model.couplings())
    y, _ = mod(torch.randn(2, 3, 32, 32, device=DEV, requires_grad=True), reverse=True)
    y.sum().backward()
