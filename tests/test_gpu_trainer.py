"""The fused training step (realnvp_hip.trainer) against the reference
trajectory and against itself under HIP-graph replay."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from formula_init import formula_state, pixels, uniform_noise

pytestmark = pytest.mark.gpu
DEV = "cuda"


def make_model(size, bd, rb):
    import flow_realnvp
    import utils
    prior = torch.distributions.Normal(torch.tensor(0.0, device=DEV), torch.tensor(1.0, device=DEV))
    m = flow_realnvp.RealNVP(3, size, prior, utils.Hyperparameters(bd, rb, True, True, True, True))
    m.load_state_dict(formula_state(m))
    return m.to(DEV)


def run_trajectory(graph):
    import utils
    from realnvp_hip.trainer import FlowTrainer
    g = load_golden("model_m32_d8_r1.npz")
    model = make_model(32, 8, 1)
    B = g["x"].shape[0]
    tr = FlowTrainer(model, B, dtype="fp32")
    lls = []
    for s in range(len(g["traj_loss"])):
        x, ld = utils.logit_transform(pixels(B, 3, 32, seed=100 + s), noise=uniform_noise(B, 3, 32, seed=200 + s))
        tr.set_input(x, ld)
        tr.reset_metrics()
        if graph and tr.graph is None:
            # capture with the first batch; warm-up steps would move the weights,
            # so capture without warm-up on a copy of the state
            state = {k: v.clone() for k, v in model.state_dict().items()}
            tr.capture(warmup=1)
            model.load_state_dict(state)
            tr.reset_optimizer()
            tr.reset_metrics()
        tr.step()
        lls.append(tr.mean_logll(1))
    return tr, model, g, lls


@pytest.mark.parametrize("graph", [False, True], ids=["eager", "hipgraph"])
def test_trainer_matches_reference_loop(graph):
    tr, model, g, lls = run_trajectory(graph)
    # step 1 is a forward of identical weights; later steps carry Adam-amplified
    # fp32 noise of near-zero gradients (see test_gpu_parity)
    np.testing.assert_allclose(lls[0], g["traj_logll"][0], rtol=2e-5)
    np.testing.assert_allclose(lls, g["traj_logll"], rtol=1e-4)
    model.eval()
    with torch.no_grad():
        lp, _ = model(torch.from_numpy(g["x"]).to(DEV))
    # Adam amplifies fp32 noise of near-zero gradients (see test_gpu_parity)
    np.testing.assert_allclose(lp.cpu().numpy(), g["traj_eval_logprob_after"], rtol=5e-4)
    assert int(tr.step_t.item()) == len(g["traj_loss"])


def test_trainer_frozen_params_untouched_and_state_dict_views():
    from realnvp_hip.trainer import FlowTrainer
    model = make_model(32, 8, 1)
    frozen = {n: p.detach().clone() for n, p in model.named_parameters() if not p.requires_grad}
    tr = FlowTrainer(model, 4, dtype="bf16")
    tr.set_pixels(pixels(4, 3, 32, seed=3).to(DEV))
    for _ in range(2):
        tr.step()
    for n, p in model.named_parameters():
        if n in frozen:
            assert torch.equal(p.detach(), frozen[n]), n
        assert p.data_ptr() >= tr.param.data_ptr()   # parameters are arena views
    bpd = tr.bits_per_dim(tr.mean_logll(2))
    assert np.isfinite(bpd) and 3.0 < bpd < 12.0


def test_bench_config_step_bf16_graph():
    """Config 1 shape (64x64x3, R4, D32) at a small batch: graph replay runs and
    produces a finite, improving loss."""
    from realnvp_hip.trainer import FlowTrainer
    import flow_realnvp
    import utils
    torch.manual_seed(0)
    prior = torch.distributions.Normal(torch.tensor(0.0, device=DEV), torch.tensor(1.0, device=DEV))
    model = flow_realnvp.RealNVP(3, 64, prior, utils.Hyperparameters(32, 4, True, True, True, True)).to(DEV)
    tr = FlowTrainer(model, 8, dtype="bf16")
    tr.set_pixels(pixels(8, 3, 64, seed=0).to(DEV))
    tr.capture(warmup=1)
    tr.reset_metrics()
    for _ in range(3):
        tr.step()
    first = tr.mean_logll(3)
    tr.reset_metrics()
    for _ in range(10):
        tr.step()
    later = tr.mean_logll(10)
    assert np.isfinite(first) and np.isfinite(later)
    assert later > first      # same batch: log-likelihood goes up


def test_side_stream_overlap_matches_single_stream():
    """Weight gradients, late weight norm and per-coupling Adam on the side
    stream give the same step as the single-stream schedule.  Gradients and
    first moments are compared normwise (the grouped wgrad's replica atomics
    make the summation order vary run to run); parameters elementwise within
    Adam's per-step bound 2*lr (sign flips of near-zero gradients)."""
    from realnvp_hip.trainer import FlowTrainer
    res = []
    for overlap in (False, False, True):
        model = make_model(32, 8, 1)
        tr = FlowTrainer(model, 4, dtype="fp32", overlap=overlap)
        tr.set_pixels(pixels(4, 3, 32, seed=5).to(DEV))
        tr.step()
        torch.cuda.synchronize()
        first = tr.grad.clone()
        for _ in range(2):
            tr.step()
        torch.cuda.synchronize()
        res.append((tr.param.clone(), tr.grad.clone(), tr.exp_avg.clone(), int(tr.step_t.item()), tr.lr, first))
    (p0, g0, m0, s0, lr, f0), (pb, gb, mb, _, _, fb), (p1, g1, m1, s1, _, f1) = res
    assert s0 == s1 == 3

    def d(a, b):
        return float((a - b).norm() / b.norm())
    # step 1 sees identical parameters: only the atomics' summation order
    # differs (a race would be O(1))
    assert d(f1, f0) < max(1e-4, 8 * d(fb, f0)), (d(f1, f0), d(fb, f0))
    # after three Adam steps the run-to-run noise is amplified by sign flips of
    # near-zero gradients (measured 1.5e-4 .. 1.3e-3 between identical runs)
    tol_g = max(1e-2, 8 * d(gb, g0))
    tol_m = max(1e-2, 8 * d(mb, m0))
    assert d(g1, g0) < tol_g, (d(g1, g0), d(gb, g0))
    assert d(m1, m0) < tol_m, (d(m1, m0), d(mb, m0))
    assert float((p1 - p0).abs().max()) <= 3 * 2 * lr * 1.01
    assert d(p1, p0) < max(1e-3, 4 * d(pb, p0))


# ---------------------------------------------------------------------------
# data parallel path (process_group) on one GPU: world-size-1 RCCL group
@pytest.fixture(scope="module")
def nccl_world1():
    import os
    import socket
    import torch.distributed as dist
    if not dist.is_initialized():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield dist.group.WORLD
    dist.destroy_process_group()


def _one_step(model, pg=None, graph=False, **kw):
    from realnvp_hip.trainer import FlowTrainer
    tr = FlowTrainer(model, 4, dtype="fp32", process_group=pg, **kw)
    tr.set_pixels(pixels(4, 3, 32, seed=5).to(DEV))
    if graph:
        tr.capture(warmup=1)
    p0 = tr.param.clone()
    tr.step()
    torch.cuda.synchronize()
    return tr, p0


@pytest.mark.parametrize("side", [False, True], ids=["onestream", "sidestream"])
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "hipgraph"])
@pytest.mark.parametrize("comm", ["overlap", "split"])
def test_process_group_step_matches_single_process(nccl_world1, comm, graph, side):
    """The DP step (bucketed all-reduce on the communication stream during
    backward, or between the captured graphs) with a world-size-1 RCCL group
    equals the single-process step: same gradients (up to the replica
    atomics' summation order), same Adam update, same step counter.  With
    side=True the weight gradients run on the side stream and each bucket's
    all-reduce waits for them through an event (trainer.py _backward)."""
    ref, p0 = _one_step(make_model(32, 8, 1))
    ref2, _ = _one_step(make_model(32, 8, 1))
    tr, q0 = _one_step(make_model(32, 8, 1), pg=nccl_world1, graph=graph, comm=comm, bucket_mb=1, overlap=side)
    assert len(tr.buckets) > 1
    assert torch.equal(p0, q0)

    def d(a, b):
        return float((a - b).norm() / b.norm())
    assert d(tr.grad, ref.grad) < max(1e-4, 8 * d(ref2.grad, ref.grad))
    assert float((tr.param - ref.param).abs().max()) <= 2 * ref.lr * 1.01
    assert d(tr.param, ref.param) < max(1e-5, 4 * d(ref2.param, ref.param))
    assert int(tr.step_t.item()) == 1
    # the linked forward adds each coupling's per-sample log-det with fp32
    # atomics (their order varies run to run): the identical-run spread, 1e-5 floor
    ll, ll2 = ref.mean_logll(1), ref2.mean_logll(1)
    np.testing.assert_allclose(tr.mean_logll(1), ll, rtol=max(1e-5, 4 * abs(ll2 - ll) / abs(ll)))


def test_capture_issues_no_eager_collective(nccl_world1, monkeypatch):
    """capture() warm-up steps issue no all-reduce, and the captured ones go
    over the capture-only group: no eager collective can be on a watchdog's
    list while the capture is open (trainer._wait_collectives_retired)."""
    import realnvp_hip.dist as D
    from realnvp_hip.trainer import FlowTrainer
    calls = []
    real = D.average_slice

    def spy(flat, lo, hi, group=None, buf=None):
        calls.append((group, torch.cuda.is_current_stream_capturing()))
        return real(flat, lo, hi, group, buf)
    monkeypatch.setattr(D, "average_slice", spy)
    tr = FlowTrainer(make_model(32, 8, 1), 4, dtype="fp32", process_group=nccl_world1, bucket_mb=1)
    tr.set_pixels(pixels(4, 3, 32, seed=5).to(DEV))
    tr.capture(warmup=2)
    assert calls and all(cap and g is tr._cap_pg for g, cap in calls), calls
    with pytest.raises(ValueError):
        tr.capture(warmup=1, restore=False)


def test_process_group_bf16_reduction(nccl_world1):
    ref, _ = _one_step(make_model(32, 8, 1))
    tr, _ = _one_step(make_model(32, 8, 1), pg=nccl_world1, comm="overlap", reduce_dtype="bf16", bucket_mb=1)
    assert float((tr.grad - ref.grad).norm() / ref.grad.norm()) < 4e-3


# ---------------------------------------------------------------------------
def _batch(s, B=4, size=32):
    import utils
    return utils.logit_transform(pixels(B, 3, size, seed=300 + s), noise=uniform_noise(B, 3, size, seed=400 + s))


def _torch_step(model, opt, s):
    x, ld = _batch(s)
    opt.zero_grad()
    lp, ws = model(x)
    ll = (lp + ld).mean()
    loss = -ll + 5e-5 * ws
    loss.backward()
    opt.step()
    return float(ll)


def _trainer_step(tr, s):
    x, ld = _batch(s)
    tr.set_input(x, ld)
    tr.reset_metrics()
    tr.step()
    return tr.mean_logll(1)


def test_optimizer_checkpoint_roundtrip_with_torch_adam():
    """train.py:139-154, 249-250: the fused trainer's Adam state saved in
    torch.optim.Adam format continues the same trajectory inside the
    reference loop (torch Adam around the drop-in), and a torch Adam
    checkpoint continues inside the fused trainer."""
    from realnvp_hip.trainer import FlowTrainer
    ma = make_model(32, 8, 1)
    tr = FlowTrainer(ma, 4, dtype="fp32")
    for s in range(2):
        _trainer_step(tr, s)
    sd = tr.state_dict()
    st = sd["optimizer"]["state"]
    assert len(st) == sum(1 for p in ma.parameters() if p.requires_grad)
    assert all(float(v["step"]) == 2.0 for v in st.values())
    # -> torch Adam around a fresh drop-in model
    mb = make_model(32, 8, 1).train()
    mb.load_state_dict(sd["model"])
    opt = torch.optim.Adam(mb.parameters(), lr=5e-4, weight_decay=5e-5)
    opt.load_state_dict(sd["optimizer"])
    ll_t = _torch_step(mb, opt, 2)
    ll_f = _trainer_step(tr, 2)
    np.testing.assert_allclose(ll_f, ll_t, rtol=1e-5)
    pa = torch.cat([p.detach().reshape(-1) for p in ma.parameters()])
    pb = torch.cat([p.detach().reshape(-1) for p in mb.parameters()])
    assert float((pa - pb).abs().max()) <= 2 * 5e-4 * 1.01
    assert float((pa - pb).norm() / pb.norm()) < 1e-3
    # <- torch Adam state into a fresh fused trainer, one more step each
    _torch_step(mb, opt, 3)
    mc = make_model(32, 8, 1)
    tc = FlowTrainer(mc, 4, dtype="fp32")
    tc.load_state_dict({"model": mb.state_dict(), "optimizer": opt.state_dict()})
    assert int(tc.step_t.item()) == 4
    ll_t = _torch_step(mb, opt, 4)
    ll_f = _trainer_step(tc, 4)
    np.testing.assert_allclose(ll_f, ll_t, rtol=1e-5)
    pc = torch.cat([p.detach().reshape(-1) for p in mc.parameters()])
    pb = torch.cat([p.detach().reshape(-1) for p in mb.parameters()])
    assert float((pc - pb).abs().max()) <= 2 * 5e-4 * 1.01
    assert float((pc - pb).norm() / pb.norm()) < 1e-3


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_fused_adam_matches_torch_adam(dtype):
    """realnvp_hip.FusedAdam in the reference loop (train.py:134, 176-200:
    model(x), loss.backward(), optimizer.step()) against torch.optim.Adam on
    the same drop-in model: the same per-step log-likelihood and parameters
    after 3 steps -- bf16: the s/t net's gradients are deterministic, so the
    trajectories agree to the update's fp32 rounding; fp32: the grouped weight
    gradient adds slab partials with atomics, so gradients that are zero in
    exact arithmetic (conv biases before a BatchNorm) are rounding noise whose
    sign Adam turns into +-lr steps (bounded as in
    test_optimizer_checkpoint_roundtrip_with_torch_adam).  Then each
    optimizer's state_dict continues inside the other."""
    from realnvp_hip import FusedAdam
    ma, mb = make_model(32, 8, 1).train(), make_model(32, 8, 1).train()
    ma.set_precision(dtype)
    mb.set_precision(dtype)
    oa = torch.optim.Adam(ma.parameters(), lr=5e-4, weight_decay=5e-5)
    ob = FusedAdam(mb.parameters(), lr=5e-4, weight_decay=5e-5)
    assert isinstance(ob, torch.optim.Optimizer)

    def cmp(steps):
        pa = torch.cat([p.detach().reshape(-1) for p in ma.parameters()])
        pb = torch.cat([p.detach().reshape(-1) for p in mb.parameters()])
        assert float((pa - pb).abs().max()) <= steps * 2 * 5e-4 * 1.01
        assert float((pa - pb).norm() / pa.norm()) < (1e-6 if dtype == "bf16" else 1e-3)
    for s in range(3):
        la, lb = _torch_step(ma, oa, s), _torch_step(mb, ob, s)
        np.testing.assert_allclose(lb, la, rtol=1e-5)
    cmp(3)
    assert int(ob.step_t.item()) == 3
    # state dicts cross over: torch Adam's into FusedAdam and back
    sa, sb = oa.state_dict(), ob.state_dict()
    assert sorted(sa["state"]) == sorted(sb["state"])
    assert all(float(sb["state"][k]["step"]) == 3.0 for k in sa["state"])
    for name in ("exp_avg", "exp_avg_sq"):
        va = torch.cat([sa["state"][k][name].reshape(-1) for k in sorted(sa["state"])])
        vb = torch.cat([sb["state"][k][name].reshape(-1) for k in sorted(sa["state"])])
        assert float((va - vb).norm() / va.norm()) < (1e-4 if dtype == "bf16" else 2e-2), name
    ob.load_state_dict(sa)
    oa.load_state_dict(sb)
    with torch.no_grad():
        for p, q in zip(mb.parameters(), ma.parameters()):
            p.copy_(q)
    la, lb = _torch_step(ma, oa, 3), _torch_step(mb, ob, 3)
    np.testing.assert_allclose(lb, la, rtol=1e-5)
    cmp(1)


def test_capture_restores_state_and_fixes_input_mode():
    """capture() leaves parameters, moments, step counter and BN buffers as
    they were (ADVICE: warm-up steps used to train silently), and a graph
    captured for set_pixels() refuses set_input() batches."""
    from realnvp_hip.trainer import FlowTrainer
    model = make_model(32, 8, 1)
    tr = FlowTrainer(model, 4, dtype="fp32")
    tr.set_pixels(pixels(4, 3, 32, seed=1).to(DEV))
    p0, rv0 = tr.param.clone(), {n: b.clone() for n, b in model.named_buffers()}
    assert tr.capture(warmup=2) == 2
    assert torch.equal(tr.param, p0) and int(tr.step_t.item()) == 0
    assert all(torch.equal(b, rv0[n]) for n, b in model.named_buffers())
    x, ld = _batch(0)
    with pytest.raises(RuntimeError):
        tr.set_input(x, ld)
    tr.drop_graph()
    tr.set_input(x, ld)
    tr.step()
    assert int(tr.step_t.item()) == 1


# ---------------------------------------------------------------------------
# data parallel path at world size 2: two ranks on the one GPU over gloo
# (RCCL needs one GPU per rank; gloo reduces device tensors through the host).
# Each rank trains on its own batch shard; the all-reduced gradient must be
# the mean of the two single-process gradients and both ranks must take the
# same Adam step.
def _dp_rank(rank, port, comm, out, side=False):
    import os
    import sys
    import torch.distributed as dist
    from conftest import PKG
    sys.path.insert(0, PKG)
    from realnvp_hip.trainer import FlowTrainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        tr = FlowTrainer(make_model(32, 8, 1), 4, dtype="fp32", process_group=dist.group.WORLD, comm=comm,
                         bucket_mb=1, overlap=side)
        tr.set_pixels(pixels(4, 3, 32, seed=5 + rank).to(DEV))
        tr.step()
        torch.cuda.synchronize()
        torch.save({"grad": tr.grad.cpu(), "param": tr.param.cpu(), "nb": len(tr.buckets),
                    "step": int(tr.step_t.item())}, out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("comm,side", [("split", False), ("overlap", False), ("overlap", True)],
                         ids=["split", "overlap", "overlap-sidestream"])
def test_process_group_world2_matches_mean_of_shards(comm, side, tmp_path):
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    outs = [str(tmp_path / ("rank%d.pt" % r)) for r in range(2)]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_dp_rank, args=(r, port, comm, outs[r], side)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join()
    assert [p.exitcode for p in procs] == [0, 0]
    res = [torch.load(o, weights_only=True) for o in outs]
    # single-process gradients of the two shards (same initial weights)
    from realnvp_hip.trainer import FlowTrainer
    refs = []
    for r in range(2):
        tr = FlowTrainer(make_model(32, 8, 1), 4, dtype="fp32")
        tr.set_pixels(pixels(4, 3, 32, seed=5 + r).to(DEV))
        p0 = tr.param.clone()
        tr.step()
        torch.cuda.synchronize()
        refs.append(tr.grad.cpu())
    p0 = p0.cpu()
    mean = 0.5 * (refs[0] + refs[1])
    # the same shard twice: the noise floor of the replica atomics
    tr = FlowTrainer(make_model(32, 8, 1), 4, dtype="fp32")
    tr.set_pixels(pixels(4, 3, 32, seed=5).to(DEV))
    tr.step()
    floor = float((tr.grad.cpu() - refs[0]).norm() / refs[0].norm())
    assert res[0]["nb"] > 1 and res[0]["step"] == res[1]["step"] == 1
    assert torch.equal(res[0]["grad"], res[1]["grad"])      # one reduced gradient on both ranks
    assert torch.equal(res[0]["param"], res[1]["param"])    # one Adam step on both ranks
    assert float((res[0]["grad"] - mean).norm() / mean.norm()) < max(1e-4, 8 * floor)
    assert float((refs[0] - mean).norm() / mean.norm()) > 1e-2   # the shards really differ
    assert float((res[0]["param"] - p0).abs().max()) <= 2 * tr.lr * 1.01


def test_checkpoint_carries_the_noise_stream():
    """FlowTrainer.state_dict() holds the dequantisation RNG (seed, Philox
    counter = step): a trainer built with another seed and resumed from the
    checkpoint draws the same noise as the unbroken run, so its next step
    (device logit_transform inside the step) is identical."""
    from realnvp_hip.trainer import FlowTrainer
    pix = pixels(4, 3, 32, seed=9).to(DEV)
    ta = FlowTrainer(make_model(32, 8, 1), 4, dtype="fp32", seed=1234)
    ta.set_pixels(pix)
    for _ in range(2):
        ta.step()
    sd = ta.state_dict()
    assert sd["rng"] == {"seed": 1234, "rank": 0, "step": 2}
    tb = FlowTrainer(make_model(32, 8, 1), 4, dtype="fp32", seed=7)
    tb.load_state_dict(sd)
    assert tb.seed == 1234 and int(tb.step_t.item()) == 2
    tb.set_pixels(pix)
    for t in (ta, tb):
        t.reset_metrics()
        t.step()
    torch.cuda.synchronize()
    # (1e-5: the linked forward adds the per-sample log-det with fp32 atomics,
    # whose order varies run to run -- measured up to 1.6e-6 between identical steps)
    np.testing.assert_allclose(tb.mean_logll(1), ta.mean_logll(1), rtol=1e-5)
    assert torch.equal(tb.xl, ta.xl)    # the same noise was drawn
    assert float((tb.param - ta.param).abs().max()) <= 2 * ta.lr * 1.01


def _resume_rank(rank, port, ckpt, out):
    """world-2 (gloo) rank: rank 0 saves after one step, every rank resumes
    from rank 0's checkpoint and takes one more step"""
    import os
    import sys
    import torch.distributed as dist
    from conftest import PKG
    sys.path.insert(0, PKG)
    from realnvp_hip.dist import rank_seed
    from realnvp_hip.trainer import FlowTrainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        tr = FlowTrainer(make_model(32, 8, 1), 4, dtype="fp32", seed=rank_seed(1000, rank),
                         process_group=dist.group.WORLD, comm="split")
        tr.set_pixels(pixels(4, 3, 32, seed=5).to(DEV))     # the same pixels on both ranks
        tr.step()
        if rank == 0:
            torch.save(tr.state_dict(), ckpt)
        dist.barrier()
        tb = FlowTrainer(make_model(32, 8, 1), 4, dtype="fp32", seed=rank_seed(1000, rank),
                         process_group=dist.group.WORLD, comm="split")
        tb.load_state_dict(torch.load(ckpt, weights_only=True))
        tb.set_pixels(pixels(4, 3, 32, seed=5).to(DEV))
        tb.step()
        torch.cuda.synchronize()
        torch.save({"seed": tb.seed, "step": int(tb.step_t.item()), "xl": tb.xl.cpu()}, out)
    finally:
        dist.destroy_process_group()


def test_resume_from_rank0_checkpoint_keeps_per_rank_noise(tmp_path):
    """data-parallel ranks resumed from rank 0's checkpoint keep
    their own dequantisation seeds (only the step counter is restored), so
    the replicas still draw different noise"""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ckpt = str(tmp_path / "ckpt.pt")
    outs = [str(tmp_path / ("rank%d.pt" % r)) for r in range(2)]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_resume_rank, args=(r, port, ckpt, outs[r])) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join()
    assert [p.exitcode for p in procs] == [0, 0]
    r0, r1 = [torch.load(o, weights_only=True) for o in outs]
    from realnvp_hip.dist import rank_seed
    assert r0["seed"] == rank_seed(1000, 0) and r1["seed"] == rank_seed(1000, 1)
    assert r0["step"] == r1["step"] == 2
    assert not torch.equal(r0["xl"], r1["xl"])     # different noise on the same pixels


def test_dropin_backward_between_trainer_steps():
    """the drop-in autograd path and the trainer share a coupling's
    backward scratch (same batch shape).  A drop-in forward/backward between
    two trainer steps must leave that scratch zero: the second trainer step
    then has the same gradient as a run without the drop-in call."""
    from realnvp_hip.trainer import FlowTrainer
    res = []
    for dropin in (False, False, True):
        model = make_model(32, 8, 1)
        tr = FlowTrainer(model, 4, dtype="fp32")
        x, ld = _batch(0)
        tr.set_input(x, ld)
        tr.step()
        if dropin:
            lp, ws = model(x)
            (-(lp + ld).mean() + 5e-5 * ws).backward()
            model.zero_grad(set_to_none=True)
        tr.step()
        torch.cuda.synchronize()
        res.append(tr.grad.clone())
    g0, g1, g2 = res

    def d(a, b):
        return float((a - b).norm() / b.norm())
    assert d(g2, g0) < max(1e-4, 8 * d(g1, g0)), (d(g2, g0), d(g1, g0))


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("shape", [(32, 8, 1, 4), (64, 32, 4, 16)], ids=["m32_d8_r1_b4", "m64_d32_r4_b16"])
def test_chained_couplings_forward_matches_unchained(shape, dtype):
    """The flow program over coupling links (rnvp_coupling_link_fwd / _bwd:
    the next coupling's in part, the squeeze / factor-out permutations and
    the prior folded into each coupling's link launch, the out_bn backward
    sums in closed form) against every in / out part, permutation and the
    prior launched on their own: per-sample log-prob and every BN running
    statistic agree to fp32 rounding (bf16: the closed-form statistics may
    flip a few bf16 roundings of h0), and so do the gradients (per-tensor
    norms, the arena) and dL/dx (against the unlinked step's own one-ulp
    input-perturbation floor).  Both schedules are also pinned to the float64
    truth separately (tests/test_gpu_deep.py
    test_trainer_config1_full_batch_{fp32,bf16}[chained|unchained])."""
    from realnvp_hip.trainer import FlowTrainer
    size, bd, rb, B = shape
    out = {}
    for chain in (0, 1, 2, 3):
        model = make_model(size, bd, rb)
        tr = FlowTrainer(model, B, dtype=dtype, chain=chain == 1)
        assert (tr.links is not None) == (chain == 1)
        if chain < 2:
            tr.set_pixels(pixels(B, 3, size, seed=3).to(DEV))
        else:
            # the chaos floor: the unlinked step on the same input moved by one ulp up / down
            xl = out[0][4]
            tr.set_input(torch.nextafter(xl, torch.full_like(xl, float("inf") if chain == 2 else -float("inf"))),
                         out[0][5])
        tr.step()
        torch.cuda.synchronize()
        bufs = torch.cat([b.detach().double().flatten() for n, b in model.named_buffers() if "running" in n])
        grads = {n: tr.grad[tr.offsets[n]:tr.offsets[n] + p.numel()].double().clone()
                 for n, p in model.named_parameters() if p.requires_grad}
        out[chain] = (tr.lp.clone(), bufs, grads, tr._g(tr.xl).double().clone(), tr.xl.clone(), tr.logdet.clone())

    def d(a, b):
        return float((a.double() - b.double()).norm() / b.double().norm())
    (a0, r0, g0, x0, _, _), (a1, r1, g1, x1, _, _) = out[0], out[1]
    tol = 1e-6 if dtype == "fp32" else 1e-3
    assert float(((a1 - a0).abs() / a0.abs()).max()) < tol
    assert d(r1, r0) < tol, d(r1, r0)
    # backward: the ~1e-7 difference of the closed-form statistics can flip a
    # ReLU-kink decision (~1e-3 each in a deep net, tests/test_gpu_deep.py) and,
    # in bf16, a few roundings of h0; the comparable quantities are the
    # per-tensor gradient norms (fp32 1e-3, bf16 6e-2: the norm-vector spread of
    # two valid bf16 steps at B = 16 is ~3e-2), the fp32 arena (1e-2) and dL/dx
    n0 = np.array([float(g0[n].norm()) for n in g0])
    n1 = np.array([float(g1[n].norm()) for n in g0])
    ntol = 1e-3 if dtype == "fp32" else 6e-2
    assert np.linalg.norm(n1 - n0) / np.linalg.norm(n0) < ntol, np.linalg.norm(n1 - n0) / np.linalg.norm(n0)
    if dtype == "fp32":
        ga, gb = torch.cat([g0[n] for n in g0]), torch.cat([g1[n] for n in g0])
        assert d(gb, ga) < 1e-2, d(gb, ga)
    # dL/dx of the flow input passes every coupling's kinks: held to 3x the
    # measured chaos floor of the unlinked step (its input moved by +-1 ulp)
    floor = max(d(out[2][3], x0), d(out[3][3], x0))
    assert d(x1, x0) < max(1e-2 if dtype == "fp32" else 6e-2, 3 * floor), (d(x1, x0), floor)


# ---------------------------------------------------------------------------
# fused row-local parameter pass (rnvp_weight_norm_bwd_adam) vs the separate
# weight-norm backward / Adam / weight-norm forward launches
def _pp_run(mode, dtype, steps=3, pg=None, overlap=False, graph=False, edit_at=None, size=32, bd=8, rb=1,
            via_data=False):
    from realnvp_hip.trainer import FlowTrainer
    tr = FlowTrainer(make_model(size, bd, rb), 4, dtype=dtype, param_pass=mode, process_group=pg, overlap=overlap,
                     bucket_mb=1)
    assert tr.fused == (mode == "fused")
    tr.set_pixels(pixels(4, 3, size, seed=5).to(DEV))
    if graph:
        tr.capture(warmup=1)
    for k in range(steps):
        if edit_at == k:
            # a change behind the trainer's back: the packed images must follow
            with torch.no_grad():
                for p in tr.model.parameters():
                    if p.requires_grad:
                        (p.data if via_data else p).mul_(0.97)
            if via_data:
                tr.invalidate_packed()   # writes through .data bypass the version counters
        tr.step()
    torch.cuda.synchronize()
    return tr


def _packed_images(tr):
    out = []
    for st in tr.stages:
        if st[0] != "coupling":
            continue
        ws = st[2].weights(tr.dtype)
        dt = torch.bfloat16 if tr.dtype == "bf16" else torch.float32
        for name in ws["geo"]:
            for kind in ("wf:", "wd:"):
                out.append(ws["arena"].view(kind + name, dt).float().clone())
            out.append(ws["arena"].view("norm:" + name, torch.float32).clone())
    return out


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _check_fused_vs_separate(fu, se, se2, what, steps=3):
    """bf16: the separate path is deterministic (its weight gradients are
    plain stores) and the fused pass computes every quantity in the separate
    kernels' operation order (explicit FMAs, the same reduction orders), so
    the two trajectories must agree BITWISE.  fp32: the grouped weight
    gradient adds slab partials with atomics, so gradients that are zero in
    exact arithmetic (a conv bias followed by a BatchNorm) are rounding noise
    whose sign Adam turns into +-lr steps: the checks are those of
    test_side_stream_overlap_matches_single_stream."""
    if fu.dtype == "bf16":
        for name in ("param", "exp_avg", "exp_avg_sq", "grad"):
            a, b, b2 = getattr(fu, name), getattr(se, name), getattr(se2, name)
            assert torch.equal(b2, b), (what, name, "separate bf16 path not deterministic")
            assert torch.equal(a, b), (what, name, _rel(a, b), int((a != b).sum()))
    else:
        for name in ("exp_avg", "grad"):
            a, b, b2 = getattr(fu, name), getattr(se, name), getattr(se2, name)
            assert _rel(a, b) < max(1e-2, 8 * _rel(b2, b)), (what, name, _rel(a, b), _rel(b2, b))
        assert float((fu.param - se.param).abs().max()) <= steps * 2 * se.lr * 1.01, what
        assert _rel(fu.param, se.param) < max(1e-3, 4 * _rel(se2.param, se.param)), what
    assert int(fu.step_t.item()) == int(se.step_t.item())
    # the images the next forward reads = weight_norm_fwd of the final parameters
    img = _packed_images(fu)
    for t in fu.wn_tables:
        fu._wn_fwd(t)
    torch.cuda.synchronize()
    ref = _packed_images(fu)
    for a, b in zip(img, ref):
        assert torch.equal(a, b), what


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("variant", ["eager", "hipgraph", "sidestream", "edited", "edited_data"])
def test_fused_param_pass_matches_separate(dtype, variant):
    kw = dict(graph=variant == "hipgraph", overlap=variant == "sidestream",
              edit_at=1 if variant in ("edited", "edited_data") else None, via_data=variant == "edited_data")
    fu = _pp_run("fused", dtype, **kw)
    se = _pp_run("separate", dtype, **kw)
    se2 = _pp_run("separate", dtype, **kw)
    _check_fused_vs_separate(fu, se, se2, (dtype, variant))


def test_fused_param_pass_config1_shape():
    """Config 1's convs (64x64, R4, D32: 3x3 rows of 4,608, 512-channel 1x1s,
    row blocks of 4 and 8) at batch 4, bf16."""
    kw = dict(size=64, bd=32, rb=4, steps=2)
    fu = _pp_run("fused", "bf16", **kw)
    se = _pp_run("separate", "bf16", **kw)
    se2 = _pp_run("separate", "bf16", **kw)
    _check_fused_vs_separate(fu, se, se2, "config1", steps=2)


def test_fused_param_pass_data_parallel(nccl_world1):
    """Data parallel: per-coupling weight-norm backward, all-reduce, then ONE
    model-wide Adam + norms + images launch (from_slabs = 0)."""
    for dtype in ("bf16", "fp32"):
        for graph in (False, True):
            fu = _pp_run("fused", dtype, pg=nccl_world1, graph=graph)
            se = _pp_run("separate", dtype, pg=nccl_world1, graph=graph)
            se2 = _pp_run("separate", dtype, pg=nccl_world1, graph=graph)
            _check_fused_vs_separate(fu, se, se2, ("dp", dtype, graph))
