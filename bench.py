"""RealNVP 64x64x3 NLL training throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

One step = the train.py:176-200 body on synthetic data: logit_transform of a
pixel batch (device noise), RealNVP forward (log_prob + weight_scale),
loss = -mean(log_prob+logdet) + 5e-5*weight_scale, backward, Adam.  Config 1
of BASELINE.json: 64x64x3, 4 res-blocks, base-dim 32, batch 64 per GPU,
s/t network in bf16 with fp32 accumulation (couplings, log-det, BN stats,
master weights and Adam in fp32).  Data parallel over RCCL for N > 1 (weak
scaling: 64 images per GPU).

Prints ONE JSON line (rank 0) with images/sec (whole job), bits/dim, the
per-kernel roofline of the dominant kernel family and the CPU oracle timed
on this host.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dl-normalizing-flows_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_PEAK_TFLOPS = 2500.0      # dense bf16 MFMA
F32_PEAK_TFLOPS = 157.3        # f32 MFMA
# BASELINE.json configs: shape, per-GPU batch, algorithmic
# bytes / image / training step (10*A + 72*X + 40*P/B)
CONFIGS = {
    "c1": dict(size=64, res_blocks=4, base_dim=32, batch=64, n_scales=5, alg_bytes=292.33e6,
               label="config 1: RealNVP 64x64x3, res-blocks 4, base-dim 32"),
    "c3": dict(size=32, res_blocks=8, base_dim=64, batch=64, n_scales=5, alg_bytes=773.78e6,
               label="config 3: RealNVP 32x32x3, res-blocks 8, base-dim 64 (923.6 M parameters)"),
    "c4": dict(size=128, res_blocks=4, base_dim=64, batch=256, n_scales=6, alg_bytes=2014.07e6,
               label="config 4: RealNVP 128x128x3, 6 scales, res-blocks 4, base-dim 64"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="c1", choices=sorted(CONFIGS), help="BASELINE.json config preset")
    p.add_argument("--batch", type=int, default=None, help="images per GPU (default: the config's)")
    p.add_argument("--size", type=int, default=None)
    p.add_argument("--res-blocks", type=int, default=None)
    p.add_argument("--base-dim", type=int, default=None)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--overlap", action="store_true", help="side stream for weight gradients (HIP graphs serialise it today)")
    p.add_argument("--comm", default="overlap", choices=["overlap", "split"], help="DP all-reduce schedule")
    p.add_argument("--reduce-dtype", default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the secondary measurements (fp32 parity mode, drop-in loop, sampling, config 3)")
    p.add_argument("--cpu-batch", type=int, default=64)
    p.add_argument("--cpu-steps", type=int, default=3)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--launch-check", action="store_true",
                   help="each rank prints its rank / world size and exits before any GPU call (tests the launcher)")
    p.add_argument("--pmc-markers", default=None,
                   help="write the instrumented step's launch families here and dispatch a marker before each "
                        "launch (for rocprofv3 --pmc passes, tools/pmc_traffic.py)")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                   help="per-family PMC HBM bytes per launch (tools/pmc_traffic.py output) for roofline.traffic")
    p.add_argument("--mfma", default=os.path.join(ROOT, "profiles", "pmc_mfma.json"),
                   help="per-family MFMA busy %% (tools/pmc_mfma.py output) for roofline.mfma_busy_pct")
    p.add_argument("--rocprof-families", default=os.path.join(ROOT, "profiles", "rocprof_families.json"),
                   help="per-family rocprof durations of the graph-replayed step (tools/trace_families.py output)")
    p.add_argument("--graph-markers", default=None,
                   help="capture a marker dispatch around every engine launch INTO the step graph and write the "
                        "families here (for a rocprofv3 kernel trace split by family, tools/trace_families.py)")
    a = p.parse_args()
    cfg = CONFIGS[a.config]
    for k in ("batch", "size", "res_blocks", "base_dim"):
        if getattr(a, k) is None:
            setattr(a, k, cfg[k])
    a.n_scales = cfg["n_scales"]
    a.custom = any(a.__dict__[k] != cfg[k] for k in ("batch", "size", "res_blocks", "base_dim"))
    return a


def synthetic_pixels(B, C, S, seed):
    """raw pixels k/255, k ~ U{0..255} (ToTensor semantics)"""
    rng = np.random.Generator(np.random.PCG64(seed))
    k = rng.integers(0, 256, size=(B, C, S, S))
    return torch.from_numpy((k / 255.0).astype(np.float32))


@__import__("functools").lru_cache(maxsize=1)
def binary_stamp():
    """Identity of the benchmarked binary: sha256 of the loaded HIP library and
    the git commit (RNVP_COMMIT on the GPU box, which has no .git)."""
    import hashlib
    from realnvp_hip import _lib
    h = hashlib.sha256(open(_lib.LIB_PATH, "rb").read()).hexdigest()[:16]
    commit = os.environ.get("RNVP_COMMIT")
    if not commit and os.path.isdir(os.path.join(ROOT, ".git")):
        import subprocess
        try:
            commit = subprocess.run(["git", "rev-parse", "HEAD"], cwd=ROOT, capture_output=True, text=True,
                                    timeout=30).stdout.strip() or None
        except (OSError, subprocess.SubprocessError):
            commit = None
    return dict(lib_sha256=h, commit=commit)


STALE = []


def _load_for(path, config):
    """a profiles/*.json family table, if it was measured on this config AND
    on this binary (its stamp's library hash equals the loaded one); a table
    of another binary is not used and is listed in the line's
    roofline.stale_tables"""
    if path and os.path.exists(path):
        t = json.load(open(path))
        if t.get("config") == config:
            st = t.get("stamp") or {}
            if st.get("lib_sha256") != binary_stamp()["lib_sha256"]:
                STALE.append(dict(table=os.path.relpath(path, ROOT), stamp=st or None))
                return {}
            return t.get("families", {})
    return {}


def kernel_roofline(trainer, markers=None, traffic=None, config=None, mfma=None, rocprof=None):
    """One instrumented eager step: HIP events around every engine launch
    (recorded on the launch stream).  Returns per-family totals and the
    roofline object of the dominant (largest total time) family.  `traffic`
    (tools/pmc_traffic.py output of the same config) supplies the PMC HBM
    bytes per launch."""
    from realnvp_hip import engine as E
    E.PROFILE = []
    E.MARKERS = markers is not None
    E.MARKER_FAMILIES = []
    torch.cuda.synchronize()
    trainer.step_eager()
    torch.cuda.synchronize()
    E.MARKERS = False
    fam = {}
    for f, nb, fl, e0, e1 in E.PROFILE:
        ms = e0.elapsed_time(e1)
        d = fam.setdefault(f, dict(ms=0.0, bytes=0.0, flops=0.0, launches=0))
        d["ms"] += ms
        d["bytes"] += nb
        d["flops"] += fl
        d["launches"] += 1
    E.PROFILE = None
    if markers is not None:
        json.dump(dict(config=config, stamp=binary_stamp(), families=E.MARKER_FAMILIES,
                       n_params=int(trainer.param.numel()),
                       alg_bytes={k: v["bytes"] / v["launches"] for k, v in fam.items()}), open(markers, "w"))
    dom = max(fam, key=lambda k: fam[k]["ms"])
    d = fam[dom]
    avg_ms = d["ms"] / d["launches"]
    bytes_per_launch = d["bytes"] / d["launches"]
    flops_per_launch = d["flops"] / d["launches"]
    gbs = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    tfs = flops_per_launch / (avg_ms * 1e-3) / 1e12
    peak_tf = BF16_PEAK_TFLOPS if trainer.dtype == "bf16" else F32_PEAK_TFLOPS
    # bound: whichever roof the family's arithmetic intensity sits under
    ai = d["flops"] / max(d["bytes"], 1.0)
    ridge = peak_tf * 1e12 / (HBM_PEAK_GBS * 1e9)
    if ai < ridge:
        roof = dict(bound="hbm", achieved=round(gbs, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(gbs / HBM_PEAK_GBS, 4))
    else:
        roof = dict(bound="mfma", achieved=round(tfs, 2), peak=peak_tf, unit="TFLOP/s",
                    frac=round(tfs / peak_tf, 4))
    roof.update(kernel=dom, launches_per_step=d["launches"], avg_launch_us=round(avg_ms * 1e3, 2),
                alg_bytes_per_launch=int(bytes_per_launch), flops_per_launch=int(flops_per_launch),
                traffic=None)
    row = _load_for(traffic, config).get(dom)
    if row:
        roof["traffic"] = row["traffic_per_launch"]
        roof["traffic_source"] = "PMC 2*FETCH_SIZE+WRITE_SIZE, %s" % os.path.relpath(traffic, ROOT)
    mf = _load_for(mfma, config)
    if dom in mf:
        roof["mfma_busy_pct"] = mf[dom]["mfma_busy_pct"]
        roof["mfma_source"] = "PMC SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs), %s" % (
            os.path.relpath(mfma, ROOT))
    rp = _load_for(rocprof, config)
    if dom in rp:
        # the same family's mean duration in the graph-replayed step (rocprof);
        # avg_launch_us above is HIP events around each launch of an eager step
        roof["rocprof_avg_launch_us"] = rp[dom]["avg_launch_us"]
        roof["rocprof_achieved"] = round(bytes_per_launch / (rp[dom]["avg_launch_us"] * 1e-6) / 1e9, 1)
        roof["rocprof_source"] = os.path.relpath(rocprof, ROOT)
    if STALE:
        roof["stale_tables"] = list(STALE)
    families = {k: dict(ms=round(v["ms"], 3), launches=v["launches"],
                        gbs=round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1),
                        tflops=round(v["flops"] / max(v["ms"], 1e-9) / 1e9, 2)) for k, v in fam.items()}
    for k, v in families.items():
        if k in mf:
            v["mfma_busy_pct"] = mf[k]["mfma_busy_pct"]
        if k in rp:
            v["rocprof_ms"] = rp[k]["total_ms"]
    return roof, families


def cpu_baseline(args):
    """The CPU oracle (fp32 torch-CPU restatement of the reference, pinned by
    tests/golden) timed on this host on a bounded sample of the workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import realnvp_oracle as O
    from formula_init import formula_value
    threads = len(os.sched_getaffinity(0))
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    torch.set_num_threads(threads)
    spec = O.FlowSpec(3, args.size, O.HP(args.base_dim, args.res_blocks), n_scales=args.n_scales)
    e = O.flow_spec_entries(spec)
    S = O.build_state(e, formula_value)
    tr = O.OracleTrainer(S, spec, O.param_names(e), O.trainable_names(e))
    B = args.cpu_batch
    pix = synthetic_pixels(B, 3, args.size, 123)
    noise = torch.rand(B, 3, args.size, args.size, generator=torch.Generator().manual_seed(1))
    x, ld = O.logit_transform(pix, noise)
    tr.step(x, ld)   # warm-up
    t0 = time.perf_counter()
    for _ in range(args.cpu_steps):
        tr.step(x, ld)
    dt = time.perf_counter() - t0
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return dict(value=round(B * args.cpu_steps / dt, 3), unit="images/sec", cores=threads, kind="port",
                sample="oracle fp32 train step (fwd+bwd+Adam), %dx%dx3 R%d D%d, batch %d, %d timed steps after 1 "
                       "warm-up, %.1fs, %s" % (args.size, args.size, args.res_blocks, args.base_dim, B,
                                               args.cpu_steps, dt, cpu_model))


def build_model(size, res_blocks, base_dim, n_scales, dev, seed):
    """random-init drop-in RealNVP, constructed on the device (no host copy of
    the parameters)"""
    import flow_realnvp
    import utils
    torch.manual_seed(seed)     # same initial weights on every rank
    prior = torch.distributions.Normal(torch.tensor(0.0, device=dev), torch.tensor(1.0, device=dev),
                                       validate_args=False)
    hp = utils.Hyperparameters(base_dim, res_blocks, True, True, True, True)
    with torch.device(dev):
        return flow_realnvp.RealNVP(3, size, prior, hp, n_scales=n_scales)


def timed(fn, steps, warmup, barrier=lambda: None):
    for _ in range(warmup):
        fn()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    barrier()
    return time.perf_counter() - t0


def secondary(args, dev):
    """Single-GPU context numbers next to the headline line: the fp32 parity
    mode of the same config, the drop-in loop train.py runs (model(x),
    loss.backward(), torch.optim.Adam), graph-replayed generation, and
    BASELINE config 3."""
    import utils
    from realnvp_hip.sampler import FlowSampler
    from realnvp_hip.trainer import FlowTrainer
    out = {}
    B = args.batch
    pix = synthetic_pixels(B, 3, args.size, seed=0).to(dev)

    # fp32 parity mode (the north star's 1e-5 log-prob mode) of the same step
    model = build_model(args.size, args.res_blocks, args.base_dim, args.n_scales, dev, args.seed)
    tr = FlowTrainer(model, B, dtype="fp32", seed=1000)
    tr.set_pixels(pix)
    tr.capture(warmup=1)
    dt = timed(tr.step, 5, 2)
    out["fp32_parity_mode"] = dict(value=round(5 * B / dt, 2), unit="images/sec", ms_per_step=round(dt / 5 * 1e3, 3),
                                   dtype="fp32", steps=5)
    del tr

    # the drop-in as train.py:176-200 drives it (eager autograd): with torch's
    # Adam as the reference builds it (train.py:134), then with the one-line
    # change to realnvp_hip.FusedAdam (one launch over a flat arena)
    from realnvp_hip import FusedAdam
    model.train()
    opt = None

    def loop_step():
        x, ld = utils.logit_transform(pix)      # device noise, seed from torch's CPU generator
        opt.zero_grad()
        lp, ws = model(x)
        loss = -(lp + ld).mean() + 5e-5 * ws
        loss.backward()
        opt.step()
    opt = torch.optim.Adam(model.parameters(), lr=5e-4, weight_decay=5e-5)
    dt = timed(loop_step, 5, 2)
    out["drop_in_loop_torch_adam"] = dict(
        value=round(5 * B / dt, 2), unit="images/sec", ms_per_step=round(dt / 5 * 1e3, 3), dtype="fp32", steps=5,
        note="model(x) + loss.backward() + torch.optim.Adam, eager (train.py:176-200 unchanged); torch's default "
             "(foreach) Adam over the 1,960 parameter tensors alone takes ~12.8 ms/step (tools/probe/adam_probe.py)")
    opt = FusedAdam(model.parameters(), lr=5e-4, weight_decay=5e-5)
    dt = timed(loop_step, 5, 2)
    out["drop_in_loop"] = dict(value=round(5 * B / dt, 2), unit="images/sec", ms_per_step=round(dt / 5 * 1e3, 3),
                               dtype="fp32", steps=5,
                               note="model(x) + loss.backward() + realnvp_hip.FusedAdam (train.py:134 changed to "
                                    "it), eager")
    # the same loop with the s/t net in bf16 (set_precision, the trainer's mode)
    model.set_precision("bf16")
    dt = timed(loop_step, 5, 2)
    out["drop_in_loop_bf16"] = dict(value=round(5 * B / dt, 2), unit="images/sec",
                                    ms_per_step=round(dt / 5 * 1e3, 3), dtype="bf16", steps=5,
                                    note="as drop_in_loop, s/t net in bf16")
    model.set_precision("fp32")
    del opt

    # generation: RealNVP.sample(n) + logit_transform(reverse=True), eval mode (train.py:253-259)
    model.eval()
    for dtype in ("fp32", "bf16"):
        with torch.no_grad():
            smp = FlowSampler(model, B, dtype=dtype)
            dt = timed(smp.sample, 10, 2)
        out["sampling_" + dtype] = dict(value=round(10 * B / dt, 2), unit="images/sec",
                                        ms_per_call=round(dt / 10 * 1e3, 3), n=B)
        del smp
    del model
    torch.cuda.empty_cache()

    # BASELINE config 3 (R8, D64, 923.6 M parameters), bf16, batch 64
    c = CONFIGS["c3"]
    model = build_model(c["size"], c["res_blocks"], c["base_dim"], c["n_scales"], dev, args.seed)
    tr = FlowTrainer(model, c["batch"], dtype="bf16", seed=1000)
    tr.set_pixels(synthetic_pixels(c["batch"], 3, c["size"], seed=0).to(dev))
    tr.capture(warmup=1)
    tr.reset_metrics()
    dt = timed(tr.step, 5, 1)
    v = 5 * c["batch"] / dt
    out["config3"] = dict(workload=c["label"] + ", per-GPU batch %d, train step fwd+bwd+Adam" % c["batch"],
                          value=round(v, 2), unit="images/sec", ms_per_step=round(dt / 5 * 1e3, 3), dtype="bf16",
                          steps=5, step_roofline_frac=round(v * c["alg_bytes"] / (HBM_PEAK_GBS * 1e9), 5))
    del tr, model
    torch.cuda.empty_cache()

    # BASELINE config 4's per-GPU slice (128x128x3, 6 scales, D64, 1.886 B
    # parameters, batch 256 = the HBM-sized local batch of the 8-GPU config)
    c = CONFIGS["c4"]
    model = build_model(c["size"], c["res_blocks"], c["base_dim"], c["n_scales"], dev, args.seed)
    tr = FlowTrainer(model, c["batch"], dtype="bf16", seed=1000)
    tr.set_pixels(synthetic_pixels(c["batch"], 3, c["size"], seed=0).to(dev))
    tr.capture(warmup=1)
    tr.step()
    tr.reset_metrics()
    dt = timed(tr.step, 3, 0)
    v = 3 * c["batch"] / dt
    out["config4"] = dict(workload=c["label"] + ", per-GPU batch %d (one rank of the 8-GPU config), train step "
                                                "fwd+bwd+Adam" % c["batch"],
                          value=round(v, 2), unit="images/sec", ms_per_step=round(dt / 3 * 1e3, 3), dtype="bf16",
                          steps=3, step_roofline_frac=round(v * c["alg_bytes"] / (HBM_PEAK_GBS * 1e9), 5),
                          bits_per_dim=round(tr.bits_per_dim(tr.mean_logll(3)), 4))
    del tr, model
    torch.cuda.empty_cache()
    return out


def dp_diagnostics(tr, pg, step_s, dev):
    """What an 8-GPU run needs to be read: the world size RCCL reports, every
    rank's own step time, and the gradient all-reduce time -- inside an eager
    instrumented step (events on the communication stream around each bucket)
    and in isolation for both wire dtypes (the bucket plan over the gradient
    arena, back to back on one stream)."""
    import torch.distributed as dist
    from realnvp_hip.dist import average_slice
    world = dist.get_world_size(pg)
    t = torch.tensor([step_s * 1e3], dtype=torch.float64, device=dev)
    ranks = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(ranks, t, group=pg)
    out = dict(world_size_rccl=world, backend=dist.get_backend(pg),
               rank_ms_per_step=[round(float(r.item()), 3) for r in ranks],
               buckets=len(tr.buckets), bucket_mb=round(tr.bucket_elems * 4 / 2 ** 20, 1),
               reduce_dtype=tr.reduce_dtype, comm=tr.comm)
    if tr.comm_stream is not None:
        tr.comm_events = []
        torch.cuda.synchronize()
        tr.step_eager()
        torch.cuda.synchronize()
        ev = tr.comm_events
        tr.comm_events = None
        out["allreduce_ms_in_step"] = round(sum(e0.elapsed_time(e1) for _, e0, e1 in ev), 3)
    iso = {}
    for rd in ("fp32", "bf16"):
        buf = torch.empty(tr.n, device=dev, dtype=torch.bfloat16) if rd == "bf16" else None
        g = torch.zeros_like(tr.grad)
        for rep in range(3):
            dist.barrier(group=pg)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for lo, hi, _ in tr.buckets:
                average_slice(g, lo, hi, pg, buf)
            e1.record()
            e1.synchronize()
        ms = e0.elapsed_time(e1)
        nbytes = tr.n * (2 if rd == "bf16" else 4)
        # ring all-reduce moves 2 (N-1)/N of the buffer through every rank's links
        iso[rd] = dict(ms=round(ms, 3), bus_gbs=round(2 * (world - 1) / world * nbytes / (ms * 1e-3) / 1e9, 1))
        del g, buf
    out["allreduce_isolated"] = iso
    return out


def launcher_command(argv, gpus, env):
    """The rank launcher `python3 bench.py --gpus N` (N > 1) starts when it was
    not itself started by torch.distributed.run (no WORLD_SIZE): one
    torch.distributed.run child that spawns N ranks on this node, rendezvous
    on 127.0.0.1.  None when this process is a rank (or N == 1) and runs the
    benchmark itself."""
    if gpus <= 1 or "WORLD_SIZE" in env:
        return None
    port = env.get("RNVP_BENCH_PORT")
    if port is None:
        import socket
        with socket.socket() as s:      # a free local port for the rendezvous
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def main():
    # `--gpus N` without a launcher: start the N ranks as children BEFORE any
    # GPU call in this process (this parent has only imported torch; it never
    # initialises HIP and never execs), pass their output through and exit
    # with their status.  Rank 0 prints the JSON line.
    args = parse()
    cmd = launcher_command(sys.argv[1:], args.gpus, os.environ)
    if cmd is not None:
        import subprocess
        sys.stdout.flush()
        raise SystemExit(subprocess.call(cmd))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d: launch %d ranks" % (args.gpus, world, args.gpus))
    if args.launch_check:
        print(json.dumps(dict(rank=rank, local_rank=local, world_size=world,
                              master=os.environ.get("MASTER_ADDR"))), flush=True)
        return
    # RNVP_BENCH_BACKEND=gloo: a rehearsal of the multi-rank path on a box with
    # fewer GPUs than ranks (ranks share devices round-robin; eager only, as
    # gloo collectives cannot be captured).  The driver's runs use RCCL.
    backend = os.environ.get("RNVP_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
        args.no_graph = True
    torch.cuda.set_device(local)
    pg = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        pg = dist.group.WORLD

    from realnvp_hip.dist import max_over_ranks, mean_over_ranks, rank_seed
    from realnvp_hip.trainer import FlowTrainer

    dev = torch.device("cuda", local)
    model = build_model(args.size, args.res_blocks, args.base_dim, args.n_scales, dev, args.seed)
    tr = FlowTrainer(model, args.batch, dtype=args.dtype, seed=rank_seed(1000, rank), process_group=pg,
                     overlap=args.overlap, comm=args.comm, reduce_dtype=args.reduce_dtype)
    tr.set_pixels(synthetic_pixels(args.batch, 3, args.size, seed=rank_seed(0, rank)).to(dev))

    cfg_key = dict(size=args.size, res_blocks=args.res_blocks, base_dim=args.base_dim, batch=args.batch,
                   dtype=args.dtype)
    if not args.no_graph:
        before = None
        if args.graph_markers:
            from realnvp_hip import engine as E

            def before():
                E.MARKERS = True
                E.MARKER_FAMILIES = []
        tr.capture(warmup=2, before_capture=before)
        if args.graph_markers:
            E.MARKERS = False
            if rank == 0:
                json.dump(dict(config=cfg_key, stamp=binary_stamp(), families=E.MARKER_FAMILIES),
                          open(args.graph_markers, "w"))

    def barrier():
        if pg is not None:
            import torch.distributed as dist
            dist.barrier()

    for _ in range(args.warmup):
        tr.step()
    tr.reset_metrics()
    dt = timed(tr.step, args.steps, 0, barrier)
    mean_ll = tr.mean_logll(args.steps)
    if pg is not None:
        dt = max_over_ranks(dt, dev, pg)
        mean_ll = mean_over_ranks(mean_ll, dev, pg)
    bpd = tr.bits_per_dim(mean_ll)
    imgs = world * args.batch * args.steps
    value = imgs / dt
    dp = dp_diagnostics(tr, pg, dt / args.steps, dev) if pg is not None else None
    roof, fams = kernel_roofline(tr, args.pmc_markers if rank == 0 else None, args.traffic, cfg_key, args.mfma,
                                 args.rocprof_families)
    alg_bytes = CONFIGS[args.config]["alg_bytes"]
    label = CONFIGS[args.config]["label"]
    if args.custom:
        label = "custom: RealNVP %dx%dx3, res-blocks %d, base-dim %d" % (args.size, args.size, args.res_blocks,
                                                                       args.base_dim)
    out = None
    if rank == 0:
        out = {
            "metric": "images/sec + bits/dim, RealNVP 64x64x3 training",
            "value": round(value, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (uniform 8-bit pixels, device Philox dequantisation noise); random init",
            "config": {"workload": "%s, per-GPU batch %d, train step fwd+bwd+Adam" % (label, args.batch),
                       "global_batch": world * args.batch, "image_size": args.size, "res_blocks": args.res_blocks,
                       "base_dim": args.base_dim, "n_scales": args.n_scales, "parallelism": "dp%d" % world,
                       "graph": not args.no_graph, "side_stream": args.overlap,
                       "allreduce": None if world == 1 else "%s, %s buckets of %d MB" % (
                           args.comm, args.reduce_dtype, 25)},
            "bits_per_dim": round(bpd, 4),
            "step_roofline_frac": None if args.custom else round(value / world * alg_bytes / (HBM_PEAK_GBS * 1e9), 5),
            "roofline": roof,
            "kernel_families": fams,
            "cpu_baseline": None,
            "binary": binary_stamp(),
        }
        if dp is not None:
            out["dp"] = dp
    del tr, model
    torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_secondary:
        out["secondary"] = secondary(args, dev)
    # the CPU baseline on rank 0 at every world size, after the timed region
    # (the other ranks wait at the closing barrier; --cpu-steps bounds it)
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if pg is not None:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
