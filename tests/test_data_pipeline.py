"""Real-data pipeline and validation loop (train.py:65-100,
214-233).  The reference's dataset (Kaggle, README.md:9) is not available, so
the pipeline is exercised on a synthetic image folder written here; the
torchvision transforms it restates are checked against PIL directly (CPU),
the device ToTensor and the graph-captured validation pass against the
drop-in model's own eager eval forward (GPU)."""
import math
import os

import numpy as np
import pytest
import torch

DEV = "cuda"


def write_folder(root, n_per_class=(5, 3), sizes=((40, 48), (64, 64), (17, 23)), seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    paths = []
    for ci, n in enumerate(n_per_class):
        d = os.path.join(root, "class_%d" % ci)
        os.makedirs(d, exist_ok=True)
        for i in range(n):
            h, w = sizes[(ci + i) % len(sizes)]
            a = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
            p = os.path.join(d, "img_%02d.png" % i)
            Image.fromarray(a).save(p)
            paths.append((p, ci))
    with open(os.path.join(root, "class_0", "notes.txt"), "w") as fh:   # not an image: skipped
        fh.write("x")
    return paths


# ----------------------------------------------------------------------- CPU
def test_image_folder_discovery_and_transform(tmp_path):
    from PIL import Image
    from realnvp_hip.data import ImageFolder
    paths = write_folder(str(tmp_path))
    ds = ImageFolder(str(tmp_path), 32)
    assert ds.classes == ["class_0", "class_1"]
    assert [s for s in ds.samples] == sorted(paths)
    assert len(ds) == 8
    for i in range(len(ds)):
        x, t = ds[i]
        assert x.dtype == torch.uint8 and tuple(x.shape) == (3, 32, 32)
        p, ct = ds.samples[i]
        assert t == ct
        # transforms.Resize((32, 32)) on a PIL image = bilinear PIL resize; CenterCrop(32) is then the identity
        ref = np.asarray(Image.open(p).convert("RGB").resize((32, 32), Image.BILINEAR)).transpose(2, 0, 1)
        assert np.array_equal(x.numpy(), ref)


def test_image_folder_already_sized_is_untouched(tmp_path):
    from PIL import Image
    from realnvp_hip.data import ImageFolder
    write_folder(str(tmp_path), n_per_class=(2,), sizes=((16, 16),))
    ds = ImageFolder(str(tmp_path), 16)
    x, _ = ds[0]
    assert np.array_equal(x.numpy(), np.asarray(Image.open(ds.samples[0][0])).transpose(2, 0, 1))


def test_image_folder_errors(tmp_path):
    from realnvp_hip.data import ImageFolder
    with pytest.raises(FileNotFoundError):
        ImageFolder(str(tmp_path), 8)
    os.makedirs(os.path.join(str(tmp_path), "empty"))
    with pytest.raises(FileNotFoundError):
        ImageFolder(str(tmp_path), 8)


def test_reference_splits_sizes_and_determinism():
    from realnvp_hip.data import reference_splits
    ds = torch.utils.data.TensorDataset(torch.arange(1000))
    tr, va = reference_splits(ds, batch_size=4, generator=torch.Generator().manual_seed(0))
    # train.py:76-83: cap at 100 batches (400), then floor(0.9 * 400) / rest
    assert (len(tr), len(va)) == (360, 40)
    tr2, va2 = reference_splits(ds, batch_size=4, generator=torch.Generator().manual_seed(0))
    assert list(tr.indices) == list(tr2.indices) and list(va.indices) == list(va2.indices)
    small = torch.utils.data.TensorDataset(torch.arange(37))
    tr, va = reference_splits(small, batch_size=64)
    assert (len(tr), len(va)) == (math.floor(37 * 0.9), 37 - math.floor(37 * 0.9))


def test_device_loader_refuses_cpu():
    from realnvp_hip.data import DeviceLoader
    with pytest.raises(RuntimeError):
        DeviceLoader(torch.utils.data.TensorDataset(torch.zeros(4, dtype=torch.uint8)), 2, "cpu")


# ----------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_u8_to_unit_bit_exact():
    from realnvp_hip.data import u8_to_unit
    for n in (0, 1, 15, 16, 17, 3 * 64 * 64 * 5 + 7):
        u8 = torch.randint(0, 256, (max(n, 1),), dtype=torch.uint8)[:n]
        ref = u8.float().div(255)                                   # transforms.ToTensor on the CPU
        got = u8_to_unit(u8.to(DEV)).cpu()
        assert torch.equal(got, ref), n
    allv = torch.arange(256, dtype=torch.uint8)
    assert torch.equal(u8_to_unit(allv.to(DEV)).cpu(), allv.float().div(255))


def _model(size=16, bd=4, rb=1):
    import flow_realnvp
    import utils
    from formula_init import formula_state
    prior = torch.distributions.Normal(torch.tensor(0.0, device=DEV), torch.tensor(1.0, device=DEV))
    m = flow_realnvp.RealNVP(3, size, prior, utils.Hyperparameters(bd, rb, True, True, True, True))
    m.load_state_dict(formula_state(m))
    return m.to(DEV)


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_evaluator_matches_dropin_eval_loop(graph):
    """FlowEvaluator's pass == the reference's validation loop written with the
    drop-in (model.eval(), logit_transform, model(x), (logll + logdet).mean()
    per batch, averaged), given the same dequantisation noise."""
    from realnvp_hip import _lib
    from realnvp_hip.engine import stream_ptr
    from realnvp_hip.evaluator import FlowEvaluator
    model = _model()
    model.train()
    with torch.no_grad():   # move the running statistics off their defaults
        model(torch.rand(8, 3, 16, 16, device=DEV) * 2 - 1)
    model.eval()
    B, n_b, seed = 4, 3, 123
    ev = FlowEvaluator(model, B, seed=seed, graph=graph)
    gen = torch.Generator().manual_seed(5)
    batches = [torch.randint(0, 256, (B, 3, 16, 16), generator=gen).float().div(255).to(DEV) for _ in range(n_b)]
    ll, bpd = ev.evaluate(batches)
    L = _lib.lib()
    n = 3 * 16 * 16
    ref = []
    with torch.no_grad():
        for k, pix in enumerate(batches):
            x = torch.empty_like(pix)
            logdet = torch.empty(B, device=DEV)
            L.logit_fwd(pix.data_ptr(), None, seed, k * B * n, None, 0.9, x.data_ptr(), logdet.data_ptr(), B, n,
                        stream_ptr())
            lp, _ = model(x)
            ref.append(float((lp + logdet).mean()))
    ref_ll = sum(ref) / n_b
    assert abs(ll - ref_ll) <= 1e-5 * abs(ref_ll), (ll, ref_ll)
    D = 3 * 16 * 16
    assert abs(bpd - (-ref_ll + math.log(256.0) * D) / (D * math.log(2.0))) < 1e-5
    # a second pass over the same batches draws fresh noise (counter advanced) but stays close
    ll2, _ = ev.evaluate(batches)
    assert ll2 != ll and abs(ll2 - ll) < 0.05 * abs(ll)


@pytest.mark.gpu
def test_folder_to_trainer_and_validation(tmp_path):
    """End to end: image folder -> reference splits -> device loader ->
    FlowTrainer steps -> FlowEvaluator validation pass (train.py:176-233)."""
    from realnvp_hip.data import DeviceLoader, ImageFolder, reference_splits
    from realnvp_hip.evaluator import FlowEvaluator
    from realnvp_hip.trainer import FlowTrainer
    write_folder(str(tmp_path), n_per_class=(14, 10))
    ds = ImageFolder(str(tmp_path), 16)
    tr_set, va_set = reference_splits(ds, 4, generator=torch.Generator().manual_seed(0))
    assert (len(tr_set), len(va_set)) == (21, 3)
    model = _model()
    tr = FlowTrainer(model, 4, dtype="fp32")
    steps = 0
    for pix, _ in DeviceLoader(tr_set, 4, DEV, shuffle=True, drop_last=True,
                               generator=torch.Generator().manual_seed(1)):
        assert pix.dtype == torch.float32 and float(pix.min()) >= 0 and float(pix.max()) <= 1
        tr.set_pixels(pix)
        tr.step()
        steps += 1
    assert steps == 5
    train_bpd = tr.bits_per_dim(tr.mean_logll(steps))
    assert math.isfinite(train_bpd)
    model.eval()
    ev = FlowEvaluator(model, 3, dtype="fp32")
    ll, bpd = ev.evaluate(DeviceLoader(va_set, 3, DEV, shuffle=False))
    assert ev.n_batches == 1 and math.isfinite(ll) and math.isfinite(bpd)
    # the uint8 pipeline delivers exactly ToTensor's pixels
    pix, _ = next(iter(DeviceLoader(va_set, 3, DEV, shuffle=False)))
    ref = torch.stack([va_set[i][0] for i in range(3)]).float().div(255)
    assert torch.equal(pix.cpu(), ref)
