"""Closed-form (RNG-free) parameter init shared by the golden generator and the
tests, so a model's weights can be regenerated on any box without shipping a
checkpoint.  Keys are reference ``state_dict`` keys.

value(name, shape) depends only on the key and the element index.
"""
import zlib

import numpy as np
import torch


def _phase(name: str) -> float:
    return (zlib.crc32(name.encode()) % 10007) / 10007.0 * 6.283185307179586


_DEVICE = None   # formula_state(..., device=d): evaluate the sinusoids there (big models)


_CHIRP = 0.0     # formula_state(..., style="chirp"): quadratic phase term


def _wave(name, shape, freq, amp, offset):
    """offset + amp * sin(freq*i + phase(name) [+ c*i^2]).  The plain wave makes
    every conv weight matrix rank 2 (sin(a*i + b) separates over the row and
    column index), so some channels are near-degenerate and ReLU decisions
    become rounding-sensitive; the chirp term (style="chirp") couples the
    indices and gives full-rank weights (the deep R=8 coupling goldens)."""
    n = int(np.prod(shape)) if len(shape) else 1
    if _DEVICE is not None:
        i = torch.arange(n, dtype=torch.float64, device=_DEVICE)
        return (offset + amp * torch.sin(freq * i + _phase(name) + _CHIRP * i * i)).float().reshape(shape)
    i = np.arange(n, dtype=np.float64)
    v = offset + amp * np.sin(freq * i + _phase(name) + _CHIRP * i * i)
    return torch.from_numpy(v.astype(np.float32)).reshape(shape)


def chirp_value(name, shape, trainable):
    """formula_value with full-rank (chirped) weights"""
    global _CHIRP
    _CHIRP = 2.3e-4
    try:
        return formula_value(name, shape, trainable)
    finally:
        _CHIRP = 0.0


def formula_value(name: str, shape, trainable: bool) -> torch.Tensor:
    leaf = name.split(".")[-1]
    shape = tuple(shape)
    if leaf == "weight_v":
        return _wave(name, shape, 0.7137, 1.0, 0.0)
    if leaf == "weight" and len(shape) == 4:  # plain conv (weight_norm=False)
        return _wave(name, shape, 0.7137, float(np.prod(shape[1:])) ** -0.5, 0.0)
    if leaf == "weight_g":
        if not trainable:
            return torch.ones(shape)
        return _wave(name, shape, 1.31, 0.1, 0.5)
    if leaf == "bias":
        return _wave(name, shape, 0.913, 0.05, 0.0)
    if leaf == "weight":                       # BatchNorm affine weight
        return _wave(name, shape, 1.07, 0.1, 1.0)
    if leaf == "scale":
        return _wave(name, shape, 1.0, 0.1, 0.5)
    if leaf == "scale_shift":
        return _wave(name, shape, 1.0, 0.05, 0.0)
    if leaf == "running_mean":
        return torch.zeros(shape)
    if leaf == "running_var":
        return torch.ones(shape)
    if leaf == "num_batches_tracked":
        return torch.zeros(shape, dtype=torch.long)
    raise KeyError(name)


def formula_state(module: torch.nn.Module, device=None, style="wave"):
    """A full state dict for ``module`` (reference or engine: same keys).
    device: evaluate on that torch device (float64 sin, rounded to float32 --
    equal to the numpy path up to the last float32 bit of a few elements;
    used for the 0.9 B-parameter config-3 model)."""
    global _DEVICE
    trainable = {n for n, p in module.named_parameters() if p.requires_grad}
    value = chirp_value if style == "chirp" else formula_value
    out = {}
    _DEVICE = device
    try:
        for k, v in module.state_dict().items():
            t = value(k, v.shape, k in trainable)
            out[k] = (t.to(device) if device is not None else t).to(v.dtype)
    finally:
        _DEVICE = None
    return out


def pixels(batch, channels, size, seed=0):
    """Synthetic raw pixels k/255, k ~ U{0..255} (ToTensor semantics), numpy PCG64."""
    rng = np.random.Generator(np.random.PCG64(seed))
    k = rng.integers(0, 256, size=(batch, channels, size, size))
    return torch.from_numpy((k / 255.0).astype(np.float32))


def uniform_noise(batch, channels, size, seed=1):
    rng = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(rng.random((batch, channels, size, size)).astype(np.float32))


# ---------------------------------------------------------------------------
# gradient projection checksums: <g, r_k> / |r_k| for K closed-form vectors
# r_k[i] = cos(2 pi frac((i + 1) * PHI_k) + k), quasi-random and regenerated on
# any box from the element index alone.  A permuted, mis-scattered or
# sign-flipped gradient with the right norm moves its projections by
# ~|g| / sqrt(n) each, like an error of its own size would.
PROJ_PHI = (0.6180339887498949, 0.4142135623730951, 0.7320508075688772, 0.2360679774997898)


def projections(g):
    """[K] float64 projection checksums of one gradient tensor (any device)."""
    t = g.detach().reshape(-1).double()
    i = torch.arange(1, t.numel() + 1, dtype=torch.float64, device=t.device)
    out = []
    for k, phi in enumerate(PROJ_PHI):
        r = torch.cos(2.0 * np.pi * torch.frac(i * phi) + k)
        out.append(float(torch.dot(t, r) / r.norm()))
    return np.array(out)


def projection_matrix(grads):
    """[n_tensors, K] projections of a list of gradient tensors"""
    return np.stack([projections(g) for g in grads])


def largest(names, sizes, n=10):
    """the n largest tensors (by element count; ties by name order): those
    whose full gradients the trainer tests compare element by element"""
    order = sorted(range(len(names)), key=lambda i: (-sizes[i], i))
    return [names[i] for i in sorted(order[:n])]
