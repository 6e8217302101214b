"""Real-data input pipeline of the training loop (train.py:65-100).

The reference reads an ImageFolder through torchvision
(Resize((S, S)) -> CenterCrop(S) -> ToTensor), keeps a random 100-batch
subset, splits it 90 / 10 into train / validation and feeds float32 batches
through DataLoader workers; each step then moves the batch to the GPU
(train.py:188-189).  torchvision is not part of this stack, so the same
semantics are restated here on PIL + torch.utils.data:

  * ``ImageFolder``: torchvision's class / sample discovery (sorted class
    sub-directories, sorted files with an image extension, target = class
    index), PIL ``convert("RGB")``, bilinear ``resize((S, S))`` (what
    transforms.Resize does to a PIL image; the CenterCrop(S) that follows a
    resize to (S, S) is the identity).  Samples stay uint8 CHW: 1 byte per
    pixel in the workers, in pinned memory and over PCIe, 4x less than the
    reference's float32 tensors.
  * ``reference_splits``: train.py:76-83 (100-batch cap, 90 / 10 split) with
    torch.utils.data.random_split, so a seeded generator gives the same
    subsets as the reference.
  * ``DeviceLoader``: DataLoader (workers, pinned memory) whose uint8 batches
    are copied to the GPU on a copy stream one batch ahead and converted by
    ``rnvp_u8_to_unit`` (ToTensor's k / 255) on the consumer's stream.
"""
import math
import os

import numpy as np
import torch
import torch.utils.data as torchdata

from . import _lib
from .engine import stream_ptr

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def _pil():
    try:
        from PIL import Image
    except ImportError as e:   # pragma: no cover - PIL ships with this image
        raise RuntimeError("the image-folder pipeline needs PIL (Pillow)") from e
    return Image


class ImageFolder(torchdata.Dataset):
    """torchvision.datasets.ImageFolder(root, transform=Compose([Resize((S, S)),
    CenterCrop(S), ToTensor()])) with the ToTensor division deferred to the
    device: items are (uint8 tensor [3, S, S], class index)."""

    def __init__(self, root, image_size):
        self.root, self.image_size = root, int(image_size)
        classes = sorted(e.name for e in os.scandir(root) if e.is_dir())
        if not classes:
            raise FileNotFoundError("no class sub-directories under %s" % root)
        self.classes = classes
        self.class_to_idx = {c: i for i, c in enumerate(classes)}
        samples = []
        for c in classes:
            d = os.path.join(root, c)
            for base, _, files in sorted(os.walk(d, followlinks=True)):
                for f in sorted(files):
                    if f.lower().endswith(IMG_EXTENSIONS):
                        samples.append((os.path.join(base, f), self.class_to_idx[c]))
        if not samples:
            raise FileNotFoundError("no images (%s) under %s" % (", ".join(IMG_EXTENSIONS), root))
        self.samples = samples
        self.targets = [t for _, t in samples]

    def __len__(self):
        return len(self.samples)

    def load(self, path):
        Image = _pil()
        with open(path, "rb") as fh:
            im = Image.open(fh)
            im = im.convert("RGB")
        S = self.image_size
        if im.size != (S, S):
            im = im.resize((S, S), Image.BILINEAR)
        return np.asarray(im, dtype=np.uint8).transpose(2, 0, 1).copy()

    def __getitem__(self, i):
        path, target = self.samples[i]
        return torch.from_numpy(self.load(path)), target


def reference_splits(dataset, batch_size, generator=None):
    """train.py:76-83: keep at most 100 batches (random subset), then a 90 / 10
    random train / validation split."""
    if len(dataset) > batch_size * 100:
        dataset, _ = torchdata.random_split(dataset, [batch_size * 100, len(dataset) - batch_size * 100],
                                            generator=generator)
    n_train = math.floor(len(dataset) * 0.9)
    train, valid = torchdata.random_split(dataset, [n_train, len(dataset) - n_train], generator=generator)
    return train, valid


def u8_to_unit(u8, out=None):
    """transforms.ToTensor's k / 255 of a uint8 device tensor (HIP kernel)."""
    if not u8.is_cuda or u8.dtype != torch.uint8:
        raise RuntimeError("u8_to_unit: expected a uint8 tensor on a HIP device")
    u8 = u8.contiguous()
    if out is None:
        out = torch.empty(u8.shape, device=u8.device, dtype=torch.float32)
    if out.shape != u8.shape or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("u8_to_unit: out must be a contiguous float32 tensor of the input's shape")
    _lib.lib().u8_to_unit(u8.data_ptr(), out.data_ptr(), u8.numel(), stream_ptr())
    return out


class DeviceLoader:
    """Iterates (pixels [B, 3, S, S] fp32 in [0, 1] on `device`, targets) over
    a dataset of uint8 images.  The host side is a torch DataLoader (workers,
    pinned memory, shuffling like train.py:86-97); the next batch's H2D copy
    runs on a copy stream while the current batch is consumed.  drop_last
    keeps every batch at the trainer's fixed (graph-captured) size."""

    def __init__(self, dataset, batch_size, device, shuffle=True, num_workers=0, drop_last=False, generator=None):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("DeviceLoader feeds a HIP device")
        self.loader = torchdata.DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, num_workers=num_workers,
                                           pin_memory=True, drop_last=drop_last, generator=generator)
        self.copy_stream = torch.cuda.Stream(device=self.device)

    def __len__(self):
        return len(self.loader)

    def _issue(self, batch):
        u8, target = batch
        with torch.cuda.stream(self.copy_stream):
            d = u8.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        return d, target, ev

    def __iter__(self):
        it = iter(self.loader)
        nxt = next(it, None)
        pending = self._issue(nxt) if nxt is not None else None
        while pending is not None:
            d, target, ev = pending
            nxt = next(it, None)
            pending = self._issue(nxt) if nxt is not None else None
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            d.record_stream(cur)
            yield u8_to_unit(d), target
