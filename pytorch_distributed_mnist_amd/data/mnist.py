"""MNIST storage: IDX reader + deterministic synthetic MNIST-shaped data.

The reference obtains MNIST through ``torchvision.datasets.MNIST(root, train,
download=True)`` with ``ToTensor()`` + ``Normalize((0.1307,), (0.3081,))``
(reference ``multi_proc_single_gpu.py:129-138``).  torchvision is not part of
this framework: we read the same on-disk files torchvision writes
(``<root>/MNIST/raw/{train,t10k}-{images-idx3,labels-idx1}-ubyte[.gz]``) and keep
them as raw uint8 — the normalisation ``(x/255 - mean)/std`` happens inside the
first GPU kernel, so the dataset lives on the device as 47 MB of uint8 instead of
188 MB of fp32 and there is no per-sample host transform at all.

With no network there is nothing to download; when the files are absent the
loader falls back to a deterministic synthetic set of the same shape (class
prototypes + noise, so it is learnable and accuracy is meaningful).
"""
from __future__ import annotations

import gzip
import os
import struct
from dataclasses import dataclass

import numpy as np
import torch

MNIST_MEAN = 0.1307
MNIST_STD = 0.3081
IMAGE_HW = 28
IMAGE_PIXELS = IMAGE_HW * IMAGE_HW
NUM_CLASSES = 10
TRAIN_SIZE = 60000
TEST_SIZE = 10000

_FILES = {
    True: ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
    False: ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte"),
}


@dataclass
class MnistSplit:
    """One split held as raw bytes: images uint8 [N, 784], labels int64 [N]."""
    images: torch.Tensor
    labels: torch.Tensor
    source: str  # "mnist" or "synthetic"

    def __len__(self) -> int:
        return int(self.images.shape[0])

    def to(self, device) -> "MnistSplit":
        return MnistSplit(self.images.to(device), self.labels.to(device), self.source)


def _open(path: str):
    if os.path.exists(path):
        return open(path, "rb")
    if os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    raise FileNotFoundError(path)


def read_idx(path: str) -> np.ndarray:
    """Parse an IDX file (magic 0x00000801 labels / 0x00000803 images)."""
    with _open(path) as f:
        raw = f.read()
    zero, dtype_code, ndim = struct.unpack(">HBB", raw[:4])
    if zero != 0 or dtype_code != 0x08:
        raise ValueError(f"{path}: not an unsigned-byte IDX file")
    dims = struct.unpack(">" + "I" * ndim, raw[4:4 + 4 * ndim])
    data = np.frombuffer(raw, dtype=np.uint8, offset=4 + 4 * ndim)
    expected = int(np.prod(dims))
    if data.size != expected:
        raise ValueError(f"{path}: expected {expected} bytes of payload, got {data.size}")
    return data.reshape(dims)


def mnist_raw_dir(root: str) -> str:
    return os.path.join(root, "MNIST", "raw")


def mnist_available(root: str) -> bool:
    d = mnist_raw_dir(root)
    for train in (True, False):
        for name in _FILES[train]:
            p = os.path.join(d, name)
            if not (os.path.exists(p) or os.path.exists(p + ".gz")):
                return False
    return True


def load_mnist(root: str, train: bool) -> MnistSplit:
    d = mnist_raw_dir(root)
    img_name, lbl_name = _FILES[train]
    images = read_idx(os.path.join(d, img_name))
    labels = read_idx(os.path.join(d, lbl_name))
    if images.ndim != 3 or images.shape[1:] != (IMAGE_HW, IMAGE_HW):
        raise ValueError(f"unexpected MNIST image shape {images.shape}")
    if labels.shape[0] != images.shape[0]:
        raise ValueError("image/label count mismatch")
    imgs = torch.from_numpy(images.reshape(images.shape[0], IMAGE_PIXELS).copy())
    lbls = torch.from_numpy(labels.astype(np.int64))
    return MnistSplit(imgs, lbls, "mnist")


def write_idx(path: str, array: np.ndarray) -> None:
    """Write an unsigned-byte IDX file (used by tests to fabricate MNIST files)."""
    array = np.ascontiguousarray(array, dtype=np.uint8)
    header = struct.pack(">HBB", 0, 0x08, array.ndim) + struct.pack(">" + "I" * array.ndim, *array.shape)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "wb") as f:
        f.write(header)
        f.write(array.tobytes())


def synthetic_split(n: int, train: bool, seed: int = 1234) -> MnistSplit:
    """Deterministic, learnable MNIST-shaped data.

    Ten smooth random prototypes (one per class); each sample is its class
    prototype, randomly shifted by up to 2 pixels and intensity-scaled, plus
    noise, quantised to uint8.  Train and test draw from the same prototypes with
    different sample seeds.
    """
    g = torch.Generator().manual_seed(seed)
    coarse = torch.rand(NUM_CLASSES, 1, 7, 7, generator=g)
    protos = torch.nn.functional.interpolate(coarse, size=(IMAGE_HW, IMAGE_HW), mode="bilinear",
                                             align_corners=False)[:, 0]
    protos = (protos - protos.amin(dim=(1, 2), keepdim=True))
    protos = protos / protos.amax(dim=(1, 2), keepdim=True).clamp_min(1e-6)
    protos = (protos ** 2) * 255.0

    # all 25 shifted copies of every prototype: [10, 5, 5, 28, 28]
    pad = torch.nn.functional.pad(protos, (2, 2, 2, 2))
    bank = torch.stack([torch.stack([pad[:, dy:dy + IMAGE_HW, dx:dx + IMAGE_HW] for dx in range(5)], 1)
                        for dy in range(5)], 1)

    gs = torch.Generator().manual_seed(seed * 7919 + (1 if train else 2))
    labels = torch.randint(0, NUM_CLASSES, (n,), generator=gs)
    images = torch.empty(n, IMAGE_HW, IMAGE_HW, dtype=torch.uint8)
    chunk = 8192
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        m = e - s
        lab = labels[s:e]
        dy = torch.randint(0, 5, (m,), generator=gs)
        dx = torch.randint(0, 5, (m,), generator=gs)
        other = torch.randint(0, NUM_CLASSES, (m,), generator=gs)
        odx = torch.randint(0, 5, (m,), generator=gs)
        mix = 0.45 * torch.rand(m, 1, 1, generator=gs)
        base = bank[lab, dy, dx] * (1 - mix) + bank[other, 4 - dy, odx] * mix
        scale = 0.6 + 0.4 * torch.rand(m, 1, 1, generator=gs)
        noise = 70.0 * torch.randn(m, IMAGE_HW, IMAGE_HW, generator=gs)
        images[s:e] = (base * scale + noise).clamp_(0, 255).to(torch.uint8)
    return MnistSplit(images.reshape(n, IMAGE_PIXELS), labels.to(torch.int64), "synthetic")


def load_split(root: str, train: bool, *, synthetic: bool = False,
               synthetic_size: int | None = None, seed: int = 1234) -> MnistSplit:
    """Real MNIST when present under ``root`` (and not forced synthetic), else synthetic."""
    if not synthetic and mnist_available(root):
        return load_mnist(root, train)
    default = TRAIN_SIZE if train else TEST_SIZE
    n = default if (synthetic_size is None or not train) else int(synthetic_size)
    return synthetic_split(n, train, seed)


def normalize_reference(images_u8: torch.Tensor) -> torch.Tensor:
    """``Normalize(ToTensor(x))`` in fp32, exactly as torchvision computes it.

    ToTensor divides by 255 in fp32; Normalize subtracts mean and divides by std
    (``torchvision.transforms.functional.normalize`` does ``sub_(mean).div_(std)``).
    """
    x = images_u8.to(torch.float32).div(255.0)
    return x.sub_(MNIST_MEAN).div_(MNIST_STD)
