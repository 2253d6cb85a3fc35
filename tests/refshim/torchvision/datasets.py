"""torchvision.datasets.MNIST over the raw IDX files (no download; see __init__)."""
import os

import numpy as np
import torch


def _read_idx(path):
    with open(path, "rb") as f:
        raw = f.read()
    ndim = raw[3]
    dims = [int.from_bytes(raw[4 + 4 * i:8 + 4 * i], "big") for i in range(ndim)]
    return np.frombuffer(raw, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


class MNIST(torch.utils.data.Dataset):
    def __init__(self, root, train=True, transform=None, target_transform=None, download=False):
        raw = os.path.join(root, "MNIST", "raw")
        pre = "train" if train else "t10k"
        self.data = torch.from_numpy(_read_idx(os.path.join(raw, f"{pre}-images-idx3-ubyte")).copy())
        self.targets = torch.from_numpy(
            _read_idx(os.path.join(raw, f"{pre}-labels-idx1-ubyte")).astype(np.int64))
        self.transform = transform
        self.target_transform = target_transform

    def __len__(self):
        return self.data.shape[0]

    def __getitem__(self, i):
        img, target = self.data[i], int(self.targets[i])
        if self.transform is not None:
            img = self.transform(img)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return img, target
