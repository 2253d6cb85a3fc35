"""Running metrics with the reference's exact print formats.

``Average`` and ``Accuracy`` mirror reference ``multi_proc_single_gpu.py:28-65``
(sample-weighted mean printed ``{:.6f}``; argmax accuracy printed ``{:.2f}%``).
The difference is *where* the sums are formed: the reference calls ``.item()``
twice per step (two blocking device->host syncs); our kernels
accumulate sum(loss*B) and #correct into a small fp64 device buffer and the
host reads it once per epoch (``DeviceMetrics``).
"""
from __future__ import annotations

import torch


class Average:
    def __init__(self):
        self.sum = 0.0
        self.count = 0

    def __str__(self):
        return "{:.6f}".format(self.average)

    @property
    def average(self):
        return self.sum / self.count if self.count else float("nan")

    def update(self, value, number):
        self.sum += value * number
        self.count += number

    @classmethod
    def from_sums(cls, total: float, count: int) -> "Average":
        a = cls()
        a.sum, a.count = float(total), int(count)
        return a


class Accuracy:
    def __init__(self):
        self.correct = 0
        self.count = 0

    def __str__(self):
        return "{:.2f}%".format(self.accuracy * 100)

    @property
    def accuracy(self):
        return self.correct / self.count if self.count else 0.0

    @torch.no_grad()
    def update(self, output, target):
        pred = output.argmax(dim=1)
        self.correct += int(pred.eq(target).sum().item())
        self.count += output.size(0)

    @classmethod
    def from_counts(cls, correct: int, count: int) -> "Accuracy":
        a = cls()
        a.correct, a.count = int(round(correct)), int(count)
        return a


class DeviceMetrics:
    """fp64 device accumulators: [loss_sum, correct, count] for train and eval.

    Kernels add into ``buf`` (graph-capturable, no host sync); ``read()`` is the
    single per-epoch synchronisation point.
    """
    TRAIN, EVAL = 0, 3

    def __init__(self, device):
        self.buf = torch.zeros(8, dtype=torch.float64, device=device)

    def reset(self, which: int) -> None:
        self.buf[which:which + 3].zero_()

    def train_view(self) -> torch.Tensor:
        return self.buf[0:3]

    def eval_view(self) -> torch.Tensor:
        return self.buf[3:6]

    def read(self, which: int):
        v = self.buf[which:which + 3].tolist()
        return Average.from_sums(v[0], int(round(v[2]))), Accuracy.from_counts(v[1], int(round(v[2])))
