"""Plain-PyTorch definitions of the two model families (CPU oracle + initialiser).

* ``Net`` is the reference model: a single ``nn.Linear(784, 10)`` applied to the
  flattened image (reference ``multi_proc_single_gpu.py:119-126``).
* ``CNN`` is the north-star model named in BASELINE.json (absent from the
  reference): conv1 1->32 3x3 + ReLU, conv2 32->64 3x3 + ReLU,
  MaxPool2d(2), flatten 9216 -> fc1 128 + ReLU -> fc2 10, trained with
  log-softmax + NLL (== ``F.cross_entropy`` on the logits, which is exactly what the
  reference's Trainer applies, ``multi_proc_single_gpu.py:88``).

These modules are used for three things only: (1) drawing the initial weights
with torch's default initialisers so a seeded run matches a seeded reference run
bit-for-bit, (2) the CPU/gloo execution path and (3) the fp32 oracle the HIP
kernels are tested against.  The GPU hot path never calls them: it runs the
fused HIP step programs in ``runtime/program.py`` over a flat parameter arena.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc = nn.Linear(784, 10)

    def forward(self, x):
        return self.fc(x.view(x.size(0), -1))


class CNN(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.fc1 = nn.Linear(9216, 128)
        self.fc2 = nn.Linear(128, 10)

    def forward(self, x):
        x = x.view(x.size(0), 1, 28, 28)
        x = F.relu(self.conv1(x))
        x = F.relu(self.conv2(x))
        x = F.max_pool2d(x, 2)
        x = torch.flatten(x, 1)
        x = F.relu(self.fc1(x))
        return self.fc2(x)


def functional_forward(model_name: str, params: dict, x: torch.Tensor) -> torch.Tensor:
    """Forward of either model from a {torch_name: tensor} dict (torch layouts)."""
    if model_name == "linear":
        return F.linear(x.reshape(x.size(0), -1), params["fc.weight"], params["fc.bias"])
    if model_name == "cnn":
        h = x.reshape(x.size(0), 1, 28, 28)
        h = F.relu(F.conv2d(h, params["conv1.weight"], params["conv1.bias"]))
        h = F.relu(F.conv2d(h, params["conv2.weight"], params["conv2.bias"]))
        h = F.max_pool2d(h, 2)
        h = torch.flatten(h, 1)
        h = F.relu(F.linear(h, params["fc1.weight"], params["fc1.bias"]))
        return F.linear(h, params["fc2.weight"], params["fc2.bias"])
    raise ValueError(f"unknown model {model_name!r}")


MODULES = {"linear": Net, "cnn": CNN}
