"""Minimal stand-in for torchvision, used ONLY to run the unmodified reference script on CPU
as a test oracle (tests/test_reference_parity.py).

torchvision is not installed in this environment and there is no network, so this package
provides exactly what the reference imports (`datasets.MNIST`, `transforms.Compose/ToTensor/
Normalize`) with torchvision's semantics, reading the torchvision on-disk layout
`<root>/MNIST/raw/{train,t10k}-{images-idx3,labels-idx1}-ubyte`, and patches the CUDA calls of
the reference so it runs on CPU with the gloo backend:
  torch.cuda.device_count -> $FAKE_NGPU, Tensor.cuda / Module.cuda -> identity,
  DistributedDataParallel(device_ids=...) -> CPU DDP, torch.load(map_location=cuda) -> CPU.
"""
import os

import numpy as np
import torch
import torch.nn as nn

from . import datasets, transforms  # noqa: F401

_ngpu = int(os.environ.get("FAKE_NGPU", "1"))
torch.cuda.device_count = lambda: _ngpu
torch.Tensor.cuda = lambda self, *a, **k: self
nn.Module.cuda = lambda self, *a, **k: self

_ddp_init = nn.parallel.DistributedDataParallel.__init__


def _ddp_cpu_init(self, module, *args, **kwargs):
    kwargs.pop("device_ids", None)
    kwargs.pop("output_device", None)
    _ddp_init(self, module, *args, **kwargs)


nn.parallel.DistributedDataParallel.__init__ = _ddp_cpu_init

_load = torch.load


def _load_cpu(f, map_location=None, **kwargs):
    return _load(f, map_location="cpu", **kwargs)


torch.load = _load_cpu
