"""Parameter layouts: torch (checkpoint) layout <-> MI355X kernel layout.

Checkpoints must stay interchangeable with the reference (``state_dict`` keys
``module.fc.weight`` etc., torch shapes; reference ``multi_proc_single_gpu.py:250-255``),
but the kernels want channels-last data:

* ``conv2.weight`` torch ``[co, ci, ky, kx]`` -> kernel ``[co, ky, kx, ci]`` so one
  3x3 tap is a contiguous K=32 slice = exactly one ``mfma_f32_16x16x32_bf16`` K-step.
* ``fc1.weight`` torch ``[128, c*h*w]`` (NCHW flatten) -> kernel ``[128, h, w, c]``
  matching the NHWC pooled activations the conv kernel writes.

Every parameter lives in one flat fp32 arena in *backward-ready order*
(last layer first), so a gradient bucket is a contiguous slice that becomes
ready as soon as its layers' backward kernels have run — the same reverse order
DDP's Reducer uses to form buckets (fc bucket first, conv bucket
second).  Conversions are pure permutations, so optimizer state converts with
the same functions.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, List, Tuple

import torch

ARENA_ALIGN = 64  # floats (256 B) between segments: 16-B vector loads never straddle


def _identity(t: torch.Tensor) -> torch.Tensor:
    return t


@dataclass
class ParamSpec:
    name: str                      # torch name, e.g. "fc1.weight"
    torch_shape: Tuple[int, ...]
    internal_shape: Tuple[int, ...]
    torch_index: int               # position in Module.parameters()
    to_internal: Callable[[torch.Tensor], torch.Tensor] = _identity
    to_torch: Callable[[torch.Tensor], torch.Tensor] = _identity
    bucket: int = 0
    # a channel of its own inside its bucket (channel_bounds): the direct xGMI transport
    # reduces it separately, so its consumers can wait for it alone
    own_channel: bool = False

    @property
    def numel(self) -> int:
        n = 1
        for s in self.torch_shape:
            n *= s
        return n


@dataclass
class ModelSpec:
    name: str
    params: List[ParamSpec]           # arena (backward-ready) order
    num_buckets: int = 1
    offsets: List[int] = field(default_factory=list)
    total: int = 0

    def __post_init__(self):
        off = 0
        self.offsets = []
        for p in self.params:
            self.offsets.append(off)
            off += p.numel
            off = (off + ARENA_ALIGN - 1) // ARENA_ALIGN * ARENA_ALIGN
        self.total = off

    def by_name(self, name: str) -> ParamSpec:
        for p in self.params:
            if p.name == name:
                return p
        raise KeyError(name)

    def offset(self, name: str) -> int:
        for p, o in zip(self.params, self.offsets):
            if p.name == name:
                return o
        raise KeyError(name)

    def torch_order(self) -> List[ParamSpec]:
        return sorted(self.params, key=lambda p: p.torch_index)

    def bucket_bounds(self) -> List[Tuple[int, int]]:
        """[(start, end)] float ranges of each gradient bucket in the arena."""
        bounds = []
        for b in range(self.num_buckets):
            idx = [i for i, p in enumerate(self.params) if p.bucket == b]
            start = self.offsets[idx[0]]
            last = idx[-1]
            end = self.offsets[last + 1] if last + 1 < len(self.params) else self.total
            bounds.append((start, end))
        return bounds

    def channel_bounds(self) -> Tuple[List[Tuple[int, int]], List[List[int]]]:
        """Buckets cut further at the parameters that take a channel of their own: ([(start,
        end)] of every channel in arena order, [channel indices of bucket b])."""
        chans, of_bucket = [], []
        for b, (bs, be) in enumerate(self.bucket_bounds()):
            cuts = [bs]
            for i, p in enumerate(self.params):
                if p.bucket == b and p.own_channel:
                    lo = self.offsets[i]
                    hi = self.offsets[i + 1] if i + 1 < len(self.params) else self.total
                    cuts += [lo, min(hi, be)]
            cuts.append(be)
            pts = sorted(set(cuts))
            of_bucket.append([])
            for lo, hi in zip(pts, pts[1:]):
                of_bucket[-1].append(len(chans))
                chans.append((lo, hi))
        return chans, of_bucket

    @property
    def num_params(self) -> int:
        return sum(p.numel for p in self.params)


def linear_spec() -> ModelSpec:
    return ModelSpec("linear", [
        ParamSpec("fc.weight", (10, 784), (10, 784), 0),
        ParamSpec("fc.bias", (10,), (10,), 1),
    ], num_buckets=1)


def _conv2_to_internal(t):   # [co, ci, ky, kx] -> [co, ky, kx, ci]
    return t.permute(0, 2, 3, 1).contiguous()


def _conv2_to_torch(t):      # [co, ky, kx, ci] -> [co, ci, ky, kx]
    return t.permute(0, 3, 1, 2).contiguous()


def _fc1_to_internal(t):     # [128, c*h*w] -> [128, h, w, c]
    return t.reshape(128, 64, 12, 12).permute(0, 2, 3, 1).contiguous()


def _fc1_to_torch(t):        # [128, h, w, c] -> [128, c*h*w]
    return t.reshape(128, 12, 12, 64).permute(0, 3, 1, 2).reshape(128, 9216).contiguous()


def _conv1_to_internal(t):   # [32, 1, 3, 3] -> [32, 9]
    return t.reshape(32, 9).contiguous()


def _conv1_to_torch(t):
    return t.reshape(32, 1, 3, 3).contiguous()


def cnn_spec() -> ModelSpec:
    # Bucket 0 = fc2 + fc1 (ready right after the fc1 backward GEMM, ~4.7 MB);
    # bucket 1 = conv2 + conv1 (ready after the fused conv backward kernel).
    # fc1.weight comes last in bucket 0, in a channel of its own: the xGMI transport reduces
    # the small fc parameters (fc2, fc1.bias) apart from it, so the optimizer waits only for
    # them while fc1.weight's 4.7 MB keep travelling until the next forward launch, which
    # carries its update (kernels/fc_carry.h)
    return ModelSpec("cnn", [
        ParamSpec("fc2.weight", (10, 128), (10, 128), 6, bucket=0),
        ParamSpec("fc2.bias", (10,), (10,), 7, bucket=0),
        ParamSpec("fc1.bias", (128,), (128,), 5, bucket=0),
        ParamSpec("fc1.weight", (128, 9216), (128, 12, 12, 64), 4,
                  _fc1_to_internal, _fc1_to_torch, bucket=0, own_channel=True),
        ParamSpec("conv2.weight", (64, 32, 3, 3), (64, 3, 3, 32), 2,
                  _conv2_to_internal, _conv2_to_torch, bucket=1),
        ParamSpec("conv2.bias", (64,), (64,), 3, bucket=1),
        ParamSpec("conv1.weight", (32, 1, 3, 3), (32, 9), 0,
                  _conv1_to_internal, _conv1_to_torch, bucket=1),
        ParamSpec("conv1.bias", (32,), (32,), 1, bucket=1),
    ], num_buckets=2)


SPECS = {"linear": linear_spec, "cnn": cnn_spec}


def get_spec(name: str) -> ModelSpec:
    try:
        return SPECS[name]()
    except KeyError:
        raise ValueError(f"unknown model {name!r}; choose from {sorted(SPECS)}") from None
