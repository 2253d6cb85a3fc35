"""Flat parameter / gradient arena.

DDP's Reducer copies every gradient into flat bucket buffers and back after the
all-reduce.  Here the parameters and gradients *are* flat
buffers from the start: one fp32 arena for master weights, one for gradients,
each parameter a view at a fixed 256-B-aligned offset (``models/specs.py``).
The backward kernels write straight into the gradient arena, a bucket is a
contiguous slice of it, the all-reduce runs in place, and the fused optimizer
kernel sweeps the whole arena in one launch — no copies, no per-tensor launches.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict

import torch

from ..models.specs import ModelSpec


class FlatArena:
    def __init__(self, spec: ModelSpec, device: torch.device):
        self.spec = spec
        self.device = torch.device(device)
        self.params = torch.zeros(spec.total, dtype=torch.float32, device=self.device)
        self.grads = torch.zeros(spec.total, dtype=torch.float32, device=self.device)

    # -- views ---------------------------------------------------------------
    def _view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        p = self.spec.by_name(name)
        off = self.spec.offset(name)
        return buf[off:off + p.numel].view(p.internal_shape)

    def param(self, name: str) -> torch.Tensor:
        return self._view(self.params, name)

    def grad(self, name: str) -> torch.Tensor:
        return self._view(self.grads, name)

    def view_of(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        """View of any arena-shaped buffer (e.g. optimizer state) for ``name``."""
        return self._view(buf, name)

    def bucket_views(self, buf: torch.Tensor | None = None):
        buf = self.grads if buf is None else buf
        return [buf[s:e] for s, e in self.spec.bucket_bounds()]

    # -- torch-layout conversion ----------------------------------------------
    def load_torch_params(self, named: Dict[str, torch.Tensor]) -> None:
        """Copy {torch_name: torch-layout tensor} into the arena."""
        with torch.no_grad():
            for p in self.spec.params:
                t = named[p.name].detach().to(torch.float32)
                if tuple(t.shape) != tuple(p.torch_shape):
                    raise ValueError(f"{p.name}: shape {tuple(t.shape)} != {p.torch_shape}")
                self.param(p.name).copy_(p.to_internal(t.cpu()).to(self.device))

    def load_module(self, module: torch.nn.Module) -> None:
        self.load_torch_params(dict(module.named_parameters()))

    def torch_tensors(self, buf: torch.Tensor) -> Dict[str, torch.Tensor]:
        """{torch_name: torch-layout CPU copy} of an arena-shaped buffer."""
        out = {}
        host = buf.detach().cpu()
        for p, off in zip(self.spec.params, self.spec.offsets):
            out[p.name] = p.to_torch(host[off:off + p.numel].view(p.internal_shape)).clone()
        return out

    def state_dict(self, prefix: str = "module.") -> "OrderedDict[str, torch.Tensor]":
        """Torch-format state dict in ``Module.parameters()`` order (CPU tensors)."""
        tensors = self.torch_tensors(self.params)
        sd = OrderedDict()
        for p in self.spec.torch_order():
            sd[prefix + p.name] = tensors[p.name]
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        named = {}
        for k, v in sd.items():
            key = k[len("module."):] if k.startswith("module.") else k
            named[key] = v
        missing = [p.name for p in self.spec.params if p.name not in named]
        unexpected = [k for k in named if k not in {p.name for p in self.spec.params}]
        if missing or unexpected:
            raise RuntimeError(f"Error(s) in loading state_dict: missing keys {missing}, "
                               f"unexpected keys {unexpected}")
        self.load_torch_params(named)

    def buffer_from_torch(self, named: Dict[str, torch.Tensor], out: torch.Tensor) -> None:
        """Fill an arena-shaped buffer ``out`` from torch-layout tensors."""
        with torch.no_grad():
            out.zero_()
            for p in self.spec.params:
                self.view_of(out, p.name).copy_(
                    p.to_internal(named[p.name].detach().to(torch.float32).cpu()).to(out.device))
