"""Cross-rank model verification before the initial weight broadcast.

The reference builds ``DistributedDataParallel(model, device_ids=[rank])``
(``multi_proc_single_gpu.py:188-189``); DDP's constructor first checks that every
rank holds the same parameters (``_verify_param_shape_across_processes``: an
all-gather of the parameter count, then the shapes) and only then broadcasts rank
0's weights.  Our ranks broadcast one flat fp32 arena, so a rank built with another
``--arch`` (or another layout) would receive bytes of a different model: this check
makes that a clear error on every rank instead of undefined behaviour.

The signature travels as a small int64 CPU tensor through ``dist.all_gather`` on the
control plane (a CPU tensor always takes the gloo backend of the default group, so
no torch NCCL communicator is created).
"""
from __future__ import annotations

import hashlib
from typing import List

import torch
import torch.distributed as dist

from .dist import distributed_is_initialized

_SIG_LEN = 5


def model_signature(spec) -> List[int]:
    """[total params, parameter tensors, arena floats, shape digest, name digest]."""
    shapes = ";".join(f"{p.name}:{'x'.join(map(str, p.torch_shape))}" for p in spec.torch_order())
    h = int.from_bytes(hashlib.sha256(shapes.encode()).digest()[:7], "little")
    n = int.from_bytes(hashlib.sha256(spec.name.encode()).digest()[:7], "little")
    return [spec.num_params, len(spec.params), spec.total, h, n]


def _describe(sig: List[int]) -> str:
    return f"{sig[0]} parameters in {sig[1]} tensors (arena of {sig[2]} floats)"


def verify_params_across_ranks(spec, rank: int, world_size: int) -> None:
    """Raise on every rank if any rank's model differs from rank 0's."""
    if world_size <= 1 or not distributed_is_initialized():
        return
    mine = torch.tensor(model_signature(spec), dtype=torch.int64)
    got = [torch.zeros(_SIG_LEN, dtype=torch.int64) for _ in range(world_size)]
    dist.all_gather(got, mine)
    ref = got[0].tolist()
    bad = [(r, g.tolist()) for r, g in enumerate(got) if g.tolist() != ref]
    if bad:
        r, sig = bad[0]
        what = ("a different set of parameter shapes" if sig[:3] == ref[:3]
                else _describe(sig))
        raise RuntimeError(
            f"parameter verification failed (DDP model check): rank {r} has {what}, while "
            f"rank 0 has {_describe(ref)} (model {spec.name!r} on rank {rank}); every rank must "
            f"build the same model (--arch) before the initial weight broadcast")
