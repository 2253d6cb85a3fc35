"""Process-group bring-up and rank/device mapping.

Reference behaviour (``multi_proc_single_gpu.py:163-183``): every rank calls
``dist.init_process_group(backend, init_method='tcp://127.0.0.1:23456',
world_size, rank)``, splits the node batch by the GPU count, and uses
``cuda:<rank>``.  Here:

* ``--backend nccl`` initialises the default group as ``cpu:gloo,cuda:nccl``:
  the TCP store and a gloo group carry the *control plane* (unique-id exchange,
  barriers, tiny host reductions) while the *data plane* (gradient buckets,
  parameter broadcast) runs on our own C++ RCCL communicator over xGMI
  (``csrc/runtime/comm.cpp``), on a dedicated HIP stream and capturable into the
  step's hipGraph.  torch's own NCCL communicator is never created.
* ``--backend gloo`` keeps everything on torch gloo (CPU path / oracle).
* the device is selected with ``torch.cuda.set_device(local_rank)`` (the
  reference never calls it; SURVEY.md §7.1 fix 3).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist
from .. import knobs


def distributed_is_initialized() -> bool:
    """Reference ``multi_proc_single_gpu.py:21-25``."""
    return dist.is_available() and dist.is_initialized()


@dataclass
class DistContext:
    rank: int
    world_size: int
    local_rank: int
    backend: str            # user-facing: "nccl" or "gloo"
    device: torch.device
    initialized: bool
    timeout_s: float = 1800.0     # --timeout: rendezvous, RCCL init and bounded host syncs

    @property
    def is_gpu(self) -> bool:
        return self.device.type == "cuda"


def pick_device(local_rank: int, want: str = "auto") -> torch.device:
    if want == "cpu":
        return torch.device("cpu")
    if want in ("auto", "cuda") and torch.cuda.is_available():
        n = torch.cuda.device_count()
        if knobs.get("PDM_SHARE_DEVICE") == "1":
            # test rehearsal only: every rank on device 0 (gloo data plane; RCCL refuses
            # two ranks on one GPU) to exercise the multi-rank GPU program on a 1-GPU box
            torch.cuda.set_device(0)
            return torch.device("cuda", 0)
        if local_rank >= n:
            raise RuntimeError(f"local rank {local_rank} has no GPU (device_count={n})")
        torch.cuda.set_device(local_rank)
        return torch.device("cuda", local_rank)
    if want == "cuda":
        raise RuntimeError("--device cuda requested but no HIP device is visible")
    return torch.device("cpu")


def init_distributed(backend: str, init_method: Optional[str], world_size: int, rank: int,
                     local_rank: int, device: torch.device, timeout_s: float = 1800.0,
                     init_pg: bool = True) -> DistContext:
    """Initialise the default process group (control plane) for this rank."""
    initialized = False
    if init_pg and not distributed_is_initialized():
        if backend == "nccl" and device.type == "cuda":
            pg_backend = "cpu:gloo,cuda:nccl"
        elif backend in ("nccl", "gloo"):
            pg_backend = "gloo"
        else:
            pg_backend = backend
        kwargs = dict(backend=pg_backend, world_size=world_size, rank=rank,
                      timeout=datetime.timedelta(seconds=timeout_s))
        if init_method:
            kwargs["init_method"] = init_method
        dist.init_process_group(**kwargs)
        initialized = True
    elif distributed_is_initialized():
        initialized = True
    return DistContext(rank=rank, world_size=world_size, local_rank=local_rank, backend=backend,
                       device=device, initialized=initialized, timeout_s=float(timeout_s))


def control_barrier() -> None:
    """Host barrier on the control plane: an all-reduce of a CPU tensor always runs on the
    gloo backend of the default group, so no torch NCCL communicator is ever created (a
    plain ``dist.barrier()`` on a ``cpu:gloo,cuda:nccl`` group may pick the cuda backend)."""
    if distributed_is_initialized():
        dist.all_reduce(torch.zeros(1))


def shutdown() -> None:
    if distributed_is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:
            pass


def default_store():
    """The rendezvous KV store of the default group (TCPStore for tcp:// / env://)."""
    from torch.distributed import distributed_c10d as c10d
    return c10d._get_default_store()


def env_rank_info():
    """(rank, world_size, local_rank) from torchrun/launch env vars, or None."""
    if "LOCAL_RANK" not in os.environ and "RANK" not in os.environ:
        return None
    local_rank = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    rank = int(os.environ.get("RANK", local_rank))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    return rank, ws, local_rank
