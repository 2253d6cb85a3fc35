"""Data parallelism over RCCL/xGMI: process group, communicators, bucketed reducer, launch."""
from .comm import Communicator, LocalComm, RcclComm, TorchComm, bounded_sync, make_comm
from .dist import (DistContext, control_barrier, distributed_is_initialized, init_distributed,
                   pick_device, shutdown)
from .launch import is_launched, launched_rank, spawn
from .reducer import GradReducer
from .verify import verify_params_across_ranks

__all__ = ["Communicator", "LocalComm", "RcclComm", "TorchComm", "make_comm", "DistContext",
           "control_barrier", "distributed_is_initialized", "init_distributed", "pick_device",
           "shutdown", "is_launched", "launched_rank", "spawn", "GradReducer", "bounded_sync",
           "verify_params_across_ranks"]
