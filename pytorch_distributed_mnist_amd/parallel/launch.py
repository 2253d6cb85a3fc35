"""Launch-mode detection and the spawn launcher.

The reference supports two launch styles but switching needs a source edit
(``multi_proc_single_gpu.py:353-359``, README lines 10-35), and its
``--local_rank`` flag breaks under torch>=2's launcher, which passes
``--local-rank=N``.  Here the mode is detected at run time:

* *launched* — ``torch.distributed.launch`` / ``torchrun`` started this process
  (``LOCAL_RANK``/``RANK`` in the environment, or an explicit ``--local-rank``):
  run one rank in this process (reference ``run_dist_launch``, :278-281);
* *spawn* — otherwise start ``world_size`` ranks with
  ``torch.multiprocessing.spawn`` (reference ``demo_spawn``/``run_spawn``, :273-285).
"""
from __future__ import annotations

import os

import torch.multiprocessing as mp


def is_launched(args) -> bool:
    if "LOCAL_RANK" in os.environ or "RANK" in os.environ:
        return True
    return getattr(args, "local_rank_given", False)


def launched_rank(args):
    """(rank, world_size, local_rank) for a launched process."""
    if "LOCAL_RANK" in os.environ or "RANK" in os.environ:
        local_rank = int(os.environ.get("LOCAL_RANK", args.local_rank))
        rank = int(os.environ.get("RANK", local_rank))
        ws = int(os.environ.get("WORLD_SIZE", args.world_size))
        return rank, ws, local_rank
    return args.local_rank, args.world_size, args.local_rank


def spawn(fn, nprocs: int, args) -> None:
    """``mp.spawn(fn, args=(args,), nprocs=nprocs)``; a failing child re-raises here."""
    mp.spawn(fn, args=(args,), nprocs=nprocs, join=True)
