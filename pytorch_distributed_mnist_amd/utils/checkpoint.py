"""Checkpoint save/load in the reference's format.

Format (reference ``multi_proc_single_gpu.py:249-271``, verified in SURVEY.md §2.8):
``checkpoints/checkpoint_{epoch}.pth.tar`` = ``torch.save({'epoch': epoch+1,
'state_dict': {'module.<name>': tensor, ...}, 'best_acc': float,
'optimizer': torch-optimizer state_dict})`` written by rank 0 every epoch, plus a
byte copy ``model_best.pth.tar`` when the test accuracy improved.

Differences (deliberate, format-invisible): the write is atomic (temp file +
``os.replace``) so a crash never leaves a truncated checkpoint, tensors are
saved on the CPU (loadable anywhere, still accepted by the reference's
``torch.load(map_location=device)``), and loading always uses
``weights_only=True`` — the format contains only tensors/dicts/lists/numbers.
"""
from __future__ import annotations

import os
import shutil
import tempfile

import torch

CHECKPOINT_DIR = "checkpoints"


def checkpoint_path(epoch: int, directory: str = CHECKPOINT_DIR) -> str:
    return os.path.join(directory, "checkpoint_{}.pth.tar".format(epoch))


def best_path(directory: str = CHECKPOINT_DIR) -> str:
    return os.path.join(directory, "model_best.pth.tar")


def _atomic_save(obj, path: str) -> None:
    d = os.path.dirname(path) or "."
    fd, tmp = tempfile.mkstemp(prefix=".tmp_ckpt_", dir=d)
    try:
        with os.fdopen(fd, "wb") as f:
            torch.save(obj, f)
        os.replace(tmp, path)
    except BaseException:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise


def save_checkpoint(state: dict, is_best: bool, epoch: int, directory: str = CHECKPOINT_DIR) -> str:
    os.makedirs(directory, exist_ok=True)
    filename = checkpoint_path(epoch, directory)
    _atomic_save(state, filename)
    if is_best:
        dst = best_path(directory)
        tmp = dst + ".tmp"
        shutil.copyfile(filename, tmp)
        os.replace(tmp, dst)
    return filename


def load_checkpoint(path: str, map_location="cpu") -> dict:
    return torch.load(path, map_location=map_location, weights_only=True)


def make_state(epoch_done: int, arena, best_acc: float, optimizer) -> dict:
    return {
        "epoch": epoch_done,
        "state_dict": arena.state_dict(prefix="module."),
        "best_acc": best_acc,
        "optimizer": optimizer.state_dict(),
    }
