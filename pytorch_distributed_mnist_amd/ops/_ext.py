"""Loader for the in-tree native extension ``pytorch_distributed_mnist_amd/_C*.so``.

The extension holds every HIP kernel (gfx950) plus the C++ runtime pieces
(RCCL communicator, bucketed gradient reducer).  It is built in-tree by
``python -m pytorch_distributed_mnist_amd.build`` (or ``__graft_entry__.build()``)
so the ``.so`` travels with the repository snapshot to the GPU box.

There is deliberately no eager/PyTorch fallback for GPU tensors: if a CUDA
(HIP) device is in use and the extension is missing, ``require()`` raises.
"""
from __future__ import annotations

import glob
import importlib.util
import os
import sys

import torch  # noqa: F401  (binds the HIP runtime / RCCL before our .so loads)
from .. import knobs

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_MOD = None
_ERR = None


def ext_path():
    override = knobs.get("PDM_EXT_PATH")   # diagnostic builds (e.g. PDM_STAMPS)
    if override:
        return override
    cands = sorted(glob.glob(os.path.join(_PKG_DIR, "_C*.so")))
    return cands[0] if cands else None


def load(required: bool = True):
    global _MOD, _ERR
    if _MOD is not None:
        return _MOD
    path = ext_path()
    if path is None:
        _ERR = ("native extension pytorch_distributed_mnist_amd/_C*.so is not built; run "
                "`python -m pytorch_distributed_mnist_amd.build`")
    else:
        try:
            spec = importlib.util.spec_from_file_location("pytorch_distributed_mnist_amd._C", path)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules["pytorch_distributed_mnist_amd._C"] = mod
            _MOD = mod
            return mod
        except Exception as e:  # pragma: no cover - depends on build
            _ERR = f"failed to load native extension {path}: {e!r}"
    if required:
        raise RuntimeError(_ERR)
    return None


def require():
    return load(required=True)


def available() -> bool:
    return load(required=False) is not None
