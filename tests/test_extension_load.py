"""The in-tree extension loads on the CPU box too (dlopen resolves every symbol; no GPU call):
a missing definition -- e.g. a declaration in one translation unit's anonymous namespace --
fails here instead of on the GPU box."""
import glob
import os

import pytest

from conftest import REPO


def test_in_tree_extension_resolves():
    if not glob.glob(os.path.join(REPO, "pytorch_distributed_mnist_amd", "_C*.so")):
        pytest.skip("extension not built (python -m pytorch_distributed_mnist_amd.build)")
    from pytorch_distributed_mnist_amd.ops import _ext
    C = _ext.require()
    for name in ("optim_step", "cnn_fwd", "cnn_bwd", "fc1_bwd", "RcclComm", "XgmiReducer",
                 "rccl_cancel_init"):
        assert hasattr(C, name), name
