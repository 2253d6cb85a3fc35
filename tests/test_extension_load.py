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


def test_fc1_head_grid_bounds():
    """fc1_head (fc1_fwd + head in one launch, PDM_FUSE_HEAD=1) only takes grids the chip holds
    at once: a head workgroup waits for every split-K workgroup of its launch."""
    if not glob.glob(os.path.join(REPO, "pytorch_distributed_mnist_amd", "_C*.so")):
        pytest.skip("extension not built (python -m pytorch_distributed_mnist_amd.build)")
    from pytorch_distributed_mnist_amd.ops import _ext
    from pytorch_distributed_mnist_amd.runtime.cnn_step import choose_splitk
    C = _ext.require()
    assert C.fc1_head_grid(32, choose_splitk(32), 32) == 32 + 8
    assert C.fc1_head_grid(256, choose_splitk(256), 256) == 256 + 64
    assert C.fc1_head_grid(512, choose_splitk(512), 512) == 256 + 128
    assert C.fc1_head_grid(1024, choose_splitk(1024), 1024) == 0      # 512 workgroups
    assert C.fc1_head_grid(4096, choose_splitk(4096), 4096) == 0      # 128-row blocks
