"""Launch-geometry helpers of the GPU step programs (pure Python, no GPU): the fc1 split-K
factor and the fp32 conv-backward work per workgroup."""
import pytest

from pytorch_distributed_mnist_amd.runtime.cnn_f32_step import conv_ipb
from pytorch_distributed_mnist_amd.runtime.cnn_step import choose_splitk


@pytest.mark.parametrize("B,cap,S", [(256, 32, 32), (32, 32, 32), (1024, 32, 8), (32, 96, 96),
                                     (64, 96, 96), (128, 96, 48), (256, 96, 32), (37, 32, 32),
                                     (2048, 32, 16), (4096, 32, 8), (8192, 32, 4)])
def test_fc1_split_k(B, cap, S):
    """~256 workgroups of (32-row m-tile, split): a divisor of 32 (9-k-step load batches) or
    48 / 96 (3-k-step batches) within the cap."""
    s = choose_splitk(B, cap=cap)
    assert s == S
    assert 32 % s == 0 or 96 % s == 0
    rows = 32 if B < 2048 else 128            # fc1_fwd's m-tile (kernels.h FC1_BIG_B)
    assert ((B + rows - 1) // rows) * s <= 256 or s == 1


@pytest.mark.parametrize("B", [1, 5, 32, 37, 64, 100, 256, 300, 1024])
def test_f32_conv_backward_units_fill_one_round(B, monkeypatch):
    """Split-bf16 conv backward: (image, band) units per workgroup so that one round of at most
    256 workgroups covers all 6 B units; the exact kernel: images per workgroup, ~2 rounds."""
    monkeypatch.delenv("PDM_F32_UPW", raising=False)
    monkeypatch.delenv("PDM_F32_IPB", raising=False)
    upw = conv_ipb(B, x3=True)
    blocks = -(-6 * B // upw)
    assert blocks <= 256 and (upw == 1 or -(-6 * B // (upw - 1)) > 256)
    ipb = conv_ipb(B, x3=False)
    assert -(-B // ipb) * 6 <= 512 + 6          # two rounds, plus one partial image group


def test_f32_conv_backward_knobs(monkeypatch):
    monkeypatch.setenv("PDM_F32_UPW", "7")
    monkeypatch.setenv("PDM_F32_IPB", "3")
    assert conv_ipb(256, x3=True) == 7
    assert conv_ipb(256, x3=False) == 3
