"""The MFMA-fragment-major operand layout (csrc/kernels.h frag_pos) and its Python builders."""
import random

import torch

from pytorch_distributed_mnist_amd.runtime.cnn_step import frag_major, frag_major_t


def frag_pos(m, k, K):   # csrc/kernels.h
    return (((m >> 4) * (K >> 5) + (k >> 5)) * 64 + ((k >> 3) & 3) * 16 + (m & 15)) * 8 + (k & 7)


def test_frag_major_matches_frag_pos():
    w = torch.arange(128 * 9216, dtype=torch.float64).reshape(128, 9216)
    f, ft = frag_major(w), frag_major_t(w)
    rnd = random.Random(0)
    for _ in range(4000):
        n, k = rnd.randrange(128), rnd.randrange(9216)
        assert f[frag_pos(n, k, 9216)] == w[n, k]          # W1: m = n (fc1_fwd B operand)
        assert ft[frag_pos(k, n, 128)] == w[n, k]          # W1^T: m = feature (dX A operand)


def test_fragment_is_one_contiguous_wave_load():
    # lane l of a 16x16x32 operand load: row l & 15, k = 8 (l >> 4) .. + 7 -> 16 B at 16 l
    w = torch.arange(64 * 96, dtype=torch.float64).reshape(64, 96)
    f = frag_major(w).view(-1, 64, 8)                       # [block][lane][8]
    for mb in range(4):
        for kb in range(3):
            blk = f[mb * 3 + kb]
            for lane in range(64):
                m, k0 = 16 * mb + (lane & 15), 32 * kb + 8 * (lane >> 4)
                assert torch.equal(blk[lane], w[m, k0:k0 + 8])
