"""Our epoch index vector == torch.utils.data.DistributedSampler (reference :142-144)."""
import pytest
import torch
from torch.utils.data import DistributedSampler

from pytorch_distributed_mnist_amd.data.sampler import (batch_bounds, distributed_indices,
                                                        num_samples_per_rank)


class _DS(torch.utils.data.Dataset):
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return i


@pytest.mark.parametrize("n", [60000, 10000, 37, 5, 3])
@pytest.mark.parametrize("ws", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("epoch", [0, 1, 3])
def test_matches_torch_sampler(n, ws, epoch):
    for rank in range(ws):
        s = DistributedSampler(_DS(n), num_replicas=ws, rank=rank)
        s.set_epoch(epoch)
        ref = list(iter(s))
        ours = distributed_indices(n, ws, rank, epoch).tolist()
        assert ours == ref
        assert len(ours) == num_samples_per_rank(n, ws)


def test_global_batch_is_world_size_invariant():
    # rank r's batch k at ws is perm positions [256k + r :: ws] -> the union over ranks of
    # batch k is the same image set at every ws ([OBS-inv]).
    n, gb = 60000, 256
    for ws in (1, 2, 4, 8):
        per = gb // ws
        sets = []
        for k in range(3):
            u = set()
            for r in range(ws):
                idx = distributed_indices(n, ws, r, 0)
                u.update(idx[k * per:(k + 1) * per].tolist())
            sets.append(u)
        if ws == 1:
            base = sets
        assert sets == base


def test_batch_bounds():
    assert batch_bounds(60000, 256)[-1] == (59904, 96)
    assert len(batch_bounds(60000, 256)) == 235
    assert len(batch_bounds(7500, 32)) == 235
    assert batch_bounds(10000, 256)[-1] == (9984, 16)


def test_prefetcher_matches_direct_computation():
    from pytorch_distributed_mnist_amd.data.sampler import EpochIndexPrefetcher, distributed_indices
    pf = EpochIndexPrefetcher(1000, 4, 3)
    try:
        for e in (0, 1, 2, 5, 6):           # in order, then a jump (not prefetched)
            assert torch.equal(pf.get(e), distributed_indices(1000, 4, 3, e))
    finally:
        pf.close()
