"""Per-rank sample order, bit-identical to ``torch.utils.data.DistributedSampler``.

The reference wraps the training set in ``data.DistributedSampler(dataset)``
(reference ``multi_proc_single_gpu.py:142-144``) with the defaults shuffle=True,
seed=0, drop_last=False, and calls ``set_epoch(epoch)`` every epoch
(``multi_proc_single_gpu.py:159-161, 231``).  The test loader is sequential and
unsharded (``multi_proc_single_gpu.py:146-149``).

Instead of a Python iterator feeding DataLoader workers, we materialise the whole
epoch's index vector once (one ``randperm`` on the host, ~1 ms for 60k) and upload
it to the device as int32; the step kernels then gather their batch straight from
the device-resident uint8 dataset.  The vector is computed with tensor ops (no
Python lists) but reproduces the sampler's padding/striding rules exactly, which
tests/test_sampler.py checks against torch's own class.
"""
from __future__ import annotations

import math

import torch


def num_samples_per_rank(n: int, world_size: int, drop_last: bool = False) -> int:
    if drop_last and n % world_size != 0:
        return math.ceil((n - world_size) / world_size)
    return math.ceil(n / world_size)


def distributed_indices(n: int, world_size: int, rank: int, epoch: int, *,
                        seed: int = 0, shuffle: bool = True,
                        drop_last: bool = False) -> torch.Tensor:
    """Indices rank ``rank`` visits in ``epoch`` (int64 CPU tensor)."""
    if not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} out of range for world_size {world_size}")
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        order = torch.randperm(n, generator=g)
    else:
        order = torch.arange(n)
    per_rank = num_samples_per_rank(n, world_size, drop_last)
    total = per_rank * world_size
    if not drop_last:
        pad = total - n
        if pad > 0:
            if pad <= n:
                order = torch.cat([order, order[:pad]])
            else:
                reps = math.ceil(pad / n)
                order = torch.cat([order, order.repeat(reps)[:pad]])
    else:
        order = order[:total]
    return order[rank:total:world_size].contiguous()


def sequential_indices(n: int) -> torch.Tensor:
    return torch.arange(n, dtype=torch.int64)


def batch_bounds(num: int, batch_size: int, drop_last: bool = False):
    """[(start, size)] of the batches a DataLoader would produce over ``num`` samples."""
    out = []
    start = 0
    while start < num:
        size = min(batch_size, num - start)
        if drop_last and size < batch_size:
            break
        out.append((start, size))
        start += size
    return out


class EpochIndexPrefetcher:
    """This rank's sample order for epoch e+1, computed on a worker thread while epoch e trains.

    The reference reshuffles inside its loop (``set_epoch``, multi_proc_single_gpu.py:231)
    and its DataLoader workers index lazily; here the whole epoch order is one
    ``randperm`` (~1.3 ms for 60k on the host).  ``get(e)`` returns epoch e's order
    (computed now if it was not prefetched) and queues epochs e+1 .. e+depth on the
    worker, so at an epoch boundary the host only hands over ready vectors (this epoch's,
    and with ``peek(e+1)`` the next one's, whose gather the device then runs early) and
    the GPU never idles behind the sampler.  torch ops release the GIL, so the worker overlaps the
    host's graph-replay loop.

    With ``int32=True`` (GPU programs) the worker also converts the order to int32, the
    form the gather kernel reads.  The worker makes no HIP call (no pinned allocation): a
    host-memory allocation from any thread would invalidate a graph capture running on the
    main thread.
    """

    def __init__(self, n: int, world_size: int, rank: int, int32: bool = False, depth: int = 2,
                 **kw):
        from concurrent.futures import ThreadPoolExecutor
        self.n, self.world_size, self.rank, self.kw = n, world_size, rank, kw
        self.int32 = int32
        self.depth = depth
        self._ex = ThreadPoolExecutor(max_workers=1, thread_name_prefix="pdm-sampler")
        self._futs = {}            # epoch -> future

    def _compute(self, epoch: int) -> torch.Tensor:
        idx = distributed_indices(self.n, self.world_size, self.rank, epoch, **self.kw)
        return idx.to(torch.int32) if self.int32 else idx

    def _future(self, epoch: int):
        f = self._futs.get(epoch)
        if f is None:
            f = self._futs[epoch] = self._ex.submit(self._compute, epoch)
        return f

    def get(self, epoch: int) -> torch.Tensor:
        """Epoch ``epoch``'s order; the next ``depth`` epochs' are then computed behind it."""
        idx = self._future(epoch).result()
        for e in list(self._futs):
            if e < epoch:
                self._futs.pop(e).cancel()
        for e in range(epoch + 1, epoch + 1 + self.depth):
            self._future(e)
        return idx

    def peek(self, epoch: int) -> torch.Tensor:
        """Epoch ``epoch``'s order (computed now if it was not prefetched), keeping it for
        the later ``get``: lets the device start on the next epoch's gather early."""
        return self._future(epoch).result()

    def close(self) -> None:
        for f in self._futs.values():
            f.cancel()
        self._ex.shutdown(wait=True)
        self._futs = {}
