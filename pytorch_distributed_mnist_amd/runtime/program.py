"""Per-rank training program: device-resident data + step kernels + graphs.

What replaces the reference's DataLoader/Trainer machinery
(``multi_proc_single_gpu.py:77-161``):

* the uint8 train/test sets are uploaded to the device once (47 + 8 MB);
* each epoch the rank's DistributedSampler-identical index vector is uploaded
  (int32, <=240 KB) and a device step counter is reset;
* a train step is a fixed chain of HIP kernels that read the batch indices via
  that counter, so the step has no host inputs at all and is captured once per
  batch size into a hipGraph (``torch.cuda.CUDAGraph`` on ROCm) — the
  full-batch graph and the ragged-tail graph;
* loss/accuracy accumulate on the device; the host reads them once per epoch.

On the CPU (gloo path) the same program runs the torch reference step.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..data.sampler import batch_bounds
from ..utils.metrics import DeviceMetrics
from .cpu_step import eval_step_cpu, train_step_cpu
from .structure import StepStructure


class TrainProgram:
    def __init__(self, model: str, dtype: str, arena, optimizer, reducer, train_split, test_split,
                 batch_size: int, eval_batch: Optional[int] = None, use_graphs: bool = True,
                 structure: Optional[StepStructure] = None):
        self.model = model
        # how the step is laid out (fusions, band splits, collective placement): read from
        # the PDM_* knobs once, here, unless the caller passes one
        self.structure = structure if structure is not None else StepStructure.from_env()
        self.dtype = dtype
        self.arena = arena
        self.optimizer = optimizer
        self.reducer = reducer
        self.device = arena.device
        self.batch_size = int(batch_size)
        if self.batch_size < 1:
            raise ValueError("per-rank batch size must be >= 1")
        self.eval_batch = int(eval_batch or self.batch_size)
        self.use_graphs = bool(use_graphs)
        self.metrics = DeviceMetrics(self.device)
        self.is_gpu = self.device.type == "cuda"
        self.train_split = train_split
        self.test_split = test_split
        self.train_idx_cpu: Optional[torch.Tensor] = None
        self._bounds = []
        self._n_train = 0
        # host sync before the once-per-epoch metric read: set by the app to a bounded
        # wait (parallel.bounded_sync) so a hung collective raises after --timeout
        self.sync_fn = None
        if self.is_gpu:
            from .gpu_step import make_gpu_step
            self.gpu = make_gpu_step(self, use_graphs=use_graphs)
        else:
            if dtype != "fp32":
                raise ValueError("the CPU path computes in fp32 only (--dtype fp32)")
            self.gpu = None

    # -- epochs ---------------------------------------------------------------
    def set_train_indices(self, indices: torch.Tensor, next_indices=None) -> None:
        """Install this rank's sample order for the coming epoch (and, on the GPU, start
        materialising the next epoch's, ``next_indices``, beside this one's first steps).

        GPU: the pinned int32 order the prefetcher hands over is read by the gather kernel in
        place; the batch bounds are arithmetic (full batches, then one ragged tail, as the
        DataLoader)."""
        self._n_train = len(indices)
        if self.gpu is not None:
            self.gpu.set_train_indices(indices, next_indices)
            return
        self.train_idx_cpu = indices.to(torch.int64)
        self._bounds = batch_bounds(len(indices), self.batch_size)

    @property
    def steps_per_epoch(self) -> int:
        return -(-self._n_train // self.batch_size)

    def train_epoch(self):
        self.metrics.reset(DeviceMetrics.TRAIN)
        self.optimizer.sync_hyperparams()
        if self.gpu is not None:
            self.gpu.begin_epoch()
            full, tail = divmod(self._n_train, self.batch_size)
            self.gpu.train_steps(self.batch_size, full)      # full batches come first
            if tail:
                self.gpu.train_step(tail)                     # ragged tail
            if self.sync_fn is not None:
                self.sync_fn("training epoch")
            self.gpu.check_device()
        else:
            buf = self.metrics.buf[0:3]
            for start, size in self._bounds:
                idx = self.train_idx_cpu[start:start + size]
                train_step_cpu(self.model, self.arena, self.train_split.images[idx],
                               self.train_split.labels[idx], self.reducer, self.optimizer, buf)
        return self.metrics.read(DeviceMetrics.TRAIN)

    # -- fc1 optimizer-state sharding (CNN, world size > 1) ------------------------------------
    def shard_supported(self) -> bool:
        return self.shard_unsupported_reason() is None

    def shard_unsupported_reason(self):
        """None when the fc1 update can be sharded here, else why not (for the user)."""
        if self.model != "cnn":
            return f"the {self.model} model has no fc1 layer to shard"
        if self.gpu is not None:
            if not hasattr(self.gpu, "shard_unsupported_reason"):
                return (f"the {self.dtype} CNN program has no sharded update "
                        "(only the bf16 CNN program does)")
            return self.gpu.shard_unsupported_reason()
        ws = self.reducer.comm.world_size
        if not self.reducer.can_shard:
            return f"the {self.reducer.kind} gradient transport has no reduce-scatter"
        if 128 % ws:
            return f"world size {ws} does not split fc1's 128 rows evenly"
        return None

    def set_shard_fc(self, on: bool = True) -> None:
        """Shard the fc1 weight's optimizer update over the ranks: its gradient is
        reduce-scattered (GPU; the gloo CPU path all-reduces it), each rank updates its
        128 / world_size rows and the updated rows are all-gathered (bf16 rows on the GPU,
        fp32 rows on the CPU).  Optimizer state of the other rows is not kept current:
        ``sync_master`` gathers it (checkpoints)."""
        if self.gpu is not None:
            self.gpu.set_shard_fc(on)
            return
        if not on:
            self.sync_master()
            self.reducer.clear_shard()
            return
        ws = self.reducer.comm.world_size
        self.reducer.set_shard(0, self.arena.spec.offset("fc1.weight"), 128 // ws * 9216)

    def sync_master(self) -> None:
        """Make the fp32 master weights and optimizer state whole on every rank (a no-op
        unless an update is sharded; collective then: every rank calls it)."""
        if self.gpu is not None:
            if hasattr(self.gpu, "sync_master"):
                self.gpu.sync_master()
            return
        sh = getattr(self.reducer, "shard", None)
        if sh is not None:
            _, start, count = sh
            n = count * self.reducer.comm.world_size
            for buf in self.optimizer.state_buffers().values():
                self.reducer.gather(buf[start:start + n])

    def use_structure(self, reducer, rccl_mode: Optional[str] = None,
                      xgmi_exchange: Optional[bool] = None) -> None:
        """Switch the step to another gradient reducer and step structure (the start-up
        check's fallbacks, parallel/startup.py; bench.py's calibration candidates): graphs
        are re-captured on next use."""
        self.reducer = reducer
        g = self.gpu
        if g is None:
            return
        if getattr(g, "shard_fc", False):
            g.set_shard_fc(False)            # (gathers the sharded state on the old reducer)
        g.reducer = reducer
        g.use_graphs = self.use_graphs and reducer.capturable
        if rccl_mode is not None and hasattr(g, "set_rccl_mode"):
            g.set_rccl_mode(rccl_mode, invalidate=False)
        if xgmi_exchange is not None and hasattr(g, "xgmi_exchange"):
            g.xgmi_exchange = bool(xgmi_exchange) and self.structure.xgmi_exchange
        g.invalidate_graphs()

    def run_steps(self, n: int, bsz: Optional[int] = None) -> None:
        """Run ``n`` full steps from the current counter (bench helper; GPU only)."""
        self.gpu.train_steps(bsz or self.batch_size, n)

    @torch.no_grad()
    def evaluate(self):
        """Full, unsharded test-set pass on every rank (reference :99-116, :142-149)."""
        self.metrics.reset(DeviceMetrics.EVAL)
        n = len(self.test_split)
        if self.gpu is not None:
            self.gpu.evaluate()
            if self.sync_fn is not None:
                self.sync_fn("evaluation")
        else:
            buf = self.metrics.buf[3:6]
            for start, size in batch_bounds(n, self.eval_batch):
                eval_step_cpu(self.model, self.arena, self.test_split.images[start:start + size],
                              self.test_split.labels[start:start + size], buf)
        return self.metrics.read(DeviceMetrics.EVAL)


def build_local_program(arch: str, dtype: str, device, batch_size: int, train_split, test_split,
                        optimizer: str = "adam", lr: float = 1e-3, momentum: float = 0.9,
                        weight_decay: float = 1e-4, seed: int = 0, use_graphs: bool = True,
                        comm=None, force_comm: bool = False, transport: str | None = None):
    """Single-rank program without a process group (tests, bench at N=1, smoke)."""
    from types import SimpleNamespace

    from ..models.reference import MODULES
    from ..models.specs import get_spec
    from ..optim.flat import build_optimizer
    from ..parallel.comm import LocalComm
    from ..parallel.reducer import GradReducer
    from .arena import FlatArena

    torch.manual_seed(seed)
    spec = get_spec(arch)
    arena = FlatArena(spec, torch.device(device))
    arena.load_module(MODULES[arch]())
    opt = build_optimizer(optimizer, arena, SimpleNamespace(lr=lr, momentum=momentum,
                                                            weight_decay=weight_decay))
    comm = comm or LocalComm()
    reducer = GradReducer(comm, arena.grads, spec.bucket_bounds(), channels=spec.channel_bounds(),
                          force=force_comm,
                          transport=transport)
    return TrainProgram(arch, dtype, arena, opt, reducer, train_split, test_split, batch_size,
                        use_graphs=use_graphs)
