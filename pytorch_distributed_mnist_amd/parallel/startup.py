"""Rank-agreed start-up check of the step structure (the app's world size > 1 path).

The reference's DDP has one fixed structure that is never in doubt
(``multi_proc_single_gpu.py:188-189``: bucketed all-reduce inside ``loss.backward()``).  This
framework picks among structures built for MI355X (the direct xGMI transport with the conv
bucket exchanged inside the optimizer launch, the same without the exchange, RCCL with the
fc1 update carried into the next forward), and the first N-GPU run of a structure is the
first time its peer traffic is real.  So before the first epoch the app runs a few steps of
each candidate in preference order through ``calibrate.calibrate`` (setup / warm / steps /
check phases, every failure agreed over the control plane, parameter fingerprints compared
over the ranks) and keeps the FIRST that passes on every rank; a failing one is reported on
stderr and the next is tried (``rccl-nocarry`` last: plain RCCL collectives).

The check trains on the start epoch's first batches, so the state it changes is put back
afterwards, pass or fail: the fp32 weights, the optimizer state and step count (snapshot
taken after the rank-0 broadcast / resume, identical on every rank) and the bf16 compute
copies.  The device data-step counter moves on; the first epoch then starts at the next
epoch boundary of the counter (GpuStepBase.set_train_indices), so the epoch's batches and
every printed line are those of a run without the check (tests/test_app_cpu.py).

A fault injected into a phase (PDM_CALIB_FAULT, calibrate._fault) raises BEFORE the phase's
work on that rank.  On the GPU the peers' collectives then wait on the device until their
deadline (the xgmi kernels' own, or the host's for RCCL), as for any rank that fails mid-step;
on the CPU / gloo rehearsal, whose data-plane collectives are synchronous host calls with no
deadline, only the 'check' phase (after the steps) can be injected without a deadlock.
"""
from __future__ import annotations

import sys
from typing import Callable, List, Optional

import torch

from .. import knobs
from .calibrate import Candidate, ControlPlane, calibrate, tensor_fingerprint


class Snapshot:
    """The training state a check may change (GPU and CPU programs)."""

    def __init__(self, program):
        self.program = program
        opt = program.optimizer
        program.sync_master()
        self.params = program.arena.params.detach().clone()
        self.state = {k: v.detach().clone() for k, v in opt.state_buffers().items()}
        self.step = opt.step_count

    @torch.no_grad()
    def restore(self) -> None:
        p, opt = self.program, self.program.optimizer
        p.arena.params.copy_(self.params)
        for k, v in opt.state_buffers().items():
            v.copy_(self.state[k])
        opt.step_count = self.step
        if p.gpu is not None:
            opt.sync_step()
            p.gpu._dev_step = self.step
            if hasattr(p.gpu, "refresh_shadows"):
                p.gpu.refresh_shadows()      # bf16 compute copies of the restored weights
            torch.cuda.synchronize(p.device)


class StructureCandidate(Candidate):
    """One step structure of a program: `apply()` switches the program to it."""

    def __init__(self, name: str, program, apply: Callable[[], None], snap: Snapshot,
                 indices: torch.Tensor, sync: Callable[[str, bool], None], abortable: bool,
                 devhang: bool = False):
        self.name, self.program, self._apply, self.snap = name, program, apply, snap
        self.indices, self._sync, self.abortable = indices, sync, abortable
        self.devhang = devhang
        self._pos = 0

    def setup(self) -> None:
        self._apply()
        p = self.program
        # fault injection (PDM_CALIB_FAULT "<rank>:<name>:devhang"): an xgmi structure whose
        # persistent collective this rank never launches -- a real device hang, bounded by
        # the transport's device deadline (reducer.GradReducer.fault_no_collective)
        p.reducer.fault_no_collective = self.devhang
        # xgmi: re-arm the transport (a structure before this one, or a device deadline,
        # left its counters elsewhere); the setup agreement orders every rank's reset before
        # any rank's first launch
        p.reducer.reset_transport()
        p.set_train_indices(self.indices)
        self._pos = 0
        if p.gpu is not None:
            p.gpu.begin_epoch()
            p.gpu.prepare(p.batch_size)          # captures (no collective runs)

    def enqueue(self, k: int) -> int:
        p = self.program
        if p.gpu is not None:
            p.gpu.train_steps(p.batch_size, k)
            return k
        from ..runtime.cpu_step import train_step_cpu
        buf = p.metrics.buf[0:3]
        for start, size in p._bounds[self._pos:self._pos + k]:
            idx = p.train_idx_cpu[start:start + size]
            train_step_cpu(p.model, p.arena, p.train_split.images[idx],
                           p.train_split.labels[idx], p.reducer, p.optimizer, buf)
        self._pos += k
        return k

    def sync(self) -> None:
        self._sync(f"start-up check ({self.name})", self.abortable)

    def check(self) -> None:
        p = self.program
        p.reducer.check()
        if p.gpu is not None:
            p.gpu.check_device()

    def fingerprint(self) -> int:
        p = self.program
        p.sync_master()
        self._sync("start-up check fingerprint", self.abortable)
        return tensor_fingerprint(p.arena.params, *p.optimizer.state_buffers().values())

    def recover(self) -> None:
        self._sync("start-up check recovery", True)
        self.snap.restore()


def check_structures(program, cands: List[tuple], indices: torch.Tensor, rank: int, ws: int,
                     sync: Callable[[str, bool], None], steps: int = 8,
                     log: Optional[Callable[[str], None]] = None) -> str:
    """Run the candidates [(name, apply, abortable)] in preference order until one passes on
    every rank; leave the program on it, with the pre-check training state restored.
    Returns the chosen name (raises if none passes)."""
    log = log or (lambda s: print(s, file=sys.stderr, flush=True))
    snap = Snapshot(program)
    full = len(indices) // program.batch_size
    k = max(1, min(int(steps), full // 2 if full >= 2 else 1))
    faults = (knobs.get("PDM_CALIB_FAULT") or "").split(",")
    objs = [StructureCandidate(n, program, fn, snap, indices, sync, ab,
                               devhang=f"{rank}:{n}:devhang" in faults) for n, fn, ab in cands]
    cal = calibrate(objs, ControlPlane(ws), rank, warm_steps=k, timed_steps=k, rounds=1,
                    budget_s=float("inf"), inject=knobs.get("PDM_CALIB_FAULT"),
                    first_ok=True, log=lambda s: None)
    best = cal.best
    if best != cands[0][0] and rank == 0:
        for n in cal.notes:
            log(f"warning: step structure {n}")
        log(f"warning: using step structure {best!r} instead of {cands[0][0]!r}")
    for n, fn, _ in cands:
        if n == best:
            fn()
            break
    program.reducer.fault_no_collective = False
    sync("start-up check", True)
    program.reducer.reset_transport()
    snap.restore()
    if ws > 1:
        from .dist import control_barrier
        control_barrier()                    # every rank re-armed before any launches
    return best
