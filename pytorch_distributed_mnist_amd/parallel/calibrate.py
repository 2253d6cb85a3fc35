"""Fault-tolerant, rank-agreed choice of the gradient transport / step structure.

``bench.py`` (and any caller that wants the fastest structure for a node) times every
candidate step structure on the real step and keeps the fastest.  On a first run on new
hardware a candidate can fail in ways a one-GPU box never shows: a capture that the runtime
refuses, a peer mapping that works on some ranks only, a transport whose device error word
trips, replicas that drift apart.  The reference has none of this (its DDP has one fixed
structure, multi_proc_single_gpu.py:188-189), so the rule here is: a candidate that fails on
ANY rank is dropped on EVERY rank, its failure is recorded, the replicas are restored from
rank 0, and calibration continues with the others.  Only when no candidate survives (or
the replicas cannot be restored, i.e. the data plane itself is gone) is the run fatal.

Deadlock freedom: every control-plane collective (gloo, CPU tensors) is issued by every
rank unconditionally and in the same order; the candidate's own work (capture, replays,
device syncs) runs between those points inside ``try``, so a rank that fails mid-phase
still arrives at the next agreement point.  Device work is bounded by the caller's
``sync`` (a deadline; on expiry the communicator is aborted and the sync raises).

Phases per candidate (each closed by an agreement):
  setup  select the structure and capture its graphs (no collective executes)
  warm   replay ``warm_steps`` steps and drain the device
  timed  barrier, ``timed_steps`` steps, drain; the slowest rank's time
  check  the transport's error word, and a fingerprint of every replica's parameters and
         optimizer state gathered over the ranks: every rank must hold the same bits
"""
from __future__ import annotations

import math
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

PHASES = ("setup", "warm", "timed", "check")


class Candidate:
    """One step structure (override the hooks; the defaults do nothing)."""

    name = "?"

    def setup(self) -> None: ...
    def enqueue(self, k: int) -> int: return 0
    def sync(self) -> None: ...
    def check(self) -> None: ...
    def fingerprint(self) -> int: return 0
    def recover(self) -> None: ...


class ControlPlane:
    """Host collectives over the control plane (gloo, CPU tensors); identity at ws = 1."""

    def __init__(self, world_size: int):
        self.ws = world_size

    def _reduce(self, x: float, op) -> float:
        if self.ws == 1:
            return x
        import torch
        import torch.distributed as dist
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=op)
        return float(t.item())

    def agree(self, ok: bool) -> bool:
        import torch.distributed as dist
        return bool(self._reduce(1.0 if ok else 0.0, dist.ReduceOp.MIN if self.ws > 1 else None))

    def allmax(self, x: float) -> float:
        import torch.distributed as dist
        return self._reduce(x, dist.ReduceOp.MAX if self.ws > 1 else None)

    def barrier(self) -> None:
        self.allmax(0.0)

    def first_error(self, err: Optional[str]) -> Optional[str]:
        """Agreement with the reason: None iff no rank failed, else the lowest failing rank's
        message (every rank gets the same answer)."""
        if self.ws == 1:
            return err
        import torch.distributed as dist
        out = [None] * self.ws
        dist.all_gather_object(out, err)
        return next((e for e in out if e is not None), None)

    def allgather_int(self, x: int) -> List[int]:
        if self.ws == 1:
            return [int(x)]
        import torch
        import torch.distributed as dist
        t = torch.tensor([int(x)], dtype=torch.int64)
        out = [torch.zeros(1, dtype=torch.int64) for _ in range(self.ws)]
        dist.all_gather(out, t)
        return [int(o.item()) for o in out]


def _fault(inject: Optional[str], rank: int, name: str, phase: str) -> None:
    """Fault injection for tests: ``"<rank>:<candidate>:<phase>[,...]"`` raises in that
    phase on that rank (phase ``diverge`` is handled by the candidate itself)."""
    if not inject:
        return
    for item in inject.split(","):
        r, n, p = (item.split(":") + ["", "", ""])[:3]
        if int(r) == rank and n == name and p == phase:
            raise RuntimeError(f"injected fault ({name}, {phase}, rank {rank})")


class Calibration:
    """Outcome: ``times`` (ms per step, survivors only), ``best``, ``notes`` (one line per
    dropped or skipped candidate)."""

    def __init__(self):
        self.times: Dict[str, float] = {}
        self.notes: List[str] = []
        self.failed: Dict[str, str] = {}
        self.best: Optional[str] = None


def calibrate(cands: Sequence[Candidate], cp: ControlPlane, rank: int, *, warm_steps: int = 16,
              timed_steps: int = 48, rounds: int = 2, budget_s: float = 120.0,
              inject: Optional[str] = None, first_ok: bool = False,
              log: Callable[[str], None] = lambda s: None) -> Calibration:
    """Time every candidate (``rounds`` passes, alternate passes in reverse order to cancel
    clock-ramp bias, the minimum per candidate) and return the agreed outcome.
    ``first_ok``: a preference order instead -- stop at the first candidate that passes
    (the app's start-up check, parallel/startup.py); ``best`` is that one."""
    res = Calibration()
    t_start = time.monotonic()
    alive = list(cands)
    for rnd in range(max(1, rounds)):
        if first_ok and res.times:
            break
        order = alive if rnd % 2 == 0 else list(reversed(alive))
        for c in order:
            if c.name in res.failed:
                continue
            # the budget is judged on the slowest rank's clock, so every rank skips together
            spent = cp.allmax(time.monotonic() - t_start)
            if spent > budget_s and (res.times or rnd > 0):
                if c.name not in res.times:
                    res.notes.append(f"{c.name}: not calibrated (budget {budget_s:.0f} s spent)")
                    res.failed[c.name] = "budget"
                continue
            ms, why = _one(c, cp, rank, warm_steps, timed_steps, inject)
            if why is None:
                res.times[c.name] = min(ms, res.times.get(c.name, math.inf))
                if first_ok:
                    break
                continue
            res.failed[c.name] = why
            res.times.pop(c.name, None)
            res.notes.append(f"{c.name} failed calibration: {why}")
            if rank == 0:
                log(f"{c.name} failed calibration: {why}")
            err = None
            try:
                c.recover()
            except Exception as e:              # noqa: BLE001 (agreed below)
                err = f"rank {rank}: {type(e).__name__}: {e}"
            err = cp.first_error(err)
            if err is not None:
                raise RuntimeError(f"calibration: replicas could not be restored after "
                                   f"{c.name} failed ({err})")
        alive = [c for c in alive if c.name not in res.failed]
    if not res.times:
        raise RuntimeError("calibration: no step structure survived: " + "; ".join(res.notes))
    res.best = next(iter(res.times)) if first_ok else min(res.times, key=res.times.get)
    return res


def _one(c: Candidate, cp: ControlPlane, rank: int, warm: int, k: int,
         inject: Optional[str]) -> Tuple[float, Optional[str]]:
    """One timed pass of one candidate: (ms per step, None) or (inf, reason)."""
    def attempt(phase, fn):
        try:
            _fault(inject, rank, c.name, phase)
            fn()
            return None
        except Exception as e:                  # noqa: BLE001 (agreed by the caller)
            return f"{phase} on rank {rank}: {type(e).__name__}: {e}"

    err = cp.first_error(attempt("setup", c.setup))
    if err is not None:
        return math.inf, err
    err = cp.first_error(attempt("warm", lambda: (c.enqueue(warm), c.sync())))
    if err is not None:
        return math.inf, err
    cp.barrier()
    box = {}

    def timed():
        t0 = time.perf_counter()
        c.enqueue(k)
        c.sync()
        box["t"] = time.perf_counter() - t0
    err = attempt("timed", timed)
    t = cp.allmax(box.get("t", math.inf) if err is None else math.inf)
    err = cp.first_error(err)
    if err is not None:
        return math.inf, err
    err = attempt("check", c.check)
    fp = None
    if err is None:
        try:
            fp = int(c.fingerprint())
        except Exception as e:                  # noqa: BLE001
            err = f"check on rank {rank}: fingerprint: {type(e).__name__}: {e}"
    fps = cp.allgather_int(fp if fp is not None else -1)
    if err is None and -1 not in fps and len(set(fps)) != 1:    # (-1: that rank failed)
        err = f"replicas diverged (parameter fingerprints {sorted(set(fps))})"
    err = cp.first_error(err)
    if err is not None:
        return math.inf, err
    return t / k * 1e3, None


def tensor_fingerprint(*tensors) -> int:
    """Exact fingerprint of tensors' bits (an int64 sum of their 32-bit words, position
    weighted so a permutation changes it): equal on every rank iff the replicas agree (up to
    a vanishing collision chance)."""
    import torch
    acc = 0
    for t in tensors:
        w = t.detach().contiguous().view(-1)
        if w.element_size() == 2:
            w = w.view(torch.int16).to(torch.int64)
        else:
            w = w.view(torch.int32).to(torch.int64)
        pos = torch.arange(1, w.numel() + 1, device=w.device, dtype=torch.int64) % 65521 + 1
        acc = (acc * 1000003 + int((w * pos).sum().item())) % (1 << 61)
    return acc
