"""Data-plane communicators.

``RcclComm`` is the MI355X path: a C++ wrapper around an RCCL communicator
(``ncclCommInitRank``) that owns its own HIP stream (``csrc/runtime/comm.cpp``).
The ``ncclUniqueId`` is exchanged through the rendezvous TCP store of the
default process group, honouring ``--init-method tcp://host:port`` /
``env://``.  Collectives are enqueued on the comm stream
behind an event recorded on the caller's stream, and the caller's stream is
made to wait for completion, so they compose with hipGraph capture.

``TorchComm`` routes through ``torch.distributed`` (gloo) and is what the CPU
path and ``--backend gloo`` use.  ``LocalComm`` is world_size 1 without any
process group (bench at N=1): every collective is the identity.
"""
from __future__ import annotations

import atexit
import itertools
import os
import threading
import time

import torch
import torch.distributed as dist

from ..ops import _ext
from .dist import default_store, distributed_is_initialized

_uid_counter = itertools.count()

# Native objects (RCCL communicators, gradient reducers, xGMI transports) whose Python owner
# was garbage-collected without close(): a GC pass can run inside a hipGraph capture, where
# tearing them down (stream syncs, RCCL finalize, frees) is prohibited and aborts the
# process, so they are parked here and released at a safe point: release_retired() (the
# next native construction, the test harness between tests) or interpreter exit.
_retired: list = []


def retire(native) -> None:
    if native is not None:
        _retired.append(native)


def release_retired() -> None:
    """Release natives parked by garbage collection (no-op inside a stream capture).
    Abandoned communicators are aborted: finalize would wait for peers that moved on."""
    if not _retired:                  # (touches no GPU state: safe in a launcher parent)
        return
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        return
    while _retired:
        obj = _retired.pop()
        if hasattr(obj, "abort"):
            obj.abort()
        del obj


atexit.register(release_retired)


class Communicator:
    rank: int = 0
    world_size: int = 1
    native: bool = False

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        raise NotImplementedError

    def close(self) -> None:
        pass


class LocalComm(Communicator):
    def __init__(self):
        self.rank, self.world_size = 0, 1

    def all_reduce_(self, t):
        return t

    def broadcast_(self, t, src=0):
        return t


class TorchComm(Communicator):
    def __init__(self):
        if not distributed_is_initialized():
            raise RuntimeError("TorchComm needs an initialised default process group")
        self.rank, self.world_size = dist.get_rank(), dist.get_world_size()

    def all_reduce_(self, t, async_op: bool = False):
        work = dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=async_op)
        return work if async_op else t

    def broadcast_(self, t, src=0):
        dist.broadcast(t, src=src)
        return t


class RcclComm(Communicator):
    """Native RCCL communicator over xGMI on a dedicated HIP stream.

    Created non-blocking with a deadline (``timeout_s``, the app's ``--timeout``): a rank
    that never joins makes the others raise instead of hanging (csrc/runtime/comm.cpp)."""
    native = True

    def __init__(self, rank: int, world_size: int, device: torch.device, tag: str | None = None,
                 timeout_s: float = 1800.0):
        _ext.require()
        release_retired()
        self.rank, self.world_size = rank, world_size
        if tag is None:
            tag = str(next(_uid_counter))
        self._tag = tag
        self._gen = 0
        self._dev = device.index if device.index is not None else torch.cuda.current_device()
        self.timeout_s = float(timeout_s)
        self._c = None
        self._create(f"pdm_amd/rccl_uid/{tag}")

    def _create(self, key: str) -> None:
        C = _ext.require()
        rank, world_size, dev, timeout_s = self.rank, self.world_size, self._dev, self.timeout_s
        if world_size == 1:
            self._c = C.RcclComm(bytes(C.rccl_unique_id()), rank, 1, dev, float(timeout_s))
            return
        # Bring-up with fail-fast: a rank that fails posts `<key>/failed` to the rendezvous
        # store; peers waiting for the unique id or polling their communicator init (the C++
        # settle loop, GIL released) see it within ~50 ms and give up, instead of waiting the
        # whole deadline for a rank that will never arrive.
        store = default_store()
        failed = f"{key}/failed"
        token = int.from_bytes(os.urandom(7), "little") | 1
        try:
            if rank == 0:
                uid = C.rccl_unique_id()
                store.set(key, uid)
            else:
                uid = _await_key(store, key, failed, self.timeout_s)
            stop = threading.Event()

            def watch():
                while not stop.wait(0.05):
                    if store.check([failed]):
                        C.rccl_cancel_init(token)
                        return
            w = threading.Thread(target=watch, name="pdm-rccl-init-watch", daemon=True)
            w.start()
            try:
                self._c = C.RcclComm(bytes(uid), rank, world_size, dev, float(timeout_s), token)
            finally:
                stop.set()
                w.join()
        except Exception as e:
            try:
                if not store.check([failed]):
                    store.set(failed, f"rank {rank}: {e}")
            except Exception:                  # noqa: BLE001 (the store may be gone too)
                pass
            raise

    @property
    def alive(self) -> bool:
        return self._c is not None

    def revive(self) -> None:
        """Replace this rank's communicator by a fresh one (a new unique id through the
        rendezvous store).  Collective: every rank calls it, in the same order -- after a
        deadline aborted the communicator on some rank (bounded_sync), the peers' communicators
        are unusable too, so every rank drops its own (abort: its peers may be gone) and joins
        the new one.  Native objects built on the old handle (GradReducer.rebind) must be
        rebuilt by the caller."""
        if self._c is not None:
            self._c.abort()
            self._c = None
        self._gen += 1
        self._create(f"pdm_amd/rccl_uid/{self._tag}/revive{self._gen}")

    @property
    def handle(self):
        return self._c

    def comm_count(self) -> int:
        """Number of ranks as the RCCL communicator itself reports them (ncclCommCount)."""
        return int(self._c.comm_count())

    def abort(self) -> None:
        if self._c is not None:
            self._c.abort()
            self._c = None

    def all_reduce_(self, t):
        self._c.all_reduce_(t)
        return t

    def broadcast_(self, t, src=0):
        self._c.broadcast_(t, src)
        return t

    def close(self):
        if self._c is not None:
            self._c.destroy()
            self._c = None

    def __del__(self):
        retire(getattr(self, "_c", None))     # never torn down from a GC pass
        self._c = None


def _await_key(store, key: str, failed: str, timeout_s: float):
    """store.get(key) that gives up as soon as another rank posts `failed`."""
    t0 = time.monotonic()
    while not store.check([key]):
        if store.check([failed]):
            raise RuntimeError(f"RCCL bring-up cancelled: {store.get(failed).decode(errors='replace')}")
        if time.monotonic() - t0 > timeout_s:
            raise RuntimeError(f"RCCL bring-up: no unique id from rank 0 within {timeout_s:.0f} s")
        time.sleep(0.01)
    return store.get(key)


def bounded_sync(device: torch.device, timeout_s: float, comm: Communicator | None = None,
                 what: str = "device work", abort: bool = True) -> None:
    """``torch.cuda.synchronize`` with a deadline.

    Everything queued on the current stream (kernels, hipGraph replays, the RCCL
    collectives they wait on) must finish within ``timeout_s``; otherwise the RCCL
    communicator is aborted (its kernels waiting for a dead peer exit) and this raises.
    This is what bounds a collective that hangs on the device: the reference inherits
    the same semantics from torch's NCCL watchdog (process-group timeout).

    ``abort=False``: raise at the deadline but leave the communicator alone -- for work whose
    every device wait is bounded by itself (the xGMI transport's kernels give up at their
    own deadline and set an error word), so the device drains without an abort and the
    communicator stays usable (bench.py's calibration of xgmi candidates)."""
    if device.type != "cuda":
        return
    ev = torch.cuda.Event()
    ev.record()
    t0 = time.monotonic()
    delay = 0.0
    while not ev.query():
        waited = time.monotonic() - t0
        if waited > timeout_s:
            if abort and isinstance(comm, RcclComm):
                comm.abort()
                raise RuntimeError(f"{what} did not finish within {timeout_s:.0f} s (a peer rank "
                                   f"is missing or hung); communicator aborted")
            raise RuntimeError(f"{what} did not finish within {timeout_s:.0f} s (a peer rank is "
                               f"missing or hung)")
        # spin for the first 50 ms (a timed window must not end with a sleep overshooting
        # the device by up to the backoff step), then back off to 1 ms polls
        if waited > 0.05:
            delay = min(max(delay * 2, 1e-4), 1e-3)
            time.sleep(delay)
    torch.cuda.synchronize(device)


def make_comm(ctx, force_native: bool = False) -> Communicator:
    """Pick the data-plane communicator for a rank's DistContext.

    ``--backend nccl`` on the GPU: the native C++ RCCL communicator.  Its bring-up is agreed
    over the control plane: if any rank fails to create it (an RCCL error, or the init
    deadline), every rank drops its own and the job continues on torch's ProcessGroupNCCL
    (``TorchComm`` on the default group's cuda:nccl backend: the same RCCL collectives, not
    capturable into the step graph, so steps run eagerly) with a warning, instead of one rank
    raising while the others wait for it."""
    if ctx.world_size == 1 and not force_native and not ctx.initialized:
        return LocalComm()
    if ctx.is_gpu and ctx.backend == "nccl":
        err, comm = None, None
        try:
            comm = RcclComm(ctx.rank, ctx.world_size, ctx.device,
                            timeout_s=getattr(ctx, "timeout_s", 1800.0))
        except Exception as e:                      # noqa: BLE001 (reported below)
            err = e
        ok = err is None
        if ctx.world_size > 1 and distributed_is_initialized():
            t = torch.tensor([1 if ok else 0], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)     # gloo: CPU tensor
            ok = bool(t.item())
        if ok:
            return comm
        if comm is not None:
            comm.abort()
        if not ctx.initialized:
            raise RuntimeError(f"RCCL communicator bring-up failed: {err}")
        import sys
        print(f"warning: native RCCL communicator unavailable on rank {ctx.rank} "
              f"({err or 'failed on another rank'}); using torch's ProcessGroupNCCL",
              file=sys.stderr, flush=True)
        return TorchComm()
    if ctx.initialized:
        return TorchComm()
    return LocalComm()
