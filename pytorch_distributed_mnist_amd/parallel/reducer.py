"""Bucketed gradient all-reduce, overlapped with backward.

Replaces DDP's C++ ``Reducer``.  Gradients already live in
one flat arena (``runtime/arena.py``) laid out in backward-ready order, so a
bucket is a contiguous slice and there is nothing to copy in:

* the step program calls ``bucket_ready(i)`` right after the kernel that
  finishes bucket i's gradients;
* a native transport records an event on the compute stream, makes its own
  high-priority stream wait on it and enqueues the bucket's collective there, so
  it overlaps the kernels the compute stream runs next;
* ``finalize()`` makes the compute stream wait for every bucket before the
  optimizer kernel, which reads ``out_grads``.

Transports (``transport=``; ``PDM_COMM`` overrides the default ``auto``):

* ``xgmi`` — the direct peer-to-peer all-reduce over xGMI (``csrc/xgmi.h``):
  the gradients are pushed into the peers' uncached hipIpc-mapped buffers and
  the sums land in an arena-sized result buffer (``out_grads``).  Its kernel is
  small enough to run beside ``cnn_bwd``, so the 4.7 MB fc bucket travels during
  the conv backward.  Sums are in fixed rank order (bit-identical on all ranks).
* ``rccl`` — ``ncclAllReduce`` on the C++ RCCL communicator, in place.
* ``auto`` — xgmi when every rank can map its peers and a numerical check of
  the transport passes on every rank, otherwise rccl (with a warning).

The reference DDP pre-divides by world_size and sums; we sum and fold the
1/world_size into the optimizer kernel (identical bits for power-of-two world
sizes).  With world_size 1 no collective is issued unless ``force`` is set
(the tests force it to exercise the native transports on a single GPU).
"""
from __future__ import annotations

import os
import sys
from typing import List, Tuple

import torch

from ..ops import _ext
from .comm import Communicator, RcclComm, TorchComm, release_retired, retire
from .xgmi_probe import probe, selfcheck
from .. import knobs

TRANSPORTS = ("auto", "xgmi", "rccl")


def default_transport() -> str:
    t = knobs.get("PDM_COMM", "auto")
    if t not in TRANSPORTS:
        raise ValueError(f"PDM_COMM={t!r}: choose from {TRANSPORTS}")
    return t


class GradReducer:
    def __init__(self, comm: Communicator, grads: torch.Tensor, bounds: List[Tuple[int, int]],
                 force: bool = False, transport: str | None = None, channels=None,
                 timeout_s: float | None = None):
        """channels: (channel bounds, channel indices per bucket) -- the buckets cut further
        for the direct xGMI transport (ModelSpec.channel_bounds); default one per bucket.
        timeout_s: bound on every xgmi device wait for a peer (default PDM_XGMI_TIMEOUT)."""
        self.comm = comm
        self.grads = grads
        self.out_grads = grads          # what the optimizer reads after finalize()
        self.bounds = list(bounds)
        if channels is None:
            channels = (list(self.bounds), [[i] for i in range(len(self.bounds))])
        self.cbounds = list(channels[0])
        self._bch = [list(c) for c in channels[1]]
        self.active = force or comm.world_size > 1
        self.grad_scale = 1.0 / comm.world_size
        self._native = None
        self._pending = {}
        self.kind = "local"
        self.transport_note = ""
        if not self.active:
            return
        transport = transport or default_transport()
        if transport not in TRANSPORTS:
            raise ValueError(f"transport {transport!r}: choose from {TRANSPORTS}")
        # auto picks xgmi on the RCCL (GPU) data plane; an explicit xgmi also runs over a
        # gloo control plane (two-ranks-on-one-GPU rehearsal, where RCCL refuses to run)
        if grads.is_cuda and (transport == "xgmi" or
                              (transport == "auto" and isinstance(comm, RcclComm))):
            try:
                x = XgmiTransport(comm, grads, self.cbounds, timeout_s=timeout_s)
                x.native.set_backward_channels(len(self._bch[0]))
            except Exception as e:           # mapping or self-check failed on some rank
                if transport == "xgmi":
                    raise
                x = None
                self.transport_note = f"xgmi unavailable ({e}); using rccl"
            if x is not None:
                self._native, self.kind, self.out_grads = x.native, "xgmi", x.result
                self._xgmi = x
                # streamed mode (default): one persistent collective launch per captured
                # step sequence, hand-offs through device words (csrc/xgmi.h)
                self.streamed = knobs.get("PDM_XGMI_STREAM", "1") != "0"
                self.sync = x.native.sync()
                self.timeout_s = x.timeout_s
                return
        if isinstance(comm, RcclComm):
            C = _ext.require()
            flat = [b for se in self.bounds for b in se]
            release_retired()
            self._native = C.GradReducer(comm.handle, grads, flat)
            self._flat = flat
            self.kind = "rccl"
        else:
            self.kind = "torch" if isinstance(comm, TorchComm) else "local"
        if self.transport_note and comm.rank == 0:
            print(f"warning: {self.transport_note}", file=sys.stderr, flush=True)

    streamed = False          # xgmi streamed mode (set in __init__)

    @property
    def num_buckets(self) -> int:
        return len(self.bounds)

    def rebind(self) -> None:
        """RCCL: rebuild the native reducer on the communicator's current handle (after
        RcclComm.revive replaced an aborted communicator); the bucket and shard setup is
        re-applied.  Other transports hold no RCCL handle: nothing to do."""
        if self.kind != "rccl":
            return
        C = _ext.require()
        retire(self._native)
        release_retired()
        self._native = C.GradReducer(self.comm.handle, self.grads, self._flat)
        if self.shard is not None:
            self._native.set_shard(*self.shard)

    def reset_transport(self) -> None:
        """xgmi: every protocol word of this rank's transport back to its initial state
        (XgmiReducer.reset: counters, generations, error words, the heap).  Needed whenever
        the step structure on this transport changes (the persistent launch then carries other
        channels, so the per-channel counters stop matching) or after a device deadline.  The
        caller guarantees that every rank resets between the same two control-plane
        agreements with its device drained (a candidate's setup phase).  No-op otherwise."""
        if self.kind == "xgmi":
            self._native.reset()

    def exchange_ok(self, bucket: int) -> bool:
        """xgmi: bucket `bucket` can be all-reduced inside the optimizer launch (its channels
        are one-shot; XgmiReducer.fill_exchange refuses a two-shot one, e.g. PDM_XGMI_MODE=two)."""
        if self.kind != "xgmi":
            return False
        desc = self._xgmi.describe
        return all(desc[c]["mode"] == "one-shot" for c in self._bch[bucket])

    # -- xgmi streamed mode -------------------------------------------------------
    def begin(self, nsteps: int, nch: int | None = None, wide: bool = False) -> None:
        """Launch the persistent collective for the next ``nsteps`` steps, carrying the first
        ``nch`` buckets (default: all; the others are exchanged in-launch by their producer,
        ``launch_optimizer(exchange=True)``); `wide`: the variant with twice the loads in
        flight, which fits only beside the small-band backward kernels."""
        if self.fault_no_collective:
            return
        n = -1 if nch is None else sum(len(self._bch[b]) for b in range(int(nch)))
        self._native.begin(nsteps, n, bool(wide))

    def end(self) -> None:
        """Join the persistent collective back into the compute stream."""
        if self.fault_no_collective:
            return
        self._native.end()

    # fault injection (bench.py PDM_CALIB_FAULT "<rank>:<xgmi candidate>:devhang"): this rank
    # never launches its persistent collective, so its buckets are never pushed to the peers
    # and its own optimizer's waits for reduced buckets are never satisfied -- a real device
    # hang on every rank, which the bounded device waits turn into error words
    fault_no_collective = False

    def bucket_of(self, offset: int) -> int:
        for i, (s, e) in enumerate(self.bounds):
            if s <= offset < e:
                return i
        raise ValueError(f"offset {offset} is in no bucket")

    def channel_of(self, offset: int) -> int:
        for i, (s, e) in enumerate(self.cbounds):
            if s <= offset < e:
                return i
        raise ValueError(f"offset {offset} is in no channel")

    def channels_of(self, bucket: int) -> list:
        """The xGMI channels bucket `bucket` is cut into (one per bucket elsewhere)."""
        return list(self._bch[bucket]) if self.kind == "xgmi" else [bucket]

    def waits_for(self, segments, exchanged=()) -> list:
        """Flat (channel, multiplier) per optimizer segment: wait for the channel holding the
        segment (-1 for the buckets in `exchanged`, which the launch all-reduces itself)."""
        skip = {c for b in exchanged for c in self._bch[b]}
        out = []
        for sg in segments:
            c = self.channel_of(sg[0])
            out += [-1, 0] if c in skip else [c, self._native.blocks(c)]
        return out

    def bucket_ready(self, i: int) -> None:
        if not self.active:
            return
        if self._native is not None:
            for c in self.channels_of(i):
                self._native.bucket_ready(c)
            return
        s, e = self.bounds[i]
        view = self.grads[s:e]
        if isinstance(self.comm, TorchComm):
            self._pending[i] = self.comm.all_reduce_(view, async_op=True)
        else:
            self.comm.all_reduce_(view)

    def all_ready(self) -> None:
        """Every bucket is complete: all-reduce them together (one grouped RCCL launch)."""
        if not self.active:
            return
        if self._native is not None:
            self._native.all_ready()
            return
        for i in range(len(self.bounds)):
            self.bucket_ready(i)

    def wait_bucket(self, i: int) -> None:
        """Make the current stream (or the host, on the torch path) wait for bucket i only."""
        if not self.active:
            return
        if self._native is not None:
            for c in self.channels_of(i):
                self._native.wait_bucket(c)
            return
        w = self._pending.pop(i, None)
        if w is not None:
            w.wait()

    def finalize(self) -> None:
        if not self.active:
            return
        if self._native is not None:
            self._native.finalize()
            return
        for w in self._pending.values():
            w.wait()
        self._pending.clear()

    # -- optimizer-state sharding of one bucket (ZeRO-1 on the fc bucket) ------------------
    shard = None              # (bucket, start, count per rank) when set

    @property
    def can_shard(self) -> bool:
        """Reduce-scatter + all-gather exist on this data plane (RCCL, or the gloo/torch
        rehearsal path); the direct xGMI all-reduce has no sharded form."""
        return self.active and (self.kind == "rccl" or self.kind == "torch")

    def set_shard(self, bucket: int, start: int, count: int) -> None:
        """Reduce-scatter the ``world_size * count`` floats of bucket `bucket` at `start`
        (rank r then holds the summed slice r) and all-reduce the rest of the bucket."""
        if not self.can_shard:
            raise RuntimeError(f"the {self.kind} transport cannot shard a bucket")
        s, e = self.bounds[bucket]
        if not (s <= start and start + self.comm.world_size * count <= e and count > 0):
            raise ValueError("shard outside its bucket")
        self.shard = (bucket, start, count)
        if self._native is not None:
            self._native.set_shard(bucket, start, count)

    def clear_shard(self) -> None:
        self.shard = None
        if self._native is not None:
            self._native.clear_shard()

    def gather(self, t: torch.Tensor) -> None:
        """In-place all-gather: rank r owns slice r of ``world_size`` equal slices of `t`
        (e.g. its rows of the bf16 W1 copy after a sharded update).  Native: on the comm
        stream behind the caller's stream; ``wait_gather`` joins it back."""
        if not self.active:
            return
        if self._native is not None:
            self._native.gather(t)
            return
        ws = self.comm.world_size
        parts = list(t.view(ws, -1).unbind(0))
        mine = parts[self.comm.rank].clone()
        torch.distributed.all_gather(parts, mine)      # gloo: copies into t's slices

    def wait_gather(self) -> None:
        if self.active and self._native is not None:
            self._native.wait_gather()

    def check(self) -> None:
        """Raise if the xgmi transport reported a peer timeout (no-op otherwise)."""
        if self.kind == "xgmi":
            self._xgmi.check()

    def close(self) -> None:
        if self.kind == "xgmi":
            self._xgmi.close()

    def __del__(self):
        retire(getattr(self, "_native", None))   # never torn down from a GC pass
        self._native = None

    @property
    def capturable(self) -> bool:
        """True when the whole reduce path can live inside a hipGraph."""
        return (not self.active) or self._native is not None


class XgmiTransport:
    """Builds and checks one rank's end of the direct xGMI all-reduce.

    Collective over the control plane: every rank exports its uncached buffer
    (hipIpcGetMemHandle), the handles go through the rendezvous store, every rank
    maps its peers, and then every rank runs three all-reduces of integer-valued
    patterns whose sums are exact and compares the result bit-for-bit.  The
    outcome is agreed with a gloo MIN, so either every rank uses xgmi or none does.
    """

    _tags = 0
    _preflight: dict = {}     # (world size, device) -> (ok, reason) of the child-process probe

    def __init__(self, comm: RcclComm, grads: torch.Tensor, bounds, timeout_s: float | None = None,
                 mode: str | None = None):
        C = _ext.require()
        from .dist import control_barrier, default_store, distributed_is_initialized
        ws, rank = comm.world_size, comm.rank
        dev = grads.device.index or 0
        mode = mode or knobs.get("PDM_XGMI_MODE", "auto")
        # bound on any wait for a peer inside the kernel (a late peer is an error, not a hang)
        timeout_s = timeout_s or float(knobs.get("PDM_XGMI_TIMEOUT", "30"))
        flat = [b for se in bounds for b in se]
        err = None
        native = None

        def agree(flag: bool) -> bool:
            if ws > 1 and distributed_is_initialized():
                t = torch.tensor([1 if flag else 0], dtype=torch.int32)
                torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN)
                return bool(t.item())
            return flag

        XgmiTransport._tags += 1
        # a peer mapping that faults would end this process: try it in child processes first
        # (xgmi_probe.py), once per process group and device (every rank builds the same
        # sequence of transports, so the cache is the same on every rank)
        self.preflight = "skipped"
        if ws > 1 and knobs.get("PDM_XGMI_PROBE", "1") != "0":
            pkey = (ws, dev)
            if pkey in XgmiTransport._preflight:
                self.preflight = "cached"
            else:
                XgmiTransport._preflight[pkey] = probe(
                    rank, ws, dev, default_store(), f"pdm_amd/xgmi_probe/{XgmiTransport._tags}",
                    agree, float(knobs.get("PDM_XGMI_PROBE_TIMEOUT_S", "120")))
                self.preflight = "passed"
            ok, why = XgmiTransport._preflight[pkey]
            if not ok:
                raise RuntimeError(f"xgmi pre-flight failed ({why})")
        try:
            native = C.XgmiReducer(rank, ws, dev, grads, flat, timeout_s, mode)
            handle = native.ipc_handle()
        except Exception as e:
            err, handle = e, b""
        handles = [handle]
        if ws > 1:
            key = f"pdm_amd/xgmi/{XgmiTransport._tags}"
            store = default_store()
            store.set(f"{key}/{rank}", handle)
            handles = [handle if r == rank else store.get(f"{key}/{r}") for r in range(ws)]
            if err is None and all(len(h) > 0 for h in handles):
                try:
                    native.open_peers([bytes(h) for h in handles])
                except Exception as e:
                    err = e
            elif err is None:
                err = RuntimeError("a peer could not export its xgmi buffer")
        else:
            if native is not None:
                native.open_peers([bytes(handle)])
        self.native = native

        # every rank has mapped every peer before any rank launches a collective kernel
        all_ok = agree(err is None) and agree(self._selfcheck(grads, bounds, ws, rank))
        if ws > 1 and distributed_is_initialized():
            control_barrier()
        if not all_ok:
            if native is not None:
                native.close()
            raise RuntimeError(f"xgmi transport check failed ({err or 'numerical self-check'})")
        self.result = native.result()
        self.describe = native.describe()
        self.timeout_s = timeout_s

    def _selfcheck(self, grads, bounds, ws, rank) -> bool:
        return selfcheck(self.native, grads, bounds, ws, rank)

    # cause bits of the device error word (csrc/xgmi.h XG_ERR_*)
    CAUSES = {1: "a peer did not arrive for the reduce-scatter / push phase",
              2: "a peer did not arrive for the all-gather phase",
              4: "the optimizer waited in vain for a reduced bucket",
              8: "the persistent collective waited in vain for this rank's backward to "
                 "publish a bucket",
              16: "waits that gave up after an earlier error (fail-fast)"}

    @classmethod
    def describe_error(cls, bits: int, first: int) -> str:
        what = [cls.CAUSES[b] for b in sorted(cls.CAUSES) if bits & b]
        root = cls.CAUSES.get(first, f"unknown cause {first:#x}") if first else "none recorded"
        return f"first cause: {root}; all causes (bits {bits:#x}): " + "; ".join(what)

    def check(self) -> None:
        e = self.native.error()
        if e:
            first = self.native.first_error()
            raise RuntimeError(f"xgmi all-reduce timed out ({self.describe_error(e, first)}); "
                               f"the gradients of this run are invalid")

    def close(self) -> None:
        if self.native is not None:
            self.native.close()
            self.native = None

    def __del__(self):
        retire(getattr(self, "native", None))    # never torn down from a GC pass
        self.native = None
