"""GPU step programs: the fixed kernel chains of one training step, and graphs.

Each model family has a ``_train_impl(B)`` that enqueues, on the current HIP
stream, every kernel of one step plus the bucket all-reduces; it has no host
inputs (batch indices come from a device step counter), so it is captured once
per batch size into a ``torch.cuda.CUDAGraph`` (hipGraph) and replayed.

Counter protocol (kernels of one step must not race on a counter): the first
kernel reads the data-step counter and only a later kernel advances it; the
optimizer-step counter is advanced before the optimizer kernel reads it (t >= 1).
CNN: ``cnn_head`` advances both.  Linear: ``lin_train`` advances the optimizer
step, ``lin_reduce`` (or, at world size 1, the optimizer launch) the data step.

Linear (reference Net, fp32):  lin_train -> [lin_reduce -> all-reduce] -> optim
CNN (bf16):  cnn_fwd -> fc1_fwd -> cnn_head -> fc1_bwd -> [all-reduce bucket 0]
             -> cnn_bwd -> conv_reduce -> [all-reduce bucket 1] -> optim
"""
from __future__ import annotations

import gc
import os

import torch

from ..ops import _ext
from .. import knobs


_GRAPH_STEPS = int(knobs.get("PDM_GRAPH_STEPS", "16"))  # steps per full graph
if _GRAPH_STEPS <= 0:
    raise ValueError(f"PDM_GRAPH_STEPS must be positive, got {_GRAPH_STEPS}")


def make_gpu_step(prog, use_graphs: bool = True):
    if prog.model == "linear":
        if prog.dtype != "fp32":
            raise ValueError("the reference Linear model runs in fp32 (--dtype fp32)")
        return LinearStep(prog, use_graphs)
    if prog.model == "cnn":
        if prog.dtype == "fp32":                 # the reference's precision, fp32 MFMA
            from .cnn_f32_step import CnnStepF32
            return CnnStepF32(prog, use_graphs)
        if prog.dtype != "bf16":
            raise ValueError(f"unsupported CNN dtype {prog.dtype!r} (bf16 or fp32)")
        from .cnn_step import CnnStep
        return CnnStep(prog, use_graphs)
    raise ValueError(prog.model)


class GpuStepBase:
    def check_device(self) -> None:
        """Raise if a kernel of this step recorded an error it could not raise itself (the
        default: none can)."""

    def __init__(self, prog, use_graphs: bool):
        self.C = _ext.require()
        self.prog = prog
        dev = prog.device
        self.device = dev
        self.arena = prog.arena
        self.opt = prog.optimizer
        self.reducer = prog.reducer
        self.train_images = prog.train_split.images.to(dev).contiguous()
        self.train_labels = prog.train_split.labels.to(device=dev, dtype=torch.int32).contiguous()
        self.test_images = prog.test_split.images.to(dev).contiguous()
        self.test_labels = prog.test_split.labels.to(device=dev, dtype=torch.int32).contiguous()
        # [train data step, (spare)]
        self.ctr = torch.zeros(2, dtype=torch.int64, device=dev)
        # the samples of two consecutive epochs in sampler order (set_train_indices): epoch e
        # in half e & 1 of the epoch buffer, located by the running data-step counter
        # (kernels.h StepRows: spe steps per epoch)
        self.ep_images = torch.empty(0, dtype=torch.uint8, device=dev)
        self.ep_labels = torch.empty(0, dtype=torch.int32, device=dev)
        self.spe = 0
        self._n_epoch = 0
        self._ctr_host = 0               # the data-step counter's value once the queue drains
        self._dev_step = None            # the optimizer-step count the device holds (host view)
        self._pending = None             # [order, half, event | None]: the next epoch's gather
        self._epoch_start = 0
        self._gather_stream = None       # stream of the ahead-of-time gathers
        self._ring = None                # pinned staging buffers of the epoch orders
        self._ring_i = 0
        self.use_graphs = bool(use_graphs) and self.reducer.capturable
        self.graphs = {}
        self.bfull = prog.batch_size
        self.structure = prog.structure
        self.metrics = prog.metrics
        self._opt_segments = None
        # step phase for double-buffered operands (CnnStep's W1^T): a step reads the buffers of
        # phase p and leaves the next step phase (p + 1) % phase_period.  A graph bakes in the
        # phase it was captured at, so graphs are keyed by it as well.
        self.phase = 0
        self.phase_period = 1

    # -- data ----------------------------------------------------------------

    def _stage(self, idx: torch.Tensor) -> list:
        """Copy an epoch order into the next pinned staging buffer of a ring of three ([buffer,
        event]); the gather kernel reads it in place (zero-copy).  The buffers are allocated
        once, on this thread and never during a graph capture (a host-memory allocation from
        any thread would invalidate a capture), and one is reused only after the event behind
        its previous reader has completed (at most two are in flight: this epoch's and the
        next's)."""
        n = idx.numel()
        if self._ring is None or self._ring[0][0].numel() != n:
            for old in self._ring or ():
                if old[1] is not None:   # a queued gather still reads this pinned buffer
                    old[1].synchronize()
            self._ring = [[torch.empty(n, dtype=torch.int32, pin_memory=True), None]
                          for _ in range(3)]
            self._ring_i = 0
        buf = self._ring[self._ring_i]
        self._ring_i = (self._ring_i + 1) % 3
        if buf[1] is not None:
            buf[1].synchronize()
        buf[0].copy_(idx)
        return buf

    def _gather(self, idx: torch.Tensor, half: int, stream) -> torch.cuda.Event:
        """Queue the gather of an epoch order into half `half` of the epoch buffer on `stream`;
        returns the event behind it."""
        n = self._n_epoch
        buf = self._stage(idx)
        with torch.cuda.stream(stream):
            self.C.gather_epoch(self.train_images, self.train_labels, buf[0],
                                self.ep_images.view(-1, 784)[half * n:(half + 1) * n],
                                self.ep_labels[half * n:(half + 1) * n],
                                # one workgroup per 64 rows (grid-striding ones taking
                                # fewer CUs beside the steps measured no better)
                                max_wgs=0)
            ev = torch.cuda.Event()
            ev.record(stream)
        buf[1] = ev
        return ev

    def set_train_indices(self, idx_cpu: torch.Tensor, next_idx=None) -> None:
        """Install this epoch's sample order; optionally start materialising the next one's.

        ``gather_epoch`` copies an epoch's samples contiguously into one half of the epoch
        buffer (the step kernels read their rows behind one counter load), reading the order
        in place from a pinned staging buffer (``EpochIndexPrefetcher`` computes it on its
        worker thread; only this thread touches pinned memory).  The data-step counter is
        never reset: epoch e = counter / spe lives in half e & 1 (kernels.h StepRows), so the
        step graphs stay valid across epochs.  With ``next_idx`` given, the next epoch's
        gather is queued on a side stream into the other half once this epoch is half-way
        through (``_issue_ahead``), behind an event after the steps queued so far (the other
        half's last reader, the previous epoch, is among them), and runs beside this epoch's
        steps.  At the next boundary that gather has long completed (the host checks its
        event) and the compute stream does not even wait for it: in steady state an epoch
        boundary enqueues nothing.  The host never waits for queued steps.
        """
        n = idx_cpu.numel()
        cur = torch.cuda.current_stream(self.device)
        if self._n_epoch != n:
            p = self._pending
            if p is not None and p[2] is not None:
                # an ahead gather still writes the old epoch buffer and reads a pinned buffer
                # of the ring about to be replaced: drain it before either is freed
                p[2].synchronize()
            self.ep_images = torch.empty(2 * n * 784, dtype=torch.uint8, device=self.device)
            self.ep_labels = torch.empty(2 * n, dtype=torch.int32, device=self.device)
            self._n_epoch = n
            self.spe = -(-n // self.bfull)
            self.graphs.clear()          # graphs captured the old buffer and geometry
            self._pending = None
        # this epoch starts at the next multiple of spe (a partial epoch before it -- tests,
        # tools -- moves the counter on)
        start = -(-self._ctr_host // self.spe) * self.spe
        if start != self._ctr_host:
            self.ctr[0:1].fill_(start)
            self._ctr_host = start
        half = (start // self.spe) & 1
        p, self._pending = self._pending, None
        if p is not None and p[0] is idx_cpu and p[1] == half and p[2] is not None:
            if not p[2].query():         # gathered ahead on the side stream: still running
                cur.wait_event(p[2])
        else:
            if p is not None and p[2] is not None:
                cur.wait_event(p[2])     # an unused ahead gather still writes a half
            self._gather(idx_cpu, half, cur)
        self._epoch_start = start
        if next_idx is not None and next_idx.numel() == n:
            if self._gather_stream is None:
                # created and used once here, not inside a timed run: HIP sets up a stream's
                # hardware queue at its first launch (~5 ms of host time)
                self._gather_stream = torch.cuda.Stream(self.device)
                with torch.cuda.stream(self._gather_stream):
                    torch.zeros(1, device=self.device)
            self._pending = [next_idx, 1 - half, None]

    def _issue_ahead(self) -> None:
        """Queue the next epoch's gather on the side stream once this epoch is half-way
        through (train_steps calls this between replays): the copy then runs beside steps in
        the middle of an epoch rather than beside the first steps after a boundary."""
        p = self._pending
        if p is None or p[2] is not None or \
                self._ctr_host - self._epoch_start < max(1, self.spe // 2):
            return
        # the side stream waits for everything queued on the compute stream so far; the other
        # half's last reader, the previous epoch, is among it
        free = torch.cuda.Event()
        free.record(torch.cuda.current_stream(self.device))
        self._gather_stream.wait_event(free)
        p[2] = self._gather(p[0], p[1], self._gather_stream)

    def skip_steps(self, k: int) -> None:
        """Move the data-step counter k steps on within the epoch (bench.py positions its
        timed window; every step is the same kernel chain on a different batch)."""
        self.ctr[0:1].add_(k)
        self._ctr_host += k
        self._issue_ahead()              # as the skipped steps would have

    def begin_epoch(self) -> None:
        self.opt.sync_hyperparams()
        if self._dev_step != self.opt.step_count:
            self.opt.sync_step()
            self._dev_step = self.opt.step_count

    # -- step ------------------------------------------------------------------
    # One hipGraph replay costs ~10-16 us of host time (MI355X_MICROARCH.md price
    # list, graph-replay-floor) — more than a whole small step's GPU time — so
    # steps are captured GRAPH_STEPS at a time (identical steps: the batch comes
    # from the device counter) and a run of n steps replays n // GRAPH_STEPS
    # multi-step graphs plus one graph of the remainder.
    GRAPH_STEPS = _GRAPH_STEPS
    GRAPH_SIZES = tuple(range(_GRAPH_STEPS, 0, -1))

    def carries_across_graphs(self, B: int) -> bool:
        """Whether a step of batch B leaves work to the next one (CnnStep: the carried fc1 update), so
        consecutive graph replays of one train_steps call hand it over: the graphs then come
        in variants by (carry in, carry out)."""
        return False

    def _graph(self, B: int, nsteps: int, phase=None, cin: bool = False, cout: bool = False):
        phase = self.phase if phase is None else phase
        key = (B, nsteps, phase, bool(cin), bool(cout))
        g = self.graphs.get(key)
        if g is None:
            g = torch.cuda.CUDAGraph()
            saved = self.phase
            self.phase = phase
            # no garbage collection inside the capture: a GC pass there may tear down native
            # objects of earlier programs (RCCL finalize, stream syncs, frees), which is
            # prohibited while capturing and aborts the process (torch.cuda.graph collects
            # once before the capture begins)
            gc_on = gc.isenabled()
            gc.disable()
            try:
                with torch.cuda.graph(g):          # captured on a side stream
                    # the persistent collective stays out of the graph when it is launched
                    # per train_steps call (collective_outside): no cross-queue edges
                    self._train_seq(B, nsteps, collective=not self.collective_outside(),
                                    cin=cin, cout=cout)
            finally:
                if gc_on:
                    gc.enable()
                self.phase = saved              # capturing runs nothing
            self.graphs[key] = g
        return g

    def _replay(self, B: int, nsteps: int, cin: bool = False, cout: bool = False) -> None:
        self._graph(B, nsteps, cin=cin, cout=cout).replay()
        self.phase = (self.phase + nsteps) % self.phase_period

    def _carry_flags(self, B: int, nreplays: int):
        """(carry in, carry out) of each of `nreplays` consecutive replays of one call."""
        if not self.carries_across_graphs(B):
            return [(False, False)] * nreplays
        return [(i > 0, i < nreplays - 1) for i in range(nreplays)]

    def _plan(self, B: int, n: int):
        """The replays of ``train_steps(B, n)``: [(steps, carry in, carry out)] -- n // GRAPH_STEPS
        full graphs, then one graph of the remainder (each graph boundary leaves the queue
        idle for ≈ 9 us: profiles/r6/window/)."""
        k = self.GRAPH_STEPS
        r = n % k
        sizes = [k] * (n // k) + ([r] if r else [])
        return [(s, ci, co) for s, (ci, co) in zip(sizes, self._carry_flags(B, len(sizes)))]

    def _variants(self, B: int, sizes):
        """Every (steps, phase, carry in, carry out) graph some ``_plan(B, n)`` replays, for the
        given graph sizes.  A graph smaller than GRAPH_STEPS only stands for the remainder,
        which is always a call's last replay, so it never carries out."""
        flags = ((False, False), (False, True), (True, True), (True, False)) \
            if self.carries_across_graphs(B) else ((False, False),)
        return [(n, ph, ci, co) for n in sizes for ph in range(self.phase_period)
                for ci, co in flags if not (co and n < self.GRAPH_STEPS)]

    def prepare(self, B: int, sizes=None) -> None:
        """Capture and upload every graph ``train_steps(B, n)`` replays (GRAPH_SIZES, or
        `sizes`, in every step phase), so no capture or first-launch upload lands inside a
        timed run.  Capturing enqueues nothing; the graphs' steps read the device counters
        when replayed."""
        if not self.use_graphs:
            return
        for n, ph, ci, co in self._variants(B, sizes or self.GRAPH_SIZES):
            g = self._graph(B, n, ph, ci, co)
            try:
                exe = g.raw_cuda_graph_exec()
            except (AttributeError, RuntimeError):
                continue
            dev = self.device.index if self.device.index is not None else \
                torch.cuda.current_device()
            self.C.graph_upload(int(exe), dev)
        torch.cuda.synchronize(self.device)

    def train_steps(self, B: int, n: int) -> None:
        """Enqueue n consecutive training steps of batch size B."""
        if n <= 0:
            return
        if self.use_graphs:
            plan = self._plan(B, n)
            if self.collective_outside():
                # one persistent collective for all n steps, launched eagerly on its own
                # stream beside the graph replays: the steps hand it their buckets through
                # device words, and the last optimizer waits for its last bucket, so
                # nothing has to join it back (a graph fork / join edge between two queues
                # costs 5-10 us on MI355X, every replay).  Every graph is captured first: a
                # capture synchronizes the device, which would wait for a running
                # collective that waits for steps not yet launched.
                ph = self.phase
                for size, ci, co in plan:
                    self._graph(B, size, ph, ci, co)
                    ph = (ph + size) % self.phase_period
                self.reducer.begin(n, self.collective_channels(), self.collective_wide(B))
            for size, ci, co in plan:
                self._issue_ahead()
                self._replay(B, size, ci, co)
                self._ctr_host += size
        else:
            self._issue_ahead()
            self._train_seq(B, n)
            self._ctr_host += n
        self._issue_ahead()
        self.opt.step_count += n
        if self._dev_step is not None:
            self._dev_step += n

    def train_step(self, B: int) -> None:
        self.train_steps(B, 1)

    def collective_outside(self) -> bool:
        """Streamed xgmi: the persistent collective is launched per train_steps call outside
        the step graphs (StepStructure.xgmi_outside) instead of inside every graph."""
        return bool(self.reducer.streamed and self.structure.xgmi_outside)

    def collective_channels(self):
        """Buckets the persistent collective carries (None: all)."""
        return None

    def collective_wide(self, B: int) -> bool:
        """Whether the wide persistent collective fits beside this step's kernels at B."""
        return False

    def _train_seq(self, B: int, n: int, collective: bool = True, cin: bool = False,
                   cout: bool = False) -> None:
        """n consecutive steps (captured together into one graph, or eager); `collective`:
        launch (and join) the persistent collective for them here; cin / cout: work carried
        in from the previous sequence / out to the next (carries_across_graphs)."""
        streamed = self.reducer.streamed and collective
        if streamed:
            # one launch for the n steps
            self.reducer.begin(n, self.collective_channels(), self.collective_wide(B))
        for _ in range(n):
            self._train_impl(B)
            self.phase = (self.phase + 1) % self.phase_period
        if streamed:
            self.reducer.end()

    def _train_impl(self, B: int) -> None:
        raise NotImplementedError

    # -- optimizer ---------------------------------------------------------------
    def optimizer_segments(self):
        """[(offset, rows, cols, shadow|None, shadow_t|None)] covering the arena."""
        return [(0, 1, self.arena.spec.total, None, None)]

    def launch_optimizer(self, segments=None, signal_ch: int = -1, bump=None,
                         metrics=None, exchange: bool = False) -> None:
        """One fused optimizer launch over `segments` (default: every parameter).

        xgmi streamed mode: bucket `signal_ch` (>= 0) is published to the persistent
        collective and the update waits for the buckets its segments belong to, by a
        one-workgroup wait kernel in front of it (every optimizer workgroup waiting for its
        own segment's bucket parked the whole grid on the GPU meanwhile; that variant was
        measured slower and removed in round 6).
        """
        if self._opt_segments is None:
            self._opt_segments = self.optimizer_segments()
        segs = self._opt_segments if segments is None else segments
        red = self.reducer
        xg = {}
        if exchange:
            # xgmi streamed, in-launch exchange of bucket 1 (the conv slabs): its workgroups
            # all-reduce their sums themselves; every other workgroup waits for its bucket
            # from the persistent collective (long done by now: it ran beside cnn_bwd)
            xg = dict(xg=red.sync, signal_ch=-1, waits=red.waits_for(segs, exchanged=(1,)),
                      timeout_s=red.timeout_s, xchg=red._native,
                      xchg_bucket=red.channels_of(1)[0])
        elif red.streamed:
            waits = red.waits_for(segs)
            uniq = []
            for i in range(0, len(waits), 2):
                if waits[i] not in uniq[0::2]:
                    uniq += waits[i:i + 2]
            self.C.xgmi_wait(red.sync, signal_ch, uniq, red.timeout_s)
        o = self.opt
        g = o.param_groups[0]
        grads = self.reducer.out_grads       # the xgmi transport's result arena, or in place
        if o.kind == "adam":
            b1, b2 = g["betas"]
            self.C.optim_step(self.C.OPT_ADAM, self.arena.params, grads, o.exp_avg,
                              o.exp_avg_sq, o._lr_dev, o._step_dev, float(b1), float(b2),
                              float(g["eps"]), float(g["weight_decay"]), 0.0, 0.0, False,
                              float(self.reducer.grad_scale), segs, bump=bump, metrics=metrics,
                              **xg)
        else:
            self.C.optim_step(self.C.OPT_SGD, self.arena.params, grads,
                              o.momentum_buffer, None, o._lr_dev, o._step_dev, 0.0, 0.0, 0.0,
                              float(g["weight_decay"]), float(g["momentum"]),
                              float(g["dampening"]), bool(g["nesterov"]),
                              float(self.reducer.grad_scale), segs, bump=bump, metrics=metrics,
                              **xg)

    def invalidate_graphs(self) -> None:
        self.graphs.clear()
        self._opt_segments = None


class LinearStep(GpuStepBase):
    """Reference Net step.  world size 1: lin_train -> optim (the optimizer sums the
    per-workgroup gradient slabs itself and advances the data-step counter);
    world size > 1: lin_train -> lin_reduce -> [all-reduce] -> optim."""

    def __init__(self, prog, use_graphs):
        super().__init__(prog, use_graphs)
        nblk = (self.bfull + self.C.LIN_ROWS - 1) // self.C.LIN_ROWS
        self.slab = torch.zeros(nblk * self.C.LIN_SLAB, dtype=torch.float32, device=self.device)
        self.W = self.arena.param("fc.weight")
        self.b = self.arena.param("fc.bias")
        self.gW = self.arena.grad("fc.weight")
        self.gb = self.arena.grad("fc.bias")
        # world size 1 (no all-reduce between backward and update): the slab reduction runs
        # inside the optimizer launch (PDM_FUSE_LIN_REDUCE=0 disables)
        self.fuse_reduce = not self.reducer.active and self.structure.fuse_lin_reduce
        self._fused = {}

    def invalidate_graphs(self) -> None:
        super().invalidate_graphs()
        self._fused = {}

    def _fused_segments(self, nblk: int):
        segs = self._fused.get(nblk)
        if segs is None:
            C, spec = self.C, self.arena.spec
            sl = lambda col: (self.slab, nblk, col, C.LIN_SLAB)
            segs = [(spec.offset("fc.weight"), 10, 784, None, None, sl(0)),
                    (spec.offset("fc.bias"), 1, 10, None, None, sl(7840))]
            self._fused[nblk] = segs
        return segs

    def _train_impl(self, B: int) -> None:
        C = self.C
        C.lin_train(self.ep_images.view(-1, 784), self.ep_labels, None, self.ctr[0:1], self.bfull,
                    B, self.W, self.b, self.slab, self.metrics.train_view(), self.opt._step_dev,
                    spe=self.spe)
        red = self.reducer
        # the step's train loss / correct partials sit in the slabs (columns 7850, 7851): the
        # launch that sums the gradient slabs adds them to the fp64 metrics in a fixed order
        nblk = (B + C.LIN_ROWS - 1) // C.LIN_ROWS
        mets = (self.slab, nblk, 10 * 784 + 10, C.LIN_SLAB, self.metrics.train_view())
        if self.fuse_reduce:
            self.launch_optimizer(self._fused_segments(nblk), bump=self.ctr[0:1], metrics=mets)
            return
        C.lin_reduce(self.slab, B, self.gW, self.gb, self.ctr[0:1],
                     red.sync if red.streamed else None, self.metrics.train_view())
        if red.streamed:
            # the optimizer publishes the bucket and waits for the persistent collective
            self.launch_optimizer(signal_ch=0)
            return
        red.bucket_ready(0)
        red.finalize()
        self.launch_optimizer()

    def evaluate(self) -> None:
        self.C.lin_eval(self.test_images, self.test_labels, self.W, self.b,
                        self.metrics.eval_view())
