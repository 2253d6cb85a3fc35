"""Throughput benchmark: the flagship training step on N GPUs of one node.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model cnn|linear]
                    [--scaling weak|strong|both]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

Metric (BASELINE.json): images/sec for the whole node, MNIST CNN (SURVEY.md §7.1:
conv 1->32 3x3 + ReLU, conv 32->64 3x3 + ReLU, maxpool 2, fc 9216->128 + ReLU,
fc 128->10, log-softmax/NLL) trained with DDP (bucketed all-reduce over xGMI) and
SGD-momentum, bf16 compute / fp32 master weights, on synthetic 1x28x28 data of MNIST
size (60k) with random-init weights.

Two scaling modes (both measured by default, one JSON line):
  weak   -- 256 images per rank (global batch 256 N): the headline `value`;
  strong -- the reference's own DDP semantics: the node batch 256 is split over the
            ranks (multi_proc_single_gpu.py:174, --batch-size 256 -> 128/64/32 per rank
            at N = 2/4/8), reported under "strong" (at N = 1 the two coincide).

A timed step is the complete training step: batch gather + normalise, forward, loss,
backward, gradient all-reduce, optimizer update.  The timed window is placed so that an
epoch boundary falls inside it (the next epoch's DistributedSampler order, prefetched on a
host thread, is uploaded and gathered in stream order), i.e. the per-epoch data work is
measured too.  W untimed warmup steps, then exactly K steps bracketed by a barrier +
device synchronize on both sides; the slowest rank's time is reported.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
from pytorch_distributed_mnist_amd import knobs
from pytorch_distributed_mnist_amd.parallel.calibrate import (Candidate, ControlPlane, calibrate,
                                                              tensor_fingerprint)

# The reference's own training loop with the CNN swapped in, PyTorch eager + DDP/RCCL on one
# MI355X (tools/reference_eager.py, DataLoader with 4 workers, fp32, SGD momentum, batch 256;
# profiles/archive/r1_r2/reference_eager_n1.jsonl).  For N GPUs the baseline is taken as N x this value,
# i.e. perfect weak scaling of the reference.
REFERENCE_CNN_IMG_S_1GPU = 135369.5
REFERENCE_LINEAR_IMG_S_1GPU = 221060.4
NODE_BATCH = 256          # reference --batch-size default (node total, S:297-300)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--model", choices=["cnn", "linear"], default="cnn")
    ap.add_argument("--batch-per-rank", type=int, default=NODE_BATCH,
                    help="per-rank batch of the weak-scaling measurement")
    ap.add_argument("--scaling", choices=["weak", "strong", "both"], default="both")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default=None,
                    help="CNN compute dtype (default bf16; fp32 = the reference's precision on the "
                         "fp32 MFMA); the Linear model always runs fp32")
    ap.add_argument("--optimizer", choices=["sgd", "adam"], default=None)
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--no-graphs", dest="graphs", action="store_false")
    ap.add_argument("--train-size", type=int, default=60000)
    ap.add_argument("--timeout", type=float, default=180.0,
                    help="deadline (s) for RCCL init and every host sync")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch + rendezvous only (gloo, CPU): each rank joins the process "
                         "group, all-reduces its rank and rank 0 prints one JSON line; tests the "
                         "self-spawn path without a GPU")
    return ap.parse_args(argv)


RCCL_MODES = ("carry", "nocarry", "side", "early", "zero")


def step_candidates(reducers: dict, model: str, B: int, shard_ok, exchange_step: bool = True) -> list:
    """Candidate step structures [(name, reducer, rccl mode, xgmi in-launch exchange)] for
    per-rank batch B: at most four, each kept for what it can win on a real N-GPU node,
    where the 4.7 MB fc bucket's all-reduce takes tens of microseconds on the wire:

      xgmi          direct xGMI transport, streamed: the fc bucket travels beside the conv
                    backward and fc1.weight's update waits for it only in the next forward;
                    the conv bucket is exchanged inside the optimizer launch (fewest launches)
      xgmi-noxchg   the same with the conv bucket through conv_reduce + the persistent
                    collective: the fallback when the in-launch exchange fails on real peers
      rccl-nocarry  one grouped RCCL launch for both buckets, the fc1 update carried into the
                    next forward: the fastest RCCL structure in every N = 1 calibration
                    (profiles/r5/final4/bench.jsonl)
      rccl          (B >= 256) carry: the fc all-reduce overlaps the conv update and the next
                    cnn_fwd; at B = 256 cnn_bwd fills every CU, so RCCL's kernel (19.7 KB LDS)
                    cannot start before it ends and 'early' gains nothing
      rccl-early    (B < 256) the fc all-reduce issued during the conv backward, whose band
                    kernels leave CUs free for RCCL's kernel (DDP's overlap in backward)

    'side' (20 us slower at every N = 1 point) and 'zero' (the sharded fc1 update) run only
    when PDM_RCCL_MODE forces them.  PDM_RCCL_MODE forces one RCCL mode."""
    forced = knobs.get("PDM_RCCL_MODE")
    if forced is not None and forced not in RCCL_MODES:
        raise SystemExit(f"PDM_RCCL_MODE={forced!r}: choose from {RCCL_MODES}")
    cands = []
    for name, red in reducers.items():
        if name == "rccl" and model == "cnn":
            if forced is not None:
                if forced == "zero" and not shard_ok(red):
                    continue
                modes = [forced]
            else:
                modes = ["nocarry", "carry" if B >= 256 else "early"]
            for m in modes:
                cands.append(("rccl" if m == "carry" else f"rccl-{m}", red, m, True))
        elif name == "xgmi" and model == "cnn":
            cands.append(("xgmi", red, "carry", True))
            if exchange_step and red.exchange_ok(1):
                cands.append(("xgmi-noxchg", red, "carry", False))
        else:
            cands.append((name, red, "carry", True))
    return cands


def launch_mode(gpus: int, env) -> str:
    """How this process runs: 'worker' (one rank of a launched job: torch.distributed.run or
    our own spawn set RANK / WORLD_SIZE), 'spawn' (--gpus N > 1 from a plain ``python`` call:
    start the N rank processes, as the reference's default entry does with mp.spawn,
    multi_proc_single_gpu.py:284-285, :359) or 'single' (N = 1, no launcher)."""
    if "WORLD_SIZE" in env:
        ws = int(env["WORLD_SIZE"])
        if ws != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}")
        return "worker" if ws > 1 else "single"
    return "spawn" if gpus > 1 else "single"


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv) -> int:
    """Start N rank processes of this script with the env:// rendezvous variables
    torch.distributed.run would set (127.0.0.1, a free port; RANK = LOCAL_RANK = i).  This
    process has not touched the GPU (only ``import torch``), so starting children is safe.
    The children inherit stdout / stderr: rank 0 prints the one JSON line.  If any rank
    fails, the others are terminated (by PID) and its exit status is returned."""
    import subprocess
    port = str(_free_port())
    procs = []
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                       LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=port, PDM_BENCH_SPAWNED="1")
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv],
                                          env=env))
        rc = 0
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    print(f"bench.py: rank {procs.index(p)} exited with {c}; stopping the others",
                          file=sys.stderr, flush=True)
                    for q in live:
                        q.terminate()
            time.sleep(0.05)
        return rc
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(10)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()


class _DryStep(Candidate):
    """A stand-in step structure for --dry-run: a CPU 'replica' advanced deterministically
    per step, a fixed cost per step, and the fault kinds calibration must survive
    (PDM_CALIB_FAULT="<rank>:<name>:<phase>": setup / warm / timed / check raise, diverge
    perturbs this rank's replica, hang stalls the device sync until its deadline)."""

    COST_MS = {"xgmi": 1.0, "xgmi-noxchg": 0.7, "rccl-nocarry": 0.8, "rccl": 0.6,
               "rccl-early": 0.4}

    def __init__(self, name, rank, state, faults):
        self.name, self.rank, self.state = name, rank, state
        self.faults = {(int(r), n, p) for r, n, p in
                       (f.split(":") for f in faults.split(",") if f)} if faults else set()

    def _f(self, phase):
        return (self.rank, self.name, phase) in self.faults

    def enqueue(self, k):
        time.sleep(k * self.COST_MS[self.name] * 1e-3)
        for _ in range(k):
            self.state.mul_(0.5).add_(1.0)
        if self._f("diverge"):
            self.state.add_(1e-3)
        return k

    def sync(self):
        if self._f("hang"):
            time.sleep(0.5)
            raise RuntimeError(f"calibration ({self.name}) did not finish within 0.5 s")

    def fingerprint(self):
        return tensor_fingerprint(self.state)

    def recover(self):
        if torch.distributed.is_initialized():
            torch.distributed.broadcast(self.state, 0)


def dry_run(a, rank: int, ws: int) -> None:
    """Launch + rendezvous + the calibration protocol on stand-in candidates (gloo, CPU):
    exercises the self-spawn path and the rank-agreed candidate drop without a GPU."""
    import torch.distributed as dist
    if knobs.get("PDM_BENCH_FAIL_RANK") == str(rank):
        sys.exit(3)                 # fault injection (tests): this rank dies before rendezvous
    total = 0.0
    if ws > 1:
        dist.init_process_group("gloo", init_method="env://", world_size=ws, rank=rank)
        t = torch.tensor([float(rank)])
        dist.all_reduce(t)
        total = float(t.item())
    state = torch.zeros(64)
    faults = knobs.get("PDM_CALIB_FAULT")
    cands = [_DryStep(n, rank, state, faults) for n in _DryStep.COST_MS]
    cal = calibrate(cands, ControlPlane(ws), rank, warm_steps=4, timed_steps=16,
                    inject=faults, log=lambda s: print(f"bench.py: {s}", file=sys.stderr,
                                                       flush=True))
    if ws > 1:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": ws, "rank_sum": total,
                          "launch": "spawned" if knobs.get("PDM_BENCH_SPAWNED") else
                          ("launcher" if ws > 1 else "single"),
                          "config": {"grad_transport": cal.best,
                                     "transport_calibration_ms_per_step":
                                         {k: round(v, 4) for k, v in cal.times.items()}},
                          "comm": {"fallback": cal.notes}}), flush=True)


def main():
    a = parse()
    mode = launch_mode(a.gpus, os.environ)
    if mode == "spawn":
        sys.exit(spawn_ranks(a.gpus, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if a.dry_run:
        dry_run(a, rank, ws)
        return
    if knobs.unknown() and rank == 0:
        print(f"bench.py: warning: unknown PDM_* variables (typos?) {knobs.unknown()}",
              file=sys.stderr, flush=True)
    from types import SimpleNamespace

    from pytorch_distributed_mnist_amd import parallel
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
    from pytorch_distributed_mnist_amd.data.sampler import EpochIndexPrefetcher
    from pytorch_distributed_mnist_amd.models.reference import MODULES
    from pytorch_distributed_mnist_amd.models.specs import get_spec
    from pytorch_distributed_mnist_amd.optim.flat import build_optimizer
    from pytorch_distributed_mnist_amd.runtime.arena import FlatArena
    from pytorch_distributed_mnist_amd.runtime.program import TrainProgram

    device = parallel.pick_device(local_rank, "cuda")
    # PDM_BENCH_BACKEND=gloo: rehearsal of the multi-rank flow on a single GPU (with
    # PDM_SHARE_DEVICE=1); the measured configuration is always nccl = RCCL
    backend = knobs.get("PDM_BENCH_BACKEND", "nccl")
    ctx = parallel.init_distributed(backend, "env://" if ws > 1 else None, ws, rank, local_rank,
                                    device, timeout_s=a.timeout, init_pg=ws > 1)
    # PDM_FORCE_COMM=1 at N=1: run the multi-GPU step structure (conv reduction, bucket
    # all-reduces through a 1-rank communicator) to price it without transfers
    force_comm = knobs.get("PDM_FORCE_COMM") == "1"
    # PDM_EMULATE_WS=N with PDM_FORCE_COMM=1 and PDM_RCCL_MODE=zero: the per-rank chain of an
    # N-rank job (the fc1 update sharded over 128 / N rows, collectives of the 1-rank
    # communicator) priced on one GPU; reported under config.emulated_world_size
    emulate = knobs.get("PDM_EMULATE_WS")
    if emulate is not None and not (force_comm and ws == 1):
        raise SystemExit("PDM_EMULATE_WS prices one rank's chain on one GPU: it needs "
                         "PDM_FORCE_COMM=1 and --gpus 1")
    model = a.model
    spec = get_spec(model)
    parallel.verify_params_across_ranks(spec, rank, ws)
    comm = parallel.make_comm(ctx, force_native=force_comm)
    dtype = (a.dtype or "bf16") if model == "cnn" else "fp32"
    optname = a.optimizer or ("sgd" if model == "cnn" else "adam")
    lr = a.lr if a.lr is not None else (0.01 if optname == "sgd" else 1e-3)

    torch.manual_seed(1234 + rank)
    arena = FlatArena(spec, device)
    arena.load_module(MODULES[model]())
    comm.broadcast_(arena.params, 0)
    opt = build_optimizer(optname, arena, SimpleNamespace(lr=lr, momentum=0.9, weight_decay=1e-4))
    bounds = spec.bucket_bounds()
    channels = spec.channel_bounds()     # the xGMI transport's finer cut (fc1.weight alone)
    # Gradient transports to choose from: with $PDM_COMM unset (auto) on the RCCL data plane
    # both the direct xGMI all-reduce and RCCL are built, and a short untimed calibration
    # run of the real step picks the faster one for this N and batch (agreed over ranks).
    want = knobs.get("PDM_COMM", "auto")
    reducers = {}
    notes = []
    # every xgmi device wait for a peer gives up after xg_timeout (error word, fail-fast); a
    # calibration candidate's host deadline is strictly longer, so a transport that hangs on
    # the device ends there, is read from its error word and dropped -- the RCCL communicator
    # is only aborted for a hang no device deadline bounds (an RCCL candidate)
    xg_timeout = float(knobs.get("PDM_XGMI_TIMEOUT", "30"))
    calib_timeout = xg_timeout + float(knobs.get("PDM_CALIB_TIMEOUT_S", "30"))
    # the one-GPU rehearsal (gloo data plane, ranks sharing device 0) calibrates the direct
    # xGMI transport against the gloo reducer, as the real node does against RCCL
    rehearsal = ws > 1 and knobs.get("PDM_SHARE_DEVICE") == "1" and \
        isinstance(comm, parallel.TorchComm) and model == "cnn"
    if (ws > 1 or force_comm) and want == "auto" and \
            (isinstance(comm, parallel.RcclComm) or rehearsal):
        try:
            reducers["xgmi"] = parallel.GradReducer(comm, arena.grads, bounds, force=force_comm,
                                                    transport="xgmi", channels=channels,
                                                    timeout_s=xg_timeout)
        except Exception as e:                # collective decision: no rank uses xgmi
            notes.append(f"xgmi unavailable: {e}")
            print(f"bench.py: xgmi transport unavailable: {e}", file=sys.stderr, flush=True)
        r1 = parallel.GradReducer(comm, arena.grads, bounds, force=force_comm,
                                  transport="rccl")
        reducers[r1.kind] = r1
    else:
        r0 = parallel.GradReducer(comm, arena.grads, bounds, force=force_comm, transport=want,
                                  channels=channels, timeout_s=xg_timeout)
        reducers[r0.kind] = r0
        if r0.transport_note:
            notes.append(r0.transport_note)
    train = synthetic_split(a.train_size, True)
    test = synthetic_split(1024, False)
    n = len(train)
    prefetch = EpochIndexPrefetcher(n, ws, rank, int32=True)
    first = next(iter(reducers.values()))

    def sync(what):
        parallel.bounded_sync(device, a.timeout, comm, what)

    def barrier():
        parallel.control_barrier()      # gloo (CPU tensor): no torch NCCL communicator

    def allmax(x: float) -> float:
        if ws > 1:
            t = torch.tensor([x], dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            x = float(t.item())
        return x

    def measure(B: int) -> dict:
        """Calibrate the transport for per-rank batch B, then time a.steps steps."""
        prog = TrainProgram(model, dtype, arena, opt, first, train, test, B, use_graphs=a.graphs)
        # the reference's epoch (DataLoader drop_last=False, S:152-157): the rank's padded
        # DistributedSampler share in full batches, then one ragged tail batch
        full, tail = divmod(-(-n // ws), B)
        spe = full + (1 if tail else 0)            # steps per epoch
        state = {"epoch": 0, "step": 0}

        orders = {}

        def order(e):
            """Epoch e's sampler order (one object per epoch: the program recognises the order
            it gathered ahead by identity)."""
            if e not in orders:
                orders[e] = prefetch.peek(e)
                orders.pop(e - 3, None)
            return orders[e]

        dbg = knobs.get("PDM_BENCH_DEBUG")
        marks = []

        def mark(what):
            if dbg:
                ev = None
                if dbg == "events" and torch.cuda.is_available():
                    # PDM_BENCH_DEBUG=events: also where the device stream is at each mark
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record()
                marks.append((what, time.perf_counter(), ev))

        def next_epoch():
            mark("get")
            prefetch.get(state["epoch"])          # queues the following epochs' orders
            idx = order(state["epoch"])
            nxt = order(state["epoch"] + 1) if \
                knobs.get("PDM_GATHER_AHEAD", "1") != "0" else None
            mark("gather")
            prog.set_train_indices(idx, nxt)
            mark("begin_epoch")
            prog.gpu.begin_epoch()
            mark("boundary done")
            state["epoch"] += 1
            state["step"] = 0

        def run(k):
            """Enqueue k steps of the epoch sequence; returns the images they train on."""
            imgs = 0
            while k > 0:
                if state["step"] >= spe:
                    next_epoch()
                if state["step"] < full:
                    m = min(k, full - state["step"])
                    mark(f"replay {m}")
                    prog.gpu.train_steps(B, m)
                    imgs += m * B
                else:                              # the epoch's ragged tail step
                    m = 1
                    mark(f"tail {tail}")
                    prog.gpu.train_steps(tail, 1)
                    imgs += tail
                state["step"] += m
                k -= m
            return imgs

        def timed(k):
            sync("warmup")
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            marks.clear()
            mark("start")
            imgs = run(k)
            mark("sync")
            sync("timed steps")
            mark("end")
            if dbg and rank == 0:
                print("bench.py: window " + " | ".join(f"{w} @{1e6 * (t - t0):.0f}"
                                                       for w, t, _ in marks), file=sys.stderr,
                      flush=True)
                evs = [(w, e) for w, _, e in marks if e is not None]
                if evs:
                    print("bench.py: window on the device " + " | ".join(
                        f"{w} @{1e3 * evs[0][1].elapsed_time(e):.1f}" for w, e in evs),
                        file=sys.stderr, flush=True)
            barrier()
            torch.cuda.synchronize()
            return allmax(time.perf_counter() - t0), imgs

        shardable = hasattr(prog.gpu, "set_shard_fc")

        def use(red, carry="carry", xchg=True):
            if shardable:
                prog.gpu.set_shard_fc(False)   # (gathers the sharded state on the old reducer)
            prog.reducer = red
            prog.gpu.reducer = red
            prog.gpu.use_graphs = bool(a.graphs) and red.capturable
            if hasattr(prog.gpu, "set_rccl_mode"):
                prog.gpu.set_rccl_mode(carry, invalidate=False)
            if hasattr(prog.gpu, "xgmi_exchange"):
                prog.gpu.xgmi_exchange = bool(xchg) and prog.structure.xgmi_exchange
            prog.gpu.invalidate_graphs()
            if shardable and (carry == "zero" or knobs.get("PDM_SHARD_FC") == "1") and \
                    red.active and prog.gpu.shard_supported():
                prog.gpu.set_shard_fc(True)

        def prepare():
            """Capture + upload the step graphs outside any timed window (a graph captured
            lazily on first use would put its capture inside a short timed run)."""
            prog.gpu.prepare(B)
            if tail:
                prog.gpu.prepare(tail, sizes=(1,))

        cands = step_candidates(reducers, model, B,
                                lambda red: shardable and prog.gpu.shard_supported(red),
                                exchange_step=hasattr(prog.gpu, "xgmi_exchange") and
                                prog.structure.xgmi_exchange)

        def fingerprint():
            """Bits of this rank's replica (master weights + optimizer state)."""
            prog.sync_master()
            sync("fingerprint")
            return tensor_fingerprint(arena.params, *opt.state_buffers().values())

        def recover():
            """After a failed candidate: drain, leave sharding, and restore every replica
            (weights, momentum, bf16 compute copies) from rank 0.  A host deadline that had
            to abort the RCCL communicator (a hang no device deadline bounds) on any rank
            leaves every rank's communicator unusable: every rank then drains its device
            and joins a fresh communicator (RcclComm.revive), and the RCCL reducer is rebuilt
            on it, so the remaining candidates and the timed run keep their data plane."""
            alive = not isinstance(comm, parallel.RcclComm) or comm.alive
            if not ControlPlane(ws).agree(alive):
                parallel.bounded_sync(device, a.timeout, None, "recovery (drain after abort)")
                comm.revive()
                for r in reducers.values():
                    r.rebind()
                print(f"bench.py: rank {rank}: RCCL communicator re-created after an abort",
                      file=sys.stderr, flush=True)
            sync("recovery")
            if shardable:
                prog.gpu.set_shard_fc(False)
            for t in (arena.params, *opt.state_buffers().values()):
                comm.broadcast_(t, 0)
            if hasattr(prog.gpu, "refresh_shadows"):
                prog.gpu.refresh_shadows()     # bf16 compute copies of the weights
            sync("recovery broadcast")

        faults = knobs.get("PDM_CALIB_FAULT") or ""

        def device_fault(name, kind):
            """PDM_CALIB_FAULT "<rank>:<candidate>:devhang|spin" on this rank (a real device
            hang: the xgmi collective never launched; or a bounded device stall past the host
            deadline)."""
            return f"{rank}:{name}:{kind}" in faults.split(",")

        class Step(Candidate):
            def __init__(self, name, red, carry, xchg):
                self.name, self.red, self.carry, self.xchg = name, red, carry, xchg

            def setup(self):
                self.red.fault_no_collective = device_fault(self.name, "devhang")
                use(self.red, self.carry, self.xchg)
                # xgmi: the candidates before this one left the transport's counters where
                # their structure (or a device deadline) left them; every rank re-arms it
                # here, and the setup agreement orders that before any rank's first launch
                self.red.reset_transport()
                prepare()                      # capture outside the calibration window

            def enqueue(self, k):
                n = run(k)
                if device_fault(self.name, "spin"):
                    prog.gpu.C.debug_spin(min(30.0, calib_timeout + 2.0))
                return n

            def sync(self):
                # the xgmi transport's device waits are bounded by xg_timeout < calib_timeout:
                # its hang drains by itself (error word, read in check()), so the deadline
                # leaves the communicator alone; an RCCL hang needs the abort to drain
                parallel.bounded_sync(device, calib_timeout, comm, f"calibration ({self.name})",
                                      abort=self.red.kind != "xgmi")

            def check(self):
                self.red.check()

            def fingerprint(self):
                return fingerprint()

            def recover(self):
                recover()

        opt.sync_hyperparams()
        next_epoch()
        steps = {name: Step(name, red, carry, xchg) for name, red, carry, xchg in cands}
        calib = {}
        if len(cands) > 1:
            cal = calibrate(list(steps.values()), ControlPlane(ws), rank,
                            budget_s=float(knobs.get("PDM_CALIB_BUDGET_S", "120")),
                            inject=knobs.get("PDM_CALIB_FAULT"),
                            log=lambda s: print(f"bench.py: {s}", file=sys.stderr, flush=True))
            calib = cal.times
            notes.extend(f"B={B}: {n}" for n in cal.notes)
            best = cal.best
        else:
            best = cands[0][0]
        for st in steps.values():
            st.red.fault_no_collective = False
        use(steps[best].red, steps[best].carry, steps[best].xchg)
        steps[best].red.reset_transport()
        parallel.control_barrier()           # every rank re-armed before any launches
        chosen = prog.reducer
        prepare()
        # put the next epoch boundary inside the timed window: continue the current epoch
        # from the step that leaves W warmup steps and then K // 2 timed full steps before
        # the boundary (every step is the same kernel chain on a different batch of the
        # sampler order).  The counter moves first, so the skipped part of the epoch also
        # issues what it would have issued (the next epoch's gather, from mid-epoch), and
        # the W warmup steps run right before the timed window as usual.
        left = spe - state["step"]
        if a.steps >= 2 and left > a.steps // 2 + a.warmup and \
                knobs.get("PDM_BENCH_BOUNDARY", "1") != "0":
            skip = left - a.steps // 2 - a.warmup
            sync("reposition")
            prog.gpu.skip_steps(skip)          # device data-step counter
            state["step"] += skip
        run(a.warmup)
        left = spe - state["step"]
        boundaries = -(-(a.steps - left) // spe) if a.steps > left else 0
        elapsed, imgs = timed(a.steps)
        chosen.check()
        prog.gpu.check_device()
        prog.sync_master()
        if not torch.isfinite(arena.params).all():
            raise RuntimeError("non-finite parameters after the benchmark")
        if ws > 1:
            # DDP keeps identical replicas: every rank must hold the same weights and
            # optimizer state bit for bit after the timed window
            fps = ControlPlane(ws).allgather_int(fingerprint())
            if len(set(fps)) != 1:
                raise RuntimeError(f"replicas diverged during the timed window ({best}): "
                                   f"fingerprints {fps}")
        ms = elapsed / a.steps * 1e3
        sharded = bool(getattr(prog.gpu, "shard_fc", False))
        conv2 = ("n/a (no convolution)" if model == "linear" else
                 "split-bf16 (hi.hi + hi.lo + lo.hi), fp32 accumulation"
                 if getattr(prog.gpu, "conv_x3", False) else
                 "fp32 MFMA" if dtype == "fp32" else "bf16 MFMA, fp32 accumulation")
        if shardable:
            prog.gpu.set_shard_fc(False)
        return {"B": B, "global_batch": B * ws, "elapsed": elapsed, "ms": ms, "shard_fc": sharded,
                "value": imgs * ws / elapsed, "images": imgs * ws, "tail": tail, "conv2": conv2,
                "epoch_steps": spe, "transport": best,
                "calib": {k: round(v, 5) for k, v in calib.items()},
                "graphs": bool(prog.gpu.use_graphs), "epoch_boundaries_timed": boundaries}

    strong_B = max(1, NODE_BATCH // ws)
    res = {}
    if a.scaling in ("weak", "both"):
        res["weak"] = measure(a.batch_per_rank)
    if a.scaling in ("strong", "both"):
        if "weak" in res and strong_B == a.batch_per_rank:
            res["strong"] = res["weak"]
        else:
            res["strong"] = measure(strong_B)
    main_mode = "weak" if "weak" in res else "strong"
    m = res[main_mode]

    comm_info = {"data_plane": type(comm).__name__, "world_size": ws}
    if isinstance(comm, parallel.RcclComm):
        comm_info["rccl_comm_count"] = comm.comm_count()      # ranks RCCL itself reports
        comm_info["rccl_version"] = int(__import__(
            "pytorch_distributed_mnist_amd.ops._ext", fromlist=["x"]).require().rccl_version())
    if "xgmi" in reducers:
        comm_info["xgmi_peers_mapped"] = int(reducers["xgmi"]._native.peers_mapped()) \
            if reducers["xgmi"]._native is not None else 0
    if notes:
        comm_info["fallback"] = notes
    if rank == 0:
        ref = REFERENCE_CNN_IMG_S_1GPU if model == "cnn" else REFERENCE_LINEAR_IMG_S_1GPU
        line = {
            "metric": "images/sec (whole node) MNIST CNN DDP at 1/2/4/8 MI355X"
            if model == "cnn" else "images/sec (whole node) MNIST Linear DDP",
            "value": round(m["value"], 1), "unit": "images/sec", "n_gpus": ws, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(m["ms"], 5), "higher_is_better": True,
            "scaling": main_mode, "vs_baseline": round(m["value"] / (ws * ref), 3),
            "dtype": dtype,
            "data": "synthetic (60k x 1x28x28 uint8, MNIST-shaped), random-init weights",
            "config": {"model": "mnist_cnn" if model == "cnn" else "mnist_linear",
                       "global_batch": m["global_batch"], "batch_per_rank": m["B"],
                       "seq_len": None, "parallelism": f"dp{ws}", "optimizer": optname,
                       "graphs": m["graphs"], "grad_transport": m["transport"],
                       "transport_calibration_ms_per_step": m["calib"],
                       "epoch_boundaries_timed": m["epoch_boundaries_timed"],
                       "epoch_steps": m["epoch_steps"], "tail_batch_per_rank": m["tail"],
                       "fc1_update_sharded": m["shard_fc"],
                       "conv2_products": m["conv2"],
                       "images_timed": m["images"]},
            "value_semantics": (
                "weak scaling: images/sec of the whole node at a fixed per-rank batch; timed "
                "window = K consecutive steps of the reference's epoch sequence (full batches "
                "+ the ragged tail, an epoch boundary inside); value = images_timed / time"
                if main_mode == "weak" else
                "strong scaling: the reference's node batch 256 split over the ranks (S:174)"),
            "comm": comm_info,
            # every PDM_* environment knob this run saw (none set = the defaults)
            "knobs": {k: v for k, v in knobs.active().items() if k != "PDM_BENCH_SPAWNED"},
            "launch": "spawned" if knobs.get("PDM_BENCH_SPAWNED") else
                      ("launcher" if ws > 1 else "single"),
        }
        if emulate is not None:
            line["config"]["emulated_world_size"] = int(emulate)
        if main_mode == "weak" and "strong" in res:
            s = res["strong"]
            line["strong"] = {"value": round(s["value"], 1), "ms_per_step": round(s["ms"], 5),
                              "global_batch": s["global_batch"], "batch_per_rank": s["B"],
                              "grad_transport": s["transport"],
                              "transport_calibration_ms_per_step": s["calib"],
                              "epoch_boundaries_timed": s["epoch_boundaries_timed"],
                              "tail_batch_per_rank": s["tail"], "images_timed": s["images"],
                              "semantics": "reference DDP: node batch 256 split over ranks (S:174)"}
        print(json.dumps(line), flush=True)
    prefetch.close()
    for red in reducers.values():
        red.close()
    comm.close()
    parallel.shutdown()


if __name__ == "__main__":
    main()
