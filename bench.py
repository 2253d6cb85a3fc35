"""Throughput benchmark: the flagship training step on N GPUs of one node.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model cnn|linear]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

Metric (BASELINE.json): images/sec for the whole node, MNIST CNN (SURVEY.md §7.1:
conv 1->32 3x3 + ReLU, conv 32->64 3x3 + ReLU, maxpool 2, fc 9216->128 + ReLU,
fc 128->10, log-softmax/NLL) trained with DDP (bucketed RCCL all-reduce over
xGMI) and SGD-momentum, bf16 compute / fp32 master weights, on synthetic
1x28x28 data of MNIST size (60k) with random-init weights.  Per-GPU batch is
fixed (weak scaling): 256 images per rank by default, the reference's per-GPU
batch at world_size 1 (its --batch-size 256 is split over the GPUs).

A timed step is the complete training step: batch gather + normalise,
forward, loss, backward, gradient all-reduce, optimizer update (incl. the
epoch-boundary reshuffles that fall inside the window).  W untimed warmup
steps, then exactly K steps bracketed by a barrier + device synchronize on
both sides; the slowest rank's time is reported.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

# The number to beat (BASELINE.md protocol): the reference's own training loop with the CNN
# swapped in, PyTorch eager + DDP/RCCL on one MI355X (tools/reference_eager.py, DataLoader with
# 4 workers, fp32, SGD momentum, batch 256; profiles/reference_eager_n1.jsonl).  For N GPUs
# the baseline is taken as N x this value, i.e. perfect weak scaling of the reference.
REFERENCE_CNN_IMG_S_1GPU = 135369.5
REFERENCE_LINEAR_IMG_S_1GPU = 221060.4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--model", choices=["cnn", "linear"], default="cnn")
    ap.add_argument("--batch-per-rank", type=int, default=256)
    ap.add_argument("--optimizer", choices=["sgd", "adam"], default=None)
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--no-graphs", dest="graphs", action="store_false")
    ap.add_argument("--train-size", type=int, default=60000)
    return ap.parse_args()


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if ws != a.gpus:
        if ws == 1 and a.gpus > 1:
            print(f"bench.py: --gpus {a.gpus} needs torch.distributed.run with {a.gpus} procs",
                  file=sys.stderr)
            sys.exit(2)
    from pytorch_distributed_mnist_amd import parallel
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
    from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
    from pytorch_distributed_mnist_amd.models.reference import MODULES
    from pytorch_distributed_mnist_amd.models.specs import get_spec
    from pytorch_distributed_mnist_amd.optim.flat import build_optimizer
    from pytorch_distributed_mnist_amd.runtime.arena import FlatArena
    from pytorch_distributed_mnist_amd.runtime.program import TrainProgram
    from types import SimpleNamespace

    device = parallel.pick_device(local_rank, "cuda")
    # PDM_BENCH_BACKEND=gloo: rehearsal of the multi-rank flow on a single GPU (with
    # PDM_SHARE_DEVICE=1); the measured configuration is always nccl = RCCL
    backend = os.environ.get("PDM_BENCH_BACKEND", "nccl")
    ctx = parallel.init_distributed(backend, "env://" if ws > 1 else None, ws, rank, local_rank,
                                    device, init_pg=ws > 1)
    # PDM_FORCE_COMM=1 at N=1: run the multi-GPU step structure (unfused conv reduction,
    # grouped RCCL all-reduce through a 1-rank communicator) to price it without transfers
    force_comm = os.environ.get("PDM_FORCE_COMM") == "1"
    comm = parallel.make_comm(ctx, force_native=force_comm)
    model = a.model
    dtype = "bf16" if model == "cnn" else "fp32"
    optname = a.optimizer or ("sgd" if model == "cnn" else "adam")
    lr = a.lr if a.lr is not None else (0.01 if optname == "sgd" else 1e-3)

    torch.manual_seed(1234 + rank)
    spec = get_spec(model)
    arena = FlatArena(spec, device)
    arena.load_module(MODULES[model]())
    comm.broadcast_(arena.params, 0)
    opt = build_optimizer(optname, arena, SimpleNamespace(lr=lr, momentum=0.9, weight_decay=1e-4))
    bounds = spec.bucket_bounds()
    # Gradient transports to choose from: with $PDM_COMM unset (auto) on the RCCL data plane
    # both the direct xGMI all-reduce and RCCL are built, and a short untimed calibration
    # run of the real step picks the faster one for this N (agreed over ranks).
    want = os.environ.get("PDM_COMM", "auto")
    reducers = {}
    if (ws > 1 or force_comm) and want == "auto" and isinstance(comm, parallel.RcclComm):
        try:
            reducers["xgmi"] = parallel.GradReducer(comm, arena.grads, bounds, force=force_comm,
                                                    transport="xgmi")
        except Exception as e:                # collective decision: no rank uses xgmi
            print(f"bench.py: xgmi transport unavailable: {e}", file=sys.stderr, flush=True)
        reducers["rccl"] = parallel.GradReducer(comm, arena.grads, bounds, force=force_comm,
                                                transport="rccl")
    else:
        r0 = parallel.GradReducer(comm, arena.grads, bounds, force=force_comm, transport=want)
        reducers[r0.kind] = r0
    train = synthetic_split(a.train_size, True)
    test = synthetic_split(1024, False)
    B = a.batch_per_rank
    first = next(iter(reducers.values()))
    prog = TrainProgram(model, dtype, arena, opt, first, train, test, B, use_graphs=a.graphs)
    n = len(train)

    state = {"epoch": 0, "step": 0}

    def next_epoch():
        prog.set_train_indices(distributed_indices(n, ws, rank, state["epoch"]))
        prog.gpu.begin_epoch()
        state["epoch"] += 1
        state["step"] = 0

    per_rank = -(-n // ws)
    full = per_rank // B                       # full-batch steps per epoch

    def run(k):
        while k > 0:
            if state["step"] >= full:
                next_epoch()
            m = min(k, full - state["step"])
            prog.gpu.train_steps(B, m)
            state["step"] += m
            k -= m

    def barrier():
        parallel.control_barrier()      # gloo (CPU tensor): no torch NCCL communicator

    def timed(k):
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(k)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if ws > 1:
            t = torch.tensor([el], dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = float(t.item())
        return el

    def use(red):
        prog.reducer = red
        prog.gpu.reducer = red
        prog.gpu.use_graphs = bool(a.graphs) and red.capturable
        prog.gpu.invalidate_graphs()

    opt.sync_hyperparams()
    next_epoch()
    calib = {}
    if len(reducers) > 1:
        for name, red in reducers.items():
            use(red)
            run(16)
            calib[name] = timed(48) / 48 * 1e3
            try:
                red.check()
                ok = 1
            except RuntimeError as e:
                print(f"bench.py: {name} transport failed calibration: {e}", file=sys.stderr,
                      flush=True)
                ok = 0
            if ws > 1:                         # every rank drops a transport any rank saw fail
                t = torch.tensor([ok], dtype=torch.int32)
                torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN)
                ok = int(t.item())
            if not ok:
                if name == "rccl":
                    raise RuntimeError("rccl transport failed calibration")
                del calib[name]
                torch.cuda.synchronize()
                # replicas (and their momentum) may differ after a failed reduce
                for t in (arena.params, *opt.state_buffers().values()):
                    comm.broadcast_(t, 0)
                if hasattr(prog.gpu, "refresh_shadows"):
                    prog.gpu.refresh_shadows()     # bf16 compute copies of the weights
        best = min(calib, key=calib.get)
        use(reducers[best])
    chosen = prog.reducer
    # capture + upload the step graphs outside the timed window (a graph captured lazily
    # on first use would put its capture inside a short timed run)
    prog.gpu.prepare(B)
    run(a.warmup)
    elapsed = timed(a.steps)
    chosen.check()
    if not torch.isfinite(arena.params).all():
        raise RuntimeError("non-finite parameters after the benchmark")
    ms = elapsed / a.steps * 1e3
    global_batch = B * ws
    value = a.steps * global_batch / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node) MNIST CNN DDP at 1/2/4/8 MI355X"
            if model == "cnn" else "images/sec (whole node) MNIST Linear DDP",
            "value": round(value, 1), "unit": "images/sec", "n_gpus": ws, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": round(value / (ws * (
                REFERENCE_CNN_IMG_S_1GPU if model == "cnn" else REFERENCE_LINEAR_IMG_S_1GPU)), 3),
            "dtype": dtype,
            "data": "synthetic (60k x 1x28x28 uint8, MNIST-shaped), random-init weights",
            "config": {"model": "mnist_cnn" if model == "cnn" else "mnist_linear",
                       "global_batch": global_batch, "batch_per_rank": B, "seq_len": None,
                       "parallelism": f"dp{ws}", "optimizer": optname,
                       "graphs": bool(prog.gpu.use_graphs), "grad_transport": chosen.kind,
                       "transport_calibration_ms_per_step":
                           {k: round(v, 5) for k, v in calib.items()}},
        }), flush=True)
    for red in reducers.values():
        red.close()
    comm.close()
    parallel.shutdown()


if __name__ == "__main__":
    main()
