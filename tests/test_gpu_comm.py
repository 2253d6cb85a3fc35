"""Native RCCL communicator + bucketed reducer on one GPU (1-rank communicator),
including capture of the reducer's fork/join into a hipGraph."""
import os
import subprocess
import sys
import time

import pytest
import torch

from conftest import REPO
from pytorch_distributed_mnist_amd.runtime.gpu_step import GpuStepBase

GRAPH_STEPS = GpuStepBase.GRAPH_STEPS

pytestmark = pytest.mark.gpu


def _comm(gpu):
    from pytorch_distributed_mnist_amd.parallel.comm import RcclComm
    return RcclComm(0, 1, gpu)


def test_rccl_allreduce_broadcast_allgather(gpu):
    comm = _comm(gpu)
    t = torch.arange(1000, dtype=torch.float32, device=gpu)
    comm.all_reduce_(t)
    comm.broadcast_(t, 0)
    g = comm.handle.all_gather(t)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), torch.arange(1000, dtype=torch.float32))
    assert g.shape == (1, 1000)
    comm.close()


def test_grad_reducer_forced_and_graph_captured(gpu):
    from pytorch_distributed_mnist_amd.parallel.reducer import GradReducer
    comm = _comm(gpu)
    grads = torch.randn(10000, device=gpu)
    ref = grads.clone()
    red = GradReducer(comm, grads, [(0, 4096), (4096, 10000)], force=True, transport="rccl")
    assert red._native is not None and red.capturable
    red.bucket_ready(0)
    red.bucket_ready(1)
    red.finalize()
    torch.cuda.synchronize()
    assert torch.equal(grads, ref)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        grads.mul_(2.0)
        red.bucket_ready(0)
        red.bucket_ready(1)
        red.finalize()
        grads.add_(1.0)
    g.replay()
    torch.cuda.synchronize()
    assert torch.allclose(grads, ref * 2 + 1)
    comm.close()


def test_grad_reducer_grouped_all_ready(gpu):
    from pytorch_distributed_mnist_amd.parallel.reducer import GradReducer
    comm = _comm(gpu)
    grads = torch.randn(10000, device=gpu)
    ref = grads.clone()
    red = GradReducer(comm, grads, [(0, 4096), (4096, 10000)], force=True, transport="rccl")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        grads.mul_(3.0)
        red.all_ready()
        red.wait_bucket(0)
        red.finalize()
        grads.sub_(1.0)
    g.replay()
    torch.cuda.synchronize()
    assert torch.allclose(grads, ref * 3 - 1)
    comm.close()


@pytest.mark.parametrize("carry", ["carry", "nocarry", "side", "early", "zero"])
@pytest.mark.parametrize("B", [256, 32])
def test_cnn_step_through_rccl_reducer_matches_local(gpu, carry, B):
    """The world_size > 1 step structure (unfused conv reduction, grouped RCCL all-reduce of
    both buckets, finalize) with a forced 1-rank RCCL communicator, graph-captured, gives
    the same parameters as the world_size-1 fast path."""
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
    from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
    from pytorch_distributed_mnist_amd.runtime.program import build_local_program
    train = synthetic_split(B * (GRAPH_STEPS + 1) + 40, True)   # a full graph, a 1-step graph
    test = synthetic_split(256, False)
    out = []
    for force in (False, True):
        comm = _comm(gpu) if force else None
        p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.05,
                                momentum=0.9, seed=4, use_graphs=True, comm=comm, force_comm=force,
                                transport="rccl")
        assert p.gpu.fuse_conv_reduce == (not force)
        p.gpu.set_rccl_mode(carry)
        if force and carry == "zero":
            p.gpu.set_shard_fc(True)           # 1 rank: the shard is all 128 rows
        p.optimizer.sync_hyperparams()
        p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
        p.train_epoch()
        torch.cuda.synchronize()
        out.append(p.arena.params.clone())
        if comm is not None:
            comm.close()
    assert torch.equal(out[0], out[1])


@pytest.mark.parametrize("transport,B", [("rccl", 32), ("rccl", 256), ("xgmi", 32), ("xgmi", 256)])
def test_fc1_update_carried_into_forward_is_bit_identical(gpu, transport, B):
    """World size > 1 (forced 1-rank communicator; RCCL nocarry and the xgmi in-launch-exchange
    step): step k's fc1 update runs in extra workgroups of step k+1's forward launch
    (kernels/fc_carry.h) instead of the optimizer.  Weights, momentum and both bf16 copies of W1
    must equal the optimizer-run update, over a graph-captured full sequence (GRAPH_STEPS - 1
    carried updates), a sequence of one and the ragged tail."""
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
    from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
    from pytorch_distributed_mnist_amd.runtime.program import build_local_program
    train = synthetic_split(B * (GRAPH_STEPS + 1) + 40, True)   # a full graph, a 1-step graph
    test = synthetic_split(256, False)
    out = []
    for carry in (False, True):
        comm = _comm(gpu)
        p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.05,
                                momentum=0.9, seed=4, use_graphs=True, comm=comm, force_comm=True,
                                transport=transport)
        assert p.reducer.kind == transport
        if transport == "rccl":
            p.gpu.set_rccl_mode("nocarry")
        p.gpu.structure = p.gpu.structure.with_(fc1_carry_fwd=carry)
        p.gpu.invalidate_graphs()
        assert p.gpu._fwd_carry_on(B) == carry
        p.optimizer.sync_hyperparams()
        p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
        p.train_epoch()
        torch.cuda.synchronize()
        p.reducer.check()
        o = p.optimizer
        out.append((p.arena.params.clone(), o.momentum_buffer.clone(), p.gpu.wf1.clone(),
                    p.gpu.wf1t.clone()))
        p.reducer.close()
        comm.close()
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [160, 256])
def test_fc1_update_carried_at_world_size_1_is_bit_identical(gpu, B, monkeypatch):
    """World size 1 with fc1_carry_local: fc1_bwd stores the fc1-weight gradient and the next
    forward launch updates from it, instead of the update fused into fc1_bwd's weight tiles.
    Same update, same bits: weights, momentum, W1 and the W1^T the next fc1_bwd reads, over
    two epochs of full graphs, a sequence of one and a (banded, fused) ragged tail."""
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
    from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
    from pytorch_distributed_mnist_amd.runtime.program import build_local_program
    train = synthetic_split(B * (GRAPH_STEPS + 1) + 40, True)   # a full graph, a 1-step graph
    test = synthetic_split(256, False)
    out = []
    for carry in ("0", "1"):
        monkeypatch.setenv("PDM_FC1_CARRY_LOCAL", carry)
        p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.05,
                                momentum=0.9, seed=4, use_graphs=True)
        assert p.gpu._fwd_carry_on(B) == (carry == "1")
        assert not p.gpu._fwd_carry_on(40)
        p.optimizer.sync_hyperparams()
        for epoch in range(2):
            p.set_train_indices(distributed_indices(len(train), 1, 0, epoch))
            p.train_epoch()
        torch.cuda.synchronize()
        o = p.optimizer
        out.append((p.arena.params.clone(), o.momentum_buffer.clone(), p.gpu.wf1.clone(),
                    p.gpu.current_wf1t().clone()))
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)


def test_fc1_grad_arena_is_current_with_carried_updates(gpu, monkeypatch):
    """World size 1, B = 256: the carried steps store the fc1-weight gradient, so the fused
    steps (a call's last step, the ragged tail) store theirs too -- after an epoch the arena
    holds the tail step's gradient, as with PDM_KEEP_GRADS=1, not an older step's."""
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
    from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
    from pytorch_distributed_mnist_amd.runtime.program import build_local_program
    B = 256
    train = synthetic_split(B * (GRAPH_STEPS + 1) + 40, True)   # a full graph, a 1-step graph
    test = synthetic_split(256, False)
    out = []
    for keep in ("0", "1"):
        monkeypatch.setenv("PDM_KEEP_GRADS", keep)
        p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.05,
                                momentum=0.9, seed=4, use_graphs=True)
        assert p.gpu._fwd_carry_on(B) and p.gpu.keep_grads == (keep == "1")
        p.optimizer.sync_hyperparams()
        p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
        p.train_epoch()
        torch.cuda.synchronize()
        out.append((p.gpu.G["fc1.weight"].clone(), p.arena.params.clone()))
    assert torch.isfinite(out[0][0]).all()
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("B", [32, 256])
def test_calibration_candidates_as_composed_match_local(gpu, B):
    """Every step structure bench.py's N > 1 calibration can pick (bench.step_candidates), with
    the production defaults composed as a real job runs them -- the xgmi streamed step with the
    in-launch conv exchange, the persistent collective outside the graphs, the fc1 update
    carried into the next forward and across graph replays; xgmi without the exchange; RCCL
    nocarry with the carried update; RCCL carry (B >= 256) / early (B < 256) -- through a
    forced 1-rank communicator, over two epochs of graph replays with the ragged tail, gives
    the world-size-1 path's weights, momentum and bf16 W1 / W1^T bit for bit.  (Each change is
    also pinned against its neighbour above; this pins the combinations.)"""
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
    from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
    from pytorch_distributed_mnist_amd.runtime.program import build_local_program
    train = synthetic_split(B * 19 + 40, True)
    test = synthetic_split(256, False)
    cands = [("local", None, None, None), ("xgmi", "xgmi", "carry", True),
             ("xgmi-noxchg", "xgmi", "carry", False), ("rccl-nocarry", "rccl", "nocarry", True),
             ("rccl" if B >= 256 else "rccl-early", "rccl", "carry" if B >= 256 else "early",
              True)]
    out = {}
    for name, transport, mode, xchg in cands:
        comm = _comm(gpu) if transport else None
        p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.05,
                                momentum=0.9, seed=4, use_graphs=True, comm=comm,
                                force_comm=comm is not None, transport=transport or "rccl")
        if transport:
            assert p.reducer.kind == transport
            p.gpu.set_rccl_mode(mode, invalidate=False)
            p.gpu.xgmi_exchange = xchg and p.structure.xgmi_exchange
            p.gpu.invalidate_graphs()
            if transport == "xgmi":
                assert p.gpu._xchg() == xchg
        p.optimizer.sync_hyperparams()
        for epoch in range(2):
            p.set_train_indices(distributed_indices(len(train), 1, 0, epoch))
            p.train_epoch()
        torch.cuda.synchronize()
        p.reducer.check()
        p.gpu.check_device()
        o = p.optimizer
        out[name] = (p.arena.params.clone(), o.momentum_buffer.clone(), p.gpu.wf1.clone(),
                     p.gpu.current_wf1t().clone())
        if transport:
            p.reducer.close()
            comm.close()
    for name, got in out.items():
        for a, b in zip(out["local"], got):
            assert torch.equal(a, b), name


def test_rccl_comm_count(gpu):
    comm = _comm(gpu)
    assert comm.comm_count() == 1
    assert comm.handle.comm_user_rank() == 0
    assert comm.handle.async_error() == 0
    comm.close()


_NEVER_JOINS = r"""
import sys, time, torch
sys.path.insert(0, sys.argv[1])
from pytorch_distributed_mnist_amd.ops import _ext
C = _ext.require()
uid = C.rccl_unique_id()
t0 = time.monotonic()
try:
    C.RcclComm(bytes(uid), 0, 2, 0, 4.0)      # rank 1 never calls init
except RuntimeError as e:
    print("RAISED %.2f %s" % (time.monotonic() - t0, e), flush=True)
    sys.exit(0)
print("NO ERROR", flush=True)
sys.exit(1)
"""


def test_rccl_init_times_out_when_a_peer_never_joins(gpu):
    """A 2-rank communicator whose rank 1 never arrives: rank 0 raises once the deadline
    (--timeout, here 4 s) passes instead of hanging (non-blocking ncclCommInitRankConfig +
    ncclCommGetAsyncError polling, csrc/runtime/comm.cpp).  Own process: the abandoned
    communicator is aborted there."""
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", _NEVER_JOINS, REPO], capture_output=True,
                       text=True, timeout=90)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RAISED")][0]
    waited = float(line.split()[1])
    assert 3.5 <= waited <= 20.0, line
    assert "timed out" in line and "never joined" in line, line
    assert time.monotonic() - t0 < 80


_CANCELLED = r"""
import sys, threading, time, torch
sys.path.insert(0, sys.argv[1])
from pytorch_distributed_mnist_amd.ops import _ext
C = _ext.require()
uid = C.rccl_unique_id()
threading.Timer(0.5, C.rccl_cancel_init, [4242]).start()   # "another rank failed"
t0 = time.monotonic()
try:
    C.RcclComm(bytes(uid), 0, 2, 0, 60.0, 4242)    # rank 1 never calls init
except RuntimeError as e:
    print("RAISED %.2f %s" % (time.monotonic() - t0, e), flush=True)
    sys.exit(0)
print("NO ERROR", flush=True)
sys.exit(1)
"""


def test_rccl_init_cancelled_when_a_peer_reports_failure(gpu):
    """Fail-fast bring-up: the init's cancel token posted (as parallel.comm's watcher thread
    does when another rank stores its failure) ends the wait at once, not at the 60 s
    deadline."""
    r = subprocess.run([sys.executable, "-c", _CANCELLED, REPO], capture_output=True,
                       text=True, timeout=90)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RAISED")][0]
    assert float(line.split()[1]) < 10.0, line
    assert "cancelled" in line, line


def test_bounded_sync_aborts_and_raises(gpu):
    """A device-side wait that outlives the deadline raises from bounded_sync."""
    from pytorch_distributed_mnist_amd.parallel.comm import bounded_sync
    a = torch.randn(4096, 4096, device=gpu)
    torch.cuda.synchronize()
    for _ in range(40):          # ~several ms of queued GEMMs, then a 1 us deadline
        a = a @ a * 1e-3
    with pytest.raises(RuntimeError, match="did not finish within"):
        bounded_sync(gpu, 1e-6, None, "queued GEMMs")
    torch.cuda.synchronize()
    bounded_sync(gpu, 30.0, None, "idle device")      # nothing queued: returns
