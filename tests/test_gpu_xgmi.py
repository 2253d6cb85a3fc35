"""Direct xGMI all-reduce transport (csrc/xgmi.h, csrc/kernels/xgmi.hip).

Single-rank cases run in-process; multi-rank cases run tests/xgmi_worker.py with
2 and 4 ranks sharing the one GPU of the box (hipIpc across processes, gloo
control plane), which exercises the same peer mappings, flags and push
schedules as ranks on different GPUs.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import REPO, free_port

pytestmark = pytest.mark.gpu


def test_xgmi_single_rank_identity_and_graph(gpu):
    from pytorch_distributed_mnist_amd.ops import _ext
    C = _ext.require()
    n = 1181120 + 18880
    grads = torch.randn(n, device=gpu)
    for mode in ("one", "two", "auto"):
        x = C.XgmiReducer(0, 1, 0, grads, [0, 1181120, 1181120, n], 10.0, mode)
        x.open_peers([bytes(x.ipc_handle())])
        res = x.result()
        x.bucket_ready(0)
        x.bucket_ready(1)
        x.finalize()
        torch.cuda.synchronize()
        assert torch.equal(res, grads)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            grads.add_(1.0)
            x.all_ready()
            x.finalize()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        assert torch.equal(res, grads)
        assert x.error() == 0
        x.close()


def test_cnn_step_through_xgmi_matches_local(gpu):
    """World-size-1 forced xgmi reducer (fc bucket during cnn_bwd, conv bucket after
    conv_reduce, optimizer reading the result arena), graph-captured, gives the same
    parameters as the world_size-1 fast path."""
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
    from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
    from pytorch_distributed_mnist_amd.parallel.comm import RcclComm
    from pytorch_distributed_mnist_amd.runtime.gpu_step import GpuStepBase
    from pytorch_distributed_mnist_amd.runtime.program import build_local_program
    train = synthetic_split(256 * (GpuStepBase.GRAPH_STEPS + 1) + 40, True)
    test = synthetic_split(256, False)
    out = []
    for force in (False, True):
        comm = RcclComm(0, 1, gpu) if force else None
        p = build_local_program("cnn", "bf16", "cuda", 256, train, test, optimizer="sgd", lr=0.05,
                                momentum=0.9, seed=4, use_graphs=True, comm=comm,
                                force_comm=force, transport="xgmi")
        assert p.reducer.kind == ("xgmi" if force else "local")
        p.optimizer.sync_hyperparams()
        p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
        p.train_epoch()
        torch.cuda.synchronize()
        p.reducer.check()
        out.append(p.arena.params.clone())
        p.reducer.close()
        if comm is not None:
            comm.close()
    assert torch.equal(out[0], out[1])


def _run_workers(nproc, tmp_path, **extra):
    # a peer that never arrives turns into an error after 10 s instead of a 60 s stall
    # 8-step graphs: the workers' 9-step epochs replay two graphs (the carry crosses a replay
    # boundary) in the step count the cross-transport tolerance below was set for
    env = dict(os.environ, PDM_SHARE_DEVICE="1", PDM_XGMI_OUT=str(tmp_path),
               PDM_XGMI_TIMEOUT=os.environ.get("PDM_XGMI_TIMEOUT", "10"), PDM_GRAPH_STEPS="8")
    env.update(extra)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", str(nproc), "--master-addr", "127.0.0.1",
                        "--master-port", str(free_port()),
                        os.path.join(REPO, "tests", "xgmi_worker.py")],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return [json.load(open(tmp_path / f"rank{i}.json")) for i in range(nproc)]


@pytest.mark.parametrize("nproc", [2, 4])
def test_xgmi_optimizer_in_launch_exchange(gpu, tmp_path, nproc):
    """The conv bucket's in-launch exchange inside the optimizer (CnnStep with the streamed
    xgmi transport): N ranks sharing one GPU, slab segments only, against the exact rank-order
    sum, eager and graph-replayed."""
    for d in _run_workers(nproc, tmp_path, PDM_XGMI_UNIT="xchg"):
        assert d["xchg_ok"], d


def test_xgmi_two_ranks_one_gpu(gpu, tmp_path):
    for d in _run_workers(2, tmp_path):
        assert d["one"] and d["two"] and d["auto"], d
        # the child-process pre-flight ran once, before the first mapping (xgmi_probe.py)
        assert d["preflight"] == ["passed", "cached", "cached"], d
        assert d["two_modes"] == ["two-shot", "two-shot"]
        assert d["auto_modes"] == ["one-shot", "one-shot"]       # 2 ranks: one-shot
        assert d["cnn_kinds"] == ["xgmi", "torch"]
        # 2-rank sums are a + b on both transports: bit-identical training
        assert d["cnn_equal"], d
        assert d["replicas_equal"]
        # the reference Net through the multi-GPU chain (lin_reduce, streamed collective)
        assert d["lin_kinds"] == ["xgmi", "torch"]
        assert d["lin_equal"] and d["lin_replicas_equal"], d


def test_xgmi_four_ranks_one_gpu(gpu, tmp_path):
    for d in _run_workers(4, tmp_path):
        assert d["one"] and d["two"] and d["auto"], d
        assert d["auto_modes"] == ["two-shot", "one-shot"]       # fc 4.7 MB, conv 75 KB
        assert d["replicas_equal"]
        # gloo sums 4 ranks in its own order; the collective itself is checked bit-exactly
        # above, the two trainings only have to stay close (bf16 weights amplify the
        # last-bit differences over 20 SGD steps)
        assert d["cnn_max_diff"] < 5e-2, d
        assert d["lin_replicas_equal"] and d["lin_max_diff"] < 1e-3, d


def test_xgmi_absent_peer_fails_fast(gpu, tmp_path):
    """A peer that never joins costs ONE timeout: after the first give-up every later
    wait of that rank (12 collective launches + 6 finalizes here) sees the error word and
    returns, and check() reports the invalid gradients instead of the run hanging."""
    d = _run_workers(2, tmp_path, PDM_XGMI_TIMEOUT="2", PDM_XGMI_ABSENT="1")[0]
    assert d["check_raised"], d
    assert d["error"] != 0, d
    # without fail-fast: >= 12 x 2 s; with it: the first timeout(s) only
    assert d["elapsed_s"] < 8.0, d


def test_xgmi_absent_peer_fails_fast_streamed(gpu, tmp_path):
    """The same through the default streamed mode: 19 graph-replayed CNN steps (four
    persistent collective launches: 8 + 8 + 2 + 1 steps) on rank 0 whose peer never
    runs a step.  The collective's first phase-0 wait times out (the recorded first
    cause); every optimizer-side wait and every later READY / peer wait fails fast, so the
    run costs about one timeout instead of one per step, and check() names the cause."""
    d = _run_workers(2, tmp_path, PDM_XGMI_TIMEOUT="2", PDM_XGMI_ABSENT="streamed")[0]
    assert d["streamed"], d
    assert d["check_raised"], d
    assert d["first_error"] == 1, d                  # XG_ERR_PEER0: the root cause
    assert d["error"] & 16, d                        # later waits failed fast
    assert "first cause: a peer did not arrive" in d["message"], d
    # without fail-fast: one 2 s timeout per step (>= 38 s); with it: about one
    assert d["elapsed_s"] < 8.0, d
