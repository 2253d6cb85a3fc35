"""DDP-style cross-rank model check before the weight broadcast (gloo, 2 ranks on CPU).

Reference: ``DistributedDataParallel(model, ...)`` (multi_proc_single_gpu.py:188-189) verifies
that every rank has the same parameters before broadcasting rank 0's.  A rank started with
another ``--arch`` must fail with a clear message on every rank, not receive foreign bytes.
"""
import os

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port


def _worker(rank, port, archs, q):
    os.environ.pop("PDM_SHARE_DEVICE", None)
    from pytorch_distributed_mnist_amd.models.specs import get_spec
    from pytorch_distributed_mnist_amd.parallel import verify_params_across_ranks
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", world_size=2, rank=rank)
    try:
        verify_params_across_ranks(get_spec(archs[rank]), rank, 2)
        q.put((rank, "ok"))
    except RuntimeError as e:
        q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def _run(archs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, port, archs, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    return out


def test_same_model_passes():
    assert _run(("cnn", "cnn")) == {0: "ok", 1: "ok"}


def test_mismatched_arch_fails_on_every_rank():
    out = _run(("cnn", "linear"))
    for r in (0, 1):
        msg = out[r]
        assert msg != "ok"
        assert "parameter verification failed" in msg
        assert "rank 1 has 7850 parameters in 2 tensors" in msg
        assert "rank 0 has 1199882 parameters in 8 tensors" in msg


def test_signature_is_layout_sensitive():
    from pytorch_distributed_mnist_amd.models.specs import get_spec
    from pytorch_distributed_mnist_amd.parallel.verify import model_signature
    a, b = model_signature(get_spec("cnn")), model_signature(get_spec("linear"))
    assert a != b and a[0] == 1199882 and b[0] == 7850
    assert model_signature(get_spec("cnn")) == a      # deterministic across processes
