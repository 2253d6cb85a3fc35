"""Native RCCL communicator + bucketed reducer on one GPU (1-rank communicator),
including capture of the reducer's fork/join into a hipGraph."""
import pytest
import torch

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


def test_cnn_step_through_rccl_reducer_matches_local(gpu):
    """The world_size > 1 step structure (unfused conv reduction, grouped RCCL all-reduce of
    both buckets, finalize) with a forced 1-rank RCCL communicator, graph-captured, gives
    the same parameters as the world_size-1 fast path."""
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
    from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
    from pytorch_distributed_mnist_amd.runtime.program import build_local_program
    train = synthetic_split(256 * 9 + 40, True)
    test = synthetic_split(256, False)
    out = []
    for force in (False, True):
        comm = _comm(gpu) if force else None
        p = build_local_program("cnn", "bf16", "cuda", 256, train, test, optimizer="sgd", lr=0.05,
                                momentum=0.9, seed=4, use_graphs=True, comm=comm, force_comm=force,
                                transport="rccl")
        assert p.gpu.fuse_conv_reduce == (not force)
        p.optimizer.sync_hyperparams()
        p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
        p.train_epoch()
        torch.cuda.synchronize()
        out.append(p.arena.params.clone())
        if comm is not None:
            comm.close()
    assert torch.equal(out[0], out[1])
