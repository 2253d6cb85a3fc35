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
    red = GradReducer(comm, grads, [(0, 4096), (4096, 10000)], force=True)
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
