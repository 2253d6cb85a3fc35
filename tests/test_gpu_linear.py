"""HIP Linear-model kernels vs a plain PyTorch fp32 reference (reference model Net)."""
import pytest
import torch
import torch.nn.functional as F

from pytorch_distributed_mnist_amd.data.mnist import normalize_reference, synthetic_split
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
from pytorch_distributed_mnist_amd.runtime.program import build_local_program

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("gather", [True, False])
@pytest.mark.parametrize("B,bfull", [(256, 256), (96, 256), (1, 8), (13, 32)])
def test_lin_train_reduce_matches_torch(gpu, B, bfull, gather):
    from pytorch_distributed_mnist_amd.ops import _ext
    C = _ext.require()
    g = torch.Generator().manual_seed(B)
    N = 600
    images = torch.randint(0, 256, (N, 784), generator=g, dtype=torch.uint8)
    labels = torch.randint(0, 10, (N,), generator=g)
    idx = torch.randperm(N, generator=g)[:2 * bfull].to(torch.int32)
    W = torch.randn(10, 784, generator=g) * 0.05
    b = torch.randn(10, generator=g) * 0.1
    step = 1
    sel = idx[step * bfull: step * bfull + B].long()
    x = normalize_reference(images[sel]).requires_grad_(False)
    Wr, br = W.clone().requires_grad_(), b.clone().requires_grad_()
    logits = F.linear(x, Wr, br)
    loss = F.cross_entropy(logits, labels[sel])
    loss.backward()
    correct = logits.argmax(1).eq(labels[sel]).sum().item()

    dev = gpu
    nblk = (bfull + C.LIN_ROWS - 1) // C.LIN_ROWS
    slab = torch.zeros(nblk * C.LIN_SLAB, device=dev)
    ctr = torch.tensor([step, 0], dtype=torch.int64, device=dev)
    ostep = torch.zeros(1, dtype=torch.int64, device=dev)
    metrics = torch.zeros(3, dtype=torch.float64, device=dev)
    gW = torch.zeros(10, 784, device=dev)
    gb = torch.zeros(10, device=dev)
    if gather:        # sampler gather: images[idx[ctr * bfull + i]]
        C.lin_train(images.to(dev), labels.to(dev, torch.int32), idx.to(dev), ctr[0:1], bfull, B,
                    W.to(dev), b.to(dev), slab, metrics, ostep)
    else:             # epoch buffer: rows ctr * bfull + i of the gathered epoch
        C.lin_train(images[idx.long()].to(dev), labels[idx.long()].to(dev, torch.int32), None,
                    ctr[0:1], bfull, B, W.to(dev), b.to(dev), slab, metrics, ostep)
    # lin_reduce also adds the train loss / correct partials (fixed order) to the metrics
    C.lin_reduce(slab, B, gW, gb, ctr[0:1], None, metrics)
    torch.cuda.synchronize()
    assert torch.allclose(gW.cpu(), Wr.grad, atol=2e-6, rtol=1e-4)
    assert torch.allclose(gb.cpu(), br.grad, atol=2e-6, rtol=1e-4)
    m = metrics.cpu()
    assert abs(m[0].item() - loss.item() * B) < 1e-4 * B
    assert m[1].item() == correct and m[2].item() == B
    assert ctr[0].item() == step + 1 and ostep.item() == 1


def test_lin_eval_matches_torch(gpu):
    from pytorch_distributed_mnist_amd.ops import _ext
    C = _ext.require()
    split = synthetic_split(1000, False)
    g = torch.Generator().manual_seed(0)
    W = torch.randn(10, 784, generator=g) * 0.05
    b = torch.randn(10, generator=g) * 0.1
    x = normalize_reference(split.images)
    logits = F.linear(x, W, b)
    loss_sum = F.cross_entropy(logits, split.labels, reduction="sum").item()
    correct = logits.argmax(1).eq(split.labels).sum().item()
    metrics = torch.zeros(3, dtype=torch.float64, device=gpu)
    C.lin_eval(split.images.to(gpu), split.labels.to(gpu, torch.int32), W.to(gpu), b.to(gpu),
               metrics)
    m = metrics.cpu()
    assert abs(m[0].item() - loss_sum) < 1e-3
    assert m[1].item() == correct and m[2].item() == 1000


@pytest.mark.parametrize("graphs", [False, True])
@pytest.mark.parametrize("opt", ["adam", "sgd"])
def test_linear_epoch_gpu_matches_cpu(gpu, graphs, opt):
    train = synthetic_split(2048 + 96, True)
    test = synthetic_split(512, False)
    progs = {}
    for dev in ("cpu", "cuda"):
        p = build_local_program("linear", "fp32", dev, 256, train, test, optimizer=opt,
                                lr=1e-3 if opt == "adam" else 0.05, seed=5, use_graphs=graphs)
        p.optimizer.sync_hyperparams()
        p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
        tl, ta = p.train_epoch()
        el, ea = p.evaluate()
        progs[dev] = (p, tl, ta, el, ea)
    pc, pg = progs["cpu"][0], progs["cuda"][0]
    assert pg.gpu.fuse_reduce            # world size 1: slab reduction inside the optimizer
    assert pg.steps_per_epoch == 9    # ragged tail of 96 included
    diff = (pc.arena.params - pg.arena.params.cpu()).abs().max().item()
    assert diff < 5e-5, diff
    assert abs(progs["cpu"][1].average - progs["cuda"][1].average) < 1e-4
    assert progs["cpu"][2].correct == progs["cuda"][2].correct
    assert abs(progs["cpu"][3].average - progs["cuda"][3].average) < 1e-4
    assert pg.optimizer.step_count == 9 and int(pg.optimizer._step_dev.item()) == 9


@pytest.mark.parametrize("opt", ["adam", "sgd"])
def test_linear_fused_reduce_matches_unfused(gpu, opt, monkeypatch):
    """World size 1 sums the gradient slabs inside the optimizer launch; the unfused chain
    (lin_reduce -> optim, the multi-GPU structure) must give the same training run."""
    train = synthetic_split(1024 + 40, True)
    test = synthetic_split(256, False)
    out = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("PDM_FUSE_LIN_REDUCE", fuse)
        p = build_local_program("linear", "fp32", "cuda", 128, train, test, optimizer=opt,
                                lr=1e-3 if opt == "adam" else 0.05, seed=3, use_graphs=True)
        assert p.gpu.fuse_reduce == (fuse == "1")
        p.optimizer.sync_hyperparams()
        p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
        tl, ta = p.train_epoch()
        out[fuse] = (p.arena.params.clone(), tl.average, ta.correct, p.gpu.ctr[0].item(),
                     int(p.optimizer._step_dev.item()))
    a, b = out["1"], out["0"]
    assert (a[0] - b[0]).abs().max().item() < 1e-6
    assert abs(a[1] - b[1]) < 1e-6 and a[2] == b[2]   # slab sums in a different order
    assert a[3] == b[3] == 9 and a[4] == b[4] == 9


def test_linear_train_metrics_bitwise_reproducible(gpu):
    """Two identical epochs give bit-identical fp64 train loss sums (fixed-order reduction of
    the per-workgroup partials, no fp64 atomics)."""
    train = synthetic_split(256 * 6, True)
    test = synthetic_split(64, False)
    out = []
    for _ in range(2):
        p = build_local_program("linear", "fp32", "cuda", 256, train, test, optimizer="adam",
                                lr=1e-3, seed=3, use_graphs=True)
        p.optimizer.sync_hyperparams()
        p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
        p.train_epoch()
        torch.cuda.synchronize()
        out.append(p.metrics.buf[0:3].clone())
    assert torch.equal(out[0], out[1]), out
