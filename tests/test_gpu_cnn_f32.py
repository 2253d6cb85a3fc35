"""CNN fp32 GPU path (``--dtype fp32``, cnn_f32.hip on v_mfma_f32_16x16x4_f32) against fp32
PyTorch autograd: the reference trains in fp32 (multi_proc_single_gpu.py:185-191), so the
gradients of one step must agree to fp32 summation-order noise (<= 1e-4 relative)."""
import pytest
import torch
import torch.nn.functional as F

from pytorch_distributed_mnist_amd.data.mnist import normalize_reference, synthetic_split
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
from pytorch_distributed_mnist_amd.models.reference import MODULES
from pytorch_distributed_mnist_amd.runtime.program import build_local_program

pytestmark = pytest.mark.gpu


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _program(B, n, lr=0.0, graphs=False, seed=0, optimizer="sgd"):
    train = synthetic_split(n, True)
    test = synthetic_split(300, False)
    prog = build_local_program("cnn", "fp32", "cuda", B, train, test, optimizer=optimizer, lr=lr,
                               momentum=0.0 if lr == 0.0 else 0.9,
                               weight_decay=0.0 if lr == 0.0 else 1e-4, seed=seed,
                               use_graphs=graphs)
    prog.optimizer.sync_hyperparams()
    return prog, train, test


def _reference_net(prog):
    net = MODULES["cnn"]()
    sd = {k[len("module."):]: v for k, v in prog.arena.state_dict().items()}
    net.load_state_dict(sd)
    return net


def _kernel_a1_active(prog, B):
    """The split-bf16 forward's ReLU decisions for conv1: a1 > 0 iff its hi or lo bf16 part
    is non-zero, read from the a1 planes it hands the backward (a1g: per image a hi and a lo
    plane, 26 x 26 pixels x 32 channels, 16-B chunk c of pixel (y, x) at c ^ (x & 3))."""
    raw = prog.gpu.a1g[:B * 676 * 32].view(torch.int16).view(B, 2, 26, 26, 4, 8).cpu()
    act = (raw[:, 0] != 0) | (raw[:, 1] != 0)                       # [B, y, x, phys chunk, 8]
    xi = torch.arange(26).view(1, 1, 26, 1)
    phys = torch.arange(4).view(1, 1, 1, 4) ^ (xi & 3)              # logical chunk -> physical
    act = act.gather(3, phys.expand(B, 26, 26, 4).unsqueeze(-1).expand(B, 26, 26, 4, 8))
    return act.reshape(B, 26, 26, 32).permute(0, 3, 1, 2)


def _fp64_grads_with_mask(prog, x, y, pmask, B, a1_active=None):
    """fp64 autograd of the step, max-pool routed by the kernel's own argmax decisions (the
    pool mask): where two window values tie within fp32 rounding, fp32 and fp64 may pick
    different positions, and a gradient routed to a neighbouring pixel is a discrete
    difference, not a precision one.  a1_active: conv1's ReLU routed the same way (the
    split-bf16 conv2 / fc1 leave conv1's fp32 ReLU decisions alone, so this changes little;
    a split-bf16 conv1 put ~15 of 1.4 M activations per 64 images on the other side of zero,
    each moving a whole dgrad value into or out of the conv1 gradients)."""
    net = _reference_net(prog).double()
    z1 = net.conv1(x.double())
    zero = torch.zeros((), dtype=torch.float64)
    a1 = F.relu(z1) if a1_active is None else torch.where(a1_active, z1, zero)
    z2 = net.conv2(a1)                                            # [B, 64, 24, 24]
    mk = pmask[:B * 9216].view(B, 12, 12, 64).permute(0, 3, 1, 2).cpu().long()
    pos = (mk & 0x80) != 0
    sidx = torch.where(pos, (mk & 0xf).float().log2().long(), torch.zeros_like(mk))
    py = torch.arange(12).view(1, 1, 12, 1)
    px = torch.arange(12).view(1, 1, 1, 12)
    flat = (2 * py + (sidx >> 1)) * 24 + 2 * px + (sidx & 1)
    pooled = torch.where(pos, z2.flatten(2).gather(2, flat.flatten(2)).view(B, 64, 12, 12),
                         torch.zeros((), dtype=torch.float64))
    out = net.fc2(F.relu(net.fc1(pooled.flatten(1))))
    F.cross_entropy(out, y).backward()
    return dict(net.named_parameters()), out


@pytest.mark.parametrize("conv,upw", [("exact", None), ("x3", None), ("x3", "4"), ("x3", "7")])
@pytest.mark.parametrize("B", [64, 37, 256])
def test_f32_gradients_match_fp32_autograd(gpu, B, conv, upw, monkeypatch):
    """One training step with lr = 0: the gradient arena holds the step's gradients (the fused
    optimizer writes the reduced conv gradients back).  Compared per parameter with fp64
    autograd of the same step (max-pool routed as the kernel routed it): <= 1e-4 relative,
    fp32 summation-order noise; and with fp32 autograd (torch's own routing).  upw: (image,
    band) units per split-bf16 conv-backward workgroup (default: one round of <= 256
    workgroups), 4 / 7 = workgroups that change image and band mid-way and a partial last one."""
    if upw is not None:
        monkeypatch.setenv("PDM_F32_UPW", upw)
    prog, train, _ = _program(B, n=max(2 * B, 300))
    prog.gpu.conv_x3 = conv == "x3"
    idx = distributed_indices(len(train), 1, 0, 0)
    prog.set_train_indices(idx)
    net = _reference_net(prog)
    prog.gpu.begin_epoch()
    prog.gpu.train_step(B)
    torch.cuda.synchronize()
    sel = idx[:B]
    x = normalize_reference(train.images[sel]).view(B, 1, 28, 28)
    out = net(x)
    loss = F.cross_entropy(out, train.labels[sel])
    loss.backward()
    a1_active = None
    if conv == "x3":
        a1_active = _kernel_a1_active(prog, B)
        with torch.no_grad():
            z1 = _reference_net(prog).double().conv1(x.double())
        flips = (a1_active != (z1 > 0)).sum().item()
        assert flips <= 1e-4 * a1_active.numel(), flips     # rare near-zero activations only
    ref64, _ = _fp64_grads_with_mask(prog, x, train.labels[sel], prog.gpu.pmask, B, a1_active)
    got = prog.arena.torch_tensors(prog.arena.grads)
    for name, p in net.named_parameters():
        r64 = rel(got[name].double(), ref64[name].grad)
        assert r64 < 1e-4, (name, r64)
        if not name.startswith("conv"):        # the conv gradients see any argmax tie flip
            assert rel(got[name], p.grad) < 1e-4, name
    tl = prog.metrics.buf[0].item()
    assert abs(tl - loss.item() * B) <= 1e-4 * B
    correct = (out.argmax(1) == train.labels[sel]).sum().item()
    assert prog.metrics.buf[1].item() == correct


@pytest.mark.parametrize("conv,tol", [("exact", 1e-4), ("x3", 1e-4)])
def test_f32_training_tracks_cpu_sgd(gpu, conv, tol):
    """Several SGD-momentum steps (graph-captured) stay within fp32 noise of the same steps
    in torch on the CPU, and the evaluation matches, in both product modes.  (A split-bf16
    conv1 -- measured, not adopted -- flipped a few ReLU decisions per step and drifted
    2e-3 from torch over these 5 steps; conv1 keeps fp32 products.)"""
    B = 64
    prog, train, test = _program(B, n=B * 5, lr=0.05, graphs=True, seed=3)
    prog.gpu.conv_x3 = conv == "x3"
    idx = distributed_indices(len(train), 1, 0, 0)
    net = _reference_net(prog)
    opt = torch.optim.SGD(net.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    prog.set_train_indices(idx)
    prog.train_epoch()
    torch.cuda.synchronize()
    for s in range(5):
        sel = idx[s * B:(s + 1) * B]
        opt.zero_grad()
        F.cross_entropy(net(normalize_reference(train.images[sel]).view(B, 1, 28, 28)),
                        train.labels[sel]).backward()
        opt.step()
    got = prog.arena.state_dict()
    for name, p in net.named_parameters():
        r = rel(got["module." + name], p.detach())
        assert r < tol, (name, r)
    tl, ta = prog.evaluate()
    with torch.no_grad():
        out = net(normalize_reference(test.images).view(-1, 1, 28, 28))
        ref_loss = F.cross_entropy(out, test.labels).item()
        ref_acc = (out.argmax(1) == test.labels).float().mean().item()
    assert abs(tl.average - ref_loss) < tol * max(1.0, ref_loss)
    assert abs(ta.accuracy - ref_acc) < 1e-6 + 2.0 / len(test.labels)


def test_f32_ws2_structure_matches_local(gpu):
    """The world-size>1 chain (conv_reduce, bucket all-reduce through a 1-rank RCCL
    communicator, one optimizer launch) gives the same parameters as the fused local chain."""
    from pytorch_distributed_mnist_amd.parallel.comm import RcclComm
    train = synthetic_split(64 * 4, True)
    test = synthetic_split(64, False)
    out = []
    for force in (False, True):
        comm = RcclComm(0, 1, gpu) if force else None
        p = build_local_program("cnn", "fp32", "cuda", 64, train, test, optimizer="sgd", lr=0.05,
                                momentum=0.9, seed=5, use_graphs=True, comm=comm,
                                force_comm=force, transport="rccl")
        p.optimizer.sync_hyperparams()
        p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
        p.train_epoch()
        torch.cuda.synchronize()
        out.append(p.arena.params.clone())
        if comm is not None:
            comm.close()
    assert torch.equal(out[0], out[1])
