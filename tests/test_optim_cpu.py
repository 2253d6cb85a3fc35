"""Flat-arena optimizers == torch.optim on CPU (bitwise), and torch-format state dicts."""
import pytest
import torch

from pytorch_distributed_mnist_amd.models import MODULES, get_spec
from pytorch_distributed_mnist_amd.optim import FlatAdam, FlatSGD
from pytorch_distributed_mnist_amd.runtime.arena import FlatArena


def _setup(arch, seed=0):
    torch.manual_seed(seed)
    m = MODULES[arch]()
    arena = FlatArena(get_spec(arch), "cpu")
    arena.load_module(m)
    return m, arena


def _set_grads(m, arena, step):
    g = torch.Generator().manual_seed(100 + step)
    for name, p in m.named_parameters():
        p.grad = torch.randn(p.shape, generator=g)
        spec = arena.spec.by_name(name)
        arena.grad(name).copy_(spec.to_internal(p.grad))


def _compare(m, arena):
    for name, p in m.named_parameters():
        spec = arena.spec.by_name(name)
        assert torch.equal(spec.to_torch(arena.param(name)), p.detach()), name


def test_adam_bitwise_vs_torch():
    for arch in ("linear", "cnn"):
        m, arena = _setup(arch)
        ref = torch.optim.Adam(m.parameters(), lr=1e-3, foreach=False)
        ours = FlatAdam(arena, lr=1e-3)
        for step in range(4):
            _set_grads(m, arena, step)
            ref.step()
            ours.step_cpu()
        _compare(m, arena)


def test_sgd_bitwise_vs_torch():
    m, arena = _setup("cnn")
    ref = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4, foreach=False)
    ours = FlatSGD(arena, lr=0.05, momentum=0.9, weight_decay=1e-4)
    for step in range(3):
        _set_grads(m, arena, step)
        ref.step()
        ours.step_cpu()
    _compare(m, arena)


def test_adam_state_dict_roundtrip_torch_format():
    m, arena = _setup("cnn")
    ref = torch.optim.Adam(m.parameters(), lr=1e-3)
    ours = FlatAdam(arena, lr=1e-3)
    for step in range(2):
        _set_grads(m, arena, step)
        ref.step()
        ours.step_cpu()
    sd_ref, sd = ref.state_dict(), ours.state_dict()
    assert sd["param_groups"][0].keys() == sd_ref["param_groups"][0].keys()
    assert sd["param_groups"][0]["params"] == sd_ref["param_groups"][0]["params"]
    for i, st in sd_ref["state"].items():
        assert set(st) == set(sd["state"][i])
        assert sd["state"][i]["step"].dtype == torch.float32 and sd["state"][i]["step"].dim() == 0
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(sd["state"][i][k], st[k])
    # load torch's state into a fresh flat optimizer, and ours into torch's
    m2, arena2 = _setup("cnn", seed=1)
    o2 = FlatAdam(arena2, lr=1e-3)
    o2.load_state_dict(sd_ref)
    assert o2.step_count == 2
    assert torch.equal(o2.exp_avg, ours.exp_avg)
    ref2 = torch.optim.Adam(m2.parameters(), lr=1e-3)
    ref2.load_state_dict(sd)


def test_sgd_state_dict_format():
    m, arena = _setup("linear")
    ref = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    ours = FlatSGD(arena, lr=0.1, momentum=0.9, weight_decay=1e-4)
    assert ours.state_dict()["state"] == {}
    _set_grads(m, arena, 0)
    ref.step()
    ours.step_cpu()
    sd = ours.state_dict()
    assert sd["param_groups"][0].keys() == ref.state_dict()["param_groups"][0].keys()
    assert set(sd["state"][0]) == {"momentum_buffer"}


def test_optimizer_kind_mismatch_is_reported():
    from pytorch_distributed_mnist_amd.models.specs import get_spec
    from pytorch_distributed_mnist_amd.optim.flat import FlatAdam, FlatSGD
    from pytorch_distributed_mnist_amd.runtime.arena import FlatArena
    arena = FlatArena(get_spec("linear"), torch.device("cpu"))
    sgd_sd = FlatSGD(arena, lr=0.1, momentum=0.9).state_dict()
    with pytest.raises(ValueError, match="--optimizer sgd"):
        FlatAdam(arena, lr=1e-3).load_state_dict(sgd_sd)
    adam_sd = FlatAdam(arena, lr=1e-3).state_dict()
    with pytest.raises(ValueError, match="--optimizer adam"):
        FlatSGD(arena, lr=0.1).load_state_dict(adam_sd)
