"""Kernel-layout arena <-> torch layouts; functional forward == nn.Module forward."""
import torch

from pytorch_distributed_mnist_amd.models import MODULES, functional_forward, get_spec
from pytorch_distributed_mnist_amd.runtime.arena import FlatArena


def test_roundtrip_and_order():
    for arch in ("linear", "cnn"):
        torch.manual_seed(0)
        m = MODULES[arch]()
        arena = FlatArena(get_spec(arch), "cpu")
        arena.load_module(m)
        sd = arena.state_dict()
        ref = m.state_dict()
        assert list(sd.keys()) == ["module." + k for k in ref.keys()]
        for k, v in ref.items():
            assert torch.equal(sd["module." + k], v)
        # offsets are 256-B aligned, buckets tile the arena
        spec = arena.spec
        assert all(o % 64 == 0 for o in spec.offsets)
        b = spec.bucket_bounds()
        assert b[0][0] == 0 and b[-1][1] == spec.total
        for (s0, e0), (s1, e1) in zip(b, b[1:]):
            assert e0 == s1


def test_cnn_internal_layout_forward_matches_module():
    torch.manual_seed(0)
    m = MODULES["cnn"]()
    arena = FlatArena(get_spec("cnn"), "cpu")
    arena.load_module(m)
    x = torch.randn(3, 784)
    views = {p.name: p.to_torch(arena.param(p.name)) for p in arena.spec.params}
    assert torch.allclose(functional_forward("cnn", views, x), m(x), atol=0, rtol=0)
    # fc1 internal layout is [n, h, w, c]: check one element by hand
    w = arena.param("fc1.weight")
    assert w.shape == (128, 12, 12, 64)
    assert w[5, 3, 7, 11] == m.fc1.weight[5, 11 * 144 + 3 * 12 + 7]
    w2 = arena.param("conv2.weight")
    assert w2[7, 1, 2, 30] == m.conv2.weight[7, 30, 1, 2]


def test_cnn_bucket_sizes():
    spec = get_spec("cnn")
    assert spec.num_params == 1199882
    (s0, e0), (s1, e1) = spec.bucket_bounds()
    assert (e0 - s0) * 4 >= 4724264 and (e1 - s1) * 4 >= 75264


def test_cnn_channel_bounds_give_fc1_weight_its_own_channel():
    """The xGMI transport cuts the fc bucket at fc1.weight (models/specs.py channel_bounds):
    the small fc parameters form channel 0, fc1.weight channel 1, the conv bucket channel 2;
    every channel is 64-float aligned (the transport's requirement) and they tile the arena."""
    spec = get_spec("cnn")
    chans, of_bucket = spec.channel_bounds()
    (s0, e0), (s1, e1) = spec.bucket_bounds()
    off = spec.offset("fc1.weight")
    assert chans == [(s0, off), (off, e0), (s1, e1)]
    assert of_bucket == [[0, 1], [2]]
    assert all(a % 64 == 0 and b % 64 == 0 for a, b in chans)
    lin = get_spec("linear")
    assert lin.channel_bounds() == (lin.bucket_bounds(), [[0]])


def test_grad_reducer_channels_map_buckets():
    """GradReducer keeps the bucket API (bucket_ready(i), wait_bucket(i)) over the xGMI
    transport's finer channels; other transports have one channel per bucket."""
    from pytorch_distributed_mnist_amd.parallel.comm import LocalComm
    from pytorch_distributed_mnist_amd.parallel.reducer import GradReducer
    spec = get_spec("cnn")
    red = GradReducer(LocalComm(), torch.zeros(spec.total), spec.bucket_bounds(),
                      channels=spec.channel_bounds())
    assert red.cbounds == spec.channel_bounds()[0]
    assert red.channels_of(0) == [0] and red.channels_of(1) == [1]      # not xgmi
    assert red.channel_of(spec.offset("fc1.weight")) == 1
    assert red.channel_of(spec.offset("fc2.bias")) == 0
    assert red.channel_of(spec.offset("conv1.bias")) == 2
