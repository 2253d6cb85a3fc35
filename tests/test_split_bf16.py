"""Precision of the split-bf16 ("bf16x3") products the fp32 CNN path runs its conv2 GEMMs with
(csrc/kernels/cnn_f32.hip f32x3_*): x = hi + lo with hi = bf16(x), lo = bf16(x - hi), and a
product taken as hi.hi + hi.lo + lo.hi with fp32 accumulation.  Emulated here in torch on the
CPU (bf16 products are exact in fp32) against fp64, next to TF32 (10-bit mantissa operands,
what cuDNN uses for fp32 convolutions by default) and plain bf16 operands."""
import torch
import torch.nn.functional as F


def _split(t):
    hi = t.to(torch.bfloat16).to(torch.float32)
    lo = (t - hi).to(torch.bfloat16).to(torch.float32)
    return hi, lo


def _tf32(t):
    # round-to-nearest to a 10-bit mantissa
    i = t.view(torch.int32)
    return ((i + 0x1000 + ((i >> 13) & 1) - 1) & ~0x1FFF).view(torch.float32)


def _rel(a, b):
    return ((a.double() - b).norm() / b.norm()).item()


def test_split_bf16_conv2_precision():
    g = torch.Generator().manual_seed(0)
    a1 = torch.relu(torch.randn(8, 32, 26, 26, generator=g))          # conv1 activations
    w2 = torch.randn(64, 32, 3, 3, generator=g) * (2.0 / 288) ** 0.5   # kaiming-scaled
    ref = F.conv2d(a1.double(), w2.double())
    ah, al = _split(a1)
    wh, wl = _split(w2)
    x3 = F.conv2d(ah, wl) + F.conv2d(al, wh) + F.conv2d(ah, wh)
    fp32 = F.conv2d(a1, w2)
    tf32 = F.conv2d(_tf32(a1), _tf32(w2))
    bf16 = F.conv2d(ah, wh)
    e_x3, e_32, e_tf, e_bf = (_rel(x, ref) for x in (x3, fp32, tf32, bf16))
    # bf16x3 sits between fp32 and TF32, orders of magnitude closer to fp32 than bf16 is
    assert e_x3 < 2e-5, e_x3
    assert e_x3 < e_tf / 10 and e_x3 < e_bf / 100, (e_x3, e_tf, e_bf)
    assert e_32 < e_x3


def test_split_is_exact_for_bf16_values_and_bounded_otherwise():
    g = torch.Generator().manual_seed(1)
    x = torch.randn(100000, generator=g) * torch.exp(torch.randn(100000, generator=g) * 5)
    hi, lo = _split(x)
    err = ((hi + lo).double() - x.double()).abs() / x.double().abs()
    assert err.max().item() <= 2.0 ** -16
    xb = x.to(torch.bfloat16).to(torch.float32)
    hb, lb = _split(xb)
    assert torch.equal(hb, xb) and (lb == 0).all()
