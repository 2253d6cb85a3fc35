"""Backward kernels on identical bf16 inputs vs an fp64 PyTorch reference.

These isolate kernel logic from bf16 rounding: every operand the kernel reads is
fed to the reference exactly, so only fp32-vs-fp64 summation order differs."""
import pytest
import torch

from pytorch_distributed_mnist_amd.runtime.cnn_step import a1_swizzled, frag_major, frag_major_t

pytestmark = pytest.mark.gpu


def _C():
    from pytorch_distributed_mnist_amd.ops import _ext
    return _ext.require()


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("B,ipb,bands", [(3, 1, 1), (5, 2, 1), (7, 3, 1),
                                         (3, 1, 2), (5, 1, 3), (4, 1, 6), (1, 1, 6)])
def test_cnn_bwd_exact(gpu, B, ipb, bands):
    """cnn_bwd (bands = 1, ipb images per workgroup) and the small-batch row-band split
    cnn_bwd_band (each image over `bands` workgroups) against fp64."""
    C = _C()
    g = torch.Generator().manual_seed(B)
    xg = torch.randint(0, 256, (B, 784), generator=g, dtype=torch.uint8)
    w1 = torch.randn(32, 9, generator=g) * 0.3
    b1 = torch.randn(32, generator=g) * 0.1
    xn = ((xg.to(torch.float32) / 255.0 - 0.1307) / 0.3081).to(torch.bfloat16).float()
    # the kernel recomputes a1 = bf16(relu(conv1(bf16 x, bf16 w1) + b1))
    a1 = torch.relu(torch.nn.functional.conv2d(
        xn.view(B, 1, 28, 28), w1.to(torch.bfloat16).float().view(32, 1, 3, 3), b1))
    a1 = a1.permute(0, 2, 3, 1).reshape(B, 676, 32).to(torch.bfloat16)
    dpool = torch.randn(B, 9216, generator=g).to(torch.bfloat16)
    s = torch.randint(0, 4, (B, 9216), generator=g)
    pos = torch.rand(B, 9216, generator=g) < 0.7
    pmask = torch.where(pos, 0x80 | (1 << s), 0).to(torch.uint8)   # cnn_fwd's encoding
    w2 = torch.randn(64, 9, 32, generator=g).to(torch.bfloat16)          # [co][tap][ci]
    w2t = w2.reshape(64, 288).t().contiguous()                             # [tap*32+ci][co]
    nblk = C.cnn_bwd_nblk(B, ipb, bands)
    assert nblk == (B * bands if bands > 1 else -(-B // ipb))
    slab = torch.full((nblk * C.CNN_CONV_SLAB,), float("nan"), device=gpu)   # every entry written
    # the band backward reads the forward's a1 image (swizzled) and normalised bf16 x
    a1g = a1_swizzled(a1).to(gpu)
    xng = xn.to(torch.bfloat16).reshape(-1).to(gpu)
    C.cnn_bwd(xg.to(gpu), w1.to(gpu), b1.to(gpu), dpool.to(gpu), pmask.to(gpu), w2t.to(gpu), B,
              ipb, slab, None, bands, a1g, xng)
    gw2 = torch.zeros(64 * 288, device=gpu)
    gb2 = torch.zeros(64, device=gpu)
    gw1 = torch.zeros(288, device=gpu)
    gb1 = torch.zeros(32, device=gpu)
    C.conv_reduce(slab, nblk, gw2, gb2, gw1, gb1)
    torch.cuda.synchronize()

    # fp64 reference
    d = torch.float64
    dp = dpool.to(d).view(B, 12, 12, 64)
    mk = pmask.view(B, 12, 12, 64).long()
    dz2 = torch.zeros(B, 24, 24, 64, dtype=d)
    for sidx in range(4):
        sel = (mk == (0x80 | (1 << sidx))).to(d)
        dz2[:, (sidx >> 1)::2, (sidx & 1)::2, :] = dp * sel
    a1n = a1.to(d).view(B, 26, 26, 32).permute(0, 3, 1, 2)                # NCHW
    dzn = dz2.permute(0, 3, 1, 2)
    W2 = w2.to(d).view(64, 3, 3, 32).permute(0, 3, 1, 2)                   # [co][ci][ky][kx]
    ref_gw2 = torch.nn.grad.conv2d_weight(a1n, W2.shape, dzn)             # [co][ci][ky][kx]
    ref_gb2 = dzn.sum((0, 2, 3))
    da1 = torch.nn.grad.conv2d_input(a1n.shape, W2, dzn)
    dz1 = da1 * (a1n > 0)
    # conv1 wgrad runs on a bf16 MFMA: dz1 and x enter it rounded to bf16
    dz1 = dz1.to(torch.bfloat16).to(d)
    x = ((xg.to(torch.float32) / 255.0 - 0.1307) / 0.3081).to(torch.bfloat16).to(d)
    x = x.view(B, 1, 28, 28)
    ref_gw1 = torch.nn.grad.conv2d_weight(x, (32, 1, 3, 3), dz1)
    ref_gb1 = dz1.sum((0, 2, 3))

    got_gw2 = gw2.cpu().double().view(64, 3, 3, 32).permute(0, 3, 1, 2)
    assert rel(got_gw2, ref_gw2) < 1e-4     # a1 recompute may round a few values differently
    assert rel(gb2.cpu().double(), ref_gb2) < 1e-5
    assert rel(gw1.cpu().double().view(32, 1, 3, 3), ref_gw1) < 1e-4
    assert rel(gb1.cpu().double(), ref_gb1) < 1e-4


@pytest.mark.parametrize("B", [64, 40, 1])
def test_fc1_bwd_exact(gpu, B):
    C = _C()
    g = torch.Generator().manual_seed(B)
    ldt = -(-B // 32) * 32
    dh = torch.zeros(ldt, 128)
    dh[:B] = torch.randn(B, 128, generator=g)
    dh = dh.to(torch.bfloat16)
    dht = dh.t().contiguous()
    pool = torch.randn(B, 9216, generator=g).to(torch.bfloat16)
    w1 = torch.randn(128, 9216, generator=g).to(torch.bfloat16)
    hb = C.cnn_head_nblk(ldt)
    head_slab = torch.randn(hb, C.CNN_HEAD_SLAB, generator=g)
    gwf1 = torch.zeros(128 * 9216, device=gpu)
    dpool = torch.zeros(B * 9216, dtype=torch.bfloat16, device=gpu)
    gwf2 = torch.zeros(1280, device=gpu)
    gbf2 = torch.zeros(10, device=gpu)
    gbf1 = torch.zeros(128, device=gpu)
    metrics = torch.zeros(3, dtype=torch.float64, device=gpu)
    # dh, dh^T and W1^T in the MFMA-fragment-major layouts (kernels.h frag_pos) the kernel reads
    C.fc1_bwd(frag_major(dh).to(gpu), frag_major(dht).to(gpu), ldt, pool.to(gpu),
              frag_major_t(w1).to(gpu), B, gwf1,
              dpool, head_slab.to(gpu), gwf2, gbf2, gbf1, metrics)
    torch.cuda.synchronize()
    d = torch.float64
    ref_gw = dh[:B].to(d).t() @ pool.to(d)
    assert rel(gwf1.cpu().double().view(128, 9216), ref_gw) < 1e-5
    ref_dp = dh[:B].to(d) @ w1.to(d)
    got_dp = dpool.cpu().double().view(B, 9216)
    assert rel(got_dp, ref_dp) < 5e-3           # output rounded to bf16
    hs = head_slab.double().sum(0)
    assert rel(gwf2.cpu().double(), hs[:1280]) < 1e-6
    assert rel(gbf2.cpu().double(), hs[1280:1290]) < 1e-6
    assert rel(gbf1.cpu().double(), hs[1290:1418]) < 1e-6
    m = metrics.cpu()
    assert abs(m[0] - hs[1418]) < 1e-3 and abs(m[1] - hs[1419]) < 1e-3 and m[2] == B
