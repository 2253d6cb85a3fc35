"""Fused optimizer kernel vs the flat CPU optimizer (torch op order)."""
import pytest
import torch

from pytorch_distributed_mnist_amd.models import get_spec
from pytorch_distributed_mnist_amd.optim import FlatAdam, FlatSGD
from pytorch_distributed_mnist_amd.runtime.arena import FlatArena

pytestmark = pytest.mark.gpu


def _pair(arch, kind, gpu):
    arenas = [FlatArena(get_spec(arch), d) for d in ("cpu", gpu)]
    g = torch.Generator().manual_seed(0)
    p0 = torch.randn(arenas[0].spec.total, generator=g)
    for a in arenas:
        a.params.copy_(p0)
    if kind == "adam":
        opts = [FlatAdam(a, lr=1e-3) for a in arenas]
    else:
        opts = [FlatSGD(a, lr=0.05, momentum=0.9, weight_decay=1e-4) for a in arenas]
    return arenas, opts


@pytest.mark.parametrize("frag", [False, True])
@pytest.mark.parametrize("kind", ["adam", "sgd"])
def test_optim_kernel_matches_cpu(gpu, kind, frag):
    """frag: fc1.weight's bf16 copies in the MFMA-fragment-major layouts the CNN step uses
    (kernels.h frag_pos), else row-major."""
    from pytorch_distributed_mnist_amd.ops import _ext
    C = _ext.require()
    (ac, ag), (oc, og) = _pair("cnn", kind, gpu)
    n = ag.spec.total
    # shadows for fc1.weight (transposed) and conv2.weight (plain)
    off_fc1 = ag.spec.offset("fc1.weight")
    off_c2 = ag.spec.offset("conv2.weight")
    sh_fc1 = torch.empty(128 * 9216, dtype=torch.bfloat16, device=gpu)
    sht_fc1 = torch.empty(9216 * 128, dtype=torch.bfloat16, device=gpu)
    sh_c2 = torch.empty(64 * 288, dtype=torch.bfloat16, device=gpu)
    sht_c2 = torch.empty(288 * 64, dtype=torch.bfloat16, device=gpu)
    segs = [(0, 1, off_fc1, None, None), (off_fc1, 128, 9216, sh_fc1, sht_fc1, None, False, frag, frag),
            (off_fc1 + 128 * 9216, 1, off_c2 - off_fc1 - 128 * 9216, None, None),
            (off_c2, 64, 288, sh_c2, sht_c2),
            (off_c2 + 64 * 288, 1, n - off_c2 - 64 * 288, None, None)]
    segs = [sg for sg in segs if sg[1] * sg[2] > 0]      # no empty gap segments
    grad_scale = 0.5
    for step in range(3):
        g = torch.randn(n, generator=torch.Generator().manual_seed(10 + step))
        ac.grads.copy_(g)
        ag.grads.copy_(g)
        oc.step_cpu(grad_scale=grad_scale)
        og.sync_hyperparams()
        og._step_dev.fill_(step + 1)
        grp = og.param_groups[0]
        if kind == "adam":
            C.optim_step(C.OPT_ADAM, ag.params, ag.grads, og.exp_avg, og.exp_avg_sq, og._lr_dev,
                         og._step_dev, 0.9, 0.999, 1e-8, 0.0, 0.0, 0.0, False, grad_scale, segs)
        else:
            C.optim_step(C.OPT_SGD, ag.params, ag.grads, og.momentum_buffer, None, og._lr_dev,
                         og._step_dev, 0.0, 0.0, 0.0, grp["weight_decay"], grp["momentum"], 0.0,
                         False, grad_scale, segs)
    torch.cuda.synchronize()
    assert torch.allclose(ag.params.cpu(), ac.params, atol=1e-6, rtol=1e-5)
    w = ag.params[off_fc1:off_fc1 + 128 * 9216]
    if frag:
        from pytorch_distributed_mnist_amd.runtime.cnn_step import frag_major, frag_major_t
        wb = w.view(128, 9216).to(torch.bfloat16)
        assert torch.equal(sh_fc1, frag_major(wb))
        assert torch.equal(sht_fc1, frag_major_t(wb))
    else:
        assert torch.equal(sh_fc1, w.to(torch.bfloat16))
        assert torch.equal(sht_fc1.view(9216, 128), w.view(128, 9216).t().to(torch.bfloat16))
    w2 = ag.params[off_c2:off_c2 + 64 * 288]
    assert torch.equal(sht_c2.view(288, 64), w2.view(64, 288).t().to(torch.bfloat16))


@pytest.mark.parametrize("kind", ["adam", "sgd"])
def test_optim_slab_segments_ragged_and_bump(gpu, kind):
    """Slab segments (the gradient is the fixed-order sum of per-workgroup slabs) with a
    numel that is not a multiple of 4 (the Linear bias: 10), and the launch's counter bump:
    same parameters as the optimizer over the pre-summed gradient."""
    from pytorch_distributed_mnist_amd.ops import _ext
    C = _ext.require()
    (ac, ag), (oc, og) = _pair("linear", kind, gpu)
    spec = ag.spec
    nslab, stride = 37, 7856
    g = torch.Generator().manual_seed(3)
    slab = torch.randn(nslab, stride, generator=g)
    want = torch.zeros(spec.total)
    grad_w = slab[:, :7840].sum(0)
    grad_b = slab[:, 7840:7850].sum(0)
    ow, ob = spec.offset("fc.weight"), spec.offset("fc.bias")
    want[ow:ow + 7840] = grad_w
    want[ob:ob + 10] = grad_b
    ac.grads.copy_(want)
    oc.step_cpu(grad_scale=1.0)
    og.sync_hyperparams()
    og._step_dev.fill_(1)
    sd = slab.reshape(-1).to(gpu)
    segs = [(ow, 10, 784, None, None, (sd, nslab, 0, stride)),
            (ob, 1, 10, None, None, (sd, nslab, 7840, stride))]
    ctr = torch.zeros(1, dtype=torch.int64, device=gpu)
    before = ag.params.clone()
    grp = og.param_groups[0]
    if kind == "adam":
        C.optim_step(C.OPT_ADAM, ag.params, ag.grads, og.exp_avg, og.exp_avg_sq, og._lr_dev,
                     og._step_dev, 0.9, 0.999, 1e-8, 0.0, 0.0, 0.0, False, 1.0, segs, bump=ctr)
    else:
        C.optim_step(C.OPT_SGD, ag.params, ag.grads, og.momentum_buffer, None, og._lr_dev,
                     og._step_dev, 0.0, 0.0, 0.0, grp["weight_decay"], grp["momentum"], 0.0,
                     False, 1.0, segs, bump=ctr)
    torch.cuda.synchronize()
    assert ctr.item() == 1
    for name, o, n in (("fc.weight", ow, 7840), ("fc.bias", ob, 10)):
        gg = ag.grads[o:o + n].cpu()
        assert torch.allclose(gg, want[o:o + n], rtol=1e-5, atol=1e-5), name
        d = (ag.params[o:o + n].cpu() - ac.params[o:o + n]).abs().max().item()
        assert d < 1e-5, (name, d)
    # the arena padding after the bias (the slab's loss / correct columns) is untouched
    assert torch.equal(ag.params[ob + 10:], before[ob + 10:])
