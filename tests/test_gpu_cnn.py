"""HIP CNN kernels (bf16 MFMA) vs plain PyTorch fp32 references.

Forward kernels are checked against a reference that rounds the same operands to
bf16 (so only fp32 summation order differs -> tight tolerance); the fused
backward is checked against fp32 autograd with a relative-norm tolerance sized
for bf16 activations/gradients.
"""
import pytest
import torch
import torch.nn.functional as F

from pytorch_distributed_mnist_amd.data.mnist import normalize_reference, synthetic_split
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
from pytorch_distributed_mnist_amd.runtime.program import build_local_program

pytestmark = pytest.mark.gpu


def bf(x):
    return x.to(torch.bfloat16).to(torch.float32)


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _program(B, opt="sgd", lr=0.0, graphs=False, n=600, seed=0):
    train = synthetic_split(n, True)
    test = synthetic_split(300, False)
    prog = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer=opt, lr=lr,
                               momentum=0.0 if lr == 0.0 else 0.9,
                               weight_decay=0.0 if lr == 0.0 else 1e-4, seed=seed,
                               use_graphs=graphs)
    prog.optimizer.sync_hyperparams()
    prog.gpu.keep_grads = True     # these tests read the gradient arena
    return prog, train, test


class _RoundFwd(torch.autograd.Function):
    """bf16 rounding in the forward, gradient passed through unchanged."""
    @staticmethod
    def forward(ctx, t):
        return bf(t)

    @staticmethod
    def backward(ctx, g):
        return g


class _RoundGrad(torch.autograd.Function):
    """Identity in the forward, bf16 rounding of the gradient in the backward."""
    @staticmethod
    def forward(ctx, t):
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        return bf(g)


def bf16_mirrored_forward(p, x):
    """The CNN forward with the kernel chain's bf16 rounding points (csrc/kernels/cnn_fwd.hip,
    cnn_bwd.hip, docs/kernels.md): x, conv1 / conv2 / fc1 weights, a1 and the pooled features
    are bf16 operands; dh (fc1 pre-activation grad, stored bf16 by cnn_head), dpool (bf16
    from fc1_bwd's dX tiles) and da1 (the conv2 dgrad after relu', the bf16 A operand of the
    conv1 weight-gradient MFMA) are rounded in the backward.  fp32 everywhere else."""
    fr, gr = _RoundFwd.apply, _RoundGrad.apply
    B = x.shape[0]
    h = fr(x.reshape(B, 1, 28, 28))
    a1 = fr(F.relu(gr(F.conv2d(h, fr(p["conv1.weight"]), p["conv1.bias"]))))
    z2 = F.relu(F.conv2d(a1, fr(p["conv2.weight"]), p["conv2.bias"]))
    pool = gr(fr(F.max_pool2d(z2, 2)))
    h = F.relu(gr(F.linear(torch.flatten(pool, 1), fr(p["fc1.weight"]), p["fc1.bias"])))
    return F.linear(h, p["fc2.weight"], p["fc2.bias"])


def _torch_params(prog):
    return prog.arena.torch_tensors(prog.arena.params)


@pytest.mark.parametrize("B,bands", [(5, 2), (7, 3), (4, 6), (1, 6)])
def test_cnn_forward_band_split(gpu, B, bands):
    """The small-batch row-band forward (each image over `bands` workgroups) computes the
    same conv1 / conv2 / pool arithmetic per output as the one-workgroup-per-image kernel:
    pooled activations, pool mask and labels are bit-identical.  In training it also hands
    the backward the normalised bf16 x (exact) and the swizzled bf16 a1 image (checked
    against a torch conv1 on the same bf16 operands)."""
    from pytorch_distributed_mnist_amd.runtime.cnn_step import a1_swizzled
    prog, train, _ = _program(B)
    st = prog.gpu
    idx = distributed_indices(len(train), 1, 0, 0)
    prog.set_train_indices(idx)
    C, P = st.C, st.P
    outs = []
    for b in (1, bands):
        for t in (st.pool, st.pmask, st.ylab, st.a1g, st.xng):
            t.view(torch.uint8).fill_(0x55) if t.dtype != torch.int32 else t.fill_(7)
        C.cnn_fwd(st.ep_images.view(-1, 784), st.ep_labels, None, st.ctr[0:1], st.bfull, B,
                  P["conv1.weight"], P["conv1.bias"], st.w2, P["conv2.bias"], st.pool, st.pmask,
                  st.xg, st.ylab, b, st.a1g, st.xng)
        torch.cuda.synchronize()
        outs.append([st.pool[:B * 9216].view(torch.uint8).clone(), st.pmask[:B * 9216].clone(),
                     st.ylab[:B].clone()])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    sel = idx[:B]
    xn = normalize_reference(train.images[sel]).to(torch.bfloat16)
    assert torch.equal(st.xng[:B * 784].cpu(), xn.reshape(-1))
    tp = _torch_params(prog)
    a1 = F.relu(F.conv2d(xn.float().view(B, 1, 28, 28), bf(tp["conv1.weight"]), tp["conv1.bias"]))
    ref = a1_swizzled(a1.permute(0, 2, 3, 1).reshape(B, 676, 32).to(torch.bfloat16))
    got = st.a1g[:B * 676 * 32].cpu()
    assert torch.allclose(got.float(), ref.float(), atol=1e-2, rtol=1e-2)
    assert (got != ref).float().mean().item() < 0.01      # bf16 rounding ties only


@pytest.mark.parametrize("B,bands", [(64, 6), (37, 2)])
def test_cnn_forward_band_split_uint8_handoff(gpu, B, bands):
    """The band forward with the uint8 hand-off of the one-image backward (kernel level: a
    band forward in front of cnn_bwd, measured slower at B = 256 and not a step structure,
    profiles/r5/fwd_bands_256/) gives cnn_fwd's pool / mask / labels and gathered image."""
    prog, train, _ = _program(B)
    st = prog.gpu
    idx = distributed_indices(len(train), 1, 0, 0)
    prog.set_train_indices(idx)
    C, P = st.C, st.P
    outs = []
    for b in (1, bands):
        for t in (st.pool, st.pmask, st.xg):
            t.view(torch.uint8).fill_(0x55)
        C.cnn_fwd(st.ep_images.view(-1, 784), st.ep_labels, None, st.ctr[0:1], st.bfull, B,
                  P["conv1.weight"], P["conv1.bias"], st.w2, P["conv2.bias"], st.pool, st.pmask,
                  st.xg, st.ylab, b, None, None)
        torch.cuda.synchronize()
        outs.append([st.pool[:B * 9216].view(torch.uint8).clone(), st.pmask[:B * 9216].clone(),
                     st.ylab[:B].clone(), st.xg[:B * 784].clone()])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert torch.equal(outs[1][3].view(B, 784).cpu(), train.images[idx[:B]])


@pytest.mark.parametrize("B", [64, 37])
def test_cnn_forward_kernels(gpu, B):
    prog, train, _ = _program(B)
    st = prog.gpu
    idx = distributed_indices(len(train), 1, 0, 0)
    prog.set_train_indices(idx)
    C = st.C
    P = st.P
    C.cnn_fwd(st.ep_images.view(-1, 784), st.ep_labels, None, st.ctr[0:1], st.bfull, B,
              P["conv1.weight"], P["conv1.bias"], st.w2, P["conv2.bias"], st.pool, st.pmask,
              st.xg, st.ylab)
    torch.cuda.synchronize()
    sel = idx[:B]
    tp = _torch_params(prog)
    x = normalize_reference(train.images[sel]).view(B, 1, 28, 28)
    assert torch.equal(st.xg[:B * 784].view(B, 784).cpu(), train.images[sel])
    assert torch.equal(st.ylab[:B].cpu(), train.labels[sel].to(torch.int32))
    # conv1/conv2 run on bf16 MFMAs with fp32 accumulation and a bf16 a1 in between:
    # reference with the same roundings -> only summation order differs
    a1 = bf(F.relu(F.conv2d(bf(x), bf(tp["conv1.weight"]), tp["conv1.bias"])))
    z2 = F.conv2d(a1, bf(tp["conv2.weight"]), tp["conv2.bias"])
    r2 = F.relu(z2)
    pooled, arg = F.max_pool2d(r2, 2, return_indices=True)
    pool = st.pool[:B * 9216].view(B, 12, 12, 64).permute(0, 3, 1, 2).float().cpu()
    assert (pool - bf(pooled)).abs().max().item() < 2e-2
    assert rel(pool, pooled) < 4e-3
    # mask: positive flag matches, and argmax agrees wherever the window has a clear winner
    mask = st.pmask[:B * 9216].view(B, 12, 12, 64).permute(0, 3, 1, 2).cpu().to(torch.int32)
    pos = (mask & 0x80) != 0
    assert ((pooled > 1e-3) <= pos).all() and (pos <= (pooled > 0)).all()
    win = r2.unfold(2, 2, 2).unfold(3, 2, 2).reshape(B, 64, 12, 12, 4)
    top2 = win.topk(2, dim=-1).values
    clear = (top2[..., 0] - top2[..., 1]) > 1e-2
    ref_s = (arg // 24 % 2) * 2 + (arg % 24 % 2)
    # one-hot argmax (0x80 | 1 << s) on positive values, 0 elsewhere
    assert (mask[~pos] == 0).all()
    assert ((mask & 0x0F) == (1 << ref_s))[clear & pos].all()
    assert (((mask & 0x0F) & ((mask & 0x0F) - 1)) == 0).all()   # one bit at most


@pytest.mark.parametrize("B,S", [(32, 32), (32, 96), (64, 48), (37, 96), (256, 32), (2048, 16),
                                 (2100, 4), (8192, 4)])
def test_fc1_fwd_split_k(gpu, B, S):
    """fc1_fwd's split-K partials (9-k-step load batches for S | 32, 3-k-step batches for
    S = 48 / 96; 128-row blocks from B = 2048 on, incl. a ragged last block) sum to
    pool . W1^T of the bf16 operands in fp32."""
    prog, _, _ = _program(B)
    st = prog.gpu
    C = st.C
    g = torch.Generator().manual_seed(B + S)
    pool = torch.randn(B, 9216, generator=g).to(torch.bfloat16)
    w1 = prog.arena.param("fc1.weight").reshape(128, 9216).float().cpu()   # kernel layout
    part = torch.full((S * B * 128,), float("nan"), device=st.pool.device)
    C.fc1_fwd(pool.to(st.pool.device), st.wf1, part, B, S)
    torch.cuda.synchronize()
    got = part.view(S, B, 128).sum(0).cpu()
    ref = pool.float() @ bf(w1).t()
    assert torch.isfinite(got).all()
    assert rel(got, ref) < 1e-5


@pytest.mark.parametrize("B", [64, 40, 300, 8192])
def test_cnn_step_gradients_match_autograd(gpu, B):
    """One step's gradients vs fp32 autograd; B = 8192 is BASELINE config 5's per-rank batch
    (32 images per conv-backward workgroup, fc1 split-K 1)."""
    prog, train, _ = _program(B, n=max(600, B))   # SGD lr=0: params unchanged, grads kept
    idx = distributed_indices(len(train), 1, 0, 0)
    prog.set_train_indices(idx)
    tp = _torch_params(prog)
    prog.gpu.begin_epoch()
    prog.metrics.reset(0)
    prog.gpu.train_step(B)
    torch.cuda.synchronize()
    sel = idx[:B]
    x = normalize_reference(train.images[sel])
    leaves = {k: v.clone().requires_grad_() for k, v in tp.items()}
    from pytorch_distributed_mnist_amd.models.reference import functional_forward
    logits = functional_forward("cnn", leaves, x)
    loss = F.cross_entropy(logits, train.labels[sel])
    loss.backward()
    got = prog.arena.torch_tensors(prog.arena.grads)
    # bf16 activations / gradients vs fp32 autograd: the conv weight gradients sum
    # ~10^5 mixed-sign bf16 products (and bf16-rounding can flip a maxpool argmax),
    # so they get a looser bound; kernel logic itself is pinned to fp64 by
    # test_gpu_cnn_bwd_exact.py.
    for name, leaf in leaves.items():
        r = rel(got[name], leaf.grad)
        assert r < (1.2e-1 if name.startswith("conv") else 5e-2), (name, r)
    # the same step in fp32 autograd with the kernels' bf16 rounding points mirrored
    # (operands rounded in the forward, dh / dpool / da1 rounded in the backward): only fp32
    # summation order and rare max-pool / ReLU ties differ, so the bound is tight
    mleaves = {k: v.clone().requires_grad_() for k, v in tp.items()}
    mloss = F.cross_entropy(bf16_mirrored_forward(mleaves, x), train.labels[sel])
    mloss.backward()
    for name, leaf in mleaves.items():
        r = rel(got[name], leaf.grad)
        assert r < (1e-2 if name.startswith("conv") else 3e-3), (name, r)
    m = prog.metrics.buf[0:3].cpu()
    assert abs(m[0].item() / B - loss.item()) < 2e-2 * max(1.0, loss.item())
    assert m[2].item() == B
    assert int(prog.gpu.ctr[0].item()) == 1 and int(prog.optimizer._step_dev.item()) == 1


def test_cnn_eval_matches_torch(gpu):
    prog, _, test = _program(64)
    tp = _torch_params(prog)
    el, ea = prog.evaluate()
    from pytorch_distributed_mnist_amd.models.reference import functional_forward
    logits = functional_forward("cnn", tp, normalize_reference(test.images))
    loss = F.cross_entropy(logits, test.labels).item()
    correct = logits.argmax(1).eq(test.labels).sum().item()
    assert el.count == len(test)
    assert abs(el.average - loss) < 2e-2 * max(1.0, loss)
    assert abs(ea.correct - correct) <= 3


@pytest.mark.parametrize("graphs", [False, True])
def test_cnn_trains_and_tracks_cpu(gpu, graphs):
    """Plain SGD (no momentum: not chaotic over a few steps) — the bf16 GPU run tracks
    the fp32 CPU run; then SGD-momentum on the GPU must learn."""
    train = synthetic_split(4096 + 64, True)
    test = synthetic_split(1000, False)
    res = {}
    for dev, dt in (("cpu", "fp32"), ("cuda", "bf16")):
        p = build_local_program("cnn", dt, dev, 256, train, test, optimizer="sgd", lr=0.05,
                                momentum=0.0, seed=3, use_graphs=graphs)
        p.optimizer.sync_hyperparams()
        p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
        tl, ta = p.train_epoch()
        el, ea = p.evaluate()
        res[dev] = (tl.average, el.average, ea.accuracy)
    c, g = res["cpu"], res["cuda"]
    assert abs(g[0] - c[0]) < 0.01 and abs(g[1] - c[1]) < 0.02 and abs(g[2] - c[2]) < 0.02, res
    p = build_local_program("cnn", "bf16", "cuda", 256, train, test, optimizer="sgd", lr=0.05,
                            momentum=0.9, seed=3, use_graphs=graphs)
    p.optimizer.sync_hyperparams()
    hist = []
    for ep in range(3):
        p.set_train_indices(distributed_indices(len(train), 1, 0, ep))
        tl, _ = p.train_epoch()
        el, ea = p.evaluate()
        hist.append((tl.average, el.average, ea.accuracy))
    assert hist[-1][0] < hist[0][0] and hist[-1][2] > 0.8, hist


def test_cnn_large_batch_epoch(gpu):
    """BASELINE config 5 shape: batch 8192 per rank (several images per conv-backward
    workgroup, split-K 1) over an enlarged synthetic set: one whole epoch of 9 full steps
    (one graph of 9 steps, or a full graph and a remainder) and the ragged 1000-image tail, which
    must give the same bits as the same epoch launched eagerly; a second epoch lowers the
    loss."""
    n = 8192 * 9 + 1000
    train = synthetic_split(n, True)
    test = synthetic_split(512, False)
    res = []
    for graphs in (True, False):
        p = build_local_program("cnn", "bf16", "cuda", 8192, train, test, optimizer="sgd",
                                lr=0.01, momentum=0.9, seed=1, use_graphs=graphs)
        p.optimizer.sync_hyperparams()
        p.set_train_indices(distributed_indices(n, 1, 0, 0))
        tl, ta = p.train_epoch()                 # 9 full steps + the 1000-image tail
        assert tl.count == n
        assert torch.isfinite(p.arena.params).all()
        assert int(p.gpu.ctr[0].item()) == 10
        torch.cuda.synchronize()
        res.append((p.arena.params.clone(), p.optimizer.momentum_buffer.clone(), tl.average))
        if graphs:
            # every graph the 9 full steps' plan replays was captured (and so replayed)
            assert {(8192, s) for s, _, _ in p.gpu._plan(8192, 9)} <= {k[:2] for k in p.gpu.graphs}
            keep = p
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert res[0][2] == res[1][2]
    keep.set_train_indices(distributed_indices(n, 1, 0, 1))
    tl2, _ = keep.train_epoch()
    assert tl2.count == n and tl2.average < res[0][2], (res[0][2], tl2.average)


def test_fused_conv_reduce_matches_separate_pass(gpu):
    """world_size 1 folds the conv slab reduction into the optimizer launch and (SGD) the
    fc1-weight update into fc1_bwd (W1^T re-derived by the optimizer, or double-buffered and
    written by fc1_bwd); every combination must give the same bits as
    conv_reduce + optimizer (same fixed summation order, same update op order), incl. a
    tail step and the bf16 weight copies the next step reads."""
    res = []
    for fuse, fuse_fc1, wt2 in ((True, True, True), (True, True, False), (True, False, False),
                                (False, False, False)):
        prog, train, _ = _program(96, lr=0.05, n=96 * 3 + 40, seed=5)
        prog.gpu.fuse_conv_reduce = fuse
        prog.gpu.fuse_fc1 = fuse_fc1
        prog.gpu.wt_double = wt2
        prog.gpu.invalidate_graphs()
        prog.set_train_indices(distributed_indices(len(train), 1, 0, 0))
        prog.train_epoch()
        torch.cuda.synchronize()
        res.append((prog.arena.params.clone(), prog.arena.grads.clone(),
                    prog.optimizer.momentum_buffer.clone(), prog.gpu.wf1.clone(),
                    prog.gpu.current_wf1t().clone()))
    for other in res[1:]:
        for a, b in zip(res[0], other):
            assert torch.equal(a, b)


@pytest.mark.parametrize("model,dtype,opt", [("cnn", "bf16", "sgd"), ("linear", "fp32", "adam")])
def test_epoch_gather_ahead_bit_identical(gpu, model, dtype, opt):
    """Double-buffered epoch buffer: with the next epoch's order handed over early
    (set_train_indices(idx, next_idx)), its gather runs on a side stream beside the current
    epoch's steps and the boundary only resets the counters.  Four epochs (graphs, ragged
    tails, both buffer slots twice, a pinned order from the prefetcher) must give the same
    bits as installing every epoch in stream order, and the device step count must follow."""
    from pytorch_distributed_mnist_amd.data.sampler import EpochIndexPrefetcher
    train = synthetic_split(96 * 5 + 40, True)
    test = synthetic_split(256, False)
    res = []
    for ahead in (False, True):
        p = build_local_program(model, dtype, "cuda", 96, train, test, optimizer=opt, lr=0.02,
                                seed=7, use_graphs=True)
        p.optimizer.sync_hyperparams()
        pf = EpochIndexPrefetcher(len(train), 1, 0, int32=True)
        losses = []
        for ep in range(4):
            nxt = pf.peek(ep + 1) if ahead and ep < 3 else None
            p.set_train_indices(pf.get(ep), nxt)
            tl, _ = p.train_epoch()
            losses.append(tl.average)
            assert int(p.gpu.opt._step_dev.item()) == p.optimizer.step_count
        pf.close()
        torch.cuda.synchronize()
        res.append((p.arena.params.clone(), losses))
    assert torch.equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1]



@pytest.mark.parametrize("n,max_wgs,host", [(1, 0, False), (63, 0, False), (64, 0, True),
                                            (1000 + 37, 0, True), (5000, 7, False)])
def test_gather_epoch_matches_indexing(gpu, n, max_wgs, host):
    """The epoch gather (data.hip: 64 rows per workgroup pass, the pass's indices read once,
    from device memory or -- the training path -- a pinned host buffer) equals plain
    indexing for images and labels, for row counts off the pass size and for a capped grid
    that strides over the rows; the step counters are reset."""
    from pytorch_distributed_mnist_amd.ops import _ext
    C = _ext.require()
    nimg = 3000
    g = torch.Generator().manual_seed(n)
    images = torch.randint(0, 256, (nimg, 784), dtype=torch.uint8, generator=g).cuda()
    labels = torch.randint(0, 10, (nimg,), dtype=torch.int32, generator=g).cuda()
    idx = torch.randint(0, nimg, (n,), dtype=torch.int32, generator=g)
    idx = idx.pin_memory() if host else idx.cuda()
    out_i = torch.full((n + 3, 784), 7, dtype=torch.uint8, device="cuda")
    out_l = torch.full((n + 3,), -1, dtype=torch.int32, device="cuda")
    ctr = torch.full((4,), 9, dtype=torch.int64, device="cuda")
    C.gather_epoch(images, labels, idx, out_i, out_l, ctr, None, 0, max_wgs)
    torch.cuda.synchronize()
    il = idx.long().cuda()
    assert torch.equal(out_i[:n], images[il]) and torch.equal(out_l[:n], labels[il])
    assert bool((out_i[n:] == 7).all()) and bool((out_l[n:] == -1).all())   # nothing past n
    assert int(ctr.abs().sum()) == 0


def test_debug_bounds_checks_report(gpu, capfd):
    """The debug-bounds build (PDM_DEBUG_BOUNDS=1, tools/gpu_r6_debug.sh) reports a violated
    check from the device without trapping: a sampler index past the dataset makes
    gather_epoch print its PDM_CHECK line, clamps the row and goes on.  (Skipped on the
    production build, where the checks are compiled out.)"""
    from pytorch_distributed_mnist_amd.ops import _ext
    C = _ext.require()
    if not C.DEBUG_BOUNDS:
        pytest.skip("production build: PDM_CHECK sites compiled out")
    n = 64
    images = torch.randint(0, 255, (n, 784), dtype=torch.uint8, device="cuda")
    labels = torch.randint(0, 10, (n,), dtype=torch.int32, device="cuda")
    idx = torch.arange(16, dtype=torch.int32, device="cuda")
    idx[3] = n + 5                                    # past the dataset
    out_i = torch.empty(16, 784, dtype=torch.uint8, device="cuda")
    out_l = torch.empty(16, dtype=torch.int32, device="cuda")
    C.gather_epoch(images, labels, idx, out_i, out_l, None, None, 0, 0)
    torch.cuda.synchronize()
    out = capfd.readouterr().out
    assert "PDM_CHECK failed: gather_epoch index" in out, out
    assert torch.equal(out_i[3], images[n - 1])      # clamped to the last row
    assert torch.equal(out_i[4], images[4])
