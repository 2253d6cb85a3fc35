"""CNN fp32 GPU step program (``--arch cnn --dtype fp32``): the reference's precision.

The reference trains in fp32 (``multi_proc_single_gpu.py:185-191``).  Same chain as the bf16
program (``cnn_step.py``) with fp32 activations, gradients and weights
(``csrc/kernels/cnn_f32.hip``).  The conv2 and fc1 GEMMs run as split-bf16 products on the
bf16 MFMA (``conv_x3``, see below) or exactly on the fp32 MFMA (``v_mfma_f32_16x16x4_f32``):

  f32_fwd      gather-free epoch buffer row, normalise, conv1 + ReLU, conv2 + ReLU + maxpool
               -> pool, mask; a1 and the normalised x for the backward
  f32_fc1_fwd  split-K fc1 GEMM -> fp32 partials
  cnn_head     fc1 reduce + bias + ReLU, fc2, CE, head backward (dh in fp32), counters
  f32_fc1_bwd  dW1 tiles | dX tiles | head-slab reduction           -> bucket 0 complete
  f32_conv_bwd conv2 dgrad + relu' + conv1 wgrad, conv2 wgrad       -> conv slabs
  world_size 1: optimizer with the conv slab reduction fused in
  world_size>1: conv_reduce -> all-reduce (both buckets) -> optimizer
"""
from __future__ import annotations

import os

import torch

from .gpu_step import GpuStepBase
from .structure import StepStructure

EVAL_CHUNK = 2048
SPLITK_TRAIN = 32        # fc1 split-K (divides 288: whole 32-float k chunks per split)


def conv_ipb(B: int, x3: bool = False, structure=None) -> int:
    """Work per fp32 conv-backward workgroup (each workgroup stages W2^T once and writes one
    slab for the work it owns).  Exact kernel: images per workgroup, all of one row band
    (StepStructure.f32_ipb / PDM_F32_IPB overrides).  Split-bf16 kernel: (image, row band)
    units per workgroup, taken image-major, so that one round of <= 256 workgroups covers the
    batch (f32_upw / PDM_F32_UPW overrides): half the slabs of 2 rounds of 3-image band groups
    at the same work per CU."""
    st = structure if structure is not None else StepStructure.from_env()
    if x3:
        if st.f32_upw:
            return max(1, int(st.f32_upw))
        return max(1, -(-B * 6 // 256))
    if st.f32_ipb:
        return max(1, int(st.f32_ipb))
    # B = 256, 100-step bench: ipb 1 / 2 / 3 / 6 = 360 / 351 / 340 / 416 us per step
    return max(1, -(-B * 6 // 512))          # <= 2 rounds of 256 workgroups


def splitk_eval(b: int) -> int:
    """Split-K for an eval chunk of b rows: ~256 fc1 workgroups."""
    mt = -(-b // 32)
    for s in (32, 16, 8, 4, 2, 1):
        if mt * s <= 256:
            return s
    return 1


class CnnStepF32(GpuStepBase):
    CONV = ("conv2.weight", "conv2.bias", "conv1.weight", "conv1.bias")

    def __init__(self, prog, use_graphs):
        super().__init__(prog, use_graphs)
        C, dev, B = self.C, self.device, self.bfull
        f32 = torch.float32
        self.ldt = -(-B // 32) * 32
        cap = max(B, EVAL_CHUNK)
        self.pool = torch.empty(cap * 9216, dtype=f32, device=dev)
        self.pmask = torch.empty(B * 9216, dtype=torch.uint8, device=dev)
        # conv1 activations for the backward: fp32, or (split-bf16 mode) the hi / lo bf16
        # planes in the backward's LDS layout -- the same bytes
        self.a1g = torch.empty(B * 676 * 32, dtype=f32, device=dev)
        # split-bf16 mode: the W2^T hi / lo planes the forward writes for the backward, and
        # conv2's weight as hi / lo planes for the forward (the optimizer keeps them current)
        self.w2x = torch.empty(2 * 9 * 32 * 128 // 4, dtype=f32, device=dev)
        self.w2split = torch.empty(2 * 64 * 288, dtype=torch.bfloat16, device=dev)
        self.xng = torch.empty(B * 784, dtype=f32, device=dev)
        self.ylab = torch.empty(cap, dtype=torch.int32, device=dev)
        part_n = max(SPLITK_TRAIN * B, splitk_eval(EVAL_CHUNK) * EVAL_CHUNK) * 128
        self.part = torch.empty(part_n, dtype=f32, device=dev)
        self.dh32 = torch.zeros(self.ldt * 128, dtype=f32, device=dev)
        self.head_slab = torch.empty(C.cnn_head_nblk(self.ldt) * C.CNN_HEAD_SLAB, dtype=f32,
                                     device=dev)
        self.dpool = torch.empty(B * 9216, dtype=f32, device=dev)
        self.conv_slab = torch.empty(max(max(C.f32_conv_bwd_nblk(b, conv_ipb(b, x3, self.structure),
                                                                 x3)
                                             for x3 in (False, True)) for b in range(1, B + 1))
                                     * C.CNN_CONV_SLAB, dtype=f32, device=dev)
        a = self.arena
        self.P = {n: a.param(n) for n in ("conv1.weight", "conv1.bias", "conv2.weight",
                                          "conv2.bias", "fc1.weight", "fc1.bias", "fc2.weight",
                                          "fc2.bias")}
        self.G = {n: a.grad(n) for n in self.P}
        self.fuse_conv_reduce = not self.reducer.active
        # conv2 and fc1 products (the step's FLOPs): "x3" (default) = split-bf16 on the bf16 MFMA
        # (hi.hi + hi.lo + lo.hi, fp32 accumulation; cnn_f32.hip f32x3_*): 4.5e-6 relative
        # error on a conv2 output against fp64, where exact fp32 gives 1.6e-7 and TF32 --
        # cuDNN's default for fp32 convolutions -- 2.9e-4 (tests/test_split_bf16.py); the
        # step's gradients stay within 1e-4 of fp64 (tests/test_gpu_cnn_f32.py).
        # "exact" = the fp32 MFMA (exact fp32 products, 1.9x the step time).
        self.conv_x3 = self.structure.f32_conv == "x3"
        if getattr(self.reducer, "streamed", False):
            # the persistent (streamed) xgmi collective is wired into the bf16 kernels' device
            # hand-off words; the fp32 program uses the transport's per-bucket launches
            self.reducer.streamed = False
        self._fused = {}
        self.refresh_shadows()

    @torch.no_grad()
    def refresh_shadows(self) -> None:
        """Re-derive the split-bf16 copy of conv2's weight (hi = bf16(w), lo = bf16(w - hi))
        from the fp32 master: the optimizer keeps it current after every update, this covers
        any other change (construction, a re-broadcast)."""
        w = self.arena.param("conv2.weight").reshape(-1)
        n = w.numel()
        hi = w.to(torch.bfloat16)
        self.w2split[:n].copy_(hi)
        self.w2split[n:].copy_((w - hi.float()).to(torch.bfloat16))

    def _seg(self, p, slab=None):
        """Optimizer segment of parameter p; conv2's weight also writes its hi / lo copy."""
        off = self.arena.spec.offset(p.name)
        if p.name == "conv2.weight":
            n = p.numel
            return (off, 1, n, self.w2split[:n], None, slab, None, None, None, self.w2split[n:])
        return (off, 1, p.numel, None, None, slab)

    def optimizer_segments(self):
        return [self._seg(p) for p in self.arena.spec.params]

    def invalidate_graphs(self) -> None:
        super().invalidate_graphs()
        self._fused = {}

    def _fused_segments(self, nblk: int):
        """Segments whose conv gradients are the fixed-order sum of `nblk` conv slabs."""
        segs = self._fused.get(nblk)
        if segs is None:
            C, spec = self.C, self.arena.spec
            col = {"conv2.weight": 0, "conv2.bias": C.CNN_CONV_SLAB_DB2,
                   "conv1.weight": C.CNN_CONV_SLAB_DW1, "conv1.bias": C.CNN_CONV_SLAB_DB1}
            slab_segs, plain = [], []
            for p in spec.params:
                if p.name in col:
                    slab_segs.append(self._seg(p, (self.conv_slab, nblk, col[p.name],
                                                   C.CNN_CONV_SLAB)))
                else:
                    plain.append(self._seg(p))
            segs = slab_segs + plain
            self._fused[nblk] = segs
        return segs

    def _train_impl(self, B: int) -> None:
        C, P, G = self.C, self.P, self.G
        ldt = -(-B // 32) * 32
        C.f32_fwd(self.ep_images.view(-1, 784), self.ep_labels, self.ctr[0:1], self.bfull, B,
                  P["conv1.weight"], P["conv1.bias"], P["conv2.weight"], P["conv2.bias"],
                  self.pool, self.pmask, self.a1g, self.xng, self.ylab, spe=self.spe,
                  x3=self.conv_x3, w2x=self.w2x, w2s=self.w2split)
        C.f32_fc1_fwd(self.pool, P["fc1.weight"], self.part, B, SPLITK_TRAIN, x3=self.conv_x3)
        C.cnn_head(self.part, SPLITK_TRAIN, B, P["fc1.bias"], P["fc2.weight"], P["fc2.bias"],
                   self.ylab, True, None, None, ldt, self.head_slab, self.metrics.train_view(),
                   self.ctr[0:1], self.opt._step_dev, None, self.dh32)
        C.f32_fc1_bwd(self.dh32, ldt, self.pool, P["fc1.weight"], B, G["fc1.weight"], self.dpool,
                      self.head_slab, G["fc2.weight"], G["fc2.bias"], G["fc1.bias"],
                      self.metrics.train_view(), x3=self.conv_x3)
        red = self.reducer
        red.bucket_ready(0)          # fc bucket: travels while the conv backward runs
        ipb = conv_ipb(B, self.conv_x3, self.structure)
        C.f32_conv_bwd(self.a1g, self.xng, self.dpool, self.pmask, P["conv2.weight"], B,
                       self.conv_slab, ipb, x3=self.conv_x3, w2x=self.w2x)
        nblk = C.f32_conv_bwd_nblk(B, ipb, self.conv_x3)
        if self.fuse_conv_reduce:
            self.launch_optimizer(self._fused_segments(nblk))
            return
        C.conv_reduce(self.conv_slab, nblk, G["conv2.weight"], G["conv2.bias"],
                      G["conv1.weight"], G["conv1.bias"])
        red.bucket_ready(1)
        red.finalize()
        self.launch_optimizer()

    def evaluate(self) -> None:
        C, P = self.C, self.P
        n = self.test_images.shape[0]
        for s in range(0, n, EVAL_CHUNK):
            b = min(EVAL_CHUNK, n - s)
            se = splitk_eval(b)
            C.f32_fwd(self.test_images[s:s + b], self.test_labels[s:s + b], None, b, b,
                      P["conv1.weight"], P["conv1.bias"], P["conv2.weight"], P["conv2.bias"],
                      self.pool, None, None, None, self.ylab, x3=self.conv_x3,
                      w2s=self.w2split)
            C.f32_fc1_fwd(self.pool, P["fc1.weight"], self.part, b, se, x3=self.conv_x3)
            C.cnn_head(self.part, se, b, P["fc1.bias"], P["fc2.weight"], P["fc2.bias"], self.ylab,
                       False, None, None, 32, None, self.metrics.eval_view(), None, None)
