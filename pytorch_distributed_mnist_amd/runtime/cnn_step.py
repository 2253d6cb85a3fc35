"""CNN (bf16) GPU step program.

Kernel chain of one training step (compute stream; all-reduces on the RCCL stream):

  cnn_fwd      gather+normalise, conv1+ReLU, conv2+ReLU+maxpool  -> pool, mask, x
  fc1_fwd      split-K fc1 GEMM                                  -> fp32 partials
  cnn_head     fc1 reduce+bias+ReLU, fc2, CE, head backward      -> dh, dh^T, head slabs
               (advances the data-step and optimizer-step counters)
  fc1_bwd      dW1 tiles | dX tiles | head-slab reduce           -> bucket 0 (fc) complete
  cnn_bwd      a1 recompute, conv2 wgrad | conv2 dgrad + conv1 wgrad -> conv slabs

  world_size 1:
  optim        conv slab reduction fused in; SGD/Adam over the arena + bf16 weight copies
  world_size > 1:
  conv_reduce  fixed-order slab sum                              -> bucket 1 (conv) complete
  [all-reduce bucket 1, then bucket 0]
  optim(conv)  after bucket 1
  optim(fc)    after bucket 0 -- inside a multi-step graph deferred to after the next
               step's cnn_fwd, which overlaps the 4.7 MB fc all-reduce

Evaluation runs cnn_fwd (no activations kept) -> fc1_fwd -> cnn_head over the
whole test set in chunks of EVAL_CHUNK images.
"""
from __future__ import annotations

import os

import torch

from .gpu_step import GpuStepBase

EVAL_CHUNK = 2048


def frag_major(w: torch.Tensor) -> torch.Tensor:
    """[M][K] -> the MFMA-fragment-major layout (csrc/kernels.h frag_pos): the 16 x 32
    fragment (m // 16, k // 32) is one 512-element block in which lane
    ((k // 8) % 4) * 16 + m % 16 holds its 8 consecutive k.  Flat 1-D result."""
    m, k = w.shape
    t = w.reshape(m // 16, 16, k // 32, 4, 8)                  # [mb][i][kb][g][j]
    return t.permute(0, 2, 3, 1, 4).contiguous().reshape(-1)   # [mb][kb][g][i][j]


def a1_swizzled(a1: torch.Tensor) -> torch.Tensor:
    """[B, 26*26, 32] conv1 activations -> the swizzled a1 image cnn_fwd_band writes and
    cnn_bwd_band reads (cnn_common.h a1_off: the 16-B chunk c // 8 of pixel (y, x) stored at
    chunk (c // 8) ^ (x & 3)).  Flat 1-D result."""
    b = a1.shape[0]
    t = a1.reshape(b, 26, 26, 4, 8)
    x = torch.arange(26).view(1, 1, 26, 1)
    src = torch.arange(4).view(1, 1, 1, 4) ^ (x & 3)           # stored chunk j holds chunk j ^ (x & 3)
    out = torch.gather(t, 3, src.expand(b, 26, 26, 4).unsqueeze(-1).expand(b, 26, 26, 4, 8))
    return out.reshape(-1).contiguous()


def frag_major_t(w: torch.Tensor) -> torch.Tensor:
    """The transpose of [rows][cols] in the fragment-major layout (kernels.h shadow_t_pos)."""
    return frag_major(w.t())


FC1_BIG_B = 2048        # csrc/kernels.h: fc1_fwd's 128-row blocks from this batch on


def choose_splitk(B: int, cap: int = 32, target_blocks: int = 256) -> int:
    """Split-K factor for fc1_fwd giving ~target_blocks workgroups of (m-tile, split): 32-row
    m-tiles, 128-row ones from B = FC1_BIG_B on; a divisor of 32 (every split holds whole
    9-step load batches of the 288 K-steps) or 48 / 96 (3-step batches)."""
    mtiles = (B + 31) // 32 if B < FC1_BIG_B else (B + 127) // 128
    best = 1
    for s in (1, 2, 4, 8, 16, 32, 48, 96):
        if s <= cap and mtiles * s <= target_blocks:
            best = s
    return best


def choose_ipb(B: int, cus: int = 256) -> int:
    """Images per cnn_bwd workgroup: one workgroup per CU once B exceeds the CU count."""
    return max(1, -(-B // cus))


BAND_CHOICES = (6, 3, 2)


def choose_bands(B: int, cus: int = 256, forced=None) -> int:
    """Row bands per image in the conv backward: small batches (the reference's per-rank
    split of the node batch, 256 / world_size) spread each image over up to 6 workgroups
    (cnn_bwd_band.hip) so that B * bands fills at most one round of the CUs; 1 = cnn_bwd
    (`forced`, StepStructure.bands / PDM_BANDS, overrides: 1 disables the split)."""
    if forced is not None:
        return int(forced)
    for s in BAND_CHOICES:
        if B * s <= cus:
            return s
    return 1


def conv_blocks(C, B: int, bands_forced=None) -> int:
    """Conv-backward workgroups (= gradient slabs) for per-rank batch B."""
    bands = choose_bands(B, forced=bands_forced)
    return C.cnn_bwd_nblk(B, choose_ipb(B) if bands == 1 else 1, bands)


class CnnStep(GpuStepBase):
    def __init__(self, prog, use_graphs):
        super().__init__(prog, use_graphs)
        C, dev, B = self.C, self.device, self.bfull
        a = self.arena
        st = self.structure
        bf16 = torch.bfloat16
        self.ldt = -(-B // 32) * 32
        cap = max(B, EVAL_CHUNK)
        # activations / workspaces (sized once; graphs capture their addresses)
        self.pool = torch.empty(cap * 9216, dtype=bf16, device=dev)
        self.pmask = torch.empty(cap * 9216, dtype=torch.uint8, device=dev)
        self.xg = torch.empty(B * 784, dtype=torch.uint8, device=dev)
        self.ylab = torch.empty(cap, dtype=torch.int32, device=dev)
        self.splitk_train = choose_splitk(B, cap=st.splitk_cap)
        self.splitk_eval = choose_splitk(min(cap, EVAL_CHUNK))
        part_n = max(self.splitk_train * B, self.splitk_eval * EVAL_CHUNK) * 128
        self.part = torch.empty(part_n, dtype=torch.float32, device=dev)
        self.dh = torch.zeros(self.ldt * 128, dtype=bf16, device=dev)
        self.dht = torch.zeros(self.ldt * 128, dtype=bf16, device=dev)
        self.head_slab = torch.empty(C.cnn_head_nblk(self.ldt) * C.CNN_HEAD_SLAB, dtype=torch.float32,
                                     device=dev)
        self.dpool = torch.empty(B * 9216, dtype=bf16, device=dev)
        self.ipb = choose_ipb(B)
        # row-band steps (small batches): the forward hands a1 and the normalised x to the
        # backward (cnn_fwd_band -> cnn_bwd_band) instead of the backward recomputing conv1
        nband = max(b for b in range(1, B + 1) if self.bands(b) > 1) if \
            any(self.bands(b) > 1 for b in range(1, B + 1)) else 0
        self.a1g = torch.empty(max(nband, 1) * 676 * 32, dtype=bf16, device=dev)
        self.xng = torch.empty(max(nband, 1) * 784, dtype=bf16, device=dev)
        # slabs for every batch size this step runs (the ragged tail may split into more
        # bands than the full batch)
        self.conv_nblk = max(conv_blocks(C, b, st.bands) for b in range(1, B + 1))
        self.conv_slab = torch.empty(self.conv_nblk * C.CNN_CONV_SLAB, dtype=torch.float32,
                                     device=dev)
        # bf16 compute copies of the weights (kept current by the optimizer kernel)
        self.wf1 = torch.empty(128 * 9216, dtype=bf16, device=dev)
        # W1^T: two copies (double buffer of the fused world-size-1 fc1 update, see below:
        # the step of phase p reads copy p and writes copy 1 - p); every other path reads and
        # writes the first
        self.wf1t2 = torch.empty(2, 9216 * 128, dtype=bf16, device=dev)
        self.wf1t = self.wf1t2[0]
        self.w2 = torch.empty(64 * 288, dtype=bf16, device=dev)
        self.w2t = torch.empty(288 * 64, dtype=bf16, device=dev)
        # parameter / gradient views (kernel layouts)
        p, g = a.param, a.grad
        self.P = {n: p(n) for n in ("conv1.weight", "conv1.bias", "conv2.bias", "fc1.bias",
                                    "fc2.weight", "fc2.bias")}
        self.G = {n: g(n) for n in ("conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias",
                                    "fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias")}
        # world_size 1 (no all-reduce between backward and update): the conv gradient
        # reduction is fused into the optimizer launch (PDM_FUSE_CONV_REDUCE=0 disables)
        self.fuse_conv_reduce = not self.reducer.active and st.fuse_conv_reduce
        # world_size 1, SGD-momentum: the fc1-weight update runs in fc1_bwd's weight-gradient
        # tiles (the gradient is still in registers; those tiles have slack next to the dX
        # tiles of the same launch); the optimizer launch then only re-derives the transposed
        # bf16 copy W1^T from the updated W1 (PDM_FUSE_FC1=0 disables)
        # (at the batches where fc1_carry_local hands it to the next forward launch instead,
        # _local_carry, fc1_bwd stores the gradient and does not update)
        self.fuse_fc1 = self.fuse_conv_reduce and self.opt.kind == "sgd" and st.fuse_fc1
        # ... and writes W1^T too, double-buffered by step parity (this step's dX tiles read
        # one half while its weight tiles write the other), so the optimizer launch skips fc1
        # entirely (PDM_FC1_WT2=0: the optimizer re-derives W1^T instead)
        self.wt_double = st.fc1_wt_double
        # the fused fc1 update consumes the fc1-weight gradient in registers; it is stored to
        # the gradient arena only when something will read it (tests comparing gradients set
        # keep_grads; PDM_KEEP_GRADS=1 forces it): 4.7 MB of writes per step otherwise
        self.keep_grads = st.keep_grads
        self.phase_period = 2 if self._wt_double_on() else 1
        self._fused = {}
        # RCCL data plane: where the fc bucket's all-reduce and update go (RCCL_MODES;
        # bench.py calibrates every mode on the real step, PDM_RCCL_MODE picks one):
        #  carry   defer the fc-bucket update past the next step's cnn_fwd, so the 4.7 MB
        #          all-reduce overlaps that forward (it only needs the conv weights)
        #  nocarry both buckets in one grouped RCCL launch, one optimizer launch (fewer
        #          launches when the transfer is short)
        #  side    the fc update on a side stream as soon as its all-reduce lands, beside the
        #          conv update and the next cnn_fwd (small per-rank batches leave CUs idle)
        #  early   the fc all-reduce issued right after fc1_bwd, during the conv backward, as
        #          DDP's Reducer does during loss.backward() (multi_proc_single_gpu.py:91); at
        #          small batches cnn_bwd_band leaves CUs free for RCCL's kernel (B = 32: 192
        #          workgroups on 256 CUs), at B = 256 the collective waits for cnn_bwd
        # world_size > 1: optimizer-state sharding of the fc1 weight (set_shard_fc): its
        # gradient is reduce-scattered instead of all-reduced, each rank updates its
        # 128 / world_size rows (fp32 master, momentum, bf16 W1 rows) and the bf16 W1 rows are
        # all-gathered; W1^T is re-derived locally.  Same arithmetic per element as the
        # replicated update; the fp32 rows a rank does not own go stale until sync_master()
        # (checkpoints, evaluation of the fp32 weights, parameter checks)
        # xgmi streamed: the conv bucket all-reduced inside the optimizer launch
        # (StepStructure.xgmi_exchange; bench.py's 'xgmi-noxchg' candidate turns it off)
        self.xgmi_exchange = st.xgmi_exchange
        self.shard_fc = False
        self._shard_rows = None
        self._side = None
        self._side_ev = None
        self.set_rccl_mode(st.rccl_mode, invalidate=False)
        self.refresh_shadows()
        self._poison_unkept_grads()

    RCCL_MODES = ("carry", "nocarry", "side", "early")

    def bands(self, B: int) -> int:
        """Row bands per image of the conv backward at batch B (choose_bands)."""
        return choose_bands(B, forced=self.structure.bands)

    def set_rccl_mode(self, mode: str, invalidate: bool = True) -> None:
        """Step structure of the fc bucket on the RCCL data plane (see __init__).  'zero' is
        carry with the fc1 update sharded over the ranks (set_shard_fc); with no reduction
        (world size 1) the structure is moot and 'zero' runs the local step."""
        shard = mode == "zero"
        if shard:
            mode = "carry"
        if mode not in self.RCCL_MODES:
            raise ValueError(f"RCCL step mode {mode!r}: choose from {self.RCCL_MODES + ('zero',)}")
        self.fc_carry = mode in ("carry", "side")
        self.fc_side = mode == "side"
        self.fc_early = mode == "early"
        if shard and self.reducer.active:
            why = self.shard_unsupported_reason()
            if why is not None:
                raise ValueError(f"RCCL step mode 'zero' (sharded fc1 update): {why}")
            self.set_shard_fc(True)
        if invalidate:
            self.invalidate_graphs()

    # -- fc1 optimizer-state sharding --------------------------------------------------------
    def shard_supported(self, reducer=None) -> bool:
        return self.shard_unsupported_reason(reducer) is None

    def shard_world_size(self, reducer=None) -> int:
        """The world size the fc1 shard is sized for: the communicator's, or with a 1-rank
        communicator the emulated one (StepStructure.emulate_ws, pricing runs)."""
        red = reducer or self.reducer
        ws = red.comm.world_size
        emu = self.structure.emulate_ws
        return int(emu) if (emu and ws == 1) else ws

    def shard_unsupported_reason(self, reducer=None):
        """None when the fc1 update can be sharded over `reducer`'s ranks, else why not."""
        red = reducer or self.reducer
        ws = self.shard_world_size(red)
        if not red.active:
            return "no gradient reduction at world size 1"
        if not red.can_shard:
            return f"the {red.kind} gradient transport has no reduce-scatter"
        if 128 % ws or (128 // ws) % 16:
            return (f"world size {ws} does not split fc1's 128 rows into shards of a multiple "
                    "of 16 rows")
        return None

    def set_shard_fc(self, on: bool) -> None:
        """Switch the fc1-weight optimizer-state sharding on or off (graphs are re-captured)."""
        if bool(on) == self.shard_fc:
            return
        if on:
            if not self.shard_supported():
                raise RuntimeError("fc1 sharding needs an RCCL or gloo data plane and a world "
                                   "size that splits 128 rows into multiples of 16")
            ws, r = self.shard_world_size(), self.reducer.comm.rank
            rows = 128 // ws
            self.reducer.set_shard(0, self.arena.spec.offset("fc1.weight"), rows * 9216)
            self._shard_rows = (r * rows, rows)
            self.shard_fc = True
        else:
            self.sync_master()
            self.reducer.clear_shard()
            self.shard_fc = False
            self._shard_rows = None
        self.invalidate_graphs()

    @torch.no_grad()
    def sync_master(self) -> None:
        """Sharded mode: all-gather the fp32 fc1 rows and their optimizer state, so every
        rank holds the full, current master weights (collective: every rank calls it)."""
        if not self.shard_fc:
            return
        off, n = self.arena.spec.offset("fc1.weight"), 128 * 9216
        for buf in (self.arena.params, *self.opt.state_buffers().values()):
            self.reducer.gather(buf[off:off + n])
        self.reducer.wait_gather()

    def _shard_segments(self):
        """Optimizer segments of a sharded step: every parameter but fc1.weight whole, and this
        rank's rows of fc1.weight (fp32 update + its rows of the fragment-major bf16 W1, which
        start on a 16-row fragment boundary); plus the transpose-only W1 -> W1^T segment run
        after the all-gather."""
        if getattr(self, "_ssegs", None) is None:
            off1 = self.arena.spec.offset("fc1.weight")
            r0, rows = self._shard_rows
            segs = []
            for sg in self.optimizer_segments():
                if sg[0] == off1:
                    segs.append((off1 + r0 * 9216, rows, 9216,
                                 self.wf1[r0 * 9216:(r0 + rows) * 9216], None, None, False, False,
                                 True))
                else:
                    segs.append(sg)
            tseg = [(off1, 128, 9216, self.wf1, self.wf1t, None, True, True, True)]
            self._ssegs = (segs, tseg)
        return self._ssegs

    @torch.no_grad()
    def refresh_shadows(self) -> None:
        """Re-derive the bf16 weight copies from the fp32 master weights."""
        self.sync_master()
        w1 = self.arena.param("fc1.weight").reshape(128, 9216)
        self.wf1.copy_(frag_major(w1.to(torch.bfloat16)))
        wt = frag_major_t(w1.to(torch.bfloat16))
        self.wf1t2[0].copy_(wt)
        self.wf1t2[1].copy_(wt)
        w2 = self.arena.param("conv2.weight").reshape(64, 288)
        self.w2.copy_(frag_major(w2.to(torch.bfloat16)))
        self.w2t.copy_(w2.t().contiguous().reshape(-1).to(torch.bfloat16))

    def optimizer_segments(self):
        spec = self.arena.spec
        segs = []
        for p in spec.params:
            off = spec.offset(p.name)
            if p.name == "fc1.weight":
                # W1 and W1^T in the MFMA-fragment-major layout fc1_fwd / fc1_bwd's dX tiles
                # read (kernels.h frag_pos)
                segs.append((off, 128, 9216, self.wf1, self.wf1t, None, False, True, True))
            elif p.name == "conv2.weight":
                # W2 fragment-major (cnn_fwd's conv2 B operand), W2^T row-major (cnn_bwd's
                # LDS image)
                segs.append((off, 64, 288, self.w2, self.w2t, None, False, False, True))
            else:
                segs.append((off, 1, p.numel, None, None))
        return segs

    def _bucket_segments(self):
        """Optimizer segments of bucket 0 (fc2 + fc1) and bucket 1 (conv2 + conv1)."""
        if getattr(self, "_bsegs", None) is None:
            if self._opt_segments is None:
                self._opt_segments = self.optimizer_segments()
            (s0, e0), _ = self.arena.spec.bucket_bounds()
            b0 = [sg for sg in self._opt_segments if s0 <= sg[0] < e0]
            b1 = [sg for sg in self._opt_segments if not (s0 <= sg[0] < e0)]
            self._bsegs = (b0, b1)
        return self._bsegs

    def _fused_segments(self, nblk: int, skip_fc1: bool = False):
        """Optimizer segments whose conv gradients are summed from `nblk` cnn_bwd slabs
        (skip_fc1: without the fc1 weight, whose update the next forward launch carries)."""
        segs = self._fused.get((nblk, skip_fc1))
        if segs is None:
            if self._opt_segments is None:
                self._opt_segments = self.optimizer_segments()
            C = self.C
            col = {"conv2.weight": 0, "conv2.bias": C.CNN_CONV_SLAB_DB2,
                   "conv1.weight": C.CNN_CONV_SLAB_DW1, "conv1.bias": C.CNN_CONV_SLAB_DB1}
            by_off = {self.arena.spec.offset(n): n for n in col}
            slab_segs, plain = [], []
            fc1_off = self.arena.spec.offset("fc1.weight")
            for sg in self._opt_segments:
                name = by_off.get(sg[0])
                if name is None and skip_fc1 and sg[0] == fc1_off:
                    continue
                if name is None and self.fuse_fc1 and sg[0] == fc1_off:
                    # updated by fc1_bwd: only W1^T = transpose(W1) is left to write, unless
                    # fc1_bwd writes it too (double-buffered)
                    if not self.wt_double:
                        plain.append((sg[0], sg[1], sg[2], sg[3], sg[4], None, True, True, True))
                elif name is None:
                    plain.append(sg)
                else:
                    sg = tuple(sg) + (None,) * (9 - len(sg))
                    slab_segs.append(sg[:5] + ((self.conv_slab, nblk, col[name], C.CNN_CONV_SLAB),) +
                                     sg[6:])
            # slab segments first: their workgroups (a 256-deep reduction each) are
            # dispatched before the streaming fc updates instead of forming the tail
            segs = slab_segs + plain
            self._fused[(nblk, skip_fc1)] = segs
        return segs

    def _segments_without_fc1(self):
        if self._opt_segments is None:
            self._opt_segments = self.optimizer_segments()
        off = self.arena.spec.offset("fc1.weight")
        return [sg for sg in self._opt_segments if sg[0] != off]

    def _local_carry(self, B: int) -> bool:
        """World size 1, SGD, fc1_carry_local: the fc1 update of a batch-B step runs in the
        next forward launch instead of fc1_bwd's weight tiles -- at the batches whose forward
        is the one-image cnn_fwd (its grid leaves room for the update's workgroups: B = 256
        53.2 vs 53.9 us per step); the band forward of B <= 128 pays more for them than fc1_bwd
        saves (B = 32: 38.6 vs 37.3; profiles/r5/fc1_carry_local/).  The last step of a
        train_steps call keeps the fused update."""
        st = self.structure
        return (not self.reducer.active and self.fuse_fc1 and st.fc1_carry_fwd and
                st.fc1_carry_local and self.bands(B) == 1)

    def _fwd_carry_on(self, B: int) -> bool:
        """SGD: step k's fc1 update runs in step k+1's forward launch (kernels/fc_carry.h) --
        at world size > 1 on the xgmi in-launch-exchange step and the RCCL nocarry step; at
        world size 1 where _local_carry says so."""
        red = self.reducer
        if not red.active:
            return self._local_carry(B)
        if not (self.structure.fc1_carry_fwd and self.opt.kind == "sgd") or self.shard_fc:
            return False
        if self._xchg():
            return True
        return (getattr(red, "kind", None) == "rccl" and getattr(red, "_native", None) is not None
                and not self.fc_carry and not self.fc_early)

    def _fc_carry(self):
        """The carried fc1 update (cnn_fwd fc_carry): the fused update's arguments, reading the
        (all-reduced) gradient, writing the W1^T copy this step's fc1_bwd reads."""
        u = self._fc_update()
        return u[:16] + (self.current_wf1t(),)

    def _fc_carry_wait(self):
        """xgmi streamed: the carried update waits for the channel of the fc1 weight, which the
        optimizer no longer waits for (its own channel: models/specs.py channel_bounds)."""
        red = self.reducer
        if not red.streamed:
            return None
        ch = red.channel_of(self.arena.spec.offset("fc1.weight"))
        return (red.sync, ch, int(red._native.blocks(ch)), float(red.timeout_s))

    def fwd_outputs(self, B: int):
        """cnn_fwd's training outputs for per-rank batch B: (xg, ylab, bands, a1g, xng) -- the
        band backward reads a1 + normalised x, the one-image backward the uint8 image."""
        fb = self.bands(B)
        if fb > 1:
            return None, self.ylab, fb, self.a1g, self.xng
        return self.xg, self.ylab, fb, None, None

    def collective_channels(self):
        return 1 if self._xchg() else None     # the conv bucket is exchanged by the optimizer

    def collective_wide(self, B: int) -> bool:
        # the 8-loads-per-lane collective (128 registers) fits beside the band backward of
        # 4- and 8-row bands only (6 / 3 bands per image), not beside 12-row bands or cnn_bwd
        return self.bands(B) >= 3

    def carries_across_graphs(self, B: int) -> bool:
        return self._fwd_carry_on(B) and self.structure.fc1_carry_graphs

    def _train_seq(self, B: int, n: int, collective: bool = True, cin: bool = False,
                   cout: bool = False) -> None:
        # multi-GPU: each step leaves its fc-bucket update to the next one, whose cnn_fwd
        # runs while the fc gradients are still being all-reduced; the last step of the
        # sequence (a graph must rejoin the comm stream) does not carry
        rccl = self.reducer.active and getattr(self.reducer, "kind", None) == "rccl"
        # sharded: the W1 all-gather and the W1^T transpose are carried past the next cnn_fwd
        carry = rccl and (self.shard_fc or (self.fc_carry and not self.fc_early))
        # SGD (world size > 1; world size 1 at B > 128): each step's fc1 update runs in the
        # next step's forward launch
        fwd = self._fwd_carry_on(B)
        streamed = self.reducer.streamed and collective
        if streamed:
            # one persistent xgmi collective for the n steps (the fc bucket only when the
            # optimizer exchanges the conv bucket itself)
            self.reducer.begin(n, self.collective_channels(), self.collective_wide(B))
        for i in range(n):
            # the fc1 update is carried across graph replays of one train_steps call too
            # (cin / cout); only the call's last step updates in its own optimizer
            self._train_impl(B, carry_in=carry and i > 0, carry_out=carry and i < n - 1,
                             fwd_in=fwd and (i > 0 or cin), fwd_out=fwd and (i < n - 1 or cout))
            self.phase = (self.phase + 1) % self.phase_period
        if streamed:
            self.reducer.end()

    def _train_impl(self, B: int, carry_in: bool = False, carry_out: bool = False,
                    fwd_in: bool = False, fwd_out: bool = False) -> None:
        """One training step (kernel chain in the module docstring).

        carry_in: the previous step's fc-bucket optimizer update is still pending; it runs
        after this step's cnn_fwd (which only needs the conv weights), so the previous fc
        all-reduce overlaps cnn_fwd.  carry_out: leave this step's fc update to the next step.
        fwd_in / fwd_out: the same for the fc1 weight alone, whose pending update runs INSIDE
        this step's forward launch (_fwd_carry_on).
        """
        C, P, G = self.C, self.P, self.G
        red = self.reducer
        xs = red.sync if red.streamed else None       # xgmi streamed-mode sync words
        ldt = -(-B // 32) * 32
        S = self.splitk_train
        bands = self.bands(B)
        C.cnn_fwd(self.ep_images.view(-1, 784), self.ep_labels, None, self.ctr[0:1], self.bfull, B,
                  P["conv1.weight"], P["conv1.bias"], self.w2, P["conv2.bias"], self.pool,
                  self.pmask, *self.fwd_outputs(B), spe=self.spe,
                  fc_carry=self._fc_carry() if fwd_in else None,
                  fc_carry_wait=self._fc_carry_wait() if fwd_in else None)
        if carry_in and self.shard_fc:
            self.reducer.wait_gather()                # this step's W1 rows from every rank
            self.launch_optimizer(self._shard_segments()[1])
        elif carry_in and self.fc_side:
            torch.cuda.current_stream(self.device).wait_event(self._side_ev)
        elif carry_in:
            self.reducer.wait_bucket(0)
            self.launch_optimizer(self._bucket_segments()[0])
        C.fc1_fwd(self.pool, self.wf1, self.part, B, S)
        C.cnn_head(self.part, S, B, P["fc1.bias"], P["fc2.weight"], P["fc2.bias"], self.ylab,
                   True, self.dh, self.dht, ldt, self.head_slab, self.metrics.train_view(),
                   self.ctr[0:1], self.opt._step_dev, xs)
        C.fc1_bwd(self.dh, self.dht, ldt, self.pool, self.current_wf1t(), B, G["fc1.weight"], self.dpool,
                  self.head_slab, G["fc2.weight"], G["fc2.bias"], G["fc1.bias"],
                  self.metrics.train_view(),
                  # (world size 1: fused unless the next forward carries it, _local_carry;
                  # when this program's full batches carry it, and so store the fc1 gradient,
                  # every fused step -- a call's last, the ragged tail -- stores it too, so the
                  # gradient arena never holds an older step's gradient)
                  self._fc_update(store_grad=self._local_carry(self.bfull))
                  if self.fuse_fc1 and not fwd_out else None)
        xgmi = getattr(self.reducer, "kind", None) == "xgmi"
        rccl_early = (self.fc_early and not xgmi and red.active and
                      getattr(red, "_native", None) is not None)
        early = xgmi and not red.streamed and self.structure.xgmi_early
        if rccl_early:
            # bucket 0 (fc, 4.7 MB) is complete: its all-reduce goes out now, on the
            # high-priority comm stream, beside the conv backward
            self.reducer.bucket_ready(0)
        if early:
            # bucket 0 (fc, 4.7 MB) is complete: its xGMI all-reduce kernel is small enough
            # to be co-resident with cnn_bwd, so it travels during the conv backward
            self.reducer.bucket_ready(0)
        ipb = choose_ipb(B) if bands == 1 else 1
        nblk = C.cnn_bwd_nblk(B, ipb, bands)
        # streamed xgmi: cnn_bwd's first workgroup publishes the fc bucket to the
        # persistent collective, which then reduces it beside cnn_bwd
        C.cnn_bwd(self.xg, P["conv1.weight"], P["conv1.bias"], self.dpool, self.pmask, self.w2t, B,
                  ipb, self.conv_slab, xs, bands, self.a1g, self.xng)
        if self.fuse_conv_reduce:
            # world_size 1: no all-reduce, the conv slab reduction runs inside the update
            self.launch_optimizer(self._fused_segments(nblk, skip_fc1=fwd_out))
            return
        if self._xchg():
            # xgmi streamed: the optimizer reduces the conv slabs AND all-reduces the conv
            # bucket in-launch (each slab workgroup exchanges its 64 sums with its peers); its
            # fc workgroups take bucket 0 from the persistent collective, which reduced it
            # beside cnn_bwd.  No conv_reduce launch, no wait launch.
            self.launch_optimizer(self._fused_segments(nblk, skip_fc1=fwd_out), exchange=True)
            return
        C.conv_reduce(self.conv_slab, nblk, G["conv2.weight"], G["conv2.bias"],
                      G["conv1.weight"], G["conv1.bias"])
        if self.shard_fc:
            # fc bucket: reduce-scatter of the fc1 weight + all-reduce of fc2 / fc1 bias (one
            # RCCL group, already on the wire if rccl_early), conv bucket all-reduced; one
            # update of every parameter but the other ranks' fc1 rows; W1 rows all-gathered
            if not rccl_early:
                self.reducer.bucket_ready(0)
            self.reducer.bucket_ready(1)
            self.reducer.finalize()
            segs, tseg = self._shard_segments()
            self.launch_optimizer(segs)
            self.reducer.gather(self.wf1)
            if not carry_out:
                self.reducer.wait_gather()
                self.launch_optimizer(tseg)
            return
        if xgmi and red.streamed:
            # the optimizer publishes the conv bucket; its fc workgroups wait for bucket 0
            # (long reduced by now), its conv workgroups for bucket 1
            self.launch_optimizer(signal_ch=red.channels_of(1)[0])
            return
        if xgmi:
            if not early:
                self.reducer.bucket_ready(0)
            # bucket 1 (conv, 75 KB, one-shot) queues behind bucket 0 on the xgmi stream;
            # one optimizer launch over the reduced arena once both have landed
            self.reducer.bucket_ready(1)
            self.reducer.finalize()
            self.launch_optimizer()
            return
        if getattr(self.reducer, "_native", None) is None:
            # gloo data plane (rehearsal / CPU-staged): plain bucket order, one update
            self.reducer.bucket_ready(0)
            self.reducer.bucket_ready(1)
            self.reducer.finalize()
            self.launch_optimizer()
            return
        # RCCL.  Both buckets are reduced after conv_reduce: RCCL's all-reduce kernel cannot
        # be co-resident with cnn_bwd (it needs 19.7 KB LDS + ~280 registers per lane per the
        # gfx950 code-object metadata of torch's librccl; cnn_bwd leaves 5.6 KB LDS and 48
        # registers per SIMD lane on every CU), so issuing bucket 0 earlier would only wait
        # for cnn_bwd or push part of it into a second round.  The small conv bucket goes
        # first (the next forward needs it); the 4.7 MB fc bucket keeps reducing while the
        # conv update and the next step's cnn_fwd run.
        if rccl_early:
            # the fc bucket is already on the wire; the conv bucket queues behind it on the
            # comm stream; one optimizer launch once both have landed
            self.reducer.bucket_ready(1)
            self.reducer.finalize()
            self.launch_optimizer()
            return
        if not self.fc_carry:
            # one grouped RCCL launch for both buckets, one optimizer launch for everything
            # (but the fc1 weight when the next forward carries its update)
            self.reducer.all_ready()
            self.reducer.finalize()
            self.launch_optimizer(self._segments_without_fc1() if fwd_out else None)
            return
        b0, b1 = self._bucket_segments()
        self.reducer.bucket_ready(1)
        self.reducer.bucket_ready(0)
        if self.fc_side:
            if self._side is None:
                self._side = torch.cuda.Stream(self.device)
                self._side_ev = torch.cuda.Event()
            with torch.cuda.stream(self._side):
                self.reducer.wait_bucket(0)          # the side stream waits for bucket 0
                self.launch_optimizer(b0)
                self._side_ev.record(self._side)
            self.reducer.wait_bucket(1)
            self.launch_optimizer(b1)
            if not carry_out:                        # a graph ends with every stream joined
                torch.cuda.current_stream(self.device).wait_event(self._side_ev)
            return
        self.reducer.wait_bucket(1)
        self.launch_optimizer(b1)
        if not carry_out:
            self.reducer.wait_bucket(0)
            self.launch_optimizer(b0)

    def _xchg(self) -> bool:
        """xgmi streamed mode with the conv bucket exchanged inside the optimizer launch (a
        one-shot conv channel only: PDM_XGMI_MODE=two falls back to conv_reduce + the
        persistent collective)."""
        red = self.reducer
        return (red.active and getattr(red, "kind", None) == "xgmi" and red.streamed and
                self.xgmi_exchange and red.exchange_ok(1))

    def _fc_update(self, store_grad: bool = False):
        """fc1_bwd's fused fc1-weight SGD update (bind.cpp make_fc_update); store_grad: store
        the gradient it consumes even without keep_grads."""
        o = self.opt
        g = o.param_groups[0]
        off = self.arena.spec.offset("fc1.weight")
        n = 128 * 9216
        return (self.C.OPT_SGD, self.arena.params[off:off + n], self.reducer.out_grads[off:off + n],
                o.momentum_buffer[off:off + n], None, self.wf1, o._lr_dev, o._step_dev, 0.0, 0.0,
                0.0, float(g["weight_decay"]), float(g["momentum"]), float(g["dampening"]),
                bool(g["nesterov"]), float(self.reducer.grad_scale),
                self.wf1t2[1 - self.phase] if self._wt_double_on() else None,
                self.keep_grads or store_grad)

    def _wt_double_on(self) -> bool:
        return self.fuse_fc1 and self.fuse_conv_reduce and self.wt_double

    def current_wf1t(self) -> torch.Tensor:
        """The W1^T copy the next fc1_bwd reads."""
        return self.wf1t2[self.phase] if self._wt_double_on() else self.wf1t

    def invalidate_graphs(self) -> None:
        super().invalidate_graphs()
        self._bsegs = None
        self._ssegs = None
        self._fused = {}
        period = 2 if self._wt_double_on() else 1
        if self.phase != self.phase % period:
            # leaving double-buffer mode at phase 1: the newest W1^T is in copy 1, and every
            # single-buffer path reads copy 0
            self.wf1t2[0].copy_(self.wf1t2[self.phase])
        self.phase_period = period
        self.phase %= period
        self._poison_unkept_grads()

    def _poison_unkept_grads(self) -> None:
        """With the fused fc1 update and keep_grads off, fc1_bwd consumes the fc1-weight
        gradient in registers and never stores it (but at the batches where the update is
        carried, _local_carry): fill that slice of the gradient arena with NaN so a later
        reader (norm logging, clipping, dumps) fails visibly instead of seeing a stale step's
        values."""
        if self.fuse_fc1 and self.fuse_conv_reduce and not self.keep_grads:
            self.G["fc1.weight"].fill_(float("nan"))

    def evaluate(self) -> None:
        C, P = self.C, self.P
        n = self.test_images.shape[0]
        S = self.splitk_eval
        for s in range(0, n, EVAL_CHUNK):
            b = min(EVAL_CHUNK, n - s)
            C.cnn_fwd(self.test_images[s:s + b], self.test_labels[s:s + b], None, None, b, b,
                      P["conv1.weight"], P["conv1.bias"], self.w2, P["conv2.bias"], self.pool,
                      self.pmask, None, self.ylab)
            C.fc1_fwd(self.pool, self.wf1, self.part, b, S)
            C.cnn_head(self.part, S, b, P["fc1.bias"], P["fc2.weight"], P["fc2.bias"], self.ylab,
                       False, None, None, 32, None, self.metrics.eval_view(), None, None)
