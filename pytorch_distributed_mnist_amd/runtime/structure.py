"""The step structure: every choice of HOW a training step is laid out that does not change
WHAT it computes (kernel fusions, band splits, split-K, graph length, where the gradient
buckets' collectives and updates go).

The defaults are the production configuration; ``bench.py`` calibrates the RCCL structure
on the node.  The ``PDM_*`` structure knobs (knobs.py) are read ONCE, by
``StepStructure.from_env()``, when a program is built; the step classes only read this
object, so no production path consults the environment while it builds or captures a step.
"""
from __future__ import annotations

from dataclasses import dataclass, replace
from typing import Optional

from .. import knobs

RCCL_MODES = ("carry", "nocarry", "side", "early", "zero")


@dataclass(frozen=True)
class StepStructure:
    # RCCL data plane: placement of the fc bucket's all-reduce and update (cnn_step.CnnStep):
    # nocarry (one grouped launch, the fc1 update carried into the next forward) is the
    # fastest RCCL structure in every N = 1 calibration (profiles/r5/final4/bench.jsonl:
    # 57.1 vs 62.3 us for carry at B = 256, 41.7 vs 46.6 at B = 32)
    rccl_mode: str = "nocarry"
    # largest fc1_fwd split-K factor
    splitk_cap: int = 32
    # world size > 1, SGD (the xgmi in-launch-exchange and RCCL nocarry steps): step k's fc1
    # update runs in extra workgroups of step k+1's forward launch instead of the optimizer
    # (kernels/fc_carry.h); the last step of a sequence updates in its own optimizer
    fc1_carry_fwd: bool = True
    # ... also from one graph replay to the next within a train_steps call (graph variants by
    # carry in / out), so only the call's last step updates fc1 in its optimizer
    fc1_carry_graphs: bool = True
    # world size 1, SGD: carry the fc1 update into the next forward launch there too, instead
    # of fusing it into fc1_bwd's weight-gradient tiles, at the batches CnnStep._local_carry
    # names (fc1_bwd then stores the gradient; a call's last step still fuses its update)
    fc1_carry_local: bool = True
    # world size 1: the conv slab reduction inside the optimizer launch
    fuse_conv_reduce: bool = True
    # world size 1, SGD: fc1's update in fc1_bwd's weight-gradient tiles
    fuse_fc1: bool = True
    # ... which also writes W1^T, double-buffered by step parity
    fc1_wt_double: bool = True
    # store the fc1 weight gradient the fused update consumes (tests / diagnostics)
    keep_grads: bool = False
    # row bands per image of the conv forward and backward (None = by batch)
    bands: Optional[int] = None
    # xgmi (per-bucket launches, PDM_XGMI_STREAM=0): the fc bucket leaves right after fc1_bwd
    xgmi_early: bool = True
    # xgmi streamed (CNN): the conv bucket all-reduced inside the optimizer launch that
    # reduces its slabs (no conv_reduce launch, no wait launch); False: conv_reduce, the
    # persistent collective, a wait launch
    xgmi_exchange: bool = True
    # xgmi streamed: the persistent collective launched eagerly per train_steps call, beside
    # the graph replays, instead of inside every step graph (fork / join edges)
    xgmi_outside: bool = True
    # Linear, world size 1: the slab reduction inside the optimizer launch
    fuse_lin_reduce: bool = True
    # fp32 CNN: conv2 / fc1 products ("x3" split-bf16, "exact" fp32 MFMA); conv-backward
    # work per workgroup (None = by batch): (image, band) units (x3) / images (exact)
    f32_conv: str = "x3"
    f32_upw: Optional[int] = None
    f32_ipb: Optional[int] = None
    # pricing only (PDM_EMULATE_WS, with a forced 1-rank communicator): size the sharded fc1
    # update for this world size -- the rank updates 128 / N rows and its collectives are
    # the 1-rank communicator's no-ops -- so an N-rank job's per-rank chain runs on one GPU
    emulate_ws: Optional[int] = None

    def __post_init__(self):
        if self.rccl_mode not in RCCL_MODES:
            raise ValueError(f"RCCL step mode {self.rccl_mode!r}: choose from {RCCL_MODES}")
        if self.f32_conv not in ("x3", "exact"):
            raise ValueError(f"PDM_F32_CONV={self.f32_conv!r}: x3 or exact")

    @classmethod
    def from_env(cls) -> "StepStructure":
        """The structure the PDM_* knobs select (unset knobs: the defaults)."""
        def flag(name, default):
            v = knobs.get(name)
            return default if v is None else v != "0"

        def opt_int(name):
            v = knobs.get(name)
            return None if v is None else int(v)

        d = cls()
        return cls(rccl_mode=knobs.get("PDM_RCCL_MODE", d.rccl_mode),
                   splitk_cap=int(knobs.get("PDM_SPLITK_CAP", str(d.splitk_cap))),
                   fc1_carry_fwd=flag("PDM_FC1_CARRY_FWD", d.fc1_carry_fwd),
                   fc1_carry_graphs=flag("PDM_FC1_CARRY_GRAPHS", d.fc1_carry_graphs),
                   fc1_carry_local=flag("PDM_FC1_CARRY_LOCAL", d.fc1_carry_local),
                   fuse_conv_reduce=flag("PDM_FUSE_CONV_REDUCE", d.fuse_conv_reduce),
                   fuse_fc1=flag("PDM_FUSE_FC1", d.fuse_fc1),
                   fc1_wt_double=flag("PDM_FC1_WT2", d.fc1_wt_double),
                   keep_grads=knobs.get("PDM_KEEP_GRADS", "0") == "1",
                   bands=opt_int("PDM_BANDS"),
                   # ranks sharing one GPU (the one-GPU rehearsal): the exchange's spinning
                   # optimizer grid would keep a peer's cnn_bwd, which needs a whole CU, off
                   # the device until the wait times out -- the wait launch is used there
                   xgmi_outside=flag("PDM_XGMI_OUTSIDE", d.xgmi_outside),
                   xgmi_exchange=flag("PDM_XGMI_XCHG", d.xgmi_exchange) and
                   knobs.get("PDM_SHARE_DEVICE") != "1",
                   fuse_lin_reduce=flag("PDM_FUSE_LIN_REDUCE", d.fuse_lin_reduce),
                   f32_conv=knobs.get("PDM_F32_CONV", d.f32_conv),
                   f32_upw=opt_int("PDM_F32_UPW"), f32_ipb=opt_int("PDM_F32_IPB"),
                   emulate_ws=opt_int("PDM_EMULATE_WS"))

    def with_(self, **kw) -> "StepStructure":
        return replace(self, **kw)
