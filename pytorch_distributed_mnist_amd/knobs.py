"""Every ``PDM_*`` environment knob in one registry.

The defaults are the production configuration; a knob exists to force one of the structures
``bench.py`` otherwise calibrates, to run a rehearsal on one GPU, or for a diagnostic or
tuning experiment.  Code reads knobs through :func:`get` (an unregistered name is a bug and
raises), ``bench.py`` echoes every knob that is set in its JSON line, and :func:`unknown`
lists ``PDM_*`` variables that match no knob (a mistyped name would otherwise be ignored
silently).
"""
from __future__ import annotations

import os
from typing import Dict, Optional

# name -> (default, kind, meaning).  kind: "structure" = picks a step structure the default
# chooses by itself, "rehearsal" = multi-rank tests on one GPU, "diag" = diagnostics and
# experiments (timed runs leave them unset), "build" = extension build options.
KNOBS: Dict[str, tuple] = {
    # step structure (bf16 CNN)
    "PDM_RCCL_MODE": ("nocarry", "structure",
                      "RCCL step structure of the fc bucket: carry / nocarry / side / early / "
                      "zero (bench.py calibrates all of them when unset)"),
    "PDM_SHARD_FC": ("0", "structure", "1: shard the fc1 update over the ranks in bench.py"),
    "PDM_COMM": ("auto", "structure", "gradient transport: auto / xgmi / rccl"),
    "PDM_FUSE_CONV_REDUCE": ("1", "structure", "0: separate conv_reduce at world size 1"),
    "PDM_FUSE_FC1": ("1", "structure", "0: fc1's SGD update in the optimizer launch, not fc1_bwd"),
    "PDM_FC1_WT2": ("1", "structure", "0: the optimizer re-derives W1^T (no double buffer)"),
    "PDM_KEEP_GRADS": ("0", "diag", "1: store the fc1 weight gradient the fused update consumes"),
    "PDM_SPLITK_CAP": ("32", "structure", "largest fc1_fwd split-K factor"),
    "PDM_FC1_CARRY_FWD": ("1", "structure", "0: the fc1 update never carried into the next "
                          "step's forward launch (world size > 1: in the optimizer launch; "
                          "world size 1: fused into fc1_bwd)"),
    "PDM_FC1_CARRY_GRAPHS": ("1", "structure", "0: the carried fc1 update stops at every graph "
                             "replay's last step instead of the train_steps call's"),
    "PDM_FC1_CARRY_LOCAL": ("1", "structure", "0: world size 1 fuses the fc1 update into "
                            "fc1_bwd at every batch instead of carrying it into the next "
                            "forward launch where that is faster (B > 128)"),
    "PDM_BANDS": (None, "structure", "row bands per image in the conv backward (1 = off)"),
    "PDM_GRAPH_STEPS": ("16", "structure", "training steps per full captured hipGraph (a remainder replays one graph of its own size)"),
    "PDM_FUSE_LIN_REDUCE": ("1", "structure", "0: separate lin_reduce at world size 1 (Linear)"),
    "PDM_F32_CONV": ("x3", "structure", "fp32 CNN conv2 products: x3 (split-bf16) / exact"),
    "PDM_F32_IPB": (None, "structure", "images per fp32 (exact) conv-backward workgroup"),
    "PDM_F32_UPW": (None, "structure", "(image, band) units per split-bf16 conv-backward workgroup"),
    # xGMI transport
    "PDM_XGMI_MODE": ("auto", "structure", "xgmi schedule: auto / one / two"),
    "PDM_XGMI_STREAM": ("1", "structure", "0: per-bucket xgmi launches, no persistent kernel"),
    "PDM_XGMI_OUTSIDE": ("1", "structure", "0: the persistent xgmi collective inside every "
                         "step graph (fork / join edges) instead of launched per train_steps"),
    "PDM_XGMI_XCHG": ("1", "structure", "0: conv bucket via conv_reduce + the persistent "
                      "collective instead of the optimizer's in-launch exchange"),
    "PDM_XGMI_TIMEOUT": ("30", "structure", "seconds any xgmi device wait for a peer may take "
                         "(bench.py's calibration deadline is this plus PDM_CALIB_TIMEOUT_S)"),
    "PDM_XGMI_PROBE": ("1", "structure", "0: no child-process pre-flight of the xgmi "
                       "peer mappings before a rank maps them itself"),
    "PDM_XGMI_PROBE_TIMEOUT_S": ("120", "structure", "seconds the xgmi pre-flight may take"),
    # bench.py
    "PDM_FORCE_COMM": ("0", "diag", "1: the world-size>1 chain at N=1 (1-rank communicator)"),
    "PDM_EMULATE_WS": (None, "diag", "with PDM_FORCE_COMM=1: price an N-rank job's per-rank "
                       "chain (fc1 update sharded over 128 / N rows, collectives stubbed)"),
    "PDM_BENCH_BACKEND": ("nccl", "rehearsal", "gloo: multi-rank bench on one GPU"),
    "PDM_BENCH_BOUNDARY": ("1", "diag", "0: no epoch boundary inside the timed window"),
    "PDM_BENCH_DEBUG": (None, "diag", "1: print the host timeline of the timed window; "
                        "events: the device timeline too (CUDA events at the marks)"),
    "PDM_BENCH_FAIL_RANK": (None, "diag", "fault injection: this rank exits (dry runs)"),
    "PDM_BENCH_SPAWNED": (None, "internal", "set by bench.py on the ranks it starts"),
    "PDM_CALIB_FAULT": (None, "diag", "fault injection into calibration: "
                        "<rank>:<candidate>:<setup|warm|timed|check|diverge|hang>[,...]"),
    "PDM_CALIB_BUDGET_S": ("120", "structure", "wall-clock budget (s) of bench.py's calibration"),
    "PDM_CALIB_TIMEOUT_S": ("30", "structure", "margin (s) of a calibration candidate's host "
                            "deadline over the xgmi device timeout (the host waits strictly "
                            "longer than any bounded device wait)"),
    "PDM_GATHER_AHEAD": ("1", "diag", "0: gather each epoch at its boundary"),
    # rehearsal / runtime
    "PDM_SHARE_DEVICE": ("0", "rehearsal", "1: every rank on device 0 (gloo / xgmi tests)"),
    "PDM_ROCTX": ("1", "diag", "0: no roctx ranges even with --trace"),
    "PDM_EXT_PATH": (None, "diag", "load this extension build instead of the in-tree one"),
    # extension build
    "PDM_DEBUG_BOUNDS": (None, "build", "device-side bounds checks"),
    "PDM_STAMPS": (None, "build", "s_memtime phase stamps (diagnostic build)"),
    "PDM_HIPCC_FLAGS": (None, "build", "extra hipcc flags"),
    "PDM_FILE_FLAGS": (None, "build", "per-file hipcc flags"),
}


def get(name: str, default: Optional[str] = None) -> Optional[str]:
    """os.environ.get for a registered knob (the registry's default is documentation: the
    call site's default is what applies, so an unset knob can be told apart)."""
    if name not in KNOBS:
        raise KeyError(f"unregistered knob {name} (add it to pytorch_distributed_mnist_amd/knobs.py)")
    return os.environ.get(name, default)


def is_set(name: str) -> bool:
    if name not in KNOBS:
        raise KeyError(f"unregistered knob {name}")
    return name in os.environ


def active() -> Dict[str, str]:
    """Every PDM_* variable set in the environment (registered or not)."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("PDM_")}


def unknown() -> Dict[str, str]:
    """PDM_* variables that match no knob (likely typos)."""
    return {k: v for k, v in active().items() if k not in KNOBS}
