"""StepStructure: the PDM_* structure knobs are read once into one object (CPU)."""
import pytest

from pytorch_distributed_mnist_amd.runtime.structure import StepStructure


def test_defaults_are_production(monkeypatch):
    for k in ("PDM_RCCL_MODE", "PDM_SPLITK_CAP", "PDM_FUSE_FC1", "PDM_BANDS", "PDM_F32_CONV",
              "PDM_FC1_CARRY_FWD", "PDM_FC1_CARRY_LOCAL"):
        monkeypatch.delenv(k, raising=False)
    s = StepStructure.from_env()
    assert s == StepStructure()
    assert s.rccl_mode == "nocarry" and s.splitk_cap == 32 and s.fuse_fc1 and s.bands is None
    # the fc1 update carried into the next forward (world size > 1): on; carried at world
    # size 1 too where that is faster (profiles/r5/fc1_carry_local/)
    assert s.fc1_carry_fwd and s.fc1_carry_local


def test_from_env_reads_each_knob(monkeypatch):
    monkeypatch.setenv("PDM_RCCL_MODE", "early")
    monkeypatch.setenv("PDM_SPLITK_CAP", "16")
    monkeypatch.setenv("PDM_FUSE_FC1", "0")
    monkeypatch.setenv("PDM_BANDS", "3")
    monkeypatch.setenv("PDM_F32_CONV", "exact")
    monkeypatch.setenv("PDM_KEEP_GRADS", "1")
    monkeypatch.setenv("PDM_FC1_CARRY_FWD", "0")
    monkeypatch.setenv("PDM_FC1_CARRY_LOCAL", "0")
    s = StepStructure.from_env()
    assert (s.rccl_mode, s.splitk_cap, s.fuse_fc1, s.bands, s.f32_conv, s.keep_grads) == \
        ("early", 16, False, 3, "exact", True)
    assert (s.fc1_carry_fwd, s.fc1_carry_local) == (False, False)
    assert s.with_(rccl_mode="nocarry").rccl_mode == "nocarry"


@pytest.mark.parametrize("kw", [{"rccl_mode": "bogus"}, {"f32_conv": "tf32"}])
def test_invalid_structure_rejected(kw):
    with pytest.raises(ValueError):
        StepStructure(**kw)


def test_program_snapshots_the_structure(monkeypatch):
    """The CPU program keeps the structure it was built with (env changes later are moot)."""
    from types import SimpleNamespace
    import torch
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
    from pytorch_distributed_mnist_amd.runtime.program import build_local_program
    monkeypatch.setenv("PDM_SPLITK_CAP", "8")
    prog = build_local_program("linear", "fp32", "cpu", 64, synthetic_split(128, True),
                               synthetic_split(64, False))
    monkeypatch.setenv("PDM_SPLITK_CAP", "4")
    assert prog.structure.splitk_cap == 8
