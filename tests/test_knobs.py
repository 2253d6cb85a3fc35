"""Environment knobs that would silently corrupt a run are rejected at import / construction."""
import os
import subprocess
import sys

import pytest

from conftest import REPO


@pytest.mark.parametrize("value,ok", [("8", True), ("16", True), ("6", True), ("0", False),
                                      ("-2", False)])
def test_graph_steps_must_be_positive(value, ok):
    env = dict(os.environ, PDM_GRAPH_STEPS=value, PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-c",
                        "import pytorch_distributed_mnist_amd.runtime.gpu_step as g; "
                        "print(g.GpuStepBase.GRAPH_SIZES)"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    assert (r.returncode == 0) == ok, r.stderr[-500:]
    if ok:
        assert r.stdout.strip() == str(tuple(range(int(value), 0, -1)))
    else:
        assert "must be positive" in r.stderr



def test_every_knob_read_in_code_is_registered():
    """All PDM_* names the package, bench.py and the build read are in knobs.KNOBS, so
    bench.py's echo and the typo warning cover every switch."""
    import glob
    import re
    from pytorch_distributed_mnist_amd import knobs
    files = glob.glob(os.path.join(REPO, "pytorch_distributed_mnist_amd", "**", "*.py"),
                      recursive=True) + [os.path.join(REPO, "bench.py")]
    used = set()
    for f in files:
        used |= set(re.findall(r'"(PDM_[A-Z0-9_]+)"', open(f).read()))
    assert used - set(knobs.KNOBS) == set(), used - set(knobs.KNOBS)
    with pytest.raises(KeyError):
        knobs.get("PDM_NOT_A_KNOB")


def test_unknown_knobs_are_reported(monkeypatch):
    from pytorch_distributed_mnist_amd import knobs
    monkeypatch.setenv("PDM_RCCL_MODEE", "early")
    monkeypatch.setenv("PDM_RCCL_MODE", "early")
    assert knobs.unknown() == {"PDM_RCCL_MODEE": "early"}
    assert knobs.get("PDM_RCCL_MODE") == "early"
