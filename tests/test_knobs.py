"""Environment knobs that would silently corrupt a run are rejected at import / construction."""
import os
import subprocess
import sys

import pytest

from conftest import REPO


@pytest.mark.parametrize("value,ok", [("8", True), ("16", True), ("6", False), ("0", False)])
def test_graph_steps_must_be_a_power_of_two(value, ok):
    env = dict(os.environ, PDM_GRAPH_STEPS=value, PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-c",
                        "import pytorch_distributed_mnist_amd.runtime.gpu_step as g; "
                        "print(g.GpuStepBase.GRAPH_SIZES)"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    assert (r.returncode == 0) == ok, r.stderr[-500:]
    if not ok:
        assert "power of two" in r.stderr

