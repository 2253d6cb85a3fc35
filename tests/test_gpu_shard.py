"""fc1 optimizer-state sharding (CnnStep.set_shard_fc, ZeRO-1 on the fc bucket): the gradient
of the fc1 weight is reduce-scattered, each rank updates its 128 / N rows and the bf16 W1 rows
are all-gathered.  Per element it is the replicated update, so the parameters and momentum
must be bit-identical to the unsharded run; checkpoints gather the full state first and keep
the reference format (multi_proc_single_gpu.py:250-255), so a sharded run resumes at ws=1."""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import REPO, free_port
from test_gpu_app import EPOCH_RE, cli

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nproc", [2, 4])
def test_sharded_fc1_update_matches_replicated(gpu, tmp_path, nproc):
    env = dict(os.environ, PDM_SHARE_DEVICE="1", PDM_SHARD_OUT=str(tmp_path))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", str(nproc), "--master-addr", "127.0.0.1",
                        "--master-port", str(free_port()),
                        os.path.join(REPO, "tests", "shard_worker.py")],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for i in range(nproc):
        d = json.load(open(tmp_path / f"rank{i}.json"))
        assert d["kinds"] == ["torch", "torch"]
        assert d["params_equal"] and d["momentum_equal"], d
        assert d["replicas_equal"] and d["eval_equal"], d


def test_sharded_cli_checkpoint_resumes_at_one_rank(gpu, tmp_path, monkeypatch):
    """--shard-fc at world size 2 (gloo data plane on one GPU): the checkpoint holds the full
    state (sync_master before rank 0 saves), loads with weights_only=True and evaluates at
    world size 1 to the epoch's printed test line."""
    monkeypatch.setenv("PDM_SHARE_DEVICE", "1")
    common = ["--arch", "cnn", "--optimizer", "sgd", "--lr", "0.05", "--seed", "5"]
    out = cli(common + ["--synthetic-size", "2048", "--epochs", "1", "--world-size", "2",
                        "--shard-fc"], tmp_path, backend="gloo")
    ep = [EPOCH_RE.match(l) for l in out if l.startswith("Epoch:")]
    assert len(ep) == 2 and all(ep), out
    ck = tmp_path / "checkpoints" / "checkpoint_0.pth.tar"
    sd = torch.load(ck, weights_only=True)
    w = sd["state_dict"]["module.fc1.weight"]
    mom = sd["optimizer"]["state"][4]["momentum_buffer"]      # fc1.weight is torch param 4
    assert w.shape == (128, 9216) and mom.shape == (128, 9216)
    # every row was updated (no rank's half left at its initial / zero state)
    assert (mom.abs().sum(1) > 0).all()
    ev = [l for l in cli(common + ["--evaluate", "--resume", str(ck)], tmp_path, backend="gloo")
          if l.startswith("test loss:")]
    assert ev == ["test loss: {}, test acc: {}%.".format(ep[0].group(5), ep[0].group(6))]
