"""Parent side of the xGMI pre-flight (parallel/xgmi_probe.py) with stand-in child programs:
a child that completes the protocol, one that dies (a GPU fault ends the process the same
way), one that hangs, one that reports a mismatch, and a two-rank gloo run where only one
rank's child dies and both ranks must leave xgmi out."""
import os
import socket
import sys
import textwrap

import pytest
import torch.multiprocessing as mp

from pytorch_distributed_mnist_amd.parallel.xgmi_probe import TAG, probe

CHILD = textwrap.dedent(f"""
    import sys, time
    how = sys.argv[1]
    def say(t):
        print("{TAG} " + t, flush=True)
    if how == "die":
        sys.exit(7)
    print("noise on stdout is ignored", flush=True)
    say("handle " + ("ab" * 8))
    if how == "hang":
        time.sleep(60)
    line = sys.stdin.readline()
    assert line.startswith("handles "), line
    say("mapped")
    assert sys.stdin.readline().strip() == "go"
    say("bad" if how == "bad" else "ok")
    sys.stdin.readline()
""")


class DictStore:
    def __init__(self):
        self.d = {}

    def set(self, k, v):
        self.d[k] = v.encode() if isinstance(v, str) else v

    def get(self, k):
        return self.d[k]


def _child(tmp_path, how):
    p = tmp_path / "child.py"
    p.write_text(CHILD)
    return [sys.executable, str(p), how]


@pytest.mark.parametrize("how,ok,why", [("good", True, ""), ("die", False, "exited with status 7"),
                                        ("hang", False, "timed out"), ("bad", False, "self-check failed")])
def test_probe_one_rank(tmp_path, how, ok, why):
    got, reason = probe(0, 1, 0, DictStore(), "k", lambda f: f, timeout_s=4.0,
                        argv=_child(tmp_path, how))
    assert got is ok
    assert why in reason


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, tmp, q):
    import torch
    import torch.distributed as dist
    from torch.distributed import distributed_c10d as c10d
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)

    def agree(flag):
        t = torch.tensor([1 if flag else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    argv = [sys.executable, os.path.join(tmp, "child.py"), "die" if rank == 1 else "good"]
    ok, reason = probe(rank, 2, 0, c10d._get_default_store(), "pdm_test/probe", agree,
                       timeout_s=20.0, argv=argv)
    q.put((rank, ok, reason))
    dist.destroy_process_group()


def test_probe_two_ranks_one_child_dies(tmp_path):
    (tmp_path / "child.py").write_text(CHILD)
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = dict((r, (ok, why)) for r, ok, why in (q.get() for _ in range(2)))
    assert res[0][0] is False and res[1][0] is False
    assert "exported no handle" in res[0][1]
    assert "exited with status 7" in res[1][1]
