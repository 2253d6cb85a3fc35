"""Fail-fast RCCL bring-up, control-plane half (CPU): a rank waiting for rank 0's unique id
gives up as soon as another rank posts its failure to the rendezvous store, instead of
waiting for the whole deadline (parallel/comm.py _await_key; the device half, the cancel
token ending the C++ init poll, is tests/test_gpu_comm.py)."""
import threading
import time
from datetime import timedelta

import pytest
from torch.distributed import TCPStore

from conftest import free_port
from pytorch_distributed_mnist_amd.parallel.comm import _await_key


def _store():
    return TCPStore("127.0.0.1", free_port(), 1, True, timeout=timedelta(seconds=30))


def test_await_key_returns_the_value():
    s = _store()
    threading.Timer(0.2, s.set, ["uid", b"abc"]).start()
    assert _await_key(s, "uid", "uid/failed", 30.0) == b"abc"


def test_await_key_gives_up_when_a_peer_failed():
    s = _store()
    threading.Timer(0.2, s.set, ["uid/failed", "rank 0: no device"]).start()
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match="cancelled: rank 0: no device"):
        _await_key(s, "uid", "uid/failed", 30.0)
    assert time.monotonic() - t0 < 5.0


def test_await_key_deadline():
    s = _store()
    with pytest.raises(RuntimeError, match="no unique id"):
        _await_key(s, "uid", "uid/failed", 0.3)
