"""Pre-flight of the direct xGMI transport in a child process.

A peer mapping that is wrong in a way no HIP call reports (a dmabuf import that maps the
wrong pages, a fabric path the driver did not set up) shows up as a GPU memory fault in the
first collective kernel, and a GPU fault ends the PROCESS that launched the kernel: here a
training rank, with the whole N-GPU job behind it.  The transport's own self-check
(``XgmiTransport._selfcheck``) catches wrong sums and late peers, not faults.  So before a
rank maps its peers itself, every rank starts one child process that builds a small
``XgmiReducer`` on the same device (a one-shot bucket and a two-shot one), exchanges hipIpc
handles with the other ranks' children and runs the same bit-exact self-check.  The child
talks to its parent only (protocol lines on stdin / stdout); the parents relay the handles
through the rendezvous store and agree on every step over the gloo control plane, so a
child that faults, hangs or reports a mismatch costs the probe and not the job: every rank
then leaves xgmi out (``bench.py`` records why; the RCCL transports remain).

    parent:  probe(rank, ws, device, store, key, agree) -> (ok, reason)
    child:   python -m pytorch_distributed_mnist_amd.parallel.xgmi_probe RANK WS DEVICE T

The child is a separate program started with ``subprocess`` (never an exec of the
GPU-initialised parent).  Knobs: ``PDM_XGMI_PROBE=0`` skips the probe,
``PDM_XGMI_PROBE_TIMEOUT_S`` bounds it (default 120 s; the child's in-kernel peer waits
are bounded at a tenth of that).
"""
from __future__ import annotations

import os
import queue
import subprocess
import sys
import threading
import time

TAG = "PDMPROBE"
SMALL = 4096                 # floats of the one-shot bucket
TOTAL = SMALL + (256 << 10)  # + a 1 MB bucket: two-shot at 3+ ranks (reducer.py threshold)


def selfcheck(native, grads, bounds, ws: int, rank: int, rounds: int = 3) -> bool:
    """All-reduce integer-valued patterns whose sums are exact and compare bit for bit
    (shared with ``XgmiTransport``).  Restores ``grads``."""
    import torch
    result = native.result()
    saved = grads.clone()
    ok = True
    n = grads.numel()
    base = (torch.arange(n, device=grads.device, dtype=torch.int64) % 251 - 125).float()
    for it in range(rounds):
        grads.copy_(base * float((it + 1) * (rank + 1)))
        native.all_ready()
        native.finalize()
        torch.cuda.synchronize(grads.device)
        want = base * float((it + 1) * ws * (ws + 1) // 2)
        for s, e in bounds:
            ok = ok and torch.equal(result[s:e], want[s:e])
    ok = ok and native.error() == 0
    grads.copy_(saved)
    torch.cuda.synchronize(grads.device)
    return bool(ok)


# ---------------------------------------------------------------------------- parent side
class _Child:
    """The child process and a reader thread that queues its protocol lines."""

    def __init__(self, argv, env):
        self.proc = subprocess.Popen(argv, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                     env=env, text=True, bufsize=1)
        self.lines: queue.Queue = queue.Queue()
        t = threading.Thread(target=self._pump, daemon=True)
        t.start()

    def _pump(self):
        for line in self.proc.stdout:
            if line.startswith(TAG + " "):
                self.lines.put(line[len(TAG) + 1:].strip())
        self.lines.put(None)                      # EOF: the child exited

    def read(self, deadline: float):
        """The next protocol line, or (None, why) on exit / timeout."""
        try:
            line = self.lines.get(timeout=max(0.0, deadline - time.monotonic()))
        except queue.Empty:
            return None, "timed out"
        if line is None:
            rc = self.proc.wait()
            return None, f"exited with status {rc}"
        return line, ""

    def send(self, text: str) -> bool:
        try:
            self.proc.stdin.write(text + "\n")
            self.proc.stdin.flush()
            return True
        except (BrokenPipeError, OSError, ValueError):
            return False

    def close(self, wait_s: float) -> None:
        try:
            self.proc.stdin.close()
        except (BrokenPipeError, OSError):
            pass
        try:
            self.proc.wait(timeout=wait_s)
        except subprocess.TimeoutExpired:
            self.proc.kill()                      # this exact child only
            self.proc.wait()


def child_argv(rank: int, ws: int, device: int, kernel_timeout_s: float) -> list:
    return [sys.executable, "-m", __name__, str(rank), str(ws), str(device), str(kernel_timeout_s)]


def probe(rank: int, ws: int, device: int, store, key: str, agree, timeout_s: float = 120.0,
          argv=None) -> tuple:
    """Run the pre-flight (collective: every rank calls it).  ``agree(flag) -> bool`` is
    the MIN of ``flag`` over ranks; ``store`` has ``set`` / ``get`` (the rendezvous store).
    Returns (ok on every rank, this rank's reason when not)."""
    deadline = time.monotonic() + timeout_s
    env = dict(os.environ)
    pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = pkg_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    argv = argv or child_argv(rank, ws, device, max(1.0, timeout_s / 10))
    reason = ""
    try:
        child = _Child(argv, env)
    except OSError as e:
        child, reason = None, f"could not start the probe process: {e}"
    # 1. every child exports its buffer; the parents relay the handles
    handle = ""
    if child is not None:
        line, why = child.read(deadline)
        if line is not None and line.startswith("handle "):
            handle = line.split(" ", 1)[1]
        else:
            reason = reason or f"no ipc handle from the probe process ({why or line})"
    store.set(f"{key}/{rank}", handle or "-")
    handles = [store.get(f"{key}/{r}") for r in range(ws)]
    handles = [h.decode() if isinstance(h, bytes) else str(h) for h in handles]
    mapped = False
    if handle and all(h != "-" for h in handles):
        if child.send("handles " + " ".join(handles)):
            line, why = child.read(deadline)
            mapped = line == "mapped"
            if not mapped:
                reason = reason or f"mapping the peers failed ({why or line})"
        else:
            reason = reason or "the probe process went away"
    elif not reason:
        reason = "a peer's probe process exported no handle"
    # 2. every child has mapped every peer before any child launches a collective kernel
    ok = False
    if agree(mapped):
        if child.send("go"):
            line, why = child.read(deadline)
            ok = line == "ok"
            if not ok:
                reason = reason or f"self-check failed ({why or line})"
        else:
            reason = reason or "the probe process went away"
    elif not reason:
        reason = "a peer's probe process could not map its peers"
    all_ok = agree(ok)
    if child is not None:
        child.send("bye")
        child.close(15.0 if ok else 2.0)     # a failed child may be stuck: do not wait long
    if not all_ok and not reason:
        reason = "the probe failed on another rank"
    return all_ok, reason


# ----------------------------------------------------------------------------- child side
def _say(text: str) -> None:
    sys.stdout.write(f"{TAG} {text}\n")
    sys.stdout.flush()


def _hear() -> str:
    line = sys.stdin.readline()
    if not line:
        raise SystemExit(4)                       # parent gone
    return line.strip()


def child_main(rank: int, ws: int, device: int, kernel_timeout_s: float) -> int:
    import torch
    from ..ops import _ext
    C = _ext.require()
    torch.cuda.set_device(device)
    grads = torch.zeros(TOTAL, device=f"cuda:{device}", dtype=torch.float32)
    bounds = [(0, SMALL), (SMALL, TOTAL)]
    native = C.XgmiReducer(rank, ws, device, grads, [b for se in bounds for b in se],
                           kernel_timeout_s, "auto")
    _say("handle " + bytes(native.ipc_handle()).hex())
    msg = _hear()
    if not msg.startswith("handles "):
        return 3
    peers = [bytes.fromhex(h) for h in msg.split()[1:]]
    native.open_peers(peers)
    _say("mapped")
    if _hear() != "go":
        return 3
    ok = selfcheck(native, grads, bounds, ws, rank)
    _say("ok" if ok else "bad")
    _hear()                                        # "bye": every rank's check is done
    native.close()
    return 0 if ok else 1


if __name__ == "__main__":
    r, w, d, t = sys.argv[1:5]
    sys.exit(child_main(int(r), int(w), int(d), float(t)))
