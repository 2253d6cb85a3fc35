"""Timing of consecutive short windows of graph-replayed training steps (N=1).

Shows how the per-step time of a short timed run (the driver times 20 steps after 5 warmup
steps) depends on what ran just before it: GPU clock ramp-up after idle, the first replay's
launch latency, the host synchronize.  Not a benchmark of record (bench.py is).

    python tools/bench_windows.py [K] [windows]
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split  # noqa: E402
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices  # noqa: E402
from pytorch_distributed_mnist_amd.runtime.program import build_local_program  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
NW = int(sys.argv[2]) if len(sys.argv) > 2 else 12
B = 256
train = synthetic_split(60000, True)
test = synthetic_split(512, False)
p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.01,
                        momentum=0.9, weight_decay=0.0, use_graphs=True)
p.optimizer.sync_hyperparams()
p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
st = p.gpu
st.begin_epoch()
st.prepare(B)
done = 0
epoch = 0


def window(k):
    global done, epoch
    if done + k > 230:                  # stay inside one epoch (234 full steps): start the next
        epoch += 1                      # (the counter runs on; the ragged tail step is skipped)
        p.set_train_indices(distributed_indices(len(train), 1, 0, epoch))
        st.begin_epoch()
        done = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st.train_steps(B, k)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    done += k
    return (t2 - t0) / k * 1e6, (t1 - t0) * 1e6


def spin(ms):
    """bf16 GEMMs (hipBLASLt) for ~ms of sustained load, ending without an idle gap."""
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(8):
            a @ a
        torch.cuda.synchronize()


st.train_steps(B, 5)
for label, pause, sp in (("after warmup 5", 0.0, 0), ("after 0.5 s idle", 0.5, 0),
                         ("after 0.5 s idle + 40 ms GEMM spin", 0.5, 40),
                         ("after 0.5 s idle + 100 ms GEMM spin", 0.5, 100)):
    if pause:
        torch.cuda.synchronize()
        time.sleep(pause)
        if sp:
            spin(sp)
        st.train_steps(B, 5)
    rows = [window(K) for _ in range(NW)]
    print(f"{label}: K={K} us/step per window: " + " ".join(f"{r[0]:.1f}" for r in rows) +
          f" | host enqueue us: " + " ".join(f"{r[1]:.0f}" for r in rows), flush=True)
# a long window for the steady state
print(f"steady K=200: {window(200)[0]:.2f} us/step", flush=True)
# kernel-only time of one 8-step graph, from events
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
st.train_steps(B, 8)
ev[1].record()
torch.cuda.synchronize()
print(f"events over one 8-step replay: {ev[0].elapsed_time(ev[1]) / 8 * 1e3:.2f} us/step", flush=True)
