"""Where the driver's 20-step window loses time beside the kernels (N = 1, B = 256).

Times (host clock, device synchronized on both sides) short sequences of graph-replayed steps
that differ in one thing each, so the differences price the graph-replay boundaries, the ragged
tail step and the host's epoch-boundary work separately:

  full20      train_steps(256, 20)                          (graphs 8 + 8 + 4)
  split       train_steps(256, 9), (256, 1), (256, 10)      (graphs 8 + 1 | 1 | 8 + 2)
  tail        train_steps(256, 9), (96, 1), (256, 10)       (the tail graph in the middle)
  boundary    as tail, positioned at the end of an epoch, with bench.py's epoch switch
              (prefetcher get + set_train_indices + begin_epoch) between the tail and the next
              call; every order the switch queues was computed beforehand
  boundary_pf as boundary, but the switch queues the sampler's randperm of later epochs on the
              prefetcher's worker thread, as the bench's boundary does

Each window follows 5 warm-up steps and a torch.cuda._sleep marker kernel (for
tools/gaps_from_trace.py).

    python tools/graph_gaps.py [reps]
"""
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split  # noqa: E402
from pytorch_distributed_mnist_amd.data.sampler import EpochIndexPrefetcher  # noqa: E402
from pytorch_distributed_mnist_amd.runtime.program import build_local_program  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 7
B, TAIL = 256, 60000 % 256
train = synthetic_split(60000, True)
test = synthetic_split(512, False)
p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.01,
                        momentum=0.9, weight_decay=0.0, use_graphs=True)
st = p.gpu
p.optimizer.sync_hyperparams()
prefetch = EpochIndexPrefetcher(len(train), 1, 0, int32=True)
orders = {}


def order(e):
    """Epoch e's order as bench.py hands it over (one object per epoch)."""
    if e not in orders:
        orders[e] = prefetch.peek(e)
    return orders[e]


epoch = 0
prefetch.get(0)
p.set_train_indices(order(0), order(1))
st.begin_epoch()
st.prepare(B)
st.prepare(TAIL, sizes=(1,))
spe = st.spe
pos = 0                                   # step within the current epoch


def new_epoch():
    global epoch, pos
    epoch += 1
    prefetch.get(epoch)                   # as bench.py's next_epoch(): queues later epochs
    p.set_train_indices(order(epoch), order(epoch + 1))
    st.begin_epoch()
    pos = 0


def worker(busy):
    """Before a boundary window: busy=False computes every order the switch will queue now;
    busy=True drops the ones after the next epoch, so the switch inside the window queues
    their randperm on the worker thread."""
    for e in (epoch + 2, epoch + 3):
        if busy:
            orders.pop(e, None)
            f = prefetch._futs.pop(e, None)
            if f is not None:
                f.result()
        else:
            order(e)
    order(epoch + 1)


def to_epoch_end(k):
    """Move the counter so that k full steps and the tail remain in this epoch."""
    global pos
    want = spe - 1 - k
    if pos > want:
        st.train_steps(B, spe - 1 - pos)   # finish this epoch (untimed)
        st.train_steps(TAIL, 1)
        new_epoch()
    st.skip_steps(want - pos)
    pos = want


def fresh_epoch_room(k):
    if pos + k > spe - 1:
        to_epoch_end(0)
        st.train_steps(TAIL, 1)
        new_epoch()


def timed(name):
    global pos
    if name.startswith("boundary"):
        to_epoch_end(9 + 5)
    else:
        fresh_epoch_room(25)
    st.train_steps(B, 5)                   # the bench's warm-up right before the window
    pos += 5
    if name.startswith("boundary"):
        worker(busy=name == "boundary_pf")
    torch.cuda._sleep(100)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if name == "full20":
        st.train_steps(B, 20)
        pos += 20
    elif name == "split":
        st.train_steps(B, 9)
        st.train_steps(B, 1)
        st.train_steps(B, 10)
        pos += 20
    elif name == "tail":
        st.train_steps(B, 9)
        st.train_steps(TAIL, 1)            # a tail-sized step mid-epoch (timing only)
        st.train_steps(B, 10)
        pos += 20
    else:
        st.train_steps(B, 9)
        st.train_steps(TAIL, 1)
        new_epoch()
        st.train_steps(B, 10)
        pos += 10
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6, (t1 - t0) * 1e6


# first-launch vs chip-idle: the first full20 after prepare (every graph exec launched for the
# first time, chip idle since the captures), then again at once, after 0.5 s idle (the same
# graph execs), and after 0.5 s idle + a 50 ms bf16 GEMM load
cold = [("first", timed("full20")), ("again", timed("full20"))]
time.sleep(0.5)
cold.append(("after 0.5 s idle", timed("full20")))
time.sleep(0.5)
a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.05:
    a @ a
cold.append(("after idle + 50 ms GEMM", timed("full20")))
print("full20 windows: " + "; ".join(f"{n} {r[0] / 20:.2f} us/step" for n, r in cold), flush=True)

names = ("full20", "split", "tail", "boundary", "boundary_pf")
res = {n: [] for n in names}
for _ in range(REPS):
    for n in names:
        res[n].append(timed(n))
for n in names:
    tot = statistics.median(r[0] for r in res[n])
    host = statistics.median(r[1] for r in res[n])
    print(f"{n:11s} window {tot:8.1f} us ({tot / 20:6.2f} us/step)   host enqueue {host:7.1f} us   "
          f"all: {' '.join(f'{r[0]:.0f}' for r in res[n])}", flush=True)
prefetch.close()
