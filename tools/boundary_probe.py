"""Host cost of each epoch-boundary operation while the GPU is busy with queued steps.

    python tools/boundary_probe.py

Queues 10 CNN steps (graph replays), then times the boundary's host calls
(the gather launch, which also resets the counters, and begin_epoch) and how long the device
stays busy after them; prints one line per trial.
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split           # noqa: E402
from pytorch_distributed_mnist_amd.data.sampler import EpochIndexPrefetcher    # noqa: E402
from pytorch_distributed_mnist_amd.runtime.program import build_local_program  # noqa: E402


def main():
    B = 256
    train = synthetic_split(60000, True)
    test = synthetic_split(512, False)
    p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.01)
    pf = EpochIndexPrefetcher(len(train), 1, 0, int32=True)
    p.optimizer.sync_hyperparams()
    p.set_train_indices(pf.get(0), pf.peek(1))
    st = p.gpu
    st.prepare(B)
    st.train_steps(B, 16)
    torch.cuda.synchronize()
    from pytorch_distributed_mnist_amd.parallel.comm import bounded_sync
    for trial in range(12):
        # trials 0-5: the next order is ready and the worker idle; 6-11: as in bench.py, the
        # worker starts the following epoch's order inside the window (get() submits it)
        if trial < 6:
            idx = pf.get(trial + 1)
            time.sleep(0.01)
        st.ctr.zero_()
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        st.train_steps(B, 10)
        if trial >= 6:
            idx = pf.get(trial + 1)
        t.append(time.perf_counter())
        st.set_train_indices(idx, pf.peek(trial + 2))   # next order gathered ahead
        t.append(time.perf_counter())
        st.begin_epoch()
        t.append(time.perf_counter())
        st.train_steps(B, 10)
        t.append(time.perf_counter())
        bounded_sync(st.device, 60.0)
        t.append(time.perf_counter())
        d = [1e6 * (b - a) for a, b in zip(t, t[1:])]
        print(f"trial {trial}: replay10(+get) {d[0]:.0f} us | gather {d[1]:.0f} | "
              f"begin_epoch {d[2]:.0f} | replay10 {d[3]:.0f} | drain {d[4]:.0f} | "
              f"total {1e6 * (t[-1] - t[0]):.0f}", flush=True)
    pf.close()


if __name__ == "__main__":
    main()
