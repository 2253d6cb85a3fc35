"""Run N eager (no hipGraph) CNN training steps at batch B: a plain target for rocprofv3
counter collection.

    python3 tools/step_loop.py [B] [N] [bf16|fp32] [force|local] [seq]

`force` runs the world-size>1 step structure through a 1-rank RCCL communicator
(unfused conv reduction, bucket all-reduces), as bench.py's PDM_FORCE_COMM=1.  `seq` enqueues
the N steps as ONE train_steps call (the layout of a graph-replayed run: work carried from
step to step, e.g. the fc1 update into the next forward launch) instead of N calls of one."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split  # noqa: E402
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices  # noqa: E402
from pytorch_distributed_mnist_amd.runtime.program import build_local_program  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
N = int(sys.argv[2]) if len(sys.argv) > 2 else 30
DT = sys.argv[3] if len(sys.argv) > 3 else "bf16"
FORCE = len(sys.argv) > 4 and sys.argv[4] == "force"
SEQ = len(sys.argv) > 5 and sys.argv[5] == "seq"
train = synthetic_split(60000, True)
test = synthetic_split(512, False)
comm = None
if FORCE:
    from pytorch_distributed_mnist_amd.parallel.comm import RcclComm
    comm = RcclComm(0, 1, torch.device("cuda", 0))
p = build_local_program("cnn", DT, "cuda", B, train, test, optimizer="sgd", lr=0.01,
                        use_graphs=False, comm=comm, force_comm=FORCE,
                        transport="rccl" if FORCE else None)
p.optimizer.sync_hyperparams()
p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
if SEQ:
    p.gpu.train_steps(B, N)
else:
    for _ in range(N):
        p.gpu.train_step(B)
torch.cuda.synchronize()
print("done", B, N, DT, "force" if FORCE else "", "seq" if SEQ else "")
