"""Run N eager (no hipGraph) CNN training steps at batch B: a plain target for rocprofv3
counter collection (python3 tools/step_loop.py [B] [N])."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split  # noqa: E402
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices  # noqa: E402
from pytorch_distributed_mnist_amd.runtime.program import build_local_program  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
N = int(sys.argv[2]) if len(sys.argv) > 2 else 30
train = synthetic_split(60000, True)
test = synthetic_split(512, False)
p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.01,
                        use_graphs=False)
p.optimizer.sync_hyperparams()
p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
for _ in range(N):
    p.gpu.train_step(B)
torch.cuda.synchronize()
print("done", B, N)
