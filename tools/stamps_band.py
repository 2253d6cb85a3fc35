"""Phase timing (s_memtime stamps, PDM_STAMPS build) of the small-batch row-band kernels
cnn_fwd_band / cnn_bwd_band inside eager training steps.

    PDM_STAMPS=1 python -m pytorch_distributed_mnist_amd.build --out build/stamps/_C...so
    PDM_EXT_PATH=build/stamps/_C...so python tools/stamps_band.py 32
"""
import sys

import torch

sys.path.insert(0, ".")
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split  # noqa: E402
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices  # noqa: E402
from pytorch_distributed_mnist_amd.runtime.program import build_local_program  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
train = synthetic_split(60000, True)
test = synthetic_split(512, False)
p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.01,
                        use_graphs=False)
p.optimizer.sync_hyperparams()
p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
for _ in range(6):
    p.gpu.train_step(B)
torch.cuda.synchronize()
C = p.gpu.C
PH = {"fwd_band": ["start", "weights+image(barrier)", "x3(barrier)", "conv1(barrier)",
                   "conv2(barrier)", "end"],
      "bwd_band": ["start", "loads issued", "zero fills", "-", "scatter done",
                   "staged(barrier)", "wgrad done w0", "dgrad done w4", "compute(barrier)", "end"]}
for which, names in PH.items():
    st = C.read_stamps(which).double()
    nb = min(256, int((st[:, 0] > 0).sum().item()))
    st = st[:nb]
    n = len(names)
    base = st[:, 0:1]
    rel = st[:, :n] - base
    med = rel.median(dim=0).values
    mx = rel.max(dim=0).values
    t0 = st[:, 0].min()
    print(f"{which}: {nb} blocks, per-block phase end (cycles from block start, median / max;"
          f" 100 MHz s_memtime -> x 24 for 2.4 GHz cycles):")
    for i, nm in enumerate(names):
        print(f"   {nm:26s} {med[i]:8.0f} {mx[i]:8.0f}")
    print("   block start skew:", (st[:, 0] - t0).max().item(), " last end:",
          (st[:, n - 1] - t0).max().item())
