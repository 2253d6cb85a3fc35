"""Phase timing of the fp32 split-bf16 kernels (f32x3_fwd, f32x3_conv_bwd) from s_memtime
stamps: run with a PDM_STAMPS build (PDM_EXT_PATH=build/stamps_f32/_C...so).

    PDM_EXT_PATH=... python tools/stamps_f32.py [B]

s_memtime ticks are shader cycles (MI355X_MICROARCH.md; ~2.4 GHz at full clock).  The stamps
cost a few percent of the phases they bracket; compare phases, not absolute totals.
"""
import sys

import torch

sys.path.insert(0, ".")
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split  # noqa: E402
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices  # noqa: E402
from pytorch_distributed_mnist_amd.runtime.program import build_local_program  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
train = synthetic_split(60000, True)
test = synthetic_split(512, False)
p = build_local_program("cnn", "fp32", "cuda", B, train, test, optimizer="sgd", lr=0.01,
                        use_graphs=False)
p.optimizer.sync_hyperparams()
p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
for _ in range(5):
    p.gpu.train_step(B)
torch.cuda.synchronize()
st = p.gpu.C.read_stamps("f32").double()


def show(title, cols, names):
    rel = st[:, cols] - st[:, cols[0]:cols[0] + 1]
    med = rel.median(dim=0).values
    mx = rel.max(dim=0).values
    print(f"{title} per-block phase, cycles since the block's start (median / max):")
    prev = 0.0
    for i, nm in enumerate(names):
        print(f"   {nm:34s} {med[i]:8.0f} {mx[i]:8.0f}   (+{med[i] - prev:6.0f})")
        prev = med[i].item()
    t0 = st[:, cols[0]].min()
    print("   block start skew:", (st[:, cols[0]] - t0).max().item(),
          " last end:", (st[:, cols[-1]] - t0).max().item())


show("f32x3_fwd", [0, 1, 2, 3, 4, 5, 6],
     ["start", "loads + W2 split + W2T planes", "barrier 1", "conv1 (wave 0)", "barrier 2",
      "conv2 end (wave 0)", "conv2 end (wave 7)"])
rel7 = (st[:, 7] - st[:, 13]).median().item()
print(f"f32x3_conv_bwd: second unit staged + barrier, cycles after the first unit's wgrad end: {rel7:.0f}")
show("f32x3_conv_bwd (first image of blocks 0..255)", [8, 9, 10, 11, 12, 13, 14, 15],
     ["start", "W2T staged + prefetch issued", "staging + barrier", "scatter + barrier",
      "dgrad end (wave 0)", "wgrad end (wave 0)", "all images (wave 0)", "end (slab written)"])
