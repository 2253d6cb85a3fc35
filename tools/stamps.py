"""Phase timing of cnn_fwd / cnn_bwd from s_memtime stamps (PDM_STAMPS build only)."""
import sys
import torch
sys.path.insert(0, ".")
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
from pytorch_distributed_mnist_amd.runtime.program import build_local_program

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
train = synthetic_split(60000, True)
test = synthetic_split(512, False)
p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.01,
                        use_graphs=False)
p.optimizer.sync_hyperparams()
p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
for _ in range(5):
    p.gpu.train_step(B)
torch.cuda.synchronize()
C = p.gpu.C
for which, names in (("fwd", ["start", "gathered(barrier)", "conv1(barrier)", "conv2end", "barrier",
                              "end"]),
                     ("bwd", ["start", "loaded(barrier)", "compute_end", "barrier", "end"])):
    st = C.read_stamps(which).double()
    n = len(names)
    base = st[:, 0:1]
    rel = (st[:, :n] - base)
    med = rel.median(dim=0).values
    mx = rel.max(dim=0).values
    t0 = st[:, 0].min()
    print(which, "per-block phase (cycles, median / max):")
    for i, nm in enumerate(names):
        print(f"   {nm:22s} {med[i]:9.0f} {mx[i]:9.0f}")
    print("   block start skew (cycles):", (st[:, 0] - t0).max().item(),
          " last end:", (st[:, n - 1] - t0).max().item())
    if which == "fwd" and B <= 256:
        hs = st[:B // 4, 10:16]            # cnn_head, blocks 0 .. B/4 - 1 (one row group each)
        hb = hs[:, 0:1]
        hm = (hs - hb).median(dim=0).values
        print("   head: partials summed / xent / dh stored / slab acc / end (rel, median):",
              " ".join(f"{v:.0f}" for v in hm[1:].tolist()))
    if which == "fwd" and B > 64:
        ws = st[64:min(B, 256), 10:16] - st[64:min(B, 256), 0:1]
        print("   conv2 end per wave 1..6 (rel, median):",
              " ".join(f"{v:.0f}" for v in ws.median(dim=0).values.tolist()),
              " wave 0:", f"{(st[64:min(B, 256), 3] - st[64:min(B, 256), 0]).median().item():.0f}")
    if which == "fwd":
        print("   image load issued (rel)", (st[:, 8] - st[:, 0]).median().item(),
              " image landed (rel)", (st[:, 9] - st[:, 0]).median().item())
    if which == "bwd":
        print("   dgrad wave4: mfma-section cycles", st[:, 8].median().item(),
              " epilogue cycles", st[:, 9].median().item(),
              " dgrad done (rel)", (st[:, 10] - st[:, 0]).median().item())
        print("   load: loads-issued (rel)", (st[:, 11] - st[:, 0]).median().item(),
              " scatter done w0 / w7 (rel)", (st[:, 12] - st[:, 0]).median().item(),
              (st[:, 15] - st[:, 0]).median().item(),
              " post-scatter barrier", (st[:, 13] - st[:, 0]).median().item(),
              " conv1 done w0", (st[:, 14] - st[:, 0]).median().item())
