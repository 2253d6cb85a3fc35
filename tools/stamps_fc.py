"""Phase timing of fc1_bwd's dX and dW tiles from s_memtime stamps (PDM_STAMPS build only).

    PDM_EXT_PATH=build/stamps/_C...so python tools/stamps_fc.py [B]
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
p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.01,
                        use_graphs=False)
p.optimizer.sync_hyperparams()
p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
st = p.gpu
for _ in range(5):
    st.train_step(B)
torch.cuda.synchronize()
C, G = st.C, st.G
ldt = -(-B // 32) * 32
for _ in range(3):   # fc1_bwd alone (cnn_bwd would overwrite the stamps)
    C.fc1_bwd(st.dh, st.dht, ldt, st.pool, st.current_wf1t(), B, G["fc1.weight"], st.dpool, st.head_slab,
              G["fc2.weight"], G["fc2.bias"], G["fc1.bias"], st.metrics.train_view(),
              st._fc_update() if st.fuse_fc1 else None)
torch.cuda.synchronize()
s = C.read_stamps("bwd").double().view(256, 16)
ndx = ldt // 32 * 24
dx = s[:min(ndx, 256), 0:4]
dw = s[:144, 8:14]
t0 = torch.cat([dx[:, 0], dw[:, 0]]).median().item()   # typical workgroup start
print("dX tiles (cycles; start relative to the median workgroup start, phases relative to the"
      " tile's own start; median / max):")
print(f"   {'start':14s} {(dx[:, 0] - t0).median().item():8.0f} {(dx[:, 0] - t0).max().item():8.0f}")
for i, nm in enumerate(["loads issued", "MFMAs done", "end"], 1):
    d = dx[:, i] - dx[:, 0]
    print(f"   {nm:14s} {d.median().item():8.0f} {d.max().item():8.0f}")
print("dW tiles:")
print(f"   {'start':14s} {(dw[:, 0] - t0).median().item():8.0f} {(dw[:, 0] - t0).max().item():8.0f}")
for i, nm in [(1, "chunk0 in LDS"), (2, "chunk1 in LDS"), (3, "MFMAs done"), (5, "end")]:
    d = dw[:, i] - dw[:, 0]
    print(f"   {nm:14s} {d.median().item():8.0f} {d.max().item():8.0f}")
