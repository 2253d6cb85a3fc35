"""One training step at batch B on a fresh program; saves the conv gradient slabs and the
conv gradients (keep_grads) to OUT, and with REF compares them bit for bit.  Used to A/B two
builds of the conv backward (PDM_EXT_PATH=... for the other build).

    python tools/slab_compare.py B OUT [REF]
"""
import sys
import torch
sys.path.insert(0, ".")
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split  # noqa: E402
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices  # noqa: E402
from pytorch_distributed_mnist_amd.runtime.program import build_local_program  # noqa: E402

B, out = int(sys.argv[1]), sys.argv[2]
train = synthetic_split(max(600, 2 * B), True)
test = synthetic_split(300, False)
p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.0,
                        momentum=0.0, weight_decay=0.0, seed=0, use_graphs=False)
p.optimizer.sync_hyperparams()
st = p.gpu
st.keep_grads = True
p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
st.begin_epoch()
p.metrics.reset(0)
st.train_step(B)
torch.cuda.synchronize()
nb = st.C.cnn_bwd_nblk(B, 1 if st.bands(B) > 1 else __import__(
    "pytorch_distributed_mnist_amd.runtime.cnn_step", fromlist=["choose_ipb"]).choose_ipb(B),
    st.bands(B))
res = {"slab": st.conv_slab[:nb * st.C.CNN_CONV_SLAB].cpu().view(nb, -1)}
for n in ("conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias"):
    res[n] = st.G[n].detach().cpu().clone()
torch.save(res, out)
if len(sys.argv) > 3:
    ref = torch.load(sys.argv[3])
    for k, v in res.items():
        d = (v - ref[k]).abs()
        print(f"B={B} {k:13s} equal={torch.equal(v, ref[k])} max|diff|={d.max().item():.3e} "
              f"rel={(d.max() / ref[k].abs().max().clamp_min(1e-30)).item():.3e}")
