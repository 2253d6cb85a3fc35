"""Per-role timing of fc1_bwd (PDM_FC1BWD_ROLE; needs a PDM_DIAG_ROLES=1 build via PDM_EXT_PATH) and of the optimizer launches at B=256."""
import os
import sys
import torch
sys.path.insert(0, ".")
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split  # noqa: E402
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices  # noqa: E402
from pytorch_distributed_mnist_amd.runtime.program import build_local_program  # noqa: E402
from pytorch_distributed_mnist_amd.runtime.cnn_step import conv_blocks  # noqa: E402
sys.path.insert(0, "tools")
from kbench import timeit  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
train = synthetic_split(60000, True)
test = synthetic_split(512, False)
p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.01, use_graphs=False)
p.optimizer.sync_hyperparams()
p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
st = p.gpu
C, P, G = st.C, st.P, st.G
ldt = -(-B // 32) * 32
st.train_step(B)
torch.cuda.synchronize()
role = os.environ.get("PDM_FC1BWD_ROLE", "all")
us = timeit(lambda: C.fc1_bwd(st.dh, st.dht, ldt, st.pool, st.current_wf1t(), B, G["fc1.weight"], st.dpool,
                              st.head_slab, G["fc2.weight"], G["fc2.bias"], G["fc1.bias"],
                              st.metrics.train_view(),
                              st._fc_update() if st.fuse_fc1 else None))
print(f"B={B} fc1_bwd role={role}: {us:.2f} us", flush=True)
if role == "all":
    nb = conv_blocks(C, B)
    print(f"optim fused: {timeit(lambda: st.launch_optimizer(st._fused_segments(nb))):.2f} us  "
          f"plain: {timeit(lambda: st.launch_optimizer()):.2f} us", flush=True)
