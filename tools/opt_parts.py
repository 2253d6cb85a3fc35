import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tools")
import torch
from kbench import timeit
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
from pytorch_distributed_mnist_amd.runtime.program import build_local_program
from pytorch_distributed_mnist_amd.runtime.cnn_step import conv_blocks
B = 256
train = synthetic_split(60000, True); test = synthetic_split(512, False)
p = build_local_program("cnn", "bf16", "cuda", B, train, test, optimizer="sgd", lr=0.01, use_graphs=False)
p.optimizer.sync_hyperparams(); p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
st = p.gpu; st.train_step(B); torch.cuda.synchronize()
segs = st._fused_segments(conv_blocks(st.C, B))
slab = [s for s in segs if len(s) > 5 and s[5] is not None]
tonly = [s for s in segs if len(s) > 6 and s[6]]
rest = [s for s in segs if s not in slab and s not in tonly]
for name, ss in (("all", segs), ("slab only", slab), ("tonly only", tonly), ("rest only", rest), ("slab+rest", slab + rest)):
    print(f"{name:12s} {timeit(lambda: st.launch_optimizer(ss)):.2f} us  ({len(ss)} segs)", flush=True)
