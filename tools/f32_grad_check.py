"""One fp32 training step (lr = 0) per configuration; relative error of every parameter's
gradient against fp64 autograd of the same step (pool routed by the kernel's own argmax).
Diagnostic companion of tests/test_gpu_cnn_f32.py (prints all parameters instead of stopping
at the first failure).

    [PDM_F32_UPW=n] python tools/f32_grad_check.py B [x3|exact]
"""
import os
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_gpu_cnn_f32 import _fp64_grads_with_mask, _program, _reference_net, rel  # noqa: E402
from pytorch_distributed_mnist_amd.data.mnist import normalize_reference  # noqa: E402
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
mode = sys.argv[2] if len(sys.argv) > 2 else "x3"
prog, train, _ = _program(B, n=max(2 * B, 300))
prog.gpu.conv_x3 = mode == "x3"
idx = distributed_indices(len(train), 1, 0, 0)
prog.set_train_indices(idx)
net = _reference_net(prog)
prog.gpu.begin_epoch()
prog.gpu.train_step(B)
torch.cuda.synchronize()
sel = idx[:B]
x = normalize_reference(train.images[sel]).view(B, 1, 28, 28)
ref64, out64 = _fp64_grads_with_mask(prog, x, train.labels[sel], prog.gpu.pmask, B)
got = prog.arena.torch_tensors(prog.arena.grads)
print(f"B={B} mode={mode} PDM_F32_UPW={os.environ.get('PDM_F32_UPW')}")
for name, p in ref64.items():
    print(f"  {name:14s} rel {rel(got[name].double(), p.grad):.3e}")
