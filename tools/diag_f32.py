"""Diagnostic: where the fp32 CNN step's gradients depart from fp64 autograd (per stage).

    python tools/diag_f32.py [B]

Runs one lr = 0 step of the fp32 GPU program, then compares, stage by stage, the kernels'
intermediate buffers (pool, pool mask, dpool, conv gradients) with an fp64 torch model of the
same batch, printing the relative error of each and where the largest conv2 weight-gradient
errors sit (co, tap, ci).
"""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from pytorch_distributed_mnist_amd.data.mnist import normalize_reference, synthetic_split  # noqa
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices  # noqa: E402
from pytorch_distributed_mnist_amd.models.reference import MODULES  # noqa: E402
from pytorch_distributed_mnist_amd.runtime.program import build_local_program  # noqa: E402


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
train = synthetic_split(max(2 * B, 300), True)
test = synthetic_split(300, False)
prog = build_local_program("cnn", "fp32", "cuda", B, train, test, optimizer="sgd", lr=0.0,
                           momentum=0.0, weight_decay=0.0, seed=0, use_graphs=False)
prog.optimizer.sync_hyperparams()
idx = distributed_indices(len(train), 1, 0, 0)
prog.set_train_indices(idx)
net = MODULES["cnn"]()
net.load_state_dict({k[len("module."):]: v for k, v in prog.arena.state_dict().items()})
net = net.double()
prog.gpu.begin_epoch()
prog.gpu.train_step(B)
torch.cuda.synchronize()
st = prog.gpu
sel = idx[:B]
x = normalize_reference(train.images[sel]).view(B, 1, 28, 28).double()
a1 = F.relu(net.conv1(x))
z2 = net.conv2(a1)
a2 = F.relu(z2)
pooled, arg = F.max_pool2d(a2, 2, return_indices=True)
pooled.retain_grad()
z2.retain_grad()
h = F.relu(net.fc1(pooled.flatten(1)))
out = net.fc2(h)
F.cross_entropy(out, train.labels[sel]).backward()
# our pooled activations are NHWC ([B][12*12][64]); torch's are NCHW
ours_pool = st.pool[:B * 9216].view(B, 12, 12, 64).permute(0, 3, 1, 2).double().cpu()
print("pool rel err", rel(ours_pool, pooled.detach()))
ours_a1 = st.a1g.view(B, 26, 26, 32).permute(0, 3, 1, 2).double().cpu()
print("a1 rel err", rel(ours_a1, a1.detach()))
# mask: argmax positions
mk = st.pmask[:B * 9216].view(B, 12, 12, 64).permute(0, 3, 1, 2).cpu().long()
pos = (mk & 0x80) != 0
sidx = torch.where(pos, (mk & 0xf).float().log2().long(), torch.zeros_like(mk))
# torch argmax index in the 24x24 map -> window position
ty, tx = arg // 24, arg % 24
tpos = (ty % 2) * 2 + (tx % 2)
tref = pooled.detach() > 0
print("mask positive mismatches", int((pos != tref).sum()), "of", pos.numel())
both = pos & tref
print("argmax mismatches among positive", int((sidx[both] != tpos[both]).sum()))
ours_dp = st.dpool[:B * 9216].view(B, 12, 12, 64).permute(0, 3, 1, 2).double().cpu()
print("dpool rel err", rel(ours_dp, pooled.grad))
got = prog.arena.torch_tensors(prog.arena.grads)
for name, p in net.named_parameters():
    print(f"{name:14s} rel err vs fp64 {rel(got[name].double(), p.grad):.3e}")
gw = got["conv2.weight"].double()
err = (gw - net.conv2.weight.grad).abs()
top = err.flatten().topk(8)
for v, i in zip(top.values.tolist(), top.indices.tolist()):
    co, ci, ky, kx = i // 288, (i // 9) % 32, (i // 3) % 3, i % 3
    print(f"  |err| {v:.3e} at co {co} ci {ci} tap ({ky},{kx}); ref {net.conv2.weight.grad.flatten()[i].item():.3e}")
print("conv2.weight grad norm", net.conv2.weight.grad.norm().item(), "max |ref|",
      net.conv2.weight.grad.abs().max().item())
