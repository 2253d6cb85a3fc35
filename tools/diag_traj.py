"""Diagnostic: GPU (bf16) vs CPU (fp32) CNN parameter trajectories, step by step."""
import sys
import torch
sys.path.insert(0, ".")
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
from pytorch_distributed_mnist_amd.runtime.program import build_local_program

train = synthetic_split(4096 + 64, True)
test = synthetic_split(1000, False)
for opt, lr, mom in (("sgd", 0.05, 0.0), ("sgd", 0.05, 0.9)):
    progs = {}
    for dev, dt in (("cpu", "fp32"), ("cuda", "bf16")):
        p = build_local_program("cnn", dt, dev, 256, train, test, optimizer=opt, lr=lr, momentum=mom,
                                weight_decay=1e-4, seed=3, use_graphs=False)
        p.optimizer.sync_hyperparams()
        p.set_train_indices(distributed_indices(len(train), 1, 0, 0))
        if p.gpu is not None:
            p.gpu.begin_epoch()
        progs[dev] = p
    pc, pg = progs["cpu"], progs["cuda"]
    from pytorch_distributed_mnist_amd.runtime.cpu_step import train_step_cpu
    for step in range(17):
        B = 256 if step < 16 else 64
        idx = pc.train_idx_cpu[step * 256: step * 256 + B]
        train_step_cpu("cnn", pc.arena, train.images[idx], train.labels[idx], pc.reducer,
                       pc.optimizer, pc.metrics.buf[0:3])
        pg.gpu.train_step(B)
        torch.cuda.synchronize()
        gc = pc.arena.torch_tensors(pc.arena.grads)
        gg = pg.arena.torch_tensors(pg.arena.grads.cpu())
        wc = pc.arena.torch_tensors(pc.arena.params)
        wg = pg.arena.torch_tensors(pg.arena.params.cpu())
        gr = {k: ((gc[k] - gg[k]).norm() / gc[k].norm()).item() for k in gc}
        wr = {k: ((wc[k] - wg[k]).norm() / wc[k].norm()).item() for k in wc}
        print(opt, mom, "step", step, "grad rel", {k: round(v, 4) for k, v in gr.items()})
        print("      param rel", {k: round(v, 5) for k, v in wr.items()})
    el, ea = pc.evaluate(); gl, ga = pg.evaluate()
    print("eval cpu", el, ea, "gpu", gl, ga, "train", pc.metrics.buf[0].item()/pc.metrics.buf[2].item(), pg.metrics.buf[0].item()/max(1,pg.metrics.buf[2].item()))
