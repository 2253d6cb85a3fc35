"""Multi-rank worker for the fc1 optimizer-state sharding test (tests/test_gpu_shard.py).

Launched with ``torch.distributed.run --nproc-per-node N`` and PDM_SHARE_DEVICE=1: every rank
on device 0 over a gloo data plane (TorchComm), the multi-rank GPU setup a one-GPU box allows.
The CNN trains two epochs replicated (every rank updates all of fc1) and again from the same
init with the fc1 update sharded (CnnStep.set_shard_fc: each rank updates its 128/N rows, the
bf16 W1 rows are all-gathered); after sync_master() the parameters and momentum must be
bit-identical to the replicated run on every rank.  Writes $PDM_SHARD_OUT/rank<r>.json.
"""
import json
import os
import sys
from types import SimpleNamespace

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def train(comm, dev, rank, ws, shard, graphs):
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
    from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
    from pytorch_distributed_mnist_amd.models.reference import MODULES
    from pytorch_distributed_mnist_amd.models.specs import get_spec
    from pytorch_distributed_mnist_amd.optim.flat import build_optimizer
    from pytorch_distributed_mnist_amd.parallel.reducer import GradReducer
    from pytorch_distributed_mnist_amd.runtime.arena import FlatArena
    from pytorch_distributed_mnist_amd.runtime.program import TrainProgram
    torch.manual_seed(1234)
    spec = get_spec("cnn")
    arena = FlatArena(spec, dev)
    arena.load_module(MODULES["cnn"]())
    opt = build_optimizer("sgd", arena, SimpleNamespace(lr=0.05, momentum=0.9, weight_decay=1e-4))
    red = GradReducer(comm, arena.grads, spec.bucket_bounds(), transport="rccl")
    train_split = synthetic_split(64 * ws * 5 + 24, True)
    prog = TrainProgram("cnn", "bf16", arena, opt, red, train_split, synthetic_split(256, False),
                        64, use_graphs=graphs)
    if shard:
        prog.gpu.set_shard_fc(True)
    opt.sync_hyperparams()
    for epoch in range(2):
        prog.set_train_indices(distributed_indices(len(train_split), ws, rank, epoch))
        prog.train_epoch()
    el, ea = prog.evaluate()                 # reads the gathered bf16 W1
    prog.sync_master()
    torch.cuda.synchronize()
    return (arena.params.clone(), opt.momentum_buffer.clone(), red.kind,
            (el.average, ea.correct))


def main():
    from pytorch_distributed_mnist_amd.parallel.comm import TorchComm
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", init_method="env://", world_size=ws, rank=rank)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = TorchComm()
    p0, m0, k0, e0 = train(comm, dev, rank, ws, False, False)
    p1, m1, k1, e1 = train(comm, dev, rank, ws, True, False)
    # replicas: every rank holds the same full state after the gathers
    parts = [torch.zeros_like(p1.cpu()) for _ in range(ws)]
    dist.all_gather(parts, p1.cpu())
    out = {"kinds": [k0, k1], "params_equal": bool(torch.equal(p0, p1)),
           "momentum_equal": bool(torch.equal(m0, m1)),
           "max_param_diff": float((p0 - p1).abs().max()),
           "replicas_equal": all(torch.equal(parts[0], q) for q in parts[1:]),
           "eval_equal": e0 == e1, "eval": [e0, e1]}
    with open(os.path.join(os.environ["PDM_SHARD_OUT"], f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
