"""The reference's training loop, run as-is in PyTorch eager on MI355X (the number to beat).

BASELINE.md asks for the reference itself measured on MI355X, with the CNN swapped in for the
CNN metric.  The reference cannot run unmodified here (torchvision is absent and there is no
network), so this tool reproduces its per-step behaviour with plain PyTorch:

  * data: a map-style dataset of uint8 28x28 images whose __getitem__ does what
    ToTensor + Normalize((0.1307,), (0.3081,)) does (reference S:132-138), served by a
    torch DataLoader with --workers worker processes and a DistributedSampler
    (reference S:142-157; pin_memory False as in S:151-156);
  * step: .cuda() of data and target, forward, F.cross_entropy, zero_grad, backward,
    optimizer.step, loss.item() and the argmax/eq/sum/.item() accuracy (reference S:77-97,
    S:61-62);
  * model: DDP (RCCL) around the SURVEY.md §7.1 CNN in fp32 (the reference computes in fp32);
    optimizer SGD momentum 0.9 / wd 1e-4 / lr 0.01 as bench.py (or Adam, reference S:191).

    python tools/reference_eager.py [--steps K] [--warmup W] [--batch 256] [--workers 4]
    python -m torch.distributed.run --nproc-per-node N ... tools/reference_eager.py

`--loader device` swaps the DataLoader for device-resident normalised tensors indexed per
step (a stronger eager baseline than the reference's own data path).  `--loader graph` is the
strongest plain-PyTorch version of the same step: device-resident data, the batch gathered by a
device-side step counter, no per-step .item() (loss / correct accumulated on the device), the
whole step (gather, forward, loss, backward, SGD/Adam) captured once into a torch.cuda.graph
(hipGraph) and replayed; `--amp bf16` runs it under torch.autocast(bfloat16) with fp32
master weights (this framework's bf16 configuration).  With --loader graph the single-GPU run
uses no DDP wrapper (nothing to reduce).  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_mnist_amd.data.mnist import synthetic_split  # noqa: E402
from pytorch_distributed_mnist_amd.models.reference import CNN, Net  # noqa: E402


class NormalizedMNIST(torch.utils.data.Dataset):
    """uint8 images -> fp32 [1,28,28] normalised per sample (ToTensor + Normalize)."""

    def __init__(self, images, labels):
        self.images = images.view(-1, 1, 28, 28)
        self.labels = labels

    def __len__(self):
        return self.images.shape[0]

    def __getitem__(self, i):
        x = self.images[i].float().div_(255.0)
        x = (x - 0.1307) / 0.3081
        return x, int(self.labels[i])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch", type=int, default=256, help="per-rank batch")
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--model", choices=["cnn", "linear"], default="cnn")
    ap.add_argument("--optimizer", choices=["sgd", "adam"], default="sgd")
    ap.add_argument("--loader", choices=["dataloader", "device", "graph"], default="dataloader")
    ap.add_argument("--amp", choices=["none", "bf16"], default="none",
                    help="--loader graph: torch.autocast(bfloat16) over forward + loss")
    ap.add_argument("--train-size", type=int, default=60000)
    a = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist.init_process_group("nccl", rank=rank, world_size=ws)

    torch.manual_seed(1234)
    model = (CNN() if a.model == "cnn" else Net()).to(dev)
    if a.loader == "graph":
        return graph_loop(a, model, dev, rank, ws)
    model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local_rank])
    if a.optimizer == "sgd":
        opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    torch.backends.cudnn.benchmark = True          # reference S:216

    split = synthetic_split(a.train_size, True)
    ds = NormalizedMNIST(split.images, split.labels)
    sampler = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=ws, rank=rank)

    def batches():
        epoch = 0
        while True:
            sampler.set_epoch(epoch)
            if a.loader == "dataloader":
                loader = torch.utils.data.DataLoader(ds, batch_size=a.batch, sampler=sampler,
                                                     num_workers=a.workers, pin_memory=False)
                yield from loader
            else:
                idx = torch.tensor(list(iter(sampler)), dtype=torch.long, device=dev)
                for s in range(0, idx.numel(), a.batch):
                    j = idx[s:s + a.batch]
                    yield x_dev[j], y_dev[j]
            epoch += 1

    if a.loader == "device":
        x_dev = ((split.images.to(dev).float() / 255.0 - 0.1307) / 0.3081).view(-1, 1, 28, 28)
        y_dev = split.labels.to(dev)
    it = batches()
    model.train()
    seen = correct_total = 0

    def step():
        nonlocal seen, correct_total
        data, target = next(it)
        data, target = data.cuda(dev), target.cuda(dev)
        output = model(data)
        loss = F.cross_entropy(output, target)
        opt.zero_grad()
        loss.backward()
        opt.step()
        _ = loss.item()
        correct_total += output.argmax(1).eq(target).sum().item()
        seen += output.size(0)
        return data.size(0)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    imgs = 0
    for _ in range(a.steps):
        imgs += step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    t = torch.tensor([el, float(imgs)], dtype=torch.float64, device=dev)
    tmax = t[:1].clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
    el, total = float(tmax.item()), float(t[1].item())
    if rank == 0:
        print(json.dumps({
            "what": "reference training loop in PyTorch eager (DDP/RCCL, fp32)",
            "model": a.model, "optimizer": a.optimizer, "loader": a.loader,
            "workers": a.workers, "n_gpus": ws, "batch_per_rank": a.batch,
            "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 4),
            "images_per_sec": round(total / el, 1),
        }), flush=True)
    dist.destroy_process_group()


def graph_loop(a, model, dev, rank, ws):
    """Device-resident data + whole-step torch.cuda.graph capture (+ optional bf16 autocast)."""
    if ws > 1:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index])
    if a.optimizer == "sgd":
        opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, capturable=True)
    split = synthetic_split(a.train_size, True)
    x_dev = ((split.images.to(dev).float() / 255.0 - 0.1307) / 0.3081).view(-1, 1, 28, 28)
    y_dev = split.labels.to(dev)
    n = x_dev.shape[0]
    per_rank = n // ws
    steps_per_epoch = per_rank // a.batch
    g = torch.Generator(device="cpu")
    g.manual_seed(0)
    perm = torch.randperm(n, generator=g)[rank:per_rank * ws:ws].to(dev)   # DistributedSampler-like
    ctr = torch.zeros((), dtype=torch.long, device=dev)
    ar = torch.arange(a.batch, device=dev)
    loss_sum = torch.zeros((), dtype=torch.float32, device=dev)
    correct = torch.zeros((), dtype=torch.long, device=dev)
    amp = a.amp == "bf16"

    def step():
        idx = perm[(ctr % steps_per_epoch) * a.batch + ar]
        x, y = x_dev[idx], y_dev[idx]
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = model(x)
            loss = F.cross_entropy(out, y)
        opt.zero_grad(set_to_none=False)
        loss.backward()
        opt.step()
        loss_sum.add_(loss.detach().float() * a.batch)
        correct.add_(out.argmax(1).eq(y).sum())
        ctr.add_(1)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):                 # warm up (optimizer state, autograd buffers)
            step()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    opt.zero_grad(set_to_none=False)
    with torch.cuda.graph(graph):
        step()
    for _ in range(a.warmup):
        graph.replay()
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        graph.replay()
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if ws > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    if rank == 0:
        print(json.dumps({
            "what": "the same CNN step in PyTorch: device-resident data, whole step captured in "
                    "a torch.cuda.graph" + (", bf16 autocast" if amp else ", fp32"),
            "model": a.model, "optimizer": a.optimizer, "loader": "graph", "amp": a.amp,
            "n_gpus": ws, "batch_per_rank": a.batch, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 4),
            "images_per_sec": round(a.steps * a.batch * ws / el, 1),
            "train_loss_mean": round(float(loss_sum.item()) / max(1, int(ctr.item()) * a.batch), 4),
        }), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
