"""CPU execution of one training / eval step (the gloo plumbing path and the oracle).

Semantics are the reference Trainer's (``multi_proc_single_gpu.py:77-116``):
normalise the gathered uint8 batch, forward, ``F.cross_entropy`` (mean), backward,
then optimizer step.  Parameters are taken from the flat arena in kernel
layout and exposed to autograd through the (permuting) torch-layout views, so
the gradients land in kernel layout directly in the gradient arena.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..data.mnist import normalize_reference
from ..models.reference import functional_forward


def _leaf_params(arena):
    leaves, torch_views = {}, {}
    for p in arena.spec.params:
        leaf = arena.param(p.name).detach().requires_grad_(True)
        leaves[p.name] = leaf
        torch_views[p.name] = p.to_torch(leaf)
    return leaves, torch_views


def train_step_cpu(model: str, arena, images_u8, labels, reducer, optimizer, metrics_buf):
    x = normalize_reference(images_u8)
    with torch.enable_grad():
        leaves, views = _leaf_params(arena)
        logits = functional_forward(model, views, x)
        loss = F.cross_entropy(logits, labels)
        names = [p.name for p in arena.spec.params]
        grads = torch.autograd.grad(loss, [leaves[n] for n in names])
    with torch.no_grad():
        for n, g in zip(names, grads):
            arena.grad(n).copy_(g)
        # buckets become ready in arena (backward) order; on CPU the all-reduces
        # are issued async and joined before the optimizer, like the GPU path.
        for b in range(reducer.num_buckets):
            reducer.bucket_ready(b)
        reducer.finalize()
        sh = getattr(reducer, "shard", None)
        if sh is None:
            optimizer.step_cpu(grad_scale=reducer.grad_scale)
        else:
            # sharded fc1 update: this rank's rows only (the other rows and their optimizer
            # state are left as they are), then every rank's updated rows all-gathered
            _, start, count = sh
            ws, r = reducer.comm.world_size, reducer.comm.rank
            own = (start + r * count, start + (r + 1) * count)
            frozen = [(start, own[0]), (own[1], start + ws * count)]
            optimizer.step_cpu(grad_scale=reducer.grad_scale, frozen=frozen)
            reducer.gather(arena.params[start:start + ws * count])
        bsz = images_u8.shape[0]
        correct = logits.argmax(dim=1).eq(labels).sum().item()
        metrics_buf[0] += loss.item() * bsz
        metrics_buf[1] += correct
        metrics_buf[2] += bsz


@torch.no_grad()
def eval_step_cpu(model: str, arena, images_u8, labels, metrics_buf):
    x = normalize_reference(images_u8)
    views = {p.name: p.to_torch(arena.param(p.name)) for p in arena.spec.params}
    logits = functional_forward(model, views, x)
    loss = F.cross_entropy(logits, labels)
    bsz = images_u8.shape[0]
    metrics_buf[0] += loss.item() * bsz
    metrics_buf[1] += logits.argmax(dim=1).eq(labels).sum().item()
    metrics_buf[2] += bsz
