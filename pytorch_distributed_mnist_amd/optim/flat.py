"""Flat-arena Adam / SGD with torch-format ``state_dict``.

The reference uses ``torch.optim.Adam(model.parameters(), lr=args.lr)``
(``multi_proc_single_gpu.py:191``) and has SGD-with-momentum commented out
(``multi_proc_single_gpu.py:192-194``).  On a GPU, torch runs Adam as ~7
``_foreach_*`` launches per step with the bias corrections computed on the host
(SURVEY.md §2.2 N8).  Here one fused HIP kernel (``csrc/kernels/optim.hip``)
updates the whole flat arena:

* the DDP 1/world_size gradient scale is folded into the kernel (``grad_scale``),
* lr and the step count live in device memory, so the step is graph-capturable,
* in bf16 mode the same pass emits the bf16 compute copies of the weights in
  every layout the forward/backward kernels read (incl. transposed copies), so
  there is no separate cast/transpose kernel.

On CPU the same update is written with torch ops in torch's own op order, which
is what the CPU/gloo path runs and what tests compare the kernel against.

``state_dict()``/``load_state_dict()`` produce/consume exactly torch's format
(per-parameter ``exp_avg``/``exp_avg_sq``/``step`` or ``momentum_buffer`` in
torch layouts, and torch's param_group key set for the installed torch), so
checkpoints interoperate with the reference.
"""
from __future__ import annotations

import copy
from typing import Dict, List, Optional

import torch

from ..runtime.arena import FlatArena


def _torch_param_group_template(kind: str) -> dict:
    """The param_group dict torch itself would produce (exact key set/defaults)."""
    p = [torch.nn.Parameter(torch.zeros(1))]
    if kind == "adam":
        opt = torch.optim.Adam(p, lr=1e-3)
    else:
        opt = torch.optim.SGD(p, lr=1e-3, momentum=0.9)
    g = copy.deepcopy(opt.state_dict()["param_groups"][0])
    g.pop("params")
    return g


class FlatOptimizer:
    kind = "base"

    def __init__(self, arena: FlatArena, hyper: dict):
        self.arena = arena
        group = _torch_param_group_template(self.kind)
        group.update(hyper)
        self.param_groups: List[dict] = [group]
        self.step_count = 0
        device = arena.device
        # Device-resident hyper-parameters (fp64): [lr], and the step counter.
        self._lr_dev = torch.zeros(1, dtype=torch.float64, device=device)
        self._step_dev = torch.zeros(1, dtype=torch.int64, device=device)
        self._lr_synced: Optional[float] = None

    @property
    def lr(self) -> float:
        return float(self.param_groups[0]["lr"])

    def sync_hyperparams(self) -> None:
        """Push host-side lr (set by adjust_learning_rate) to the device scalar."""
        if self._lr_synced != self.lr:
            self._lr_dev.fill_(self.lr)
            self._lr_synced = self.lr

    def sync_step(self) -> None:
        self._step_dev.fill_(self.step_count)

    def _check_kind(self, sd: dict) -> None:
        """Refuse a torch optimizer state_dict written by the other optimizer kind."""
        group = sd["param_groups"][0]
        kind = "adam" if "betas" in group else ("sgd" if "dampening" in group else None)
        if kind is not None and kind != self.kind:
            raise ValueError(f"checkpoint holds {kind} optimizer state but --optimizer {self.kind} "
                             f"was selected; pass --optimizer {kind}")

    # subclasses: step(grad_scale), state buffers, (de)serialisation
    def state_buffers(self) -> Dict[str, torch.Tensor]:
        raise NotImplementedError

    def _freeze(self, frozen):
        """Save the [start, end) ranges of the parameters and optimizer state that this step
        must leave unchanged (another rank's shard); returns a restore function."""
        if not frozen:
            return lambda: None
        bufs = [self.arena.params, *self.state_buffers().values()]
        saved = [(b, s, e, b[s:e].clone()) for b in bufs for s, e in frozen if e > s]

        def restore():
            for b, s, e, v in saved:
                b[s:e].copy_(v)
        return restore

    def zero_grad(self, set_to_none: bool = True) -> None:
        # Gradients are overwritten (not accumulated) by the backward kernels,
        # so there is nothing to clear; kept for API parity with torch.optim.
        return None

    def _torch_groups(self) -> List[dict]:
        g = dict(self.param_groups[0])
        g["params"] = list(range(len(self.arena.spec.params)))
        return [g]


class FlatAdam(FlatOptimizer):
    kind = "adam"

    def __init__(self, arena: FlatArena, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        super().__init__(arena, {"lr": lr, "betas": tuple(betas), "eps": eps,
                                 "weight_decay": weight_decay})
        self.exp_avg = torch.zeros_like(arena.params)
        self.exp_avg_sq = torch.zeros_like(arena.params)

    def state_buffers(self):
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq}

    def step_cpu(self, grad_scale: float = 1.0, frozen=None) -> None:
        """torch ``_single_tensor_adam`` math on the flat buffers (CPU path)."""
        restore = self._freeze(frozen)
        self._adam_cpu(grad_scale)
        restore()

    def _adam_cpu(self, grad_scale):
        g0 = self.param_groups[0]
        beta1, beta2 = g0["betas"]
        lr, eps, wd = g0["lr"], g0["eps"], g0["weight_decay"]
        p, grad = self.arena.params, self.arena.grads
        if grad_scale != 1.0:
            grad = grad * grad_scale
        if wd != 0:
            grad = grad.add(p, alpha=wd)
        self.step_count += 1
        step = self.step_count
        self.exp_avg.lerp_(grad, 1 - beta1)
        self.exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
        bias_correction1 = 1 - beta1 ** step
        bias_correction2 = 1 - beta2 ** step
        step_size = lr / bias_correction1
        bias_correction2_sqrt = bias_correction2 ** 0.5
        denom = (self.exp_avg_sq.sqrt() / bias_correction2_sqrt).add_(eps)
        p.addcdiv_(self.exp_avg, denom, value=-step_size)

    def state_dict(self) -> dict:
        state = {}
        m = self.arena.torch_tensors(self.exp_avg)
        v = self.arena.torch_tensors(self.exp_avg_sq)
        if self.step_count > 0:
            for p in self.arena.spec.torch_order():
                state[p.torch_index] = {
                    "step": torch.tensor(float(self.step_count), dtype=torch.float32),
                    "exp_avg": m[p.name],
                    "exp_avg_sq": v[p.name],
                }
        return {"state": state, "param_groups": self._torch_groups()}

    def load_state_dict(self, sd: dict) -> None:
        self._check_kind(sd)
        group = sd["param_groups"][0]
        for k, v in group.items():
            if k != "params":
                self.param_groups[0][k] = tuple(v) if k == "betas" else v
        state = sd.get("state", {})
        if not state:
            self.step_count = 0
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            return
        by_index = {p.torch_index: p for p in self.arena.spec.params}
        m_named, v_named, steps = {}, {}, set()
        for idx, st in state.items():
            p = by_index[int(idx)]
            m_named[p.name] = st["exp_avg"]
            v_named[p.name] = st["exp_avg_sq"]
            steps.add(int(float(st["step"])))
        if len(steps) != 1:
            raise ValueError(f"per-parameter Adam steps differ: {sorted(steps)}")
        self.step_count = steps.pop()
        self.arena.buffer_from_torch(m_named, self.exp_avg)
        self.arena.buffer_from_torch(v_named, self.exp_avg_sq)


class FlatSGD(FlatOptimizer):
    kind = "sgd"

    def __init__(self, arena: FlatArena, lr: float, momentum: float = 0.0, weight_decay: float = 0.0,
                 dampening: float = 0.0, nesterov: bool = False):
        super().__init__(arena, {"lr": lr, "momentum": momentum, "weight_decay": weight_decay,
                                 "dampening": dampening, "nesterov": nesterov})
        self.momentum_buffer = torch.zeros_like(arena.params)

    def state_buffers(self):
        return {"momentum_buffer": self.momentum_buffer}

    def step_cpu(self, grad_scale: float = 1.0, frozen=None) -> None:
        """torch ``_single_tensor_sgd`` math on the flat buffers (CPU path)."""
        restore = self._freeze(frozen)
        self._sgd_cpu(grad_scale)
        restore()

    def _sgd_cpu(self, grad_scale):
        g0 = self.param_groups[0]
        lr, mom, wd = g0["lr"], g0["momentum"], g0["weight_decay"]
        damp, nesterov = g0["dampening"], g0["nesterov"]
        p, d_p = self.arena.params, self.arena.grads
        if grad_scale != 1.0:
            d_p = d_p * grad_scale
        if wd != 0:
            d_p = d_p.add(p, alpha=wd)
        if mom != 0:
            buf = self.momentum_buffer
            if self.step_count == 0:
                buf.copy_(d_p)
            else:
                buf.mul_(mom).add_(d_p, alpha=1 - damp)
            d_p = d_p.add(buf, alpha=mom) if nesterov else buf
        p.add_(d_p, alpha=-lr)
        self.step_count += 1

    def state_dict(self) -> dict:
        state = {}
        if self.step_count > 0 and self.param_groups[0]["momentum"] != 0:
            b = self.arena.torch_tensors(self.momentum_buffer)
            for p in self.arena.spec.torch_order():
                state[p.torch_index] = {"momentum_buffer": b[p.name]}
        return {"state": state, "param_groups": self._torch_groups()}

    def load_state_dict(self, sd: dict) -> None:
        self._check_kind(sd)
        group = sd["param_groups"][0]
        for k, v in group.items():
            if k != "params":
                self.param_groups[0][k] = v
        state = sd.get("state", {})
        by_index = {p.torch_index: p for p in self.arena.spec.params}
        named = {}
        for idx, st in state.items():
            if "momentum_buffer" in st and st["momentum_buffer"] is not None:
                named[by_index[int(idx)].name] = st["momentum_buffer"]
        if named:
            self.arena.buffer_from_torch(named, self.momentum_buffer)
            self.step_count = max(self.step_count, 1)
        else:
            self.momentum_buffer.zero_()
            self.step_count = 0


def build_optimizer(name: str, arena: FlatArena, args) -> FlatOptimizer:
    if name == "adam":
        return FlatAdam(arena, lr=args.lr)
    if name == "sgd":
        return FlatSGD(arena, lr=args.lr, momentum=args.momentum, weight_decay=args.weight_decay)
    raise ValueError(f"unknown optimizer {name!r}")


def adjust_learning_rate(optimizer, epoch: int, args) -> None:
    """Step decay: lr = lr0 * 0.1 ** (epoch // 10)  (reference ``multi_proc_single_gpu.py:257-261``)."""
    lr = args.lr * (0.1 ** (epoch // 10))
    for param_group in optimizer.param_groups:
        param_group["lr"] = lr
