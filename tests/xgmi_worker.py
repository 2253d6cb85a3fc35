"""Multi-rank worker for the xGMI transport tests (tests/test_gpu_xgmi.py).

Launched with ``torch.distributed.run --nproc-per-node N`` and PDM_SHARE_DEVICE=1:
every rank sits on device 0 over a gloo control plane — the only multi-rank GPU
setup a one-GPU box allows (RCCL refuses two ranks on one device; hipIpc between
processes on one device is allowed).  The peer mappings, flag protocol, one-shot
and two-shot schedules and the graph capture are the same code that runs over
xGMI between GPUs.  Writes one JSON file per rank into $PDM_XGMI_OUT.
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

FC, CONV = 1181120, 18880          # the CNN's bucket sizes (floats)
_LOG = None


def log(msg):
    """Progress line into $PDM_XGMI_LOG_DIR/rank<r>.log (diagnosis of a stuck rank)."""
    if _LOG is not None:
        _LOG.write(msg + "\n")
        _LOG.flush()


def rank_order_sum(data, ws):
    parts = [torch.zeros_like(data) for _ in range(ws)]
    dist.all_gather(parts, data)
    want = parts[0].clone()
    for p in parts[1:]:
        want += p
    return want


PREFLIGHT = []


def check_collective(comm, dev, rank, ws, mode):
    from pytorch_distributed_mnist_amd.parallel.reducer import GradReducer
    os.environ["PDM_XGMI_MODE"] = mode
    n = FC + CONV
    grads = torch.zeros(n, device=dev)
    red = GradReducer(comm, grads, [(0, FC), (FC, n)], transport="xgmi")
    assert red.kind == "xgmi", red.kind
    gen = torch.Generator().manual_seed(100 + rank)
    ok = True
    log(f"{mode}: reducer up {red._xgmi.describe} (pre-flight {red._xgmi.preflight})")
    PREFLIGHT.append(red._xgmi.preflight)
    for _ in range(4):                                   # eager, bucket by bucket
        data = torch.randn(n, generator=gen)
        want = rank_order_sum(data, ws)
        grads.copy_(data.to(dev))
        red.bucket_ready(0)
        red.bucket_ready(1)
        red.finalize()
        torch.cuda.synchronize()
        ok = ok and torch.equal(red.out_grads.cpu(), want)
        log(f"{mode}: eager ok={ok} err={red._xgmi.native.error()}")
    # captured: 3 all-reduces per replay, data changed by a captured kernel in between
    g = torch.cuda.CUDAGraph()
    scale = torch.ones(1, device=dev)
    with torch.cuda.graph(g):
        for _ in range(3):
            grads.mul_(scale)
            red.all_ready()
            red.finalize()
    for it in range(3):
        data = torch.randn(n, generator=gen)
        want = rank_order_sum(data * (2.0 ** (it + 1)) ** 3, ws)
        grads.copy_(data.to(dev))
        scale.fill_(2.0 ** (it + 1))
        g.replay()
        torch.cuda.synchronize()
        ok = ok and torch.equal(red.out_grads.cpu(), want)
    log(f"{mode}: graph ok={ok}")
    red.check()
    desc = red._xgmi.describe
    red.close()
    return bool(ok), [d["mode"] for d in desc]


def exchange_unit(comm, dev, rank, ws):
    """The optimizer's in-launch exchange of the conv bucket alone (slab segments only,
    lr = 0), the part of the streamed CNN step that ranks sharing ONE GPU cannot run inside a
    whole step (a spinning optimizer grid would keep the peer's cnn_bwd, which needs a whole
    CU, off the device): the gradients it leaves in the result arena must equal the rank-order
    sum of every rank's slab sums -- eager calls (both stage parities) and graph replays."""
    from pytorch_distributed_mnist_amd.ops import _ext
    from pytorch_distributed_mnist_amd.parallel.reducer import GradReducer
    C = _ext.require()
    n = FC + CONV
    grads = torch.zeros(n, device=dev)
    red = GradReducer(comm, grads, [(0, FC), (FC, n)], transport="xgmi")
    assert red.kind == "xgmi"
    SL, nslab = C.CNN_CONV_SLAB, 6
    cols = torch.arange(SL, dtype=torch.float32)
    base = torch.stack([((cols % 97) - 48) * (rank + 1) + j for j in range(nslab)])   # exact sums
    slab = base.reshape(-1).to(dev).contiguous()
    params = torch.zeros(n, device=dev)
    mom = torch.zeros(n, device=dev)
    lr = torch.zeros(1, dtype=torch.float64, device=dev)
    step = torch.ones(1, dtype=torch.int64, device=dev)
    # (arena offset, rows, cols, slab column) of conv2.weight / .bias, conv1.weight / .bias
    parts = [(FC, 64, 288, 0), (FC + 18432, 1, 64, C.CNN_CONV_SLAB_DB2),
             (FC + 18496, 1, 288, C.CNN_CONV_SLAB_DW1), (FC + 18816, 1, 32, C.CNN_CONV_SLAB_DB1)]
    segs = [(off, r, c, None, None, (slab, nslab, col0, SL)) for off, r, c, col0 in parts]

    def launch():
        C.optim_step(C.OPT_SGD, params, red.out_grads, mom, None, lr, step, 0.0, 0.0, 0.0, 0.0,
                     0.0, 0.0, False, 1.0, segs, xg=red.sync, signal_ch=-1,
                     waits=red.waits_for(segs, exchanged=(1,)), timeout_s=red.timeout_s,
                     xchg=red._native, xchg_bucket=1)

    def expected(scale):
        mine = (base * scale).sum(0)                   # this rank's slab sums, per column
        tot = rank_order_sum(mine, ws)
        want = torch.full((CONV,), float("nan"))     # nan: padding, not compared
        for off, r, c, col0 in parts:
            want[off - FC:off - FC + r * c] = tot[col0:col0 + r * c]
        return want

    ok = True
    info = []

    def check(tag, scale):
        got, want = red.out_grads[FC:n].cpu(), expected(scale)
        seg = ~torch.isnan(want)
        good = torch.equal(got[seg], want[seg])
        if not good:
            bad = ((got != want) & seg).nonzero().flatten()
            i = int(bad[0])
            info.append(f"{tag}: {bad.numel()} wrong, first at {i}: got {float(got[i])} "
                        f"want {float(want[i])} (err {red._xgmi.native.error()})")
        return good

    for it in range(3):                               # eager: both stage parities, twice
        slab.copy_((base * (it + 1)).reshape(-1).to(dev))
        launch()
        torch.cuda.synchronize()
        ok = check(f"eager {it}", it + 1) and ok
        log(f"xchg eager {it} ok={ok}")
    scale = torch.ones(1, device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(3):
            slab.mul_(scale)
            launch()
    for it in range(2):
        slab.copy_(base.reshape(-1).to(dev))
        scale.fill_(2.0)
        g.replay()
        torch.cuda.synchronize()
        ok = check(f"graph {it}", 8.0) and ok
        log(f"xchg graph {it} ok={ok}")
    red.check()
    red.close()
    return {"xchg_ok": bool(ok), "xchg_info": info}


def train_model(arch, comm, dev, rank, ws, transport):
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
    from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
    from pytorch_distributed_mnist_amd.models.reference import MODULES
    from pytorch_distributed_mnist_amd.models.specs import get_spec
    from pytorch_distributed_mnist_amd.optim.flat import build_optimizer
    from pytorch_distributed_mnist_amd.parallel.reducer import GradReducer
    from pytorch_distributed_mnist_amd.runtime.arena import FlatArena
    from pytorch_distributed_mnist_amd.runtime.program import TrainProgram
    os.environ["PDM_XGMI_MODE"] = "auto"
    torch.manual_seed(1234)
    spec = get_spec(arch)
    arena = FlatArena(spec, dev)
    arena.load_module(MODULES[arch]())
    cnn = arch == "cnn"
    opt = build_optimizer("sgd" if cnn else "adam", arena,
                          SimpleNamespace(lr=0.05 if cnn else 1e-3, momentum=0.9, weight_decay=1e-4))
    red = GradReducer(comm, arena.grads, spec.bucket_bounds(), transport=transport)
    train = synthetic_split(128 * ws * 9 + 40, True)   # 9 steps: graphs of 8 and 1 (the test sets 8)
    test = synthetic_split(256, False)
    prog = TrainProgram(arch, "bf16" if cnn else "fp32", arena, opt, red, train, test, 128,
                        use_graphs=True)
    opt.sync_hyperparams()
    for epoch in range(2):
        prog.set_train_indices(distributed_indices(len(train), ws, rank, epoch))
        prog.train_epoch()
        log(f"{arch} {transport}: epoch {epoch} done")
    torch.cuda.synchronize()
    red.check()
    kind = red.kind
    out = arena.params.clone()
    red.close()
    return out, kind


def absent_peer(comm, dev, rank, ws):
    """Rank 0 runs eager all-reduces that no other rank joins: the first wait gives up
    at the deadline, every later one fails fast on the error word."""
    import time
    from pytorch_distributed_mnist_amd.parallel.reducer import GradReducer
    os.environ["PDM_XGMI_MODE"] = "auto"
    n = FC + CONV
    grads = torch.ones(n, device=dev)
    red = GradReducer(comm, grads, [(0, FC), (FC, n)], transport="xgmi")
    out = {}
    if rank == 0:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(6):
            red.bucket_ready(0)
            red.bucket_ready(1)
            red.finalize()
        torch.cuda.synchronize()
        out["elapsed_s"] = time.perf_counter() - t0
        out["error"] = int(red._xgmi.native.error()) if hasattr(red, "_xgmi") else -1
        try:
            red.check()
            out["check_raised"] = False
        except RuntimeError:
            out["check_raised"] = True
    dist.barrier()                     # peers keep their mappings until rank 0 is done
    red.close()
    return out


def absent_peer_streamed(comm, dev, rank, ws):
    """Streamed mode (the default): rank 0 trains CNN steps whose persistent collective
    never sees its peer.  The collective's first phase-0 wait gives up at the deadline;
    the optimizer-side waits of every later step and the persistent kernel's READY
    waits fail fast on the error word, so the whole run costs about one timeout."""
    import time
    from pytorch_distributed_mnist_amd.data.mnist import synthetic_split
    from pytorch_distributed_mnist_amd.data.sampler import distributed_indices
    from pytorch_distributed_mnist_amd.models.reference import MODULES
    from pytorch_distributed_mnist_amd.models.specs import get_spec
    from pytorch_distributed_mnist_amd.optim.flat import build_optimizer
    from pytorch_distributed_mnist_amd.parallel.reducer import GradReducer
    from pytorch_distributed_mnist_amd.runtime.arena import FlatArena
    from pytorch_distributed_mnist_amd.runtime.program import TrainProgram
    os.environ["PDM_XGMI_MODE"] = "auto"
    spec = get_spec("cnn")
    arena = FlatArena(spec, dev)
    arena.load_module(MODULES["cnn"]())
    red = GradReducer(comm, arena.grads, spec.bucket_bounds(), transport="xgmi")
    out = {"streamed": bool(red.streamed)}
    if rank == 0:
        opt = build_optimizer("sgd", arena, SimpleNamespace(lr=0.05, momentum=0.9,
                                                            weight_decay=1e-4))
        train = synthetic_split(64 * 40, True)
        prog = TrainProgram("cnn", "bf16", arena, opt, red, train, synthetic_split(64, False),
                            64, use_graphs=True)
        opt.sync_hyperparams()
        prog.set_train_indices(distributed_indices(len(train), 1, 0, 0))
        prog.gpu.prepare(64)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        prog.gpu.train_steps(64, 2 * prog.gpu.GRAPH_STEPS + 3)     # two full graphs and one of 3 steps
        torch.cuda.synchronize()
        out["elapsed_s"] = time.perf_counter() - t0
        out["error"] = int(red._xgmi.native.error())
        out["first_error"] = int(red._xgmi.native.first_error())
        try:
            red.check()
            out["check_raised"] = False
        except RuntimeError as e:
            out["check_raised"] = True
            out["message"] = str(e)
    dist.barrier()                     # peers keep their mappings until rank 0 is done
    red.close()
    return out


def main():
    global _LOG
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if os.environ.get("PDM_XGMI_LOG_DIR"):
        os.makedirs(os.environ["PDM_XGMI_LOG_DIR"], exist_ok=True)
        _LOG = open(os.path.join(os.environ["PDM_XGMI_LOG_DIR"], f"rank{rank}.log"), "w")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from pytorch_distributed_mnist_amd.parallel.comm import TorchComm
    comm = TorchComm()
    res = {"rank": rank}
    absent = os.environ.get("PDM_XGMI_ABSENT")
    if os.environ.get("PDM_XGMI_UNIT") == "xchg":
        res.update(exchange_unit(comm, dev, rank, ws))
        with open(os.path.join(os.environ["PDM_XGMI_OUT"], f"rank{rank}.json"), "w") as f:
            json.dump(res, f)
        dist.destroy_process_group()
        return
    if absent in ("1", "streamed"):
        res.update(absent_peer(comm, dev, rank, ws) if absent == "1" else
                   absent_peer_streamed(comm, dev, rank, ws))
        with open(os.path.join(os.environ["PDM_XGMI_OUT"], f"rank{rank}.json"), "w") as f:
            json.dump(res, f)
        dist.destroy_process_group()
        return
    for mode in ("one", "two", "auto"):
        ok, modes = check_collective(comm, dev, rank, ws, mode)
        res[mode] = ok
        res[mode + "_modes"] = modes
    res["preflight"] = PREFLIGHT
    p_x, kind_x = train_model("cnn", comm, dev, rank, ws, "xgmi")
    p_g, kind_g = train_model("cnn", comm, dev, rank, ws, None)       # gloo data plane
    res["cnn_kinds"] = [kind_x, kind_g]
    res["cnn_max_diff"] = float((p_x - p_g).abs().max())
    res["cnn_equal"] = bool(torch.equal(p_x, p_g))
    # every rank holds the same replica
    parts = [torch.zeros_like(p_x.cpu()) for _ in range(ws)]
    dist.all_gather(parts, p_x.cpu())
    res["replicas_equal"] = all(torch.equal(parts[0], q) for q in parts[1:])
    # the reference Net (Linear, fp32, Adam): lin_train -> lin_reduce -> all-reduce -> optim
    l_x, lkind_x = train_model("linear", comm, dev, rank, ws, "xgmi")
    l_g, lkind_g = train_model("linear", comm, dev, rank, ws, None)
    res["lin_kinds"] = [lkind_x, lkind_g]
    res["lin_max_diff"] = float((l_x - l_g).abs().max())
    res["lin_equal"] = bool(torch.equal(l_x, l_g))
    parts = [torch.zeros_like(l_x.cpu()) for _ in range(ws)]
    dist.all_gather(parts, l_x.cpu())
    res["lin_replicas_equal"] = all(torch.equal(parts[0], q) for q in parts[1:])
    with open(os.path.join(os.environ["PDM_XGMI_OUT"], f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
