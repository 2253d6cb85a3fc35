"""Command-line surface.

Every reference flag is kept with its default (reference
``multi_proc_single_gpu.py:289-334``).  ``--local_rank`` also
accepts the ``--local-rank`` spelling torch>=2's launcher passes.

Additions are opt-in and default to the reference's behaviour:
``--arch {linear,cnn}``, ``--optimizer {adam,sgd}`` (sgd finally consumes
``--momentum``/``--wd`` as the commented-out reference code would,
:192-194), ``--dtype {fp32,bf16}``, ``--synthetic``/``--synthetic-size``,
``--device``, ``--no-graphs``, ``--checkpoint-dir``, ``--timeout``, ``--perf``
and ``--rank-prefix``.
"""
from __future__ import annotations

import argparse
import sys


class _LocalRankAction(argparse.Action):
    def __call__(self, parser, namespace, values, option_string=None):
        setattr(namespace, self.dest, int(values))
        setattr(namespace, "local_rank_given", True)


def build_parser() -> argparse.ArgumentParser:
    parser = argparse.ArgumentParser(
        description="MI355X-native distributed MNIST training (DDP over RCCL/xGMI)")
    parser.add_argument('--root', type=str, default='data')
    parser.add_argument('-j', '--workers', default=4, type=int, metavar='N',
                        help='number of data loading workers (default: 4); kept for CLI '
                             'parity — data is device-resident, no worker processes run')
    parser.add_argument('--epochs', type=int, default=20)
    parser.add_argument('--start-epoch', default=0, type=int, metavar='N',
                        help='manual epoch number (useful on restarts)')
    parser.add_argument('--batch-size', type=int, default=256,
                        help='mini-batch size(default: 256), this is the total batch size of '
                             'all GPUs on the current node when use Distributed Data Parallel')
    parser.add_argument('--lr', '--learning-rate', default=1e-3, type=float,
                        metavar='LR', help='initial learning rate', dest='lr')
    parser.add_argument('--momentum', default=0.9, type=float, metavar='M', help='momentum')
    parser.add_argument('--wd', '--weight-decay', default=1e-4, type=float,
                        metavar='W', help='weight decay (default: 1e-4)', dest='weight_decay')
    parser.add_argument('--resume', default='', type=str, metavar='PATH',
                        help='path to latest checkpoint (default: none)')
    parser.add_argument('-e', '--evaluate', dest='evaluate', action='store_true',
                        help='evaluate model on validation set')
    parser.add_argument('--backend', type=str, default='nccl',
                        help='Name of the backend to use (nccl = RCCL on ROCm, or gloo).')
    parser.add_argument('--local_rank', '--local-rank', type=int, default=0, dest='local_rank',
                        action=_LocalRankAction)
    parser.add_argument('-i', '--init-method', type=str, default='tcp://127.0.0.1:23456',
                        help='URL specifying how to initialize the package.')
    parser.add_argument('-s', '--world-size', type=int, default=1,
                        help='Number of processes participating in the job.')
    parser.add_argument('-r', '--rank', type=int, default=0, help='Rank of the current process.')
    parser.add_argument('--seed', default=None, type=int,
                        help='seed for initializing training (applied inside every rank).')
    # ---- additions (opt-in; defaults reproduce the reference) ----
    g = parser.add_argument_group("MI355X framework options")
    g.add_argument('--arch', choices=['linear', 'cnn'], default='linear',
                   help="linear = reference Net (Linear 784->10); cnn = north-star CNN")
    g.add_argument('--optimizer', choices=['adam', 'sgd'], default='adam')
    g.add_argument('--dtype', choices=['auto', 'fp32', 'bf16'], default='auto',
                   help='compute dtype of activations / GEMM inputs (master weights stay fp32); '
                        'auto = bf16 for the CNN on GPU, fp32 otherwise (the reference Linear '
                        'model and every CPU run)')
    g.add_argument('--synthetic', action='store_true',
                   help='use deterministic synthetic MNIST-shaped data even if MNIST is on disk')
    g.add_argument('--synthetic-size', type=int, default=None,
                   help='number of synthetic training samples (default 60000)')
    g.add_argument('--device', choices=['auto', 'cuda', 'cpu'], default='auto')
    g.add_argument('--no-graphs', dest='graphs', action='store_false',
                   help='launch kernels eagerly instead of replaying captured hipGraphs')
    g.add_argument('--comm', choices=['auto', 'xgmi', 'rccl'], default=None,
                   help='gradient all-reduce transport on GPU with --backend nccl: xgmi = direct '
                        'peer-to-peer pushes over xGMI (hipIpc), rccl = ncclAllReduce; auto '
                        '(default, or $PDM_COMM) = xgmi when every rank passes its self-check')
    g.add_argument('--shard-fc', action='store_true',
                   help='bf16 CNN, world size > 1 over rccl (or gloo): shard the fc1 weight\'s '
                        'optimizer update over the ranks (reduce-scatter of its gradient, each '
                        'rank updates 128 / world_size rows, all-gather of the bf16 rows); '
                        'checkpoints gather the full state first and keep the reference format')
    g.add_argument('--structure-check', choices=['auto', 'on', 'off'], default='auto',
                   help='world size > 1: before the first epoch, run a few steps of each step '
                        'structure in preference order and keep the first that passes on every '
                        'rank, restoring the training state afterwards (auto: on the GPU when '
                        'there is a fallback structure; on: also with a single structure, e.g. '
                        'on CPU/gloo, where the fallback is the same reducer rebuilt)')
    g.add_argument('--checkpoint-dir', default='checkpoints')
    g.add_argument('--timeout', type=float, default=1800.0,
                   help='deadline in seconds for the rendezvous, RCCL communicator init and every '
                        'host sync on the device (a missing peer raises instead of hanging)')
    g.add_argument('--perf', action='store_true',
                   help='print an extra per-epoch throughput line on rank 0')
    g.add_argument('--trace', action='store_true',
                   help='emit roctx ranges (epoch/train/evaluate/checkpoint) for rocprofv3 '
                        '--marker-trace')
    g.add_argument('--rank-prefix', action='store_true',
                   help="prefix every per-rank line with '[rank r] '")
    parser.set_defaults(local_rank_given=False)
    return parser


def parse_args(argv=None):
    return build_parser().parse_args(sys.argv[1:] if argv is None else argv)
