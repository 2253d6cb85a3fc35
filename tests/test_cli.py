"""CLI surface parity with the reference (multi_proc_single_gpu.py:289-334)."""
from pytorch_distributed_mnist_amd.config import parse_args


def test_reference_defaults():
    a = parse_args([])
    assert a.root == "data" and a.workers == 4 and a.epochs == 20 and a.start_epoch == 0
    assert a.batch_size == 256 and a.lr == 1e-3 and a.momentum == 0.9
    assert a.weight_decay == 1e-4 and a.resume == "" and a.evaluate is False
    assert a.backend == "nccl" and a.local_rank == 0
    assert a.init_method == "tcp://127.0.0.1:23456" and a.world_size == 1 and a.rank == 0
    assert a.seed is None
    # additions default to the reference behaviour
    assert a.arch == "linear" and a.optimizer == "adam" and a.dtype == "auto"


def test_short_and_alias_flags():
    a = parse_args(["-j", "8", "--learning-rate", "0.1", "--weight-decay", "0.5", "-e",
                    "-i", "tcp://127.0.0.1:1", "-s", "4", "-r", "2", "--seed", "7"])
    assert a.workers == 8 and a.lr == 0.1 and a.weight_decay == 0.5 and a.evaluate
    assert a.init_method == "tcp://127.0.0.1:1" and a.world_size == 4 and a.rank == 2
    assert a.seed == 7


def test_local_rank_both_spellings():
    assert parse_args(["--local_rank", "3"]).local_rank == 3
    a = parse_args(["--local-rank=2"])          # torch>=2 launcher spelling
    assert a.local_rank == 2 and a.local_rank_given
    assert not parse_args([]).local_rank_given
