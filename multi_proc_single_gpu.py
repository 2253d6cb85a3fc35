"""Entry point with the reference's file name and CLI.

    python multi_proc_single_gpu.py --world-size 4                      # spawn mode
    python -m torch.distributed.launch --nproc_per_node=4 \\
        multi_proc_single_gpu.py --world-size 4                         # launch mode
    torchrun --nproc-per-node 4 multi_proc_single_gpu.py --world-size 4

The launch mode is detected at run time (no source edit, unlike the reference's
``multi_proc_single_gpu.py:353-359``).  All logic lives in
``pytorch_distributed_mnist_amd.app``.
"""
from pytorch_distributed_mnist_amd.app import main, run, run_dist_launch, run_spawn  # noqa: F401

if __name__ == '__main__':
    main()
