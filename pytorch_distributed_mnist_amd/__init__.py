"""MI355X-native distributed MNIST training framework.

Same capabilities and CLI as flybirdtian/pytorch_distributed_mnist, built
MI355X-first: hand-written gfx950 HIP kernels for the whole training step,
a flat parameter arena, a C++ RCCL communicator + bucketed gradient reducer
over xGMI, and hipGraph-replayed steps.  See README.md and SURVEY.md.
"""
__version__ = "0.1.0"
