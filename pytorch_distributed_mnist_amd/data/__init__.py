"""Device-resident MNIST data: IDX reader, synthetic data, DistributedSampler-identical order."""
from .mnist import MnistSplit, load_split, normalize_reference, synthetic_split
from .sampler import batch_bounds, distributed_indices, num_samples_per_rank

__all__ = ["MnistSplit", "load_split", "normalize_reference", "synthetic_split", "batch_bounds",
           "distributed_indices", "num_samples_per_rank"]
