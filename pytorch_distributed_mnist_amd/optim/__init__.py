"""Fused flat-arena optimizers with torch-compatible state dicts."""
from .flat import FlatAdam, FlatOptimizer, FlatSGD, adjust_learning_rate, build_optimizer

__all__ = ["FlatAdam", "FlatSGD", "FlatOptimizer", "adjust_learning_rate", "build_optimizer"]
