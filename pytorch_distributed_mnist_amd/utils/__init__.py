"""Metrics, checkpointing, logging and timing helpers."""
from .checkpoint import best_path, checkpoint_path, load_checkpoint, make_state, save_checkpoint
from .metrics import Accuracy, Average, DeviceMetrics

__all__ = ["Average", "Accuracy", "DeviceMetrics", "save_checkpoint", "load_checkpoint",
           "make_state", "checkpoint_path", "best_path"]
