"""Trainer facade with the reference's API.

Reference ``Trainer(model, optimizer, train_loader, test_loader, device)`` with
``train()`` / ``evaluate()`` returning ``(Average, Accuracy)``
(``multi_proc_single_gpu.py:68-116``).  Here a Trainer drives a
``TrainProgram`` (device-resident data, fused step kernels, graph replay) and
returns the same metric objects, read from the device once per epoch.
"""
from __future__ import annotations

import time

import torch

from .utils import trace


class Trainer:
    def __init__(self, program):
        self.program = program
        self.last_train_seconds = 0.0
        self.last_eval_seconds = 0.0

    def _sync(self):
        if self.program.is_gpu:
            torch.cuda.synchronize(self.program.device)

    def train(self, indices=None, next_indices=None):
        """One training epoch.  ``indices``: this rank's sample order for the epoch (the
        reference's ``set_epoch`` reshuffle, :231), installed inside the timed region so the
        epoch time includes the boundary work (epoch gather).  ``next_indices``: the next
        epoch's order, if known (its gather then runs beside this epoch's first steps)."""
        self._sync()
        t0 = time.perf_counter()
        with trace.range("train"):
            if indices is not None:
                with trace.range("sampler upload"):
                    self.program.set_train_indices(indices, next_indices)
            result = self.program.train_epoch()   # reading the metrics synchronises
        self.last_train_seconds = time.perf_counter() - t0
        return result

    def evaluate(self):
        t0 = time.perf_counter()
        with trace.range("evaluate"):
            result = self.program.evaluate()
        self.last_eval_seconds = time.perf_counter() - t0
        return result
