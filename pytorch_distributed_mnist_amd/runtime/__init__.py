"""Flat parameter arena, step programs and graph capture."""
from .arena import FlatArena
from .program import TrainProgram

__all__ = ["FlatArena", "TrainProgram"]
