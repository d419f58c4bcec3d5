"""Optimizers with explicit gradients over the flat parameter buffer (reference ``optim/``)."""
from .flat import FlatAdam, FlatSGD, make_optimizer

__all__ = ["FlatSGD", "FlatAdam", "make_optimizer"]
