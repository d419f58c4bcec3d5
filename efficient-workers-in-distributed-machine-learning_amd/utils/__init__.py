"""Utilities: metrics/byte accounting, checkpoints, seeding, fault injection."""
from .metrics import MetricsLogger, accuracy, byte_summary, reference_equivalent_bytes

__all__ = ["MetricsLogger", "accuracy", "byte_summary", "reference_equivalent_bytes"]
