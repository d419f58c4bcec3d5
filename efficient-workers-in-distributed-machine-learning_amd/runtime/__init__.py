"""Roles and drivers: the trainer (workers / PS server) and the standalone evaluator."""
from .evaluator import DistributedEvaluator
from .trainer import FaultInjected, Trainer, resolve_device, run

__all__ = ["Trainer", "run", "resolve_device", "FaultInjected", "DistributedEvaluator"]
