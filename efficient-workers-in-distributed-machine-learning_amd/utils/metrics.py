"""Accuracy, byte accounting and per-step JSONL metrics.

Parity:
  * ``accuracy`` = the reference's precision@k (``nn_ops.py:13-26`` and its 3 copies);
  * byte accounting replaces ``total_byte_sent += sys.getsizeof(tensor.storage())``
    (``distributed_worker.py:346``, nbytes + 72 B of CPython overhead) with exact payload sizes,
    the algorithmic RCCL wire bytes, and the *reference-equivalent* figure the report plots
    ("comm cost per iteration" = sum over the 2 workers of push + pull);
  * the per-step worker log line (``distributed_worker.py:228-231``) becomes one JSON record per
    step (``--metrics-file``) plus a rate-limited human line every ``--log-interval`` steps.
"""
import json
import os
import time

import torch

MiB = float(1 << 20)


def accuracy(output: torch.Tensor, target: torch.Tensor, topk=(1,)):
    """precision@k in percent for each k."""
    maxk = min(max(topk), output.shape[1])
    _, pred = output.topk(maxk, 1, True, True)
    correct = pred.t().eq(target.view(1, -1).expand_as(pred.t()))
    n = target.shape[0]
    return [correct[:min(k, maxk)].reshape(-1).float().sum().mul_(100.0 / n) for k in topk]


def reference_equivalent_bytes(payload_bytes_push: int, payload_bytes_pull: int,
                               workers: int = 2) -> int:
    """The report's metric: sum over ``workers`` of (bytes pushed + bytes pulled) per iteration."""
    return workers * (payload_bytes_push + payload_bytes_pull)


def byte_summary(stats, world: int, sync_every: int = 1) -> dict:
    """Per-step communication summary from an exchange's StepStats."""
    P = stats.payload_bytes
    D = stats.dense_bytes
    # in the all-to-all topology a rank "pushes" its payload and "pulls" the peers' payloads;
    # the reference-equivalent metric is quoted for its 2-worker setup: push P + pull P each.
    ref_equiv = reference_equivalent_bytes(P, P) / sync_every
    dense_ref = reference_equivalent_bytes(D, D)
    return {
        "payload_bytes_per_rank": P,
        "dense_fp32_bytes": D,
        "compression_ratio": (D / P) if P else None,
        "wire_bytes_sent_per_rank": stats.wire_bytes_sent / sync_every,
        "wire_bytes_total": stats.wire_bytes_sent * world / sync_every,
        "ref_equiv_MiB_per_step": ref_equiv / MiB,
        "dense_ref_equiv_MiB_per_step": dense_ref / MiB,
        "ref_equiv_reduction": (dense_ref / ref_equiv) if ref_equiv else None,
    }


class MetricsLogger:
    def __init__(self, path=None, rank=0, quiet=False):
        self.rank = rank
        self.quiet = quiet
        self.f = None
        if path:
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
            root, ext = os.path.splitext(path)
            self.f = open(f"{root}.rank{rank}{ext or '.jsonl'}", "a", buffering=1)
        self.t0 = time.time()

    def record(self, rec: dict):
        if self.f:
            self.f.write(json.dumps(rec) + "\n")

    def info(self, msg: str):
        if not self.quiet and self.rank == 0:
            print(msg, flush=True)

    def close(self):
        if self.f:
            self.f.close()
            self.f = None
