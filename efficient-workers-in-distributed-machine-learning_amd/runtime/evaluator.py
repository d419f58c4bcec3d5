"""Standalone polling evaluator.

Parity: ``src/distributed_evaluator.py:56-141`` -- a separate process that polls the training
directory for the checkpoint the workers publish, loads it and reports test loss / accuracy, the
filesystem being the only channel between trainer and evaluator (``PS/images/system_overview.jpg``).

Fixed defects: the loss is cross-entropy on the logits (the reference
computes NLL on raw logits), a checkpoint is evaluated once per *new* version (the reference keys on
a path that ignores the step and so re-evaluates or misses versions), and the loop can stop
(``--once``, ``--max-evals``, ``--timeout``).  Reads both the legacy ``model_step_`` state_dict
and the rank-0 ``latest`` -> ``step_N.pt`` checkpoints, always with ``weights_only=True``.
"""
import os
import time

import torch
import torch.nn.functional as F

from ..data import DeviceLoader, load_dataset
from ..models import build_model
from ..utils.metrics import accuracy


def _resolve(model_dir):
    """Newest checkpoint in ``model_dir``: (path, version key, is_full_checkpoint)."""
    latest = os.path.join(model_dir, "latest")
    if os.path.exists(latest):
        p = os.path.realpath(latest)
        return p, (p, os.path.getmtime(p)), True
    legacy = os.path.join(model_dir, "model_step_")
    if os.path.exists(legacy):
        return legacy, (legacy, os.path.getmtime(legacy)), False
    return None, None, False


class DistributedEvaluator:
    def __init__(self, network, dataset, model_dir, eval_batch_size=10000, data_dir=None,
                 device="cpu", eval_freq=50, synthetic_size=0, seed=0):
        self.network, self.model_dir = network, model_dir
        self.device = torch.device(device)
        self.eval_freq = eval_freq
        x, y, info = load_dataset(dataset, data_dir, train=False, synthetic_size=synthetic_size,
                                  seed=seed, device=self.device)
        self.info = info
        self.loader = DeviceLoader(x, y, info, min(eval_batch_size, x.shape[0]), shuffle=False,
                                   augment=False, device=self.device, drop_last=False)
        self.model = build_model(network, info["classes"]).to(self.device)
        self._seen = None
        self.history = []

    def load(self, path, full):
        obj = torch.load(path, map_location=self.device, weights_only=True)
        sd = obj["model"] if full else obj
        self.model.load_state_dict(sd)
        return int(obj.get("step", -1)) if full else -1

    @torch.no_grad()
    def evaluate_model(self):
        self.model.eval()
        loss, c1, c5, n = 0.0, 0.0, 0.0, 0
        self.loader.set_epoch(0)
        for x, y in self.loader:
            out = self.model(x).float()
            loss += float(F.cross_entropy(out, y, reduction="sum"))
            a1, a5 = accuracy(out, y, (1, 5))
            c1 += float(a1) * y.shape[0] / 100
            c5 += float(a5) * y.shape[0] / 100
            n += y.shape[0]
        return {"test_loss": loss / n, "top1": 100 * c1 / n, "top5": 100 * c5 / n, "samples": n}

    def poll_once(self):
        path, key, full = _resolve(self.model_dir)
        if path is None or key == self._seen:
            return None
        self._seen = key
        step = self.load(path, full)
        res = self.evaluate_model()
        res.update(step=step, path=path)
        self.history.append(res)
        print(f"Test set (step {step}): Avg. loss: {res['test_loss']:.4f}, "
              f"Accuracy: {res['top1']:.2f}% (top5 {res['top5']:.2f}%)", flush=True)
        return res

    def evaluate(self, poll_s=10.0, max_evals=None, timeout_s=None):
        t0 = time.time()
        while True:
            self.poll_once()
            if max_evals is not None and len(self.history) >= max_evals:
                return self.history
            if timeout_s is not None and time.time() - t0 > timeout_s:
                return self.history
            time.sleep(poll_s)
