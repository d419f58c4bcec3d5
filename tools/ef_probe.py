"""Error-feedback stability probe on the torch oracle (CPU or GPU): loss curve of a short run
with no error feedback, plain error feedback, and momentum-corrected (DGC) error feedback.

    python tools/ef_probe.py [--network ResNet50] [--batch 32] [--steps 38] [--modes none,plain,dgc]

VERDICT r2 Weak #1 reproduced plain error feedback's spike with this configuration (ResNet-50
CIFAR, batch 32, top-1 % + QSGD-8, momentum 0.9, lr 0.01): peak loss 12.67 (chance 2.30).  Prints
one JSON line per mode: peak and final loss and the per-step curve.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(mode, a):
    import torch

    import ewdml
    from ewdml.runtime.trainer import Trainer

    flags = ["--network", a.network, "--dataset", a.dataset, "--batch-size", str(a.batch),
             "--compress", a.compress, "--topk-ratio", str(a.ratio), "--momentum", "0.9",
             "--lr", str(a.lr), "--synthetic-size", str(a.synthetic or max(2048, 4 * a.batch)),
             "--eval-freq",
             "0", "--quiet", "--max-steps", str(a.steps), "--device", a.device,
             "--log-interval", "1000000", "--seed", str(a.seed)]
    if mode != "none":
        flags += ["--error-feedback", "--ef-mode", mode]
    if a.hip_graph != "off":
        flags += ["--hip-graph", a.hip_graph]
    flags += a.extra.split()
    if a.dense_below:
        flags += ["--topk-dense-below", str(a.dense_below)]
    if a.warmup:
        flags += ["--topk-warmup", a.warmup, "--topk-warmup-epochs", str(a.warmup_epochs)]
    torch.manual_seed(a.seed)
    tr = Trainer(ewdml.parse_args(flags))
    losses = []
    for _ in range(a.steps):
        loss, _ = tr.train_step()
        losses.append(round(float(loss.detach()), 4))
    tail = losses[-max(1, len(losses) // 6):]
    every = max(1, len(losses) // 30)
    return {"mode": mode, "ef_mode": getattr(tr.exchange, "ef_mode", None),
            "compress": a.compress, "warmup": a.warmup, "dense_below": a.dense_below,
            "extra": a.extra, "peak": max(losses), "final": losses[-1],
            "tail_mean": round(sum(tail) / len(tail), 4),
            "curve": [round(sum(losses[i:i + every]) / len(losses[i:i + every]), 3)
                      for i in range(0, len(losses), every)]}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--network", default="ResNet50")
    p.add_argument("--dataset", default="Cifar10")
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--steps", type=int, default=38)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--ratio", type=float, default=0.01)
    p.add_argument("--compress", default="topk_qsgd")
    p.add_argument("--modes", default="none,plain,dgc")
    p.add_argument("--device", default="cpu")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--warmup", default="")
    p.add_argument("--dense-below", type=int, default=0)
    p.add_argument("--hip-graph", default="off")
    p.add_argument("--synthetic", type=int, default=0)
    p.add_argument("--extra", default="", help="more distributed_nn.py flags")
    p.add_argument("--warmup-epochs", type=float, default=1.0)
    a = p.parse_args()
    for m in a.modes.split(","):
        print(json.dumps(run(m, a)), flush=True)


if __name__ == "__main__":
    main()
