"""Standalone evaluator (same role and flags as the reference's ``src/distributed_evaluator.py``):
polls ``--model-dir`` for the checkpoint published by rank 0 and prints test loss / accuracy.

    python distributed_evaluator.py --network LeNet --dataset MNIST --model-dir output/models/
"""
import argparse

from ewdml.runtime.evaluator import DistributedEvaluator


def parse(argv=None):
    p = argparse.ArgumentParser(description="ewdml distributed evaluator")
    p.add_argument("--eval-batch-size", type=int, default=10000)
    p.add_argument("--eval-freq", type=int, default=50)
    p.add_argument("--model-dir", type=str, default="output/models/")
    p.add_argument("--dataset", type=str, default="MNIST")
    p.add_argument("--network", type=str, default="LeNet")
    p.add_argument("--data-dir", type=str, default=None)
    p.add_argument("--device", type=str, default="cpu")
    p.add_argument("--poll-seconds", type=float, default=10.0)
    p.add_argument("--once", action="store_true", help="evaluate the current checkpoint and exit")
    p.add_argument("--max-evals", type=int, default=None)
    p.add_argument("--timeout", type=float, default=None)
    p.add_argument("--synthetic-size", type=int, default=0)
    return p.parse_args(argv)


def main(argv=None):
    a = parse(argv)
    ev = DistributedEvaluator(a.network, a.dataset, a.model_dir, a.eval_batch_size, a.data_dir,
                              a.device, a.eval_freq, a.synthetic_size)
    if a.once:
        return ev.poll_once()
    return ev.evaluate(a.poll_seconds, a.max_evals, a.timeout)


if __name__ == "__main__":
    main()
