"""Reproduce the report's "average communication cost per iteration" chart (BASELINE.md,
``Report.zip:Comm Cost.png``) from the *actual* packed payload sizes of this framework.

The report's metric is the sum over its 2 workers of (bytes pushed + bytes pulled) per iteration,
in MiB.  For each method we compute it from ``Layout.build`` of the real bucket plans:

  1  push dense fp32 grads, pull dense fp32 weights
  2  push int8 QSGD, pull dense fp32 weights
  3  push + pull dense fp32 grads
  4  int8 QSGD both ways
  5  top-k -> int8 QSGD both ways (u16 chunk-local indices)
  6  method 5, communicating every 20 iterations

Usage: python tools/methods_table.py [--ratio 0.4] [--markdown]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ewdml.compress.plan import BucketPlan, Layout  # noqa: E402
from ewdml.models import build_model  # noqa: E402
from ewdml.parallel.flat import FlatModel  # noqa: E402

MiB = float(1 << 20)
PUBLISHED = {  # BASELINE.md, methods 1..6
    "VGG11": [148, 92.5, 148, 37, 29.6, 1.48],
    "LeNet": [6.56, 4.1, 6.56, 1.64, 1.312, 0.066],
}


def plan_of(name, ratio):
    flat = FlatModel(build_model(name), bucket_bytes=1 << 40)
    p = flat.buckets[0].plan
    return BucketPlan(p.numels, p.offsets, ratio, 0, p.length), flat.param_numel


def table(name, ratio, bits=8):
    plan, n = plan_of(name, ratio)
    dense = 4 * n
    q = Layout.build("qsgd", plan, bits).nbytes
    tk = Layout.build("topk_qsgd", plan, bits).nbytes
    workers = 2
    rows = [
        dense + dense, q + dense, dense + dense, q + q, tk + tk, (tk + tk) / 20,
    ]
    return [workers * r / MiB for r in rows]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--ratio", type=float, default=0.4, help="top-k ratio (report: K=0.4)")
    ap.add_argument("--bits", type=int, default=8)
    ap.add_argument("--markdown", action="store_true")
    a = ap.parse_args(argv)
    out = []
    for name in ("VGG11", "LeNet"):
        ours = table(name, a.ratio, a.bits)
        ours1 = table(name, 0.01, a.bits)
        out.append(f"\n{name}: MiB per iteration (2 workers, push+pull)")
        out.append("| method | published | ours (top-k %g) | ours (top-k 0.01) |" % a.ratio)
        out.append("|---|---|---|---|")
        for m in range(6):
            out.append(f"| {m + 1} | {PUBLISHED[name][m]} | {ours[m]:.4f} | {ours1[m]:.4f} |")
    txt = "\n".join(out)
    print(txt)
    return txt


if __name__ == "__main__":
    main()
