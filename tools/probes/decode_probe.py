"""Time the fused top-k decode + update (ops.topk_decode_apply) on VGG-11's bucket for N ranks'
payloads (N = 1, 2, 4, 8): the receive side of the all-gather at 1-8 GPUs, on one GPU.

    python tools/probes/decode_probe.py [--ratio 0.01] [--reps 50]
EWDML_EXT=<other _C .so> times a different build (A/B of a kernel change).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

import ewdml  # noqa: F401
from ewdml import ops
from ewdml.compress.plan import BucketPlan, Layout
from ewdml.models import build_model


def main():
    a = argparse.ArgumentParser()
    a.add_argument("--ratio", type=float, default=0.01)
    a.add_argument("--reps", type=int, default=50)
    args = a.parse_args()
    ops.require()
    dev = torch.device("cuda")
    m = build_model("VGG11", 10)
    numels = [p.numel() for p in m.parameters()][::-1]
    offs, o = [], 0
    for n in numels:
        offs.append(o)
        o += (n + 63) // 64 * 64
    plan = BucketPlan(numels, offs, args.ratio, 0, o)
    lay = Layout.build("topk_qsgd", plan, 8)
    dp = ops.DevicePlan(plan, dev)
    g = torch.Generator(device=dev).manual_seed(0)
    pays = []
    for r in range(8):
        grad = torch.randn(plan.length, device=dev, generator=g)
        pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=dev)
        ops.topk_encode(dp, grad, pay, lay, 127, "max", 1234 + r)
        pays.append(pay)
    recv = torch.stack(pays)
    param = torch.randn(plan.length, device=dev)
    for n in (1, 2, 4, 8):
        rv = recv[:n].contiguous()
        for _ in range(3):
            ops.topk_decode_apply(dp, rv, lay, 127, param=param, mom=None, lr=1e-9,
                                  grad_scale=1.0 / n)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            ops.topk_decode_apply(dp, rv, lay, 127, param=param, mom=None, lr=1e-9,
                                  grad_scale=1.0 / n)
        e1.record()
        torch.cuda.synchronize()
        print(f"N={n}  decode+update {e0.elapsed_time(e1) * 1e3 / args.reps:7.1f} us "
              f"({lay.nbytes} B per rank, {plan.num_chunks} chunks)")


if __name__ == "__main__":
    main()
