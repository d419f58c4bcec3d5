"""Time the top-k + QSGD-8 encode (ops.topk_encode, 4 launches) on VGG-11's bucket, with
momentum-corrected error feedback (the bench's codec) and without, by HIP events.

    python tools/probes/encode_probe.py [--ratio 0.01] [--reps 50]
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
    a.add_argument("--modes", default="plain,ef,dgc")
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
    grad = torch.randn(plan.length, device=dev, generator=g) * 1e-3
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=dev)
    resid = torch.zeros(plan.length, device=dev)
    vel = torch.zeros(plan.length, device=dev)
    param = torch.randn(plan.length, device=dev)
    dgc = dict(velocity=vel, momentum=0.9, dampening=0.0, nesterov=False, weight_decay=0.0,
               param=param, mask=True)
    modes = (("plain", {}), ("ef", dict(resid=resid)), ("dgc", dict(resid=resid, dgc=dgc)))
    for name, kw in modes:
        if name not in args.modes.split(","):
            continue
        for _ in range(3):
            ops.topk_encode(dp, grad, pay, lay, 127, "max", 7, **kw)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            ops.topk_encode(dp, grad, pay, lay, 127, "max", 7, **kw)
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:6s} encode {e0.elapsed_time(e1) * 1e3 / args.reps:7.1f} us "
              f"({plan.length} elements, {plan.num_chunks} chunks)")


if __name__ == "__main__":
    main()
