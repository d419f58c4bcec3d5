"""Time the fused top-k decode + update (ops.topk_decode_apply) on a model's bucket for N ranks'
payloads (N = 1, 2, 4, 8): the receive side of the all-gather at 1-8 GPUs, on one GPU.

    python tools/probes/decode_probe.py [--model VGG11] [--ratio 0.01] [--bits 8] [--reps 50]
        [--json out.json]   # {"model", "ratio", "bits", "decode_us": {N: us}} for the step model
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
    a.add_argument("--model", default="VGG11")
    a.add_argument("--bits", type=int, default=8)
    a.add_argument("--json", default=None)
    args = a.parse_args()
    ops.require()
    dev = torch.device("cuda")
    m = build_model(args.model, 1000 if "imagenet" in args.model.lower() else 10)
    numels = [p.numel() for p in m.parameters()][::-1]
    # buckets as the trainer cuts them: at most 128 tensors (ops.MAX_TENSORS_PER_BUCKET), 64 MiB
    groups, cur, cur_b = [], [], 0
    for n in numels:
        if cur and (len(cur) == ops.MAX_TENSORS_PER_BUCKET or cur_b + 4 * n > 64 << 20):
            groups.append(cur)
            cur, cur_b = [], 0
        cur.append(n)
        cur_b += 4 * n
    groups.append(cur)
    lv = 127 if args.bits == 8 else 7
    g = torch.Generator(device=dev).manual_seed(0)
    buckets = []
    for gi, grp in enumerate(groups):
        offs, o = [], 0
        for n in grp:
            offs.append(o)
            o += (n + 63) // 64 * 64
        plan = BucketPlan(grp, offs, args.ratio, 0, o)
        lay = Layout.build("topk_qsgd", plan, args.bits)
        dp = ops.DevicePlan(plan, dev)
        pays = []
        for r in range(8):
            grad = torch.randn(plan.length, device=dev, generator=g)
            pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=dev)
            ops.topk_encode(dp, grad, pay, lay, lv, "max", 1234 + r + 8 * gi)
            pays.append(pay)
        buckets.append((dp, lay, torch.stack(pays), torch.randn(plan.length, device=dev)))
    nbytes = sum(b[1].nbytes for b in buckets)
    nchunks = sum(b[0].plan.num_chunks for b in buckets)
    res = {}

    def step(n):
        for dp, lay, recv, param in buckets:
            ops.topk_decode_apply(dp, recv[:n].contiguous() if n < 8 else recv, lay, lv,
                                  param=param, mom=None, lr=1e-9, grad_scale=1.0 / n)

    for n in (1, 2, 4, 8):
        for _ in range(3):
            step(n)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            step(n)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.reps
        res[n] = round(us, 2)
        print(f"N={n}  decode+update {us:7.1f} us ({nbytes} B per rank, {nchunks} chunks, "
              f"{len(buckets)} bucket(s))")
    if args.json:
        import json

        with open(args.json, "w") as f:
            json.dump({"model": args.model, "ratio": args.ratio, "bits": args.bits,
                       "payload_bytes": nbytes, "buckets": len(buckets), "decode_us": res}, f)


if __name__ == "__main__":
    main()
