"""Time the fp32 MFMA conv kernels per VGG-11 layer shape (forward, backward-data, weight
gradient) with HIP events; prints us and TF/s per direction.

    python tools/probes/conv_f32_probe.py [--batch 128] [--reps 20] [--shapes vgg|big] [--wino]
--wino adds the Winograd F(2x2, 3x3) forward (weight + input transforms, 16 GEMMs, output
transform: "wfwd"), backward data ("wbwd") and weight gradient ("wwgrad") on the same shapes (TF/s counted at direct FLOPs).
EWDML_CF_PLAN="bm,bn,split" forces a launch plan (ops/csrc/conv_f32.hip cf_plan).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

import ewdml  # noqa: F401
from ewdml import ops
from ewdml.ops import _ptr, _stream
from ewdml.ops.conv import _ws

VGG = [(64, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4), (512, 512, 4), (512, 512, 2)]
BIG = [(512, 128, 16)]  # long k-loop: steady-state loop efficiency


def main():
    a = argparse.ArgumentParser()
    a.add_argument("--batch", type=int, default=128)
    a.add_argument("--reps", type=int, default=20)
    a.add_argument("--shapes", default="vgg")
    a.add_argument("--dirs", default="fwd,bwd,wgrad")
    a.add_argument("--miopen", action="store_true", help="also time F.conv2d (MIOpen) forward")
    a.add_argument("--wino", action="store_true", help="also time the Winograd path")
    a.add_argument("--tile", type=int, default=0, help="Winograd m (2 or 4; default: auto)")
    args = a.parse_args()
    C_ = ops.require()
    dev = torch.device("cuda")
    ws = _ws(dev)
    N = args.batch
    tot = {}
    for C, Nc, HW in (VGG if args.shapes == "vgg" else BIG):
        x = torch.randn(N, HW, HW, C, device=dev)
        w = torch.randn(Nc, 3, 3, C, device=dev) * 0.05
        y = torch.empty(N, HW, HW, Nc, device=dev)
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        flop = 2.0 * N * HW * HW * Nc * C * 9
        calls = {
            "fwd": lambda: C_.conv_f32_fwd(_ptr(x), _ptr(w), _ptr(y), _ptr(ws), ws.numel(), N, HW,
                                           HW, C, Nc, 3, 0, 0, _stream()),
            "bwd": lambda: C_.conv_f32_bwd_data(_ptr(y), _ptr(w), _ptr(dx), _ptr(ws), ws.numel(),
                                                N, HW, HW, C, Nc, 3, 0, 0, 0, 0, 0, 0, 0, 0,
                                                _stream()),
            "wgrad": lambda: C_.conv_f32_wgrad(_ptr(y), _ptr(x), _ptr(dw), _ptr(ws), ws.numel(), N,
                                               HW, HW, C, Nc, 3, _stream()),
        }
        if args.wino:
            from ewdml.ops.conv import _wino_fits

            m = args.tile or (4 if _wino_fits(N, C, Nc, HW, HW, 4) else 2)
            aa = (m + 2) ** 2
            t = N * (HW // m) * (HW // m)
            U = torch.empty(aa * Nc * C, device=dev)
            buf = torch.empty(aa * t * (C + Nc), device=dev)
            calls["wfwd"] = lambda: C_.wino_f32_fwd(
                _ptr(x), _ptr(w), _ptr(U), _ptr(y), _ptr(buf), _ptr(buf) + 4 * aa * t * C, N, HW,
                HW, C, Nc, m, 0, 0, _stream())
            calls["wbwd"] = lambda: C_.wino_f32_bwd_data(
                _ptr(y), _ptr(w), _ptr(U), _ptr(dx), _ptr(buf), _ptr(buf) + 4 * aa * t * Nc, N,
                HW, HW, C, Nc, m, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, _stream())
            D = torch.empty(aa * t * Nc, device=dev)
            dU = torch.empty(aa * Nc * C, device=dev)
            slabs = torch.empty(4 * aa * Nc * C + 64, device=dev)
            calls["wwgrad"] = lambda: C_.wino_f32_wgrad(
                _ptr(y), _ptr(buf), _ptr(dw), _ptr(D), 0, _ptr(dU), _ptr(slabs), slabs.numel(), N,
                HW, HW, C, Nc, m, 0, _stream())
        if args.miopen:
            xm = x.permute(0, 3, 1, 2)  # NCHW view of NHWC memory: channels_last
            wm = w.permute(0, 3, 1, 2)
            calls["miopen_fwd"] = lambda: torch.nn.functional.conv2d(xm, wm, padding=1)
        line = f"C={C:4d} Nc={Nc:4d} HW={HW:3d}" + (f" m={m}" if args.wino else "")
        extra = (["miopen_fwd"] if args.miopen else []) + (["wfwd", "wbwd", "wwgrad"] if args.wino
                                                            else [])
        for d in args.dirs.split(",") + extra:
            f = calls[d]
            for _ in range(3):
                f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                f()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.reps
            tot[d] = tot.get(d, 0.0) + us
            line += f"  {d} {us:7.1f}us {flop / us / 1e6:6.1f}TF"
        print(line, flush=True)
    print("totals us:", {k: round(v, 1) for k, v in tot.items()}, "sum", round(sum(tot.values()), 1))


if __name__ == "__main__":
    main()
