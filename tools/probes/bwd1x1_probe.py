"""Backward data of ResNet-50's stride-1 1x1 convs two ways: the backward-data GEMM on w (its B
operand rows-contiguous in LDS: one ds_read_b32 per MFMA operand) vs the forward GEMM on the
transposed weight wT [C][Nc] (B k-contiguous: ds_read_b128), same products.

    python tools/probes/bwd1x1_probe.py [--reps 20]
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

# (N, HW, C, Nc): x [N][HW][HW][C] -> y [..][Nc]; bwd data: dx [..][C] from dy [..][Nc]
SHAPES = [(128, 32, 256, 64), (128, 32, 64, 256), (128, 16, 512, 128), (128, 16, 128, 512),
          (128, 8, 1024, 256), (128, 8, 256, 1024), (128, 4, 2048, 512), (128, 4, 512, 2048),
          (64, 56, 256, 64), (64, 56, 64, 256), (64, 28, 128, 512), (64, 7, 512, 2048)]


def main():
    a = argparse.ArgumentParser()
    a.add_argument("--reps", type=int, default=20)
    args = a.parse_args()
    C_ = ops.require()
    dev = torch.device("cuda")
    ws = _ws(dev)
    tot = [0.0, 0.0]
    for N, HW, C, Nc in SHAPES:
        dy = torch.randn(N, HW, HW, Nc, device=dev)
        w = torch.randn(Nc, 1, 1, C, device=dev) * 0.05
        wT = w.view(Nc, C).t().contiguous().view(C, 1, 1, Nc)
        dx = torch.empty(N, HW, HW, C, device=dev)
        dx2 = torch.empty_like(dx)
        calls = {
            "bwd": lambda: C_.conv_f32_bwd_data(_ptr(dy), _ptr(w), _ptr(dx), _ptr(ws), ws.numel(),
                                                N, HW, HW, C, Nc, 1, 0, 0, 0, 0, 0, 0, 0, 0,
                                                _stream()),
            "fwdT": lambda: C_.conv_f32_fwd(_ptr(dy), _ptr(wT), _ptr(dx2), _ptr(ws), ws.numel(), N,
                                            HW, HW, Nc, C, 1, 0, 0, _stream()),
        }
        res = {}
        for name, f in calls.items():
            for _ in range(3):
                f()
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            for _ in range(args.reps):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[name] = e0.elapsed_time(e1) * 1000 / args.reps
        err = float((dx - dx2).abs().max())
        same = bool(torch.equal(dx, dx2))
        tot[0] += res["bwd"]
        tot[1] += res["fwdT"]
        flop = 2.0 * N * HW * HW * C * Nc
        print(f"N={N} {HW}x{HW} C={C} Nc={Nc}: bwd {res['bwd']:7.1f} us ({flop / res['bwd'] / 1e6:5.1f} TF/s)"
              f"  fwd(wT) {res['fwdT']:7.1f} us ({flop / res['fwdT'] / 1e6:5.1f} TF/s)  max|d|={err:.2e} bitwise={same}")
    print(f"total bwd {tot[0]:.1f} us, fwd(wT) {tot[1]:.1f} us")


if __name__ == "__main__":
    main()
