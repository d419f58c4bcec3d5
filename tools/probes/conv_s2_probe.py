"""Time the fp32 stride-2 conv kernels (ops/csrc/conv_f32.hip k_cf_gemm<..., 2>) per ResNet
down-sampling shape against MIOpen (F.conv2d / aten.convolution_backward), HIP events, us and
TF/s per direction.

    python tools/conv_s2_probe.py [--batch 128] [--reps 20] [--hw 32]
--hw is the input map of the first stage (32: CIFAR, 56: the 224x224 ImageNet stem).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch
import torch.nn.functional as F

import ewdml  # noqa: F401
from ewdml import ops
from ewdml.ops import _ptr, _stream
from ewdml.ops.conv import _ws


def shapes(hw):
    # (C_in, C_out, H, k): ResNet-50 layer2-4 first-block conv2 (3x3/2) and shortcut (1x1/2)
    return [(128, 128, hw, 3), (256, 512, hw, 1), (256, 256, hw // 2, 3), (512, 1024, hw // 2, 1),
            (512, 512, hw // 4, 3), (1024, 2048, hw // 4, 1)]


def timed(fn, reps):
    fn()
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--hw", type=int, default=32)
    a = p.parse_args()
    C_ = ops.require()
    torch.backends.cudnn.benchmark = True  # MIOpen find mode, as the trainer runs it
    dev = torch.device("cuda")
    ws = _ws(dev)
    N = a.batch
    tot = {}
    print(f"{'shape':>26} {'dir':>6} {'hip us':>8} {'miopen us':>10} {'hip TF/s':>9}")
    for C, Nc, H, k in shapes(a.hw):
        x = torch.randn(N, C, H, H, device=dev).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Nc, C, k, k, device=dev) / (k * C ** 0.5)).contiguous(
            memory_format=torch.channels_last)
        Ho = H // 2
        y = torch.empty(N, Nc, Ho, Ho, device=dev).contiguous(memory_format=torch.channels_last)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        part = torch.empty(2 * max(N * Ho * Ho // 64, 1024) * Nc, device=dev)
        flop = 2.0 * N * Ho * Ho * Nc * C * k * k
        pad = k // 2
        runs = {
            "fwd": (lambda: C_.conv_f32_fwd_s2(_ptr(x), _ptr(w), _ptr(y), _ptr(ws), ws.numel(), N,
                                               H, H, C, Nc, k, _ptr(part), part.numel(),
                                               _stream()),
                    lambda: F.conv2d(x, w, stride=2, padding=pad)),
            "bwd": (lambda: C_.conv_f32_bwd_data_s2(_ptr(dy), _ptr(w), _ptr(dx), N, H, H, C, Nc, k,
                                                    0, _stream()),
                    lambda: torch.ops.aten.convolution_backward(
                        dy, x, w, None, [2, 2], [pad, pad], [1, 1], False, [0, 0], 1,
                        [True, False, False])),
            "wgrad": (lambda: C_.conv_f32_wgrad_s2(_ptr(dy), _ptr(x), _ptr(dw), _ptr(ws),
                                                   ws.numel(), N, H, H, C, Nc, k, _stream()),
                      lambda: torch.ops.aten.convolution_backward(
                          dy, x, w, None, [2, 2], [pad, pad], [1, 1], False, [0, 0], 1,
                          [False, True, False])),
        }
        for d, (hip, mio) in runs.items():
            th, tm = timed(hip, a.reps), timed(mio, a.reps)
            tot[d] = (tot.get(d, (0, 0))[0] + th, tot.get(d, (0, 0))[1] + tm)
            print(f"{f'{C}->{Nc} {H}x{H} k{k}':>26} {d:>6} {th:8.1f} {tm:10.1f} "
                  f"{flop / th / 1e6:9.1f}", flush=True)
    for d, (th, tm) in tot.items():
        print(f"{'total':>26} {d:>6} {th:8.1f} {tm:10.1f}")


if __name__ == "__main__":
    main()
