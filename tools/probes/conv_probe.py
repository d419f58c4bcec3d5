"""Per-layer timing of VGG-11's conv shapes (bs128, CIFAR, NHWC bf16) through MIOpen, and of the
equivalent im2col GEMM shapes through hipBLASLt, to size hand-written kernels against.

    python tools/conv_probe.py
"""
import torch
import torch.nn.functional as F

LAYERS = [(3, 64, 32), (64, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4), (512, 512, 4),
          (512, 512, 2), (512, 512, 2)]


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def hip_times(x, w, dy):
    """(fwd, bwd_data, wgrad) us of the MFMA kernels (ops/conv.py), None if unsupported."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from ewdml import ops
    from ewdml.ops import conv

    if not conv.supported(x, w):
        return None
    C_ = ops.require()
    N, C, H, W = x.shape
    Nc = w.shape[0]
    ws = conv._ws(x.device)
    y = torch.empty_like(dy)
    dx = torch.empty_like(x)
    dw = torch.empty_like(w)
    st = ops._stream
    if C == 3:  # stem kernels: forward and weight gradient (no input gradient)
        tf = timeit(lambda: C_.conv_stem_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), N, H, W,
                                             Nc, 0, 0, st()))
        tw = timeit(lambda: C_.conv_stem_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr(),
                                               ws.data_ptr(), ws.numel(), N, H, W, Nc, st()))
        return tf, float("nan"), tw
    tf = timeit(lambda: C_.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), ws.data_ptr(),
                                       ws.numel(), N, H, W, C, Nc, 3, 0, 0, st()))
    tb = timeit(lambda: C_.conv_bwd_data(dy.data_ptr(), w.data_ptr(), dx.data_ptr(),
                                            ws.data_ptr(), ws.numel(), N, H, W, C, Nc, 3, 0, 0,
                                            0, 0, 0, 0, 0, 0, st()))
    tw = timeit(lambda: C_.conv_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr(),
                                         ws.data_ptr(), ws.numel(), N, H, W, C, Nc, 3, st()))
    return tf, tb, tw


def main():
    torch.backends.cudnn.benchmark = True
    htot = [0.0, 0.0, 0.0]
    B = 128
    tot = [0.0, 0.0, 0.0, 0.0]
    print("cin cout hw | conv fwd us  TF/s | gemm(M,N,K) us TF/s | bwd_data us | wrw us")
    for cin, cout, hw in LAYERS:
        x = torch.randn(B, cin, hw, hw, device="cuda", dtype=torch.bfloat16).to(
            memory_format=torch.channels_last)
        w = torch.randn(cout, cin, 3, 3, device="cuda", dtype=torch.bfloat16).to(
            memory_format=torch.channels_last)
        x.requires_grad_(True)
        w.requires_grad_(True)
        fl = 2.0 * B * hw * hw * cout * cin * 9
        t_f = timeit(lambda: F.conv2d(x, w, padding=1))
        y = F.conv2d(x, w, padding=1)
        dy = torch.randn_like(y)
        t_bd = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]))
        t_bw = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
        M, N, K = B * hw * hw, cout, 9 * cin
        a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        bt = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        t_g = timeit(lambda: a @ bt.t())
        tot[0] += t_f
        tot[1] += t_g
        tot[2] += t_bd
        tot[3] += t_bw
        print(f"{cin:3d} {cout:4d} {hw:2d} | {t_f:8.1f} {fl / t_f / 1e6:6.0f} | ({M},{N},{K}) "
              f"{t_g:7.1f} {fl / t_g / 1e6:6.0f} | {t_bd:8.1f} | {t_bw:8.1f}")
        h = hip_times(x.detach(), w.detach(), dy.contiguous(memory_format=torch.channels_last))
        if h is not None:
            for i in range(3):
                htot[i] += h[i] if h[i] == h[i] else 0.0
            print(f"      hip mfma | fwd {h[0]:8.1f} ({fl / h[0] / 1e6:6.0f} TF/s) | bwd_data "
                  f"{h[1]:8.1f} ({fl / h[1] / 1e6:6.0f}) | wgrad {h[2]:8.1f} ({fl / h[2] / 1e6:6.0f})")
    print(f"total: fwd {tot[0]:.1f} gemm {tot[1]:.1f} bwd_data {tot[2]:.1f} wrw {tot[3]:.1f} us")
    print(f"hip mfma total (supported layers): fwd {htot[0]:.1f} bwd_data {htot[1]:.1f} "
          f"wgrad {htot[2]:.1f} us")


if __name__ == "__main__":
    main()
