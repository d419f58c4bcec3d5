"""Launch the MFMA conv kernels a few times per VGG layer shape (for rocprofv3 --pmc runs).

    rocprofv3 --pmc SQ_WAVE_CYCLES ... --output-format csv -d out -- python3 tools/conv_pmc.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LAYERS = [(64, 128, 16), (256, 256, 8), (512, 512, 4), (512, 512, 2)]


def main():
    from ewdml import ops
    from ewdml.ops import conv

    C_ = ops.require()
    B = 128
    for cin, cout, hw in LAYERS:
        x = torch.randn(B, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = torch.randn(cout, cin, 3, 3, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn(B, cout, hw, hw, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y, dx, dw = torch.empty_like(dy), torch.empty_like(x), torch.empty_like(w)
        ws = conv._ws(x.device)
        st = ops._stream()
        for _ in range(3):
            C_.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), ws.data_ptr(), ws.numel(), B,
                        hw, hw, cin, cout, 3, 0, 0, st)
            C_.conv_bwd_data(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), ws.data_ptr(),
                             ws.numel(), B, hw, hw, cin, cout, 3, 0, 0, 0, 0, 0, 0, 0, 0, st)
            C_.conv_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), ws.data_ptr(), ws.numel(),
                          B, hw, hw, cin, cout, 3, st)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
