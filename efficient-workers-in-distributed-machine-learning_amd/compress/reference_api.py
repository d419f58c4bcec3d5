"""Tensor-level compressor classes with the reference's call signatures.

Parity:
  * ``QSGDCompressor().compress(t) -> (levels, norm)``, ``.decompress((levels, norm)) -> t``
    (``Compresssor/qsgd.py:5-40``; Horovod flavour ``horovod_compression.py:11-43`` with static
    methods and ``decompress(levels, ctx=norm)``);
  * ``TopKCompressor(ratio).compress(t) -> ((values, indices), (numel, shape))``,
    ``.decompress(tensors, ctx)`` (``Compresssor/TopK.py:20-35``).

Differences: levels are real ``int8`` (s <= 127), a zero norm gives zeros,
not NaN, and the rounding variates come from the counter RNG.  These are convenience/compat
helpers for single tensors; training uses the bucketed codecs (``codecs.py``) and HIP kernels.
"""
import torch

from . import oracle


class QSGDCompressor:
    def __init__(self, quantum_num: int = 127, norm: str = "l2", seed: int = 0):
        if not 1 <= quantum_num <= 127:
            raise ValueError("quantum_num must be in [1, 127] to fit int8 codes")
        self.quantum_num = quantum_num
        self.norm = norm
        self.seed = seed
        self.calls = 0

    def compress(self, tensor: torch.Tensor):
        flat = tensor.detach().flatten().to(torch.float32)
        scale = oracle._scale_of(flat, self.norm)
        key = (self.seed * 0x9E3779B9 + self.calls) & 0xFFFFFFFF
        self.calls += 1
        idx = torch.arange(flat.numel(), device=flat.device)
        q = oracle.quantize(flat, scale, self.quantum_num, idx, key)
        norm = torch.tensor([scale], dtype=torch.float32, device=tensor.device)
        return q.to(torch.int8).view(tensor.shape), norm

    def decompress(self, tensor_compressed, ctx=None):
        if ctx is None:
            levels, norm = tensor_compressed
        else:  # Horovod signature: decompress(levels, ctx=norm)
            levels, norm = tensor_compressed, ctx
        step = oracle.dequant_step(self.quantum_num, float(norm.flatten()[0]))
        return levels.to(torch.float32) * step


class TopKCompressor:
    def __init__(self, compress_ratio: float):
        self.compress_ratio = compress_ratio

    def compress(self, tensor: torch.Tensor):
        flat = tensor.flatten()
        k = max(1, int(flat.numel() * self.compress_ratio))
        idx = oracle.topk_indices(flat, k)
        return (flat[idx], idx), (tensor.numel(), tensor.size())

    def decompress(self, tensors, ctx):
        values, indices = tensors
        numel, shape = ctx
        out = torch.zeros(numel, dtype=values.dtype, device=values.device)
        out.scatter_(0, indices, values)
        return out.view(shape)


class TopKQSGDCompressor:
    """Method 5: top-k, then QSGD of the kept values (scale = max |g| by default)."""

    def __init__(self, compress_ratio: float = 0.01, quantum_num: int = 127, norm: str = "max"):
        self.topk = TopKCompressor(compress_ratio)
        self.qsgd = QSGDCompressor(quantum_num, norm)

    def compress(self, tensor):
        (vals, idx), ctx = self.topk.compress(tensor)
        levels, norm = self.qsgd.compress(vals)
        return (levels, norm, idx), ctx

    def decompress(self, tensors, ctx):
        levels, norm, idx = tensors
        vals = self.qsgd.decompress((levels, norm))
        return self.topk.decompress((vals, idx), ctx)
