"""Counter-based RNG shared bit-for-bit by the HIP kernels and the torch oracle.

QSGD's stochastic rounding needs one uniform variate per quantised element.  The reference draws
them with ``torch.empty_like(t).uniform_()`` (``Compresssor/qsgd.py:23``), which is neither
reproducible across ranks nor free.  Here a variate is a pure function of
(seed, step, rank, flat element index): ``u = mix32(idx ^ key) >> 8`` scaled to [0, 1), with
``key = stream_key(seed, step, rank)``.  ``mix32`` is the "lowbias32" integer finaliser (two
multiply-xorshift rounds).  The same function lives in ``ops/csrc/common.h`` (``ew_mix32``); the
kernel tests assert identical payload bytes on CPU and GPU.
"""
import torch

M32 = 0xFFFFFFFF
_C1 = 0x7FEB352D
_C2 = 0x846CA68B


def mix32_int(x: int) -> int:
    x &= M32
    x ^= x >> 16
    x = (x * _C1) & M32
    x ^= x >> 15
    x = (x * _C2) & M32
    x ^= x >> 16
    return x


def stream_key(seed: int, step: int, rank: int) -> int:
    """Per-(seed, step, rank) key; computed on the host and passed to kernels as a uint32."""
    k = mix32_int((step * 0x9E3779B9 + rank * 0x85EBCA6B + 0x632BE59B) & M32)
    return mix32_int((seed & M32) ^ k)


def _mul32(x: torch.Tensor, c: int) -> torch.Tensor:
    # (x * c) mod 2^32 for 0 <= x < 2^32 held in int64, without int64 overflow.
    lo = x * (c & 0xFFFF)
    hi = ((x * (c >> 16)) & 0xFFFF) << 16
    return (lo + hi) & M32


def mix32(x: torch.Tensor) -> torch.Tensor:
    x = x & M32
    x = x ^ (x >> 16)
    x = _mul32(x, _C1)
    x = x ^ (x >> 15)
    x = _mul32(x, _C2)
    return x ^ (x >> 16)


def uniform(idx: torch.Tensor, key: int) -> torch.Tensor:
    """Uniform float32 variates in [0, 1) with 24 random bits for int64 element indices."""
    h = mix32((idx.to(torch.int64) & M32) ^ (key & M32))
    return (h >> 8).to(torch.float32) * (1.0 / 16777216.0)
