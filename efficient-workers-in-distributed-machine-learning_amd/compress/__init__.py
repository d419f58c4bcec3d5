"""Gradient compression: bucket plans, packed payload layouts, codecs, torch oracle, RNG.

``reference_api`` keeps the reference's tensor-level compressor classes (``QSGDCompressor``,
``TopKCompressor``, Horovod-style ``Compression``) on top of the packed formats.
"""
from .codecs import KINDS, Codec, make_codec
from .plan import CHUNK, BucketPlan, Layout
from .reference_api import QSGDCompressor, TopKCompressor, TopKQSGDCompressor

__all__ = ["Codec", "make_codec", "KINDS", "BucketPlan", "Layout", "CHUNK",
           "QSGDCompressor", "TopKCompressor", "TopKQSGDCompressor"]
