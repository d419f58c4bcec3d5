"""Static description of a gradient bucket and of the packed payloads exchanged for it.

A *bucket* is a contiguous range of the flat gradient buffer holding whole parameter tensors
(see ``parallel/flat.py``).  Each tensor is cut into *chunks* of ``CHUNK`` = 8192 elements; a chunk
is the unit of work of every encode/decode kernel and the base of the 16-bit sparse indices.

Top-k semantics follow the reference exactly: per tensor, ``k = max(1, int(numel * ratio))``
(``Compresssor/TopK.py:7``).  Selected entries are emitted sorted by index, so an entry is stored as
a chunk-local ``uint16`` offset plus its code, and one ``uint16`` count per chunk says how many
entries each chunk owns.  That is what gets VGG-11 at top-1 % + 8-bit QSGD to ~132x fewer bytes than
dense fp32 instead of the 80x that int32 indices would give.

Dense selections index better with a bitmap: a tensor whose k is above ~1/16 of its elements
(the report's K = 0.4, or small tensors sent whole) stores one bit per element (uint32 words,
``bitmap`` section) instead of 2 bytes per entry; the choice is made per tensor at plan time from
k and numel alone, so every rank still sends the same fixed size.  At K = 0.4 with 8-bit codes
that is 0.525 B per element against the list's 1.2 B and the report's 0.8 B (value + index byte).

Payload layouts (every section starts 16-byte aligned; all ranks send identical sizes, so the
exchange is a fixed-size all-gather with no size handshake):

``topk_qsgd``: scales f32[T] | counts u16[C] | idx u16[K] | codes i8[K] (bits=8) or nibbles[K/2]
``topk``     : scales f32[T] (unused, kept for a uniform header) | counts | idx | values f32[K]
``qsgd``     : scales f32[T] | codes i8[D'] or nibbles  (dense; D' = numels padded to 16 per tensor)
"""
from dataclasses import dataclass, field
from typing import List

import os

import torch

CHUNK = 8192
BM_WORDS = CHUNK // 32  # bitmap words per chunk
# predictive top-k encode (ops/csrc/topk_codec.hip): a tensor keeps at most this many candidates
# (elements at or above its predicted threshold) per step: CAND_K_MULT * k + CAND_SLACK, capped at
# numel; more (or fewer than k) and that tensor takes the exact full-pass path for the step
CAND_K_MULT = 8
CAND_SLACK = 4096
# ... but a tensor of at most this many elements keeps all of them (bound 0, never a miss;
# EWDML_CAND_ALL_MAX, default 0 = off: measured slower, profiles/ab/README.md "Round 6")
CAND_ALL_MAX = int(os.environ.get("EWDML_CAND_ALL_MAX", "0"))


def cand_cap(n: int, k: int) -> int:
    """Candidate-list capacity of a tensor of n elements keeping k."""
    return n if n <= CAND_ALL_MAX else min(n, CAND_K_MULT * k + CAND_SLACK)


def _align(n: int, a: int = 16) -> int:
    return (n + a - 1) // a * a


@dataclass
class BucketPlan:
    """Tensors of one bucket.  ``offsets`` are element offsets relative to the bucket start."""

    numels: List[int]
    offsets: List[int]
    ratio: float = 1.0
    bucket_offset: int = 0  # element offset of the bucket inside the flat buffer
    length: int = 0  # bucket length in elements (>= last offset + numel; includes align pad)
    # tensors of at most this many elements are sent whole (k = numel): BatchNorm scales/shifts
    # and biases, whose sparsified updates would otherwise arrive once per ~1/ratio steps
    dense_below: int = 0
    # "auto": per tensor, u16 index list or a 1-bit-per-element bitmap, whichever is smaller;
    # "list": always the index list
    index_mode: str = "auto"
    ks: List[int] = field(default_factory=list)
    chunk_tensor: List[int] = field(default_factory=list)
    chunk_start: List[int] = field(default_factory=list)  # relative to bucket start
    chunk_len: List[int] = field(default_factory=list)
    tensor_chunk0: List[int] = field(default_factory=list)
    tensor_nchunks: List[int] = field(default_factory=list)
    tensor_entry0: List[int] = field(default_factory=list)
    tensor_code0: List[int] = field(default_factory=list)  # dense code offset (16-aligned)
    tensor_idx0: List[int] = field(default_factory=list)  # index-list position (-1: bitmap)
    tensor_bm0: List[int] = field(default_factory=list)  # bitmap word offset (-1: index list)
    tensor_cap: List[int] = field(default_factory=list)  # candidate capacity (predictive encode)
    tensor_cap0: List[int] = field(default_factory=list)  # its offset in the candidate list

    def __post_init__(self):
        assert len(self.numels) == len(self.offsets) and self.numels
        if not self.length:
            self.length = self.offsets[-1] + self.numels[-1]
        self.ks = [n if n <= self.dense_below else max(1, int(n * self.ratio))
                   for n in self.numels]
        if self.index_mode not in ("auto", "list"):
            raise ValueError("index_mode must be 'auto' or 'list'")
        e = c = ix = bw = 0
        for t, (n, off) in enumerate(zip(self.numels, self.offsets)):
            nch = (n + CHUNK - 1) // CHUNK
            self.tensor_chunk0.append(len(self.chunk_tensor))
            self.tensor_nchunks.append(nch)
            for j in range(nch):
                self.chunk_tensor.append(t)
                self.chunk_start.append(off + j * CHUNK)
                self.chunk_len.append(min(CHUNK, n - j * CHUNK))
            self.tensor_entry0.append(e)
            e += self.ks[t]
            self.tensor_code0.append(c)
            c += _align(n, 16)
            words = (n + 31) // 32  # chunk j's words start at 256 j: one flat bit per element
            if self.index_mode == "auto" and 4 * words < 2 * self.ks[t]:
                self.tensor_idx0.append(-1)
                self.tensor_bm0.append(bw)
                bw += words
            else:
                self.tensor_idx0.append(ix)
                self.tensor_bm0.append(-1)
                ix += self.ks[t]
        self.total_k = e
        self.total_codes = c
        self.total_idx = ix
        self.total_bm_words = bw
        cap0 = 0
        for n, k in zip(self.numels, self.ks):
            cap = cand_cap(n, k)
            self.tensor_cap.append(cap)
            self.tensor_cap0.append(cap0)
            cap0 += cap
        self.total_cap = cap0

    @property
    def num_tensors(self) -> int:
        return len(self.numels)

    @property
    def num_chunks(self) -> int:
        return len(self.chunk_tensor)

    @property
    def numel(self) -> int:
        return sum(self.numels)

    # ---- device tables consumed by the kernels -------------------------------------------
    @property
    def tensor_cblocks(self) -> List[int]:
        """Blocks per tensor of the predictive encode's candidate passes (one per CHUNK
        candidates of capacity)."""
        return [max(1, (c + CHUNK - 1) // CHUNK) for c in self.tensor_cap]

    @property
    def num_cblocks(self) -> int:
        return sum(self.tensor_cblocks)

    def tensor_table(self, device) -> torch.Tensor:
        """int32 [T, 12]: offset, numel, k, chunk0, nchunks, entry0, code0, idx0, bm0, cap0, cap,
        candidate blocks (csrc/common.h TensorRow)."""
        rows = [[o, n, k, c0, nc, e0, d0, i0, b0, q0, q, nb]
                for o, n, k, c0, nc, e0, d0, i0, b0, q0, q, nb in zip(
                    self.offsets, self.numels, self.ks, self.tensor_chunk0, self.tensor_nchunks,
                    self.tensor_entry0, self.tensor_code0, self.tensor_idx0, self.tensor_bm0,
                    self.tensor_cap0, self.tensor_cap, self.tensor_cblocks)]
        return torch.tensor(rows, dtype=torch.int32, device=device)

    def cblock_table(self, device) -> torch.Tensor:
        """int32 [G, 2]: tensor, block index within the tensor (predictive encode passes)."""
        rows = [[t, j] for t, nb in enumerate(self.tensor_cblocks) for j in range(nb)]
        return torch.tensor(rows, dtype=torch.int32, device=device)

    def chunk_table(self, device) -> torch.Tensor:
        """int32 [C, 4]: tensor, start (rel. bucket), len, local chunk index."""
        rows = []
        for c, (t, s, ln) in enumerate(zip(self.chunk_tensor, self.chunk_start, self.chunk_len)):
            rows.append([t, s, ln, c - self.tensor_chunk0[t]])
        return torch.tensor(rows, dtype=torch.int32, device=device)


@dataclass(frozen=True)
class Layout:
    """Byte offsets of the payload sections for one bucket and one codec."""

    kind: str
    bits: int
    scales: int
    counts: int
    idx: int
    codes: int
    nbytes: int
    bitmap: int = 0  # byte offset of the uint32 bitmap words (top-k kinds)

    @staticmethod
    def build(kind: str, plan: BucketPlan, bits: int = 8) -> "Layout":
        T, C, K = plan.num_tensors, plan.num_chunks, plan.total_k
        scales = 0
        off = _align(4 * T)
        bitmap = 0
        if kind in ("topk_qsgd", "topk"):
            counts = off
            off = _align(off + 2 * C)
            idx = off
            off = _align(off + 2 * plan.total_idx)
            bitmap = off
            off = _align(off + 4 * plan.total_bm_words)
            codes = off
            if kind == "topk":
                off += 4 * K
            else:
                off += K if bits == 8 else (K + 1) // 2
        elif kind == "qsgd":
            counts = idx = off
            codes = off
            off += plan.total_codes if bits == 8 else plan.total_codes // 2
        else:
            raise ValueError(kind)
        return Layout(kind, bits, scales, counts, idx, codes, _align(off), bitmap)
