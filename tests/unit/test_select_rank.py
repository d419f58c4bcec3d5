"""The top-k selects' ranked digit-0 bin (ops/csrc/topk_codec.hip pk1_select_cands and
k_pk_select's pass 1): after the first radix digit picks the bin holding the k-th largest key,
ranking that bin's few keys directly gives the threshold and the tie count the two remaining
radix digits give.  Checked here on a model of both procedures over random key sets (the GPU
tests check the kernels bitwise against the three-launch encode and the oracle)."""
import numpy as np
import pytest


def _radix(keys, k, B, s0, s1):
    """Three digits over rel = key - B: [.. : s0], [s0 - 1 : s1], [s1 - 1 : 0]; returns
    (threshold rel, ties to keep) as the kernels' digit selects do (bins scanned from the top)."""
    rel = keys - B
    prefix, k_rem = 0, k
    for shift, hi in ((s0, None), (s1, s0), (0, s1)):
        sel = rel if hi is None else rel[(rel >> hi) == (prefix >> hi)]
        digit = (sel >> shift) & (((1 << (hi - shift)) - 1) if hi is not None else 0xFFFFFFFF)
        counts = np.bincount(digit, minlength=int(digit.max()) + 1 if len(digit) else 1)
        run = 0
        for b in range(len(counts) - 1, -1, -1):
            if run + counts[b] >= k_rem:
                prefix |= b << shift
                k_rem -= run
                break
            run += counts[b]
    return prefix, k_rem


def _ranked(keys, k, B, s0):
    """Digit 0 as above, then the selected bin's keys ranked directly."""
    rel = keys - B
    d0 = rel >> s0
    counts = np.bincount(d0)
    run, k_rem = 0, k
    for b in range(len(counts) - 1, -1, -1):
        if run + counts[b] >= k_rem:
            k_rem -= run
            binkeys = rel[d0 == b]
            break
        run += counts[b]
    for mine in binkeys:
        gt = int((binkeys > mine).sum())
        eq = int((binkeys == mine).sum())
        if gt < k_rem <= gt + eq:
            return int(mine), k_rem - gt
    raise AssertionError("no threshold")


@pytest.mark.parametrize("seed", range(40))
def test_ranked_bin_matches_radix_digits(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(20, 3000))
    # fp32 magnitudes as their bit patterns (the kernels' keys), with deliberate ties
    mags = np.abs(rng.standard_normal(n).astype(np.float32)) * np.float32(10.0 ** rng.integers(-4, 2))
    if seed % 3 == 0:
        mags[rng.integers(0, n, n // 4)] = mags[0]
    keys = mags.view(np.uint32).astype(np.int64)
    k = int(rng.integers(1, n + 1))
    B = int(keys.min()) if seed % 2 else 0
    span = int(keys.max() - B)
    bl = span.bit_length()
    s0 = bl - 11 if bl > 11 else 0
    s1 = s0 - 10 if s0 > 10 else 0
    thr, ties = _radix(keys, k, B, s0, s1)
    assert _ranked(keys, k, B, s0) == (thr, ties)
    # the definition: exactly k keys are kept (those above the threshold + `ties` equal ones)
    rel = keys - B
    assert int((rel > thr).sum()) + ties == k and 1 <= ties <= int((rel == thr).sum())
