"""Sharded parameter server (``--topology sharded``, ``parallel/sharded.py``; SURVEY 7.3 item
4(b)) on CPU/Gloo: shard cutting, replica agreement at world sizes 2 and 3, equality with the
dense all-reduce when the codec is lossless, and the wire-byte model."""
import pytest
import torch

from .helpers import run_world
from .test_exchange import _same_params, _train

pytestmark = pytest.mark.slow


def test_shard_plans_cover_bucket():
    from ewdml.compress import CHUNK, BucketPlan
    from ewdml.parallel.sharded import shard_plans

    numels = [5, 3 * CHUNK + 7, 100, 2 * CHUNK]
    offsets, o = [], 0
    for n in numels:
        offsets.append(o)
        o += n + 11  # alignment padding between tensors
    plan = BucketPlan(numels, offsets, 0.01, 0, o)
    for n in (1, 2, 3, 8, 64):
        sh = shard_plans(plan, n, 1000)
        assert len(sh) == n
        assert sh[0][0] == 0 and sum(ln for _, ln, _ in sh) == plan.length
        covered = 0
        for s0, ln, sp in sh:
            assert s0 % CHUNK == 0
            if sp is None:
                continue
            assert sp.bucket_offset == 1000 + s0
            for off, num in zip(sp.offsets, sp.numels):
                assert 0 <= off and off + num <= ln
            covered += sum(sp.numels)
        assert covered == sum(numels)


@pytest.mark.parametrize("world,flags", [
    (2, ["--compress", "topk_qsgd"]),
    (3, ["--compress", "topk_qsgd"]),
    (2, ["--compress", "qsgd"]),
    (3, ["--compress", "topk_qsgd", "--bucket-mb", "0.5"]),
])
def test_sharded_replicas_identical(tmp_path, world, flags):
    res = run_world(_train, world, tmp_path, args=(["--topology", "sharded"] + flags, 3))
    _same_params(res)
    assert all(res[0]["losses"])


def test_sharded_lossless_equals_dense_allreduce(tmp_path):
    # top-k with ratio 1 ships every value in fp32: owner average + re-encode is exact, so the
    # sharded server must reproduce the dense all-reduce step
    sh = run_world(_train, 2, tmp_path / "sh", args=(
        ["--topology", "sharded", "--compress", "topk", "--topk-ratio", "1.0", "--amp", "none"], 3))
    ar = run_world(_train, 2, tmp_path / "ar", args=(["--compress", "none", "--amp", "none"], 3))
    torch.testing.assert_close(sh[0]["params"], ar[0]["params"], rtol=1e-5, atol=1e-6)


def test_sharded_rejects_dense_codec():
    import ewdml

    cfg = ewdml.parse_args(["--topology", "sharded", "--compress", "none"])
    assert cfg.topology == "sharded"
    from ewdml.parallel.sharded import ShardedPSExchange

    with pytest.raises(ValueError, match="compressing codec"):
        ShardedPSExchange(None, None, "none", None)
