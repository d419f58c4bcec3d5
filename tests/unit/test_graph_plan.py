"""``--hip-graph auto`` decision for the all-to-all exchange (parallel/engine.plan_graph_mode):
the one-graph step at N = 1 and for top-k payloads, segmented overlap for large dense collectives
at N > 1 on the own (capturable) communicator."""
import pytest

from ewdml.parallel.engine import OVERLAP_MIN_WIRE_BYTES, plan_graph_mode

VGG = 9_756_426  # VGG-11-BN parameters
R50 = 23_520_842  # ResNet-50 (CIFAR) parameters
LENET = 431_080


@pytest.mark.parametrize("codec", ["none", "bf16", "qsgd", "topk_qsgd", "topk"])
def test_one_rank_keeps_the_single_graph(codec):
    p = plan_graph_mode(1, "local", codec, VGG)
    assert p["mode"] == "full" and p["wire_bytes"] == 0


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("codec", ["topk_qsgd", "topk"])
def test_topk_payloads_stay_in_one_graph(world, codec):
    p = plan_graph_mode(world, "rccl-stream", codec, R50, bucket_bytes=64 << 20)
    assert p["mode"] == "full" and p["bucket_bytes"] == 64 << 20


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dense_fp32_vgg_overlaps_at_n_gt_1(world):
    p = plan_graph_mode(world, "rccl-stream", "none", VGG, bucket_bytes=64 << 20)
    assert p["mode"] == "segmented"
    assert p["wire_bytes"] == int(2 * (world - 1) / world * 4 * VGG)
    assert p["splits"] == 2  # 39 MB of payload: one comm graph per 32 MiB
    # buckets on both sides of every split point
    assert 4 * VGG // p["bucket_bytes"] >= 2 * (p["splits"] + 1) - 1


def test_dense_resnet50_splits_are_capped():
    p = plan_graph_mode(8, "rccl-stream", "none", R50)
    assert p["mode"] == "segmented" and p["splits"] == 3
    assert p["bucket_bytes"] <= 16 << 20


def test_dense_qsgd_all_gather_grows_with_world():
    p2 = plan_graph_mode(2, "rccl-stream", "qsgd", VGG)
    p8 = plan_graph_mode(8, "rccl-stream", "qsgd", VGG)
    assert p8["wire_bytes"] == 7 * p2["wire_bytes"]
    assert p2["mode"] == p8["mode"] == "segmented"


def test_small_dense_collective_is_not_worth_a_split():
    p = plan_graph_mode(2, "rccl-stream", "none", LENET)
    assert p["wire_bytes"] < OVERLAP_MIN_WIRE_BYTES and p["mode"] == "full"


@pytest.mark.parametrize("kind", ["process-group", "local"])
def test_uncapturable_collectives_or_no_overlap(kind):
    assert plan_graph_mode(8, kind, "none", VGG)["mode"] == "full"
    assert plan_graph_mode(8, "rccl-stream", "none", VGG, overlap=False)["mode"] == "full"
