"""``--hip-graph auto`` decision for the all-to-all exchange (parallel/engine.plan_graph_mode) and
the N > 1 step model behind it (parallel/step_model.py): the one-graph step at N = 1; for a
configuration with measured N = 1 numbers, the mode the model predicts faster (and both
predictions, for the scaling run to be checked against); otherwise the codec-kind rule."""
import pytest

from ewdml.parallel import step_model as sm
from ewdml.parallel.engine import OVERLAP_MIN_WIRE_BYTES, plan_graph_mode

VGG = 9_756_426  # VGG-11-BN parameters
R50 = 23_520_842  # ResNet-50 (CIFAR) parameters
LENET = 431_080


@pytest.mark.parametrize("codec", ["none", "bf16", "qsgd", "topk_qsgd", "topk"])
def test_one_rank_keeps_the_single_graph(codec):
    p = plan_graph_mode(1, "local", codec, VGG, model="VGG11")
    assert p["mode"] == "full" and p["wire_bytes"] == 0


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("codec", ["topk_qsgd", "topk"])
@pytest.mark.parametrize("model", [None, "VGG11", "ResNet50"])
def test_topk_payloads_stay_in_one_graph(world, codec, model):
    """Model or rule: a few hundred KiB all-gather cannot repay the segmented step's cost."""
    p = plan_graph_mode(world, "rccl-stream", codec, R50 if model != "VGG11" else VGG,
                        bucket_bytes=64 << 20, model=model)
    assert p["mode"] == "full" and p["bucket_bytes"] == 64 << 20
    if model is not None:
        assert p["predicted_ms"]["full"] < p["predicted_ms"]["segmented"]
        assert p["reason"].startswith("step model")


def test_model_dense_vgg_overlaps_on_few_links_only():
    """Dense fp32 VGG-11 (39 MB all-reduce): with 1-3 xGMI links per rank the collective costs
    more than the segmented step's N = 1 penalty and overlap wins; at N = 8 (7 links) the
    all-reduce is short enough that the one-graph step is predicted faster."""
    modes = {w: plan_graph_mode(w, "rccl-stream", "none", VGG, bucket_bytes=64 << 20,
                                model="VGG11") for w in (2, 4, 8)}
    assert modes[2]["mode"] == modes[4]["mode"] == "segmented"
    assert modes[8]["mode"] == "full"
    for w, p in modes.items():
        assert p["wire_bytes"] == int(2 * (w - 1) / w * 4 * VGG)
        pr = p["predicted_ms"]
        assert (pr["segmented"] < pr["full"]) == (p["mode"] == "segmented")
    seg = modes[2]
    assert seg["splits"] == 2  # 39 MB of payload: one comm graph per 32 MiB
    assert 4 * VGG // seg["bucket_bytes"] >= 2 * (seg["splits"] + 1) - 1


def test_rule_without_a_profile():
    """No measured profile (e.g. an untuned model): dense collectives overlap, top-k stays one
    graph."""
    p = plan_graph_mode(8, "rccl-stream", "none", R50, model="resnet101")
    assert p["mode"] == "segmented" and p["splits"] == 3 and "predicted_ms" not in p
    assert p["bucket_bytes"] <= 16 << 20
    assert plan_graph_mode(8, "rccl-stream", "topk_qsgd", R50, model=None)["mode"] == "full"


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
    assert plan_graph_mode(8, kind, "none", VGG, model="VGG11")["mode"] == "full"
    assert plan_graph_mode(8, "rccl-stream", "none", VGG, overlap=False,
                           model="VGG11")["mode"] == "full"


def test_step_model_terms():
    prof = sm.profile_for("VGG11", "topk_qsgd")
    assert prof is not None and sm.profile_for("resnet50_imagenet", "none") is None
    # decode: measured points, linear in between
    assert prof.decode_at(1) == 10.7 and prof.decode_at(8) == 27.5
    assert 13.2 < prof.decode_at(3) < 18.4
    # collectives: zero on one rank, bandwidth term shrinks per peer as links are added
    assert sm.allgather_us(1, 1e6) == 0.0 and sm.allreduce_us(1, 1e6) == 0.0
    assert sm.bus_gbps(8) == 7 * sm.bus_gbps(2)
    big = 39e6
    assert sm.allreduce_us(8, big) < sm.allreduce_us(2, big)
    # the prediction at N = 1 is the measurement itself
    p1 = sm.predict(prof, 1, "topk_qsgd", 295296, 4 * VGG)
    assert p1["full"] == prof.full_ms and p1["comm_us"] == 0.0
    p8 = sm.predict(prof, 8, "topk_qsgd", 295296, 4 * VGG)
    assert p8["decode_delta_us"] == pytest.approx(27.5 - 10.7)
    assert prof.full_ms < p8["full"] < prof.full_ms * 1.1  # top-k: a few % at 8 ranks
