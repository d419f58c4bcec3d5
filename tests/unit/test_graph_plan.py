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


@pytest.mark.parametrize("model,numel,worlds", [("VGG11", VGG, (2, 4, 8)),
                                                 ("ResNet50", R50, (2, 4))])
def test_model_dense_collectives_overlap(model, numel, worlds):
    """Dense fp32 all-reduce (VGG-11 39 MB, ResNet-50 94 MB) with the calibrated N = 1 profiles:
    the segmented step's measured world-1 penalty (device stream hand-offs: 83 us on VGG-11) is
    below what overlapping the all-reduce with backward hides at these worlds, so the model picks
    segmented; at every world the mode is the one predicted faster."""
    for w in (2, 4, 8):
        p = plan_graph_mode(w, "rccl-stream", "none", numel, bucket_bytes=64 << 20, model=model)
        assert p["wire_bytes"] == int(2 * (w - 1) / w * 4 * numel)
        pr = p["predicted_ms"]
        assert p["mode"] == ("segmented" if pr["segmented"] < pr["full"] else "full")
        if w in worlds:
            assert p["mode"] == "segmented", (w, pr)
    seg = plan_graph_mode(2, "rccl-stream", "none", numel, bucket_bytes=64 << 20, model=model)
    assert seg["splits"] >= 2  # >= 39 MB of payload: one comm graph per 32 MiB
    assert 4 * numel // seg["bucket_bytes"] >= 2 * (seg["splits"] + 1) - 1


def test_half_codec_all_reduce_bytes():
    """a bf16 all-reduce moves 2 bytes per element, not 4 (its collective term is
    half the fp32 one's)."""
    p32 = plan_graph_mode(4, "rccl-stream", "none", VGG, bucket_bytes=64 << 20, model="VGG11")
    p16 = plan_graph_mode(4, "rccl-stream", "bf16", VGG, bucket_bytes=64 << 20, model="VGG11")
    assert p16["wire_bytes"] * 2 == p32["wire_bytes"]
    assert p16["predicted_ms"]["comm_us"] < 0.55 * p32["predicted_ms"]["comm_us"]


def test_model_error_n1_on_committed_preset_lines():
    """The step model at N = 1 against the committed preset lines of this round's kernels
    (bench.py model_error_n1): within 3 % on every BASELINE preset, top-k and dense."""
    import json
    import os

    lines = []
    for name in ("bench_presets_r06.jsonl", "bench_presets_r06_final.jsonl"):
        path = os.path.join(os.path.dirname(__file__), "..", "..", "profiles", "validation", name)
        lines += [json.loads(l) for l in open(path) if l.startswith("{")]
    assert len(lines) >= 10
    for r in lines:
        c = r["config"]
        model = {"vgg11_bn": "VGG11"}.get(c["model"], c["model"])
        codec = "none" if c["codec"] == "none" else "topk_qsgd"
        prof = sm.profile_for(model, codec, r["dtype"])
        assert prof is not None, (model, codec)
        pred = sm.predict(prof, 1, codec, r["payload_bytes_per_rank"], 4 * 1e6)["full"]
        err = pred / r["ms_per_step"] - 1
        assert abs(err) <= 0.03, (model, codec, pred, r["ms_per_step"])


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
    assert prof is not None and sm.profile_for("resnet101", "none") is None
    assert sm.profile_for("VGG11", "topk_qsgd", "bf16") is None  # fp32 profiles only
    # decode: measured points, linear in between
    d = {int(k): v for k, v in prof.decode_us.items()}
    assert prof.decode_at(1) == d[1] and prof.decode_at(8) == d[8]
    assert d[2] < prof.decode_at(3) < d[4]
    # collectives: zero on one rank, bandwidth term shrinks per peer as links are added
    assert sm.allgather_us(1, 1e6) == 0.0 and sm.allreduce_us(1, 1e6) == 0.0
    assert sm.bus_gbps(8) == 7 * sm.bus_gbps(2)
    big = 39e6
    assert sm.allreduce_us(8, big) < sm.allreduce_us(2, big)
    # the prediction at N = 1 is the measurement itself
    p1 = sm.predict(prof, 1, "topk_qsgd", 295296, 4 * VGG)
    assert p1["full"] == prof.full_ms and p1["comm_us"] == 0.0
    p8 = sm.predict(prof, 8, "topk_qsgd", 295296, 4 * VGG)
    assert p8["decode_delta_us"] == pytest.approx(d[8] - d[1])
    assert prof.full_ms < p8["full"] < prof.full_ms * 1.1  # top-k: a few % at 8 ranks
