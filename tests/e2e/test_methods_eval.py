"""The measured Methods 1-6 harness (tools/methods_eval.py): its byte column equals the packed
layouts' (tools/methods_table.py, plus the flat buffer's alignment padding on dense legs) -- the
wire counters of a real 1-server + 2-worker Gloo run
move exactly the bytes the layouts predict.  Method 6 syncs compressed model deltas and adopts the
best worker's delta out of the same all-gather (no weight broadcast; LeNet has no BN buffers), so
it is Method 5's payload every 20 steps."""
import os
import sys

import pytest

pytestmark = pytest.mark.slow

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


@pytest.mark.parametrize("method", [1, 2, 3, 4, 5, 6])
def test_methods_eval_bytes_match_layouts(method):
    from tools.methods_eval import MiB, run_method
    from tools.methods_table import table

    steps = 20
    r = run_method(method, 0.4, steps, every=20, target=99.0)
    static = table("LeNet", 0.4)
    from ewdml.models import build_model
    from ewdml.parallel.flat import FlatModel

    flat = FlatModel(build_model("LeNet"))
    # dense payloads are the flat buffer: parameters + per-tensor 16-float alignment padding
    pad = 4 * (flat.numel - flat.param_numel) / MiB
    dense_legs = {1: 4, 2: 2, 3: 4}.get(method, 0)  # 2 workers x (push, pull) legs sent dense
    if method <= 5:
        expect = static[method - 1] + dense_legs * pad
    else:
        expect = static[4] / 20
    assert r["MiB_per_iter"] == pytest.approx(expect, rel=1e-9)
    assert 0 < r["top1"] <= 100


@pytest.mark.gpu
@pytest.mark.parametrize("method", [3, 5, 6])
def test_methods_eval_on_the_gpu_bytes_and_time_to_accuracy(method):
    """The MI355X path of the harness (three Gloo ranks sharing one GPU, HIP codecs and graphs):
    the same byte column as the layouts predict, and a time-to-accuracy record."""
    from ewdml.models import build_model
    from ewdml.parallel.flat import FlatModel
    from tools.methods_eval import MiB, run_method
    from tools.methods_table import table

    steps = 40
    r = run_method(method, 0.4, steps, every=20, target=99.0, device="cuda", targets=(10.0,))
    static = table("LeNet", 0.4)
    flat = FlatModel(build_model("LeNet"))
    pad = 4 * (flat.numel - flat.param_numel) / MiB
    expect = static[method - 1] + {3: 4}.get(method, 0) * pad if method <= 5 else static[4] / 20
    assert r["MiB_per_iter"] == pytest.approx(expect, rel=1e-9)
    assert r["device"] == "cuda" and r["train_s"] > 0
    assert "10.0" in r["hit"] and r["hit"]["10.0"][0] in (20, 40)
