"""World 8 -- the target node's rank count -- on CPU/Gloo: the all-gather exchange's N = 8 payload
strides, the parameter server with 1 + 7 ranks, 8-way sharding, Method 6's best-worker choice
among 8, and the phase-timing summary over ranks (the reference exercised its
distributed path only as several ranks on one host, ``src/run_pytorch_single.sh:1-18``)."""
import json

import pytest
import torch

from .helpers import run_world
from .test_exchange import BASE, _same_params

pytestmark = pytest.mark.slow


def _train8(rank, world, flags, steps):
    import ewdml
    from ewdml.runtime import Trainer

    cfg = ewdml.parse_args(BASE + ["--synthetic-size", "1024"] + flags +
                           ["--max-steps", str(steps)])
    tr = Trainer(cfg)
    for _ in range(steps):
        tr.train_step()
    ex = tr.exchange
    return {"params": tr.flat.data.clone(), "payload": ex.last.payload_bytes,
            "dense": tr.flat.numel * 4, "wire_recv": ex.last.wire_bytes_recv,
            "best": list(getattr(ex, "best_rank_history", []))}


def test_world8_allgather_topk_qsgd(tmp_path):
    res = run_world(_train8, 8, tmp_path, args=(["--compress", "topk_qsgd", "--error-feedback",
                                                 "--ef-warmup", "none"], 3))
    _same_params(res)
    r = res[0]
    assert r["dense"] / r["payload"] >= 100
    assert r["wire_recv"] == 7 * r["payload"]  # seven peers' payloads


def test_world8_parameter_server_1_plus_7(tmp_path):
    res = run_world(_train8, 8, tmp_path, args=(["--topology", "ps", "--method", "5"], 3))
    _same_params(res)  # pull-grad: the server's replica tracks the 7 workers'


def test_world8_sharded(tmp_path):
    res = run_world(_train8, 8, tmp_path, args=(["--topology", "sharded", "--compress",
                                                 "topk_qsgd"], 3))
    _same_params(res)


def test_world8_method6_best_worker(tmp_path):
    res = run_world(_train8, 8, tmp_path, args=(["--method", "6", "--sync-every", "2"], 4))
    _same_params(res)  # after the step-4 sync every rank holds the winner's model
    assert all(r["best"] == res[0]["best"] for r in res) and len(res[0]["best"]) == 2
    assert all(0 <= b < 8 for b in res[0]["best"])


def _fit(rank, world, flags, out):
    import ewdml
    from ewdml.runtime import Trainer

    cfg = ewdml.parse_args(BASE + flags + ["--max-steps", "4", "--phase-timing",
                                           "--summary-file", out])
    return Trainer(cfg).fit()["summary"]


@pytest.mark.parametrize("flags,world", [(["--topology", "ps", "--method", "4"], 3),
                                         (["--compress", "topk_qsgd"], 2)])
def test_phase_timing_summary_over_ranks(tmp_path, flags, world):
    out = str(tmp_path / "summary.json")
    res = run_world(_fit, world, tmp_path, args=(flags, out))
    assert res[1:] == [None] * (world - 1)  # rank 0 writes it
    summ = json.load(open(out))
    assert summ["world"] == world and len(summ["ranks"]) == world
    for r in summ["ranks"]:
        assert r["comm_ms_mean"] > 0 and r["compute_ms_mean"] >= 0
        assert r["bytes_sent_total"] > 0 and r["bytes_recv_total"] > 0
    assert summ["max"]["comm_ms_mean"] >= summ["mean"]["comm_ms_mean"]
    if "ps" in flags:  # the server aggregates, the workers push and pull
        assert "aggregate" in summ["ranks"][0]["phase_ms_mean"]
        assert "forward" in summ["ranks"][1]["phase_ms_mean"]
