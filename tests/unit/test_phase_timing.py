"""--phase-timing: the step's timeline partitioned into forward / backward / encode /
collective / decode_update phases (the reference's per-worker send / fetch / computation times,
``src/distributed_worker.py:130-155, 214-231``), cumulative bytes in the JSONL, and rank 0's
summary.json with the communication / computation split."""
import json
import os

import pytest

import ewdml
from ewdml.parallel.engine import Stopwatch
from ewdml.runtime import Trainer

BASE = ["--network", "LeNet", "--dataset", "MNIST", "--batch-size", "32", "--synthetic-size",
        "512", "--momentum", "0.9", "--lr", "0.05", "--eval-freq", "0", "--quiet", "--device",
        "cpu", "--log-interval", "1", "--max-steps", "5", "--phase-timing"]


def _records(path):
    root, ext = os.path.splitext(path)
    with open(f"{root}.rank0{ext}") as f:
        return [json.loads(ln) for ln in f if ln.strip()]


@pytest.mark.parametrize("codec", ["topk_qsgd", "none"])
def test_phases_partition_the_step(tmp_path, codec):
    mf = str(tmp_path / "m.jsonl")
    tr = Trainer(ewdml.parse_args(BASE + ["--compress", codec, "--metrics-file", mf,
                                          "--train-dir", str(tmp_path)]))
    out = tr.fit()
    recs = [r for r in _records(mf) if "phase_ms" in r]
    assert len(recs) == 5
    for r in recs:
        ph = r["phase_ms"]
        for k in ("forward", "backward", "encode", "collective", "decode_update"):
            assert k in ph, (k, ph)
        part = sum(v for k, v in ph.items() if not k.startswith("side:"))
        # the phases are consecutive intervals of one timeline: they sum to the step time
        assert part == pytest.approx(r["step_ms"], rel=0.05, abs=0.05)
        assert r["comm_ms"] + r["compute_ms"] == pytest.approx(part, rel=1e-6, abs=1e-3)
    assert recs[-1]["payload_bytes_total"] == 5 * recs[-1]["payload_bytes_per_rank"]
    summ = json.load(open(tmp_path / "summary.json"))
    assert summ == out["summary"]
    assert summ["world"] == 1 and len(summ["ranks"]) == 1
    assert summ["mean"]["phase_ms_mean"]["forward"] > 0
    assert summ["max"]["compute_ms_mean"] >= summ["mean"]["compute_ms_mean"] > 0


def test_summary_without_phase_timing(tmp_path):
    tr = Trainer(ewdml.parse_args([a for a in BASE if a != "--phase-timing"] +
                                  ["--train-dir", str(tmp_path)]))
    tr.fit()
    summ = json.load(open(tmp_path / "summary.json"))
    r = summ["ranks"][0]
    assert r["steps"] == 5 and r["step_ms_mean"] > 0 and "phase_ms_mean" not in r


def test_stopwatch_split():
    comm, comp = Stopwatch.split({"forward": 1.0, "backward": 2.0, "collective": 0.5,
                                  "comm_wait": 0.25, "side:comm_graph": 9.0, "encode": 0.5})
    assert comm == 0.75 and comp == 3.5
