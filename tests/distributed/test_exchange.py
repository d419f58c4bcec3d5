"""Multi-process exchange tests on CPU/Gloo (BASELINE.json config #1: LeNet, world_size=2,
top-k 1 % + QSGD, plumbing without a GPU)."""
import os

import pytest
import torch

from .helpers import run_world

pytestmark = pytest.mark.slow

BASE = ["--network", "LeNet", "--dataset", "MNIST", "--batch-size", "16", "--synthetic-size",
        "512", "--momentum", "0.9", "--lr", "0.05", "--eval-freq", "0", "--quiet",
        "--device", "cpu", "--log-interval", "1000", "--no-error-feedback"]


def _train(rank, world, flags, steps):
    import ewdml
    from ewdml.runtime import Trainer

    cfg = ewdml.parse_args(BASE + flags + ["--max-steps", str(steps)])
    tr = Trainer(cfg)
    losses = []
    for _ in range(steps):
        loss, _ = tr.train_step()
        losses.append(None if loss is None else float(loss))
    return {"params": tr.flat.data.clone(), "losses": losses,
            "bytes": tr.exchange.last.payload_bytes, "rank": rank}


def _same_params(results, ranks=None):
    ranks = ranks if ranks is not None else range(len(results))
    ps = [results[r]["params"] for r in ranks]
    for p in ps[1:]:
        assert torch.equal(p, ps[0])


@pytest.mark.parametrize("flags", [
    ["--compress", "topk_qsgd"],
    ["--compress", "topk_qsgd", "--qsgd-bits", "4", "--qsgd-levels", "7"],
    ["--compress", "topk", "--topk-ratio", "0.05"],
    ["--compress", "qsgd", "--qsgd-norm", "l2"],
    ["--compress", "none"],
    ["--compress", "bf16"],
    ["--compress", "topk_qsgd", "--error-feedback"],
    ["--compress", "topk_qsgd", "--error-feedback", "--ef-mode", "plain"],
    ["--compress", "topk_qsgd", "--error-feedback", "--weight-decay", "5e-4", "--nesterov",
     "--topk-warmup", "0.25,0.05", "--topk-warmup-epochs", "0.25", "--topk-dense-below", "64"],
    ["--compress", "topk_qsgd", "--no-overlap", "--bucket-mb", "0.5"],
])
def test_allgather_replicas_identical(tmp_path, flags):
    res = run_world(_train, 2, tmp_path, args=(flags, 4))
    _same_params(res)
    assert all(res[0]["losses"])


def _warmup_schedule(rank, world):
    import ewdml
    from ewdml.runtime import Trainer

    cfg = ewdml.parse_args(BASE + ["--compress", "topk_qsgd", "--error-feedback", "--topk-warmup",
                                   "0.25,0.0625", "--topk-warmup-epochs", "1", "--max-steps",
                                   "40"])
    tr = Trainer(cfg)
    spe = len(tr.loader)
    seen = []
    for _ in range(2 * spe + 1):
        tr.train_step()
        seen.append((tr.exchange.codec.ratio, tr.exchange.last.payload_bytes))
    return {"seen": seen, "spe": spe, "ef": tr.exchange.ef_mode,
            "params": tr.flat.data.clone()}


def test_topk_warmup_schedule(tmp_path):
    """--topk-warmup: 25 % for the first half epoch, 6.25 % for the second, then --topk-ratio;
    payload sizes follow; replicas stay identical; momentum-corrected EF by default."""
    res = run_world(_warmup_schedule, 2, tmp_path)
    _same_params(res)
    seen, spe = res[0]["seen"], res[0]["spe"]
    half = spe // 2
    assert res[0]["ef"] == "dgc"
    assert all(r == 0.25 for r, _ in seen[:half])
    assert all(r == 0.0625 for r, _ in seen[half + 1:spe])
    assert all(r == 0.01 for r, _ in seen[spe:])
    assert seen[0][1] > seen[spe - 1][1] > seen[-1][1]


def test_world3_topk_qsgd_identical(tmp_path):
    res = run_world(_train, 3, tmp_path, args=(["--compress", "topk_qsgd"], 3))
    _same_params(res)


def test_dense_allreduce_equals_average(tmp_path):
    res = run_world(_worker_dense, 2, tmp_path)
    # single-process reference: average grads of both batches
    import torch.nn.functional as F
    from ewdml.models import build_model
    from ewdml.parallel.flat import FlatModel

    m = build_model("LeNet")
    flat = FlatModel(m, bucket_bytes=16 << 20)
    flat.data.copy_(res[0]["p0"])
    g = torch.zeros_like(flat.grad)
    for r in res:
        flat.zero_grad()
        F.cross_entropy(m(r["x"]), r["y"]).backward()
        g += flat.grad
    g /= 2
    lr = 0.05
    expected = res[0]["p0"] - lr * g  # first step: momentum buffer = g
    torch.testing.assert_close(res[0]["p1"], expected, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(res[1]["p1"], res[0]["p1"], rtol=0, atol=0)


def _worker_dense(rank, world):
    import ewdml
    from ewdml.runtime import Trainer

    cfg = ewdml.parse_args(BASE + ["--compress", "none", "--max-steps", "1", "--amp", "none"])
    tr = Trainer(cfg)
    x, y = tr.loader.next()
    p0 = tr.flat.data.clone()
    tr.train_step(x, y)
    return {"p0": p0, "p1": tr.flat.data.clone(), "x": x, "y": y}


@pytest.mark.parametrize("method", [1, 2, 3, 4, 5])
def test_ps_topology_methods(tmp_path, method):
    flags = ["--method", str(method), "--topology", "ps"]
    res = run_world(_train, 3, tmp_path, args=(flags, 3))
    _same_params(res, [1, 2])  # workers identical
    if method >= 3:  # pull-grad: the server's replica tracks the workers'
        _same_params(res)
    assert res[0]["losses"] == [None, None, None]


def test_ps_matches_allreduce_dense(tmp_path):
    ps = run_world(_train, 3, tmp_path / "ps",
                   args=(["--topology", "ps", "--compress", "none", "--amp", "none"], 3))
    ar = run_world(_train, 2, tmp_path / "ar",
                   args=(["--compress", "none", "--amp", "none"], 3))
    torch.testing.assert_close(ps[1]["params"], ar[0]["params"], rtol=1e-5, atol=1e-6)


def test_method6_local_sgd_select_best(tmp_path):
    res = run_world(_train, 2, tmp_path, args=(["--method", "6", "--sync-every", "3"], 6))
    _same_params(res)  # after the step-6 sync everyone holds the best rank's weights


def _method6(rank, world, ef=False):
    import ewdml
    from ewdml.runtime import Trainer

    cfg = ewdml.parse_args(BASE + ["--method", "6", "--sync-every", "3", "--max-steps", "3"] +
                           (["--error-feedback"] if ef else []))
    tr = Trainer(cfg)
    ex = tr.exchange
    for _ in range(2):
        tr.train_step()
    tr.loader.seek(2)
    x, y = tr.loader.next()
    anchor = ex.anchor.clone()
    tr.train_step(x, y)  # the sync step
    best = ex.best_rank_history[-1]
    inner = ex.inner
    rows = inner.recv[0].view(inner.N, -1)
    delta = torch.zeros_like(tr.flat.grad)
    inner.codec.decode(0, rows[best:best + 1], delta, 1.0)
    resid = inner.resid
    return {"mode": ex.mode, "params": tr.flat.data.clone(), "expect": anchor + delta,
            "wire": ex.last.wire_bytes_sent + ex.last.wire_bytes_recv,
            "dense": tr.flat.numel * 4, "nb": len(tr.flat.buckets), "best": best,
            "resid": None if resid is None else float(resid.abs().sum())}


def test_method6_adopts_the_winners_compressed_delta(tmp_path):
    """--method 6 defaults to compressed model-delta sync: every rank applies the best rank's
    compressed delta out of the all-gather (no dense weight broadcast)."""
    res = run_world(_method6, 2, tmp_path)
    _same_params(res)
    r = res[0]
    assert r["mode"] == "model" and r["nb"] == 1
    torch.testing.assert_close(r["params"], r["expect"], rtol=0, atol=0)
    assert r["wire"] < r["dense"] / 20  # a compressed payload each way, no dense weights


def test_method6_error_feedback_keeps_only_the_winners_residual(tmp_path):
    """Method 6 with error feedback (the CLI default for top-k codecs): every rank adopts
    anchor + decode(winner's payload) as documented in parallel/local_sgd.py; the winner keeps the
    part of its delta that top-k dropped in its residual (sent with its next delta), the other
    ranks zero theirs."""
    res = run_world(_method6, 2, tmp_path, args=(True,))
    _same_params(res)
    best = res[0]["best"]
    assert res[1]["best"] == best
    for r in res:
        torch.testing.assert_close(r["params"], r["expect"], rtol=0, atol=0)
    assert res[best]["resid"] > 0
    assert res[1 - best]["resid"] == 0


def test_local_sgd_grad_mode_resyncs_replicas(tmp_path):
    """grad mode without best-worker selection: local steps drift the replicas apart; every sync
    point re-broadcasts rank 0's weights, so after a sync step all ranks hold the same model."""
    res = run_world(_train, 2, tmp_path, args=(["--compress", "topk_qsgd", "--sync-every", "3",
                                                "--sync-mode", "grad"], 6))
    _same_params(res)


def test_local_sgd_model_mode(tmp_path):
    res = run_world(_train, 2, tmp_path,
                    args=(["--compress", "topk_qsgd", "--topk-ratio", "0.2", "--sync-every", "2",
                           "--sync-mode", "model"], 4))
    _same_params(res)


def test_payload_bytes_lenet(tmp_path):
    res = run_world(_train, 2, tmp_path, args=(["--compress", "topk_qsgd"], 1))
    assert res[0]["bytes"] == res[1]["bytes"]
    assert 431080 * 4 / res[0]["bytes"] > 125


def _train_slow(rank, world, flags, steps, slow_rank, delay):
    import time

    import ewdml
    from ewdml.runtime import Trainer

    cfg = ewdml.parse_args(BASE + flags + ["--max-steps", str(steps)])
    tr = Trainer(cfg)
    chosen = []
    for _ in range(steps):
        if rank == slow_rank:
            time.sleep(delay)  # a straggler: its push arrives after the others'
        tr.train_step()
        if rank == 0:
            chosen.append(list(tr.exchange.last_aggregated))
    return {"params": tr.flat.data.clone(), "chosen": chosen}


def test_ps_k_of_n_aggregation_drops_straggler(tmp_path):
    """--mode kill --num-aggregate 2 with 3 workers: the server averages the first two pushes to
    arrive, so a consistently slow worker is left out every step; replicas stay identical."""
    flags = ["--topology", "ps", "--mode", "kill", "--num-aggregate", "2", "--compress", "none",
             "--amp", "none"]
    res = run_world(_train_slow, 4, tmp_path, args=(flags, 3, 3, 0.6))
    assert res[0]["chosen"] == [[1, 2]] * 3
    _same_params(res)


def test_ps_kill_threshold_aborts_on_a_stalled_worker(tmp_path):
    """A worker still missing --kill-threshold seconds after the k-th push arrived aborts the job
    (the server raises) instead of hanging it; the threshold applies to that push only."""
    flags = ["--topology", "ps", "--mode", "kill", "--num-aggregate", "1", "--compress", "none",
             "--amp", "none", "--kill-threshold", "0.5", "--comm-timeout", "60"]
    assert run_world(_train_slow, 3, tmp_path, args=(flags, 2, 2, 4.0), expect_fail=True) is None
    err = [f for f in tmp_path.iterdir() if f.name.endswith(".err")]
    assert any("did not push bucket" in f.read_text() for f in err)


def test_ps_k_of_n_inactive_without_kill_mode(tmp_path):
    flags = ["--topology", "ps", "--num-aggregate", "1", "--compress", "none", "--amp", "none"]
    res = run_world(_train_slow, 3, tmp_path, args=(flags, 2, 2, 0.0))
    assert res[0]["chosen"] == [[1, 2]] * 2
