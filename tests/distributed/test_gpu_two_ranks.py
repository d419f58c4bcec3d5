"""Two ranks sharing ``cuda:0`` over Gloo: the HIP top-k/QSGD codecs, the all-gather exchange and
the fused decode+SGD run with world 2 on the GPU (the 1-GPU box cannot host two RCCL ranks).
Gloo collectives cannot be captured into a HIP graph, so ``--hip-graph full`` also exercises the
cross-rank agreement of the capture fallback (``Trainer._try_capture``): every rank must drop to
eager together or the all-gather schedule would deadlock.  Reference pattern:
``src/run_pytorch_single.sh:1-18`` (several ranks on one host)."""
import pytest
import torch

from .helpers import run_world

pytestmark = pytest.mark.gpu

BASE = ["--network", "LeNet", "--dataset", "MNIST", "--batch-size", "16", "--synthetic-size",
        "512", "--momentum", "0.9", "--lr", "0.05", "--eval-freq", "0", "--quiet",
        "--device", "cuda", "--log-interval", "1000", "--no-error-feedback"]


def _train(rank, world, flags, steps):
    import os

    os.environ["LOCAL_RANK"] = "0"  # both ranks share the box's one GPU
    import ewdml
    from ewdml import ops
    from ewdml.runtime import Trainer

    torch.cuda.set_device(0)
    ops.require()
    cfg = ewdml.parse_args(BASE + flags + ["--max-steps", str(steps)])
    tr = Trainer(cfg)
    losses = []
    for _ in range(steps):
        loss, _ = tr.train_step()
        losses.append(None if loss is None else float(loss.detach()))
    torch.cuda.synchronize()
    return {"params": tr.flat.data.float().cpu(), "losses": losses,
            "bytes": tr.exchange.last.payload_bytes, "graph": tr.graph_mode}


@pytest.mark.parametrize("flags,graph", [
    (["--compress", "topk_qsgd", "--hip-graph", "off"], "off"),
    # gloo collectives cannot be captured: "full" is downgraded to split graphs up front
    (["--compress", "topk_qsgd", "--hip-graph", "full", "--graph-warmup", "1"], "split"),
    (["--compress", "topk_qsgd", "--hip-graph", "split", "--graph-warmup", "1"], "split"),
])
def test_two_ranks_on_one_gpu_identical(tmp_path, flags, graph):
    res = run_world(_train, 2, tmp_path, args=(flags, 4))
    assert torch.isfinite(res[0]["params"]).all()
    assert torch.equal(res[0]["params"], res[1]["params"])
    assert all(l is not None and l == l for l in res[0]["losses"])
    assert res[0]["bytes"] == res[1]["bytes"] > 0
    assert res[0]["graph"] == res[1]["graph"] == graph


@pytest.mark.parametrize("flags,graph", [
    (["--compress", "topk_qsgd", "--hip-graph", "auto", "--graph-warmup", "1"], "split"),
    (["--compress", "topk_qsgd", "--topology", "sharded", "--graph-warmup", "1"], "split"),
    (["--compress", "topk_qsgd", "--topology", "ps", "--graph-warmup", "1"], None),
])
def test_four_ranks_on_one_gpu_identical(tmp_path, flags, graph):
    """Four ranks on the box's one GPU (Gloo between them): the all-gather exchange with N = 4
    payload strides, the 4-way sharded exchange and a 1 + 3 parameter server, split-graphed where
    the topology allows; the replicas stay bitwise identical."""
    res = run_world(_train, 4, tmp_path, args=(flags, 4))
    assert torch.isfinite(res[0]["params"]).all()
    for r in res[1:]:
        assert torch.equal(res[0]["params"], r["params"])
    if graph is not None:
        assert all(r["graph"] == graph for r in res)
    else:  # parameter server: the workers split-graph, the server captures nothing
        assert all(r["graph"] == "split" for r in res[1:])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("ef", [False, True])
def test_eight_ranks_on_one_gpu_identical(tmp_path, ef):
    """Eight ranks on the box's one GPU (Gloo between them, the size of the 8-GPU node): the HIP
    encode, the all-gather of 8 payload slots and the rank-ordered decode of all 8 (past the 8
    ranks whose first entries the decode prefetches) keep the replicas bitwise identical, with
    and without momentum-corrected error feedback (the headline codec)."""
    flags = ["--compress", "topk_qsgd", "--hip-graph", "auto", "--graph-warmup", "1"]
    if ef:
        flags += ["--error-feedback"]
    res = run_world(_train, 8, tmp_path, args=(flags, 3))
    assert torch.isfinite(res[0]["params"]).all()
    for r in res[1:]:
        assert torch.equal(res[0]["params"], r["params"])
        assert r["bytes"] == res[0]["bytes"] > 0
    assert all(r["graph"] == "split" for r in res)
