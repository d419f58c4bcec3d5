"""End-to-end training on one MI355X through the HIP kernels: eager vs HIP-graph execution, the
flagship VGG-11 bf16 step, and the Horovod-style optimizer wrapper."""
import pytest
import torch

import ewdml
from ewdml import ops

pytestmark = pytest.mark.gpu

LENET = ["--network", "LeNet", "--dataset", "MNIST", "--batch-size", "32", "--synthetic-size",
         "1024", "--momentum", "0.9", "--lr", "0.05", "--eval-freq", "0", "--quiet", "--device",
         "cuda", "--amp", "none", "--graph-warmup", "2", "--no-error-feedback"]


def _run(flags, steps):
    from ewdml.runtime import Trainer

    torch.manual_seed(0)
    tr = Trainer(ewdml.parse_args(flags + ["--max-steps", str(steps)]))
    losses = []
    for _ in range(steps):
        loss, _ = tr.train_step()
        losses.append(float(loss.detach()))
    torch.cuda.synchronize()
    return tr, losses


@pytest.mark.parametrize("codec", ["topk_qsgd", "qsgd", "none", "bf16"])
def test_graph_modes_match_eager(codec):
    ops.require()
    import warnings

    ref, l_ref = _run(LENET + ["--compress", codec, "--hip-graph", "off"], 8)
    for mode in ("split", "full", "segmented"):
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            tr, l = _run(LENET + ["--compress", codec, "--hip-graph", mode], 8)
        # an empty trailing compute segment is dropped, not captured as an empty graph
        assert not [w for w in caught if "Graph is empty" in str(w.message)], mode
        assert tr.graph_mode == mode and tr._graphs is not None
        rel = (tr.flat.data - ref.flat.data).norm() / ref.flat.data.norm()
        assert rel < 1e-3, f"{mode}: params differ from eager by {rel:.2e}"
        assert abs(l[-1] - l_ref[-1]) < 1e-2


@pytest.mark.parametrize("extra", [["--compress", "topk_qsgd"],
                                   ["--compress", "topk_qsgd", "--error-feedback", "--ef-warmup",
                                    "none"],
                                   ["--compress", "none", "--optimizer", "adam", "--lr", "0.001"]])
def test_unrolled_graph_steps_bitwise_single_graph_steps(extra):
    """Trainer.train_steps(n, U): runs of U steps replayed as one graph (bench --graph-unroll)
    leave bitwise the parameters and loss of n one-step replays, across an epoch boundary (32
    batches per epoch: the runs stop before it and single steps cross it)."""
    from ewdml.runtime import Trainer

    ops.require()
    flags = LENET + extra + ["--hip-graph", "full"]
    res = []
    for unroll in (1, 4):
        torch.manual_seed(0)
        tr = Trainer(ewdml.parse_args(flags + ["--max-steps", "60"]))
        for _ in range(3):
            tr.train_step()
        loss, _ = tr.train_steps(38, unroll)
        torch.cuda.synchronize()
        assert tr.step == 41 and tr.opt.steps == 41
        assert (tr._ugraph is not None) == (unroll > 1)
        res.append((tr.flat.data.clone(), float(loss)))
    assert torch.equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1]


@pytest.mark.parametrize("opt", ["adam", "amsgrad"])
def test_adam_graph_matches_eager(opt):
    """Adam's bias correction follows the step count inside a replayed HIP graph (a device step
    counter, not the host value frozen at capture): graph and eager runs stay together."""
    ops.require()
    flags = LENET + ["--compress", "none", "--optimizer", opt, "--lr", "0.001"]
    ref, l_ref = _run(flags + ["--hip-graph", "off"], 10)
    for mode in ("split", "full"):
        tr, l = _run(flags + ["--hip-graph", mode], 10)
        assert tr._graphs is not None and tr.opt.steps == 10
        assert int(tr.opt.step_t.item()) == 10
        rel = float((tr.flat.data - ref.flat.data).norm() / ref.flat.data.norm())
        assert rel < 1e-4, f"{mode}: params differ from eager by {rel:.2e}"


@pytest.mark.parametrize("codec,splits", [("topk_qsgd", 2), ("none", 1), ("none", 3)])
def test_segmented_graph_matches_full_graph(codec, splits):
    """--hip-graph segmented (linear compute segments split at bucket boundaries, per-bucket
    encode + collective graphs on the comm stream, apply graph): same kernels on the same data
    as the one-graph step, so the trajectory is bitwise the full graph's; the comm graphs are
    real (several buckets, one launch each)."""
    ops.require()
    flags = ["--network", "VGG11", "--dataset", "Cifar10", "--batch-size", "32",
             "--synthetic-size", "512", "--momentum", "0.9", "--eval-freq", "0", "--quiet",
             "--device", "cuda", "--graph-warmup", "2", "--amp", "none", "--bucket-mb", "6",
             "--compress", codec, "--error-feedback", "--ef-warmup", "none"]
    full, lf = _run(flags + ["--hip-graph", "full"], 7)
    seg, ls = _run(flags + ["--hip-graph", "segmented", "--overlap-splits", str(splits)], 7)
    assert seg.graph_mode == "segmented" and seg._graphs[0] == "segmented"
    sc = seg._graphs[1]
    assert len(seg.flat.buckets) >= 3 and 1 <= len(sc.comms) <= splits
    assert len(sc.segments) == len(sc.comms) + 1
    # device hand-offs (the default): the apply rides in the last segment, no apply graph
    assert sc.device and sc.apply is None and sc.handoff_errors() == 0
    assert lf == ls
    assert torch.equal(full.flat.data, seg.flat.data)


def test_segmented_event_handoff_matches_device_handoff(monkeypatch):
    """The two segmented-step hand-offs (cross-stream events + an apply graph, or the device
    flag kernels of ops/csrc/stream_flag.hip with the apply in the last segment) run the same
    kernels on the same data: bitwise the same trajectory."""
    ops.require()
    flags = ["--network", "VGG11", "--dataset", "Cifar10", "--batch-size", "32",
             "--synthetic-size", "512", "--momentum", "0.9", "--eval-freq", "0", "--quiet",
             "--device", "cuda", "--graph-warmup", "2", "--amp", "none", "--bucket-mb", "6",
             "--compress", "none", "--hip-graph", "segmented", "--overlap-splits", "2"]
    res = []
    for mode in ("event", "device"):
        monkeypatch.setenv("EWDML_SEG_HANDOFF", mode)
        tr, l = _run(flags, 9)
        sc = tr._graphs[1]
        assert sc.device == (mode == "device") and len(sc.comms) >= 1
        assert sc.handoff_errors() == 0
        res.append((tr.flat.data.clone(), l))
    assert res[0][1] == res[1][1]
    assert torch.equal(res[0][0], res[1][0])


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_lr_schedule_in_graph_without_recapture(opt):
    """The learning rate lives in device memory (optim/flat.py DeviceScalar): a warm-up schedule
    changes it every step without re-capturing the step graph, and the trajectory follows the
    eager run's."""
    ops.require()
    flags = LENET + ["--compress", "topk_qsgd", "--optimizer", opt, "--lr-warmup-epochs", "1",
                     "--lr-warmup-start", "0.1", "--graph-warmup", "1"]
    if opt == "adam":
        flags += ["--compress", "none", "--lr", "0.001"]
    ref, _ = _run(flags + ["--hip-graph", "off"], 12)
    tr, _ = _run(flags + ["--hip-graph", "full"], 12)
    assert tr.captures == 1 and tr._graphs is not None
    assert float(tr.opt.lr_t.item()) == pytest.approx(tr.opt.lr)
    assert tr.opt.lr < tr.base_lr  # still warming up
    # LeNet's MIOpen convolutions are not bitwise between eager and captured runs, and a last-bit
    # difference can move a top-k choice: the same 1e-3 bound as test_graph_modes_match_eager
    rel = float((tr.flat.data - ref.flat.data).norm() / ref.flat.data.norm())
    assert rel < 1e-3, rel


def test_graph_replay_refreshes_rng_key():
    """The QSGD rounding key lives in device memory and changes every replay."""
    tr, _ = _run(LENET + ["--compress", "topk_qsgd", "--hip-graph", "full"], 5)
    k1 = int(tr.exchange.key_dev.item())
    tr.train_step()
    torch.cuda.synchronize()
    assert int(tr.exchange.key_dev.item()) != k1


def test_vgg11_bf16_full_graph_step():
    ops.require()
    flags = ["--network", "VGG11", "--dataset", "Cifar10", "--batch-size", "16",
             "--synthetic-size", "256", "--momentum", "0.9", "--eval-freq", "0", "--quiet",
             "--device", "cuda", "--hip-graph", "full", "--graph-warmup", "2", "--amp", "bf16",
             "--no-error-feedback"]
    tr, losses = _run(flags, 6)
    assert all(torch.isfinite(torch.tensor(losses)))
    assert tr.exchange.last.payload_bytes == 295312
    assert ops.library_path() is not None


def test_error_feedback_gpu_matches_cpu_oracle_one_step():
    """One EF step through the HIP path equals the CPU oracle path."""
    from ewdml.runtime import Trainer

    flags = LENET + ["--compress", "topk_qsgd", "--error-feedback", "--max-steps", "1"]
    torch.manual_seed(0)
    g = Trainer(ewdml.parse_args(flags))
    x, y = g.loader.next()
    c = Trainer(ewdml.parse_args([f if f != "cuda" else "cpu" for f in flags]))
    c.flat.data.copy_(g.flat.data.cpu())
    g.train_step(x, y)
    c.train_step(x.cpu(), y.cpu())
    torch.testing.assert_close(g.flat.data.cpu(), c.flat.data, rtol=1e-4, atol=1e-5)


def test_distributed_optimizer_on_gpu():
    import torch.nn.functional as F

    from ewdml.models import MnistNet

    m = MnistNet().cuda()
    opt = ewdml.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.5),
                                     compression=ewdml.Compression.qsgd())
    x = torch.randn(32, 1, 28, 28, device="cuda")
    y = torch.randint(0, 10, (32,), device="cuda")
    before = [p.detach().clone() for p in m.parameters()]
    for _ in range(3):
        opt.zero_grad()
        F.nll_loss(m(x), y).backward()
        opt.step()
    assert any(not torch.equal(b, p) for b, p in zip(before, m.parameters()))


def test_bf16_params_match_fp32_master_path(monkeypatch):
    """--param-dtype auto (bf16 compute copies of conv/linear weights) computes what autocast
    computes from fp32 parameters: same trajectory up to kernel nondeterminism.  (The fused
    classifier head only takes bf16 weights and draws its own dropout masks: both runs use
    PyTorch's head here so the masks match.)"""
    from ewdml.ops import head

    monkeypatch.setattr(head, "_ENABLED", False)
    base = ["--network", "VGG11", "--dataset", "Cifar10", "--batch-size", "32",
            "--synthetic-size", "256", "--momentum", "0.9", "--eval-freq", "0", "--quiet",
            "--device", "cuda", "--hip-graph", "off", "--compress", "topk_qsgd", "--amp", "bf16",
            "--no-error-feedback"]
    a, la = _run(base + ["--param-dtype", "auto"], 4)
    b, lb = _run(base + ["--param-dtype", "fp32"], 4)
    assert a.flat.shadow is not None and b.flat.shadow is None
    rel = (a.flat.data - b.flat.data).norm() / b.flat.data.norm()
    assert rel < 1e-3, rel
    assert abs(la[-1] - lb[-1]) < 5e-2
    # the bf16 compute copy equals the rounded master
    assert torch.equal(a.flat.shadow, a.flat.data.to(torch.bfloat16))


def test_bf16_params_checkpoint_holds_fp32_master(tmp_path):
    from ewdml.runtime import Trainer
    from ewdml.utils import checkpoint as ckpt

    flags = ["--network", "LeNet", "--dataset", "MNIST", "--batch-size", "32", "--synthetic-size",
             "256", "--eval-freq", "2", "--quiet", "--device", "cuda", "--max-steps", "2",
             "--train-dir", str(tmp_path) + "/", "--amp", "bf16"]
    tr = Trainer(ewdml.parse_args(flags))
    tr.fit()
    st = ckpt.load(ckpt.latest(str(tmp_path)))
    assert st["model"]["conv1.weight"].dtype == torch.float32
    torch.testing.assert_close(st["model"]["conv1.weight"].cuda(),
                               tr.flat.master_view(tr.model.conv1.weight))


def test_capture_after_single_eager_step():
    """bench.py may capture after one eager step (driver's --warmup 2): must work."""
    flags = ["--network", "VGG11", "--dataset", "Cifar10", "--batch-size", "16",
             "--synthetic-size", "256", "--momentum", "0.9", "--eval-freq", "0", "--quiet",
             "--device", "cuda", "--hip-graph", "full", "--graph-warmup", "1"]
    tr, losses = _run(flags, 4)
    assert tr._graphs is not None and all(torch.isfinite(torch.tensor(losses)))


def test_capture_failure_falls_back_to_eager(monkeypatch):
    """A capture that fails after the encode was forked onto the side stream (the unjoined case)
    must leave a trainer that keeps training eagerly, matching a never-graphed run."""
    from ewdml.runtime import Trainer

    ops.require()
    ref, _ = _run(LENET + ["--compress", "topk_qsgd", "--hip-graph", "off"], 6)
    torch.manual_seed(0)
    tr = Trainer(ewdml.parse_args(LENET + ["--compress", "topk_qsgd", "--hip-graph", "full",
                                           "--max-steps", "6"]))
    orig = tr.exchange.finish

    def finish(*a, **k):
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("injected capture failure")
        return orig(*a, **k)

    monkeypatch.setattr(tr.exchange, "finish", finish)
    losses = [float(tr.train_step()[0].detach()) for _ in range(6)]
    torch.cuda.synchronize()
    assert tr.graph_mode == "off" and tr._graphs is None
    assert all(l == l for l in losses)
    rel = (tr.flat.data - ref.flat.data).norm() / ref.flat.data.norm()
    assert rel < 1e-3, f"params differ from the eager run by {rel:.2e}"


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench_pg(codec, comm, extra=(), env_extra=None):
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, EWDML_FORCE_PG="1", EWDML_COMM=comm, **(env_extra or {}))
    for _ in range(2):  # a rendezvous port taken between _free_port and the launcher: a new port
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
               "1", "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
               "--gpus", "1", "--steps", "4", "--warmup", "4", "--batch-size", "64",
               "--compress", codec, "--no-extras", "--graph-unroll", "1", *extra]
        r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
        if not (r.returncode != 0 and "EADDRINUSE" in r.stderr and "failed to listen" in r.stderr):
            break
    if r.returncode != 0:
        errs = [ln for ln in r.stderr.splitlines()
                if ("rror" in ln or "what()" in ln or "Watchdog" in ln) and "frame #" not in ln]
        raise AssertionError("bench failed (rc %d):\n%s\n--- stdout tail:\n%s"
                             % (r.returncode, "\n".join(errs[:30]), r.stdout[-1500:]))
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("codec", ["topk_qsgd", "none"])
def test_own_rccl_communicator_matches_process_group(codec):
    """The stream-ordered RCCL communicator (ops/csrc/rccl_comm.hip) in a world of one
    (EWDML_FORCE_PG=1): the step graph captures its collectives, and the training trajectory is
    bit-identical to the same run with the collectives on the process group."""
    own = _bench_pg(codec, "rccl")
    pg = _bench_pg(codec, "pg")
    assert own["config"]["comm"] == "rccl-stream" and pg["config"]["comm"] == "process-group"
    # process-group collectives stay outside the graphs (split): their watchdog must not see an
    # event recorded inside a capture
    assert own["config"]["hip_graph"] == "full" and pg["config"]["hip_graph"] == "split"
    assert own["final_loss"] == pg["final_loss"]
    assert own["payload_bytes_per_rank"] == pg["payload_bytes_per_rank"]


def test_unrolled_bench_through_own_rccl_communicator():
    """bench.py's timed loop with 8 steps per graph launch through the own RCCL communicator
    (world 1, EWDML_FORCE_PG=1: the collectives are captured in the graph, eight sets of them in
    the unrolled one): the same final loss, bytes and healthy codec as one graph per step."""
    extra = ("--steps", "16", "--warmup", "12", "--graph-unroll")
    u8 = _bench_pg("topk_qsgd", "rccl", extra=extra + ("8",))
    u1 = _bench_pg("topk_qsgd", "rccl", extra=extra + ("1",))
    assert u8["config"]["comm"] == "rccl-stream" and u8["config"]["hip_graph"] == "full"
    assert u8["graph_unroll"] == 8 and u1["graph_unroll"] == 1
    # the same 28 steps (4 + one 8-step replay of warmup, then 16 timed) on both
    assert u8["warmup_steps_run"] == u1["warmup_steps_run"] == 12
    assert u8["final_loss"] == u1["final_loss"]
    assert u8["replicas_identical"] is not False
    assert "error" not in (u8["codec_health"] or {})
    assert u8["payload_bytes_per_rank"] == u1["payload_bytes_per_rank"]


def test_comm_probe_passes_and_failure_falls_back_to_process_group():
    """The first-contact probe of the own RCCL communicator (parallel/probe.py: rank-coded
    all-gather / all-reduce / broadcast, eager and captured in a HIP graph replayed twice) passes
    on the real communicator; with one rank's probe result corrupted (EWDML_PROBE_CORRUPT) the
    communicator is dropped and the step's collectives run on the process group with split
    graphs -- and the run still trains with identical bytes."""
    ok = _bench_pg("topk_qsgd", "rccl")
    assert ok["comm_probe"] == {"ok": True, "eager": True, "graph": True}
    assert ok["config"]["comm"] == "rccl-stream" and ok["config"]["hip_graph"] == "full"
    assert ok["replicas_identical"] is True and ok["rccl_world"] == 1
    bad = _bench_pg("topk_qsgd", "rccl", env_extra={"EWDML_PROBE_CORRUPT": "0:graph"})
    assert bad["comm_probe"]["ok"] is False and bad["comm_probe"]["eager"] is True
    assert bad["comm_probe"]["graph"] is False
    assert bad["config"]["comm"] == "process-group" and bad["config"]["hip_graph"] == "split"
    assert bad["rccl_world"] == 0
    assert bad["final_loss"] == ok["final_loss"]  # same trajectory on the fallback transport
    assert bad["payload_bytes_per_rank"] == ok["payload_bytes_per_rank"]


def test_auto_plan_at_n8_runs_segmented_through_rccl():
    """--hip-graph auto as planned for 8 ranks (EWDML_PLAN_AS_WORLD=8) on the real RCCL
    communicator (world of one) takes the mode the step model predicts faster
    (parallel/step_model.py), for the dense and the top-k exchange; and the segmented step --
    comm graphs with the all-reduce on their own stream beside backward -- runs through RCCL with
    the replicas check and the JSON fields holding."""
    for codec, extra in (("none", ("--error-feedback", "off")), ("topk_qsgd", ())):
        rec = _bench_pg(codec, "rccl", extra=extra, env_extra={"EWDML_PLAN_AS_WORLD": "8"})
        plan = rec["graph_plan"]
        pred = plan["predicted_ms"]
        want = "segmented" if pred["segmented"] < pred["full"] else "full"
        assert plan["mode"] == want and rec["config"]["hip_graph"] == want, (codec, plan)
        assert rec["predicted_ms_per_step"] == pred[want]
    dense = _bench_pg("none", "rccl", extra=("--error-feedback", "off", "--hip-graph", "segmented"),
                      env_extra={"EWDML_PLAN_AS_WORLD": "8"})
    assert dense["config"]["hip_graph"] == "segmented" and dense["overlap_comm_graphs"] >= 1
    assert dense["replicas_identical"] is True
    assert dense["final_loss"] == dense["final_loss"]


@pytest.mark.parametrize("codec", ["topk_qsgd", "none"])
def test_bench_through_rccl_process_group(codec):
    """bench.py under torch.distributed.run with a real RCCL communicator (world of one,
    EWDML_FORCE_PG=1): the multi-GPU code path -- RCCL all-gather of the packed payloads issued
    in place from the payload slot (or the dense all-reduce), captured in the step's HIP graph --
    that the 8-GPU scaling run takes, on the one GPU this box has."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, EWDML_FORCE_PG="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "1", "--steps", "4", "--warmup", "4", "--batch-size", "64",
           "--compress", codec, "--no-extras"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        errs = [ln for ln in r.stderr.splitlines()
                if ("rror" in ln or "what()" in ln or "Watchdog" in ln) and "frame #" not in ln]
        raise AssertionError("bench failed (rc %d):\n%s\n--- stdout tail:\n%s"
                             % (r.returncode, "\n".join(errs[:30]), r.stdout[-1500:]))
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["config"]["hip_graph"] == "full"  # the capture of the RCCL collective succeeded
    assert rec["config"]["comm"] == "rccl-stream"
    assert rec["value"] > 0 and rec["n_gpus"] == 1
    assert rec["final_loss"] == rec["final_loss"]  # not NaN


def test_method6_sync_graph_through_rccl():
    """Method 6 under torch.distributed.run with the own RCCL communicator (world of one,
    EWDML_FORCE_PG=1): the sync step -- compressed delta all-gather, the on-device best-worker
    choice (score all-gather, argmax) and the BN-buffer all-gathers -- is captured with its RCCL
    collectives, as the 8-GPU run needs."""
    rec = _bench_pg("topk_qsgd", "rccl", extra=("--extra=--method 6 --sync-every 3",))
    assert rec["config"]["comm"] == "rccl-stream" and rec["config"]["hip_graph"] == "full"
    assert rec["final_loss"] == rec["final_loss"]


@pytest.mark.parametrize("codec", ["topk_qsgd", "qsgd"])
def test_sharded_topology_hip_codecs(codec):
    """--topology sharded through the HIP codecs on shard plans (world of one: one shard per
    bucket, bucket_offset of the shard = the bucket's): lossless top-k equals the dense step, the
    compressing codecs train."""
    ops.require()
    ref, _ = _run(LENET + ["--compress", "none", "--hip-graph", "off"], 4)
    tr, _ = _run(LENET + ["--compress", "topk", "--topk-ratio", "1.0", "--topology", "sharded"], 4)
    # graph A (forward, backward, push encodes) -> eager collectives -> graph B (decode + step)
    assert tr.graph_mode == "split" and tr._graphs is not None
    rel = (tr.flat.data - ref.flat.data).norm() / ref.flat.data.norm()
    assert rel < 1e-5, f"sharded lossless top-k differs from dense by {rel:.2e}"
    tr, losses = _run(LENET + ["--compress", codec, "--topology", "sharded"], 6)
    assert all(torch.isfinite(torch.tensor(losses)))
    assert tr.exchange.last.payload_bytes > 0


def _ps_rank(rank, world, flags, steps):
    import os

    os.environ["LOCAL_RANK"] = "0"  # every rank on the box's one GPU (Gloo between them)
    from ewdml.runtime import Trainer

    torch.manual_seed(0)
    tr = Trainer(ewdml.parse_args(LENET + flags + ["--max-steps", str(steps)]))
    for _ in range(steps):
        tr.train_step()
    torch.cuda.synchronize()
    return {"params": tr.flat.data.cpu(), "mode": tr.graph_mode,
            "graphs": tr._graphs is not None, "bytes": tr.exchange.last.payload_bytes}


@pytest.mark.parametrize("method", [1, 4])
def test_ps_worker_split_graphs_match_eager(tmp_path, method):
    """Parameter-server workers (server + 2 workers on the one GPU, Gloo between them) run
    graph A (forward, backward, push encode with the step's device RNG key) -> eager gather /
    broadcast -> graph B (pull decode + update): same trajectory as the eager protocol."""
    from ..distributed.helpers import run_world

    ops.require()
    flags = ["--topology", "ps", "--method", str(method)]
    eager = run_world(_ps_rank, 3, tmp_path / "eager", args=(flags + ["--hip-graph", "off"], 6))
    graph = run_world(_ps_rank, 3, tmp_path / "graph", args=(flags + ["--hip-graph", "auto"], 6))
    for r in (1, 2):
        assert graph[r]["mode"] == "split" and graph[r]["graphs"]
        rel = float((graph[r]["params"] - eager[r]["params"]).norm() / eager[r]["params"].norm())
        assert rel < 1e-4, f"worker {r}: graph run differs from eager by {rel:.2e}"
    torch.testing.assert_close(graph[1]["params"], graph[2]["params"], rtol=0, atol=0)
    assert graph[1]["bytes"] == eager[1]["bytes"] > 0


@pytest.mark.parametrize("extra", [["--method", "6"],
                                   ["--compress", "topk_qsgd", "--sync-mode", "model"]])
def test_local_sgd_sync_graph_matches_eager(extra):
    """Local SGD (Method 6) captures two graphs -- the local step (fused pointer-table SGD on
    autograd's gradients) and the sync step (local step, model delta, compressed all-gather, the
    on-device best-worker choice, anchor update) -- and replays each at its steps: the trajectory
    is the eager one."""
    ops.require()
    flags = LENET + extra + ["--sync-every", "3"]
    ref, l_ref = _run(flags + ["--hip-graph", "off"], 10)
    tr, l = _run(flags + ["--hip-graph", "full"], 10)
    assert tr.graph_mode == "full" and tr.captures == 2
    assert tr._graphs is not None and any(v[0] is not None for v in tr._gslots.values())
    # eager and captured LeNet steps are not bitwise alike (test_graph_modes_match_eager)
    rel = float((tr.flat.data - ref.flat.data).norm() / ref.flat.data.norm())
    assert rel < 1e-5, f"graph run differs from eager by {rel:.2e}"
    assert tr.exchange.inner.step_idx == ref.exchange.inner.step_idx == 3
    assert max(abs(a - b) for a, b in zip(l, l_ref)) < 1e-4


def test_local_sgd_pointer_grads_match_views(monkeypatch):
    """Local steps read autograd's gradients through pointer tables (no accumulate-adds into
    attached .grad views): the views-mode trajectory."""
    ops.require()
    flags = LENET + ["--method", "6", "--sync-every", "3", "--hip-graph", "off"]
    ptr, _ = _run(flags, 7)
    assert not ptr.flat.attach_grads
    monkeypatch.setenv("EWDML_GRAD_VIEWS", "1")
    views, _ = _run(flags, 7)
    assert views.flat.attach_grads
    # LeNet's MIOpen convolutions are not run-to-run bitwise: compare at a tight tolerance
    rel = float((ptr.flat.data - views.flat.data).norm() / views.flat.data.norm())
    assert rel < 1e-5, f"pointer-mode local steps differ from views mode by {rel:.2e}"


def _m6_rank(rank, world, steps):
    import os

    os.environ["LOCAL_RANK"] = "0"  # both ranks on the box's one GPU (Gloo between them)
    from ewdml.runtime import Trainer

    torch.manual_seed(0)
    tr = Trainer(ewdml.parse_args(LENET + ["--method", "6", "--sync-every", "3", "--seed",
                                           str(rank), "--max-steps", str(steps)]))
    for _ in range(steps):
        tr.train_step()
    torch.cuda.synchronize()
    ex = tr.exchange
    return {"params": tr.flat.data.cpu(), "best": list(ex.best_rank_history),
            "bn": [b.cpu() for b in tr.model.buffers()], "mode": tr.graph_mode}


def test_method6_device_best_worker_two_ranks(tmp_path):
    """Method 6 with two ranks on the GPU: the on-device best-worker choice (all-gathered scores,
    argmax, the winner's payload row and BN buffers by index) leaves both replicas identical
    after every sync, with the same winner recorded on both."""
    from ..distributed.helpers import run_world

    ops.require()
    res = run_world(_m6_rank, 2, tmp_path, args=(6,))
    torch.testing.assert_close(res[0]["params"], res[1]["params"], rtol=0, atol=0)
    for a, b in zip(res[0]["bn"], res[1]["bn"]):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    assert res[0]["best"] == res[1]["best"] and len(res[0]["best"]) == 2


RESNET = ["--network", "ResNet50", "--dataset", "Cifar10", "--batch-size", "32",
          "--synthetic-size", "256", "--momentum", "0.9", "--lr", "0.02", "--eval-freq", "0",
          "--quiet", "--device", "cuda", "--amp", "none", "--graph-warmup", "2"]


@pytest.mark.parametrize("graph", ["off", "full", "segmented"])
@pytest.mark.parametrize("codec", ["topk_qsgd", "none"])
def test_wgrad_side_stream_is_bitwise_single_stream(graph, codec):
    """--wgrad-stream (ResNet-50: weight gradients of the MFMA convs on a second stream beside
    the backward-data chain, joined before any gradient is read) trains bit for bit as the
    single-stream step: eager, one captured graph (fork / join inside it) and segmented graphs
    (the exchange's bucket hooks join before they encode)."""
    ops.require()
    from ewdml.ops import conv as cv

    # deterministic runs to compare: MIOpen's stride-2 backward solvers accumulate with atomics
    # (run-to-run bits differ), so the six stride-2 convs take the MFMA kernels here
    cv.set_stride2(True)
    flags = RESNET + ["--compress", codec, "--hip-graph", graph]
    try:
        ref, l_ref = _run(flags + ["--wgrad-stream", "off"], 4)
        ref2, l_ref2 = _run(flags + ["--wgrad-stream", "off"], 4)
        assert l_ref2 == l_ref, "single-stream runs differ: nothing to compare against"
        _check_side_run(flags, ref, l_ref)
    finally:
        cv.set_stride2(False)
    ref.close()
    ref2.close()


def _check_side_run(flags, ref, l_ref):
    from ewdml.ops import conv as cv

    assert not ref.wgrad_stream
    before = cv.SIDE_LAUNCHES
    tr, l = _run(flags + ["--wgrad-stream", "auto"], 4)
    assert tr.wgrad_stream and cv.SIDE_LAUNCHES > before  # auto: on for ResNet-50
    assert l == l_ref
    assert torch.equal(tr.flat.data.view(torch.int32), ref.flat.data.view(torch.int32))
    assert not cv._WGRAD_SIDE and not cv._SIDE_QUEUE and not cv._SIDE_PENDING
    tr.close()


@pytest.mark.parametrize("ef", [True, False])
@pytest.mark.parametrize("graph", ["off", "full"])
def test_world_of_one_encode_apply_bitwise_decode(monkeypatch, graph, ef):
    """A world of one: the top-k write pass applies the update (GradientExchange.
    enable_local_apply, no decode launch) -- the trajectory is bitwise the one with the decode of
    the one-rank all-gather (EWDML_LOCAL_APPLY=0), eager and through the captured (unrolled)
    graphs, whose device RNG key the write pass now advances."""
    from ewdml.runtime import Trainer

    ops.require()
    flags = LENET + ["--compress", "topk_qsgd", "--hip-graph", graph, "--max-steps", "40"] + (
        ["--error-feedback", "--ef-warmup", "none"] if ef else [])  # (LENET: no EF otherwise)
    res = []
    for on in ("0", "1"):
        monkeypatch.setenv("EWDML_LOCAL_APPLY", on)
        torch.manual_seed(0)
        tr = Trainer(ewdml.parse_args(flags))
        assert tr.exchange.local_apply == (on == "1")
        for _ in range(4):
            tr.train_step()
        loss, _ = tr.train_steps(12, 4 if graph == "full" else 1)
        torch.cuda.synchronize()
        res.append((tr.flat.data.clone(), float(loss), tr.exchange.key_state.clone()))
        tr.close()
    assert torch.equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1]
    assert torch.equal(res[0][2], res[1][2])


@pytest.mark.parametrize("graph", ["off", "full"])
def test_producer_staging_bitwise_encode_staging(graph):
    """The small-map backward runs the exchange's momentum-corrected error-feedback staging for
    VGG-11's conv7 / conv8 weights itself (ops/csrc/dgc_stage.h: velocity and e written, the
    gradient never stored, the tensor stamped) and the encode reads e for those tensors: the
    trajectory -- parameters, residual, velocity -- is bitwise the one where the encode stages
    every tensor, eager and in the captured graph."""
    from ewdml.ops import conv as cmod
    from ewdml.runtime import Trainer

    ops.require()
    flags = ["--network", "VGG11", "--dataset", "Cifar10", "--batch-size", "64",
             "--synthetic-size", "1024", "--momentum", "0.9", "--lr", "0.02", "--eval-freq", "0",
             "--quiet", "--device", "cuda", "--amp", "none", "--graph-warmup", "2",
             "--compress", "topk_qsgd", "--error-feedback", "--ef-warmup", "none",
             "--hip-graph", graph, "--max-steps", "20"]
    res = []
    saved = cmod._PRODUCER_STAGE
    try:
        for on in (False, True):
            cmod._PRODUCER_STAGE = on
            rides = cmod.STAGE_RIDES
            torch.manual_seed(0)
            tr = Trainer(ewdml.parse_args(flags))
            for _ in range(8):
                tr.train_step()
            torch.cuda.synchronize()
            ex = tr.exchange
            assert (cmod.STAGE_RIDES > rides) == on
            res.append((tr.flat.data.clone(), ex.resid.clone(), ex.vel.clone()))
            if on:
                assert all(int(s.abs().sum()) == 0 for s in ex.stamps)  # re-armed by the encode
            tr.close()
    finally:
        cmod._PRODUCER_STAGE = saved
    for name, a, b in zip(("params", "resid", "vel"), *res):
        assert torch.equal(a, b), name
