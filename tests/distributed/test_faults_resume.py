"""Checkpoint/resume and failure handling on CPU/Gloo (SURVEY sections 5.3-5.4)."""
import os
import subprocess
import sys

import pytest
import torch

from .helpers import free_port, run_world

pytestmark = pytest.mark.slow
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BASE = ["--network", "LeNet", "--dataset", "MNIST", "--batch-size", "16", "--synthetic-size",
        "512", "--momentum", "0.9", "--lr", "0.05", "--quiet", "--device", "cpu",
        "--log-interval", "1000", "--compress", "topk_qsgd", "--error-feedback"]


def _fit(rank, world, flags):
    import ewdml
    from ewdml.runtime import Trainer

    tr = Trainer(ewdml.parse_args(BASE + flags))
    tr.fit()
    return {"params": tr.flat.data.clone(), "mom": tr.opt.mom.clone(), "step": tr.step}


def test_resume_reproduces_uninterrupted_run(tmp_path):
    full = run_world(_fit, 2, tmp_path / "a", args=(["--max-steps", "6", "--eval-freq", "0",
                                                     "--train-dir", str(tmp_path / "ca") + "/"],))
    d = str(tmp_path / "cb") + "/"
    run_world(_fit, 2, tmp_path / "b", args=(["--max-steps", "3", "--eval-freq", "3",
                                              "--train-dir", d],))
    assert os.path.islink(os.path.join(d, "latest"))
    assert os.path.exists(os.path.join(d, "model_step_"))
    res = run_world(_fit, 2, tmp_path / "c", args=(["--max-steps", "6", "--eval-freq", "0",
                                                    "--resume", "--train-dir", d],))
    assert res[0]["step"] == 6
    assert torch.equal(res[0]["params"], full[0]["params"])
    assert torch.equal(res[0]["mom"], full[0]["mom"])
    assert torch.equal(res[1]["params"], res[0]["params"])


def test_local_sgd_resume_reproduces_uninterrupted_run(tmp_path):
    """Method 6 (compressed model deltas, best-worker choice) resumed between two syncs: every
    rank's drifted replica and momentum, the common anchor and the sync count come back, so the
    run continues exactly as the uninterrupted one."""
    m6 = ["--method", "6", "--sync-every", "4", "--eval-freq", "0"]
    full = run_world(_fit, 2, tmp_path / "a", args=(m6 + ["--max-steps", "9", "--train-dir",
                                                          str(tmp_path / "ca") + "/"],))
    d = str(tmp_path / "cb") + "/"
    run_world(_fit, 2, tmp_path / "b", args=(m6[:-1] + ["3", "--max-steps", "6",
                                                        "--train-dir", d],))
    res = run_world(_fit, 2, tmp_path / "c", args=(m6 + ["--max-steps", "9", "--resume",
                                                         "--train-dir", d],))
    for r in (0, 1):
        assert res[r]["step"] == 9
        assert torch.equal(res[r]["params"], full[r]["params"])
        assert torch.equal(res[r]["mom"], full[r]["mom"])


def test_injected_fault_aborts_all_ranks_without_hang(tmp_path):
    port = free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE="2", LOCAL_RANK=str(r), PYTHONPATH=ROOT)
        cmd = [sys.executable, os.path.join(ROOT, "distributed_nn.py")] + BASE + [
            "--max-steps", "50", "--eval-freq", "0", "--inject-fault", "1:2",
            "--comm-timeout", "60", "--train-dir", str(tmp_path) + "/"]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    codes = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=180)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError("a rank hung after the injected fault")
        codes.append(p.returncode)
    assert codes[1] != 0  # the faulty rank
    assert codes[0] != 0  # the healthy rank aborts too instead of hanging


REF_CKPT = "/root/reference/PyTorch-parameter-server/src/model_step_.zip"


@pytest.mark.skipif(not os.path.exists(REF_CKPT), reason="reference checkout not mounted")
def test_reference_lenet_checkpoint_loads():
    """The reference ships a LeNet state_dict (torch zip format); it loads into our LeNet with the
    safe loader, and our evaluator path can score it."""
    from ewdml.models import build_model

    sd = torch.load(REF_CKPT, map_location="cpu", weights_only=True)
    m = build_model("LeNet")
    m.load_state_dict(sd)
    assert sum(v.numel() for v in sd.values()) == 431080
    with torch.no_grad():
        assert m(torch.zeros(1, 1, 28, 28)).shape == (1, 10)


def _fit_bn(rank, world, flags):
    import ewdml
    from ewdml.runtime import Trainer

    tr = Trainer(ewdml.parse_args(flags))
    tr.fit()
    bn = [m for m in tr.model.modules() if isinstance(m, torch.nn.BatchNorm2d)][0]
    return {"rm": bn.running_mean.clone(), "nbt": int(bn.num_batches_tracked)}


def test_ps_topology_checkpoint_holds_worker_bn_statistics(tmp_path):
    """Parameter-server topology with a BN model: rank 0 (the server) never runs a forward, so
    the checkpoint it writes must carry the first worker's running statistics, not the initial
    ones; the other workers keep their own."""
    d = str(tmp_path / "ck") + "/"
    flags = ["--network", "VGG11", "--dataset", "Cifar10", "--batch-size", "4",
             "--synthetic-size", "64", "--momentum", "0.9", "--lr", "0.01", "--quiet",
             "--device", "cpu", "--log-interval", "1000", "--topology", "ps", "--compress",
             "none", "--amp", "none", "--max-steps", "2", "--eval-freq", "2", "--train-dir", d]
    res = run_world(_fit_bn, 3, tmp_path / "w", args=(flags,))
    assert res[1]["nbt"] == 2 and float(res[1]["rm"].abs().sum()) > 0
    from ewdml.utils import checkpoint as ckpt

    st = ckpt.load(ckpt.latest(d))
    rm = [v for k, v in st["model"].items() if k.endswith("running_mean")][0]
    nbt = [v for k, v in st["model"].items() if k.endswith("num_batches_tracked")][0]
    assert int(nbt) == 2
    torch.testing.assert_close(rm, res[1]["rm"])
    # worker 2 kept its own statistics (different data shard)
    assert not torch.equal(res[2]["rm"], res[1]["rm"])
