"""First-contact self-validation of a multi-rank run (CPU/Gloo, world 2 and 8):

* the collective probe (parallel/probe.py) passes on a healthy transport and, when one rank's
  result is corrupted (test hook EWDML_PROBE_CORRUPT), every rank reaches the same failed verdict
  (on the GPU the own RCCL communicator is then dropped everywhere:
  tests/e2e/test_gpu_train.py::test_comm_probe_failure_falls_back_to_process_group);
* the replica fingerprint check that bench.py runs after its timed steps flags a rank whose
  parameters differ by one bit."""
import os

import pytest
import torch

from .helpers import run_world

pytestmark = pytest.mark.slow


def _probe(rank, world, corrupt):
    if corrupt is not None:
        os.environ["EWDML_PROBE_CORRUPT"] = corrupt
    from ewdml.parallel.comm import Comm
    from ewdml.parallel.probe import probe_collectives

    return probe_collectives(Comm(), "cpu", graph=False)


@pytest.mark.parametrize("world", [2, 8])
def test_probe_passes_on_a_healthy_transport(tmp_path, world):
    res = run_world(_probe, world, tmp_path, args=(None,))
    assert all(r["ok"] and r["local_ok"] and r["eager"] for r in res)


def test_probe_failure_on_one_rank_is_agreed_by_all(tmp_path):
    res = run_world(_probe, 2, tmp_path, args=("1",))
    assert [r["ok"] for r in res] == [False, False]
    assert res[0]["local_ok"] and not res[1]["local_ok"]


def _replicas(rank, world, flip):
    from ewdml.parallel.comm import Comm
    from ewdml.parallel.engine import check_replicas

    t = torch.linspace(-1, 1, 10007)
    if flip and rank == world - 1:
        t.view(torch.int32)[5000] ^= 1  # one bit of one parameter
    return check_replicas(Comm(), t)


@pytest.mark.parametrize("flip", [False, True])
def test_replica_check(tmp_path, flip):
    res = run_world(_replicas, 2, tmp_path, args=(flip,))
    assert [r["identical"] for r in res] == [not flip] * 2
