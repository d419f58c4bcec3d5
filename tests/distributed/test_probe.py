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


def _probe_capture_fails(rank, world, bad_rank):
    """The graph phase on Gloo with stand-in capture / replay: the replay issues a collective (as
    the captured RCCL collectives do), so a rank replaying while a peer has no graph would hang."""
    os.environ["EWDML_PROBE_CORRUPT"] = f"{bad_rank}:capture"
    import torch.distributed as dist

    from ewdml.parallel import probe
    from ewdml.parallel.comm import Comm

    replays = []

    def capture(comm, device, fail=False):
        if fail:
            raise RuntimeError("injected")
        return "state"

    def replay(comm, device, state, corrupt):
        replays.append(state)
        t = torch.ones(4)
        dist.all_reduce(t)
        return bool(t[0] == world)

    probe._graph_supported = lambda device: True
    probe._graph_capture = capture
    probe._graph_replay = replay
    res = probe.probe_collectives(Comm(), "cpu", graph=True)
    res["replays"] = len(replays)
    return res


@pytest.mark.parametrize("bad_rank", [0, 1])
def test_probe_capture_failure_skips_every_replay(tmp_path, bad_rank):
    """a capture that raises on one rank makes every rank skip the replays (agreed
    before them) and fail the probe, instead of hanging its peers inside a replayed collective."""
    res = run_world(_probe_capture_fails, 2, tmp_path, args=(bad_rank,))
    assert [r["ok"] for r in res] == [False, False]
    assert [r["replays"] for r in res] == [0, 0]
    assert res[bad_rank]["error"] and "injected" in res[bad_rank]["error"]


def _probe_graph_ok(rank, world):
    from ewdml.parallel import probe
    from ewdml.parallel.comm import Comm

    probe._graph_supported = lambda device: True
    probe._graph_capture = lambda comm, device, fail=False: "state"
    probe._graph_replay = lambda comm, device, state, corrupt: not corrupt
    return probe.probe_collectives(Comm(), "cpu", graph=True)


def test_probe_graph_phase_passes_when_every_rank_captures(tmp_path):
    res = run_world(_probe_graph_ok, 2, tmp_path)
    assert all(r["ok"] and r["graph"] for r in res)
