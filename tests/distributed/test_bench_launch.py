"""bench.py under the driver's exact multi-rank launch line (torch.distributed.run, one rank per
device, MASTER_ADDR 127.0.0.1), on CPU/Gloo with two ranks: the JSON contract, whole-job
aggregation and the dp-N config fields.  The GPU variant (RCCL, one rank) is
`tests/e2e/test_gpu_train.py::test_bench_through_rccl_process_group`."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.slow

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("preset,batch", [("lenet", 32), ("vgg11", 4)])
def test_bench_two_ranks_gloo(preset, batch):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--preset", preset,
           "--batch-size", str(batch), "--hip-graph", "off"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["global_batch"] == 2 * batch
    # whole-job images/s from the slowest rank's clock
    assert rec["value"] == pytest.approx(2 * batch * 1e3 / rec["ms_per_step"], rel=1e-3)
    assert rec["higher_is_better"] is True and rec["scaling"] == "weak"
    # every rank sends the same fixed-size payload: the wire total is world x payload
    assert rec["grad_bytes_per_step_on_wire"] == 2 * rec["payload_bytes_per_rank"]
    assert rec["compression_ratio"] > 100
    # headline at the reference's precision with the accuracy-preserving codec; the extra
    # configurations are measured in the same run
    assert rec["dtype"] == "fp32" and rec["config"]["error_feedback"] is True
    for k in ("value_fp32_no_ef", "value_bf16", "ms_per_step_bf16"):
        assert rec[k] > 0, k
    assert rec["overlap_effective"] is (rec["config"]["buckets"] > 1)
    # the self-validation of a multi-rank run: every measured configuration left the replicas
    # bitwise identical (local SGD's replicas legitimately differ between syncs: not checked)
    assert rec["replicas_identical"] is True
    for k in ("fp32_no_ef", "bf16", "dense_fp32"):
        assert rec[f"replicas_identical_{k}"] is True, k
    assert rec["comm"] == "process-group" and rec["rccl_world"] == 0
    assert rec["step_ms_min"] <= rec["step_ms_max"] == pytest.approx(rec["ms_per_step"], rel=1e-3)
    if preset == "vgg11":
        assert rec["config"]["model"] == "vgg11_bn"
        assert rec["metric"].startswith("grad bytes/step on wire + images/sec, VGG-11")
        assert rec["vs_baseline"] is not None
