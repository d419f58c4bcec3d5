"""Failure detection on the GPU data plane.

The step's collectives run on the own RCCL communicator (``ops/csrc/rccl_comm.hip``), which no
process-group watchdog observes.  The native step watchdog polls an event recorded after each
step; when one stays pending past ``--comm-timeout`` it aborts the communicator and ends the
process with a non-zero code instead of hanging.  The stall is simulated in a world of one
(EWDML_FORCE_PG=1, a real RCCL communicator) by a test-only kernel that waits on a host-pinned
flag; the watchdog releases the flag on abort and the kernel is bounded by its own clock, so the
grid always drains.
"""
import os
import subprocess
import sys
import textwrap
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = textwrap.dedent("""
    import os, sys, time
    sys.path.insert(0, {root!r})
    import torch
    import ewdml
    from ewdml import ops
    from ewdml.parallel.comm import init_distributed
    torch.cuda.set_device(0)
    comm = init_distributed(device=torch.device("cuda", 0))
    assert comm.kind == "rccl-stream", comm.kind
    C = ops.require()
    x = torch.arange(64, dtype=torch.float32, device="cuda")
    out = torch.zeros(64, device="cuda")
    comm.all_gather(out, x)  # the communicator works
    comm.arm_watchdog({timeout}, exit_code=17)
    comm.watch()
    torch.cuda.synchronize()
    time.sleep(0.3)
    assert C.rccl_watch_pending(comm.watchdog) == 0  # completed steps are retired
    flag = C.test_flag_alloc()
    C.watchdog_release_flag(comm.watchdog, flag)
    if {stall}:
        C.test_spin(flag, 60.0, torch.cuda.current_stream().cuda_stream)
    comm.all_gather(out, x)
    comm.watch()
    print("ARMED", time.time(), flush=True)
    torch.cuda.synchronize()
    print("COMPLETED", flush=True)
    comm.close()
    C.test_flag_free(flag)
""")


def _run_child(stall: bool, timeout: float):
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, EWDML_FORCE_PG="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    code = CHILD.format(root=ROOT, timeout=timeout, stall=stall)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=180)
    t_end = time.time()
    armed = [float(ln.split()[1]) for ln in r.stdout.splitlines() if ln.startswith("ARMED")]
    return r, (t_end - armed[0]) if armed else None


def test_watchdog_aborts_a_stalled_step_and_exits_nonzero():
    timeout = 2.0
    r, waited = _run_child(True, timeout)
    assert r.returncode == 17, (r.returncode, r.stdout[-500:], r.stderr[-1500:])
    assert "ewdml watchdog" in r.stderr and "aborting the RCCL communicator" in r.stderr
    # (the released stream may let the main thread run on for the bounded drain wait before
    # the exit: what matters is that the process ends, non-zero, within the bound)
    assert waited is not None and waited < timeout + 5.0, waited


def test_watchdog_quiet_on_healthy_steps():
    r, _ = _run_child(False, 5.0)
    assert r.returncode == 0, (r.returncode, r.stderr[-1500:])
    assert "COMPLETED" in r.stdout and "ewdml watchdog" not in r.stderr
