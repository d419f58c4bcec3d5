"""First-contact self-check of the data-plane communicator.

The step's collectives (payload all-gather, dense all-reduce, parameter broadcast) run on the own
RCCL communicator and are captured inside the step's HIP graph.  Before a multi-GPU run trusts
them, every rank issues rank-coded collectives through the same ``Comm`` methods the exchange
uses -- eagerly, and captured in a HIP graph that is replayed twice with fresh inputs -- and
compares the results with their closed forms.  All ranks then agree (control-plane all-reduce over
the process group, like ``Trainer._try_capture``): one failing rank makes every rank fall back to
process-group collectives with split graphs, so a silently wrong transport cannot produce a
number.

The reference has no counterpart (its Gloo/MPI collectives are trusted as-is:
``src/distributed_nn.py:81``, ``horvod_pytorch.py:187-201``); this is the check SURVEY 5.3 asks
of a data plane that cannot be exercised at N > 1 before the scaling run.

Test hook: ``EWDML_PROBE_CORRUPT=<rank>[,<rank>...]`` flips one byte of the listed ranks' probe
results (``<rank>:graph`` only in the captured replays); ``<rank>:capture`` makes that rank's graph
capture raise (every rank must then skip the replays: a replay holds collectives that would wait
forever for the rank that has no graph).
"""
import os

import torch

# sizes are odd on purpose (no accidental alignment); the all-gather moves bytes like the payloads
_AG_N = 4099
_AR_N = 2053
_BC_N = 1031


def _corrupt_phase(rank: int):
    """None, 'all' or 'graph' for this rank (test hook)."""
    spec = os.environ.get("EWDML_PROBE_CORRUPT", "")
    for item in spec.split(","):
        item = item.strip()
        if not item:
            continue
        r, _, phase = item.partition(":")
        if int(r) == rank:
            return phase or "all"
    return None


def _inputs(rank: int, world: int, salt: int, device):
    """Rank-coded inputs and the closed-form results of the three collectives."""
    i = torch.arange(_AG_N, dtype=torch.int64, device=device)
    ag_in = ((i * 7 + rank * 31 + salt * 101) % 251).to(torch.uint8)
    ag_exp = torch.cat([((i * 7 + r * 31 + salt * 101) % 251).to(torch.uint8)
                        for r in range(world)])
    j = torch.arange(_AR_N, dtype=torch.int64, device=device)
    base = ((j + salt) % 13 + 1).to(torch.float32)
    ar_in = base * float(rank + 1)
    ar_exp = base * float(world * (world + 1) // 2)  # exact in fp32 for these magnitudes
    root = world - 1  # a non-zero root where possible
    k = torch.arange(_BC_N, dtype=torch.int64, device=device)
    bc_in = ((k * 3 + rank * 17 + salt) % 1009).to(torch.float32)
    bc_exp = ((k * 3 + root * 17 + salt) % 1009).to(torch.float32)
    return (ag_in, ag_exp), (ar_in, ar_exp), (bc_in, bc_exp, root)


def _check(got, exp) -> bool:
    return bool(torch.equal(got.cpu(), exp.cpu()))


def _eager(comm, device, corrupt: bool) -> bool:
    rank, world = comm.rank, comm.world
    (ag_in, ag_exp), (ar_in, ar_exp), (bc_in, bc_exp, root) = _inputs(rank, world, 0, device)
    out = torch.zeros(world * _AG_N, dtype=torch.uint8, device=device)
    # in place from this rank's slot, like the payload all-gather (GradientExchange)
    slot = out[rank * _AG_N:(rank + 1) * _AG_N]
    slot.copy_(ag_in)
    _wait(comm.all_gather(out, slot, async_op=True))
    _wait(comm.all_reduce(ar_in, async_op=True))
    _wait(comm.broadcast(bc_in, src=root, async_op=True))
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    if corrupt:
        out[0] ^= 0x5A
    return _check(out, ag_exp) and _check(ar_in, ar_exp) and _check(bc_in, bc_exp)


def _wait(work):
    if work is not None:
        work.wait()


def _graph_capture(comm, device, fail: bool = False):
    """The three collectives captured in one HIP graph on a side stream (as the step graph
    captures them).  Returns the replay state; raises if the capture fails (``fail``: test
    hook).  Nothing here waits on a peer: capture only records the collectives."""
    rank, world = comm.rank, comm.world
    if fail:
        raise RuntimeError(f"probe capture failure injected on rank {rank}")
    out = torch.zeros(world * _AG_N, dtype=torch.uint8, device=device)
    slot = out[rank * _AG_N:(rank + 1) * _AG_N]
    ar = torch.zeros(_AR_N, dtype=torch.float32, device=device)
    bc = torch.zeros(_BC_N, dtype=torch.float32, device=device)
    src = (torch.zeros(_AG_N, dtype=torch.uint8, device=device), torch.zeros_like(ar),
           torch.zeros_like(bc))
    (_, _), (_, _), (_, _, root) = _inputs(rank, world, 0, device)
    s = torch.cuda.Stream(device=device)
    s.wait_stream(torch.cuda.current_stream(device))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
        slot.copy_(src[0])
        ar.copy_(src[1])
        bc.copy_(src[2])
        comm.all_gather(out, slot)
        comm.all_reduce(ar)
        comm.broadcast(bc, src=root)
    return g, out, ar, bc, src


def _graph_replay(comm, device, state, corrupt: bool) -> bool:
    """Replay the captured probe twice with new inputs copied into the static buffers between
    replays: each replay must read the current inputs and produce their closed forms.  Every rank
    calls it (the replays hold collectives), only after all ranks captured."""
    rank, world = comm.rank, comm.world
    g, out, ar, bc, (src_ag, src_ar, src_bc) = state
    ok = True
    for salt in (1, 2):
        (ag_in, ag_exp), (ar_in, ar_exp), (bc_in, bc_exp, _) = _inputs(rank, world, salt, device)
        src_ag.copy_(ag_in)
        src_ar.copy_(ar_in)
        src_bc.copy_(bc_in)
        out.zero_()
        torch.cuda.synchronize(device)
        g.replay()
        torch.cuda.synchronize(device)
        if corrupt:
            ar[1] += 1.0
        ok = ok and _check(out, ag_exp) and _check(ar, ar_exp) and _check(bc, bc_exp)
    return ok


def _graph_supported(device) -> bool:
    return device.type == "cuda"


def probe_collectives(comm, device, graph: bool = True) -> dict:
    """Run the probe on every rank and agree on the outcome (collective: every rank calls it with
    the same ``graph``).  Returns ``{"ok", "eager", "graph", "local_ok", "error"}``; ``ok`` is the
    all-rank verdict.  A rank whose probe raised counts as failed.  The ranks agree (process-group
    all-reduce, the control plane) after the eager phase and again after capturing the graph, so
    the captured collectives are replayed only when every rank holds its graph: a rank whose
    capture raised never leaves its peers waiting inside a replay."""
    device = torch.device(device)
    phase = _corrupt_phase(comm.rank)
    res = {"eager": None, "graph": None}
    err = None
    try:
        res["eager"] = _eager(comm, device, corrupt=phase == "all")
    except Exception as e:  # noqa: BLE001 - a raising probe is a failed probe
        err = repr(e)
    if graph and _graph_supported(device):
        eager_bad = comm.all_reduce_scalars([0.0 if err is None else 1.0], op="max")[0]
        state = None
        if eager_bad == 0.0:
            try:
                state = _graph_capture(comm, device, fail=phase == "capture")
            except Exception as e:  # noqa: BLE001
                err = repr(e)
            cap_bad = comm.all_reduce_scalars([0.0 if state is not None else 1.0], op="max")[0]
            if cap_bad == 0.0:
                try:
                    res["graph"] = _graph_replay(comm, device, state,
                                                 corrupt=phase in ("all", "graph"))
                except Exception as e:  # noqa: BLE001
                    err = repr(e)
            else:
                res["graph"] = False  # some rank has no graph: nobody replays
            del state
        else:
            res["graph"] = False
    local_ok = err is None and res["eager"] is not False and res["graph"] is not False
    bad = comm.all_reduce_scalars([0.0 if local_ok else 1.0], op="max")[0]
    res.update(ok=bad == 0.0, local_ok=local_ok, error=err)
    return res
