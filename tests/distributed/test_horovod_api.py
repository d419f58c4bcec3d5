"""Multi-rank tests of the Horovod-style API (``ewdml.parallel.horovod``) on CPU/Gloo worlds of 2, 3
and 4 ranks: the reference's flow ``broadcast_parameters`` -> ``broadcast_optimizer_state`` ->
``DistributedOptimizer(compression, op=Average|Sum|Adasum, gradient_predivide_factor,
backward_passes_per_step)`` (``horvod_pytorch.py:173-201``)."""
import pytest
import torch

from .helpers import run_world

pytestmark = pytest.mark.slow


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))


def _data(rank, n=8):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(n, 16, generator=g), torch.randint(0, 4, (n,), generator=g)


def _step(rank, world, compression, op, predivide=1.0, bpps=1, momentum=0.0):
    from ewdml.parallel import horovod as hvd

    hvd.init(backend="gloo")
    m = _model()
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=momentum)
    hvd.broadcast_parameters(m.state_dict(), root_rank=0)
    hvd.broadcast_optimizer_state(opt, root_rank=0)
    comp = {"none": hvd.Compression.none, "fp16": hvd.Compression.fp16,
            "qsgd": hvd.Compression.qsgd(), "topk_qsgd": hvd.Compression.topk_qsgd(0.25)}[compression]
    dopt = hvd.DistributedOptimizer(opt, m.named_parameters(), compression=comp, op=op,
                                    gradient_predivide_factor=predivide,
                                    backward_passes_per_step=bpps)
    p0 = [p.detach().clone() for p in m.parameters()]
    # the rank's own gradient, from an unwrapped copy (the wrapped model's .grad is exchanged in
    # place, overlapped with backward)
    import copy

    ref = copy.deepcopy(m)
    for q, p in zip(ref.parameters(), p0):
        q.data.copy_(p)
    ref.zero_grad()
    for k in range(bpps):
        x, y = _data(rank * 10 + k)
        torch.nn.functional.cross_entropy(ref(x), y).backward()
    local = [q.grad.detach().clone() for q in ref.parameters()]
    dopt.zero_grad()
    for k in range(bpps):
        x, y = _data(rank * 10 + k)
        torch.nn.functional.cross_entropy(m(x), y).backward()
    dopt.synchronize()
    reduced = [p.grad.detach().clone() for p in m.parameters()]
    dopt.step()
    return {"p0": p0, "p1": [p.detach().clone() for p in m.parameters()], "local": local,
            "reduced": reduced}


def _same(res, key):
    for r in res[1:]:
        for a, b in zip(res[0][key], r[key]):
            assert torch.equal(a, b), key


@pytest.mark.parametrize("compression", ["none", "fp16", "qsgd", "topk_qsgd"])
def test_distributed_optimizer_replicas_identical(tmp_path, compression):
    from ewdml.parallel import horovod as hvd

    res = run_world(_step, 3, tmp_path, args=(compression, hvd.Average))
    _same(res, "p0")
    _same(res, "p1")  # every rank decodes the same payloads in the same order
    _same(res, "reduced")
    if compression == "none":  # dense: exactly the average of the ranks' gradients
        for i, red in enumerate(res[0]["reduced"]):
            avg = sum(r["local"][i] for r in res) / len(res)
            torch.testing.assert_close(red, avg, rtol=1e-6, atol=1e-7)
        for i, p in enumerate(res[0]["p1"]):
            torch.testing.assert_close(p, res[0]["p0"][i] - 0.1 * res[0]["reduced"][i])
    elif compression == "fp16":
        for i, red in enumerate(res[0]["reduced"]):
            avg = sum(r["local"][i] for r in res) / len(res)
            torch.testing.assert_close(red, avg, rtol=2e-3, atol=2e-4)


def test_op_sum_and_predivide(tmp_path):
    from ewdml.parallel import horovod as hvd

    s = run_world(_step, 2, tmp_path / "s", args=("none", hvd.Sum))
    for i, red in enumerate(s[0]["reduced"]):
        torch.testing.assert_close(red, s[0]["local"][i] + s[1]["local"][i], rtol=1e-6, atol=1e-7)
    a = run_world(_step, 2, tmp_path / "a", args=("none", hvd.Average, 2.0))
    for i, red in enumerate(a[0]["reduced"]):  # predivide + post-scale: still the average
        torch.testing.assert_close(red, (a[0]["local"][i] + a[1]["local"][i]) / 2, rtol=1e-6,
                                   atol=1e-7)


def test_backward_passes_per_step(tmp_path):
    """Two backward passes accumulate locally, then one reduction and one optimizer step."""
    from ewdml.parallel import horovod as hvd

    res = run_world(_step, 2, tmp_path, args=("none", hvd.Average, 1.0, 2))
    _same(res, "p1")
    for i, red in enumerate(res[0]["reduced"]):
        torch.testing.assert_close(red, (res[0]["local"][i] + res[1]["local"][i]) / 2,
                                   rtol=1e-6, atol=1e-7)
    # the local gradients are sums of two passes: larger than one pass's
    one = run_world(_step, 2, tmp_path / "one", args=("none", hvd.Average, 1.0, 1))
    assert not torch.allclose(one[0]["local"][0], res[0]["local"][0])


def _adasum_ref(vs):
    vs = [v.double() for v in vs]
    while len(vs) > 1:
        nxt = []
        for i in range(0, len(vs) - 1, 2):
            a, b = vs[i], vs[i + 1]
            d = torch.dot(a, b)
            nxt.append((1 - d / (2 * torch.dot(a, a))) * a + (1 - d / (2 * torch.dot(b, b))) * b)
        if len(vs) % 2:
            nxt.append(vs[-1])
        vs = nxt
    return vs[0]


@pytest.mark.parametrize("world", [2, 3, 4])
def test_adasum_closed_form(tmp_path, world):
    """The pairwise-tree exchange (horovod.adasum_tree: point-to-point swaps between the tree's
    groups, a trailing smaller group serving several ranks at world 3) gives every rank the
    closed-form tree of rank-ordered Adasum pairs."""
    from ewdml.parallel import horovod as hvd

    res = run_world(_step, world, tmp_path, args=("none", hvd.Adasum))
    _same(res, "reduced")
    flat = [torch.cat([g.reshape(-1) for g in r["local"]]) for r in res]
    ref = _adasum_ref(flat)
    got = torch.cat([g.reshape(-1) for g in res[0]["reduced"]])
    torch.testing.assert_close(got.double(), ref, rtol=1e-5, atol=1e-7)
    if world == 2:  # orthogonal-ish gradients add, parallel ones average: check the formula
        a, b = flat
        d = float(torch.dot(a.double(), b.double()))
        assert abs(float(torch.dot(ref, ref)) - float(torch.dot(got.double(), got.double()))) \
            < 1e-4 * (1 + abs(d))


def _bcast(rank, world):
    from ewdml.parallel import horovod as hvd

    hvd.init(backend="gloo")
    m = _model(seed=rank)  # different initialisation per rank
    opt = torch.optim.SGD(m.parameters(), lr=0.05 * (rank + 1), momentum=0.9)
    if rank == 0:  # only the root has momentum buffers
        x, y = _data(0)
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    hvd.broadcast_parameters(m.state_dict(), root_rank=0)
    hvd.broadcast_optimizer_state(opt, root_rank=0)
    mom = [opt.state[p]["momentum_buffer"].clone() for p in m.parameters()]
    return {"params": [p.detach().clone() for p in m.parameters()], "mom": mom,
            "lr": opt.param_groups[0]["lr"]}


def test_broadcast_parameters_and_optimizer_state(tmp_path):
    res = run_world(_bcast, 3, tmp_path)
    _same(res, "params")
    _same(res, "mom")  # created on ranks 1, 2 from the root's description, then filled
    assert all(r["lr"] == res[0]["lr"] for r in res)
    assert float(sum(m.abs().sum() for m in res[0]["mom"])) > 0
