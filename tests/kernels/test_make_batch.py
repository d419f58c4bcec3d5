"""Fused input-pipeline kernel (ops/csrc/data.hip) against its torch oracle, its device-side
batch position (advanced by the kernel, also under HIP-graph replay), and the loader contract."""
import pytest
import torch

from ewdml.data.loader import DeviceLoader, fused_draws, reference_fused_batch

pytestmark = pytest.mark.gpu


def _data(n=64, c=3, h=32, w=32):
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 256, (n, c, h, w), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 10, (n,), generator=g)
    return x.cuda(), y.cuda()


@pytest.mark.parametrize("augment", [False, True])
@pytest.mark.parametrize("channels_last", [False, True])
def test_make_batch_matches_oracle(augment, channels_last):
    from ewdml import ops

    x, y = _data()
    B = 8
    perm = torch.randperm(64, generator=torch.Generator().manual_seed(1)).cuda()
    state = torch.tensor([2, 5], dtype=torch.int64, device="cuda")  # pos 2, epoch 5
    done = torch.zeros(ops.TICKET_INTS, dtype=torch.int32, device="cuda")
    fmt = torch.channels_last if channels_last else torch.contiguous_format
    out = torch.empty((B, 3, 32, 32), device="cuda", memory_format=fmt)
    oy = torch.empty(B, dtype=torch.int64, device="cuda")
    mean, istd = [0.49, 0.48, 0.45], [1 / 0.25, 1 / 0.24, 1 / 0.26]
    ops.make_batch(x, y, perm, state, done, out, oy, mean, istd, augment=augment, seed=3, rank=1)
    torch.cuda.synchronize()
    ref, ry = reference_fused_batch(x, y, perm, 2, B, mean, istd, augment, 3, 1, 5)
    assert torch.equal(out.float(), ref)
    assert torch.equal(oy, ry)
    assert state.tolist() == [3, 5] and int(done.abs().sum()) == 0
    # bf16 output = round-to-nearest of the fp32 result
    outb = torch.empty((B, 3, 32, 32), device="cuda", dtype=torch.bfloat16, memory_format=fmt)
    state[0] = 2
    ops.make_batch(x, y, perm, state, done, outb, oy, mean, istd, augment=augment, seed=3, rank=1)
    assert torch.equal(outb, ref.to(torch.bfloat16))


def test_draws_cover_offsets_and_flips():
    seen = {fused_draws(0, 0, 0, s) for s in range(4000)}
    assert {d[0] for d in seen} == set(range(9)) and {d[1] for d in seen} == set(range(9))
    assert {d[2] for d in seen} == {0, 1}


def test_make_batch_in_graph_advances_position():
    x, y = _data()
    info = {"mean": (0.5, 0.5, 0.5), "std": (0.25, 0.25, 0.25)}
    ld = DeviceLoader(x, y, info, 8, augment=True, seed=0, device="cuda", fused=True,
                      channels_last=True)
    ref = DeviceLoader(x, y, info, 8, augment=True, seed=0, device="cuda", fused=True,
                       channels_last=True)
    assert ld.fused and len(ld) == 8
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ld.begin_step()
        ld.emit()
        ld.advance()  # eager warmup of the kernel on the capture stream
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            bx, by = ld.emit()
    torch.cuda.current_stream().wait_stream(s)
    ref.next()
    for _ in range(10):  # crosses an epoch boundary (8 batches per epoch)
        ld.begin_step()
        g.replay()
        ld.advance()
        rx, ry = ref.next()
        torch.cuda.synchronize()
        assert torch.equal(bx, rx) and torch.equal(by, ry)
    assert ld.epoch == ref.epoch == 1
