"""HIP kernels vs the torch oracle (compress/oracle.py), on one MI355X.

Exactness contract: top-k selection, int8/int4/fp32 payload bytes and decoded sums are bitwise
equal to the oracle (max-norm scales are exact; the kernels are built with -ffp-contract=off).
L2-norm scales and the optimizer updates are compared with tight tolerances.
"""
import pytest
import torch

from ewdml import ops
from ewdml.compress import oracle
from ewdml.compress.plan import BucketPlan, Layout
from ewdml.compress.rng import stream_key

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _plan(numels, ratio, bucket_offset=0):
    offs, o = [], 0
    for n in numels:
        offs.append(o)
        o += (n + 63) // 64 * 64
    return BucketPlan(numels, offs, ratio, bucket_offset, o)


def _grad(plan, seed=0, ties=False):
    g = torch.zeros(plan.length)
    gen = torch.Generator().manual_seed(seed)
    for off, n in zip(plan.offsets, plan.numels):
        x = torch.randn(n, generator=gen) * (0.1 + torch.rand(1, generator=gen))
        if ties:  # quantised values -> many exact ties at the threshold
            x = torch.round(x * 4) / 4
        g[off:off + n] = x
    return g


SHAPES = [
    [10], [500, 10], [20 * 25, 20, 50 * 500, 50], [8192 * 3 + 5, 7, 64, 100003],
    [2359296], [1, 2, 3, 4, 5],
]


@pytest.mark.parametrize("numels", SHAPES)
@pytest.mark.parametrize("ratio", [0.01, 0.4, 1.0])
@pytest.mark.parametrize("kind,bits", [("topk_qsgd", 8), ("topk_qsgd", 4), ("topk", 8)])
def test_topk_encode_matches_oracle(numels, ratio, kind, bits):
    ops.require()
    plan = _plan(numels, ratio, bucket_offset=4096)
    lay = Layout.build(kind, plan, bits)
    levels = 127 if bits == 8 else 7
    g = _grad(plan, seed=len(numels))
    key = stream_key(3, 11, 1)
    ref = oracle.encode_topk(g.clone(), plan, lay, levels, "max", key)
    dp = ops.DevicePlan(plan, DEV)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
    ops.topk_encode(dp, g.to(DEV), pay, lay, levels, "max", key)
    got = pay.cpu()
    assert torch.equal(got, ref), f"payload mismatch at {(got != ref).nonzero()[:10].flatten()}"


def test_topk_repeated_encodes_reuse_scratch():
    """Consecutive encodes on one DevicePlan (no per-encode memset: the write kernel clears the
    histograms for the next encode) stay bit-exact, including after a different gradient."""
    ops.require()
    plan = _plan([20 * 25, 20, 50 * 500, 50, 2359296], 0.01)
    lay = Layout.build("topk_qsgd", plan, 8)
    dp = ops.DevicePlan(plan, DEV)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
    for it in range(4):
        g = _grad(plan, seed=10 + it, ties=(it == 2))
        key = stream_key(5, it, 0)
        ref = oracle.encode_topk(g.clone(), plan, lay, 127, "max", key)
        ops.topk_encode(dp, g.to(DEV), pay, lay, 127, "max", key)
        assert torch.equal(pay.cpu(), ref), f"encode {it} differs"
    # the write pass's look-back (max-norm scale) never had to give up on a predecessor
    assert ops.topk_lookback_errors(dp) == 0


def test_topk_ties_exact_count():
    ops.require()
    plan = _plan([8192 * 4 + 17, 333], 0.05)
    lay = Layout.build("topk_qsgd", plan, 8)
    g = _grad(plan, seed=5, ties=True)
    key = stream_key(0, 0, 0)
    ref = oracle.encode_topk(g.clone(), plan, lay, 127, "max", key)
    dp = ops.DevicePlan(plan, DEV)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
    ops.topk_encode(dp, g.to(DEV), pay, lay, 127, "max", key)
    assert torch.equal(pay.cpu(), ref)


def test_topk_l2_norm_close():
    ops.require()
    plan = _plan([100003, 4097], 0.02)
    lay = Layout.build("topk_qsgd", plan, 8)
    g = _grad(plan, seed=9)
    key = stream_key(1, 2, 0)
    ref = oracle.encode_topk(g.clone(), plan, lay, 127, "l2", key)
    dp = ops.DevicePlan(plan, DEV)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
    ops.topk_encode(dp, g.to(DEV), pay, lay, 127, "l2", key)
    got = pay.cpu()
    T = plan.num_tensors
    s_ref = ref[:4 * T].view(torch.float32)
    s_got = got[:4 * T].view(torch.float32)
    torch.testing.assert_close(s_got, s_ref, rtol=1e-5, atol=0)
    # indices and counts identical; codes may differ by at most 1 where the scale's last bit moved
    assert torch.equal(got[lay.counts:lay.codes], ref[lay.counts:lay.codes])
    c_ref = ref[lay.codes:lay.codes + plan.total_k].view(torch.int8).int()
    c_got = got[lay.codes:lay.codes + plan.total_k].view(torch.int8).int()
    assert (c_ref - c_got).abs().max() <= 1


@pytest.mark.parametrize("kind,bits", [("topk_qsgd", 8), ("topk_qsgd", 4), ("topk", 8)])
@pytest.mark.parametrize("ratio,N", [(0.03, 5), (0.06, 5), (0.03, 11), (0.4, 5)])
def test_topk_decode_matches_oracle(kind, bits, ratio, N):
    """ratio 0.4: most tensors are bitmap-indexed (plan.py), the 20-element one keeps the list;
    0.06: u16 lists with more entries per chunk than threads; N = 11: past the ranks whose first
    entries the decode prefetches."""
    ops.require()
    plan = _plan([20 * 25, 20, 8192 * 5 + 3, 50, 70001], ratio, bucket_offset=128)
    if ratio > 0.1:
        assert plan.tensor_bm0[2] >= 0 and plan.total_bm_words > 0
    lay = Layout.build(kind, plan, bits)
    levels = 127 if bits == 8 else 7
    pays = []
    for r in range(N):
        g = _grad(plan, seed=100 + r)
        pays.append(oracle.encode_topk(g, plan, lay, levels, "max", stream_key(0, 4, r)))
    recv = torch.stack(pays)
    ref = oracle.decode_sum(recv, plan, lay, levels, 1.0 / N)
    dp = ops.DevicePlan(plan, DEV)
    out = torch.full((plan.length,), float("nan"), device=DEV)
    ops.topk_decode_apply(dp, recv.to(DEV), lay, levels, grad_out=out, grad_scale=1.0 / N)
    got = out.cpu()
    for off, n in zip(plan.offsets, plan.numels):
        assert torch.equal(got[off:off + n], ref[off:off + n])


def test_topk_decode_fused_sgd():
    ops.require()
    plan = _plan([9000, 64, 33333], 0.05)
    lay = Layout.build("topk_qsgd", plan, 8)
    N = 3
    recv = torch.stack([oracle.encode_topk(_grad(plan, seed=r), plan, lay, 127, "max",
                                           stream_key(0, 0, r)) for r in range(N)])
    p0 = torch.randn(plan.length)
    m0 = torch.randn(plan.length)
    hp = dict(lr=0.05, momentum=0.9, dampening=0.1, weight_decay=1e-4, nesterov=False)
    for first in (True, False):
        p, m = p0.clone(), m0.clone()
        g = oracle.decode_sum(recv, plan, lay, 127, 1.0 / N)
        for off, n in zip(plan.offsets, plan.numels):
            oracle.sgd_apply(p[off:off + n], m[off:off + n], g[off:off + n], first=first, **hp)
        dp = ops.DevicePlan(plan, DEV)
        pd, md = p0.to(DEV), m0.to(DEV)
        ops.topk_decode_apply(dp, recv.to(DEV), lay, 127, param=pd, mom=md,
                              grad_scale=1.0 / N, first=first, **hp)
        torch.testing.assert_close(pd.cpu(), p, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(md.cpu(), m, rtol=1e-6, atol=1e-7)


def test_topk_error_feedback_matches_oracle():
    ops.require()
    plan = _plan([40000, 1000], 0.01)
    lay = Layout.build("topk_qsgd", plan, 8)
    g = _grad(plan, seed=1)
    r0 = _grad(plan, seed=2) * 0.1
    key = stream_key(0, 1, 0)
    r_ref = r0.clone()
    ref = oracle.encode_topk(g.clone(), plan, lay, 127, "max", key, residual=r_ref)
    dp = ops.DevicePlan(plan, DEV)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
    r_dev = r0.to(DEV)
    ops.topk_encode(dp, g.to(DEV), pay, lay, 127, "max", key, resid=r_dev)
    assert torch.equal(pay.cpu(), ref)
    for off, n in zip(plan.offsets, plan.numels):
        assert torch.equal(r_dev.cpu()[off:off + n], r_ref[off:off + n])


@pytest.mark.parametrize("kind,bits", [("topk_qsgd", 8), ("topk_qsgd", 4), ("topk", 8)])
@pytest.mark.parametrize("wd,nesterov,damp", [(0.0, False, 0.0), (5e-4, False, 0.1),
                                              (1e-4, True, 0.0)])
@pytest.mark.parametrize("mode", ["dgc", "local"])
def test_topk_dgc_matches_oracle(kind, bits, wd, nesterov, damp, mode):
    """Momentum-corrected error feedback (DGC): velocity, residual and payload bitwise equal to
    oracle.dgc_accumulate + encode_topk over consecutive steps (the velocity is cleared at the
    sent coordinates, so the selection moves from step to step)."""
    ops.require()
    plan = _plan([40000, 1000, 8192 * 3 + 5], 0.01, bucket_offset=256)
    lay = Layout.build(kind, plan, bits)
    levels = 127 if bits == 8 else 7
    dp = ops.DevicePlan(plan, DEV)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
    p0 = _grad(plan, seed=40)
    r_ref, v_ref = torch.zeros(plan.length), torch.zeros(plan.length)
    r_dev, v_dev, p_dev = r_ref.to(DEV), v_ref.to(DEV), p0.to(DEV)
    for it in range(3):
        g = _grad(plan, seed=30 + it)
        key = stream_key(2, it, 1)
        hp = dict(momentum=0.9, dampening=damp, nesterov=nesterov, weight_decay=wd)
        if mode == "local":  # no masking, lr-scaled residual (the device lr)
            lr = 0.05 * (it + 1)
            hp.update(mask=False, lr=lr)
        ref = oracle.encode_topk(g.clone(), plan, lay, levels, "max", key, residual=r_ref,
                                 dgc=dict(velocity=v_ref, param=p0, **hp))
        lr_t = torch.tensor([hp.get("lr", 0.0)], dtype=torch.float32, device=DEV)
        ops.topk_encode(dp, g.to(DEV), pay, lay, levels, "max", key, resid=r_dev,
                        dgc=dict(velocity=v_dev, param=p_dev, lr_t=lr_t, **hp))
        assert torch.equal(pay.cpu(), ref), f"step {it}: payload"
        for off, n in zip(plan.offsets, plan.numels):
            assert torch.equal(r_dev.cpu()[off:off + n], r_ref[off:off + n]), f"step {it}: resid"
            assert torch.equal(v_dev.cpu()[off:off + n], v_ref[off:off + n]), f"step {it}: vel"
        if mode == "dgc":
            assert (v_ref == 0).sum() >= plan.total_k  # masked where sent


def test_topk_decode_without_momentum_buffer():
    """mom=None (momentum ran on the sender): p -= lr * mean, the momentum buffer untouched."""
    ops.require()
    plan = _plan([9000, 64, 33333], 0.05)
    lay = Layout.build("topk_qsgd", plan, 8)
    N = 3
    recv = torch.stack([oracle.encode_topk(_grad(plan, seed=r), plan, lay, 127, "max",
                                           stream_key(0, 0, r)) for r in range(N)])
    p0 = torch.randn(plan.length)
    g = oracle.decode_sum(recv, plan, lay, 127, 1.0 / N)
    p = p0.clone()
    for off, n in zip(plan.offsets, plan.numels):
        oracle.sgd_apply(p[off:off + n], None, g[off:off + n], 0.05, 0.0, 0.0, 0.0, False, False)
    dp = ops.DevicePlan(plan, DEV)
    pd = p0.to(DEV)
    ops.topk_decode_apply(dp, recv.to(DEV), lay, 127, param=pd, mom=None, lr=0.05,
                          grad_scale=1.0 / N)
    for off, n in zip(plan.offsets, plan.numels):  # torch's CPU add(alpha=) may fuse: ~1 ulp
        torch.testing.assert_close(pd.cpu()[off:off + n], p[off:off + n], rtol=1e-6, atol=1e-7)
    with pytest.raises(ValueError):
        ops.topk_decode_apply(dp, recv.to(DEV), lay, 127, param=pd, mom=None, lr=0.05,
                              momentum=0.9)


@pytest.mark.parametrize("bits,norm", [(8, "max"), (4, "max"), (8, "l2")])
def test_qsgd_dense_roundtrip(bits, norm):
    ops.require()
    plan = _plan([8192 * 2 + 13, 10, 5000], 1.0, bucket_offset=64)
    lay = Layout.build("qsgd", plan, bits)
    levels = 127 if bits == 8 else 7
    N = 4
    dp = ops.DevicePlan(plan, DEV)
    pays_ref, pays_dev = [], []
    for r in range(N):
        g = _grad(plan, seed=20 + r)
        key = stream_key(7, 3, r)
        ref = oracle.encode_qsgd(g.clone(), plan, lay, levels, norm, key)
        pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
        ops.qsgd_encode(dp, g.to(DEV), pay, lay, levels, norm, key)
        pays_ref.append(ref)
        pays_dev.append(pay)
        if norm == "max":
            assert torch.equal(pay.cpu(), ref)
    recv = torch.stack(pays_ref)
    out = torch.zeros(plan.length, device=DEV)
    ops.qsgd_decode_apply(dp, recv.to(DEV), lay, levels, grad_out=out, grad_scale=1.0 / N)
    ref_dec = oracle.decode_sum(recv, plan, lay, levels, 1.0 / N)
    for off, n in zip(plan.offsets, plan.numels):
        assert torch.equal(out.cpu()[off:off + n], ref_dec[off:off + n])


def test_sgd_and_adam_flat():
    ops.require()
    n = 100000
    p0, m0, g = torch.randn(n), torch.randn(n), torch.randn(n)
    hp = dict(lr=0.1, momentum=0.9, dampening=0.0, weight_decay=1e-3, nesterov=True)
    p, m = p0.clone(), m0.clone()
    oracle.sgd_apply(p, m, g * 0.5, first=False, **hp)
    pd, md = p0.cuda(), m0.cuda()
    ops.sgd_flat(pd, md, g.cuda(), grad_scale=0.5, first=False, **hp)
    torch.testing.assert_close(pd.cpu(), p, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(md.cpu(), m, rtol=1e-6, atol=1e-7)
    # bf16 gradient input
    gb = g.to(torch.bfloat16)
    p, m = p0.clone(), m0.clone()
    oracle.sgd_apply(p, m, gb.float(), first=True, **hp)
    pd, md = p0.cuda(), m0.cuda()
    ops.sgd_flat(pd, md, gb.cuda(), first=True, **hp)
    torch.testing.assert_close(pd.cpu(), p, rtol=1e-6, atol=1e-7)
    # adam / amsgrad
    for ams in (False, True):
        p = p0.clone()
        mm, vv, vx = torch.zeros(n), torch.zeros(n), torch.zeros(n)
        for t in (1, 2, 3):
            oracle.adam_apply(p, mm, vv, vx, g * t, 1e-3, 0.9, 0.999, 1e-8, 1e-2, t, ams)
        pd = p0.cuda()
        mmd, vvd, vxd = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV), \
            torch.zeros(n, device=DEV)
        import math
        for t in (1, 2, 3):
            ls = 1e-3 * math.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
            ops.adam_flat(pd, mmd, vvd, vxd, (g * t).cuda(), ls, 0.9, 0.999, 1e-8, 1e-2, 1.0, ams)
        torch.testing.assert_close(pd.cpu(), p, rtol=1e-5, atol=1e-6)


def test_cast_scale_bf16_fp16():
    ops.require()
    x = torch.randn(4096 * 3, device=DEV) * 100
    for dt in (torch.bfloat16, torch.float16):
        out = torch.empty(x.numel(), dtype=dt, device=DEV)
        ops.cast_scale(x, out, 0.25)
        assert torch.equal(out, (x * 0.25).to(dt))


def test_bad_operands_rejected():
    ops.require()
    plan = _plan([1000], 0.1)
    lay = Layout.build("topk_qsgd", plan, 8)
    dp = ops.DevicePlan(plan, DEV)
    with pytest.raises(ValueError):
        ops.topk_encode(dp, torch.zeros(10, device=DEV), torch.zeros(lay.nbytes,
                        dtype=torch.uint8, device=DEV), lay, 127, "max", 0)
    with pytest.raises(ValueError):
        ops.topk_encode(dp, torch.zeros(plan.length, device=DEV), torch.zeros(
            lay.nbytes, dtype=torch.uint8, device=DEV), lay, 200, "max", 0)


def _split(plan, g, dtype=torch.float32):
    return [g[o:o + n].clone().to(dtype).to(DEV) for o, n in zip(plan.offsets, plan.numels)]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("kind", ["topk_qsgd", "qsgd"])
def test_encode_from_per_tensor_pointers(dtype, kind):
    """Encoding autograd's own per-tensor gradients (fp32 or bf16, read through the pointer
    table) equals encoding the same values from a flat fp32 buffer."""
    ops.require()
    plan = _plan([8192 + 7, 64, 30000, 5], 0.02, bucket_offset=256)
    lay = Layout.build(kind, plan, 8)
    g = _grad(plan, seed=3)
    if dtype == torch.bfloat16:  # the flat reference holds the same (bf16-representable) values
        for o, n in zip(plan.offsets, plan.numels):
            g[o:o + n] = g[o:o + n].to(torch.bfloat16).float()
    key = stream_key(2, 5, 1)
    enc = oracle.encode_qsgd if kind == "qsgd" else oracle.encode_topk
    ref = enc(g.clone(), plan, lay, 127, "max", key)
    dp = ops.DevicePlan(plan, DEV)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
    fn = ops.qsgd_encode if kind == "qsgd" else ops.topk_encode
    fn(dp, _split(plan, g, dtype), pay, lay, 127, "max", key)
    assert torch.equal(pay.cpu(), ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_error_feedback_bf16_grads_stage_in_residual(dtype):
    ops.require()
    plan = _plan([20000, 300], 0.01)
    lay = Layout.build("topk_qsgd", plan, 8)
    g = _grad(plan, seed=7)
    for o, n in zip(plan.offsets, plan.numels):
        g[o:o + n] = g[o:o + n].to(dtype).float()
    r0 = _grad(plan, seed=8) * 0.05
    key = stream_key(0, 3, 0)
    r_ref = r0.clone()
    ref = oracle.encode_topk(g.clone(), plan, lay, 127, "max", key, residual=r_ref)
    dp = ops.DevicePlan(plan, DEV)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
    grads = _split(plan, g, dtype)
    before = [t.clone() for t in grads]
    r_dev = r0.to(DEV)
    ops.topk_encode(dp, grads, pay, lay, 127, "max", key, resid=r_dev)
    assert torch.equal(pay.cpu(), ref)
    for o, n in zip(plan.offsets, plan.numels):
        assert torch.equal(r_dev.cpu()[o:o + n], r_ref[o:o + n])
    for a, b in zip(grads, before):  # the gradients themselves are not modified
        assert torch.equal(a, b)


def test_decode_writes_bf16_shadow():
    ops.require()
    plan = _plan([9000, 64, 33333], 0.05)
    lay = Layout.build("topk_qsgd", plan, 8)
    recv = torch.stack([oracle.encode_topk(_grad(plan, seed=r), plan, lay, 127, "max",
                                           stream_key(0, 0, r)) for r in range(2)]).to(DEV)
    dp = ops.DevicePlan(plan, DEV)
    p = torch.randn(plan.length, device=DEV)
    m = torch.zeros(plan.length, device=DEV)
    sh = torch.zeros(plan.length, dtype=torch.bfloat16, device=DEV)
    ops.topk_decode_apply(dp, recv, lay, 127, param=p, mom=m, lr=0.1, momentum=0.9,
                          grad_scale=0.5, first=True, shadow=sh)
    for o, n in zip(plan.offsets, plan.numels):
        assert torch.equal(sh[o:o + n], p[o:o + n].to(torch.bfloat16))
    # flat SGD shadow too
    g = torch.randn(plan.length, device=DEV)
    sh2 = torch.zeros_like(sh)
    ops.sgd_flat(p, m, g, 0.1, 0.9, shadow=sh2)
    assert torch.equal(sh2, p.to(torch.bfloat16))


def test_pack_grads_mixed_dtypes():
    ops.require()
    plan = _plan([1000, 8192 * 2 + 3, 17], 1.0)
    dp = ops.DevicePlan(plan, DEV)
    g = _grad(plan, seed=11)
    grads = _split(plan, g, torch.float32)
    grads[1] = grads[1].to(torch.bfloat16)
    for dt in (torch.float32, torch.bfloat16):
        dst = torch.zeros(plan.length, dtype=dt, device=DEV)
        ops.pack_grads(dp, grads, dst, 0.5)
        for t, o, n in zip(grads, plan.offsets, plan.numels):
            assert torch.equal(dst[o:o + n], (t.float() * 0.5).to(dt))


@pytest.mark.parametrize("kind,bits", [("topk_qsgd", 8), ("topk_qsgd", 4), ("topk", 8)])
@pytest.mark.parametrize("ratio,N", [(0.01, 2), (0.06, 5), (0.03, 11), (0.4, 3)])
def test_topk_decode_sparse_update_bitwise(kind, bits, ratio, N):
    """Without momentum buffer and weight decay the decode (its own kernel: half a chunk of LDS
    at a time) reads and writes only the float4s whose averaged gradient is non-zero: bitwise the
    dense update (p - lr * (+0) is p, -0.0 parameters included), shadow copy too.  Index lists
    (0.06: more entries per chunk than threads), bitmaps (0.4), ranks past the prefetched ones
    (N = 11), entries in both halves of a chunk and a partial last chunk (33333)."""
    ops.require()
    plan = _plan([9000, 64, 33333], ratio)
    lay = Layout.build(kind, plan, bits)
    lv = 127 if bits == 8 else 7
    recv = torch.stack([oracle.encode_topk(_grad(plan, seed=r), plan, lay, lv, "max",
                                           stream_key(0, 0, r)) for r in range(N)]).to(DEV)
    p0 = torch.randn(plan.length, device=DEV)
    p0[::7] = -0.0
    dp = ops.DevicePlan(plan, DEV)
    sparse, sh_s = p0.clone(), torch.zeros(plan.length, dtype=torch.bfloat16, device=DEV)
    ops.topk_decode_apply(dp, recv, lay, lv, param=sparse, mom=None, lr=0.05,
                          grad_scale=1.0 / N, shadow=sh_s)
    dense, sh_d = p0.clone(), torch.zeros(plan.length, dtype=torch.bfloat16, device=DEV)
    mom = torch.zeros(plan.length, device=DEV)  # a momentum buffer forces the dense pass
    ops.topk_decode_apply(dp, recv, lay, lv, param=dense, mom=mom, lr=0.05, momentum=0.0,
                          grad_scale=1.0 / N, shadow=sh_d)
    torch.cuda.synchronize()
    assert torch.equal(sparse.view(torch.int32), dense.view(torch.int32))
    changed = sparse.view(torch.int32) != p0.view(torch.int32)
    assert 0 < int(changed.sum()) <= N * plan.total_k
    # the shadow is written where the parameters were (the rest stays as it was: zeros here)
    assert torch.equal(sh_s[changed], sh_d[changed])


def test_sgd_from_pointer_table_matches_flat():
    """Local SGD's fused step reads each tensor's gradient in place (pointer table, fp32 and
    bf16): bitwise the flat-buffer SGD over the gathered gradient."""
    ops.require()
    plan = _plan([9000, 64, 33333, 5], 1.0)
    dp = ops.DevicePlan(plan, DEV)
    grads = [torch.randn(n, device=DEV) for n in plan.numels]
    grads[1] = grads[1].to(torch.bfloat16)
    flat_g = torch.zeros(plan.length, device=DEV)
    for g, off, n in zip(grads, plan.offsets, plan.numels):
        flat_g[off:off + n] = g.float()
    p0, m0 = torch.randn(plan.length, device=DEV), torch.randn(plan.length, device=DEV)
    hp = dict(lr=0.1, momentum=0.9, dampening=0.0, weight_decay=1e-3, nesterov=True)
    p1, m1 = p0.clone(), m0.clone()
    ops.sgd_ptrs(dp, grads, p1, m1, first=False, **hp)
    p2, m2 = p0.clone(), m0.clone()
    ops.sgd_flat(p2, m2, flat_g, first=False, **hp)
    torch.cuda.synchronize()
    for off, n in zip(plan.offsets, plan.numels):
        assert torch.equal(p1[off:off + n], p2[off:off + n])
        assert torch.equal(m1[off:off + n], m2[off:off + n])


@pytest.mark.parametrize("kind,bits", [("topk_qsgd", 8), ("topk_qsgd", 4), ("topk", 8)])
@pytest.mark.parametrize("ratio", [0.01, 0.4])
def test_topk_predictive_encode_fast_and_full_paths(kind, bits, ratio):
    """The predictive encode (candidates at or above beta x the previous threshold; ops/csrc/
    topk_codec.hip k_pk_*) is bitwise the oracle on both paths: the fast path (a tensor's
    candidates number >= k and fit its list) and the full passes it falls back to when the
    threshold moved too far -- down (too few candidates: the gradient shrank 1000x) or up (too
    many: it grew back).  The counters record which path each tensor took."""
    ops.require()
    plan = _plan([20 * 25, 20, 50 * 500, 50, 8192 * 3 + 5, 2359296, 100003], ratio,
                 bucket_offset=512)
    lay = Layout.build(kind, plan, bits)
    levels = 127 if bits == 8 else 7
    dp = ops.DevicePlan(plan, DEV)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
    g0 = _grad(plan, seed=21)
    noise = _grad(plan, seed=22) * 0.01
    seq = [g0, g0 * 1.02 + noise, g0 * 1e-3, g0, g0 * 1.01 - noise]
    big = [n > c for n, c in zip(plan.numels, plan.tensor_cap)]
    T, nbig = plan.num_tensors, sum(big)
    # full passes, only for the tensors larger than their candidate list (the others take every
    # element as a candidate: bound 0, always the fast path): the first encode (no prediction
    # yet), the 1000x shrink (too few candidates) and the growth (too many)
    expect_full = 3 * nbig
    for it, g in enumerate(seq):
        key = stream_key(4, it, 2)
        ref = oracle.encode_topk(g.clone(), plan, lay, levels, "max", key)
        ops.topk_encode(dp, g.to(DEV), pay, lay, levels, "max", key)
        assert torch.equal(pay.cpu(), ref), f"encode {it}: payload differs"
    st = ops.topk_stats(dp)
    assert st["lookback_errors"] == 0
    assert st["full"] == expect_full, st
    assert st["fast"] == T * len(seq) - st["full"]
    if ratio == 0.01:
        assert nbig >= 3  # the fallback really ran


def test_topk_predictive_encode_dgc_steady_state():
    """Momentum-corrected error feedback over 14 steps from zero state (VGG's largest tensor among
    others): payload, residual and velocity stay bitwise the oracle's on every step.  While the
    velocity builds up (e grows ~2x per step at first) the candidate bound lags and tensors take
    the full passes; once it settles every tensor takes the candidate path."""
    ops.require()
    plan = _plan([1728, 64, 2359296, 512, 262144, 5120], 0.01, bucket_offset=64)
    lay = Layout.build("topk_qsgd", plan, 8)
    dp = ops.DevicePlan(plan, DEV)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
    r_ref, v_ref = torch.zeros(plan.length), torch.zeros(plan.length)
    r_dev, v_dev = r_ref.to(DEV), v_ref.to(DEV)
    hp = dict(momentum=0.9, dampening=0.0, nesterov=False, weight_decay=0.0)
    per_step = []
    for it in range(14):
        g = _grad(plan, seed=60 + it)
        key = stream_key(1, it, 0)
        ref = oracle.encode_topk(g.clone(), plan, lay, 127, "max", key, residual=r_ref,
                                 dgc=dict(velocity=v_ref, param=None, **hp))
        ops.topk_encode(dp, g.to(DEV), pay, lay, 127, "max", key, resid=r_dev,
                        dgc=dict(velocity=v_dev, param=None, **hp))
        assert torch.equal(pay.cpu(), ref), f"step {it}: payload"
        assert torch.equal(r_dev.cpu(), r_ref), f"step {it}: resid"
        assert torch.equal(v_dev.cpu(), v_ref), f"step {it}: vel"
        per_step.append(ops.topk_stats(dp)["full"])
    full = [b - a for a, b in zip([0] + per_step[:-1], per_step)]
    assert ops.topk_stats(dp)["lookback_errors"] == 0
    assert sum(full[-6:]) == 0, f"full-pass tensors per step: {full}"


@pytest.mark.parametrize("predict", ["1", "0"])
def test_lookback_failure_is_reported(monkeypatch, predict):
    """a write block that gives up on its decoupled look-back (bounded by polls, not
    wall time) must not pass silently -- the counter reports it, and the exchange's health check
    (read at every log record and by bench.py) raises."""
    ops.require()
    monkeypatch.setattr(ops, "_TOPK_PREDICT", predict == "1")
    plan = _plan([8192 * 6, 100], 0.01)
    lay = Layout.build("topk_qsgd", plan, 8)
    dp = ops.DevicePlan(plan, DEV)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
    g = _grad(plan, seed=3).to(DEV)
    ops.topk_encode(dp, g, pay, lay, 127, "max", 1)
    assert ops.topk_stats(dp)["lookback_errors"] == 0
    ops.set_lookback_fault(True)
    try:
        ops.topk_encode(dp, g, pay, lay, 127, "max", 2)
        torch.cuda.synchronize()
    finally:
        ops.set_lookback_fault(False)
    # chunk 1 polls to the bound; a later chunk may see the word chunk 1 publishes after giving
    # up, so 1..5 of the 6-chunk tensor's chunks report
    assert 1 <= ops.topk_stats(dp)["lookback_errors"] <= 5

    class _Ex:  # the exchange's check on a codec holding this plan
        cuda = True

        class codec:
            kind, allreduce = "topk_qsgd", False
            _bound = {0.01: (None, None, [dp])}

    from ewdml.parallel.engine import GradientExchange

    with pytest.raises(RuntimeError, match="look-back"):
        GradientExchange.codec_health(_Ex)
    # and the next payload publishes NaN scales: every rank's decoded update goes non-finite at
    # once, so a corrupted exchange cannot train on silently until the next health check
    ops.topk_encode(dp, g, pay, lay, 127, "max", 3)
    torch.cuda.synchronize()
    T = plan.num_tensors
    assert torch.isnan(pay[:4 * T].view(torch.float32)).all()


def test_fused_select_beside_a_long_gemm():
    """the fused select's per-tensor barriers with a concurrent kernel on
    another stream holding CUs (a segmented graph runs encodes beside backward GEMMs).  The GEMM
    does not wait on the encode, so it drains and the select's blocks all become resident: no
    barrier gives up, and every payload is bitwise the oracle's."""
    ops.require()
    C_ = ops.require()
    assert C_.topk_fused_select_max_blocks() > 0  # the fused kernel is in use on this GPU
    plan = _plan([1728, 64, 2359296, 512, 262144, 5120], 0.01, bucket_offset=64)
    lay = Layout.build("topk_qsgd", plan, 8)
    dp = ops.DevicePlan(plan, DEV)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
    r_ref, v_ref = torch.zeros(plan.length), torch.zeros(plan.length)
    r_dev, v_dev = r_ref.to(DEV), v_ref.to(DEV)
    hp = dict(momentum=0.9, dampening=0.0, nesterov=False, weight_decay=0.0)
    a = torch.randn(6144, 6144, device=DEV)
    side = torch.cuda.Stream()
    for it in range(10):
        g = _grad(plan, seed=80 + it)
        key = stream_key(1, it, 0)
        ref = oracle.encode_topk(g.clone(), plan, lay, 127, "max", key, residual=r_ref,
                                 dgc=dict(velocity=v_ref, param=None, **hp))
        gd = g.to(DEV)
        torch.cuda.synchronize()
        busy = [a @ a for _ in range(3)]  # ~10 ms of GEMMs on the default stream
        with torch.cuda.stream(side):
            ops.topk_encode(dp, gd, pay, lay, 127, "max", key, resid=r_dev,
                            dgc=dict(velocity=v_dev, param=None, **hp))
        torch.cuda.synchronize()
        del busy
        assert torch.equal(pay.cpu(), ref), f"step {it}: payload"
    st = ops.topk_stats(dp)
    assert st["lookback_errors"] == 0, st
    assert st["fast"] > 0  # the candidate (fused select) path ran


SMALL = [20 * 25, 20, 50 * 500, 50, 800 * 500, 500, 5000, 10]  # LeNet's 8 tensors


@pytest.mark.parametrize("ef", ["none", "plain", "dgc"])
@pytest.mark.parametrize("kind,bits", [("topk_qsgd", 8), ("topk_qsgd", 4), ("topk", 8)])
def test_topk_one_launch_encode_matches_oracle(ef, kind, bits):
    """Small buckets (every chunk block resident: LeNet's 431,080 elements in 53 chunks) encode in
    ONE launch (ops/csrc/topk_codec.hip k_pk_one: stage + candidates, the tensor's select in its
    last block, the ordered write), on the candidate path and on the full passes it falls back
    to (the first encode, a 1000x shrink, the growth back; ties at the threshold): payload,
    residual and velocity bitwise the oracle's at every step."""
    C_ = ops.require()
    plan = _plan(SMALL, 0.01, bucket_offset=128)
    assert plan.num_chunks <= C_.topk_one_max_blocks(), "the one-launch encode is not in use"
    lay = Layout.build(kind, plan, bits)
    levels = 127 if bits == 8 else 7
    dp = ops.DevicePlan(plan, DEV)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
    g0 = _grad(plan, seed=31)
    seq = [g0, g0 * 1.01, g0 * 1e-3, g0, _grad(plan, seed=32, ties=True)] + [
        _grad(plan, seed=40 + i) * (1.0 + 0.01 * i) for i in range(6)]
    r_ref = torch.zeros(plan.length) if ef != "none" else None
    v_ref = torch.zeros(plan.length) if ef == "dgc" else None
    r_dev = r_ref.to(DEV) if r_ref is not None else None
    v_dev = v_ref.to(DEV) if v_ref is not None else None
    hp = dict(momentum=0.9, dampening=0.0, nesterov=False, weight_decay=0.0)
    for it, g in enumerate(seq):
        key = stream_key(7, it, 1)
        dgc_ref = dict(velocity=v_ref, param=None, **hp) if ef == "dgc" else None
        dgc_dev = dict(velocity=v_dev, param=None, **hp) if ef == "dgc" else None
        ref = oracle.encode_topk(g.clone(), plan, lay, levels, "max", key, residual=r_ref,
                                 dgc=dgc_ref)
        ops.topk_encode(dp, g.to(DEV), pay, lay, levels, "max", key, resid=r_dev, dgc=dgc_dev)
        assert torch.equal(pay.cpu(), ref), f"step {it}: payload"
        if r_ref is not None:
            assert torch.equal(r_dev.cpu(), r_ref), f"step {it}: resid"
        if v_ref is not None:
            assert torch.equal(v_dev.cpu(), v_ref), f"step {it}: vel"
    st = ops.topk_stats(dp)
    assert st["lookback_errors"] == 0, st
    assert st["fast"] > 0 and st["full"] > 0, st  # both paths ran


@pytest.mark.parametrize("numels", [SMALL, [1728, 64, 2359296, 512, 262144, 5120]])
@pytest.mark.parametrize("kind,bits", [("topk_qsgd", 8), ("topk_qsgd", 4), ("topk", 8)])
def test_topk_encode_apply_matches_decode(numels, kind, bits):
    """A world of one: the encode's write pass applies the update itself (ops.topk_encode
    apply=..., on the one-launch and the three-launch encodes) -- parameters, bf16 shadow and the
    advanced RNG key state bitwise those of the encode followed by the sparse decode of the
    one-rank all-gather (k_topk_decode_sparse), step after step under DGC error feedback."""
    ops.require()
    plan = _plan(numels, 0.01, bucket_offset=64)
    lay = Layout.build(kind, plan, bits)
    levels = 127 if bits == 8 else 7
    hp = dict(momentum=0.9, dampening=0.0, nesterov=False, weight_decay=0.0)
    gen = torch.Generator().manual_seed(5)
    p0 = torch.randn(plan.length, generator=gen).to(DEV)
    runs = []
    for fused in (False, True):
        dp = ops.DevicePlan(plan, DEV)
        pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
        r = torch.zeros(plan.length, device=DEV)
        v = torch.zeros(plan.length, device=DEV)
        p = p0.clone()
        sh = p0.to(torch.bfloat16)  # the invariant the trainer keeps: shadow = bf16(param)
        k3 = int(stream_key(9, 3, 0))
        ks = torch.tensor([3, k3 - (1 << 32) if k3 >= 1 << 31 else k3], dtype=torch.int32,
                          device=DEV)
        for it in range(8):
            g = _grad(plan, seed=70 + it).to(DEV)
            dgc = dict(velocity=v, param=None, **hp)
            kd = ks[1:2]
            if fused:
                ops.topk_encode(dp, g, pay, lay, levels, "max", 0, resid=r, key_tensor=kd,
                                dgc=dgc, apply=dict(param=p, shadow=sh, lr=0.05, grad_scale=1.0,
                                                    key_state=ks, key_seed=9, key_rank=0))
            else:
                ops.topk_encode(dp, g, pay, lay, levels, "max", 0, resid=r, key_tensor=kd,
                                dgc=dgc)
                ops.topk_decode_apply(dp, pay.view(1, -1), lay, levels, param=p, mom=None,
                                      lr=0.05, grad_scale=1.0, shadow=sh, key_state=ks,
                                      key_seed=9, key_rank=0)
        torch.cuda.synchronize()
        runs.append((p, sh, ks, r, v, pay))
    for name, a, b in zip(("param", "shadow", "key_state", "resid", "vel", "payload"), *runs):
        assert torch.equal(a.view(torch.uint8) if a.dtype != torch.uint8 else a,
                           b.view(torch.uint8) if b.dtype != torch.uint8 else b), name
    assert not torch.equal(runs[0][0], p0)


@pytest.mark.parametrize("ef", ["none", "plain"])
@pytest.mark.parametrize("kind,bits", [("topk_qsgd", 8), ("topk", 8)])
def test_topk_encode_dense_apply_matches_decode(ef, kind, bits):
    """A world of one without momentum correction (the reference's Method 5: the momentum runs
    on the receiver): the one-launch encode applies the dense momentum step over its chunk after
    the write -- parameters, momentum, bf16 shadow and key state bitwise the encode followed by
    the decode's dense pass (k_topk_decode_apply with a momentum buffer), step after step."""
    ops.require()
    plan = _plan(SMALL, 0.01, bucket_offset=64)
    lay = Layout.build(kind, plan, bits)
    levels = 127 if bits == 8 else 7
    gen = torch.Generator().manual_seed(6)
    p0 = torch.randn(plan.length, generator=gen).to(DEV)
    m0 = torch.randn(plan.length, generator=gen).to(DEV) * 0.1
    hp = dict(lr=0.05, momentum=0.9, dampening=0.0, weight_decay=1e-4, nesterov=True)
    runs = []
    for fused in (False, True):
        dp = ops.DevicePlan(plan, DEV)
        assert ops.topk_one_launch(dp)
        pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
        r = torch.zeros(plan.length, device=DEV) if ef == "plain" else None
        p, m = p0.clone(), m0.clone()
        sh = p0.to(torch.bfloat16)
        k3 = int(stream_key(9, 3, 0))
        ks = torch.tensor([3, k3 - (1 << 32) if k3 >= 1 << 31 else k3], dtype=torch.int32,
                          device=DEV)
        for it in range(6):
            g = _grad(plan, seed=90 + it).to(DEV)
            first = it == 0
            if fused:
                ops.topk_encode(dp, g, pay, lay, levels, "max", 0, resid=r, key_tensor=ks[1:2],
                                apply=dict(param=p, mom=m, shadow=sh, grad_scale=1.0,
                                           key_state=ks, key_seed=9, key_rank=0, first=first,
                                           **hp))
            else:
                ops.topk_encode(dp, g, pay, lay, levels, "max", 0, resid=r, key_tensor=ks[1:2])
                ops.topk_decode_apply(dp, pay.view(1, -1), lay, levels, param=p, mom=m,
                                      grad_scale=1.0, shadow=sh, key_state=ks, key_seed=9,
                                      key_rank=0, first=first, **hp)
        torch.cuda.synchronize()
        runs.append((p, m, sh, ks, pay))
    for name, a, b in zip(("param", "mom", "shadow", "key_state", "payload"), *runs):
        assert torch.equal(a.view(torch.uint8) if a.dtype != torch.uint8 else a,
                           b.view(torch.uint8) if b.dtype != torch.uint8 else b), name
