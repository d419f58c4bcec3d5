"""Where does a HIP top-k encode differ from the oracle?  Runs the repeated-encode sequence of
tests/kernels/test_hip_codecs.py::test_topk_repeated_encodes_reuse_scratch and prints, per encode,
which payload sections differ (scales / counts / idx / bitmap / codes) and for which tensors."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from ewdml import ops  # noqa: E402
from ewdml.compress import oracle  # noqa: E402
from ewdml.compress.plan import BucketPlan, Layout  # noqa: E402
from ewdml.compress.rng import stream_key  # noqa: E402


def _plan(numels, ratio):
    offs, o = [], 0
    for n in numels:
        offs.append(o)
        o += (n + 63) // 64 * 64
    return BucketPlan(numels, offs, ratio, 0, o)


def _grad(plan, seed, ties):
    g = torch.zeros(plan.length)
    gen = torch.Generator().manual_seed(seed)
    for off, n in zip(plan.offsets, plan.numels):
        x = torch.randn(n, generator=gen) * (0.1 + torch.rand(1, generator=gen))
        if ties:
            x = torch.round(x * 4) / 4
        g[off:off + n] = x
    return g


def diff(plan, lay, got, ref):
    T, C = plan.num_tensors, plan.num_chunks
    sec = {"scales": (lay.scales, 4 * T), "counts": (lay.counts, 2 * C),
           "idx": (lay.idx, 2 * plan.total_idx), "bitmap": (lay.bitmap, 4 * plan.total_bm_words),
           "codes": (lay.codes, plan.total_k)}
    out = []
    for k, (o, n) in sec.items():
        a, b = got[o:o + n], ref[o:o + n]
        if not torch.equal(a, b):
            out.append(f"{k}: {int((a != b).sum())} bytes differ")
    cg = got[lay.counts:lay.counts + 2 * C].view(torch.int16)
    cr = ref[lay.counts:lay.counts + 2 * C].view(torch.int16)
    for t in range(T):
        c0, nc = plan.tensor_chunk0[t], plan.tensor_nchunks[t]
        if not torch.equal(cg[c0:c0 + nc], cr[c0:c0 + nc]):
            d = (cg[c0:c0 + nc] != cr[c0:c0 + nc]).nonzero().flatten()[:5].tolist()
            out.append(f"  tensor {t} (n={plan.numels[t]}, k={plan.ks[t]}): counts differ at "
                       f"chunks {d}: got {cg[c0:c0 + nc][d].tolist()} ref {cr[c0:c0 + nc][d].tolist()}"
                       f" sums {int(cg[c0:c0 + nc].sum())} / {int(cr[c0:c0 + nc].sum())}")
    return out


def main():
    ops.require()
    plan = _plan([20 * 25, 20, 50 * 500, 50, 2359296], 0.01)
    lay = Layout.build("topk_qsgd", plan, 8)
    dp = ops.DevicePlan(plan, "cuda")
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device="cuda")
    for it in range(4):
        g = _grad(plan, 10 + it, it == 2)
        key = stream_key(5, it, 0)
        ref = oracle.encode_topk(g.clone(), plan, lay, 127, "max", key)
        ops.topk_encode(dp, g.cuda(), pay, lay, 127, "max", key)
        got = pay.cpu()
        print(f"encode {it} (ties={it == 2}): {'OK' if torch.equal(got, ref) else 'DIFF'}")
        for line in diff(plan, lay, got, ref):
            print("   ", line)
    print("lookback errors:", ops.topk_lookback_errors(dp))
    # the ties gradient on a fresh plan
    dp2 = ops.DevicePlan(plan, "cuda")
    g = _grad(plan, 12, True)
    ref = oracle.encode_topk(g.clone(), plan, lay, 127, "max", 7)
    ops.topk_encode(dp2, g.cuda(), pay, lay, 127, "max", 7)
    print("fresh plan, ties:", "OK" if torch.equal(pay.cpu(), ref) else "DIFF")
    for line in diff(plan, lay, pay.cpu(), ref):
        print("   ", line)


if __name__ == "__main__":
    main()


def detail():
    plan = _plan([20 * 25, 20, 50 * 500, 50, 2359296], 0.01)
    lay = Layout.build("topk_qsgd", plan, 8)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device="cuda")
    g = _grad(plan, 12, True)
    for norm in ("l2", "max"):
        dp = ops.DevicePlan(plan, "cuda")
        ref = oracle.encode_topk(g.clone(), plan, lay, 127, norm, 7)
        ops.topk_encode(dp, g.cuda(), pay, lay, 127, norm, 7)
        got = pay.cpu()
        ig = got[lay.idx:lay.idx + 2 * plan.total_idx].view(torch.int16).long() & 0xFFFF
        ir = ref[lay.idx:lay.idx + 2 * plan.total_idx].view(torch.int16).long() & 0xFFFF
        bad = (ig != ir).nonzero().flatten()
        print(f"{norm}: idx mismatches {bad.numel()}",
              "first at entry", bad[:3].tolist(), "got", ig[bad[:8]].tolist(), "ref",
              ir[bad[:8]].tolist())
        if bad.numel():
            e = int(bad[0])
            print("   got around:", ig[max(0, e - 4):e + 6].tolist())
            print("   ref around:", ir[max(0, e - 4):e + 6].tolist())
            t = 4
            off = plan.offsets[t]
            x = g[off:off + plan.numels[t]].abs()
            kth = torch.topk(x, plan.ks[t]).values.min()
            print("   kth", float(kth), "#gt", int((x > kth).sum()), "#eq", int((x == kth).sum()),
                  "k", plan.ks[t])


def lookback_words():
    """Read the write pass's look-back words back and compare the inclusive prefixes with the
    host's cumulative (#gt, #eq) per chunk."""
    plan = _plan([20 * 25, 20, 50 * 500, 50, 2359296], 0.01)
    lay = Layout.build("topk_qsgd", plan, 8)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device="cuda")
    g = _grad(plan, 12, True)
    dp = ops.DevicePlan(plan, "cuda")
    ops.topk_encode(dp, g.cuda(), pay, lay, 127, "max", 7)
    torch.cuda.synchronize()
    T, C = plan.num_tensors, plan.num_chunks
    NREP, NB0, NB1, NB2, TS = 8, 2048, 1024, 1024, 32
    words = 4 * T + NREP * T * (1 + NB0 + NB1 + NB2) + 5 * C + T
    base = dp.scratch.data_ptr()
    inv_end = base + 4 * words
    tick = (inv_end + TS * 4 - 1) & ~(TS * 4 - 1)
    lb_err = tick + 4 * (5 * TS * T)
    lb = lb_err + 4 * TS
    off = lb - base
    w = dp.scratch[off:off + 8 * C].cpu().view(torch.int64)
    state = dp.scratch[:16 * T].cpu().view(torch.int32)
    t = 4
    c0, nc = plan.tensor_chunk0[t], plan.tensor_nchunks[t]
    x = g[plan.offsets[t]:plan.offsets[t] + plan.numels[t]].abs().view(torch.int32)
    thr = int(state[4 * t]) & 0x7FFFFFFF
    print("thr key", thr, "need", int(state[4 * t + 1]))
    cg = ce = 0
    bad = 0
    for j in range(nc):
        seg = x[j * 8192:(j + 1) * 8192]
        cg += int((seg > thr).sum())
        ce += int((seg == thr).sum())
        v = int(w[c0 + j]) & ((1 << 64) - 1)
        st, gt, eq = v >> 62, (v >> 31) & 0x7FFFFFFF, v & 0x7FFFFFFF
        if st != 2 or gt != cg or eq != ce:
            if bad < 8:
                print(f"chunk {j}: status {st} word gt {gt} eq {eq}  host inclusive gt {cg} eq {ce}")
            bad += 1
    print("bad words:", bad, "of", nc)


def chunk_view():
    plan = _plan([20 * 25, 20, 50 * 500, 50, 2359296], 0.01)
    lay = Layout.build("topk_qsgd", plan, 8)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device="cuda")
    g = _grad(plan, 12, True)
    dp = ops.DevicePlan(plan, "cuda")
    ref = oracle.encode_topk(g.clone(), plan, lay, 127, "max", 7)
    ops.topk_encode(dp, g.cuda(), pay, lay, 127, "max", 7)
    got = pay.cpu()
    t = 4
    c0, nc, i0, k = plan.tensor_chunk0[t], plan.tensor_nchunks[t], plan.tensor_idx0[t], plan.ks[t]
    cnt = ref[lay.counts:lay.counts + 2 * plan.num_chunks].view(torch.int16).long()[c0:c0 + nc]
    ig = got[lay.idx:lay.idx + 2 * plan.total_idx].view(torch.int16).long()[i0:i0 + k] & 0xFFFF
    ir = ref[lay.idx:lay.idx + 2 * plan.total_idx].view(torch.int16).long()[i0:i0 + k] & 0xFFFF
    x = g[plan.offsets[t]:plan.offsets[t] + plan.numels[t]].abs()
    e = 0
    shown = 0
    for j in range(nc):
        n = int(cnt[j])
        a, b = ig[e:e + n], ir[e:e + n]
        if not torch.equal(a, b) and shown < 3:
            seg = x[j * 8192:(j + 1) * 8192]
            print(f"chunk {j}: entries [{e}, {e + n}) count {n}; #gt {int((seg > 2.75).sum())} "
                  f"#eq {int((seg == 2.75).sum())}")
            d = (a != b).nonzero().flatten()
            print("   first diff at", d[:4].tolist(), "got", a[d[:6]].tolist(), "ref",
                  b[d[:6]].tolist())
            print("   got sorted?", bool((a[1:] > a[:-1]).all()), "dups", n - a.unique().numel(),
                  "got max", int(a.max()), "ref max", int(b.max()))
            shown += 1
        e += n


def lb_values():
    plan = _plan([20 * 25, 20, 50 * 500, 50, 2359296], 0.01)
    lay = Layout.build("topk_qsgd", plan, 8)
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device="cuda")
    g = _grad(plan, 12, True)
    dp = ops.DevicePlan(plan, "cuda")
    ops.topk_encode(dp, g.cuda(), pay, lay, 127, "max", 7)
    torch.cuda.synchronize()
    T, C = plan.num_tensors, plan.num_chunks
    NREP, NB0, NB1, NB2 = 8, 2048, 1024, 1024
    w0 = 4 * T + NREP * T * (1 + NB0 + NB1 + NB2)  # cnt_gt
    sc = dp.scratch.cpu().view(torch.int32)
    off = sc[w0 + 2 * C:w0 + 3 * C]
    ties = sc[w0 + 3 * C:w0 + 4 * C]
    t = 4
    c0, nc = plan.tensor_chunk0[t], plan.tensor_nchunks[t]
    x = g[plan.offsets[t]:plan.offsets[t] + plan.numels[t]].abs()
    state = dp.scratch[:16 * T].cpu().view(torch.int32)
    need = int(state[4 * t + 1])
    gb = eb = 0
    for j in range(0, 50):
        seg = x[j * 8192:(j + 1) * 8192]
        gt, eq = int((seg > 2.75).sum()), int((seg == 2.75).sum())
        tc = min(max(need - eb, 0), eq)
        if j >= 44:
            print(f"chunk {j}: kernel off {int(off[c0 + j])} ties {int(ties[c0 + j])}  host off "
              f"{gb + min(eb, need)} ties {tc}  (gb {gb} eb {eb} need {need})")  # noqa
        gb += gt
        eb += eq
    print(list(range(0)))


def host_prefix_until(plan, x, j1):
    pass


lb_values()
