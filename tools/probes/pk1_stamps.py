"""Phase stamps of the one-launch small-bucket encode (ops/csrc/topk_codec.hip k_pk_one) on
LeNet's bucket, steady-state DGC error feedback.  Run with EWDML_PK1_STAMPS=1:

    EWDML_PK1_STAMPS=1 python tools/probes/pk1_stamps.py

Prints, per tensor, the spread of each phase over its blocks in us from the launch's first
stamp: 0 start, 1 staged, 2 candidates appended (ticket), 6/7 select begin/end (tensor-last
block), 3 selected (generation seen), 4 written; inside the tensor-last block's select: 8 pass 0
(keys staged), 9 fold, 10 digit 0, 12 the selected bin's keys compacted, 11 ranked (or digits 1 and 2), 13 the
prediction stored."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from ewdml import ops  # noqa: E402
from ewdml.compress.plan import BucketPlan, Layout  # noqa: E402

SHAPES = [20 * 25, 20, 50 * 500, 50, 800 * 500, 500, 5000, 10]


def main():
    assert os.environ.get("EWDML_PK1_STAMPS") == "1", "set EWDML_PK1_STAMPS=1"
    offs, o = [], 0
    for n in SHAPES:
        offs.append(o)
        o += (n + 63) // 64 * 64
    plan = BucketPlan(SHAPES, offs, 0.01, 0, o)
    lay = Layout.build("topk_qsgd", plan, 8)
    dp = ops.DevicePlan(plan, "cuda")
    pay = torch.zeros(lay.nbytes, dtype=torch.uint8, device="cuda")
    r = torch.zeros(plan.length, device="cuda")
    v = torch.zeros(plan.length, device="cuda")
    hp = dict(velocity=v, param=None, momentum=0.9, dampening=0.0, nesterov=False,
              weight_decay=0.0)
    gen = torch.Generator(device="cuda").manual_seed(0)
    for it in range(40):
        g = torch.randn(plan.length, device="cuda", generator=gen) * 0.01
        ops.topk_encode(dp, g, pay, lay, 127, "max", it + 1, resid=r, dgc=hp)
    torch.cuda.synchronize()
    print("stats", ops.topk_stats(dp))
    st = ops.require().topk_one_stamps()
    C = plan.num_chunks
    rows = [st[16 * b:16 * b + 16] for b in range(C)]
    t0 = min(rw[0] for rw in rows)
    us = lambda x: (x - t0) / 100.0  # noqa: E731 - 100 MHz ticks
    chunk_t = [int(x) for x in plan.chunk_table("cpu")[:, 0].tolist()]
    for t in range(plan.num_tensors):
        bs = [b for b in range(C) if chunk_t[b] == t]
        ph = {i: [us(rows[b][i]) for b in bs if rows[b][i]] for i in (0, 1, 2, 6, 8, 9, 10, 12, 11, 13, 7, 3, 4)}
        desc = "  ".join(f"{i}:{min(x):6.2f}-{max(x):6.2f}" if x else f"{i}:-"
                         for i, x in ph.items())
        last = [b for b in bs if rows[b][14]]
        mn = f"  M={rows[last[0]][14]} bin={rows[last[0]][15]}" if last else ""
        print(f"tensor {t} ({plan.numels[t]} el, {len(bs)} blocks, k={plan.ks[t]})  {desc}{mn}")
    print("launch span us", max(us(rw[4]) for rw in rows))


if __name__ == "__main__":
    main()
