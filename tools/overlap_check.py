"""Did the exchange run beside backward?  Reads a rocprofv3 ``--kernel-trace --output-format csv``
run and reports, over the timed window (after bench.py's EWDML_PROF_GAP idle gap), how much of the
exchange kernels' time (codec encode, gradient pack, RCCL) intersects compute kernels running on
another queue/stream.

Usage: python tools/overlap_check.py <trace dir> [--steps K] [--out file]
"""
import argparse
import csv
import glob
import os
import re

EXCHANGE = re.compile(r"k_topk_(hist|count|write)|k_qsgd_(stats|scale|quant)|k_pack|nccl|rccl|"
                      r"Rccl|ncclDevKernel|ncclKernel", re.I)
SKIP = re.compile(r"k_watch_mark|k_topk_decode|k_qsgd_decode")


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                q = r.get("Queue_Id") or r.get("Stream_Id") or r.get("Correlation_Id", "")
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r.get("Kernel_Name", "?"), str(r.get("Stream_Id") or q)))
    rows.sort()
    return rows


def window(rows, gap_ns=150_000_000):
    end, cut = rows[0][1], None
    for s, e, *_ in rows[1:]:
        if s - end >= gap_ns:
            cut = s
        end = max(end, e)
    return [r for r in rows if cut is None or r[0] >= cut]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    win = window(load(a.trace))
    ex = [r for r in win if EXCHANGE.search(r[2]) and not SKIP.search(r[2])]
    comp = [r for r in win if not EXCHANGE.search(r[2]) and not SKIP.search(r[2])]
    lines = [f"kernels in window: {len(win)} ({len(ex)} exchange, {len(comp)} other)"]
    # per exchange kernel: the part of its interval covered by compute kernels on other streams
    comp_by_stream = {}
    for s, e, n, st in comp:
        comp_by_stream.setdefault(st, []).append((s, e))
    tot_ex = tot_ov = 0
    names = {}
    for s, e, n, st in ex:
        cov = []
        for cst, ivs in comp_by_stream.items():
            if cst == st:
                continue
            for cs, ce in ivs:
                if ce > s and cs < e:
                    cov.append((max(cs, s), min(ce, e)))
        cov.sort()
        ov, cur_s, cur_e = 0, None, None
        for cs, ce in cov:
            if cur_e is None or cs > cur_e:
                if cur_e is not None:
                    ov += cur_e - cur_s
                cur_s, cur_e = cs, ce
            else:
                cur_e = max(cur_e, ce)
        if cur_e is not None:
            ov += cur_e - cur_s
        tot_ex += e - s
        tot_ov += ov
        k = re.sub(r"\(.*", "", n)[:60]
        a_ = names.setdefault(k, [0, 0, 0])
        a_[0] += 1
        a_[1] += e - s
        a_[2] += ov
    streams = sorted({r[3] for r in win})
    lines.append(f"streams/queues seen: {streams}")
    lines.append(f"exchange kernel time per step: {tot_ex / 1e3 / a.steps:.1f} us, of which "
                 f"{tot_ov / 1e3 / a.steps:.1f} us ({100.0 * tot_ov / max(1, tot_ex):.0f} %) ran "
                 "while compute kernels ran on another stream")
    lines.append("kernel | calls | us/step | overlapped us/step")
    for k, (c, t, o) in sorted(names.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"{k} | {c} | {t / 1e3 / a.steps:.1f} | {o / 1e3 / a.steps:.1f}")
    txt = "\n".join(lines) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
