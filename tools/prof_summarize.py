"""Summarise a rocprofv3 ``--kernel-trace --output-format csv`` run into a small text report.

Usage: python tools/prof_summarize.py <dir containing *kernel_trace.csv> <out.txt> [--steps K]
       [--delete]

Reports per-kernel totals over the last K-step window (the timed region of bench.py: the final
``steps`` iterations), GPU busy fraction (union of kernel intervals / wall span), and kernels per
step.  ``--delete`` removes the raw trace CSVs afterwards (gpurun copies back <= 64 MiB).
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r.get("Kernel_Name", "?")))
    rows.sort()
    return rows


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    # drop the argument list (first "(" not inside a template) but keep template args
    depth, cut = 0, len(n)
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0 and i > 0:
            cut = i
            break
    return n[:cut][:110] or name[:110]


def timed_window(rows, frac=0.5, gap_ns=150_000_000):
    """Rows (start, end, name, ...) of the timed loop: the window between two idle gaps >= gap_ns
    (bench.py EWDML_PROF_GAP=1 sleeps before and after it), or everything after a single gap;
    falls back to the last ``frac`` of the trace.  Returns (rows, description)."""
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    gaps = []  # (idle start, idle end)
    end = rows[0][1]
    for r in rows[1:]:
        s, e = r[0], r[1]
        if s - end >= gap_ns:
            gaps.append((end, s))
        end = max(end, e)
    # bench.py (EWDML_PROF_GAP=1) idles before and after each timed loop: of the windows between
    # two consecutive gaps, the first one the GPU kept >= 90 % busy (the headline's timed steps;
    # the extra measurements that follow each add a setup window and a timed window of their own),
    # else the one with the most kernels (teardown after the loop can add idle gaps of its own); a
    # trace with one gap: everything after it
    stop = None
    if len(gaps) >= 2:
        def stats(a, b):
            w = [r for r in rows if a <= r[0] < b]
            if not w:
                return 0, 0.0
            busy, cs, ce = 0, w[0][0], w[0][1]
            for s, e, *_ in w[1:]:
                if s > ce:
                    busy += ce - cs
                    cs, ce = s, e
                else:
                    ce = max(ce, e)
            busy += ce - cs
            return len(w), busy / max(1, max(r[1] for r in w) - w[0][0])

        st = [stats(gaps[j][1], gaps[j + 1][0]) for j in range(len(gaps) - 1)]
        dense = [j for j, (n, f) in enumerate(st) if n >= 10 and f >= 0.9]
        if dense:
            i = dense[0]
            how = "between two idle gaps (the first >= 90 % busy window)"
        else:
            i = max(range(len(st)), key=lambda j: (st[j][0], j))
            how = "between two idle gaps (the busiest window)"
        cut, stop = gaps[i][1], gaps[i + 1][0]
    elif gaps:
        cut = gaps[-1][1]
        how = "after last idle gap"
    else:
        cut = t0 + (t1 - t0) * (1 - frac)
        how = f"last {frac:.0%} of trace"
    return [r for r in rows if r[0] >= cut and (stop is None or r[0] < stop)], how


def summarize(rows, frac=0.5, gap_ns=150_000_000, steps=None):
    """Per-kernel report of the timed window (``timed_window``)."""
    if not rows:
        return "no kernels\n"
    win, how = timed_window(rows, frac, gap_ns)
    span = max(r[1] for r in win) - win[0][0]
    busy = 0
    cur_s, cur_e = win[0][0], win[0][1]
    for s, e, _ in win[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in win:
        agg[short(n)][0] += 1
        agg[short(n)][1] += e - s
    per = f", per step {span / 1e6 / steps:.3f} ms" if steps else ""
    out = [f"window: {how}, {len(win)} kernels, span {span / 1e6:.3f} ms{per}, "
           f"GPU busy {busy / 1e6:.3f} ms ({100 * busy / span:.1f}%)",
           f"{'calls':>7} {'total_ms':>10} {'avg_us':>9}" + (" us/step " if steps else "") +
           "  kernel"]
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:60]:
        ps = f" {t / 1e3 / steps:>9.2f}" if steps else ""
        out.append(f"{c:>7} {t / 1e6:>10.3f} {t / c / 1e3:>9.2f}{ps}  {n}")
    # where the idle time is: the largest gaps between consecutive kernels, with their neighbours
    gaps, end_prev, name_prev = [], win[0][1], win[0][2]
    for s, e, n in win[1:]:
        if s > end_prev:
            gaps.append((s - end_prev, name_prev, n))
        if e >= end_prev:
            end_prev, name_prev = e, n
    if gaps:
        tot = sum(g[0] for g in gaps)
        out.append("")
        out.append(f"idle: {tot / 1e3:.1f} us in {len(gaps)} gaps"
                   + (f" ({tot / 1e3 / steps:.1f} us/step)" if steps else "") + "; largest:")
        for g, a, b in sorted(gaps, reverse=True)[:8]:
            out.append(f"{g / 1e3:>9.2f} us  {short(a)[:50]}  ->  {short(b)[:50]}")
    if steps:  # the last step's kernels in launch order: duration and idle gap before each
        per_step = len(win) // steps
        last = win[-per_step:]
        out.append("")
        out.append(f"last step, {per_step} kernels in order:  gap_us  dur_us  kernel")
        prev_end = last[0][0]
        for s, e, n in last:
            out.append(f"{max(0, s - prev_end) / 1e3:>8.2f} {(e - s) / 1e3:>7.2f}  {short(n)[:90]}")
            prev_end = max(prev_end, e)
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    d, out = sys.argv[1], sys.argv[2]
    rows = load(d)
    steps = None
    if "--steps" in sys.argv:
        steps = int(sys.argv[sys.argv.index("--steps") + 1])
    txt = summarize(rows, steps=steps)
    with open(out, "w") as f:
        f.write(txt)
    print(txt[:3000])
    if "--delete" in sys.argv:
        for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
            if "stats" not in os.path.basename(f):
                os.remove(f)
        for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
            os.remove(f)
