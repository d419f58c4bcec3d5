"""Per-kernel roofline of bench.py's timed step from one kernel trace plus rocprofv3 --pmc passes.

    python tools/roofline.py <trace dir> <out.txt> --steps K <pmc dir> [<pmc dir> ...]

* Durations and calls per step come from the kernel-trace run (``prof_summarize.timed_window``: the
  timed loop only, un-profiled clocks apart from the tracer itself).
* Counters come from the --pmc passes (which serialise dispatches and include the warmup steps):
  each counter is averaged per (kernel, grid size) over every dispatch that has it, then weighted
  by that (kernel, grid)'s calls per step in the trace window.
* Columns: calls/step, us/step, MB read (FETCH_SIZE, raw: on gfx950 it tallies a wide coalesced
  streaming read at half its bytes, MI355X_MICROARCH.md "HBM"), MB written (WRITE_SIZE), TB/s on
  raw read + write and on 2 x read + write (the two bracket the real HBM rate), MFMA TF/s
  (SQ_VALU_MFMA_BUSY_CYCLES x 64 FLOP per busy SIMD cycle, the f32 MFMA rate, over the traced
  duration) and its share of the 157.3 TF/s f32 peak, LDS bank-conflict cycles per LDS instruction.
"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import prof_summarize as ps  # noqa: E402

F32_PEAK_TF = 157.3
HBM_TBS = 6.3  # achievable (MI355X_MICROARCH.md "HBM")


def load_trace(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                grid = 1
                for ax in "XYZ":
                    grid *= int(r.get(f"Grid_Size_{ax}", 1) or 1)
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r.get("Kernel_Name", "?"), grid))
    rows.sort()
    return rows


def load_pmc(dirs):
    acc = defaultdict(lambda: defaultdict(list))  # (short, grid) -> counter -> values
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    key = (ps.short(r.get("Kernel_Name", "?")), int(r.get("Grid_Size", 0) or 0))
                    acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def table(trace_rows, pmc, steps):
    win, how = ps.timed_window(trace_rows)
    span = max(r[1] for r in win) - win[0][0]
    per = defaultdict(lambda: defaultdict(lambda: [0, 0]))  # short -> grid -> [calls, ns]
    for s, e, n, g in win:
        c = per[ps.short(n)][g]
        c[0] += 1
        c[1] += e - s
    out_rows = []
    tot = defaultdict(float)
    for name, grids in per.items():
        calls = sum(c for c, _ in grids.values())
        ns = sum(t for _, t in grids.values())
        ctr = defaultdict(float)
        have = set()
        for g, (c, _) in grids.items():
            m = pmc.get((name, g))
            if m is None:
                continue
            for k, v in m.items():
                ctr[k] += v * c
                have.add(k)
        us = ns / 1e3 / steps
        rd = ctr["FETCH_SIZE"] * 1024 / 1e6 / steps if "FETCH_SIZE" in have else None
        wr = ctr["WRITE_SIZE"] * 1024 / 1e6 / steps if "WRITE_SIZE" in have else None
        mf = ctr["SQ_VALU_MFMA_BUSY_CYCLES"] / steps if "SQ_VALU_MFMA_BUSY_CYCLES" in have else None
        lds_i = ctr.get("SQ_INSTS_LDS", 0.0)
        lds_c = ctr.get("SQ_LDS_BANK_CONFLICT", 0.0)
        out_rows.append(dict(name=name, calls=calls / steps, us=us, rd=rd, wr=wr, mfma=mf,
                             conf=(lds_c / lds_i) if lds_i > 0 else None))
        tot["us"] += us
        for k, v in (("rd", rd), ("wr", wr), ("mfma", mf)):
            if v is not None:
                tot[k] += v
    out_rows.sort(key=lambda r: -r["us"])

    def f(v, fmt):
        return format(v, fmt) if v is not None else "-".rjust(len(format(0.0, fmt)))

    lines = [f"window: {how}; {len(win)} kernels over {steps} steps, {span / 1e6 / steps:.3f} ms "
             f"per step (traced); counters averaged per (kernel, grid) over the --pmc passes",
             f"{'calls':>5} {'us/step':>8} {'MB rd':>7} {'MB wr':>7} {'TB/s':>5} {'TB/s2r':>6} "
             f"{'TF/s':>6} {'%f32pk':>6} {'conf/lds':>8}  kernel"]
    for r in out_rows:
        sec = r["us"] * 1e-6
        bw = (r["rd"] + r["wr"]) * 1e6 / sec / 1e12 if r["rd"] is not None and r["wr"] is not None else None
        bw2 = (2 * r["rd"] + r["wr"]) * 1e6 / sec / 1e12 if bw is not None else None
        tf = r["mfma"] * 64 / sec / 1e12 if r["mfma"] is not None else None
        pk = 100 * tf / F32_PEAK_TF if tf is not None else None
        lines.append(f"{r['calls']:>5.1f} {r['us']:>8.2f} {f(r['rd'], '7.2f')} {f(r['wr'], '7.2f')} "
                     f"{f(bw, '5.2f')} {f(bw2, '6.2f')} {f(tf, '6.1f')} {f(pk, '6.1f')} "
                     f"{f(r['conf'], '8.3f')}  {r['name'][:80]}")
    sec = tot["us"] * 1e-6
    lines.append("")
    lines.append(f"total busy {tot['us']:.1f} us/step; read {tot['rd']:.1f} MB (raw FETCH_SIZE), "
                 f"written {tot['wr']:.1f} MB; MFMA {tot['mfma'] * 64 / 1e9:.2f} GFLOP/step "
                 f"= {tot['mfma'] * 64 / sec / 1e12 if sec else 0:.1f} TF/s over busy time "
                 f"({100 * tot['mfma'] * 64 / sec / 1e12 / F32_PEAK_TF if sec else 0:.1f} % of "
                 f"{F32_PEAK_TF} TF/s)")
    return "\n".join(lines) + "\n"


def main():
    args = [a for a in sys.argv[1:]]
    steps = 1
    if "--steps" in args:
        i = args.index("--steps")
        steps = int(args[i + 1])
        del args[i:i + 2]
    trace_dir, out, pmc_dirs = args[0], args[1], args[2:]
    txt = table(load_trace(trace_dir), load_pmc(pmc_dirs), steps)
    with open(out, "w") as fh:
        fh.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
