"""Average rocprofv3 --pmc counters per kernel name (and per grid size).

    python tools/pmc_summarize.py <dir with *counter_collection.csv> [name filter]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "?").replace("(anonymous namespace)::", "")
                name = name.replace("void ", "").split("(")[0][:60]
                if filt not in name:
                    continue
                key = (name, r.get("Grid_Size", ""), r.get("Workgroup_Size", ""))
                acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for key in sorted(acc):
        cs = acc[key]
        vals = "  ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items()))
        print(f"{key[0]} grid={key[1]} wg={key[2]}: {vals}")


if __name__ == "__main__":
    main()
