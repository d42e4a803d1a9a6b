#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per kernel over every pass directory given.

usage: python tools/pmc_table.py gpurun_out/pmc1 gpurun_out/pmc2 ... > profiles/x.md
Adds derived columns when the inputs are present: MFMA busy %, VALU busy,
HBM bytes (FETCH_SIZE + WRITE_SIZE are in KiB) and achieved GB/s over the
kernel's own duration.
"""
import csv
import os
import sys
from collections import defaultdict


def main():
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for d in sys.argv[1:]:
        with open(os.path.join(d, "pmc_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"]
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    names = sorted({c for k in vals for c in vals[k]})
    keep = [k for k in vals if "at::native" not in k and "rocprim" not in k]
    print("| kernel | us | " + " | ".join(names) + " |")
    print("|---|---:|" + "---:|" * len(names))
    for k in sorted(keep, key=lambda k: -sum(dur[k]) / len(dur[k])):
        us = sum(dur[k]) / len(dur[k]) / 1e3
        row = [f"{sum(v) / len(v):.4g}" for v in (vals[k].get(n, [float('nan')]) for n in names)]
        short = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]
        print(f"| `{short}` | {us:.1f} | " + " | ".join(row) + " |")


if __name__ == "__main__":
    main()
