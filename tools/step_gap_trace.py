#!/usr/bin/env python3
"""Timeline of the MLP step kernels in a rocprofv3 kernel trace of bench.py (tools/sessions/gpu_step_gaps.sh):
per step the start offset, each kernel's duration and the idle gap before it, so the driver window's
fixed cost (first-launch latency, slow first steps, gaps) is visible.
usage: python tools/step_gap_trace.py <r_kernel_trace.csv> [n_steps]"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))

    def nm(s):
        m = re.search(r"::(\w+_kernel)", s)
        return m.group(1) if m else s[:32]

    t = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm(r["Kernel_Name"])) for r in rows]
    idx = [i for i, x in enumerate(t) if x[2].startswith("mlp_fwd3")]
    first = idx[0]
    t0 = t[first][0]
    prev_end = t[first - 1][1] if first else t0
    print(f"{'kernel':28s} {'start us':>10s} {'dur us':>8s} {'gap us':>8s}")
    for s, e, k in t[first: first + 3 * n + 2]:
        print(f"{k[:28]:28s} {(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} {(s - prev_end) / 1e3:8.1f}")
        prev_end = e
    span = t[first + 3 * n - 1][1] - t0
    print(f"{n} steps: {span / 1e3:.1f} us of kernels+gaps = {span / n / 1e3:.2f} us per step")


if __name__ == "__main__":
    main()
