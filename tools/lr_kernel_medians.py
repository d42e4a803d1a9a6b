#!/usr/bin/env python3
"""Median device time per (LR kernel, models in the launch) from a rocprofv3 kernel trace.
usage: python tools/lr_kernel_medians.py <r_kernel_trace.csv>"""
import collections
import csv
import sys

KERNELS = ("qn_direction", "qn_update", "logreg_eval", "logreg_grad")


def main(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        for k in KERNELS:
            if k in r["Kernel_Name"]:
                d[(k, int(r["Grid_Size_Y"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (k, gy), v in sorted(d.items()):
        v.sort()
        print(f"{k:14s} gridY={gy:4d} n={len(v):4d} median {v[len(v) // 2]:7.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
