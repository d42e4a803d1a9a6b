#!/usr/bin/env python3
"""Median duration of consecutive groups of dispatches of one kernel in a rocprofv3
kernel_trace.csv: usage trace_groups.py <kernel_trace.csv> <name-substring> <group-size>."""
import csv
import sys


def main():
    path, sub, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    for i in range(0, len(d), n):
        g = sorted(d[i:i + n])
        print(f"group {i // n}: n={len(g)} median {g[len(g) // 2]:.1f} us  min {g[0]:.1f} us")


if __name__ == "__main__":
    main()
