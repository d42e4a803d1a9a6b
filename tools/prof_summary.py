#!/usr/bin/env python3
"""Turn a rocprofv3 ``*_kernel_stats.csv`` into a markdown table (for profiles/).

usage: python tools/prof_summary.py gpurun_out/prof/bench_kernel_stats.csv "title" > profiles/x.md
"""
import csv
import sys


def main():
    path, title = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    rows = list(csv.DictReader(open(path)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n\nSource: `{path}` (rocprofv3 --kernel-trace --stats)\n")
    print("| kernel | calls | avg us | total us | % |")
    print("|---|---:|---:|---:|---:|")
    for r in rows:
        name = r["Name"].replace("|", "/")
        if len(name) > 110:
            name = name[:107] + "..."
        print(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
              f"{float(r['TotalDurationNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    print(f"\nTotal kernel time: {total / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
