#!/usr/bin/env python3
"""Kernel time and idle gaps inside the LAST forest fit of a rocprofv3 kernel_trace.csv:
usage fit_breakdown.py <kernel_trace.csv> <fits in the trace> [top]."""
import collections
import csv
import sys


def main():
    path, nfits = sys.argv[1], int(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 14
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    hs = [i for i, r in enumerate(rows) if "tree_hist_split" in r["Kernel_Name"]]
    per = len(hs) // nfits
    seg = rows[hs[-per - 1] + 1:hs[-1] + 1]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    agg, cnt = collections.Counter(), collections.Counter()
    for r in seg:
        k = r["Kernel_Name"][:100]
        agg[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[k] += 1
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(seg, seg[1:])]
    print(f"last fit: window {(t1 - t0) / 1e3:.1f} us, kernel busy {sum(agg.values()):.1f} us, "
          f"idle gaps {sum(g for g in gaps if g > 0):.1f} us, {len(seg)} dispatches")
    for k, v in agg.most_common(top):
        print(f"{v:9.1f} {cnt[k]:4d}  {k}")


if __name__ == "__main__":
    main()
