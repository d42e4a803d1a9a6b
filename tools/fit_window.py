#!/usr/bin/env python3
"""Kernel time inside the LAST forest fit of a rocprofv3 kernel trace (bench --config rf/rf9):
the window spans the last N tree_hist_split dispatches; prints busy vs wall and the top kernels."""
import csv
import sys
from collections import Counter

path, nlev = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
hs = [r for r in rows if "tree_hist_split" in r["Kernel_Name"]]
last = hs[-nlev:]
t0, t1 = int(last[0]["Start_Timestamp"]), int(last[-1]["End_Timestamp"])
for r in last:
    print(r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"],
          round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1))
inside = [r for r in rows if t0 <= int(r["Start_Timestamp"]) <= t1]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in inside)
print(f"window {(t1 - t0) / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us")
c = Counter()
for r in inside:
    c[r["Kernel_Name"][:90]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, v in c.most_common(10):
    print(f"{v / 1e3:9.1f}  {k}")
