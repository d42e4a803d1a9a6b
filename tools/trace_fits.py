#!/usr/bin/env python3
"""Per-fit kernel breakdown of a rocprofv3 kernel trace: fits are delimited by a marker kernel that
runs once per fit (default ``sort_columns``, findSplits' column sort).

usage: python tools/trace_fits.py <kernel_trace.csv> [marker] [fit indices, e.g. 3,4,8,9]"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    n = re.sub(r"^void ", "", name)
    n = n.replace("(anonymous namespace)::", "")
    n = re.split(r"[(<]", n, 1)[0] + ("<" + n.split("<", 1)[1].split(">", 1)[0] + ">" if "<" in n.split("(", 1)[0] else "")
    return n[:70]


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "sort_columns"
    show = {int(x) for x in sys.argv[3].split(",")} if len(sys.argv) > 3 else None
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    bounds = idx + [len(rows)]
    for j in range(len(idx)):
        seg = rows[bounds[j]:bounds[j + 1]]
        tot, cnt = collections.Counter(), collections.Counter()
        for r in seg:
            n = short(r["Kernel_Name"])
            tot[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            cnt[n] += 1
        span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
        print(f"--- fit {j}: {len(seg)} kernels, busy {sum(tot.values()):.1f} us, span {span:.1f} us")
        if show is None or j in show:
            for n, v in tot.most_common(16):
                print(f"   {v:8.1f} us {cnt[n]:4d}x  {n}")


if __name__ == "__main__":
    main()
