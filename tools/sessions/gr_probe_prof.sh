#!/bin/bash
# rocprofv3 kernel trace of tools/gr_probe.py: kernel-only durations of each reduction variant
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/grprobe"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o t -- \
  python3 "$ROOT/tools/gr_probe.py" > "$OUT/probe.log" 2>&1 || exit $?
cd "$ROOT" && python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/t_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "grad_reduce_adam" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
names = ["step(3 train)", "reduce+adam", "reduce+store", "adam only", "store only", "region0", "region1", "region2", "region3"]
print(len(d), "dispatches")
i = 0
for n, c in zip(names, [3, 53, 53, 53, 53, 53, 53, 53, 53]):
    seg = sorted(d[i:i + c]); i += c
    if seg:
        print(f"{n:16s} median {seg[len(seg)//2]:6.2f} us  min {seg[0]:6.2f} us")
PY
