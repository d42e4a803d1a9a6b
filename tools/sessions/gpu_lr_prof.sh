#!/bin/bash
# LogisticRegression fit profile: wall time per fit + host cProfile (tools/lr_probe.py) and the
# kernel statistics of the same run (rocprofv3 --kernel-trace --stats), for LR and LR-CV.
#   usage: gpurun --timeout 900 -- bash tools/gpu_lr_prof.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/lrprof_${1:-x}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for m in lr lrcv; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$m" -o r -- \
      python3 "$ROOT/tools/lr_probe.py" --model $m --fits 5 > "$OUT/probe_$m.txt" 2>&1)
  rc=$?
  head -4 "$OUT/probe_$m.txt"
  [ $rc -ne 0 ] && exit $rc
  python3 "$ROOT/tools/prof_summary.py" "$OUT/prof_$m/r_kernel_stats.csv" "lr_probe --model $m" | sed -n 6,16p | cut -c1-150
done
echo done
