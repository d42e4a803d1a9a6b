#!/bin/bash
# Persistent LR solve: the GPU LR tests (bitwise equality with the launch sequence among them), then the
# reference-suite LR / LR-CV fit times with the persistent solve on (default) and off, and a kernel trace.
#   usage: gpurun --timeout 900 -- bash tools/gpu_lr_persist.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/lrpersist_${1:-x}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_logreg.py -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest.txt" 2>&1
rc=$?
tail -25 "$OUT/pytest.txt"
[ $rc -ne 0 ] && exit $rc
for mode in 1 0; do
  HAR_LR_PERSISTENT=$mode timeout -k 10 200 python tools/lr_probe.py --model lr --fits 5 > "$OUT/probe_lr_$mode.txt" 2>&1 || exit 1
  echo "persistent=$mode"; head -4 "$OUT/probe_lr_$mode.txt"
done
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o r -- \
    python3 "$ROOT/tools/lr_probe.py" --model lr --fits 5 > "$OUT/probe_prof.txt" 2>&1) || exit 1
python3 tools/prof_summary.py "$OUT/prof/r_kernel_stats.csv" "lr_probe persistent" | sed -n 6,16p | cut -c1-150
