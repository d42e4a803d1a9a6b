#!/bin/bash
# LR solver cache: the GPU LR tests, then the reference-suite LR and LR-CV fit times (tools/lr_probe.py).
#   usage: gpurun --timeout 600 -- bash tools/gpu_lr_cache.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/lrcache_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_logreg.py -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest.txt" 2>&1
rc=$?
tail -6 "$OUT/pytest.txt"
[ $rc -ne 0 ] && exit $rc
for m in lr lrcv; do
  timeout -k 10 200 python tools/lr_probe.py --model $m --fits 5 > "$OUT/probe_$m.txt" 2>&1 || exit 1
  echo "$m"; sed -n 2,5p "$OUT/probe_$m.txt"
done
