#!/bin/bash
# LR-CV fit time vs the L-BFGS workgroup budget (HAR_QN_WORKGROUPS: chunks per model = budget / models,
# capped at 32) and the grad-reduce waves per workgroup (HAR_GR_W) at the small / flagship batches.
#   usage: gpurun --timeout 900 -- bash tools/gpu_qnwg_ab.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/qnwg_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_logreg.py -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -2 "$OUT/pytest.txt"
timeout -k 10 200 python tools/lr_probe.py --model lr --fits 5 > "$OUT/lr.txt" 2>&1 || exit 1
echo "LR $(grep 'mean of' "$OUT/lr.txt")"
for wg in 512 1024 2048 4096; do
  HAR_QN_WORKGROUPS=$wg timeout -k 10 200 python tools/lr_probe.py --model lrcv --fits 5 > "$OUT/lrcv_$wg.txt" 2>&1 || exit 1
  echo "QN_WORKGROUPS=$wg $(grep 'mean of' "$OUT/lrcv_$wg.txt")"
done
for w in 16 8 4; do
  HAR_GR_W=$w timeout -k 10 200 python tools/mlp_phase_probe.py 65536 256 512 > "$OUT/grw$w.txt" 2>&1 || exit 1
  echo "GR_W=$w"; grep -v amdgpu.ids "$OUT/grw$w.txt"
done
