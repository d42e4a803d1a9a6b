#!/bin/bash
# grad_reduce_adam waves per workgroup (HAR_GR_W 4 / 8 / 16) at the small-batch and flagship batches.
#   usage: gpurun --timeout 600 -- bash tools/gpu_grw_ab.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/grw_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
for w in 16 8 4; do
  HAR_GR_W=$w timeout -k 10 200 python tools/mlp_phase_probe.py 65536 256 512 > "$OUT/w$w.txt" 2>&1 || exit 1
  echo "GR_W=$w"; grep -v amdgpu.ids "$OUT/w$w.txt"
done
