#!/bin/bash
# MLP kernel tests + the phase probe (flagship and small batch).
#   usage: gpurun --timeout 600 -- bash tools/gpu_mlp_quick2.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/mq2_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_distributed.py -x -q \
    --timeout 120 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 200 python tools/mlp_phase_probe.py 65536 256 > "$OUT/probe.txt" 2>&1 || exit 1
grep -v amdgpu.ids "$OUT/probe.txt"
