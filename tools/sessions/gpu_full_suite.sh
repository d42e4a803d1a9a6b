#!/bin/bash
# The whole GPU test suite in one process (as the driver runs it at round end).
#   usage: gpurun --timeout 1200 -- bash tools/gpu_full_suite.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/full_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.txt" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest.txt" | tail -3
exit $rc
