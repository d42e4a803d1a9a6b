#!/bin/bash
# The whole GPU test suite (device DP tests with gloo ranks sharing the GPU included) + smoke.
#   usage: gpurun --timeout 1200 -- bash tools/gpu_dp_tests.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/suite_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.txt" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.txt" | tail -15
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1
  echo "smoke rc=$?"; tail -3 "$OUT/smoke.txt"
fi
exit $rc
