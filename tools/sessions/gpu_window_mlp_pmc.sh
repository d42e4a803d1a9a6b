#!/bin/bash
# One gpurun call: window kernel tests + A/B timing (v3 register kernel vs legacy), then the MLP
# step's PMC passes (tools/pmc_groups_step.txt).  Each GPU step has its own limit; a fault, abort
# or timeout ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_window.py -m gpu -q -x --timeout 120 --timeout-method thread \
    > "$OUT/pytest_window.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_window.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/window_probe.py > "$OUT/window_probe.txt" 2>&1
rc=$?; cat "$OUT/window_probe.txt"
[ $rc -ne 0 ] && exit $rc
if [ "${SKIP_PMC:-0}" = "0" ]; then
  PMC_GROUPS="$ROOT/tools/pmc_groups_step.txt" BENCH_ARGS="--no-wisdm --graph 0" bash tools/pmc_session.sh
  rc=$?
  [ $rc -ne 0 ] && exit $rc
fi
echo done
