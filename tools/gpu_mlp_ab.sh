#!/bin/bash
# MLP backward scheduling A/B + window kernel check on one gpurun call.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/mlpab_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_window.py -m gpu -q -x \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for v in ${VARIANTS:-0 1 2 3}; do
  HAR_BWD_VARIANT=$v timeout -k 10 200 python -u tools/mlp_phase_probe.py 65536 > "$OUT/probe_$v.txt" 2>&1
  rc=$?; echo "variant $v"; cat "$OUT/probe_$v.txt"; [ $rc -ne 0 ] && exit $rc
  HAR_BWD_VARIANT=$v timeout -k 10 200 python -u tools/mlp_phase_probe.py --stamps > "$OUT/stamps_$v.txt" 2>&1
  rc=$?; cat "$OUT/stamps_$v.txt"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 200 python -u tools/window_probe.py > "$OUT/window_probe.txt" 2>&1
rc=$?; cat "$OUT/window_probe.txt"; [ $rc -ne 0 ] && exit $rc
echo done
