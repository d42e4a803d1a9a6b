#!/bin/bash
# The reference's own workload (WISDM, Main/main.py flow) end to end on one MI355X,
# plus the deeper presets; artefacts land in gpurun_out/reference_run/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/reference_run"
mkdir -p "$OUT"
python tools/build_native.py > /dev/null || exit 3
DATA="${HAR_WISDM_CSV:-$ROOT/tests/data/wisdm_data.csv}"
for preset in reference rf-deep mlp all-numeric; do
  timeout -k 10 600 python main.py --preset $preset --data "$DATA" --device cuda \
      --out-dir "$OUT/$preset" --report ${EXTRA:-} > "$OUT/$preset.log" 2>&1
  rc=$?
  tail -1 "$OUT/$preset.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "preset $preset fatal $rc"; exit $rc; fi
done
