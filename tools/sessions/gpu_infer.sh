#!/bin/bash
# Serving path check: the MLP kernel tests, then bench --config infer (step INFER pipeline on / off).
#   usage: gpurun --timeout 600 -- bash tools/gpu_infer.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/infer_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 120 \
    --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -2 "$OUT/pytest.txt"
for on in 1 0; do
  HAR_MLP_STEP_INFER=$on timeout -k 10 200 python bench.py --config infer --steps 50 --warmup 10 \
      --out "$OUT/infer_$on.json" > "$OUT/infer_$on.log" 2>&1 || { tail -20 "$OUT/infer_$on.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/infer_$on.json'));print('step-infer=$on', 'ms', round(d['ms_per_step'],5), 'value %.4g' % d['value'], 'acc', d['test_accuracy'])"
done
