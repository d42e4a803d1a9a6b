#!/bin/bash
# LR A/B: the device-LR GPU tests once, then the reference suite bench under each HAR_QN_WORKGROUPS
# budget given (default: 512 768 1024).
#   usage: gpurun --timeout 900 -- bash tools/gpu_lr_ab.sh <tag> [budgets...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/lrab_${1:-x}"
shift || true
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -m pytest tests/test_gpu_logreg.py tests/test_gpu_models.py tests/test_gpu_distributed.py -m gpu \
    --timeout 120 --timeout-method thread -q -x -k "logreg or lr or LogisticRegression or crossval or cv" > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && [ $rc -ne 5 ] && exit $rc
for wg in ${@:-512 768 1024}; do
  HAR_QN_WORKGROUPS=$wg timeout -k 10 300 python bench.py --config reference --steps 5 --warmup 1 \
      --out "$OUT/bench_reference_$wg.json" > "$OUT/bench_$wg.log" 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/bench_reference_$wg.json'))['reference_suite']['models'];print('wg $wg', {k:(round(v['fit_s']*1e3,2),round(v['first_fit_s']*1e3,2),round(v['accuracy'],4)) for k,v in d.items()})"
done
