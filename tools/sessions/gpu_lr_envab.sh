#!/bin/bash
# LR env A/B on one box: the device-LR GPU tests once, then the reference suite bench and the grad
# kernel's phase stamps under each env assignment of VARS (';'-separated, e.g. "HAR_LR_COLBLK=0;HAR_LR_COLBLK=1").
#   usage: VARS="A=1;A=0" gpurun --timeout 900 -- bash tools/gpu_lr_envab.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/lrenv_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -m pytest tests/test_gpu_logreg.py tests/test_gpu_models.py tests/test_gpu_distributed.py tests/test_wolfe.py -m gpu \
    --timeout 120 --timeout-method thread -q -x -k "logreg or lr or LogisticRegression or crossval or cv or wolfe" > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && [ $rc -ne 5 ] && exit $rc
IFS=';' read -ra VS <<< "${VARS:-X=0}"
i=0
for v in "${VS[@]}"; do
  env $v timeout -k 10 300 python bench.py --config reference --steps 5 --warmup 1 \
      --out "$OUT/bench_$i.json" > "$OUT/bench_$i.log" 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/bench_$i.json'))['reference_suite']['models'];print('$v', {k:(round(v['fit_s']*1e3,3),round(v['accuracy'],4)) for k,v in d.items() if k in ('lr','lrcv','LR','LR-CV') or 'lr' in k.lower()})"
  env $v timeout -k 10 200 python tools/lr_stamps.py --model lr > "$OUT/stamps_$i.txt" 2>&1 || exit $?
  grep -E -- "^---|entry -> last|finalize|pass B|one-hot slices|element sweep" "$OUT/stamps_$i.txt" || true
  i=$((i+1))
done
echo done
