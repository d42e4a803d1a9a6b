#!/bin/bash
# LR quick check: device-LR GPU tests, the reference suite bench, and its kernel stats.
#   usage: gpurun --timeout 900 -- bash tools/gpu_lr_quick.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/lrq_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -m pytest tests/test_gpu_logreg.py tests/test_gpu_models.py tests/test_gpu_distributed.py -m gpu --timeout 120 --timeout-method thread -q -x -k "logreg or lr or LogisticRegression or crossval or cv" > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && [ $rc -ne 5 ] && exit $rc
timeout -k 10 300 python bench.py --config reference --steps 3 --warmup 1 --out "$OUT/bench_reference.json" > "$OUT/bench.log" 2>&1 || exit $?
python -c "import json;d=json.load(open('$OUT/bench_reference.json'))['reference_suite']['models'];print({k:(round(v['fit_s']*1e3,2),round(v['accuracy'],4)) for k,v in d.items()})"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o r -- \
  python3 "$ROOT/bench.py" --config reference --steps 3 --warmup 1 > "$OUT/prof.log" 2>&1 || exit $?
python3 "$ROOT/tools/prof_summary.py" "$OUT/prof/r_kernel_stats.csv" "reference suite" | sed -n 6,14p | cut -c1-150
