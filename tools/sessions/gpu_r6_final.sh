#!/bin/bash
# Round-6 record run on one MI355X: the whole GPU test suite (one process, as the driver runs it), smoke(),
# then every bench config the docs quote (driver command first), the window probe.
#   usage: gpurun --timeout 1200 -- bash tools/sessions/gpu_r6_final.sh <tag> [skip-tests]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/r6f_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.txt" 2>&1
  rc=$?; grep -E "passed|failed|error" "$OUT/pytest.txt" | tail -3; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1
  rc=$?; tail -1 "$OUT/smoke.txt"; [ $rc -ne 0 ] && exit $rc
fi
b() {  # $1 = tag, rest = bench args
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --out "$OUT/bench_$tag.json" > "$OUT/bench_$tag.log" 2>&1
  local rc=$?
  python3 -c "import json;d=json.load(open('$OUT/bench_$tag.json'));print('$tag', 'ms', round(d['ms_per_step'],5), 'value %.4g' % d['value'], 'acc', d.get('test_accuracy', d.get('synthetic_test_accuracy')))" || tail -5 "$OUT/bench_$tag.log"
  return $rc
}
b driver --gpus 1 --steps 20 --warmup 5 || exit $?
b reference --config reference --steps 5 --warmup 2 || exit $?
python3 - "$OUT/bench_reference.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.get("models", d.get("reference_suite", {}).get("models", {})).items():
    print(" ", k, {x: v.get(x) for x in ("fit_s", "first_fit_s", "accuracy")})
PY
b stream_1b --config stream --stream-pass --samples-per-gpu 1000000000 --steps 3 --warmup 1 --no-wisdm || exit $?
b driver2 --gpus 1 --steps 20 --warmup 5 || exit $?
HAR_WINDOW_AB=0 timeout -k 10 200 python -u tools/window_probe.py > "$OUT/window.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/window.txt"
echo done
