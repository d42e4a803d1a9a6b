#!/bin/bash
# Round-4 record run: every bench config on one MI355X (1 GPU), window probe, MLP probe.
#   usage: gpurun --timeout 1200 -- bash tools/gpu_r4_final.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r4f_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
b() {  # $1 = tag, rest = bench args
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --out "$OUT/bench_$tag.json" > "$OUT/bench_$tag.log" 2>&1
  local rc=$?
  python3 -c "import json;d=json.load(open('$OUT/bench_$tag.json'));print('$tag', 'ms', round(d['ms_per_step'],5), 'value %.4g' % d['value'], 'acc', d.get('test_accuracy', d.get('synthetic_test_accuracy')))" || tail -5 "$OUT/bench_$tag.log"
  return $rc
}
b driver --gpus 1 --steps 20 --warmup 5 || exit $?
b mlp500 --steps 500 --warmup 20 --no-wisdm || exit $?
b reference --config reference --steps 5 --warmup 2 || exit $?
python3 - "$OUT/bench_reference.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.get("models", d.get("reference_suite", {}).get("models", {})).items():
    print(" ", k, {x: v.get(x) for x in ("fit_s", "first_fit_s", "accuracy")})
PY
b rf --config rf --steps 5 --warmup 2 || exit $?
b rf9 --config rf9 --steps 5 --warmup 2 || exit $?
b stream --config stream --steps 50 --warmup 10 || exit $?
b stream_ov --config stream --steps 50 --warmup 10 --stream-overlap 1 || exit $?
b infer --config infer --steps 50 --warmup 10 || exit $?
HAR_WINDOW_AB=0 timeout -k 10 200 python -u tools/window_probe.py > "$OUT/window.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/window.txt"
echo done
