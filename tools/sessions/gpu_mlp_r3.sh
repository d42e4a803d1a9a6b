#!/bin/bash
# MLP step iteration on one gpurun call: the step's GPU tests, the per-kernel phase probe (graph-
# replayed kernel times + in-kernel stamps) and three plain bench runs.
#   usage: gpurun --timeout 900 -- bash tools/gpu_mlp_r3.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/mlp_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -k "mlp or step or fused" -q -x \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/mlp_phase_probe.py 65536 > "$OUT/probe.txt" 2>&1
rc=$?; cat "$OUT/probe.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/mlp_phase_probe.py --stamps > "$OUT/stamps.txt" 2>&1
rc=$?; cat "$OUT/stamps.txt"; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 180 python bench.py --no-wisdm --steps 200 --warmup 20 --out "$OUT/bench_$i.json" > "$OUT/bench_$i.log" 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/bench_$i.json'));print('run $i ms/step', d['ms_per_step'], 'acc', d['synthetic_test_accuracy'])"
done
echo done
