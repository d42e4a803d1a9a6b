#!/bin/bash
# One gpurun call: MLP scheduling-variant A/B (probe only), the N = 1 bench in the three graph
# modes, and the LogisticRegression fit profile (tools/gpu_lr_prof.sh).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r3c_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "variants or mlp_step" \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for v in 0 1 2 3; do
  HAR_BWD_VARIANT=$v timeout -k 10 200 python -u tools/mlp_phase_probe.py 65536 > "$OUT/probe_$v.txt" 2>&1
  rc=$?; echo "variant $v: $(grep 65536 "$OUT/probe_$v.txt")"; [ $rc -ne 0 ] && exit $rc
done
for gm in 0 1 2; do
  timeout -k 10 200 python bench.py --no-wisdm --steps 200 --warmup 20 --graph $gm --out "$OUT/bench_graph$gm.json" \
      > "$OUT/bench_graph$gm.log" 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/bench_graph$gm.json'));print('graph $gm ms/step', round(d['ms_per_step'],5), d['hip_graph'], d['phase_ms'])"
done
bash tools/gpu_lr_prof.sh "${1:-x}"
