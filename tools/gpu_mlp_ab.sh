#!/bin/bash
# MLP iteration: MLP GPU tests, then the flagship bench with the h1 recompute on / off (A/B).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
python tools/build_native.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "mlp or MLP or determin or fault or graph" > gpurun_out/pytest_mlp.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_mlp.log; [ $rc -ne 0 ] && exit $rc
for rh in 1 0 1 0; do
  HAR_MLP_RECOMPUTE_H1=$rh timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-wisdm \
      --out gpurun_out/bench_mlp_rh$rh.json > gpurun_out/bench_mlp_rh$rh.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_mlp_rh$rh.log; exit $rc; }
  python -c "import json;r=json.load(open('gpurun_out/bench_mlp_rh$rh.json'));print('recompute_h1=$rh', round(r['ms_per_step'],4), r['synthetic_test_accuracy'])"
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_mlp_rh" \
    -o b -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 2 --no-wisdm > "$GRAFT_REPO_ROOT/gpurun_out/prof_mlp_rh.log" 2>&1
echo "prof rc=$?"
