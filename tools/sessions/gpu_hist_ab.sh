#!/bin/bash
# A/B of the forest histogram accumulation (uint32 vs fp32 LDS atomics) on rf / rf9, after the tree tests.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
python tools/build_native.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread \
    -k "forest or tree or level or subtraction or hist" > gpurun_out/pytest_tree.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_tree.log; [ $rc -ne 0 ] && exit $rc
for fa in 0 1; do
  for cfg in rf rf9; do
    HAR_HIST_FLOAT_ATOMICS=$fa timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 \
        --out gpurun_out/bench_${cfg}_fa$fa.json > gpurun_out/bench_${cfg}_fa$fa.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_${cfg}_fa$fa.log; exit $rc; }
    python -c "import json;r=json.load(open('gpurun_out/bench_${cfg}_fa$fa.json'));print('$cfg float_atomics=$fa', round(r['ms_per_step'],3), r['test_accuracy'])"
  done
done
