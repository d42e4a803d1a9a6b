#!/bin/bash
# Forest iteration on one MI355X: tree GPU tests -> rf / rf9 / dt (subtraction on / off) benches ->
# rocprofv3 kernel trace of the rf bench (per-fit busy vs idle from tools/fit_breakdown.py).
#   usage: gpurun --timeout 900 -- bash tools/gpu_forest.sh
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
python tools/build_native.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py -x -v --timeout 120 --timeout-method thread \
    -k "forest or tree or level or subtraction or subsets or graph" > gpurun_out/pytest_tree.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_tree.log | tail -40; [ $rc -ne 0 ] && exit $rc
for run in "rf" "rf9" "dt" "dt --no-subtract"; do
  tag=$(echo "$run" | tr -d ' -')
  timeout -k 10 300 python bench.py --config $run --steps 5 --warmup 2 --out gpurun_out/bench_$tag.json \
      > gpurun_out/bench_$tag.log 2>&1
  rc=$?; tail -c 300 gpurun_out/bench_$tag.log; echo; [ $rc -ne 0 ] && exit $rc
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_rf" \
    -o b -- python3 "$GRAFT_REPO_ROOT/bench.py" --config rf --steps 5 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof_rf.log" 2>&1
rc=$?; echo "prof rf rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python "$GRAFT_REPO_ROOT/tools/forest_host_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/probe_rf.log" 2>&1; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/probe_rf.log"
cd "$GRAFT_REPO_ROOT" && python tools/fit_breakdown.py gpurun_out/prof_rf/b_kernel_trace.csv 6 20 | tee gpurun_out/rf_fit_levels.txt
