set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
python tools/build_native.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread tests/test_gpu_models.py -k "mlp" > gpurun_out/pytest_mlp.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/pytest_mlp.log | tail -15; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-wisdm --out gpurun_out/bench_mlp.json > gpurun_out/bench.log 2>&1
rc=$?; tail -c 700 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_mlp2" -o b -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 2 --no-wisdm > "$GRAFT_REPO_ROOT/gpurun_out/prof_mlp2.log" 2>&1
echo "prof rc=$?"
