set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python tools/build_native.py > gpurun_out/build.log 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for g in 0 1 2; do timeout -k 10 200 python bench.py --steps 200 --warmup 10 --graph $g > gpurun_out/bench_graph$g.json; tail -1 gpurun_out/bench_graph$g.json | cut -c150-260; done
