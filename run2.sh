set -e
mkdir -p gpurun_out/r7
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r7/pytest_gpu.log 2>&1
timeout -k 10 180 python bench.py --config rf > gpurun_out/r7/bench_rf.json 2> gpurun_out/r7/bench_rf.err
timeout -k 10 240 python bench.py --config rf9 > gpurun_out/r7/bench_rf9.json 2> gpurun_out/r7/bench_rf9.err
