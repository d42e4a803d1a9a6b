#!/bin/bash
# Short vs long bench runs: where does the driver's 20-step window lose time against 200 steps?
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; mkdir -p gpurun_out/short
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "mlp" --timeout 120 \
    --timeout-method thread > gpurun_out/short/pytest.log 2>&1 || { tail -5 gpurun_out/short/pytest.log; exit 1; }
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --out gpurun_out/short/$tag.json > gpurun_out/short/$tag.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('gpurun_out/short/$tag.json'));print('$tag', round(d['ms_per_step'],5))"
}
run drv_a --gpus 1 --steps 20 --warmup 5
run drv_nowisdm --gpus 1 --steps 20 --warmup 5 --no-wisdm
run s20_w50 --gpus 1 --steps 20 --warmup 50 --no-wisdm
run s200_w5 --gpus 1 --steps 200 --warmup 5 --no-wisdm
run s200_w20 --gpus 1 --steps 200 --warmup 20 --no-wisdm
