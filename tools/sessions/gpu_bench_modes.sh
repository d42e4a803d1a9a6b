#!/bin/bash
# The driver's bench command (N = 1, 20 steps after 5 warm-up) twice, then a long eager run.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; mkdir -p gpurun_out/drv
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/drv/drv_$i.json > gpurun_out/drv/drv_$i.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('gpurun_out/drv/drv_$i.json'));print('driver-style', d['ms_per_step'], d['hip_graph'], d.get('test_accuracy'))"
done
timeout -k 10 200 python bench.py --no-wisdm --steps 200 --warmup 20 --out gpurun_out/drv/long.json > gpurun_out/drv/long.log 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/drv/long.json'));print('long eager', d['ms_per_step'])"
