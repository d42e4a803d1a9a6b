#!/bin/bash
# Round-6 session e: MLP step tests + stamps + bench, window oracle tests (large counts), kfold test.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
mkdir -p gpurun_out/r6e
timeout -k 10 400 python -u -m pytest tests/test_window.py tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu -k "window or kfold" > gpurun_out/r6e/pytest_window.log 2>&1; rc=$?; tail -3 gpurun_out/r6e/pytest_window.log; [ $rc -ne 0 ] && exit $rc
bash tools/sessions/gpu_r6_mlp.sh e "mlp or step or frag or rccl" stamps
