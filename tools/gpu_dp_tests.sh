#!/bin/bash
# Device DP tests (gloo ranks sharing the GPU) + the other multi-process GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dp.py \
  > gpurun_out/dp_tests.log 2>&1
rc=$?
tail -30 gpurun_out/dp_tests.log
exit $rc
