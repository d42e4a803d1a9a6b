#!/bin/bash
# Window featurizer: GPU tests + A/B timing probe (v3 vs legacy kernels).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; mkdir -p gpurun_out/winq
timeout -k 10 300 python -u -m pytest tests/test_window.py tests/test_raw.py -m gpu -q -x --timeout 120 --timeout-method thread \
    > gpurun_out/winq/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/winq/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/window_probe.py > gpurun_out/winq/probe.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/winq/probe.txt; exit $rc
