#!/bin/bash
# LR tests + host probe, then the stream benches.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
python tools/build_native.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_logreg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lr.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_lr.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/lr_probe.py --model lr > gpurun_out/lr_probe.log 2>&1 || exit 1
timeout -k 10 300 python tools/lr_probe.py --model lrcv --fits 3 > gpurun_out/lrcv_probe.log 2>&1 || exit 1
grep -h "fit 2\|mean of" gpurun_out/lr_probe.log gpurun_out/lrcv_probe.log
bash tools/gpu_stream.sh
