set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6d
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_rccl.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "mlp or step or frag or rccl" > gpurun_out/r6d/pytest_default.log 2>&1; rc=$?; tail -2 gpurun_out/r6d/pytest_default.log; [ $rc -ne 0 ] && exit $rc
HAR_MLP_H1=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "mlp or step" > gpurun_out/r6d/pytest_h1.log 2>&1; rc=$?; tail -2 gpurun_out/r6d/pytest_h1.log; [ $rc -ne 0 ] && exit $rc
VARS="-;HAR_MLP_H1=1" ROUNDS=3 bash tools/sessions/gpu_r6_abenv.sh h1
