#!/bin/bash
# Round-6 MLP iteration: the step's GPU tests, the per-kernel probe, the driver's bench command twice.
#   usage: gpurun --timeout 900 -- bash tools/sessions/gpu_r6_mlp.sh <tag> [pytest -k expr] [stamps]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/r6mlp_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "STEP $2 failed: status $1"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_rccl.py -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "${2:-mlp or step or frag or rccl}" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; fatal $rc pytest
timeout -k 10 200 python -u tools/mlp_phase_probe.py 65536 > "$OUT/probe.txt" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/probe.txt"; fatal $rc probe
if [ "${3:-}" = "stamps" ]; then
  timeout -k 10 200 python -u tools/mlp_phase_probe.py --stamps > "$OUT/stamps.txt" 2>&1
  rc=$?; grep -E -- "---|prologue|tile 4|epilogue|total|real" "$OUT/stamps.txt"; fatal $rc stamps
fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
  rc=$?; python -c "import json,sys; r=json.loads(open('$OUT/bench_$i.json').read().strip().splitlines()[-1]); print('bench', r['ms_per_step'], {k: round(v['fit_s']*1e3,3) for k,v in r.get('reference_suite',{}).get('models',{}).items()})"; fatal $rc bench
done
echo done
