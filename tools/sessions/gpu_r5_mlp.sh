#!/bin/bash
# Round-5 MLP iteration: step / fragment tests, per-kernel probe of env variants (VARS),
# stamps, driver-command bench.
#   usage: gpurun --timeout 900 -- bash tools/gpu_r5_mlp.sh <tag> [pytest -k expr]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r5mlp_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ] && [ "$1" -ne 5 ]; then echo "STEP $2 fatal status $1"; exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests -m gpu -k "${2:-mlp or frag or fused or infer}" -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; fatal $rc pytest
# probe variants: VARS="A=1 B=2;C=3" (';'-separated env sets; default: the built-in settings)
IFS=';' read -r -a vars <<< "${VARS:-HAR_MLP_FWD_STAGGER=0}"
i=0
for v in "${vars[@]}"; do
  env $v timeout -k 10 200 python -u tools/mlp_phase_probe.py 65536 > "$OUT/probe_v$i.txt" 2>&1
  rc=$?; echo "variant $i: $v"; grep -v amdgpu.ids "$OUT/probe_v$i.txt"; fatal $rc probe
  i=$((i + 1))
done
timeout -k 10 200 python -u tools/mlp_phase_probe.py --stamps > "$OUT/stamps.txt" 2>&1
rc=$?; grep -E -- "---|prologue|tile 4|total|real" "$OUT/stamps.txt"; fatal $rc stamps
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
  rc=$?; tail -c 400 "$OUT/bench_$i.json"; echo; fatal $rc bench
done
echo done
