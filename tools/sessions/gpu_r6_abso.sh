#!/bin/bash
# Round-6 same-box A/B of two native builds: GPU tests of the in-tree build (A), then the per-kernel probe
# and the driver's bench command alternated between A and ab/<name>/_har_native.so (B).
#   usage: gpurun -- bash tools/sessions/gpu_r6_abso.sh <tag> <name> [rounds] [pytest -k expr]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/abso_$1"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_rccl.py -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "${4:-mlp or step or frag or rccl}" > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for r in $(seq 1 "${3:-3}"); do
  for v in A B; do
    if [ $v = A ]; then so=""; else so="$ROOT/ab/$2/_har_native.so"; fi
    HAR_NATIVE_SO="$so" timeout -k 10 200 python -u tools/mlp_phase_probe.py 65536 > "$OUT/probe_${v}_$r.txt" 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 "$OUT/probe_${v}_$r.txt"; exit $rc; }
    HAR_NATIVE_SO="$so" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-wisdm > "$OUT/${v}_$r.json" 2> "$OUT/${v}_$r.err"
    rc=$?; [ $rc -ne 0 ] && { echo "bench $v $r failed: $rc"; tail -3 "$OUT/${v}_$r.err"; exit $rc; }
    echo "$v $r probe: $(grep -E '^ +65536' "$OUT/probe_${v}_$r.txt") bench: $(python3 -c "import json,sys; print(round(json.load(open(sys.argv[1]))['ms_per_step'], 5))" "$OUT/${v}_$r.json")"
  done
done
echo done
