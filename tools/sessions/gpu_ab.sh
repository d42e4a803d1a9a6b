#!/bin/bash
# A/B of native builds on ONE box: the driver's bench command alternated between the in-tree build
# (A) and ab/<name>/_har_native.so (B), ROUNDS times each; ms_per_step lines -> gpurun_out/ab_<tag>/.
#   usage: gpurun -- bash tools/gpu_ab.sh <tag> <name> [rounds]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/ab_$1"
mkdir -p "$OUT"
cd "$ROOT"
for r in $(seq 1 "${3:-3}"); do
  for v in A B; do
    if [ $v = A ]; then so=""; else so="$ROOT/ab/$2/_har_native.so"; fi
    HAR_NATIVE_SO="$so" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-wisdm > "$OUT/${v}_$r.json" 2> "$OUT/${v}_$r.err"
    rc=$?; [ $rc -ne 0 ] && { echo "bench $v $r failed: $rc"; tail -3 "$OUT/${v}_$r.err"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],5), round(d['phase_ms']['compute'],5))" "$OUT/${v}_$r.json" $v $r
  done
done
echo done
