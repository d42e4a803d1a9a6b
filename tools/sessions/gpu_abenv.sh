#!/bin/bash
# Env-variant A/B/... of the driver's bench command on ONE box, interleaved over ROUNDS rounds:
#   VARS="A=1;A=2 B=3" gpurun -- bash tools/gpu_abenv.sh <tag> [rounds]
# (a variant of "-" = the defaults; HAR_NATIVE_SO=<path> in a variant selects another build)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/abenv_$1"
mkdir -p "$OUT"
cd "$ROOT"
IFS=';' read -r -a vars <<< "${VARS:--}"
for r in $(seq 1 "${2:-3}"); do
  i=0
  for v in "${vars[@]}"; do
    [ "$v" = "-" ] && v=""
    env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-wisdm > "$OUT/v${i}_$r.json" 2> "$OUT/v${i}_$r.err"
    rc=$?; [ $rc -ne 0 ] && { echo "bench [$v] $r failed: $rc"; tail -3 "$OUT/v${i}_$r.err"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '|', sys.argv[3], round(d['ms_per_step'],5))" "$OUT/v${i}_$r.json" "$r" "$v"
    i=$((i + 1))
  done
done
echo done
