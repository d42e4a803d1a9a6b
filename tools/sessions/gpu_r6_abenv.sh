#!/bin/bash
# Round-6 env A/B of the MLP step: the per-kernel probe under each VARS set (';'-separated env sets,
# "-" = none), interleaved over ROUNDS rounds, then the driver bench command per set.
#   usage: VARS="-;HAR_MLP_WT=1" gpurun -- bash tools/sessions/gpu_r6_abenv.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/r6ab_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
IFS=';' read -r -a vars <<< "${VARS:--}"
for r in $(seq 1 "${ROUNDS:-2}"); do
  i=0
  for v in "${vars[@]}"; do
    [ "$v" = "-" ] && v=""
    env $v timeout -k 10 200 python -u tools/mlp_phase_probe.py 65536 > "$OUT/probe_r${r}_v$i.txt" 2>&1
    rc=$?; echo "round $r variant $i [$v]: $(grep -E '^ +65536' "$OUT/probe_r${r}_v$i.txt")"
    [ $rc -ne 0 ] && { cat "$OUT/probe_r${r}_v$i.txt" | tail -5; exit $rc; }
    i=$((i + 1))
  done
done
i=0
for v in "${vars[@]}"; do
  [ "$v" = "-" ] && v=""
  env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-wisdm > "$OUT/bench_v$i.json" 2> "$OUT/bench_v$i.err"
  rc=$?; echo "bench variant $i [$v]: $(python -c "import json; print(json.loads(open('$OUT/bench_v$i.json').read().strip().splitlines()[-1])['ms_per_step'])")"
  [ $rc -ne 0 ] && exit $rc
  i=$((i + 1))
done
echo done
