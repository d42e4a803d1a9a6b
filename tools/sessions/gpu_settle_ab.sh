#!/bin/bash
# Driver command (5 warm-up + 20 timed steps) with 0 / 100 / 300 / 1000 ms of untimed clock-settle
# steps before the warm-up (bench.py --settle-ms), two runs each, plus a 500-step steady-state run.
#   usage: gpurun --timeout 900 -- bash tools/gpu_settle_ab.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/settle_${1:-x}"
mkdir -p "$OUT"
for ms in 0 100 300 1000; do
  for i in 1 2; do
    timeout -k 10 200 python "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --settle-ms $ms \
        --out "$OUT/s${ms}_$i.json" > "$OUT/s${ms}_$i.log" 2>&1 || exit 1
    python -c "import json;d=json.load(open('$OUT/s${ms}_$i.json'));print('settle $ms', d['ms_per_step'], d['settle_ms'])"
  done
done
timeout -k 10 200 python "$ROOT/bench.py" --gpus 1 --steps 500 --warmup 20 --no-wisdm --out "$OUT/long.json" \
    > "$OUT/long.log" 2>&1 || exit 1
python -c "import json;d=json.load(open('$OUT/long.json'));print('w20 s500', d['ms_per_step'])"
