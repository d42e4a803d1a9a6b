#!/bin/bash
# Quick MLP A/B: three plain bench runs + one rocprofv3 kernel-stats run of the B=65536 step.
#   usage: gpurun --timeout 600 -- bash tools/gpu_mlp_quick.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/mlpq_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
for i in 1 2 3; do
  timeout -k 10 180 python bench.py --no-wisdm --steps 200 --warmup 20 --out "$OUT/bench_$i.json" > "$OUT/bench_$i.log" 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/bench_$i.json'));print('run $i ms/step', d['ms_per_step'])"
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o b -- \
  python3 "$ROOT/bench.py" --no-wisdm --steps 20 --warmup 2 --graph 0 > "$OUT/prof.log" 2>&1 || exit $?
python3 "$ROOT/tools/prof_summary.py" "$OUT/prof/b_kernel_stats.csv" 2>/dev/null | head -12 || true
