#!/bin/bash
# Kernel-trace statistics of the flagship bench (driver command) and of the reference suite on the final
# round-6 build: rocprofv3 --kernel-trace --stats (no counters), summaries -> gpurun_out/trace6
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/trace6"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/mlp" -o t -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-wisdm > "$OUT/mlp.log" 2>&1
rc=$?; echo "mlp trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ref" -o t -- \
    python3 "$ROOT/bench.py" --config reference --steps 3 --warmup 1 > "$OUT/ref.log" 2>&1
rc=$?; echo "ref trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOT"
python3 tools/prof_summary.py "$OUT/mlp/t_kernel_stats.csv" "flagship bench (driver command) under rocprofv3" > "$OUT/mlp.md"
python3 tools/prof_summary.py "$OUT/ref/t_kernel_stats.csv" "reference suite bench under rocprofv3" > "$OUT/ref.md"
sed -n 1,16p "$OUT/mlp.md" | cut -c1-150
echo done
