#!/bin/bash
# LR kernel A/B: rocprofv3 kernel traces of the reference suite under each HAR_QN_WORKGROUPS budget,
# summarized as per-kernel medians (tools/lr_kernel_medians.py).
#   usage: gpurun --timeout 900 -- bash tools/gpu_lr_kab.sh <tag> [budgets...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/lrkab_${1:-x}"
shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
for wg in ${@:-512 768}; do
  (cd /tmp && HAR_QN_WORKGROUPS=$wg timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_$wg" -o r -- \
      python3 "$ROOT/bench.py" --config reference --steps 3 --warmup 1 --out "$OUT/bench_$wg.json" > "$OUT/prof_$wg.log" 2>&1) || exit $?
  echo "== HAR_QN_WORKGROUPS=$wg"
  python3 "$ROOT/tools/lr_kernel_medians.py" "$OUT/prof_$wg/r_kernel_trace.csv"
done
