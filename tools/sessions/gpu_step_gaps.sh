#!/bin/bash
# Kernel trace of the driver's bench command (5 warm-up + 20 timed steps): where the window's fixed
# cost over the steady-state step goes (tools/step_gap_trace.py).
#   usage: gpurun --timeout 600 -- bash tools/gpu_step_gaps.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/gaps_${1:-x}"
mkdir -p "$OUT"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o r -- \
    python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --out "$OUT/bench.json" > "$OUT/bench.log" 2>&1) || exit 1
python3 "$ROOT/tools/step_gap_trace.py" "$OUT/prof/r_kernel_trace.csv" 25 > "$OUT/gaps.txt"
tail -30 "$OUT/gaps.txt"
