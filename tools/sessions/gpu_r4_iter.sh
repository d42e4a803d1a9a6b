#!/bin/bash
# Round-4 quick iteration: MLP step tests + probe + stamps, window tests + probe.
#   usage: gpurun --timeout 900 -- bash tools/gpu_r4_iter.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/it_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ] && [ "$1" -ne 5 ]; then echo "STEP $2 fatal status $1"; exit "$1"; fi; }
timeout -k 10 400 python -u -m pytest tests -m gpu -k "${2:-mlp_step or frag or fused or window}" -x -q --timeout 200 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; fatal $rc pytest
timeout -k 10 200 python -u tools/mlp_phase_probe.py 65536 256 > "$OUT/probe.txt" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/probe.txt"; fatal $rc probe
timeout -k 10 200 python -u tools/mlp_phase_probe.py --stamps > "$OUT/stamps.txt" 2>&1
rc=$?; grep -E -- "---|tile 4|total" "$OUT/stamps.txt"; fatal $rc stamps
HAR_WINDOW_AB=0 timeout -k 10 200 python -u tools/window_probe.py > "$OUT/window.txt" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/window.txt"; fatal $rc window
echo done
