#!/bin/bash
# Same-box A/B of a window-kernel environment switch: tools/window_probe.py without and with "<VAR>=<value>".
#   usage: gpurun -- bash tools/sessions/gpu_r6_winenv.sh <tag> <VAR> <value> [rounds]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/winenv_$1"
mkdir -p "$OUT"
cd "$ROOT"
for r in $(seq 1 "${4:-2}"); do
  for v in off on; do
    if [ $v = on ]; then export "$2=$3"; else unset "$2"; fi
    HAR_WINDOW_AB=0 timeout -k 10 200 python -u tools/window_probe.py > "$OUT/probe_${v}_$r.txt" 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 "$OUT/probe_${v}_$r.txt"; exit $rc; }
    echo "== $v $r"; grep -v amdgpu.ids "$OUT/probe_${v}_$r.txt"
  done
done
echo done
