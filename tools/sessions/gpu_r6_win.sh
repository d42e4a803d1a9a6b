#!/bin/bash
# Round-6 window featurizer A/B: GPU window tests of the in-tree build (A), then tools/window_probe.py
# alternated between A and ab/<name>/_har_native.so (B) on the same box.
#   usage: gpurun -- bash tools/sessions/gpu_r6_win.sh <tag> <name> [rounds]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/win_$1"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_window.py tests/test_raw.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for r in $(seq 1 "${3:-2}"); do
  for v in A B; do
    if [ $v = A ]; then so=""; else so="$ROOT/ab/$2/_har_native.so"; fi
    HAR_WINDOW_AB=0 HAR_NATIVE_SO="$so" timeout -k 10 200 python -u tools/window_probe.py > "$OUT/probe_${v}_$r.txt" 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 "$OUT/probe_${v}_$r.txt"; exit $rc; }
    echo "== $v $r"; grep -v amdgpu.ids "$OUT/probe_${v}_$r.txt"
  done
done
echo done
