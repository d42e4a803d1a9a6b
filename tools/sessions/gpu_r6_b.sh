#!/bin/bash
# Round-6 session b: one-hot-aware tree path — its tests, the tree / forest GPU tests, the tree probe
# (reference suite DT / RF fit times) and a kernel trace of those fits.
#   usage: gpurun --timeout 900 -- bash tools/sessions/gpu_r6_b.sh <tag> [pytest -k expr]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/r6b_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tree_sparse.py -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_sparse.log" 2>&1
rc=$?; tail -15 "$OUT/pytest_sparse.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ref_tree_probe.py > "$OUT/tree_probe.txt" 2>&1
rc=$?; grep model "$OUT/tree_probe.txt"; [ $rc -ne 0 ] && exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tree_trace" -o tree -- \
    python3 "$ROOT/tools/ref_tree_probe.py" --repeats 3 > "$OUT/tree_trace.log" 2>&1)
rc=$?; grep model "$OUT/tree_trace.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    -k "${2:-tree or forest or distributed or crossval or cv}" > "$OUT/pytest_trees.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_trees.log"; [ $rc -ne 0 ] && exit $rc
echo done
