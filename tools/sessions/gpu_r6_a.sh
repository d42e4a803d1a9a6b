#!/bin/bash
# Round-6 session a: RCCL tests on the forced 1-rank group, the driver bench, a rocprofv3 kernel trace of
# the reference suite's tree fits.   usage: gpurun --timeout 900 -- bash tools/sessions/gpu_r6_a.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/r6a_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_rccl.log" 2>&1
rc=$?; tail -15 "$OUT/pytest_rccl.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; tail -c 600 "$OUT/bench.json"; echo; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ref_tree_probe.py > "$OUT/tree_probe.txt" 2>&1
rc=$?; cat "$OUT/tree_probe.txt" | grep model; [ $rc -ne 0 ] && exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tree_trace" -o tree -- \
    python3 "$ROOT/tools/ref_tree_probe.py" --repeats 3 > "$OUT/tree_trace.log" 2>&1)
rc=$?; grep model "$OUT/tree_trace.log"; [ $rc -ne 0 ] && exit $rc
echo done
