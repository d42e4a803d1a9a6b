#!/bin/bash
# Config-4 1B-sample full pass: bench record + a rocprofv3 kernel trace of the same run (where the pass's
# time goes outside the MLP steps).  -> gpurun_out/stream_<tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/stream_${1:-x}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 400 python -u bench.py --config stream --stream-pass --samples-per-gpu 1000000000 --steps 3 --warmup 1 \
    --no-wisdm --out "$OUT/bench_stream_1b.json" > "$OUT/bench.log" 2>&1
rc=$?; python3 -c "import json;d=json.load(open('$OUT/bench_stream_1b.json'));print('pass ms', d['ms_per_step'], 'steps', d.get('mlp_steps_per_pass'), 'acc', d.get('test_accuracy'))" || tail -5 "$OUT/bench.log"
[ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- \
    python3 "$ROOT/bench.py" --config stream --stream-pass --samples-per-gpu 1000000000 --steps 2 --warmup 1 --no-wisdm \
    > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 "$ROOT/tools/prof_summary.py" "$OUT/trace/t_kernel_stats.csv" "stream 1B pass" | sed -n 1,22p | cut -c1-160
echo done
