#!/bin/bash
# One gpurun call: window tests + A/B probe, the config-4 1B-sample stream pass on one GPU, the
# stream / rf / rf9 benches, then the reference's main.py flow (tools/reference_run.sh).  Each GPU
# step has its own limit; a fault / abort / timeout (exit > 1) ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
step() {  # $1 = name, $2 = limit (s), rest = command
  local name=$1 lim=$2
  shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -3 "$OUT/$name.log" | cut -c1-400
  echo "STEP $name rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
}
step pytest_window 300 python -u -m pytest tests/test_window.py -m gpu -q -x --timeout 120 --timeout-method thread
step window_probe 200 python -u tools/window_probe.py
cat "$OUT/window_probe.log"
if [ "${WINDOW_ONLY:-0}" = "1" ]; then exit 0; fi
step bench_stream_1b 400 python -u bench.py --config stream --stream-pass --samples-per-gpu 1000000000 --steps 3 --warmup 1 \
    --out "$OUT/bench_stream_1b.json"
step bench_stream 300 python -u bench.py --config stream --steps 50 --warmup 10 --out "$OUT/bench_stream.json"
step bench_rf 300 python -u bench.py --config rf --steps 5 --warmup 2 --out "$OUT/bench_rf.json"
step bench_rf9 300 python -u bench.py --config rf9 --steps 5 --warmup 2 --out "$OUT/bench_rf9.json"
step reference_run 900 bash tools/reference_run.sh
echo done
