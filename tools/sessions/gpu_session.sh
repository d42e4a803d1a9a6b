#!/bin/bash
# One gpurun session: GPU tests -> benches -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fault / abort / timeout ends the script
# (exit codes 124, 134, 137, 139 or >128), plain test failures (exit 1) do not.
#   usage: gpurun --timeout 1200 -- bash tools/gpu_session.sh [tests|bench|ref|benchall|prof|all] [pytest args]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
WHAT="${1:-all}"
shift || true

fatal() {  # $1 = exit code, $2 = step
  local rc=$1
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ] && [ "$rc" -ne 5 ]; then
    echo "STEP $2 ended with fatal status $rc — stopping" | tee -a "$OUT/session.log"
    exit "$rc"
  fi
}

echo "== session $WHAT $(date)" | tee -a "$OUT/session.log"
python tools/build_native.py > "$OUT/build.log" 2>&1 || { echo "build failed"; cat "$OUT/build.log"; exit 3; }

if [ "$WHAT" = "tests" ] || [ "$WHAT" = "all" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x "$@" > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  tail -25 "$OUT/pytest_gpu.log"
  fatal $rc pytest
fi

if [ "$WHAT" = "bench" ] || [ "$WHAT" = "all" ] || [ "$WHAT" = "benchall" ]; then
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 --out "$OUT/bench_mlp.json" > "$OUT/bench.log" 2>&1
  rc=$?
  tail -2 "$OUT/bench.log"
  fatal $rc bench
fi

if [ "$WHAT" = "ref" ] || [ "$WHAT" = "bench" ] || [ "$WHAT" = "all" ] || [ "$WHAT" = "benchall" ]; then
  timeout -k 10 300 python bench.py --config reference --steps 5 --warmup 2 --out "$OUT/bench_reference.json" \
      > "$OUT/bench_reference.log" 2>&1
  rc=$?
  tail -c 600 "$OUT/bench_reference.log"
  fatal $rc bench_reference
fi

if [ "$WHAT" = "benchall" ]; then
  for cfg in rf stream rf9; do
    # the stream config trains while it times: 60 steps, as in its recorded accuracy
    if [ "$cfg" = "stream" ]; then st=50; wu=10; else st=5; wu=2; fi  # forests: fit graph captured on the 2nd fit
    timeout -k 10 400 python bench.py --config $cfg --steps $st --warmup $wu --out "$OUT/bench_$cfg.json" \
        > "$OUT/bench_$cfg.log" 2>&1
    rc=$?
    tail -2 "$OUT/bench_$cfg.log"
    fatal $rc "bench_$cfg"
  done
fi

if [ "$WHAT" = "prof" ] || [ "$WHAT" = "all" ]; then
  export TMPDIR=/tmp
  PCFG="${PROF_CONFIG:-mlp}"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$PCFG" -o bench -- \
      python3 "$ROOT/bench.py" --config "$PCFG" --steps "${PROF_STEPS:-20}" --warmup 2 --graph 0 > "$OUT/prof_$PCFG.log" 2>&1)
  rc=$?
  tail -2 "$OUT/prof_$PCFG.log"
  fatal $rc rocprof
fi
echo "== done" | tee -a "$OUT/session.log"
