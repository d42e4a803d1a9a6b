#!/bin/bash
# PMC counter passes over the flagship bench (one rocprofv3 --pmc run per counter group;
# never combined with tracing domains).  usage: bash tools/pmc_session.sh [list]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
if [ "${1:-}" = "list" ]; then
  timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
fi
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o pmc -- \
      python3 "$ROOT/bench.py" --steps ${PMC_STEPS:-5} --warmup 2 ${BENCH_ARGS:-} > "$OUT/pmc$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp): rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done < "${PMC_GROUPS:-$ROOT/tools/pmc_groups.txt}"
exit 0
