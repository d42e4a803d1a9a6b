#!/bin/bash
# PMC passes over the MLP step (one rocprofv3 --pmc run per counter group of tools/pmc_groups_step.txt,
# never combined with tracing) + a kernel-trace stats pass; summaries -> gpurun_out/pmc5_<tag>.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc5_${1:-x}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-wisdm > "$OUT/trace.log" 2>&1
rc=$?; echo "trace pass: rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/mlp$i" -o pmc -- \
      python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-wisdm > "$OUT/mlp$i.log" 2>&1
  rc=$?; echo "mlp pass $i: rc=$rc"; [ $rc -ne 0 ] && exit $rc
done < "$ROOT/tools/${2:-pmc_groups_step.txt}"
cd "$ROOT"
python3 tools/pmc_table.py $(ls -d $OUT/mlp[0-9]* | grep -v "\.log$") > "$OUT/pmc.md" 2>&1; head -12 "$OUT/pmc.md"
echo done
