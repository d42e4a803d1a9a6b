#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter group, never combined with tracing): the MLP step
# (bench.py) and the window featurizer (tools/window_probe.py, v3 kernels only).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_${1:-x}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/mlp$i" -o pmc -- \
      python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-wisdm > "$OUT/mlp$i.log" 2>&1
  rc=$?; echo "mlp pass $i: rc=$rc"; [ $rc -ne 0 ] && exit $rc
done < "$ROOT/tools/pmc_groups_step.txt"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE" "FETCH_SIZE"; do
  i=$((i + 1))
  HAR_WINDOW_AB=0 timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/win$i" -o pmc -- \
      python3 "$ROOT/tools/window_probe.py" > "$OUT/win$i.log" 2>&1
  rc=$?; echo "window pass $i: rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
echo done
