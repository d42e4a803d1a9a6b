#!/bin/bash
# LR solve diagnostics: fit times at different phase-kernel chunk budgets (HAR_QN_WORKGROUPS) and two
# PMC passes over the single fit (never combined with tracing).  -> gpurun_out/lrpmc_<tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/lrpmc_${1:-x}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for wg in 512 128 32; do
  HAR_QN_WORKGROUPS=$wg timeout -k 10 120 python3 "$ROOT/tools/lr_probe.py" --model lr --fits 3 > "$OUT/wg$wg.txt" 2>&1
  rc=$?; echo "workgroups $wg: $(grep -m3 '^fit\|^mean' "$OUT/wg$wg.txt" | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
done
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CU_CYCLES"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc -- \
      python3 "$ROOT/tools/lr_probe.py" --model lr --fits 1 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i: rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
echo done
