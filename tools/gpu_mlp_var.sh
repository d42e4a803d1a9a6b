#!/bin/bash
# MLP kernel-variant A/B (HAR_MLP_VARIANT, har_mlp_set_variant): probe kernel times per variant.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/mlpvar_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
for rep in 1 2; do
for v in ${VARIANTS:-0 1 2 3}; do
  HAR_MLP_VARIANT=$v timeout -k 10 200 python -u tools/mlp_phase_probe.py 65536 > "$OUT/probe_${v}_$rep.txt" 2>&1
  rc=$?; echo "variant $v rep $rep: $(grep 65536 "$OUT/probe_${v}_$rep.txt")"; [ $rc -ne 0 ] && exit $rc
done
done
echo done
