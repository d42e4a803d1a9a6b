#!/bin/bash
# Dense-design LR (WISDM numeric43: 43 dense columns) fit times with the matrix-core evaluation
# (default) and with the VALU evaluation (HAR_LR_EVAL_MFMA=0), + the evaluation kernel's trace medians.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/lrdense_${1:-x}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for mf in 1 0; do
  for m in lr lrcv; do
    HAR_LR_EVAL_MFMA=$mf timeout -k 10 200 python3 "$ROOT/tools/lr_probe.py" --model $m --fits 5 --encoding numeric43 \
        > "$OUT/${m}_mf$mf.txt" 2>&1 || exit $?
    echo "mfma=$mf $m: $(grep -m3 '^fit\|^mean' "$OUT/${m}_mf$mf.txt" | tr '\n' ' ')"
  done
  (cd /tmp && HAR_LR_EVAL_MFMA=$mf timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr$mf" -o r -- \
      python3 "$ROOT/tools/lr_probe.py" --model lrcv --fits 2 --encoding numeric43 > "$OUT/tr$mf.log" 2>&1) || exit $?
  python3 "$ROOT/tools/lr_kernel_medians.py" "$OUT/tr$mf/r_kernel_trace.csv" | sed "s/^/mfma=$mf /"
done
echo done
