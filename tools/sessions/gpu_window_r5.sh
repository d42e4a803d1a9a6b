#!/bin/bash
# Round-5 window featurizer iteration: window / raw GPU tests, the kernel probe (tools/window_probe.py,
# v3 only) and PMC passes over it (one rocprofv3 --pmc run per counter group, never with tracing).
#   usage: gpurun --timeout 900 -- bash tools/gpu_window_r5.sh <tag> [pmc]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/win5_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
export HAR_WINDOW_AB=0
timeout -k 10 300 python -u -m pytest tests/test_window.py tests/test_raw.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; if [ $rc -ne 0 ] && [ $rc -ne 5 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/window_probe.py > "$OUT/probe.txt" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/probe.txt"; [ $rc -ne 0 ] && exit $rc
[ "${2:-}" != "pmc" ] && { echo done; exit 0; }
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE" "FETCH_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o pmc -- \
      python3 "$ROOT/tools/window_probe.py" > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc pass $i: rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
cd "$ROOT"
python3 tools/pmc_table.py "$OUT/pmc1" "$OUT/pmc2" "$OUT/pmc3" > "$OUT/pmc.md" 2>&1; cat "$OUT/pmc.md" | cut -c1-400
echo done
