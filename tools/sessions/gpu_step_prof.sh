#!/bin/bash
# MLP step profiling session: correctness tests of the step kernels, per-kernel timing (phase probe),
# in-kernel phase stamps, then rocprofv3 PMC passes (one run per counter group) over the probe.
#   usage: gpurun --timeout 900 -- bash tools/gpu_step_prof.sh <tag> [pmc]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/step_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "mlp" > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/mlp_phase_probe.py 65536 262144 > "$OUT/probe.log" 2>&1 || exit $?
cat "$OUT/probe.log"
timeout -k 10 120 python tools/mlp_phase_probe.py --stamps 65536 > "$OUT/stamps.log" 2>&1 || exit $?
grep -E "prologue|tile 1 |tile 7 |epilogue|total|real" "$OUT/stamps.log"
if [ "${2:-}" = "pmc" ]; then
  export TMPDIR=/tmp
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i + 1))
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o pmc -- \
        python3 "$ROOT/tools/mlp_phase_probe.py" 65536 > "$OUT/pmc$i.log" 2>&1) || exit $?
  done < "$ROOT/tools/pmc_groups_step.txt"
  python3 tools/pmc_table.py "$OUT"/pmc1 "$OUT"/pmc2 > "$OUT/pmc.md" 2>&1
  grep -E "mlp_step|mlp_fwd3|mlp_bwd3|grad_reduce|kernel \|" "$OUT/pmc.md" | cut -c1-600
fi
