#!/bin/bash
# Small-batch MLP step records: probe (graph-replayed step at B = 256 / 512), kernel trace of it, the
# bench's WISDM fit fields, main.py --preset mlp.  -> gpurun_out/small_<tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/small_${1:-x}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 200 python -u tools/mlp_phase_probe.py 256 512 > "$OUT/probe.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/probe.txt"
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- \
    python3 "$ROOT/tools/mlp_phase_probe.py" 256 > "$OUT/trace.log" 2>&1) || exit $?
python3 "$ROOT/tools/prof_summary.py" "$OUT/trace/t_kernel_stats.csv" "small step B=256" | sed -n 5,9p | cut -c1-150
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 || exit $?
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('bench ms', d['ms_per_step'], 'wisdm fit', d.get('wisdm_mlp_fit_s'), 'first', d.get('wisdm_mlp_first_fit_s'), 'acc', d.get('test_accuracy'))"
timeout -k 10 300 python -u main.py --preset mlp --out-dir "$OUT/main_mlp" > "$OUT/main_mlp.log" 2>&1 || { tail -5 "$OUT/main_mlp.log"; exit 1; }
grep -h "trained in\|Accuracy\|accuracy" "$OUT/main_mlp.log" "$OUT"/main_mlp/result.txt 2>/dev/null | head -6
echo done
