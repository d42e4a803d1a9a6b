#!/bin/bash
# Round-4 iteration on one gpurun call: selected GPU tests, the MLP phase probe (B = 65536 and 256, graph
# replayed kernel times + in-kernel stamps), three plain bench runs and a reference-suite bench.
#   usage: gpurun --timeout 1200 -- bash tools/gpu_r4.sh <tag> [pytest -k expression]
# Every GPU step has its own time limit; a fault / abort / timeout ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r4_${1:-x}"
KEXPR="${2:-mlp or step or fused or frag}"
mkdir -p "$OUT"
cd "$ROOT"
fatal() {  # $1 = exit code, $2 = step: stop on anything but pass / test failure
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ] && [ "$1" -ne 5 ]; then echo "STEP $2 fatal status $1"; exit "$1"; fi
}
timeout -k 10 600 python -u -m pytest tests -m gpu -k "$KEXPR" -q -x --timeout 200 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1
rc=$?; tail -4 "$OUT/pytest.log"; fatal $rc pytest
timeout -k 10 200 python -u tools/mlp_phase_probe.py 65536 256 > "$OUT/probe.txt" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/probe.txt"; fatal $rc probe
HAR_MLP_BWD=3 timeout -k 10 200 python -u tools/mlp_phase_probe.py 65536 > "$OUT/probe_bwd3.txt" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/probe_bwd3.txt" | sed 's/^/[bwd3] /'; fatal $rc probe_bwd3
timeout -k 10 200 python -u tools/mlp_phase_probe.py --stamps > "$OUT/stamps.txt" 2>&1
rc=$?; grep -E -- "---|prologue|epilogue|total|clock|tile 4" "$OUT/stamps.txt"; fatal $rc stamps
timeout -k 10 240 python -u tools/mlp_fit_probe.py > "$OUT/fit_probe.txt" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/fit_probe.txt"; fatal $rc fit_probe
timeout -k 10 240 python -u tools/mlp_fit_probe.py --hidden 128 > "$OUT/fit_probe128.txt" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/fit_probe128.txt"; fatal $rc fit_probe128
for i in 1 2 3; do
  timeout -k 10 180 python bench.py --no-wisdm --steps 200 --warmup 20 --out "$OUT/bench_$i.json" > "$OUT/bench_$i.log" 2>&1
  rc=$?; fatal $rc bench
  python -c "import json;d=json.load(open('$OUT/bench_$i.json'));print('run $i ms/step', d['ms_per_step'], 'acc', d['synthetic_test_accuracy'])"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --out "$OUT/bench_driver.json" > "$OUT/bench_driver.log" 2>&1
rc=$?; fatal $rc bench_driver
python - "$OUT/bench_driver.json" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
print("driver-cmd ms/step", d["ms_per_step"], "wisdm acc", d.get("test_accuracy"), "wisdm fit s", d.get("wisdm_mlp_fit_s"))
for k, v in d.get("reference_suite", {}).get("models", {}).items():
    print(" ", k, {x: v.get(x) for x in ("fit_s", "first_fit_s", "accuracy")})
EOF
echo done
