#!/bin/bash
# Reference-suite iteration: tree / findSplits GPU tests, then bench --config reference and rf.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
python tools/build_native.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "tree or forest or thresh or split or level or graph or reference or etl or bin" > gpurun_out/pytest_ref.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ref.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config reference --steps 5 --warmup 2 --out gpurun_out/bench_reference.json \
    > gpurun_out/bench_reference.log 2>&1 || { tail -5 gpurun_out/bench_reference.log; exit 1; }
python - <<'PY'
import json
r = json.load(open("gpurun_out/bench_reference.json")); rs = r.get("reference_suite", r)
print({k: (round(v["fit_s"] * 1e3, 2), round(v["accuracy"], 4)) for k, v in rs["models"].items()})
PY
for cfg in rf rf9; do
  timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --out gpurun_out/bench_$cfg.json > gpurun_out/bench_$cfg.log 2>&1 || exit 1
  python -c "import json;r=json.load(open('gpurun_out/bench_$cfg.json'));print('$cfg', round(r['ms_per_step'],3), r['test_accuracy'])"
done
