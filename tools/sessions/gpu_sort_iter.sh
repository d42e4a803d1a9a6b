set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sort_columns or thresh or split or forest or tree" > gpurun_out/pytest_sort.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_sort.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config reference --steps 5 --warmup 2 --out gpurun_out/bench_reference.json > gpurun_out/bench_reference.log 2>&1 || { tail -5 gpurun_out/bench_reference.log; exit 1; }
python -c "
import json; r=json.load(open('gpurun_out/bench_reference.json')); rs=r.get('reference_suite',r)
print({k: (round(v['fit_s']*1e3,2), round(v['accuracy'],4)) for k,v in rs['models'].items()})"
for cfg in rf rf9; do
  timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --out gpurun_out/bench_$cfg.json > gpurun_out/bench_$cfg.log 2>&1 || exit 1
  python -c "import json;r=json.load(open('gpurun_out/bench_$cfg.json'));print('$cfg', round(r['ms_per_step'],3), r['test_accuracy'])"
done
