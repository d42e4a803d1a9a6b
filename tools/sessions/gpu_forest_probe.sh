set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python tools/forest_host_probe.py > gpurun_out/probe_rf.log 2>&1 || exit $?
timeout -k 10 200 python tools/forest_host_probe.py --dt --rows 60000 > gpurun_out/probe_dt.log 2>&1 || exit $?
for run in "dt --rows 1000000" "dt --rows 1000000 --no-subtract"; do
  tag=$(echo "$run" | tr -d ' -')
  timeout -k 10 300 python bench.py --config $run --steps 5 --warmup 2 --out gpurun_out/bench_$tag.json > gpurun_out/bench_$tag.log 2>&1 || exit $?
  python -c "import json;r=json.load(open('gpurun_out/bench_$tag.json'));print('$tag', round(r['ms_per_step'],3), r['test_accuracy'])"
done
tail -3 gpurun_out/probe_rf.log gpurun_out/probe_dt.log
