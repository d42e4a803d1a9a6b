set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for run in "stream" "stream --stream-pass" "infer"; do
  tag=$(echo "$run" | tr -d ' -')
  if [ "$run" = "stream" ]; then st=50; wu=10; elif [ "$run" = "infer" ]; then st=20; wu=5; else st=3; wu=1; fi
  timeout -k 10 400 python bench.py --config $run --steps $st --warmup $wu --out gpurun_out/bench_$tag.json > gpurun_out/bench_$tag.log 2>&1 || { tail -5 gpurun_out/bench_$tag.log; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/bench_$tag.json'));print('$tag', round(r['ms_per_step'],4), '%.3e' % r['value'], r.get('test_accuracy'), r.get('samples_per_s'))"
done
