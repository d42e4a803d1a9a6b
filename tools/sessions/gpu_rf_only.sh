cd "$GRAFT_REPO_ROOT"
for cfg in rf rf9; do
  timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --out gpurun_out/bench_$cfg.json > gpurun_out/bench_$cfg.log 2>&1 || exit 1
done
