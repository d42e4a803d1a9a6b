#!/bin/bash
# The DP MLP step on a forced 1-rank RCCL group (HAR_DIST_FORCE_PG=1): sharded optimizer (reduce-scatter +
# all-gather) vs one all-reduce (HAR_MLP_SHARDED_OPT=0), eager, 3 rounds; ms/step + phase_ms.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
mkdir -p gpurun_out/dp1
for r in 1 2 3; do
  for sh in 1 0; do
    HAR_MLP_SHARDED_OPT=$sh HAR_DIST_FORCE_PG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-wisdm \
        > gpurun_out/dp1/s${sh}_$r.json 2> gpurun_out/dp1/s${sh}_$r.err || { tail -3 gpurun_out/dp1/s${sh}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d.get('phase_ms') or {}; print('sharded', sys.argv[2], 'run', sys.argv[3], 'ms', round(d['ms_per_step'],5), {k: (round(v,4) if isinstance(v,float) else v) for k,v in p.items()})" gpurun_out/dp1/s${sh}_$r.json $sh $r
  done
done
