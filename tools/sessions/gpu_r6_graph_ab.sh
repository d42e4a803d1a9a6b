#!/bin/bash
# Same-box A/B of the flagship step's launch mode: eager (--graph 0) vs whole-step HIP graph (--graph 1).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/graph_ab"
mkdir -p "$OUT"
cd "$ROOT"
for r in 1 2 3; do
  for m in 0 1; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-wisdm --graph $m > "$OUT/g${m}_$r.json" 2> "$OUT/g${m}_$r.err"
    rc=$?; [ $rc -ne 0 ] && { tail -3 "$OUT/g${m}_$r.err"; exit $rc; }
    echo "graph=$m run $r: $(python3 -c "import json,sys; print(round(json.load(open(sys.argv[1]))['ms_per_step'], 5))" "$OUT/g${m}_$r.json")"
  done
done
