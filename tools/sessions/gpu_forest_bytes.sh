#!/bin/bash
# DP forest wire volume: the analytic per-level table (tools/forest_bytes.py, one
# GPU) and bench.py --config rf9 / rf with --rf-parallel data under an 8-rank gloo job whose ranks share
# the box's one GPU (HAR_DIST_SHARE_DEVICE), in the r3 mode (HAR_TREE_DP_BOUND=1: collectives sized by the
# bound 2^d x trees) and the r4 mode (exact level counts, fp16 when exact); plus the tree-parallel mode.
#   usage: gpurun --timeout 1200 -- bash tools/gpu_forest_bytes.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/fbytes_${1:-x}"
mkdir -p "$OUT"
cd "$ROOT"
fatal() { if [ "$1" -ne 0 ]; then echo "STEP $2 fatal status $1"; exit "$1"; fi; }
timeout -k 10 240 python -u tools/forest_bytes.py rf9 --rows-per-gpu 60000 --world 8 > "$OUT/table_rf9.md" 2>&1
rc=$?; cat "$OUT/table_rf9.md" | grep -v amdgpu.ids; fatal $rc table_rf9
timeout -k 10 240 python -u tools/forest_bytes.py rf --rows-per-gpu 60000 --world 8 > "$OUT/table_rf.md" 2>&1
rc=$?; tail -3 "$OUT/table_rf.md"; fatal $rc table_rf
run8() {  # $1 = tag, $2 = HAR_TREE_DP_BOUND (0 / 1), rest = bench args
  local tag=$1 bound=$2; shift 2
  timeout -k 10 400 env HAR_TREE_DP_WIRE=${HAR_TREE_DP_WIRE:-packed} HAR_DIST_BACKEND=gloo HAR_DIST_SHARE_DEVICE=1 OMP_NUM_THREADS=2 HAR_TREE_DP_BOUND=$bound \
      python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29611 \
      bench.py --gpus 8 --steps 1 --warmup 0 --no-wisdm "$@" --out "$OUT/$tag.json" > "$OUT/$tag.log" 2>&1
  local rc=$?
  python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag', d['ms_per_step'], 'ms', d.get('rf_parallel'), d.get('collectives_per_step'), 'acc', d.get('test_accuracy'))" 2>/dev/null || tail -5 "$OUT/$tag.log"
  return $rc
}
run8 rf9_exact 0 --config rf9 --rows 4000 --trees 100 --rf-parallel data
rc=$?; fatal $rc rf9_exact
HAR_TREE_DP_WIRE=fp16 run8 rf9_fp16 0 --config rf9 --rows 4000 --trees 100 --rf-parallel data
rc=$?; fatal $rc rf9_fp16
run8 rf9_bound 1 --config rf9 --rows 4000 --trees 100 --rf-parallel data
rc=$?; fatal $rc rf9_bound
run8 rf9_tree 0 --config rf9 --rows 4000 --trees 100 --rf-parallel tree
rc=$?; fatal $rc rf9_tree
run8 rf_exact 0 --config rf --rows 8000 --rf-parallel data
rc=$?; fatal $rc rf_exact
HAR_TREE_DP_WIRE=fp16 run8 rf_fp16 0 --config rf --rows 8000 --rf-parallel data
rc=$?; fatal $rc rf_fp16
run8 rf_bound 1 --config rf --rows 8000 --rf-parallel data
rc=$?; fatal $rc rf_bound
echo done
