set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_win" -o w -- python3 "$GRAFT_REPO_ROOT/tools/window_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_win.log" 2>&1 || exit 1
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE" "FETCH_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcw$i" -o pmc -- python3 "$GRAFT_REPO_ROOT/tools/window_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/pmcw$i.log" 2>&1 || exit 1
done
echo done
