set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_window.py tests/test_raw.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_win.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_win.log; [ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_win" -o w -- python3 "$GRAFT_REPO_ROOT/tools/window_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_win.log" 2>&1
echo "prof rc=$?"
