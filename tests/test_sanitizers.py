"""Host sanitizers over the native CSV parser (SURVEY.md §5 race detection): ASan+UBSan
and TSan builds parse the WISDM file plus truncated / random buffers and compare the
multithreaded parse with the single-threaded one.  (GPU ASan / xnack+ is not
available on the MI355X pool, so device kernels are covered by the fp32-oracle tests.)"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_csv_parser_asan_ubsan_tsan(wisdm_csv, tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(REPO, "tools", "sanitize", "run.sh"), wisdm_csv], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.count("csv sanitizer run: OK") == 2


@pytest.mark.skipif(not os.path.exists(os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")), reason="needs hipcc")
def test_kernel_launch_guards_asan_ubsan(tmp_path):
    """Every kernel source's host launcher under -Xarch_host ASan + UBSan: contract-violating
    calls (shapes, alignment, bounds, negative counts) return their documented error codes before
    anything reaches the device, and the host sizing helpers have no integer overflow."""
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(REPO, "tools", "sanitize", "guards.sh"), "8"], env=env,
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "guard sanitizer run: OK" in r.stdout
