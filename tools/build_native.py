#!/usr/bin/env python3
"""Build the in-tree native extension ``_har_native`` for gfx950.

Every ``csrc/kernels/*.hip`` and ``csrc/host/*.cpp`` file is compiled to an
object with ``hipcc --offload-arch=gfx950`` (in parallel, incrementally), then
linked with ``csrc/bind.cpp`` (pybind11) into
``activity-recognition-using-apache-spark_amd/_har_native.so`` — importable as
``har._har_native``.  The ``.so`` is git-ignored but travels to the GPU box with
the gpurun snapshot.  No torch headers are involved, so a full rebuild takes
well under a minute.

Staleness is content based, not mtime based: every object records the SHA-256
of its source, all headers and its flags (``<obj>.sha``), and the whole library
embeds the hash of all of them (``source_hash()`` in the module), which
``ops/_native.py`` compares with the tree at import time — a library built
from other sources is rebuilt (or refused when auto-build is off), even if
its file times look newer.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "activity-recognition-using-apache-spark_amd")
OBJ = os.path.join(ROOT, "build", "obj")
OUT = os.path.join(PKG, "_har_native.so")
ARCH = os.environ.get("HAR_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _headers():
    hs = []
    for d, _, fs in os.walk(CSRC):
        hs += [os.path.join(d, f) for f in fs if f.endswith(".h")]
    return hs


def _sources():
    srcs = []
    for sub, ext in (("kernels", ".hip"), ("host", ".cpp")):
        d = os.path.join(CSRC, sub)
        srcs += sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(ext))
    srcs.append(os.path.join(CSRC, "bind.cpp"))
    return srcs


def _flags(src):
    import pybind11

    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC,
              "-Wno-unused-result", "-Wno-unused-variable"]
    if src.endswith(".hip"):
        return common + ["-x", "hip", "-munsafe-fp-atomics"]
    inc = ["-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"]]
    return common + inc + ["-D__HIP_PLATFORM_AMD__"]


def _obj_for(src):
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(OBJ, rel + ".o")


def _digest(paths, extra=()) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.relpath(p, ROOT).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    for e in extra:
        h.update(str(e).encode())
    return h.hexdigest()


def _flag_key(flags) -> str:
    """Compile flags without machine-specific absolute paths (the tree is checked out at a
    different path on the GPU box, and the hash must still match there)."""
    return " ".join("<path>" if f.startswith("/") else f for f in flags)


def source_hash() -> str:
    """Hash of every input of the library (sources, headers, compile flags, arch)."""
    srcs = _sources()
    return _digest(sorted(srcs + _headers()), [ARCH] + [_flag_key(_flags(s)) for s in srcs])[:32]


def _read(p):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError:
        return None


def _stale(target, digest):
    return not os.path.exists(target) or _read(target + ".sha") != digest


def needs_build() -> bool:
    return _stale(OUT, source_hash())


def build(verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(OBJ, exist_ok=True)
    headers = sorted(_headers())
    srcs = _sources()
    lib_hash = source_hash()

    def compile_one(src):
        obj = _obj_for(src)
        flags = _flags(src)
        if src.endswith("bind.cpp"):
            flags = flags + [f'-DHAR_SOURCE_HASH="{lib_hash}"']
        digest = _digest([src] + headers, [ARCH, _flag_key(flags)])
        if not _stale(obj, digest):
            return obj, None
        cmd = [HIPCC] + flags + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            return obj, f"{src}:\n{r.stdout}\n{r.stderr}"
        with open(obj + ".sha", "w") as f:
            f.write(digest)
        return obj, None

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(compile_one, srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("native build failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    if _stale(OUT, lib_hash):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", OUT] + objs + \
              ["-L/opt/rocm/lib", "-lamdhip64", "-lpthread", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        with open(OUT + ".sha", "w") as f:
            f.write(lib_hash)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=8)
    a = ap.parse_args()
    print(build(verbose=a.verbose, jobs=a.jobs))
    sys.exit(0)
