"""Loader for the in-tree native extension ``_har_native`` (gfx950 HIP kernels +
C++ host runtime), built by ``tools/build_native.py``.

Policy: on a machine with a GPU, every device op REQUIRES the extension — a
missing or stale build raises instead of silently running a PyTorch fallback
(the round-end checks record which ``.so`` files were loaded).  On a CPU-only
machine the ops run their PyTorch reference implementations, which are also the
test oracles.
"""
from __future__ import annotations

import importlib
import os
import threading

import torch

_LOCK = threading.Lock()
_MOD = None
_ERR = None


def _import():
    global _MOD, _ERR
    with _LOCK:
        if _MOD is not None or _ERR is not None:
            return _MOD
        try:
            import sys
            alt = os.environ.get("HAR_NATIVE_SO")
            if alt:
                # A/B tooling only (tools/sessions/gpu_ab.sh): load another build of the extension, e.g. the
                # previous commit's, so two builds are compared on the same GPU box; no source check
                from importlib.machinery import ExtensionFileLoader
                from importlib.util import module_from_spec, spec_from_file_location

                loader = ExtensionFileLoader("har._har_native", alt)
                spec = spec_from_file_location("har._har_native", alt, loader=loader)
                mod = module_from_spec(spec)
                loader.exec_module(mod)
                sys.modules["har._har_native"] = mod
                _MOD = mod
                return _MOD
            root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            tools = os.path.join(root, "tools")
            bn = None
            if os.path.isdir(os.path.join(root, "csrc")):
                if tools not in sys.path:
                    sys.path.insert(0, tools)
                import build_native as bn  # type: ignore
                if os.environ.get("HAR_AUTOBUILD", "1") == "1" and bn.needs_build():
                    bn.build()
            mod = importlib.import_module("har._har_native")
            if bn is not None:  # the loaded binary must come from exactly these sources
                want = bn.source_hash()
                got = mod.source_hash() if hasattr(mod, "source_hash") else "none"
                if got != want:
                    raise RuntimeError(f"_har_native.so was built from other sources (hash {got}, tree {want}); "
                                       "rebuild with python tools/build_native.py")
            _MOD = mod
        except Exception as e:  # pragma: no cover
            _ERR = e
        return _MOD


def host_module():
    """Native module for host-side routines (CSV parser); None if unavailable."""
    return _import()


def kernels():
    """Native module for device kernels; raises if it cannot be loaded."""
    mod = _import()
    if mod is None:
        raise RuntimeError(f"har native extension unavailable (GPU ops require it): {_ERR!r}")
    return mod


def available() -> bool:
    return _import() is not None


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    """data pointer of an optional tensor (0 for None)."""
    return 0 if t is None else t.data_ptr()


def use_device_kernels(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU — the HIP kernels are then mandatory."""
    return t.is_cuda
