"""Phase timers and roctx ranges.

The reference times ``fit``/``transform`` with ``time()`` deltas rounded to ms
(``Main/main.py:116-124`` and five copies).  Its "Prediction made in" number is
lazy-plan time; here every timer synchronizes the device so
that the number is real work.  On ROCm ``torch.cuda.nvtx`` emits roctx ranges,
which ``rocprofv3 --marker-trace`` shows around each kernel family.
"""
from __future__ import annotations

import contextlib
import time
from collections import OrderedDict

import torch


def device_sync(device=None):
    if torch.cuda.is_available():
        if device is None or (isinstance(device, torch.device) and device.type == "cuda") or \
                (isinstance(device, str) and device.startswith("cuda")):
            torch.cuda.synchronize()


@contextlib.contextmanager
def roctx_range(name: str):
    """roctx range (no-op without a GPU)."""
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


class PhaseTimer:
    """Accumulates wall time per named phase, device-synchronized on both ends."""

    def __init__(self, device=None):
        self.device = device
        self.totals: "OrderedDict[str, float]" = OrderedDict()

    @contextlib.contextmanager
    def phase(self, name: str):
        device_sync(self.device)
        t0 = time.perf_counter()
        with roctx_range(name):
            yield
        device_sync(self.device)
        self.totals[name] = self.totals.get(name, 0.0) + time.perf_counter() - t0

    def get(self, name: str) -> float:
        return self.totals.get(name, 0.0)

    def as_dict(self):
        return dict(self.totals)


class Stopwatch:
    """``t0 = time(); ...; round(time()-t0, 3)`` with device sync."""

    def __init__(self, device=None):
        self.device = device
        device_sync(device)
        self.t0 = time.perf_counter()

    def elapsed(self, digits: int = 3) -> float:
        device_sync(self.device)
        return round(time.perf_counter() - self.t0, digits)
