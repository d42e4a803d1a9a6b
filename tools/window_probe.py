"""Window featurizer kernel probe: the rf (60k x 200 x 3, stride 200), rf9 (60k x 500 x 9) and
stream (65536 x 200 x 3 -> bf16 MLP rows) shapes, 20 launches each (time them with rocprofv3).

The streams come from ``generate_stream`` (the bench's synthetic accelerometer data, so the
peak / histogram branches see realistic signals), and ~0.5 s of GEMMs run first so the launches
are timed at steady clocks rather than during the power-state ramp of a fresh process."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from har.data.synth import StreamSpec, generate_stream  # noqa: E402
from har.features.window import n_features, window_features, window_features_mlp  # noqa: E402

dev = torch.device("cuda:0")
streams = []
for nw, W, A, hz in ((60000, 200, 3, 20.0), (60000, 500, 9, 50.0)):
    s, _ = generate_stream(nw, StreamSpec(axes=A, window=W, hz=hz), dev)
    streams.append((s, W, hz))
nw = 65536
s3, _ = generate_stream(nw, StreamSpec(), dev)
F = n_features(3)
mean, inv = torch.zeros(F, device=dev), torch.ones(F, device=dev)
out = torch.empty(nw, 64, dtype=torch.bfloat16, device=dev)

a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
t0 = time.time()
while time.time() - t0 < 0.5:
    for _ in range(20):
        a @ a
    torch.cuda.synchronize()

from har.ops import _native  # noqa: E402

mod = _native.kernels()


def timed(fn, reps=20):
    """us per launch (HIP events around `reps` back-to-back launches, best of 3)"""
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


modes = [("v3", 0), ("legacy", 1)] if os.environ.get("HAR_WINDOW_AB", "1") != "0" else [("v3", 0)]
for name, legacy in modes:
    mod.window_set_legacy(legacy)
    for s, W, hz in streams:
        us = timed(lambda: window_features(s, W, W, hz))
        gb = s.numel() * 4 / 1e9
        print(f"{name:7s} {s.shape[1]} axes W={W} stride={W}: {us:8.1f} us  {gb / us * 1e3:6.2f} TB/s ({gb:.3f} GB)")
    us = timed(lambda: window_features_mlp(s3, 200, 200, 20.0, mean, inv, 64, -1.0, out=out))
    print(f"{name:7s} 3 axes W=200 MLP rows : {us:8.1f} us  {s3.numel() * 4 / us / 1e6:6.2f} TB/s")
    us = timed(lambda: window_features(s3, 200, 100, 20.0))
    print(f"{name:7s} 3 axes W=200 stride=100: {us:8.1f} us  {s3.numel() * 4 / us / 1e6:6.2f} TB/s ({s3.shape[0] // 100 - 1} windows)")
    # the 1B-sample stream pass's kernel: 50%-overlapping windows straight into bf16 MLP rows
    out2 = torch.empty(s3.shape[0] // 100 - 1, 64, dtype=torch.bfloat16, device=dev)
    us = timed(lambda: window_features_mlp(s3, 200, 100, 20.0, mean, inv, 64, -1.0, out=out2))
    print(f"{name:7s} 3 axes W=200 stride=100 MLP rows: {us:8.1f} us  ({out2.shape[0] / us * 1e-3:.2f} G windows/s)")
mod.window_set_legacy(0)
torch.cuda.synchronize()
print("ok")
