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

for s, W, hz in streams:
    for _ in range(20):
        window_features(s, W, W, hz)
for _ in range(20):
    window_features_mlp(s3, 200, 200, 20.0, mean, inv, 64, -1.0, out=out)
torch.cuda.synchronize()
print("ok")
