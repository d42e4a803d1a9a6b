"""Time the fused MLP forward kernel alone (events around N launches) for each HAR_MLP_FWD_DBG
variant given on the command line (debug experiment: 1 = no h1/dact2 stores, 2 = stage 2 cut to
one k-chunk, 3 = both)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from har.models.mlp import MLPEngine, pad_input_bf16  # noqa: E402
from har.ops import _native  # noqa: E402

B = int(os.environ.get("PROBE_B", "65536"))
dev = torch.device("cuda:0")
eng = MLPEngine([43, 256, 256, 6], B, dev)
X = pad_input_bf16(torch.randn(B, 43, device=dev), 64)
y = torch.randint(0, 6, (B,), device=dev, dtype=torch.int32)
mod = _native.kernels()
L = eng.layout
H = 256


def launch():
    mod.mlp_fwd_head(X.data_ptr(), 64, eng._w(eng.Pb, "W0").data_ptr(), eng._w(eng.P, "b0").data_ptr(),
                     eng._w(eng.Pb, "W1").data_ptr(), eng._w(eng.P, "b1").data_ptr(), H,
                     eng._w(eng.Pb, "Wout").data_ptr(), eng._w(eng.P, "bout").data_ptr(), y.data_ptr(), B, 6,
                     1.0 / B, eng.acts[1].data_ptr(), eng.dbuf[1].data_ptr(), eng.fslab.data_ptr(),
                     eng.fblock_loss.data_ptr(), eng.fblock_correct.data_ptr(), _native.stream_ptr())


for _ in range(20):
    launch()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200):
    launch()
e1.record()
torch.cuda.synchronize()
dbg = os.environ.get("HAR_MLP_FWD_DBG", "0")
print(f"B={B} HAR_MLP_FWD_DBG={dbg}: {e0.elapsed_time(e1) / 200 * 1e3:.1f} us per forward")
