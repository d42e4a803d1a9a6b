#!/usr/bin/env python3
"""Per-kernel timing of the flagship MLP step (43-256-256-6) at several batch sizes: the full
step, the fused forward alone, the fused backward alone and the gradient reduction + Adam alone
(HIP events around 100 back-to-back launches of one kernel).  The slope over batch size is the
per-row cost of a kernel, the intercept its fixed (launch / prologue / epilogue) cost.

    python tools/mlp_phase_probe.py [B ...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from har.models.mlp import MLPEngine, pad_input_bf16  # noqa: E402
from har.ops import _native  # noqa: E402


def timed(fn, reps=100, graph=None):
    """us per call: min over 3 runs of `reps` back-to-back calls.  graph=True captures the `reps`
    calls in one HIP graph and times its replay (device time, no host launch cost: a short kernel
    launched from Python is otherwise host-bound); default from HAR_PROBE_GRAPH (1)."""
    if graph is None:
        graph = os.environ.get("HAR_PROBE_GRAPH", "1") != "0"
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    run = None
    if graph:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(reps):
                    fn()
        torch.cuda.current_stream().wait_stream(s)
        run = g.replay
    else:
        def run():
            for _ in range(reps):
                fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def stamps(B=65536):
    """One step with the stamped kernel instantiations: per-phase shader cycles (median / max over
    waves) and the real-time (100 MHz) entry / exit spread of the workgroups."""
    import numpy as np

    dev = torch.device("cuda")
    eng = MLPEngine([43, 256, 256, 6], B, dev, seed=1)
    g = torch.Generator(device=dev).manual_seed(0)
    X = pad_input_bf16(torch.randn(B, 43, device=dev, generator=g), eng.layout.in_pad)
    y = torch.randint(0, 6, (B,), device=dev, generator=g).to(torch.int32)
    for _ in range(3):
        eng.train_step(X, y, B)
    buf = torch.zeros(2 * 256 * 8 * 40, dtype=torch.int64, device=dev)
    mod = _native.kernels()
    mod.mlp_set_stamps(buf.data_ptr())
    try:
        for _ in range(3):  # the last of three stamped steps is read
            buf.zero_()
            eng.train_step(X, y, B)
        torch.cuda.synchronize()
    finally:
        mod.mlp_set_stamps(0)
    st = buf.cpu().numpy().view(np.uint64).astype(np.float64).reshape(2, 256 * 8, 40)
    bwd4 = os.environ.get("HAR_MLP_BWD", "4") != "3"
    roles = [("forward", 0, None)]
    if bwd4:  # mlp_bwd4: waves 0..3 of a workgroup produce, 4..7 consume (own loops, own phase stamps)
        roles += [("backward producers (waves 0-3)", 1, True), ("backward consumers (waves 4-7)", 1, False)]
    else:
        roles += [("backward", 1, None)]
    for name, k, producer in roles:
        s = st[k]
        live = s[:, 0] > 0
        if producer is not None:
            live &= ((np.arange(s.shape[0]) % 8) < 4) == producer
        s = s[live]
        print(f"--- {name}: {live.sum()} waves stamped")
        # forward slots 10.. / backward slots 26.. hold tile-4 sub-phases
        lim = 10 if (k == 0 and (s[:, 10] > 0).all()) else 26 if (k == 1 and ((s[:, 26] > 0) | (s[:, 29] > 0)).all()) else 34
        ntile = int(((s[:, 2:lim] > 0).sum(1)).max())
        rows = [("prologue (weights in regs)", s[:, 1] - s[:, 0])]
        for t in range(min(ntile, 32)):
            end = s[:, 3 + t] if t + 1 < ntile else s[:, 34]
            rows.append((f"tile {t}", end - s[:, 2 + t]))
        rows.append(("epilogue", s[:, 35] - s[:, 34]))
        rows.append(("total (entry -> exit)", s[:, 35] - s[:, 0]))
        for nm, v in rows:
            print(f"  {nm:28s} median {np.median(v):9.0f}  max {v.max():9.0f} cycles")
        if k == 0 and (s[:, 10] > 0).all():  # forward sub-phases of tile 4 (stamped slots 10..13)
            sub = [("  tile 4: softmax", s[:, 10] - s[:, 6]), ("  tile 4: stage 5", s[:, 11] - s[:, 10]),
                   ("  tile 4: stages 2+3 (next tile)", s[:, 12] - s[:, 11]),
                   ("  tile 4: stage 1 + X loads", s[:, 13] - s[:, 12]), ("  tile 4: to next tile (barrier)", s[:, 7] - s[:, 13])]
            for nm, v in sub:
                print(f"  {nm:28s} median {np.median(v):9.0f}  max {v.max():9.0f} cycles")
        if k == 1 and bwd4 and producer and (s[:, 26] > 0).all():  # mlp_bwd4 producer phases of tile 4
            sub = [("  tile 4: dact2 refill wait", s[:, 32] - s[:, 6]),
                   ("  tile 4: dact2 (tile 5) -> LDS", s[:, 26] - s[:, 32]), ("  tile 4: X stage + refills", s[:, 27] - s[:, 26]),
                   ("  tile 4: h1 recompute (tile 5)", s[:, 28] - s[:, 27]), ("  tile 4: (c) dW0 + db0 (tile 3)", s[:, 33] - s[:, 28]),
                   ("  tile 4: barrier", s[:, 7] - s[:, 33])]
            for nm, v in sub:
                print(f"  {nm:28s} median {np.median(v):9.0f}  max {v.max():9.0f} cycles")
        if k == 1 and bwd4 and producer is False and (s[:, 29] > 0).all():  # mlp_bwd4 consumer phases
            sub = [("  tile 4: (a) dact1", s[:, 29] - s[:, 6]), ("  tile 4: (b) dW1 + db1", s[:, 30] - s[:, 29]),
                   ("  tile 4: barrier", s[:, 7] - s[:, 30])]
            for nm, v in sub:
                print(f"  {nm:28s} median {np.median(v):9.0f}  max {v.max():9.0f} cycles")
        if k == 1 and not bwd4 and (s[:, 26] > 0).all():  # backward sub-phases of tile 4 (stamped slots 26..30)
            sub = [("  tile 4: dact2 -> LDS", s[:, 26] - s[:, 6]), ("  tile 4: X stage + refills", s[:, 27] - s[:, 26]),
                   ("  tile 4: h1 recompute", s[:, 28] - s[:, 27]), ("  tile 4: (a) + (b) + db1", s[:, 29] - s[:, 28]),
                   ("  tile 4: (c) dW0", s[:, 30] - s[:, 29]), ("  tile 4: barrier", s[:, 7] - s[:, 30])]
            for nm, v in sub:
                print(f"  {nm:28s} median {np.median(v):9.0f}  max {v.max():9.0f} cycles")
        t0 = s[:, 38].min()
        ent, ex = (s[:, 38] - t0) * 10.0, (s[:, 39] - t0) * 10.0  # ns
        print(f"  real time: entry spread {ent.max():.0f} ns (median {np.median(ent):.0f}), "
              f"exit median {np.median(ex):.0f} ns max {ex.max():.0f} ns; "
              f"clock ~{np.median((s[:, 35] - s[:, 0]) / np.maximum(ex - ent, 1)):.2f} GHz")


def main():
    dev = torch.device("cuda")
    if sys.argv[1:2] == ["--stamps"]:
        return stamps(int(sys.argv[2]) if len(sys.argv) > 2 else 65536)
    sizes = [int(a) for a in sys.argv[1:]] or [16384, 32768, 65536, 131072, 262144]
    print(f"{'B':>8s} {'step':>8s} {'fwd':>8s} {'bwd':>8s} {'reduce':>8s} {'eager':>8s}  (us, min of 3 x 100 launches; "
          "graph-replayed unless HAR_PROBE_GRAPH=0, eager = the step launched from Python)")
    for B in sizes:
        eng = MLPEngine([43, 256, 256, 6], B, dev, seed=1)
        g = torch.Generator(device=dev).manual_seed(0)
        X = pad_input_bf16(torch.randn(B, 43, device=dev, generator=g), eng.layout.in_pad)
        y = torch.randint(0, 6, (B,), device=dev, generator=g).to(torch.int32)
        eng.train_step(X, y, B)
        torch.cuda.synchronize()
        step = timed(lambda: eng.train_step(X, y, B))
        step_eager = timed(lambda: eng.train_step(X, y, B), graph=False)
        if eng.last_path == "small":  # B <= 512: the small-batch step (mlp_small.hip + reduction / Adam)
            print(f"{B:8d} {step:8.1f}  (small-batch path: one tile kernel + reduction / Adam; eager {step_eager:.1f})")
            continue
        phases = getattr(eng, "phase_fns", None)
        if phases is None:
            print(f"{B:8d} {step:8.1f}  (engine exposes no phase_fns)")
            continue
        t = {k: timed(f) for k, f in phases(X, y, B).items()}
        print(f"{B:8d} {step:8.1f} " + " ".join(f"{t.get(k, float('nan')):8.1f}" for k in ("fwd", "bwd", "reduce")) + f" {step_eager:8.1f}")
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
