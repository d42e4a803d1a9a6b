#!/usr/bin/env python3
"""Flagship benchmark: WISDM-shaped 6-class 3-layer MLP, bf16 MFMA, data parallel.

BASELINE.json config 3 ("WISDM 6-class 3-layer MLP bf16, DP all-reduce on
8xMI355X"), metric "windows/sec (whole node) + test accuracy".  One process per
GPU (``torch.distributed.run``), RCCL all-reduce of the flat gradient bucket
over xGMI each step, weak scaling (fixed per-GPU batch).

A step = forward + backward + all-reduce + Adam on ``--batch`` windows per GPU
(every window of the global batch goes through the full training step; nothing
is skipped inside the timed region).  Data: synthetic WISDM-shaped windows
(43 features = the WISDM transformed feature set width, 6 classes,
class-conditional Gaussians, generated on device) — there is no network for
the dataset; random-init weights.  After the timed region the model is scored
on held-out synthetic windows (``test_accuracy``).

``vs_baseline`` divides by the reference's published WISDM training throughput
(LogisticRegression, 3793 windows / 9.061 s = 418.6 windows/s, run A,
BASELINE.md §3) — the only train-windows/s number the reference publishes.

Usage: python bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

BASELINE_WINDOWS_PER_S = 418.6
METRIC = "windows/sec (whole node) + test accuracy on WISDM 6-class at 1/2/4/8 MI355X"
N_FEATURES = 43
N_CLASSES = 6
WINDOW_SAMPLES = 200  # 10 s @ 20 Hz (WISDM v1.1 transformed windows)


def synthetic_windows(n: int, seed: int, device, class_seed: int = 2018):
    """Class-conditional Gaussian windows: x = mu[y] + noise; mu shared by all ranks."""
    g = torch.Generator(device="cpu").manual_seed(class_seed)
    mu = torch.randn(N_CLASSES, N_FEATURES, generator=g) * 0.6
    prior = torch.tensor([2081, 1625, 632, 528, 306, 246], dtype=torch.float64)  # WISDM class mix
    gd = torch.Generator(device=device).manual_seed(seed)
    y = torch.multinomial(prior.to(device).float(), n, replacement=True, generator=gd)
    x = mu.to(device)[y] + torch.randn(n, N_FEATURES, device=device, generator=gd)
    return x, y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=65536, help="windows per GPU per step")
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--graph", type=int, default=1, help="capture the step in a HIP graph")
    ap.add_argument("--out", type=str, default="")
    args = ap.parse_args()

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from har.models.mlp import MLPEngine, pad_input_bf16
    from har.parallel import dist as hdist

    ctx = hdist.init(expected_world=args.gpus)
    dev = ctx.device
    rank, world = ctx.rank, ctx.world_size
    B = args.batch
    layers = [N_FEATURES, args.hidden, args.hidden, N_CLASSES]
    eng = MLPEngine(layers, B, dev, lr=args.lr, seed=1234, process_group=ctx.group, world_size=world)

    # resident per-rank training shard: 8 batches worth of windows
    n_local = B * 8
    X, y = synthetic_windows(n_local, seed=100 + rank, device=dev)
    Xin = pad_input_bf16(X, eng.layout.in_pad) if eng.native else X
    y32 = y.to(torch.int32).contiguous()
    nb = n_local // B
    global_batch = B * world

    def step(i):
        j = i % nb
        eng.train_step(Xin[j * B:(j + 1) * B], y32[j * B:(j + 1) * B], global_batch)

    graph = None
    if eng.native and args.graph:
        # warm the allocator / kernels on a side stream, then capture one step per batch slot
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for i in range(3):
                step(i)
        torch.cuda.current_stream().wait_stream(s)
        graphs = []
        for j in range(nb):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step(j)
            graphs.append(g)
        graph = graphs

    def run(i):
        if graph is not None:
            graph[i % nb].replay()
        else:
            step(i)

    for i in range(args.warmup):
        run(i)
    hdist.barrier(ctx)
    hdist.sync(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        run(i)
    hdist.sync(dev)
    hdist.barrier(ctx)
    elapsed = time.perf_counter() - t0
    elapsed = hdist.max_over_ranks(ctx, elapsed)
    ms = elapsed * 1e3 / args.steps
    value = global_batch * args.steps / elapsed

    # held-out accuracy (synthetic windows, rank-local; averaged)
    Xt, yt = synthetic_windows(65536, seed=999, device=dev)
    pred = torch.argmax(eng.logits(Xt), dim=1)
    acc = float((pred == yt).float().mean())
    acc = hdist.mean_over_ranks(ctx, acc)

    rec = {"metric": METRIC, "value": value, "unit": "windows/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": value / BASELINE_WINDOWS_PER_S, "dtype": "bf16",
           "data": "synthetic WISDM-shaped windows (43 features, 6 classes, class-conditional Gaussian); "
                   "random-init weights",
           "config": {"model": f"WISDM 6-class 3-layer MLP bf16 ({'-'.join(map(str, layers))})",
                      "global_batch": global_batch, "seq_len": WINDOW_SAMPLES, "parallelism": f"dp{world}"},
           "test_accuracy": acc, "test_accuracy_data": "held-out synthetic windows",
           "hip_graph": graph is not None, "device": torch.cuda.get_device_name(dev) if eng.native else "cpu"}
    if rank == 0:
        line = json.dumps(rec)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    hdist.shutdown(ctx)


if __name__ == "__main__":
    main()
