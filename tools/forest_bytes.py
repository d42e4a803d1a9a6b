#!/usr/bin/env python3
"""Per-level histogram wire volume of the data-parallel forest: grows the
forest of ``bench.py --config rf9`` (or ``rf``) on one device, reads the node count and the largest
node weight of every level from the fitted arrays, and prints what one rank puts on the wire per
level under the owner reduction (reduce-scatter of the per-node histogram store):

* r3 (``HAR_TREE_DP_BOUND=1``): the store sized by the host bound min(2^d T, T N), fp32;
* r4: the store sized by the level's real node count (one 16-byte read per level), padded to a
  multiple of P, fp16 when every count is exactly representable (largest node weight <= 2048).

    python tools/forest_bytes.py [rf9|rf] [--rows-per-gpu 60000] [--world 8] [--trees N] [--depth 10]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="rf9", choices=["rf9", "rf"])
    ap.add_argument("--rows-per-gpu", type=int, default=60000)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--trees", type=int, default=0)
    ap.add_argument("--depth", type=int, default=10)
    args = ap.parse_args()
    import bench  # noqa: E402  (the bench's featurizer and stream spec)
    from har.data.synth import StreamSpec
    from har.models.tree import RandomForestClassifier, subset_size
    from har.ops import tree as T

    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    nine = args.config == "rf9"
    K = 12 if nine else 6
    spec = StreamSpec(num_classes=K, axes=9 if nine else 3, hz=50.0 if nine else 20.0, window=500 if nine else 200,
                      seed=2018)
    n_all = args.rows_per_gpu * args.world
    X, y = bench._featurized(n_all, spec, dev, first_window=0)
    if not nine:
        X = X[:, :bench.N_FEATURES].contiguous()
    Tn = args.trees or (500 if nine else 100)
    F = X.shape[1]
    m = subset_size("auto", F, Tn)
    est = RandomForestClassifier(numTrees=Tn, maxDepth=args.depth, maxBins=32, seed=7, device=dev)
    thr = T.thresholds_for(X, 32, seed=7)
    model = est.fit_tensors(X, y, K, thresholds=thr)
    a = model.arrs
    feat, left, right = a.feature.cpu().numpy(), a.left.cpu().numpy(), a.right.cpu().numpy()
    st = a.stats.double().cpu().numpy()
    weight = st.sum(2)
    gini = 1.0 - ((st / np.maximum(weight, 1e-300)[:, :, None]) ** 2).sum(2)
    # depth of every node by a walk from the roots; a level's candidates (what its collectives carry)
    # = its split nodes plus the impure leaves of weight >= 2 that the split search rejected
    per_level = {}
    for t in range(Tn):
        stack = [(0, 0)]
        while stack:
            n, d = stack.pop()
            split = feat[t, n] >= 0
            if split or (d < args.depth and gini[t, n] > 1e-12 and weight[t, n] >= 2):
                c, w, pk = per_level.get(d, (0, 0.0, 0))
                # packed wire words of the node: m x bins x present classes, fields by node weight
                kp = int((st[t, n] > 0).sum())
                wt = float(weight[t, n])
                bw = 1 if wt < 256 else 2 if wt < 65536 else 4
                per_level[d] = (c + 1, max(w, wt), pk + -(-m * 32 * kp // (4 // bw)))
            if split:
                stack += [(left[t, n], d + 1), (right[t, n], d + 1)]
    P = args.world
    slot = m * 32 * K
    rows = []
    tot_old = tot_new = tot_pk = 0
    A_bound = Tn
    for d in range(args.depth):
        A, wmax, words = per_level.get(d, (0, 0.0, 0))
        if A == 0:
            break
        old = A_bound * slot * 4
        S = -(-A // P)
        narrow = wmax <= 2048
        new = P * S * slot * (2 if narrow else 4)
        pk = words * 4  # word-balanced owner rows: ~ the total words (+ < one node's words per rank)
        tot_old += old
        tot_new += new
        tot_pk += pk
        rows.append(f"| {d} | {A_bound} | {A} | {wmax:.0f} | {'fp16' if narrow else 'fp32'} | {old / 2**20:.1f} | "
                    f"{new / 2**20:.2f} | {pk / 2**20:.2f} | {old / max(pk, 1):.1f}x |")
        A_bound = min(2 * A_bound, Tn * n_all)
    print(f"# DP forest histogram wire volume per rank, {args.config}: {Tn} trees, depth {args.depth}, {K} classes, "
          f"{F} features (m = {m} per node), {args.rows_per_gpu} rows x {P} ranks\n")
    print("Level = split level d; bound = r3 store nodes min(2^d T, T N); real = the level's candidates in the fitted forest; "
          "max w = largest node weight at d (fp16 exact <= 2048). Bytes: one rank's reduce-scatter input. "
          "exact = the dense store sized by the real node count (fp16 when max w <= 2048, HAR_TREE_DP_WIRE=fp16); "
          "packed = present classes only, 8 / 16 / 32-bit integer fields by node weight (default).\n")
    print("| level | r3 bound nodes | real nodes | max w | exact wire | r3 MiB | exact MiB | packed MiB | r3 / packed |")
    print("|---:|---:|---:|---:|---|---:|---:|---:|---:|")
    print("\n".join(rows))
    print(f"\nper forest: r3 {tot_old / 2**20:.1f} MiB, exact {tot_new / 2**20:.2f} MiB ({tot_old / max(tot_new, 1):.1f}x less), "
          f"packed {tot_pk / 2**20:.2f} MiB ({tot_old / max(tot_pk, 1):.1f}x less); device {dev}")


if __name__ == "__main__":
    main()
