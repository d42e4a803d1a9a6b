#!/usr/bin/env python3
"""The reference suite's tree fits alone (DecisionTree depth 3, RandomForest 100 x depth 4 on the WISDM
reference encoding, Main/main.py:297,478), for a rocprofv3 kernel trace of just those fits.

usage: python tools/ref_tree_probe.py [--repeats 5] [--models dt,rf]
Prints per model the fit times (first eager, then graph capture / replays) and the accuracy."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeats", type=int, default=5)
    ap.add_argument("--models", default="dt,rf")
    ap.add_argument("--wisdm", default=os.path.join(ROOT, "tests", "data", "wisdm_data.csv"))
    a = ap.parse_args()
    import torch

    from har.suite import run_reference_suite

    r = run_reference_suite(torch.device("cuda:0"), a.wisdm, models=a.models.split(","), repeats=a.repeats, warmup=1)
    for name, m in r["models"].items():
        print(json.dumps({"model": name, "fit_ms_median": round(m["fit_s"] * 1e3, 4),
                          "fit_ms_every": [round(t * 1e3, 4) for t in m["fit_s_every"]],
                          "kinds": m["fit_kind_every"], "accuracy": m["accuracy"]}))


if __name__ == "__main__":
    main()
