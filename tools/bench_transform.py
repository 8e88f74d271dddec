#!/usr/bin/env python3
"""LightGBMClassificationModel.transform throughput (batch scoring, K9) at the headline shape: a 100-tree,
31-leaf model trained on the 11M x 28 Higgs-shape data of bench.py, scoring the same float32 DataFrame
(rawPrediction + probability + prediction columns). One step = one transform of the whole partition:
chunked pinned upload of the float32 rows, one device ensemble pass, probabilities from the raw scores.
Prints one JSON line (rows/s). Synthetic data."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=11_000_000)
    ap.add_argument("--features", type=int, default=28)
    ap.add_argument("--iterations", type=int, default=100)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    import torch

    from bench import higgs_like
    from synapseml_amd.core.dataframe import DataFrame
    from synapseml_amd.lightgbm import LightGBMClassifier

    X, y = higgs_like(args.rows, args.features, seed=1234)
    df = DataFrame({"features": X, "label": y})
    model = LightGBMClassifier(numIterations=args.iterations, numLeaves=31, deviceType="gpu").fit(df)
    for _ in range(args.warmup):
        out = model.transform(df)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = model.transform(df)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    host = model.getModel().native.predict(np.ascontiguousarray(X[:20000], np.float64), 1, 0, -1)[:, 0]
    err = float(np.max(np.abs(out["probability"][:20000, 1] - host)))
    print(json.dumps({"bench": "lightgbm_transform", "metric": "rows/sec LightGBMClassificationModel.transform",
                      "value": round(args.rows * args.steps / el, 1), "ms_per_transform": round(el / args.steps * 1e3, 2),
                      "rows": args.rows, "features": args.features, "trees": args.iterations, "input_dtype": "float32",
                      "outputs": "rawPrediction, probability, prediction", "max_abs_prob_err_vs_host": err,
                      "data": "synthetic Higgs-shape (bench.py)"}), flush=True)


if __name__ == "__main__":
    main()
