#!/usr/bin/env python3
"""Same-host comparators for the headline (BASELINE.md "Same-host comparators"): the reference publishes no
throughput, so the GPU fit is put next to CPU learners on the SAME synthetic Higgs-shape data and the SAME
settings (100 iterations, 31 leaves, 255 bins, lr 0.1, min 20 rows per leaf, binary):

  * scikit-learn HistGradientBoostingClassifier (max_leaf_nodes=31, max_bins=255, learning_rate=0.1,
    max_iter=100, min_samples_leaf=20, early_stopping=False) - timed ``fit`` on the float32 matrix
  * this framework's own C++ CPU engine (``LightGBMClassifier(deviceType="cpu").fit``, all threads)
  * this framework's GPU engine (``deviceType="gpu"``), the number bench.py reports

Each line is one JSON record: rows/s = N_rows / fit wall seconds, plus the holdout AUC on the first rows.
Threads: OMP_NUM_THREADS (the GPU box gives a 1-GPU job 16 CPU threads).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import higgs_like  # noqa: E402


def _auc(y, p):
    from sklearn.metrics import roc_auc_score

    return float(roc_auc_score(y, p))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=11_000_000)
    ap.add_argument("--iterations", type=int, default=100)
    ap.add_argument("--which", default="gpu,cpu,sklearn")
    args = ap.parse_args()
    X, y = higgs_like(args.rows, 28, seed=1234)
    nh = min(200_000, args.rows)
    Xh, yh = X[:nh].astype(np.float64), y[:nh]
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    base = {"rows": args.rows, "features": 28, "iterations": args.iterations, "cpu_threads": threads,
            "data": "synthetic Higgs-shape (bench.higgs_like, seed 1234)"}
    for which in args.which.split(","):
        rec = dict(base, learner=which)
        if which in ("gpu", "cpu"):
            from synapseml_amd.core.dataframe import DataFrame
            from synapseml_amd.lightgbm import LightGBMClassifier

            if which == "gpu":
                import torch

                if not torch.cuda.is_available():
                    continue
            df = DataFrame({"features": X, "label": y})
            est = LightGBMClassifier(numIterations=args.iterations, learningRate=0.1, numLeaves=31, maxBin=255,
                                     binSampleCount=200000, minDataInLeaf=20, objective="binary",
                                     deviceType=which)
            # warm-up outside the clock: library / HIP module load, allocator (a small fit on CPU)
            est.fit(df if which == "gpu" else DataFrame({"features": X[:20000], "label": y[:20000]}))
            t0 = time.perf_counter()
            m = est.fit(df)
            dt = time.perf_counter() - t0
            p = m.getModel().score(Xh, raw=False, classification=True)[:, 1]
            rec.update(fit_s=round(dt, 3), rows_per_s=round(args.rows / dt, 1), holdout_auc=round(_auc(yh, p), 5),
                       learner="synapseml_amd LightGBMClassifier deviceType=" + which)
        elif which == "sklearn":
            from sklearn.ensemble import HistGradientBoostingClassifier

            clf = HistGradientBoostingClassifier(max_leaf_nodes=31, max_bins=255, learning_rate=0.1,
                                                 max_iter=args.iterations, min_samples_leaf=20,
                                                 early_stopping=False, random_state=0)
            t0 = time.perf_counter()
            clf.fit(X, y)
            dt = time.perf_counter() - t0
            p = clf.predict_proba(Xh)[:, 1]
            import sklearn

            rec.update(fit_s=round(dt, 3), rows_per_s=round(args.rows / dt, 1), holdout_auc=round(_auc(yh, p), 5),
                       learner=f"sklearn {sklearn.__version__} HistGradientBoostingClassifier")
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
