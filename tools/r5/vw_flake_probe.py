"""Repeat the GPU VW classifier quality fit (batch 256, 3 passes) with the staging pipeline on and off, and
the model scored on the device and on the host, to find which path loses accuracy intermittently."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from sklearn.metrics import roc_auc_score  # noqa: E402

from synapseml_amd.core.dataframe import DataFrame  # noqa: E402
from synapseml_amd.vw import VowpalWabbitClassifier  # noqa: E402


def binary(n=20000, d=20, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d))
    w = rng.normal(size=d)
    y = (X @ w + 0.3 * rng.normal(size=n) > 0).astype(np.float64)
    return DataFrame({"features": X, "label": y}), y


df, y = binary()
BATCH = int(sys.argv[2]) if len(sys.argv) > 2 else 256
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    for fused in ("1", "0"):
        os.environ["SML_VW_STAGE_LEARN"] = fused
        m = VowpalWabbitClassifier(deviceType="gpu", labelConversion=True, passThroughArgs="--loss_function logistic",
                                   numPasses=3, gpuBatchSize=BATCH).fit(df)
        a_dev = roc_auc_score(y, m.transform(df)["probability"][:, 1])
        h = m.copy()
        h.set("deviceType", "cpu")
        a_host = roc_auc_score(y, h.transform(df)["probability"][:, 1])
        st = m.getPerformanceStatistics()
        print(f"rep={rep} fused={fused} auc_dev={a_dev:.4f} auc_host={a_host:.4f} loss={float(st['averageLoss'][0]):.5f}",
              flush=True)
