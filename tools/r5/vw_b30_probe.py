"""Bisect the b30 scoring accuracy: fused stage+learn vs staged-then-learned, and device vs host scoring."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from synapseml_amd.core.dataframe import DataFrame  # noqa: E402
from synapseml_amd.vw import VowpalWabbitClassifier  # noqa: E402

rng = np.random.default_rng(2)
X = rng.normal(size=(20000, 8))
y = (X[:, 0] - X[:, 1] > 0).astype(np.float64)
df = DataFrame({"features": X, "label": y})
for bits in (18, 30):
    for fused in ("1", "0"):
        os.environ["SML_VW_STAGE_LEARN"] = fused
        m = VowpalWabbitClassifier(deviceType="gpu", numBits=bits, labelConversion=True,
                                   passThroughArgs="--loss_function logistic", gpuBatchSize=256).fit(df)
        acc_dev = float(np.mean(m.transform(df)["prediction"] == y))
        h = m.copy()
        h.set("deviceType", "cpu")
        acc_host = float(np.mean(h.transform(df)["prediction"] == y)) if bits < 30 else float("nan")
        st = m.getPerformanceStatistics()
        print(f"bits={bits} fused={fused} acc_dev={acc_dev:.4f} acc_host={acc_host:.4f} "
              f"loss={float(st['averageLoss'][0]):.5f} model_bytes={len(m.getNativeModel())}", flush=True)
