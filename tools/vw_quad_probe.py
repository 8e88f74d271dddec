#!/usr/bin/env python3
"""Diagnostic: the -q ab regression of tests/test_vw_gpu.py::test_gpu_quadratic_interactions_syncs_and_initial_model
with its RMSEs printed (run with SML_VW_HOT_AGG=0/1 to compare the constant-slot aggregation), plus the same
fit scored on the device (_GpuScorer) against the exported host model."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from synapseml_amd.core.dataframe import DataFrame  # noqa: E402
from synapseml_amd.vw import VowpalWabbitRegressor  # noqa: E402

rng = np.random.default_rng(3)
n = 20000
A = rng.normal(size=(n, 3))
B = rng.normal(size=(n, 3))
y = A[:, 0] * B[:, 1] - 0.5 * A[:, 2] * B[:, 0] + 0.05 * rng.normal(size=n)
df = DataFrame({"a": A, "b": B, "label": y})
out = {"hot_agg": os.environ.get("SML_VW_HOT_AGG", "1")}
for name, extra in (("lin", {}), ("quad", {"passThroughArgs": "-q ab"}), ("quad_sync3", {"passThroughArgs": "-q ab", "numSyncsPerPass": 3})):
    for bs in (1, 256):
        m = VowpalWabbitRegressor(deviceType="gpu", featuresCol="a", additionalFeatures=["b"], numPasses=4,
                                  gpuBatchSize=bs, **extra).fit(df)
        p = m.transform(df)["prediction"]
        out[f"{name}_b{bs}"] = round(float(np.sqrt(np.mean((p - y) ** 2))), 4)
print(json.dumps(out), flush=True)
