import numpy as np, difflib
from synapseml_amd.core import DataFrame
from synapseml_amd.lightgbm import LightGBMClassifier
from synapseml_amd.parallel.runtime import run_partitions
import sys; sys.path.insert(0,'tests')
from test_distributed_cpu import _ModelText
if __name__ == '__main__':
    rng = np.random.default_rng(5)
    n = 8000
    X = rng.standard_normal((n, 7))
    y = (X[:, 0] + X[:, 1] * X[:, 2] - 0.5 * X[:, 3] > 0).astype(float)
    kw = dict(deviceType="cpu", numIterations=6, numThreads=2)
    base = LightGBMClassifier(**kw)
    one = base.fit(DataFrame({"features": X, "label": y})).getNativeModel().split("parameters:")[0]
    ref = base._last_reference
    df = DataFrame({"features": X, "label": y}, num_partitions=2)
    txt = run_partitions(_ModelText(LightGBMClassifier(referenceDataset=ref, **kw)), df, num_workers=2)[0]
    d = list(difflib.unified_diff(one.splitlines(), txt.splitlines(), lineterm='', n=0))
    print("\n".join(x[:300] for x in d[:30]))
    