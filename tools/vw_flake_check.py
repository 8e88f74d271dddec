import sys, json
sys.path.insert(0, ".")
import numpy as np
from sklearn.metrics import roc_auc_score
from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.vw import VowpalWabbitClassifier
def _binary(n=20000, d=20, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d)); w = rng.normal(size=d)
    y = (X @ w + 0.3 * rng.normal(size=n) > 0).astype(np.float64)
    return DataFrame({"features": X, "label": y}), y
df, y = _binary()
aucs = []
for i in range(int(sys.argv[1])):
    m = VowpalWabbitClassifier(deviceType="gpu", labelConversion=True, passThroughArgs="--loss_function logistic", numPasses=3, gpuBatchSize=256).fit(df)
    aucs.append(round(roc_auc_score(y, m.transform(df)["probability"][:, 1]), 4))
print(json.dumps({"aucs": aucs}), flush=True)
