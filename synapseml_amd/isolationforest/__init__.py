"""Isolation forest anomaly detection (reference:
core/.../isolationforest/IsolationForest.scala, which wraps LinkedIn's
isolation-forest; params and outputs follow that library: outlierScore =
2^(−E[h(x)] / c(ψ)), predictedLabel from a contamination-quantile threshold).

Trees are stored as flat arrays; scoring walks all (row, tree) pairs level by
level with vectorised gathers."""
from __future__ import annotations

import numpy as np

from ..core.contracts import HasFeaturesCol
from ..core.dataframe import DataFrame
from ..core.linalg import as_matrix
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Estimator, Model

EULER = 0.5772156649015329


def avg_path_length(n) -> np.ndarray:
    n = np.asarray(n, dtype=np.float64)
    out = np.zeros_like(n)
    big = n > 2
    out[big] = 2.0 * (np.log(n[big] - 1.0) + EULER) - 2.0 * (n[big] - 1.0) / n[big]
    out[n == 2] = 1.0
    return out


class _Params(HasFeaturesCol):
    numEstimators = Param("The number of trees in the ensemble.", 100, T.toInt)
    bootstrap = Param("If true, draw sample for each tree with replacement.", False, T.toBoolean)
    maxSamples = Param("The number of samples used to train each tree (<= 1.0: fraction of the data).", 256.0,
                       T.toFloat)
    maxFeatures = Param("The number of features used to train each tree (<= 1.0: fraction).", 1.0, T.toFloat)
    contamination = Param("The fraction of outliers in the training data set.", 0.0, T.toFloat)
    contaminationError = Param("The error allowed when calculating the threshold required to achieve the "
                               "specified contamination fraction.", 0.0, T.toFloat)
    randomSeed = Param("The seed used for the random number generator.", 1, T.toInt)
    predictionCol = Param("The column name of the predicted label.", "predictedLabel", T.toString)
    scoreCol = Param("The column name of the outlier score.", "outlierScore", T.toString)


class IsolationForestModel(Model, _Params):
    trees = Param("flattened isolation trees", None, complex=True)
    numSamples = Param("samples per tree", 256, T.toInt)
    outlierScoreThreshold = Param("score threshold for the predicted label", 0.5, T.toFloat)

    def getInnerModel(self):  # noqa: N802
        """the fitted forest itself (reference IsolationForestModel.getInnerModel returns the wrapped
        linkedin model; here the flattened trees live on this stage)"""
        return self

    def scores(self, X: np.ndarray) -> np.ndarray:
        feat, thr, left, right, size, fidx = self.getTrees()
        T_ = len(fidx)
        n = X.shape[0]
        depth = np.zeros((n, T_))
        for t in range(T_):
            f, th, l, r, sz = feat[t], thr[t], left[t], right[t], size[t]
            Xt = X[:, fidx[t]]
            node = np.zeros(n, dtype=np.int64)
            d = np.zeros(n)
            active = f[node] >= 0
            while active.any():
                nd = node[active]
                go_left = Xt[active, f[nd]] < th[nd]
                node[active] = np.where(go_left, l[nd], r[nd])
                d[active] += 1
                active = f[node] >= 0
            depth[:, t] = d + avg_path_length(sz[node])
        return 2.0 ** (-depth.mean(1) / avg_path_length([self.getNumSamples()])[0])

    def _transform(self, df):
        s = self.scores(as_matrix(df[self.getFeaturesCol()]))
        return df.withColumn(self.getScoreCol(), s).withColumn(
            self.getPredictionCol(), (s >= self.getOutlierScoreThreshold()).astype(np.float64))


class IsolationForest(Estimator, _Params):
    def _grow(self, X, rng, height_limit):
        feat, thr, left, right, size = [], [], [], [], []

        def build(idx, depth):
            me = len(feat)
            feat.append(-1)
            thr.append(0.0)
            left.append(-1)
            right.append(-1)
            size.append(len(idx))
            if depth >= height_limit or len(idx) <= 1:
                return me
            sub = X[idx]
            lo, hi = sub.min(0), sub.max(0)
            cand = np.nonzero(hi > lo)[0]
            if len(cand) == 0:
                return me
            f = int(rng.choice(cand))
            t = float(rng.uniform(lo[f], hi[f]))
            m = sub[:, f] < t
            feat[me], thr[me] = f, t
            left[me] = build(idx[m], depth + 1)
            right[me] = build(idx[~m], depth + 1)
            return me

        build(np.arange(X.shape[0]), 0)
        return (np.asarray(feat), np.asarray(thr), np.asarray(left), np.asarray(right), np.asarray(size, float))

    def _fit(self, df):
        X = as_matrix(df[self.getFeaturesCol()])
        n, d = X.shape
        rng = np.random.default_rng(self.getRandomSeed())
        ms = self.getMaxSamples()
        psi = int(ms * n) if ms <= 1.0 else int(min(ms, n))
        psi = max(2, min(psi, n))
        mf = self.getMaxFeatures()
        nf = int(mf * d) if mf <= 1.0 else int(min(mf, d))
        nf = max(1, nf)
        height = int(np.ceil(np.log2(psi)))
        trees = [[], [], [], [], [], []]
        for _ in range(self.getNumEstimators()):
            rows = rng.choice(n, size=psi, replace=self.getBootstrap())
            cols = np.sort(rng.choice(d, size=nf, replace=False))
            t = self._grow(X[np.ix_(rows, cols)], rng, height)
            for k in range(5):
                trees[k].append(t[k])
            trees[5].append(cols)
        m = IsolationForestModel(featuresCol=self.getFeaturesCol(), predictionCol=self.getPredictionCol(),
                                 scoreCol=self.getScoreCol(), numSamples=psi,
                                 contamination=self.getContamination(), numEstimators=self.getNumEstimators())
        m.set("trees", trees)
        c = self.getContamination()
        if c > 0:
            s = m.scores(X)
            m.set("outlierScoreThreshold", float(np.quantile(s, 1.0 - c)))
        return m


__all__ = ["IsolationForest", "IsolationForestModel", "avg_path_length"]
