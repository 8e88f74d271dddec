"""Causal inference (reference: core/.../causal/{DoubleMLEstimator,
OrthoForestDMLEstimator, DiffInDiffEstimator, SyntheticControlEstimator,
SyntheticDiffInDiffEstimator, ResidualTransformer, opt/MirrorDescent,
opt/ConstrainedLeastSquare}.scala).

* DoubleML: cross-fitted residual-on-residual ATE, repeated ``maxIter``
  times over random sample splits; CI from percentiles, p-value from a
  one-sample t-test of the raw effects.
* OrthoForestDML: residualise, then a forest of regression trees (native
  GBDT engine, rf mode) on the heterogeneity features fits the local effect
  with target ỹ/t̃ and weights t̃²; per-row effect = mean over trees, bounds
  from tree quantiles.
* DiffInDiff: OLS on y ~ 1 + treat + post + treat·post (weighted).
* SyntheticControl / SyntheticDiffInDiff: simplex-constrained least squares
  (exponentiated-gradient mirror descent) for unit (and time) weights, then
  a weighted difference-in-differences."""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from ..core.contracts import HasFeaturesCol, HasWeightCol
from ..core.dataframe import DataFrame
from ..core.linalg import DenseVector, as_matrix
from ..core.params import Param, Params, TypeConverters as T
from ..core.pipeline import Estimator, Model, Transformer


def _obj(values) -> np.ndarray:
    arr = np.empty(len(values), dtype=object)
    for i, v in enumerate(values):
        arr[i] = v
    return arr


class ResidualTransformer(Transformer):
    observedCol = Param("observed data (label column)", "label", T.toString)
    predictedCol = Param("predicted data (prediction or probability columns)", "prediction", T.toString)
    outputCol = Param("output column name", "residual", T.toString)
    classIndex = Param("The index of the class to compute residual for classification outputs", 1, T.toInt)

    def _transform(self, df):
        obs = np.asarray(df[self.getObservedCol()], np.float64)
        pred = df[self.getPredictedCol()]
        if pred.ndim == 2:
            p = pred[:, self.getClassIndex()].astype(np.float64)
        elif pred.dtype == object:
            p = np.asarray([np.asarray(v.toArray() if hasattr(v, "toArray") else v)[self.getClassIndex()]
                            for v in pred], dtype=np.float64)
        else:
            p = pred.astype(np.float64)
        return df.withColumn(self.getOutputCol(), obs - p)


class OrthoForestVariableTransformer(Transformer):
    """Per-row target and weight of the orthogonal forest: outcome residual / treatment residual and
    treatment residual squared (reference: causal/OrthoForestVariableTransformer.scala:23-88)."""

    treatmentResidualCol = Param("Treatment Residual Col", "TResid", T.toString)
    outcomeResidualCol = Param("Outcome Residual Col", "OResid", T.toString)
    outputCol = Param("The name of the output column", "_tmp_tsOutcome", T.toString)
    weightsCol = Param("Weights Col", "_tmp_twOutcome", T.toString)

    def _transform(self, df):
        cols = {}
        for name in (self.getTreatmentResidualCol(), self.getOutcomeResidualCol()):
            c = df[name]
            if not np.issubdtype(c.dtype, np.floating):
                raise TypeError(f"{name} must be of type double, got {c.dtype}")
            cols[name] = c.astype(np.float64)
        t, o = cols[self.getTreatmentResidualCol()], cols[self.getOutcomeResidualCol()]
        with np.errstate(divide="ignore", invalid="ignore"):
            ratio = o / t
        return df.withColumn(self.getOutputCol(), ratio).withColumn(self.getWeightsCol(), t * t)


class _DMLParams(HasFeaturesCol, HasWeightCol):
    treatmentCol = Param("treatment column", "treatment", T.toString)
    outcomeCol = Param("outcome column", "outcome", T.toString)
    treatmentModel = Param("treatment model to run", None, complex=True)
    outcomeModel = Param("outcome model to run", None, complex=True)
    maxIter = Param("maximum number of iterations", 1, T.toInt)
    sampleSplitRatio = Param("Sample split ratio for cross-fitting", [0.5, 0.5], T.toListFloat)
    confidenceLevel = Param("confidence level, default value is 0.975", 0.975, T.toFloat)
    parallelism = Param("the number of threads to use when running parallel algorithms", 10, T.toInt)

    def _predict(self, model, df, label: str) -> np.ndarray:
        est = model.copy()
        for p, v in (("labelCol", label), ("featuresCol", self.getFeaturesCol())):
            if est.hasParam(p):
                est.set(p, v)
        fitted = est.fit(df)
        return fitted

    def _residuals(self, train: DataFrame, test: DataFrame, rng=None):
        tcol, ycol = self.getTreatmentCol(), self.getOutcomeCol()
        tm = self._predict(self.getTreatmentModel(), train, tcol)
        om = self._predict(self.getOutcomeModel(), train, ycol)
        to = tm.transform(test)
        oo = om.transform(test)
        t_obs = np.asarray(test[tcol], np.float64)
        y_obs = np.asarray(test[ycol], np.float64)
        if "probability" in to.columns and to["probability"].ndim == 2:
            t_hat = to["probability"][:, 1]
        else:
            t_hat = np.asarray(to["prediction"], np.float64)
        y_hat = np.asarray(oo["prediction"], np.float64) if "prediction" in oo.columns else \
            np.asarray(oo["probability"][:, 1])
        return t_obs - t_hat, y_obs - y_hat


class DoubleMLModel(Model, _DMLParams):
    rawTreatmentEffects = Param("raw treatment effect results for all iterations", [], T.toListFloat)

    def getAvgTreatmentEffect(self) -> float:  # noqa: N802
        v = self.getRawTreatmentEffects()
        return float(np.mean(v))

    def getPValue(self) -> float:  # noqa: N802
        from scipy import stats

        v = np.asarray(self.getRawTreatmentEffects())
        if len(v) < 2 or np.std(v) == 0:
            return 0.0 if abs(np.mean(v)) > 0 else 1.0
        return float(stats.ttest_1samp(v, 0.0).pvalue)

    def getConfidenceInterval(self) -> List[float]:  # noqa: N802
        v = np.asarray(self.getRawTreatmentEffects())
        cl = self.getConfidenceLevel()
        return [float(np.percentile(v, 100 * (1 - cl))), float(np.percentile(v, 100 * cl))]

    def _transform(self, df):
        return df


class DoubleMLEstimator(Estimator, _DMLParams):
    def _fit(self, df):
        ratio = np.asarray(self.getSampleSplitRatio(), float)
        ratio = ratio / ratio.sum()
        effects = []
        for it in range(self.getMaxIter()):
            a, b = df.randomSplit(list(ratio), seed=it)
            num = den = 0.0
            for tr, te in ((a, b), (b, a)):
                tres, yres = self._residuals(tr, te)
                num += float(np.sum(tres * yres))
                den += float(np.sum(tres * tres))
            effects.append(num / den if den else 0.0)
        m = DoubleMLModel(treatmentCol=self.getTreatmentCol(), outcomeCol=self.getOutcomeCol(),
                          confidenceLevel=self.getConfidenceLevel(), rawTreatmentEffects=effects)
        return m


class OrthoForestDMLModel(Model, _DMLParams):
    heterogeneityVecCol = Param("Vector to divide the treatment by", "X", T.toString)
    outputCol = Param("output column", "EffectAverage", T.toString)
    outputLowCol = Param("output column", "EffectLowerBound", T.toString)
    outputHighCol = Param("output column", "EffectUpperBound", T.toString)
    forest = Param("fitted per-tree effect models", None, complex=True)

    def _transform(self, df):
        X = as_matrix(df[self.getHeterogeneityVecCol()])
        tmp = DataFrame({"features": X})
        preds = np.stack([np.asarray(t.transform(tmp)["prediction"], np.float64) for t in self.getForest()], 1)
        cl = self.getConfidenceLevel()
        return (df.withColumn(self.getOutputCol(), preds.mean(1))
                .withColumn(self.getOutputLowCol(), np.percentile(preds, 100 * (1 - cl), axis=1))
                .withColumn(self.getOutputHighCol(), np.percentile(preds, 100 * cl, axis=1)))


class OrthoForestDMLEstimator(Estimator, _DMLParams):
    heterogeneityVecCol = Param("Vector to divide the treatment by", "X", T.toString)
    confounderVecCol = Param("Confounders to control for", "XW", T.toString)
    numTrees = Param("Number of trees", 20, T.toInt)
    maxDepth = Param("Max Depth of Tree", 5, T.toInt)
    minSamplesLeaf = Param("Max Depth of Tree", 10, T.toInt)
    treatmentResidualCol = Param("Treatment Residual Column", "TResid", T.toString)
    outcomeResidualCol = Param("Outcome Residual Column", "OResid", T.toString)
    outputCol = Param("output column", "EffectAverage", T.toString)
    outputLowCol = Param("output column", "EffectLowerBound", T.toString)
    outputHighCol = Param("output column", "EffectUpperBound", T.toString)

    def _fit(self, df):
        from ..models import DecisionTreeRegressor

        feat = self.getFeaturesCol()
        work = df.withColumn(feat, as_matrix(df[self.getConfounderVecCol()]))
        a, b = work.randomSplit([0.5, 0.5], seed=0)
        parts = []
        for tr, te in ((a, b), (b, a)):
            tres, yres = self._residuals(tr, te)
            parts.append((te, tres, yres))
        X = np.concatenate([as_matrix(p[0][self.getHeterogeneityVecCol()]) for p in parts])
        tres = np.concatenate([p[1] for p in parts])
        yres = np.concatenate([p[2] for p in parts])
        safe = np.where(np.abs(tres) < 1e-6, np.sign(tres + 1e-12) * 1e-6, tres)
        tr_col, or_col = self.getTreatmentResidualCol(), self.getOutcomeResidualCol()
        vt = OrthoForestVariableTransformer(treatmentResidualCol=tr_col, outcomeResidualCol=or_col).transform(
            DataFrame({tr_col: safe, or_col: yres}))
        target = vt["_tmp_tsOutcome"]
        wts = tres * tres
        rng = np.random.default_rng(0)
        forest = []
        for t in range(self.getNumTrees()):
            idx = rng.choice(len(target), size=len(target) // 2, replace=False)
            d = DataFrame({"features": X[idx], "label": target[idx], "w": wts[idx]})
            forest.append(DecisionTreeRegressor(maxDepth=self.getMaxDepth(), minInstancesPerNode=self.getMinSamplesLeaf(),
                                                weightCol="w", seed=t, deviceType="cpu").fit(d))
        m = OrthoForestDMLModel(heterogeneityVecCol=self.getHeterogeneityVecCol(), outputCol=self.getOutputCol(),
                                outputLowCol=self.getOutputLowCol(), outputHighCol=self.getOutputHighCol(),
                                confidenceLevel=self.getConfidenceLevel())
        return m.set("forest", forest)


# ---------------------------------------------------------------------- difference in differences
@dataclass
class DiffInDiffSummary:
    treatmentEffect: float  # noqa: N815
    standardError: float  # noqa: N815
    timeWeights: Optional[np.ndarray] = None  # noqa: N815
    unitWeights: Optional[np.ndarray] = None  # noqa: N815
    timeIntercept: Optional[float] = None  # noqa: N815
    unitIntercept: Optional[float] = None  # noqa: N815
    lossHistoryTimeWeights: Optional[List[float]] = None  # noqa: N815
    lossHistoryUnitWeights: Optional[List[float]] = None  # noqa: N815


class _DiDParams(Params):
    treatmentCol = Param("treatment column", "treatment", T.toString)
    postTreatmentCol = Param("post treatment indicator column", "postTreatment", T.toString)
    outcomeCol = Param("outcome column", "outcome", T.toString)


class DiffInDiffModel(Model, _DiDParams):
    timeCol = Param("time column", "time", T.toString)
    unitCol = Param("unit column", "unit", T.toString)
    # the synthetic estimators' index DataFrames: position in timeWeights / unitWeights <-> time / unit value
    # (BaseDiffInDiffEstimator.scala:105-119)
    timeIndex = Param("time index", None, complex=True)
    timeIndexCol = Param("time index column", "time_index", T.toString)
    unitIndex = Param("unit index", None, complex=True)
    unitIndexCol = Param("unit index column", "unit_index", T.toString)

    def getSummary(self) -> DiffInDiffSummary:  # noqa: N802
        if getattr(self, "_summary", None) is None:
            raise RuntimeError("No summary available for this DiffInDiffModel")
        return self._summary

    def getTimeWeights(self) -> Optional[DataFrame]:  # noqa: N802
        s = self.getSummary()
        if s.timeWeights is None:
            return None
        return DataFrame({self.getTimeCol(): self._time_index, "value": s.timeWeights})

    def getUnitWeights(self) -> Optional[DataFrame]:  # noqa: N802
        s = self.getSummary()
        if s.unitWeights is None:
            return None
        return DataFrame({self.getUnitCol(): self._unit_index, "value": s.unitWeights})

    def _transform(self, df):
        return df

    def _set_indexes(self, units, times) -> None:
        """timeIndex / unitIndex DataFrames (value, index) as the reference's synthetic estimators set them."""
        self._unit_index, self._time_index = _obj(units), _obj(times)
        self.set("timeIndex", DataFrame({self.getTimeCol(): _obj(times),
                                         self.getTimeIndexCol(): np.arange(len(times), dtype=np.int64)}))
        self.set("unitIndex", DataFrame({self.getUnitCol(): _obj(units),
                                         self.getUnitIndexCol(): np.arange(len(units), dtype=np.int64)}))


def _weighted_did(y, treat, post, w) -> DiffInDiffSummary:
    X = np.stack([np.ones_like(y), treat, post, treat * post], 1)
    sw = np.sqrt(w)
    beta, *_ = np.linalg.lstsq(X * sw[:, None], y * sw, rcond=None)
    res = y - X @ beta
    dof = max(1, len(y) - X.shape[1])
    sigma2 = float((w * res * res).sum() / dof)
    cov = sigma2 * np.linalg.pinv((X * w[:, None]).T @ X)
    return DiffInDiffSummary(float(beta[3]), float(np.sqrt(max(cov[3, 3], 0.0))))


class DiffInDiffEstimator(Estimator, _DiDParams):
    def _fit(self, df):
        y = np.asarray(df[self.getOutcomeCol()], np.float64)
        t = np.asarray(df[self.getTreatmentCol()], np.float64)
        p = np.asarray(df[self.getPostTreatmentCol()], np.float64)
        m = DiffInDiffModel(treatmentCol=self.getTreatmentCol(), postTreatmentCol=self.getPostTreatmentCol(),
                            outcomeCol=self.getOutcomeCol())
        m._summary = _weighted_did(y, t, p, np.ones_like(y))
        return m


def simplex_least_squares(A: np.ndarray, b: np.ndarray, zeta: float = 0.0, intercept: bool = True,
                          step: float = 0.5, max_iter: int = 500, tol: float = 1e-8, no_change: int = 0):
    """min ||A w + c - b||² + zeta² ||w||²  s.t. w ≥ 0, Σw = 1 (exponentiated-gradient mirror descent;
    reference opt/MirrorDescent.scala + ConstrainedLeastSquare.scala)."""
    n = A.shape[1]
    w = np.full(n, 1.0 / n)
    hist = []
    scale = max(1e-12, float(np.abs(A).max()) ** 2 * A.shape[0])
    stall = 0
    for it in range(max_iter):
        c = float(np.mean(b - A @ w)) if intercept else 0.0
        r = A @ w + c - b
        loss = float(r @ r + zeta ** 2 * w @ w)
        hist.append(loss)
        g = 2 * (A.T @ r + zeta ** 2 * w) / scale
        w = w * np.exp(-step * g)
        w = w / w.sum()
        if it > 0 and abs(hist[-2] - loss) < tol * max(1.0, abs(loss)):
            stall += 1
            if no_change <= 0 or stall >= no_change:
                break
        else:
            stall = 0
    c = float(np.mean(b - A @ w)) if intercept else 0.0
    return w, c, hist


class _SyntheticParams(_DiDParams):
    timeCol = Param("time column", "time", T.toString)
    unitCol = Param("unit column", "unit", T.toString)
    maxIter = Param("maximum number of iterations", 100, T.toInt)
    stepSize = Param("Step size to be used for each iteration of optimization", 1.0, T.toFloat)
    tol = Param("the convergence tolerance for iterative algorithms", 1e-3, T.toFloat)
    numIterNoChange = Param("Early termination when number of iterations without change reached.", None, T.toInt)
    localSolverThreshold = Param("threshold for collecting data on the driver", 1_000_000, T.toInt)
    epsilon = Param("threshold below which weights are treated as zero", 1e-10, T.toFloat)
    handleMissingOutcome = Param("How to handle missing outcomes: skip | zero | impute", "zero", T.toString)

    def _panel(self, df):
        units = sorted(set(df[self.getUnitCol()].tolist()), key=str)
        times = sorted(set(df[self.getTimeCol()].tolist()), key=lambda v: (str(type(v)), v))
        ui = {u: i for i, u in enumerate(units)}
        ti = {t: i for i, t in enumerate(times)}
        Y = np.full((len(units), len(times)), np.nan)
        treat = np.zeros(len(units))
        post = np.zeros(len(times))
        for u, t, y, tr, p in zip(df[self.getUnitCol()].tolist(), df[self.getTimeCol()].tolist(),
                                  df[self.getOutcomeCol()].tolist(), df[self.getTreatmentCol()].tolist(),
                                  df[self.getPostTreatmentCol()].tolist()):
            Y[ui[u], ti[t]] = y
            treat[ui[u]] = max(treat[ui[u]], float(tr))
            post[ti[t]] = max(post[ti[t]], float(p))
        if np.isnan(Y).any():
            mode = self.getHandleMissingOutcome()
            if mode == "zero":
                Y = np.nan_to_num(Y)
            elif mode == "impute":
                col_mean = np.nanmean(Y, axis=0)
                Y = np.where(np.isnan(Y), col_mean[None, :], Y)
        return units, times, Y, treat.astype(bool), post.astype(bool)

    def _did_from_weights(self, Y, treat, post, uw, tw):
        """Weighted DiD over the panel with unit/time weights (treated units and post periods weight 1/n)."""
        rows = []
        for i in range(Y.shape[0]):
            for j in range(Y.shape[1]):
                wu = uw[i] if not treat[i] else 1.0 / treat.sum()
                wt = tw[j] if not post[j] else 1.0 / post.sum()
                if wu * wt <= 0:
                    continue
                rows.append((Y[i, j], float(treat[i]), float(post[j]), wu * wt))
        y, t, p, w = map(np.asarray, zip(*rows))
        return _weighted_did(y, t, p, w)


class SyntheticControlEstimator(Estimator, _SyntheticParams):
    def _fit(self, df):
        units, times, Y, treat, post = self._panel(df)
        pre = ~post
        ctrl = ~treat
        target = Y[treat][:, pre].mean(0)
        uw, c, hist = simplex_least_squares(Y[ctrl][:, pre].T, target, 0.0, intercept=False,
                                            step=self.getStepSize(), max_iter=self.getMaxIter(), tol=self.getTol(),
                                            no_change=self.getNumIterNoChange() or 0)
        uw[uw < self.getEpsilon()] = 0.0
        full_uw = np.zeros(len(units))
        full_uw[ctrl] = uw / uw.sum()
        tw = np.full(len(times), 1.0 / max(1, pre.sum()))
        s = self._did_from_weights(Y, treat, post, full_uw, tw)
        s.unitWeights = full_uw
        s.lossHistoryUnitWeights = hist
        m = DiffInDiffModel(treatmentCol=self.getTreatmentCol(), postTreatmentCol=self.getPostTreatmentCol(),
                            outcomeCol=self.getOutcomeCol(), timeCol=self.getTimeCol(), unitCol=self.getUnitCol())
        m._summary = s
        m._set_indexes(units, times)
        return m


class SyntheticDiffInDiffEstimator(Estimator, _SyntheticParams):
    def _fit(self, df):
        units, times, Y, treat, post = self._panel(df)
        pre, ctrl = ~post, ~treat
        Yc = Y[ctrl]
        # time weights: pre-period combination matching the post-period mean of controls
        tw_pre, tc, th = simplex_least_squares(Yc[:, pre], Yc[:, post].mean(1), 0.0, intercept=True,
                                               step=self.getStepSize(), max_iter=self.getMaxIter(),
                                               tol=self.getTol(), no_change=self.getNumIterNoChange() or 0)
        # unit weights with the SDID regulariser zeta = (N_tr T_post)^(1/4) * sd(ΔY_controls)
        diffs = np.diff(Yc[:, pre], axis=1)
        zeta = (treat.sum() * post.sum()) ** 0.25 * (float(np.std(diffs)) if diffs.size else 0.0)
        uw_c, uc, uh = simplex_least_squares(Yc[:, pre].T, Y[treat][:, pre].mean(0), zeta, intercept=True,
                                             step=self.getStepSize(), max_iter=self.getMaxIter(),
                                             tol=self.getTol(), no_change=self.getNumIterNoChange() or 0)
        uw = np.zeros(len(units))
        uw[ctrl] = uw_c
        tw = np.zeros(len(times))
        tw[pre] = tw_pre
        s = self._did_from_weights(Y, treat, post, uw, tw)
        s.unitWeights, s.timeWeights = uw, tw
        s.unitIntercept, s.timeIntercept = uc, tc
        s.lossHistoryUnitWeights, s.lossHistoryTimeWeights = uh, th
        m = DiffInDiffModel(treatmentCol=self.getTreatmentCol(), postTreatmentCol=self.getPostTreatmentCol(),
                            outcomeCol=self.getOutcomeCol(), timeCol=self.getTimeCol(), unitCol=self.getUnitCol())
        m._summary = s
        m._set_indexes(units, times)
        return m


__all__ = ["DoubleMLEstimator", "DoubleMLModel", "OrthoForestDMLEstimator", "OrthoForestDMLModel",
           "DiffInDiffEstimator", "DiffInDiffModel", "DiffInDiffSummary", "SyntheticControlEstimator",
           "SyntheticDiffInDiffEstimator", "ResidualTransformer", "OrthoForestVariableTransformer",
           "simplex_least_squares"]
