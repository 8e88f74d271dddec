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


def commons_percentile(values, p: float) -> float:
    """Apache commons-math ``Percentile.evaluate(p)`` (default estimation: position p(n+1)/100 with linear
    interpolation, clamped to the sample range) - the estimator the reference's confidence intervals and
    BLB bounds use (DoubleMLEstimator.scala percentile, OrthoForestDMLEstimator.scala getBLBBounds)."""
    v = np.sort(np.asarray(values, np.float64))
    n = len(v)
    if n == 0:
        return float("nan")
    if n == 1:
        return float(v[0])
    pos = p * (n + 1) / 100.0
    if pos < 1:
        return float(v[0])
    if pos >= n:
        return float(v[-1])
    lo = int(np.floor(pos))
    return float(v[lo - 1] + (pos - lo) * (v[lo] - v[lo - 1]))


def _commons_percentile_rows(sorted_rows: np.ndarray, p: float) -> np.ndarray:
    """commons_percentile over each row of an already sorted (k, n) matrix"""
    n = sorted_rows.shape[1]
    if n == 1:
        return sorted_rows[:, 0].copy()
    pos = p * (n + 1) / 100.0
    if pos < 1:
        return sorted_rows[:, 0].copy()
    if pos >= n:
        return sorted_rows[:, -1].copy()
    lo = int(np.floor(pos))
    return sorted_rows[:, lo - 1] + (pos - lo) * (sorted_rows[:, lo] - sorted_rows[:, lo - 1])


def _model_kind(model) -> str:
    """'binary' for probabilistic classifiers, 'continuous' for regressors (reference DoubleMLParams
    ensureSupportedEstimator: anything else is refused)"""
    if model.hasParam("probabilityCol"):
        return "binary"
    if model.hasParam("predictionCol"):
        return "continuous"
    raise TypeError(f"DoubleMLEstimator only supports regressors and probabilistic classifiers as treatment or "
                    f"outcome model types, but got {type(model).__name__}")


def _check_col_for_model(col: np.ndarray, name: str, model) -> None:
    """Column type vs model type (reference DoubleMLEstimator.validateColTypeWithModel)"""
    kind = _model_kind(model)
    if col.dtype == bool:
        if kind == "continuous":
            raise TypeError(f"column '{name}' in dataset is boolean data type, but you set to use a regression "
                            "model for it.")
    elif np.issubdtype(col.dtype, np.integer):
        if kind == "binary" and not np.isin(col, (0, 1)).all():
            raise ValueError(f"column '{name}' in dataset is integer data type and you set to use a classification "
                             "model for it, its all values must be either 0 or 1, but it has other values.")
    elif np.issubdtype(col.dtype, np.floating):
        if kind == "binary":
            raise TypeError(f"column '{name}' in dataset is double or long data type, but you set to use a "
                            "classification model for it.")
    else:
        raise TypeError(f"column '{name}' must be of type DoubleType, LongType, IntegerType or BooleanType "
                        f"but got {col.dtype}")


def _ols_slope(x: np.ndarray, y: np.ndarray) -> float:
    """slope of a gaussian / identity GLM y ~ 1 + x (the reference's GeneralizedLinearRegression with
    fitIntercept=true on the residuals)"""
    xc = x - x.mean()
    den = float(xc @ xc)
    return float(xc @ (y - y.mean())) / den if den > 0 else 0.0


class _DMLParams(HasFeaturesCol, HasWeightCol):
    treatmentCol = Param("treatment column", "treatment", T.toString)
    outcomeCol = Param("outcome column", "outcome", T.toString)
    treatmentModel = Param("treatment model to run", None, complex=True)
    outcomeModel = Param("outcome model to run", None, complex=True)
    maxIter = Param("maximum number of iterations", 1, T.toInt)
    sampleSplitRatio = Param("Sample split ratio for cross-fitting", [0.5, 0.5], T.toListFloat)
    confidenceLevel = Param("confidence level, default value is 0.975", 0.975, T.toFloat)
    parallelism = Param("the number of threads to use when running parallel algorithms", 10, T.toInt)

    def _models(self):
        """(treatment, outcome) estimators; the reference defaults both to LogisticRegression"""
        from ..models import LogisticRegression

        tm = self.getTreatmentModel() or LogisticRegression()
        om = self.getOutcomeModel() or LogisticRegression()
        return tm, om

    def _fit_nuisance(self, model, df, label: str, features: str):
        est = model.copy()
        for p, v in (("labelCol", label), ("featuresCol", features)):
            if est.hasParam(p):
                est.set(p, v)
        if self.isSet("weightCol") and self.getWeightCol():
            if not est.hasParam("weightCol"):
                raise ValueError(f"The selected {label} model does not support sample weight, but the weightCol "
                                 f"parameter was set. Please select a model that supports sample weight.")
            est.set("weightCol", self.getWeightCol())
        return est.fit(df)

    @staticmethod
    def _prediction(model, out) -> np.ndarray:
        """P(class 1) of a probabilistic classifier, else the prediction (ResidualTransformer classIndex 1)"""
        if model.hasParam("probabilityCol"):
            col = out[model.getProbabilityCol() if hasattr(model, "getProbabilityCol") else "probability"]
            return np.asarray(col[:, 1] if getattr(col, "ndim", 1) == 2 else
                              [np.asarray(v.toArray() if hasattr(v, "toArray") else v)[1] for v in col], np.float64)
        return np.asarray(out[model.getPredictionCol() if hasattr(model, "getPredictionCol") else "prediction"],
                          np.float64)

    def _residuals(self, train: DataFrame, test: DataFrame, features: Optional[str] = None):
        """treatment and outcome nuisance models fit on `train`, residuals observed - predicted on `test`"""
        tcol, ycol = self.getTreatmentCol(), self.getOutcomeCol()
        feats = features or self.getFeaturesCol()
        tmodel, omodel = self._models()
        tm = self._fit_nuisance(tmodel, train, tcol, feats)
        om = self._fit_nuisance(omodel, train, ycol, feats)
        t_hat = self._prediction(tmodel, tm.transform(test))
        y_hat = self._prediction(omodel, om.transform(test))
        return np.asarray(test[tcol], np.float64) - t_hat, np.asarray(test[ycol], np.float64) - y_hat


class DoubleMLModel(Model, _DMLParams):
    rawTreatmentEffects = Param("raw treatment effect results for all iterations", [], T.toListFloat)

    def getAvgTreatmentEffect(self) -> float:  # noqa: N802
        v = self.getRawTreatmentEffects()
        return float(np.sum(v) / len(v))

    def getPValue(self) -> float:  # noqa: N802
        """two-sided one-sample t-test of the raw effects against 0 (commons-math TTest.tTest(0, values);
        it needs at least two iterations)"""
        from scipy import stats

        v = np.asarray(self.getRawTreatmentEffects(), np.float64)
        if len(v) < 2:
            raise ValueError("the p-value needs maxIter >= 2 (a t-test of the per-iteration effects)")
        if np.std(v) == 0:
            return 0.0 if abs(np.mean(v)) > 0 else 1.0
        return float(stats.ttest_1samp(v, 0.0).pvalue)

    def getConfidenceInterval(self) -> List[float]:  # noqa: N802
        v = self.getRawTreatmentEffects()
        cl = self.getConfidenceLevel()
        return [commons_percentile(v, 100 * (1 - cl)), commons_percentile(v, 100 * cl)]

    def _transform(self, df):
        return df


class DoubleMLEstimator(Estimator, _DMLParams):
    """Double machine learning ATE (reference core/.../causal/DoubleMLEstimator.scala:63-268): each of
    ``maxIter`` iterations (run on ``parallelism`` threads) redraws the data with replacement (not when
    maxIter == 1), splits it by ``sampleSplitRatio``, fits the treatment / outcome nuisance models on one
    half and takes residuals on the other, both ways, and averages the two slopes of outcome residual on
    treatment residual (GLM with intercept). Failed iterations are dropped; all failing is an error."""

    def _one_ate(self, df: DataFrame, it: int) -> float:
        work = df if self.getMaxIter() == 1 else df.sample(1.0, seed=it, withReplacement=True)
        ratio = np.asarray(self.getSampleSplitRatio(), float)
        a, b = work.randomSplit(list(ratio / ratio.sum()), seed=it)
        slopes = []
        for tr, te in ((a, b), (b, a)):
            tres, yres = self._residuals(tr, te)
            ok = np.isfinite(tres) & np.isfinite(yres)  # VectorAssembler handleInvalid=skip
            slopes.append(_ols_slope(tres[ok], yres[ok]))
        return float(sum(slopes) / len(slopes))

    def _fit(self, df):
        if self.getMaxIter() <= 0:
            raise ValueError("maxIter should be larger than 0!")
        tmodel, omodel = self._models()
        _check_col_for_model(np.asarray(df[self.getTreatmentCol()]), self.getTreatmentCol(), tmodel)
        _check_col_for_model(np.asarray(df[self.getOutcomeCol()]), self.getOutcomeCol(), omodel)
        from concurrent.futures import ThreadPoolExecutor

        def run(it):
            try:
                return self._one_ate(df, it)
            except Exception as e:  # reference: logged and skipped
                import logging

                logging.getLogger(__name__).warning("ATE calculation failed on iteration %d: %s", it, e)
                return None

        with ThreadPoolExecutor(max_workers=max(1, min(self.getParallelism(), self.getMaxIter()))) as ex:
            ates = [a for a in ex.map(run, range(1, self.getMaxIter() + 1)) if a is not None]
        if not ates:
            raise RuntimeError("ATE calculation failed on all iterations. Please check the log for details.")
        m = DoubleMLModel(rawTreatmentEffects=ates)
        for name in ("treatmentCol", "outcomeCol", "confidenceLevel", "maxIter", "sampleSplitRatio", "parallelism",
                     "featuresCol"):
            m.set(name, self.getOrDefault(name))
        return m


class OrthoForestDMLModel(Model, _DMLParams):
    heterogeneityVecCol = Param("Vector to divide the treatment by", "X", T.toString)
    outputCol = Param("output column", "EffectAverage", T.toString)
    outputLowCol = Param("output column", "EffectLowerBound", T.toString)
    outputHighCol = Param("output column", "EffectUpperBound", T.toString)
    forest = Param("fitted per-tree effect models", None, complex=True)

    def _blb_bounds(self, preds: np.ndarray, rng) -> np.ndarray:
        """Bag of little bootstraps over each row's per-tree effects (reference getBLBBounds): groups of
        ceil(sqrt(n)) trees, 100 draws with replacement per group, per-group lower / median / upper
        percentile, averaged over the groups -> (rows, 3)"""
        rows, n = preds.shape
        b = int(np.ceil(np.sqrt(n)))
        cl = self.getConfidenceLevel()
        acc = np.zeros((rows, 3))
        groups = [(s, min(n, s + b)) for s in range(0, n, b)]
        for s, e in groups:
            draws = preds[:, s:e][np.arange(rows)[:, None], rng.integers(0, e - s, size=(rows, 100))]
            draws.sort(axis=1)
            acc[:, 0] += _commons_percentile_rows(draws, 100 * (1 - cl))
            acc[:, 1] += _commons_percentile_rows(draws, 50)
            acc[:, 2] += _commons_percentile_rows(draws, 100 * cl)
        return acc / len(groups)

    def _transform(self, df):
        X = as_matrix(df[self.getHeterogeneityVecCol()])
        tmp = DataFrame({"features": X})
        preds = np.stack([np.asarray(t.transform(tmp)["prediction"], np.float64) for t in self.getForest()], 1)
        lo_med_hi = self._blb_bounds(preds, np.random.default_rng(0))
        return (df.withColumn(self.getOutputLowCol(), lo_med_hi[:, 0])
                .withColumn(self.getOutputCol(), lo_med_hi[:, 1])
                .withColumn(self.getOutputHighCol(), lo_med_hi[:, 2]))


class OrthoForestDMLEstimator(Estimator, _DMLParams):
    """Orthogonal random forest DML (reference OrthoForestDMLEstimator.scala:30-160): cross-fitted treatment /
    outcome residuals on the confounders, target = outcome residual / treatment residual with weight =
    treatment residual^2 (OrthoForestVariableTransformer), a random forest of ``numTrees`` depth-``maxDepth``
    trees on the heterogeneity features per residual half; the model's per-row effect and bounds come from a
    bag of little bootstraps over all trees."""

    heterogeneityVecCol = Param("Vector to divide the treatment by", "X", T.toString)
    confounderVecCol = Param("Confounders to control for", "XW", T.toString)
    numTrees = Param("Number of trees", 20, T.toInt)
    maxDepth = Param("Max Depth of Tree", 5, T.toInt)
    minSamplesLeaf = Param("Max Depth of Tree", 10, T.toInt)
    treatmentResidualCol = Param("Treatment Residual Column", "TreatmentResidual", T.toString)
    outcomeResidualCol = Param("Outcome Residual Column", "OutcomeResidual", T.toString)
    outputCol = Param("output column", "EffectAverage", T.toString)
    outputLowCol = Param("output column", "EffectLowerBound", T.toString)
    outputHighCol = Param("output column", "EffectUpperBound", T.toString)

    def _models(self):
        from ..models import GBTRegressor

        tm = self.getTreatmentModel() or GBTRegressor(seed=0)
        om = self.getOutcomeModel() or GBTRegressor(seed=0)
        return tm, om

    def _fit(self, df):
        from ..models import DecisionTreeRegressor

        if self.getNumTrees() <= 0:
            raise ValueError("You need at least one tree in a forest")
        tcol = df[self.getTreatmentCol()]
        if not np.issubdtype(np.asarray(tcol).dtype, np.floating):
            raise TypeError(f"TreatmentCol must be of type DoubleType but got {np.asarray(tcol).dtype}")
        ratio = np.asarray(self.getSampleSplitRatio(), float)
        a, b = df.randomSplit(list(ratio / ratio.sum()), seed=0)
        tr_col, or_col = self.getTreatmentResidualCol(), self.getOutcomeResidualCol()
        forest = []
        for half, (tr, te) in enumerate(((a, b), (b, a))):
            tres, yres = self._residuals(tr, te, features=self.getConfounderVecCol())
            vt = OrthoForestVariableTransformer(treatmentResidualCol=tr_col, outcomeResidualCol=or_col).transform(
                DataFrame({tr_col: tres, or_col: yres}))
            target, wts = np.asarray(vt["_tmp_tsOutcome"]), np.asarray(vt["_tmp_twOutcome"])
            ok = np.isfinite(target) & (wts > 0)
            X = as_matrix(te[self.getHeterogeneityVecCol()])[ok]
            target, wts = target[ok], wts[ok]
            rng = np.random.default_rng(half)
            for t in range(self.getNumTrees()):
                # random forest member: bootstrap rows, one tree
                idx = rng.integers(0, len(target), len(target))
                d = DataFrame({"features": X[idx], "label": target[idx], "w": wts[idx]})
                forest.append(DecisionTreeRegressor(maxDepth=self.getMaxDepth(),
                                                    minInstancesPerNode=self.getMinSamplesLeaf(), weightCol="w",
                                                    seed=1000 * half + t, deviceType="cpu").fit(d))
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
