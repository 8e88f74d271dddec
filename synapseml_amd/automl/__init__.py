"""Hyperparameter search and model selection (reference:
core/.../automl/{TuneHyperparameters, FindBestModel, HyperparamBuilder,
ParamSpace, EvaluationUtils}.scala, Python HyperparamBuilder.py)."""
from __future__ import annotations

import itertools
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Dict, Iterator, List, Sequence, Tuple

import numpy as np

from ..core.contracts import HasEvaluationMetric, HasSeed
from ..core.dataframe import DataFrame
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Estimator, Model, Transformer
from ..models.evaluation import (auc, classification_metrics, positive_scores, regression_metrics, roc_curve)


# ---------------------------------------------------------------------- hyperparameter spaces
class Dist:
    def get_next(self, rng) -> Any:
        raise NotImplementedError

    def values(self) -> List[Any]:
        raise NotImplementedError


class DiscreteHyperParam(Dist):
    def __init__(self, values: Sequence[Any], seed: int = 0):
        self._values = list(values)

    def get_next(self, rng):
        return self._values[int(rng.integers(0, len(self._values)))]

    def values(self):
        return list(self._values)

    def get(self):
        """the wrapped distribution (reference HyperparamBuilder.py DiscreteHyperParam.get)"""
        return self


class RangeHyperParam(Dist):
    """Uniform range; integer-valued when both bounds are ints (IntRangeHyperParam & co.)."""

    def __init__(self, min_value, max_value, seed: int = 0, isDouble: bool = None):  # noqa: N803
        self.min, self.max = min_value, max_value
        self.is_int = isinstance(min_value, (int, np.integer)) and isinstance(max_value, (int, np.integer)) \
            if isDouble is None else not isDouble

    def get_next(self, rng):
        if self.is_int:
            return int(rng.integers(self.min, self.max))
        return float(self.min + (self.max - self.min) * rng.random())

    def get(self):
        """the wrapped distribution (reference HyperparamBuilder.py RangeHyperParam.get)"""
        return self

    def values(self):
        if self.is_int:
            return list(range(self.min, self.max))
        raise ValueError("a continuous range has no finite value list; use DiscreteHyperParam for grids")


IntRangeHyperParam = RangeHyperParam
LongRangeHyperParam = RangeHyperParam
FloatRangeHyperParam = lambda a, b, seed=0: RangeHyperParam(float(a), float(b), seed)  # noqa: E731
DoubleRangeHyperParam = FloatRangeHyperParam


class HyperparamBuilder:
    def __init__(self):
        self._hp: List[Tuple[Any, str, Dist]] = []

    def addHyperparam(self, est, param, values: Dist) -> "HyperparamBuilder":  # noqa: N802
        name = param if isinstance(param, str) else getattr(param, "name", str(param))
        self._hp.append((est, name, values))
        return self

    def build(self) -> List[Tuple[Any, str, Dist]]:
        return list(self._hp)


class ParamSpace:
    def paramMaps(self) -> Iterator[Dict[Tuple[str, str], Any]]:  # noqa: N802
        raise NotImplementedError


class GridSpace(ParamSpace):
    def __init__(self, hyperparams: List[Tuple[Any, str, Dist]]):
        self.hp = hyperparams

    def space(self):
        """the wrapped search space (reference HyperparamBuilder.py GridSpace.space)"""
        return self

    def paramMaps(self):  # noqa: N802
        keys = [(est, name) for est, name, _ in self.hp]
        for combo in itertools.product(*[d.values() for _, _, d in self.hp]):
            yield {(est.uid, name): v for (est, name), v in zip(keys, combo)}


class RandomSpace(ParamSpace):
    def __init__(self, hyperparams: List[Tuple[Any, str, Dist]], seed: int = 0):
        self.hp = hyperparams
        self.rng = np.random.default_rng(seed)

    def space(self):
        """the wrapped search space (reference HyperparamBuilder.py RandomSpace.space)"""
        return self

    def paramMaps(self):  # noqa: N802
        while True:
            yield {(est.uid, name): d.get_next(self.rng) for est, name, d in self.hp}


# ---------------------------------------------------------------------- evaluation helpers
_CLS_METRICS = {"accuracy", "precision", "recall", "AUC", "areaUnderROC", "classification", "all"}
_REG_METRICS = {"mse", "rmse", "r2", "mae", "regression"}
_LOWER_BETTER = {"mse", "rmse", "mae"}


def _kind_of(model) -> str:
    from ..train import TrainedRegressorModel

    if isinstance(model, TrainedRegressorModel):
        return "regression"
    for attr in ("getProbabilityCol", "getRawPredictionCol"):
        if hasattr(model, attr):
            return "classification"
    name = type(model).__name__.lower()
    return "regression" if "regress" in name else "classification"


def evaluate_model(model, scored: DataFrame, metric: str) -> float:
    """Metric of a scored validation set (ComputeModelStatistics semantics)."""
    from ..train import SCORED_LABELS, SCORES, TrainedClassifierModel, TrainedRegressorModel

    if isinstance(model, TrainedClassifierModel):
        lab, pred, raw = model.getLabelCol(), SCORED_LABELS, SCORES
    elif isinstance(model, TrainedRegressorModel):
        lab, pred, raw = model.getLabelCol(), SCORES, None
    else:
        lab = model.getLabelCol() if model.hasParam("labelCol") else "label"
        pred = model.getPredictionCol() if model.hasParam("predictionCol") else "prediction"
        raw = model.getRawPredictionCol() if model.hasParam("rawPredictionCol") else None
        if raw is None and model.hasParam("probabilityCol"):
            raw = model.getProbabilityCol()
        if lab not in scored and "label" in scored:
            lab = "label"
    if metric in _REG_METRICS or (metric == "all" and _kind_of(model) == "regression"):
        m = regression_metrics(scored[lab], scored[pred])
        return m["mse" if metric in ("regression", "all") else metric]
    y_raw = scored[lab].tolist()
    p_raw = scored[pred].tolist()
    levels = sorted(set(y_raw) | set(p_raw), key=lambda v: (str(type(v)), v))
    table = {l: i for i, l in enumerate(levels)}
    y = np.asarray([table[v] for v in y_raw])
    p = np.asarray([table[v] for v in p_raw])
    if metric in ("AUC", "areaUnderROC"):
        return auc(y, positive_scores(scored[raw]))
    m = classification_metrics(y, p)
    return m["accuracy" if metric in ("classification", "all") else metric]


def larger_is_better(metric: str) -> bool:
    return metric not in _LOWER_BETTER


def _kfold(df: DataFrame, k: int, seed: int) -> List[Tuple[DataFrame, DataFrame]]:
    rng = np.random.default_rng(seed)
    fold = rng.integers(0, k, size=df.count())
    return [(df.filter(fold != i), df.filter(fold == i)) for i in range(k)]


# ---------------------------------------------------------------------- TuneHyperparameters
class TuneHyperparametersModel(Model):
    bestModel = Param("the best model found", None, complex=True)
    bestMetric = Param("the best metric from the runs", None, T.toFloat)

    def _transform(self, df):
        return self.getBestModel().transform(df)

    def getBestModelInfo(self) -> str:  # noqa: N802
        return f"{type(self.getBestModel()).__name__}: {self.getBestMetric()}"


class TuneHyperparameters(Estimator, HasEvaluationMetric, HasSeed):
    models = Param("Estimators to run", [], complex=True)
    numFolds = Param("Number of folds", 3, T.toInt)
    numRuns = Param("Termination criteria for randomized search", 10, T.toInt)
    parallelism = Param("The number of models to run in parallel", 1, T.toInt)
    paramSpace = Param("Parameter space for generating hyperparameters", None, complex=True)

    def _fit(self, df):
        models = list(self.getModels())
        metric = self.getEvaluationMetric()
        space = self.getParamSpace()
        gen = space.paramMaps() if space is not None else iter(lambda: {}, None)
        runs = []
        for i in range(self.getNumRuns()):
            try:
                pm = next(gen)
            except StopIteration:
                break
            runs.append(pm)
        if not runs:
            runs = [{}]
        splits = _kfold(df, self.getNumFolds(), self.getSeed())

        def run_one(idx_pm):
            idx, pm = idx_pm
            est = models[idx % len(models)]
            own = {name: v for (uid, name), v in pm.items() if uid == est.uid}
            scores = []
            for tr, va in splits:
                m = est.copy(own).fit(tr)
                scores.append(evaluate_model(m, m.transform(va), metric))
            return float(np.mean(scores))

        with ThreadPoolExecutor(max_workers=max(1, self.getParallelism())) as ex:
            scores = list(ex.map(run_one, list(enumerate(runs))))
        better = larger_is_better(metric)
        best = int(np.argmax(scores) if better else np.argmin(scores))
        est = models[best % len(models)]
        own = {name: v for (uid, name), v in runs[best].items() if uid == est.uid}
        best_model = est.copy(own).fit(df)
        out = TuneHyperparametersModel(bestMetric=scores[best])
        out.all_metrics = scores
        out.all_params = runs
        return out.set("bestModel", best_model)


# ---------------------------------------------------------------------- FindBestModel
class BestModel(Model):
    bestModel = Param("the best model found", None, complex=True)
    scoredDataset = Param("dataset scored by best model", None, complex=True)
    rocCurve = Param("the roc curve of the best model", None, complex=True)
    bestModelMetrics = Param("the metrics from the best model", None, complex=True)
    allModelMetrics = Param("all model metrics", None, complex=True)

    def _transform(self, df):
        return self.getBestModel().transform(df)

    def getEvaluationResults(self) -> DataFrame:  # noqa: N802
        return self.getAllModelMetrics()


class FindBestModel(Estimator, HasEvaluationMetric):
    models = Param("List of models to be evaluated", [], complex=True)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(evaluationMetric="accuracy")

    def _fit(self, df):
        metric = self.getEvaluationMetric()
        results = []
        for m in self.getModels():
            scored = m.transform(df)
            results.append((m, scored, evaluate_model(m, scored, metric)))
        vals = [r[2] for r in results]
        best = int(np.argmax(vals) if larger_is_better(metric) else np.argmin(vals))
        bm, scored, _ = results[best]
        all_metrics = DataFrame({"model_name": np.asarray([type(r[0]).__name__ + "_" + r[0].uid for r in results],
                                                          dtype=object), metric: np.asarray(vals, dtype=float)})
        out = BestModel()
        out.set("bestModel", bm)
        out.set("scoredDataset", scored)
        out.set("allModelMetrics", all_metrics)
        best_metrics = {metric: vals[best]}
        roc = None
        if _kind_of(bm) == "classification":
            try:
                from ..train import SCORES, TrainedClassifierModel

                lab = bm.getLabelCol() if bm.hasParam("labelCol") else "label"
                raw = SCORES if isinstance(bm, TrainedClassifierModel) else bm.getRawPredictionCol()
                y_raw = scored[lab].tolist()
                levels = sorted(set(y_raw), key=lambda v: (str(type(v)), v))
                if len(levels) == 2:
                    y = np.asarray([levels.index(v) for v in y_raw], float)
                    fpr, tpr = roc_curve(y, positive_scores(scored[raw]))
                    roc = DataFrame({"false_positive_rate": fpr, "true_positive_rate": tpr})
                    best_metrics["AUC"] = float(np.trapezoid(tpr, fpr))
            except Exception:  # noqa: BLE001 - ROC is optional metadata
                roc = None
        out.set("rocCurve", roc)
        out.set("bestModelMetrics", DataFrame({k: [v] for k, v in best_metrics.items()}))
        return out


__all__ = ["DiscreteHyperParam", "RangeHyperParam", "IntRangeHyperParam", "LongRangeHyperParam",
           "FloatRangeHyperParam", "DoubleRangeHyperParam", "HyperparamBuilder", "GridSpace", "RandomSpace",
           "TuneHyperparameters", "TuneHyperparametersModel", "FindBestModel", "BestModel", "evaluate_model"]
