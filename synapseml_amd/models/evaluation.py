"""Evaluators with SparkML's API (BinaryClassificationEvaluator,
MulticlassClassificationEvaluator, RegressionEvaluator) and the metric
functions shared with ComputeModelStatistics / TuneHyperparameters /
FindBestModel."""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np

from ..core.contracts import HasLabelCol, HasPredictionCol, HasRawPredictionCol, HasWeightCol
from ..core.dataframe import DataFrame
from ..core.linalg import Vector
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Evaluator


def positive_scores(col) -> np.ndarray:
    """Score of the positive class from a raw-prediction / probability column or scalar scores."""
    if isinstance(col, np.ndarray) and col.ndim == 2:
        return col[:, -1].astype(np.float64)
    vals = col.tolist()
    if vals and isinstance(vals[0], (Vector, list, tuple, np.ndarray)):
        return np.asarray([np.asarray(v.toArray() if isinstance(v, Vector) else v, dtype=np.float64)[-1]
                           for v in vals])
    return np.asarray(vals, dtype=np.float64)


def roc_curve(y: np.ndarray, s: np.ndarray, w=None) -> Tuple[np.ndarray, np.ndarray]:
    w = np.ones_like(s) if w is None else w
    order = np.argsort(-s, kind="mergesort")
    s, y, w = s[order], y[order], w[order]
    distinct = np.r_[np.nonzero(np.diff(s))[0], len(s) - 1]
    tps = np.cumsum(y * w)[distinct]
    fps = np.cumsum((1 - y) * w)[distinct]
    tpr = np.r_[0.0, tps / max(tps[-1], 1e-300)] if len(tps) else np.array([0.0, 1.0])
    fpr = np.r_[0.0, fps / max(fps[-1], 1e-300)] if len(fps) else np.array([0.0, 1.0])
    return fpr, tpr


def auc(y, s, w=None) -> float:
    fpr, tpr = roc_curve(np.asarray(y, float), np.asarray(s, float), w)
    return float(np.trapezoid(tpr, fpr))


def area_under_pr(y, s, w=None) -> float:
    y = np.asarray(y, float)
    s = np.asarray(s, float)
    w = np.ones_like(s) if w is None else w
    order = np.argsort(-s, kind="mergesort")
    s, y, w = s[order], y[order], w[order]
    distinct = np.r_[np.nonzero(np.diff(s))[0], len(s) - 1]
    tps = np.cumsum(y * w)[distinct]
    fps = np.cumsum((1 - y) * w)[distinct]
    prec = tps / np.maximum(tps + fps, 1e-300)
    rec = tps / max(tps[-1], 1e-300)
    prec = np.r_[prec[0] if len(prec) else 1.0, prec]
    rec = np.r_[0.0, rec]
    return float(np.trapezoid(prec, rec))


def confusion_matrix(y, p, k=None) -> np.ndarray:
    y = np.asarray(y, dtype=np.int64)
    p = np.asarray(p, dtype=np.int64)
    k = k or int(max(y.max(initial=0), p.max(initial=0))) + 1
    m = np.zeros((k, k))
    np.add.at(m, (y, p), 1)
    return m


def classification_metrics(y, p) -> Dict[str, float]:
    cm = confusion_matrix(y, p)
    k = cm.shape[0]
    total = cm.sum()
    acc = np.trace(cm) / total if total else 0.0
    out = {"accuracy": float(acc)}
    if k == 2:
        tp, fp, fn = cm[1, 1], cm[0, 1], cm[1, 0]
        out["precision"] = float(tp / (tp + fp)) if tp + fp > 0 else 0.0
        out["recall"] = float(tp / (tp + fn)) if tp + fn > 0 else 0.0
    else:
        out["precision"] = float(acc)  # micro-averaged == accuracy
        out["recall"] = float(acc)
        per_acc = [(total - cm[i].sum() - cm[:, i].sum() + 2 * cm[i, i]) / total for i in range(k)]
        out["average_accuracy"] = float(np.mean(per_acc))
        prec = [cm[i, i] / cm[:, i].sum() if cm[:, i].sum() else 0.0 for i in range(k)]
        rec = [cm[i, i] / cm[i].sum() if cm[i].sum() else 0.0 for i in range(k)]
        out["macro_averaged_precision"] = float(np.mean(prec))
        out["macro_averaged_recall"] = float(np.mean(rec))
    return out


def regression_metrics(y, p, w=None) -> Dict[str, float]:
    y = np.asarray(y, float)
    p = np.asarray(p, float)
    w = np.ones_like(y) if w is None else np.asarray(w, float)
    ws = w.sum()
    err = p - y
    mse = float((w * err * err).sum() / ws)
    ym = (w * y).sum() / ws
    ss_tot = (w * (y - ym) ** 2).sum()
    return {"mse": mse, "rmse": float(np.sqrt(mse)), "r2": float(1 - (w * err * err).sum() / ss_tot) if ss_tot else
            0.0, "mae": float((w * np.abs(err)).sum() / ws), "var": float((w * (p - (w * p).sum() / ws) ** 2).sum() / ws)}


class BinaryClassificationEvaluator(Evaluator, HasLabelCol, HasRawPredictionCol, HasWeightCol):
    metricName = Param("areaUnderROC | areaUnderPR", "areaUnderROC", T.toString)

    def _evaluate(self, df):
        y = np.asarray(df[self.getLabelCol()], float)
        s = positive_scores(df[self.getRawPredictionCol()])
        w = np.asarray(df[self.getWeightCol()], float) if self.getWeightCol() else None
        if self.getMetricName() == "areaUnderPR":
            return area_under_pr(y, s, w)
        return auc(y, s, w)

    def isLargerBetter(self):  # noqa: N802
        return True


class MulticlassClassificationEvaluator(Evaluator, HasLabelCol, HasPredictionCol, HasWeightCol):
    metricName = Param("f1 | accuracy | weightedPrecision | weightedRecall | logLoss", "f1", T.toString)

    def _evaluate(self, df):
        y = np.asarray(df[self.getLabelCol()], np.int64)
        p = np.asarray(df[self.getPredictionCol()], np.float64).astype(np.int64)
        cm = confusion_matrix(y, p)
        k = cm.shape[0]
        support = cm.sum(1)
        prec = np.array([cm[i, i] / cm[:, i].sum() if cm[:, i].sum() else 0.0 for i in range(k)])
        rec = np.array([cm[i, i] / cm[i].sum() if cm[i].sum() else 0.0 for i in range(k)])
        f1 = np.where(prec + rec > 0, 2 * prec * rec / np.maximum(prec + rec, 1e-300), 0.0)
        wts = support / support.sum()
        m = self.getMetricName()
        if m == "accuracy":
            return float(np.trace(cm) / cm.sum())
        if m == "weightedPrecision":
            return float((prec * wts).sum())
        if m == "weightedRecall":
            return float((rec * wts).sum())
        return float((f1 * wts).sum())

    def isLargerBetter(self):  # noqa: N802
        return self.getMetricName() != "logLoss"


class RegressionEvaluator(Evaluator, HasLabelCol, HasPredictionCol, HasWeightCol):
    metricName = Param("rmse | mse | r2 | mae | var", "rmse", T.toString)

    def _evaluate(self, df):
        w = np.asarray(df[self.getWeightCol()], float) if self.getWeightCol() else None
        return regression_metrics(df[self.getLabelCol()], df[self.getPredictionCol()], w)[self.getMetricName()]

    def isLargerBetter(self):  # noqa: N802
        return self.getMetricName() in ("r2", "var")
