"""Auto-featurizing trainers and model statistics (reference:
core/.../train/{TrainClassifier, TrainRegressor, AutoTrainer,
ComputeModelStatistics, ComputePerInstanceStatistics}.scala)."""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from ..core.contracts import HasEvaluationMetric, HasInputCols, HasLabelCol
from ..core.dataframe import DataFrame
from ..core.linalg import DenseVector, Vector
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Estimator, Model, Pipeline, PipelineModel, Transformer
from ..featurize import Featurize, ValueIndexer
from ..models import (DecisionTreeClassifier, DecisionTreeRegressor, GBTClassifier, GBTRegressor,
                      LogisticRegression, MultilayerPerceptronClassifier, RandomForestClassifier,
                      RandomForestRegressor)
from ..models.evaluation import auc, classification_metrics, confusion_matrix, positive_scores, regression_metrics

SCORES = "scores"
SCORED_LABELS = "scored_labels"
SCORED_PROBABILITIES = "scored_probabilities"
CLASSIFICATION_KIND = "Classification"
REGRESSION_KIND = "Regression"


def _score_md(kind: str, model_uid: str, label: str = "label") -> dict:
    return {"score_model": {"kind": kind, "uid": model_uid, "label": label}}


class _AutoTrainer(Estimator, HasLabelCol, HasInputCols):
    model = Param("Model to run", None, complex=True)
    featuresCol = Param("The name of the features column", None, T.toString)
    numFeatures = Param("Number of features to hash to", 0, T.toInt)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(featuresCol=self.uid + "_features")

    def _featurize_params(self, learner):
        tree = isinstance(learner, (DecisionTreeClassifier, RandomForestClassifier, GBTClassifier,
                                    DecisionTreeRegressor, RandomForestRegressor, GBTRegressor))
        from ..lightgbm import LightGBMClassifier, LightGBMRegressor

        tree = tree or isinstance(learner, (LightGBMClassifier, LightGBMRegressor))
        return (not tree), isinstance(learner, MultilayerPerceptronClassifier), (1 << 12) if tree else (1 << 18)

    def _featurize(self, df, learner):
        ohe, mlp, nf = self._featurize_params(learner)
        nf = self.getNumFeatures() or nf
        cols = self.getInputCols() or [c for c in df.columns if c != self.getLabelCol()]
        fz = Featurize(inputCols=cols, outputCol=self.getFeaturesCol(), oneHotEncodeCategoricals=ohe,
                       numFeatures=nf).fit(df)
        return fz, fz.transform(df), mlp


class TrainedClassifierModel(Model, HasLabelCol):
    model = Param("the fitted featurization + learner pipeline", None, complex=True)
    featuresCol = Param("The name of the features column", None, T.toString)
    levels = Param("original label levels when the label was reindexed", None, T.identity)

    def _transform(self, df):
        pm = self.getModel()
        levels = self.getLevels()
        work = df
        lab = self.getLabelCol()
        if levels is not None and lab in df:
            table = {l: i for i, l in enumerate(levels)}
            work = df.withColumn(lab, np.asarray([table.get(v, np.nan) for v in df[lab].tolist()], float))
        out = pm.transform(work)
        learner = pm.getStages()[-1]
        raw = getattr(learner, "getRawPredictionCol", lambda: "rawPrediction")()
        prob = getattr(learner, "getProbabilityCol", lambda: "probability")()
        pred = learner.getPredictionCol()
        res = out
        if raw in res:
            res = res.withColumnRenamed(raw, SCORES)
        if prob in res:
            res = res.withColumnRenamed(prob, SCORED_PROBABILITIES)
        p = res[pred]
        if levels is not None:
            vals = [levels[int(v)] for v in p.tolist()]
            arr = np.empty(len(vals), dtype=object)
            for i, v in enumerate(vals):
                arr[i] = v
            if vals and all(isinstance(v, (int, float, np.number)) and not isinstance(v, bool) for v in vals):
                arr = np.asarray(vals)
            res = res.drop(pred).withColumn(SCORED_LABELS, arr, metadata=_score_md(CLASSIFICATION_KIND, self.uid, lab))
            if lab in df:
                res = res.withColumn(lab, df[lab])
        else:
            res = res.drop(pred).withColumn(SCORED_LABELS, p, metadata=_score_md(CLASSIFICATION_KIND, self.uid, lab))
        return res.drop(self.getFeaturesCol())


class TrainClassifier(_AutoTrainer):
    reindexLabel = Param("Re-index the label column", True, T.toBoolean)
    labels = Param("Sorted label values on the labels column", None, T.toListString)

    def _fit(self, df):
        lab = self.getLabelCol()
        levels = None
        work = df
        if self.getReindexLabel():
            if self.getLabels():
                levels = list(self.getLabels())
                conv = [type(df[lab][0])(l) if not isinstance(df[lab][0], str) else l for l in levels] \
                    if df.count() else levels
                levels = conv
            else:
                vi = ValueIndexer(inputCol=lab, outputCol=lab).fit(df)
                levels = [l for l in vi.getLevels() if l is not None]
            table = {l: i for i, l in enumerate(levels)}
            work = df.withColumn(lab, np.asarray([table[v] for v in df[lab].tolist()], dtype=np.float64))
        learner = self.getModel() or LogisticRegression()
        learner = learner.copy()
        if learner.hasParam("labelCol"):
            learner.set("labelCol", lab)
        if learner.hasParam("featuresCol"):
            learner.set("featuresCol", self.getFeaturesCol())
        fz, feat, mlp = self._featurize(work, learner)
        if mlp:
            layers = list(learner.getLayers())
            from ..core.linalg import as_matrix

            layers[0] = as_matrix(feat[self.getFeaturesCol()][:1]).shape[1]
            learner.set("layers", layers)
        fitted = learner.fit(feat)
        m = TrainedClassifierModel(labelCol=lab, featuresCol=self.getFeaturesCol(),
                                   levels=levels if self.getReindexLabel() else None)
        return m.set("model", PipelineModel([fz, fitted]))


class TrainedRegressorModel(Model, HasLabelCol):
    model = Param("the fitted featurization + learner pipeline", None, complex=True)
    featuresCol = Param("The name of the features column", None, T.toString)

    def _transform(self, df):
        pm = self.getModel()
        out = pm.transform(df)
        pred = pm.getStages()[-1].getPredictionCol()
        p = out[pred]
        return out.drop(pred).withColumn(SCORES, p, metadata=_score_md(REGRESSION_KIND, self.uid, self.getLabelCol())) \
            .drop(self.getFeaturesCol())


class TrainRegressor(_AutoTrainer):
    def _fit(self, df):
        from ..models import LinearRegression

        lab = self.getLabelCol()
        work = df.withColumn(lab, np.asarray(df[lab], dtype=np.float64))
        learner = (self.getModel() or LinearRegression()).copy()
        learner.set("labelCol", lab)
        learner.set("featuresCol", self.getFeaturesCol())
        fz, feat, _ = self._featurize(work, learner)
        fitted = learner.fit(feat)
        m = TrainedRegressorModel(labelCol=lab, featuresCol=self.getFeaturesCol())
        return m.set("model", PipelineModel([fz, fitted]))


def _score_info(df: DataFrame, scored_labels: Optional[str], scores: Optional[str]) -> dict:
    for c in (scored_labels, scores, SCORED_LABELS, SCORES):
        if c and c in df:
            md = df.metadata(c).get("score_model")
            if md:
                return md
    return {}


def _detect_kind(df: DataFrame, scored_labels: Optional[str], scores: Optional[str]) -> Optional[str]:
    return _score_info(df, scored_labels, scores).get("kind")


def _label_col(stage, df, scored_labels, scores) -> str:
    if stage.isSet("labelCol"):
        return stage.getLabelCol()
    return _score_info(df, scored_labels, scores).get("label", stage.getLabelCol())


class ComputeModelStatistics(Transformer, HasLabelCol, HasEvaluationMetric):
    scoresCol = Param("Scores or raw prediction column name", None, T.toString)
    scoredLabelsCol = Param("Scored labels column name", None, T.toString)

    def _transform(self, df):
        metric = self.getEvaluationMetric()
        lab = _label_col(self, df, self.getScoredLabelsCol(), self.getScoresCol())
        sl = self.getScoredLabelsCol() or (SCORED_LABELS if SCORED_LABELS in df else "prediction")
        sc = self.getScoresCol() or (SCORES if SCORES in df else None)
        kind = _detect_kind(df, sl, sc)
        if metric in ("classification", "accuracy", "precision", "recall", "AUC", "areaUnderROC"):
            kind = CLASSIFICATION_KIND
        elif metric in ("regression", "mse", "rmse", "r2", "mae"):
            kind = REGRESSION_KIND
        if kind is None:
            kind = CLASSIFICATION_KIND if sl in df and sl != "prediction" else REGRESSION_KIND
        if kind == REGRESSION_KIND:
            pred_col = sc if sc and sc in df and df[sc].ndim == 1 and df[sc].dtype.kind == "f" else sl
            m = regression_metrics(df[lab], df[pred_col])
            out = {"mean_squared_error": [m["mse"]], "root_mean_squared_error": [m["rmse"]], "R^2": [m["r2"]],
                   "mean_absolute_error": [m["mae"]]}
            return DataFrame(out)
        y_raw = df[lab].tolist()
        p_raw = df[sl].tolist()
        levels = sorted(set(y_raw) | set(p_raw), key=lambda v: (str(type(v)), v))
        table = {l: i for i, l in enumerate(levels)}
        y = np.asarray([table[v] for v in y_raw])
        p = np.asarray([table[v] for v in p_raw])
        k = max(2, len(levels))
        cm = confusion_matrix(y, p, k)
        m = classification_metrics(y, p)
        out = {"evaluation_type": [CLASSIFICATION_KIND], "confusion_matrix": [cm]}
        if k == 2:
            out.update({"accuracy": [m["accuracy"]], "precision": [m["precision"]], "recall": [m["recall"]]})
            if sc and sc in df:
                out["AUC"] = [auc(y, positive_scores(df[sc]))]
        else:
            out.update({"accuracy": [m["accuracy"]], "precision": [m["precision"]], "recall": [m["recall"]],
                        "average_accuracy": [m["average_accuracy"]],
                        "macro_averaged_precision": [m["macro_averaged_precision"]],
                        "macro_averaged_recall": [m["macro_averaged_recall"]]})
        res = DataFrame({k2: np.asarray(v, dtype=object) if k2 in ("confusion_matrix", "evaluation_type") else v
                         for k2, v in out.items()})
        return res


class ComputePerInstanceStatistics(Transformer, HasLabelCol, HasEvaluationMetric):
    scoresCol = Param("Scores or raw prediction column name", None, T.toString)
    scoredLabelsCol = Param("Scored labels column name", None, T.toString)
    scoredProbabilitiesCol = Param("Scored probabilities column name", None, T.toString)

    def _transform(self, df):
        lab = _label_col(self, df, self.getScoredLabelsCol(), self.getScoresCol())
        kind = _detect_kind(df, self.getScoredLabelsCol(), self.getScoresCol())
        if self.getEvaluationMetric() == "regression" or kind == REGRESSION_KIND:
            sc = self.getScoresCol() or SCORES
            err = np.asarray(df[sc], float) - np.asarray(df[lab], float)
            return df.withColumn("L1_loss", np.abs(err)).withColumn("L2_loss", err * err)
        prob_col = self.getScoredProbabilitiesCol() or SCORED_PROBABILITIES
        probs = df[prob_col]
        P = probs if probs.ndim == 2 else np.stack([v.toArray() if isinstance(v, Vector) else np.asarray(v)
                                                    for v in probs])
        y_raw = df[lab].tolist()
        try:
            y = np.asarray(y_raw, dtype=np.int64)
        except (TypeError, ValueError):
            levels = sorted(set(y_raw))
            y = np.asarray([levels.index(v) for v in y_raw])
        p = np.clip(P[np.arange(len(y)), y], 1e-15, 1.0)
        return df.withColumn("log_loss", -np.log(p))


__all__ = ["TrainClassifier", "TrainedClassifierModel", "TrainRegressor", "TrainedRegressorModel",
           "ComputeModelStatistics", "ComputePerInstanceStatistics", "SCORES", "SCORED_LABELS",
           "SCORED_PROBABILITIES"]
