"""Shared column-param mixins (reference: core/.../core/contracts/Params.scala)."""
from __future__ import annotations

from .params import Param, Params, TypeConverters as T


class HasInputCol(Params):
    inputCol = Param("The name of the input column", None, T.toString)


class HasInputCols(Params):
    inputCols = Param("The names of the input columns", None, T.toListString)


class HasOutputCol(Params):
    outputCol = Param("The name of the output column", None, T.toString)


class HasOutputCols(Params):
    outputCols = Param("The names of the output columns", None, T.toListString)


class HasLabelCol(Params):
    labelCol = Param("The name of the label column", "label", T.toString)


class HasFeaturesCol(Params):
    featuresCol = Param("The name of the features column", "features", T.toString)


class HasWeightCol(Params):
    weightCol = Param("The name of the weight column", None, T.toString)


class HasPredictionCol(Params):
    predictionCol = Param("The name of the prediction column", "prediction", T.toString)


class HasRawPredictionCol(Params):
    rawPredictionCol = Param("The name of the raw prediction column", "rawPrediction", T.toString)


class HasProbabilityCol(Params):
    probabilityCol = Param("The name of the probability column", "probability", T.toString)


class HasValidationIndicatorCol(Params):
    validationIndicatorCol = Param("Indicates whether the row is for training or validation", None, T.toString)


class HasInitScoreCol(Params):
    initScoreCol = Param("The name of the initial score column", None, T.toString)


class HasGroupCol(Params):
    groupCol = Param("The name of the group column", None, T.toString)


class HasSeed(Params):
    seed = Param("Random seed", 0, T.toInt)


class HasBatchSize(Params):
    batchSize = Param("The max size of the buffer", 10, T.toInt)


class HasEvaluationMetric(Params):
    evaluationMetric = Param("Metric to evaluate models with", "all", T.toString)


class HasScoredLabelsCol(Params):
    scoredLabelsCol = Param("Scored labels column name", None, T.toString)


class HasScoresCol(Params):
    scoresCol = Param("Scores or raw prediction column name", None, T.toString)


class HasScoredProbabilitiesCol(Params):
    scoredProbabilitiesCol = Param("Scored probabilities column name", None, T.toString)


class HasErrorCol(Params):
    errorCol = Param("column to hold http errors", None, T.toString)
