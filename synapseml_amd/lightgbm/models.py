"""LightGBM estimators and models: classifier, regressor, ranker
(reference: lightgbm/.../LightGBMClassifier.scala, LightGBMRegressor.scala,
LightGBMRanker.scala, LightGBMModelMethods.scala)."""
from __future__ import annotations

from typing import Optional

import numpy as np

from ..core.contracts import HasGroupCol, HasProbabilityCol, HasRawPredictionCol
from ..core.dataframe import DataFrame
from ..core.linalg import as_matrix
from ..core.pipeline import Model
from ..core.params import Param, TypeConverters as T
from ..core.utils import ParamsStringBuilder
from .base import LightGBMBase
from .booster import LightGBMBooster
from .params import LightGBMModelParams


def _features_matrix(df: DataFrame, col: str) -> np.ndarray:
    """the feature rows for scoring: a float32 / float64 dense column as is (no float64 copy of a float32
    partition: the device scorer reads float32 rows), other layouts densified to float64"""
    c = df[col]
    if isinstance(c, np.ndarray) and c.ndim == 2:
        return np.ascontiguousarray(c) if c.dtype in (np.float32, np.float64) else np.ascontiguousarray(c, np.float64)
    return as_matrix(c)


class _LightGBMModelBase(Model, LightGBMModelParams):
    """Shared model methods (LightGBMModelMethods.scala:13-133)."""

    def setPredictDisableShapeCheck(self, value=None):  # noqa: N802
        """reference mixin.py:83-95: a missing / falsy value means False"""
        self.set("predictDisableShapeCheck", bool(value))
        return self

    def getModel(self) -> LightGBMBooster:  # noqa: N802
        return self.getLightGBMBooster()

    def _booster(self) -> LightGBMBooster:
        b = self.getLightGBMBooster()
        b.setNumIterations(self.getNumIterations())
        b.setStartIteration(self.getStartIteration())
        return b

    def getFeatureImportances(self, importance_type: str = "split") -> list:  # noqa: N802
        return list(self.getLightGBMBooster().getFeatureImportances(importance_type))

    def getFeatureShaps(self, vector) -> list:  # noqa: N802
        x = np.asarray(vector.toArray() if hasattr(vector, "toArray") else vector, dtype=np.float64)
        return list(self._booster().featuresShap(x[None, :], self.getPredictDisableShapeCheck())[0])

    def getDenseFeatureShaps(self, values) -> list:  # noqa: N802
        return self.getFeatureShaps(np.asarray(values, dtype=np.float64))

    def getSparseFeatureShaps(self, size, indices, values) -> list:  # noqa: N802
        x = np.zeros(size)
        x[np.asarray(indices, dtype=np.int64)] = values
        return self.getFeatureShaps(x)

    def getBoosterBestIteration(self) -> int:  # noqa: N802
        return self.getLightGBMBooster().bestIteration

    def getBoosterNumTotalIterations(self) -> int:  # noqa: N802
        return self.getLightGBMBooster().numTotalIterations

    def getBoosterNumTotalModel(self) -> int:  # noqa: N802
        return self.getLightGBMBooster().numTotalModel

    def getBoosterNumFeatures(self) -> int:  # noqa: N802
        return self.getLightGBMBooster().numFeatures

    def getBoosterNumClasses(self) -> int:  # noqa: N802
        return self.getLightGBMBooster().numClasses

    def saveNativeModel(self, filename: str, overwrite: bool = True) -> None:  # noqa: N802
        self.getLightGBMBooster().saveNativeModel(filename, overwrite)

    def getNativeModel(self) -> str:  # noqa: N802
        return self.getLightGBMBooster().modelStr

    def _extra_outputs(self, df: DataFrame, X: np.ndarray) -> DataFrame:
        b = self._booster()
        if self.getLeafPredictionCol():
            df = df.withColumn(self.getLeafPredictionCol(), b.predictLeaf(X, self.getPredictDisableShapeCheck(),
                                                                          self.getDeviceType()))
        if self.getFeaturesShapCol():
            df = df.withColumn(self.getFeaturesShapCol(), b.featuresShap(X, self.getPredictDisableShapeCheck()))
        return df

    @classmethod
    def loadNativeModelFromString(cls, model: str, **kw):  # noqa: N802
        m = cls(**kw)
        m.setLightGBMBooster(LightGBMBooster(model))
        m._post_load()
        return m

    @classmethod
    def loadNativeModelFromFile(cls, filename: str, **kw):  # noqa: N802
        with open(filename) as f:
            return cls.loadNativeModelFromString(f.read(), **kw)

    def _post_load(self) -> None:
        pass


# ============================================================== classifier
class LightGBMClassificationModel(_LightGBMModelBase, HasRawPredictionCol, HasProbabilityCol):
    actualNumClasses = Param("Inferred number of classes based on dataset metadata or, if there is no metadata, unique count", None, T.toInt)
    thresholds = Param("Thresholds in multi-class classification to adjust the probability of predicting each class", None, T.toListFloat)

    @property
    def numClasses(self) -> int:  # noqa: N802
        return self.getActualNumClasses() or max(2, self.getLightGBMBooster().numClasses)

    def _post_load(self) -> None:
        self.setActualNumClasses(max(2, self.getLightGBMBooster().numClasses))

    def _transform(self, df: DataFrame) -> DataFrame:
        X = _features_matrix(df, self.getFeaturesCol())
        b = self._booster()
        dsc = self.getPredictDisableShapeCheck()
        dev = self.getDeviceType()
        raw = prob = None
        if self.getRawPredictionCol() or self.getProbabilityCol() or self.getPredictionCol():
            # one ensemble pass yields both the raw scores and the probabilities
            raw, prob = b.score_both(X, classification=True, disable_shape_check=dsc, device=dev)
        if self.getRawPredictionCol():
            df = df.withColumn(self.getRawPredictionCol(), raw)
        if self.getProbabilityCol():
            df = df.withColumn(self.getProbabilityCol(), prob)
        if self.getPredictionCol():
            th = self.getThresholds()
            if th is None and raw is not None:
                pred = np.argmax(raw, axis=1)
            else:
                if prob is None:
                    prob = b.score(X, raw=False, classification=True, disable_shape_check=dsc, device=dev)
                if th is not None:
                    t = np.asarray(th, dtype=np.float64)
                    if len(t) != prob.shape[1]:
                        raise ValueError(f"thresholds length {len(t)} != numClasses {prob.shape[1]}")
                    pred = np.argmax(prob / np.where(t == 0, 1e-300, t), axis=1)
                else:
                    pred = np.argmax(prob, axis=1)
            df = df.withColumn(self.getPredictionCol(), pred.astype(np.float64))
        return self._extra_outputs(df, X)


class LightGBMClassifier(LightGBMBase, HasRawPredictionCol, HasProbabilityCol):
    """Gradient-boosted trees for binary / multiclass classification."""

    isUnbalance = Param("Set to true if training data is unbalanced in binary classification scenario", False, T.toBoolean)
    maxNumClasses = Param("Number of max classes to infer numClass in multi-class classification.", 100, T.toInt)
    thresholds = Param("Thresholds in multi-class classification", None, T.toListFloat)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(objective="binary")

    def _is_classification(self) -> bool:
        return True

    def _num_class(self, df: DataFrame) -> int:
        if self.getObjective() == "binary":
            return 1
        md = df.metadata(self.getLabelCol())
        if "num_classes" in md:
            return int(md["num_classes"])
        from ..parallel import distributed as D

        lab = np.asarray(df[self.getLabelCol()], dtype=np.float64)
        mx = int(lab.max()) + 1 if len(lab) else 1
        if D.world_size() > 1:
            mx = max(D.all_gather_object(mx))
        if mx > self.getMaxNumClasses():
            raise ValueError(f"inferred {mx} classes > maxNumClasses={self.getMaxNumClasses()}")
        return mx

    def _extra_params(self, sb: ParamsStringBuilder, num_class: int) -> None:
        binary = self.getObjective() == "binary"
        sb.appendParamValueIfNotThere("num_class", None if binary else num_class)
        sb.appendParamValueIfNotThere("is_unbalance", self.getIsUnbalance() if binary else None)
        sb.appendParamValueIfNotThere("boost_from_average", self.getBoostFromAverage())

    def _make_model(self, booster: LightGBMBooster, num_class: int) -> LightGBMClassificationModel:
        m = LightGBMClassificationModel()
        self._copyValues(m)
        m.setLightGBMBooster(booster)
        m.setActualNumClasses(2 if num_class == 1 else num_class)
        m.set("numIterations", -1)
        m.set("startIteration", 0)
        m.parent = self
        return m


# ============================================================== regressor
class LightGBMRegressionModel(_LightGBMModelBase):
    def _transform(self, df: DataFrame) -> DataFrame:
        X = _features_matrix(df, self.getFeaturesCol())
        b = self._booster()
        pred = b.score(X, raw=False, classification=False, disable_shape_check=self.getPredictDisableShapeCheck(),
                       device=self.getDeviceType())[:, 0]
        df = df.withColumn(self.getPredictionCol(), pred)
        return self._extra_outputs(df, X)


class LightGBMRegressor(LightGBMBase):
    """Regression objectives: regression_l2, regression_l1, huber, fair,
    poisson, quantile, mape, gamma, tweedie (LightGBMRegressor.scala:25-36)."""

    alpha = Param("parameter for Huber loss and Quantile regression", 0.9, T.toFloat)
    tweedieVariancePower = Param("control the variance of tweedie distribution, must be between 1 and 2", 1.5, T.toFloat)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(objective="regression")

    def _extra_params(self, sb: ParamsStringBuilder, num_class: int) -> None:
        sb.appendParamValueIfNotThere("alpha", self.getAlpha())
        sb.appendParamValueIfNotThere("tweedie_variance_power", self.getTweedieVariancePower())
        sb.appendParamValueIfNotThere("boost_from_average", self.getBoostFromAverage())

    def _make_model(self, booster: LightGBMBooster, num_class: int) -> LightGBMRegressionModel:
        m = LightGBMRegressionModel()
        self._copyValues(m)
        m.setLightGBMBooster(booster)
        m.set("numIterations", -1)
        m.set("startIteration", 0)
        m.parent = self
        return m


# ============================================================== ranker
class LightGBMRankerModel(_LightGBMModelBase):
    def _transform(self, df: DataFrame) -> DataFrame:
        X = _features_matrix(df, self.getFeaturesCol())
        pred = self._booster().score(X, raw=True, classification=False,
                                     disable_shape_check=self.getPredictDisableShapeCheck(),
                                     device=self.getDeviceType())[:, 0]
        df = df.withColumn(self.getPredictionCol(), pred)
        return self._extra_outputs(df, X)


class LightGBMRanker(LightGBMBase, HasGroupCol):
    """LambdaRank with query groups (LightGBMRanker.scala:26-121)."""

    maxPosition = Param("optimized NDCG at this position", 20, T.toInt)
    labelGain = Param("graded relevance for each label in NDCG", [], T.toListFloat)
    evalAt = Param("NDCG and MAP evaluation positions, separated by comma", [1, 2, 3, 4, 5], T.toListInt)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(objective="lambdarank", groupCol="group")

    def _group_col(self) -> Optional[str]:
        return self.getGroupCol()

    def _extra_params(self, sb: ParamsStringBuilder, num_class: int) -> None:
        sb.appendParamValueIfNotThere("max_position", self.getMaxPosition())
        sb.appendParamListIfNotThere("label_gain", self.getLabelGain())
        sb.appendParamListIfNotThere("eval_at", self.getEvalAt())

    def _make_model(self, booster: LightGBMBooster, num_class: int) -> LightGBMRankerModel:
        m = LightGBMRankerModel()
        self._copyValues(m)
        m.setLightGBMBooster(booster)
        m.set("numIterations", -1)
        m.set("startIteration", 0)
        m.parent = self
        return m


# reference lightgbm/mixin.py: the model-method mixin of the three LightGBM model classes
LightGBMModelMixin = _LightGBMModelBase
