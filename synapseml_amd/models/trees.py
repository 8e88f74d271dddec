"""Tree learners with SparkML's API (DecisionTree / RandomForest / GBT
classifiers and regressors, as used by TrainClassifier & friends) on top of
the native GBDT engine (csrc/gbdt: histogram tree growth on the GPU or the
OpenMP host backend) — one tree implementation for the whole framework."""
from __future__ import annotations

import numpy as np

from ..core.contracts import (HasFeaturesCol, HasLabelCol, HasPredictionCol, HasProbabilityCol, HasRawPredictionCol,
                              HasSeed, HasWeightCol)
from ..core.params import Param, Params, TypeConverters as T
from ..core.pipeline import Estimator, Model


class _TreeParams(HasFeaturesCol, HasLabelCol, HasWeightCol, HasPredictionCol, HasSeed):
    maxDepth = Param("Maximum depth of the tree", 5, T.toInt)
    maxBins = Param("Max number of bins for discretizing continuous features", 32, T.toInt)
    minInstancesPerNode = Param("Minimum number of instances each child must have after split", 1, T.toInt)
    minInfoGain = Param("Minimum information gain for a split to be considered at a tree node", 0.0, T.toFloat)
    deviceType = Param("cpu | gpu", "auto", T.toString)

    def _common(self):
        import torch

        dev = self.getDeviceType()
        if dev == "auto":
            dev = "gpu" if torch.cuda.is_available() else "cpu"
        return dict(featuresCol=self.getFeaturesCol(), labelCol=self.getLabelCol(),
                    maxDepth=self.getMaxDepth(), numLeaves=max(2, min(131072, 2 ** self.getMaxDepth())),
                    maxBin=max(2, self.getMaxBins()), minDataInLeaf=self.getMinInstancesPerNode(),
                    minGainToSplit=self.getMinInfoGain(), seed=self.getSeed(), deviceType=dev,
                    minSumHessianInLeaf=0.0, **({"weightCol": self.getWeightCol()} if self.getWeightCol() else {}))


class _WrappedModel(Model, HasFeaturesCol, HasPredictionCol):
    inner = Param("the wrapped native booster model", None, complex=True)

    def _transform(self, df):
        m = self.getInner()
        m.setPredictionCol(self.getPredictionCol())
        return m.transform(df)

    @property
    def featureImportances(self):  # noqa: N802
        imp = np.asarray(self.getInner().getFeatureImportances("gain"), dtype=np.float64)
        s = imp.sum()
        from ..core.linalg import DenseVector

        return DenseVector(imp / s if s > 0 else imp)


class _ClsModel(_WrappedModel, HasRawPredictionCol, HasProbabilityCol):
    def _transform(self, df):
        m = self.getInner()
        m.setPredictionCol(self.getPredictionCol())
        m.setProbabilityCol(self.getProbabilityCol())
        m.setRawPredictionCol(self.getRawPredictionCol())
        return m.transform(df)


class _TreeClassifier(Estimator, _TreeParams, HasRawPredictionCol, HasProbabilityCol):
    _model_cls = _ClsModel

    def _lgbm_params(self) -> dict:
        raise NotImplementedError

    def _fit(self, df):
        from ..lightgbm import LightGBMClassifier

        y = np.asarray(df[self.getLabelCol()], dtype=np.float64)
        k = int(y.max()) + 1 if len(y) else 2
        params = self._common()
        params.update(self._lgbm_params())
        if k > 2:
            params["objective"] = "multiclass"
        est = LightGBMClassifier(**params)
        inner = est.fit(df)
        m = self._model_cls(featuresCol=self.getFeaturesCol(), predictionCol=self.getPredictionCol(),
                            rawPredictionCol=self.getRawPredictionCol(), probabilityCol=self.getProbabilityCol())
        return m.set("inner", inner)


class _TreeRegressor(Estimator, _TreeParams):
    _model_cls = _WrappedModel

    def _lgbm_params(self) -> dict:
        raise NotImplementedError

    def _fit(self, df):
        from ..lightgbm import LightGBMRegressor

        params = self._common()
        params.update(self._lgbm_params())
        inner = LightGBMRegressor(**params).fit(df)
        m = self._model_cls(featuresCol=self.getFeaturesCol(), predictionCol=self.getPredictionCol())
        return m.set("inner", inner)


class DecisionTreeClassificationModel(_ClsModel):
    pass


class DecisionTreeClassifier(_TreeClassifier):
    _model_cls = DecisionTreeClassificationModel

    def _lgbm_params(self):
        return dict(numIterations=1, learningRate=1.0, boostFromAverage=True)


class DecisionTreeRegressionModel(_WrappedModel):
    pass


class DecisionTreeRegressor(_TreeRegressor):
    _model_cls = DecisionTreeRegressionModel

    def _lgbm_params(self):
        return dict(numIterations=1, learningRate=1.0)


class RandomForestClassificationModel(_ClsModel):
    pass


class _ForestParams(Params):
    numTrees = Param("Number of trees to train (>= 1)", 20, T.toInt)
    subsamplingRate = Param("Fraction of the training data used for learning each decision tree", 1.0, T.toFloat)
    featureSubsetStrategy = Param("auto | all | onethird | sqrt | log2 | (0.0-1.0]", "auto", T.toString)

    def _forest(self, n_features: int, classification: bool) -> dict:
        s = self.getFeatureSubsetStrategy()
        if s == "auto":
            s = "sqrt" if classification else "onethird"
        frac = {"all": 1.0, "onethird": 1.0 / 3, "sqrt": np.sqrt(max(1, n_features)) / max(1, n_features),
                "log2": np.log2(max(2, n_features)) / max(1, n_features)}.get(s)
        if frac is None:
            frac = float(s)
        sub = self.getSubsamplingRate()
        # SparkML samples the candidate features at every node (featureSubsetStrategy), LightGBM's
        # feature_fraction is per tree: the per-node form is feature_fraction_bynode
        return dict(boostingType="rf", numIterations=self.getNumTrees(), baggingFraction=min(sub, 0.999),
                    baggingFreq=1, featureFraction=1.0, featureFractionByNode=min(1.0, max(frac, 1e-6)))


class RandomForestClassifier(_TreeClassifier, _ForestParams):
    _model_cls = RandomForestClassificationModel

    def _fit(self, df):
        from ..core.linalg import as_matrix

        self._nf = as_matrix(df[self.getFeaturesCol()][:1]).shape[1] if df.count() else 1
        return super()._fit(df)

    def _lgbm_params(self):
        return self._forest(getattr(self, "_nf", 1), True)


class RandomForestRegressionModel(_WrappedModel):
    pass


class RandomForestRegressor(_TreeRegressor, _ForestParams):
    _model_cls = RandomForestRegressionModel

    def _fit(self, df):
        from ..core.linalg import as_matrix

        self._nf = as_matrix(df[self.getFeaturesCol()][:1]).shape[1] if df.count() else 1
        return super()._fit(df)

    def _lgbm_params(self):
        return self._forest(getattr(self, "_nf", 1), False)


class GBTClassificationModel(_ClsModel):
    pass


class _GBTParams(Params):
    maxIter = Param("max number of iterations (>= 0)", 20, T.toInt)
    stepSize = Param("Step size (learning rate) in interval (0, 1]", 0.1, T.toFloat)
    subsamplingRate = Param("Fraction of the training data used for learning each decision tree", 1.0, T.toFloat)

    def _gbt(self) -> dict:
        p = dict(numIterations=self.getMaxIter(), learningRate=self.getStepSize())
        if self.getSubsamplingRate() < 1.0:
            p.update(baggingFraction=self.getSubsamplingRate(), baggingFreq=1)
        return p


class GBTClassifier(_TreeClassifier, _GBTParams):
    _model_cls = GBTClassificationModel

    def _lgbm_params(self):
        return self._gbt()


class GBTRegressionModel(_WrappedModel):
    pass


class GBTRegressor(_TreeRegressor, _GBTParams):
    _model_cls = GBTRegressionModel

    def _lgbm_params(self):
        return self._gbt()
