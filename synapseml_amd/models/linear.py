"""Base learners the reference borrows from SparkML (used by TrainClassifier /
TrainRegressor / TuneHyperparameters / the explainers' tests): logistic and
linear regression, naive Bayes, multilayer perceptron. GEMM-shaped training
runs on the GPU through torch (L-BFGS on the device) when one is visible;
tree learners live in trees.py on top of the native GBDT engine."""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from ..core.contracts import (HasFeaturesCol, HasLabelCol, HasPredictionCol, HasProbabilityCol, HasRawPredictionCol,
                              HasSeed, HasWeightCol)
from ..core.dataframe import DataFrame
from ..core.linalg import DenseVector, SparseVector, Vector, as_matrix
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Estimator, Model


def _device():
    import torch

    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


def features_matrix(df: DataFrame, col: str) -> np.ndarray:
    return np.asarray(as_matrix(df[col]), dtype=np.float64)


class _ProbModelMixin:
    def _emit(self, df: DataFrame, raw: np.ndarray, prob: np.ndarray) -> DataFrame:
        out = df.withColumn(self.getRawPredictionCol(), raw).withColumn(self.getProbabilityCol(), prob)
        pred = np.argmax(prob, axis=1).astype(np.float64)
        th = getattr(self, "getThresholds", None)
        if th is not None and th():
            t = np.asarray(th(), dtype=np.float64)
            scaled = prob / np.where(t > 0, t, 1e-300)
            pred = np.argmax(scaled, axis=1).astype(np.float64)
        return out.withColumn(self.getPredictionCol(), pred)


# ---------------------------------------------------------------------- logistic regression
class LogisticRegressionModel(Model, HasFeaturesCol, HasPredictionCol, HasRawPredictionCol, HasProbabilityCol,
                              _ProbModelMixin):
    coefficientMatrix = Param("coefficients (numClasses x numFeatures)", None, complex=True)
    interceptVector = Param("intercepts (numClasses)", None, complex=True)
    numClasses = Param("number of classes", 2, T.toInt)
    thresholds = Param("per-class thresholds", None, T.toListFloat)

    @property
    def coefficients(self) -> DenseVector:
        W = np.asarray(self.getCoefficientMatrix())
        return DenseVector(W[-1] if W.shape[0] == 1 or self.getNumClasses() == 2 else W.ravel())

    @property
    def intercept(self) -> float:
        return float(np.asarray(self.getInterceptVector())[-1])

    def _scores(self, X: np.ndarray) -> np.ndarray:
        W = np.asarray(self.getCoefficientMatrix())
        b = np.asarray(self.getInterceptVector())
        return X @ W.T + b

    def _transform(self, df):
        X = features_matrix(df, self.getFeaturesCol())
        s = self._scores(X)
        if s.shape[1] == 1:
            raw = np.concatenate([-s, s], axis=1)
            from scipy.special import expit

            p1 = expit(s[:, 0])  # overflow-free logistic
            prob = np.stack([1 - p1, p1], axis=1)
        else:
            raw = s
            e = np.exp(s - s.max(1, keepdims=True))
            prob = e / e.sum(1, keepdims=True)
        return self._emit(df, raw, prob)


class LogisticRegression(Estimator, HasFeaturesCol, HasLabelCol, HasWeightCol, HasPredictionCol,
                         HasRawPredictionCol, HasProbabilityCol):
    maxIter = Param("max number of iterations", 100, T.toInt)
    regParam = Param("regularization parameter (L2 when elasticNetParam = 0)", 0.0, T.toFloat)
    elasticNetParam = Param("ElasticNet mixing parameter in [0, 1]", 0.0, T.toFloat)
    tol = Param("convergence tolerance", 1e-6, T.toFloat)
    fitIntercept = Param("whether to fit an intercept term", True, T.toBoolean)
    standardization = Param("whether to standardize features before fitting", True, T.toBoolean)
    family = Param("auto | binomial | multinomial", "auto", T.toString)
    thresholds = Param("per-class thresholds", None, T.toListFloat)
    threshold = Param("binary threshold", 0.5, T.toFloat)

    def _fit(self, df):
        import torch

        X = features_matrix(df, self.getFeaturesCol())
        y = np.asarray(df[self.getLabelCol()], dtype=np.float64).astype(np.int64)
        w = np.asarray(df[self.getWeightCol()], dtype=np.float64) if self.getWeightCol() else np.ones(len(y))
        k = int(y.max()) + 1 if len(y) else 2
        k = max(k, 2)
        binomial = self.getFamily() == "binomial" or (self.getFamily() == "auto" and k == 2)
        W, b = fit_logistic(X, y, w, k, binomial, self.getRegParam(), self.getElasticNetParam(), self.getMaxIter(),
                            self.getTol(), self.getFitIntercept(), self.getStandardization())
        thr = self.getThresholds()
        if thr is None and binomial and self.getThreshold() != 0.5:
            t = self.getThreshold()
            thr = [1 - t, t]
        m = LogisticRegressionModel(featuresCol=self.getFeaturesCol(), predictionCol=self.getPredictionCol(),
                                    rawPredictionCol=self.getRawPredictionCol(),
                                    probabilityCol=self.getProbabilityCol(), numClasses=k, thresholds=thr)
        m.set("coefficientMatrix", W)
        m.set("interceptVector", b)
        del torch
        return m


def fit_logistic(X, y, w, k, binomial, reg, enet, max_iter, tol, fit_intercept, standardize):
    """L-BFGS on the device; L2 penalty on standardized coefficients (Spark semantics), L1 part via a
    smooth pseudo-Huber approximation."""
    import torch

    dev = _device()
    Xt = torch.as_tensor(X, dtype=torch.float32, device=dev)
    mu = Xt.mean(0) if standardize else torch.zeros(Xt.shape[1], device=dev)
    sd = Xt.std(0, unbiased=True) if standardize and Xt.shape[0] > 1 else torch.ones(Xt.shape[1], device=dev)
    sd = torch.where(sd > 0, sd, torch.ones_like(sd))
    Xs = (Xt - mu) / sd if standardize else Xt
    yt = torch.as_tensor(y, device=dev)
    wt = torch.as_tensor(w, dtype=torch.float32, device=dev)
    ncoef = 1 if binomial else k
    Wp = torch.zeros(ncoef, X.shape[1], device=dev, requires_grad=True)
    bp = torch.zeros(ncoef, device=dev, requires_grad=fit_intercept)
    opt = torch.optim.LBFGS([Wp] + ([bp] if fit_intercept else []), max_iter=max(1, max_iter), tolerance_grad=tol,
                            tolerance_change=tol * 1e-3, history_size=10, line_search_fn="strong_wolfe")
    wsum = wt.sum()
    l2 = reg * (1 - enet)
    l1 = reg * enet

    def closure():
        opt.zero_grad()
        s = Xs @ Wp.T + bp
        if binomial:
            loss = torch.nn.functional.binary_cross_entropy_with_logits(s[:, 0], yt.float(), weight=wt,
                                                                        reduction="sum") / wsum
        else:
            loss = (torch.nn.functional.cross_entropy(s, yt, reduction="none") * wt).sum() / wsum
        if l2 > 0:
            loss = loss + 0.5 * l2 * (Wp * Wp).sum()
        if l1 > 0:
            loss = loss + l1 * torch.sqrt(Wp * Wp + 1e-8).sum()
        loss.backward()
        return loss

    opt.step(closure)
    with torch.no_grad():
        W = (Wp / sd).cpu().double().numpy()
        b = (bp - (Wp / sd) @ mu).cpu().double().numpy() if standardize else bp.cpu().double().numpy()
    return W, b


# ---------------------------------------------------------------------- linear regression
class LinearRegressionModel(Model, HasFeaturesCol, HasPredictionCol):
    coefficients_ = Param("coefficients", None, complex=True)
    intercept_ = Param("intercept", 0.0, T.toFloat)

    @property
    def coefficients(self) -> DenseVector:
        return DenseVector(np.asarray(self.getCoefficients_()))

    @property
    def intercept(self) -> float:
        return float(self.getIntercept_())

    def _transform(self, df):
        X = features_matrix(df, self.getFeaturesCol())
        return df.withColumn(self.getPredictionCol(), X @ np.asarray(self.getCoefficients_()) + self.getIntercept_())


class LinearRegression(Estimator, HasFeaturesCol, HasLabelCol, HasWeightCol, HasPredictionCol):
    maxIter = Param("max number of iterations", 100, T.toInt)
    regParam = Param("regularization parameter", 0.0, T.toFloat)
    elasticNetParam = Param("ElasticNet mixing parameter", 0.0, T.toFloat)
    fitIntercept = Param("whether to fit an intercept term", True, T.toBoolean)
    standardization = Param("whether to standardize the training features", True, T.toBoolean)
    solver = Param("auto | normal | l-bfgs", "auto", T.toString)
    tol = Param("convergence tolerance", 1e-6, T.toFloat)

    def _fit(self, df):
        X = features_matrix(df, self.getFeaturesCol())
        y = np.asarray(df[self.getLabelCol()], dtype=np.float64)
        w = np.asarray(df[self.getWeightCol()], dtype=np.float64) if self.getWeightCol() else np.ones(len(y))
        coef, icpt = fit_linear(X, y, w, self.getRegParam(), self.getFitIntercept(), self.getStandardization())
        m = LinearRegressionModel(featuresCol=self.getFeaturesCol(), predictionCol=self.getPredictionCol())
        m.set("coefficients_", coef)
        m.set("intercept_", icpt)
        return m


def fit_linear(X, y, w, reg=0.0, fit_intercept=True, standardize=True) -> Tuple[np.ndarray, float]:
    """Weighted ridge via the normal equations (the Gram matrix is one device GEMM)."""
    import torch

    dev = _device()
    Xt = torch.as_tensor(X, dtype=torch.float64, device=dev)
    yt = torch.as_tensor(y, dtype=torch.float64, device=dev)
    wt = torch.as_tensor(w, dtype=torch.float64, device=dev)
    ws = wt.sum()
    if fit_intercept:
        xm = (Xt * wt[:, None]).sum(0) / ws
        ym = (yt * wt).sum() / ws
    else:
        xm = torch.zeros(Xt.shape[1], dtype=torch.float64, device=dev)
        ym = torch.zeros((), dtype=torch.float64, device=dev)
    Xc = Xt - xm
    yc = yt - ym
    sd = torch.sqrt(((Xc * Xc) * wt[:, None]).sum(0) / ws) if standardize else torch.ones_like(xm)
    sd = torch.where(sd > 0, sd, torch.ones_like(sd))
    Xn = Xc / sd
    G = (Xn * wt[:, None]).T @ Xn / ws
    r = (Xn * wt[:, None]).T @ yc / ws
    lam = reg * torch.eye(G.shape[0], dtype=torch.float64, device=dev)
    beta = torch.linalg.lstsq(G + lam, r.unsqueeze(1)).solution.squeeze(1) / sd
    icpt = (ym - xm @ beta) if fit_intercept else torch.zeros((), dtype=torch.float64)
    return beta.cpu().numpy(), float(icpt)


# ---------------------------------------------------------------------- naive Bayes
class NaiveBayesModel(Model, HasFeaturesCol, HasPredictionCol, HasRawPredictionCol, HasProbabilityCol,
                      _ProbModelMixin):
    pi = Param("log class priors", None, complex=True)
    theta = Param("log conditional probabilities", None, complex=True)
    modelType = Param("multinomial | bernoulli | gaussian", "multinomial", T.toString)
    sigma = Param("per-class variances (gaussian)", None, complex=True)
    thresholds = Param("per-class thresholds", None, T.toListFloat)

    def _transform(self, df):
        X = features_matrix(df, self.getFeaturesCol())
        pi, th = np.asarray(self.getPi()), np.asarray(self.getTheta())
        mt = self.getModelType()
        if mt == "multinomial":
            raw = X @ th.T + pi
        elif mt == "bernoulli":
            neg = np.log1p(-np.exp(th))
            raw = X @ (th - neg).T + neg.sum(1) + pi
        else:
            var = np.asarray(self.getSigma())
            raw = pi - 0.5 * (np.log(2 * np.pi * var).sum(1) + (((X[:, None, :] - th[None]) ** 2) / var[None]).sum(2))
        e = np.exp(raw - raw.max(1, keepdims=True))
        return self._emit(df, raw, e / e.sum(1, keepdims=True))


class NaiveBayes(Estimator, HasFeaturesCol, HasLabelCol, HasWeightCol, HasPredictionCol, HasRawPredictionCol,
                 HasProbabilityCol):
    smoothing = Param("The smoothing parameter", 1.0, T.toFloat)
    modelType = Param("multinomial | bernoulli | gaussian", "multinomial", T.toString)

    def _fit(self, df):
        X = features_matrix(df, self.getFeaturesCol())
        y = np.asarray(df[self.getLabelCol()], dtype=np.int64)
        w = np.asarray(df[self.getWeightCol()], dtype=np.float64) if self.getWeightCol() else np.ones(len(y))
        k = int(y.max()) + 1
        lam = self.getSmoothing()
        counts = np.bincount(y, weights=w, minlength=k)
        pi = np.log(counts + lam) - np.log(counts.sum() + k * lam)
        mt = self.getModelType()
        m = NaiveBayesModel(featuresCol=self.getFeaturesCol(), predictionCol=self.getPredictionCol(),
                            rawPredictionCol=self.getRawPredictionCol(), probabilityCol=self.getProbabilityCol(),
                            modelType=mt)
        if mt == "gaussian":
            mean = np.stack([np.average(X[y == c], axis=0, weights=w[y == c]) for c in range(k)])
            var = np.stack([np.average((X[y == c] - mean[c]) ** 2, axis=0, weights=w[y == c]) for c in range(k)])
            var = var + 1e-9 * X.var(0).max()
            m.set("theta", mean)
            m.set("sigma", var)
        else:
            if (X < 0).any():
                raise ValueError("Naive Bayes requires nonnegative feature values")
            if mt == "bernoulli":
                X = (X > 0).astype(np.float64)
            fc = np.stack([(X[y == c] * w[y == c, None]).sum(0) for c in range(k)])
            if mt == "multinomial":
                th = np.log(fc + lam) - np.log(fc.sum(1, keepdims=True) + X.shape[1] * lam)
            else:
                th = np.log(fc + lam) - np.log(counts[:, None] + 2 * lam)
            m.set("theta", th)
        m.set("pi", pi)
        return m


# ---------------------------------------------------------------------- MLP
class MultilayerPerceptronClassificationModel(Model, HasFeaturesCol, HasPredictionCol, HasRawPredictionCol,
                                              HasProbabilityCol, _ProbModelMixin):
    layers = Param("layer sizes including input and output", [], T.toListInt)
    weights = Param("flattened weights", None, complex=True)
    thresholds = Param("per-class thresholds", None, T.toListFloat)

    def _net(self):
        import torch

        layers = self.getLayers()
        mods = []
        for i in range(len(layers) - 1):
            mods.append(torch.nn.Linear(layers[i], layers[i + 1]).double())
            if i < len(layers) - 2:
                mods.append(torch.nn.Sigmoid())
        net = torch.nn.Sequential(*mods)
        torch.nn.utils.vector_to_parameters(torch.as_tensor(np.asarray(self.getWeights()), dtype=torch.float64),
                                            net.parameters())
        return net

    def _transform(self, df):
        import torch

        X = torch.as_tensor(features_matrix(df, self.getFeaturesCol()), dtype=torch.float64)
        with torch.no_grad():
            raw = self._net()(X).numpy()
        e = np.exp(raw - raw.max(1, keepdims=True))
        return self._emit(df, raw, e / e.sum(1, keepdims=True))


class MultilayerPerceptronClassifier(Estimator, HasFeaturesCol, HasLabelCol, HasPredictionCol, HasRawPredictionCol,
                                     HasProbabilityCol, HasSeed):
    layers = Param("Sizes of layers from input layer to output layer", [], T.toListInt)
    maxIter = Param("max number of iterations", 100, T.toInt)
    stepSize = Param("Step size (learning rate) for gd", 0.03, T.toFloat)
    solver = Param("l-bfgs | gd", "l-bfgs", T.toString)
    blockSize = Param("Block size for stacking input data in matrices", 128, T.toInt)
    tol = Param("convergence tolerance", 1e-6, T.toFloat)

    def _fit(self, df):
        import torch

        torch.manual_seed(self.getSeed())
        dev = _device()
        X = torch.as_tensor(features_matrix(df, self.getFeaturesCol()), dtype=torch.float32, device=dev)
        y = torch.as_tensor(np.asarray(df[self.getLabelCol()], dtype=np.int64), device=dev)
        layers = self.getLayers()
        mods = []
        for i in range(len(layers) - 1):
            mods.append(torch.nn.Linear(layers[i], layers[i + 1]))
            if i < len(layers) - 2:
                mods.append(torch.nn.Sigmoid())
        net = torch.nn.Sequential(*mods).to(dev)
        if self.getSolver() == "l-bfgs":
            opt = torch.optim.LBFGS(net.parameters(), max_iter=self.getMaxIter(), tolerance_grad=self.getTol(),
                                    line_search_fn="strong_wolfe")

            def closure():
                opt.zero_grad()
                loss = torch.nn.functional.cross_entropy(net(X), y)
                loss.backward()
                return loss

            opt.step(closure)
        else:
            opt = torch.optim.SGD(net.parameters(), lr=self.getStepSize())
            for _ in range(self.getMaxIter()):
                for s in range(0, X.shape[0], self.getBlockSize()):
                    opt.zero_grad()
                    torch.nn.functional.cross_entropy(net(X[s:s + self.getBlockSize()]),
                                                      y[s:s + self.getBlockSize()]).backward()
                    opt.step()
        wvec = torch.nn.utils.parameters_to_vector(net.parameters()).detach().cpu().double().numpy()
        m = MultilayerPerceptronClassificationModel(featuresCol=self.getFeaturesCol(),
                                                    predictionCol=self.getPredictionCol(),
                                                    rawPredictionCol=self.getRawPredictionCol(),
                                                    probabilityCol=self.getProbabilityCol(), layers=layers)
        m.set("weights", wvec)
        return m
