"""Weighted least squares and Lasso used by the local explainers (reference:
core/.../explainers/{LeastSquaresRegression, LassoRegression,
RegressionBase}.scala). Solved per instance in float64."""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class RegressionResult:
    coefficients: np.ndarray
    intercept: float
    rSquared: float  # noqa: N815
    loss: float


def _r2(y, yhat, w):
    ym = np.sum(w * y) / np.sum(w)
    ss_tot = np.sum(w * (y - ym) ** 2)
    ss_res = np.sum(w * (y - yhat) ** 2)
    return float(1 - ss_res / ss_tot) if ss_tot > 0 else 1.0


def least_squares(X: np.ndarray, y: np.ndarray, w: np.ndarray, fit_intercept: bool = True) -> RegressionResult:
    X = np.asarray(X, np.float64)
    y = np.asarray(y, np.float64)
    w = np.asarray(w, np.float64)
    if fit_intercept:
        A = np.concatenate([np.ones((X.shape[0], 1)), X], axis=1)
    else:
        A = X
    sw = np.sqrt(w)[:, None]
    sol, *_ = np.linalg.lstsq(A * sw, y * sw[:, 0], rcond=None)
    b0 = float(sol[0]) if fit_intercept else 0.0
    coef = sol[1:] if fit_intercept else sol
    yhat = A @ sol
    return RegressionResult(coef, b0, _r2(y, yhat, w), float(np.sum(w * (y - yhat) ** 2) / np.sum(w)))


def lasso(X: np.ndarray, y: np.ndarray, w: np.ndarray, alpha: float, fit_intercept: bool = True,
          max_iter: int = 1000, tol: float = 1e-8) -> RegressionResult:
    """Weighted Lasso by coordinate descent: min 1/(2 Σw) Σ w (y - b0 - Xβ)² + alpha ||β||₁."""
    if alpha <= 0:
        return least_squares(X, y, w, fit_intercept)
    X = np.asarray(X, np.float64)
    y = np.asarray(y, np.float64)
    w = np.asarray(w, np.float64) / np.sum(w)
    if fit_intercept:
        xm = w @ X
        ym = float(w @ y)
    else:
        xm = np.zeros(X.shape[1])
        ym = 0.0
    Xc = X - xm
    yc = y - ym
    beta = np.zeros(X.shape[1])
    col_sq = (w[:, None] * Xc * Xc).sum(0)
    r = yc.copy()
    for _ in range(max_iter):
        max_d = 0.0
        for j in range(X.shape[1]):
            if col_sq[j] == 0:
                continue
            old = beta[j]
            rho = float((w * Xc[:, j]) @ r) + col_sq[j] * old
            new = np.sign(rho) * max(abs(rho) - alpha, 0.0) / col_sq[j]
            if new != old:
                r -= Xc[:, j] * (new - old)
                beta[j] = new
                max_d = max(max_d, abs(new - old))
        if max_d < tol:
            break
    b0 = ym - float(xm @ beta) if fit_intercept else 0.0
    yhat = X @ beta + b0
    return RegressionResult(beta, b0, _r2(y, yhat, w), float(np.sum(w * (y - yhat) ** 2)))
