"""Data-balance analysis (reference: core/.../exploratory/
{AggregateBalanceMeasure, DistributionBalanceMeasure, FeatureBalanceMeasure,
DataBalanceParams}.scala). Outputs are dicts keyed by the reference's metric
names (the reference's struct columns)."""
from __future__ import annotations

from typing import Dict, List

import numpy as np

from ..core.contracts import HasLabelCol, HasOutputCol
from ..core.dataframe import DataFrame
from ..core.params import Param, Params, TypeConverters as T
from ..core.pipeline import Transformer


def _obj(values) -> np.ndarray:
    arr = np.empty(len(values), dtype=object)
    for i, v in enumerate(values):
        arr[i] = v
    return arr


class _DataBalanceParams(HasOutputCol):
    sensitiveCols = Param("Sensitive columns to use.", [], T.toListString)
    verbose = Param("Whether to show intermediate measures and calculations, such as Positive Rate.", False,
                    T.toBoolean)


def _counts(df: DataFrame, cols: List[str]) -> Dict[tuple, int]:
    out: Dict[tuple, int] = {}
    for k in zip(*[df[c].tolist() for c in cols]):
        out[k] = out.get(k, 0) + 1
    return out


class AggregateBalanceMeasure(Transformer, _DataBalanceParams):
    epsilon = Param("Epsilon value for Atkinson Index. Inverse of alpha (1 - alpha).", 1.0, T.toFloat)
    errorTolerance = Param("Error tolerance value for Atkinson Index.", 1e-12, T.toFloat)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(outputCol="AggregateBalanceMeasure")

    def _transform(self, df):
        n = df.count()
        p = np.asarray(list(_counts(df, self.getSensitiveCols()).values()), dtype=np.float64) / n
        k = len(p)
        norm = p / p.mean()
        alpha = 1.0 - self.getEpsilon()
        if abs(alpha) < self.getErrorTolerance():
            atk = 1.0 - np.exp(np.log(norm).sum()) ** (1.0 / k)
        else:
            atk = 1.0 - ((norm ** alpha).sum() / k) ** (1.0 / alpha)
        res = {"atkinson_index": float(atk), "theil_l_index": float((-np.log(norm)).sum() / k),
               "theil_t_index": float((norm * np.log(norm)).sum() / k)}
        return DataFrame({self.getOutputCol(): _obj([res])})


class DistributionBalanceMeasure(Transformer, _DataBalanceParams):
    featureNameCol = Param("Output column name for feature names.", "FeatureName", T.toString)
    referenceDistribution = Param("An ordered list of reference distributions that correspond to each of the "
                                  "sensitive columns.", None, T.identity)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(outputCol="DistributionBalanceMeasure")

    def _transform(self, df):
        from scipy import stats

        n = df.count()
        names, results = [], []
        refs = self.getReferenceDistribution()
        if refs is not None and len(refs) != len(self.getSensitiveCols()):
            raise ValueError("The reference distribution must have the same length and order as the sensitive "
                             "columns: " + ", ".join(self.getSensitiveCols()))
        for i, c in enumerate(self.getSensitiveCols()):
            cnt = _counts(df, [c])
            keys = [k[0] for k in cnt]
            obs_c = np.asarray([cnt[(k,)] for k in keys], dtype=np.float64)
            obs_p = obs_c / n
            m = len(keys)
            if refs is None or not refs[i]:
                ref_p = np.full(m, 1.0 / m)
            else:
                ref_p = np.asarray([float(refs[i].get(str(k), refs[i].get(k, 0.0))) for k in keys])
            ref_c = ref_p * n

            def rel_entr(a, b):
                tot = 0.0
                for x, z in zip(a, b):
                    if x == 0 and z >= 0:
                        continue
                    if x > 0 and z > 0:
                        tot += x * np.log(x / z)
                    else:
                        return float("inf")
                return float(tot)

            avg = (obs_p + ref_p) / 2
            chi = np.where((ref_c == 0) & (obs_c != 0), np.inf,
                           (obs_c - ref_c) ** 2 / np.where(ref_c == 0, 1, ref_c)).sum()
            res = {"kl_divergence": rel_entr(obs_p, ref_p),
                   "js_dist": float(np.sqrt((rel_entr(ref_p, avg) + rel_entr(obs_p, avg)) / 2)),
                   "inf_norm_dist": float(np.abs(obs_p - ref_p).max()),
                   "total_variation_dist": float(np.abs(obs_p - ref_p).sum() * 0.5),
                   "wasserstein_dist": float(np.abs(obs_p - ref_p).mean()),
                   "chi_sq_stat": float(chi),
                   "chi_sq_p_value": 1.0 if np.isinf(chi) else float(1 - stats.chi2.cdf(chi, m - 1))}
            names.append(c)
            results.append(res)
        return DataFrame({self.getFeatureNameCol(): _obj(names), self.getOutputCol(): _obj(results)})


class FeatureBalanceMeasure(Transformer, _DataBalanceParams, HasLabelCol):
    featureNameCol = Param("Output column name for feature names.", "FeatureName", T.toString)
    classACol = Param("Output column name for the first feature value to compare.", "ClassA", T.toString)
    classBCol = Param("Output column name for the second feature value to compare.", "ClassB", T.toString)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(outputCol="FeatureBalanceMeasure")

    @staticmethod
    def _assoc(pos_feat, feat, pos, total) -> Dict[str, float]:
        pY, pX, pXY = pos / total, feat / total, pos_feat / total
        with np.errstate(divide="ignore", invalid="ignore"):
            dp = pXY / pX
            pmi = -np.inf if dp == 0 else float(np.log(dp))
            a = total ** 2 * (1 - 2 * pX - 2 * pY + 2 * pXY + 2 * pX * pY)
            b = total * (2 * pX + 2 * pY - 4 * pXY - 1)
            c = total ** 2 * np.sqrt((pX - pX ** 2) * (pY - pY ** 2))
            return {"dp": float(dp), "sdc": float(pXY / (pX + pY)), "ji": float(pXY / (pX + pY - pXY)),
                    "llr": float(np.log(pXY / pY)) if pXY > 0 else -np.inf, "pmi": pmi,
                    "n_pmi_y": 0.0 if pY == 0 else pmi / float(np.log(pY)),
                    "n_pmi_xy": 0.0 if pXY == 0 else pmi / float(np.log(pXY)),
                    "s_pmi": 0.0 if pX * pY == 0 else float(np.log(pXY ** 2 / (pX * pY))) if pXY > 0 else -np.inf,
                    "krc": float((a + b) / c) if c else np.nan,
                    "t_test": float((pXY - pX * pY) / np.sqrt(pX * pY))}

    def _transform(self, df):
        y = (np.asarray(df[self.getLabelCol()], np.float64).astype(np.int64) > 0).astype(np.float64)
        n = float(len(y))
        pos = float(y.sum())
        names, ca, cb, res = [], [], [], []
        for c in self.getSensitiveCols():
            vals = df[c].tolist()
            stats_ = {}
            for v, t in zip(vals, y):
                pf, f = stats_.get(v, (0.0, 0.0))
                stats_[v] = (pf + t, f + 1)
            metrics = {v: self._assoc(pf, f, pos, n) for v, (pf, f) in stats_.items()}
            keys = sorted(metrics, key=lambda v: (str(type(v)), v))
            for a in keys:
                for b in keys:
                    if not (a > b):
                        continue
                    gaps = {m: (0.0 if metrics[a][m] == metrics[b][m] else metrics[a][m] - metrics[b][m])
                            for m in metrics[a]}
                    if self.getVerbose():
                        gaps["prA"], gaps["prB"] = metrics[a]["dp"], metrics[b]["dp"]
                    names.append(c)
                    ca.append(a)
                    cb.append(b)
                    res.append(gaps)
        return DataFrame({self.getFeatureNameCol(): _obj(names), self.getClassACol(): _obj(ca),
                          self.getClassBCol(): _obj(cb), self.getOutputCol(): _obj(res)})


__all__ = ["AggregateBalanceMeasure", "DistributionBalanceMeasure", "FeatureBalanceMeasure"]
