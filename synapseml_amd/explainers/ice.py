"""ICE / PDP explainer (reference: core/.../explainers/ICEExplainer.scala:
126-364, ICEFeature.scala). For each explained feature the sampled rows are
replicated once per grid value, the whole grid is scored in one batched
model.transform, then grouped: ``individual`` — per-row map value → target
vector, ``average`` — PDP map value → mean target, ``feature`` — PDP-based
importance (std of the PDP for numeric features, (max − min)/4 for
categorical ones)."""
from __future__ import annotations

from typing import Dict, List

import numpy as np

from ..core.dataframe import DataFrame
from ..core.linalg import DenseVector
from ..core.params import Param, TypeConverters as T
from .local import LocalExplainer, _obj


class ICETransformer(LocalExplainer):
    categoricalFeatures = Param("The list of categorical features to explain ({name, numTopValues, outputColName})",
                                [], T.identity)
    numericFeatures = Param("The list of numeric features to explain ({name, numSplits, rangeMin, rangeMax, "
                            "outputColName})", [], T.identity)
    kind = Param("Whether to return the partial dependence plot (PDP) averaged across all the samples in the dataset "
                 "or individual feature importance (ICE) per instance", "individual", T.toString)
    featureNameCol = Param("Output column name which corresponds to names of the features used in calculation of "
                           "PDP-based-feature-importance option (kind == `feature`)", "featureNames", T.toString)
    dependenceNameCol = Param("Output column name which corresponds to dependence values of "
                              "PDP-based-feature-importance option (kind == `feature`)", "pdpBasedDependence",
                              T.toString)

    @staticmethod
    def _spec(f) -> dict:
        return dict(f) if isinstance(f, dict) else {"name": str(f)}

    def _values(self, df: DataFrame, f: dict, categorical: bool) -> list:
        col = df[f["name"]].tolist()
        if categorical:
            counts: Dict = {}
            for v in col:
                counts[v] = counts.get(v, 0) + 1
            top = sorted(counts, key=lambda k: (-counts[k], str(k)))[: int(f.get("numTopValues", 100))]
            return top
        x = np.asarray(col, dtype=np.float64)
        lo = f.get("rangeMin", float(np.nanmin(x)))
        hi = f.get("rangeMax", float(np.nanmax(x)))
        k = int(f.get("numSplits", 10))
        return list(np.linspace(lo, hi, k + 1))

    def _transform(self, df):
        kind = self.getKind().lower()
        n = self.getNumSamples()
        sampled = df
        if n:
            rng = np.random.default_rng(0)
            idx = np.sort(rng.permutation(df.count())[:n])
            sampled = df._take_rows(idx)
        classes = self._classes_for(sampled)
        feats = [(self._spec(f), True) for f in self.getCategoricalFeatures() or []] + \
                [(self._spec(f), False) for f in self.getNumericFeatures() or []]
        results_ind = {}
        pdp_cols = {}
        feat_rows = []
        m = sampled.count()
        for f, categorical in feats:
            name = f["name"]
            out_col = f.get("outputColName") or name + "_dependence"
            values = self._values(df, f, categorical)
            V = len(values)
            rep = sampled._take_rows(np.tile(np.arange(m), V))
            newcol = np.repeat(np.asarray(values, dtype=object if categorical else np.float64), m)
            if not categorical and sampled[name].dtype.kind in "iu":
                newcol = newcol.astype(sampled[name].dtype)
            rep = rep.withColumn(name, newcol if not categorical else _obj(list(newcol)))
            scored = self.getModel().transform(rep)
            tg = np.stack(self._targets(scored, classes * V))  # [V*m, K]
            tg = tg.reshape(V, m, -1)
            if kind == "individual":
                col = []
                for r in range(m):
                    col.append({values[v]: DenseVector(tg[v, r]) for v in range(V)})
                results_ind[out_col] = _obj(col)
            else:
                pdp = tg.mean(1)  # [V, K]
                if kind == "average":
                    pdp_cols[out_col] = _obj([{values[v]: DenseVector(pdp[v]) for v in range(V)}])
                else:
                    dep = (pdp.max(0) - pdp.min(0)) / 4.0 if categorical else pdp.std(0, ddof=1)
                    feat_rows.append((out_col, DenseVector(dep)))
        if kind == "individual":
            out = sampled
            for c, v in results_ind.items():
                out = out.withColumn(c, v)
            return out
        if kind == "average":
            return DataFrame(pdp_cols)
        return DataFrame({self.getFeatureNameCol(): _obj([r[0] for r in feat_rows]),
                          self.getDependenceNameCol(): _obj([r[1] for r in feat_rows])})
