"""Model-agnostic local explainers (reference: core/.../explainers/
{LocalExplainer, KernelSHAPBase, KernelSHAPSampler, LIMEBase, LIMESampler,
TabularSHAP, VectorSHAP, ImageSHAP, TextSHAP, TabularLIME, VectorLIME,
ImageLIME, TextLIME, SharedParams}.scala).

For every instance a set of perturbed samples is generated, ALL samples of
ALL instances are scored by the wrapped model in one batched ``transform``
(the hot path — the wrapped model runs on the GPU when it is a GPU model),
then a weighted least-squares (KernelSHAP) or Lasso (LIME) fit per instance
and target class yields the explanation vectors and their r² (metricsCol).

KernelSHAP output per target class: [φ₀, φ₁, …, φ_M] (intercept first);
LIME output per target class: [β₁, …, β_M]."""
from __future__ import annotations

from math import comb
from typing import Any, List, Optional, Tuple

import numpy as np

from ..core.contracts import HasInputCol, HasInputCols, HasOutputCol
from ..core.dataframe import DataFrame
from ..core.linalg import DenseVector, SparseVector, Vector
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Transformer
from .regression import lasso, least_squares
from .superpixel import censor, slic


def _obj(values) -> np.ndarray:
    arr = np.empty(len(values), dtype=object)
    for i, v in enumerate(values):
        arr[i] = v
    return arr


class LocalExplainer(Transformer, HasOutputCol):
    model = Param("The model to be interpreted.", None, complex=True)
    targetCol = Param("The column name of the prediction target to explain (i.e. the response variable).",
                      "probability", T.toString)
    targetClasses = Param("The indices of the classes for multinomial classification models. Default: 0.", [],
                          T.toListInt)
    targetClassesCol = Param("The name of the column that specifies the indices of the classes", None, T.toString)
    metricsCol = Param("Column name for fitting metrics", "r2", T.toString)
    numSamples = Param("Number of samples to generate.", None, T.toInt)

    # ---- target extraction (SharedParams.extractTarget)
    def _targets(self, scored: DataFrame, classes_per_row: List[List[int]]) -> List[np.ndarray]:
        col = scored[self.getTargetCol()]
        out = []
        if col.ndim == 2:
            mat = col.astype(np.float64)
            for i, cls in enumerate(classes_per_row):
                out.append(mat[i, cls] if cls else mat[i])
            return out
        for i, v in enumerate(col.tolist()):
            cls = classes_per_row[i]
            if isinstance(v, dict):
                keys = cls if cls else sorted(v)
                out.append(np.asarray([float(v[k]) for k in keys]))
            elif isinstance(v, (Vector, list, tuple, np.ndarray)):
                a = np.asarray(v.toArray() if isinstance(v, Vector) else v, dtype=np.float64).reshape(-1)
                out.append(a[cls] if cls else a)
            else:
                out.append(np.asarray([float(v)]))
        return out

    def _classes_for(self, df: DataFrame) -> List[List[int]]:
        if self.getTargetClassesCol():
            return [list(v) if v is not None else [] for v in df[self.getTargetClassesCol()].tolist()]
        return [list(self.getTargetClasses() or [])] * df.count()

    # subclass API --------------------------------------------------------------
    def _prepare(self, df: DataFrame) -> Any:
        return None

    def _num_features(self, df: DataFrame, i: int, ctx) -> int:
        raise NotImplementedError

    def _samples(self, df: DataFrame, i: int, ctx, rng) -> Tuple[np.ndarray, np.ndarray, DataFrame]:
        """-> (regression inputs [S, M], sample weights [S], DataFrame of rows to score [S * R])."""
        raise NotImplementedError

    def _fit(self, X, y, w) -> Tuple[np.ndarray, float]:
        raise NotImplementedError

    def _transform(self, df):
        if self.getModel() is None:
            raise ValueError("model must be set")
        ctx = self._prepare(df)
        rng = np.random.default_rng(getattr(self, "_seed", 0))
        n = df.count()
        per = []
        frames = []
        for i in range(n):
            X, w, rows = self._samples(df, i, ctx, rng)
            reps = rows.count() // max(1, X.shape[0])
            per.append((X, w, reps, rows.count()))
            frames.append(rows)
        scored = self.getModel().transform(DataFrame.union_all(frames)) if frames else None
        classes = self._classes_for(df)
        outs, metrics = [], []
        off = 0
        for i, (X, w, reps, cnt) in enumerate(per):
            part = scored.slice(off, off + cnt)
            off += cnt
            tg = np.stack(self._targets(part, [classes[i]] * cnt))  # [S*R, K]
            y = tg.reshape(X.shape[0], reps, -1).mean(1)  # average over background rows
            vecs, r2s = [], []
            for k in range(y.shape[1]):
                coef, r2 = self._fit(X, y[:, k], w)
                vecs.append(DenseVector(coef))
                r2s.append(r2)
            outs.append(vecs)
            metrics.append(DenseVector(r2s))
        return df.withColumn(self.getOutputCol(), _obj(outs)).withColumn(self.getMetricsCol(), _obj(metrics))


# ---------------------------------------------------------------------- KernelSHAP
def effective_num_samples(num_samples, m: int) -> int:
    """coalition budget: the numSamples param (default 2 * M + 2048, shap's default) clamped to
    [M + 2, 2^M] (KernelSHAPBase.scala:132-139)"""
    value = num_samples if num_samples else 2 * m + 2048
    return int(min(max(value, m + 2), 2 ** m if m < 63 else value))


def shap_sample_sizes(m: int, num_samples: int, kernel_weight) -> List[Tuple[int, float]]:
    """(number of coalitions, weight) per coalition-size slot, in the reference's order
    (KernelSHAPSampler.scala generateSampleSizes): sizes k and M - k are paired slots (k < M / 2), the
    Shapley-kernel size weights (M - 1) / (k (M - k)) (doubled for paired slots) decide how the budget is
    shared. While a size class fits its share completely it is enumerated exactly (weight kernel_weight(k));
    the budget left over is then spread over the remaining sizes (paired: ceil(share / 2) each side, or one
    coalition on the k side when the share is below one) with unit weight."""
    if not (m > 0 and 0 < num_samples <= 2 ** m - 2):
        raise ValueError(f"need M > 0 and 0 < numSamples <= 2^M - 2 (M={m}, numSamples={num_samples})")
    num_subsets, num_paired = m // 2, (m - 1) // 2
    w = np.array([(m - 1) / (i * (m - i)) for i in range(1, num_subsets + 1)], dtype=np.float64)
    w[:num_paired] *= 2.0

    def share(k: int) -> float:
        return float(w[k - 1] / w[k - 1:].sum())

    out: List[Tuple[int, float]] = []
    left = num_samples
    k = 1
    while k <= num_subsets:
        paired = k <= num_paired
        combo = comb(m, k) * (2 if paired else 1)
        if share(k) * left < combo:
            break
        sizes = [combo // 2, combo // 2] if paired else [combo]
        out += [(int(x), kernel_weight(k)) for x in sizes]
        left -= sum(sizes)
        if left <= 0:
            break
        k += 1
    remaining = num_samples - sum(x for x, _ in out)
    if remaining > 0:
        k, left, rest = len(out) // 2 + 1, remaining, []
        while True:
            alloc = share(k) * left
            if k <= num_paired:
                sizes = [int(np.ceil(alloc / 2))] * 2 if alloc >= 1 else [1, 0]
            else:
                sizes = [int(alloc)]
            rest += sizes
            left -= sum(sizes)
            if left <= 0:
                break
            k += 1
        out += [(x, 1.0) for x in rest]
    return out


def shap_coalitions(m: int, num_samples: int, rng, inf_weight: float) -> Tuple[np.ndarray, np.ndarray]:
    """Coalitions and weights of KernelSHAP (KernelSHAPSampler.scala generateCoalitions): the empty and the
    full coalition with weight infWeight, then the slots of :func:`shap_sample_sizes` - slot i covers size
    i / 2 (even i) or M - (i - 1) / 2 (odd i); a slot holding every coalition of its size enumerates them,
    otherwise its coalitions are drawn uniformly at random. The kernel weight of an enumerated size follows
    the reference, which uses the sample budget N where the Shapley kernel has M:
    (N - 1) / (k (N - k)) / C(M, k)."""
    import itertools

    if m == 0:
        return np.zeros((1, 0)), np.ones(1)
    n = effective_num_samples(num_samples, m)
    kern = lambda k: (n - 1) / (k * (n - k)) / comb(m, k)  # noqa: E731
    slots = [(1, inf_weight), (1, inf_weight)] + (shap_sample_sizes(m, n - 2, kern) if n > 2 else [])
    rows, weights = [], []
    for i, (size, wt) in enumerate(slots):
        k = i // 2 if i % 2 == 0 else m - (i - 1) // 2
        if size <= 0:
            continue
        if size == comb(m, k):
            subsets = itertools.combinations(range(m), k)
        else:
            subsets = (rng.permutation(m)[:k] for _ in range(size))
        for sub in subsets:
            z = np.zeros(m)
            z[list(sub)] = 1.0
            rows.append(z)
            weights.append(wt)
    return np.asarray(rows), np.asarray(weights, dtype=np.float64)


class _KernelSHAPBase(LocalExplainer):
    infWeight = Param("The double value to represent infinite weight. Default: 1E8.", 1e8, T.toFloat)

    def _budget(self, m: int) -> int:
        return effective_num_samples(self.getNumSamples(), m)

    def _fit(self, X, y, w):
        r = least_squares(X, y, w, fit_intercept=True)
        return np.concatenate([[r.intercept], r.coefficients]), r.rSquared


def _background_values(bg: DataFrame, cols: List[str]) -> List[np.ndarray]:
    return [bg[c] for c in cols]


class TabularSHAP(_KernelSHAPBase, HasInputCols):
    backgroundData = Param("A dataframe containing background data", None, complex=True)

    def _prepare(self, df):
        bg = self.getBackgroundData() if self.getBackgroundData() is not None else df
        return bg

    def _samples(self, df, i, bg, rng):
        cols = self.getInputCols()
        m = len(cols)
        Z, w = shap_coalitions(m, self._budget(m), rng, self.getInfWeight())
        B = bg.count()
        S = Z.shape[0]
        inst = {c: df[c][i] for c in cols}
        rows = {}
        for c in df.columns:
            base = np.repeat(df[c][i:i + 1], S * B, axis=0)
            rows[c] = base
        for j, c in enumerate(cols):
            bgc = bg[c]
            vals = np.tile(bgc, (S,) + (1,) * (bgc.ndim - 1)) if bgc.ndim > 1 else np.tile(bgc, S)
            take = np.repeat(Z[:, j] > 0, B)
            col = vals.copy() if vals.dtype != object else vals.copy()
            if col.dtype == object:
                for t in np.nonzero(take)[0]:
                    col[t] = inst[c]
            else:
                col[take] = inst[c]
            rows[c] = col
        return Z, w, DataFrame(rows)


class VectorSHAP(_KernelSHAPBase, HasInputCol):
    backgroundData = Param("A dataframe containing background data", None, complex=True)

    def _prepare(self, df):
        from ..core.linalg import as_matrix

        bg = self.getBackgroundData() if self.getBackgroundData() is not None else df
        return as_matrix(bg[self.getInputCol()])

    def _samples(self, df, i, bgm, rng):
        from ..core.linalg import as_matrix

        x = as_matrix(df[self.getInputCol()][i:i + 1])[0]
        m = len(x)
        Z, w = shap_coalitions(m, self._budget(m), rng, self.getInfWeight())
        samples = np.where(Z[:, None, :] > 0, x[None, None, :], bgm[None, :, :]).reshape(-1, m)
        rows = {c: np.repeat(df[c][i:i + 1], len(samples), axis=0) for c in df.columns if c != self.getInputCol()}
        rows[self.getInputCol()] = samples
        return Z, w, DataFrame(rows)


class ImageSHAP(_KernelSHAPBase, HasInputCol):
    cellSize = Param("Number that controls the size of the superpixels", 16.0, T.toFloat)
    modifier = Param("Controls the trade-off spatial and color distance", 130.0, T.toFloat)
    superpixelCol = Param("The column holding the superpixel decompositions", "superpixels", T.toString)

    def _samples(self, df, i, ctx, rng):
        from ..image.schema import make_image_row, to_array

        img = to_array(df[self.getInputCol()][i])
        labels = slic(img, self.getCellSize(), self.getModifier())
        m = int(labels.max()) + 1
        Z, w = shap_coalitions(m, self.getNumSamples() or (2 * m + 2048), rng, self.getInfWeight())
        imgs = [make_image_row(censor(img, labels, z)) for z in Z]
        rows = {c: np.repeat(df[c][i:i + 1], len(imgs), axis=0) for c in df.columns if c != self.getInputCol()}
        rows[self.getInputCol()] = _obj(imgs)
        return Z, w, DataFrame(rows)


class TextSHAP(_KernelSHAPBase, HasInputCol):
    tokensCol = Param("The column holding the tokens", "tokens", T.toString)

    def _samples(self, df, i, ctx, rng):
        text = df[self.getInputCol()][i]
        toks = text.split()
        m = len(toks)
        Z, w = shap_coalitions(m, self.getNumSamples() or (2 * m + 2048), rng, self.getInfWeight())
        texts = [" ".join(t for t, z in zip(toks, zz) if z > 0) for zz in Z]
        rows = {c: np.repeat(df[c][i:i + 1], len(texts), axis=0) for c in df.columns if c != self.getInputCol()}
        rows[self.getInputCol()] = _obj(texts)
        return Z, w, DataFrame(rows)

    def _transform(self, df):
        out = super()._transform(df)
        return out.withColumn(self.getTokensCol(), _obj([t.split() for t in df[self.getInputCol()].tolist()]))


# ---------------------------------------------------------------------- LIME
class _LIMEBase(LocalExplainer):
    regularization = Param("Regularization param for the lasso. Default value: 0.", 0.0, T.toFloat)
    kernelWidth = Param("Kernel width. Default value: sqrt (number of features) * 0.75", 0.75, T.toFloat)

    def _n(self) -> int:
        return self.getNumSamples() or 1000

    def _kernel(self, d: np.ndarray) -> np.ndarray:
        t = d / self.getKernelWidth()
        return np.sqrt(np.exp(-t * t))

    def _fit(self, X, y, w):
        r = lasso(X, y, w, self.getRegularization(), fit_intercept=True)
        return r.coefficients, r.rSquared


class TabularLIME(_LIMEBase, HasInputCols):
    backgroundData = Param("A dataframe containing background data", None, complex=True)
    categoricalFeatures = Param("Name of features that should be treated as categorical variables.", [],
                                T.toListString)

    def _prepare(self, df):
        bg = self.getBackgroundData() if self.getBackgroundData() is not None else df
        stats = {}
        for c in self.getInputCols():
            col = bg[c]
            if c in (self.getCategoricalFeatures() or []) or col.dtype.kind not in "biuf":
                vals = col.tolist()
                stats[c] = ("cat", vals)
            else:
                x = col.astype(np.float64)
                stats[c] = ("num", float(np.std(x)) or 1.0)
        return stats

    def _samples(self, df, i, stats, rng):
        cols = self.getInputCols()
        n = self._n()
        X = np.zeros((n, len(cols)))
        dist = np.zeros(n)
        rows = {c: np.repeat(df[c][i:i + 1], n, axis=0) for c in df.columns}
        for j, c in enumerate(cols):
            kind, s = stats[c]
            xi = df[c][i]
            if kind == "num":
                samp = float(xi) + rng.standard_normal(n) * s
                rows[c] = samp.astype(df[c].dtype) if df[c].dtype.kind == "f" else samp
                X[:, j] = samp
                dist += ((samp - float(xi)) / s) ** 2
            else:
                samp = [s[k] for k in rng.integers(0, len(s), size=n)]
                same = np.asarray([v == xi for v in samp], dtype=np.float64)
                rows[c] = _obj(samp) if df[c].dtype == object else np.asarray(samp)
                X[:, j] = same
                dist += 1.0 - same
        w = self._kernel(np.sqrt(dist / max(1, len(cols))))
        return X, w, DataFrame(rows)


class VectorLIME(_LIMEBase, HasInputCol):
    backgroundData = Param("A dataframe containing background data", None, complex=True)

    def _prepare(self, df):
        from ..core.linalg import as_matrix

        bg = self.getBackgroundData() if self.getBackgroundData() is not None else df
        sd = as_matrix(bg[self.getInputCol()]).std(0)
        return np.where(sd > 0, sd, 1.0)

    def _samples(self, df, i, sd, rng):
        from ..core.linalg import as_matrix

        x = as_matrix(df[self.getInputCol()][i:i + 1])[0]
        n = self._n()
        samples = x[None, :] + rng.standard_normal((n, len(x))) * sd[None, :]
        d = np.sqrt((((samples - x) / sd) ** 2).mean(1))
        rows = {c: np.repeat(df[c][i:i + 1], n, axis=0) for c in df.columns if c != self.getInputCol()}
        rows[self.getInputCol()] = samples
        return samples, self._kernel(d), DataFrame(rows)


class _OnOffLIME(_LIMEBase):
    samplingFraction = Param("The fraction of superpixels (for image) or tokens (for text) to keep on", 0.7,
                             T.toFloat)

    def _states(self, m: int, rng) -> Tuple[np.ndarray, np.ndarray]:
        n = self._n()
        Z = (rng.random((n, m)) < self.getSamplingFraction()).astype(np.float64)
        Z[0] = 1.0
        d = np.sqrt(1.0 - Z.mean(1)) if m else np.zeros(n)
        return Z, self._kernel(d)


class ImageLIME(_OnOffLIME, HasInputCol):
    cellSize = Param("Number that controls the size of the superpixels", 16.0, T.toFloat)
    modifier = Param("Controls the trade-off spatial and color distance", 130.0, T.toFloat)
    superpixelCol = Param("The column holding the superpixel decompositions", "superpixels", T.toString)

    def _samples(self, df, i, ctx, rng):
        from ..image.schema import make_image_row, to_array

        img = to_array(df[self.getInputCol()][i])
        labels = slic(img, self.getCellSize(), self.getModifier())
        Z, w = self._states(int(labels.max()) + 1, rng)
        imgs = [make_image_row(censor(img, labels, z)) for z in Z]
        rows = {c: np.repeat(df[c][i:i + 1], len(imgs), axis=0) for c in df.columns if c != self.getInputCol()}
        rows[self.getInputCol()] = _obj(imgs)
        return Z, w, DataFrame(rows)


class TextLIME(_OnOffLIME, HasInputCol):
    tokensCol = Param("The column holding the tokens", "tokens", T.toString)

    def _samples(self, df, i, ctx, rng):
        toks = df[self.getInputCol()][i].split()
        Z, w = self._states(len(toks), rng)
        texts = [" ".join(t for t, z in zip(toks, zz) if z > 0) for zz in Z]
        rows = {c: np.repeat(df[c][i:i + 1], len(texts), axis=0) for c in df.columns if c != self.getInputCol()}
        rows[self.getInputCol()] = _obj(texts)
        return Z, w, DataFrame(rows)

    def _transform(self, df):
        out = super()._transform(df)
        return out.withColumn(self.getTokensCol(), _obj([t.split() for t in df[self.getInputCol()].tolist()]))
