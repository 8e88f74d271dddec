"""Utility stages (reference: core/.../stages/{Cacher, ClassBalancer,
DropColumns, EnsembleByKey, Explode, Lambda, MultiColumnAdapter,
PartitionConsolidator, RenameColumn, Repartition, SelectColumns,
StratifiedRepartition, SummarizeData, TextPreprocessor, Timer, UDFTransformer,
UnicodeNormalize}.scala)."""
from __future__ import annotations

import time
import unicodedata
from typing import Any, Callable, Dict, List, Optional

import numpy as np

from ..core.contracts import HasInputCol, HasInputCols, HasLabelCol, HasOutputCol, HasOutputCols, HasSeed
from ..core.dataframe import DataFrame
from ..core.linalg import DenseVector, Vector
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Estimator, Model, PipelineModel, PipelineStage, Transformer


class Cacher(Transformer):
    disable = Param("Whether or disable caching (so that you can turn it off during evaluation)", False, T.toBoolean)

    def _transform(self, df):
        return df if self.getDisable() else df.cache()


class DropColumns(Transformer):
    cols = Param("Comma separated list of column names", [], T.toListString)

    def _transform(self, df):
        for c in self.getCols():
            if c not in df:
                raise ValueError(f"DataFrame does not contain specified column: {c}")
        return df.drop(*self.getCols())


class SelectColumns(Transformer):
    cols = Param("Comma separated list of selected column names", [], T.toListString)

    def _transform(self, df):
        for c in self.getCols():
            if c not in df:
                raise ValueError(f"DataFrame does not contain specified column: {c}")
        return df.select(*self.getCols())


class RenameColumn(Transformer, HasInputCol, HasOutputCol):
    def _transform(self, df):
        return df.withColumnRenamed(self.getInputCol(), self.getOutputCol())


class Repartition(Transformer):
    n = Param("Number of partitions", 1, T.toInt)
    disable = Param("Whether to disable repartitioning (so that one can turn it off for evaluation)", False,
                    T.toBoolean)

    def _transform(self, df):
        if self.getDisable():
            return df
        if self.getN() <= 0:
            raise ValueError("Number of partitions must be positive")
        return df.repartition(self.getN())


class PartitionConsolidator(Transformer):
    """Funnels all partitions of a worker into one (one per process here)."""

    def _transform(self, df):
        return df.coalesce(1)


class Explode(Transformer, HasInputCol, HasOutputCol):
    def _transform(self, df):
        col = df[self.getInputCol()]
        idx, vals = [], []
        for i, v in enumerate(col.tolist()):
            for x in (v if v is not None else []):
                idx.append(i)
                vals.append(x)
        out = df._take_rows(np.asarray(idx, dtype=np.int64))
        arr = np.empty(len(vals), dtype=object)
        for i, v in enumerate(vals):
            arr[i] = v
        if vals and all(isinstance(v, (int, float, bool, np.number)) for v in vals):
            arr = np.asarray(vals)
        return out.withColumn(self.getOutputCol(), arr)


class Lambda(Transformer):
    transformFunc = Param("holder for dataframe function", None, complex=True)
    transformSchemaFunc = Param("the output schema after the transformation", None, complex=True)

    def _transform(self, df):
        return self.getTransformFunc()(df)

    def transformSchema(self, schema):  # noqa: N802
        f = self.getTransformSchemaFunc()
        return f(schema) if f else schema


class UDFTransformer(Transformer, HasInputCol, HasInputCols, HasOutputCol):
    udf = Param("User Defined Python Function to be applied to the DF input col", None, complex=True)

    def setUDF(self, f):  # noqa: N802
        return self.set("udf", f)

    def getUDF(self):  # noqa: N802
        return self.getUdf()

    def _transform(self, df):
        f = self.getUdf()
        if self.getInputCols():
            cols = [df[c] for c in self.getInputCols()]
            vals = [f(*args) for args in zip(*[c.tolist() for c in cols])]
        else:
            col = df[self.getInputCol()]
            vals = [f(v) for v in (col.tolist() if col.ndim == 1 else [DenseVector(r) for r in col])]
        arr = np.empty(len(vals), dtype=object)
        for i, v in enumerate(vals):
            arr[i] = v
        if vals and all(isinstance(v, (int, float, bool, np.number)) for v in vals):
            arr = np.asarray(vals)
        return df.withColumn(self.getOutputCol(), arr)


class UnicodeNormalize(Transformer, HasInputCol, HasOutputCol):
    form = Param("Unicode normalization form: NFC, NFD, NFKC, NFKD", "NFKD", T.toString)
    lower = Param("Lowercase text", True, T.toBoolean)

    def _transform(self, df):
        form, lower = self.getForm(), self.getLower()
        out = np.empty(df.count(), dtype=object)
        for i, v in enumerate(df[self.getInputCol()].tolist()):
            if v is None:
                out[i] = None
                continue
            s = v.lower() if lower else v
            out[i] = unicodedata.normalize(form, s)
        return df.withColumn(self.getOutputCol(), out)


# ---------------------------------------------------------------------- ClassBalancer
class ClassBalancerModel(Model, HasInputCol, HasOutputCol):
    weights = Param("the dataframe of weights", None, complex=True)
    broadcastJoin = Param("whether to broadcast join", True, T.toBoolean)

    def _transform(self, df):
        w = self.getWeights()
        table = dict(zip(w[self.getInputCol()].tolist(), w[self.getOutputCol()].tolist()))
        return df.withColumn(self.getOutputCol(),
                             np.asarray([table.get(v, np.nan) for v in df[self.getInputCol()].tolist()], float))


class ClassBalancer(Estimator, HasInputCol, HasOutputCol):
    broadcastJoin = Param("Whether to broadcast the class to weight mapping to the worker", True, T.toBoolean)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(outputCol="weight")

    def _fit(self, df):
        counts = df.groupBy(self.getInputCol()).count()
        mx = float(np.max(counts["count"]))
        weights = counts.withColumn(self.getOutputCol(), mx / counts["count"].astype(float)).drop("count")
        m = ClassBalancerModel(inputCol=self.getInputCol(), outputCol=self.getOutputCol(),
                               broadcastJoin=self.getBroadcastJoin())
        return m.set("weights", weights)


# ---------------------------------------------------------------------- EnsembleByKey
class EnsembleByKey(Transformer):
    keys = Param("Keys to group by", [], T.toListString)
    cols = Param("Cols to ensemble", [], T.toListString)
    colNames = Param("Names of the result of each col", None, T.toListString)
    strategy = Param("How to ensemble the scores, ex: mean", "mean", T.toString)
    collapseGroup = Param("Whether to collapse all items in group to one entry", True, T.toBoolean)
    vectorDims = Param("the dimensions of any vector columns, used to avoid materialization", None, T.identity)

    def _transform(self, df):
        if self.getStrategy() != "mean":
            raise ValueError(f"unsupported strategy {self.getStrategy()}")
        keys = self.getKeys()
        names = self.getColNames() or [f"mean({c})" for c in self.getCols()]
        groups: Dict[tuple, List[int]] = {}
        for i, k in enumerate(zip(*[df[c].tolist() for c in keys])):
            groups.setdefault(k, []).append(i)
        agg: Dict[str, list] = {k: [] for k in keys}
        for n in names:
            agg[n] = []
        for key, idx in groups.items():
            for kn, kv in zip(keys, key):
                agg[kn].append(kv)
            for c, n in zip(self.getCols(), names):
                col = df[c]
                if col.ndim == 2:
                    agg[n].append(DenseVector(col[idx].mean(0)))
                elif col.dtype == object:
                    vecs = [v.toArray() if isinstance(v, Vector) else np.asarray(v, float) for v in col[idx]]
                    agg[n].append(DenseVector(np.mean(vecs, axis=0)))
                elif col.dtype.kind in "fiu":
                    agg[n].append(float(col[idx].astype(float).mean()))
                else:
                    raise ValueError(f"Cannot operate on type {col.dtype} with strategy mean")
        out = DataFrame(agg)
        if self.getCollapseGroup():
            return out
        rest = df.drop(*[c for c in names if c in df])
        return rest.join(out, keys)


# ---------------------------------------------------------------------- StratifiedRepartition
class StratifiedRepartition(Transformer, HasLabelCol, HasSeed):
    mode = Param("Specify equal to repartition with replacement across all labels, specify original to keep the "
                 "ratios in the original dataset, or specify mixed to use a heuristic", "mixed", T.toString)

    def _transform(self, df):
        labels = df[self.getLabelCol()].tolist()
        uniq = sorted(set(labels), key=lambda x: (str(type(x)), x))
        counts = {l: labels.count(l) for l in uniq}
        p = df.getNumPartitions()
        mode = self.getMode()
        if mode == "equal":
            mx = max(max(counts.values()), p)
            frac = {l: mx / c for l, c in counts.items()}
        elif mode == "mixed":
            mx = max(max(counts.values()), p)
            eq = {l: mx / c for l, c in counts.items()}
            norm = sum(eq.values()) / len(counts)
            frac = {l: f / norm for l, f in eq.items()}
        elif mode == "original":
            frac = {l: 1.0 for l in counts}
        else:
            raise ValueError(f"Unknown mode specified to StratifiedRepartition: {mode}")
        rng = np.random.default_rng(self.getSeed())
        rows = []
        for l in uniq:
            idx = [i for i, v in enumerate(labels) if v == l]
            f = frac[l]
            k = int(round(len(idx) * f)) if f != 1.0 else len(idx)
            take = rng.choice(idx, size=k, replace=f > 1.0) if f != 1.0 else np.asarray(idx)
            rows.append(np.asarray(take, dtype=np.int64))
        # round-robin the rows of every label over the partitions so each partition sees all labels
        assign: List[List[int]] = [[] for _ in range(p)]
        for arr in rows:
            for j, r in enumerate(arr):
                assign[j % p].append(int(r))
        order = np.concatenate([np.asarray(a, dtype=np.int64) for a in assign]) if rows else np.zeros(0, np.int64)
        out = df._take_rows(order)
        out._bounds = [0] + list(np.cumsum([len(a) for a in assign]))
        return out


# ---------------------------------------------------------------------- SummarizeData
class SummarizeData(Transformer):
    counts = Param("Compute count statistics", True, T.toBoolean)
    basic = Param("Compute basic statistics", True, T.toBoolean)
    sample = Param("Compute sample statistics", True, T.toBoolean)
    percentiles = Param("Compute percentiles", True, T.toBoolean)
    errorThreshold = Param("Threshold for quantiles - 0 is exact", 0.0, T.toFloat)

    def _transform(self, df):
        out: Dict[str, list] = {"Feature": []}
        fields = []
        if self.getCounts():
            fields += ["Count", "Unique_Value_Count", "Missing_Value_Count"]
        if self.getBasic():
            fields += ["Min", "1st_Quartile", "Median", "3rd_Quartile", "Max"]
        if self.getSample():
            fields += ["Sample_Variance", "Sample_Standard_Deviation", "Sample_Skewness", "Sample_Kurtosis"]
        if self.getPercentiles():
            fields += ["P0_5", "P1", "P5", "P95", "P99", "P99_5"]
        for f in fields:
            out[f] = []
        for name in df.columns:
            col = df[name]
            if col.ndim != 1:
                continue
            out["Feature"].append(name)
            numeric = col.dtype.kind in "biuf"
            x = col.astype(float) if numeric else None
            if self.getCounts():
                if numeric:
                    miss = np.isnan(x)
                    vals = x[~miss]
                    uniq = len(np.unique(vals))
                else:
                    miss = np.asarray([v is None or (isinstance(v, float) and np.isnan(v)) for v in col.tolist()])
                    uniq = len({repr(v) for v, m in zip(col.tolist(), miss) if not m})
                out["Count"].append(float(len(col) - miss.sum()))
                out["Unique_Value_Count"].append(float(uniq))
                out["Missing_Value_Count"].append(float(miss.sum()))
            v = x[~np.isnan(x)] if numeric else None
            if self.getBasic():
                qs = np.quantile(v, [0, 0.25, 0.5, 0.75, 1.0], method="inverted_cdf") if numeric and len(v) else \
                    [np.nan] * 5
                for f, q in zip(["Min", "1st_Quartile", "Median", "3rd_Quartile", "Max"], qs):
                    out[f].append(float(q))
            if self.getSample():
                if numeric and len(v) > 1:
                    var = float(np.var(v, ddof=1))
                    m = v.mean()
                    m2 = np.mean((v - m) ** 2)
                    skew = float(np.mean((v - m) ** 3) / m2 ** 1.5) if m2 > 0 else np.nan
                    kurt = float(np.mean((v - m) ** 4) / m2 ** 2 - 3) if m2 > 0 else np.nan
                    stats = [var, float(np.sqrt(var)), skew, kurt]
                else:
                    stats = [np.nan] * 4
                for f, s in zip(["Sample_Variance", "Sample_Standard_Deviation", "Sample_Skewness",
                                 "Sample_Kurtosis"], stats):
                    out[f].append(s)
            if self.getPercentiles():
                qs = np.quantile(v, [0.005, 0.01, 0.05, 0.95, 0.99, 0.995], method="inverted_cdf") \
                    if numeric and len(v) else [np.nan] * 6
                for f, q in zip(["P0_5", "P1", "P5", "P95", "P99", "P99_5"], qs):
                    out[f].append(float(q))
        return DataFrame(out)


# ---------------------------------------------------------------------- TextPreprocessor
class Trie:
    """Longest-match replacement trie with the reference's scanning rules
    (TextPreprocessor.scala:15-83): after a replacement the rest of the
    current word is skipped; a key ending exactly at the end of the text is
    not matched (the reference checks a node's value only while input
    remains)."""

    def __init__(self, norm: Callable[[str], str] = lambda c: c):
        self.children: Dict[str, "Trie"] = {}
        self.value = ""
        self.norm = norm

    def put(self, key: str, value: str) -> "Trie":
        node = self
        for ch in key:
            ch = self.norm(ch)
            node = node.children.setdefault(ch, Trie(self.norm))
        node.value = value
        return self

    def putAll(self, m: Dict[str, str]) -> "Trie":  # noqa: N802
        for k, v in m.items():
            self.put(k, v)
        return self

    def get(self, ch: str) -> Optional["Trie"]:
        return self.children.get(self.norm(ch))

    def mapText(self, text: str) -> str:  # noqa: N802
        out: List[str] = []
        n = len(text)
        pos = 0

        def is_alpha(c):
            return c.isalnum() or c == "_"

        while pos < n:
            # scan(chars = text[pos:])
            rest = pos + 1
            matched = text[pos]
            has_match = False
            cpos = pos + 1
            trie = self.get(text[pos])
            while True:
                if trie is None or cpos >= n:
                    out.append(matched)
                    pos = rest
                    if has_match:
                        while pos < n and is_alpha(text[pos]):
                            pos += 1
                    break
                if not trie.value:
                    has_match = False
                    trie = trie.get(text[cpos])
                    cpos += 1
                else:
                    rest = cpos
                    matched = trie.value
                    has_match = True
                    trie = trie.get(text[cpos])
                    cpos += 1
        return "".join(out)


class TextPreprocessor(Transformer, HasInputCol, HasOutputCol):
    map = Param("Map of substring match to replacement", {}, T.identity)
    normFunc = Param("Name of normalization function to apply", "identity", T.toString)

    _NORMS = {"identity": lambda c: c, "lowerCase": str.lower, "upperCase": str.upper}

    def _transform(self, df):
        if self.getNormFunc() not in self._NORMS:
            raise ValueError(f"invalid normFunc {self.getNormFunc()}")
        trie = Trie(self._NORMS[self.getNormFunc()]).putAll(self.getMap() or {})
        out = np.empty(df.count(), dtype=object)
        for i, v in enumerate(df[self.getInputCol()].tolist()):
            out[i] = None if v is None else trie.mapText(v)
        return df.withColumn(self.getOutputCol(), out)


# ---------------------------------------------------------------------- Timer
class TimerModel(Model):
    transformer = Param("inner model to time", None, complex=True)
    logToScala = Param("Whether to output the time to the console", True, T.toBoolean)
    disableMaterialization = Param("Whether to disable timing (so that one can turn it off for evaluation)", True,
                                   T.toBoolean)

    def _transform(self, df):
        t0 = time.perf_counter_ns()
        out = self.getTransformer().transform(df)
        dt = time.perf_counter_ns() - t0
        msg = _fmt_time(dt, True, None if self.getDisableMaterialization() else out.count(), self.getTransformer())
        self.last_message = msg
        if self.getLogToScala():
            print(msg)
        return out


class Timer(Estimator):
    stage = Param("The stage to time", None, complex=True)
    logToScala = Param("Whether to output the time to the console", True, T.toBoolean)
    disableMaterialization = Param("Whether to disable timing (so that one can turn it off for evaluation)", True,
                                   T.toBoolean)

    def _fit(self, df):
        st = self.getStage()
        t0 = time.perf_counter_ns()
        if isinstance(st, Estimator):
            inner = st.fit(df)
        else:
            inner = st
        dt = time.perf_counter_ns() - t0
        msg = _fmt_time(dt, False, None if self.getDisableMaterialization() else df.count(), st)
        self.last_message = msg
        if self.getLogToScala() and isinstance(st, Estimator):
            print(msg)
        return TimerModel(logToScala=self.getLogToScala(),
                          disableMaterialization=self.getDisableMaterialization()).set("transformer", inner)


def _fmt_time(ns: int, is_transform: bool, count: Optional[int], stage) -> str:
    verb = "transform" if is_transform else "fit"
    amount = f"{count} rows" if count is not None else ""
    return f"{type(stage).__name__} took {ns / 1e9:.3f}s to {verb} {amount}".strip()


# ---------------------------------------------------------------------- MultiColumnAdapter
class MultiColumnAdapter(Estimator, HasInputCols, HasOutputCols):
    baseStage = Param("base pipeline stage to apply to every column", None, complex=True)

    def _fit(self, df):
        ins, outs = self.getInputCols(), self.getOutputCols()
        if len(ins) != len(outs):
            raise ValueError("inputCols and outputCols must have the same length")
        for i in ins:
            if i not in df:
                raise ValueError(f"DataFrame does not contain specified column: {i}")
        for o in outs:
            if o in df:
                raise ValueError(f"DataFrame already contains column: {o}")
        stages = []
        for i, o in zip(ins, outs):
            s = self.getBaseStage().copy()
            if s.hasParam("inputCol"):
                s.set("inputCol", i)
                s.set("outputCol", o)
            else:
                s.set("inputCols", [i])
                s.set("outputCols", [o])
            stages.append(s.fit(df) if isinstance(s, Estimator) else s)
        return PipelineModel(stages)
