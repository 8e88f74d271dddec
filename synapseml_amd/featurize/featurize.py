"""Featurization stages (reference: core/.../featurize/{ValueIndexer,
IndexToValue, CleanMissingData, DataConversion, CountSelector,
Featurize}.scala and featurize/text/{TextFeaturizer, MultiNGram,
PageSplitter}.scala)."""
from __future__ import annotations

import datetime as _dt
import re
from typing import Any, Dict, List, Optional

import numpy as np

from ..core.contracts import HasInputCol, HasInputCols, HasOutputCol, HasOutputCols
from ..core.dataframe import DataFrame
from ..core.linalg import DenseVector, SparseVector, Vector
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Estimator, Model, Pipeline, PipelineModel, Transformer
from .ml import (IDF, HashingTF, NGram, OneHotEncoder, RegexTokenizer, StopWordsRemover, VectorAssembler, _obj)

NUM_FEATURES_DEFAULT = 262144


def _is_missing(v) -> bool:
    return v is None or (isinstance(v, float) and np.isnan(v))


def _sort_key(v):
    if isinstance(v, (bool, np.bool_)):
        return (0, int(v))
    if isinstance(v, (int, float, np.number)):
        return (1, float(v))
    return (2, str(v))


def categorical_metadata(levels: List[Any], has_null: bool, name: str, dtype: str) -> dict:
    return {"ml_attr": {"type": "nominal", "vals": [str(l) for l in levels], "name": name},
            "mml_categorical": {"levels": list(levels), "hasNullLevel": has_null, "dataType": dtype}}


# ---------------------------------------------------------------------- ValueIndexer
class ValueIndexerModel(Model, HasInputCol, HasOutputCol):
    levels = Param("Levels in categorical array", [], T.identity)
    dataType = Param("The datatype of the levels", "string", T.toString)

    def _transform(self, df):
        levels = list(self.getLevels())
        non_null = [l for l in levels if not _is_missing(l)]
        has_null = len(non_null) != len(levels)
        table = {l: i for i, l in enumerate(non_null)}
        unknown = len(non_null) if not has_null else len(non_null) + 1
        idx = []
        for v in df[self.getInputCol()].tolist():
            if _is_missing(v):
                idx.append(len(non_null))
            else:
                idx.append(table.get(v, unknown))
        md = categorical_metadata(non_null, has_null, self.getOutputCol(), self.getDataType())
        return df.withColumn(self.getOutputCol(), np.asarray(idx, dtype=np.int64), metadata=md)


class ValueIndexer(Estimator, HasInputCol, HasOutputCol):
    def _fit(self, df):
        col = df[self.getInputCol()]
        vals = col.tolist()
        distinct = []
        seen = set()
        has_null = False
        for v in vals:
            if _is_missing(v):
                has_null = True
                continue
            if v not in seen:
                seen.add(v)
                distinct.append(v)
        if col.dtype.kind == "f":
            dtype = "double"
        elif col.dtype.kind in "iu":
            dtype = "long"
        elif col.dtype.kind == "b":
            dtype = "boolean"
        else:
            dtype = "string"
            if any(not isinstance(v, str) for v in distinct):
                if all(isinstance(v, (bool, np.bool_)) for v in distinct):
                    dtype = "boolean"
                elif all(isinstance(v, (int, np.integer)) for v in distinct):
                    dtype = "long"
                elif all(isinstance(v, (int, float, np.number)) for v in distinct):
                    dtype = "double"
                else:
                    raise TypeError(f"Unsupported Categorical type for column: {self.getInputCol()}")
        levels = sorted(distinct, key=_sort_key)
        if has_null:
            levels = [None] + levels
        return ValueIndexerModel(inputCol=self.getInputCol(), outputCol=self.getOutputCol(), levels=levels,
                                 dataType=dtype)


class IndexToValue(Transformer, HasInputCol, HasOutputCol):
    def _transform(self, df):
        md = df.metadata(self.getInputCol()).get("mml_categorical")
        if md is None:
            raise ValueError(f"column {self.getInputCol()} is not Categorical")
        levels = [l for l in md["levels"] if not _is_missing(l)]
        out = []
        for i in df[self.getInputCol()].tolist():
            i = int(i)
            if i == len(levels) and md.get("hasNullLevel"):
                out.append(None)
            elif 0 <= i < len(levels):
                out.append(levels[i])
            else:
                raise IndexError(f"Invalid metadata: Index greater than number of levels in metadata, index: {i}, "
                                 f"levels: {len(levels)}")
        arr = _obj(out)
        if out and all(isinstance(v, (int, float, np.number)) and not isinstance(v, bool) for v in out):
            arr = np.asarray(out)
        return df.withColumn(self.getOutputCol(), arr)


# ---------------------------------------------------------------------- CleanMissingData
class CleanMissingDataModel(Model, HasInputCols, HasOutputCols):
    colsToFill = Param("The columns to fill with", [], T.toListString)
    fillValues = Param("what to replace in the columns", [], T.identity)

    def _transform(self, df):
        out = df
        for c, o, v in zip(self.getInputCols(), self.getOutputCols(), self.getFillValues()):
            col = df[c]
            if col.dtype.kind in "f":
                out = out.withColumn(o, np.where(np.isnan(col), float(v), col))
            elif col.dtype.kind in "iub":
                out = out.withColumn(o, col.copy())
            else:
                vals = [(type_cast(v, col) if _is_missing(x) else x) for x in col.tolist()]
                out = out.withColumn(o, _obj(vals) if col.dtype == object else np.asarray(vals))
        return out


def type_cast(v, col):
    if isinstance(v, str):
        sample = next((x for x in col.tolist() if not _is_missing(x)), None)
        if isinstance(sample, bool):
            return v.lower() == "true"
        if isinstance(sample, (int, np.integer)):
            return int(v)
        if isinstance(sample, float):
            return float(v)
    return v


class CleanMissingData(Estimator, HasInputCols, HasOutputCols):
    cleaningMode = Param("Cleaning mode", "Mean", T.toString)
    customValue = Param("Custom value for replacement", None, T.toString)

    def _fit(self, df):
        mode = self.getCleaningMode()
        vals = []
        for c in self.getInputCols():
            col = df[c]
            if mode in ("Mean", "Median"):
                if col.dtype.kind not in "iuf":
                    raise TypeError("Only numeric types supported for numeric imputation")
                x = col.astype(float)
                x = x[~np.isnan(x)]
                vals.append(float(np.mean(x)) if mode == "Mean" else float(np.quantile(x, 0.5, method="inverted_cdf")))
            elif mode == "Custom":
                v = self.getCustomValue()
                vals.append(float(v) if col.dtype.kind in "f" else v)
            else:
                raise ValueError(f"unknown cleaning mode {mode}")
        return CleanMissingDataModel(inputCols=self.getInputCols(), outputCols=self.getOutputCols(),
                                     colsToFill=self.getInputCols(), fillValues=vals)


# ---------------------------------------------------------------------- DataConversion
class DataConversion(Transformer):
    cols = Param("Comma separated list of columns whose type will be converted", [], T.toListString)
    convertTo = Param("The result type", "", T.toString)
    dateTimeFormat = Param("Format for DateTime when making DateTime:String conversions", "yyyy-MM-dd HH:mm:ss",
                           T.toString)

    _NP = {"boolean": np.bool_, "byte": np.int8, "short": np.int16, "integer": np.int32, "long": np.int64,
           "float": np.float32, "double": np.float64}

    def _py_fmt(self) -> str:
        f = self.getDateTimeFormat()
        for a, b in (("yyyy", "%Y"), ("MM", "%m"), ("dd", "%d"), ("HH", "%H"), ("mm", "%M"), ("ss", "%S"),
                     ("SSS", "%f")):
            f = f.replace(a, b)
        return f

    def _transform(self, df):
        for c in self.getCols():
            if c not in df:
                raise KeyError(f"DataFrame does not contain specified column: {c}")
        out = df
        to = self.getConvertTo()
        for c in [c.strip() for c in self.getCols()]:
            col = out[c]
            if to in self._NP:
                if col.dtype == object and col.size and isinstance(col[0], _dt.datetime):
                    if to != "long":
                        raise ValueError("Date only converts to string or long")
                    out = out.withColumn(c, np.asarray([int(v.timestamp() * 1000) for v in col], np.int64))
                elif col.dtype == object:
                    conv = [self._NP[to](float(v) if to not in ("boolean",) else (str(v).lower() == "true"))
                            for v in col.tolist()]
                    out = out.withColumn(c, np.asarray(conv, dtype=self._NP[to]))
                else:
                    out = out.withColumn(c, col.astype(self._NP[to]))
            elif to == "string":
                if col.dtype == object and col.size and isinstance(col[0], _dt.datetime):
                    out = out.withColumn(c, _obj([v.strftime(self._py_fmt()) for v in col]))
                elif col.dtype.kind == "b":
                    out = out.withColumn(c, _obj(["true" if v else "false" for v in col.tolist()]))
                else:
                    out = out.withColumn(c, _obj([None if v is None else str(v) for v in col.tolist()]))
            elif to == "toCategorical":
                out = ValueIndexer(inputCol=c, outputCol=c).fit(out).transform(out)
            elif to == "clearCategorical":
                out = IndexToValue(inputCol=c, outputCol=c).transform(out)
            elif to == "date":
                if col.dtype.kind in "iu":
                    out = out.withColumn(c, _obj([_dt.datetime.fromtimestamp(v / 1000.0) for v in col.tolist()]))
                else:
                    out = out.withColumn(c, _obj([_dt.datetime.strptime(v, self._py_fmt()) for v in col.tolist()]))
            else:
                raise ValueError(f"unsupported conversion {to}")
        return out


# ---------------------------------------------------------------------- CountSelector
class CountSelectorModel(Model, HasInputCol, HasOutputCol):
    indices = Param("An array of indices to select features from a vector column.", [], T.toListInt)

    def _transform(self, df):
        keep = np.asarray(self.getIndices(), dtype=np.int64)
        pos = {int(i): j for j, i in enumerate(keep.tolist())}
        out = []
        for v in df[self.getInputCol()].tolist():
            if isinstance(v, SparseVector):
                sel = [(pos[int(i)], x) for i, x in zip(v.indices, v.values) if int(i) in pos]
                out.append(SparseVector(len(keep), [s[0] for s in sel], [s[1] for s in sel]))
            else:
                a = v.toArray() if isinstance(v, Vector) else np.asarray(v, float)
                out.append(DenseVector(a[keep]))
        return df.withColumn(self.getOutputCol(), _obj(out))


class CountSelector(Estimator, HasInputCol, HasOutputCol):
    def _fit(self, df):
        used = set()
        col = df[self.getInputCol()]
        rows = col.tolist() if col.ndim == 1 else [DenseVector(r) for r in col]
        for v in rows:
            if isinstance(v, SparseVector):
                used.update(int(i) for i, x in zip(v.indices, v.values))
            else:
                a = v.toArray() if isinstance(v, Vector) else np.asarray(v, float)
                used.update(np.nonzero(a)[0].tolist())
        return CountSelectorModel(inputCol=self.getInputCol(), outputCol=self.getOutputCol(), indices=sorted(used))


# ---------------------------------------------------------------------- text
class TextFeaturizerModel(Model, HasInputCol, HasOutputCol):
    stages_ = Param("fitted inner pipeline", None, complex=True)

    def _transform(self, df):
        return self.getStages_().transform(df)


class TextFeaturizer(Estimator, HasInputCol, HasOutputCol):
    useTokenizer = Param("Whether to tokenize the input", True, T.toBoolean)
    tokenizerGaps = Param("Indicates whether regex splits on gaps (true) or matches tokens (false)", True,
                          T.toBoolean)
    minTokenLength = Param("Minimum token length, >= 0.", 0, T.toInt)
    tokenizerPattern = Param("Regex pattern used to match delimiters if gaps is true or tokens if gaps is false",
                             r"\s+", T.toString)
    toLowercase = Param("Indicates whether to convert all characters to lowercase before tokenizing.", True,
                        T.toBoolean)
    useStopWordsRemover = Param("Whether to remove stop words from tokenized data", False, T.toBoolean)
    caseSensitiveStopWords = Param("Whether to do a case sensitive comparison over the stop words", False,
                                   T.toBoolean)
    defaultStopWordLanguage = Param("Which language to use for the stop word remover", "english", T.toString)
    stopWords = Param("The words to be filtered out.", None, T.toString)
    useNGram = Param("Whether to enumerate N grams", False, T.toBoolean)
    nGramLength = Param("The size of the Ngrams", 2, T.toInt)
    useHashingTF = Param("Whether to use a hashing TF", True, T.toBoolean)
    binary = Param("If true, all nonegative word counts are set to 1", False, T.toBoolean)
    numFeatures = Param("Set the number of features to hash each document to", NUM_FEATURES_DEFAULT, T.toInt)
    useIDF = Param("Whether to scale the Term Frequencies by IDF", True, T.toBoolean)
    minDocFreq = Param("The minimum number of documents in which a term should appear.", 1, T.toInt)

    def _fit(self, df):
        stages = []
        cur = self.getInputCol()
        k = 0

        def nxt():
            nonlocal k
            k += 1
            return f"{self.uid}__{k}"

        if self.getUseTokenizer():
            o = nxt()
            stages.append(RegexTokenizer(inputCol=cur, outputCol=o, gaps=self.getTokenizerGaps(),
                                         pattern=self.getTokenizerPattern(), minTokenLength=self.getMinTokenLength(),
                                         toLowercase=self.getToLowercase()))
            cur = o
        if self.getUseStopWordsRemover():
            o = nxt()
            sw = self.getStopWords()
            stages.append(StopWordsRemover(inputCol=cur, outputCol=o, caseSensitive=self.getCaseSensitiveStopWords(),
                                           stopWords=sw.split(",") if sw else None))
            cur = o
        if self.getUseNGram():
            o = nxt()
            stages.append(NGram(inputCol=cur, outputCol=o, n=self.getNGramLength()))
            cur = o
        if self.getUseHashingTF():
            o = nxt() if self.getUseIDF() else self.getOutputCol()
            stages.append(HashingTF(inputCol=cur, outputCol=o, numFeatures=self.getNumFeatures(),
                                    binary=self.getBinary()))
            cur = o
        if self.getUseIDF():
            stages.append(IDF(inputCol=cur, outputCol=self.getOutputCol(), minDocFreq=self.getMinDocFreq()))
        pm = Pipeline(stages).fit(df)
        tmp = [s.getOutputCol() for s in pm.getStages() if s.getOutputCol() != self.getOutputCol()]
        dropper = _Drop(tmp)
        full = PipelineModel(pm.getStages() + [dropper])
        return TextFeaturizerModel(inputCol=self.getInputCol(), outputCol=self.getOutputCol()).set("stages_", full)


class _Drop(Transformer):
    def __init__(self, cols=None, **kw):
        super().__init__(**kw)
        self._cols = list(cols or [])

    def _transform(self, df):
        return df.drop(*[c for c in self._cols if c in df])


class MultiNGram(Transformer, HasInputCol, HasOutputCol):
    lengths = Param("the collection of lengths to use for ngram extraction", [1, 2, 3], T.toListInt)

    def _transform(self, df):
        out = []
        for toks in df[self.getInputCol()].tolist():
            if toks is None:
                out.append(None)
                continue
            grams = []
            for n in self.getLengths():
                grams.extend(" ".join(toks[i:i + n]) for i in range(len(toks) - n + 1))
            out.append(grams)
        return df.withColumn(self.getOutputCol(), _obj(out))


class PageSplitter(Transformer, HasInputCol, HasOutputCol):
    maximumPageLength = Param("the maximum number of characters to be in a page", 5000, T.toInt)
    minimumPageLength = Param("the the minimum number of characters to have on a page in order to preserve work "
                              "boundaries", 4500, T.toInt)
    boundaryRegex = Param("how to split into words", r"\s", T.toString)

    def split(self, text: str) -> List[str]:
        mx, mn = self.getMaximumPageLength(), self.getMinimumPageLength()
        pat = re.compile(self.getBoundaryRegex())
        pages = []
        while text:
            if len(text) <= mx:
                pages.append(text)
                break
            cut = None
            for m in pat.finditer(text, mn, mx + 1):
                cut = m.start()
            if cut is None or cut < mn:
                cut = mx
            pages.append(text[:cut])
            text = text[cut:]
        return pages

    def _transform(self, df):
        return df.withColumn(self.getOutputCol(), _obj([None if t is None else self.split(t)
                                                        for t in df[self.getInputCol()].tolist()]))


# ---------------------------------------------------------------------- Featurize
class Featurize(Estimator, HasInputCols, HasOutputCol):
    oneHotEncodeCategoricals = Param("One-hot encode categorical columns", True, T.toBoolean)
    numFeatures = Param("Number of features to hash string columns to", NUM_FEATURES_DEFAULT, T.toInt)
    imputeMissing = Param("Whether to impute missing values", True, T.toBoolean)

    def _fit(self, df):
        stages: List = []
        final_cols = []
        cur = df
        for c in self.getInputCols():
            col = cur[c]
            md = cur.metadata(c).get("ml_attr", {})
            is_cat = self.getOneHotEncodeCategoricals() and md.get("type") == "nominal"
            name = c
            if is_cat:
                o = f"{c}_{self.uid}_ohe"
                enc = OneHotEncoder(inputCols=[name], outputCols=[o]).fit(cur)
                stages.append(enc)
                cur = enc.transform(cur)
                final_cols.append(o)
                continue
            if col.ndim == 2 or (col.dtype == object and col.size and isinstance(col[0], Vector)):
                final_cols.append(name)
                continue
            if col.dtype.kind in "biuf":
                o = f"{c}_{self.uid}_dbl"
                caster = _Cast(name, o)
                stages.append(caster)
                cur = caster.transform(cur)
                name = o
                if self.getImputeMissing():
                    o2 = f"{c}_{self.uid}_imp"
                    cm = CleanMissingData(inputCols=[name], outputCols=[o2]).fit(cur)
                    stages.append(cm)
                    cur = cm.transform(cur)
                    name = o2
                final_cols.append(name)
                continue
            sample = next((v for v in col.tolist() if v is not None), None)
            if isinstance(sample, (_dt.datetime, _dt.date)):
                o = f"{c}_{self.uid}_ts"
                st = _TimestampFeatures(name, o)
                stages.append(st)
                cur = st.transform(cur)
                final_cols.append(o)
                continue
            # strings: fill nulls, hash-TF/IDF, drop unused slots
            o1, o2 = f"{c}_{self.uid}_tf", f"{c}_{self.uid}_cs"
            fill = _FillEmpty(name)
            stages.append(fill)
            cur = fill.transform(cur)
            tf = TextFeaturizer(inputCol=name, outputCol=o1, numFeatures=self.getNumFeatures()).fit(cur)
            stages.append(tf)
            cur = tf.transform(cur)
            cs = CountSelector(inputCol=o1, outputCol=o2).fit(cur)
            stages.append(cs)
            cur = cs.transform(cur)
            final_cols.append(o2)
        asm = VectorAssembler(inputCols=final_cols, outputCol=self.getOutputCol(), handleInvalid="keep")
        stages.append(asm)
        temp = [c for c in cur.columns if c not in df.columns and c != self.getOutputCol()]
        stages.append(_Drop(temp))
        return PipelineModel(stages)


class _Cast(Transformer):
    def __init__(self, src=None, dst=None, **kw):
        super().__init__(**kw)
        self._src, self._dst = src, dst

    def _transform(self, df):
        return df.withColumn(self._dst, df[self._src].astype(np.float64))


class _FillEmpty(Transformer):
    def __init__(self, col=None, **kw):
        super().__init__(**kw)
        self._col = col

    def _transform(self, df):
        return df.withColumn(self._col, _obj(["" if v is None else str(v) for v in df[self._col].tolist()]))


class _TimestampFeatures(Transformer):
    def __init__(self, src=None, dst=None, **kw):
        super().__init__(**kw)
        self._src, self._dst = src, dst

    def _transform(self, df):
        out = []
        for ts in df[self._src].tolist():
            if not isinstance(ts, _dt.datetime):
                ts = _dt.datetime(ts.year, ts.month, ts.day)
            out.append([ts.timestamp() * 1000.0, ts.year, ts.isoweekday(), ts.month, ts.day, ts.hour, ts.minute,
                        ts.second])
        return df.withColumn(self._dst, np.asarray(out, dtype=np.float64).reshape(-1, 8))
