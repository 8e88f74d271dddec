"""Feature primitives the reference takes from SparkML (Tokenizer,
RegexTokenizer, StopWordsRemover, NGram, HashingTF, IDF, OneHotEncoder,
StringIndexer, VectorAssembler, SQL casts). There is no SparkML here, so the
framework carries its own with Spark's semantics: HashingTF index =
nonNegativeMod(murmur3_x86_32(utf8(term), seed 42), numFeatures); IDF =
log((m + 1) / (df + 1)) with terms below minDocFreq zeroed; OneHotEncoder
drops the last category by default."""
from __future__ import annotations

import re
from typing import Dict, List, Optional

import numpy as np

from ..core.contracts import HasInputCol, HasInputCols, HasOutputCol, HasOutputCols
from ..core.dataframe import DataFrame
from ..core.linalg import DenseVector, SparseVector, Vector
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Estimator, Model, Transformer
from ..ops import native

ENGLISH_STOP_WORDS = (
    "i me my myself we our ours ourselves you your yours yourself yourselves he him his himself she her hers herself "
    "it its itself they them their theirs themselves what which who whom this that these those am is are was were be "
    "been being have has had having do does did doing a an the and but if or because as until while of at by for "
    "with about against between into through during before after above below to from up down in out on off over "
    "under again further then once here there when where why how all any both each few more most other some such no "
    "nor not only own same so than too very s t can will just don should now i'll you'll he'll she'll we'll they'll "
    "i'd you'd he'd she'd we'd they'd i'm you're he's she's it's we're they're i've we've you've they've isn't "
    "aren't wasn't weren't haven't hasn't hadn't don't doesn't didn't won't wouldn't shan't shouldn't mustn't can't "
    "couldn't cannot could here's how's let's ought that's there's what's when's where's who's why's would").split()


def _obj(values) -> np.ndarray:
    arr = np.empty(len(values), dtype=object)
    for i, v in enumerate(values):
        arr[i] = v
    return arr


def murmur3_spark(term: str, seed: int = 42) -> int:
    h = int(native.load("_vw").murmur3(term.encode("utf-8"), seed & 0xFFFFFFFF))
    return h - (1 << 32) if h >= (1 << 31) else h


class Tokenizer(Transformer, HasInputCol, HasOutputCol):
    def _transform(self, df):
        return df.withColumn(self.getOutputCol(), _obj([None if v is None else v.lower().split(" ")
                                                        for v in df[self.getInputCol()].tolist()]))


class RegexTokenizer(Transformer, HasInputCol, HasOutputCol):
    gaps = Param("Set regex to match gaps or tokens", True, T.toBoolean)
    pattern = Param("regex pattern used for tokenizing", r"\s+", T.toString)
    minTokenLength = Param("minimum token length (>= 0)", 1, T.toInt)
    toLowercase = Param("whether to convert all characters to lowercase before tokenizing", True, T.toBoolean)

    def tokenize(self, s: str) -> List[str]:
        if self.getToLowercase():
            s = s.lower()
        pat = re.compile(self.getPattern())
        toks = pat.split(s) if self.getGaps() else pat.findall(s)
        return [t for t in toks if len(t) >= self.getMinTokenLength()]

    def _transform(self, df):
        return df.withColumn(self.getOutputCol(), _obj([None if v is None else self.tokenize(v)
                                                        for v in df[self.getInputCol()].tolist()]))


class StopWordsRemover(Transformer, HasInputCol, HasOutputCol):
    stopWords = Param("The words to be filtered out", None, T.toListString)
    caseSensitive = Param("whether to do a case-sensitive comparison over the stop words", False, T.toBoolean)

    def _transform(self, df):
        sw = self.getStopWords() or ENGLISH_STOP_WORDS
        cs = self.getCaseSensitive()
        swset = set(sw) if cs else {w.lower() for w in sw}
        out = []
        for toks in df[self.getInputCol()].tolist():
            out.append(None if toks is None else [t for t in toks if (t if cs else t.lower()) not in swset])
        return df.withColumn(self.getOutputCol(), _obj(out))


class NGram(Transformer, HasInputCol, HasOutputCol):
    n = Param("number elements per n-gram (>=1)", 2, T.toInt)

    def _transform(self, df):
        n = self.getN()
        out = [None if t is None else [" ".join(t[i:i + n]) for i in range(len(t) - n + 1)]
               for t in df[self.getInputCol()].tolist()]
        return df.withColumn(self.getOutputCol(), _obj(out))


class HashingTF(Transformer, HasInputCol, HasOutputCol):
    numFeatures = Param("Number of features. Should be greater than 0", 1 << 18, T.toInt)
    binary = Param("If true, all non zero counts are set to 1", False, T.toBoolean)

    def vectorize(self, terms) -> SparseVector:
        nf = self.getNumFeatures()
        counts: Dict[int, float] = {}
        for t in terms:
            i = murmur3_spark(str(t)) % nf
            counts[i] = 1.0 if self.getBinary() else counts.get(i, 0.0) + 1.0
        idx = np.asarray(sorted(counts), dtype=np.int32)
        return SparseVector(nf, idx, np.asarray([counts[i] for i in idx.tolist()], dtype=np.float64))

    def _transform(self, df):
        return df.withColumn(self.getOutputCol(), _obj([None if t is None else self.vectorize(t)
                                                        for t in df[self.getInputCol()].tolist()]))


class IDFModel(Model, HasInputCol, HasOutputCol):
    idf = Param("inverse document frequency per feature", None, complex=True)

    def _transform(self, df):
        w = np.asarray(self.getIdf())
        out = []
        for v in df[self.getInputCol()].tolist():
            if isinstance(v, SparseVector):
                out.append(SparseVector(v.size, v.indices, v.values * w[v.indices]))
            else:
                a = v.toArray() if isinstance(v, Vector) else np.asarray(v, float)
                out.append(DenseVector(a * w))
        return df.withColumn(self.getOutputCol(), _obj(out))


class IDF(Estimator, HasInputCol, HasOutputCol):
    minDocFreq = Param("minimum number of documents in which a term should appear for filtering", 0, T.toInt)

    def _fit(self, df):
        col = df[self.getInputCol()].tolist()
        size = col[0].size if col else 0
        dfreq = np.zeros(size)
        for v in col:
            if isinstance(v, SparseVector):
                dfreq[v.indices[v.values != 0]] += 1
            else:
                dfreq += np.asarray(v.toArray() if isinstance(v, Vector) else v) != 0
        m = len(col)
        idf = np.log((m + 1.0) / (dfreq + 1.0))
        idf[dfreq < self.getMinDocFreq()] = 0.0
        return IDFModel(inputCol=self.getInputCol(), outputCol=self.getOutputCol()).set("idf", idf)


class StringIndexerModel(Model, HasInputCol, HasOutputCol):
    labels = Param("Ordered list of labels", [], T.identity)
    handleInvalid = Param("error | skip | keep", "error", T.toString)

    def _transform(self, df):
        table = {l: i for i, l in enumerate(self.getLabels())}
        vals, keep = [], []
        for v in df[self.getInputCol()].tolist():
            if v in table:
                vals.append(float(table[v]))
                keep.append(True)
            elif self.getHandleInvalid() == "keep":
                vals.append(float(len(table)))
                keep.append(True)
            elif self.getHandleInvalid() == "skip":
                vals.append(np.nan)
                keep.append(False)
            else:
                raise ValueError(f"Unseen label: {v}")
        out = df.withColumn(self.getOutputCol(), np.asarray(vals),
                            metadata={"ml_attr": {"type": "nominal", "vals": [str(l) for l in self.getLabels()],
                                                  "name": self.getOutputCol()}})
        return out.filter(np.asarray(keep)) if not all(keep) else out


class StringIndexer(Estimator, HasInputCol, HasOutputCol):
    stringOrderType = Param("frequencyDesc | frequencyAsc | alphabetDesc | alphabetAsc", "frequencyDesc", T.toString)
    handleInvalid = Param("error | skip | keep", "error", T.toString)

    def _fit(self, df):
        vals = [v for v in df[self.getInputCol()].tolist() if v is not None]
        counts: Dict = {}
        for v in vals:
            counts[v] = counts.get(v, 0) + 1
        order = self.getStringOrderType()
        if order == "frequencyDesc":
            labels = sorted(counts, key=lambda k: (-counts[k], str(k)))
        elif order == "frequencyAsc":
            labels = sorted(counts, key=lambda k: (counts[k], str(k)))
        elif order == "alphabetDesc":
            labels = sorted(counts, key=str, reverse=True)
        else:
            labels = sorted(counts, key=str)
        return StringIndexerModel(inputCol=self.getInputCol(), outputCol=self.getOutputCol(), labels=labels,
                                  handleInvalid=self.getHandleInvalid())


class OneHotEncoderModel(Model, HasInputCols, HasOutputCols):
    categorySizes = Param("original number of categories for each feature", [], T.toListInt)
    dropLast = Param("whether to drop the last category", True, T.toBoolean)
    handleInvalid = Param("error | keep", "error", T.toString)

    def _transform(self, df):
        out = df
        for c, o, k in zip(self.getInputCols(), self.getOutputCols(), self.getCategorySizes()):
            keep_extra = self.getHandleInvalid() == "keep"
            size = k + (1 if keep_extra else 0) - (1 if self.getDropLast() else 0)
            vecs = []
            for v in df[c].tolist():
                i = int(v) if v is not None and not (isinstance(v, float) and np.isnan(v)) else -1
                if i < 0 or i >= k:
                    if not keep_extra:
                        raise ValueError(f"invalid category {v} in column {c}")
                    i = k
                vecs.append(SparseVector(size, [i], [1.0]) if i < size else SparseVector(size, [], []))
            out = out.withColumn(o, _obj(vecs))
        return out


class OneHotEncoder(Estimator, HasInputCols, HasOutputCols, HasInputCol, HasOutputCol):
    dropLast = Param("whether to drop the last category", True, T.toBoolean)
    handleInvalid = Param("error | keep", "error", T.toString)

    def _fit(self, df):
        ins = self.getInputCols() or ([self.getInputCol()] if self.getInputCol() else [])
        outs = self.getOutputCols() or ([self.getOutputCol()] if self.getOutputCol() else [])
        sizes = []
        for c in ins:
            md = df.metadata(c).get("ml_attr", {})
            if "vals" in md:
                sizes.append(len(md["vals"]))
            else:
                vals = np.asarray([v for v in df[c].tolist() if v is not None], dtype=float)
                sizes.append(int(np.nanmax(vals)) + 1 if len(vals) else 0)
        return OneHotEncoderModel(inputCols=ins, outputCols=outs, categorySizes=sizes, dropLast=self.getDropLast(),
                                  handleInvalid=self.getHandleInvalid())


class VectorAssembler(Transformer, HasInputCols, HasOutputCol):
    handleInvalid = Param("error | skip | keep", "error", T.toString)

    def _transform(self, df):
        n = df.count()
        cols = self.getInputCols()
        pieces = []
        sparse = False
        for c in cols:
            col = df[c]
            if col.ndim == 2:
                pieces.append(("dense", col.astype(np.float64)))
            elif col.dtype.kind in "biuf":
                pieces.append(("dense", col.astype(np.float64).reshape(-1, 1)))
            else:
                vs = col.tolist()
                if any(isinstance(v, SparseVector) for v in vs):
                    sparse = True
                pieces.append(("obj", vs))
        if not sparse:
            mats = []
            for kind, p in pieces:
                if kind == "dense":
                    mats.append(p)
                else:
                    mats.append(np.stack([v.toArray() if isinstance(v, Vector) else np.asarray(v, float)
                                          for v in p]) if n else np.zeros((0, 0)))
            m = np.concatenate(mats, axis=1) if mats else np.zeros((n, 0))
            if self.getHandleInvalid() == "error" and np.isnan(m).any():
                raise ValueError("Encountered NaN while assembling a row with handleInvalid = \"error\"")
            return df.withColumn(self.getOutputCol(), m)
        out = []
        for i in range(n):
            idx, val, off = [], [], 0
            for kind, p in pieces:
                if kind == "dense":
                    row = p[i]
                    nz = np.nonzero(row)[0]
                    idx.extend((nz + off).tolist())
                    val.extend(row[nz].tolist())
                    off += p.shape[1]
                else:
                    v = p[i]
                    if isinstance(v, SparseVector):
                        idx.extend((v.indices + off).tolist())
                        val.extend(v.values.tolist())
                        off += v.size
                    else:
                        a = v.toArray() if isinstance(v, Vector) else np.asarray(v, float).reshape(-1)
                        nz = np.nonzero(a)[0]
                        idx.extend((nz + off).tolist())
                        val.extend(a[nz].tolist())
                        off += len(a)
            out.append(SparseVector(off, idx, val))
        return df.withColumn(self.getOutputCol(), _obj(out))


class FastVectorAssembler(VectorAssembler):
    """Assembler that keeps categorical slot metadata without a pass over the data (reference:
    SPX/ml/feature/FastVectorAssembler.scala). Columnar assembly above never scans rows for
    attribute metadata, so this is the same kernel under the reference's name."""
