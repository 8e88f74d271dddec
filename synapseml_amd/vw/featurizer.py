"""Hashing featurizers (reference: vw/.../VowpalWabbitFeaturizer.scala,
featurizer/*.scala, VowpalWabbitInteractions.scala,
VowpalWabbitMurmurWithPrefix.scala). Feature index = mask & murmur3(colName +
value, murmur3(outputCol, seed)); numeric columns hash the column name and keep
the value; zero values are dropped; duplicates are summed (sumCollisions)."""
from __future__ import annotations

from typing import Dict, List

import numpy as np

from ..core.contracts import HasInputCols, HasOutputCol
from ..core.dataframe import DataFrame
from ..core.linalg import CsrColumn, DenseVector, SparseVector
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Transformer
from ..ops import native


def _vw():
    return native.load("_vw")


_GPU_HASH_MIN = 200_000  # strings per call above which the device kernel pays for its copies


def hash_strings(strings, seed: int, mask: int = 0xFFFFFFFF, device: str = "auto") -> np.ndarray:
    """murmur3_32(utf8(s), seed) & mask for every string, in one native call over the packed UTF-8
    bytes (Arrow layout). ``device``: "gpu" runs the batched HIP kernel (K13), "cpu" the host loop,
    "auto" the kernel for large batches when a device is present."""
    enc = [x.encode("utf-8") for x in strings]
    lens = np.fromiter((len(b) for b in enc), dtype=np.int64, count=len(enc))
    offs = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    data = np.frombuffer(b"".join(enc), dtype=np.uint8) if enc else np.zeros(0, np.uint8)
    vw = _vw()
    if device == "auto":
        on_gpu = len(enc) >= _GPU_HASH_MIN and bool(vw.gpu_available())
    else:
        on_gpu = device == "gpu"
    return vw.murmur_offsets(data, offs, seed & 0xFFFFFFFF, mask & 0xFFFFFFFF, on_gpu)


def murmur_hash(s: str, seed: int) -> int:
    """VW murmur3_32 of the UTF-8 bytes of ``s`` (signed like the JVM int)."""
    h = int(_vw().murmur3(s.encode("utf-8"), seed & 0xFFFFFFFF))
    return h - (1 << 32) if h >= (1 << 31) else h


class VowpalWabbitMurmur:
    """Static murmur3_32 entry point of the VW native library
    (``VowpalWabbitMurmur.hash(str|bytes, seed)``, used at
    VowpalWabbitMurmurWithPrefix.scala:32,77 and VowpalWabbitUtil.scala:23).
    Strings hash their UTF-8 bytes; the result is a signed 32-bit int."""

    @staticmethod
    def hash(value, seed: int) -> int:  # noqa: A003
        data = value.encode("utf-8") if isinstance(value, str) else bytes(value)
        h = int(_vw().murmur3(data, seed & 0xFFFFFFFF))
        return h - (1 << 32) if h >= (1 << 31) else h


class VowpalWabbitMurmurWithPrefix:
    """Murmur hashing with a fixed string prefix (VowpalWabbitMurmurWithPrefix.scala:15-79)."""

    def __init__(self, prefix: str):
        self.prefix = prefix

    def hash(self, value: str, seed: int) -> int:
        return murmur_hash(self.prefix + value, seed)


def sort_and_distinct(indices: np.ndarray, values: np.ndarray, sum_collisions: bool = True):
    """VectorUtils.sortAndDistinct: sort by index, merge duplicates."""
    if len(indices) == 0:
        return indices.astype(np.int32), values.astype(np.float64)
    order = np.argsort(indices, kind="stable")
    idx = indices[order]
    val = values[order]
    uniq, first = np.unique(idx, return_index=True)
    if sum_collisions:
        sums = np.add.reduceat(val, first)
    else:
        sums = val[first]
    return uniq.astype(np.int32), sums.astype(np.float64)


class HasNumBits(Transformer):
    numBits = Param("Number of bits used to mask", 30, T.toInt)


class VowpalWabbitFeaturizer(HasNumBits, HasInputCols, HasOutputCol):
    seed = Param("Hash seed", 0, T.toInt)
    stringSplitInputCols = Param("Input cols that should be split at word boundaries", [], T.toListString)
    sumCollisions = Param("Sums collisions if true, otherwise removes them", True, T.toBoolean)
    prefixStringsWithColumnName = Param("Prefix string features with column name", True, T.toBoolean)
    preserveOrderNumBits = Param("Number of bits used to preserve the feature order", 0, T.toInt)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(outputCol="features", inputCols=[])

    def _all_cols(self) -> List[str]:
        return list(self.getInputCols() or []) + list(self.getStringSplitInputCols() or [])

    def _transform(self, df: DataFrame) -> DataFrame:
        nb, po = self.getNumBits(), self.getPreserveOrderNumBits()
        if nb + po > 30:
            raise ValueError(f"Number of bits used for hashing ({nb}) and for order preserving ({po}) must be <= 30")
        for c in self._all_cols():
            if c not in df:
                raise ValueError(f"missing input column {c}")
        mask = (1 << nb) - 1
        ns_hash = murmur_hash(self.getOutputCol(), self.getSeed()) & 0xFFFFFFFF
        vw = _vw()
        prefix_on = self.getPrefixStringsWithColumnName()
        split_cols = set(self.getStringSplitInputCols() or [])
        n = df.count()
        # features accumulate as COO chunks (row, index, value) in column order; one stable sort by row then
        # keeps each row's features in column order, as the per-row concatenation did
        R: List[np.ndarray] = []
        I: List[np.ndarray] = []
        V: List[np.ndarray] = []

        def add_coo(rows, idx, val):
            R.append(np.asarray(rows, dtype=np.int64))
            I.append(np.asarray(idx, dtype=np.int64))
            V.append(np.asarray(val, dtype=np.float64))

        def add(i, idx, val):
            idx = np.asarray(idx, dtype=np.int64)
            add_coo(np.full(len(idx), i, np.int64), idx, val)

        for c in self._all_cols():
            col = df[c]
            pre = c if prefix_on else ""
            if isinstance(col, CsrColumn):  # columnar sparse vectors: indices kept (masked to the table)
                ip, ind, val = col.csr()
                ind = ind.astype(np.int64)
                add_coo(np.repeat(np.arange(n, dtype=np.int64), np.diff(ip)), ind & mask if col.size >= mask + 1 else ind,
                        val)
                continue
            if isinstance(col, np.ndarray) and col.ndim == 2:  # dense vector column
                width = col.shape[1]
                idx = np.arange(width, dtype=np.int64) & mask if width >= mask + 1 else np.arange(width)
                add_coo(np.repeat(np.arange(n, dtype=np.int64), width), np.tile(idx, n), col.reshape(-1))
                continue
            if col.dtype.kind in "biuf":
                h = int(vw.murmur3(c.encode(), ns_hash)) & mask
                vals = col.astype(np.float64)
                nz = np.flatnonzero(vals)
                add_coo(nz, np.full(len(nz), h, np.int64), np.ones(len(nz)) if col.dtype.kind == "b" else vals[nz])
                continue
            # object columns: strings, string lists, maps, vectors
            vals = col.tolist()
            strs = [i for i, v in enumerate(vals) if isinstance(v, str)]
            if strs and len(strs) == sum(v is not None for v in vals):
                # a string column: every row's tokens hashed in one native call (K13 on the GPU for big columns)
                toks = [vals[i].split() if c in split_cols else [vals[i]] for i in strs]
                flat = [pre + t for tk in toks for t in tk]
                hs = hash_strings(flat, ns_hash, mask).astype(np.int64)
                cnt = np.fromiter((len(tk) for tk in toks), dtype=np.int64, count=len(toks))
                add_coo(np.repeat(np.asarray(strs, np.int64), cnt), hs, np.ones(len(hs)))
                continue
            for i, v in enumerate(vals):
                if v is None:
                    continue
                if isinstance(v, str):
                    toks = v.split() if c in split_cols else [v]
                    hs = vw.murmur_batch(toks, ns_hash, pre) & mask
                    add(i, hs, np.ones(len(toks)))
                elif isinstance(v, (list, tuple)) and (not v or isinstance(v[0], str)):
                    hs = vw.murmur_batch([str(t) for t in v], ns_hash, pre) & mask
                    add(i, hs, np.ones(len(v)))
                elif isinstance(v, dict):
                    keys = [str(k) for k in v.keys()]
                    mvals = np.asarray([float(x) if not isinstance(x, str) else 1.0 for x in v.values()])
                    if any(isinstance(x, str) for x in v.values()):
                        keys = [f"{k}{x}" if isinstance(x, str) else k for k, x in v.items()]
                    hs = vw.murmur_batch(keys, ns_hash, c) & mask
                    nz = mvals != 0
                    add(i, hs[nz], mvals[nz])
                elif isinstance(v, SparseVector):
                    add(i, v.indices.astype(np.int64) & mask if v.size >= mask + 1 else v.indices, v.values)
                elif isinstance(v, (DenseVector, np.ndarray, list, tuple)):
                    a = np.asarray(v, dtype=np.float64)
                    add(i, np.arange(len(a)), a)
                elif isinstance(v, (bool, np.bool_)):
                    if v:
                        add(i, [int(vw.murmur3(c.encode(), ns_hash)) & mask], [1.0])
                else:
                    fv = float(v)
                    if fv != 0:
                        add(i, [int(vw.murmur3(c.encode(), ns_hash)) & mask], [fv])
        size = (1 << 30) if po > 0 else (1 << nb)
        rows = np.concatenate(R) if R else np.zeros(0, np.int64)
        idx = np.concatenate(I) if I else np.zeros(0, np.int64)
        val = np.concatenate(V) if V else np.zeros(0)
        order = np.argsort(rows, kind="stable")
        rows, idx, val = rows[order], idx[order], val[order]
        counts = np.bincount(rows, minlength=n) if len(rows) else np.zeros(n, np.int64)
        starts = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
        if po > 0:
            if len(counts) and counts.max() > (1 << po):
                raise ValueError(f"Too many features {int(counts.max())} for preserveOrderNumBits={po}")
            pos = np.arange(len(rows), dtype=np.int64) - starts[rows]
            idx = idx | (pos << (30 - po))
        # VectorUtils.sortAndDistinct per row: sort by index (stable), merge duplicates (sum or keep the first)
        order = np.lexsort((idx, rows))
        rows, idx, val = rows[order], idx[order], val[order]
        first = np.ones(len(rows), dtype=bool)
        if len(rows) > 1:
            first[1:] = (rows[1:] != rows[:-1]) | (idx[1:] != idx[:-1])
        heads = np.flatnonzero(first)
        out_val = np.add.reduceat(val, heads) if (self.getSumCollisions() and len(heads)) else val[heads]
        out_rows, out_idx = rows[heads], idx[heads]
        indptr = np.zeros(n + 1, np.int64)
        np.cumsum(np.bincount(out_rows, minlength=n) if len(out_rows) else np.zeros(n, np.int64), out=indptr[1:])
        return df.withColumn(self.getOutputCol(), CsrColumn(indptr, out_idx.astype(np.int32), out_val, size))


class VowpalWabbitInteractions(HasNumBits, HasInputCols, HasOutputCol):
    """Quadratic (and higher) feature crosses of sparse vectors for non-VW
    learners (VowpalWabbitInteractions.scala): index = mask & (h1 * FNV ^ h2)."""

    sumCollisions = Param("Sums collisions if true, otherwise removes them", True, T.toBoolean)

    def _transform(self, df: DataFrame) -> DataFrame:
        mask = (1 << self.getNumBits()) - 1
        fnv = 16777619
        cols = [df[c] for c in self.getInputCols()]
        n = df.count()
        out = np.empty(n, dtype=object)

        def as_sparse(v):
            if isinstance(v, SparseVector):
                return v.indices.astype(np.int64), v.values
            a = np.asarray(v, dtype=np.float64)
            nz = np.nonzero(a)[0]
            return nz.astype(np.int64), a[nz]

        for i in range(n):
            idx, val = as_sparse(cols[0][i])
            for c in cols[1:]:
                i2, v2 = as_sparse(c[i])
                idx = ((idx[:, None] * fnv) ^ i2[None, :]).ravel() & mask
                val = (val[:, None] * v2[None, :]).ravel()
            si, sv = sort_and_distinct(idx, val, self.getSumCollisions())
            out[i] = SparseVector(1 << self.getNumBits(), si, sv)
        return df.withColumn(self.getOutputCol(), out)
