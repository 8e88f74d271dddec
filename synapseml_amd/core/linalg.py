"""Dense / sparse vectors (the pyspark.ml.linalg surface the reference uses).

The reference's models take ``Vector`` feature columns (Spark ML). These are
small, numpy-backed equivalents; columns of them are stored either as a 2-D
ndarray (dense, the fast path) or as an object array of vectors.
"""
from __future__ import annotations

from typing import Iterable, Sequence

import numpy as np


class Vector:
    size: int

    def toArray(self) -> np.ndarray:  # noqa: N802 - Spark API name
        raise NotImplementedError

    def __len__(self) -> int:
        return self.size

    def __iter__(self):
        return iter(self.toArray())

    def __array__(self, dtype=None, copy=None):
        a = self.toArray()
        return a.astype(dtype) if dtype is not None else a


class DenseVector(Vector):
    __slots__ = ("values",)

    def __init__(self, values: Iterable[float]):
        self.values = np.asarray(list(values) if not isinstance(values, np.ndarray) else values, dtype=np.float64)

    @property
    def size(self) -> int:
        return int(self.values.shape[0])

    def toArray(self) -> np.ndarray:  # noqa: N802
        return self.values

    def __getitem__(self, i):
        return self.values[i]

    def __eq__(self, other) -> bool:
        if isinstance(other, Vector):
            return self.size == other.size and np.array_equal(self.toArray(), other.toArray())
        return False

    def __hash__(self) -> int:
        return hash(self.values.tobytes())

    def __repr__(self) -> str:
        return f"DenseVector({self.values.tolist()})"


class SparseVector(Vector):
    __slots__ = ("_size", "indices", "values")

    def __init__(self, size: int, indices, values=None):
        if values is None and isinstance(indices, dict):
            items = sorted(indices.items())
            indices = [k for k, _ in items]
            values = [v for _, v in items]
        self._size = int(size)
        self.indices = np.asarray(indices, dtype=np.int32)
        self.values = np.asarray(values, dtype=np.float64)
        if len(self.indices) != len(self.values):
            raise ValueError("indices and values must have the same length")

    @property
    def size(self) -> int:
        return self._size

    def toArray(self) -> np.ndarray:  # noqa: N802
        a = np.zeros(self._size, dtype=np.float64)
        a[self.indices] = self.values
        return a

    def __getitem__(self, i):
        pos = np.searchsorted(self.indices, i)
        if pos < len(self.indices) and self.indices[pos] == i:
            return self.values[pos]
        return 0.0

    def __eq__(self, other) -> bool:
        if isinstance(other, Vector):
            return self.size == other.size and np.array_equal(self.toArray(), other.toArray())
        return False

    def __hash__(self) -> int:
        return hash((self._size, self.indices.tobytes(), self.values.tobytes()))

    def __repr__(self) -> str:
        return f"SparseVector({self._size}, {self.indices.tolist()}, {self.values.tolist()})"


class CsrColumn:
    """A column of sparse vectors stored as ONE CSR matrix (indptr int64, indices int32/uint32, values float32 or
    float64, a common size) instead of an object array of :class:`SparseVector` rows.

    Rows read back as SparseVector (so row-wise code keeps working), while the engines take the CSR arrays
    without a per-row Python loop: VW's namespace blocks and LightGBM's CSR push are zero-copy views, and
    slicing a contiguous row range (partitions) only rebases ``indptr``. It supports the subset of the numpy
    1-D array surface the DataFrame uses (len, ndim / dtype / shape, int / slice / mask / index-array
    ``__getitem__``, iteration, ``tolist``); ``np.asarray`` materialises the object-array form."""

    ndim = 1
    dtype = np.dtype(object)

    def __init__(self, indptr, indices, values, size: int):
        self.indptr = np.asarray(indptr, dtype=np.int64)
        self.indices = np.asarray(indices)
        self.values = np.asarray(values)
        self.size = int(size)
        if self.indptr.ndim != 1 or len(self.indptr) < 1:
            raise ValueError("indptr must be a 1-D array of n + 1 offsets")
        if len(self.indices) != len(self.values):
            raise ValueError("indices and values must have the same length")

    @property
    def shape(self):
        return (len(self.indptr) - 1,)

    def __len__(self) -> int:
        return len(self.indptr) - 1

    def row(self, i: int) -> SparseVector:
        a, b = self.indptr[i] - self.indptr[0], self.indptr[i + 1] - self.indptr[0]
        return SparseVector(self.size, self.indices[a:b].astype(np.int32), self.values[a:b])

    def csr(self):
        """(indptr rebased to 0, indices, values) of the rows, without copying when already rebased"""
        base = int(self.indptr[0])
        ip = self.indptr - base if base else self.indptr
        return ip, self.indices[: ip[-1]] if len(self.indices) != ip[-1] else self.indices, \
            self.values[: ip[-1]] if len(self.values) != ip[-1] else self.values

    def __getitem__(self, key):
        n = len(self)
        if isinstance(key, (int, np.integer)):
            k = int(key)
            if k < 0:
                k += n
            if not 0 <= k < n:
                raise IndexError(key)
            return self.row(k)
        if isinstance(key, slice):
            a, b, step = key.indices(n)
            if step == 1:
                b = max(a, b)
                s, e = int(self.indptr[a]), int(self.indptr[b])
                base = int(self.indptr[0])
                return CsrColumn(self.indptr[a:b + 1] - s, self.indices[s - base:e - base],
                                 self.values[s - base:e - base], self.size)
            key = np.arange(a, b, step)
        idx = np.asarray(key)
        if idx.dtype == bool:
            if len(idx) != n:
                raise IndexError("boolean index length mismatch")
            idx = np.flatnonzero(idx)
        idx = idx.astype(np.int64)
        idx[idx < 0] += n
        ip, ind, val = self.csr()
        lens = ip[idx + 1] - ip[idx]
        out_ip = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        # gather of the selected rows' nonzeros: source position = row start + offset within the row
        src = np.repeat(ip[idx] - out_ip[:-1], lens) + np.arange(out_ip[-1], dtype=np.int64)
        return CsrColumn(out_ip, ind[src], val[src], self.size)

    def __iter__(self):
        for i in range(len(self)):
            yield self.row(i)

    def tolist(self) -> list:
        return list(self)

    def __array__(self, dtype=None, copy=None):
        out = np.empty(len(self), dtype=object)
        for i in range(len(self)):
            out[i] = self.row(i)
        return out

    @staticmethod
    def concat(cols) -> "CsrColumn":
        parts = [c.csr() for c in cols]
        sizes = {c.size for c in cols}
        offs = np.cumsum([0] + [p[0][-1] for p in parts])
        ip = np.concatenate([parts[0][0][:1]] + [p[0][1:] + o for p, o in zip(parts, offs[:-1])])
        return CsrColumn(ip, np.concatenate([p[1] for p in parts]), np.concatenate([p[2] for p in parts]),
                         max(sizes) if sizes else 0)

    @staticmethod
    def from_rows(rows, size: int = 0) -> "CsrColumn":
        ip, ii, vv = [0], [], []
        for r in rows:
            if isinstance(r, SparseVector):
                ii.append(r.indices)
                vv.append(r.values)
                size = max(size, r.size)
            else:
                a = np.asarray(r, dtype=np.float64)
                nz = np.flatnonzero(a)
                ii.append(nz.astype(np.int32))
                vv.append(a[nz])
                size = max(size, len(a))
            ip.append(ip[-1] + len(ii[-1]))
        return CsrColumn(np.asarray(ip, np.int64), np.concatenate(ii) if ii else np.zeros(0, np.int32),
                         np.concatenate(vv) if vv else np.zeros(0), size)

    def __repr__(self) -> str:
        return f"CsrColumn(rows={len(self)}, size={self.size}, nnz={int(self.indptr[-1] - self.indptr[0])})"


class Vectors:
    @staticmethod
    def dense(*values) -> DenseVector:
        if len(values) == 1 and not isinstance(values[0], (int, float)):
            return DenseVector(values[0])
        return DenseVector(values)

    @staticmethod
    def sparse(size: int, indices, values=None) -> SparseVector:
        return SparseVector(size, indices, values)

    @staticmethod
    def zeros(size: int) -> DenseVector:
        return DenseVector(np.zeros(size))


def as_matrix(col) -> np.ndarray:
    """Vector column -> dense 2-D float64 matrix."""
    if isinstance(col, np.ndarray) and col.ndim == 2:
        return np.ascontiguousarray(col, dtype=np.float64)
    rows = list(col)
    if not rows:
        return np.zeros((0, 0))
    width = max(len(r) for r in rows)
    out = np.zeros((len(rows), width), dtype=np.float64)
    for i, r in enumerate(rows):
        if isinstance(r, SparseVector):
            out[i, r.indices] = r.values
        else:
            a = np.asarray(r, dtype=np.float64)
            out[i, : a.shape[0]] = a
    return out


def as_csr(col):
    """Vector column -> (indptr int64, indices int32, values float64, width)."""
    if isinstance(col, CsrColumn):
        ip, ind, val = col.csr()
        return ip, ind.astype(np.int32, copy=False), val.astype(np.float64, copy=False), col.size
    rows = list(col) if not (isinstance(col, np.ndarray) and col.ndim == 2) else None
    if rows is None:
        m = np.asarray(col, dtype=np.float64)
        nz = m != 0
        indptr = np.concatenate([[0], np.cumsum(nz.sum(1))]).astype(np.int64)
        rr, cc = np.nonzero(nz)
        return indptr, cc.astype(np.int32), m[rr, cc], m.shape[1]
    indptr = [0]
    idx, val = [], []
    width = 0
    for r in rows:
        if isinstance(r, SparseVector):
            idx.append(r.indices)
            val.append(r.values)
            width = max(width, r.size)
            indptr.append(indptr[-1] + len(r.indices))
        else:
            a = np.asarray(r, dtype=np.float64)
            nz = np.nonzero(a)[0]
            idx.append(nz.astype(np.int32))
            val.append(a[nz])
            width = max(width, a.shape[0])
            indptr.append(indptr[-1] + len(nz))
    cat_i = np.concatenate(idx).astype(np.int32) if idx else np.zeros(0, np.int32)
    cat_v = np.concatenate(val).astype(np.float64) if val else np.zeros(0)
    return np.asarray(indptr, np.int64), cat_i, cat_v, width


def is_sparse_column(col) -> bool:
    if isinstance(col, CsrColumn):
        return True
    if isinstance(col, np.ndarray) and col.ndim == 2:
        return False
    for r in col[:10] if hasattr(col, "__getitem__") else []:
        return isinstance(r, SparseVector)
    return False


def to_vector_column(mat: np.ndarray) -> np.ndarray:
    """2-D matrix kept as-is (the dense vector column layout)."""
    return np.ascontiguousarray(mat)


def vector_list(values: Sequence) -> list:
    return [v if isinstance(v, Vector) else DenseVector(v) for v in values]
