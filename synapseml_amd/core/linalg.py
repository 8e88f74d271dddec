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
