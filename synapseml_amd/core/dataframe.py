"""Columnar, partitioned DataFrame: the orchestration substrate.

The reference runs on Spark DataFrames. There is no JVM or
pyspark here, so the framework carries its own DataFrame with
the subset of Spark semantics SynapseML relies on: named columns, partitions
(``repartition``/``coalesce``/``getNumPartitions``), ``mapPartitions``,
``withColumn``/``select``/``filter``, ``randomSplit``, collect/count, column
metadata (ML attributes such as categorical slots).

Storage is one numpy array per column. A dense vector column is a 2-D float
array (rows x width) - the layout the native engines consume without copies;
sparse/ragged vector columns are object arrays of :class:`SparseVector`, or one
CSR matrix (:class:`~synapseml_amd.core.linalg.CsrColumn`) that the engines take
zero-copy.
"""
from __future__ import annotations

import itertools
from typing import Any, Callable, Dict, Iterable, List, Optional, Sequence

import numpy as np

from .linalg import CsrColumn, DenseVector, SparseVector, Vector


class Row(dict):
    """dict with attribute access, like pyspark.sql.Row."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def asDict(self) -> dict:  # noqa: N802
        return dict(self)


def _as_column(values: Any, n: Optional[int] = None) -> np.ndarray:
    if isinstance(values, (np.ndarray, CsrColumn)):
        return values
    if isinstance(values, (list, tuple)):
        if values and isinstance(values[0], Vector):
            if all(isinstance(v, DenseVector) for v in values):
                widths = {v.size for v in values}
                if len(widths) == 1:
                    return np.stack([v.values for v in values])
            arr = np.empty(len(values), dtype=object)
            for i, v in enumerate(values):
                arr[i] = v
            return arr
        if values and isinstance(values[0], (list, tuple, np.ndarray, dict, str, bytes, type(None))):
            arr = np.empty(len(values), dtype=object)
            for i, v in enumerate(values):
                arr[i] = v
            return arr
        return np.asarray(values)
    if np.isscalar(values) and n is not None:
        return np.full(n, values)
    try:
        import pandas as pd

        if isinstance(values, pd.Series):
            return _as_column(values.tolist()) if values.dtype == object else values.to_numpy()
    except ImportError:  # pragma: no cover
        pass
    return np.asarray(values)


def _take(col: np.ndarray, idx) -> np.ndarray:
    return col[idx]


class DataFrame:
    def __init__(self, columns: Dict[str, Any], num_partitions: int = 1,
                 metadata: Optional[Dict[str, dict]] = None, partition_bounds: Optional[List[int]] = None):
        self._cols: Dict[str, np.ndarray] = {}
        n = None
        for k, v in columns.items():
            c = _as_column(v, n)
            if n is None:
                n = len(c)
            elif len(c) != n:
                raise ValueError(f"column {k!r} has {len(c)} rows, expected {n}")
            self._cols[k] = c
        self._n = 0 if n is None else n
        self._meta: Dict[str, dict] = dict(metadata or {})
        if partition_bounds is not None:
            self._bounds = list(partition_bounds)
        else:
            p = max(1, int(num_partitions))
            self._bounds = [self._n * i // p for i in range(p + 1)]

    # ---------------------------------------------------------------- basics
    @property
    def columns(self) -> List[str]:
        return list(self._cols.keys())

    @property
    def dtypes(self) -> List[tuple]:
        out = []
        for k, c in self._cols.items():
            if c.ndim == 2:
                out.append((k, "vector"))
            elif c.dtype == object:
                first = next((x for x in c if x is not None), None)
                out.append((k, "vector" if isinstance(first, Vector) else type(first).__name__ if first is not None else "null"))
            else:
                out.append((k, str(c.dtype)))
        return out

    @property
    def schema(self) -> Dict[str, str]:
        return dict(self.dtypes)

    def count(self) -> int:
        return self._n

    def __len__(self) -> int:
        return self._n

    def __getitem__(self, name: str) -> np.ndarray:
        return self._cols[name]

    def __contains__(self, name: str) -> bool:
        return name in self._cols

    def col(self, name: str) -> np.ndarray:
        return self._cols[name]

    def metadata(self, name: str) -> dict:
        return self._meta.get(name, {})

    def withMetadata(self, name: str, md: dict) -> "DataFrame":  # noqa: N802
        m = dict(self._meta)
        m[name] = dict(md)
        return self._replace(meta=m)

    def _replace(self, cols=None, meta=None, bounds=None) -> "DataFrame":
        df = DataFrame.__new__(DataFrame)
        df._cols = dict(self._cols) if cols is None else cols
        first = next(iter(df._cols.values()), None)
        df._n = 0 if first is None else len(first)
        df._meta = dict(self._meta) if meta is None else meta
        if bounds is not None:
            df._bounds = bounds
        elif df._n == self._n:
            df._bounds = list(self._bounds)
        else:
            p = self.getNumPartitions()
            df._bounds = [df._n * i // p for i in range(p + 1)]
        return df

    # ---------------------------------------------------------------- partitions
    def getNumPartitions(self) -> int:  # noqa: N802
        return len(self._bounds) - 1

    def partition_bounds(self) -> List[tuple]:
        return [(self._bounds[i], self._bounds[i + 1]) for i in range(self.getNumPartitions())]

    def repartition(self, n: int, *cols: str) -> "DataFrame":
        n = max(1, int(n))
        if cols:
            # hash partition by key columns: rows of one key end up together
            keys = [self._cols[c] for c in cols]
            h = np.zeros(self._n, dtype=np.int64)
            for k in keys:
                h = h * 1000003 + np.asarray([hash(x) for x in k.tolist()], dtype=np.int64)
            part = np.mod(h, n)
            order = np.argsort(part, kind="stable")
            df = self._take_rows(order)
            counts = np.bincount(part, minlength=n)
            bounds = [0] + list(np.cumsum(counts))
            df._bounds = [int(b) for b in bounds]
            return df
        return self._replace(bounds=[self._n * i // n for i in range(n + 1)])

    def coalesce(self, n: int) -> "DataFrame":
        n = max(1, min(int(n), self.getNumPartitions()))
        old = self._bounds
        p = self.getNumPartitions()
        nb = [old[(p * i) // n] for i in range(n)] + [old[-1]]
        return self._replace(bounds=nb)

    def partitions(self) -> List["DataFrame"]:
        return [self.slice(a, b) for a, b in self.partition_bounds()]

    def slice(self, a: int, b: int) -> "DataFrame":
        cols = {k: v[a:b] for k, v in self._cols.items()}
        return self._replace(cols=cols, bounds=[0, b - a])

    def mapPartitions(self, fn: Callable[["DataFrame"], "DataFrame"]) -> "DataFrame":  # noqa: N802
        parts = [fn(p) for p in self.partitions()]
        return DataFrame.union_all(parts, keep_partitions=True)

    # ---------------------------------------------------------------- columns
    def select(self, *cols) -> "DataFrame":
        names = []
        for c in cols:
            if isinstance(c, (list, tuple)):
                names.extend(c)
            else:
                names.append(c)
        if names == ["*"]:
            return self
        cols_ = {k: self._cols[k] for k in names}
        meta = {k: v for k, v in self._meta.items() if k in cols_}
        return self._replace(cols=cols_, meta=meta)

    def withColumn(self, name: str, values, metadata: Optional[dict] = None) -> "DataFrame":  # noqa: N802
        if callable(values) and not isinstance(values, np.ndarray):
            values = values(self)
        c = _as_column(values, self._n)
        if len(c) != self._n:
            raise ValueError(f"withColumn {name!r}: {len(c)} values for {self._n} rows")
        cols = dict(self._cols)
        cols[name] = c
        meta = dict(self._meta)
        if metadata is not None:
            meta[name] = metadata
        elif name in meta:
            meta.pop(name)
        return self._replace(cols=cols, meta=meta)

    def withColumnRenamed(self, old: str, new: str) -> "DataFrame":  # noqa: N802
        cols = {(new if k == old else k): v for k, v in self._cols.items()}
        meta = {(new if k == old else k): v for k, v in self._meta.items()}
        return self._replace(cols=cols, meta=meta)

    def drop(self, *names: str) -> "DataFrame":
        cols = {k: v for k, v in self._cols.items() if k not in names}
        meta = {k: v for k, v in self._meta.items() if k not in names}
        return self._replace(cols=cols, meta=meta)

    # ---------------------------------------------------------------- rows
    def _take_rows(self, idx) -> "DataFrame":
        cols = {k: v[idx] for k, v in self._cols.items()}
        return self._replace(cols=cols)

    def filter(self, cond) -> "DataFrame":
        if callable(cond) and not isinstance(cond, np.ndarray):
            cond = cond(self)
        mask = np.asarray(cond, dtype=bool)
        df = self._take_rows(mask)
        # keep partitioning proportional
        p = self.getNumPartitions()
        counts = [int(mask[a:b].sum()) for a, b in self.partition_bounds()]
        df._bounds = [0] + list(itertools.accumulate(counts))
        assert len(df._bounds) == p + 1
        return df

    where = filter

    def limit(self, n: int) -> "DataFrame":
        return self.slice(0, min(n, self._n))

    def orderBy(self, *cols: str, ascending: bool = True) -> "DataFrame":  # noqa: N802
        keys = [self._cols[c] for c in reversed(cols)]
        order = np.lexsort(keys) if keys else np.arange(self._n)
        if not ascending:
            order = order[::-1]
        return self._take_rows(order)

    sort = orderBy

    def randomSplit(self, weights: Sequence[float], seed: int = 0) -> List["DataFrame"]:  # noqa: N802
        w = np.asarray(weights, dtype=np.float64)
        w = w / w.sum()
        rng = np.random.default_rng(seed)
        u = rng.random(self._n)
        edges = np.concatenate([[0.0], np.cumsum(w)])
        return [self.filter((u >= edges[i]) & (u < edges[i + 1])) for i in range(len(w))]

    def sample(self, fraction: float, seed: int = 0, withReplacement: bool = False) -> "DataFrame":  # noqa: N803
        rng = np.random.default_rng(seed)
        if withReplacement:
            idx = rng.integers(0, self._n, size=int(round(self._n * fraction)))
            return self._take_rows(np.sort(idx))
        return self.filter(rng.random(self._n) < fraction)

    def union(self, other: "DataFrame") -> "DataFrame":
        return DataFrame.union_all([self, other], keep_partitions=True)

    unionAll = union

    @staticmethod
    def union_all(parts: List["DataFrame"], keep_partitions: bool = False) -> "DataFrame":
        parts = [p for p in parts if p is not None]
        if not parts:
            return DataFrame({})
        names = parts[0].columns
        cols = {}
        for k in names:
            arrs = [p._cols[k] for p in parts]
            if all(isinstance(a, CsrColumn) for a in arrs):
                cols[k] = CsrColumn.concat(arrs)
                continue
            arrs = [np.asarray(a) if isinstance(a, CsrColumn) else a for a in arrs]
            if any(a.dtype == object for a in arrs) or len({a.ndim for a in arrs}) > 1:
                out = np.empty(sum(len(a) for a in arrs), dtype=object)
                i = 0
                for a in arrs:
                    for x in (a if a.ndim == 1 else [DenseVector(r) for r in a]):
                        out[i] = x
                        i += 1
                cols[k] = out
            elif len({a.shape[1:] for a in arrs}) > 1:
                out = np.empty(sum(len(a) for a in arrs), dtype=object)
                i = 0
                for a in arrs:
                    for r in a:
                        out[i] = DenseVector(r)
                        i += 1
                cols[k] = out
            else:
                cols[k] = np.concatenate(arrs)
        bounds = [0]
        if keep_partitions:
            for p in parts:
                for a, b in p.partition_bounds():
                    bounds.append(bounds[-1] + (b - a))
        else:
            bounds = [0, sum(len(p) for p in parts)]
        df = DataFrame(cols, partition_bounds=bounds)
        df._meta = dict(parts[0]._meta)
        return df

    def distinct_values(self, name: str) -> list:
        c = self._cols[name]
        if c.dtype == object:
            seen, out = set(), []
            for x in c:
                if x not in seen:
                    seen.add(x)
                    out.append(x)
            return out
        return list(np.unique(c))

    def groupBy(self, *keys: str) -> "GroupedData":  # noqa: N802
        return GroupedData(self, list(keys))

    def join(self, other: "DataFrame", on, how: str = "inner") -> "DataFrame":
        on = [on] if isinstance(on, str) else list(on)
        right_index: Dict[tuple, List[int]] = {}
        rk = list(zip(*[other._cols[k].tolist() for k in on]))
        for i, k in enumerate(rk):
            right_index.setdefault(k, []).append(i)
        lk = list(zip(*[self._cols[k].tolist() for k in on]))
        li, ri = [], []
        for i, k in enumerate(lk):
            for j in right_index.get(k, []):
                li.append(i)
                ri.append(j)
            if how == "left" and k not in right_index:
                li.append(i)
                ri.append(-1)
        li = np.asarray(li, dtype=np.int64)
        ri = np.asarray(ri, dtype=np.int64)
        cols = {k: v[li] for k, v in self._cols.items()}
        for k, v in other._cols.items():
            if k in on:
                continue
            if how == "left":
                col = np.empty(len(ri), dtype=object)
                for t, j in enumerate(ri):
                    col[t] = None if j < 0 else v[j]
                cols[k] = col
            else:
                cols[k] = v[ri]
        return DataFrame(cols, num_partitions=self.getNumPartitions())

    # ---------------------------------------------------------------- actions
    def collect(self) -> List[Row]:
        names = self.columns
        out = []
        for i in range(self._n):
            r = Row()
            for k in names:
                v = self._cols[k][i]
                if self._cols[k].ndim == 2:
                    v = DenseVector(v)
                elif isinstance(v, np.generic):
                    v = v.item()
                r[k] = v
            out.append(r)
        return out

    def head(self, n: int = 1) -> List[Row]:
        return self.limit(n).collect()

    def take(self, n: int) -> List[Row]:
        return self.head(n)

    def first(self) -> Optional[Row]:
        h = self.head(1)
        return h[0] if h else None

    def cache(self) -> "DataFrame":
        return self

    persist = cache

    def unpersist(self) -> "DataFrame":
        return self

    def show(self, n: int = 20) -> None:  # pragma: no cover - cosmetic
        print(self.toPandas().head(n))

    def toPandas(self):  # noqa: N802
        import pandas as pd

        data = {}
        for k, v in self._cols.items():
            if v.ndim == 2:
                data[k] = [DenseVector(r) for r in v]
            else:
                data[k] = v
        return pd.DataFrame(data)

    @staticmethod
    def fromPandas(pdf, num_partitions: int = 1) -> "DataFrame":  # noqa: N802
        cols = {}
        for k in pdf.columns:
            s = pdf[k]
            cols[str(k)] = _as_column(s.tolist()) if s.dtype == object else s.to_numpy()
        return DataFrame(cols, num_partitions=num_partitions)

    def toArrow(self):  # noqa: N802
        """Arrow table (the columnar interchange Spark's ``mapInArrow`` / ``toArrow`` speak).
        2-D numeric columns (vectors, tensors) become fixed-size-list columns without a copy
        of the row data into Python objects."""
        import pyarrow as pa

        arrays, names = [], []
        for k, v in self._cols.items():
            if v.ndim == 2 and v.dtype != object:
                flat = pa.array(np.ascontiguousarray(v).reshape(-1))
                arrays.append(pa.FixedSizeListArray.from_arrays(flat, v.shape[1]))
            elif v.dtype == object:
                arrays.append(pa.array([_arrow_value(x) for x in v]))
            else:
                arrays.append(pa.array(v))
            names.append(k)
        return pa.Table.from_arrays(arrays, names=names)

    @staticmethod
    def fromArrow(table, num_partitions: int = 1) -> "DataFrame":  # noqa: N802
        """DataFrame from an Arrow table or record batches; fixed-size-list numeric columns
        become 2-D arrays (the layout the native engines ingest directly)."""
        import pyarrow as pa

        if isinstance(table, pa.RecordBatch):
            table = pa.Table.from_batches([table])
        elif isinstance(table, (list, tuple)):
            table = pa.Table.from_batches(list(table))
        cols = {}
        for name, col in zip(table.column_names, table.columns):
            t = col.type
            if pa.types.is_fixed_size_list(t) and (pa.types.is_floating(t.value_type) or pa.types.is_integer(t.value_type)):
                flat = col.combine_chunks().flatten().to_numpy(zero_copy_only=False)
                cols[name] = flat.reshape(len(col), t.list_size)
            elif ((pa.types.is_list(t) or pa.types.is_large_list(t)) and
                  (pa.types.is_floating(t.value_type) or pa.types.is_integer(t.value_type)) and col.null_count == 0
                  and _uniform_list_width(col) is not None):
                # array<double> (Spark's vector_to_array): equal-length rows become a 2-D array from the flat
                # values buffer, with no per-row Python objects
                w = _uniform_list_width(col)
                flat = col.combine_chunks().flatten().to_numpy(zero_copy_only=False)
                cols[name] = flat.reshape(len(col), w)
            elif pa.types.is_floating(t) or pa.types.is_integer(t) or pa.types.is_boolean(t):
                cols[name] = col.to_numpy()
            else:
                cols[name] = _as_column(col.to_pylist())
        return DataFrame(cols, num_partitions=num_partitions)

    @staticmethod
    def fromRows(rows: Iterable[dict], num_partitions: int = 1) -> "DataFrame":  # noqa: N802
        rows = list(rows)
        if not rows:
            return DataFrame({})
        names = list(rows[0].keys())
        return DataFrame({k: [r[k] for r in rows] for k in names}, num_partitions=num_partitions)

    def __repr__(self) -> str:
        return f"DataFrame[{', '.join(f'{k}: {t}' for k, t in self.dtypes)}] ({self._n} rows, {self.getNumPartitions()} partitions)"


def _uniform_list_width(col):
    """Common length of every row of a list column, or None when the lengths differ."""
    arr = col.combine_chunks()
    off = arr.offsets.to_numpy(zero_copy_only=False)
    if len(off) < 2:
        return 0
    d = np.diff(off)
    return int(d[0]) if (d == d[0]).all() else None


def _arrow_value(x):
    if isinstance(x, DenseVector):
        return x.toArray().tolist()
    if isinstance(x, np.ndarray):
        return x.tolist()
    if isinstance(x, np.generic):
        return x.item()
    return x


class GroupedData:
    def __init__(self, df: DataFrame, keys: List[str]):
        self.df = df
        self.keys = keys

    def _groups(self):
        key_rows = list(zip(*[self.df[k].tolist() for k in self.keys]))
        groups: Dict[tuple, List[int]] = {}
        for i, k in enumerate(key_rows):
            groups.setdefault(k, []).append(i)
        return groups

    def agg(self, **aggs: tuple) -> DataFrame:
        """agg(out=("col", "sum"|"mean"|"count"|"max"|"min"|"collect_list"|callable))"""
        groups = self._groups()
        out: Dict[str, list] = {k: [] for k in self.keys}
        for name in aggs:
            out[name] = []
        for key, idx in groups.items():
            for kname, kv in zip(self.keys, key):
                out[kname].append(kv)
            for name, (col, fn) in aggs.items():
                vals = self.df[col][idx]
                if callable(fn):
                    out[name].append(fn(vals))
                elif fn == "sum":
                    out[name].append(np.sum(vals))
                elif fn == "mean":
                    out[name].append(np.mean(vals))
                elif fn == "count":
                    out[name].append(len(idx))
                elif fn == "max":
                    out[name].append(np.max(vals))
                elif fn == "min":
                    out[name].append(np.min(vals))
                elif fn == "collect_list":
                    out[name].append(list(vals))
                else:
                    raise ValueError(f"unknown aggregate {fn}")
        return DataFrame(out)

    def count(self) -> DataFrame:
        groups = self._groups()
        out: Dict[str, list] = {k: [] for k in self.keys}
        out["count"] = []
        for key, idx in groups.items():
            for kname, kv in zip(self.keys, key):
                out[kname].append(kv)
            out["count"].append(len(idx))
        return DataFrame(out)


def createDataFrame(data, columns: Optional[Sequence[str]] = None, num_partitions: int = 1) -> DataFrame:  # noqa: N802
    """Build a DataFrame from a dict of columns, a list of rows/tuples or pandas."""
    try:
        import pandas as pd

        if isinstance(data, pd.DataFrame):
            return DataFrame.fromPandas(data, num_partitions)
    except ImportError:  # pragma: no cover
        pass
    if isinstance(data, dict):
        return DataFrame(data, num_partitions=num_partitions)
    rows = list(data)
    if not rows:
        return DataFrame({c: [] for c in (columns or [])})
    if isinstance(rows[0], dict):
        return DataFrame.fromRows(rows, num_partitions)
    if columns is None:
        columns = [f"_{i + 1}" for i in range(len(rows[0]))]
    return DataFrame({c: [r[i] for r in rows] for i, c in enumerate(columns)}, num_partitions=num_partitions)
