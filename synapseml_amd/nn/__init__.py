"""Maximum-inner-product nearest neighbours (reference: core/.../nn/
{BallTree, ConditionalBallTree, KNN, ConditionalKNN}.scala).

``BallTree`` / ``ConditionalBallTree`` reproduce the reference's exact
branch-and-bound search on the host. ``KNNModel.transform`` is exact MIPS as
a blocked GEMM (queries × keysᵀ) + top-k on the device when a GPU is visible
— on the MI355X a dense GEMM over all keys beats tree traversal — and falls
back to the ball tree on the host."""
from __future__ import annotations

import heapq
from typing import Any, Dict, List, Optional, Sequence, Set

import numpy as np

from ..core.contracts import HasFeaturesCol, HasLabelCol, HasOutputCol
from ..core.dataframe import DataFrame
from ..core.linalg import as_matrix
from ..core.params import Param, Params, TypeConverters as T
from ..core.pipeline import Estimator, Model


class _Node:
    __slots__ = ("idx", "center", "radius", "left", "right", "labels")

    def __init__(self, idx, center, radius, left=None, right=None):
        self.idx, self.center, self.radius, self.left, self.right = idx, center, radius, left, right
        self.labels = None


class BestMatch:
    __slots__ = ("index", "distance")

    def __init__(self, index: int, distance: float):
        self.index, self.distance = index, distance

    def __repr__(self):
        return f"BestMatch({self.index}, {self.distance:.4g})"


class BallTree:
    """Ball tree for maximum inner product search: bound = q·c + |q|·r."""

    def __init__(self, keys, values: Sequence[Any], leafSize: int = 50):  # noqa: N803
        self.keys = np.asarray(keys, dtype=np.float64)
        self.values = list(values)
        self.leaf_size = leafSize
        self.root = self._build(np.arange(len(self.keys)))

    def _build(self, idx: np.ndarray) -> _Node:
        pts = self.keys[idx]
        center = pts.mean(0)
        radius = float(np.sqrt(((pts - center) ** 2).sum(1).max())) if len(idx) else 0.0
        if len(idx) <= self.leaf_size:
            return _Node(idx, center, radius)
        # two far-apart pivots
        a = int(np.argmax(((pts - pts[0]) ** 2).sum(1)))
        b = int(np.argmax(((pts - pts[a]) ** 2).sum(1)))
        da = ((pts - pts[a]) ** 2).sum(1)
        db = ((pts - pts[b]) ** 2).sum(1)
        left = idx[da <= db]
        right = idx[da > db]
        if len(left) == 0 or len(right) == 0:
            return _Node(idx, center, radius)
        return _Node(idx, center, radius, self._build(left), self._build(right))

    @staticmethod
    def _bound(q, qn, node):
        return float(q @ node.center) + qn * node.radius

    def _search(self, q, k, node, heap, allowed: Optional[Set[int]] = None):
        qn = float(np.linalg.norm(q))
        if len(heap) == k and heap[0][0] > self._bound(q, qn, node):
            return
        if node.left is None:
            ids = node.idx if allowed is None else [i for i in node.idx if i in allowed]
            for i in ids:
                d = float(q @ self.keys[i])
                item = (d, -int(i))
                if len(heap) < k:
                    heapq.heappush(heap, item)
                elif item > heap[0]:
                    heapq.heapreplace(heap, item)
            return
        children = sorted([node.left, node.right], key=lambda n: -self._bound(q, qn, n))
        for c in children:
            self._search(q, k, c, heap, allowed)

    def findMaximumInnerProducts(self, queryPoint, k: int = 1) -> List[BestMatch]:  # noqa: N802,N803
        heap: list = []
        self._search(np.asarray(queryPoint, np.float64), k, self.root, heap)
        return [BestMatch(-i, d) for d, i in sorted(heap, reverse=True)]


class ConditionalBallTree(BallTree):
    def __init__(self, keys, values, labels: Sequence[Any], leafSize: int = 50):  # noqa: N803
        self.labels = list(labels)
        super().__init__(keys, values, leafSize)

    def save(self, filename: str) -> None:
        """keys, values, labels and leaf size as JSON (rebuilt deterministically on load; reference
        nn/ConditionalBallTree.py save / load)"""
        import json

        with open(filename, "w") as f:
            json.dump({"keys": self.keys.tolist(), "values": list(self.values), "labels": list(self.labels),
                       "leafSize": self.leaf_size}, f)

    @staticmethod
    def load(filename: str) -> "ConditionalBallTree":
        import json

        with open(filename) as f:
            d = json.load(f)
        return ConditionalBallTree(np.asarray(d["keys"], np.float64), d["values"], d["labels"], d["leafSize"])

    def findMaximumInnerProducts(self, queryPoint, conditioner: Set[Any], k: int = 1):  # noqa: N802,N803
        allowed = {i for i, l in enumerate(self.labels) if l in conditioner}
        heap: list = []
        if allowed:
            self._search(np.asarray(queryPoint, np.float64), k, self.root, heap, allowed)
        return [BestMatch(-i, d) for d, i in sorted(heap, reverse=True)]


def _device_mips(Q: np.ndarray, K: np.ndarray, k: int, mask: Optional[np.ndarray] = None, block: int = 8192):
    """Exact top-k inner products via blocked device GEMM; ties broken by smaller index like the tree."""
    import torch

    dev = torch.device("cuda")
    Kt = torch.as_tensor(K, dtype=torch.float32, device=dev)
    out_v, out_i = [], []
    for s in range(0, len(Q), block):
        q = torch.as_tensor(Q[s:s + block], dtype=torch.float32, device=dev)
        sc = q @ Kt.T
        if mask is not None:
            sc = sc.masked_fill(~torch.as_tensor(mask[s:s + block], device=dev), float("-inf"))
        v, i = torch.topk(sc, min(k, K.shape[0]), dim=1)
        out_v.append(v.cpu().numpy())
        out_i.append(i.cpu().numpy())
    return np.concatenate(out_v), np.concatenate(out_i)


def _use_gpu() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


class _KNNParams(HasFeaturesCol, HasOutputCol):
    valuesCol = Param("column holding values for each feature (key) that will be returned when queried",
                      "values", T.toString)
    leafSize = Param("max size of the leaves of the tree", 50, T.toInt)
    k = Param("number of matches to return", 5, T.toInt)


def _obj(values) -> np.ndarray:
    arr = np.empty(len(values), dtype=object)
    for i, v in enumerate(values):
        arr[i] = v
    return arr


class KNNModel(Model, _KNNParams):
    ballTree = Param("the ballTree model used for performing queries", None, complex=True)

    def _transform(self, df):
        bt: BallTree = self.getBallTree()
        Q = as_matrix(df[self.getFeaturesCol()])
        k = self.getK()
        res = []
        if _use_gpu() and len(Q):
            vals, idx = _device_mips(Q, bt.keys, k)
            for r in range(len(Q)):
                res.append([{"value": bt.values[int(i)], "distance": float(v)} for v, i in zip(vals[r], idx[r])])
        else:
            for q in Q:
                res.append([{"value": bt.values[m.index], "distance": m.distance}
                            for m in bt.findMaximumInnerProducts(q, k)])
        return df.withColumn(self.getOutputCol(), _obj(res))


class KNN(Estimator, _KNNParams):
    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(outputCol=self.uid + "_output")

    def _fit(self, df):
        bt = BallTree(as_matrix(df[self.getFeaturesCol()]), df[self.getValuesCol()].tolist(), self.getLeafSize())
        m = KNNModel(featuresCol=self.getFeaturesCol(), valuesCol=self.getValuesCol(), outputCol=self.getOutputCol(),
                     k=self.getK(), leafSize=self.getLeafSize())
        return m.set("ballTree", bt)


class ConditionalKNNModel(Model, _KNNParams, HasLabelCol):
    conditionerCol = Param("column holding identifiers for features that will be returned when queried",
                           "conditioner", T.toString)
    ballTree = Param("the ballTree model used for performing queries", None, complex=True)

    def _transform(self, df):
        bt: ConditionalBallTree = self.getBallTree()
        Q = as_matrix(df[self.getFeaturesCol()])
        conds = [set(c) for c in df[self.getConditionerCol()].tolist()]
        k = self.getK()
        res = []
        if _use_gpu() and len(Q):
            labels = np.asarray(bt.labels, dtype=object)
            mask = np.stack([np.asarray([l in c for l in labels]) for c in conds])
            vals, idx = _device_mips(Q, bt.keys, k, mask)
            for r in range(len(Q)):
                res.append([{"value": bt.values[int(i)], "distance": float(v), "label": bt.labels[int(i)]}
                            for v, i in zip(vals[r], idx[r]) if np.isfinite(v)])
        else:
            for q, c in zip(Q, conds):
                res.append([{"value": bt.values[m.index], "distance": m.distance, "label": bt.labels[m.index]}
                            for m in bt.findMaximumInnerProducts(q, c, k)])
        return df.withColumn(self.getOutputCol(), _obj(res))


class ConditionalKNN(Estimator, _KNNParams, HasLabelCol):
    conditionerCol = Param("column holding identifiers for features that will be returned when queried",
                           "conditioner", T.toString)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(outputCol=self.uid + "_output")

    def _fit(self, df):
        bt = ConditionalBallTree(as_matrix(df[self.getFeaturesCol()]), df[self.getValuesCol()].tolist(),
                                 df[self.getLabelCol()].tolist(), self.getLeafSize())
        m = ConditionalKNNModel(featuresCol=self.getFeaturesCol(), valuesCol=self.getValuesCol(),
                                outputCol=self.getOutputCol(), k=self.getK(), leafSize=self.getLeafSize(),
                                labelCol=self.getLabelCol(), conditionerCol=self.getConditionerCol())
        return m.set("ballTree", bt)


__all__ = ["BallTree", "ConditionalBallTree", "BestMatch", "KNN", "KNNModel", "ConditionalKNN",
           "ConditionalKNNModel"]
