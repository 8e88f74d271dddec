"""SLIC-style superpixels (reference: core/.../image/Superpixel.scala:44-340,
SuperpixelTransformer.scala): grid seeds every ``cellSize`` pixels, k-means in
(color, position) space restricted to a 2S window, ``modifier`` weighs colour
against spatial distance."""
from __future__ import annotations

from typing import List

import numpy as np

from ..core.contracts import HasInputCol, HasOutputCol
from ..core.dataframe import DataFrame
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Transformer


def slic(img: np.ndarray, cell_size: float = 16.0, modifier: float = 130.0, iters: int = 5) -> np.ndarray:
    """HWC uint8 -> int32 label map."""
    a = img.astype(np.float64)
    if a.ndim == 2:
        a = a[:, :, None]
    h, w, _ = a.shape
    S = max(1, int(round(cell_size)))
    ys = np.arange(S // 2, h, S)
    xs = np.arange(S // 2, w, S)
    if len(ys) == 0:
        ys = np.array([h // 2])
    if len(xs) == 0:
        xs = np.array([w // 2])
    centers = [(float(y), float(x), a[y, x].copy()) for y in ys for x in xs]
    yy, xx = np.mgrid[0:h, 0:w]
    labels = np.zeros((h, w), np.int32)
    for _ in range(iters):
        dist = np.full((h, w), np.inf)
        for k, (cy, cx, cc) in enumerate(centers):
            y0, y1 = max(0, int(cy) - S), min(h, int(cy) + S + 1)
            x0, x1 = max(0, int(cx) - S), min(w, int(cx) + S + 1)
            patch = a[y0:y1, x0:x1]
            dc = ((patch - cc) ** 2).sum(-1)
            ds = (yy[y0:y1, x0:x1] - cy) ** 2 + (xx[y0:y1, x0:x1] - cx) ** 2
            d = dc / max(modifier, 1e-9) ** 2 + ds / S ** 2
            sub = dist[y0:y1, x0:x1]
            m = d < sub
            sub[m] = d[m]
            labels[y0:y1, x0:x1][m] = k
        new = []
        for k in range(len(centers)):
            m = labels == k
            if m.any():
                new.append((float(yy[m].mean()), float(xx[m].mean()), a[m].mean(0)))
            else:
                new.append(centers[k])
        centers = new
    # compact label ids
    _, inv = np.unique(labels, return_inverse=True)
    return inv.reshape(h, w).astype(np.int32)


def clusters_of(labels: np.ndarray) -> List[List[tuple]]:
    out = []
    for k in range(int(labels.max()) + 1):
        ys, xs = np.nonzero(labels == k)
        out.append(list(zip(xs.tolist(), ys.tolist())))
    return out


def censor(img: np.ndarray, labels: np.ndarray, state: np.ndarray) -> np.ndarray:
    """Keep superpixels whose state is 1, black out the rest."""
    keep = np.asarray(state, bool)[labels]
    out = img.copy()
    out[~keep] = 0
    return out


class SuperpixelTransformer(Transformer, HasInputCol, HasOutputCol):
    cellSize = Param("Number that controls the size of the superpixels", 16.0, T.toFloat)
    modifier = Param("Controls the trade-off spatial and color distance", 130.0, T.toFloat)

    def _transform(self, df):
        from ..image.schema import to_array

        out = np.empty(df.count(), dtype=object)
        for i, v in enumerate(df[self.getInputCol()].tolist()):
            a = to_array(v)
            out[i] = None if a is None else {"clusters": clusters_of(slic(a, self.getCellSize(), self.getModifier()))}
        return df.withColumn(self.getOutputCol(), out)
