"""Off-policy estimators as mergeable aggregators (reference:
vw/.../policyeval/{Ips,Snips,CressieRead,CressieReadInterval}.scala).
Each has zero/reduce/merge/finish like a Spark Aggregator, plus
``evaluate(df, ...)`` that reduces DataFrame columns (partition-wise, then
merged). Sums use Kahan summation (KahanSum.scala)."""
from __future__ import annotations

import math
from dataclasses import dataclass, field, replace
from typing import Optional

import numpy as np

from ..core.dataframe import DataFrame


class KahanSum:
    """Compensated sum (reference: vw/.../KahanSum.scala:16-68)."""

    __slots__ = ("sum", "c")

    def __init__(self, s: float = 0.0, c: float = 0.0):
        self.sum = float(s)
        self.c = float(c)

    def __add__(self, x):
        if isinstance(x, KahanSum):
            out = KahanSum(self.sum, self.c)
            out = out + x.sum
            out.c += x.c
            return out
        y = float(x) - self.c
        t = self.sum + y
        return KahanSum(t, (t - self.sum) - y)

    def toDouble(self) -> float:  # noqa: N802
        return self.sum - self.c

    def __float__(self) -> float:
        return self.toDouble()


def _ksum(a: np.ndarray) -> float:
    k = KahanSum()
    for v in np.asarray(a, dtype=np.float64).tolist():
        k = k + v
    return k.toDouble()


class Ips:
    def zero(self):
        return {"n": 0.0, "wr": 0.0}

    def reduce(self, acc, probLog, reward, probPred, count=1.0):  # noqa: N803
        w = probPred / probLog
        return {"n": acc["n"] + count, "wr": acc["wr"] + reward * w * count}

    def merge(self, a, b):
        return {"n": a["n"] + b["n"], "wr": a["wr"] + b["wr"]}

    def finish(self, acc) -> float:
        return -1.0 if acc["n"] == 0 else acc["wr"] / acc["n"]

    def evaluate(self, df: DataFrame, probLog="probLog", reward="reward", probPred="probPred", count=None) -> float:  # noqa: N803
        c = np.asarray(df[count], float) if count else np.ones(df.count())
        w = np.asarray(df[probPred], float) / np.asarray(df[probLog], float)
        return self.finish({"n": _ksum(c), "wr": _ksum(np.asarray(df[reward], float) * w * c)})


class Snips(Ips):
    def zero(self):
        return {"wn": 0.0, "wr": 0.0}

    def reduce(self, acc, probLog, reward, probPred, count=1.0):  # noqa: N803
        w = probPred / probLog
        return {"wn": acc["wn"] + w * count, "wr": acc["wr"] + reward * w * count}

    def merge(self, a, b):
        return {"wn": a["wn"] + b["wn"], "wr": a["wr"] + b["wr"]}

    def finish(self, acc) -> float:
        return -1.0 if acc["wn"] == 0 else acc["wr"] / acc["wn"]

    def evaluate(self, df: DataFrame, probLog="probLog", reward="reward", probPred="probPred", count=None) -> float:  # noqa: N803
        c = np.asarray(df[count], float) if count else np.ones(df.count())
        w = np.asarray(df[probPred], float) / np.asarray(df[probLog], float)
        return self.finish({"wn": _ksum(w * c), "wr": _ksum(np.asarray(df[reward], float) * w * c)})


@dataclass
class CressieReadBuffer:
    wMin: float = 0.0
    wMax: float = 0.0
    n: float = 0.0
    sumw: float = 0.0
    sumwsq: float = 0.0
    sumwr: float = 0.0
    sumwrsqr: float = 0.0
    sumr: float = 0.0


class CressieRead:
    """Distributionally robust point estimate (CressieRead.scala)."""

    def zero(self) -> CressieReadBuffer:
        return CressieReadBuffer()

    def reduce(self, acc: CressieReadBuffer, probLog, reward, probPred, count, wMin, wMax):  # noqa: N803
        w = probPred / probLog
        cw = count * w
        cwsq = cw * cw
        return CressieReadBuffer(min(acc.wMin, wMin), max(acc.wMax, wMax), acc.n + count, acc.sumw + cw,
                                 acc.sumwsq + cwsq, acc.sumwr + cw * reward, acc.sumwrsqr + cwsq * reward,
                                 acc.sumr + count * reward)

    def merge(self, a: CressieReadBuffer, b: CressieReadBuffer) -> CressieReadBuffer:
        return CressieReadBuffer(min(a.wMin, b.wMin), max(a.wMax, b.wMax), a.n + b.n, a.sumw + b.sumw,
                                 a.sumwsq + b.sumwsq, a.sumwr + b.sumwr, a.sumwrsqr + b.sumwrsqr, a.sumr + b.sumr)

    def finish(self, acc: CressieReadBuffer) -> float:
        n = acc.n
        wfake = acc.wMax if acc.sumw < n else acc.wMin
        if math.isinf(wfake):
            gamma, beta = -(1 + n) / n, 0.0
        else:
            a = (wfake + acc.sumw) / (1 + n)
            b = (wfake * wfake + acc.sumwsq) / (1 + n)
            assert a * a <= b
            gamma, beta = (b - a) / (a * a - b), (1 - a) / (a * a - b)
        vhat = (-gamma * acc.sumwr - beta * acc.sumwrsqr) / (1 + n)
        missing = max(0.0, 1 - (-gamma * acc.sumw - beta * acc.sumwsq) / (1 + n))
        return vhat + missing * (acc.sumr / n)

    def evaluate(self, df: DataFrame, probLog="probLog", reward="reward", probPred="probPred", count=None,  # noqa: N803
                 wMin=0.0, wMax=float("inf")) -> float:  # noqa: N803
        acc = self.zero()
        c = df[count] if count else np.ones(df.count())
        for pl, r, pp, cc in zip(df[probLog], df[reward], df[probPred], c):
            acc = self.reduce(acc, float(pl), float(r), float(pp), float(cc), wMin, wMax)
        return self.finish(acc)


@dataclass
class BanditEstimator:
    lower: float
    upper: float


class CressieReadInterval:
    """Confidence interval (CressieReadInterval.scala). Note: the reference
    computes ``(1 / 2)`` with integer division (= 0) in its bound; that
    behaviour is kept for parity."""

    alpha = 0.05
    atol = 1e-9

    def __init__(self, empiricalBounds: bool = True):  # noqa: N803
        self.empirical = empiricalBounds

    def evaluate(self, df: DataFrame, probLog="probLog", reward="reward", probPred="probPred", count=None,  # noqa: N803
                 wMin=0.0, wMax=float("inf"), rewardMin=0.0, rewardMax=1.0) -> BanditEstimator:  # noqa: N803
        from scipy.stats import f as fdist

        pl = np.asarray(df[probLog], float)
        r = np.asarray(df[reward], float)
        pp = np.asarray(df[probPred], float)
        c = np.asarray(df[count], float) if count else np.ones(len(pl))
        if not self.empirical and ((r > rewardMax) | (r < rewardMin)).any():
            raise ValueError(f"Reward is out of bounds: {rewardMin} < reward < {rewardMax}")
        w = pp / pl
        cw = c * w
        cwsq = cw * cw
        n = c.sum()
        if n == 0:
            return BanditEstimator(-1, -1)
        rmin, rmax = (r.min(), r.max()) if self.empirical else (rewardMin, rewardMax)
        sumw, sumwsq, sumwr = cw.sum(), cwsq.sum(), (cw * r).sum()
        sumwsqr, sumwsqrsq = (cwsq * r).sum(), (cwsq * r * r).sum()
        unc = wMax if sumw < n else wMin
        if math.isinf(unc):
            ug = 1 + 1 / n
        else:
            ua = (unc + sumw) / (1 + n)
            ub = (unc * unc + sumwsq) / (1 + n)
            ug = (1 + n) * (ua - 1) * (ua - 1) / (ub - ua * ua)
        delta = 1 - fdist.ppf(self.alpha, 1, n)
        phi = (-ug - delta) / (2 * (1 + n))

        def inner(wfake, sign, rr):
            if math.isinf(wfake):
                return None
            barw = (wfake + sumw) / (1 + n)
            barwsq = (wfake * wfake + sumwsq) / (1 + n)
            barwr = sign * (wfake * rr + sumwr) / (1 + n)
            barwsqr = sign * (wfake * wfake * rr + sumwsqr) / (1 + n)
            barwsqrsq = (wfake * wfake * rr * rr + sumwsqrsq) / (1 + n)
            if barwsq <= barw * barw:
                return None
            x = barwr + ((1 - barw) * (barwsqr - barw * barwr) / (barwsq - barw * barw))
            y = (barwsqr - barw * barwr) ** 2 / (barwsq - barw * barw) - (barwsqrsq - barwr * barwr)
            z = phi  # reference: phi + (1 / 2) * ..., with integer (1 / 2) == 0
            if abs(y * x) < self.atol * self.atol:
                return x - math.sqrt(2) * self.atol
            if z <= 0 and y * z >= 0:
                return x - math.sqrt(2 * y * z)
            return None

        def bound(rr, sign):
            cands = [v for v in (inner(wMin, sign, rr), inner(wMax, sign, rr)) if v is not None]
            best = min(cands) if cands else (rmin if sign > 0 else -rmax)
            return min(rmax, max(rmin, sign * best))

        return BanditEstimator(bound(rmin, 1), bound(rmax, -1))
