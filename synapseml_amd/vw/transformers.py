"""Bandit-log plumbing transformers.

* ``VowpalWabbitDSJsonTransformer`` — parses decision-service JSON lines
  (reference: vw/.../VowpalWabbitDSJsonTransformer.scala:18-110) into the
  header columns ``EventId``, ``rewards`` (a dict of reward aliases →
  float, default ``{"reward": "_label_cost"}``), ``probLog``
  (``_label_probability``) and ``chosenActionIndex`` (``_labelIndex``), plus
  the parsed ``json`` column.
* ``VowpalWabbitCSETransformer`` — counterfactual statistics estimation
  (VowpalWabbitCSETransformer.scala:18-222): importance-weight statistics
  and, per reward, min/max reward, SNIPS, IPS, Cressie-Read and both
  Cressie-Read intervals, optionally stratified by columns.
* ``VectorZipper`` — zips input columns into one array column
  (VectorZipper.scala).
"""
from __future__ import annotations

import json
from typing import Dict, List

import numpy as np

from ..core.contracts import HasInputCols, HasOutputCol
from ..core.dataframe import DataFrame
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Transformer
from .policyeval import CressieRead, CressieReadInterval, Ips, Snips

EventIdColName = "EventId"
JsonColName = "json"
ProbabilityLoggedColName = "probLog"
ProbabilityPredictedColName = "probPred"
ChosenActionIndexColName = "chosenActionIndex"
RewardsColName = "rewards"
LabelProbability = "_label_probability"
LabelIndex = "_labelIndex"
HeaderColNames = [EventIdColName, RewardsColName, ProbabilityLoggedColName, ChosenActionIndexColName]


class VowpalWabbitDSJsonTransformer(Transformer):
    dsJsonColumn = Param("Column containing ds-json. defaults to \"value\".", "value", T.toString)
    rewards = Param("Extract bandit reward(s) from DS json. Defaults to _label_cost.",
                    {"reward": "_label_cost"}, T.identity)

    def _transform(self, df: DataFrame) -> DataFrame:
        col = self.getDsJsonColumn()
        rewards: Dict[str, str] = dict(self.getRewards())
        n = df.count()
        parsed = np.empty(n, dtype=object)
        eid = np.empty(n, dtype=object)
        rew = np.empty(n, dtype=object)
        prob = np.zeros(n, dtype=np.float32)
        chosen = np.zeros(n, dtype=np.int32)
        for i, line in enumerate(df[col].tolist()):
            j = json.loads(line) if isinstance(line, (str, bytes)) else dict(line)
            parsed[i] = j
            eid[i] = j.get(EventIdColName)
            rew[i] = {alias: (float(j[key]) if j.get(key) is not None else None) for alias, key in rewards.items()}
            prob[i] = float(j.get(LabelProbability, np.nan))
            chosen[i] = int(j.get(LabelIndex, -1))
        return (df.withColumn(JsonColName, parsed).withColumn(EventIdColName, eid)
                .withColumn(RewardsColName, rew).withColumn(ProbabilityLoggedColName, prob)
                .withColumn(ChosenActionIndexColName, chosen))


def _top_action(pred) -> int:
    """First element's action of a VW action-probability list."""
    if pred is None or len(pred) == 0:
        return -1
    first = pred[0]
    if isinstance(first, dict):
        return int(first["action"])
    if isinstance(first, (tuple, list)):
        return int(first[0])
    return int(np.argmax(np.asarray(pred, dtype=np.float64)))


class VowpalWabbitCSETransformer(Transformer):
    minImportanceWeight = Param("Clip importance weight at this lower bound. Defaults to 0.", 0.0, T.toFloat)
    maxImportanceWeight = Param("Clip importance weight at this upper bound. Defaults to 100.", 100.0, T.toFloat)
    metricsStratificationCols = Param("Optional list of column names to stratify rewards by.", [], T.toListString)

    def _transform(self, df: DataFrame) -> DataFrame:
        n = df.count()
        chosen = np.asarray(df[ChosenActionIndexColName], np.int64)
        probpred = np.asarray([1.0 if _top_action(p) == c else 0.0 for p, c in zip(df["predictions"].tolist(), chosen)],
                              dtype=np.float64)
        problog = np.asarray(df[ProbabilityLoggedColName], np.float64)
        w = probpred / problog
        rewards = df[RewardsColName].tolist()
        names = list(rewards[0].keys()) if n else []
        rcols = {k: np.asarray([float(r[k]) if r[k] is not None else np.nan for r in rewards]) for k in names}
        # min/max reward are global (cross-joined before stratifying in the reference)
        mm = {k: (float(np.nanmin(v)), float(np.nanmax(v))) for k, v in rcols.items()}
        strat = list(self.getMetricsStratificationCols() or [])
        if strat:
            keys = list(zip(*[df[c].tolist() for c in strat]))
        else:
            keys = [()] * n
        groups: Dict[tuple, List[int]] = {}
        for i, k in enumerate(keys):
            groups.setdefault(k, []).append(i)
        wmin, wmax = self.getMinImportanceWeight(), self.getMaxImportanceWeight()
        out: Dict[str, list] = {c: [] for c in strat}
        gnames = ["exampleCount", "probPredNonZeroCount", "minimumImportanceWeight", "maximumImportanceWeight",
                  "averageImportanceWeight", "averageSquaredImportanceWeight",
                  "proportionOfMaximumImportanceWeight", "importance weight quantiles (0.25, 0.5, 0.75, 0.95)"]
        for g in gnames + names:
            out[g] = []
        for key, idx in groups.items():
            idx = np.asarray(idx)
            for c, v in zip(strat, key):
                out[c].append(v)
            wi = w[idx]
            out["exampleCount"].append(len(idx))
            out["probPredNonZeroCount"].append(int((probpred[idx] > 0).sum()))
            out["minimumImportanceWeight"].append(float(wi.min()))
            out["maximumImportanceWeight"].append(float(wi.max()))
            out["averageImportanceWeight"].append(float(wi.mean()))
            out["averageSquaredImportanceWeight"].append(float((wi * wi).mean()))
            out["proportionOfMaximumImportanceWeight"].append(float(wi.max() / len(idx)))
            out["importance weight quantiles (0.25, 0.5, 0.75, 0.95)"].append(
                [float(x) for x in np.quantile(wi, [0.25, 0.5, 0.75, 0.95])])
            sub = DataFrame({"probLog": problog[idx], "probPred": probpred[idx]})
            for k in names:
                s2 = sub.withColumn("reward", rcols[k][idx])
                rmin, rmax = mm[k]
                ci = CressieReadInterval(False)
                try:
                    interval = ci.evaluate(s2, wMin=wmin, wMax=wmax, rewardMin=rmin, rewardMax=rmax)
                except ValueError:
                    interval = None
                emp = CressieReadInterval(True).evaluate(s2, wMin=wmin, wMax=wmax, rewardMin=rmin, rewardMax=rmax)
                out[k].append({
                    "minReward": rmin, "maxReward": rmax,
                    "snips": Snips().evaluate(s2), "ips": Ips().evaluate(s2),
                    "cressieRead": CressieRead().evaluate(s2, wMin=wmin, wMax=wmax),
                    "cressieReadInterval": None if interval is None else
                    {"lower": interval.lower, "upper": interval.upper},
                    "cressieReadIntervalEmpirical": {"lower": emp.lower, "upper": emp.upper},
                })
        return DataFrame(out)


class VectorZipper(Transformer, HasInputCols, HasOutputCol):
    def _transform(self, df: DataFrame) -> DataFrame:
        cols = [df[c] for c in self.getInputCols()]
        n = df.count()
        out = np.empty(n, dtype=object)
        for i in range(n):
            out[i] = [c[i] for c in cols]
        return df.withColumn(self.getOutputCol(), out)
