"""Anomaly Detector transformers (reference: cognitive/.../services/anomaly/
AnomalyDetection.scala:26-290, MultivariateAnomalyDetection.scala).

``SimpleDetectAnomalies`` groups rows into one series per ``groupbyCol``
value, sorts each series by timestamp, detects over the whole series in one
request and explodes the per-point verdicts back onto the original rows."""
from __future__ import annotations

import json
from typing import Any, Dict, List

import numpy as np

from ..core.dataframe import DataFrame
from ..core.params import Param, TypeConverters as T
from .base import CognitiveServicesBase, HasAsyncReply, ServiceParam


class _AnomalyBase(CognitiveServicesBase):
    granularity = ServiceParam("Can only be one of yearly, monthly, weekly, daily, hourly or minutely.")
    maxAnomalyRatio = ServiceParam("Optional argument, advanced model parameter, max anomaly ratio")
    sensitivity = ServiceParam("Optional argument, advanced model parameter, between 0-99")
    customInterval = ServiceParam("Custom Interval is used to set non-standard time interval")
    period = ServiceParam("Optional argument, periodic value of a time series.")
    imputeMode = ServiceParam("Optional argument, impute mode of a time series.")
    imputeFixedValue = ServiceParam("Optional argument, fixed value to use in imputeMode=fixed")
    series = ServiceParam("Time series data points [{timestamp, value}] (at least 12).", required=True)

    def _entity(self, vals):
        body = self._body_params(vals, exclude=("series",))
        body["series"] = [{"timestamp": p["timestamp"], "value": float(p["value"])} if isinstance(p, dict)
                          else {"timestamp": p[0], "value": float(p[1])} for p in vals["series"]]
        return json.dumps(body).encode("utf-8"), "application/json"


class DetectLastAnomaly(_AnomalyBase):
    url_path = "/anomalydetector/v1.1-preview.1/timeseries/last/detect"


class DetectAnomalies(_AnomalyBase):
    url_path = "/anomalydetector/v1.1-preview.1/timeseries/entire/detect"


_PER_POINT = ("isAnomaly", "isPositiveAnomaly", "isNegativeAnomaly", "expectedValues", "upperMargins",
              "lowerMargins", "severity")


def explode_entire(resp: Dict[str, Any], count: int) -> List[Dict[str, Any]]:
    """Entire-series response -> one single-point record per input point."""
    if not isinstance(resp, dict):
        return [None] * count
    out = []
    for i in range(count):
        rec = {}
        for k in _PER_POINT:
            if k in resp and resp[k] is not None and i < len(resp[k]):
                rec[k[:-1] if k.endswith("Values") or k.endswith("Margins") else k] = resp[k][i]
        rec["period"] = resp.get("period")
        out.append(rec)
    return out


class SimpleDetectAnomalies(_AnomalyBase):
    url_path = "/anomalydetector/v1.1-preview.1/timeseries/entire/detect"
    timestampCol = Param("column representing the time of the series", "timestamp", T.toString)
    valueCol = Param("column representing the value of the series", "value", T.toString)
    groupbyCol = Param("column that groups the series", None, T.toString)

    def _transform(self, df):
        ts = df[self.getTimestampCol()].tolist()
        vs = df[self.getValueCol()].tolist()
        gcol = self.getGroupbyCol()
        groups = df[gcol].tolist() if gcol else [0] * df.count()
        order: Dict[Any, List[int]] = {}
        for i, g in enumerate(groups):
            order.setdefault(g, []).append(i)
        keys = list(order)
        series, rows_of = [], []
        for g in keys:
            idx = sorted(order[g], key=lambda i: str(ts[i]))
            rows_of.append(idx)
            series.append([{"timestamp": str(ts[i]), "value": float(vs[i])} for i in idx])
        inner = self.copy()
        inner.set("series", {"kind": "col", "value": "__series"})
        scol = np.empty(len(series), dtype=object)
        for i, s in enumerate(series):
            scol[i] = s
        res = CognitiveServicesBase._transform(inner, DataFrame({"__series": scol}))
        outs = np.empty(df.count(), dtype=object)
        errs = np.empty(df.count(), dtype=object)
        for gi, idx in enumerate(rows_of):
            recs = explode_entire(res[self.getOutputCol()][gi], len(idx))
            for j, i in enumerate(idx):
                outs[i] = recs[j]
                errs[i] = res[self.getErrorCol()][gi]
        return df.withColumn(self.getOutputCol(), outs).withColumn(self.getErrorCol(), errs)


class SimpleFitMultivariateAnomaly(CognitiveServicesBase, HasAsyncReply):
    """Train a multivariate model from data already uploaded to storage (``source`` URL)."""

    url_path = "/anomalydetector/v1.1/multivariate/models"
    source = ServiceParam("The blob link to the input data (zip or container)", required=True)
    startTime = ServiceParam("A required field, start time of data to be used for training", required=True)
    endTime = ServiceParam("A required field, end time of data to be used for training", required=True)
    slidingWindow = ServiceParam("An optional field, indicates how many history points will be used")
    alignMode = ServiceParam("An optional field, indicates how we align different variables (Inner|Outer)")
    fillNAMethod = ServiceParam("An optional field, indicates how missed values will be filled")
    paddingValue = ServiceParam("optional field, only be useful if FillNAMethod is set to Fixed")
    displayName = ServiceParam("optional field, name of the model")

    def _entity(self, vals):
        body = {"dataSource": vals["source"], "startTime": vals["startTime"], "endTime": vals["endTime"]}
        for k in ("slidingWindow", "displayName"):
            if k in vals:
                body[k] = vals[k]
        align = {k: vals[k] for k in ("alignMode", "fillNAMethod", "paddingValue") if k in vals}
        if align:
            body["alignPolicy"] = align
        return json.dumps(body).encode("utf-8"), "application/json"


class DetectMultivariateAnomaly(CognitiveServicesBase, HasAsyncReply):
    url_path = "/anomalydetector/v1.1/multivariate/models/"
    modelId = ServiceParam("Format - uuid. Model identifier.", required=True)
    source = ServiceParam("The blob link to the input data", required=True)
    startTime = ServiceParam("start time of data to be used for detection", required=True)
    endTime = ServiceParam("end time of data to be used for detection", required=True)
    topContributorCount = ServiceParam("number of top contributors for each anomaly")

    def _base_url(self, vals):
        return self.getUrl().rstrip("/") + "/" + vals["modelId"] + ":detect-batch"

    def _entity(self, vals):
        body = {"dataSource": vals["source"], "startTime": vals["startTime"], "endTime": vals["endTime"],
                "topContributorCount": vals.get("topContributorCount", 10)}
        return json.dumps(body).encode("utf-8"), "application/json"


__all__ = ["DetectLastAnomaly", "DetectAnomalies", "SimpleDetectAnomalies", "SimpleFitMultivariateAnomaly",
           "DetectMultivariateAnomaly", "explode_entire"]
