"""Anomaly Detector transformers (reference: cognitive/.../services/anomaly/
AnomalyDetection.scala:26-290, MultivariateAnomalyDetection.scala).

``SimpleDetectAnomalies`` groups rows into one series per ``groupbyCol``
value, sorts each series by timestamp, detects over the whole series in one
request and explodes the per-point verdicts back onto the original rows."""
from __future__ import annotations

import json
from typing import Any, Dict, List

import numpy as np

import time

from ..core.dataframe import DataFrame
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Estimator, Model
from .base import CognitiveServicesBase, HasAsyncReply, HasServiceParams, ServiceParam, ServiceValue


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


# ---------------------------------------------------------------- multivariate (v1.1, OneTable schema)
def iso_instant(v) -> str:
    """ISO-8601 instant string (reference convertTimeFormat: DateTimeFormatter.ISO_INSTANT), UTC 'Z' form."""
    import datetime as _dt

    if isinstance(v, np.datetime64):
        v = v.astype("datetime64[us]").item()
    if hasattr(v, "to_pydatetime"):
        v = v.to_pydatetime()
    if isinstance(v, str):
        t = v.strip().replace("Z", "+00:00")
        try:
            v = _dt.datetime.fromisoformat(t)
        except ValueError as e:
            raise ValueError(f"Timestamp {v!r} is not in ISO-8601 instant form, e.g. 2021-01-01T00:00:00Z") from e
    if not isinstance(v, _dt.datetime):
        raise ValueError(f"cannot read {v!r} as a timestamp")
    if v.tzinfo is not None:
        v = v.astimezone(_dt.timezone.utc).replace(tzinfo=None)
    s = v.strftime("%Y-%m-%dT%H:%M:%S")
    if v.microsecond:
        s += ("%.6f" % (v.microsecond / 1e6))[1:].rstrip("0")
    return s + "Z"


class _MADParams(HasServiceParams, HasAsyncReply):
    """Shared params and HTTP helpers of the multivariate estimator / model
    (reference: MultivariateAnomalyDetection.scala:60-420, MADUtils + MADBase)."""

    url = Param("Url of the service", None, T.toString)
    subscriptionKey = ServiceParam("the API key to use")
    AADToken = ServiceParam("AAD Token used for authentication")
    CustomAuthHeader = ServiceParam("A Custom Value for Authorization Header")
    timestampCol = Param("Timestamp column name", "timestamp", T.toString)
    inputCols = Param("The names of the input columns", None, T.toListString)
    startTime = Param("A required field, start time of data to be used for detection/generating multivariate "
                      "anomaly detection model, should be date-time.", None, iso_instant)
    endTime = Param("A required field, end time of data to be used for detection/generating multivariate anomaly "
                    "detection model, should be date-time.", None, iso_instant)
    intermediateSaveDir = Param("Directory (any fsspec URL; wasbs:// and abfss:// map to blob https URLs) where "
                                "the intermediate CSV is written for the service to read", None, T.toString)
    outputCol = Param("The name of the output column", "result", T.toString)
    errorCol = Param("column to hold http errors", "error", T.toString)
    timeout = Param("number of seconds to wait before closing the connection", 60.0, T.toFloat)

    url_path = ""
    host_template = "https://{location}.api.cognitive.microsoft.{domain}/"

    def setLocation(self, location: str):  # noqa: N802
        from .base import location_domain

        return self.setUrl(self.host_template.format(location=location, domain=location_domain(location))
                           + self.url_path)

    def _mad_headers(self, content_type="application/json") -> dict:
        vals = self._resolve({})
        return CognitiveServicesBase._headers(self, vals, content_type)

    _headers = CognitiveServicesBase._headers
    subscription_key_header = CognitiveServicesBase.subscription_key_header

    def _mad_send(self, session, method: str, url: str, body=None):
        import requests

        h = self._mad_headers()
        for attempt, wait in enumerate((0.0, 0.1, 0.5, 1.0)):
            time.sleep(wait)
            r = session.request(method, url, headers=h, data=None if body is None else json.dumps(body).encode(),
                                timeout=self.getTimeout())
            if r.status_code != 429 and r.status_code < 500:
                break
        if r.status_code >= 400:
            raise requests.HTTPError(f"{type(self).__name__}: {method} {url} -> {r.status_code} {r.text[:500]}")
        return r

    def _blob_source(self, path: str) -> str:
        from urllib.parse import urlparse

        u = urlparse(path)
        if u.scheme in ("wasb", "wasbs", "abfs", "abfss"):
            container, _, host = u.netloc.partition("@")
            account = host.split(".")[0]
            return f"https://{account}.blob.core.windows.net/{container}/{u.path.lstrip('/')}"
        return path

    def _upload(self, df) -> str:
        """Write timestamp + input columns (timestamps as ISO instants, sorted) as one CSV under
        intermediateSaveDir/<uid>.csv; returns the data-source URL the service reads."""
        import fsspec

        d = self.getIntermediateSaveDir()
        if not d:
            raise ValueError(f"{type(self).__name__}: intermediateSaveDir is not set")
        cols = [self.getTimestampCol()] + list(self.getInputCols() or [])
        ts = [iso_instant(t) for t in df[cols[0]].tolist()]
        order = sorted(range(len(ts)), key=lambda i: ts[i])
        data = {c: df[c].tolist() for c in cols[1:]}
        path = d.rstrip("/") + f"/{self.uid}.csv"
        with fsspec.open(path, "w") as fh:
            fh.write(",".join(cols) + "\n")
            for i in order:
                fh.write(",".join([ts[i]] + [repr(float(data[c][i])) for c in cols[1:]]) + "\n")
        return self._blob_source(path)

    def _poll_json(self, session, url: str, status_of, done=("ready", "failed")) -> dict:
        for _ in range(self.getMaxPollingRetries() + 1):
            js = self._mad_send(session, "GET", url).json()
            st = str(status_of(js) or "").lower()
            if st in done:
                return js
            if st not in ("created", "running", ""):
                raise RuntimeError(f"Received unknown status code: {st}")
            time.sleep(self.getPollingDelay() / 1000.0)
        raise TimeoutError(f"{type(self).__name__}: {url} did not complete within {self.getMaxPollingRetries()} tries")

    def _models_url(self) -> str:
        u = self.getUrl()
        if not u:
            raise ValueError(f"{type(self).__name__}: url is not set (setUrl / setLocation)")
        return u if u.endswith("/") else u + "/"

    def _check_model(self, session, model_id: str) -> dict:
        js = self._mad_send(session, "GET", self._models_url() + model_id).json()
        info = js.get("modelInfo", {})
        st = str(info.get("status", "")).lower()
        if st == "failed":
            raise RuntimeError(f"Caught errors during fitting: {json.dumps(info.get('errors'))}")
        if st in ("created", "running"):
            raise RuntimeError(f"model {model_id} is not ready yet")
        return js


class SimpleFitMultivariateAnomaly(Estimator, _MADParams):
    """Estimator: uploads the timestamp + inputCols table, trains a multivariate model and polls until it is
    ready; returns a :class:`SimpleDetectMultivariateAnomaly` bound to the model id
    (reference: MultivariateAnomalyDetection.scala:421-540)."""

    url_path = "anomalydetector/v1.1/multivariate/models"
    slidingWindow = Param("An optional field, indicates how many history points will be used to determine the "
                          "anomaly score of one subsequent point.", 300, T.toInt)
    alignMode = Param("An optional field, indicates how we align different variables into the same time-range "
                      "(Inner | Outer)", "Outer", T.toString)
    fillNAMethod = Param("An optional field, indicates how missed values will be filled (Previous | Subsequent | "
                         "Linear | Zero | Fixed)", "Linear", T.toString)
    paddingValue = Param("optional field, is only useful if FillNAMethod is set to Fixed.", None, T.toInt)
    displayName = Param("optional field, name of the model", None, T.toString)

    def setSlidingWindow(self, v):  # noqa: N802
        if not 28 <= int(v) <= 2880:
            raise ValueError("slidingWindow must be between 28 and 2880 (both inclusive).")
        return self.set("slidingWindow", v)

    def setAlignMode(self, v):  # noqa: N802
        if str(v).lower() not in ("inner", "outer"):
            raise ValueError("alignMode must be either `inner` or `outer`.")
        return self.set("alignMode", v)

    def setFillNAMethod(self, v):  # noqa: N802
        if str(v).lower() not in ("previous", "subsequent", "linear", "zero", "fixed"):
            raise ValueError("fillNAMethod must be one of [Previous, Subsequent, Linear, Zero, Fixed].")
        return self.set("fillNAMethod", v)

    def _fit(self, df):
        import requests

        session = requests.Session()
        align = {"alignMode": self.getAlignMode(), "fillNAMethod": self.getFillNAMethod()}
        if self.getPaddingValue() is not None:
            align["paddingValue"] = self.getPaddingValue()
        body = {"dataSource": self._upload(df), "dataSchema": "OneTable", "startTime": self.getStartTime(),
                "endTime": self.getEndTime(), "slidingWindow": self.getSlidingWindow(), "alignPolicy": align}
        if self.getDisplayName():
            body["displayName"] = self.getDisplayName()
        r = self._mad_send(session, "POST", self.getUrl(), body)
        loc = r.headers.get("Location") or r.headers.get("location")
        js = r.json() if r.content else {}
        if loc:
            js = self._poll_json(session, loc, lambda j: (j.get("modelInfo") or {}).get("status"))
        info = js.get("modelInfo", {})
        if str(info.get("status", "")).lower() == "failed":
            raise RuntimeError(f"Caught errors during fitting: {json.dumps(info.get('errors'))}")
        model = SimpleDetectMultivariateAnomaly(modelId=js["modelId"], url=self._models_url() + "",
                                                timestampCol=self.getTimestampCol(), inputCols=self.getInputCols(),
                                                intermediateSaveDir=self.getIntermediateSaveDir(),
                                                outputCol=self.getOutputCol(), errorCol=self.getErrorCol(),
                                                pollingDelay=self.getPollingDelay(),
                                                maxPollingRetries=self.getMaxPollingRetries())
        for n in ("subscriptionKey", "AADToken", "CustomAuthHeader"):
            if self.isSet(n):
                model.set(n, self.getOrDefault(n))
        if info.get("diagnosticsInfo") is not None:
            model.setDiagnosticsInfo(info["diagnosticsInfo"])
        return model


class SimpleDetectMultivariateAnomaly(Model, _MADParams):
    """Batch inference with a trained model: uploads the rows, posts ``<modelId>:detect-batch``, polls the
    result and joins the per-timestamp verdicts back onto the rows sorted by time (``outputCol`` = the
    result's ``value`` record, ``isAnomaly``, ``errorCol``) (reference: MultivariateAnomalyDetection.scala:
    578-660)."""

    url_path = "anomalydetector/v1.1/multivariate/models/"
    modelId = Param("Format - uuid. Model identifier.", None, T.toString)
    diagnosticsInfo = Param("diagnosticsInfo for training a multivariate anomaly detection model", None,
                            T.identity)
    topContributorCount = Param("This is a number that you want to return the top contributors.", 10, T.toInt)

    def _transform(self, df):
        import requests

        session = requests.Session()
        self._check_model(session, self.getModelId())
        ts = [iso_instant(t) for t in df[self.getTimestampCol()].tolist()]
        body = {"dataSource": self._upload(df), "topContributorCount": self.getTopContributorCount(),
                "startTime": self.getStartTime() or min(ts), "endTime": self.getEndTime() or max(ts)}
        r = self._mad_send(session, "POST", self._models_url() + f"{self.getModelId()}:detect-batch", body)
        js = r.json() if r.content else {}
        result_id = js.get("resultId")
        if result_id is None:
            raise RuntimeError(f"detect-batch returned no resultId: {js}")
        base = self._models_url().rstrip("/").rsplit("/", 1)[0] + "/detect-batch/"
        res = self._poll_json(session, base + result_id, lambda j: (j.get("summary") or {}).get("status"))
        summ = res.get("summary", {})
        if str(summ.get("status", "")).lower() == "failed":
            raise RuntimeError(f"Failure during inference: {json.dumps(summ.get('errors'))}")
        by_ts = {}
        for rec in res.get("results", []):
            by_ts[iso_instant(rec["timestamp"])] = rec
        order = sorted(range(len(ts)), key=lambda i: ts[i])
        out = df._take_rows(np.asarray(order, dtype=np.int64))
        outs = np.empty(len(order), dtype=object)
        errs = np.empty(len(order), dtype=object)
        flags = np.empty(len(order), dtype=object)
        for j, i in enumerate(order):
            rec = by_ts.get(ts[i])
            val = None if rec is None else rec.get("value")
            outs[j] = val
            errs[j] = None if rec is None else rec.get("errors")
            flags[j] = None if val is None else val.get("isAnomaly")
        return out.withColumn(self.getOutputCol(), outs).withColumn("isAnomaly", flags) \
            .withColumn(self.getErrorCol(), errs)


class DetectLastMultivariateAnomaly(CognitiveServicesBase):
    """Synchronous detection of the last point of each sliding window: rows sorted by time, each row sends
    the previous ``batchSize`` rows (itself included) of every input variable to ``<modelId>:detect-last``;
    adds ``isAnomaly`` and ``DetectDataTimestamp`` from the first result (reference:
    MultivariateAnomalyDetection.scala:664-770)."""

    url_path = "anomalydetector/v1.1/multivariate/models/"
    modelId = Param("Format - uuid. Model identifier.", None, T.toString)
    inputVariablesCols = Param("The names of the input variables columns", None, T.toListString)
    timestampCol = Param("Timestamp column name", "timestamp", T.toString)
    topContributorCount = Param("This is a number that you want to return the top contributors.", 10, T.toInt)
    batchSize = Param("The size of the sliding window (rows sent with each request)", 300, T.toInt)
    window = ServiceParam("the rows of the sliding window ending at this row", required=True)

    def _base_url(self, vals):
        u = self.getUrl()
        if not u:
            raise ValueError(f"{type(self).__name__}: url is not set (setUrl / setLocation)")
        return (u if u.endswith("/") else u + "/") + f"{self.getModelId()}:detect-last"

    def _entity(self, vals):
        w = vals["window"]
        variables = [{"variable": v, "timestamps": w["timestamps"], "values": w[v]}
                     for v in self.getInputVariablesCols()]
        return json.dumps({"variables": variables, "topContributorCount": self.getTopContributorCount()}) \
            .encode("utf-8"), "application/json"

    def _transform(self, df):
        import requests

        probe = _MADParams()
        probe.setUrl(self.getUrl())
        for n in ("subscriptionKey", "AADToken", "CustomAuthHeader"):
            if self.isSet(n):
                probe.set(n, self.getOrDefault(n))
        probe._check_model(requests.Session(), self.getModelId())
        ts = [iso_instant(t) for t in df[self.getTimestampCol()].tolist()]
        order = sorted(range(len(ts)), key=lambda i: ts[i])
        sdf = df._take_rows(np.asarray(order, dtype=np.int64))
        cols = {v: [float(x) for x in sdf[v].tolist()] for v in self.getInputVariablesCols()}
        sts = [ts[i] for i in order]
        bs = self.getBatchSize()
        win = np.empty(len(order), dtype=object)
        for j in range(len(order)):
            lo = max(0, j - bs)  # rowsBetween(-batchSize, 0)
            rec = {"timestamps": sts[lo:j + 1]}
            for v, vals in cols.items():
                rec[v] = vals[lo:j + 1]
            win[j] = rec
        inner = self.copy()
        inner.set("window", ServiceValue(kind="col", value="__window"))
        res = CognitiveServicesBase._transform(inner, sdf.withColumn("__window", win))
        outs = res[self.getOutputCol()].tolist()
        flags = np.empty(len(outs), dtype=object)
        when = np.empty(len(outs), dtype=object)
        for j, o in enumerate(outs):
            r0 = (o or {}).get("results") or [None]
            flags[j] = None if r0[0] is None else (r0[0].get("value") or {}).get("isAnomaly")
            when[j] = None if r0[0] is None else r0[0].get("timestamp")
        return res.drop("__window").withColumn("isAnomaly", flags).withColumn("DetectDataTimestamp", when)


__all__ = ["DetectLastAnomaly", "DetectAnomalies", "SimpleDetectAnomalies", "SimpleFitMultivariateAnomaly",
           "SimpleDetectMultivariateAnomaly", "DetectLastMultivariateAnomaly", "DetectMultivariateAnomaly",
           "explode_entire", "iso_instant"]
