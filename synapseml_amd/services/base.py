"""Cognitive-service transformers: shared machinery (reference:
cognitive/.../services/CognitiveServiceBase.scala:32-518, param/ServiceParam).

A ``ServiceParam`` holds either a scalar (``setX(v)``) or the name of a
column to read per row (``setXCol(c)``). Every service transformer turns a
row's resolved values into one HTTP request (URL + query params, auth
headers, entity), sends the partition's requests with ``concurrency`` worker
threads through the HTTP stack's retry handler, optionally polls an
``Operation-Location`` for asynchronous APIs, and writes the parsed JSON
reply to ``outputCol`` and HTTP failures to ``errorCol``. Rows whose required
values are null are skipped (null output, null error), like the reference's
``shouldSkip``.

Auth precedence follows ``addHeaders``: subscription key header, else
``Authorization: Bearer <AAD token>``, else a custom ``Authorization``
value."""
from __future__ import annotations

import json
import time
import uuid
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Dict, List, Optional, Tuple
from urllib.parse import quote, urlencode

import numpy as np

from ..core.contracts import HasOutputCol
from ..core.params import Param, Params, TypeConverters as T
from ..core.pipeline import Transformer
from ..io.http import ConcurrencyParams, _jsonable, _to_response, error_of, response_string, send_with_retries


def _obj(values) -> np.ndarray:
    arr = np.empty(len(values), dtype=object)
    for i, v in enumerate(values):
        arr[i] = v
    return arr


class ServiceValue(dict):
    """{"kind": "value"|"col", "value": ...}: JSON-serialisable param payload."""

    @staticmethod
    def of(v) -> "ServiceValue":
        if isinstance(v, ServiceValue):
            return v
        if isinstance(v, dict) and v.get("kind") in ("value", "col") and set(v) == {"kind", "value"}:
            return ServiceValue(v)
        return ServiceValue(kind="value", value=v)


class ServiceParam(Param):
    def __init__(self, doc: str = "", default: Any = None, required: bool = False, url_param: bool = False,
                 payload_name: Optional[str] = None, name: Optional[str] = None):
        super().__init__(doc, None if default is None else ServiceValue(kind="value", value=default),
                         ServiceValue.of, name=name)
        self.required = required
        self.url_param = url_param
        self.payload_name = payload_name

    @property
    def payload(self) -> str:
        return self.payload_name or self.name


def _cap(n: str) -> str:
    return n[0].upper() + n[1:]


class HasServiceParams(Params):
    """Adds ``setXCol``/``getXCol`` and scalar ``getX`` for every ServiceParam."""

    @classmethod
    def _params_hook(cls):
        for name, p in cls._params_decl.items():
            if not isinstance(p, ServiceParam):
                continue
            c = _cap(name)
            cur = getattr(cls, "get" + c, None)
            if cur is None or getattr(cur, "__qualname__", "").startswith("_make_getter"):
                setattr(cls, "get" + c, _scalar_getter(name))
            if not hasattr(cls, "set" + c + "Col"):
                setattr(cls, "set" + c + "Col", _col_setter(name))
            if not hasattr(cls, "get" + c + "Col"):
                setattr(cls, "get" + c + "Col", _col_getter(name))

    def service_params(self) -> List[ServiceParam]:
        return [p for p in self._params_decl.values() if isinstance(p, ServiceParam)]

    def _vector_cols(self) -> Dict[str, str]:
        out = {}
        for p in self.service_params():
            v = self.getOrDefault(p.name)
            if isinstance(v, dict) and v.get("kind") == "col":
                out[p.name] = v["value"]
        return out

    def _resolve(self, row: Dict[str, Any]) -> Dict[str, Any]:
        vals = {}
        for p in self.service_params():
            v = self.getOrDefault(p.name)
            if v is None:
                continue
            val = row.get(v["value"]) if v.get("kind") == "col" else v["value"]
            if isinstance(val, np.generic):
                val = val.item()
            if val is not None:
                vals[p.name] = val
        return vals


def _scalar_getter(name):
    def g(self):  # noqa: D401 - scalar value of a ServiceParam
        v = self.getOrDefault(name)
        if v is None:
            return None
        if v.get("kind") == "col":
            raise ValueError(f"{name} is bound to column {v['value']!r}; use get{_cap(name)}Col")
        return v["value"]

    return g


def _col_setter(name):
    def s(self, col: str):
        return self.set(name, ServiceValue(kind="col", value=col))

    return s


def _col_getter(name):
    def g(self):
        v = self.getOrDefault(name)
        return v["value"] if isinstance(v, dict) and v.get("kind") == "col" else None

    return g


def location_domain(location: str) -> str:
    if location in ("usgovarizona", "usgovvirginia"):
        return "us"
    if location in ("chinaeast2", "chinanorth"):
        return "cn"
    return "com"


class HasAsyncReply(Params):
    pollingDelay = Param("number of milliseconds to wait between polling", 300, T.toInt)
    maxPollingRetries = Param("number of times to poll", 1000, T.toInt)
    suppressMaxRetriesException = Param("set true to suppress the maxumimum retries exception and report in the "
                                        "error column", False, T.toBoolean)


class CognitiveServicesBase(Transformer, HasServiceParams, ConcurrencyParams, HasOutputCol):
    url = Param("Url of the service", None, T.toString)
    errorCol = Param("column to hold http errors", None, T.toString)
    subscriptionKey = ServiceParam("the API key to use")
    AADToken = ServiceParam("AAD Token used for authentication")
    CustomAuthHeader = ServiceParam("A Custom Value for Authorization Header")
    handler = Param("Which strategy to use when handling requests", None, complex=True)

    url_path = ""
    method = "POST"
    subscription_key_header = "Ocp-Apim-Subscription-Key"
    host_template = "https://{location}.api.cognitive.microsoft.{domain}/"
    retries_ms: Tuple[int, ...] = (100, 500, 1000)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(outputCol=self.uid + "_output", errorCol=self.uid + "_error")

    # --------------------------------------------------------------- endpoint helpers
    def setLocation(self, location: str):  # noqa: N802
        host = self.host_template.format(location=location, domain=location_domain(location))
        return self.setUrl(host + self.url_path.lstrip("/"))

    def setEndpoint(self, endpoint: str):  # noqa: N802
        return self.setUrl(endpoint.rstrip("/") + "/" + self.url_path.lstrip("/"))

    def setCustomServiceName(self, name: str):  # noqa: N802
        return self.setUrl(f"https://{name}.cognitiveservices.azure.com/" + self.url_path.lstrip("/"))

    def setDefaultAADToken(self, v: str):  # noqa: N802
        return self._setDefault(AADToken=ServiceValue(kind="value", value=v))

    # --------------------------------------------------------------- request construction
    def _required_names(self) -> List[str]:
        return [p.name for p in self.service_params() if p.required]

    def _should_skip(self, vals: Dict[str, Any]) -> bool:
        return any(vals.get(n) is None for n in self._required_names())

    def _query(self, vals: Dict[str, Any]) -> List[Tuple[str, str]]:
        q = []
        for p in self.service_params():
            if p.url_param and p.name in vals:
                v = vals[p.name]
                if isinstance(v, (list, tuple)):
                    q.extend((p.payload, str(x)) for x in v)
                else:
                    q.append((p.payload, str(v).lower() if isinstance(v, bool) else str(v)))
        return q

    def _base_url(self, vals: Dict[str, Any]) -> str:
        u = self.getUrl()
        if not u:
            raise ValueError(f"{type(self).__name__}: url is not set (setUrl / setLocation / setEndpoint)")
        return u

    def _url(self, vals: Dict[str, Any]) -> str:
        u = self._base_url(vals)
        q = self._query(vals)
        if q:
            u += ("&" if "?" in u else "?") + urlencode(q)
        return u

    def _headers(self, vals: Dict[str, Any], content_type: Optional[str]) -> Dict[str, str]:
        h = {}
        if vals.get("subscriptionKey"):
            h[self.subscription_key_header] = vals["subscriptionKey"]
        elif vals.get("AADToken"):
            h["Authorization"] = "Bearer " + vals["AADToken"]
            h["x-ms-workload-resource-moniker"] = str(uuid.uuid4())
        elif vals.get("CustomAuthHeader"):
            h["Authorization"] = vals["CustomAuthHeader"]
            h["x-ms-workload-resource-moniker"] = str(uuid.uuid4())
        if content_type:
            h["Content-Type"] = content_type
        return h

    def _body_params(self, vals: Dict[str, Any], exclude=()) -> Dict[str, Any]:
        skip = {"subscriptionKey", "AADToken", "CustomAuthHeader", *exclude}
        out = {}
        for p in self.service_params():
            if p.url_param or p.name in skip or p.name not in vals:
                continue
            out[p.payload] = _jsonable(vals[p.name])
        return out

    def _entity(self, vals: Dict[str, Any]) -> Tuple[Optional[bytes], Optional[str]]:
        """Request entity (bytes, content type). Default: JSON object of the body params."""
        return json.dumps(self._body_params(vals)).encode("utf-8"), "application/json"

    def _postprocess(self, parsed: Any, vals: Dict[str, Any]) -> Any:
        return parsed

    def _parse(self, resp: dict) -> Any:
        s = response_string(resp)
        if s is None or s == "":
            return None
        try:
            return json.loads(s)
        except ValueError:
            return s

    # --------------------------------------------------------------- execution
    def _modify_polling_url(self, url: str) -> str:
        """Hook for services whose polling URL needs extra query parameters (reference: modifyPollingURI)."""
        return url

    def _poll(self, session, resp, headers) -> dict:
        loc = None
        for h in resp["headers"]:
            if h["name"].lower() in ("operation-location", "location"):
                loc = h["value"]
        if not loc:
            return resp
        loc = self._modify_polling_url(loc)
        delay = self.getPollingDelay() / 1000.0
        auth = {k: v for k, v in headers.items() if k != "Content-Type"}
        for _ in range(self.getMaxPollingRetries()):
            r = session.get(loc, headers=auth, timeout=self.getTimeout())
            out = _to_response(r)
            if r.status_code != 200:
                return out
            try:
                status = str(json.loads(r.content or b"{}").get("status", "")).lower()
            except ValueError:
                return out
            if status in ("succeeded", "failed", "partiallycompleted", "partiallysucceeded", "completed",
                          "cancelled", "canceled"):
                return out
            time.sleep(delay)
        if self.getSuppressMaxRetriesException():
            return {"statusLine": {"statusCode": 504, "reasonPhrase": "max polling retries"}, "headers": [],
                    "entity": {"content": b"max polling retries exceeded"}}
        raise TimeoutError(f"{type(self).__name__}: polling {loc} exceeded {self.getMaxPollingRetries()} retries")

    def _send(self, session, req: Tuple[str, str, Dict[str, str], Optional[bytes]]) -> dict:
        method, url, headers, body = req
        handler = self.getHandler()
        rq = {"requestLine": {"method": method, "uri": url},
              "headers": [{"name": k, "value": v} for k, v in headers.items()],
              "entity": None if body is None else {"content": body}}
        resp = handler(session, rq, self.getTimeout()) if handler else \
            send_with_retries(session, rq, self.retries_ms, self.getTimeout())
        if isinstance(self, HasAsyncReply) and resp["statusLine"]["statusCode"] == 202:
            resp = self._poll(session, resp, headers)
        return resp

    def _requests_for(self, df) -> Tuple[List[Optional[tuple]], List[Dict[str, Any]]]:
        missing = [n for n in self._required_names() if self.getOrDefault(n) is None]
        if missing:
            raise ValueError(f"Missing required params: ({', '.join(missing)})")
        bad = set(self._vector_cols().values()) - set(df.columns)
        if bad:
            raise ValueError(f"Could not find dynamic columns: {sorted(bad)} in columns: {sorted(df.columns)}")
        cols = sorted(set(self._vector_cols().values()))
        data = {c: df[c].tolist() if df[c].ndim == 1 else list(df[c]) for c in cols}
        reqs, allvals = [], []
        for i in range(df.count()):
            vals = self._resolve({c: data[c][i] for c in cols})
            allvals.append(vals)
            if self._should_skip(vals):
                reqs.append(None)
                continue
            body, ctype = self._entity(vals) if self.method in ("POST", "PUT", "PATCH") else (None, None)
            reqs.append((self.method, self._url(vals), self._headers(vals, ctype), body))
        return reqs, allvals

    def _transform(self, df):
        import requests

        reqs, allvals = self._requests_for(df)
        session = requests.Session()

        def one(r):
            return None if r is None else self._send(session, r)

        if self.getConcurrency() <= 1:
            resps = [one(r) for r in reqs]
        else:
            with ThreadPoolExecutor(max_workers=self.getConcurrency()) as ex:
                resps = list(ex.map(one, reqs))
        outs, errs = [], []
        for resp, vals in zip(resps, allvals):
            err = error_of(resp)
            errs.append(err)
            outs.append(None if resp is None or err is not None else self._postprocess(self._parse(resp), vals))
        return df.withColumn(self.getOutputCol(), _obj(outs)).withColumn(self.getErrorCol(), _obj(errs))


class HasAPIVersion(Params):
    apiVersion = ServiceParam("version of the api", url_param=True, payload_name="api-version")


def url_join(*parts: str) -> str:
    out = parts[0]
    for p in parts[1:]:
        out = out.rstrip("/") + "/" + quote(str(p).lstrip("/"), safe="/:?=&")
    return out


__all__ = ["ServiceParam", "ServiceValue", "HasServiceParams", "CognitiveServicesBase", "HasAsyncReply",
           "HasAPIVersion", "location_domain", "url_join"]
