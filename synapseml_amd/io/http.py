"""HTTP on DataFrames (reference: core/.../io/http/{HTTPTransformer,
SimpleHTTPTransformer, HTTPClients, HTTPSchema, Parsers}.scala).

Requests and responses are plain dicts shaped like the reference's
HTTPRequestData / HTTPResponseData rows. Requests of a partition are sent
with ``concurrency`` worker threads; the default handler retries with the
reference's back-off list, waits ``Retry-After`` seconds on 429 (which does
not consume a retry), retries 5xx codes and returns other 4xx codes as-is."""
from __future__ import annotations

import json
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np

from ..core.contracts import HasInputCol, HasOutputCol
from ..core.dataframe import DataFrame
from ..core.params import Param, Params, TypeConverters as T
from ..core.pipeline import PipelineModel, Transformer


def _obj(values) -> np.ndarray:
    arr = np.empty(len(values), dtype=object)
    for i, v in enumerate(values):
        arr[i] = v
    return arr


# ---------------------------------------------------------------------- schema helpers
def make_request(url: str, method: str = "GET", headers: Optional[Dict[str, str]] = None,
                 entity: Optional[bytes] = None, content_type: Optional[str] = None) -> dict:
    hdrs = [{"name": k, "value": v} for k, v in (headers or {}).items()]
    ent = None
    if entity is not None:
        ent = {"content": entity if isinstance(entity, bytes) else str(entity).encode("utf-8"),
               "contentEncoding": None, "contentLength": len(entity),
               "contentType": {"name": "Content-Type", "value": content_type or "application/json"},
               "isChunked": False, "isRepeatable": True, "isStreaming": False}
    return {"requestLine": {"method": method, "uri": url,
                            "protocolVersion": {"protocol": "HTTP", "major": 1, "minor": 1}},
            "headers": hdrs, "entity": ent}


def response_string(resp: Optional[dict]) -> Optional[str]:
    if resp is None or resp.get("entity") is None:
        return None
    c = resp["entity"]["content"]
    return c.decode("utf-8", errors="replace") if isinstance(c, (bytes, bytearray)) else str(c)


def _to_response(r) -> dict:
    return {"headers": [{"name": k, "value": v} for k, v in r.headers.items()],
            "entity": {"content": r.content, "contentEncoding": r.encoding,
                       "contentLength": len(r.content),
                       "contentType": {"name": "Content-Type", "value": r.headers.get("Content-Type")},
                       "isChunked": False, "isRepeatable": True, "isStreaming": False},
            "statusLine": {"protocolVersion": {"protocol": "HTTP", "major": 1, "minor": 1},
                           "statusCode": r.status_code, "reasonPhrase": r.reason},
            "locale": "en_US"}


def send_with_retries(session, req: dict, retries_ms: Sequence[int], timeout: float,
                      extra_codes_to_retry: Sequence[int] = ()) -> Optional[dict]:
    """HandlingUtils.advanced semantics (HTTPClients.scala:86-135)."""
    retries = list(retries_ms)
    while True:
        try:
            ent = req.get("entity")
            r = session.request(req["requestLine"]["method"], req["requestLine"]["uri"],
                                headers={h["name"]: h["value"] for h in req.get("headers") or []},
                                data=ent["content"] if ent else None, timeout=timeout)
        except Exception:
            if not retries:
                raise
            time.sleep(retries.pop(0) / 1000.0)
            continue
        code = r.status_code
        if code in (200, 201, 202):
            return _to_response(r)
        if code == 429:
            ra = r.headers.get("Retry-After")
            if ra:
                time.sleep(float(ra))
            if not retries:
                return _to_response(r)
            time.sleep(retries[0] / 1000.0)  # rate limiting does not consume a retry
            continue
        retry = code in extra_codes_to_retry or not str(code).startswith("4")  # 4xx (except 429) are final
        if not retry or not retries:
            return _to_response(r)
        time.sleep(retries.pop(0) / 1000.0)


def advanced_handler(*retries_ms: int) -> Callable:
    def handler(session, req, timeout):
        return send_with_retries(session, req, retries_ms, timeout)

    return handler


def basic_handler(session, req, timeout):
    return send_with_retries(session, req, (), timeout)


class ConcurrencyParams(Params):
    concurrency = Param("max number of concurrent calls", 1, T.toInt)
    timeout = Param("number of seconds to wait before closing the connection", 60.0, T.toFloat)
    concurrentTimeout = Param("max number seconds to wait on futures if concurrency >= 1", None, T.toFloat)


class HasHandler(Params):
    handler = Param("Which strategy to use when handling requests", None, complex=True)


class HTTPTransformer(Transformer, ConcurrencyParams, HasInputCol, HasOutputCol, HasHandler):
    def _send_all(self, reqs: List[Optional[dict]]) -> List[Optional[dict]]:
        import requests

        handler = self.getHandler() or advanced_handler(100, 500, 1000)
        session = requests.Session()

        def one(req):
            if req is None:
                return None
            return handler(session, req, self.getTimeout())

        if self.getConcurrency() <= 1:
            return [one(r) for r in reqs]
        with ThreadPoolExecutor(max_workers=self.getConcurrency()) as ex:
            return list(ex.map(one, reqs))

    def _transform(self, df):
        return df.withColumn(self.getOutputCol(), _obj(self._send_all(df[self.getInputCol()].tolist())))


# ---------------------------------------------------------------------- parsers
class HTTPInputParser(Transformer, HasInputCol, HasOutputCol):
    pass


class JSONInputParser(HTTPInputParser):
    url = Param("Url of the service", None, T.toString)
    method = Param("method to use for request, (PUT, POST, PATCH)", "POST", T.toString)
    headers = Param("headers of the request", {}, T.identity)

    def _transform(self, df):
        out = []
        for v in df[self.getInputCol()].tolist():
            body = json.dumps(_jsonable(v)).encode("utf-8")
            out.append(make_request(self.getUrl(), self.getMethod(),
                                    dict({"Content-Type": "application/json"}, **(self.getHeaders() or {})), body))
        return df.withColumn(self.getOutputCol(), _obj(out))


class CustomInputParser(HTTPInputParser):
    udf = Param("User Defined Function to be applied to the DF input col", None, complex=True)

    def _transform(self, df):
        f = self.getUdf()
        return df.withColumn(self.getOutputCol(), _obj([f(v) for v in df[self.getInputCol()].tolist()]))


class HTTPOutputParser(Transformer, HasInputCol, HasOutputCol):
    pass


class JSONOutputParser(HTTPOutputParser):
    dataType = Param("format to parse the column to (optional field names to keep)", None, T.identity)
    postProcessor = Param("optional transformation to postprocess json output", None, complex=True)

    def _transform(self, df):
        out = []
        for r in df[self.getInputCol()].tolist():
            s = response_string(r)
            v = None if s is None else json.loads(s)
            if self.getPostProcessor() is not None and v is not None:
                v = self.getPostProcessor()(v)
            out.append(v)
        return df.withColumn(self.getOutputCol(), _obj(out))


class StringOutputParser(HTTPOutputParser):
    def _transform(self, df):
        return df.withColumn(self.getOutputCol(), _obj([response_string(r) for r in df[self.getInputCol()].tolist()]))


class CustomOutputParser(HTTPOutputParser):
    udf = Param("User Defined Function to be applied to the DF input col", None, complex=True)

    def _transform(self, df):
        f = self.getUdf()
        return df.withColumn(self.getOutputCol(), _obj([f(v) for v in df[self.getInputCol()].tolist()]))


def _jsonable(v):
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, np.generic):
        return v.item()
    if isinstance(v, dict):
        return {k: _jsonable(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if hasattr(v, "toArray"):
        return v.toArray().tolist()
    return v


def error_of(resp: Optional[dict]) -> Optional[dict]:
    if resp is None:
        return None
    code = resp["statusLine"]["statusCode"]
    if 200 <= code < 300:
        return None
    return {"response": response_string(resp), "status": resp["statusLine"]}


class SimpleHTTPTransformer(Transformer, ConcurrencyParams, HasInputCol, HasOutputCol, HasHandler):
    errorCol = Param("column to hold http errors", None, T.toString)
    flattenOutputBatches = Param("whether to flatten the output batches", None, T.toBoolean)
    inputParser = Param("format to parse the column to", None, complex=True)
    outputParser = Param("format to parse the column to", None, complex=True)
    miniBatcher = Param("Minibatcher to use", None, complex=True)

    def __init__(self, **kw):
        super().__init__(**kw)
        self._setDefault(errorCol=self.uid + "_errors")

    def setUrl(self, url: str):  # noqa: N802
        ip = self.getInputParser() or JSONInputParser()
        if not isinstance(ip, JSONInputParser):
            raise ValueError("this setting is only available when using a JSONInputParser")
        ip.setUrl(url)
        return self.set("inputParser", ip)

    def _transform(self, df):
        from ..stages.batching import FlattenBatch

        work = df
        mb = self.getMiniBatcher()
        if mb is not None:
            work = mb.transform(work)
        ip = (self.getInputParser() or JSONInputParser()).copy()
        ip.set("inputCol", self.getInputCol())
        ip.set("outputCol", "__parsed_input")
        work = ip.transform(work)
        client = HTTPTransformer(inputCol="__parsed_input", outputCol="__unparsed_output",
                                 concurrency=self.getConcurrency(), timeout=self.getTimeout())
        client.set("handler", self.getHandler() or advanced_handler(0, 50, 100, 500))
        work = client.transform(work)
        resp = work["__unparsed_output"].tolist()
        errs = [error_of(r) for r in resp]
        work = work.withColumn(self.getErrorCol(), _obj(errs)).withColumn(
            "__unparsed_output", _obj([None if e is not None else r for r, e in zip(resp, errs)]))
        op = (self.getOutputParser() or JSONOutputParser()).copy()
        op.set("inputCol", "__unparsed_output")
        op.set("outputCol", self.getOutputCol())
        work = op.transform(work).drop("__parsed_input", "__unparsed_output")
        if mb is not None and self.getFlattenOutputBatches() is not False:
            work = FlattenBatch().transform(work)
        return work


__all__ = ["HTTPTransformer", "SimpleHTTPTransformer", "JSONInputParser", "JSONOutputParser", "StringOutputParser",
           "CustomInputParser", "CustomOutputParser", "make_request", "response_string", "advanced_handler",
           "basic_handler", "send_with_retries"]
