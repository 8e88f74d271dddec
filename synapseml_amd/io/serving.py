"""Model serving over HTTP (reference: SPX/sql/execution/streaming/
{HTTPSource, DistributedHTTPSource, continuous/HTTPSourceV2, HTTPSinkV2,
ServingUDFs}.scala and CORE/io/IOImplicits.scala:100-187).

MI355X-first shape: one server per GPU process. HTTP handler threads enqueue
requests; a single batching loop drains up to ``max_batch_size`` requests (or
waits at most ``max_wait_ms`` for the first one to have company), turns them
into one DataFrame(id, request) micro-batch, runs the user's transform —
typically a pipeline whose heavy stage is a device model, so a whole batch is
one device launch sequence — and routes the reply column back by id.

``parse_request`` / ``make_reply`` mirror the reference's DataFrame
extensions (parsingCheck none/partial/full; 400 "JSON Parsing Failure")."""
from __future__ import annotations

import itertools
import json
import queue
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Dict, List, Optional, Union

import numpy as np

from ..core.dataframe import DataFrame
from .http import _jsonable, make_request


def _obj(values) -> np.ndarray:
    arr = np.empty(len(values), dtype=object)
    for i, v in enumerate(values):
        arr[i] = v
    return arr


def make_response(entity, code: int = 200, reason: str = "Success", content_type: Optional[str] = None) -> dict:
    if isinstance(entity, (bytes, bytearray)):
        body, ct = bytes(entity), content_type or "application/octet-stream"
    elif isinstance(entity, str):
        body, ct = entity.encode("utf-8"), content_type or "text/plain"
    else:
        body, ct = json.dumps(_jsonable(entity)).encode("utf-8"), content_type or "application/json"
    return {"statusLine": {"statusCode": code, "reasonPhrase": reason},
            "headers": [{"name": "Content-Type", "value": ct}],
            "entity": {"content": body, "contentLength": len(body)}}


def request_to_string(req: dict) -> Optional[str]:
    ent = req.get("entity") if req else None
    if not ent:
        return None
    c = ent["content"]
    return c.decode("utf-8", errors="replace") if isinstance(c, (bytes, bytearray)) else str(c)


def _full_ok(v) -> bool:
    if v is None:
        return False
    if isinstance(v, dict):
        return all(_full_ok(x) for x in v.values())
    if isinstance(v, list):
        return all(_full_ok(x) for x in v)
    return True


def parse_request(df: DataFrame, schema: Union[str, List[str], Dict[str, type]], id_col: str = "id",
                  request_col: str = "request", parsing_check: str = "none",
                  server: Optional["ServingServer"] = None) -> DataFrame:
    """Parse request bodies into columns.

    ``schema="binary"`` returns (id, bytes). Otherwise bodies are parsed as
    JSON objects and ``schema`` names the fields (types are applied when a
    dict of callables is given). Missing fields become None. With
    ``parsing_check`` "partial"/"full" unparseable rows are answered with 400
    through ``server`` and dropped."""
    reqs = df[request_col].tolist()
    ids = df[id_col].tolist()
    if schema == "binary":
        return DataFrame({id_col: _obj(ids), "bytes": _obj([(r.get("entity") or {}).get("content") for r in reqs])})
    fields = list(schema.keys()) if isinstance(schema, dict) else list(schema)
    check = parsing_check.lower()
    if check not in ("none", "partial", "full"):
        raise ValueError(f"Need to use either full, partial, or none. Received {parsing_check}")
    keep, rows = [], []
    for i, r in enumerate(reqs):
        body = request_to_string(r)
        try:
            parsed = json.loads(body) if body is not None else None
            if not isinstance(parsed, dict):
                parsed = None
        except ValueError:
            parsed = None
        row = None
        if parsed is not None:
            row = {}
            for f in fields:
                v = parsed.get(f)
                if v is not None and isinstance(schema, dict) and schema[f] is not None:
                    try:
                        v = schema[f](v)
                    except (TypeError, ValueError):
                        v = None
                row[f] = v
        ok = True if check == "none" else (row is not None if check == "partial" else _full_ok(row))
        if not ok:
            if server is not None:
                server.reply(ids[i], make_response(
                    f"JSON Parsing error, expected schema:\n {fields}\n received:\n {body}", 400,
                    "JSON Parsing Failure"))
            continue
        keep.append(i)
        rows.append(row or {f: None for f in fields})
    out = {id_col: _obj([ids[i] for i in keep])}
    for f in fields:
        out[f] = _obj([r[f] for r in rows])
    return DataFrame(out)


def make_reply(df: DataFrame, reply_col: str, name: str = "reply") -> DataFrame:
    return df.withColumn(name, _obj([v if isinstance(v, dict) and "statusLine" in v else make_response(v)
                                     for v in df[reply_col].tolist()]))


class _Pending:
    __slots__ = ("event", "response", "t0")

    def __init__(self):
        self.event = threading.Event()
        self.response: Optional[dict] = None
        self.t0 = time.perf_counter()


class ServingServer:
    """Batched HTTP serving of a DataFrame transform.

    ``transform(df)`` receives DataFrame(id, request) and must return a
    DataFrame with ``id`` and a ``reply`` column (see ``make_reply``); rows it
    drops are answered by ``parse_request`` or get a 500."""

    def __init__(self, transform: Callable[[DataFrame], DataFrame], host: str = "127.0.0.1", port: int = 0,
                 api: str = "", max_batch_size: int = 64, max_wait_ms: float = 1.0, reply_col: str = "reply",
                 request_timeout: float = 60.0):
        self.transform_fn = transform
        self.api = api.strip("/")
        self.max_batch_size = max_batch_size
        self.max_wait_ms = max_wait_ms
        self.reply_col = reply_col
        self.request_timeout = request_timeout
        self._q: "queue.Queue" = queue.Queue()
        self._pending: Dict[int, _Pending] = {}
        self._lock = threading.Lock()
        self._ids = itertools.count()
        self._stop = threading.Event()
        self.batch_sizes: List[int] = []
        self.latencies_ms: List[float] = []
        outer = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):  # silence default stderr logging
                pass

            def _handle(self):
                path = self.path.split("?")[0].strip("/")
                if outer.api and path != outer.api:
                    self.send_response(404)
                    self.send_header("Content-Length", "0")
                    self.end_headers()
                    return
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n) if n else None
                req = make_request(self.path, self.command, dict(self.headers.items()), body,
                                   self.headers.get("Content-Type"))
                resp = outer._submit(req)
                ent = resp.get("entity") or {}
                content = ent.get("content") or b""
                self.send_response(resp["statusLine"]["statusCode"], resp["statusLine"].get("reasonPhrase"))
                for h in resp.get("headers") or []:
                    self.send_header(h["name"], h["value"])
                self.send_header("Content-Length", str(len(content)))
                self.end_headers()
                self.wfile.write(content)

            do_GET = do_POST = do_PUT = _handle

        self._httpd = ThreadingHTTPServer((host, port), Handler)
        self._httpd.daemon_threads = True
        self.host, self.port = self._httpd.server_address[:2]
        self._threads = [threading.Thread(target=self._httpd.serve_forever, daemon=True),
                         threading.Thread(target=self._batch_loop, daemon=True)]

    @property
    def address(self) -> str:
        return f"http://{self.host}:{self.port}/{self.api}"

    def start(self) -> "ServingServer":
        for t in self._threads:
            t.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        self._httpd.shutdown()
        self._httpd.server_close()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    def _submit(self, req: dict) -> dict:
        rid = next(self._ids)
        p = _Pending()
        with self._lock:
            self._pending[rid] = p
        self._q.put((rid, req))
        if not p.event.wait(self.request_timeout):
            with self._lock:
                self._pending.pop(rid, None)
            return make_response("request timed out", 504, "Gateway Timeout")
        return p.response

    def reply(self, rid: int, response: dict) -> None:
        with self._lock:
            p = self._pending.pop(rid, None)
        if p is not None:
            p.response = response
            self.latencies_ms.append((time.perf_counter() - p.t0) * 1e3)
            p.event.set()

    def _batch_loop(self) -> None:
        while not self._stop.is_set():
            try:
                first = self._q.get(timeout=0.05)
            except queue.Empty:
                continue
            batch = [first]
            deadline = time.perf_counter() + self.max_wait_ms / 1e3
            while len(batch) < self.max_batch_size:
                try:
                    batch.append(self._q.get_nowait())
                    continue
                except queue.Empty:
                    pass
                left = deadline - time.perf_counter()
                if left <= 0:
                    break
                try:
                    batch.append(self._q.get(timeout=left))
                except queue.Empty:
                    break
            self.batch_sizes.append(len(batch))
            ids = [b[0] for b in batch]
            df = DataFrame({"id": _obj(ids), "request": _obj([b[1] for b in batch])})
            try:
                out = self.transform_fn(df)
                for rid, rep in zip(out["id"].tolist(), out[self.reply_col].tolist()):
                    self.reply(rid, rep if isinstance(rep, dict) and "statusLine" in rep else make_response(rep))
            except Exception as e:  # noqa: BLE001 - reported to the client
                for rid in ids:
                    self.reply(rid, make_response(f"{type(e).__name__}: {e}", 500, "Internal Server Error"))
            for rid in ids:  # rows the transform dropped without replying
                self.reply(rid, make_response("no reply produced", 500, "Internal Server Error"))


def serve(transform: Callable[[DataFrame], DataFrame], host: str = "127.0.0.1", port: int = 0, api: str = "",
          **kw) -> ServingServer:
    return ServingServer(transform, host, port, api, **kw).start()


__all__ = ["ServingServer", "serve", "parse_request", "make_reply", "make_response", "request_to_string"]
