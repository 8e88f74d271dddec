"""Model serving over HTTP (reference: SPX/sql/execution/streaming/
{HTTPSource, DistributedHTTPSource, continuous/HTTPSourceV2, HTTPSinkV2,
ServingUDFs}.scala and CORE/io/IOImplicits.scala:100-187).

MI355X-first shape: one server per GPU process. HTTP handler threads enqueue
requests; a single batching loop drains up to ``max_batch_size`` requests (or
waits at most ``max_wait_ms`` for the first one to have company; 0 = take what
is queued and go, so an idle server answers at once and batches form under
load while the previous batch runs), turns them
into one DataFrame(id, request) micro-batch, runs the user's transform —
typically a pipeline whose heavy stage is a device model, so a whole batch is
one device launch sequence — and routes the reply column back by id.

``parse_request`` / ``make_reply`` mirror the reference's DataFrame
extensions (parsingCheck none/partial/full; 400 "JSON Parsing Failure")."""
from __future__ import annotations

import asyncio
import itertools
import json
import socket
import threading
import time
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


class ServingServer:
    """Batched HTTP serving of a DataFrame transform.

    ``transform(df)`` receives DataFrame(id, request) and must return a
    DataFrame with ``id`` and a ``reply`` column (see ``make_reply``); rows it
    drops are answered by ``parse_request`` or get a 500.

    One asyncio event loop (its own thread) owns every connection: it parses
    HTTP/1.1 requests itself (persistent connections, TCP_NODELAY, one write
    per reply) and scores in the loop thread, so an idle server answers a
    request with no thread hand-off at all. Requests that arrive while a batch
    is scoring queue up and form the next micro-batch (``max_batch_size``);
    ``max_wait_ms`` > 0 additionally holds the first request of a batch that
    long for company."""

    def __init__(self, transform: Callable[[DataFrame], DataFrame], host: str = "127.0.0.1", port: int = 0,
                 api: str = "", max_batch_size: int = 64, max_wait_ms: float = 0.0, reply_col: str = "reply",
                 request_timeout: float = 60.0, reuse_port: bool = False, worker_id: Optional[str] = None):
        self.transform_fn = transform
        self.api = api.strip("/")
        self.max_batch_size = max_batch_size
        self.max_wait_ms = max_wait_ms
        self.reply_col = reply_col
        self.request_timeout = request_timeout
        self._ids = itertools.count()
        self._queue: list = []
        self._pending: Dict[int, tuple] = {}
        self._scheduled = False
        self._conns: set = set()
        self.batch_sizes: List[int] = []
        self.latencies_ms: List[float] = []
        self._loop = asyncio.new_event_loop()
        self._sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        if reuse_port:
            # several worker processes (one per GPU) listen on one port; the kernel spreads connections
            self._sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
        self.worker_id = worker_id  # echoed as X-Served-By on every reply
        self._sock.bind((host, port))
        self._sock.listen(1024)
        self._sock.setblocking(False)
        self.host, self.port = self._sock.getsockname()[:2]
        self._server = None
        self._thread = threading.Thread(target=self._run_loop, daemon=True)
        self._ready = threading.Event()

    @property
    def address(self) -> str:
        return f"http://{self.host}:{self.port}/{self.api}"

    def start(self) -> "ServingServer":
        if not self._thread.is_alive():  # idempotent: `with serve(...)` after start() is fine
            self._thread.start()
        self._ready.wait(30)
        return self

    def stop(self) -> None:
        if self._loop.is_running():
            try:
                asyncio.run_coroutine_threadsafe(self._shutdown(), self._loop).result(10)
            except Exception:  # noqa: BLE001 - best effort
                pass
            self._loop.call_soon_threadsafe(self._loop.stop)
            self._thread.join(10)
        self._sock.close()

    async def _shutdown(self) -> None:
        if self._server is not None:
            self._server.close()
        tasks = [t for t in self._conns if not t.done()]
        for t in tasks:
            t.cancel()
        await asyncio.gather(*tasks, return_exceptions=True)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # ------------------------------------------------------------------ event loop
    def _run_loop(self) -> None:
        asyncio.set_event_loop(self._loop)

        async def boot():
            self._server = await asyncio.start_server(self._conn, sock=self._sock)

        self._loop.run_until_complete(boot())
        self._ready.set()
        try:
            self._loop.run_forever()
        finally:
            if self._server is not None:
                self._server.close()

    async def _conn(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        task = asyncio.current_task()
        self._conns.add(task)
        sock = writer.get_extra_info("socket")
        if sock is not None:
            # replies are small: without TCP_NODELAY, Nagle + the client's delayed ACK add ~40 ms
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        try:
            while True:
                line = await reader.readline()
                if not line or not line.strip():
                    break
                parts = line.decode("latin-1").split()
                if len(parts) < 2:
                    break
                method, target = parts[0], parts[1]
                headers: Dict[str, str] = {}
                while True:
                    h = await reader.readline()
                    if not h or h in (b"\r\n", b"\n"):
                        break
                    k, _, v = h.decode("latin-1").partition(":")
                    headers[k.strip()] = v.strip()
                low = {k.lower(): v for k, v in headers.items()}
                n = int(low.get("content-length") or 0)
                body = await reader.readexactly(n) if n else None
                close = low.get("connection", "").lower() == "close"
                path = target.split("?")[0].strip("/")
                if self.api and path != self.api:
                    writer.write(b"HTTP/1.1 404 Not Found\r\nContent-Length: 0\r\n\r\n")
                else:
                    resp = await self._submit(make_request(target, method, headers, body, low.get("content-type")))
                    writer.write(_serialize(resp, self.worker_id))
                await writer.drain()
                if close:
                    break
        except (asyncio.IncompleteReadError, ConnectionError, asyncio.CancelledError):
            pass
        finally:
            self._conns.discard(task)
            try:
                writer.close()
            except RuntimeError:  # loop shutting down
                pass

    async def _submit(self, req: dict) -> dict:
        rid = next(self._ids)
        fut = self._loop.create_future()
        self._pending[rid] = (fut, time.perf_counter())
        self._queue.append((rid, req))
        if not self._scheduled:
            self._scheduled = True
            if self.max_wait_ms > 0:
                self._loop.call_later(self.max_wait_ms / 1e3, self._drain)
            else:
                self._loop.call_soon(self._drain)
        try:
            return await asyncio.wait_for(fut, self.request_timeout)
        except asyncio.TimeoutError:
            self._pending.pop(rid, None)
            return make_response("request timed out", 504, "Gateway Timeout")

    def _drain(self) -> None:
        self._scheduled = False
        while self._queue:
            batch = self._queue[: self.max_batch_size]
            del self._queue[: self.max_batch_size]
            self._run_batch(batch)

    def reply(self, rid: int, response: dict) -> None:
        """Answer request ``rid`` (callable from the transform or from another thread)."""
        if threading.current_thread() is not self._thread:
            self._loop.call_soon_threadsafe(self.reply, rid, response)
            return
        entry = self._pending.pop(rid, None)
        if entry is not None and not entry[0].done():
            self.latencies_ms.append((time.perf_counter() - entry[1]) * 1e3)
            entry[0].set_result(response)

    def _run_batch(self, batch: list) -> None:
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


def _serialize(resp: dict, worker_id: Optional[str] = None) -> bytes:
    st = resp.get("statusLine") or {}
    code = int(st.get("statusCode", 200))
    reason = st.get("reasonPhrase") or ""
    content = (resp.get("entity") or {}).get("content") or b""
    if isinstance(content, str):
        content = content.encode("utf-8")
    head = [f"HTTP/1.1 {code} {reason}"]
    for h in resp.get("headers") or []:
        if h["name"].lower() != "content-length":
            head.append(f"{h['name']}: {h['value']}")
    if worker_id is not None:
        head.append(f"X-Served-By: {worker_id}")
    head.append(f"Content-Length: {len(content)}")
    return ("\r\n".join(head) + "\r\n\r\n").encode("latin-1") + content


def serve(transform: Callable[[DataFrame], DataFrame], host: str = "127.0.0.1", port: int = 0, api: str = "",
          **kw) -> ServingServer:
    return ServingServer(transform, host, port, api, **kw).start()


__all__ = ["ServingServer", "serve", "parse_request", "make_reply", "make_response", "request_to_string"]
