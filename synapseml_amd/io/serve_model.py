"""Serve a saved pipeline over HTTP: ``python -m synapseml_amd.io.serve_model --model DIR``
(reference: the Spark Serving deployment pattern — readStream.server() -> parseRequest ->
model.transform -> makeReply -> writeStream.server(), io/http/HTTPTransformer +
DistributedHTTPSource; here one ServingServer process per GPU, see tools/k8s/serving.yaml).

Request body: a JSON object with the model's input column(s), e.g. ``{"features": [..28 floats..]}``.
Reply: a JSON object with the requested output columns of the transformed row."""
from __future__ import annotations

import argparse
import signal
import threading
from typing import List, Optional

import numpy as np

from ..core.dataframe import DataFrame
from .serving import ServingServer, make_response, parse_request


def _jsonable(v):
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, np.generic):
        return v.item()
    if hasattr(v, "toArray"):
        return v.toArray().tolist()
    return v


def model_handler(model, input_cols: List[str], output_cols: Optional[List[str]] = None):
    """DataFrame(id, request) -> DataFrame(id, reply) around ``model.transform`` (one batched call per batch)."""

    def handle(df: DataFrame) -> DataFrame:
        parsed = parse_request(df, input_cols, parsing_check="none")
        n = parsed.count()
        cols = {}
        for c in input_cols:
            vals = parsed[c].tolist()
            if vals and all(isinstance(v, list) for v in vals) and len({len(v) for v in vals}) == 1:
                cols[c] = np.asarray(vals, dtype=np.float64)  # dense vector column
            else:
                a = np.empty(n, dtype=object)
                a[:] = vals
                cols[c] = a
        out = model.transform(DataFrame(cols))
        keep = output_cols or [c for c in out.columns if c not in input_cols]
        reps = np.empty(n, dtype=object)
        for i in range(n):
            reps[i] = make_response({c: _jsonable(out[c][i]) for c in keep})
        return DataFrame({"id": parsed["id"], "reply": reps})

    return handle


def main(argv=None) -> None:
    from ..core.serialize import load_stage

    ap = argparse.ArgumentParser()
    ap.add_argument("--model", required=True, help="directory written by stage.save()")
    ap.add_argument("--input-cols", default="features")
    ap.add_argument("--output-cols", default="")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8898)
    ap.add_argument("--api", default="")
    ap.add_argument("--max-batch-size", type=int, default=64)
    a = ap.parse_args(argv)
    model = load_stage(a.model)
    outs = [c for c in a.output_cols.split(",") if c] or None
    srv = ServingServer(model_handler(model, a.input_cols.split(","), outs), a.host, a.port, a.api,
                        max_batch_size=a.max_batch_size).start()
    print(f"serving {type(model).__name__} at {srv.address}", flush=True)
    done = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: done.set())
    try:
        done.wait()
    except KeyboardInterrupt:
        pass
    srv.stop()


if __name__ == "__main__":
    main()
