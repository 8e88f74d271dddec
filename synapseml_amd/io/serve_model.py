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


class DistributedServing:
    """One serving worker process per device on ONE port (reference: DistributedHTTPSource - a server
    per executor behind the cluster's load balancer - and ``readStream.distributedServer()``).

    Every worker loads the saved pipeline, pins its GPU through ``HIP_VISIBLE_DEVICES`` and listens
    with ``SO_REUSEPORT``: the kernel balances incoming connections across the workers, so each GPU
    batches and scores its own share of the traffic with no front-end process. Replies carry
    ``X-Served-By: <worker>``. The parent never touches the GPU; workers are child processes."""

    def __init__(self, model_dir: str, num_workers: int, port: int, host: str = "127.0.0.1", input_cols: str = "features",
                 output_cols: str = "", api: str = "", max_batch_size: int = 64, gpus: Optional[List[int]] = None,
                 startup_timeout: float = 120.0):
        import os
        import subprocess
        import sys
        import time
        import urllib.request

        if port <= 0:
            raise ValueError("DistributedServing needs an explicit port (every worker binds it)")
        self.port, self.host, self.api = port, host, api
        self.procs = []
        for w in range(num_workers):
            env = dict(os.environ)
            if gpus is not None:
                env["HIP_VISIBLE_DEVICES"] = str(gpus[w % len(gpus)])
            cmd = [sys.executable, "-m", "synapseml_amd.io.serve_model", "--model", model_dir, "--host", host,
                   "--port", str(port), "--input-cols", input_cols, "--output-cols", output_cols, "--api", api,
                   "--max-batch-size", str(max_batch_size), "--reuse-port", "--worker-id", str(w)]
            self.procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                               text=True))
        # each worker prints one "serving ..." line once it listens. Its output is read on a thread that
        # feeds a queue, so a worker that hangs silently (model load, GPU init) cannot block the parent past
        # the deadline; the same thread keeps draining the pipe afterwards (a full pipe blocks a worker)
        import queue as _queue
        import threading as _threading

        ready: "_queue.Queue" = _queue.Queue()

        def _pump(w, f):
            announced = False
            for line in f:
                if not announced and line.startswith("serving"):
                    announced = True
                    ready.put((w, line))
            if not announced:
                ready.put((w, None))  # exited without listening

        for w, p in enumerate(self.procs):
            _threading.Thread(target=_pump, args=(w, p.stdout), daemon=True).start()
        deadline = time.monotonic() + startup_timeout
        pending = set(range(num_workers))
        while pending:
            try:
                w, line = ready.get(timeout=max(0.0, deadline - time.monotonic()))
            except _queue.Empty:
                self.stop()
                raise RuntimeError(f"serving workers {sorted(pending)} did not start within {startup_timeout}s")
            if line is None:
                self.stop()
                raise RuntimeError(f"serving worker {w} exited before listening (code {self.procs[w].poll()})")
            pending.discard(w)

    @property
    def address(self) -> str:
        return f"http://{self.host}:{self.port}/{self.api}"

    def stop(self) -> None:
        import signal as _signal

        for p in self.procs:
            if p.poll() is None:
                p.send_signal(_signal.SIGTERM)
        for p in self.procs:
            try:
                p.wait(20)
            except Exception:  # noqa: BLE001 - escalate below
                p.kill()
                p.wait(5)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()


def _worker_gpus(spec: Optional[str]) -> Optional[List[int]]:
    """Device ids the serving workers are spread over (one per worker, round robin): ``--gpus``, else
    SML_SERVE_GPUS (a count), else the visible devices - counted without initialising a GPU in the
    parent (HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES, else torch's device count, which on this image
    does not initialise the runtime). None when there is no GPU."""
    import os

    if spec:
        return [int(x) for x in spec.split(",") if x.strip()]
    n = int(os.environ.get("SML_SERVE_GPUS", "0"))
    if n:
        return list(range(n))
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:
            return list(range(len([x for x in v.split(",") if x.strip()])))
    try:
        import torch

        n = torch.cuda.device_count()
    except Exception:  # noqa: BLE001 - no torch / no ROCm: CPU workers
        n = 0
    return list(range(n)) if n else None


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
    ap.add_argument("--workers", type=int, default=1, help="worker processes on the port (one per GPU)")
    ap.add_argument("--reuse-port", action="store_true", help="bind with SO_REUSEPORT (set for workers)")
    ap.add_argument("--worker-id", default=None)
    ap.add_argument("--gpus", default=None, help="comma-separated device ids for the workers (default: all visible)")
    ap.add_argument("--mode", choices=("microbatch", "continuous"), default="microbatch",
                    help="continuous: per-request partition tasks with epochs (io/streaming.py)")
    ap.add_argument("--num-partitions", type=int, default=2, help="continuous mode: partition tasks")
    ap.add_argument("--epoch-ms", type=float, default=30000.0, help="continuous mode: epoch (checkpoint) interval")
    ap.add_argument("--checkpoint-location", default=None, help="continuous mode: offsets/commits directory")
    a = ap.parse_args(argv)
    if a.workers > 1 and a.mode == "continuous":
        # the multi-worker front end runs micro-batch workers only; continuous mode's epochs/offsets are per
        # process (one checkpoint location each), so scale it with one replica per GPU instead
        ap.error("--mode continuous serves from one process: use --workers 1 per replica (one checkpoint "
                 "location per replica), not --workers > 1")
    if a.workers > 1:
        srv_d = DistributedServing(a.model, a.workers, a.port, a.host, a.input_cols, a.output_cols, a.api,
                                   a.max_batch_size, gpus=_worker_gpus(a.gpus))
        print(f"serving {a.workers} workers at {srv_d.address}", flush=True)
        done = threading.Event()
        signal.signal(signal.SIGTERM, lambda *_: done.set())
        try:
            done.wait()
        except KeyboardInterrupt:
            pass
        srv_d.stop()
        return
    model = load_stage(a.model)
    outs = [c for c in a.output_cols.split(",") if c] or None
    handler = model_handler(model, a.input_cols.split(","), outs)
    if a.mode == "continuous":
        from .streaming import ContinuousServingServer

        srv = ContinuousServingServer(handler, a.host, a.port, a.api, num_partitions=a.num_partitions,
                                      epoch_length_ms=a.epoch_ms, checkpoint_location=a.checkpoint_location).start()
    else:
        srv = ServingServer(handler, a.host, a.port, a.api, max_batch_size=a.max_batch_size,
                            reuse_port=a.reuse_port, worker_id=a.worker_id).start()
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
