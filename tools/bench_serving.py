#!/usr/bin/env python3
"""Serving latency of a LightGBM model behind the batched HTTP server —
the reference's published serving claim (Spark Serving,
continuous mode, "as low as 1 ms"; docs/Deploy Models/Overview.md:18-19).

One process serves ``parse_request -> LightGBMClassificationModel.transform
-> make_reply`` (28 float features, 100 trees x 31 leaves); clients send JSON
requests over persistent HTTP/1.1 connections. Reported: round-trip latency
p50/p90/p99 of sequential requests from one client, and throughput with
--clients concurrent clients (requests coalesce into device-sized micro-
batches under load). Synthetic data."""
from __future__ import annotations

import argparse
import http.client
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=2000)
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--device", default="cpu", help="model scoring device (cpu or gpu)")
    a = ap.parse_args()
    from synapseml_amd.core import DataFrame
    from synapseml_amd.io.serving import make_reply, parse_request, serve
    from synapseml_amd.lightgbm import LightGBMClassifier

    rng = np.random.default_rng(0)
    X = rng.standard_normal((20000, 28))
    y = (X[:, 0] + X[:, 1] * X[:, 2] > 0).astype(float)
    model = LightGBMClassifier(numIterations=100, numLeaves=31, deviceType=a.device).fit(
        DataFrame({"features": X, "label": y}))
    fields = [f"f{i}" for i in range(28)]

    def pipeline(df):
        p = parse_request(df, fields)
        feats = np.column_stack([np.asarray(p[f], dtype=np.float64) for f in fields]) if p.count() else \
            np.zeros((0, 28))
        scored = model.transform(DataFrame({"id": p["id"], "features": feats}))
        prob = scored["probability"][:, 1] if scored.count() else np.zeros(0)
        return make_reply(DataFrame({"id": scored["id"], "p": np.asarray(prob, dtype=object)}), "p")

    bodies = [json.dumps({f: float(v) for f, v in zip(fields, row)}).encode() for row in X[:256]]
    srv = serve(pipeline, api="score")

    def client_code(n, off):
        """A sequential client as a program of its own (no GIL shared with the server): prints its
        latencies and the wall time of its request loop."""
        return (
            "import http.client, json, sys, time\n"
            f"bodies = {[b.decode() for b in bodies[:64]]!r}\n"
            f"c = http.client.HTTPConnection('{srv.host}', {srv.port})\n"
            "lat = []\n"
            "t_start = time.perf_counter()\n"
            f"for i in range({n}):\n"
            "    t0 = time.perf_counter()\n"
            f"    c.request('POST', '/score', body=bodies[({off} + i) % len(bodies)].encode(), "
            "headers={'Content-Type': 'application/json'})\n"
            "    r = c.getresponse(); r.read(); assert r.status == 200\n"
            "    lat.append((time.perf_counter() - t0) * 1e3)\n"
            "print(json.dumps({'lat': lat, 'wall': time.perf_counter() - t_start}))\n")

    def client_proc(n, off):
        import subprocess

        out = subprocess.run([sys.executable, "-c", client_code(n, off)], capture_output=True, text=True,
                             check=True).stdout
        return json.loads(out.strip().splitlines()[-1])["lat"]

    def client_procs(k, n):
        """k concurrent client processes of n requests each: (latencies, request-loop wall seconds)"""
        import subprocess

        ps = [subprocess.Popen([sys.executable, "-c", client_code(n, 13 * j)], stdout=subprocess.PIPE, text=True)
              for j in range(k)]
        res = [json.loads(p.communicate()[0].strip().splitlines()[-1]) for p in ps]
        if any(p.returncode for p in ps):
            raise RuntimeError("a serving client failed")
        return np.concatenate([np.asarray(r["lat"]) for r in res]), max(r["wall"] for r in res)

    def client(n, lat, off):
        c = http.client.HTTPConnection(srv.host, srv.port)
        for i in range(n):
            t0 = time.perf_counter()
            c.request("POST", "/score", body=bodies[(off + i) % len(bodies)], headers={"Content-Type": "application/json"})
            r = c.getresponse()
            r.read()
            lat.append((time.perf_counter() - t0) * 1e3)
            assert r.status == 200
        c.close()

    try:
        warm = []
        client(200, warm, 0)
        k0 = len(srv.latencies_ms)
        seq = client_proc(a.requests, 7)
        server_side = np.asarray(srv.latencies_ms[k0:])
        # concurrent clients, each its own process: the throughput is the server's, not the client threads'
        # share of the server's GIL (r1 ran them as threads of the serving process)
        per = max(1, a.requests // a.clients)
        allc, dt = client_procs(a.clients, per)
    finally:
        srv.stop()
    s = np.asarray(seq)
    print(json.dumps({
        "bench": "serving_latency", "model": "LightGBMClassifier 100 trees x 31 leaves, 28 features",
        "scoring_device": a.device, "sequential_requests": len(s),
        "p50_ms": round(float(np.percentile(s, 50)), 3), "p90_ms": round(float(np.percentile(s, 90)), 3),
        "p99_ms": round(float(np.percentile(s, 99)), 3),
        "server_queue_to_reply_p50_ms": round(float(np.percentile(server_side, 50)), 3), "clients": a.clients,
        "throughput_req_per_s": round(len(allc) / dt, 1),
        "concurrent_p50_ms": round(float(np.percentile(allc, 50)), 3),
        "mean_batch_size_under_load": round(float(np.mean(srv.batch_sizes[-max(1, len(allc) // 2):])), 2),
        "reference_claim": "Spark Serving continuous mode 'as low as 1 ms' (BASELINE.md P4)"}), flush=True)


if __name__ == "__main__":
    main()
