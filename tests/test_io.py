"""HTTP-on-DataFrame, serving and binary IO tests against local 127.0.0.1
servers (reference: core/src/test/.../io/{http,split1,split2}/*Suite.scala)."""
import json
import os
import threading
import urllib.request

import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.io import (HTTPTransformer, JSONOutputParser, PowerBIWriter, ServingServer, SimpleHTTPTransformer,
                              StringOutputParser, advanced_handler, make_reply, make_request, parse_request,
                              read_binary_files, response_string, zip_bytes)
from synapseml_amd.stages.batching import FixedMiniBatchTransformer


def _obj(v):
    a = np.empty(len(v), dtype=object)
    for i, x in enumerate(v):
        a[i] = x
    return a


def _echo_server(**kw):
    def fn(df):
        p = parse_request(df, {"x": float, "name": str})
        return make_reply(p.withColumn("out", _obj([{"y": (x or 0) * 2, "name": n}
                                                     for x, n in zip(p["x"].tolist(), p["name"].tolist())])),
                          "out")
    return ServingServer(fn, **kw).start()


def test_serving_roundtrip_and_batching():
    srv = _echo_server(max_batch_size=16, max_wait_ms=20)
    try:
        results = [None] * 32

        def call(i):
            req = urllib.request.Request(srv.address, data=json.dumps({"x": i, "name": f"n{i}"}).encode(),
                                         headers={"Content-Type": "application/json"}, method="POST")
            results[i] = json.loads(urllib.request.urlopen(req, timeout=10).read())

        ts = [threading.Thread(target=call, args=(i,)) for i in range(32)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        assert [r["y"] for r in results] == [2.0 * i for i in range(32)]
        assert results[5]["name"] == "n5"
        assert max(srv.batch_sizes) > 1  # concurrent requests were batched
    finally:
        srv.stop()


def test_parse_request_full_check_replies_400():
    def fn(df):
        p = parse_request(df, ["a", "b"], parsing_check="full", server=srv)
        return make_reply(p.withColumn("o", _obj([a + b for a, b in zip(p["a"].tolist(), p["b"].tolist())])), "o")

    srv = ServingServer(fn).start()
    try:
        ok = urllib.request.urlopen(urllib.request.Request(srv.address, data=b'{"a":1,"b":2}', method="POST"))
        assert json.loads(ok.read()) == 3
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(urllib.request.Request(srv.address, data=b'{"a":1}', method="POST"))
        assert e.value.code == 400
    finally:
        srv.stop()


def test_simple_http_transformer_json_and_errors():
    def fn(df):
        p = parse_request(df, ["x"])
        reps = []
        from synapseml_amd.io import make_response
        for x in p["x"].tolist():
            reps.append(make_response({"error": "neg"}, 400, "Bad") if x < 0 else {"sq": x * x})
        return p.withColumn("reply", _obj(reps))

    srv = ServingServer(fn).start()
    try:
        df = DataFrame({"data": _obj([{"x": 1}, {"x": -2}, {"x": 3}])})
        t = SimpleHTTPTransformer(inputCol="data", outputCol="results", concurrency=2)
        t.setUrl(srv.address)
        t.set("handler", advanced_handler())
        out = t.transform(df)
        res = out["results"].tolist()
        assert res[0] == {"sq": 1} and res[1] is None and res[2] == {"sq": 9}
        errs = out[t.getErrorCol()].tolist()
        assert errs[0] is None and errs[1]["status"]["statusCode"] == 400
    finally:
        srv.stop()


def test_simple_http_minibatch_flatten():
    def fn(df):
        p = parse_request(df, "binary")
        reps = [json.loads(b.decode())["v"] if False else [r["x"] + 1 for r in json.loads(b.decode())]
                for b in p["bytes"].tolist()]
        return p.withColumn("reply", _obj(reps))

    srv = ServingServer(fn).start()
    try:
        df = DataFrame({"data": _obj([{"x": i} for i in range(7)])})
        t = SimpleHTTPTransformer(inputCol="data", outputCol="res")
        t.setUrl(srv.address)
        t.set("miniBatcher", FixedMiniBatchTransformer(batchSize=3))
        out = t.transform(df)
        assert out.count() == 7
        assert list(out["res"]) == [i + 1 for i in range(7)]
    finally:
        srv.stop()


def test_http_retries_on_5xx_and_429():
    calls = {"n": 0}

    from synapseml_amd.io import make_response

    def fn(df):
        calls["n"] += len(df)
        if calls["n"] == 1:
            return df.withColumn("reply", _obj([make_response("busy", 503, "Unavailable")]))
        if calls["n"] in (2, 3):
            r = make_response("slow down", 429, "Too Many")
            r["headers"].append({"name": "Retry-After", "value": "0"})
            return df.withColumn("reply", _obj([r]))
        return df.withColumn("reply", _obj(["ok"]))

    srv = ServingServer(fn).start()
    try:
        df = DataFrame({"req": _obj([make_request(srv.address, "POST", {}, b"{}")])})
        t = HTTPTransformer(inputCol="req", outputCol="resp")
        t.set("handler", advanced_handler(1, 1))  # 429s do not consume retries
        out = t.transform(df)
        r = out["resp"].tolist()[0]
        assert r["statusLine"]["statusCode"] == 200 and response_string(r) == "ok"
        assert calls["n"] == 4
    finally:
        srv.stop()


def test_string_and_404():
    srv = ServingServer(lambda df: df.withColumn("reply", _obj(["hi"] * len(df))), api="my_api").start()
    try:
        df = DataFrame({"req": _obj([make_request(srv.address, "GET"),
                                     make_request(f"http://127.0.0.1:{srv.port}/other", "GET")])})
        out = HTTPTransformer(inputCol="req", outputCol="resp").set("handler", advanced_handler()).transform(df)
        s = StringOutputParser(inputCol="resp", outputCol="s").transform(out)
        assert s["s"].tolist()[0] == "hi"
        assert out["resp"].tolist()[1]["statusLine"]["statusCode"] == 404
    finally:
        srv.stop()


def test_powerbi_writer_posts_batches():
    got = []

    def fn(df):
        p = parse_request(df, "binary")
        for b in p["bytes"].tolist():
            got.append(json.loads(b.decode()))
        return p.withColumn("reply", _obj([{}] * len(p)))

    srv = ServingServer(fn).start()
    try:
        df = DataFrame({"a": np.arange(5), "b": _obj(list("vwxyz"))})
        PowerBIWriter.write(df, srv.address, {"batchSize": "2"})
        flat = [r for batch in got for r in batch]
        assert len(got) == 3 and sorted(r["a"] for r in flat) == list(range(5))
        with pytest.raises(ValueError):
            PowerBIWriter.write(df, srv.address, {"bogus": "1"})
    finally:
        srv.stop()


def test_read_binary_files_zip_and_sampling(tmp_path):
    (tmp_path / "a.bin").write_bytes(b"\x00\x01")
    (tmp_path / "sub").mkdir()
    (tmp_path / "sub" / "b.txt").write_bytes(b"hello")
    (tmp_path / "c.zip").write_bytes(zip_bytes({"m1.txt": b"one", "m2.txt": b"two"}))
    df = read_binary_files(str(tmp_path), recursive=True)
    paths = [os.path.relpath(p, tmp_path) for p in df["path"].tolist()]
    assert paths == ["a.bin", "c.zip/m1.txt", "c.zip/m2.txt", "sub/b.txt"]
    assert df["bytes"].tolist()[1] == b"one"
    flat = read_binary_files(str(tmp_path), recursive=False, inspectZip=False)
    assert len(flat) == 2
    s1 = read_binary_files(str(tmp_path), recursive=True, sampleRatio=0.5, seed=3)
    s2 = read_binary_files(str(tmp_path), recursive=True, sampleRatio=0.5, seed=3)
    assert s1["path"].tolist() == s2["path"].tolist()


def test_serve_saved_model_end_to_end(tmp_path):
    """Save a trained classifier, serve it with serve_model's handler, score over HTTP."""
    import json
    import urllib.request

    import numpy as np

    from synapseml_amd.core import DataFrame
    from synapseml_amd.core.serialize import load_stage
    from synapseml_amd.io.serve_model import model_handler
    from synapseml_amd.io.serving import ServingServer
    from synapseml_amd.lightgbm import LightGBMClassifier

    rng = np.random.default_rng(0)
    X = rng.standard_normal((600, 4))
    y = (X[:, 0] > 0).astype(float)
    m = LightGBMClassifier(numIterations=10, numLeaves=7, deviceType="cpu").fit(DataFrame({"features": X, "label": y}))
    m.save(str(tmp_path / "m"))
    model = load_stage(str(tmp_path / "m"))
    with ServingServer(model_handler(model, ["features"], ["prediction", "probability"])).start() as srv:
        for row, lab in ((X[0], y[0]), (X[1], y[1])):
            body = json.dumps({"features": row.tolist()}).encode()
            r = json.loads(urllib.request.urlopen(urllib.request.Request(srv.address, data=body, method="POST"),
                                                  timeout=10).read())
            assert r["prediction"] == lab and len(r["probability"]) == 2


def test_distributed_serving_reuse_port(tmp_path):
    """Two worker processes share one port via SO_REUSEPORT (reference DistributedHTTPSource);
    every reply is correct and carries the id of the worker that scored it."""
    import json
    import socket
    import urllib.request

    import numpy as np

    from synapseml_amd.core import DataFrame
    from synapseml_amd.io.serve_model import DistributedServing
    from synapseml_amd.lightgbm import LightGBMClassifier

    rng = np.random.default_rng(1)
    X = rng.standard_normal((400, 4))
    y = (X[:, 1] > 0).astype(float)
    LightGBMClassifier(numIterations=8, numLeaves=7, deviceType="cpu").fit(
        DataFrame({"features": X, "label": y})).save(str(tmp_path / "m"))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    seen = set()
    with DistributedServing(str(tmp_path / "m"), 2, port, output_cols="prediction") as d:
        for i in range(40):
            body = json.dumps({"features": X[i].tolist()}).encode()
            resp = urllib.request.urlopen(urllib.request.Request(d.address, data=body, method="POST"), timeout=20)
            seen.add(resp.headers["X-Served-By"])
            assert json.loads(resp.read())["prediction"] == y[i]
    assert seen <= {"0", "1"} and seen
    assert all(p.poll() is not None for p in d.procs)
