"""Continuous-mode serving (io/streaming.py; reference HTTPSourceV2 / HTTPSinkV2): per-request partition
tasks, epochs committed to a checkpoint location, crashed-task replay, restart on the same checkpoint."""
import json
import os
import threading
import urllib.request

import numpy as np
import pytest

from synapseml_amd.io import read_stream
from synapseml_amd.io.serving import make_reply, parse_request
from synapseml_amd.io.streaming import ContinuousServingServer, _interval_ms


def _post(url, payload, timeout=30):
    req = urllib.request.Request(url, data=json.dumps(payload).encode(), headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return r.status, r.read().decode()


def _double(df):
    p = parse_request(df, {"x": float})
    return make_reply(p.withColumn("y", np.asarray(p["x"], float) * 2), "y")


def test_trigger_interval_parsing():
    assert _interval_ms("1 second") == 1000.0 and _interval_ms("250 milliseconds") == 250.0
    assert _interval_ms("2 minutes") == 120000.0 and _interval_ms(40) == 40.0
    with pytest.raises(ValueError):
        _interval_ms("soon")


def test_continuous_query_answers_each_request_and_commits_epochs(tmp_path):
    ckpt = str(tmp_path / "ckpt")
    q = (read_stream().continuous_server().address("127.0.0.1", 0, "dbl").option("numPartitions", 3).load()
         .map(_double)
         .write_stream().continuous_server().reply_to("dbl").option("checkpointLocation", ckpt)
         .queryName("doubler").trigger(continuous="100 milliseconds").start())
    try:
        out = {}

        def hit(i):
            out[i] = _post(q.address, {"x": i})

        ths = [threading.Thread(target=hit, args=(i,)) for i in range(40)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert all(out[i] == (200, str(float(2 * i))) for i in range(40)), out
        srv = q.server
        assert set(srv.batch_sizes) <= {1} or not srv.batch_sizes  # no micro-batches in continuous mode
        import time

        deadline = time.time() + 10
        while time.time() < deadline and not srv.committed:
            time.sleep(0.05)
        assert srv.committed and q.lastProgress["epoch"] == srv.committed[-1]
        assert sum(p["numInputRows"] for p in q.recentProgress) <= 40
        commits = sorted(int(n) for n in os.listdir(os.path.join(ckpt, "commits")) if n.isdigit())
        assert commits == sorted(srv.committed)
        assert os.path.exists(os.path.join(ckpt, "offsets", str(commits[0])))
    finally:
        q.stop()
    assert not q.isActive and q.awaitTermination(0.1)


def test_crashed_task_replays_its_epoch(tmp_path):
    """A transform that raises on the first attempt of a request 'crashes' the partition task; the restarted
    task replays the epoch's unanswered requests, so the client still gets the right reply."""
    seen = {}
    lock = threading.Lock()

    def flaky(df):
        p = parse_request(df, {"x": float})
        x = float(p["x"][0])
        with lock:
            seen[x] = seen.get(x, 0) + 1
            first = seen[x] == 1
        if x == 7.0 and first:
            raise RuntimeError("executor lost")
        return make_reply(p.withColumn("y", np.asarray(p["x"], float) + 1), "y")

    srv = ContinuousServingServer(flaky, api="f", num_partitions=2, epoch_length_ms=50,
                                  checkpoint_location=str(tmp_path)).start()
    try:
        assert _post(srv.address, {"x": 7}) == (200, "8.0")
        assert _post(srv.address, {"x": 1}) == (200, "2.0")
        assert seen[7.0] == 2 and sum(srv.task_attempts.values()) == 1
    finally:
        srv.stop()


def test_always_failing_request_gets_500_after_max_task_failures():
    def bad(df):
        raise ValueError("poison")

    srv = ContinuousServingServer(bad, api="b", num_partitions=1, epoch_length_ms=50, max_task_failures=3).start()
    try:
        with pytest.raises(urllib.error.HTTPError) as ei:
            _post(srv.address, {"x": 1})
        assert ei.value.code == 500
        assert srv.task_attempts[0] == 3
    finally:
        srv.stop()


def test_restart_on_same_checkpoint_resumes_epochs(tmp_path):
    ckpt = str(tmp_path / "ck")
    import time

    s1 = ContinuousServingServer(_double, api="r", num_partitions=1, epoch_length_ms=30, checkpoint_location=ckpt).start()
    try:
        assert _post(s1.address, {"x": 2}) == (200, "4.0")
        deadline = time.time() + 10
        while time.time() < deadline and len(s1.committed) < 2:
            time.sleep(0.02)
        last = max(s1.committed)
    finally:
        s1.stop()
    s2 = ContinuousServingServer(_double, api="r", num_partitions=1, epoch_length_ms=30, checkpoint_location=ckpt)
    try:
        assert s2.start_epoch == last + 1 >= 2
        s2.start()
        assert _post(s2.address, {"x": 5}) == (200, "10.0")
    finally:
        s2.stop()


def test_micro_batch_builder_and_validation():
    q = (read_stream().server().address("127.0.0.1", 0, "mb").load().map(_double)
         .write_stream().server().reply_to("mb").trigger(processingTime="5 milliseconds").start())
    try:
        assert _post(q.address, {"x": 3}) == (200, "6.0")
    finally:
        q.stop()
    s = read_stream().continuous_server().address("127.0.0.1", 0, "c").load()
    with pytest.raises(ValueError, match="replyTo"):
        s.write_stream().reply_to("other").start()
    with pytest.raises(ValueError, match="continuous"):
        s.write_stream().continuous_server().trigger(processingTime="1 second").start()


def test_serve_model_cli_continuous_mode(tmp_path):
    """serve_model --mode continuous: the deployable entry point (and the helm chart's command) runs the
    continuous server on a saved pipeline."""
    import subprocess
    import sys
    import time

    from synapseml_amd.core.dataframe import DataFrame as DF
    from synapseml_amd.lightgbm import LightGBMRegressor
    from synapseml_amd.parallel.runtime import find_open_port

    rng = np.random.default_rng(0)
    X = rng.standard_normal((400, 3))
    m = LightGBMRegressor(numIterations=3).fit(DF({"features": X, "label": X[:, 0]}))
    m.save(str(tmp_path / "m"))
    port = find_open_port(24100)
    p = subprocess.Popen([sys.executable, "-m", "synapseml_amd.io.serve_model", "--model", str(tmp_path / "m"),
                          "--port", str(port), "--host", "127.0.0.1", "--mode", "continuous", "--epoch-ms", "50",
                          "--checkpoint-location", str(tmp_path / "ck")], stdout=subprocess.PIPE, text=True)
    try:
        line = p.stdout.readline()
        assert "serving" in line, line
        code, body = _post(f"http://127.0.0.1:{port}/", {"features": [0.5, 0.0, 0.0]})
        assert code == 200 and "prediction" in body
        deadline = time.time() + 10
        while time.time() < deadline and not os.path.isdir(tmp_path / "ck" / "commits"):
            time.sleep(0.05)
        assert os.listdir(tmp_path / "ck" / "commits")
    finally:
        p.terminate()
        p.wait(20)


def test_helm_chart_renders_both_modes():
    """The chart's templates reference only values that exist (a tiny renderer for the {{ .Values.x }} /
    if / range subset the chart uses - helm itself is not in this image)."""
    import re

    import yaml

    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "helm", "synapseml-amd")
    values = yaml.safe_load(open(os.path.join(root, "values.yaml")))
    chart = yaml.safe_load(open(os.path.join(root, "Chart.yaml")))
    assert chart["name"] == "synapseml-amd"
    for t in os.listdir(os.path.join(root, "templates")):
        src = open(os.path.join(root, "templates", t)).read()
        for ref in re.findall(r"\.Values\.([\w.]+)", src):
            cur = values
            for k in ref.split("."):
                assert isinstance(cur, dict) and k in cur, f"{t}: .Values.{ref} missing"
                cur = cur[k]
        assert src.count("{{- if") + src.count("{{ if") == src.count("{{- end") + src.count("{{ end") - \
            src.count("{{- range")


def test_serve_model_rejects_continuous_with_workers():
    """Continuous mode keeps epochs/offsets per process: --workers > 1 (micro-batch workers only) with
    --mode continuous is refused instead of silently dropping the continuous options."""
    from synapseml_amd.io import serve_model

    with pytest.raises(SystemExit) as e:
        serve_model.main(["--model", "/nonexistent", "--workers", "2", "--mode", "continuous"])
    assert e.value.code == 2
