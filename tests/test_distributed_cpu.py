"""Data-parallel training across 2 processes (gloo) must match one process on
the union of the shards when both use the same bin boundaries."""
import os

import numpy as np
import pytest

from synapseml_amd.core import DataFrame
from synapseml_amd.lightgbm import LightGBMClassifier, LightGBMRegressor
from synapseml_amd.parallel.runtime import distributed_fit, run_partitions


def _allreduce_task(part, rank, world):
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(part.count())])
    dist.all_reduce(t)
    return float(t.item())


def test_run_partitions_rendezvous():
    df = DataFrame({"x": np.arange(10.0)}, num_partitions=4)
    res = run_partitions(_allreduce_task, df, num_workers=2)
    assert res == [10.0, 10.0]


@pytest.mark.parametrize("est_cls", [LightGBMClassifier, LightGBMRegressor])
def test_data_parallel_matches_single_process(est_cls):
    rng = np.random.default_rng(0)
    n = 6000
    X = rng.standard_normal((n, 8))
    y = (X[:, 0] + X[:, 1] * X[:, 2] > 0).astype(float)
    if est_cls is LightGBMRegressor:
        y = X[:, 0] * 2 + X[:, 1] ** 2
    df = DataFrame({"features": X, "label": y}, num_partitions=2)
    base = est_cls(deviceType="cpu", numIterations=8, numThreads=1)
    base.fit(df)
    ref = base._last_reference
    single = est_cls(deviceType="cpu", numIterations=8, numThreads=1, referenceDataset=ref).fit(df)
    dist_model = distributed_fit(est_cls(deviceType="cpu", numIterations=8, numThreads=1, referenceDataset=ref), df,
                                 num_workers=2)
    col = "probability" if est_cls is LightGBMClassifier else "prediction"
    a = single.transform(df)[col]
    b = dist_model.transform(df)[col]
    np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6)
    def splits(m):
        return [l for l in m.getNativeModel().splitlines() if l.startswith(("split_feature=", "threshold="))]

    assert splits(single) == splits(dist_model)


def _sleepy_allreduce(part, rank, world):
    import torch
    import torch.distributed as dist

    t = torch.ones(1)
    dist.all_reduce(t)  # a dead peer would leave this blocked until the timeout
    return float(t.item())


@pytest.mark.parametrize("kind", ["raise", "crash_after_init", "crash_before"])
def test_rank_failure_aborts_fast(monkeypatch, kind):
    """A failing / dying rank aborts the whole job promptly with a driver-visible error (fault injection,
    SURVEY §5.3) instead of blocking the other ranks in collectives until the timeout."""
    import time

    monkeypatch.setenv("SML_FAULT_INJECT", f"1:{kind}")
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match="worker 1"):
        run_partitions(_sleepy_allreduce, DataFrame({"x": np.arange(4)}, num_partitions=2), num_workers=2,
                       timeout_s=300)
    assert time.monotonic() - t0 < 120


def test_rank_death_mid_fit_fails_every_rank(monkeypatch):
    """A rank that dies inside the boosting loop must fail the fit on the surviving ranks with a CommError
    (the histogram allreduce cannot complete) - never a warning plus a truncated model."""
    import time

    rng = np.random.default_rng(0)
    X = rng.standard_normal((4000, 6))
    y = (X[:, 0] > 0).astype(float)
    df = DataFrame({"features": X, "label": y}, num_partitions=2)
    monkeypatch.setenv("SML_FAULT_INJECT", "1:crash_iter=3")
    t0 = time.monotonic()
    with pytest.raises(RuntimeError) as ei:
        # fail_fast=False: the driver lets the survivor run to its own end, so what it raised is reported
        distributed_fit(LightGBMClassifier(deviceType="cpu", numIterations=20, numThreads=1, timeout=60.0), df,
                        num_workers=2, timeout_s=300, fail_fast=False)
    msg = str(ei.value)
    assert "worker 1: exit code 19" in msg, msg[-2000:]
    assert "worker 0: CommError" in msg, msg[-2000:]
    assert time.monotonic() - t0 < 200


def test_empty_partition_rank_still_joins(monkeypatch):
    monkeypatch.setenv("SML_FAULT_INJECT", "1:empty")
    out = run_partitions(_allreduce_task, DataFrame({"x": np.arange(8.0)}, num_partitions=2), num_workers=2)
    assert len(out) == 2


def test_voting_parallel_two_ranks():
    """voting_parallel (PV-Tree): with topK >= #features every feature is reduced, so the
    model equals data-parallel; with topK=1 only voted features are reduced and the model still learns."""
    from sklearn.metrics import roc_auc_score

    rng = np.random.default_rng(1)
    n = 6000
    X = rng.standard_normal((n, 8))
    y = (X[:, 0] + 0.8 * X[:, 1] * X[:, 2] - 0.5 * X[:, 3] > 0).astype(float)
    df = DataFrame({"features": X, "label": y}, num_partitions=2)
    ref = LightGBMClassifier(deviceType="cpu", numIterations=1).fit(df) and None
    base = LightGBMClassifier(deviceType="cpu", numIterations=1)
    base.fit(df)
    ref = base._last_reference
    kw = dict(deviceType="cpu", numIterations=10, numThreads=1, referenceDataset=ref)
    data_m = distributed_fit(LightGBMClassifier(**kw), df, num_workers=2)
    vote_all = distributed_fit(LightGBMClassifier(parallelism="voting_parallel", topK=8, **kw), df, num_workers=2)
    vote_1 = distributed_fit(LightGBMClassifier(parallelism="voting_parallel", topK=1, **kw), df, num_workers=2)
    splits = lambda m: [l for l in m.getNativeModel().splitlines() if l.startswith(("split_feature=", "threshold="))]
    assert splits(vote_all) == splits(data_m)
    assert "[tree_learner: voting]" in vote_1.getNativeModel()
    p = vote_1.transform(df)["probability"][:, 1]
    assert roc_auc_score(y, p) > 0.85


def _port_task(part, rank, world):
    import os

    import torch
    import torch.distributed as dist

    t = torch.ones(1)
    dist.all_reduce(t)
    return int(os.environ["MASTER_PORT"]), float(t.item())


def test_network_init_retries_with_backoff(monkeypatch):
    """NetworkInit retry semantics (NetworkManager.scala:195-218): a rank whose first rendezvous fails makes
    the driver relaunch every rank after a delay; with no retries left the job fails naming the cause."""
    import time

    monkeypatch.setenv("SML_FAULT_INJECT", "1:netinit_fail")
    df = DataFrame({"x": np.arange(4)}, num_partitions=2)
    t0 = time.monotonic()
    res = run_partitions(_port_task, df, num_workers=2, initial_delay_s=0.2)
    assert [r[1] for r in res] == [2.0, 2.0]
    assert time.monotonic() - t0 < 120
    with pytest.raises(RuntimeError, match="network init failed after 0 retries"):
        run_partitions(_port_task, df, num_workers=2, network_retries=0)


def test_listen_port_semantics():
    """defaultListenPort: first open port at or above it (findOpenPort); driverListenPort: used as given,
    an error when taken (LightGBMParams.scala:39-49)."""
    import socket

    from synapseml_amd.parallel.runtime import find_open_port, rendezvous_port

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        s.listen(1)
        busy = s.getsockname()[1]
        assert find_open_port(busy) > busy
        with pytest.raises(RuntimeError, match="already in use"):
            rendezvous_port(driver_listen_port=busy)
    free = find_open_port(busy)
    assert rendezvous_port(driver_listen_port=free) == free
    with pytest.raises(ValueError):
        find_open_port(70000)
    df = DataFrame({"x": np.arange(4)}, num_partitions=2)
    res = run_partitions(_port_task, df, num_workers=2, port=free)
    assert [r[0] for r in res] == [free, free]


def test_distributed_fit_uses_estimator_ports():
    from synapseml_amd.parallel.runtime import find_open_port

    rng = np.random.default_rng(1)
    X = rng.standard_normal((400, 4))
    y = (X[:, 0] > 0).astype(float)
    df = DataFrame({"features": X, "label": y}, num_partitions=2)
    port = find_open_port(23000)
    m = distributed_fit(LightGBMClassifier(numIterations=3, driverListenPort=port), df, num_workers=2)
    assert m.getNativeModel()


def _retry_task(part, rank, world):
    from synapseml_amd.parallel.distributed import init_with_retries

    calls = {"n": 0}

    def make():
        calls["n"] += 1
        if rank == 1 and calls["n"] == 1:
            raise OSError("transient bootstrap failure")
        return f"comm{calls['n']}"

    c = init_with_retries(make, "test comm", delay_s=0.05)
    try:
        init_with_retries(lambda: (_ for _ in ()).throw(OSError("down")) if rank == 0 else "ok", "dead comm",
                          retries=1, delay_s=0.01)
        failed = None
    except RuntimeError as e:
        failed = str(e)
    return c, calls["n"], failed


def test_collective_init_retries_together():
    """A communicator that fails to initialise on one rank is retried on every rank together; when it keeps
    failing, every rank raises with the failing rank named."""
    res = run_partitions(_retry_task, DataFrame({"x": np.arange(4)}, num_partitions=2), num_workers=2)
    assert [r[0] for r in res] == ["comm2", "comm2"] and [r[1] for r in res] == [2, 2]
    assert all(r[2] and "rank 0: OSError: down" in r[2] and "after 1 retries" in r[2] for r in res)


def _p2p_decision_task(part, rank, world):
    import os

    from synapseml_amd.parallel import distributed as D

    sentinel = object()
    if rank == 1:
        os.environ["LOCAL_WORLD_SIZE"] = "1"  # this rank believes it is alone on its node
    c = D.maybe_p2p(sentinel, -1)
    return c is sentinel, dict(D.p2p_status)


def _p2p_disabled_on_one_rank(part, rank, world):
    import os

    from synapseml_amd.parallel import distributed as D

    sentinel = object()
    if rank == 0:
        os.environ["SML_GBDT_P2P"] = "0"
    c = D.maybe_p2p(sentinel, -1)
    return c is sentinel, dict(D.p2p_status)


@pytest.mark.parametrize("task", [_p2p_decision_task, _p2p_disabled_on_one_rank])
def test_p2p_fallback_is_collective(task):
    """maybe_p2p's fallback (distributed.py): when any rank sees a multi-node layout (LOCAL_WORLD_SIZE !=
    world) or has P2P disabled, EVERY rank keeps the plain RCCL/host communicator - no rank enters the IPC
    self-test alone."""
    res = run_partitions(task, DataFrame({"x": np.arange(4)}, num_partitions=2), num_workers=2)
    assert all(kept for kept, _ in res)
    assert all(st.get("active") is False and "multi-node" in st.get("reason", "") for _, st in res)


class _FakeComm:
    def __init__(self, tag):
        self.tag, self.aborted = tag, False

    def abort(self):
        self.aborted = True


def _prepare_failure_task(part, rank, world):
    """prepare() fails on rank 1 in the first attempt; make() is collective (a gloo barrier stands in for
    ncclCommInitRank). Without the readiness agreement rank 0 would sit in the barrier forever."""
    import torch.distributed as dist

    from synapseml_amd.parallel.distributed import init_with_retries

    st = {"prep": 0, "make": 0, "built": []}

    def prepare():
        st["prep"] += 1
        if rank == 1 and st["prep"] == 1:
            raise OSError("device not ready")
        return f"uid{st['prep']}" if rank == 0 else None

    def make(uid):
        st["make"] += 1
        dist.barrier()  # collective: both ranks must be inside
        c = _FakeComm(uid)
        st["built"].append(c)
        if rank == 0 and st["make"] == 1 and uid == "uid-never":
            raise OSError("unreachable")
        return c

    c = init_with_retries(make, "collective comm", delay_s=0.01, prepare=prepare)
    return c.tag, st["prep"], st["make"]


def _make_failure_aborts_task(part, rank, world):
    """make() fails on rank 1 after rank 0 built its half: rank 0 must abort its communicator before the
    retry (a half-built RCCL communicator is never left alive)."""
    from synapseml_amd.parallel.distributed import init_with_retries

    built = []

    def make(uid):
        c = _FakeComm(uid)
        built.append(c)
        if rank == 1 and len(built) == 1:
            raise OSError("init failed inside the collective")
        return c

    c = init_with_retries(make, "collective comm", delay_s=0.01, prepare=lambda: "uid")
    return [b.aborted for b in built], c.aborted


def test_collective_init_agrees_on_readiness_before_entering():
    res = run_partitions(_prepare_failure_task, DataFrame({"x": np.arange(4)}, num_partitions=2), num_workers=2,
                         timeout_s=120)
    # the uid is rank 0's second prepare() result on every rank; make() was entered once, together
    assert res == [("uid2", 2, 1), ("uid2", 2, 1)]


def test_failed_collective_init_aborts_peers_communicators():
    res = run_partitions(_make_failure_aborts_task, DataFrame({"x": np.arange(4)}, num_partitions=2),
                         num_workers=2, timeout_s=120)
    assert res[0] == ([True, False], False)
    assert res[1] == ([False, False], False)  # rank 1's first make raised before returning a communicator


def test_comm_cache_evicts_aborted(monkeypatch):
    from synapseml_amd.parallel import distributed as D

    c = _FakeComm("x")
    D._comm_cache[("host", 2)] = c
    D.evict_comm("test")
    assert c.aborted and not D._comm_cache


def test_bench_launches_n_ranks_on_cpu():
    """bench.py --gpus 2 started without a torchrun environment launches 2 ranks itself (child process)
    and the JSON line reports a 2-rank data-parallel world; a rank whose world != --gpus refuses."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--device", "cpu",
                          "--rows", "20000", "--iterations", "3", "--steps", "1", "--warmup", "0"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["config"]["parallelism"] == "dp2" and rec["config"]["world"] == 2
    assert rec["config"]["data_plane_world"] == 2 and rec["config"]["global_batch"] == 40000
    env1 = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    bad = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--device", "cpu",
                          "--rows", "2000", "--iterations", "1", "--steps", "1", "--warmup", "0"],
                         env=env1, capture_output=True, text=True, timeout=120)
    assert bad.returncode != 0 and "WORLD_SIZE=1" in bad.stderr


def _checksum_task(part, rank, world):
    from synapseml_amd.core.linalg import CsrColumn

    f = part["f"]
    csr = part["sv"]
    return (float(np.asarray(f, np.float64).sum()), str(f.dtype), f.shape, isinstance(csr, CsrColumn),
            float(csr.values.sum()) if isinstance(csr, CsrColumn) else None, list(part["s"]), float(part["y"].sum()))


def test_partitions_reach_workers_through_shared_memory():
    """Partition hand-off (runtime._share_partition): numeric and CSR columns arrive as shared-memory views with
    their dtype / shape, object columns pickled; the driver unlinks every segment afterwards."""
    import glob

    from synapseml_amd.core.linalg import CsrColumn

    before = set(glob.glob("/dev/shm/psm_*"))
    rng = np.random.default_rng(0)
    f = rng.standard_normal((1000, 7)).astype(np.float32)
    ip = np.arange(0, 2001, 2, dtype=np.int64)
    sv = CsrColumn(ip, rng.integers(0, 50, 2000).astype(np.int32), rng.random(2000), 50)
    s = np.array([f"r{i}" for i in range(1000)], dtype=object)
    df = DataFrame({"f": f, "sv": sv, "s": s, "y": np.arange(1000.0)}, num_partitions=2)
    res = run_partitions(_checksum_task, df, num_workers=2)
    for r, (a, b) in enumerate(df.partition_bounds()):
        fs, dt, shape, is_csr, vs, strs, ys = res[r]
        assert dt == "float32" and shape == (b - a, 7) and is_csr
        np.testing.assert_allclose(fs, f[a:b].astype(np.float64).sum(), rtol=1e-6)
        np.testing.assert_allclose(vs, sv[a:b].values.sum())
        assert strs == list(s[a:b]) and ys == float(np.arange(a, b).sum())
    if not os.environ.get("PYTEST_XDIST_WORKER"):  # (other workers' jobs create segments concurrently)
        assert set(glob.glob("/dev/shm/psm_*")) <= before


def test_partitions_fall_back_to_pickle_when_shm_is_small(monkeypatch):
    """A /dev/shm without room for the partition (Docker's 64 MB default) must not SIGBUS the driver: the
    partition travels pickled, with the same contents."""
    from synapseml_amd.parallel import runtime as R

    monkeypatch.setenv("SML_SHM_HANDOFF", "0")
    assert not R._shm_fits(1)
    rng = np.random.default_rng(1)
    f = rng.standard_normal((400, 3)).astype(np.float32)
    from synapseml_amd.core.linalg import CsrColumn

    ip = np.arange(0, 801, 2, dtype=np.int64)
    sv = CsrColumn(ip, rng.integers(0, 9, 800).astype(np.int32), rng.random(800), 9)
    s = np.array([f"r{i}" for i in range(400)], dtype=object)
    df = DataFrame({"f": f, "sv": sv, "s": s, "y": np.arange(400.0)}, num_partitions=2)
    desc, shm = R._share_partition(df.partitions()[0])
    assert shm is None
    res = run_partitions(_checksum_task, df, num_workers=2)
    a, b = df.partition_bounds()[1]
    assert res[1][1] == "float32" and res[1][2] == (b - a, 3) and res[1][6] == float(np.arange(a, b).sum())


def _lgbm_df(n=4000, parts=2, seed=3):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, 6))
    y = (X[:, 0] - X[:, 1] * X[:, 2] > 0).astype(float)
    return DataFrame({"features": X, "label": y}, num_partitions=parts)


def _splits(m):
    return [l for l in m.getNativeModel().splitlines() if l.startswith(("split_feature=", "threshold=", "leaf_value="))]


def test_num_tasks_fans_out_like_distributed_fit():
    """LightGBMClassifier(numTasks=2).fit(df) runs 2 partition tasks itself (LightGBMBase.scala:449-456,
    608-628) and returns the main task's model: the same model as an explicit distributed_fit."""
    df = _lgbm_df()
    base = LightGBMClassifier(deviceType="cpu", numIterations=6, numThreads=1)
    base.fit(df.coalesce(1))
    ref = base._last_reference
    est = LightGBMClassifier(deviceType="cpu", numIterations=6, numThreads=1, referenceDataset=ref, numTasks=2,
                             useBarrierExecutionMode=True)
    fanned = est.fit(df)
    explicit = distributed_fit(LightGBMClassifier(deviceType="cpu", numIterations=6, numThreads=1,
                                                  referenceDataset=ref), df, num_workers=2)
    assert _splits(fanned) == _splits(explicit)
    tm = est.getTaskMeasures()
    assert len(tm) == 2 and all(t and "training_iterations_ms" in t[0] for t in tm)
    np.testing.assert_allclose(fanned.transform(df)["probability"], explicit.transform(df)["probability"])


def test_num_tasks_default_uses_executor_tasks(monkeypatch):
    """numTasks=0: min(executor tasks, partitions) (determineNumTasks); one executor task keeps the fit in
    this process, SML_EXECUTOR_TASKS=2 (two CPU executors) fans a 3-partition DataFrame out to 2 tasks."""
    from synapseml_amd.parallel import runtime as R

    df = _lgbm_df(parts=3)
    assert R.determine_num_tasks(0, df, use_gpu=False) == 1
    assert R.determine_num_tasks(5, df, use_gpu=False) == 5
    monkeypatch.setenv("SML_EXECUTOR_TASKS", "2")
    assert R.determine_num_tasks(0, df, use_gpu=False) == 2
    assert R.determine_num_tasks(0, df.coalesce(1), use_gpu=False) == 1
    calls = []
    real = R.fan_out

    def spy(fn, d, n, use_gpu, **kw):
        calls.append(n)
        return real(fn, d, n, use_gpu, **kw)

    monkeypatch.setattr(R, "fan_out", spy)
    m = LightGBMClassifier(deviceType="cpu", numIterations=3, numThreads=1).fit(df)
    assert calls == [2] and m.transform(df)["probability"].shape[0] == len(df)


def test_inert_params_warn(caplog):
    import logging

    df = _lgbm_df(n=600, parts=1)
    with caplog.at_level(logging.WARNING, logger="synapseml_amd.lightgbm"):
        LightGBMClassifier(deviceType="cpu", numIterations=2, dataTransferMode="bulk", chunkSize=5).fit(df)
    msgs = " ".join(r.getMessage() for r in caplog.records)
    assert "dataTransferMode" in msgs and "chunkSize" in msgs
    caplog.clear()
    with caplog.at_level(logging.WARNING, logger="synapseml_amd.lightgbm"):
        LightGBMClassifier(deviceType="cpu", numIterations=2).fit(df)
    assert not any("has no effect" in r.getMessage() for r in caplog.records)




class _ModelText:
    def __init__(self, est):
        self.est = est

    def __call__(self, part, rank, world):
        m = self.est.fit(part)
        return m.getNativeModel().split("parameters:")[0] if rank == 0 else None


@pytest.mark.parametrize("est_cls,extra", [(LightGBMClassifier, {}),
                                           (LightGBMRegressor, {"lambdaL2": 1.0}),
                                           (LightGBMClassifier, {"numLeaves": 63, "minDataInLeaf": 5})])
def test_n_ranks_give_the_1_rank_model_bitwise(est_cls, extra):
    """The fixed-point histograms travel as int64 with a scale built from global quantities only (global row
    count, global max |g| / max h), so 1, 2 and 4 ranks train byte-identical models on the same rows and bin
    boundaries (VerifyLightGBMClassifierStream.scala:95-101 checks the same for streaming vs bulk)."""
    rng = np.random.default_rng(5)
    n = 8000
    X = rng.standard_normal((n, 7))
    y = (X[:, 0] + X[:, 1] * X[:, 2] - 0.5 * X[:, 3] > 0).astype(float)
    if est_cls is LightGBMRegressor:
        y = X[:, 0] * 2 + X[:, 1] ** 2 + 0.1 * rng.standard_normal(n)
    kw = dict(deviceType="cpu", numIterations=6, numThreads=2, **extra)
    base = est_cls(**kw)
    df1 = DataFrame({"features": X, "label": y})
    one = base.fit(df1).getNativeModel().split("parameters:")[0]
    ref = base._last_reference
    for world in (2, 4):
        df = DataFrame({"features": X, "label": y}, num_partitions=world)
        txt = run_partitions(_ModelText(est_cls(referenceDataset=ref, **kw)), df, num_workers=world)[0]
        assert txt == one, f"world {world} model differs from the 1-rank model"


def _return_partition(part, rank, world):
    return part.withColumn("twice", np.asarray(part["id"]) * 2)


def test_worker_result_may_view_the_shared_partition():
    """A task result that keeps the partition's shared-memory columns (a transformed partition) is serialised
    before the worker unmaps the segment (it used to read unmapped memory and die after an empty result file,
    which the driver then reported as an unpickling error)."""
    df = DataFrame({"features": np.ones((60, 4), np.float32), "id": np.arange(60.0)}, num_partitions=3)
    res = run_partitions(_return_partition, df, num_workers=2)
    assert [r.count() for r in res] == [20, 40]
    assert np.concatenate([r["twice"] for r in res]).tolist() == (np.arange(60.0) * 2).tolist()
