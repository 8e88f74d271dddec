"""The multi-GPU data plane executed on one MI355X (RcclComm and the VW weight allreduce had
never run on hardware). A world-1 RCCL communicator runs every collective for real (ncclAllReduce on the
engine stream), and SML_GBDT_COMM_WORLD1=1 makes the GBDT backend take its full data-parallel path on it:
one histogram allreduce per split, device-timed (hipEvents), with the polling wait that turns a failed
collective into a CommError."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _gbdt():
    from synapseml_amd.ops import native

    return native.gbdt()


def _rccl_world1():
    import torch

    g = _gbdt()
    return g.rccl_comm(g.rccl_unique_id(), 0, 1, torch.cuda.current_device())


def test_rccl_world1_device_and_host_allreduce():
    g = _gbdt()
    c = _rccl_world1()
    assert (c.rank, c.world) == (0, 1)
    x = np.linspace(-3.0, 5.0, 4099).tolist()
    out = g.comm_device_allreduce(c, x, 3)  # 3 back-to-back ncclAllReduce on the device buffer
    np.testing.assert_array_equal(np.asarray(out), np.asarray(x))
    h = np.arange(7, dtype=np.float64)
    c.allreduce_host(h)  # staged through the device
    np.testing.assert_array_equal(h, np.arange(7, dtype=np.float64))
    assert g.comm_device_allreduce_us(c, 2 * 7168 + 2, 20) > 0.0


def _data(n=120000, f=10, seed=4):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, f)).astype(np.float32)
    y = (X[:, 0] + X[:, 1] * X[:, 2] + 0.5 * rng.standard_normal(n) > 0).astype(np.float32)
    return X, y


def _train(X, y, comm, iters=8):
    g = _gbdt()
    p = "objective=binary num_leaves=31 learning_rate=0.1 device_type=gpu"
    ref = g.DatasetReference.from_sample(X[:50000].astype(np.float64), len(X), p, [f"f{i}" for i in range(X.shape[1])])
    ds = g.Dataset(ref, len(X))
    ds.push_dense_gpu(X, 0)
    ds.set_label(y)
    b = g.Booster(ds, p, comm)
    for _ in range(iters):
        b.update()
    b.synchronize()
    return b


def test_gbdt_data_parallel_path_on_world1_rccl(monkeypatch):
    """Every split's histogram goes through ncclAllReduce (identity at world 1): same trees as the
    single-process path, and the device-timed comm time is reported."""
    X, y = _data()
    base = _train(X, y, None)
    monkeypatch.setenv("SML_GBDT_COMM_WORLD1", "1")
    c = _rccl_world1()
    dist = _train(X, y, c)
    s = dist.stats()
    # one allreduce per histogram: the root + one smaller child per further split (30 splits of 31 leaves)
    assert s["comm_calls"] >= 8 * 2 and s["comm_calls"] <= 8 * 31, s
    assert s["comm_ms"] >= 0.0, s
    split = lambda m: [l for l in m.splitlines() if l.startswith(("split_feature=", "threshold=", "leaf_count="))]
    assert split(dist.save_model_string()) == split(base.save_model_string())
    np.testing.assert_allclose(dist.predict(X[:5000].astype(np.float64), 0, 0, -1),
                               base.predict(X[:5000].astype(np.float64), 0, 0, -1), rtol=1e-12, atol=1e-12)


def test_vw_gpu_allreduce_average_world1():
    """GpuSgd::AllReduceAverage on a world-1 RCCL communicator (weighted ncclAllReduce of the touched
    blocks, divided by the summed weight): the exported model is unchanged and the sync moved bytes."""
    from synapseml_amd.ops import native

    vw = native.load("_vw")
    cfg = vw.GpuSgdConfig()
    cfg.bits = 16
    cfg.loss = 1
    sgd = vw.GpuSgd(cfg, 0)
    rng = np.random.default_rng(0)
    n, k = 4000, 8
    idx = rng.integers(0, 1 << 16, size=n * k).astype(np.uint32)
    val = rng.standard_normal(n * k).astype(np.float32)
    ip = np.arange(0, n * k + 1, k, dtype=np.int64)
    lab = (rng.random(n) > 0.5).astype(np.float32) * 2 - 1
    sgd.learn(ip, idx, val, lab, None, 64)
    m0 = sgd.export_model("--loss_function logistic -b 16")
    p0 = sgd.predict(ip, idx, val)
    assert np.abs(p0).sum() > 0
    comm = vw.nccl_comm(vw.nccl_unique_id(), 0, 1)
    sgd.allreduce_average(comm)
    assert sgd.last_sync_bytes > 0 and sgd.last_sync_blocks > 0
    np.testing.assert_allclose(sgd.predict(ip, idx, val), p0, rtol=1e-6, atol=1e-6)
    assert len(sgd.export_model("--loss_function logistic -b 16")) == len(m0)


def test_vw_gpu_2p30_table_sync_and_export_keep_host_rss_flat():
    """A 2^30-slot table (16 GiB in HBM): learning, a world-1 RCCL sync and a model export only move
    the touched blocks / nonzeros through the host - the process RSS does not grow by the table size."""
    import psutil

    from synapseml_amd.ops import native

    vw = native.load("_vw")
    cfg = vw.GpuSgdConfig()
    cfg.bits = 30
    cfg.loss = 1
    proc = psutil.Process()
    sgd = vw.GpuSgd(cfg, 0)
    rss0 = proc.memory_info().rss
    rng = np.random.default_rng(1)
    n, k = 20000, 16
    vocab = rng.integers(0, 1 << 32, size=5000, dtype=np.uint64).astype(np.uint32)  # 5000 hashed features
    idx = vocab[rng.integers(0, len(vocab), size=n * k)]
    val = np.ones(n * k, np.float32)
    ip = np.arange(0, n * k + 1, k, dtype=np.int64)
    lab = (rng.random(n) > 0.5).astype(np.float32) * 2 - 1
    sgd.learn(ip, idx, val, lab, None, 1024)
    comm = vw.nccl_comm(vw.nccl_unique_id(), 0, 1)
    sgd.allreduce_average(comm)
    # touched blocks only: at most one 4096-slot block per distinct feature, a sliver of the 2^18 blocks
    assert 0 < sgd.last_sync_blocks <= len(vocab)
    assert sgd.last_sync_bytes <= len(vocab) * 4096 * 20 + (1 << 18)
    model = sgd.export_model("--loss_function logistic -b 30")
    assert len(model) < 36 * len(vocab) + 4096  # the nonzeros (<= 3 per touched slot, 12 B each) + header
    grown = proc.memory_info().rss - rss0
    assert grown < (2 << 30), f"host RSS grew by {grown / 2**30:.2f} GiB"
    del sgd


def _train_p(X, y, comm, p, iters=8):
    g = _gbdt()
    ref = g.DatasetReference.from_sample(X[:50000].astype(np.float64), len(X), p, [f"f{i}" for i in range(X.shape[1])])
    ds = g.Dataset(ref, len(X))
    ds.push_dense_gpu(X, 0)
    ds.set_label(y)
    b = g.Booster(ds, p, comm)
    for _ in range(iters):
        b.update()
    b.synchronize()
    return b


@pytest.mark.parametrize("top_k", [1, 2, 20])
def test_gbdt_voting_parallel_on_world1_rccl(monkeypatch, top_k):
    """Device PV-Tree (tree_learner=voting): local search, vote, vote allreduce, selection, selected-feature
    histogram allreduce, global search - every kernel and both ncclAllReduce calls per split executed.
    At world 1 the local gains are the global ones, so the best feature is always among the voted ones and
    the trees equal the single-process trees for any top_k (top_k=1 reduces 2 of the 10 features)."""
    X, y = _data()
    p = "objective=binary num_leaves=31 learning_rate=0.1 device_type=gpu"
    base = _train_p(X, y, None, p)
    monkeypatch.setenv("SML_GBDT_COMM_WORLD1", "1")
    c = _rccl_world1()
    vote = _train_p(X, y, c, p + f" tree_learner=voting top_k={top_k}")
    s = vote.stats()
    # two collectives per split search: the root + one per further split
    assert s["comm_calls"] >= 8 * 2 * 2 and s["comm_calls"] <= 8 * 2 * 31, s
    split = lambda m: [l for l in m.splitlines() if l.startswith(("split_feature=", "threshold=", "leaf_count="))]
    assert split(vote.save_model_string()) == split(base.save_model_string())
    np.testing.assert_allclose(vote.predict(X[:5000].astype(np.float64), 0, 0, -1),
                               base.predict(X[:5000].astype(np.float64), 0, 0, -1), rtol=1e-12, atol=1e-12)
