"""Vowpal Wabbit-style estimators and models (reference: vw/.../
VowpalWabbitBase.scala, VowpalWabbitBaseLearner.scala, VowpalWabbitBaseSpark
.scala, VowpalWabbitClassifier.scala, VowpalWabbitRegressor.scala,
VowpalWabbitGeneric.scala, VowpalWabbitContextualBandit.scala,
VowpalWabbitBaseProgressive.scala).

Training: every partition/rank owns a native learner built from the VW
command line (passThroughArgs first, then the typed params); rows are
marshalled in columnar batches (no per-row JNI calls); at pass boundaries (and
``numSyncsPerPass`` times within a pass) the weight tables are averaged across
ranks with an allreduce (RCCL/gloo replaces VW's spanning tree,
VowpalWabbitClusterUtil.scala); rank 0's model is returned. ``splitCol``
training broadcasts the model per split and averages (mergeModels).
"""
from __future__ import annotations

import os
import re
import time
from typing import List, Optional

import numpy as np

from ..core.contracts import (HasFeaturesCol, HasLabelCol, HasPredictionCol, HasProbabilityCol,
                              HasRawPredictionCol, HasWeightCol)
from ..core.dataframe import DataFrame
from ..core.linalg import CsrColumn, DenseVector, SparseVector
from ..core.params import Param, TypeConverters as T
from ..core.pipeline import Estimator, Model, Transformer
from ..core.utils import ParamsStringBuilder, StopWatch
from ..ops import native
from ..parallel import distributed as D
from .featurizer import murmur_hash


def _vw():
    return native.load("_vw")


def _initial_model_bytes(model):
    """VowpalWabbitPythonBase.setInitialModel (reference vw/.../VowpalWabbitPythonBase.py:22-26) takes a fitted
    model; raw model bytes are accepted too"""
    if model is None or isinstance(model, (bytes, bytearray)):
        return None if model is None else bytes(model)
    get = getattr(model, "getModel", None)
    if get is None:
        raise TypeError(f"setInitialModel expects a fitted VowpalWabbit model or model bytes, got {type(model).__name__}")
    return bytes(get())


class VowpalWabbitBaseParams(HasFeaturesCol):
    passThroughArgs = Param("VW command line arguments passed", "", T.toString)
    additionalFeatures = Param("Additional feature columns", [], T.toListString)
    hashSeed = Param("Seed used for hashing", 0, T.toInt)
    numBits = Param("Number of bits used", 18, T.toInt)
    learningRate = Param("Learning rate", None, T.toFloat)
    powerT = Param("t power value", None, T.toFloat)
    l1 = Param("l_1 lambda", None, T.toFloat)
    l2 = Param("l_2 lambda", None, T.toFloat)
    interactions = Param("Interaction terms as specified by -q", [], T.toListString)
    ignoreNamespaces = Param("Namespaces to be ignored (first letter only)", None, T.toString)
    initialModel = Param("Initial model to start from", None, complex=True)
    numPasses = Param("Number of passes over the data", 1, T.toInt)
    numSyncsPerPass = Param("Number of times weights should be synchronized within each pass", 0, T.toInt)

    def setInitialModel(self, model):  # noqa: N802
        self.set("initialModel", _initial_model_bytes(model))
        return self
    useBarrierExecutionMode = Param("Use barrier execution mode, on by default.", True, T.toBoolean)
    splitCol = Param("The column to split on for inter-pass sync", None, T.toString)
    splitColValues = Param("Sorted values to use to select each split to train on", None)
    predictionIdCol = Param("The ID column returned for predictions", None, T.toString)
    deviceType = Param("cpu (exact sequential VW semantics) or gpu (hogwild mini-batch SGD on the MI355X)", "cpu",
                       T.toString)
    gpuBatchSize = Param("Mini-batch size of the GPU learner", 1024, T.toInt)


def build_args(est, extra: Optional[ParamsStringBuilder] = None) -> str:
    sb = ParamsStringBuilder(prefix="--", delimiter=" ")
    sb.append(est.getPassThroughArgs())
    sb.appendParamValueIfNotThere("hash_seed", est.getHashSeed())
    if "-b " not in (" " + sb.result + " "):
        sb.appendParamValueIfNotThere("bit_precision", est.getNumBits())
    if " -l " not in (" " + sb.result + " "):
        sb.appendParamValueIfNotThere("learning_rate", est.getLearningRate())
    sb.appendParamValueIfNotThere("power_t", est.getPowerT())
    sb.appendParamValueIfNotThere("l1", est.getL1())
    sb.appendParamValueIfNotThere("l2", est.getL2())
    sb.appendParamValueIfNotThere("ignore", est.getIgnoreNamespaces())
    for q in est.getInteractions() or []:
        if f"-q {q}" not in sb.result and f"--quadratic {q}" not in sb.result:
            sb.append(f"-q {q}")
    if extra is not None:
        sb.append(extra.result)
    sb.appendParamFlagIfNotThere("no_stdin")
    if est.getNumPasses() > 1:
        sb.appendParamValueIfNotThere("passes", est.getNumPasses())
        sb.appendParamFlagIfNotThere("holdout_off")
    return sb.result


def namespace_blocks(df: DataFrame, cols: List[str], hash_seed: int):
    """Columns -> [(featureGroup, indptr, indices, values)] for the native
    batch API. Dense vector columns get index = murmur(col, seed) + i, sparse
    vectors keep their (already hashed) indices (VowpalWabbitUtil.scala:11-40)."""
    blocks = []
    n = df.count()
    for c in cols:
        col = df[c]
        ns_hash = murmur_hash(c, hash_seed) & 0xFFFFFFFF
        group = c[0]
        if isinstance(col, CsrColumn):  # columnar sparse rows: zero-copy (indices are already hashed)
            ip, ind, val = col.csr()
            blocks.append((group, ip, ind.astype(np.uint32, copy=False), val.astype(np.float32, copy=False)))
            continue
        if isinstance(col, np.ndarray) and col.ndim == 2:
            width = col.shape[1]
            nz = col != 0
            indptr = np.concatenate([[0], np.cumsum(nz.sum(1))]).astype(np.int64)
            rr, cc = np.nonzero(nz)
            idx = ((cc.astype(np.uint64) + ns_hash) & 0xFFFFFFFF).astype(np.uint32)
            blocks.append((group, indptr, idx, col[rr, cc].astype(np.float32)))
            continue
        indptr = [0]
        ii, vv = [], []
        for v in col.tolist():
            if isinstance(v, SparseVector):
                ii.append(v.indices.astype(np.uint32))
                vv.append(v.values.astype(np.float32))
                indptr.append(indptr[-1] + len(v.indices))
            else:
                a = np.asarray(v.toArray() if isinstance(v, DenseVector) else v, dtype=np.float64)
                nzi = np.nonzero(a)[0]
                ii.append(((nzi.astype(np.uint64) + ns_hash) & 0xFFFFFFFF).astype(np.uint32))
                vv.append(a[nzi].astype(np.float32))
                indptr.append(indptr[-1] + len(nzi))
        blocks.append((group, np.asarray(indptr, np.int64),
                       np.concatenate(ii).astype(np.uint32) if ii else np.zeros(0, np.uint32),
                       np.concatenate(vv).astype(np.float32) if vv else np.zeros(0, np.float32)))
    assert all(len(b[1]) == n + 1 for b in blocks)
    return blocks


def _block_slice(blocks, a: int, b: int):
    out = []
    for g, ip, ii, vv in blocks:
        s, e = ip[a], ip[b]
        out.append((g, (ip[a:b + 1] - s).astype(np.int64), ii[s:e], vv[s:e]))
    return out


def _host_allreduce_f32(arr: np.ndarray) -> None:
    if D.world_size() <= 1:
        return
    import torch

    t = torch.from_numpy(arr)
    if D.backend() == "nccl":
        tt = t.cuda()
        D._dist().all_reduce(tt)
        arr[...] = tt.cpu().numpy()
    else:
        D._dist().all_reduce(t)


_nccl_cache: dict = {}


def _merged_csr(blocks, n: int, constant: bool):
    """Concatenate namespace blocks row-wise into one CSR (+ VW constant feature)."""
    counts = np.zeros(n, np.int64)
    for _, ip, _, _ in blocks:
        counts += np.diff(ip)
    if constant:
        counts += 1
    indptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    idx = np.empty(indptr[-1], np.uint32)
    val = np.empty(indptr[-1], np.float32)
    pos = indptr[:-1].copy()
    for _, ip, ii, vv in blocks:
        lens = np.diff(ip)
        rows = np.repeat(np.arange(n), lens)
        within = np.arange(len(ii)) - np.repeat(ip[:-1], lens)
        dst = pos[rows] + within
        idx[dst] = ii
        val[dst] = vv
        pos += lens
    if constant:
        idx[pos] = 11650396  # VW constant-feature hash
        val[pos] = 1.0
    return indptr, idx, val


_FNV_PRIME = np.uint32(16777619)


def _quadratic_pairs(args: str) -> List[str]:
    """Two-namespace interactions from -q / --quadratic / --interactions (VW command line)."""
    out = []
    for m in re.finditer(r"(?:^|\s)(?:-q|--quadratic|--interactions)(?:\s+|=)(\S+)", args):
        v = m.group(1)
        if len(v) != 2 or ":" in v:
            raise ValueError(f"deviceType='gpu' supports two-namespace interactions only; got {v!r}")
        out.append(v)
    return out


def _interaction_block(blocks, pair: str, n: int):
    """Host expansion of one quadratic interaction into a CSR block, with the
    native learner's hashing (vw_core.cpp ForEachFeature: (a * FNV) ^ b, value
    a.x * b.x; a namespace crossed with itself keeps pairs j >= i). The GPU
    kernel masks indices to num_bits <= 32, so 32-bit products are exact."""
    def last(g):
        found = [b for b in blocks if b[0] == g]
        return found[-1] if found else None

    A, B = last(pair[0]), last(pair[1])
    if A is None or B is None:
        return (pair, np.zeros(n + 1, np.int64), np.zeros(0, np.uint32), np.zeros(0, np.float32))
    same = A is B
    ia, a_idx, a_val = A[1], A[2], A[3]
    ib, b_idx, b_val = B[1], B[2], B[3]
    la, lb = np.diff(ia), np.diff(ib)
    npair = la * lb
    rows = np.repeat(np.arange(n), npair)
    k = np.arange(int(npair.sum())) - np.repeat(np.concatenate([[0], np.cumsum(npair)[:-1]]), npair)
    lbr = lb[rows]
    i = k // np.maximum(lbr, 1)
    j = k - i * lbr
    if same:
        keep = j >= i
        rows, i, j = rows[keep], i[keep], j[keep]
    ga, gb = ia[rows] + i, ib[rows] + j
    idx = (a_idx[ga].astype(np.uint32) * _FNV_PRIME) ^ b_idx[gb].astype(np.uint32)
    val = (a_val[ga] * b_val[gb]).astype(np.float32)
    indptr = np.concatenate([[0], np.cumsum(np.bincount(rows, minlength=n))]).astype(np.int64)
    return (pair, indptr, idx.astype(np.uint32), val)


class _GpuTrainedModel:
    """What the training loop hands back from the GPU learner: the model bytes (host learner format, built
    from the device table's nonzeros - the table itself never crosses to the host) and the identifying
    args, with the same surface the CPU learner's native object offers _fit (save_model / args / ...)."""

    def __init__(self, model: bytes, args: str, info: dict):
        self._model, self.args = model, args
        self.hash_seed, self.num_bits = int(info["hash_seed"]), int(info["bits"])

    def save_model(self) -> bytes:
        return self._model


def _expand_interactions(specs, chars: List[str]) -> List[tuple]:
    """VW interaction strings (-q / --cubic / --interactions) -> concrete namespace tuples over `chars` (the
    namespaces present). A ':' position ranges over the present namespaces in sorted order and each unordered
    multiset is kept once (its first arrangement: `::` gives ab, never ba), as vw_core.cpp ForEachFeature does
    per example; explicit namespaces that are absent contribute nothing and are dropped."""
    present = sorted(chars)
    out = []
    for q in specs:
        if len(q) not in (2, 3):
            continue
        if ":" not in q:
            if all(c in chars for c in q):
                out.append(tuple(q))
            continue
        seen = set()
        pools = [present if c == ":" else [c] for c in q]
        import itertools

        for combo in itertools.product(*pools):
            if not all(c in chars for c in combo):
                continue
            key = tuple(sorted(combo))
            if key in seen:
                continue
            seen.add(key)
            out.append(combo)
    return out


def _device_plan(blocks, info, shared_blocks=None):
    """Namespace blocks -> GpuSgd.stage_plan arguments: (gpu blocks [(group, level, ip, idx, val)], ngroups,
    interactions as group-id triples). Ignored namespaces are dropped; blocks sharing a first letter form one
    namespace (the host learner's Example::Get merge); `shared_blocks` (CB) are level-1 blocks read through the
    row map."""
    ignore = set(info.get("ignore", ""))
    chars: List[str] = []
    gpu_blocks = []
    for level, bl in ((0, blocks), (1, shared_blocks or [])):
        for g, ip, ii, vv in bl:
            if g in ignore:
                continue
            if g not in chars:
                chars.append(g)
            gpu_blocks.append((chars.index(g), level, np.ascontiguousarray(ip, np.int64),
                               np.ascontiguousarray(ii, np.uint32), np.ascontiguousarray(vv, np.float32)))
    specs = [q for q in info.get("interactions", "").split(",") if q]
    inter = [tuple(chars.index(c) for c in t) + ((-1,) if len(t) == 2 else ()) for t in _expand_interactions(specs, chars)]
    return gpu_blocks, len(chars), inter


def _gpu_refusals(info) -> List[str]:
    """options the device learner does not run (deviceType='gpu' refuses them rather than silently running
    something else)"""
    bad = ["loss_function " + info["loss_function"]] if info["loss_function"] not in (
        "squared", "classic", "logistic", "hinge", "quantile") else []
    if info["cb_adf"] == "1" and info.get("cb_type", "mtr") not in ("mtr", "dr", "ips"):
        bad.append("cb_type " + info["cb_type"])
    return bad


def _gpu_config(vwmod, info):
    cfg = vwmod.GpuSgdConfig()
    cfg.bits = int(info["bits"])
    cfg.lr = float(info["learning_rate"])
    cfg.power_t = float(info["power_t"])
    cfg.initial_t = float(info["initial_t"])
    cfg.l2 = float(info["l2"])
    cfg.l1 = float(info["l1"])
    cfg.tau = float(info.get("loss_quantile_tau", "0.5"))
    cfg.loss = {"logistic": 1, "hinge": 2, "quantile": 3}.get(info["loss_function"], 0)
    cfg.adaptive, cfg.normalized, cfg.invariant = (info[k] == "1" for k in ("adaptive", "normalized", "invariant"))
    cfg.oaa = int(info["oaa"])
    cfg.csoaa = int(info["csoaa"])
    if int(info.get("cats", "0")) > 0:
        cfg.cats = int(info["cats"])
        cfg.cats_min, cfg.cats_max, cfg.cats_bw = (float(info[k]) for k in ("min_value", "max_value", "bandwidth"))
    if info["cb_adf"] == "1":
        cfg.cb = {"mtr": 0, "dr": 1, "ips": 2}[info.get("cb_type", "mtr")]
        cfg.cb_explore = info.get("cb_explore", "0") == "1"
        cfg.epsilon = float(info.get("epsilon", "0.05"))
    return cfg


def _vw_fan_out(est, df: DataFrame):
    """The reference's VW fit runs one task per partition, min(executor tasks, partitions) of them
    (VowpalWabbitBase.scala:124-137, VowpalWabbitBaseLearner.scala:180-211), the tasks averaging their weights
    through VW's allreduce, and keeps the first partition's model. Returns that model when this fit fans out
    (GPU: one rank per visible MI355X - the device learner averages over RCCL), else None."""
    from ..parallel import runtime as R
    from ..utils.cluster import _device_count

    if R.in_partition_task():
        return None
    use_gpu = (est.getOrDefault("deviceType") or "cpu").lower() == "gpu" and _device_count() > 0
    n = R.determine_num_tasks(0, df, use_gpu)
    if use_gpu:
        n = min(n, max(1, _device_count()))
    if n <= 1:
        return None
    barrier = bool(est.getOrDefault("useBarrierExecutionMode")) if est.hasParam("useBarrierExecutionMode") else False
    return R.fan_out(R._FitTask(est.copy(), barrier=barrier), df, n, use_gpu)[0]


def _gpu_learner(args: str, model_bytes=None):
    vwmod = _vw()
    info = vwmod.describe_args(args)  # parses + validates the command line without a host table
    bad = _gpu_refusals(info)
    if bad:
        raise ValueError(f"deviceType='gpu' does not run {', '.join(bad)}; use deviceType='cpu' (args: {args})")
    if not vwmod.gpu_available():
        raise RuntimeError("deviceType='gpu' requested but no HIP device is visible")
    import os

    g = vwmod.GpuSgd(_gpu_config(vwmod, info), D.local_device())
    if model_bytes is not None:  # initialModel: warm start (weights, adaptive / normalizer state, schedule)
        g.import_model(bytes(model_bytes))
    return vwmod, info, g


def _gpu_sync_comm(vwmod):
    world = D.world_size()
    if world <= 1:
        return None
    # (the control plane may be gloo or nccl: the averaging runs on the learner's own RCCL communicator,
    # whose unique id travels over the control plane)
    if world in _nccl_cache and getattr(_nccl_cache[world], "aborted", False):
        del _nccl_cache[world]  # aborted by a failed sync of an earlier fit: rebuild
    if world not in _nccl_cache:
        import os

        timeout_ms = float(os.environ.get("SML_RCCL_INIT_TIMEOUT_MS", "120000"))
        # readiness agreement + bounded collective init + abort on any rank's failure (distributed.py)
        _nccl_cache[world] = D.init_with_retries(
            lambda uid: vwmod.nccl_comm(uid, D.rank(), world, timeout_ms), "VW RCCL communicator",
            prepare=lambda: vwmod.nccl_unique_id() if D.rank() == 0 else None)
    return _nccl_cache[world]


def _evict_nccl(comm) -> None:
    for k, v in list(_nccl_cache.items()):
        if v is comm:
            del _nccl_cache[k]
    abort = getattr(comm, "abort", None)
    if abort is not None:
        abort()


def _sync_bounds(est, n: int) -> np.ndarray:
    """row bounds of the sync segments of one pass: numSyncsPerPass intermediate averages + the end-of-pass
    one, the same count on every rank whatever its row count (VowpalWabbitSyncSchedule.scala:36-72)"""
    segs = max(0, int(est.getNumSyncsPerPass() or 0)) + 1
    return np.linspace(0, n, segs + 1).astype(np.int64)


def _gpu_learn_staged(est, g, comm, n: int, first_learned: bool = False):
    """The sync schedule over the staged rows, re-read from HBM by every pass and segment (VW's cache file).
    ``first_learned``: pass 0's first segment was already learned while the pass staged (stage_plan's
    learn_r1); its sync still runs here."""
    bounds = _sync_bounds(est, n)
    sync_bytes = []
    for p in range(max(1, est.getNumPasses())):
        for k, (s0, s1) in enumerate(zip(bounds[:-1], bounds[1:])):
            if s1 > s0 and not (first_learned and p == 0 and k == 0):
                g.learn_staged(int(s0), int(s1), int(est.getGpuBatchSize()))
            if comm is not None:
                try:
                    g.allreduce_average(comm)
                except RuntimeError:
                    # the native call aborted the communicator (a peer died / the sync timed out): drop it so a
                    # later fit in this process builds a fresh one, and fail this fit on every rank
                    _evict_nccl(comm)
                    raise
                sync_bytes.append(int(g.last_sync_bytes))
    return sync_bytes


def _train_partition_gpu(est, df: DataFrame, args: str, model_bytes=None):
    """Device-resident hogwild mini-batch learner (csrc/vw/vw_gpu.hip, K12).

    Runs VW's update rule - adaptive + normalized + invariant by default, or the subset the command line
    selects (--sgd / --adaptive / --normalized / --invariant) - for squared / logistic loss, scalar learners
    and --oaa K. The partition's namespace blocks go to HBM as they are and the example rows are built there
    (device featurization: -q / --cubic / --interactions incl. ':' wildcards, ignored namespaces, the
    constant). gpuBatchSize=1 is the exact sequential learner; larger batches update concurrently with
    atomics (hogwild). Ranks average the blocks they touched at every sync with RCCL (VW's weighted
    averaging), and the model is exported from the device nonzeros."""
    if int(_vw().describe_args(args).get("cats", "0")) > 0:  # CATS labels ("ca action:cost:pdf") are VW text
        raise ValueError(f"deviceType='gpu' does not run cats in a vector-column estimator; use VowpalWabbitGeneric "
                         f"(args: {args})")
    vwmod, info, g = _gpu_learner(args, model_bytes)
    if info["cb_adf"] == "1":
        raise ValueError("deviceType='gpu' runs --cb_adf / --cb_explore_adf through VowpalWabbitContextualBandit or "
                         "VowpalWabbitGeneric (multi-line examples), not a single-line estimator")
    t0 = time.perf_counter_ns()
    cols = [est.getFeaturesCol()] + list(est.getAdditionalFeatures() or [])
    blocks = namespace_blocks(df, cols, est.getHashSeed())
    labels, multiclass, costs = est._labels(df)
    if int(info["oaa"]) > 0:
        if multiclass is None:
            raise ValueError("--oaa needs integer class labels")
        labels = np.asarray(multiclass, np.float32)
    n = df.count()
    wcol = est.getWeightCol()
    weights = np.asarray(df[wcol], np.float32) if wcol and wcol in df else None
    gb, ng, inter = _device_plan(blocks, info)
    # scalar / oaa learners learn pass 0's first sync segment while the pass's blocks cross PCIe (chunked
    # upload on the copy stream, each chunk expanded and learned as it lands); csoaa stages its cost lists
    # after the plan, so it stages first
    fused = int(info["csoaa"]) == 0 and os.environ.get("SML_VW_STAGE_LEARN", "1") != "0"
    g.stage_plan(gb, ng, inter, info["constant"] == "1", None, n, np.ascontiguousarray(labels, dtype=np.float32),
                 None if weights is None else np.ascontiguousarray(weights, dtype=np.float32),
                 learn_r1=int(_sync_bounds(est, n)[1]) if fused else 0, batch=int(est.getGpuBatchSize()))
    if int(info["csoaa"]) > 0:
        if costs is None:
            raise ValueError("--csoaa needs per-row (class, cost) lists")
        cptr = np.concatenate([[0], np.cumsum([len(c) for c in costs])]).astype(np.int64)
        g.stage_costs(cptr, np.asarray([k for c in costs for k, _ in c], np.int32),
                      np.asarray([v for c in costs for _, v in c], np.float32))
    t1 = time.perf_counter_ns()
    sync_bytes = _gpu_learn_staged(est, g, _gpu_sync_comm(vwmod), n, first_learned=fused)
    t2 = time.perf_counter_ns()
    model = g.export_model(args, final=True)  # the learner's last use: its table is cleared for reuse
    t3 = time.perf_counter_ns()
    lab = np.asarray(labels)
    if weights is None:  # unit weights: no n-long ones / product arrays
        wsum = float(n)
        lsum = float(lab.sum(dtype=np.float64))
    else:
        w64 = np.asarray(weights, np.float64)
        wsum = float(w64.sum())
        lsum = float(np.dot(lab.astype(np.float64), w64))
    stats = {"numberOfExamplesPerPass": int(n), "weightedExampleSum": wsum,
             "weightedLabelSum": lsum, "averageLoss": float(g.sum_loss) / max(wsum, 1e-300),
             "bestConstant": lsum / max(wsum, 1e-300),
             "totalNumberOfFeatures": float(sum(len(b[3]) for b in gb)),
             "passes": int(max(1, est.getNumPasses())), "ipsEstimate": 0.0, "snipsEstimate": 0.0,
             "syncBytes": int(sum(sync_bytes)), "timeTotalNs": t2 - t0, "timeNativeIngestNs": t1 - t0,
             "timeLearnNs": t2 - t1, "timeMultipassNs": 0, "timeExportNs": t3 - t2}  # export: nonzeros -> bytes
    return _GpuTrainedModel(model, args, info), stats


class _GpuScorer:
    """A VW model scored on the MI355X: the model's nonzeros are scattered into an HBM table (no dense host
    table at any size - a 2^30-slot model is a 16 GiB device allocation, never a host one) and examples are
    featurized and scored on the device (VowpalWabbitBaseModelSpark.scala:46-60 scores through native VW)."""

    def __init__(self, args: str, model: bytes):
        vwmod = _vw()
        self.info = vwmod.describe_args(args)
        bad = _gpu_refusals(self.info)
        if bad or int(self.info["ngram"]) or not vwmod.gpu_available():
            raise ValueError("model not scoreable on the device: " + ", ".join(bad or ["no HIP device / ngram"]))
        import os

        self.g = vwmod.GpuSgd(_gpu_config(vwmod, self.info), D.local_device())
        self.g.import_model(bytes(model))

    def predict(self, blocks, n: int, shared_blocks=None, row_map=None):
        gb, ng, inter = _device_plan(blocks, self.info, shared_blocks)
        self.g.stage_plan(gb, ng, inter, self.info["constant"] == "1", row_map, n, None, None)
        return self.g.predict_staged()

    def predict_cb(self, action_blocks, shared_blocks, aip):
        """contextual bandit scoring: per example the action probabilities (cb_explore: epsilon-greedy pmf)
        or the action scores, in action order"""
        aip = np.asarray(aip, np.int64)
        ne = len(aip) - 1
        counts = np.diff(aip)
        row_map = np.repeat(np.arange(ne, dtype=np.int64), counts)
        gb, ng, inter = _device_plan(action_blocks, self.info, shared_blocks)
        self.g.stage_plan(gb, ng, inter, self.info["constant"] == "1", row_map, int(aip[-1]), None, None)
        z = np.zeros(ne, np.float32)
        self.g.stage_cb(aip, np.full(ne, -1, np.int32), z, np.ones(ne, np.float32))
        scores, best = self.g.predict_staged()
        out = []
        eps = float(self.info.get("epsilon", "0.05"))
        explore = self.info.get("cb_explore", "0") == "1"
        for e in range(ne):
            A = int(counts[e])
            if explore:
                p = np.full(A, eps / max(A, 1))
                if A:
                    p[int(best[e])] += 1.0 - eps
                out.append(p.tolist())
            else:
                out.append([float(x) for x in scores[aip[e]:aip[e + 1]]])
        return out


class VowpalWabbitModelBase(Model, VowpalWabbitBaseParams, HasPredictionCol):
    def getNativeModel(self) -> bytes:  # noqa: N802
        """the binary VW model (reference VowpalWabbitPythonBase.py getNativeModel)"""
        return bytes(self.getModel())

    model = Param("The VW model bytes", None, complex=True)
    performanceStatistics = Param("Training statistics", None, complex=True)
    testArgs = Param("Additional arguments passed to VW at test time", "", T.toString)
    vwArgs = Param("Arguments the model was trained with", "", T.toString)

    def _native_model(self):
        # keyed on the model object itself (held by the cache, compared with `is`): an id() key can be reused by
        # a new bytes object once the old model is garbage-collected, and would then score with stale weights
        cache = getattr(self, "_vw_cache", None)
        model, targs = self.getModel(), self.getTestArgs()
        if cache is None or cache[0] is not model or cache[1] != targs:
            m = _vw().VW(self.getVwArgs() + " --testonly " + (targs or ""), model)
            self._vw_cache = (model, targs, m)
        return self._vw_cache[2]

    def getPerformanceStatistics(self) -> DataFrame:  # noqa: N802
        return self.getOrDefault("performanceStatistics")

    def getReadableModel(self) -> str:  # noqa: N802
        return self._native_model().readable_model()

    def saveNativeModel(self, path: str) -> None:  # noqa: N802
        with open(path, "wb") as f:
            f.write(self.getModel())

    def _gpu_scorer(self):
        """device scorer for deviceType='gpu' models (None: score on the host learner)"""
        if (self.getDeviceType() or "cpu").lower() != "gpu":
            return None
        args = self.getVwArgs() + " --testonly " + (self.getTestArgs() or "")
        if "--probabilities" in args:
            return None  # oaa probabilities: host learner
        model = self.getModel()
        cache = getattr(self, "_gpu_cache", None)
        if cache is None or cache[0] is not model or cache[1] != args:
            try:
                self._gpu_cache = (model, args, _GpuScorer(args, model))
            except ValueError:
                self._gpu_cache = (model, args, None)
        return self._gpu_cache[2]

    def _predict_raw(self, df: DataFrame, multiclass: bool = False):
        cols = [self.getFeaturesCol()] + list(self.getAdditionalFeatures() or [])
        blocks = namespace_blocks(df, cols, self.getHashSeed())
        n = df.count()
        gs = self._gpu_scorer()
        if gs is not None:
            preds, _ = gs.predict(blocks, n)
            preds = np.asarray(preds, dtype=np.float64)
            if gs.info["link_logistic"] == "1":
                preds = 1.0 / (1.0 + np.exp(-preds))
            return preds, []
        vw = self._native_model()
        preds, scores = vw.learn_batch(blocks, np.zeros(n, np.float32), None, None, None, False)
        return np.asarray(preds, dtype=np.float64), scores

    def _transform(self, df: DataFrame) -> DataFrame:
        raw, _ = self._predict_raw(df)
        return df.withColumn(self.getPredictionCol(), raw)


class VowpalWabbitBase(Estimator, VowpalWabbitBaseParams, HasLabelCol, HasWeightCol, HasPredictionCol):
    _model_cls = VowpalWabbitModelBase

    def _extra_args(self) -> Optional[ParamsStringBuilder]:
        return None

    def _labels(self, df: DataFrame):
        return np.asarray(df[self.getLabelCol()], dtype=np.float32), None, None

    def _train_partition(self, df: DataFrame, args: str, model_bytes=None):
        if (self.getDeviceType() or "cpu").lower() == "gpu":
            return _train_partition_gpu(self, df, args, model_bytes)
        vw = _vw().VW(args, model_bytes)
        world = D.world_size()
        if world > 1:
            vw.set_allreduce(world, _host_allreduce_f32)
        total = StopWatch()
        ingest = StopWatch()
        learn = StopWatch()
        multipass = StopWatch()
        total.start()
        cols = [self.getFeaturesCol()] + list(self.getAdditionalFeatures() or [])
        blocks = ingest.measure(lambda: namespace_blocks(df, cols, self.getHashSeed()))
        labels, multiclass, costs = self._labels(df)
        wcol = self.getWeightCol()
        weights = np.asarray(df[wcol], np.float32) if wcol and wcol in df else None
        n = df.count()
        syncs = self.getNumSyncsPerPass()
        # every rank must fire the same number of syncs (VowpalWabbitSyncSchedule.scala:36-72)
        if syncs > 0 and world > 1:
            max_n = max(D.all_gather_object(n))
        else:
            max_n = n
        splits = [int(max_n * (k + 1) / (syncs + 1)) for k in range(syncs)] if syncs > 0 else []
        start = 0
        for s in splits + [None]:
            end = n if s is None else min(n, s)
            if end > start:
                learn.measure(lambda: vw.learn_batch(
                    _block_slice(blocks, start, end), labels[start:end],
                    None if weights is None else weights[start:end],
                    None if multiclass is None else multiclass[start:end],
                    None if costs is None else costs[start:end], True))
            start = max(start, end)
            if s is not None and world > 1:
                vw.end_pass()
        if self.getNumPasses() > 1:
            multipass.measure(vw.perform_remaining_passes)
        elif world > 1:
            vw.end_pass()
        total.pause()
        stats = vw.stats()
        stats.update(timeTotalNs=total.elapsed_ns, timeNativeIngestNs=ingest.elapsed_ns, timeLearnNs=learn.elapsed_ns,
                     timeMultipassNs=multipass.elapsed_ns)
        return vw, stats

    def _stats_df(self, vw, stats: dict) -> DataFrame:
        tot = max(1, stats["timeTotalNs"])
        row = {"partitionId": D.rank(), "arguments": vw.args, "learningRate": float(self.getLearningRate() or 0.5),
               "powerT": float(self.getPowerT() or 0.5), "hashSeed": vw.hash_seed, "numBits": vw.num_bits}
        row.update({k: v for k, v in stats.items()})
        for k in ["timeNativeIngestNs", "timeLearnNs", "timeMultipassNs"]:
            row[k.replace("Ns", "Percentage")] = stats[k] / tot
        return DataFrame({k: [v] for k, v in row.items()})

    def _fit(self, df: DataFrame):
        if not self.getSplitCol():
            fanned = _vw_fan_out(self, df)
            if fanned is not None:
                return fanned
        args = build_args(self, self._extra_args())
        init = self.getInitialModel()
        if self.getSplitCol():
            vw, stats = self._train_splits(df, args, init)
        else:
            vw, stats = self._train_partition(df, args, init)
        m = self._model_cls()
        self._copyValues(m)
        m.set("model", bytes(vw.save_model()))
        m.set("vwArgs", args)
        m.set("performanceStatistics", self._stats_df(vw, stats))
        self._post_fit(m)
        return m

    def _post_fit(self, model) -> None:
        pass

    def _train_splits(self, df: DataFrame, args: str, init):
        """Spark-coordinated path (VowpalWabbitBaseLearner.scala:307-354): per
        split value train every partition from the current model, then average."""
        col = df[self.getSplitCol()]
        values = self.getSplitColValues() or sorted(set(col.tolist()))
        model = init
        vw = stats = None
        for v in values:
            part = df.filter(col == v)
            models = []
            for p in part.partitions():
                if p.count() == 0:
                    continue
                vw, stats = self._train_partition(p, args, model)
                models.append(vw)
            if models:
                models = [_vw().VW(args, m.save_model()) if isinstance(m, _GpuTrainedModel) else m for m in models]
                vw = _vw().merge_models(models) if len(models) > 1 else models[0]
                model = bytes(vw.save_model())
        return vw, stats

    def parallelFit(self, df: DataFrame, paramMaps: list):  # noqa: N802
        """Fit one model per param map (VowpalWabbitPythonBase.parallelFit)."""
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(max_workers=min(8, len(paramMaps) or 1)) as ex:
            return list(ex.map(lambda pm: self.copy(pm).fit(df), paramMaps))


# ============================================================ regressor
class VowpalWabbitRegressionModel(VowpalWabbitModelBase, HasRawPredictionCol):
    def _transform(self, df: DataFrame) -> DataFrame:
        raw, _ = self._predict_raw(df)
        return df.withColumn(self.getRawPredictionCol(), raw).withColumn(self.getPredictionCol(), raw)


class VowpalWabbitRegressor(VowpalWabbitBase):
    _model_cls = VowpalWabbitRegressionModel


# ============================================================ classifier
class VowpalWabbitClassificationModel(VowpalWabbitModelBase, HasRawPredictionCol, HasProbabilityCol):
    numClassesModel = Param("Number of classes.", 2, T.toInt)

    def _transform(self, df: DataFrame) -> DataFrame:
        raw, scores = self._predict_raw(df)
        if self.getNumClassesModel() == 2:
            if "--link logistic" in self.getVwArgs():
                p = raw
            else:
                p = 1.0 / (1.0 + np.exp(-raw))
            prob = np.stack([1 - p, p], 1)
            return (df.withColumn(self.getRawPredictionCol(), raw).withColumn(self.getProbabilityCol(), prob)
                    .withColumn(self.getPredictionCol(), (p > 0.5).astype(np.float64)))
        if scores and "--probabilities" in self.getVwArgs():
            probs = np.asarray(scores, dtype=np.float64)
            return (df.withColumn(self.getRawPredictionCol(), probs).withColumn(self.getProbabilityCol(), probs)
                    .withColumn(self.getPredictionCol(), np.argmax(probs, 1).astype(np.float64)))
        return df.withColumn(self.getRawPredictionCol(), raw).withColumn(self.getPredictionCol(), raw)


class VowpalWabbitClassifier(VowpalWabbitBase, HasRawPredictionCol, HasProbabilityCol):
    _model_cls = VowpalWabbitClassificationModel
    labelConversion = Param("Convert 0/1 Spark ML style labels to -1/1 VW style labels.", False, T.toBoolean)
    numClasses = Param("Number of classes. Defaults to binary. Needs to match oaa/csoaa.", 2, T.toInt)

    def _labels(self, df: DataFrame):
        y = np.asarray(df[self.getLabelCol()], dtype=np.float64)
        if self.getNumClasses() != 2:
            return y.astype(np.float32), y.astype(np.int32), None
        if self.getLabelConversion():
            y = y * 2 - 1
        return y.astype(np.float32), None, None

    def _post_fit(self, model) -> None:
        model.set("numClassesModel", self.getNumClasses())


# ============================================================ generic (VW text format)
def _object_column(values) -> np.ndarray:
    col = np.empty(len(values), dtype=object)
    for i, v in enumerate(values):
        col[i] = v
    return col


class VowpalWabbitGenericModel(Model, HasPredictionCol):
    model = Param("The VW model bytes", None, complex=True)
    vwArgs = Param("Arguments the model was trained with", "", T.toString)
    inputCol = Param("Column with examples in VW text format", "value", T.toString)
    testArgs = Param("Additional test-time arguments", "", T.toString)

    def _transform(self, df: DataFrame) -> DataFrame:
        """Adds the columns of the learner's prediction type, as the reference's schema map does
        (VowpalWabbitPrediction.scala:18-101, VowpalWabbitSchema.scala): scalar -> prediction, confidence;
        scalars -> predictions; multiclass / prob -> prediction; action_scores -> predictions [(action, score)];
        action_probs -> predictions [(action, probability)]; pdf -> segments [(left, right, pdfValue)];
        action_pdf_value -> action, pdf."""
        vw = _vw().VW(self.getVwArgs() + " --testonly " + self.getTestArgs(), self.getModel())
        lines = [str(s) for s in df[self.getInputCol()].tolist()]
        ptype, recs = vw.predict_text_structured(lines, False)
        kind = ptype.split("::")[-1]
        obj = lambda xs: _object_column(xs)  # noqa: E731
        if kind == "pdf":
            segs = [[{"left": float(a), "right": float(b), "pdfValue": float(v)} for a, b, v in r] for r in recs]
            return df.withColumn("segments", obj(segs))
        if kind == "action_pdf_value":
            return (df.withColumn("action", np.asarray([r[0] for r in recs], np.float64))
                    .withColumn("pdf", np.asarray([r[1] for r in recs], np.float64)))
        if kind in ("action_probs", "action_scores"):
            field = "probability" if kind == "action_probs" else "score"
            return df.withColumn("predictions", obj([[{"action": int(a), field: float(v)} for a, v in r] for r in recs]))
        if kind == "scalars":
            return df.withColumn("predictions", obj([list(map(float, r)) for r in recs]))
        if kind == "multiclass":
            return df.withColumn(self.getPredictionCol(), np.asarray(recs, np.int64))
        out = df.withColumn(self.getPredictionCol(), np.asarray([r[0] for r in recs], np.float64))
        return out.withColumn("confidence", np.asarray([r[1] for r in recs], np.float64))

    def getReadableModel(self) -> str:  # noqa: N802
        return _vw().VW(self.getVwArgs(), self.getModel()).readable_model()


class VowpalWabbitGeneric(Estimator, HasPredictionCol):
    """Learn from VW-format strings (VowpalWabbitGeneric.scala:19-131)."""

    passThroughArgs = Param("VW command line arguments passed", "", T.toString)
    inputCol = Param("Column with examples in VW text format", "value", T.toString)
    numPasses = Param("Number of passes over the data", 1, T.toInt)
    initialModel = Param("Initial model to start from", None, complex=True)
    numSyncsPerPass = Param("Number of times weights should be synchronized within each pass", 0, T.toInt)
    deviceType = Param("cpu (exact sequential VW semantics) or gpu (hogwild mini-batch SGD on the MI355X: scalar, "
                       "--oaa, --csoaa, --cb_adf / --cb_explore_adf and --cats_pdf / --cats)", "cpu", T.toString)
    gpuBatchSize = Param("Mini-batch size of the GPU learner", 1024, T.toInt)

    def setInitialModel(self, model):  # noqa: N802
        self.set("initialModel", _initial_model_bytes(model))
        return self

    def _fit_gpu(self, lines: List[str], args: str) -> "VowpalWabbitGenericModel":
        """Text examples parsed on the host (the learner's hashing / ngrams), then learned on the device:
        single-line examples (labels, importance weights, --oaa classes, --csoaa cost lists) or blank-line
        separated ADF groups for --cb_adf / --cb_explore_adf (shared line + one line per action)."""
        vwmod, info, g = _gpu_learner(args, self.getInitialModel())
        cb = info["cb_adf"] == "1"
        d = vwmod.parse_blocks(args, lines, cb)
        if cb:
            aip = np.asarray(d["aip"], np.int64)
            ne = len(aip) - 1
            row_map = np.repeat(np.arange(ne, dtype=np.int64), np.diff(aip))
            gb, ng, inter = _device_plan(d["actions"], info, d["shared"])
            g.stage_plan(gb, ng, inter, info["constant"] == "1", row_map, int(aip[-1]), None, None)
            g.stage_cb(aip, d["chosen"], d["cost"], d["prob"])
            n = ne
        else:
            n = len(d["labels"])
            labels = np.asarray(d["multiclass"], np.float32) if int(info["oaa"]) > 0 else d["labels"]
            weights = np.where(d["has_label"] > 0, d["weights"], 0.0).astype(np.float32)
            gb, ng, inter = _device_plan(d["blocks"], info)
            g.stage_plan(gb, ng, inter, info["constant"] == "1", None, n, np.ascontiguousarray(labels, np.float32),
                         weights)
            if int(info["csoaa"]) > 0:
                g.stage_costs(d["cptr"], d["ccls"], d["ccost"])
            if int(info.get("cats", "0")) > 0:  # --cats_pdf / --cats: "ca action:cost:pdf" labels
                g.stage_cats(d["cats_action"], d["cats_cost"], d["cats_pdf"], d["cats_has"])
        _gpu_learn_staged(self, g, _gpu_sync_comm(vwmod), n)
        m = VowpalWabbitGenericModel()
        m.set("model", bytes(g.export_model(args)))
        m.set("vwArgs", args)
        m.set("inputCol", self.getInputCol())
        m.set("predictionCol", self.getPredictionCol())
        self._gpu_stats = g.cb_stats if cb else None
        return m

    def _fit(self, df: DataFrame):
        fanned = _vw_fan_out(self, df)
        if fanned is not None:
            return fanned
        args = self.getPassThroughArgs() + (f" --passes {self.getNumPasses()}" if self.getNumPasses() > 1 else "")
        if (self.getDeviceType() or "cpu").lower() == "gpu":
            return self._fit_gpu([str(s) for s in df[self.getInputCol()].tolist()], args)
        vw = _vw().VW(args, self.getInitialModel())
        if D.world_size() > 1:
            vw.set_allreduce(D.world_size(), _host_allreduce_f32)
        lines = [str(s) for s in df[self.getInputCol()].tolist()]
        if "--cb" in args:
            # multi-line examples separated by empty lines
            group: List[str] = []
            for l in lines + [""]:
                if l.strip():
                    group.append(l)
                elif group:
                    vw.learn_text_multi(group, True)
                    group = []
        else:
            vw.learn_text(lines, True)
        if self.getNumPasses() > 1:
            vw.perform_remaining_passes()
        elif D.world_size() > 1:
            vw.end_pass()
        m = VowpalWabbitGenericModel()
        m.set("model", bytes(vw.save_model()))
        m.set("vwArgs", args)
        m.set("inputCol", self.getInputCol())
        m.set("predictionCol", self.getPredictionCol())
        return m


class VowpalWabbitGenericProgressive(Transformer, HasPredictionCol):
    """Online 1-step-ahead predictions while learning (VowpalWabbitGenericProgressive.scala)."""

    passThroughArgs = Param("VW command line arguments passed", "", T.toString)
    inputCol = Param("Column with examples in VW text format", "value", T.toString)

    def _transform(self, df: DataFrame) -> DataFrame:
        out = []
        for part in df.partitions():
            vw = _vw().VW(self.getPassThroughArgs())
            out.append(np.asarray(vw.learn_text([str(s) for s in part[self.getInputCol()].tolist()], True), np.float64))
        return df.withColumn(self.getPredictionCol(), np.concatenate(out) if out else np.zeros(0))


class VowpalWabbitProgressive(Transformer, VowpalWabbitBaseParams, HasLabelCol, HasPredictionCol):
    """Progressive validation over Spark-vector features (VowpalWabbitBaseProgressive.scala)."""

    def _transform(self, df: DataFrame) -> DataFrame:
        args = build_args(self)
        out = []
        for part in df.partitions():
            vw = _vw().VW(args)
            cols = [self.getFeaturesCol()] + list(self.getAdditionalFeatures() or [])
            blocks = namespace_blocks(part, cols, self.getHashSeed())
            preds, _ = vw.learn_batch(blocks, np.asarray(part[self.getLabelCol()], np.float32), None, None, None, True)
            out.append(np.asarray(preds, np.float64))
        return df.withColumn(self.getPredictionCol(), np.concatenate(out) if out else np.zeros(0))


# reference vw/VowpalWabbitPythonBase.py: the Python-side base mixins
VowpalWabbitPythonBase = VowpalWabbitBase
VowpalWabbitPythonBaseModel = VowpalWabbitModelBase
