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

import re
import time
from typing import List, Optional

import numpy as np

from ..core.contracts import (HasFeaturesCol, HasLabelCol, HasPredictionCol, HasProbabilityCol,
                              HasRawPredictionCol, HasWeightCol)
from ..core.dataframe import DataFrame
from ..core.linalg import DenseVector, SparseVector
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


def _train_partition_gpu(est, df: DataFrame, args: str, model_bytes=None):
    """Device-resident hogwild mini-batch learner (csrc/vw/vw_gpu.hip, K12).

    Runs VW's update rule - adaptive + normalized + invariant by default, or the subset the command line
    selects (--sgd / --adaptive / --normalized / --invariant) - for squared / logistic loss, scalar
    learners and --oaa K, with -q interactions expanded on the host. gpuBatchSize=1 is the exact
    sequential learner; larger batches update concurrently with atomics (hogwild). csoaa, contextual
    bandits, CATS, l1, ngrams, ignore and cubic interactions run on the CPU learner and are rejected here
    rather than silently run elsewhere. Ranks average the blocks they touched at every sync with RCCL
    (VW's weighted averaging), and the model is exported from the device nonzeros."""
    vwmod = _vw()
    info = vwmod.describe_args(args)  # parses + validates the command line without a host table
    bad = [k for k in ("csoaa", "cats", "ngram") if int(info[k])] + (["cb_adf"] if info["cb_adf"] == "1" else []) + \
        (["l1"] if float(info["l1"]) else []) + (["ignore"] if info["ignore"] else []) + \
        (["loss_function " + info["loss_function"]] if info["loss_function"] not in ("squared", "logistic") else []) + \
        (["cubic interactions"] if any(len(q) > 2 for q in info["interactions"].split(",") if q) else [])
    if bad:
        raise ValueError(f"deviceType='gpu' does not run {', '.join(bad)}; use deviceType='cpu' (args: {args})")
    if not vwmod.gpu_available():
        raise RuntimeError("deviceType='gpu' requested but no HIP device is visible")
    cfg = vwmod.GpuSgdConfig()
    cfg.bits = int(info["bits"])
    cfg.lr = float(info["learning_rate"])
    cfg.power_t = float(info["power_t"])
    cfg.initial_t = float(info["initial_t"])
    cfg.l2 = float(info["l2"])
    cfg.loss = 1 if info["loss_function"] == "logistic" else 0
    cfg.adaptive, cfg.normalized, cfg.invariant = (info[k] == "1" for k in ("adaptive", "normalized", "invariant"))
    cfg.oaa = int(info["oaa"])
    import os

    dev = int(os.environ.get("LOCAL_RANK", "0"))
    g = vwmod.GpuSgd(cfg, dev)
    if model_bytes is not None:  # initialModel: warm start (weights, adaptive / normalizer state, schedule)
        g.import_model(bytes(model_bytes))
    t0 = time.perf_counter_ns()
    cols = [est.getFeaturesCol()] + list(est.getAdditionalFeatures() or [])
    blocks = namespace_blocks(df, cols, est.getHashSeed())
    labels, multiclass, _ = est._labels(df)
    if cfg.oaa > 0:
        if multiclass is None:
            raise ValueError("--oaa needs integer class labels")
        labels = np.asarray(multiclass, np.float32)
    n = df.count()
    blocks = blocks + [_interaction_block(blocks, pq, n) for pq in _quadratic_pairs(args)]
    indptr, idx, val = _merged_csr(blocks, n, info["constant"] == "1")
    wcol = est.getWeightCol()
    weights = np.asarray(df[wcol], np.float32) if wcol and wcol in df else None
    t1 = time.perf_counter_ns()
    world = D.world_size()
    comm = None
    if world > 1:
        if D.backend() != "nccl":
            raise RuntimeError("the GPU VW learner averages over RCCL: start the ranks with the nccl backend")
        key = world
        if key not in _nccl_cache:
            uid = vwmod.nccl_unique_id() if D.rank() == 0 else None
            _nccl_cache[key] = vwmod.nccl_comm(D.broadcast_object(uid, 0), D.rank(), world)
        comm = _nccl_cache[key]
    # numSyncsPerPass intermediate weight averages + the end-of-pass one, the same count on every rank
    # whatever its row count (VowpalWabbitSyncSchedule.scala:36-72)
    segs = max(0, int(est.getNumSyncsPerPass() or 0)) + 1
    bounds = np.linspace(0, n, segs + 1).astype(np.int64)
    sync_bytes = []
    # the partition's CSR goes to HBM once; every pass and sync segment learns from there (VW's cache file)
    g.stage(indptr, idx, val, np.ascontiguousarray(labels, dtype=np.float32),
            None if weights is None else np.ascontiguousarray(weights, dtype=np.float32))
    for _ in range(max(1, est.getNumPasses())):
        for s0, s1 in zip(bounds[:-1], bounds[1:]):
            if s1 > s0:
                g.learn_staged(int(s0), int(s1), int(est.getGpuBatchSize()))
            if comm is not None:
                g.allreduce_average(comm)
                sync_bytes.append(int(g.last_sync_bytes))
    t2 = time.perf_counter_ns()
    lab = np.asarray(labels, np.float64)
    wts = np.ones(n) if weights is None else weights.astype(np.float64)
    wsum = float(wts.sum())
    stats = {"numberOfExamplesPerPass": int(n), "weightedExampleSum": wsum,
             "weightedLabelSum": float((lab * wts).sum()), "averageLoss": float(g.sum_loss) / max(wsum, 1e-300),
             "bestConstant": float((lab * wts).sum()) / max(wsum, 1e-300), "totalNumberOfFeatures": float(len(idx)),
             "passes": int(max(1, est.getNumPasses())), "ipsEstimate": 0.0, "snipsEstimate": 0.0,
             "syncBytes": int(sum(sync_bytes)), "timeTotalNs": t2 - t0, "timeNativeIngestNs": t1 - t0,
             "timeLearnNs": t2 - t1, "timeMultipassNs": 0}
    return _GpuTrainedModel(g.export_model(args), args, info), stats


class VowpalWabbitModelBase(Model, VowpalWabbitBaseParams, HasPredictionCol):
    def getNativeModel(self) -> bytes:  # noqa: N802
        """the binary VW model (reference VowpalWabbitPythonBase.py getNativeModel)"""
        return bytes(self.getModel())

    model = Param("The VW model bytes", None, complex=True)
    performanceStatistics = Param("Training statistics", None, complex=True)
    testArgs = Param("Additional arguments passed to VW at test time", "", T.toString)
    vwArgs = Param("Arguments the model was trained with", "", T.toString)

    def _native_model(self):
        cache = getattr(self, "_vw_cache", None)
        key = (id(self.getModel()), self.getTestArgs())
        if cache is None or cache[0] != key:
            m = _vw().VW(self.getVwArgs() + " --testonly " + (self.getTestArgs() or ""), self.getModel())
            self._vw_cache = (key, m)
        return self._vw_cache[1]

    def getPerformanceStatistics(self) -> DataFrame:  # noqa: N802
        return self.getOrDefault("performanceStatistics")

    def getReadableModel(self) -> str:  # noqa: N802
        return self._native_model().readable_model()

    def saveNativeModel(self, path: str) -> None:  # noqa: N802
        with open(path, "wb") as f:
            f.write(self.getModel())

    def _predict_raw(self, df: DataFrame, multiclass: bool = False):
        vw = self._native_model()
        cols = [self.getFeaturesCol()] + list(self.getAdditionalFeatures() or [])
        blocks = namespace_blocks(df, cols, self.getHashSeed())
        n = df.count()
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

    def setInitialModel(self, model):  # noqa: N802
        self.set("initialModel", _initial_model_bytes(model))
        return self

    def _fit(self, df: DataFrame):
        args = self.getPassThroughArgs() + (f" --passes {self.getNumPasses()}" if self.getNumPasses() > 1 else "")
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
