"""Contextual bandits with action-dependent features (reference:
vw/.../VowpalWabbitContextualBandit.scala): shared features (Vector column),
per-action features (Array[Vector] columns), chosen action (1-based), cost
label and logged propensity; ``--cb_explore_adf`` with epsilon-greedy
exploration; online IPS/SNIPS metrics (ContextualBanditMetrics :54-82);
``parallelFit`` over param maps."""
from __future__ import annotations

from typing import List

import numpy as np

from ..core.dataframe import DataFrame
from ..core.linalg import DenseVector, SparseVector
from ..core.params import Param, Params, TypeConverters as T
from ..core.utils import ParamsStringBuilder
from .featurizer import murmur_hash
from .learners import (VowpalWabbitBase, VowpalWabbitModelBase, _host_allreduce_f32, _vw, build_args)
from ..parallel import distributed as D


def _vec_to_arrays(v, ns_hash):
    if isinstance(v, SparseVector):
        return v.indices.astype(np.uint32), v.values.astype(np.float32)
    a = np.asarray(v.toArray() if isinstance(v, DenseVector) else v, dtype=np.float64)
    nz = np.nonzero(a)[0]
    return ((nz.astype(np.uint64) + ns_hash) & 0xFFFFFFFF).astype(np.uint32), a[nz].astype(np.float32)


def _blocks_rows(df: DataFrame, cols: List[str], seed: int):
    blocks = []
    for c in cols:
        nh = murmur_hash(c, seed) & 0xFFFFFFFF
        ip, ii, vv = [0], [], []
        for v in df[c].tolist() if df[c].ndim == 1 else [DenseVector(r) for r in df[c]]:
            i, x = _vec_to_arrays(v, nh)
            ii.append(i)
            vv.append(x)
            ip.append(ip[-1] + len(i))
        blocks.append((c[0], np.asarray(ip, np.int64), np.concatenate(ii) if ii else np.zeros(0, np.uint32),
                       np.concatenate(vv) if vv else np.zeros(0, np.float32)))
    return blocks


def _blocks_actions(df: DataFrame, cols: List[str], seed: int):
    """Array[Vector] columns -> CSR over all actions + row->action offsets."""
    n = df.count()
    first = df[cols[0]].tolist()
    counts = [len(a) for a in first]
    action_indptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    blocks = []
    for c in cols:
        nh = murmur_hash(c, seed) & 0xFFFFFFFF
        ip, ii, vv = [0], [], []
        for row in df[c].tolist():
            for v in row:
                i, x = _vec_to_arrays(v, nh)
                ii.append(i)
                vv.append(x)
                ip.append(ip[-1] + len(i))
        blocks.append((c[0], np.asarray(ip, np.int64), np.concatenate(ii) if ii else np.zeros(0, np.uint32),
                       np.concatenate(vv) if vv else np.zeros(0, np.float32)))
    assert len(action_indptr) == n + 1
    return blocks, action_indptr


class _CBParams(Params):
    sharedCol = Param("Column name of shared features", "shared", T.toString)
    additionalSharedFeatures = Param("Additional namespaces for the shared example", [], T.toListString)


class VowpalWabbitContextualBanditModel(VowpalWabbitModelBase, _CBParams):
    def _transform(self, df: DataFrame) -> DataFrame:
        shared = _blocks_rows(df, [self.getSharedCol()] + list(self.getAdditionalSharedFeatures() or []),
                              self.getHashSeed())
        actions, aip = _blocks_actions(df, [self.getFeaturesCol()] + list(self.getAdditionalFeatures() or []),
                                       self.getHashSeed())
        n = df.count()
        gs = self._gpu_scorer()
        if gs is not None:  # scored on the device (no host weight table)
            out = np.empty(n, dtype=object)
            for i, p in enumerate(gs.predict_cb(actions, shared, aip)):
                out[i] = p
            return df.withColumn(self.getPredictionCol(), out)
        vw = self._native_model()
        res = vw.learn_cb(shared, actions, aip, np.zeros(n, np.int32), np.zeros(n, np.float32),
                          np.ones(n, np.float32), False)
        out = np.empty(n, dtype=object)
        for i, probs in enumerate(res):
            p = sorted(probs, key=lambda t: t[0])
            out[i] = [float(x[1]) for x in p]
        return df.withColumn(self.getPredictionCol(), out)


class VowpalWabbitContextualBandit(VowpalWabbitBase, _CBParams):
    _model_cls = VowpalWabbitContextualBanditModel
    probabilityCol = Param("Column name of probability of chosen action", "probability", T.toString)
    chosenActionCol = Param("Column name of chosen action", "chosenAction", T.toString)
    epsilon = Param("epsilon used for exploration", 0.05, T.toFloat)

    def _extra_args(self):
        args = self.getPassThroughArgs() or ""
        import re

        if re.search(r"--(cb_explore|cb|cb_adf)( |$)", args):
            raise NotImplementedError("VowpalWabbitContextualBandit requires '--cb_explore_adf' problems")
        sb = ParamsStringBuilder(prefix="--", delimiter=" ")
        if "--cb_explore_adf" not in args:
            sb.append("--cb_explore_adf")
        if "--epsilon" not in args:
            sb.appendParamValueIfNotThere("epsilon", self.getEpsilon())
        return sb

    def _train_partition_gpu(self, df: DataFrame, args: str, model_bytes=None):
        """--cb_explore_adf on the device (vw_gpu.hip cb_kernel): action rows featurized in HBM with their
        example's shared namespaces, one block per example scores the actions, epsilon-greedy pmf, IPS/SNIPS
        and the --cb_type (mtr / dr / ips) update; gpuBatchSize=1 is the sequential learner."""
        import time

        from .learners import _GpuTrainedModel, _device_plan, _gpu_learn_staged, _gpu_learner, _gpu_sync_comm

        t0 = time.perf_counter_ns()
        vwmod, info, g = _gpu_learner(args, model_bytes)
        shared = _blocks_rows(df, [self.getSharedCol()] + list(self.getAdditionalSharedFeatures() or []),
                              self.getHashSeed())
        actions, aip = _blocks_actions(df, [self.getFeaturesCol()] + list(self.getAdditionalFeatures() or []),
                                       self.getHashSeed())
        n = df.count()
        row_map = np.repeat(np.arange(n, dtype=np.int64), np.diff(aip))
        gb, ng, inter = _device_plan(actions, info, shared)
        g.stage_plan(gb, ng, inter, info["constant"] == "1", row_map, int(aip[-1]), None, None)
        g.stage_cb(aip, np.asarray(df[self.getChosenActionCol()], np.int32) - 1,
                   np.asarray(df[self.getLabelCol()], np.float32), np.asarray(df[self.getProbabilityCol()], np.float32))
        t1 = time.perf_counter_ns()
        _gpu_learn_staged(self, g, _gpu_sync_comm(vwmod), n)
        t2 = time.perf_counter_ns()
        ips, snips_den, ex = g.cb_stats
        st = {"numberOfExamplesPerPass": int(n), "weightedExampleSum": float(ex), "weightedLabelSum": 0.0,
              "averageLoss": float(ips) / max(ex, 1.0), "bestConstant": 0.0, "totalNumberOfFeatures": 0.0,
              "passes": int(max(1, self.getNumPasses())), "ipsEstimate": float(ips) / max(ex, 1.0),
              "snipsEstimate": float(ips) / snips_den if snips_den else 0.0, "syncBytes": 0,
              "timeTotalNs": t2 - t0, "timeNativeIngestNs": t1 - t0, "timeLearnNs": t2 - t1, "timeMultipassNs": 0}
        return _GpuTrainedModel(g.export_model(args), args, info), st

    def _train_partition(self, df: DataFrame, args: str, model_bytes=None):
        import time

        if (self.getDeviceType() or "cpu").lower() == "gpu":
            return self._train_partition_gpu(df, args, model_bytes)
        t0 = time.perf_counter_ns()
        vw = _vw().VW(args, model_bytes)
        if D.world_size() > 1:
            vw.set_allreduce(D.world_size(), _host_allreduce_f32)
        shared = _blocks_rows(df, [self.getSharedCol()] + list(self.getAdditionalSharedFeatures() or []),
                              self.getHashSeed())
        actions, aip = _blocks_actions(df, [self.getFeaturesCol()] + list(self.getAdditionalFeatures() or []),
                                       self.getHashSeed())
        t1 = time.perf_counter_ns()
        vw.learn_cb(shared, actions, aip, np.asarray(df[self.getChosenActionCol()], np.int32),
                    np.asarray(df[self.getLabelCol()], np.float32), np.asarray(df[self.getProbabilityCol()], np.float32),
                    True)
        t2 = time.perf_counter_ns()
        if self.getNumPasses() > 1:
            vw.perform_remaining_passes()
        elif D.world_size() > 1:
            vw.end_pass()
        t3 = time.perf_counter_ns()
        st = vw.stats()
        st.update(timeTotalNs=t3 - t0, timeNativeIngestNs=t1 - t0, timeLearnNs=t2 - t1, timeMultipassNs=t3 - t2)
        return vw, st

    def fit(self, df: DataFrame, params=None):
        if isinstance(params, (list, tuple)):
            return self.parallelFit(df, list(params))
        return super().fit(df, params)


class ContextualBanditMetrics:
    """Running IPS / SNIPS estimates (VowpalWabbitContextualBandit.scala:54-82)."""

    def __init__(self):
        self.snips_numerator = 0.0
        self.total_events = 0
        self.snips_denominator = 0.0
        self.policy_cost = 0.0

    def addExample(self, probLoggingPolicy: float, reward: float, probEvalPolicy: float, count: int = 1):  # noqa: N802,N803
        self.total_events += count
        if probEvalPolicy > 0:
            w = probEvalPolicy / probLoggingPolicy
            self.snips_numerator += reward * w
            self.snips_denominator += w
            self.policy_cost += reward * w

    def getIpsEstimate(self) -> float:  # noqa: N802
        return self.snips_numerator / self.total_events if self.total_events else 0.0

    def getSnipsEstimate(self) -> float:  # noqa: N802
        return self.snips_numerator / self.snips_denominator if self.snips_denominator else 0.0
