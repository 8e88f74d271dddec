"""Distributed LightGBM-style training driver (reference:
lightgbm/.../LightGBMBase.scala, BasePartitionTask.scala, TrainUtils.scala).

Flow of one ``fit``: optional sequential batches (``numBatches``, :45-60) ->
per batch: column preparation, validation split, categorical slots, bin
boundaries from a row sample (``samplingMode`` global/subset/fixed, or a cached
``referenceDataset``), native Dataset construction, booster creation (+ merge
of ``modelString`` for continued training), the iteration loop with delegate
hooks, learning-rate resets, custom objective, train/valid evaluation and early
stopping (TrainUtils.scala:98-169), and truncation to the best iteration.

Data parallel: when a process group with world > 1 is active each rank holds
its partition; rank 0's sample defines the shared bin boundaries (broadcast,
C8 in SURVEY §2.5) and histograms are allreduced over RCCL inside the engine.
"""
from __future__ import annotations

import logging
import json
import os
import time
from typing import List, Optional

import numpy as np

from ..core.dataframe import DataFrame
from ..core.linalg import SparseVector, as_csr, as_matrix
from ..core.pipeline import Estimator
from ..core.utils import ParamsStringBuilder
from ..ops import native
from ..parallel import distributed as D
from .booster import LightGBMBooster
from .params import LightGBMParams

log = logging.getLogger("synapseml_amd.lightgbm")

# A fitted model keeps only its trees: the training booster's backend (device buffers, pinned staging),
# datasets and validation state are released as the fit returns. The buffers go back to the process's device
# pool, the stream / pinned staging to the backend object cache and the label vectors to the host block pool,
# so the next fit gets them back without allocating (~1 ms; a background-thread release measured no faster
# end to end - it contended with the next fit's sampling and upload; r6 pass 14).
def _release_training(nb) -> None:
    nb.release_training()


def _group_order(g) -> Optional[np.ndarray]:
    """Row order that makes each query group contiguous (groups in first-appearance order, rows stable
    inside a group), or None when the rows already are grouped (the common case: no copy at all).

    Vectorised (LightGBMRanker.scala:88-120 needs contiguous groups). The column is cut into runs of equal
    ids; when no id starts two runs the rows are grouped. Otherwise the run ids are factorised (a hash pass
    over runs, first-appearance codes) and the runs are stably ordered by code and expanded back to rows."""
    a = np.asarray(g)
    n = len(a)
    if n < 2:
        return None
    starts, grouped = _group_runs(a)
    if grouped:
        return None
    run_ids = a[starts]
    import pandas as pd

    codes, _ = pd.factorize(run_ids, sort=False)
    lens = np.diff(np.append(starts, n))
    run_order = np.argsort(codes, kind="stable")
    rs, rl = starts[run_order], lens[run_order]
    # expand runs to row indices: row i of the output = rs[run] + (i - first output row of that run)
    out_first = np.concatenate(([0], np.cumsum(rl)[:-1]))
    idx = np.arange(n, dtype=np.int64)
    idx -= np.repeat(out_first - rs, rl)
    return idx

def _group_runs(a: np.ndarray):
    """(first row of every run of equal ids, whether every id forms a single run). Integer ids: one parallel
    native scan (12.5M ids ~1 ms; numpy's compare + nonzero + unique ~8 ms); other ids: numpy."""
    if a.dtype.kind in "iu" and len(a) >= 2:
        starts, grouped = native.gbdt().group_runs(np.ascontiguousarray(a, dtype=np.int64))
        return starts, bool(grouped)
    brk = np.flatnonzero(a[1:] != a[:-1]) + 1
    starts = np.concatenate(([0], brk))
    return starts, len(np.unique(a[starts])) == len(starts)


class InstrumentationMeasures(dict):
    """Per-phase wall-clock timings (reference: LightGBMPerformance.scala:11-183)."""

    def mark(self, name: str, value_ms: float) -> None:
        self[name] = self.get(name, 0.0) + value_ms


def _features(df: DataFrame, col: str, matrix_type: str):
    c = df[col]
    if isinstance(c, np.ndarray) and c.ndim == 2:
        if matrix_type == "sparse":
            return "sparse", as_csr(c)
        # float32 feature matrices stay float32 end to end (the native push and the K1 device encoder take
        # them as is, and ValueToBin compares in double either way): an 11M x 28 float64 copy would be a
        # 2.5 GB host pass inside fit
        dt = np.float32 if c.dtype == np.float32 else np.float64
        return "dense", np.ascontiguousarray(c, dtype=dt)
    sparse = matrix_type == "sparse" or (matrix_type == "auto" and any(isinstance(v, SparseVector) for v in c[:10]))
    if sparse:
        return "sparse", as_csr(c)
    return "dense", as_matrix(c)


def _slice_features(kind, data, idx):
    if kind == "dense":
        return data[idx]
    indptr, indices, values, width = data
    rows = np.nonzero(idx)[0] if idx.dtype == bool else idx
    new_ptr = [0]
    ii, vv = [], []
    for r in rows:
        a, b = indptr[r], indptr[r + 1]
        ii.append(indices[a:b])
        vv.append(values[a:b])
        new_ptr.append(new_ptr[-1] + (b - a))
    return (np.asarray(new_ptr, np.int64), np.concatenate(ii).astype(np.int32) if ii else np.zeros(0, np.int32),
            np.concatenate(vv) if vv else np.zeros(0), width)


def _num_rows(kind, data) -> int:
    return data.shape[0] if kind == "dense" else len(data[0]) - 1


def _num_cols(kind, data) -> int:
    return data.shape[1] if kind == "dense" else data[3]


def _sample_dense(kind, data, idx) -> np.ndarray:
    if kind == "dense":
        return np.ascontiguousarray(data[idx])
    indptr, indices, values, width = data
    out = np.zeros((len(idx), width))
    for i, r in enumerate(idx):
        a, b = indptr[r], indptr[r + 1]
        out[i, indices[a:b]] = values[a:b]
    return out


def _injected_iteration_crash() -> Optional[int]:
    """Test-only fault injection: ``SML_FAULT_INJECT="<rank>:crash_iter=<k>"`` makes that rank's
    process exit at boosting iteration k, while its peers wait in the histogram allreduce."""
    for item in filter(None, os.environ.get("SML_FAULT_INJECT", "").split(",")):
        r, _, kind = item.partition(":")
        if r.strip() == str(D.rank()) and kind.strip().startswith("crash_iter="):
            return int(kind.strip().split("=", 1)[1])
    return None


class LightGBMBase(Estimator, LightGBMParams):
    _objective_default = "regression"

    def _init_state(self) -> None:
        self._measures: List[InstrumentationMeasures] = []

    # ------------------------------------------------------------- public helpers
    def getPerformanceMeasures(self) -> List[InstrumentationMeasures]:  # noqa: N802
        return list(getattr(self, "_measures", []))

    # ------------------------------------------------------------- hooks
    def _is_classification(self) -> bool:
        return False

    def _num_class(self, df: DataFrame) -> int:
        return 1

    def _extra_params(self, sb: ParamsStringBuilder, num_class: int) -> None:
        pass

    def _make_model(self, booster: LightGBMBooster, num_class: int):
        raise NotImplementedError

    def _group_col(self) -> Optional[str]:
        return None

    # ------------------------------------------------------------- params string
    def _categorical_indexes(self, df: DataFrame, num_cols: int) -> List[int]:
        idx = set(self.getCategoricalSlotIndexes() or [])
        names = self.getCategoricalSlotNames() or []
        slot_names = self._slot_names(df, num_cols)
        for n in names:
            if n in slot_names:
                idx.add(slot_names.index(n))
        md = df.metadata(self.getFeaturesCol())
        for i, attr in enumerate(md.get("ml_attr", {}).get("attrs", {}).get("nominal", [])):
            if "idx" in attr:
                idx.add(int(attr["idx"]))
        for i in md.get("categorical_slots", []):
            idx.add(int(i))
        return sorted(i for i in idx if 0 <= i < num_cols)

    def _slot_names(self, df: DataFrame, num_cols: int) -> List[str]:
        names = list(self.getSlotNames() or [])
        if not names:
            md = df.metadata(self.getFeaturesCol())
            names = list(md.get("slot_names", []))
        if len(names) != num_cols:
            names = [f"Column_{i}" for i in range(num_cols)]
        for n in names:
            if any(ch in n for ch in '",:[]{}'):
                raise ValueError(f"Invalid slot name {n!r}: slot names cannot contain \" , : [ ] {{ }}")
        return names

    def _check_parallelism(self, use_gpu: bool, world: int) -> None:
        """data_parallel (full-histogram allreduce per split) and voting_parallel (PV-Tree: local top-k votes,
        only the 2*topK most-voted features' histograms reduced) run on both backends and any number of ranks
        (reference LightGBMParams.scala:25-35); anything else is refused before any data moves."""
        if self.getParallelism() not in ("data_parallel", "voting_parallel"):
            raise ValueError(f"parallelism={self.getParallelism()!r}: expected 'data_parallel' or 'voting_parallel'")

    def _train_params(self, num_class: int, cat_idx: List[int], num_machines: int) -> str:
        sb = ParamsStringBuilder()
        sb.append(self.getPassThroughArgs())
        sb.appendParamValueIfNotThere("is_pre_partition", "True")
        sb.appendParamValueIfNotThere("boosting_type", self.getBoostingType())
        sb.appendParamValueIfNotThere("tree_learner", "data" if self.getParallelism() == "data_parallel" else
                                      ("voting" if self.getParallelism() == "voting_parallel" else self.getParallelism()))
        sb.appendParamValueIfNotThere("top_k", self.getTopK())
        sb.appendParamValueIfNotThere("num_leaves", self.getNumLeaves())
        sb.appendParamValueIfNotThere("max_bin", self.getMaxBin())
        sb.appendParamValueIfNotThere("bin_construct_sample_cnt", self.getBinSampleCount())
        sb.appendParamValueIfNotThere("min_data_in_bin", self.getMinDataPerBin())
        sb.appendParamValueIfNotThere("bagging_fraction", self.getBaggingFraction())
        sb.appendParamValueIfNotThere("pos_bagging_fraction", self.getPosBaggingFraction())
        sb.appendParamValueIfNotThere("neg_bagging_fraction", self.getNegBaggingFraction())
        sb.appendParamValueIfNotThere("bagging_freq", self.getBaggingFreq())
        sb.appendParamValueIfNotThere("feature_fraction", self.getFeatureFraction())
        sb.appendParamValueIfNotThere("feature_fraction_bynode", self.getFeatureFractionByNode())
        sb.appendParamValueIfNotThere("max_depth", self.getMaxDepth())
        sb.appendParamValueIfNotThere("min_sum_hessian_in_leaf", self.getMinSumHessianInLeaf())
        sb.appendParamValueIfNotThere("lambda_l1", self.getLambdaL1())
        sb.appendParamValueIfNotThere("lambda_l2", self.getLambdaL2())
        metric = self.getMetric()
        sb.appendParamValueIfNotThere("metric", metric if metric else None)
        sb.appendParamValueIfNotThere("min_gain_to_split", self.getMinGainToSplit())
        sb.appendParamValueIfNotThere("max_delta_step", self.getMaxDeltaStep())
        sb.appendParamValueIfNotThere("min_data_in_leaf", self.getMinDataInLeaf())
        sb.appendParamValueIfNotThere("num_iterations", self.getNumIterations())
        sb.appendParamValueIfNotThere("learning_rate", self.getLearningRate())
        sb.appendParamValueIfNotThere("num_machines", num_machines)
        # `timeout` (seconds, the reference's network timeout) bounds how long a collective may block before
        # the engine aborts the communicator and fails the fit on every rank (native `time_out` is minutes)
        sb.appendParamValueIfNotThere("time_out", max(1, int(-(-float(self.getTimeout()) // 60))))
        sb.appendParamValueIfNotThere("verbosity", self.getVerbosity())
        sb.appendParamValueIfNotThere("early_stopping_round", self.getEarlyStoppingRound())
        sb.appendParamListIfNotThere("categorical_feature", cat_idx)
        sb.appendParamListIfNotThere("max_bin_by_feature", self.getMaxBinByFeature())
        sb.appendParamValueIfNotThere("top_rate", self.getTopRate())
        sb.appendParamValueIfNotThere("other_rate", self.getOtherRate())
        sb.appendParamListIfNotThere("monotone_constraints", self.getMonotoneConstraints())
        sb.appendParamValueIfNotThere("monotone_constraints_method", self.getMonotoneConstraintsMethod())
        sb.appendParamValueIfNotThere("monotone_penalty", self.getMonotonePenalty())
        # dataset
        sb.appendParamValueIfNotThere("is_enable_sparse", self.getIsEnableSparse())
        sb.appendParamValueIfNotThere("use_missing", self.getUseMissing())
        sb.appendParamValueIfNotThere("zero_as_missing", self.getZeroAsMissing())
        if self.getBoostingType() == "dart":
            sb.appendParamValueIfNotThere("drop_rate", self.getDropRate())
            sb.appendParamValueIfNotThere("max_drop", self.getMaxDrop())
            sb.appendParamValueIfNotThere("skip_drop", self.getSkipDrop())
            sb.appendParamValueIfNotThere("xgboost_dart_mode", self.getXGBoostDartMode())
            sb.appendParamValueIfNotThere("uniform_drop", self.getUniformDrop())
        # objective
        sb.appendParamValueIfNotThere("objective", "custom" if self.getFobj() is not None else self.getObjective())
        # execution
        sb.appendParamValueIfNotThere("num_threads", self.getNumThreads())
        sb.appendParamValueIfNotThere("device_type", self.getDeviceType())
        # seeds
        sb.appendParamValueIfNotThere("seed", self.getSeed())
        sb.appendParamValueIfNotThere("deterministic", self.getDeterministic())
        sb.appendParamValueIfNotThere("bagging_seed", self.getBaggingSeed())
        sb.appendParamValueIfNotThere("feature_fraction_seed", self.getFeatureFractionSeed())
        sb.appendParamValueIfNotThere("extra_seed", self.getExtraSeed())
        sb.appendParamValueIfNotThere("drop_seed", self.getDropSeed())
        sb.appendParamValueIfNotThere("data_random_seed", self.getDataRandomSeed())
        sb.appendParamValueIfNotThere("objective_seed", self.getObjectiveSeed())
        # categorical
        sb.appendParamValueIfNotThere("min_data_per_group", self.getMinDataPerGroup())
        sb.appendParamValueIfNotThere("max_cat_threshold", self.getMaxCatThreshold())
        sb.appendParamValueIfNotThere("cat_l2", self.getCatl2())
        sb.appendParamValueIfNotThere("cat_smooth", self.getCatSmooth())
        sb.appendParamValueIfNotThere("max_cat_to_onehot", self.getMaxCatToOnehot())
        self._extra_params(sb, num_class)
        return sb.result

    # ------------------------------------------------------------- fit
    # ------------------------------------------------------------- checkpoints
    # Params that change where checkpoints go or how often, not what is trained.
    _CKPT_EXCLUDE = ("checkpointDir", "checkpointInterval", "resumeFromCheckpoint", "delegate", "fobj",
                     "referenceDataset", "modelString")

    def _ckpt_fingerprint(self, df: DataFrame) -> str:
        """Identity of one training job: training params (minus checkpoint bookkeeping and
        non-JSON values), the row count, the feature width and a strided content sample of the
        features and labels. A checkpoint is only resumed when its fingerprint matches."""
        import hashlib

        pm = {}
        for name, v in sorted(self.extractParamMap().items()):
            if name in self._CKPT_EXCLUDE or callable(v):
                continue
            try:
                json.dumps(v)
            except TypeError:
                v = repr(type(v))
            pm[name] = v
        h = hashlib.sha256(json.dumps(pm, sort_keys=True, default=str).encode())
        n = len(df)
        h.update(str(n).encode())
        idx = np.unique(np.linspace(0, max(0, n - 1), num=min(n, 64)).astype(np.int64)) if n else np.zeros(0, np.int64)
        for col in (self.getFeaturesCol(), self.getLabelCol()):
            if col not in df:
                continue
            vals = df[col]
            try:
                sample = as_matrix(vals[idx]) if getattr(vals, "dtype", None) == object else np.asarray(vals)[idx]
                arr = np.ascontiguousarray(np.asarray(sample, dtype=np.float64))
                h.update(str(arr.shape).encode())
                h.update(arr.tobytes())
            except Exception:  # sparse / exotic columns: the row count and params still pin the job
                h.update(repr(type(vals)).encode())
        if D.world_size() > 1:
            # every rank holds a different partition: the job is the set of all partitions
            parts = D.all_gather_object(h.hexdigest())
            return hashlib.sha256("|".join(parts).encode()).hexdigest()
        return h.hexdigest()

    def _ckpt_latest(self, fingerprint: Optional[str] = None) -> Optional[dict]:
        """The checkpoint to resume from, or None. Rank 0 decides (only it writes checkpoints) and
        broadcasts the decision, so every rank takes the same path even when the checkpoint
        directory is not shared between hosts."""
        d = self.getCheckpointDir()
        if not d or not self.getResumeFromCheckpoint():
            return None
        meta = None
        if D.rank() == 0:
            # rank 0 always reaches the broadcast: a failed read travels to every rank as an error marker,
            # so all ranks raise together instead of the others waiting in the broadcast forever
            try:
                p = os.path.join(d, "latest.json")
                if os.path.exists(p):
                    with open(p) as f:
                        meta = json.load(f)
                    if fingerprint is not None and meta.get("fingerprint") != fingerprint:
                        log.warning("checkpoint %s was written by a different job (params or data differ); "
                                    "starting fresh", p)
                        meta = None
                    else:
                        with open(os.path.join(d, meta["model"])) as f:
                            meta["model_str"] = f.read()
            except Exception as e:  # noqa: BLE001 - reported on every rank below
                meta = {"__error__": f"{type(e).__name__}: {e}"}
        meta = D.broadcast_object(meta, 0)
        if meta is not None and "__error__" in meta:
            raise RuntimeError(f"cannot resume from checkpoint directory {d!r}: {meta['__error__']}")
        return meta

    def _ckpt_write(self, model_str: str, batch: int, iteration: int, complete: bool) -> None:
        d = self.getCheckpointDir()
        if not d or D.rank() != 0:
            return
        os.makedirs(d, exist_ok=True)
        name = f"model_b{batch}_i{iteration}.txt"
        tmp = os.path.join(d, name + ".tmp")
        with open(tmp, "w") as f:
            f.write(model_str)
        os.replace(tmp, os.path.join(d, name))
        meta = {"model": name, "batch": batch, "iteration": iteration, "complete": complete,
                "fingerprint": getattr(self, "_ckpt_fp", None)}
        tmp = os.path.join(d, "latest.json.tmp")
        with open(tmp, "w") as f:
            json.dump(meta, f)
        os.replace(tmp, os.path.join(d, "latest.json"))

    # Params of the reference's JVM data-transfer path. Here partitions reach HBM as columnar blocks through one
    # path whatever their value, so an explicit setting is reported instead of silently ignored.
    _INERT_PARAMS = {
        "dataTransferMode": "partitions are always pushed as columnar blocks (the streaming and bulk JVM paths "
                            "do not exist here)",
        "executionMode": "deprecated in the reference; partitions are always pushed as columnar blocks",
        "useSingleDatasetMode": "each task (one process per MI355X) always builds exactly one Dataset",
        "microBatchSize": "rows are pushed in whole columnar blocks, not JVM micro-batches",
        "chunkSize": "rows are pushed in whole columnar blocks, not JVM chunked arrays",
        "maxStreamingOMPThreads": "the host encoder sizes its own thread pool",
        "repartitionByGroupingColumn": "ranker rows are grouped inside each task instead of by a Spark shuffle",
    }

    def _warn_inert_params(self) -> None:
        for name, why in self._INERT_PARAMS.items():
            if self.hasParam(name) and self.isSet(name):
                log.warning("%s=%r has no effect: %s", name, self.getOrDefault(name), why)

    def _fit(self, df: DataFrame):
        from ..parallel import runtime as R

        self._warn_inert_params()
        if not R.in_partition_task():
            from ..utils.cluster import _device_count

            # counting devices does not initialise HIP in this (driver) process, which only spawns the tasks
            use_gpu = self.getDeviceType() == "gpu" and _device_count() > 0
            ntasks = R.determine_num_tasks(self.getNumTasks(), df, use_gpu)
            if ntasks > 1:
                return self._fit_tasks(df, ntasks, use_gpu)
        return self._fit_local(df)

    def _fit_tasks(self, df: DataFrame, ntasks: int, use_gpu: bool):
        """Fan the fit out over ``ntasks`` partition tasks, one process (and one MI355X) each, as the
        reference's fit does with barrier / plain mapPartitions (LightGBMBase.scala:608-628); the tasks
        rendezvous on driverListenPort / defaultListenPort, train data-parallel (histogram allreduce over
        RCCL) and the main task's model is returned (BasePartitionTask.scala:450-461)."""
        from ..parallel import runtime as R

        kw = {"timeout_s": max(60.0, float(self.getTimeout()))}
        dp = int(self.getDriverListenPort() or 0)
        if dp > 0:
            kw["port"] = R.rendezvous_port(dp)
        else:
            kw["default_listen_port"] = int(self.getDefaultListenPort() or 0)
        log.info("fit: %d partition tasks (%s)", ntasks, "gpu" if use_gpu else "cpu")
        est = self.copy()
        res = R.fan_out(R._FitTask(est, barrier=bool(self.getUseBarrierExecutionMode()), with_measures=True), df,
                        ntasks, use_gpu, **kw)
        model = res[0][0]
        self._measures = list(res[0][1] or [])
        self._task_measures = [r[1] for r in res]
        return model

    def getTaskMeasures(self) -> list:  # noqa: N802
        """Per-task instrumentation of the last fanned-out fit, in task order
        (LightGBMPerformance.setTaskMeasures)."""
        return list(getattr(self, "_task_measures", []))

    def _fit_local(self, df: DataFrame):
        self._measures = []
        nb = self.getNumBatches()
        batches = df.randomSplit([1.0] * nb, seed=self.getSeed() or 0) if nb and nb > 0 else [df]
        model_str = self.getModelString() or None
        booster = None
        num_class = self._num_class(df)
        delegate = self.getDelegate()
        self._ckpt_fp = self._ckpt_fingerprint(df) if self.getCheckpointDir() else None
        ck = self._ckpt_latest(self._ckpt_fp)
        start_batch, self._resume_done = 0, 0
        if ck is not None:
            model_str = ck["model_str"]
            start_batch = ck["batch"] + (1 if ck["complete"] else 0)
            self._resume_done = 0 if ck["complete"] else ck["iteration"]
            log.info("resuming from checkpoint %s (batch %d, iteration %d)", ck["model"], ck["batch"], ck["iteration"])
            if start_batch >= len(batches):
                return self._make_model(LightGBMBooster(model_str), num_class)
        for bi, batch in enumerate(batches):
            if bi < start_batch:
                continue
            if delegate is not None:
                delegate.beforeTrainBatch(bi, log, batch, booster)
            booster = self._train_batch(batch, model_str, bi, num_class)
            # the model text is only needed to continue into the next batch or for a checkpoint
            model_str = booster.modelStr if (bi + 1 < len(batches) or self.getCheckpointDir()) else None
            self._resume_done = 0
            if self.getCheckpointDir():
                self._ckpt_write(model_str, bi, self.getNumIterations(), True)
            if delegate is not None:
                delegate.afterTrainBatch(bi, log, batch, booster)
        return self._make_model(booster, num_class)

    def _prepare(self, df: DataFrame):
        """Column extraction; ranker rows are grouped contiguously."""
        gcol = self._group_col()
        if gcol:
            order = _group_order(df[gcol])
            if order is not None:
                df = df._take_rows(order)
        return df

    def _train_batch(self, df: DataFrame, model_str: Optional[str], batch_index: int, num_class: int):
        m = InstrumentationMeasures()
        t_start = time.perf_counter()
        g = native.gbdt()
        t0 = time.perf_counter()
        df = self._prepare(df)
        m.mark("prepare_ms", (time.perf_counter() - t0) * 1e3)
        vcol = self.getValidationIndicatorCol()
        valid_df = None
        if vcol and vcol in df:
            vmask = np.asarray(df[vcol], dtype=bool)
            valid_df = df.filter(vmask)
            df = df.filter(~vmask)
        kind, data = _features(df, self.getFeaturesCol(), self.getMatrixType())
        n = _num_rows(kind, data)
        ncols = _num_cols(kind, data)
        world = D.world_size()
        if world > 1:
            ncols = max(D.all_gather_object(ncols))
        cat_idx = self._categorical_indexes(df, ncols)
        names = self._slot_names(df, ncols)
        params = self._train_params(num_class, cat_idx, world)
        use_gpu = self.getDeviceType() == "gpu" and native.gpu_available()
        self._check_parallelism(use_gpu, world)
        # K1 input staging: a large dense partition starts its host->HBM copy now, on a native thread, so it
        # overlaps the row sampling and bin-boundary construction below (the encode then runs in HBM)
        upload = g.DeviceRows(data) if (kind == "dense" and use_gpu and n >= (1 << 16)) else None
        # --- bin boundaries (reference dataset)
        t0 = time.perf_counter()
        ref_bytes = self.getReferenceDataset()
        if ref_bytes:
            ref = g.DatasetReference.deserialize(bytes(ref_bytes))
        else:
            sample = None
            if D.rank() == 0 or world == 1:
                sample = self._sample_rows(kind, data, n)
            if world > 1:
                # "global" sampling gathers a proportional sample from every rank
                if self.getSamplingMode() == "global":
                    parts = D.all_gather_object(self._sample_rows(kind, data, n, share=1.0 / world))
                    sample = np.concatenate([p for p in parts if p is not None and len(p)], axis=0)
                ser = None
                if D.rank() == 0:
                    tot = n * world
                    ser = bytes(g.DatasetReference.from_sample(sample, tot, params, names).serialize())
                ser = D.broadcast_object(ser, 0)
                ref = g.DatasetReference.deserialize(ser)
            else:
                ref = g.DatasetReference.from_sample(sample, n, params, names)
            self._last_reference = bytes(ref.serialize())
        m.mark("sampling_ms", (time.perf_counter() - t0) * 1e3)
        # --- datasets
        delegate = self.getDelegate()
        if delegate is not None:
            delegate.beforeGenerateTrainDataset(batch_index, D.rank(), None, df.schema, log, params)
        t0 = time.perf_counter()
        train = self._build_dataset(g, ref, df, kind, data, n, num_class, upload=upload)
        upload = None  # the raw rows' HBM copy is released (back to the device pool)
        m.mark("dataset_creation_ms", (time.perf_counter() - t0) * 1e3)
        if delegate is not None:
            delegate.afterGenerateTrainDataset(batch_index, D.rank(), None, df.schema, log, params)
        valid = None
        if valid_df is not None and len(valid_df) > 0:
            if delegate is not None:
                delegate.beforeGenerateValidDataset(batch_index, D.rank(), None, df.schema, log, params)
            t0 = time.perf_counter()
            vk, vd = _features(valid_df, self.getFeaturesCol(), self.getMatrixType())
            valid = self._build_dataset(g, ref, valid_df, vk, vd, _num_rows(vk, vd), num_class)
            m.mark("validation_dataset_creation_ms", (time.perf_counter() - t0) * 1e3)
            if delegate is not None:
                delegate.afterGenerateValidDataset(batch_index, D.rank(), None, df.schema, log, params)
        # --- booster
        t0 = time.perf_counter()
        comm = D.gbdt_comm(use_gpu) if world > 1 else None
        nb = g.Booster(train, params, comm)
        if model_str:
            nb.merge(g.Booster.from_model_string(model_str))
        if valid is not None:
            nb.add_valid(valid, "valid")
        m.mark("booster_init_ms", (time.perf_counter() - t0) * 1e3)
        # iterations from earlier batches / modelString; a mid-batch checkpoint's iterations of THIS batch
        # are counted by _iterate (it starts at _resume_done), so they are not part of the base
        base_iters = nb.current_iteration - getattr(self, "_resume_done", 0)
        best = self._iterate(nb, valid is not None, batch_index, m, n, num_class)
        if best is not None and best >= 0:
            # keep iterations up to and including the best one (BasePartitionTask.scala:450-457)
            nb.truncate(base_iters + best + 1)
        m.mark("total_ms", (time.perf_counter() - t_start) * 1e3)
        t0 = time.perf_counter()
        m["backend"] = nb.backend
        m["native_stats"] = nb.stats()
        t1 = time.perf_counter()
        self._measures.append(m)
        booster = LightGBMBooster(native_booster=nb, best_iteration=best if best is not None else -1)
        _release_training(nb)
        t2 = time.perf_counter()
        del train, valid, data
        t3 = time.perf_counter()
        # after total_ms: the device timings' sync, the training state's release, the datasets' teardown
        m.mark("stats_sync_ms", (t1 - t0) * 1e3)
        m.mark("release_ms", (t2 - t1) * 1e3)
        m.mark("dataset_free_ms", (t3 - t2) * 1e3)
        return booster

    def _sample_rows(self, kind, data, n, share: float = 1.0):
        cnt = int(min(n, max(1, int(self.getBinSampleCount() * share))))
        rng = np.random.default_rng(self.getDataRandomSeed())
        mode = self.getSamplingMode()
        if n == 0:
            return np.zeros((0, _num_cols(kind, data)))
        if kind == "dense" and mode != "fixed" and isinstance(data, np.ndarray) and data.dtype in (np.float32,
                                                                                                   np.float64):
            # native: Floyd sampling of distinct rows + a parallel gather, in the input dtype (no float64 copy)
            pop = data[:min(n, self.getSamplingSubsetSize())] if mode == "subset" else data
            return native.gbdt().sample_dense_rows(np.ascontiguousarray(pop), min(cnt, len(pop)),
                                                   int(self.getDataRandomSeed()) & 0xFFFFFFFFFFFFFFFF)
        if mode == "fixed":
            idx = np.arange(cnt)
        elif mode == "subset":
            sub = min(n, self.getSamplingSubsetSize())
            idx = np.sort(rng.choice(sub, size=min(cnt, sub), replace=False))
        else:
            idx = np.sort(rng.choice(n, size=cnt, replace=False))
        return _sample_dense(kind, data, idx)

    def _build_dataset(self, g, ref, df: DataFrame, kind, data, n, num_class, upload=None):
        ds = g.Dataset(ref, n)
        # the per-row columns first: with a background upload in flight (K1 staging) their host copies run
        # while the feature bytes cross PCIe instead of after the encode (~4 ms for 11M labels)
        ds.set_label(self._labels(df))
        wcol = self.getWeightCol()
        if wcol and wcol in df:
            ds.set_weight(np.asarray(df[wcol], dtype=np.float32))
        icol = self.getInitScoreCol()
        if icol and icol in df:
            s = df[icol]
            if isinstance(s, np.ndarray) and s.ndim == 2:
                arr = np.ascontiguousarray(s.T, dtype=np.float64).ravel()  # class-major
            elif s.dtype == object:
                arr = np.ascontiguousarray(as_matrix(s).T).ravel()
            else:
                arr = np.asarray(s, dtype=np.float64)
            ds.set_init_score(arr)
        gcol = self._group_col()
        if gcol and gcol in df:
            vals = np.asarray(df[gcol])
            # runs of equal consecutive group ids (rows are already grouped)
            starts = _group_runs(vals)[0] if len(vals) else np.zeros(0, np.int64)
            sizes = np.diff(np.append(starts, len(vals)))
            ds.set_group(np.asarray(sizes, dtype=np.int32))
        if kind == "dense":
            # K1: large dense partitions are bin-encoded on the MI355X (bit-identical with the host encoder)
            on_gpu = n >= (1 << 16) and self.getDeviceType() == "gpu" and native.gpu_available()
            if upload is not None:
                ds.push_device_rows(upload, 0)
            elif on_gpu:
                ds.push_dense_gpu(data, 0)
            else:
                chunk = 1 << 20
                for s in range(0, n, chunk):
                    ds.push_dense(data[s: s + chunk], s)
        else:
            indptr, indices, values, _ = data
            ds.push_csr(indptr, indices, values, 0)
        return ds

    def _labels(self, df: DataFrame) -> np.ndarray:
        return np.asarray(df[self.getLabelCol()], dtype=np.float32)

    def _iterate(self, nb, has_valid: bool, batch_index: int, m: InstrumentationMeasures, n: int, num_class: int):
        delegate = self.getDelegate()
        fobj = self.getFobj()
        lr = self.getLearningRate()
        es = self.getEarlyStoppingRound()
        tol = self.getImprovementTolerance()
        names = nb.eval_names()
        best_score = [None] * len(names)
        best_iter = [0] * len(names)
        best_result = None
        provide_train = self.getIsProvideTrainingMetric()
        t0 = time.perf_counter()
        it = getattr(self, "_resume_done", 0)  # iterations already in a resumed checkpoint of this batch
        num_iter = self.getNumIterations()
        ck_every = self.getCheckpointInterval() if self.getCheckpointDir() else 0
        finished = False
        crash_at = _injected_iteration_crash()
        while not finished and it < num_iter:
            if crash_at is not None and it == crash_at:
                os._exit(19)  # test-only (SML_FAULT_INJECT="<rank>:crash_iter=<k>"): this rank dies mid-fit
            if delegate is not None:
                delegate.beforeTrainIteration(batch_index, D.rank(), it, log, None, nb, has_valid)
                new_lr = delegate.getLearningRate(batch_index, D.rank(), it, log, None, lr)
                if new_lr != lr:
                    nb.reset_parameter(f"learning_rate={new_lr}")
                    lr = new_lr
            try:
                if fobj is not None:
                    K = nb.num_model_per_iteration
                    preds = nb.train_scores().reshape(K, -1).T if K > 1 else nb.train_scores()
                    grad, hess = fobj(preds, None)
                    grad = np.asarray(grad, dtype=np.float32)
                    hess = np.asarray(hess, dtype=np.float32)
                    if K > 1 and grad.ndim == 2:
                        grad = np.ascontiguousarray(grad.T).ravel()
                        hess = np.ascontiguousarray(hess.T).ravel()
                    finished = nb.update(grad, hess)
                else:
                    finished = nb.update()
            except RuntimeError as e:
                # a failed or timed-out collective (peer died, link broke, ranks diverged) fails the job on
                # every rank; anything else ends this task's training early (TrainUtils.scala:89-95). The
                # aborted communicator is evicted so a later fit in this process builds a fresh one.
                if isinstance(e, native.gbdt().CommError):
                    D.evict_comm(str(e))
                    raise
                log.warning("training stopped early on this task: %s", e)
                finished = True
            train_res = dict(nb.eval(0)) if provide_train and not finished else None
            valid_res = None
            if has_valid and not finished:
                res = nb.eval(1)
                valid_res = dict(res)
                for i, (name, score) in enumerate(res):
                    higher = name.startswith(("auc", "ndcg@", "map@", "average_precision"))
                    better = (best_score[i] is None or
                              ((score - best_score[i] > tol) if higher else (score - best_score[i] < tol)))
                    if better:
                        best_score[i] = score
                        best_iter[i] = it
                    elif es > 0 and it - best_iter[i] >= es:
                        finished = True
                        best_result = best_iter[i]
            if delegate is not None:
                delegate.afterTrainIteration(batch_index, D.rank(), it, log, None, nb, has_valid, finished,
                                             train_res, valid_res)
            it += 1
            if ck_every > 0 and it % ck_every == 0 and not finished and it < num_iter:
                self._ckpt_write(nb.save_model_string(), batch_index, it, False)
        try:
            nb.synchronize()
        except RuntimeError as e:
            if isinstance(e, native.gbdt().CommError):
                D.evict_comm(str(e))
            raise
        m.mark("training_iterations_ms", (time.perf_counter() - t0) * 1e3)
        return best_result
