#!/usr/bin/env python3
"""VowpalWabbitClassifier hashed-sparse training throughput on the MI355X —
BASELINE.json config "VowpalWabbitClassifier 1B-feature hashed sparse
synthetic, 8xMI355X model allreduce".

Per GPU: a 2^bits weight table (default 2^30 = 1B features; 16 B per slot:
weight, adaptive sum of squared gradients, normalizer = 16 GiB resident in HBM), --rows examples per pass with ~--nnz hashed
features each (32-bit hashed ids from a 2^24 vocabulary, Zipf-like). One step = one pass:
host -> device transfer of the pass's CSR (overlapped with learning), hogwild
mini-batches of VW's default adaptive + normalized + invariant update on the
device (K12, logistic loss), then (N > 1) the endPass weighted average over
RCCL of the 64 KiB table blocks some rank touched. Prints one
JSON line with examples/s over all GPUs, the per-pass allreduce time and the
held-out logistic loss. Synthetic data; labels from a planted sparse model."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


_VOCAB = {}


def vocabulary(size_log2=24):
    """Hashed feature ids: 2^24 distinct 32-bit murmur-like hashes and a planted weight per id."""
    if size_log2 not in _VOCAB:
        r = np.random.default_rng(12345)
        ids = r.integers(0, 2 ** 32, size=2 ** size_log2, dtype=np.uint64).astype(np.uint32)
        wt = (r.standard_normal(2 ** size_log2) * 0.4).astype(np.float32)
        _VOCAB[size_log2] = (ids, wt)
    return _VOCAB[size_log2]


def make_pass(n, nnz, seed):
    rng = np.random.default_rng(seed)
    ids, wt = vocabulary()
    counts = rng.integers(max(1, nnz // 2), nnz * 3 // 2 + 1, size=n)
    indptr = np.zeros(n + 1, np.int64)
    np.cumsum(counts, out=indptr[1:])
    tot = int(indptr[-1])
    # Zipf-like popularity: frequent ids repeat across examples, the tail is rare
    v = np.minimum((rng.pareto(1.1, size=tot) * 2000).astype(np.int64), len(ids) - 1)
    idx = ids[v]
    val = np.ones(tot, np.float32)
    margin = np.add.reduceat(wt[v], indptr[:-1])
    y = np.where(margin + 0.3 * rng.standard_normal(n) > 0, 1.0, -1.0).astype(np.float32)
    return indptr, idx, val, y


def estimator_bench(args, world: int, rank: int) -> None:
    """One step = one ``VowpalWabbitClassifier(numBits=30, deviceType='gpu').fit(df)`` on the rank's partition:
    the hashed-feature column is a CSR-backed sparse vector column (zero-copy namespace block), the fit uploads
    it, builds the example rows on the device (constant feature included), learns one pass of hogwild
    mini-batches with VW's default update, averages the touched blocks over RCCL (N > 1) and exports the model
    from the device nonzeros."""
    import torch

    from synapseml_amd.core.dataframe import DataFrame
    from synapseml_amd.core.linalg import CsrColumn
    from synapseml_amd.parallel import distributed as D
    from synapseml_amd.vw import VowpalWabbitClassifier

    ip, idx, val, y = make_pass(args.rows, args.nnz, seed=1000 * rank)
    df = DataFrame({"features": CsrColumn(ip, idx, val, 1 << 32), "label": y.astype(np.float64)})
    hold = make_pass(100_000, args.nnz, seed=999_999)
    hdf = DataFrame({"features": CsrColumn(hold[0], hold[1], hold[2], 1 << 32), "label": hold[3].astype(np.float64)})
    est = VowpalWabbitClassifier(numBits=args.bits, deviceType="gpu", gpuBatchSize=args.batch,
                                 passThroughArgs="--loss_function logistic")
    model = None
    for _ in range(args.warmup):
        model = est.fit(df)
    torch.cuda.synchronize()
    D.barrier()
    t0 = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        model = est.fit(df)
        stats.append({k: float(model.getPerformanceStatistics()[k][0])
                      for k in ("timeNativeIngestNs", "timeLearnNs", "timeTotalNs", "syncBytes", "timeExportNs")
                      if k in model.getPerformanceStatistics()})
    torch.cuda.synchronize()
    D.barrier()
    elapsed = time.perf_counter() - t0
    if args.profile and rank == 0:  # host-side breakdown of one more fit (outside the timed region)
        import cProfile
        import pstats

        pr = cProfile.Profile()
        pr.enable()
        est.fit(df)
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats("cumulative").print_stats(30)
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        raw = model.transform(hdf)["rawPrediction"]
        m = hold[3] * raw
        logloss = float(np.mean(np.log1p(np.exp(-np.clip(m, -50, 50)))))
        ph = {k: round(float(np.mean([s[k] for s in stats])) / 1e6, 2) for k in stats[0]}
        fit_ms = elapsed / args.steps * 1e3
        print(json.dumps({
            "bench": "vw_classifier_fit", "metric": "examples/sec VowpalWabbitClassifier.fit (whole fit, whole job)",
            "value": round(args.rows * world * args.steps / elapsed, 1), "unit": "examples / fit wall second",
            "n_gpus": world, "bits": args.bits, "table_gib": round((2 ** args.bits) * 16 / 2 ** 30, 2),
            "rows_per_gpu": args.rows, "nnz_per_row": args.nnz, "batch": args.batch, "ms_per_fit": round(fit_ms, 1),
            "phases_ms": {"stage_and_first_segment_learn": ph["timeNativeIngestNs"],
                          "remaining_learn_and_sync": ph["timeLearnNs"], "engine_total": ph["timeTotalNs"],
                          "export_model": ph.get("timeExportNs"),
                          "export_model_and_other": round(fit_ms - ph["timeTotalNs"], 2)},
            "sync_mib": round(stats[-1]["syncBytes"] / 2 ** 20, 2), "holdout_logloss": round(logloss, 4),
            "model_mib": round(len(model.getNativeModel()) / 2 ** 20, 2),
            "timed_region": "VowpalWabbitClassifier(numBits, deviceType='gpu').fit(df) end to end (DataFrame built "
                            "before timing)",
            "data": "synthetic hashed sparse (Zipf ids from a 2^24 vocabulary, planted linear model)"}), flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--api", choices=("estimator", "kernel"), default="estimator",
                    help="estimator: VowpalWabbitClassifier(deviceType='gpu').fit(df) end to end (default); "
                         "kernel: the GpuSgd learner alone on a pre-built CSR")
    ap.add_argument("--bits", type=int, default=30)
    ap.add_argument("--rows", type=int, default=2_000_000, help="examples per pass per GPU")
    ap.add_argument("--nnz", type=int, default=64)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=16384, help="hogwild mini-batch (examples in flight)")
    ap.add_argument("--profile", action="store_true", help="estimator mode: cProfile one extra fit (stderr)")
    ap.add_argument("--resident", action="store_true",
                    help="kernel mode: the pass is staged in HBM once and every step re-learns it from there")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench_vw: --gpus {args.gpus} but WORLD_SIZE={world}")
    import torch

    if not torch.cuda.is_available():
        raise SystemExit("bench_vw needs an MI355X")
    if world > torch.cuda.device_count():
        sys.exit(f"bench_vw: {world} ranks but {torch.cuda.device_count()} visible GPU(s)")
    torch.cuda.set_device(local_rank)
    from synapseml_amd.ops import native
    from synapseml_amd.parallel import distributed as D

    if world > 1:
        D.init_from_env("nccl")
    if args.api == "estimator":
        return estimator_bench(args, world, rank)
    vw = native.load("_vw")
    cfg = vw.GpuSgdConfig()
    cfg.bits = args.bits
    cfg.lr = 0.5
    cfg.power_t = 0.5
    cfg.loss = 1  # adaptive / normalized / invariant default on, as in VW
    g = vw.GpuSgd(cfg, local_rank)
    comm = None
    if world > 1:
        uid = vw.nccl_unique_id() if rank == 0 else None
        comm = vw.nccl_comm(D.broadcast_object(uid, 0), rank, world)
    passes = [make_pass(args.rows, args.nnz, seed=1000 * rank + s) for s in range(2)]
    hold = make_pass(100_000, args.nnz, seed=999_999)
    ar_ms, sync_mb = [], []

    if args.resident:
        ip0, ix0, vl0, y0 = passes[0]
        g.stage(ip0, ix0, vl0, y0)

    def one_pass(i):
        if args.resident:
            g.learn_staged(0, args.rows, args.batch)
        else:
            ip, ix, vl, y = passes[i % 2]
            g.learn(ip, ix, vl, y, None, args.batch)
        if comm is not None:
            t = time.perf_counter()
            g.allreduce_average(comm)
            ar_ms.append((time.perf_counter() - t) * 1e3)
            sync_mb.append(g.last_sync_bytes / 2 ** 20)

    for i in range(args.warmup):
        one_pass(i)
    torch.cuda.synchronize()
    D.barrier()
    ar_ms.clear()
    sync_mb.clear()
    t0 = time.perf_counter()
    for i in range(args.steps):
        one_pass(i)
    torch.cuda.synchronize()
    D.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        p = g.predict(hold[0], hold[1], hold[2])
        m = hold[3] * p
        logloss = float(np.mean(np.log1p(np.exp(-np.clip(m, -50, 50)))))
        print(json.dumps({
            "bench": "vw_hashed_sgd_kernel", "metric": "examples/sec GpuSgd learner (kernel only, whole job)",
            "value": round(args.rows * world * args.steps / elapsed, 1), "n_gpus": world, "bits": args.bits,
            "table_gib": round((2 ** args.bits) * 16 / 2 ** 30, 2), "rows_per_gpu_per_pass": args.rows,
            "nnz_per_row": args.nnz, "batch": args.batch, "ms_per_pass": round(elapsed / args.steps * 1e3, 2),
            "allreduce_ms_per_pass": round(float(np.mean(ar_ms)), 2) if ar_ms else None,
            "allreduce_mib_per_pass": round(float(np.mean(sync_mb)), 1) if sync_mb else None,
            "holdout_logloss": round(logloss, 4), "pass_data": "resident in HBM" if args.resident else "uploaded per pass",
            "data": "synthetic hashed sparse (2^24-id vocabulary of 32-bit hashes, Zipf-like popularity, planted model)"}), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    from bench import _parse_gpus, launch_ranks

    if "WORLD_SIZE" not in os.environ and _parse_gpus(sys.argv[1:]) > 1:
        sys.exit(launch_ranks(_parse_gpus(sys.argv[1:]), os.path.abspath(__file__), sys.argv[1:]))
    main()
