#!/usr/bin/env python3
"""LightGBMRanker (lambdarank) training throughput — BASELINE.json config
"LightGBMRanker 100M-row synthetic on 8xMI355X, RCCL histogram allreduce".

Per GPU: --rows rows (default 12.5M = 100M / 8, weak scaling) of 28 float
features in query groups of 20-180 documents with graded relevance 0-4.
One step = one complete ``LightGBMRanker(numIterations=100).fit(df)`` on the
rank's DataFrame partition (group prep, sampling, device bin encode, 100
lambdarank iterations, model). Single GPU: ``python tools/bench_ranker.py``;
N GPUs: ``python tools/bench_ranker.py --gpus N`` (launches N ranks). Prints
one JSON line (rank 0): training rows per second of fit wall time over all
GPUs, a phase breakdown, and NDCG@10 on a held-out slice (outside timing).
Data is synthetic (no datasets are downloadable here)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def ranking_data(n: int, f: int, seed: int):
    rng = np.random.default_rng(seed)
    sizes = []
    tot = 0
    while tot < n:
        s = int(min(rng.integers(20, 181), n - tot))
        sizes.append(s)
        tot += s
    sizes = np.asarray(sizes, np.int32)
    X = rng.standard_normal((n, f), dtype=np.float32)
    # relevance: nonlinear score plus a per-query offset and noise, graded 0..4
    qoff = np.repeat(rng.standard_normal(len(sizes)).astype(np.float32) * 0.5, sizes)
    s = 0.9 * X[:, 0] - 0.6 * X[:, 1] * X[:, 2] + 0.5 * np.sin(2 * X[:, 3]) + 0.3 * X[:, 4] + qoff
    s += 0.6 * rng.standard_normal(n, dtype=np.float32)
    y = np.clip(np.floor((s - np.quantile(s, 0.35)) * 1.4), 0, 4).astype(np.float32)
    return X, y, sizes


def ndcg_at(scores, labels, sizes, k=10):
    out, b = [], 0
    for c in sizes:
        sc, lb = scores[b:b + c], labels[b:b + c]
        b += c
        order = np.argsort(-sc, kind="stable")[:k]
        disc = 1.0 / np.log2(np.arange(2, 2 + len(order)))
        dcg = ((2.0 ** lb[order] - 1) * disc).sum()
        ideal = ((2.0 ** np.sort(lb)[::-1][:k] - 1) * disc[: min(k, c)]).sum()
        out.append(dcg / ideal if ideal > 0 else 1.0)
    return float(np.mean(out))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--rows", type=int, default=12_500_000, help="rows per GPU (weak scaling)")
    ap.add_argument("--features", type=int, default=28)
    ap.add_argument("--steps", type=int, default=3, help="timed fits")
    ap.add_argument("--warmup", type=int, default=1, help="untimed fits")
    ap.add_argument("--iterations", type=int, default=100, help="numIterations per fit (reference default 100)")
    ap.add_argument("--leaves", type=int, default=31)
    ap.add_argument("--device", default="gpu")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench_ranker: --gpus {args.gpus} but WORLD_SIZE={world}")
    import torch

    use_gpu = args.device == "gpu" and torch.cuda.is_available()
    if use_gpu:
        if world > torch.cuda.device_count():
            sys.exit(f"bench_ranker: {world} ranks but {torch.cuda.device_count()} visible GPU(s)")
        torch.cuda.set_device(local_rank)
    from synapseml_amd.core.dataframe import DataFrame
    from synapseml_amd.lightgbm import LightGBMRanker
    from synapseml_amd.parallel import distributed as D

    if world > 1:
        D.init_from_env("nccl" if use_gpu else "gloo")
    X, y, sizes = ranking_data(args.rows, args.features, seed=77 + rank)
    # query ids: contiguous groups, unique across ranks (int64 column of the training DataFrame)
    qid = np.repeat(np.arange(len(sizes), dtype=np.int64) + (rank << 40), sizes)
    df = DataFrame({"features": X, "label": y, "query": qid})
    n_hold = min(100_000, args.rows)
    hold_q = int(np.searchsorted(np.cumsum(sizes), n_hold)) + 1
    nh = int(sizes[:hold_q].sum())
    Xh, yh, sh = X[:nh].astype(np.float64), y[:nh], sizes[:hold_q]
    est = LightGBMRanker(numIterations=args.iterations, learningRate=0.1, numLeaves=args.leaves, maxBin=255,
                         minDataInLeaf=20, groupCol="query", evalAt=[10], deviceType="gpu" if use_gpu else "cpu")

    def sync():
        if use_gpu:
            torch.cuda.synchronize()

    model = None
    for _ in range(args.warmup):
        model = est.fit(df)
    sync()
    D.barrier()
    t0 = time.perf_counter()
    measures = []
    for _ in range(args.steps):
        model = est.fit(df)
        measures.append(est.getPerformanceMeasures()[0])
    sync()
    D.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if use_gpu else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    phases = {k: round(float(np.mean([m.get(k, 0.0) for m in measures])), 2)
              for k in ("sampling_ms", "dataset_creation_ms", "booster_init_ms", "training_iterations_ms", "total_ms")}
    if rank == 0:
        nd = ndcg_at(model.getModel().score(Xh, raw=True, classification=False)[:, 0], yh, sh)
        fit_s = elapsed / args.steps
        print(json.dumps({
            "bench": "lightgbm_ranker_fit", "metric": "rows/sec LightGBMRanker.fit (whole fit, whole job)",
            "value": round(args.rows * world * args.steps / elapsed, 1), "unit": "training rows / fit wall seconds",
            "n_gpus": world if use_gpu else 0, "rows_per_gpu": args.rows, "queries_per_gpu": int(len(sizes)),
            "steps": args.steps, "warmup": args.warmup, "ms_per_fit": round(fit_s * 1e3, 1),
            "num_iterations": args.iterations, "fit_phases_ms": phases,
            "group_prep_and_other_ms": round(phases["total_ms"] - phases["sampling_ms"] - phases["dataset_creation_ms"]
                                             - phases["booster_init_ms"] - phases["training_iterations_ms"], 2),
            "iteration_ms": round(phases["training_iterations_ms"] / args.iterations, 3),
            "row_iterations_per_s": round(args.rows * world * args.iterations / (phases["training_iterations_ms"] / 1e3), 1),
            "ndcg@10_holdout_slice": round(nd, 4), "backend": measures[-1].get("backend"),
            "timed_region": "LightGBMRanker(numIterations=100).fit(df) end to end (DataFrame built before timing)",
            "data": "synthetic (28 float features, query groups of 20-180 docs, relevance 0-4)"}), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    from bench import _parse_gpus, launch_ranks

    if "WORLD_SIZE" not in os.environ and _parse_gpus(sys.argv[1:]) > 1:
        sys.exit(launch_ranks(_parse_gpus(sys.argv[1:]), os.path.abspath(__file__), sys.argv[1:]))
    main()
