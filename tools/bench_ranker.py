#!/usr/bin/env python3
"""LightGBMRanker (lambdarank) training throughput — BASELINE.json config
"LightGBMRanker 100M-row synthetic on 8xMI355X, RCCL histogram allreduce".

Per GPU: --rows rows (default 12.5M = 100M / 8, weak scaling) of 28 float
features in query groups of 20-180 documents with graded relevance 0-4.
One step = one boosting iteration (lambdarank gradients on the device, K2
ranking kernel -> 31-leaf tree -> score update). Single GPU:
``python tools/bench_ranker.py``; N GPUs: ``torchrun --nproc-per-node N
tools/bench_ranker.py``. Prints one JSON line (rank 0): rows/s over all GPUs
and NDCG@10 of the trained model on a held-out slice (outside the timing).
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
    ap.add_argument("--rows", type=int, default=12_500_000, help="rows per GPU (weak scaling)")
    ap.add_argument("--features", type=int, default=28)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--leaves", type=int, default=31)
    ap.add_argument("--device", default="gpu")
    args = ap.parse_args()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = args.device == "gpu" and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local_rank)
    from synapseml_amd.parallel import distributed as D

    if world > 1:
        D.init_from_env("nccl" if use_gpu else "gloo")
    from synapseml_amd.ops import native

    g = native.gbdt()
    X, y, sizes = ranking_data(args.rows, args.features, seed=77 + rank)
    params = (f"objective=lambdarank num_iterations={args.warmup + args.steps} learning_rate=0.1 "
              f"num_leaves={args.leaves} max_bin=255 min_data_in_leaf=20 eval_at=10 "
              f"device_type={'gpu' if use_gpu else 'cpu'} num_machines={world} tree_learner=data")
    names = [f"f{i}" for i in range(args.features)]
    ser = None
    if rank == 0:
        idx = np.sort(np.random.default_rng(1).choice(args.rows, size=min(200_000, args.rows), replace=False))
        ser = bytes(g.DatasetReference.from_sample(X[idx].astype(np.float64), args.rows * world, params, names)
                    .serialize())
    ref = g.DatasetReference.deserialize(D.broadcast_object(ser, 0))
    ds = g.Dataset(ref, args.rows)
    if use_gpu:
        ds.push_dense_gpu(X, 0)
    else:
        ds.push_dense(X, 0)
    ds.set_label(y)
    ds.set_group(sizes)
    n_hold = min(100_000, args.rows)
    hold_q = int(np.searchsorted(np.cumsum(sizes), n_hold)) + 1
    Xh, yh, sh = X[: int(sizes[:hold_q].sum())].astype(np.float64), y[: int(sizes[:hold_q].sum())], sizes[:hold_q]
    del X
    comm = D.gbdt_comm(use_gpu) if world > 1 else None
    booster = g.Booster(ds, params, comm)

    def sync():
        booster.synchronize()
        if use_gpu:
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        booster.update()
    sync()
    D.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        booster.update()
    sync()
    D.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if use_gpu else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        nd = ndcg_at(booster.predict(Xh, 0, 0, -1)[:, 0], yh, sh)
        st = booster.stats()
        print(json.dumps({
            "bench": "lightgbm_ranker", "metric": "rows/sec LightGBMRanker lambdarank (row-iterations/s, whole job)",
            "value": round(args.rows * world * args.steps / elapsed, 1), "n_gpus": world if use_gpu else 0,
            "rows_per_gpu": args.rows, "queries_per_gpu": int(len(sizes)), "steps": args.steps,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "ndcg@10_holdout_slice": round(nd, 4),
            "grad_ms_total": round(st.get("grad_ms", 0.0), 2), "backend": booster.backend,
            "data": "synthetic (28 float features, query groups of 20-180 docs, relevance 0-4)"}), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
