#!/usr/bin/env python3
"""Headline benchmark: ``LightGBMClassifier.fit`` throughput on a Higgs-shape
synthetic DataFrame (11M rows x 28 float features per GPU), 1..8 MI355X.

Metric (BASELINE.md:35, primary): ``N_rows / fit_wall_s`` — rows of the
training DataFrame per second of the WHOLE public ``fit`` call at the
reference's defaults (numIterations 100, numLeaves 31, maxBin 255,
binSampleCount 200000, learningRate 0.1, minDataInLeaf 20, binary objective).
The timed region is everything the reference's ``LightGBMBase.train``
(lightgbm/.../LightGBMBase.scala:36-65,396-447) does after the DataFrame
exists: column extraction, row sampling + bin boundaries (reference dataset),
dataset construction (K1 device bin encode), booster creation, 100 boosting
iterations, and the returned LightGBMClassificationModel with its model
string (forced inside the timed loop: the engine builds the text lazily).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for
N > 1 it runs under torch.distributed.run with one rank per GPU (exact int64
histogram allreduce inside the engine, one per batched round: the one-shot P2P
allreduce over xGMI for messages up to 1 MB, RCCL above; gloo control plane). Started WITHOUT a torchrun
environment and ``--gpus N > 1``, this script launches
``python -m torch.distributed.run --nproc-per-node N bench.py ...`` as a child
process before anything touches the GPU (the parent never imports torch),
streams the ranks' output and exits with the child's code. Every rank checks
that the world it joined has exactly N ranks and, on the GPU, N distinct
devices (``--allow-shared-device`` opts into a rehearsal with ranks sharing a
device); otherwise it fails. One step = one complete ``fit``.
W untimed warmup fits, then exactly K timed fits bracketed by barrier +
device synchronize; time is the max over ranks. ``value`` = total rows x K /
seconds (whole job). Per-GPU rows are fixed as N grows (weak scaling).
The secondary metric (N_rows x numIterations / iteration-loop seconds) and a
per-phase breakdown are reported under ``config``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "rows/sec LightGBMClassifier 11M×28 Higgs-shape synthetic; 1/2/4/8 MI355X"


def higgs_like(n: int, f: int, seed: int):
    """Higgs-shape synthetic: 21 'low-level' heavy-tailed kinematic features
    and 7 'high-level' nonlinear combinations; label from a noisy nonlinear
    score (roughly balanced, AUC ceiling well below 1 like HIGGS)."""
    rng = np.random.default_rng(seed)
    low = f - 7 if f > 7 else f
    X = np.empty((n, f), dtype=np.float32)
    X[:, :low] = rng.standard_normal((n, low), dtype=np.float32)
    X[:, 0:low:3] = np.abs(X[:, 0:low:3]) * 1.5  # pt-like, positive
    for j in range(low, f):
        a, b = (j * 7) % low, (j * 11 + 3) % low
        X[:, j] = np.sqrt(X[:, a] ** 2 + X[:, b] ** 2 + 1.0) + 0.1 * rng.standard_normal(n, dtype=np.float32)
    s = (0.8 * X[:, 0] - 0.6 * X[:, 1] * X[:, 2] + 0.5 * np.sin(X[:, 3] * 2) + 0.4 * X[:, low] - 0.3 * X[:, low + 1]
         + 0.25 * (X[:, 4] > 0.5)) if f > 7 else X[:, 0]
    s = s - np.median(s)
    y = (s + 1.2 * rng.standard_normal(n, dtype=np.float32) > 0).astype(np.float32)
    return X, y


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, script: str, argv: list) -> int:
    """Run ``script argv`` as n torchrun ranks in a CHILD process (no exec, no torch import here: this
    process must not initialise the GPU). Returns the child's exit code."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", script] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 8) // max(n, 1))))
    return subprocess.call(cmd, env=env)


def _parse_gpus(argv: list) -> int:
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            return int(argv[i + 1])
        if a.startswith("--gpus="):
            return int(a.split("=", 1)[1])
    return 1


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5, help="timed fits")
    ap.add_argument("--warmup", type=int, default=1, help="untimed fits")
    ap.add_argument("--rows", type=int, default=11_000_000, help="rows per GPU (weak scaling)")
    ap.add_argument("--features", type=int, default=28)
    ap.add_argument("--leaves", type=int, default=31)
    ap.add_argument("--iterations", type=int, default=100, help="numIterations of each fit (reference default 100)")
    ap.add_argument("--device", default="gpu")
    ap.add_argument("--save-model", default=None, help="write the last model's text here (after timing)")
    ap.add_argument("--profile", action="store_true", help="cProfile one more fit after timing (stderr, host side)")
    ap.add_argument("--allow-shared-device", action="store_true",
                    help="rehearsal only: allow more ranks than visible GPUs (ranks share devices)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but this process is one of WORLD_SIZE={world} ranks; "
              "refusing to report a run whose world differs from the requested GPU count", file=sys.stderr)
        sys.exit(2)

    import torch

    use_gpu = args.device == "gpu" and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
    from synapseml_amd.parallel import distributed as D

    # Control plane: gloo over TCP for every world size. The histogram data plane is the engine's own RCCL
    # communicator (ncclUniqueId handed out over this control plane, P2P one-shot over xGMI on top), so
    # nothing needs an NCCL default group - and the device identities below are agreed on BEFORE any RCCL
    # object exists: ranks that share a GPU are refused (or run the rehearsal) with a clear message instead of
    # RCCL's "Duplicate GPU detected" crash.
    if world > 1:
        D.init_from_env("gloo")
    distinct = 0
    shared = False
    if use_gpu:
        # the devices really in use, by identity (uuid / PCI location), over every rank
        pr = torch.cuda.get_device_properties(torch.cuda.current_device())
        ident = str(getattr(pr, "uuid", "")) + ":%s:%s:%s" % (getattr(pr, "pci_domain_id", ""),
                                                              getattr(pr, "pci_bus_id", ""), getattr(pr, "pci_device_id", ""))
        distinct = len(set(D.all_gather_object(ident)))
        shared = distinct < world
        if shared and not args.allow_shared_device:
            print(f"bench.py: {world} ranks run on {distinct} distinct GPU(s); refusing to report it as a "
                  f"{world}-GPU measurement (pass --allow-shared-device for a shared-device rehearsal)",
                  file=sys.stderr)
            sys.exit(3)
        if shared:
            # ranks share devices: RCCL cannot put two ranks on one device, so histograms go over the one-shot
            # IPC allreduce on a host base communicator
            os.environ["SML_GBDT_SHARED_DEVICE"] = "1"
    from synapseml_amd.core.dataframe import DataFrame
    from synapseml_amd.lightgbm import LightGBMClassifier
    from synapseml_amd.ops import native

    native.gbdt()
    t_gen = time.perf_counter()
    X, y = higgs_like(args.rows, args.features, seed=1234 + rank)
    # this rank's partition of the training DataFrame (one process per GPU = one Spark executor)
    df = DataFrame({"features": X, "label": y})
    gen_s = time.perf_counter() - t_gen
    del X

    est = LightGBMClassifier(numIterations=args.iterations, learningRate=0.1, numLeaves=args.leaves, maxBin=255,
                             binSampleCount=200000, minDataInLeaf=20, objective="binary",
                             deviceType="gpu" if use_gpu else "cpu", metric="auc")

    def sync():
        if use_gpu:
            torch.cuda.synchronize()

    model = None
    for _ in range(args.warmup):
        model = est.fit(df)
        model.getNativeModel()
    sync()
    D.barrier()
    sync()
    t0 = time.perf_counter()
    measures = []
    for _ in range(args.steps):
        model = est.fit(df)
        # the returned model's LightGBM text, as the reference's fit serialises the booster before it returns
        # (BasePartitionTask.scala:450-461); this engine builds the text lazily, so it is forced here
        model.getNativeModel()
        measures.append(est.getPerformanceMeasures()[0])
    sync()
    D.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if args.profile and world == 1:  # outside the timed region (one rank: a fit is collective)
        import cProfile
        import pstats

        pr = cProfile.Profile()
        pr.enable()
        est.fit(df).getNativeModel()
        sync()
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats("cumulative").print_stats(35)
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-phase breakdown (ms, mean over the timed fits) from the estimator's instrumentation measures
    phases = {}
    for k in ("sampling_ms", "dataset_creation_ms", "booster_init_ms", "training_iterations_ms", "total_ms"):
        vals = [m.get(k, 0.0) for m in measures]
        phases[k] = round(float(np.mean(vals)), 2) if vals else None
    native_stats = measures[-1].get("native_stats", {}) if measures else {}
    iter_s = (phases["training_iterations_ms"] or 0.0) / 1e3
    # sanity (outside the timed region): AUC of the last model on 200k fresh rows of the same distribution
    # (a different seed from every rank's training rows: a real holdout, not a train AUC)
    auc = None
    n_hold = min(200_000, args.rows)
    if rank == 0 and model is not None:
        try:
            from sklearn.metrics import roc_auc_score

            X_hold, y_hold = higgs_like(n_hold, args.features, seed=987_654)
            p = model.getModel().score(X_hold.astype(np.float64), raw=False, classification=True)[:, 1]
            auc = float(roc_auc_score(y_hold, p))
        except Exception:  # pragma: no cover
            auc = None
    if args.save_model and rank == 0 and model is not None:
        with open(args.save_model, "w") as fh:
            fh.write(model.getNativeModel())
    total_rows = args.rows * world
    value = total_rows * args.steps / elapsed
    comm = next(iter(D._comm_cache.values()), None) if world > 1 else None
    comm_world = int(comm.world) if comm is not None else world
    if comm_world != world:
        print(f"bench.py: communicator world {comm_world} != {world} ranks", file=sys.stderr)
        sys.exit(4)
    n_devices = distinct if use_gpu else 0
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "rows/s (training rows / LightGBMClassifier.fit wall seconds, %d iterations, whole job)" % args.iterations,
            "n_gpus": n_devices,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            # gradients/hessians fp32 (as the reference's LightGBM), histogram sums 64-bit fixed point per
            # (feature, bin) with a per-row quantum <= 2^-38 of max|g| (at least fp64-of-fp32 precision),
            # split gains and leaf values fp64
            "dtype": "fp32",
            "data": "synthetic Higgs-shape (21 heavy-tailed + 7 derived float32 features), noisy nonlinear labels",
            "config": {
                "model": "LightGBMClassifier(binary, numIterations=%d, numLeaves=%d, maxBin=255, lr=0.1, "
                         "minDataInLeaf=20, binSampleCount=200000)" % (args.iterations, args.leaves),
                "global_batch": total_rows,
                "seq_len": args.features,
                "parallelism": f"dp{world}",
                "rows_per_gpu": args.rows,
                "world": world,
                "distinct_devices": n_devices,
                "shared_device_rehearsal": bool(shared),
                "data_plane_world": comm_world,
                "control_plane": "gloo" if world > 1 else None,
                "data_plane": (None if world == 1 else type(comm).__name__ if comm is None else
                               ("rccl" if use_gpu and not shared else "host") +
                               ("+p2p-ipc" if D.p2p_status.get("active") else "")),
                "timed_region": "LightGBMClassifier.fit(df) end to end + the model's LightGBM text "
                                "(DataFrame built before timing)",
                "fit_phases_ms": phases,
                "iteration_loop_row_iters_per_s": round(total_rows * args.iterations / iter_s, 1) if iter_s else None,
                "iteration_ms": round(phases["training_iterations_ms"] / args.iterations, 3)
                if phases["training_iterations_ms"] else None,
                "backend": measures[-1].get("backend") if measures else None,
                "holdout_auc": auc,
                "holdout_rows": n_hold,
                "datagen_s": round(gen_s, 2),
                "native_comm_ms": native_stats.get("comm_ms"),
                "native_comm_calls": native_stats.get("comm_calls"),
                # histogram bytes: the host-side bound (every expansion slot of every round) and what this rank
                # actually pushed through the device-sized P2P transport (only each round's expansions)
                "comm_bytes_bound": native_stats.get("comm_bytes_max"),
                "comm_bytes_pushed": native_stats.get("comm_dev_bytes"),
                "histogram_accumulation": "int64 fixed point per (feature, bin), exact int64 block reduce -> fp64",
                "histogram_allreduce": (None if world == 1 else "host (gloo)" if not use_gpu else
                                        "p2p-ipc one-shot" if D.p2p_status.get("active") else
                                        "rccl (%s)" % D.p2p_status.get("reason", "")),
            },
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    if "WORLD_SIZE" not in os.environ and _parse_gpus(sys.argv[1:]) > 1:
        sys.exit(launch_ranks(_parse_gpus(sys.argv[1:]), os.path.abspath(__file__), sys.argv[1:]))
    main()
