#!/usr/bin/env python3
"""ONNXModel ResNet-50 batch inference, data-parallel over GPUs — BASELINE.json
config "ONNXModel ResNet-50 batch inference on synthetic 224x224 image
DataFrame, 8-GPU DP".

Each rank (one per GPU: ``python tools/bench_onnx_dp.py --gpus N`` launches the N
ranks itself; plain ``python`` for one GPU) holds its own DataFrame partition of
--images synthetic 3x224x224 float tensors and runs the public
``ONNXModel.transform`` (model-zoo ResNet-50 v2 topology, random-init
weights from our ONNX writer, mini-batch --batch, softmax/argmax post
processing) on its GPU — partition-parallel inference as in the reference
(ONNXModel.scala:242-251). No collective is on the inference path; the ranks
only agree on the timing (max over ranks). Prints one JSON line per
precision: images/s over all GPUs."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--images", type=int, default=4096, help="images per GPU")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--precisions", default="fp32,fp16")
    a = ap.parse_args()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus or world > torch.cuda.device_count():
        sys.exit(f"bench_onnx_dp: --gpus {a.gpus}, WORLD_SIZE={world}, {torch.cuda.device_count()} visible GPU(s)")
    torch.cuda.set_device(local_rank)
    from synapseml_amd.core.dataframe import DataFrame
    from synapseml_amd.onnx import ONNXModel, writer
    from synapseml_amd.parallel import distributed as D

    if world > 1:
        D.init_from_env("nccl")
    payload = writer.resnet50_v2(seed=0)
    rng = np.random.default_rng(rank)
    imgs = rng.random((a.images, 3, 224, 224), dtype=np.float32)
    df = DataFrame({"data": imgs})
    for prec in a.precisions.split(","):
        m = (ONNXModel().setModelPayload(payload).setDeviceType("GPU").setPrecision(prec)
             .setFeedDict({"data": "data"}).setFetchDict({"logits": "resnetv24_dense0_fwd"})
             .setArgMaxDict({"logits": "label"}).setMiniBatchSize(a.batch))
        m.transform(df.limit(a.batch))  # warm-up: session build, fusions, hipGraph capture
        torch.cuda.synchronize()
        D.barrier()
        t0 = time.perf_counter()
        out = m.transform(df)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        assert out.count() == a.images
        if world > 1:
            import torch.distributed as dist

            t = torch.tensor([dt], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        if rank == 0:
            print(json.dumps({"bench": "onnx_resnet50_dp", "metric": "images/sec ONNXModel ResNet-50 (whole job)",
                              "value": round(a.images * world / dt, 1), "n_gpus": world, "precision": prec,
                              "images_per_gpu": a.images, "mini_batch": a.batch, "s": round(dt, 3),
                              "data": "synthetic 3x224x224 float tensors, random-init ResNet-50 v2"}), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    from bench import _parse_gpus, launch_ranks

    if "WORLD_SIZE" not in os.environ and _parse_gpus(sys.argv[1:]) > 1:
        sys.exit(launch_ranks(_parse_gpus(sys.argv[1:]), os.path.abspath(__file__), sys.argv[1:]))
    main()
