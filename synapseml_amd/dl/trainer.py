"""Data-parallel fine-tuning loop shared by the deep-learning estimators
(reference: deep-learning/.../dl/DeepVisionClassifier.py via horovod
TorchEstimator + PyTorch Lightning).

MI355X-first: one process per GPU, ``torch.distributed`` (nccl = RCCL over
xGMI) with DistributedDataParallel bucketed gradient all-reduce overlapped
with backward; bf16 autocast and channels_last on the device; the whole
epoch's tensors stay resident in HBM (288 GB leaves room for the dataset),
so each step is a slice, not a host→device copy. On CPU (tests) the same
loop runs in fp32, optionally under ``gloo`` for multi-process runs."""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class TrainConfig:
    epochs: int = 1
    batch_size: int = 32
    learning_rate: float = 1e-3
    optimizer: str = "adam"
    loss: str = "cross_entropy"
    weight_decay: float = 0.0
    seed: int = 0
    use_gpu: bool = True
    channels_last: bool = True
    log_every: int = 50


def _optimizer(name: str, params, lr: float, wd: float):
    name = name.lower()
    if name == "adam":
        return torch.optim.Adam(params, lr=lr, weight_decay=wd)
    if name == "adamw":
        return torch.optim.AdamW(params, lr=lr, weight_decay=wd)
    if name == "sgd":
        return torch.optim.SGD(params, lr=lr, momentum=0.9, weight_decay=wd)
    if name == "rmsprop":
        return torch.optim.RMSprop(params, lr=lr, weight_decay=wd)
    raise ValueError(f"unsupported optimizer {name!r} (adam, adamw, sgd, rmsprop)")


def _loss(name: str) -> Callable:
    name = name.lower()
    if name in ("cross_entropy", "crossentropy"):
        return F.cross_entropy
    if name in ("nll", "nll_loss"):
        return F.nll_loss
    if name in ("mse", "mse_loss"):
        return lambda out, y: F.mse_loss(out.squeeze(-1), y.float())
    raise ValueError(f"unsupported loss {name!r}")


def device_for(cfg: TrainConfig) -> torch.device:
    if cfg.use_gpu and torch.cuda.is_available():
        import os

        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    return torch.device("cpu")


def fit(model: nn.Module, inputs, labels: torch.Tensor, cfg: TrainConfig,
        forward: Optional[Callable] = None, shard: bool = True) -> dict:
    """Train ``model`` on (inputs, labels). ``inputs`` is a tensor [N, ...] or a dict of tensors (text).

    Returns history {loss: [...per epoch...], steps}. Under an initialised process group each rank trains
    its contiguous shard (``shard=False``: the inputs already are this rank's partition) and gradients are
    averaged by DDP."""
    dev = device_for(cfg)
    torch.manual_seed(cfg.seed)
    dist = torch.distributed.is_available() and torch.distributed.is_initialized()
    rank = torch.distributed.get_rank() if dist else 0
    world = torch.distributed.get_world_size() if dist else 1
    model = model.to(dev)
    is_img = isinstance(inputs, torch.Tensor) and inputs.dim() == 4
    if dev.type == "cuda" and cfg.channels_last and is_img:
        model = model.to(memory_format=torch.channels_last)
    n = labels.shape[0]
    lo, hi = (rank * n // world, (rank + 1) * n // world) if shard else (0, n)

    def _take(t):
        return t[lo:hi].to(dev, non_blocking=True)

    X = {k: _take(v) for k, v in inputs.items()} if isinstance(inputs, dict) else _take(inputs)
    if dev.type == "cuda" and cfg.channels_last and is_img:
        X = X.contiguous(memory_format=torch.channels_last)
    Y = _take(labels)
    net = model
    if dist:
        kw = {"device_ids": [dev.index]} if dev.type == "cuda" else {}
        net = torch.nn.parallel.DistributedDataParallel(model, bucket_cap_mb=64, **kw)
    params = [p for p in model.parameters() if p.requires_grad]
    opt = _optimizer(cfg.optimizer, params, cfg.learning_rate, cfg.weight_decay)
    loss_fn = _loss(cfg.loss)
    fwd = forward or (lambda m, x: m(x))
    m_local = hi - lo
    # every rank runs the same number of steps (DDP collectives must match)
    per_rank = n // world if shard else n
    if dist and not shard:
        t = torch.tensor([n], device=dev if dev.type == "cuda" else "cpu")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        per_rank = int(t.item())
    steps = max(1, math.ceil(per_rank / cfg.batch_size))
    hist = {"loss": [], "steps": 0}
    g = torch.Generator(device="cpu").manual_seed(cfg.seed + rank)
    net.train()
    for _ in range(cfg.epochs):
        perm = torch.randperm(max(1, m_local), generator=g).to(dev)
        tot, cnt = 0.0, 0
        for s in range(steps):
            idx = perm[(s * cfg.batch_size) % max(1, m_local):][:cfg.batch_size]
            xb = {k: v[idx] for k, v in X.items()} if isinstance(X, dict) else X[idx]
            yb = Y[idx]
            with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=dev.type == "cuda"):
                out = fwd(net, xb)
            loss = loss_fn(out.float(), yb)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            tot += float(loss.detach())
            cnt += 1
            hist["steps"] += 1
        hist["loss"].append(tot / max(1, cnt))
    model.eval()
    return hist


@torch.no_grad()
def predict(model: nn.Module, inputs, batch_size: int = 256, use_gpu: bool = True,
            forward: Optional[Callable] = None) -> torch.Tensor:
    dev = device_for(TrainConfig(use_gpu=use_gpu))
    model = model.to(dev).eval()
    fwd = forward or (lambda m, x: m(x))
    n = next(iter(inputs.values())).shape[0] if isinstance(inputs, dict) else inputs.shape[0]
    outs = []
    for s in range(0, n, batch_size):
        xb = {k: v[s:s + batch_size].to(dev) for k, v in inputs.items()} if isinstance(inputs, dict) \
            else inputs[s:s + batch_size].to(dev)
        with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=dev.type == "cuda"):
            outs.append(fwd(model, xb).float().cpu())
    return torch.cat(outs) if outs else torch.empty(0)


__all__ = ["TrainConfig", "fit", "predict", "device_for"]
