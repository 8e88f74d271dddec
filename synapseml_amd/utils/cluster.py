"""Process / device topology (reference: core/.../core/utils/ClusterUtil.scala:22-190,
which derives tasks per executor and executor counts from Spark conf).

Here a "worker" is one process pinned to one MI355X (or a CPU process when no
GPU is visible); the topology comes from the torch.distributed environment
(RANK / WORLD_SIZE / LOCAL_RANK / LOCAL_WORLD_SIZE) and the visible devices."""
from __future__ import annotations

import os
import socket
from dataclasses import dataclass
from typing import List


@dataclass
class ClusterInfo:
    rank: int
    world_size: int
    local_rank: int
    local_world_size: int
    num_nodes: int
    devices_per_node: int
    host: str
    backend: str

    @property
    def is_driver(self) -> bool:
        return self.rank == 0


def _device_count() -> int:
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # pragma: no cover - torch always present in this stack
        return 0


def cluster_info() -> ClusterInfo:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    devs = _device_count()
    return ClusterInfo(rank=int(os.environ.get("RANK", "0")), world_size=world,
                       local_rank=int(os.environ.get("LOCAL_RANK", "0")), local_world_size=local_world,
                       num_nodes=max(1, world // max(1, local_world)), devices_per_node=devs,
                       host=os.environ.get("MASTER_ADDR", socket.gethostname()),
                       backend="nccl" if devs > 0 else "gloo")


def num_workers_for(num_rows: int, min_rows_per_worker: int = 1) -> int:
    """Workers to use for a job of ``num_rows`` (never more workers than rows)."""
    info = cluster_info()
    workers = info.world_size if info.world_size > 1 else max(1, info.devices_per_node)
    return max(1, min(workers, num_rows // max(1, min_rows_per_worker)))


def rows_per_partition(num_rows: int, num_partitions: int) -> List[int]:
    base, extra = divmod(num_rows, max(1, num_partitions))
    return [base + (1 if i < extra else 0) for i in range(num_partitions)]


__all__ = ["ClusterInfo", "cluster_info", "num_workers_for", "rows_per_partition"]
