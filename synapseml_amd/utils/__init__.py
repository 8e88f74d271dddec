"""Framework utilities (reference: core/src/main/scala/.../core/utils/*,
io/http/SharedVariable.scala, python synapse/ml/{downloader, plot,
core/spark/FluentAPI, core/platform}).

* ``cluster``   — device / process topology (ClusterUtil)
* ``shared``    — per-process shared singletons (SharedVariable / SharedSingleton)
* ``concurrency`` — bounded-concurrency async map and retries (AsyncUtils, FaultToleranceUtils)
* ``equality``  — stage / model equality (ModelEquality)
* ``platform``  — platform detection and secret lookup
* ``downloader``— local model repository (ModelDownloader)
* ``plot``      — confusion-matrix / ROC plots
* ``fluent``    — ``df.mlTransform`` / ``df.mlFit``
"""
from . import cluster, concurrency, downloader, equality, fluent, platform, plot, shared  # noqa: F401
from .cluster import ClusterInfo, cluster_info
from .concurrency import buffered_map, retry
from .downloader import ModelDownloader, ModelSchema
from .equality import assert_stages_equal
from .shared import SharedSingleton, SharedVariable

__all__ = ["ClusterInfo", "cluster_info", "buffered_map", "retry", "ModelDownloader", "ModelSchema",
           "assert_stages_equal", "SharedSingleton", "SharedVariable", "cluster", "concurrency", "downloader",
           "equality", "fluent", "platform", "plot", "shared"]
