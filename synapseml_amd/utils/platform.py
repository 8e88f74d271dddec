"""Platform detection and secret lookup (reference:
core/src/main/python/synapse/ml/core/platform/Platform.py:15-95)."""
from __future__ import annotations

import os

PLATFORM_SYNAPSE_INTERNAL = "synapse_internal"
PLATFORM_SYNAPSE = "synapse"
PLATFORM_BINDER = "binder"
PLATFORM_DATABRICKS = "databricks"
PLATFORM_FABRIC = "fabric"
PLATFORM_UNKNOWN = "unknown"
SECRET_STORE = "mmlspark-build-keys"


def current_platform() -> str:
    if os.environ.get("AZURE_SERVICE") == "Microsoft.ProjectArcadia":
        return PLATFORM_SYNAPSE if os.environ.get("SPARK_CLUSTER_TYPE", "synapse") == "synapse" \
            else PLATFORM_SYNAPSE_INTERNAL
    if os.environ.get("FABRIC_TENANT_ID") or os.environ.get("TRIDENT_RUNTIME"):
        return PLATFORM_FABRIC
    if os.path.isdir("/dbfs"):
        return PLATFORM_DATABRICKS
    if os.environ.get("BINDER_LAUNCH_HOST") is not None:
        return PLATFORM_BINDER
    return PLATFORM_UNKNOWN


def running_on_synapse_internal() -> bool:
    return current_platform() == PLATFORM_SYNAPSE_INTERNAL


def running_on_synapse() -> bool:
    return current_platform() == PLATFORM_SYNAPSE


def running_on_binder() -> bool:
    return current_platform() == PLATFORM_BINDER


def running_on_databricks() -> bool:
    return current_platform() == PLATFORM_DATABRICKS


def running_on_fabric() -> bool:
    return current_platform() == PLATFORM_FABRIC


def find_secret(secret_name: str, keyvault: str = SECRET_STORE) -> str:
    """Secrets come from the environment here: ``<KEYVAULT>_<SECRET>`` or ``<SECRET>`` (upper-cased, '-' -> '_').
    Hosted key vault clients are not available offline."""
    norm = lambda s: s.upper().replace("-", "_")  # noqa: E731
    for k in (f"{norm(keyvault)}_{norm(secret_name)}", norm(secret_name)):
        if os.environ.get(k):
            return os.environ[k]
    raise RuntimeError(f"Could not find {secret_name} in keyvault {keyvault}: set the environment variable "
                       f"{norm(secret_name)} (or replace this call with the secret string).")


def materializing_display(data) -> None:
    print(data)


__all__ = ["current_platform", "running_on_synapse", "running_on_synapse_internal", "running_on_binder",
           "running_on_databricks", "running_on_fabric", "find_secret", "materializing_display"]
