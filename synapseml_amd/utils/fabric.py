"""Fabric / token helpers (reference: core/.../fabric/{FabricClient, TokenLibrary, OpenAITokenLibrary}.scala).

Hosted token services are not reachable offline; tokens come from the environment
(``SYNAPSEML_AAD_TOKEN`` / ``SYNAPSEML_OPENAI_TOKEN``) and the ML workload endpoint from
``SYNAPSEML_FABRIC_ENDPOINT``. Cognitive-service transformers use these as their default auth when
``running_on_fabric()``."""
from __future__ import annotations

import json
import os
import urllib.request
from typing import Dict, Optional

from .platform import running_on_fabric


class TokenLibrary:
    @staticmethod
    def getAccessToken(audience: str = "ml") -> Optional[str]:  # noqa: N802
        return os.environ.get("SYNAPSEML_AAD_TOKEN")

    @staticmethod
    def getAuthHeader() -> Optional[str]:  # noqa: N802
        tok = TokenLibrary.getAccessToken()
        return None if tok is None else "Bearer " + tok


class OpenAITokenLibrary(TokenLibrary):
    @staticmethod
    def getAccessToken(audience: str = "openai") -> Optional[str]:  # noqa: N802
        return os.environ.get("SYNAPSEML_OPENAI_TOKEN") or os.environ.get("SYNAPSEML_AAD_TOKEN")


class FabricClient:
    @staticmethod
    def MLWorkloadEndpointML() -> Optional[str]:  # noqa: N802
        return os.environ.get("SYNAPSEML_FABRIC_ENDPOINT")

    @staticmethod
    def available() -> bool:
        return running_on_fabric() and FabricClient.MLWorkloadEndpointML() is not None


# feature names used for certified events (reference: logging/FeatureNames.scala)
FEATURE_NAMES = {"lightgbm": "LightGBM", "vw": "VowpalWabbit", "onnx": "ONNX", "services": "AiServices",
                 "explainers": "Explainers", "causal": "Causal", "recommendation": "Recommendation",
                 "featurize": "Featurize", "stages": "Core", "automl": "AutoML", "dl": "DeepLearning"}


class CertifiedEventClient:
    """Posts certified usage events to the Fabric telemetry endpoint (reference:
    logging/fabric/CertifiedEventClient.scala:13-37). Only active when ``FabricClient.available()``;
    ``install()`` subscribes it to every fit/transform payload of core.logging."""

    @staticmethod
    def feature_name(payload: Dict) -> str:
        mod = str(payload.get("module", "")).split(".")
        return FEATURE_NAMES.get(mod[1] if len(mod) > 1 else "", "SynapseML")

    @staticmethod
    def log_to_certified_events(feature_name: str, activity_name: str, attributes: Dict,
                                endpoint: Optional[str] = None, timeout: float = 5.0) -> Optional[int]:
        endpoint = endpoint or FabricClient.MLWorkloadEndpointML()
        if endpoint is None:
            return None
        body = json.dumps({"timestamp": __import__("time").time(), "feature_name": feature_name,
                           "activity_name": activity_name, "attributes": attributes}).encode()
        req = urllib.request.Request(endpoint.rstrip("/") + "/telemetry", data=body, method="POST",
                                     headers={"Content-Type": "application/json"})
        auth = TokenLibrary.getAuthHeader()
        if auth:
            req.add_header("Authorization", auth)
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return r.status

    # events are posted by one daemon thread from a bounded queue: telemetry never adds latency to a
    # fit/transform (serving mini-batches included); when the endpoint is slow and the queue is full,
    # new events are dropped rather than blocking the caller
    _queue = None
    _lock = __import__("threading").Lock()
    dropped = 0

    @staticmethod
    def _worker(q) -> None:
        while True:
            item = q.get()
            try:
                CertifiedEventClient.log_to_certified_events(*item)
            except Exception:  # noqa: BLE001 - telemetry failures are never surfaced to the workload
                pass
            finally:
                q.task_done()

    @classmethod
    def _enqueue(cls, item) -> None:
        import queue
        import threading

        with cls._lock:
            if cls._queue is None:
                cls._queue = queue.Queue(maxsize=1024)
                threading.Thread(target=cls._worker, args=(cls._queue,), daemon=True,
                                 name="sml-certified-events").start()
        try:
            cls._queue.put_nowait(item)
        except queue.Full:
            cls.dropped += 1

    @staticmethod
    def flush(timeout: float = 5.0) -> None:
        """Wait (up to `timeout`) until queued events were posted (tests, process exit)."""
        import time

        q = CertifiedEventClient._queue
        end = time.monotonic() + timeout
        while q is not None and q.unfinished_tasks and time.monotonic() < end:
            time.sleep(0.01)

    @staticmethod
    def sink(payload: Dict) -> None:
        if payload.get("method") not in ("fit", "transform"):
            return
        attrs = {k: str(v) for k, v in payload.items() if k in ("className", "method", "modelUid", "errorType")}
        CertifiedEventClient._enqueue((CertifiedEventClient.feature_name(payload),
                                       f"{payload.get('className')}.{payload.get('method')}", attrs))

    @staticmethod
    def install(force: bool = False) -> bool:
        from ..core.logging import add_event_sink

        if force or FabricClient.available():
            add_event_sink(CertifiedEventClient.sink)
            return True
        return False


__all__ = ["TokenLibrary", "OpenAITokenLibrary", "FabricClient", "CertifiedEventClient", "FEATURE_NAMES"]
