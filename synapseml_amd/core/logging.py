"""Structured usage logging (reference: core/.../logging/SynapseMLLogging.scala
:19-172 and the Python SynapseMLLogger). One JSON payload per constructor /
fit / transform with uid, class, method, library version, column count,
execution seconds and error. Emitted on the ``synapseml_amd`` logger at DEBUG;
nothing is sent anywhere (no telemetry endpoint)."""
from __future__ import annotations

import json
import logging
import re
import time
import traceback

LIBRARY_NAME = "synapseml_amd"
LIBRARY_VERSION = "0.1.0"
PROTOCOL_VERSION = "0.0.1"

logger = logging.getLogger(LIBRARY_NAME)

# Shared Access Signatures must never reach a log (reference: logging/common/Scrubber.scala SASScrubber)
_SAS = re.compile(r"(?i)sig=[a-z0-9%]{43,63}%3d")


def scrub(message: str) -> str:
    """Replace SAS token signatures (``sig=...%3d``) in a message before it is logged."""
    return _SAS.sub("sig=####", message)


def payload(stage, method: str, num_cols=None, seconds=None, error=None) -> dict:
    p = {
        "modelUid": getattr(stage, "uid", None),
        "className": type(stage).__name__,
        "module": type(stage).__module__,
        "method": method,
        "libraryVersion": LIBRARY_VERSION,
        "libraryName": LIBRARY_NAME,
        "protocolVersion": PROTOCOL_VERSION,
    }
    if num_cols is not None:
        p["dfInfo"] = {"input": {"numCols": num_cols}}
    if seconds is not None:
        p["executionSeconds"] = seconds
    if error is not None:
        p["errorType"] = type(error).__name__
        p["errorMessage"] = scrub(str(error))
    return p


_sinks: list = []


def add_event_sink(fn) -> None:
    """Receive every usage payload (dict) - e.g. utils.fabric.CertifiedEventClient's sink."""
    if fn not in _sinks:
        _sinks.append(fn)


def remove_event_sink(fn) -> None:
    if fn in _sinks:
        _sinks.remove(fn)


def _emit(p: dict) -> None:
    if logger.isEnabledFor(logging.DEBUG):
        logger.debug(json.dumps(p))
    for fn in list(_sinks):
        try:
            fn(p)
        except Exception:  # noqa: BLE001 - telemetry never breaks a fit/transform
            logger.debug("event sink failed", exc_info=True)


def log_verb(stage, method: str, fn, df=None):
    t0 = time.perf_counter()
    ncols = len(df.columns) if df is not None and hasattr(df, "columns") else None
    active = bool(_sinks) or logger.isEnabledFor(logging.DEBUG)
    try:
        out = fn()
    except Exception as e:
        if active:
            _emit(payload(stage, method, ncols, time.perf_counter() - t0, e))
            if logger.isEnabledFor(logging.DEBUG):
                logger.debug(scrub(traceback.format_exc()))
        raise
    if active:
        _emit(payload(stage, method, ncols, time.perf_counter() - t0))
    return out


class SynapseMLLogger:
    """Python-side usage logger (reference core/.../python/synapse/ml/core/logging/SynapseMLLogger.py): a
    class that owns a ``uid`` and emits the same payloads as the stages do - constructor (``log_class``),
    free-form messages, and fit / transform / any verb through the ``log_verb`` / ``log_fit`` /
    ``log_transform`` method decorators (timing, input column count, errors)."""

    def __init__(self, library_name: str = None, library_version: str = None, uid: str = None,
                 log_level: int = logging.INFO):
        import uuid

        self.library_name = library_name or LIBRARY_NAME
        self.library_version = library_version or LIBRARY_VERSION
        self.uid = uid or f"{self.library_name}_{uuid.uuid4()}"
        self.logger = logging.getLogger(self.library_name)
        self.logger.setLevel(log_level)

    @classmethod
    def safe_get_spark_context(cls):
        return None  # no Spark: one process per GPU

    @classmethod
    def get_hadoop_conf_entries(cls) -> dict:
        return {}

    def get_required_log_fields(self, uid: str, class_name: str, method: str) -> dict:
        return {"modelUid": uid, "className": class_name, "method": method, "libraryVersion": self.library_version,
                "libraryName": self.library_name, "protocolVersion": PROTOCOL_VERSION}

    def _log(self, info: dict) -> None:
        info = {k: (scrub(v) if isinstance(v, str) else v) for k, v in info.items()}
        self.logger.log(self.logger.level or logging.INFO, json.dumps(info))
        for fn in list(_sinks):
            try:
                fn(info)
            except Exception:  # noqa: BLE001
                logger.debug("event sink failed", exc_info=True)

    def log_message(self, message: str) -> None:
        self._log({"message": message, "libraryName": self.library_name})

    @classmethod
    def get_error_fields(cls, e: Exception) -> dict:
        return {"errorType": type(e).__name__, "errorMessage": scrub(str(e))}

    def log_class(self, feature_name: str) -> None:
        self._log(dict(self.get_required_log_fields(self.uid, type(self).__name__, "constructor"),
                       featureName=feature_name))

    @classmethod
    def get_column_number(cls, args, kwargs):
        for v in list(args) + list(kwargs.values()):
            if hasattr(v, "columns"):
                return len(v.columns)
        return None

    @staticmethod
    def log_verb(method_name: str = None):
        import functools

        def get_wrapper(func):
            @functools.wraps(func)
            def wrapper(self, *args, **kwargs):
                base = self.get_required_log_fields(self.uid, type(self).__name__, method_name or func.__name__)
                ncols = SynapseMLLogger.get_column_number(args, kwargs)
                t0 = time.perf_counter()
                try:
                    out = func(self, *args, **kwargs)
                except Exception as e:
                    self._log(dict(base, executionSeconds=time.perf_counter() - t0, **self.get_error_fields(e)))
                    raise
                info = dict(base, executionSeconds=time.perf_counter() - t0)
                if ncols is not None:
                    info["dfInfo"] = {"input": {"numCols": ncols}}
                self._log(info)
                return out

            return wrapper

        return get_wrapper

    @staticmethod
    def log_transform():
        return SynapseMLLogger.log_verb("transform")

    @staticmethod
    def log_fit():
        return SynapseMLLogger.log_verb("fit")
