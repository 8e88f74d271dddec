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
