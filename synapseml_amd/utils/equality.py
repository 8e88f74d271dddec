"""Stage equality for tests and round-trip checks (reference:
core/.../core/utils/ModelEquality.scala, test fuzzing's experiment-result
comparison)."""
from __future__ import annotations

from typing import Any

import numpy as np


def values_equal(a: Any, b: Any, rtol: float = 1e-9, atol: float = 1e-12) -> bool:
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        try:
            a2, b2 = np.asarray(a), np.asarray(b)
            if a2.shape != b2.shape:
                return False
            if a2.dtype.kind in "fc" or b2.dtype.kind in "fc":
                return bool(np.allclose(a2, b2, rtol=rtol, atol=atol, equal_nan=True))
            return all(values_equal(x, y) for x, y in zip(a2.ravel().tolist(), b2.ravel().tolist()))
        except (TypeError, ValueError):
            return False
    if isinstance(a, dict) and isinstance(b, dict):
        return a.keys() == b.keys() and all(values_equal(a[k], b[k]) for k in a)
    if isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)):
        return len(a) == len(b) and all(values_equal(x, y) for x, y in zip(a, b))
    if isinstance(a, float) and isinstance(b, float):
        return (np.isnan(a) and np.isnan(b)) or abs(a - b) <= atol + rtol * abs(b)
    if hasattr(a, "extractParamMap") and hasattr(b, "extractParamMap"):
        return stages_equal(a, b)
    if hasattr(a, "toArray") and hasattr(b, "toArray"):
        return values_equal(a.toArray(), b.toArray())
    try:
        return bool(a == b)
    except Exception:  # noqa: BLE001 - incomparable objects
        return a is b


def stages_equal(a, b) -> bool:
    if type(a) is not type(b):
        return False
    pa, pb = a.extractParamMap(), b.extractParamMap()
    if pa.keys() != pb.keys():
        return False
    return all(values_equal(pa[k], pb[k]) for k in pa if not callable(pa[k]))


def assert_stages_equal(a, b) -> None:
    if type(a) is not type(b):
        raise AssertionError(f"stage types differ: {type(a).__name__} vs {type(b).__name__}")
    pa, pb = a.extractParamMap(), b.extractParamMap()
    for k in sorted(set(pa) | set(pb)):
        if callable(pa.get(k)):
            continue
        if not values_equal(pa.get(k), pb.get(k)):
            raise AssertionError(f"param {k!r} differs: {pa.get(k)!r} vs {pb.get(k)!r}")


__all__ = ["values_equal", "stages_equal", "assert_stages_equal"]
