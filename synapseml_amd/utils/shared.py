"""Per-process shared state (reference: core/.../io/http/SharedVariable.scala:17-63).

``SharedVariable(constructor)`` lazily builds one value per process and key
(the reference keys a JVM-wide map by a UUID so every task in an executor
reuses e.g. an HTTP client or a loaded model); ``SharedSingleton`` is the
same with thread-safe construction of a single instance."""
from __future__ import annotations

import threading
import uuid
from typing import Callable, Dict, Generic, TypeVar

T = TypeVar("T")

_REGISTRY: Dict[str, object] = {}
_LOCK = threading.Lock()


class SharedVariable(Generic[T]):
    def __init__(self, constructor: Callable[[], T], key: str = None):
        self._ctor = constructor
        self.key = key or uuid.uuid4().hex

    def get(self) -> T:
        v = _REGISTRY.get(self.key)
        if v is None:
            with _LOCK:
                v = _REGISTRY.get(self.key)
                if v is None:
                    v = self._ctor()
                    _REGISTRY[self.key] = v
        return v  # type: ignore[return-value]

    def __getstate__(self):
        # the key travels to worker processes; each builds its own value there
        return {"key": self.key, "_ctor": self._ctor}

    def __setstate__(self, st):
        self.key, self._ctor = st["key"], st["_ctor"]

    def clear(self) -> None:
        with _LOCK:
            _REGISTRY.pop(self.key, None)


class SharedSingleton(SharedVariable[T]):
    @property
    def instance(self) -> T:
        return self.get()


__all__ = ["SharedVariable", "SharedSingleton"]
