"""Runtime helpers (reference: core/.../core/utils/*).

* ParamsStringBuilder: native config strings with "append if not already
  present" semantics (ParamsStringBuilder.scala:35-206): passThroughArgs go in
  first and win over typed params.
* StopWatch: ns timers used by the performance measures.
* retry_with_timeout: FaultToleranceUtils backoff list 0,100,200,500 ms.
"""
from __future__ import annotations

import re
import time
from typing import Callable, Iterable, List, Optional, TypeVar

T = TypeVar("T")


class ParamsStringBuilder:
    def __init__(self, prefix: str = "", delimiter: str = "=", sep: str = " "):
        self.prefix = prefix
        self.delimiter = delimiter
        self.sep = sep
        self.parts: List[str] = []

    def _contains(self, name: str) -> bool:
        pat = re.compile(r"(^|\s)" + re.escape(self.prefix + name) + r"(" + re.escape(self.delimiter) + r"|\s|$)")
        return bool(pat.search(self.result))

    def append(self, raw: Optional[str]) -> "ParamsStringBuilder":
        if raw:
            self.parts.append(raw.strip())
        return self

    def appendParamValueIfNotThere(self, name: str, value) -> "ParamsStringBuilder":  # noqa: N802
        if value is None or self._contains(name):
            return self
        if isinstance(value, bool):
            value = "true" if value else "false"
        self.parts.append(f"{self.prefix}{name}{self.delimiter}{value}")
        return self

    def appendParamListIfNotThere(self, name: str, values: Optional[Iterable]) -> "ParamsStringBuilder":  # noqa: N802
        vals = list(values or [])
        if not vals or self._contains(name):
            return self
        self.parts.append(f"{self.prefix}{name}{self.delimiter}{','.join(str(v) for v in vals)}")
        return self

    def appendParamFlagIfNotThere(self, name: str, condition: bool = True) -> "ParamsStringBuilder":  # noqa: N802
        if condition and not self._contains(name):
            self.parts.append(f"{self.prefix}{name}")
        return self

    @property
    def result(self) -> str:
        return self.sep.join(p for p in self.parts if p)


class StopWatch:
    def __init__(self):
        self.elapsed_ns = 0
        self._t = None

    def start(self):
        self._t = time.perf_counter_ns()

    def pause(self):
        if self._t is not None:
            self.elapsed_ns += time.perf_counter_ns() - self._t
            self._t = None

    def restart(self):
        self.elapsed_ns = 0
        self.start()

    def measure(self, fn: Callable[[], T]) -> T:
        self.start()
        try:
            return fn()
        finally:
            self.pause()

    def elapsed_ms(self) -> float:
        return self.elapsed_ns / 1e6


def retry_with_timeout(fn: Callable[[], T], backoffs_ms=(0, 100, 200, 500), timeout_s: Optional[float] = None) -> T:
    last: Optional[BaseException] = None
    t0 = time.time()
    for b in backoffs_ms:
        if b:
            time.sleep(b / 1000.0)
        try:
            return fn()
        except Exception as e:  # noqa: BLE001 - mirrors FaultToleranceUtils
            last = e
        if timeout_s is not None and time.time() - t0 > timeout_s:
            break
    assert last is not None
    raise last


def find_unused_column_name(prefix: str, columns: Iterable[str]) -> str:
    cols = set(columns)
    if prefix not in cols:
        return prefix
    i = 1
    while f"{prefix}_{i}" in cols:
        i += 1
    return f"{prefix}_{i}"
