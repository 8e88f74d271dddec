"""Bounded-concurrency mapping and retries (reference: core/.../core/utils/
AsyncUtils.scala (bufferedAwait), FaultToleranceUtils.scala:10-31)."""
from __future__ import annotations

import time
from concurrent.futures import ThreadPoolExecutor, TimeoutError as FutTimeout
from typing import Callable, Iterable, Iterator, Optional, Sequence, TypeVar

from ..core.utils import retry_with_timeout

T = TypeVar("T")
R = TypeVar("R")


def buffered_map(fn: Callable[[T], R], items: Iterable[T], concurrency: int,
                 timeout_s: Optional[float] = None) -> Iterator[R]:
    """Ordered map with at most ``concurrency`` calls in flight (results yielded in input order as they
    complete). A per-item ``timeout_s`` raises ``TimeoutError``."""
    if concurrency <= 1:
        for it in items:
            yield fn(it)
        return
    with ThreadPoolExecutor(max_workers=concurrency) as ex:
        pending = []
        it = iter(items)
        for x in it:
            pending.append(ex.submit(fn, x))
            if len(pending) >= concurrency:
                try:
                    yield pending.pop(0).result(timeout=timeout_s)
                except FutTimeout as e:
                    raise TimeoutError(f"buffered_map item exceeded {timeout_s}s") from e
        for f in pending:
            try:
                yield f.result(timeout=timeout_s)
            except FutTimeout as e:
                raise TimeoutError(f"buffered_map item exceeded {timeout_s}s") from e


def retry(fn: Callable[[], T], backoffs_ms: Sequence[int] = (0, 100, 200, 500),
          timeout_s: Optional[float] = None) -> T:
    """Call ``fn`` until it succeeds, sleeping each back-off in turn (FaultToleranceUtils.retryWithTimeout)."""
    return retry_with_timeout(fn, backoffs_ms, timeout_s)


def wait_until(pred: Callable[[], bool], timeout_s: float, poll_s: float = 0.05) -> bool:
    end = time.monotonic() + timeout_s
    while time.monotonic() < end:
        if pred():
            return True
        time.sleep(poll_s)
    return pred()


__all__ = ["buffered_map", "retry", "wait_until"]
