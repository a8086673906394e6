"""Failure detection and fault injection (SURVEY.md §5, row "Failure
detection / elastic recovery / fault injection").

The reference degrades silently: provider errors become ``""`` or zero vectors
(reference ``core/providers.py:17-19, 45-47, 55-57``), a JSON parse error in
fact extraction prints and returns with the drained memories lost
(``memory_system.py:697-699``), and ``check_for_updates`` swallows everything
(``:1425-1427``). This module gives the engine:

* a typed error hierarchy (:class:`LazzaroError` and subclasses) so callers can
  tell a provider outage from a store or collective failure;
* named **fault points** compiled into every boundary where a real failure can
  happen -- provider calls, store commits, collectives, kernel launches. A
  point is a dictionary lookup when nothing is armed. Tests (or an operator,
  via ``LZK_FAULTS="name:count[:ErrorClass],..."``) arm a point to make its next
  ``count`` passes raise;
* :func:`retry` with bounded exponential backoff for transient failures.

Recovery policies built on top of these live where the state is:
``core.consolidation`` re-queues a failed consolidation batch instead of
dropping it, ``core.memory_system`` keeps the in-memory graph authoritative and
retries a failed persistence on the next save, and ``parallel.elastic``
detects dead ranks by heartbeat and re-forms the process group.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from typing import Callable, Dict, Optional, Tuple, Type

log = logging.getLogger("lazzaro_amd.faults")


class LazzaroError(RuntimeError):
    """Base class of every error the engine raises on purpose."""


class ProviderError(LazzaroError):
    """An LLM or embedding provider failed (network, quota, bad response)."""


class EmbeddingError(ProviderError):
    """Embeddings could not be produced, or came back degenerate (zero/NaN)."""


class StoreError(LazzaroError):
    """The persistent store could not commit or read."""


class CommError(LazzaroError):
    """A collective failed or timed out (peer died, network partition)."""


class RankFailure(CommError):
    """One or more ranks stopped responding; ``ranks`` lists them."""

    def __init__(self, ranks, msg: str = ""):
        self.ranks = sorted(set(int(r) for r in ranks))
        super().__init__(msg or f"ranks {self.ranks} failed")


class KernelError(LazzaroError):
    """A HIP kernel launch returned an error code."""


class InjectedFault(LazzaroError):
    """Raised by an armed fault point whose error class was not specified."""


_ERRORS: Dict[str, Type[BaseException]] = {c.__name__: c for c in (
    LazzaroError, ProviderError, EmbeddingError, StoreError, CommError, KernelError, InjectedFault,
    RuntimeError, TimeoutError, OSError, ValueError)}


class FaultInjector:
    """Registry of armed fault points (thread-safe)."""

    def __init__(self):
        self._armed: Dict[str, Tuple[int, Type[BaseException]]] = {}
        self._hits: Dict[str, int] = {}
        self._lock = threading.Lock()
        spec = os.environ.get("LZK_FAULTS", "")
        if spec:
            self.load_spec(spec)

    def load_spec(self, spec: str) -> None:
        for item in filter(None, (s.strip() for s in spec.split(","))):
            parts = item.split(":")
            name = parts[0]
            count = int(parts[1]) if len(parts) > 1 and parts[1] else 1
            exc = _ERRORS.get(parts[2], InjectedFault) if len(parts) > 2 else InjectedFault
            self.arm(name, count, exc)

    def arm(self, name: str, count: int = 1, exc: Type[BaseException] = InjectedFault) -> None:
        with self._lock:
            self._armed[name] = (int(count), exc)

    def disarm(self, name: Optional[str] = None) -> None:
        with self._lock:
            if name is None:
                self._armed.clear()
            else:
                self._armed.pop(name, None)

    def hits(self, name: str) -> int:
        return self._hits.get(name, 0)

    def check(self, name: str) -> None:
        if not self._armed:  # fast path: nothing armed anywhere
            return
        with self._lock:
            ent = self._armed.get(name)
            if ent is None:
                return
            count, exc = ent
            if count <= 1:
                del self._armed[name]
            else:
                self._armed[name] = (count - 1, exc)
            self._hits[name] = self._hits.get(name, 0) + 1
        log.warning("fault injected at %s", name)
        raise exc(f"injected fault at {name}")


injector = FaultInjector()


def fault_point(name: str) -> None:
    """Raise if ``name`` is armed (see :class:`FaultInjector`)."""
    injector.check(name)


class armed:
    """Context manager for tests: ``with armed("store.commit", 2, StoreError): ...``."""

    def __init__(self, name: str, count: int = 1, exc: Type[BaseException] = InjectedFault):
        self.name, self.count, self.exc = name, count, exc

    def __enter__(self):
        injector.arm(self.name, self.count, self.exc)
        return injector

    def __exit__(self, *a):
        injector.disarm(self.name)
        return False


def retry(fn: Callable, *, attempts: int = 3, base_delay: float = 0.05, max_delay: float = 2.0,
          retry_on: Tuple[Type[BaseException], ...] = (Exception,), on_error: Callable = None):
    """Call ``fn()`` up to ``attempts`` times with exponential backoff; the
    last failure propagates."""
    delay = base_delay
    for i in range(attempts):
        try:
            return fn()
        except retry_on as e:  # noqa: PERF203
            if on_error is not None:
                on_error(i, e)
            if i == attempts - 1:
                raise
            time.sleep(delay)
            delay = min(max_delay, delay * 2)
    return None  # pragma: no cover


def degenerate_embedding(v) -> bool:
    """True for the zero / non-finite vectors failing providers return."""
    try:
        import math
        s = 0.0
        for x in v:
            if not math.isfinite(x):
                return True
            s += abs(x)
        return s == 0.0
    except TypeError:
        return True
