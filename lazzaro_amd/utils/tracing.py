"""Tracing / profiling (SURVEY.md §5 "Tracing / profiling").

The reference only wall-clocks retrieval and consolidation with time.time()
(memory_system.py:287-298, :655, :782-784). Here every engine stage can be
timed with HIP events on the stream it runs on (no host sync in the hot path;
events are resolved lazily) and annotated with roctx ranges so rocprofv3
timelines show ``lzk:<stage>`` spans around the kernels:

    from lazzaro_amd.utils.tracing import tracer
    with tracer.stage("search"):
        ...
    tracer.summary()   # {"search": {"calls": n, "total_ms": .., "avg_ms": .., "p50_ms": .., "p95_ms": ..}}

Enabled by ``LZK_TRACE=1`` (or ``tracer.enable()``); disabled it costs one
attribute check per stage.
"""
from __future__ import annotations

import ctypes
import os
import threading
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List

import torch


class _Roctx:
    def __init__(self):
        self.lib = None
        try:
            import torch as _t
            p = os.path.join(os.path.dirname(_t.__file__), "lib", "libroctx64.so")
            for cand in (p, "libroctx64.so"):
                try:
                    self.lib = ctypes.CDLL(cand)
                    break
                except OSError:
                    continue
            if self.lib is not None:
                self.lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                self.lib.roctxRangePop.restype = ctypes.c_int
        except Exception:
            self.lib = None

    def push(self, name: str) -> None:
        if self.lib is not None:
            self.lib.roctxRangePushA(("lzk:" + name).encode())

    def pop(self) -> None:
        if self.lib is not None:
            self.lib.roctxRangePop()


class Tracer:
    def __init__(self):
        self.enabled = os.environ.get("LZK_TRACE", "0") == "1"
        self._pending: List = []
        self._times: Dict[str, List[float]] = defaultdict(list)
        self._lock = threading.Lock()
        self._roctx = None

    def enable(self, on: bool = True) -> None:
        self.enabled = on

    @contextmanager
    def stage(self, name: str, device=None):
        if not self.enabled:
            yield
            return
        if self._roctx is None:
            self._roctx = _Roctx()
        self._roctx.push(name)
        gpu = torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")
        if gpu:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            try:
                yield
            finally:
                e.record()
                self._roctx.pop()
                with self._lock:
                    self._pending.append((name, s, e))
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self._roctx.pop()
                with self._lock:
                    self._times[name].append((time.perf_counter() - t0) * 1e3)

    def _resolve(self) -> None:
        with self._lock:
            pend, self._pending = self._pending, []
        for name, s, e in pend:
            e.synchronize()
            self._times[name].append(s.elapsed_time(e))

    def summary(self) -> Dict[str, Dict[str, float]]:
        self._resolve()
        out = {}
        for k, v in self._times.items():
            vs = sorted(v)
            out[k] = {"calls": len(v), "total_ms": round(sum(v), 3), "avg_ms": round(sum(v) / len(v), 4),
                      "p50_ms": round(vs[len(vs) // 2], 4),
                      "p95_ms": round(vs[min(len(vs) - 1, int(0.95 * len(vs)))], 4)}
        return out

    def reset(self) -> None:
        self._resolve()
        self._times.clear()


tracer = Tracer()
