"""Rank failure detection and elastic recovery ("Failure
detection / elastic recovery"; the reference has no process groups at all).

Model: one process per GPU, tenants placed by rendezvous hashing
(:mod:`.placement`), every tenant's durable state in the shared versioned
columnar store (``store/colstore``). A dead rank therefore loses no data --
only ownership has to move:

1. **Detect** -- :class:`Heartbeat` bumps a per-rank counter in a shared
   key-value store (``torch.distributed`` ``FileStore`` on the shared db
   directory, or the rendezvous ``TCPStore``) from a daemon thread;
   :func:`detect_failed` samples the counters twice and reports the ranks
   that did not advance. Clock-free, so it also works across hosts, and it
   never touches the (possibly wedged) communicator.
2. **Re-form** -- :func:`reform_group` tears the old process group down
   locally and rendezvouses the survivors in a fresh group (new store key
   per generation), ranks renumbered densely.
3. **Re-place** -- :class:`ElasticPlacement` keeps the ORIGINAL rank ids of
   the survivors and uses rendezvous hashing restricted to them, so tenants
   of surviving ranks stay put and only the dead ranks' tenants move (each to
   its runner-up rank), which then reloads them from the store.

Collective failures surface as :class:`~lazzaro_amd.utils.faults.CommError`
from :class:`~lazzaro_amd.parallel.comm.Communicator`.
"""
from __future__ import annotations

import threading
import time
from datetime import timedelta
from typing import Callable, Dict, Iterable, List, Optional

import torch.distributed as dist

from ..utils.faults import RankFailure


class Heartbeat:
    """Per-rank liveness counter in a ``torch.distributed.Store``."""

    def __init__(self, store, rank: int, world: int, prefix: str = "lzk/hb", interval: float = 0.2):
        self.store, self.rank, self.world = store, int(rank), int(world)
        self.prefix, self.interval = prefix, float(interval)
        self._stop = threading.Event()
        self._thr: Optional[threading.Thread] = None

    def key(self, r: int) -> str:
        return f"{self.prefix}/{r}"

    def beat(self) -> None:
        self.store.add(self.key(self.rank), 1)

    def start(self) -> "Heartbeat":
        self.beat()

        def run():
            while not self._stop.wait(self.interval):
                try:
                    self.beat()
                except Exception:  # store gone: stop quietly (we are probably shutting down)
                    return
        self._thr = threading.Thread(target=run, name=f"lzk-heartbeat-{self.rank}", daemon=True)
        self._thr.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thr is not None:
            self._thr.join(timeout=5)

    def counters(self, ranks: Iterable[int]) -> Dict[int, int]:
        out = {}
        for r in ranks:
            k = self.key(r)
            out[r] = int(self.store.add(k, 0)) if self.store.check([k]) else 0
        return out


def detect_failed(hb: Heartbeat, window: float = 1.0, ranks: Optional[Iterable[int]] = None) -> List[int]:
    """Ranks whose heartbeat counter did not advance within ``window`` s."""
    ranks = list(range(hb.world)) if ranks is None else list(ranks)
    c0 = hb.counters(ranks)
    time.sleep(window)
    c1 = hb.counters(ranks)
    return sorted(r for r in ranks if r != hb.rank and c1[r] == c0[r])


def reform_group(store_factory: Callable[[int, int], object], survivors: List[int], my_rank: int,
                 backend: str = "gloo", generation: int = 1, timeout: float = 60.0) -> int:
    """Destroy the current process group (locally) and rendezvous the
    survivors in a new one. ``store_factory(generation, new_world)`` returns
    the store for the new group. Returns this process's new (dense) rank."""
    survivors = sorted(survivors)
    if my_rank not in survivors:
        raise RankFailure([my_rank], "this rank is not among the survivors")
    if dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:
            pass
    new_rank = survivors.index(my_rank)
    store = store_factory(generation, len(survivors))
    dist.init_process_group(backend, store=store, rank=new_rank, world_size=len(survivors),
                            timeout=timedelta(seconds=timeout))
    return new_rank


class ElasticPlacement:
    """Tenant -> ORIGINAL rank id among the live ranks (rendezvous hashing)."""

    def __init__(self, world: int, alive: Optional[Iterable[int]] = None):
        self.world = int(world)
        self.alive = sorted(range(self.world) if alive is None else set(alive))

    def owner(self, tenant: str) -> int:
        from ..store.colstore import _rt
        if len(self.alive) == self.world:
            return int(_rt().tenant_rank(tenant, self.world))
        return int(_rt().tenant_rank_among(tenant, self.alive))

    def remove(self, dead: Iterable[int]) -> "ElasticPlacement":
        return ElasticPlacement(self.world, [r for r in self.alive if r not in set(dead)])

    def moved(self, tenants: Iterable[str], after: "ElasticPlacement") -> Dict[str, int]:
        """Tenants whose owner changes between self and ``after`` -> new owner."""
        out = {}
        for t in tenants:
            a, b = self.owner(t), after.owner(t)
            if a != b:
                out[t] = b
        return out
