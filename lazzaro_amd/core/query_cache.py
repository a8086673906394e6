"""Thread-safe LRU of query embeddings and retrieval results (reference
``core/query_cache.py:7-59``): md5-keyed, ``max_size`` entries, one entry holds
both the embedding and the result list.

Fix vs reference (SURVEY.md App. C "cache hit inflation"): ``get_results``
only counts a hit when a result list is actually present; an entry holding
just an embedding is a miss for results. Keys/eviction are unchanged.
"""
from __future__ import annotations

import hashlib
import threading
import time
from collections import OrderedDict
from typing import Any, List, Optional


class QueryCache:
    def __init__(self, max_size: int = 1000):
        self.max_size = max_size
        self.cache: "OrderedDict[str, dict]" = OrderedDict()
        self.lock = threading.Lock()
        self.hits = 0
        self.misses = 0

    @staticmethod
    def _hash_query(query: str) -> str:
        return hashlib.md5(query.encode()).hexdigest()

    def _lookup(self, query: str, field: str) -> Optional[Any]:
        key = self._hash_query(query)
        with self.lock:
            ent = self.cache.get(key)
            if ent is not None and ent.get(field) is not None:
                self.cache.move_to_end(key)
                self.hits += 1
                return ent[field]
            self.misses += 1
            return None

    def _store(self, query: str, field: str, value: Any, evict: bool) -> None:
        key = self._hash_query(query)
        with self.lock:
            ent = self.cache.get(key)
            if ent is None:
                self.cache[key] = {field: value, "timestamp": time.time()}
            else:
                ent[field] = value
                self.cache.move_to_end(key)
            if evict:
                while len(self.cache) > self.max_size:
                    self.cache.popitem(last=False)

    def get_embedding(self, query: str) -> Optional[List[float]]:
        return self._lookup(query, "embedding")

    def set_embedding(self, query: str, embedding: List[float]) -> None:
        self._store(query, "embedding", embedding, evict=True)

    def get_results(self, query: str) -> Optional[List[str]]:
        return self._lookup(query, "results")

    def set_results(self, query: str, results: List[str]) -> None:
        self._store(query, "results", results, evict=True)

    def invalidate_results(self) -> None:
        """Drop cached result lists (called when the tenant's index changes)."""
        with self.lock:
            for ent in self.cache.values():
                ent.pop("results", None)

    def get_hit_rate(self) -> float:
        tot = self.hits + self.misses
        return self.hits / tot if tot else 0.0
