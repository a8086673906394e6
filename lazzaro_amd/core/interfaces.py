"""Pluggable engine protocols (reference ``core/interfaces.py:3-102``):
``LLMProvider``, ``EmbeddingProvider`` and the ``Store`` persistence/search
protocol. Same method names and signatures; providers written for the
reference work unchanged."""
from __future__ import annotations

from typing import Any, Dict, Iterator, List, Optional, Protocol


class LLMProvider(Protocol):
    def completion(self, messages: List[Dict[str, str]], response_format: Dict = None) -> str:
        """Chat completion; ``response_format={"type": "json_object"}`` asks for JSON."""
        ...

    def completion_stream(self, messages: List[Dict[str, str]],
                          response_format: Dict = None) -> Iterator[str]:
        """Streaming completion yielding text chunks."""
        ...


class EmbeddingProvider(Protocol):
    def embed(self, text: str) -> List[float]:
        ...

    def batch_embed(self, texts: List[str]) -> List[List[float]]:
        ...


class Store(Protocol):
    """Full graph persistence + vector search for one or many tenants."""

    def add_nodes(self, nodes: List[Dict[str, Any]], user_id: str = "default"): ...

    def get_nodes(self, user_id: str = "default") -> List[Dict[str, Any]]: ...

    def get_latest_version(self) -> int: ...

    def search_nodes(self, query_emb: List[float], user_id: str = "default",
                     limit: int = 5) -> List[str]: ...

    def delete_nodes(self, node_ids: List[str], user_id: str = "default"): ...

    def add_edges(self, edges: List[Dict[str, Any]], user_id: str = "default"): ...

    def delete_edges(self, source_id: Optional[str] = None, user_id: str = "default"): ...

    def get_edges(self, source_id: Optional[str] = None,
                  user_id: str = "default") -> List[Dict[str, Any]]: ...

    def save_profile(self, profile_data: Dict[str, Any], user_id: str = "default"): ...

    def load_profile(self, user_id: str = "default") -> Optional[Dict[str, Any]]: ...

    def close(self): ...
