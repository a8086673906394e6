"""Core orchestration layer (reference ``src/lazzaro/core``)."""
from .buffer_graph import BufferGraph  # noqa: F401
from .memory_shard import MemoryShard  # noqa: F401
from .memory_system import MemorySystem  # noqa: F401
from .profile import Profile  # noqa: F401
from .query_cache import QueryCache  # noqa: F401

__all__ = ["MemorySystem", "MemoryShard", "BufferGraph", "Profile", "QueryCache"]
