"""Port of reference tests/test_basic.py (data-model defaults, init defaults)."""
from unittest.mock import patch

from lazzaro_amd.core.memory_system import MemorySystem
from lazzaro_amd.models.graph import Edge, Node


def test_node_creation():
    n = Node(id="test_1", content="Hello world")
    assert n.id == "test_1" and n.content == "Hello world" and n.type == "semantic"
    assert n.salience == 0.5 and n.access_count == 0 and n.is_super_node is False
    assert n.child_ids == [] and n.parent_id is None and n.shard_key == "default"


def test_edge_creation():
    e = Edge(source="a", target="b")
    assert (e.source, e.target, e.weight, e.edge_type, e.co_occurrence) == ("a", "b", 1.0, "relates_to", 1)


def test_node_dict_roundtrip_ignores_unknown_keys():
    n = Node(id="x", content="c", embedding=[1.0, 2.0])
    d = n.to_dict()
    d["vector"] = [9.0]
    d["metadata"] = {}
    m = Node.from_dict(d)
    assert m == n


@patch("lazzaro_amd.core.memory_system.openai")
def test_memory_system_init(mock_openai):
    ms = MemorySystem(openai_api_key="fake-key", enable_async=False)
    assert ms.model == "gpt-4o-mini"
    assert ms.enable_sharding and ms.enable_hierarchy and ms.enable_caching
    assert ms.max_buffer_size == 10 and ms.prune_threshold == 0.5 and ms.consolidate_every == 3
    assert ms.vector_store is ms.store
    ms.close()
