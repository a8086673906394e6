"""Port of reference tests/test_v03_migration.py: instance A persists nodes /
edges / profile, instance B loads them, then B detects A's later write via the
table version (two MemorySystems on one directory stand in for 2 processes)."""
from lazzaro_amd.core.memory_shard import MemoryShard
from lazzaro_amd.core.memory_system import MemorySystem
from lazzaro_amd.models.graph import Edge, Node


class MockLLM:
    def completion(self, messages, response_format=None):
        return "{}"

    def completion_stream(self, messages, response_format=None):
        yield ""


class MockEmbedder:
    def embed(self, text):
        return [0.1] * 1536

    def batch_embed(self, texts):
        return [[0.1] * 1536 for _ in texts]


def test_full_persistence_and_sync():
    a = MemorySystem(db_dir="test_v03_db", user_id="test_user", llm_provider=MockLLM(),
                     embedding_provider=MockEmbedder())
    a.shards["work"] = MemoryShard("work")
    a.shards["work"].add_node(Node(id="node_1", content="Fact 1", embedding=[0.1] * 1536, shard_key="work"))
    a.shards["work"].add_edge(Edge(source="node_1", target="node_X", weight=0.9))
    a.profile.update_domain("preferences", "Loves minimalism")
    a._save_to_persistence()

    b = MemorySystem(db_dir="test_v03_db", user_id="test_user", load_from_disk=True,
                     llm_provider=MockLLM(), embedding_provider=MockEmbedder())
    assert len(b.buffer.nodes) == 1 and b.buffer.nodes["node_1"].content == "Fact 1"
    found = [sh.edges[("node_1", "node_X")] for sh in b.shards.values() if ("node_1", "node_X") in sh.edges]
    assert found and abs(found[0].weight - 0.9) < 1e-5
    assert "Loves minimalism" in b.profile.get_context()
    assert b.node_counter == 1

    a.shards["personal"] = MemoryShard("personal")
    a.shards["personal"].add_node(Node(id="node_2", content="Fact 2", embedding=[0.2] * 1536,
                                       shard_key="personal"))
    a._save_to_persistence()
    assert b.check_for_updates() is True
    assert "node_2" in b.buffer.nodes and len(b.buffer.nodes) == 2
    # our own saves are not "updates from elsewhere"
    assert a.check_for_updates() is False
    a.close()
    b.close()
