"""Intent of the reference's stale tests (test_vector_store.py,
test_lancedb_integration.py, test_persistence.py), which target the pre-v0.3
API: served here through lazzaro_amd.compat shims and HBMStore aliases."""
import os
from unittest.mock import MagicMock

from lazzaro_amd.compat import LanceDBVectorStore, PersistenceManager
from lazzaro_amd.core.memory_shard import MemoryShard
from lazzaro_amd.core.memory_system import MemorySystem
from lazzaro_amd.models.graph import Node


def test_vector_store_add_and_search():
    vs = LanceDBVectorStore(db_dir="test_vector_db")
    vs.add([{"id": "node_1", "content": "I like apples", "embedding": [0.1] * 1536, "type": "semantic",
             "salience": 0.8, "shard_key": "food", "timestamp": 1234.5},
            {"id": "node_2", "content": "I hate oranges", "embedding": [-0.1] * 1536, "type": "semantic",
             "salience": 0.5, "shard_key": "food", "timestamp": 1235.0}])
    assert vs.search([0.1] * 1536, limit=1) == ["node_1"]
    assert vs.search([-0.1] * 1536, limit=1) == ["node_2"]
    vs.close()


def test_vector_store_delete():
    vs = LanceDBVectorStore(db_dir="test_vector_db")
    vs.add([{"id": "node_1", "content": "test", "embedding": [0.1] * 1536}])
    assert len(vs.search([0.1] * 1536, limit=1)) == 1
    vs.delete(["node_1"])
    assert vs.search([0.1] * 1536, limit=1) == []
    vs.close()


def _emb():
    m = MagicMock()
    m.embed.return_value = [0.1] * 1536
    m.batch_embed.return_value = [[0.1] * 1536]
    return m


def test_sync_on_load():
    ms = MemorySystem(openai_api_key="fake", db_dir="test_int_db", embedding_provider=_emb(),
                      load_from_disk=False)
    sh = MemoryShard("default")
    sh.add_node(Node(id="manual_node", content="Manual content", embedding=[0.2] * 1536))
    ms.shards["default"] = sh
    ms._save_to_persistence()
    ms.close()
    ms2 = MemorySystem(openai_api_key="fake", db_dir="test_int_db", embedding_provider=_emb(),
                       load_from_disk=True)
    assert "manual_node" in ms2.buffer.nodes
    assert "manual_node" in ms2.vector_store.search([0.2] * 1536, limit=1)
    ms2.close()


def test_delete_sync_on_eviction():
    ms = MemorySystem(openai_api_key="fake", db_dir="test_int_db", embedding_provider=_emb(),
                      load_from_disk=False)
    ms.start_conversation()
    ms.add_to_short_term("Delete me later")
    node = Node(id="node_to_delete", content="Delete me later", embedding=[0.3] * 1536)
    ms._get_or_create_shard("default").add_node(node)
    ms.vector_store.add([{"id": node.id, "content": node.content, "embedding": node.embedding}])
    assert "node_to_delete" in ms.vector_store.search([0.3] * 1536)
    ms.max_buffer_size = 0
    ms._enforce_buffer_limit()
    assert "node_to_delete" not in ms.vector_store.search([0.3] * 1536)
    ms.close()


def test_persistence_manager_save_load_and_backup():
    pm = PersistenceManager(db_dir="test_db", filename="test.pkl")
    assert pm.save({"foo": "bar", "num": 123})
    assert os.path.exists("test_db/test.pkl") and not os.path.exists("test_db/test.pkl.bak")
    assert pm.load() == {"foo": "bar", "num": 123}
    pm.save({"v": 2})
    assert os.path.exists("test_db/test.pkl.bak")
    assert pm.load() == {"v": 2}
