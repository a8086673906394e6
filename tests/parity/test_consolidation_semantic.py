"""Port of reference tests/test_consolidation_semantic.py: near-duplicate facts
across two conversations merge into one node; salience = decay(0.9) = 0.893."""
import json
from unittest.mock import MagicMock

from lazzaro_amd.core.memory_system import MemorySystem


def test_semantic_merging():
    llm, emb = MagicMock(), MagicMock()
    ms = MemorySystem(llm_provider=llm, embedding_provider=emb, enable_async=False, load_from_disk=False)
    llm.completion.return_value = json.dumps({"memories": [
        {"content": "User prefers Python for data science", "type": "semantic", "salience": 0.8, "topic": "work"}]})
    emb.batch_embed.return_value = [[0.1] * 1536]
    ms.start_conversation()
    ms.add_to_short_term("I like Python for DS")
    ms.end_conversation()
    assert ms.buffer.size()[0] == 1
    nid = list(ms.buffer.nodes.keys())[0]
    assert ms.buffer.nodes[nid].content == "User prefers Python for data science"

    llm.completion.return_value = json.dumps({"memories": [
        {"content": "The user has a preference for the Python programming language in data science tasks",
         "type": "semantic", "salience": 0.9, "topic": "work"}]})
    emb.batch_embed.return_value = [[0.1001] * 1536]
    ms.start_conversation()
    ms.add_to_short_term("Python is my go-to for data work")
    ms.end_conversation()
    assert ms.buffer.size()[0] == 1, "semantic duplicates must merge"
    node = ms.buffer.get_node(nid)
    assert abs(node.salience - 0.893) < 1e-3
    assert node.access_count == 1
    ms.close()
