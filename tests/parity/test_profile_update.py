"""Port of reference tests/test_profile_update.py: run_consolidation on a
4-node chain updates exactly the 4 profile domains the LLM returns."""
import json
from unittest.mock import MagicMock

from lazzaro_amd.core.memory_system import MemorySystem
from lazzaro_amd.models.graph import Edge, Node


def test_multi_field_profile_update():
    ms = MemorySystem(openai_api_key="dummy", llm_provider=MagicMock(), embedding_provider=MagicMock(),
                      load_from_disk=False, auto_consolidate=False)
    ms._get_embedding = MagicMock(return_value=[0.1] * 10)
    ms._batch_embed = MagicMock(return_value=[[0.1] * 10] * 10)
    mems = ["I love programming in Python for data science.",
            "I tend to be very detail-oriented and patient when debugging.",
            "I have 5 years of experience building scalable distributed systems.",
            "I prefer concise, direct communication in meetings."]
    for i, c in enumerate(mems):
        ms.buffer.add_node(Node(id=f"seed_{i}", content=c, embedding=[0.1] * 10, shard_key="default"))
    for i in range(len(mems) - 1):
        ms.buffer.add_edge(Edge(source=f"seed_{i}", target=f"seed_{i+1}", weight=0.8))
    insights = {"preferences": "User prefers Python/Data Science and concise communication.",
                "personality_traits": "Detail-oriented and patient.",
                "knowledge_domains": "Experienced in scalable distributed systems.",
                "interaction_style": "Direct communication style."}

    def fake_llm(messages, response_format=None):
        if any("Analyze these related memories" in m["content"] for m in messages):
            return json.dumps(insights)
        return "{}"

    ms._call_llm = fake_llm
    res = ms.run_consolidation()
    assert "Updated" in res
    for d, v in insights.items():
        assert ms.profile.data[d] == v
    assert ms.profile.data["key_experiences"] == ""
    ms.close()
