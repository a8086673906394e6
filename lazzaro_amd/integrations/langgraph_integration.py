"""LangGraph node factories (reference integrations/langgraph_integration.py:5-71).
No langgraph import is needed: nodes are plain ``state -> update`` callables."""
from __future__ import annotations

from typing import Any, Dict

from ._common import context_block, record_turn


def _text(m) -> str:
    return m.content if hasattr(m, "content") else (m.get("content", "") if isinstance(m, dict) else str(m))


class LazzaroLangGraph:
    def __init__(self, memory_system):
        self.memory_system = memory_system

    def get_memory_node(self):
        def memory_node(state: Dict[str, Any]):
            msgs = state.get("messages", [])
            q = _text(msgs[-1]) if msgs else state.get("input", "")
            if not q:
                return {"lazzaro_context": ""}
            return {"lazzaro_context": context_block(self.memory_system, q, "Past Memories:")}
        return memory_node

    def get_record_node(self):
        def record_node(state: Dict[str, Any]):
            msgs = state.get("messages", [])
            if len(msgs) < 2:
                return {}
            record_turn(self.memory_system, _text(msgs[-2]), _text(msgs[-1]))
            return {}
        return record_node
