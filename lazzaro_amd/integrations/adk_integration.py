"""Google ADK plugin (reference integrations/adk_integration.py:5-60): a
JSON-schema retrieval tool plus an ``observe`` hook."""
from __future__ import annotations

from ._common import record_turn, retrieve


class LazzaroADKPlugin:
    def __init__(self, memory_system):
        self.memory_system = memory_system

    def as_tool(self):
        return {
            "name": "lazzaro_memory_retrieval",
            "description": "Retrieve relevant past memories and user profile information.",
            "parameters": {"type": "object",
                           "properties": {"query": {"type": "string",
                                                    "description": "The current user query to find relevant memories for."}},
                           "required": ["query"]},
            "func": self.retrieve,
        }

    def retrieve(self, query: str) -> str:
        prof, texts = retrieve(self.memory_system, query)
        parts = []
        if prof:
            parts.append(f"User Profile: {prof}")
        if texts:
            parts.append("Relevant Memories:\n" + "\n".join(texts))
        return "\n\n".join(parts) if parts else "No relevant memories found."

    def observe(self, user_input: str, agent_output: str) -> None:
        record_turn(self.memory_system, user_input, agent_output)
