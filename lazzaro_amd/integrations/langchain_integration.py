"""LangChain memory adapter (reference integrations/langchain_integration.py:7-71).

Subclasses ``langchain_core.memory.BaseMemory`` when langchain is installed;
otherwise it is a plain class with the same interface (``memory_variables``,
``load_memory_variables``, ``save_context``, ``clear``)."""
from __future__ import annotations

from typing import Any, Dict, List, Optional

from ._common import context_block, record_turn

try:  # optional dependency
    from langchain_core.memory import BaseMemory as _Base  # type: ignore
    from langchain_core.messages import AIMessage as _AIMessage  # type: ignore
    HAVE_LANGCHAIN = True
except Exception:  # pragma: no cover - exercised when langchain is absent
    _Base = object
    _AIMessage = None
    HAVE_LANGCHAIN = False


class LazzaroLangChainMemory(_Base):  # type: ignore[misc]
    memory_system: Any = None
    memory_key: str = "history"
    input_key: Optional[str] = None
    output_key: Optional[str] = None
    return_messages: bool = False

    def __init__(self, memory_system, **kwargs):
        if HAVE_LANGCHAIN:
            super().__init__(memory_system=memory_system, **kwargs)
        else:
            self.memory_system = memory_system
            for k, v in kwargs.items():
                setattr(self, k, v)

    @property
    def memory_variables(self) -> List[str]:
        return [self.memory_key]

    def load_memory_variables(self, inputs: Dict[str, Any]) -> Dict[str, Any]:
        msg = inputs.get(self.input_key) or inputs.get("input") or ""
        if not msg:
            return {self.memory_key: [] if self.return_messages else ""}
        ctx = context_block(self.memory_system, msg, "Relevant Past Memories:")
        if self.return_messages:
            if _AIMessage is None:
                return {self.memory_key: [{"type": "ai", "content": ctx}] if ctx else []}
            return {self.memory_key: [_AIMessage(content=ctx)] if ctx else []}
        return {self.memory_key: ctx}

    def save_context(self, inputs: Dict[str, Any], outputs: Dict[str, str]) -> None:
        u = inputs.get(self.input_key) or inputs.get("input") or ""
        a = outputs.get(self.output_key) or outputs.get("output") or ""
        record_turn(self.memory_system, u, a)

    def clear(self) -> None:
        self.memory_system.end_conversation()
